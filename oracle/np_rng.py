"""Pure-Python restatement of the NumPy Generator(PCG64) draws the reference's reset makes —
TEST INFRASTRUCTURE (checks the device-side NumPy-exact reset, gym-usv_amd/csrc/usv_kernels.hip
`NpPcg64`, and is itself checked against numpy in tests/test_np_rng.py).

Algorithms (numpy 2.x, numpy/random/src): PCG64 = 128-bit LCG with the XSL-RR output, stepped
before each output; next_uint32 buffers the high half of a 64-bit draw; next_double =
(next64 >> 11) * 2^-53; random_standard_normal = ziggurat over the ki/wi/fi tables
(np_ziggurat.inc, extracted by tools/gen_np_ziggurat.py); Generator.uniform(lo, hi) =
lo + (hi - lo) * next_double; Generator.integers(lo, hi) with hi - lo - 1 < 2^32 = Lemire's
bounded draw over next_uint32.  Used by the reference at simple_env.py:234-290.
"""
from __future__ import annotations

import math
import os
import re

import numpy as np

M128 = (1 << 128) - 1
MULT = (2549297995355413924 << 64) + 4865540595714422341
ZIG_R = 3.6541528853610088
ZIG_INV_R = 0.27366123732975828
_INC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "gym-usv_amd", "csrc", "np_ziggurat.inc")


def _tables():
    src = open(_INC).read()
    blocks = re.findall(r"(\w+)\[256\] = \{(.*?)\};", src, flags=re.S)
    t = {}
    for name, body in blocks:
        vals = [v.strip() for v in body.split(",") if v.strip()]
        t[name] = [int(v[:-3], 16) for v in vals] if name == "kNpZigKi" else [float.fromhex(v) for v in vals]
    return t["kNpZigKi"], t["kNpZigWi"], t["kNpZigFi"]


KI, WI, FI = _tables()


def pcg64_words(seed):
    """(state, inc, has_uint32, uinteger) of Generator(PCG64(SeedSequence(seed))) as numpy holds it."""
    st = np.random.PCG64(np.random.SeedSequence(seed)).state
    return st["state"]["state"], st["state"]["inc"], st["has_uint32"], st["uinteger"]


class Pcg64:
    def __init__(self, state, inc, has_uint32=0, uinteger=0):
        self.state, self.inc, self.has32, self.u32 = state, inc, has_uint32, uinteger

    def next64(self):
        self.state = (self.state * MULT + self.inc) & M128
        hi, lo = self.state >> 64, self.state & ((1 << 64) - 1)
        x, rot = hi ^ lo, self.state >> 122
        return ((x >> rot) | (x << ((64 - rot) & 63))) & ((1 << 64) - 1)

    def next32(self):
        if self.has32:
            self.has32 = 0
            return self.u32
        v = self.next64()
        self.has32, self.u32 = 1, v >> 32
        return v & 0xFFFFFFFF

    def next_double(self):
        return (self.next64() >> 11) * (1.0 / 9007199254740992.0)

    def standard_normal(self):
        while True:
            r = self.next64()
            idx = r & 0xFF
            r >>= 8
            sign = r & 1
            rabs = (r >> 1) & 0x000FFFFFFFFFFFFF
            x = rabs * WI[idx]
            if sign:
                x = -x
            if rabs < KI[idx]:
                return x
            if idx == 0:
                while True:
                    xx = -ZIG_INV_R * math.log1p(-self.next_double())
                    yy = -math.log1p(-self.next_double())
                    if yy + yy > xx * xx:
                        return -(ZIG_R + xx) if (rabs >> 8) & 1 else ZIG_R + xx
            elif (FI[idx - 1] - FI[idx]) * self.next_double() + FI[idx] < math.exp(-0.5 * x * x):
                return x

    def normal(self, loc, scale):
        return loc + scale * self.standard_normal()

    def uniform(self, lo, hi):
        return lo + (hi - lo) * self.next_double()

    def integers(self, lo, hi):
        """Generator.integers(lo, hi) for hi - lo <= 2^32 (Lemire, 32-bit)."""
        rng = hi - 1 - lo
        excl = rng + 1
        m = self.next32() * excl
        left = m & 0xFFFFFFFF
        if left < excl:
            thr = (0xFFFFFFFF - rng) % excl
            while left < thr:
                m = self.next32() * excl
                left = m & 0xFFFFFFFF
        return lo + (m >> 32)


class Mt19937:
    """np.random's legacy RandomState stream (MT19937) as the legacy envs' resets draw it
    (np.random.uniform, usv_asmc_env.py:258-279); mirrors the device NpMt."""

    def __init__(self, seed):
        _, key, pos, _, _ = np.random.RandomState(seed).get_state(legacy=True)
        self.key, self.pos = [int(k) for k in key], int(pos)

    def _twist(self):
        k = self.key
        for i in range(624):
            y = (k[i] & 0x80000000) | (k[(i + 1) % 624] & 0x7FFFFFFF)
            k[i] = k[(i + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        self.pos = 0

    def next32(self):
        if self.pos >= 624:
            self._twist()
        y = self.key[self.pos]
        self.pos += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF

    def uniform(self, lo, hi):
        a, b = self.next32() >> 5, self.next32() >> 6
        return lo + (hi - lo) * ((a * 67108864.0 + b) / 9007199254740992.0)
