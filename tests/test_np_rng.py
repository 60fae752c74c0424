"""NumPy-exact reset mode (USV_RESET_NUMPY_PCG64), CPU side: the Python restatement of NumPy's
Generator(PCG64) draws (oracle/np_rng.py, which the device NpPcg64 mirrors) against numpy
itself, the USV_FIELD_NP_RNG word layout, and the device reset's draw order against the oracle's
reset (itself pinned by the reference-generated golden rollouts)."""
import math

import numpy as np
import pytest

from oracle import np_rng as R
from oracle import usv_oracle as O


@pytest.mark.parametrize("seed", [0, 1, 7, 1000, 123456789])
def test_pcg64_draws_match_numpy(seed):
    g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
    p = R.Pcg64(*R.pcg64_words(seed))
    pick = np.random.default_rng(seed + 1).integers(0, 4, size=3000)
    for k, c in enumerate(pick):
        if c == 0:
            a, b = g.normal(scale=0.5), p.normal(0.0, 0.5)
        elif c == 1:
            a, b = g.uniform(-np.pi, np.pi), p.uniform(-np.pi, np.pi)
        elif c == 2:
            a, b = g.integers(15, 30), p.integers(15, 30)
        else:
            a, b = g.standard_normal(), p.standard_normal()
        assert a == b, (k, c)
    st = g.bit_generator.state
    assert (st["state"]["state"], st["has_uint32"], st["uinteger"]) == (p.state, p.has32, p.u32)


def test_ziggurat_tail_paths_match_numpy():
    """200k normals: the wedge (fi / exp) and idx-0 tail (log1p) branches all occur."""
    g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(7)))
    p = R.Pcg64(*R.pcg64_words(7))
    a = g.standard_normal(200000)
    b = np.array([p.standard_normal() for _ in range(200000)])
    assert np.array_equal(a, b)
    assert np.abs(a).max() > R.ZIG_R            # the idx-0 tail was drawn


def test_np_rng_words_layout():
    from gym_usv_amd.vector_env import np_rng_words
    w = np_rng_words([5, 6]).view(np.uint32).astype(np.uint64)
    for i, sd in enumerate((5, 6)):
        st, inc, h, u = R.pcg64_words(sd)
        words = [int(w[i, 2 * k]) | (int(w[i, 2 * k + 1]) << 32) for k in range(4)]
        assert words == [st >> 64, st & ((1 << 64) - 1), inc >> 64, inc & ((1 << 64) - 1)]
        assert (int(w[i, 8]), int(w[i, 9])) == (h, u)


def np_reset_py(g):
    """Statement-for-statement mirror of the device np_reset (usv_kernels.hip)."""
    kb = 20.0
    sx = 0.5 * g.standard_normal() + kb / 2
    sy = 0.5 * g.standard_normal() + kb / 2
    g.standard_normal(); g.standard_normal(); g.next_double()
    psi = g.uniform(-math.pi, math.pi)
    ang, dist = g.uniform(-math.pi, math.pi), g.uniform(100, 110)
    tx, ty = g.uniform(0, kb), g.uniform(0, kb)
    u, v, r = g.uniform(0.0, 0.15), g.uniform(0.0, 0.15), g.uniform(0.0, 0.15)
    mu = g.uniform(1.50, 3)
    g.next_double(); g.next_double()
    mr = g.uniform(3, 6)
    refv = g.uniform(0.75, mu)
    n = g.integers(15, 30)
    obs = []
    for _ in range(n):
        ox, oy = g.uniform(0, kb), g.uniform(0, kb)
        if not (math.hypot(sx - ox, sy - oy) < 0.5 or math.hypot(tx - ox, ty - oy) < 0.5):
            obs.append((ox, oy))
    if not obs:
        obs.append((g.uniform(0, kb), g.uniform(0, kb)))
    rad = [g.uniform(0.15, 0.5) for _ in obs]
    return dict(position=[sx, sy, psi], path_end=[sx + math.cos(ang) * dist, sy + math.sin(ang) * dist],
                target=[tx, ty], velocity=[u, v, r], max_u=mu, max_r=mr, ref_v=refv,
                ox=[o[0] for o in obs], oy=[o[1] for o in obs], orad=rad)


def test_device_reset_draw_order_matches_oracle():
    """Seeded resets and three continued (unseeded) resets per env: the device algorithm's
    statement order reproduces the oracle's numpy reset exactly."""
    n = 64
    orc = O.SimpleEnvBatch(n)
    gens = [R.Pcg64(*R.pcg64_words(2000 + i)) for i in range(n)]
    for rnd in range(4):
        orc.reset(seeds=list(range(2000, 2000 + n)) if rnd == 0 else None)
        for i in range(n):
            d = np_reset_py(gens[i])
            k = len(d["ox"])
            assert orc.n_obs[i] == k
            np.testing.assert_array_equal(orc.position[i], d["position"])
            np.testing.assert_array_equal(orc.path_end[i], d["path_end"])
            np.testing.assert_array_equal(orc.target[i], d["target"])
            np.testing.assert_array_equal(orc.velocity[i], d["velocity"])
            assert (orc.max_action[i, 0], orc.max_action[i, 2], orc.ref_v[i]) == (d["max_u"], d["max_r"], d["ref_v"])
            np.testing.assert_array_equal(orc.ox[i, :k], d["ox"])
            np.testing.assert_array_equal(orc.oy[i, :k], d["oy"])
            np.testing.assert_array_equal(orc.orad[i, :k], d["orad"])


@pytest.mark.parametrize("seed", [0, 2000, 4003])
def test_mt19937_uniform_matches_numpy_random(seed):
    """The legacy envs' np.random.seed + np.random.uniform stream (usv_asmc_env.py:258-279),
    across several MT19937 twists."""
    rs = np.random.RandomState(seed)
    m = R.Mt19937(seed)
    for k in range(2000):
        lo, hi = [(-2.5, 2.5), (-np.pi, np.pi), (15, 30), (0.4, 1.4)][k % 4]
        assert rs.uniform(lo, hi) == m.uniform(lo, hi), k
