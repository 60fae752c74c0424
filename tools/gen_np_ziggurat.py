"""Extract NumPy's standard-normal ziggurat tables (ki_double, wi_double, fi_double) from the
libnpyrandom.a that ships with the installed numpy, and write them as C++ constants for the
device-side NumPy-exact reset (gym-usv_amd/csrc/np_ziggurat.inc).

The reference draws its reset with numpy.random.Generator(PCG64).normal (simple_env.py:234-237),
whose algorithm is NumPy's random_standard_normal ziggurat over these 256-entry tables.  The
tables are data in numpy's static library; this script reads them by symbol from the object's
.rodata and then checks them by replaying numpy's own normal draws (tests/test_np_rng.py does
the same on every CPU test run).

    python tools/gen_np_ziggurat.py
"""
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(os.path.dirname(np.__file__), "random", "lib", "libnpyrandom.a")
OBJ = "src_distributions_distributions.c.o"


def rodata_tables():
    with tempfile.TemporaryDirectory() as d:
        subprocess.check_call(["ar", "x", LIB, OBJ], cwd=d)
        path = os.path.join(d, OBJ)
        syms = {}
        for line in subprocess.check_output(["nm", path], text=True).splitlines():
            p = line.split()
            if len(p) == 3 and p[2] in ("ki_double", "wi_double", "fi_double"):
                syms[p[2]] = int(p[0], 16)
        sec = subprocess.check_output(["readelf", "-S", "-W", path], text=True)
        off = None
        for line in sec.splitlines():
            if " .rodata " in line + " ":
                f = line.split()
                i = f.index(".rodata")
                off = int(f[i + 3], 16)       # Address, Off columns follow the type
                break
        data = open(path, "rb").read()
    out = {}
    for name, fmt in (("ki_double", "<256Q"), ("wi_double", "<256d"), ("fi_double", "<256d")):
        out[name] = struct.unpack_from(fmt, data, off + syms[name])
    return out


def main():
    t = rodata_tables()
    assert t["ki_double"][0] != 0 and 0 < t["wi_double"][1] < 1e-14 and t["fi_double"][0] == 1.0, "bad extraction"
    dst = os.path.join(ROOT, "gym-usv_amd", "csrc", "np_ziggurat.inc")
    with open(dst, "w") as f:
        f.write("// NumPy's standard-normal ziggurat tables (random_standard_normal), extracted from the\n"
                f"// installed numpy {np.__version__} by tools/gen_np_ziggurat.py.  Data, not code.\n")
        f.write("__constant__ unsigned long long kNpZigKi[256] = {\n")
        f.write(",\n".join("  0x%016xULL" % v for v in t["ki_double"]) + "};\n")
        for name, key in (("kNpZigWi", "wi_double"), ("kNpZigFi", "fi_double")):
            f.write(f"__constant__ double {name}[256] = {{\n")
            f.write(",\n".join("  %s" % float.hex(v) for v in t[key]) + "};\n")
    print("wrote", dst)


if __name__ == "__main__":
    sys.exit(main())
