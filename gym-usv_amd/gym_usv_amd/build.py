"""Build libusvhip.so in-tree for gfx950 (hipcc; no JIT cache, so the .so travels with the repo).

    python -m gym_usv_amd.build        (from gym-usv_amd/, or via __graft_entry__.build())
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(PKG))
CSRC = os.path.join(os.path.dirname(PKG), "csrc")
INCLUDE = os.path.join(ROOT, "include")
ARCH = os.environ.get("USV_OFFLOAD_ARCH", "gfx950")


# The block-queue step takes its next pair's LDS ticket one pair ahead; the atomic optimizer would
# rewrite that single-lane atomicAdd into a wave reduction whose result is consumed at once, exposing
# the LDS atomic's latency every pair.
DEVICE_FLAGS = ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


def sources():
    return [os.path.join(CSRC, "usv_kernels.hip")]


def deps():
    """Every file the build reads: the sources, everything under csrc/ they include (.hpp, .h, .inc)
    and the public header."""
    return sources() + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h", ".inc"))] + \
        [os.path.join(INCLUDE, "usv_hip.h")]


# product library, and the debug build whose hand-counted vmcnt waits are all vmcnt(0)
VARIANTS = {"product": ("libusvhip.so", []), "safe": ("libusvhip_safe.so", ["-DUSV_SAFE_VMCNT"])}


def _stale(out):
    return not os.path.exists(out) or any(os.path.getmtime(d) > os.path.getmtime(out) for d in deps())


def _cmd(variant):
    name, defs = VARIANTS[variant]
    out = os.path.join(PKG, name)
    return out, [hipcc(), "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared", "-Wall",
                 *DEVICE_FLAGS, *defs, f"-I{INCLUDE}", "-o", out + ".tmp"] + sources()


def build_library(force=False, verbose=True, variant="product"):
    out, cmd = _cmd(variant)
    if not force and not _stale(out):
        return out
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_all(force=False, verbose=True):
    """Every variant, compiled concurrently (one hipcc process each).  Every job is waited for; the
    variants that compiled are installed even if another failed (the product library does not depend
    on the vmcnt(0) debug build), failed jobs leave no temporary output, and the first failure is
    raised at the end."""
    jobs = []
    for v in VARIANTS:
        out, cmd = _cmd(v)
        if force or _stale(out):
            if verbose:
                print(" ".join(cmd), flush=True)
            jobs.append((out, subprocess.Popen(cmd)))
    failed = []
    for out, p in jobs:
        if p.wait() == 0:
            os.replace(out + ".tmp", out)
        else:
            failed.append((p.returncode, out))
            if os.path.exists(out + ".tmp"):
                os.remove(out + ".tmp")
    if failed:
        rc, out = failed[0]
        raise subprocess.CalledProcessError(rc, "hipcc " + out)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
