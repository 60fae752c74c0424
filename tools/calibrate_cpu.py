"""CPU-baseline calibration — build container only, needs /root/reference.

Times, per core (one single-threaded process each, same protocol as bench.py's cpu_baseline leg:
1 env, seeded random actions, TimeLimit + reset), the reference's own env step imported read-only
through tests/golden/refharness.py, and the oracle restatement (oracle/usv_oracle.py) that bench.py
times on the GPU box, where the reference does not exist.  Writes profiles/cpu_calibration.json:
per env id, both per-core rates and ratio = oracle / reference.  bench.py reports the ratio next to
its measured cpu_baseline so the port's number can be read in reference units.

    python tools/calibrate_cpu.py [--seconds 10] [--procs 4]
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIMITS = {"usv-simple": 500, "usv-asmc-simple": 1000}


def _ref_worker(args):
    env_id, seconds, seed = args
    os.environ["OMP_NUM_THREADS"] = "1"
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import refharness
    refharness.load_reference()
    import gym_usv.envs as E
    cls = {"usv-simple": E.UsvSimpleEnv, "usv-asmc-simple": E.UsvSimpleASMCEnv}[env_id]
    env = cls(render_mode=None)
    env.reset(seed=seed)
    rng = np.random.default_rng(seed)
    n, el, t0 = 0, 0, time.perf_counter()
    while True:
        _, _, te, tr, _ = env.step(rng.uniform([0.2, -1], [1, 1]).astype(np.float32))
        el += 1
        if te or tr or el >= LIMITS[env_id]:
            env.reset()
            el = 0
        n += 1
        if n % 16 == 0 and time.perf_counter() - t0 >= seconds:
            return n, time.perf_counter() - t0


def _port_worker(args):
    sys.path.insert(0, ROOT)
    import bench
    return bench._cpu_worker(args)


def rate(worker, env_id, seconds, procs):
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.map(worker, [(env_id, seconds, 1000 + i) for i in range(procs)])
    return sum(n / t for n, t in res) / procs


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--procs", type=int, default=4)
    a = ap.parse_args()
    out = {"host": cpu_model(), "procs": a.procs, "seconds": a.seconds,
           "protocol": "per-core env-steps/s, 1 env per single-threaded process, random actions, "
                       "TimeLimit + reset; reference imported read-only (numba absent: pure-Python lidar)"}
    for env_id in ("usv-simple", "usv-asmc-simple"):
        ref = rate(_ref_worker, env_id, a.seconds, a.procs)
        port = rate(_port_worker, env_id, a.seconds, a.procs)
        out[env_id] = {"reference_per_core": round(ref, 1), "oracle_per_core": round(port, 1),
                       "ratio_oracle_over_reference": round(port / ref, 3)}
        print(env_id, out[env_id], flush=True)
    p = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    json.dump(out, open(p, "w"), indent=1)
    print("wrote", p)


if __name__ == "__main__":
    main()
