"""Phase timeline of the step kernel from the diagnostic build's per-block s_memrealtime stamps.

    hipcc ... -DUSV_DIAG_STAMPS -o /tmp/libdiag.so gym-usv_amd/csrc/usv_kernels.hip
    USV_LIB_PATH=/tmp/libdiag.so python tools/stamps.py [--envs 65536] [--variant 32,7]

Stamps (100 MHz ticks, per block): 0 start, 1 dynamics-wave phase-1 done, 2 after barrier 1,
3 wave-0 lidar loop done, 4 wave-0 resets done, 5 after barrier 2, 6 end.  Diagnostic only.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-usv_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--variant", default="32,7")
    ap.add_argument("--warm", type=int, default=50)
    args = ap.parse_args()
    os.environ["USV_STEP_VARIANT"] = args.variant
    import gym_usv_amd
    lib = gym_usv_amd.load_library()
    lib.usv_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    env = gym_usv_amd.make_vec("usv-simple", args.envs, seed=1)
    env.reset(seed=1)
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(args.warm):
        env.step(torch.rand(args.envs, 2, device="cuda", generator=g))
    a = torch.rand(args.envs, 2, device="cuda", generator=g)
    torch.cuda.synchronize()
    env.step(a)
    torch.cuda.synchronize()
    epb = int(args.variant.split(",")[0])
    nb = (args.envs + epb - 1) // epb
    buf = np.zeros(32768 * 8, dtype=np.uint64)
    assert lib.usv_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) == 0
    st = buf.reshape(32768, 8)[:nb, :7].astype(np.int64)
    t0 = st[:, 0].min()
    st = (st - t0) * 10 / 1000.0   # us
    ph = {"phase1 (dyn wave)": st[:, 1] - st[:, 0], "barrier1 wait": st[:, 2] - st[:, 1],
          "lidar loop (wave0)": st[:, 3] - st[:, 2], "resets (wave0)": st[:, 4] - st[:, 3],
          "barrier2 wait": st[:, 5] - st[:, 4], "phase3": st[:, 6] - st[:, 5],
          "block total": st[:, 6] - st[:, 0]}
    out = {"envs": args.envs, "variant": args.variant, "blocks": nb,
           "kernel_span_us": float(st[:, 6].max()),
           "block_start_us_pcts": np.percentile(st[:, 0], [0, 25, 50, 75, 100]).round(2).tolist(),
           "block_end_us_pcts": np.percentile(st[:, 6], [0, 25, 50, 75, 100]).round(2).tolist()}
    for k, v in ph.items():
        out[k] = {"mean": round(float(v.mean()), 3), "p50": round(float(np.median(v)), 3),
                  "p99": round(float(np.percentile(v, 99)), 3), "max": round(float(v.max()), 3)}
    # concurrency: blocks alive over time
    ts = np.linspace(0, st[:, 6].max(), 12)
    out["alive_blocks_over_time"] = [int(((st[:, 0] <= t) & (st[:, 6] > t)).sum()) for t in ts]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
