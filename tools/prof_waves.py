"""Per-wave cycle breakdown of the wave-per-env scan (diagnostic build, -DUSV_DIAG_PROF).

    hipcc ... -DUSV_DIAG_PROF -o /tmp/libprof.so gym-usv_amd/csrc/usv_kernels.hip
    USV_LIB_PATH=/tmp/libprof.so python tools/prof_waves.py [--envs 65536] [--variant 64,7,1]

Slots (shader-clock cycles per wave, s_memtime): 0 prologue + dynamics (+ barrier),
1 DMA wait at the top of each scan iteration, 2 lidar, 3 emit (obs rows, flags),
4 loop bookkeeping, 5 epilogue (rewards, resets); slot 7 counts scan iterations.
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
    ap.add_argument("--variant", default="64,7,1")
    ap.add_argument("--env-id", default="usv-simple")
    ap.add_argument("--warm", type=int, default=200)
    args = ap.parse_args()
    os.environ["USV_STEP_VARIANT"] = args.variant
    import gym_usv_amd
    lib = gym_usv_amd.load_library()
    lib.usv_diag_prof.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    env = gym_usv_amd.make_vec(args.env_id, args.envs, seed=1)
    env.reset(seed=1)
    g = torch.Generator(device="cuda").manual_seed(0)
    lo, span = torch.tensor([0.2, -1.0], device="cuda"), torch.tensor([0.8, 2.0], device="cuda")
    for _ in range(args.warm):
        env.step(torch.rand(args.envs, 2, device="cuda", generator=g) * span + lo)
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    a = torch.rand(args.envs, 2, device="cuda", generator=g) * span + lo
    t0.record()
    env.step(a)
    t1.record()
    torch.cuda.synchronize()
    buf = np.zeros(16384 * 8, dtype=np.uint64)
    assert lib.usv_diag_prof(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) == 0
    epb = int(args.variant.split(",")[0])
    waves = (args.envs + epb - 1) // epb * 4
    p = buf.reshape(16384, 8)[:waves].astype(np.float64)
    names = ["prologue+dyn", "dma_wait", "lidar", "emit", "loop", "epilogue"]
    tot = p[:, :6].sum(1)
    out = {"variant": args.variant, "envs": args.envs, "waves": waves,
           "kernel_us": round(t0.elapsed_time(t1) * 1e3, 2),
           "iters_per_wave": float(p[:, 7].mean()),
           "wave_cycles_mean": round(float(tot.mean())), "wave_cycles_p99": round(float(np.percentile(tot, 99))),
           "wave_cycles_max": round(float(tot.max()))}
    for i, nm in enumerate(names):
        out[nm] = {"mean": round(float(p[:, i].mean())), "share": round(float(p[:, i].sum() / tot.sum()), 3)}
    out["lidar_cycles_per_iter"] = round(float(p[:, 2].sum() / max(1, p[:, 7].sum())))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
