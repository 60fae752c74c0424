"""Per-wave section cycles of the wave-per-env scan (kinds 1 / 2) from the diagnostic build (-DUSV_DIAG_PROF).

    bash tools/build_diag.sh PROF   (-> diagbuild/prof.so)
    USV_LIB_PATH=diagbuild/prof.so python tools/scan_prof.py [--envs 65536] [--precision f64] [--variant 32,7,2]

Slots (shader-clock cycles per wave, s_memtime): 0 prologue (start -> barrier), 4 iteration top
(priority, vm_wait for the rows), 1 next rows' DMA issue, 2 lidar, 3 emit (sensor stores, final obs),
5 epilogue (reward / flags / autoresets); 7 = iterations (count).  Diagnostic only.
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

NAMES = {0: "prologue", 4: "iter_top", 1: "dma_issue", 2: "lidar", 3: "emit", 5: "epilogue"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--warm", type=int, default=200)
    ap.add_argument("--precision", default="f64")
    ap.add_argument("--variant", default="32,7,2")
    ap.add_argument("--env-id", default="usv-simple")
    args = ap.parse_args()
    import gym_usv_amd
    lib = gym_usv_amd.load_library()
    lib.usv_diag_prof.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    env = gym_usv_amd.make_vec(args.env_id, args.envs, seed=1, precision=args.precision,
                               kernel_variant=args.variant, copy=False)
    env.reset(seed=1)
    dt = torch.float64 if args.precision == "f64" else torch.float32
    g = torch.Generator(device="cuda").manual_seed(0)
    lo = torch.tensor([0.2, -1.0], device="cuda", dtype=dt)
    span = torch.tensor([0.8, 2.0], device="cuda", dtype=dt)
    for _ in range(args.warm):
        env.step(torch.rand(args.envs, 2, device="cuda", generator=g, dtype=dt) * span + lo)
    a = torch.rand(args.envs, 2, device="cuda", generator=g, dtype=dt) * span + lo
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    env.step(a)
    e1.record()
    torch.cuda.synchronize()
    epb = int(args.variant.split(",")[0])           # envs per 4-wave block (kinds 1, 2)
    nw = min(16384, (args.envs + epb - 1) // epb * 4)
    buf = np.zeros(16384 * 8, dtype=np.uint64)
    assert lib.usv_diag_prof(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) == 0
    q = buf.reshape(16384, 8)[:nw].astype(np.float64)
    iters = q[:, 7]
    life = sum(q[:, k] for k in NAMES)
    out = {"event_us": round(e0.elapsed_time(e1) * 1e3, 2), "waves": nw,
           "iters_per_wave": float(iters.mean()),
           "life_cycles_mean": float(life.mean()), "life_cycles_p90": float(np.percentile(life, 90))}
    for k, nm in NAMES.items():
        out[nm] = {"mean_per_wave": round(float(q[:, k].mean()), 1),
                   "per_iter": round(float(q[:, k].sum() / max(1.0, iters.sum())), 1),
                   "share": round(float(q[:, k].sum() / life.sum()), 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
