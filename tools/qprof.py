"""Per-wave section cycles of the block-queue step from the diagnostic build (-DUSV_DIAG_QPROF).

    bash tools/build_diag.sh QPROF   (-> diagbuild/qprof.so)
    USV_LIB_PATH=diagbuild/qprof.so python tools/qprof.py [--envs 65536]

Slots (shader-clock cycles per wave, summed over the wave's pairs): 10 phase 1 (start -> barrier),
0 barrier wait, 1 iteration top (ticket, DMA issue, record reads), 2 lidar setup + scan, 3 passes,
4 slot readback, 5 stores / reward / done path, 6 vm_wait, 7 resets, 11 loop exits;
8 pairs, 9 passes (counts).  Diagnostic only.
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

NAMES = {10: "phase1", 0: "barrier", 1: "iter_top", 2: "lidar_setup", 3: "passes", 4: "readback",
         5: "stores", 6: "vm_wait", 7: "resets", 11: "exits"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--warm", type=int, default=200)
    ap.add_argument("--env-id", default="usv-simple")
    ap.add_argument("--variant", default=None, help="kernel variant epb,lid,kind (e.g. 128,263,5: row spans on)")
    args = ap.parse_args()
    import gym_usv_amd
    lib = gym_usv_amd.load_library()
    lib.usv_diag_qprof.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    env = gym_usv_amd.make_vec(args.env_id, args.envs, seed=1, kernel_variant=args.variant)
    env.reset(seed=1)
    g = torch.Generator(device="cuda").manual_seed(0)
    lo, span = torch.tensor([0.2, -1.0], device="cuda"), torch.tensor([0.8, 2.0], device="cuda")
    for _ in range(args.warm):
        env.step(torch.rand(args.envs, 2, device="cuda", generator=g) * span + lo)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a = torch.rand(args.envs, 2, device="cuda", generator=g) * span + lo
    torch.cuda.synchronize()
    e0.record()
    env.step(a)
    e1.record()
    torch.cuda.synchronize()
    nw = args.envs // 128 * 16
    buf = np.zeros(16384 * 12, dtype=np.uint32)
    assert lib.usv_diag_qprof(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) == 0
    q = buf.reshape(16384, 12)[:nw].astype(np.float64)
    pairs, passes = q[:, 8], q[:, 9]
    life = sum(q[:, k] for k in NAMES)
    out = {"env_id": args.env_id, "event_us": round(e0.elapsed_time(e1) * 1e3, 2), "waves": nw,
           "pairs_per_wave": [float(pairs.mean()), float(pairs.min()), float(pairs.max())],
           "passes_per_pair": float(passes.sum() / pairs.sum()),
           "life_cycles_mean": float(life.mean()), "life_cycles_p90": float(np.percentile(life, 90))}
    for k, nm in NAMES.items():
        out[nm] = {"mean_per_wave": round(float(q[:, k].mean()), 1),
                   "per_pair": round(float(q[:, k].sum() / pairs.sum()), 1),
                   "share": round(float(q[:, k].sum() / life.sum()), 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
