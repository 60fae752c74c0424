"""Per-wave timeline of the fused wave kernel (kind 1) from the diagnostic build's stamps.

    bash tools/build_diag.sh STAMPS   (-> diagbuild/stamps.so)
    USV_LIB_PATH=diagbuild/stamps.so python tools/wave_timeline.py [--envs 65536] [--variant 16,7,1]

Stamps (s_memrealtime, 100 MHz, per wave): 0 start, 1 dynamics done, 2 after the block barrier,
3 scan done, 5 first pair done (block queue), 6 end; slot 4 = pairs scanned (block queue); slot 7 =
HW_ID | XCC_ID << 32.  Diagnostic only.
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


def pct(v):
    return np.percentile(v, [0, 10, 50, 90, 99, 100]).round(2).tolist()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--variant", default="16,7,1")
    ap.add_argument("--warm", type=int, default=100)
    ap.add_argument("--env-id", default="usv-simple")
    ap.add_argument("--precision", default="f32")
    args = ap.parse_args()
    import gym_usv_amd
    lib = gym_usv_amd.load_library()
    lib.usv_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    env = gym_usv_amd.make_vec(args.env_id, args.envs, seed=1, kernel_variant=args.variant, copy=False,
                               precision=args.precision)
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
    epb = int(args.variant.split(",")[0])
    nw = (args.envs + epb - 1) // epb * 4
    buf = np.zeros(32768 * 8, dtype=np.uint64)
    assert lib.usv_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) == 0
    v = args.variant.split(",")
    if len(v) > 2 and v[2] == "3":
        nw = (args.envs + epb - 1) // epb          # one-wave blocks
    if len(v) > 2 and v[2] in ("4", "5"):
        nw = (args.envs + epb - 1) // epb * (8 if epb == 64 else 16)   # block-queue blocks
    raw = buf.reshape(32768, 8)[:nw].copy()
    raw[raw[:, 2] == 0, 2] = raw[raw[:, 2] == 0, 1]   # scan kernels: no barrier stamp
    st = raw[:, [0, 1, 2, 3, 6]].astype(np.int64)
    t0 = st[:, 0].min()
    st = (st - t0) / 100.0   # us
    hw = raw[:, 7] & 0xFFFFFFFF
    xcc = (raw[:, 7] >> 32) & 0xF
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    sid = ((xcc * 8 + se) * 16 + cu) * 4 + simd
    out = {"envs": args.envs, "variant": args.variant, "waves": int(nw),
           "event_us": round(e0.elapsed_time(e1) * 1e3, 2),
           "span_us": float(st[:, 4].max()),
           "start_us": pct(st[:, 0]), "end_us": pct(st[:, 4]),
           "dyn_us": pct(st[:, 1] - st[:, 0]), "barrier_us": pct(st[:, 2] - st[:, 1]),
           "scan_us": pct(st[:, 3] - st[:, 2]), "epi_us": pct(st[:, 4] - st[:, 3]),
           "life_us": pct(st[:, 4] - st[:, 0]),
           "distinct_simds": int(len(np.unique(sid)))}
    # first-round waves (start within 1 us of t0) vs later ones
    first = st[:, 0] < 1.0
    out["first_round_waves"] = int(first.sum())
    for nm, m in (("first", first), ("later", ~first)):
        if m.any():
            out[nm + "_dyn_us"] = round(float((st[m, 1] - st[m, 0]).mean()), 3)
            out[nm + "_life_us"] = round(float((st[m, 4] - st[m, 0]).mean()), 3)
    ts = np.linspace(0, st[:, 4].max(), 16)
    out["alive_waves_over_time"] = [int(((st[:, 0] <= t) & (st[:, 4] > t)).sum()) for t in ts]
    out["in_dyn_over_time"] = [int(((st[:, 0] <= t) & (st[:, 1] > t)).sum()) for t in ts]
    out["in_scan_over_time"] = [int(((st[:, 2] <= t) & (st[:, 3] > t)).sum()) for t in ts]
    _, per = np.unique(sid, return_counts=True)
    out["waves_per_simd"] = pct(per)
    out["end_us_by_xcc"] = {int(x): [round(float(st[xcc == x, 4].mean()), 2), round(float(st[xcc == x, 4].max()), 2)]
                            for x in np.unique(xcc)}
    out["scan_us_by_xcc"] = {int(x): round(float((st[xcc == x, 3] - st[xcc == x, 2]).mean()), 2) for x in np.unique(xcc)}
    wpb = (8 if epb == 64 else 16) if (len(v) > 2 and v[2] in ("4", "5")) else (1 if (len(v) > 2 and v[2] == "3") else 4)
    blk = st[: (nw // wpb) * wpb, 4].reshape(-1, wpb)
    out["block_end_spread_us"] = pct(blk.max(1) - blk.min(1))
    out["block_end_us"] = pct(blk.max(1))
    # co-residency: the blocks that ran on each CU, their start / end, and which one is younger
    if len(v) > 2 and v[2] in ("4", "5"):
        blk_id = np.arange(nw) // wpb
        cu_id = (xcc * 8 + se) * 16 + cu
        per_cu = {}
        for b in np.unique(blk_id[: (nw // wpb) * wpb]):
            m = blk_id == b
            per_cu.setdefault(int(cu_id[m][0]), []).append((float(st[m, 0].min()), float(st[m, 4].max()), int(b)))
        pairs = [sorted(x) for x in per_cu.values() if len(x) == 2]
        # dispatch: is block b on XCD b % 8, and when does it start (by b % 8, by b // 8)
        nb = nw // wpb
        bx = np.array([int(xcc[b * wpb]) for b in range(nb)])
        bs = np.array([float(st[b * wpb:(b + 1) * wpb, 0].min()) for b in range(nb)])
        out["xcc_eq_block_mod8"] = round(float(np.mean(bx == np.arange(nb) % 8)), 3)
        out["block_start_by_mod8"] = {int(x): round(float(bs[np.arange(nb) % 8 == x].mean()), 2) for x in range(8)}
        grp = np.arange(nb) // 8
        out["block_start_by_group_deciles"] = pct([bs[grp == q].mean() for q in np.unique(grp)])
        out["cus"] = len(per_cu)
        out["blocks_per_cu"] = pct([len(x) for x in per_cu.values()])
        if pairs:
            older_end = np.array([p[0][1] for p in pairs])
            younger_end = np.array([p[1][1] for p in pairs])
            out["older_block_start_end_us"] = [round(float(np.mean([p[0][0] for p in pairs])), 2), pct(older_end)]
            out["younger_block_start_end_us"] = [round(float(np.mean([p[1][0] for p in pairs])), 2), pct(younger_end)]
            out["younger_has_larger_block_id"] = round(float(np.mean([p[1][2] > p[0][2] for p in pairs])), 3)
            out["younger_id_ge_half_grid"] = round(float(np.mean([p[1][2] >= nw // wpb // 2 for p in pairs])), 3)
            out["older_ends_first"] = round(float(np.mean(older_end <= younger_end)), 3)
        # per CU: first wave start, last wave end; which CUs set the launch's end
        cus = sorted(per_cu)
        cs = np.array([min(x[0] for x in per_cu[c]) for c in cus])
        ce = np.array([max(x[1] for x in per_cu[c]) for c in cus])
        out["cu_start_us"], out["cu_end_us"], out["cu_busy_us"] = pct(cs), pct(ce), pct(ce - cs)
        out["corr_cu_start_end"] = round(float(np.corrcoef(cs, ce)[0, 1]), 3)
        cx = np.array(cus) // 128
        out["cu_end_by_xcc"] = {int(x): [round(float(ce[cx == x].mean()), 2), round(float(ce[cx == x].max()), 2)]
                                for x in np.unique(cx)}
        out["cu_start_by_xcc"] = {int(x): round(float(cs[cx == x].mean()), 2) for x in np.unique(cx)}
        out["cu_busy_by_xcc"] = {int(x): round(float((ce - cs)[cx == x].mean()), 2) for x in np.unique(cx)}
        oe = np.array([min(x[1] for x in per_cu[c]) - min(x[0] for x in per_cu[c]) for c in cus])
        out["older_busy_by_xcc"] = {int(x): round(float(oe[cx == x].mean()), 2) for x in np.unique(cx)}
        cse = np.array(cus) // 16
        out["cu_end_by_se_mean"] = pct([ce[cse == q].mean() for q in np.unique(cse)])
        slow = np.argsort(-ce)[:8]
        out["slowest_cus"] = [[int(cus[i]), round(float(cs[i]), 2),
                               [round(x[1] - x[0], 2) for x in sorted(per_cu[cus[i]])],
                               round(float(ce[i]), 2)] for i in slow]
        pairs_w = (raw[:, 4] & 0xFFFF).astype(np.int64)
        wsum_w = (raw[:, 4] >> 16).astype(np.int64)      # window sizes of the wave's pairs (work)
        out["pairs_per_wave"] = pct(pairs_w)
        # is the CU-to-CU spread work?  per CU: the window sizes its waves scanned against its busy time
        cw = np.array([wsum_w[np.isin(blk_id, [x[2] for x in per_cu[c]])].sum() for c in cus], dtype=np.float64)
        if cw.std() > 0:
            busy = ce - cs
            out["cu_work_windows"] = pct(cw)
            out["corr_cu_work_busy"] = round(float(np.corrcoef(cw, busy)[0, 1]), 3)
            out["corr_cu_work_end"] = round(float(np.corrcoef(cw, ce)[0, 1]), 3)
            slope = np.polyfit(cw, busy, 1)
            out["cu_busy_us_per_1000_windows"] = round(float(slope[0] * 1000), 3)
            resid = busy - np.polyval(slope, cw)
            out["cu_busy_residual_us"] = pct(resid)
            bw = np.array([wsum_w[blk_id == b].sum() for b in range(nb)], dtype=np.float64)
            be = np.array([float(st[blk_id == b, 4].max() - st[blk_id == b, 0].min()) for b in range(nb)])
            out["corr_block_work_busy"] = round(float(np.corrcoef(bw, be)[0, 1]), 3)
        # per role (older / younger block of a CU): phase-1 end (stamp 1), barrier exit (2), end (6),
        # pairs scanned per wave
        role = np.zeros(nw, np.int64)
        for c in cus:
            bl = sorted(per_cu[c])
            if len(bl) == 2:
                role[blk_id == bl[1][2]] = 1
        for nm, r in (("older", 0), ("younger", 1)):
            m = role == r
            fp = (raw[m, 5].astype(np.int64) - int(t0)) / 100.0       # stamp 5: first pair done
            out[nm + "_roles"] = {"start": pct(st[m, 0]), "dyn_end": pct(st[m, 1]), "barrier_exit": pct(st[m, 2]),
                                  "first_pair_end": pct(fp),
                                  "end": pct(st[m, 4]), "pairs": pct(pairs_w[m]),
                                  "pairs_total_per_block": float(pairs_w[m].sum() / max(1, m.sum() // wpb))}
        # pairs finished by both blocks of a CU over time is not stamped; the wave ends are
        ends = np.sort(st[:, 4])
        out["wave_end_deciles_us"] = np.percentile(ends, np.arange(0, 101, 10)).round(2).tolist()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
