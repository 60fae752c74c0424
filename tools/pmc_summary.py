"""Summarise rocprofv3 outputs for the step kernel into profiles/<round>_summary.json and
profiles/pmc_summary.json (read by bench.py for roofline.traffic).

    python tools/pmc_summary.py --kt DIR --fetch DIR --write DIR --key usv-simple/65536/f32/window --round r01

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (TCC_EA0_RDREQ/WRREQ based, include Infinity
Cache hits).  On gfx950 FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced
read, global_load and LDS-DMA alike, while WRITE_SIZE is exact for streaming stores
(MI355X_MICROARCH.md, HBM section).  The step kernel's reads are dominated by the 16-B/lane
LDS-DMA of the obstacle rows, so the reported traffic is 2 x FETCH_SIZE + WRITE_SIZE; the raw sum
is kept alongside.
"""
import argparse
import csv
import glob
import json
import os
import re

# every step-kernel family: step_kernel, step_kernel_wave, step_q_kernel, scan_kernel (split step)
STEP_RE = re.compile(r"usv::(step\w*_kernel|scan_kernel)")


def rows(d, pattern):
    f = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    if not f:
        raise SystemExit(f"no {pattern} under {d}")
    return list(csv.DictReader(open(f[0])))


def all_rows(d, pattern):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True)):
        out += list(csv.DictReader(open(f)))
    if not out:
        raise SystemExit(f"no {pattern} under {d}")
    return out


def counter(d, name, skip=5, regex=None):
    """Per step: the sum over the step's kernels (names matching `regex`, default the step kernels) of
    each kernel's mean per dispatch of `name`, over every counter CSV under `d` (one per --pmc pass)."""
    regex = regex or STEP_RE
    per = {}
    for r in all_rows(d, "*counter_collection.csv"):
        if regex.search(r["Kernel_Name"]) and r["Counter_Name"] == name:
            per.setdefault(r["Kernel_Name"].split("(")[0], []).append(float(r["Counter_Value"]))
    if not per:
        raise SystemExit(f"no step-kernel {name} samples under {d}")
    total = 0.0
    for v in per.values():
        v = v[skip:] or v
        total += sum(v) / len(v)
    return total, min(len(v) for v in per.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kt", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--round", default="r01")
    ap.add_argument("--out", default="profiles")
    ap.add_argument("--sq", default=None, help="directory of SQ counter passes (SQ_INSTS_VALU / SALU)")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--kernels", default=None,
                    help="regex of the kernels one step launches (default: the step kernels; usv-asmc-simple "
                         "kind 6 also runs asmc_chain_kernel)")
    a = ap.parse_args()
    rx = re.compile(a.kernels) if a.kernels else STEP_RE
    stats = [r for r in rows(a.kt, "*kernel_stats.csv") if "usv::" in r["Name"]]
    step = [r for r in stats if rx.search(r["Name"])]
    fetch_kib, nf = counter(a.fetch, "FETCH_SIZE", regex=rx)
    write_kib, nw = counter(a.write, "WRITE_SIZE", regex=rx)
    summ = {
        "key": a.key,
        "kernel_stats": [{k: r[k] for k in ("Name", "Calls", "AverageNs", "MinNs", "MaxNs", "Percentage")}
                         for r in stats[:8]],
        "step_kernel": step[0]["Name"] if step else None,
        "step_kernels": [r["Name"] for r in step],
        # every kernel of one step (their average durations summed)
        "step_kernel_avg_ns": sum(float(r["AverageNs"]) for r in step) if step else None,
        "fetch_kib_per_launch": fetch_kib, "write_kib_per_launch": write_kib,
        "fetch_samples": nf, "write_samples": nw,
        "hbm_bytes_per_launch": round((2 * fetch_kib + write_kib) * 1024),
        "hbm_bytes_per_launch_raw": round((fetch_kib + write_kib) * 1024),
        "correction": "2 x FETCH_SIZE (16-B/lane reads, gfx950) + WRITE_SIZE",
    }
    if a.sq:          # wave-instruction counts per launch, for roofline.valu_frac (bench.py)
        for name in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES"):
            try:
                v, _ = counter(a.sq, name, regex=rx)
            except SystemExit:
                continue
            summ[name.lower() + "_per_launch"] = v
            summ[name.lower() + "_per_env"] = v / a.envs
    os.makedirs(a.out, exist_ok=True)
    json.dump(summ, open(os.path.join(a.out, f"{a.round}_summary.json"), "w"), indent=1)
    agg_p = os.path.join(a.out, "pmc_summary.json")
    agg = json.load(open(agg_p)) if os.path.exists(agg_p) else {}
    agg[a.key] = {"hbm_bytes_per_launch": summ["hbm_bytes_per_launch"],
                  "hbm_bytes_per_launch_raw": summ["hbm_bytes_per_launch_raw"],
                  "step_kernel_avg_ns": summ["step_kernel_avg_ns"], "round": a.round}
    for k in ("sq_insts_valu_per_launch", "sq_insts_salu_per_launch"):
        if k in summ:
            agg[a.key][k] = summ[k]
    json.dump(agg, open(agg_p, "w"), indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
