"""Summarise a tools/pmc_split.sh output directory: per-kernel average duration and per-wave /
per-env instruction counts.  python tools/pmc_report.py gpurun_out/pmc_<tag> [--envs 65536]"""
import argparse
import collections
import csv
import glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--envs", type=int, default=65536)
    a = ap.parse_args()
    for f in glob.glob(f"{a.dir}/kt/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "usv" in r["Name"]:
                print(f"{r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1000:8.2f} us")
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{a.dir}/p*/**/*counter_collection.csv", recursive=True)):
        for row in csv.DictReader(open(f)):
            if "usv" in row["Kernel_Name"] and "reset_kernel" not in row["Kernel_Name"]:
                acc[row["Kernel_Name"][:48]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for kname, d in acc.items():
        m = {k: sum(v[5:] or v) / len(v[5:] or v) for k, v in d.items()}
        per_env = {k.replace("SQ_", ""): round(v / a.envs, 1) for k, v in m.items()
                   if k.startswith("SQ_INSTS") or k.startswith("SQ_ACTIVE") or k.startswith("SQ_WAIT")}
        print(kname, "waves", int(m.get("SQ_WAVES", 0)), "per env:", per_env)


if __name__ == "__main__":
    main()
