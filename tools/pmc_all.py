"""Mean per dispatch (skipping the first 5) of every counter collected under a directory of
rocprofv3 --pmc runs, for the usv step kernels, plus per-env values.

    python tools/pmc_all.py gpurun_out/diag_<tag> [--envs 65536]
"""
import argparse
import collections
import csv
import glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--envs", type=int, default=65536)
    a = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{a.dir}/**/*counter_collection.csv", recursive=True)):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if "usv::" in k and "reset_kernel" not in k:
                acc[k.split("(")[0]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for kname, d in acc.items():
        print(kname)
        for c, v in sorted(d.items()):
            v = v[5:] or v
            m = sum(v) / len(v)
            print(f"  {c:26s} {m:16.1f}   per env {m / a.envs:10.3f}")


if __name__ == "__main__":
    main()
