"""Summarise tools/exp_write_ab.sh output directories (gpurun_out/writeab_<envs>/) into one JSON:
per library build, WRITE_SIZE / FETCH_SIZE KiB per step-kernel launch and the event-timed step of
each round.   python tools/collect_writeab.py gpurun_out/writeab_65536 gpurun_out/writeab_524288 > out.json"""
import csv
import glob
import json
import os
import re
import sys


def kib(d, c):
    v = [float(r["Counter_Value"]) for f in glob.glob(f"{d}/{c}/**/*counter_collection.csv", recursive=True)
         for r in csv.DictReader(open(f)) if re.search(r"usv::step\w*_kernel", r["Kernel_Name"])]
    v = v[5:] or v
    return round(sum(v) / len(v), 1) if v else None


out = {}
for d in sys.argv[1:]:
    envs = int(d.rstrip("/").rsplit("_", 1)[1])
    res = {}
    for lib in sorted(x for x in os.listdir(d) if os.path.isdir(os.path.join(d, x))):
        rounds = []
        for f in sorted(glob.glob(os.path.join(d, f"{lib}.*.json"))):
            try:
                b = json.loads(open(f).read().strip().splitlines()[-1])
                rounds.append({"step_us": round(b["roofline"]["kernel_ms"] * 1e3, 2), "frac": b["roofline"]["frac"]})
            except Exception:
                pass
        res[lib] = {"write_kib_per_launch": kib(os.path.join(d, lib), "write"),
                    "fetch_kib_per_launch": kib(os.path.join(d, lib), "fetch"), "rounds": rounds}
    out[str(envs)] = res
print(json.dumps(out, indent=1))
