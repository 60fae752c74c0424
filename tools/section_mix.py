"""Static instruction mix of the block-queue step kernel per loop section (no GPU).

    python tools/section_mix.py [--kernel REGEX]

Compiles csrc/usv_kernels.hip to gfx950 assembly with -DUSV_DIAG -DUSV_DIAG_SECTIONS (QMARK(i) becomes
an assembly comment) and counts, between consecutive markers in the listing's layout order, the
instructions by class: VALU (v_*, lane moves counted apart), SALU (s_* ALU, exec-mask and compare
ops), waits / nops / branches, LDS (ds_*), VMEM (global_* / buffer_*), SMEM.  Sections of
step_q_body: 10 = phase 1 (dynamics, first DMAs) up to the barrier; 0 -> 1 = pair-loop top (ticket,
next pair's DMA, span set-up); 1 -> 2 = lidar set-up (per-obstacle records, windows, prefix scan);
2 -> 3 = the passes (marks, max-scan, pair tests, ds_min); 3 -> 4 = slot read-back; 4 -> 5 =
stores, the next pair's record, done handling; 5 -> 6 = the vmcnt wait; 11 / 7 = same-step resets.
Static counts: the pass code runs 1.65 times per pair at C3 and branches run once or not at all,
so this attributes the pipes' work to sections, it does not replace the SQ counters.
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def classify(op):
    if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return "lane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_sleep", "s_setprio")):
        return "wait_nop"
    if op.startswith(("s_branch", "s_cbranch", "s_endpgm")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default=r"_ZN3usv13step_q_kernelILi0ELb1ELb0ELb1ELb0ELb0EEEv")
    ap.add_argument("--asm", default="/tmp/usv_sections.s")
    args = ap.parse_args()
    src = os.path.join(ROOT, "gym-usv_amd", "csrc", "usv_kernels.hip")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "--cuda-device-only", "-S",
                    "-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "-I" + os.path.join(ROOT, "include"),
                    "-DUSV_DIAG", "-DUSV_DIAG_SECTIONS", *os.environ.get("XDEFS", "").split(), "-o", args.asm, src], check=True,
                   stderr=subprocess.DEVNULL)
    t = open(args.asm).read()
    names = [n for n in re.findall(r"^(_Z\w+):", t, re.M) if re.match(args.kernel, n)]
    if not names:
        sys.exit(f"no kernel matches {args.kernel}")
    name = names[0]
    i = t.find("\n" + name + ":")
    body = t[i:t.find(".Lfunc_end", i)].split("\n")
    sec = "entry"
    mix = collections.OrderedDict()
    for line in body:
        m = re.search(r";@@QMARK (\d+)", line)
        if m:
            sec = m.group(1)
            continue
        if not line.startswith("\t") or line.strip().startswith((".", ";")):
            continue
        op = line.strip().split()[0]
        mix.setdefault(sec, collections.Counter())[classify(op)] += 1
    out = {"kernel": name, "sections": {k: dict(v) for k, v in mix.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
