#!/usr/bin/env python3
"""Summarise tools/gs_phase.sh: per variant, the blend kernel's (gs_sort_blend_kernel<false>) average launch
time (kernel trace) and per-launch SQ counters, and the differences between consecutive variants (what the
removed phase cost).   tools/gs_phase.py <out-dir> [variants in order]"""
import csv
import glob
import os
import sys

KERNEL = "gs_sort_blend_kernel<false>"
SHOW = ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM",
        "SQ_INSTS_BRANCH", "SQ_INSTS_VALU_TRANS_F32", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES",
        "SQ_ACTIVE_INST_VALU", "SQ_BUSY_CU_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_WAVES"]


def load(d):
    out = {}
    kt = glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True)
    for r in csv.DictReader(open(kt[0])) if kt else []:
        if KERNEL in r["Name"]:
            out["us"] = float(r["AverageNs"]) / 1e3
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        acc = {}
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        for k, v in acc.items():
            out[k] = sum(v) / len(v)
    return out


def main():
    d = sys.argv[1]
    vs = sys.argv[2:] or sorted(os.path.basename(p) for p in glob.glob(os.path.join(d, "*")) if os.path.isdir(p))
    data = {v: load(os.path.join(d, v)) for v in vs}
    cols = ["us"] + SHOW
    print("| variant | " + " | ".join(c.replace("SQ_", "") for c in cols) + " |")
    print("|---" * (len(cols) + 1) + "|")
    for v in vs:
        print(f"| {v} | " + " | ".join(f"{data[v].get(c, float('nan')):.4g}" for c in cols) + " |")
    print()
    print("differences (previous variant minus this one: the cost of the phase it removes)")
    for a, b in zip(vs, vs[1:]):
        print(f"| {a} - {b} | " + " | ".join(f"{data[a].get(c, float('nan')) - data[b].get(c, float('nan')):.4g}"
                                              for c in cols) + " |")


if __name__ == "__main__":
    main()
