#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counters (one or more output directories), for quick
investigations: tools/pmc_kernels.py <dir> [<dir> ...] [--match SUBSTR]

Prints, per kernel name (and VGPR count), the dispatch count and the average of every collected
counter per dispatch, plus a few derived ratios when their inputs are present:
  lds_util   = SQ_LDS_IDX_ACTIVE / SQ_BUSY_CU_CYCLES    (LDS-array busy share of the busy CU cycles)
  valu_share = SQ_ACTIVE_INST_VALU / SQ_BUSY_CU_CYCLES  (per CU: 4 SIMDs, so up to ~4)
  wait_share = SQ_WAIT_ANY / SQ_WAVE_CYCLES
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(argv):
    match = None
    if "--match" in argv:
        i = argv.index("--match")
        match = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    cnt = defaultdict(lambda: defaultdict(list))
    for d in argv:
        for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    name = r["Kernel_Name"]
                    if match and match not in name:
                        continue
                    cnt[(name[:70], r.get("VGPR_Count", "?"))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (name, vg), c in sorted(cnt.items()):
        n = max(len(v) for v in c.values())
        avg = {k: sum(v) / len(v) for k, v in c.items()}
        print(f"{name}  vgpr={vg}  dispatches={n}")
        for k in sorted(avg):
            print(f"    {k:32s} {avg[k]:16.1f}")
        def ratio(a, b, label):
            if a in avg and b in avg and avg[b]:
                print(f"    {label:32s} {avg[a] / avg[b]:16.4f}")
        ratio("SQ_LDS_IDX_ACTIVE", "SQ_BUSY_CU_CYCLES", "lds_util")
        ratio("SQ_ACTIVE_INST_VALU", "SQ_BUSY_CU_CYCLES", "valu_share (per CU)")
        ratio("SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "wait_share")
        ratio("SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES", "wait_inst_lds_share")
        ratio("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "bank_conflict_share")


if __name__ == "__main__":
    main(sys.argv[1:])
