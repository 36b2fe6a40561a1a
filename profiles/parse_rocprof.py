#!/usr/bin/env python3
"""Summarise a profiles/profile.sh run (gpurun_out/prof_<tag>/) into committed files:

  profiles/<tag>_kernel_stats.csv    rocprofv3 --kernel-trace --stats summary (as produced)
  profiles/<tag>_summary.md          per-kernel average duration + HBM bytes per dispatch
  profiles/traffic_latest.json       HBM bytes per launch of pt_camera_kernel (read by bench.py)

HBM bytes per dispatch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE/WRITE_SIZE are in KiB and
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read (MI355X_MICROARCH.md §HBM).
The instrumented (counting) pt_camera_kernel<true> dispatch is told apart by its VGPR count.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _find(d, pat):
    hits = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return sorted(hits)


def _counters(d):
    rows = []
    for f in _find(d, "*counter_collection.csv"):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def main(tag, workload):
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = _find(os.path.join(base, "kt"), "*kernel_stats.csv")
    if not stats:
        raise SystemExit(f"no kernel_stats.csv under {base}/kt")
    dst = os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv")
    shutil.copy(stats[0], dst)
    with open(stats[0]) as fh:
        krows = list(csv.DictReader(fh))
    traces = _find(os.path.join(base, "kt"), "*kernel_trace.csv")
    per_vgpr = defaultdict(list)
    if traces:
        with open(traces[0]) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "")
                dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                per_vgpr[(name, r.get("VGPR_Count", "?"))].append(dur)
    by_kernel = defaultdict(lambda: defaultdict(list))  # (name, vgpr) -> counter -> values
    for sub in ("fetch", "write"):
        for r in _counters(os.path.join(base, sub)):
            key = (r["Kernel_Name"], r.get("VGPR_Count", "?"))
            by_kernel[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    lines = [f"# rocprofv3 summary — {tag}", "", f"workload: {workload}", "",
             "## kernel-trace --stats (as reported)", "",
             "| kernel | calls | avg ms | total ms | % |", "|---|---|---|---|---|"]
    for r in krows:
        lines.append(f"| {r['Name'][:90]} | {r['Calls']} | {float(r['AverageNs']) / 1e6:.4f} | "
                     f"{float(r['TotalDurationNs']) / 1e6:.3f} | {float(r['Percentage']):.2f} |")
    lines += ["", "## per dispatch kind (kernel trace, split by VGPR count)", "",
              "| kernel | VGPRs | dispatches | avg ms |", "|---|---|---|---|"]
    for (name, vg), durs in sorted(per_vgpr.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| {name[:90]} | {vg} | {len(durs)} | {sum(durs) / len(durs) / 1e6:.4f} |")
    lines += ["", "## HBM traffic per dispatch (separate --pmc passes)", "",
              "| kernel | VGPRs | FETCH_SIZE KiB | WRITE_SIZE KiB | HBM bytes (2*F+W)*1024 |", "|---|---|---|---|---|"]
    traffic = {}
    for (name, vg), cnt in sorted(by_kernel.items()):
        f = cnt.get("FETCH_SIZE", [])
        w = cnt.get("WRITE_SIZE", [])
        fa = sum(f) / len(f) if f else float("nan")
        wa = sum(w) / len(w) if w else float("nan")
        hbm = (2 * fa + wa) * 1024
        lines.append(f"| {name[:90]} | {vg} | {fa:.1f} | {wa:.1f} | {hbm:.4g} |")
        if "pt_camera_kernel<false" in name:
            traffic.setdefault("candidates", []).append({"name": name, "vgpr": vg, "hbm": hbm,
                                                         "fetch_kib": fa, "write_kib": wa})
    # the timed (non-instrumented) pt kernel is the <false> instantiation (profile.sh keeps full names)
    cands = traffic.get("candidates", [])
    import hashlib
    lib = os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", "libptgs.so")
    out = {"tag": tag, "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest()}
    if cands:
        c = cands[0]
        out["pt_camera_kernel"] = {"workload": workload, "hbm_bytes_per_launch": c["hbm"], "vgpr": c["vgpr"],
                                   "fetch_kib": c["fetch_kib"], "write_kib": c["write_kib"],
                                   "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024"}
    with open(os.path.join(ROOT, "profiles", f"{tag}_summary.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    with open(os.path.join(ROOT, "profiles", "traffic_latest.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("\n".join(lines))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01",
         sys.argv[2] if len(sys.argv) > 2 else "C3 1920x1080 64spp 250000tri")
