#!/usr/bin/env python3
"""Summarise a profiles/profile.sh run (gpurun_out/prof_<tag>/) into committed files:

  profiles/<tag>_kernel_stats.csv    rocprofv3 --kernel-trace --stats summary (as produced)
  profiles/<tag>_summary.md          per-kernel duration, HBM bytes, L2 hit rate, VALU utilisation
  profiles/traffic_latest.json       per-kernel HBM bytes per launch + duration (read by bench.py,
                                     keyed to the sha256 of the profiled libptgs.so)

HBM bytes per dispatch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE/WRITE_SIZE are in KiB and
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read (MI355X_MICROARCH.md §HBM).
L2 hit rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum).
VALU lane utilisation = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU) (active lanes per issued
VALU cycle); VALU issue share = SQ_ACTIVE_INST_VALU / SQ_ACTIVE_INST_ANY; wave wait share =
SQ_WAIT_ANY / SQ_WAVE_CYCLES.
Dispatch kinds of one kernel name are told apart by their VGPR count (the instrumented counting
pt_camera_kernel<true> differs from the timed one).
"""
import csv
import glob
import hashlib
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# kernels bench.py reports a roofline for: short key -> substring of the demangled name
TRACKED = {"pt_camera_kernel": "pt_camera_kernel<false", "gs_sort_blend_kernel": "gs_sort_blend_kernel<false",
           "gs_bin_fused_kernel": "gs_bin_fused_kernel<false, 512", "gs_bin_fused_kernel_ov": "gs_bin_fused_kernel<false, 256",
           "pt_extend_kernel": "pt_extend_kernel", "pt_shade_kernel": "pt_shade_kernel",
           "pt_shadow_kernel": "pt_shadow_kernel", "pt_raygen_kernel": "pt_raygen_kernel"}


def _find(d, pat):
    return sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))


def _counters(d):
    rows = []
    for f in _find(d, "*counter_collection.csv"):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def _short(name):
    m = re.search(r"ptgs::(\w+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main(tag, workload):
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = _find(os.path.join(base, "kt"), "*kernel_stats.csv")
    if not stats:
        raise SystemExit(f"no kernel_stats.csv under {base}/kt")
    shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    with open(stats[0]) as fh:
        krows = list(csv.DictReader(fh))
    per_kind = defaultdict(list)  # (name, vgpr) -> durations (ns)
    for f in _find(os.path.join(base, "kt"), "*kernel_trace.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                per_kind[(r.get("Kernel_Name", ""), r.get("VGPR_Count", "?"))].append(
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    cnt = defaultdict(lambda: defaultdict(list))  # (name, vgpr) -> counter -> per-dispatch values
    for sub in ("fetch", "write", "tcc", "sq"):
        for r in _counters(os.path.join(base, sub)):
            cnt[(r["Kernel_Name"], r.get("VGPR_Count", "?"))][r["Counter_Name"]].append(float(r["Counter_Value"]))

    def avg(c, k):
        v = c.get(k, [])
        return sum(v) / len(v) if v else float("nan")

    lines = [f"# rocprofv3 summary — {tag}", "", f"workload: {workload}", "",
             "## kernel-trace --stats (as reported)", "",
             "| kernel | calls | avg ms | total ms | % |", "|---|---|---|---|---|"]
    for r in krows:
        lines.append(f"| {r['Name'][:90]} | {r['Calls']} | {float(r['AverageNs']) / 1e6:.4f} | "
                     f"{float(r['TotalDurationNs']) / 1e6:.3f} | {float(r['Percentage']):.2f} |")
    lines += ["", "## per dispatch kind (kernel trace split by VGPR count; counters from separate --pmc passes)", "",
              "| kernel | VGPRs | dispatches | avg ms | FETCH KiB | WRITE KiB | HBM bytes (2F+W)·1024 | HBM GB/s | "
              "frac of 8 TB/s | L2 hit | VALU lanes | VALU issue | wave wait |",
              "|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    # the hash of the library the box profiled (profile.sh writes it next to the traces); a run without it
    # falls back to the local library, which must then be the one that was sent
    sha_file = os.path.join(base, "lib_sha256.txt")
    if os.path.exists(sha_file):
        lib_sha = open(sha_file).read().split()[0]
    else:
        lib_sha = hashlib.sha256(open(os.path.join(ROOT, "pathtracer_gaussiansplatting_amd", "libptgs.so"),
                                      "rb").read()).hexdigest()
    out = {"tag": tag, "workload": workload,
           "lib_sha256": lib_sha,
           "formula": {"hbm_bytes": "(2*FETCH_SIZE + WRITE_SIZE) * 1024", "l2_hit": "TCC_HIT/(TCC_HIT+TCC_MISS)",
                       "valu_lanes": "SQ_THREAD_CYCLES_VALU/(64*SQ_ACTIVE_INST_VALU)"},
           "kernels": {}}
    for (name, vg), durs in sorted(per_kind.items(), key=lambda kv: -sum(kv[1])):
        c = cnt.get((name, vg), {})
        ms = sum(durs) / len(durs) / 1e6
        fa, wa = avg(c, "FETCH_SIZE"), avg(c, "WRITE_SIZE")
        hbm = (2 * fa + wa) * 1024
        gbs = hbm / (ms * 1e-3) / 1e9 if ms > 0 else float("nan")
        hit, miss = avg(c, "TCC_HIT_sum"), avg(c, "TCC_MISS_sum")
        l2 = _div(hit, hit + miss)
        lanes = _div(avg(c, "SQ_THREAD_CYCLES_VALU"), 64 * avg(c, "SQ_ACTIVE_INST_VALU"))
        issue = _div(avg(c, "SQ_ACTIVE_INST_VALU"), avg(c, "SQ_ACTIVE_INST_ANY"))
        wait = _div(avg(c, "SQ_WAIT_ANY"), avg(c, "SQ_WAVE_CYCLES"))
        lines.append(f"| {name[:80]} | {vg} | {len(durs)} | {ms:.4f} | {fa:.1f} | {wa:.1f} | {hbm:.4g} | {gbs:.1f} | "
                     f"{gbs / 8000:.4f} | {l2:.3f} | {lanes:.3f} | {issue:.3f} | {wait:.3f} |")
        for key, pat in TRACKED.items():
            if pat in name and key not in out["kernels"]:
                out["kernels"][key] = {"name": _short(name), "vgpr": vg, "dispatches": len(durs), "avg_ms": ms,
                                       "fetch_kib": fa, "write_kib": wa, "hbm_bytes_per_launch": hbm,
                                       "hbm_gbs": gbs, "l2_hit": l2, "valu_lane_util": lanes,
                                       "valu_issue_share": issue, "wave_wait_share": wait}
    lines += _two_queue_timeline(base)
    with open(os.path.join(ROOT, "profiles", f"{tag}_summary.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    out = _finite(out)
    with open(os.path.join(ROOT, "profiles", "traffic_latest.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("\n".join(lines))
    print(json.dumps(out, indent=1))


def _two_queue_timeline(base, count=16):
    """The 3DGS dispatches of the kernel trace on a timeline (frames in flight put the front end and the
    blend on two queues): the first 16 consecutive ones from 40% into the trace that show both queues in a
    steady state (blends within 15 us of each other), times relative to the first."""
    import csv
    import glob
    f = sorted(glob.glob(os.path.join(base, "kt", "*kernel_trace.csv")))
    if not f:
        return []
    rows = sorted((r for r in csv.DictReader(open(f[0])) if "gs_bin_fused" in r["Kernel_Name"] or
                   "gs_sort_blend" in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
    if len({r["Queue_Id"] for r in rows}) < 2:
        return []
    def steady(w):  # both queues, and every blend within 15 us of the previous blend's end
        bl = [r for r in w if "gs_sort_blend" in r["Kernel_Name"]]
        gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(bl, bl[1:])]
        return len({r["Queue_Id"] for r in w}) > 1 and len(bl) > 3 and max(gaps) < 15000
    start = next((i for i in range(int(len(rows) * 0.4), len(rows) - count) if steady(rows[i:i + count])),
                 int(len(rows) * 0.6))
    sub = rows[start:start + count]
    t0 = int(sub[0]["Start_Timestamp"])
    out = ["", "## two-queue timeline (frames in flight: front end and blend of consecutive frames)", "",
           "| start us | end us | dur us | queue | kernel |", "|---|---|---|---|---|"]
    for r in sub:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ptgs::", "")
        out.append(f"| {(a - t0) / 1e3:.1f} | {(b - t0) / 1e3:.1f} | {(b - a) / 1e3:.1f} | {r['Queue_Id']} | {name} |")
    return out


def _div(a, b):
    return a / b if b else float("nan")


def _finite(x):
    """NaN (a counter pass that did not see the kernel) -> null, so the JSON stays standard."""
    if isinstance(x, dict):
        return {k: _finite(v) for k, v in x.items()}
    if isinstance(x, float) and x != x:
        return None
    return x


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02",
         sys.argv[2] if len(sys.argv) > 2 else "C3 1920x1080 64spp 250000tri + C2 100000 Gaussians 1920x1080")
