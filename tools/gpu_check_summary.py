#!/usr/bin/env python3
"""Summarise a tools/gpu_check.sh run (gpurun_out/check_<tag>/) into profiles/<tag>_gputest.txt (pass
counts, per-test durations, smoke line, library sha256, git HEAD) and profiles/<tag>_bench.json (the
bench's JSON line).   tools/gpu_check_summary.py <tag> [<git rev>]"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", f"check_{tag}")
    rev = sys.argv[2] if len(sys.argv) > 2 else subprocess.run(
        ["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
    read = lambda f: open(os.path.join(src, f)).read() if os.path.exists(os.path.join(src, f)) else ""
    pytest_log, smoke, bench, sha = read("pytest.log"), read("smoke.log"), read("bench.log"), read("lib_sha256.txt")
    lines = [f"# GPU check {tag} (tools/gpu_check.sh on one gpurun MI355X box, builder-run; source tree {rev})", ""]
    lines.append(f"libptgs.so sha256: {sha.split()[0] if sha else 'n/a'}")
    summary = [l for l in pytest_log.splitlines() if re.search(r"\d+ (passed|failed)", l)]
    lines.append("pytest -m gpu: " + (summary[-1].strip("= ") if summary else "n/a"))
    lines += [l for l in pytest_log.splitlines() if l.startswith("pytest rc=")]
    lines += [l for l in smoke.splitlines() if l.startswith("smoke")]
    lines += ["", "## slowest tests"]
    grab = False
    for l in pytest_log.splitlines():
        if "slowest" in l:
            grab = True
            continue
        if grab:
            if re.match(r"^\d+\.\d+s ", l):
                lines.append(l)
            elif l.strip():
                break
    open(os.path.join(ROOT, "profiles", f"{tag}_gputest.txt"), "w").write("\n".join(lines) + "\n")
    js = [l for l in bench.splitlines() if l.startswith("{")]
    if js:
        d = json.loads(js[-1])
        d["_provenance"] = f"builder gpurun ({tag}): python bench.py --gpus 1 --steps 20 --warmup 5, source tree {rev}"
        json.dump(d, open(os.path.join(ROOT, "profiles", f"{tag}_bench.json"), "w"), indent=1)
    print("\n".join(lines[:8]))


if __name__ == "__main__":
    main()
