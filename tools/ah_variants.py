#!/usr/bin/env python3
"""Build libptgs_<name>.so variants whose pt_wavefront.hip object (or name@<source>) gets extra compiler
flags (the any-hit inlining investigation, tools/ah_repro.py; compiler-flag A/B of a kernel file):
name[@source]=flag,flag,... ; the other objects are the default ones.
   tools/ah_variants.py ahinl_b6481=-DPTGS_WF_AH_CALL=false,-mllvm,-opt-bisect-limit=6481 ..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from pathtracer_gaussiansplatting_amd import build as B
    for spec in sys.argv[1:]:
        name, flags = spec.split("=", 1)
        src = "pt_wavefront.hip"
        if "@" in name:  # name@source.hip=flags: another source file
            name, src = name.split("@", 1)
        flags = flags.split(",") if flags else []
        bdir = B.BUILD + "_" + name
        os.makedirs(bdir, exist_ok=True)
        obj = os.path.join(bdir, src + ".o")
        cmd = ([B._hipcc()] + B.COMMON + B.EXTRA.get(src, []) + flags +
               [f"--offload-arch={B.ARCH}", "-c", os.path.join(B.CSRC, src), "-o", obj])
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            print(name, "FAILED", r.stderr[-2000:])
            continue
        B.build(variant=name)  # the other objects; pt_wavefront.hip.o is newer than its sources: kept
        print("built", name, flush=True)


if __name__ == "__main__":
    main()
