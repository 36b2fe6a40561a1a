#!/usr/bin/env python3
"""Build libptgs_<name>.so variants whose pt_wavefront.hip object gets extra compiler flags (for the
any-hit inlining investigation, tools/ah_repro.py): name=flag,flag,... ; the other objects are the
default ones (shared per variant directory).
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
        flags = flags.split(",") if flags else []
        bdir = B.BUILD + "_" + name
        os.makedirs(bdir, exist_ok=True)
        obj = os.path.join(bdir, "pt_wavefront.hip.o")
        cmd = ([B._hipcc()] + B.COMMON + B.EXTRA["pt_wavefront.hip"] + flags +
               [f"--offload-arch={B.ARCH}", "-c", os.path.join(B.CSRC, "pt_wavefront.hip"), "-o", obj])
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            print(name, "FAILED", r.stderr[-2000:])
            continue
        B.build(variant=name)  # the other objects; pt_wavefront.hip.o is newer than its sources: kept
        print("built", name, flush=True)


if __name__ == "__main__":
    main()
