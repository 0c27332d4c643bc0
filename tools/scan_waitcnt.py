#!/usr/bin/env python3
"""Flag kernels whose gfx950 ISA waits for an older vector load while a younger store is in
flight (s_waitcnt vmcnt(N > 0) with a store among the last N vector memory instructions and a
load before them, in text order).  That shape preceded xform_h8's intermittently skipped
stores.  Text order only: an aid for review, not a proof.

Usage: python tools/scan_waitcnt.py [source.hip ...]   (default: the RS kernel sources)
"""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "alpenglow_amd", "csrc")
INC = os.path.join(os.path.dirname(HERE), "include")


def scan(asm: str):
    out = []
    for m in re.finditer(r"^(_Z\S+):", asm, re.M):
        end = asm.find(".Lfunc_end", m.end())
        hist, flagged = [], 0
        for line in asm[m.end():end].splitlines():
            t = line.strip()
            if t.startswith(("global_store", "buffer_store")):
                hist.append("S")
            elif t.startswith(("global_load", "buffer_load")):
                hist.append("L")
            elif t.startswith("s_waitcnt") and "vmcnt(" in t:
                n = int(re.search(r"vmcnt\((\d+)\)", t).group(1))
                if n > 0 and "S" in hist[-n:] and "L" in hist[:-n]:
                    flagged += 1
        if flagged:
            out.append((m.group(1), flagged))
    return out


def main():
    srcs = sys.argv[1:] or ["rs_kernels.hip", "rs_xform64.hip", "rs_decode_c.hip"]
    with tempfile.TemporaryDirectory() as d:
        for src in srcs:
            s = os.path.join(d, os.path.basename(src) + ".s")
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-fno-slp-vectorize",
                            f"-I{INC}", f"-I{CSRC}", "-mllvm", "-amdgpu-promote-alloca-to-vector-limit=2048",
                            "--cuda-device-only", "-S", "-x", "hip", os.path.join(CSRC, os.path.basename(src)), "-o", s],
                           check=True, capture_output=True)
            for name, n in scan(open(s).read()):
                print(f"{os.path.basename(src)}: {name[:100]}  {n} wait(s)")


if __name__ == "__main__":
    main()
