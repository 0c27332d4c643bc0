#!/usr/bin/env python3
"""VGPR / spill / LDS use of the gfx950 kernels in a built object (no GPU needed).

Usage: python tools/kernel_resources.py [alpenglow_amd/_lib/obj/rs_kernels.hip.o] [name-filter]
Unbundles the object's .hip_fatbin with the ROCm LLVM tools and reads the code-object notes.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    obj = sys.argv[1] if len(sys.argv) > 1 else "alpenglow_amd/_lib/obj/rs_kernels.hip.o"
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    for blk in notes.split("  - .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        if filt not in name:
            continue
        g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "-"])[1]
        print(f"{name[:100]:100s} vgpr {g('vgpr_count'):>4} spill {g('vgpr_spill_count'):>3} "
              f"sgpr_spill {g('sgpr_spill_count'):>3} scratch {g('private_segment_fixed_size'):>4} "
              f"lds {g('group_segment_fixed_size'):>6}")


if __name__ == "__main__":
    main()
