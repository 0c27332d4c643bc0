"""Builds libalpenglow_rs.so in-tree (alpenglow_amd/_lib/) for gfx950.

Steps:
  1. compile and run csrc/gen_consts.cpp -> csrc/rs_consts.inc (FFT skew constants and
     their 16x16 GF(2) multiply matrices; committed, regenerated and checked here);
  2. hipcc --offload-arch=gfx950 the kernels and the host library into one shared object.

Usage: python -m alpenglow_amd.build [--force]
"""

from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
OBJDIR = os.path.join(LIBDIR, os.environ.get("AG_RS_OBJ_DIR", "obj"))
LIB = os.path.join(LIBDIR, os.environ.get("AG_RS_LIB_NAME", "libalpenglow_rs.so"))
INCLUDE = os.path.join(os.path.dirname(HERE), "include")

ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else "hipcc")
CXX = os.environ.get("CXX_HOST", "g++")

SOURCES = ["rs_kernels.hip", "rs_xform64.hip", "rs_decode_c.hip", "merkle.hip", "cipher.hip", "ed25519.hip", "wire.hip", "slice.hip", "shredder.hip", "rs_api.cpp", "rs_patterns.cpp", "gf16.cpp"]
HEADERS = ["gf16.hpp", "rs_device.hpp", "rs_xform.hpp", "rs_launch.hpp", "rs_consts.inc", "rs_patterns.hpp", "merkle.hpp", "sha256.hpp", "cipher.hpp", "ed25519.hpp", "ed25519_core.hpp", "wire.hpp", "slice.hpp", "shredder.hpp", "unaligned.hpp"]
# -fno-slp-vectorize: the SLP vectoriser packs the bitsliced XOR networks into <2 x i32>
# ops, which lengthens live ranges (measured +40 VGPRs on the transform kernel).
# -amdgpu-promote-alloca-to-vector-limit: keeps the four-Russians tables of decode_x and
# decode_syn (4 x 16 words, wave-uniform picks) in VGPRs (v_movrels) instead of scratch.
# rs_kernels.hip and rs_decode_c.hip need 2048 (at 512 two of decode_syn's four tables land in scratch; no
# other RS kernel's VGPR or scratch use changes, checked with
# -Rpass-analysis=kernel-resource-usage); the other sources keep 512, the setting their
# kernels were measured with (2048 would change the Ed25519 kernels' scratch use).
HIP_FLAGS = [*os.environ.get("AG_RS_EXTRA_HIPFLAGS", "").split(),
             "-O3", "-std=c++20", "-fPIC", f"--offload-arch={ARCH}", "-fno-slp-vectorize",
             "-Wall", "-Wno-unused-command-line-argument", f"-I{INCLUDE}", f"-I{CSRC}"]


def _deps(source: str, seen=None) -> list[str]:
    """The csrc headers `source` includes, transitively (rebuild only what a header touches)."""
    import re

    seen = set() if seen is None else seen
    path = os.path.join(CSRC, source)
    if not os.path.exists(path):
        return []
    for h in re.findall(r'#include "([^"/]+)"', open(path).read()):
        if h not in seen:
            seen.add(h)
            _deps(h, seen)
    return sorted(seen)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def gen_consts() -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    gen = os.path.join(OBJDIR, "gen_consts")
    srcs = [os.path.join(CSRC, "gen_consts.cpp"), os.path.join(CSRC, "gf16.cpp")]
    if _mtime(gen) < max(_mtime(s) for s in srcs + [os.path.join(CSRC, "gf16.hpp")]):
        _run([CXX, "-O2", "-std=c++17", f"-I{CSRC}", *srcs, "-o", gen])
    # per-process output and an atomic replace: concurrent builds (parallel test workers) must
    # never read or install a half-written table
    out = os.path.join(OBJDIR, f"rs_consts.{os.getpid()}.inc")
    _run([gen, out])
    dst = os.path.join(CSRC, "rs_consts.inc")
    new = open(out).read()
    if not os.path.exists(dst) or open(dst).read() != new:
        tmp = f"{dst}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            f.write(new)
        os.replace(tmp, dst)
    os.remove(out)
    return dst


def build(force: bool = False) -> str:
    if shutil.which(HIPCC) is None and not os.path.exists(HIPCC):
        raise RuntimeError("hipcc not found: cannot build the HIP extension")
    gen_consts()
    os.makedirs(OBJDIR, exist_ok=True)
    objs, jobs = [], []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OBJDIR, s + ".o")
        objs.append(obj)
        deps = [os.path.join(CSRC, h) for h in _deps(s)] + [os.path.join(INCLUDE, "alpenglow_rs.h")]
        limit = 2048 if s in ("rs_kernels.hip", "rs_xform64.hip", "rs_decode_c.hip") else 512
        cmd = [HIPCC, *HIP_FLAGS, "-mllvm", f"-amdgpu-promote-alloca-to-vector-limit={limit}", "-c", src, "-o", obj]
        # the stamp holds the full compile command: a flag change (AG_RS_EXTRA_HIPFLAGS
        # diagnostics, the promote-alloca limit) rebuilds the object even when no file changed
        stamp = obj + ".cmd"
        old = open(stamp).read() if os.path.exists(stamp) else None
        if force or old != " ".join(cmd) or _mtime(obj) < max(_mtime(src), *(_mtime(d) for d in deps)):
            jobs.append((cmd, stamp))
    def _compile(job):
        cmd, stamp = job
        if os.path.exists(stamp):
            os.remove(stamp)
        _run(cmd)
        with open(stamp, "w") as f:
            f.write(" ".join(cmd))
    with cf.ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        list(ex.map(_compile, jobs))
    if force or jobs or _mtime(LIB) < max(_mtime(o) for o in objs):
        tmp = LIB + ".tmp"
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp])
        os.replace(tmp, LIB)
    return LIB


PYCODER = os.path.join(LIBDIR, "_pycoder" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))


def build_pycoder(force: bool = False) -> str:
    """The CPython binding of the per-call coder path (csrc/pycoder.c; host code, gcc)."""
    src = os.path.join(CSRC, "pycoder.c")
    hdr = os.path.join(INCLUDE, "alpenglow_rs.h")
    if force or _mtime(PYCODER) < max(_mtime(src), _mtime(hdr)):
        os.makedirs(LIBDIR, exist_ok=True)
        tmp = PYCODER + ".tmp"
        _run([os.environ.get("CC_HOST", "gcc"), "-O2", "-shared", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter",
              f"-I{sysconfig.get_paths()['include']}", f"-I{INCLUDE}", src, "-o", tmp])
        os.replace(tmp, PYCODER)
    return PYCODER


if __name__ == "__main__":
    build_pycoder(force="--force" in sys.argv)
    print(build(force="--force" in sys.argv))
