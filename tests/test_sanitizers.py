"""AddressSanitizer + UndefinedBehaviorSanitizer builds of the host-only code (CPU, no GPU).

The reference runs ASan / LSan / TSan weekly (/root/reference/.github/workflows/sanitizers.yml);
SURVEY.md §5 asks for the same on this build's host C/C++.  Three programs, each compiled with
-fsanitize=address,undefined -fno-sanitize-recover=all (leak detection on) and run here:

* tests/native/patterns_selfcheck.cpp + alpenglow_amd/csrc/rs_patterns.cpp + gf16.cpp: the
  decoders' host bookkeeping (flag packing, GF(2^16) Gauss-Jordan, the syndrome and correction
  decoders' tables, the W = 64 / 128 window masks) checked against the field's definitions;
* alpenglow_amd/csrc/gen_consts.cpp + gf16.cpp: the constant generator (one restart: its
  tables must equal the committed rs_consts.inc's, and it self-checks every program);
* tests/native/oracle_selfcheck.c + oracle/rs_oracle.c + oracle/rs_cpu_avx2.c: the C oracle and
  the restated Avx2 engine (encode agreement, decode round trips, threaded block entry points).
"""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "alpenglow_amd", "csrc")
NATIVE = os.path.join(ROOT, "tests", "native")
BUILD = os.path.join(NATIVE, "_build")
SAN = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=all"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


def _build(cmd):
    os.makedirs(BUILD, exist_ok=True)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]


def _run(exe, *args):
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ missing")
def test_patterns_asan_ubsan():
    exe = os.path.join(BUILD, "patterns_selfcheck_san")
    _build(["g++", "-std=c++20", *SAN, "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", f"-I{CSRC}",
            os.path.join(NATIVE, "patterns_selfcheck.cpp"), os.path.join(CSRC, "rs_patterns.cpp"),
            os.path.join(CSRC, "gf16.cpp"), "-o", exe])
    assert _run(exe).strip() == "ok"


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ missing")
def test_gen_consts_asan_ubsan():
    exe = os.path.join(BUILD, "gen_consts_san")
    out = os.path.join(BUILD, "rs_consts_san.inc")
    _build(["g++", "-std=c++17", *SAN, f"-I{CSRC}", os.path.join(CSRC, "gen_consts.cpp"),
            os.path.join(CSRC, "gf16.cpp"), "-o", exe])
    # one restart (the full search is ~30 s natively): the programs differ from the committed
    # ones, so compare the tables and rely on the generator's own program self-checks
    _run(exe, out, "--restarts", "1")
    got, want = open(out).read(), open(os.path.join(CSRC, "rs_consts.inc")).read()
    for table in ("kSkewLog", "kMulRow", "kBasisMat"):
        pick = lambda src: src[src.index(table):src.index("};", src.index(table))]  # noqa: E731
        assert pick(got) == pick(want), table


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc missing")
def test_oracle_asan_ubsan():
    exe = os.path.join(BUILD, "oracle_selfcheck_san")
    _build(["gcc", "-std=c11", *SAN, "-pthread", os.path.join(NATIVE, "oracle_selfcheck.c"),
            os.path.join(ROOT, "oracle", "rs_oracle.c"), os.path.join(ROOT, "oracle", "rs_cpu_avx2.c"), "-o", exe])
    assert _run(exe).strip() == "ok"
