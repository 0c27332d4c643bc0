"""CPU tests of the C-ABI library: it builds, loads, exports every symbol the header
declares, agrees with the oracle on host logic (rate rule, generated constants), and fails
loudly -- never falls back to the CPU -- when no GPU is present."""

import os
import re
import subprocess

import numpy as np
import pytest

import rs_oracle as o
from alpenglow_amd import build, rs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "alpenglow_rs.h")


@pytest.fixture(scope="module")
def lib():
    build.build()
    return rs.load()


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ag_\w+)\s*\(", text)))


def test_header_declares_what_python_binds():
    assert header_symbols() == sorted(rs.EXPORTS)


def test_library_exports_every_header_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", rs.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (ag_\w+)", out))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing
    for s in header_symbols():
        assert hasattr(lib, s)


def test_library_contains_gfx950_code_object(lib):
    blob = open(rs.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_abi_version_and_status_strings(lib):
    assert lib.ag_rs_abi_version() == 1
    assert lib.ag_rs_status_string(9) == b"not enough shards"
    assert lib.ag_rs_status_string(21) == b"invalid padding"


@pytest.mark.parametrize("k,m", [(32, 32), (16, 4), (64, 64), (32, 64), (32, 33), (20, 30), (30, 20),
                                 (1, 1), (1, 65535), (65535, 1), (100, 3), (3, 100)])
def test_rate_rule_matches_oracle(lib, k, m):
    assert rs.use_high_rate(k, m) == o.use_high_rate(k, m)


def test_unsupported_counts(lib):
    for k, m in [(0, 1), (1, 0), (65536, 2), (40000, 40000)]:
        with pytest.raises(rs.RSError) as e:
            rs.use_high_rate(k, m)
        assert e.value.kind == "UnsupportedShardCount"


def test_fast_path_geometry(lib):
    assert rs.has_fast_path(32, 32, 1024) and rs.has_fast_path(32, 32, 32768)
    assert rs.has_fast_path(20, 30, 64)
    assert rs.has_fast_path(32, 32, 62)          # tail chunk: restrided onto the same kernels
    assert rs.has_fast_path(32, 32, 1000) and rs.has_fast_path(32, 64, 1022) and rs.has_fast_path(16, 4, 2)
    assert not rs.has_fast_path(32, 32, 63)      # odd: InvalidShardSize
    assert rs.has_fast_path(32, 64, 1024)        # LowRate: one transform launch per chunk
    assert rs.has_fast_path(32, 33, 1024)
    assert not rs.has_fast_path(16, 64, 1024)    # LowRate chunk 16 -> generic kernel
    assert rs.has_fast_path(16, 4, 1024)          # multi-chunk small encode
    assert rs.has_fast_path(64, 64, 1024)         # 64-point transform
    assert not rs.has_fast_path(16, 8, 1024)      # chunk 8 -> generic kernel
    assert rs.has_fast_path(64, 33, 1024)         # tie with k > m: LowRate, 64-point


def test_generated_constants_match_oracle_skew():
    build.gen_consts()
    text = open(os.path.join(build.CSRC, "rs_consts.inc")).read()
    body = text.split("kSkewLog[kSkewConstCount] = {")[1].split("};")[0]
    vals = [int(x) for x in re.findall(r"\d+", body)]
    _, _, skew, _ = o.tables()
    assert vals == [int(x) for x in skew[:len(vals)]]
    # spot-check a multiply matrix row against the oracle's field multiply
    rows = text.split("kMulRow[kSkewConstCount][16] = {")[1]
    first = [int(x, 16) for x in re.findall(r"0x([0-9a-f]{4})", rows)[: 16 * 8]]
    s = 2  # skew index 2
    mat = first[16 * s: 16 * s + 16]
    for i in range(16):
        col = int(o.mul(np.array([1 << i]), int(skew[s]))[0])
        for bit in range(16):
            assert ((mat[bit] >> i) & 1) == ((col >> bit) & 1)


def test_no_device_fails_loudly(lib):
    if rs.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(rs.RSError) as e:
        rs.Context(0)
    assert e.value.kind == "NoDevice"


def test_private_context_objects_fail_loudly_without_device(lib):
    """The per-object contexts (ReedSolomonCoder / Encoder / Decoder with ctx=None) take the
    same loud path: no GPU, no object, never a CPU fallback."""
    if rs.device_count() > 0:
        pytest.skip("a GPU is present")
    for make in (lambda: rs.ReedSolomonCoder(None, 32), lambda: rs.ReedSolomonEncoder(None, 32, 32, 1024),
                 lambda: rs.ReedSolomonDecoder(None, 32, 32, 1024)):
        with pytest.raises(rs.RSError) as e:
            make()
        assert e.value.kind == "NoDevice"


def test_pycoder_binding_marshalling(lib):
    """The CPython binding of the per-call coder path (csrc/pycoder.c) is built, bound to the
    loaded library, and rejects malformed shred lists before any device call."""
    build.build_pycoder()
    pc = rs._coder_binding()
    assert pc is not None
    with pytest.raises(ValueError):
        pc.deshred(0, [None] * 3, 32, 32)
    with pytest.raises(TypeError):
        pc.deshred(0, [None] * 63 + [b"not a tuple"], 32, 32)
    with pytest.raises(TypeError):
        pc.deshred(0, [None] * 63 + [(True, 12345)], 32, 32)
    # the coding-output size comes from the coder: a negative or foreign num_coding (or a
    # handle that is no coder) is refused before anything is allocated or called
    with pytest.raises(ValueError):
        pc.shred(0, b"abc", -1)
    with pytest.raises(ValueError):
        pc.shred(0, b"abc", 32)
    with pytest.raises(ValueError):
        pc.deshred(0, [None] * 64, 32, 32)
    # a RawShreds built from packed bytes splits on access and compares by content
    raw = rs.RawShreds(packed=(bytes(range(8)), bytes(range(8, 12)), 2))
    assert raw.data == [b"\x00\x01", b"\x02\x03", b"\x04\x05", b"\x06\x07"] and raw.coding == [b"\x08\x09", b"\x0a\x0b"]
    assert raw == rs.RawShreds(data=list(raw.data), coding=list(raw.coding))
