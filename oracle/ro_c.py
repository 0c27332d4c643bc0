"""ctypes binding of the C oracle (oracle/rs_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg; never by the product package.
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "liboracle_rs.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        sz, p = ctypes.c_size_t, ctypes.c_void_p
        L.ro_encode.argtypes = [sz, sz, sz, p, p]
        L.ro_decode.argtypes = [sz, sz, sz, p, p, p, p, p]
        L.ro_encode_blocks.argtypes = [sz, sz, sz, sz, p, sz, p, sz, ctypes.c_int]
        L.ro_decode_blocks.argtypes = [sz, sz, sz, sz, p, sz, p, p, p, sz, ctypes.c_int]
        L.ro_use_high_rate.argtypes = [sz, sz]
        L.ro_tables.argtypes = [p, p, p, p]
        L.rb_encode.argtypes = [sz, sz, sz, p, p]
        L.rb_decode.argtypes = [sz, sz, sz, p, p, p, p, p]
        L.rb_encode_blocks.argtypes = [sz, sz, sz, sz, p, sz, p, sz, ctypes.c_int]
        L.rb_decode_blocks.argtypes = [sz, sz, sz, sz, p, sz, p, p, p, sz, ctypes.c_int]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def encode(orig: np.ndarray, m: int) -> np.ndarray:
    """orig: (k, S) uint8 -> (m, S) uint8 recovery shards."""
    orig = np.ascontiguousarray(orig, dtype=np.uint8)
    k, S = orig.shape
    rec = np.zeros((m, S), dtype=np.uint8)
    st = lib().ro_encode(k, m, S, _ptr(orig), _ptr(rec))
    if st:
        raise RuntimeError(f"ro_encode status {st}")
    return rec


def decode(orig: np.ndarray, orig_present, rec: np.ndarray, rec_present) -> np.ndarray:
    """Returns a copy of ``orig`` with the absent originals restored (crate algorithm,
    every present shard used)."""
    orig = np.ascontiguousarray(orig, dtype=np.uint8)
    rec = np.ascontiguousarray(rec, dtype=np.uint8)
    k, S = orig.shape
    m = rec.shape[0]
    op = np.ascontiguousarray(orig_present, dtype=np.uint8)
    rp = np.ascontiguousarray(rec_present, dtype=np.uint8)
    out = orig.copy()
    st = lib().ro_decode(k, m, S, _ptr(orig), _ptr(op), _ptr(rec), _ptr(rp), _ptr(out))
    if st:
        raise RuntimeError(f"ro_decode status {st}")
    return out


def avx2_available() -> bool:
    return bool(lib().rb_avx2_available())


def encode_blocks(blocks: np.ndarray, m: int, threads: int = 1, engine: str = "scalar") -> np.ndarray:
    """blocks: (n, k, S) uint8 -> (n, m, S) recovery.  engine "avx2": the crate's Avx2
    engine restated (rs_cpu_avx2.c; S % 64 == 0), "scalar": the log/exp-table oracle."""
    blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
    n, k, S = blocks.shape
    out = np.zeros((n, m, S), dtype=np.uint8)
    f = lib().rb_encode_blocks if engine == "avx2" else lib().ro_encode_blocks
    st = f(k, m, S, n, _ptr(blocks), k * S, _ptr(out), m * S, threads)
    if st:
        raise RuntimeError(f"ro_encode_blocks status {st}")
    return out


def decode_blocks(codewords: np.ndarray, k: int, orig_present, rec_present,
                  threads: int = 1, engine: str = "scalar") -> np.ndarray:
    """codewords: (n, k+m, S) -> (n, k, S) originals with absent ones restored."""
    codewords = np.ascontiguousarray(codewords, dtype=np.uint8)
    n, km, S = codewords.shape
    out = np.ascontiguousarray(codewords[:, :k, :]).copy()
    op = np.ascontiguousarray(orig_present, dtype=np.uint8)
    rp = np.ascontiguousarray(rec_present, dtype=np.uint8)
    f = lib().rb_decode_blocks if engine == "avx2" else lib().ro_decode_blocks
    st = f(k, km - k, S, n, _ptr(codewords), km * S, _ptr(op), _ptr(rp), _ptr(out), k * S, threads)
    if st:
        raise RuntimeError(f"ro_decode_blocks status {st}")
    return out


def tables():
    exp = np.zeros(65536, np.uint16)
    log = np.zeros(65536, np.uint16)
    skew = np.zeros(65535, np.uint16)
    lw = np.zeros(65536, np.uint16)
    lib().ro_tables(_ptr(exp), _ptr(log), _ptr(skew), _ptr(lw))
    return exp, log, skew, lw
