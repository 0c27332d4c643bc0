"""ctypes binding of oracle/shredder_cpu.c, the composed RegularShredder on the CPU.

TEST INFRASTRUCTURE ONLY -- bench_shredder.py's cpu_baseline leg (a "port": the crate's
Avx2 RS engine restated, OpenSSL's SHA-256 and Ed25519) and tests/test_shredder_cpu.py;
never imported by the product package.
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libshredder_cpu.so")
_lib = None

SHRED, DESHRED, RECEIVE = 1, 2, 4


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        L = ctypes.CDLL(LIB_PATH)
        sz, p, i = ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int
        L.sc_run.argtypes = [i, i, sz, p, sz, p, p, p, p, p, p, p, p, p]
        L.sc_run.restype = i
        L.sc_phase_us.argtypes = [i, p, sz, p, p, p]
        L.sc_phase_us.restype = i
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def run(what: int, threads: int, payloads: np.ndarray, lens, slots, slice_idx, is_last, seed: bytes, pk: bytes,
        outputs: bool = False):
    """Shred n framed payloads (rows of `payloads`) and, per `what`, receive / deshred them
    again.  Returns (status, coding [n, 32, S] or None, roots [n, 32] or None, sigs [n, 64] or
    None); status 0 when every slice round-tripped."""
    n = payloads.shape[0]
    lens = np.ascontiguousarray(lens, np.uint32)
    slots = np.ascontiguousarray(slots, np.uint64)
    slice_idx = np.ascontiguousarray(slice_idx, np.uint64)
    is_last = np.ascontiguousarray(is_last, np.uint8)
    S = (int(lens.max()) + 64 - int(lens.max()) % 64) // 32 if n else 0
    coding = np.zeros((n, 32, S), np.uint8) if outputs else None
    roots = np.zeros((n, 32), np.uint8) if outputs else None
    sigs = np.zeros((n, 64), np.uint8) if outputs else None
    sd, pkb = np.frombuffer(seed, np.uint8).copy(), np.frombuffer(pk, np.uint8).copy()
    st = lib().sc_run(what, threads, n, _p(payloads), payloads.strides[0], _p(lens), _p(slots), _p(slice_idx),
                      _p(is_last), _p(sd), _p(pkb), _p(coding), _p(roots), _p(sigs))
    return st, coding, roots, sigs


def phase_us(payload: bytes, seed: bytes, pk: bytes, reps: int = 50):
    """Single-thread microseconds per slice: (shred, deshred, receive)."""
    out = (ctypes.c_double * 3)()
    buf = np.frombuffer(payload, np.uint8).copy()
    sd, pkb = np.frombuffer(seed, np.uint8).copy(), np.frombuffer(pk, np.uint8).copy()
    st = lib().sc_phase_us(reps, _p(buf), len(payload), _p(sd), _p(pkb), out)
    if st:
        raise RuntimeError(f"sc_phase_us failed: {st}")
    return tuple(out)
