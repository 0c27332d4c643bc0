"""Generates tests/golden/rs_golden.json from the numpy oracle (oracle/rs_oracle.py).

These are RESTATEMENT GOLDENS: the reference (Rust + the unvendored crate
reed-solomon-simd 3.1.0) cannot be built or run in this container, and its own tests
hold no known-answer vectors for coding-shred bytes, so parity at the reference boundary
is "unpinned" (SURVEY.md section 8c).  The fixtures freeze the oracle's outputs so that
(a) the oracle cannot drift silently and (b) the GPU path is checked against fixed bytes,
not only against a live oracle.  Inputs are regenerated from splitmix64 seeds
(BASELINE.md section 2), so only seeds, shapes and expected outputs are stored.

Usage: python tests/golden/make_golden.py
"""

from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import rs_oracle as o  # noqa: E402

FULL_BYTES_LIMIT = 4096  # store full hex below this many output bytes, else sha256


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def shards_from_seed(seed: int, n: int, S: int) -> list[bytes]:
    raw = o.splitmix64_bytes(seed, n * S)
    return [raw[i * S:(i + 1) * S] for i in range(n)]


def out_record(shards: list[bytes]) -> dict:
    cat = b"".join(shards)
    rec = {"sha256": sha(cat), "bytes": len(cat)}
    if len(cat) <= FULL_BYTES_LIMIT:
        rec["hex"] = cat.hex()
    return rec


ENCODE_CASES = [
    # (k, m, S) -- 32:32 over every layout class (S < 64, S % 64 != 0, multi-chunk), the
    # BASELINE sweep geometries, the reference's other shredders (32:64 CodingOnly,
    # 32:33 PETS) and odd counts for both rates.
    (32, 32, 2), (32, 32, 32), (32, 32, 62), (32, 32, 64), (32, 32, 1024), (32, 32, 2048),
    (32, 32, 4160), (16, 4, 128), (64, 64, 64), (32, 64, 1024), (32, 33, 66),
    (20, 30, 128), (3, 7, 2), (100, 3, 130), (1, 1, 64), (33, 32, 64), (32, 31, 64),
]

DECODE_CASES = [
    # (k, m, S, erased original indices, erased recovery indices)
    (32, 32, 2048, list(range(32)), []),                     # benches/shredder.rs:49-53
    (32, 32, 2048, list(range(16)), []),                     # BASELINE C3
    (32, 32, 1024, [0], list(range(1, 32))),                 # shredder.rs:684-688
    (32, 32, 1024, list(range(16)), list(range(16, 32))),    # shredder.rs:690-695 (middle)
    (32, 32, 64, [5, 9, 31], [0, 1, 2]),
    (16, 4, 128, [1, 7, 12], [2]),
    (64, 64, 64, list(range(0, 64, 2)), list(range(1, 64, 2))),
    (32, 64, 1024, list(range(32)), list(range(32))),        # CodingOnly: coding shreds only
    (32, 33, 66, [31], [0]),                                 # PETS: key shred never sent
    (3, 7, 2, [0, 2], [1, 3, 5]),
]

PAYLOAD_SIZES = [0, 31, 32767] + list(range(16383, 16415))  # reed_solomon.rs:244-276


def main():
    exp, log, skew, log_walsh = o.tables()
    doc = {
        "note": "restatement goldens from oracle/rs_oracle.py (parity unpinned vs the crate)",
        "tables": {
            "exp_sha256": sha(exp.astype("<u2").tobytes()),
            "log_sha256": sha(log.astype("<u2").tobytes()),
            "skew_sha256": sha(skew.astype("<u2").tobytes()),
            "log_walsh_sha256": sha(log_walsh.astype("<u2").tobytes()),
            "skew_first_256": [int(x) for x in skew[:256]],
        },
        "encode": [],
        "decode": [],
        "coder": [],
    }
    seed = 0xA11CE
    for k, m, S in ENCODE_CASES:
        seed += 1
        orig = shards_from_seed(seed, k, S)
        rec = o.encode(orig, m)
        doc["encode"].append({"k": k, "m": m, "S": S, "seed": seed, "use_high_rate": o.use_high_rate(k, m),
                              "recovery": out_record(rec)})
    for k, m, S, eo, er in DECODE_CASES:
        seed += 1
        orig = shards_from_seed(seed, k, S)
        rec = o.encode(orig, m)
        og = {i: orig[i] for i in range(k) if i not in eo}
        rg = {j: rec[j] for j in range(m) if j not in er}
        res = o.decode(k, m, og, rg)
        assert all(res[i] == orig[i] for i in eo)
        doc["decode"].append({"k": k, "m": m, "S": S, "seed": seed, "erased_original": eo,
                              "erased_recovery": er,
                              "restored": out_record([res[i] for i in sorted(res)])})
    for n in PAYLOAD_SIZES:
        seed += 1
        payload = o.splitmix64_bytes(seed, n)
        raw = o.coder_shred(payload, 32)
        doc["coder"].append({"payload_len": n, "seed": seed, "num_coding": 32,
                             "shred_bytes": len(raw.data[0]),
                             "data_sha256": sha(b"".join(raw.data)),
                             "coding_sha256": sha(b"".join(raw.coding))})
    path = os.path.join(HERE, "rs_golden.json")
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print(path)


if __name__ == "__main__":
    main()
