"""Extracts the reference's EMPTY_ROOTS digests (crypto/merkle.rs:62-157) into
tests/golden/merkle_empty_roots.json -- data only (32 expected SHA-256 outputs), the pin for
oracle/merkle_oracle.py and the library's SHA-256.  Run once where /root/reference exists:

    python tests/golden/make_merkle_golden.py
"""
import json
import os
import re

SRC = "/root/reference/src/crypto/merkle.rs"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "merkle_empty_roots.json")

text = open(SRC).read()
block = text[text.index("const EMPTY_ROOTS"):]
block = block[: block.index("];")]
digests = re.findall(r'"([0-9a-f]{64})"', block)
assert len(digests) == 32, len(digests)
json.dump({"source": "crypto/merkle.rs:62-157 EMPTY_ROOTS (hash_leaf([]), then hash_pair(node, node) per height)",
           "empty_roots": digests}, open(OUT, "w"), indent=1)
print(OUT, len(digests))
