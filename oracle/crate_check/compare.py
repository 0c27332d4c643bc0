"""Compares the crate check's output (oracle/crate_check/src/main.rs) with the restatement
goldens.  Exit 0 when every hash agrees: the oracle (and with it the GPU path, which the GPU
tests hold to these goldens) is then pinned against the crate.  Usage: compare.py OUT.txt"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
g = json.load(open(os.path.join(HERE, "..", "..", "tests", "golden", "rs_golden.json")))
want = {("encode", i): [c["recovery"]["sha256"]] for i, c in enumerate(g["encode"])}
want.update({("decode", i): [c["restored"]["sha256"]] for i, c in enumerate(g["decode"])})
want.update({("coder", i): [c["data_sha256"], c["coding_sha256"]] for i, c in enumerate(g["coder"])})
got = {}
for line in open(sys.argv[1]):
    f = line.split()
    if f:
        got[(f[0], int(f[1]))] = f[2:]
bad = [k for k in want if got.get(k) != want[k]]
print(f"{len(want) - len(bad)} of {len(want)} cases agree with the crate")
for k in bad:
    print("MISMATCH", k, "crate", got.get(k), "oracle", want[k])
sys.exit(1 if bad else 0)
