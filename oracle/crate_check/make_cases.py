"""Writes the cases of tests/golden/rs_golden.json as the crate check's stdin lines
(oracle/crate_check/src/main.rs).  Test infrastructure; see Cargo.toml."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
g = json.load(open(os.path.join(HERE, "..", "..", "tests", "golden", "rs_golden.json")))
lst = lambda v: ",".join(str(x) for x in v) or "-"
for c in g["encode"]:
    print("encode", c["k"], c["m"], c["S"], c["seed"])
for c in g["decode"]:
    print("decode", c["k"], c["m"], c["S"], c["seed"], lst(c["erased_original"]), lst(c["erased_recovery"]))
for c in g["coder"]:
    print("coder", c["payload_len"], c["seed"], c["num_coding"])
