"""The crate-check recipe (oracle/crate_check/, SURVEY.md §8(c)'s upgrade path to a true oracle)
cannot run here (no cargo, no registry).  These CPU tests keep its plumbing honest: the case
list covers every golden, and compare.py accepts hashes equal to the goldens and names a
mismatch -- so the day a maintainer runs the crate, a disagreement cannot pass silently."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CC = os.path.join(ROOT, "oracle", "crate_check")


def _cases():
    r = subprocess.run([sys.executable, os.path.join(CC, "make_cases.py")], capture_output=True, text=True, check=True)
    return r.stdout.splitlines()


def _golden_lines():
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "rs_golden.json")))
    out = [f"encode {i} {c['recovery']['sha256']}" for i, c in enumerate(g["encode"])]
    out += [f"decode {i} {c['restored']['sha256']}" for i, c in enumerate(g["decode"])]
    out += [f"coder {i} {c['data_sha256']} {c['coding_sha256']}" for i, c in enumerate(g["coder"])]
    return g, out


def test_cases_cover_goldens():
    g, _ = _golden_lines()
    kinds = [ln.split()[0] for ln in _cases()]
    assert kinds.count("encode") == len(g["encode"]) and kinds.count("decode") == len(g["decode"])
    assert kinds.count("coder") == len(g["coder"])
    # the power-of-two rate tie with k > m (32:31) is among them: the crate pins the tie-break
    assert "encode 32 31 64" in " ".join(ln.rsplit(" ", 1)[0] for ln in _cases())


def test_compare_accepts_and_rejects(tmp_path):
    _, lines = _golden_lines()
    good = tmp_path / "good.txt"
    good.write_text("\n".join(lines) + "\n")
    r = subprocess.run([sys.executable, os.path.join(CC, "compare.py"), str(good)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    bad = tmp_path / "bad.txt"
    bad.write_text("\n".join(lines[:-1] + [lines[-1][:-1] + ("0" if lines[-1][-1] != "0" else "1")]) + "\n")
    r = subprocess.run([sys.executable, os.path.join(CC, "compare.py"), str(bad)], capture_output=True, text=True)
    assert r.returncode == 1 and "MISMATCH" in r.stdout
