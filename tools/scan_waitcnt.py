#!/usr/bin/env python3
"""CFG-aware scan of gfx950 kernel ISA for two shapes around vector stores.

1. LOAD-BEHIND-STORE: an `s_waitcnt vmcnt(N)` with N > 0 on a path where a vector load is
   older than the last N vector memory operations and a store is among those N.  Such a wait
   relies on loads and stores retiring in issue order.
2. EXEC-AFTER-STORE: a scalar write of EXEC (s_and_saveexec, s_or_b64 exec, ...) within W
   instructions of a vector store on some path (W = --window, default 1): the store's lanes
   must be latched before EXEC changes.

The kernel's basic blocks (labels, s_branch / s_cbranch_*, s_endpgm, s_setpc) form a CFG; a
forward dataflow carries, per block entry, the set of possible (outstanding vector-memory
history, instructions since the last store) states, merged at joins.  A `vmcnt(N)` wait cuts
the history to its last N entries, so every report names a real path through the code, not a
text-order neighbour.  Reports carry the ISA line number.

Usage: python tools/scan_waitcnt.py [--window W] [source.hip | file.s ...]
       (default: the RS kernel sources, compiled to gfx950 assembly)
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "alpenglow_amd", "csrc")
INC = os.path.join(os.path.dirname(HERE), "include")
HIST = 24  # vector memory operations remembered per path (vmcnt is 6 bits; waits here are small)

EXEC_W = re.compile(r"^s_\w+\s+exec(_lo|_hi)?\b|^s_\w*saveexec\w*\s")


def kind(t: str):
    if t.startswith(("global_store", "buffer_store", "flat_store", "global_atomic", "buffer_atomic")):
        return "S"
    if t.startswith(("global_load", "buffer_load", "flat_load")):
        return "L"
    return None


def blocks_of(lines):
    """Split a function body into basic blocks: [(start_line, [instr...], succ_labels, falls)]."""
    blocks, cur, label = [], [], None
    labels = {}

    def close(falls):
        nonlocal cur, label
        blocks.append({"label": label, "ins": cur, "succ": [], "falls": falls})
        cur, label = [], None

    for no, raw in lines:
        t = raw.strip()
        m = re.match(r"^(\.LBB\S*):", t)
        if not m and (not t or t.startswith((";", "."))):
            continue
        if m:
            if cur or label is not None:
                close(True)
            label = m.group(1)
            continue
        cur.append((no, t))
        op = t.split()[0]
        if op == "s_branch" or op.startswith("s_cbranch") or op in ("s_endpgm", "s_setpc_b64"):
            tgt = t.split()[1] if len(t.split()) > 1 and op != "s_endpgm" else None
            blk_succ = [tgt] if tgt and tgt.startswith(".LBB") else []
            falls = op.startswith("s_cbranch")
            blocks.append({"label": label, "ins": cur, "succ": blk_succ, "falls": falls})
            cur, label = [], None
    if cur or label is not None:
        close(False)
    for i, b in enumerate(blocks):
        if b["label"]:
            labels[b["label"]] = i
    for i, b in enumerate(blocks):
        s = [labels[x] for x in b["succ"] if x in labels]
        if b["falls"] and i + 1 < len(blocks):
            s.append(i + 1)
        b["next"] = s
    return blocks


def transfer(state, ins, window, reports):
    hist, since = state
    for no, t in ins:
        k = kind(t)
        if k:
            hist = (hist + k)[-HIST:]
            since = 0 if k == "S" else (since + 1 if since is not None and since + 1 < window else None)
            continue
        if t.startswith("s_waitcnt") and "vmcnt(" in t:
            n = int(re.search(r"vmcnt\((\d+)\)", t).group(1))
            if n > 0 and "S" in hist[-n:] and "L" in hist[:-n]:
                reports.add(("LOAD-BEHIND-STORE", no, t))
            hist = hist[-n:] if n else ""
        if EXEC_W.match(t) and since is not None and since < window:
            reports.add(("EXEC-AFTER-STORE", no, t))
        if since is not None:
            since = since + 1 if since + 1 < window else None
    return hist, since


def scan_function(lines, window):
    blocks = blocks_of(lines)
    if not blocks:
        return set()
    states = [set() for _ in blocks]
    states[0].add(("", None))
    work = [0]
    reports = set()
    while work:
        i = work.pop()
        for st in list(states[i]):
            out = transfer(st, blocks[i]["ins"], window, reports)
            for j in blocks[i]["next"]:
                if out not in states[j]:
                    states[j].add(out)
                    work.append(j)
    return reports


def scan(asm: str, window: int):
    out = []
    lines = asm.splitlines()
    for m in re.finditer(r"^(_Z\S+):", asm, re.M):
        start = asm.count("\n", 0, m.start())
        end_pos = asm.find(".Lfunc_end", m.end())
        end = asm.count("\n", 0, end_pos)
        body = [(no + 1, lines[no]) for no in range(start + 1, end)]
        rep = scan_function(body, window)
        if rep:
            out.append((m.group(1), sorted(rep, key=lambda r: r[1])))
    return out


def to_asm(src, d):
    if src.endswith(".s"):
        return open(src).read()
    s = os.path.join(d, os.path.basename(src) + ".s")
    path = src if os.path.exists(src) else os.path.join(CSRC, os.path.basename(src))
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-fno-slp-vectorize",
                    f"-I{INC}", f"-I{CSRC}", "-mllvm", "-amdgpu-promote-alloca-to-vector-limit=2048",
                    "--cuda-device-only", "-S", "-x", "hip", path, "-o", s], check=True, capture_output=True)
    return open(s).read()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--window", type=int, default=1)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("srcs", nargs="*", default=["rs_kernels.hip", "rs_xform64.hip", "rs_decode_c.hip"])
    args = ap.parse_args()
    total = 0
    with tempfile.TemporaryDirectory() as d:
        for src in args.srcs:
            for name, reps in scan(to_asm(src, d), args.window):
                kinds = {}
                for r in reps:
                    kinds[r[0]] = kinds.get(r[0], 0) + 1
                total += len(reps)
                print(f"{os.path.basename(src)}: {name[:110]}  {kinds}")
                if args.verbose:
                    for r in reps[:12]:
                        print(f"    line {r[1]}: {r[0]}: {r[2]}")
    print(f"{total} report(s)")


if __name__ == "__main__":
    main()
