"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc/p*/pmc_counter_collection.csv) per kernel.

HBM traffic per launch follows MI355X_MICROARCH.md: FETCH_SIZE (KiB) reads exactly half
the bytes of a wide coalesced stream on gfx950 -> doubled; WRITE_SIZE (KiB) is exact for
16-B-per-lane stores.  Writes profiles/pmc_traffic.json for bench.py when --shape is
given (n, k, m, S of the profiled bench run).
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("--dir", default="gpurun_out/pmc")
ap.add_argument("--shape", default=None, help="n,k,m,S of the profiled run")
ap.add_argument("--out", default=None)
args = ap.parse_args()

vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(args.dir, "p*", "pmc_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = "encode" if ("xform8_kernel<32, 0" in name or "xform_kernel<4, 32, 0" in name) else \
                "reconstruct" if ("xform8_kernel<0, 32" in name or "xform_kernel<4, 0, 32" in name) else \
                (re.search(r"(\w+(<[^()]*>)?)\(", name.replace("(anonymous namespace)", "")) or
                 re.search(r"(\w+)", name)).group(1)[:60]
        vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {}
for k, cs in vals.items():
    summary[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    s = summary[k]
    if "FETCH_SIZE" in s and "WRITE_SIZE" in s:
        s["hbm_bytes_per_launch"] = (2 * s["FETCH_SIZE"] + s["WRITE_SIZE"]) * 1024
print(json.dumps(summary, indent=1))
if args.shape and args.out:
    n, kk, m, S = [int(x) for x in args.shape.split(",")]
    doc = {"note": "HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE (x2, gfx950 wide-stream "
                   "correction) + WRITE_SIZE, separate passes (MI355X_MICROARCH.md HBM section)",
           "kernels": {}}
    for name in ("encode", "reconstruct"):
        if name in summary and "hbm_bytes_per_launch" in summary[name]:
            doc["kernels"][name] = {"shape": [n, kk, m, S],
                                    "hbm_bytes_per_launch": summary[name]["hbm_bytes_per_launch"],
                                    "fetch_size_kib": summary[name]["FETCH_SIZE"],
                                    "write_size_kib": summary[name]["WRITE_SIZE"]}
    json.dump(doc, open(args.out, "w"), indent=1)
