"""Per-kernel launch durations from a rocprofv3 kernel trace (kt_kernel_trace.csv):
average over all launches and over the last N launches (bench.py's timed steps, after the
warmup's clock ramp).  Usage: python tools/trace_steady.py TRACE.csv [N]"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dur = defaultdict(list)
for r in rows:
    dur[r["Kernel_Name"].rsplit("(", 1)[0].replace("(anonymous namespace)::", "")].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
print(f"# {sys.argv[1]}: per-kernel launch durations (ms); 'last' = the final {last} launches")
for name, d in dur.items():
    tail = d[-last:]
    print(f"{name:70s} launches {len(d):3d}  avg_all {sum(d) / len(d):.4f}  avg_last{len(tail)} {sum(tail) / len(tail):.4f}")
