"""Summarise a rocprofv3 --kernel-trace --stats directory: top kernels + per-step GPU busy time."""
import csv
import sys

d = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"GPU kernel time {tot / 1e6:.2f} ms total, {tot / 1e6 / steps:.2f} ms per step ({steps} steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{float(r['TotalDurationNs']) / tot * 100:6.2f}%  calls={int(r['Calls']) / steps:8.1f}/step  "
          f"avg={float(r['AverageNs']) / 1e3:9.1f}us  {r['Name'][:100]}")
tr = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
if tr:
    t0 = min(int(r["Start_Timestamp"]) for r in tr)
    t1 = max(int(r["End_Timestamp"]) for r in tr)
    print(f"trace span {(t1 - t0) / 1e6:.2f} ms; busy {tot / (t1 - t0) * 100:.1f}%")
