"""Per-kernel busy / traffic table of one bench workload from the rocprofv3 passes of
tools/gpu_round.sh (steps `mfma` and `pmc`): MFMA busy and bf16 FLOP utilisation
(pmc_mfma.json, tools/pmc_mfma.py), HBM read / write bytes per call from the FETCH_SIZE /
WRITE_SIZE passes (gfx950 corrections as tools/pmc_traffic.py: FETCH x2 x 1 KiB, WRITE x 1 KiB),
sorted by MFMA work and bytes moved.

usage: python tools/pmc_table.py <round dir with pmc_mfma.json, pmc_FETCH_SIZE/, pmc_WRITE_SIZE/> [top N]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n[:n.index("(")] if "(" in n else n


def counter(sub, name, scale):
    f = glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True)[0]
    tot, calls = defaultdict(float), defaultdict(set)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != name:
            continue
        k = short(r["Kernel_Name"])
        tot[k] += float(r["Counter_Value"]) * scale
        calls[k].add(r["Dispatch_Id"])
    return {k: tot[k] / len(calls[k]) for k in tot}


rd = counter("pmc_FETCH_SIZE", "FETCH_SIZE", 2 * 1024.0)
wr = counter("pmc_WRITE_SIZE", "WRITE_SIZE", 1024.0)
mf = json.load(open(os.path.join(d, "pmc_mfma.json")))["kernels"]
rows = []
for k, v in mf.items():
    rows.append((k, v["calls"], v["mfma_busy"], v["mfma_flop_util"], v["mfma_gflop_per_call"], rd.get(k), wr.get(k)))
rows.sort(key=lambda r: -(r[1] * (r[4] or 0)) - 1e-6 * r[1] * ((r[5] or 0) + (r[6] or 0)))
print(f"{'kernel':70s} {'calls':>6s} {'busy':>6s} {'flopU':>6s} {'GF/call':>8s} {'rd MB':>8s} {'wr MB':>8s}")
for k, c, b, u, gf, r, w in rows[:top]:
    print(f"{k[:70]:70s} {c:6d} {b:6.3f} {u:6.3f} {gf:8.2f} {(r or 0) / 1e6:8.2f} {(w or 0) / 1e6:8.2f}")
