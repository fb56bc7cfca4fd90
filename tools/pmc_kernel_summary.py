"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv: for the kernels with the most
summed GRBM_GUI_ACTIVE (or dispatches), every collected counter's mean per dispatch.
usage: python tools/pmc_kernel_summary.py <dir> [top]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 8
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
per = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for r in csv.DictReader(open(f)):
    per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    names[r["Dispatch_Id"]] = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for k, cs in per.items():
    n = names[k]
    cnt[n] += 1
    for c, v in cs.items():
        agg[n][c] += v
key = "GRBM_GUI_ACTIVE" if any("GRBM_GUI_ACTIVE" in a for a in agg.values()) else None
order = sorted(agg, key=lambda n: -(agg[n].get(key, 0.0) if key else cnt[n]))[:top]
for n in order:
    cs = agg[n]
    print(f"{cnt[n]:5d} dispatches  {n[:110]}")
    print("       " + "  ".join(f"{c}={v / cnt[n]:.4g}" for c, v in sorted(cs.items())))
