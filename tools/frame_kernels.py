"""Launches per frame from a rocprofv3 kernel trace of tools/lat_prof.py (B=1 graph replays).

The stem convolution is the first kernel of every forward; the kernels between the last two stem
launches are one replayed frame.  Prints the frame's launch count, its GPU span (first start to
last end), the summed kernel time and a per-kernel histogram.

usage: python tools/frame_kernels.py <dir with *kernel_trace.csv> [stem substring]
"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
stem = sys.argv[2] if len(sys.argv) > 2 else "k_conv_stem"
f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))))
idx = [i for i, r in enumerate(rows) if stem in r[2]]
if len(idx) < 2:
    sys.exit(f"fewer than two '{stem}' launches in {f}")
frame = rows[idx[-2]:idx[-1]]
span = (frame[-1][1] - frame[0][0]) / 1e3
busy = sum(e - s for s, e, _ in frame) / 1e3
print(f"launches per frame {len(frame)}; GPU span {span:.1f} us; summed kernel time {busy:.1f} us "
      f"({len(idx)} frames in the trace)")
hist = collections.Counter()
tsum = collections.defaultdict(float)
for s, e, n in frame:
    k = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    hist[k] += 1
    tsum[k] += (e - s) / 1e3
for k, c in sorted(hist.items(), key=lambda kv: -tsum[kv[0]]):
    print(f"{c:5d}  {tsum[k]:8.1f} us  {k[:150]}")
