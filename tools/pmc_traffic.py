"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; one counter
per pass because TCC has 4 slots and they cost 3 + 2).

Corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): FETCH_SIZE is in KiB and on gfx950 reports
half the bytes of a wide coalesced streaming read -> x2; WRITE_SIZE is exact for 16 B/lane
stores.  Prints a per-kernel-family table and writes JSON for bench.py's roofline.traffic.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json>
"""
import csv
import glob
import json
import sys
from collections import defaultdict

FAMILIES = {
    "gemm": ("gemm_glds_kernel", "gemm_kernel", "gemm_pp256_kernel", "gemm_sk_kernel", "gemm_skr_kernel", "k_conv3x3_c32"),
    "mhc_fused": ("mhc_fused_kernel", "mhc_fused2_kernel", "mhc_fused_pipe_kernel"),
}


def load(d, counter):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] != counter:
            continue
        key = r["Dispatch_Id"]
        per[key] += float(r["Counter_Value"])
        names[key] = r["Kernel_Name"]
    return per, names


def family(name):
    for fam, pats in FAMILIES.items():
        if any(p in name for p in pats):
            return fam
    return "other"


def main():
    fetch, names = load(sys.argv[1], "FETCH_SIZE")
    write, wnames = load(sys.argv[2], "WRITE_SIZE")
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for k, v in fetch.items():
        a = agg[family(names[k])]
        a[0] += 1
        a[1] += 2.0 * v * 1024.0          # KiB -> B, gfx950 x2 read correction
    wagg = defaultdict(lambda: [0, 0.0])
    for k, v in write.items():
        a = wagg[family(wnames[k])]
        a[0] += 1
        a[1] += v * 1024.0
    out = {}
    for fam in sorted(set(agg) | set(wagg)):
        n, rb, _ = agg[fam]
        wn, wb = wagg[fam]
        out[fam] = {"launches": n, "read_bytes_per_launch": rb / max(n, 1),
                    "write_bytes_per_launch": wb / max(wn, 1),
                    "bytes_per_launch": rb / max(n, 1) + wb / max(wn, 1)}
        print(f"{fam:10s} launches={n:6d} read/launch={rb / max(n, 1) / 1e6:9.3f} MB "
              f"write/launch={wb / max(wn, 1) / 1e6:9.3f} MB")
    json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
