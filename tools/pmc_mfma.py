"""MFMA utilisation, LDS bank conflicts and issue mix per kernel from rocprofv3 --pmc passes.

usage: python tools/pmc_mfma.py <out.json> <pass_dir> [<pass_dir> ...]

Every pass directory holds one rocprofv3 counter_collection.csv (one pass per directory: the SQ
block has 8 slots, GRBM 2).  Values are summed per dispatch over the counter's instances, then
per kernel name.  Definitions (MI355X_MICROARCH.md, "Per-instruction cycle constants", "DVFS"):
  cycles      = GRBM_GUI_ACTIVE / 8            (the counter is summed over the 8 XCDs)
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (cycles * 1024 SIMDs)   -- fraction of SIMD-cycles
                with the matrix pipe busy (the counter is MFMA pipe cycles, 32 per 32x32x16 bf16)
  mfma_flop   = SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512                 -- executed bf16 MFMA FLOP
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE           -- extra LDS cycles share
Kernels are grouped into the bench's families (gemm / mhc_fused / other) as in pmc_traffic.py.
"""
import csv
import glob
import json
import sys
from collections import defaultdict

FAMILIES = {
    "gemm": ("gemm_glds_kernel", "gemm_kernel", "gemm_pp256_kernel", "gemm_sk_kernel", "k_conv3x3_c32",
             "gemm_sk2_kernel", "gemm_stk_kernel"),
    "mhc_fused": ("mhc_fused_kernel", "mhc_fused2_kernel", "mhc_fused3_kernel"),
}


def family(name):
    for fam, pats in FAMILIES.items():
        if any(p in name for p in pats):
            return fam
    return "other"


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0][:90]


def main():
    out_path, dirs = sys.argv[1], sys.argv[2:]
    per = defaultdict(lambda: defaultdict(float))     # dispatch -> counter -> value
    kname = {}
    for d in dirs:
        files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
        if not files:
            print(f"(no counter_collection.csv under {d})")
            continue
        for r in csv.DictReader(open(files[0])):
            key = (d, r["Dispatch_Id"])
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            kname[key] = r["Kernel_Name"]
    by_name = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(int))
    for key, cs in per.items():
        n = short(kname[key])
        for c, v in cs.items():
            by_name[n][c] += v
            calls[n][c] += 1

    def derived(cs, nc):
        o = {}
        cyc = cs.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in cs:
            # per-dispatch averages: both counters come from the same pass when present
            o["mfma_busy"] = round(cs["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024.0), 4)
        if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in cs:
            o["mfma_gflop_per_call"] = round(cs["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / 1e9 /
                                             max(nc.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 1), 1), 3)
        if cs.get("SQ_LDS_IDX_ACTIVE"):
            o["lds_conflict_frac"] = round(cs.get("SQ_LDS_BANK_CONFLICT", 0.0) / cs["SQ_LDS_IDX_ACTIVE"], 4)
        if cyc and "GRBM_GUI_ACTIVE" in nc:
            o["cycles_per_call"] = round(cyc / nc["GRBM_GUI_ACTIVE"])
        for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in cs and cs.get("SQ_WAVE_CYCLES"):
                o[c.lower() + "_frac"] = round(cs[c] / cs["SQ_WAVE_CYCLES"], 4)
        return o

    rows = []
    fam = defaultdict(lambda: defaultdict(float))
    famc = defaultdict(lambda: defaultdict(int))
    for n, cs in by_name.items():
        d = derived(cs, calls[n])
        d["calls"] = max(calls[n].values())
        d["family"] = family(n)
        rows.append((cs.get("GRBM_GUI_ACTIVE", 0.0), n, d))
        for c, v in cs.items():
            fam[d["family"]][c] += v
            famc[d["family"]][c] += calls[n][c]
    rows.sort(key=lambda r: -r[0])
    out = {"families": {f: derived(cs, famc[f]) for f, cs in fam.items()},
           "kernels": {n: d for _, n, d in rows[:40]}}
    print(f"{'kernel':90s} {'calls':>6s} {'mfma_busy':>9s} {'GF/call':>9s} {'ldsconf':>8s}")
    for _, n, d in rows[:40]:
        print(f"{n:90s} {d['calls']:6d} {d.get('mfma_busy', float('nan')):9.4f} "
              f"{d.get('mfma_gflop_per_call', float('nan')):9.3f} {d.get('lds_conflict_frac', float('nan')):8.4f}")
    for f, d in out["families"].items():
        print(f"family {f:10s} {d}")
    json.dump(out, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
