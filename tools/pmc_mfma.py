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
    "mhc_fused": ("mhc_fused_kernel", "mhc_fused2_kernel", "mhc_fused_pipe_kernel"),
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
    # per pass: kernel name -> counter -> summed value, and the number of dispatches
    passes = []
    for d in dirs:
        files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
        if not files:
            print(f"(no counter_collection.csv under {d})")
            continue
        per = defaultdict(lambda: defaultdict(float))
        kname = {}
        for r in csv.DictReader(open(files[0])):
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            kname[r["Dispatch_Id"]] = r["Kernel_Name"]
        agg = defaultdict(lambda: defaultdict(float))
        calls = defaultdict(int)
        for k, cs in per.items():
            n = short(kname[k])
            calls[n] += 1
            for c, v in cs.items():
                agg[n][c] += v
        passes.append((agg, calls))

    def metrics(rows):
        """rows: list of (counter dict, calls) from different passes of the same kernel(s); every
        ratio uses the cycles (GRBM_GUI_ACTIVE / 8 XCDs) of its own pass."""
        o = {}
        for cs, nc in rows:
            cyc = cs.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
            if not cyc:
                continue
            o.setdefault("cycles_per_call", round(cyc / max(nc, 1)))
            o.setdefault("calls", nc)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in cs:
                o["mfma_busy"] = round(cs["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024.0), 4)
            if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in cs:
                fl = cs["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512
                o["mfma_gflop_per_call"] = round(fl / 1e9 / max(nc, 1), 3)
                # executed bf16 MFMA FLOP per cycle over the chip peak (1024 SIMDs x 1024 FLOP/clk)
                o["mfma_flop_util"] = round(fl / (cyc * 1024.0 * 1024.0), 4)
            if cs.get("SQ_LDS_IDX_ACTIVE"):
                o["lds_conflict_frac"] = round(cs.get("SQ_LDS_BANK_CONFLICT", 0.0) / cs["SQ_LDS_IDX_ACTIVE"], 4)
            for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in cs and cs.get("SQ_WAVE_CYCLES"):
                    o[c.lower() + "_frac"] = round(cs[c] / cs["SQ_WAVE_CYCLES"], 4)
        return o

    names = set()
    for agg, _ in passes:
        names |= set(agg)
    kern = {n: metrics([(agg[n], calls[n]) for agg, calls in passes if n in agg]) for n in names}
    fam_rows = []
    for agg, calls in passes:
        fa = defaultdict(lambda: defaultdict(float))
        fc = defaultdict(int)
        for n, cs in agg.items():
            f = family(n)
            fc[f] += calls[n]
            for c, v in cs.items():
                fa[f][c] += v
        fam_rows.append((fa, fc))
    fams = {f: metrics([(fa[f], fc[f]) for fa, fc in fam_rows if f in fa]) for f in FAMILIES.keys() | {"other"}}
    order = sorted(names, key=lambda n: -kern[n].get("cycles_per_call", 0) * kern[n].get("calls", 0))
    out = {"note": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024 SIMDs); mfma_flop_util = executed bf16 "
                   "MFMA FLOP (SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512) / (cycles x 1024 SIMDs x 1024 FLOP/clk); "
                   "cycles = GRBM_GUI_ACTIVE / 8 of the same rocprofv3 pass",
           "families": fams, "kernels": {n: kern[n] for n in order[:40]}}
    print(f"{'kernel':80s} {'calls':>6s} {'busy':>7s} {'flopU':>7s} {'GF/call':>8s} {'ldsconf':>8s} {'us/call':>8s}")
    for n in order[:40]:
        d = kern[n]
        print(f"{n[:80]:80s} {d.get('calls', 0):6d} {d.get('mfma_busy', float('nan')):7.4f} "
              f"{d.get('mfma_flop_util', float('nan')):7.4f} {d.get('mfma_gflop_per_call', float('nan')):8.3f} "
              f"{d.get('lds_conflict_frac', float('nan')):8.4f} {d.get('cycles_per_call', 0) / 2100:8.1f}")
    for f, d in fams.items():
        print(f"family {f:10s} {d}")
    json.dump(out, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
