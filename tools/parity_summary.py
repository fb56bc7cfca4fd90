"""Summary of the parity records the GPU tests write (tests/conftest.py record_parity ->
gpurun_out/parity/*.json): mHC layer bf16 vs the reference's own bf16 error, every fused variant
forced, the large-T policy cases, the timed-step / streaming graph outputs and the bf16 training
anchors.  usage: python tools/parity_summary.py <parity dir> > SUMMARY.txt"""
import glob
import json
import os
import sys

d = sys.argv[1]


def load(name):
    with open(os.path.join(d, name + ".json")) as f:
        return json.load(f)


def names(prefix):
    return sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(d, prefix + "*.json")))


print("bf16 parity anchored to the reference's OWN bf16 error (S8: the reference under an emulated CUDA autocast")
print("bf16 policy) and to an absolute bound (MHC_BF16_BOUND = 1.5e-2 rel-L2 vs fp64, ~3x the HIP level)\n")
print("mHC layer (T=64), default kernel, rel-L2 vs the reference fp64 run")
for n in names("mhc_bf16_"):
    r = load(n)
    print(f"  {n[9:]:18s} hip {r['hip_bf16_vs_f64']:.4f}  ref_bf16 {r['ref_bf16_vs_f64']:.4f}  ratio {r['ratio']:.3f}")
print("\nevery kernel variant FORCED on the same fixtures (rel-L2 vs fp64; ratio = / the reference's bf16 error)")
for n in names("mhc_variants_"):
    r = load(n)
    v = {k: x for k, x in r.items() if isinstance(x, dict)}
    cells = "  ".join(f"{k} {x['hip_bf16_vs_f64']:.4f} ({x['ratio_to_ref_bf16']:.3f})" for k, x in sorted(v.items()))
    print(f"  {n[13:]:18s} ref_bf16 {r['ref_bf16_vs_f64']:.4f}: {cells}")
print("\nlarge-T fixtures (the token counts that cross the kernel-selection thresholds), automatic policy")
for n in names("mhc_large_"):
    r = load(n)
    print(f"  {n[10:]:24s} variant 0x{int(r['variant'] or 0):x}  hip {r['hip_bf16_vs_f64']:.4f}  bound {r['bound']}")
for n in names("timed_step_"):
    r = load(n)
    print(f"\n{n}: {r['config']} vs fixture {r['fixture']}")
    print("  worst image rel-L2, bf16 graph vs fp32 HIP:", r["worst_image_rel_l2_bf16_graph_vs_fp32_hip"],
          "bounds", r["bounds"])
    print("  class agreement vs reference fp64 (margin 1e-2):", r["class_agreement_vs_ref_f64_margin_1e-2"])
    v = r.get("vs_reference_bf16")
    if v:
        print(f"  {v['bound']}")
        for k, x in v.items():
            if isinstance(x, dict):
                print("   ", k, {a: b for a, b in x.items()})
for n in names("streaming_"):
    r = load(n)
    print(f"\n{n}: {r['config']}")
    print("  graph vs reference fp64 logits rel-L2", r["graph_vs_ref_f64"]["logits_rel_l2"],
          "class agreement", [round(a, 4) for a in r["graph_vs_ref_f64"]["class_agreement_margin_1e-2"]])
for n in names("train_bf16_"):
    r = load(n)
    print(f"\n{n}")
    for part, x in r.items():
        if not isinstance(x, dict) or "group_norm_rel" not in x:
            continue
        ref = x.get("ref_bf16_group_norm_rel") or x.get("ref640_bf16_group_norm_rel")
        extra = f" ({x['statistic']}, x seeds {x['x_seeds']})" if "statistic" in x else ""
        print(f"  {part}{extra}")
        for k in sorted(x["group_norm_rel"]):
            rr = ref.get(k) if ref else None
            print(f"    {k:24s} hip {x['group_norm_rel'][k]:.4f}" + (f"  ref_bf16 {rr:.4f}  ratio {x['group_norm_rel'][k] / max(rr, 1e-2):.2f}" if rr else ""))
    if "config" in r:
        print(f"  {r['config']}: loss rel {r['loss_rel']:.4f}, group mean {r['groups']['hip_mean']:.4f} vs reference-640 {r['groups']['ref_bf16_mean']:.4f}")
