"""GPU parity of the mHC layer, the blocks and the full HybridVision forward against the
reference (golden fixtures from oracle/gen_golden.py).

Contract: fp32 mode -- logits/boxes within atol 1e-3 of the reference run in
float64 (and of the reference fp32 run), class indices bit-exact on cells whose reference
top-1/top-2 margin is >= 1e-4.  bf16 mode (the perf mode) is reported as relative-L2 and
margin-filtered class agreement with looser bounds written in each test.
"""
import numpy as np
import pytest
import torch

from conftest import MODEL_CFG, formula_state_dict, golden, record_parity, run_options
from oracle import cases
from oracle import weights as W

pytestmark = pytest.mark.gpu


MHC_BF16_BOUND = 1.5e-2     # 3x HIP's measured bf16 mHC level vs the reference fp64 run


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


# ------------------------------------------------------------------------------ mHC layer
@pytest.mark.parametrize("fam", ["wc", "init"])
@pytest.mark.parametrize("D,e", cases.MHC_CASES)
def test_mhc_fp32_matches_reference(gpu_device, fam, D, e):
    from hv_amd import ManifoldHyperConnection
    from hv_amd.runtime import HVOptions
    g = golden(f"mhc_{fam}_D{D}_e{e}")
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=False)
    W.load_formula_weights(m, fam)
    m = m.to(gpu_device).eval()
    x = cases.mhc_input(D, e).to(gpu_device)
    for fold in (True, False):
        m.hv_options = HVOptions(fold_max_d=4096 if fold else 0)     # per-layer option
        y = m(x).cpu().numpy()
        np.testing.assert_allclose(y, g["y64"], rtol=0, atol=1e-3)
        np.testing.assert_allclose(y, g["y"], rtol=0, atol=1e-3)


@pytest.mark.parametrize("fam", ["wc", "init"])
@pytest.mark.parametrize("D,e", cases.MHC_CASES)
def test_mhc_bf16_agreement(gpu_device, fam, D, e):
    """bf16 mode held to the reference's OWN bf16 error: the reference under its autocast policy
    (S8, oracle/autocast_emu.py: bf16 matmuls/linears, fp32 LayerNorm -- manifold_layers.py:186,
    248) is `err_vs_f64` rel-L2 from its fp64 run on the same input (fixture *_bf16ref); the HIP
    bf16 mHC must be within 2x that AND within MHC_BF16_BOUND = 1.5e-2 rel-L2, 3x HIP's own
    measured level (0.003 init / 0.005 wc: the centred coefficients keep HIP at the bf16 level,
    while the reference's un-centred H_res + H_post sum loses 0.02-0.12 on wc and 0.18-1.2 at
    init, so a 2x-reference bound alone would pass a 100x regression)."""
    from conftest import record_parity
    from hv_amd import ManifoldHyperConnection
    g = golden(f"mhc_{fam}_D{D}_e{e}")
    gb = golden(f"mhc_{fam}_D{D}_e{e}_bf16ref")
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=True)
    W.load_formula_weights(m, fam)
    m = m.to(gpu_device).eval()
    y = m(cases.mhc_input(D, e).to(gpu_device)).float().cpu().numpy()
    err, ref = rel_l2(y, g["y64"]), float(gb["err_vs_f64"])
    record_parity(f"mhc_bf16_{fam}_D{D}_e{e}", {"hip_bf16_vs_f64": err, "ref_bf16_vs_f64": ref,
                                                 "ratio": err / ref, "bound_ratio": 2.0, "bound_abs": MHC_BF16_BOUND})
    assert err <= 2.0 * ref, (err, ref)
    assert err <= MHC_BF16_BOUND, err


def _mhc_variants(D, e):
    """Every kernel that can run the (D, e) site, by the HV_MV_* bits that force it."""
    from hv_amd import _lib as L
    v = {"chain": None}
    if D in (32, 64):
        v.update({"pipe": L.MV_WIDE, "pipe_merge": L.MV_WIDE | L.MV_PIPE, "perwave": L.MV_WIDE | L.MV_PERWAVE,
                  "perwave8": L.MV_WIDE | L.MV_ONE_GROUP8})
    if (D, e) == (128, 4):
        v.update({"split_hidden": L.MV_WIDE, "split_hidden_w": L.MV_WIDE | L.MV_SPLITW,
                  "perwave": L.MV_WIDE | L.MV_PERWAVE128})
    if (D, e) == (256, 2):
        v.update({"split_hidden": L.MV_SPLIT256, "split_hidden_w": L.MV_SPLIT256 | L.MV_SPLITW,
                  "perwave8": L.MV_WIDE})
    if (D, e) in ((128, 4), (256, 2), (256, 4)):
        v.update({"tok32": L.MV_TOK, "tok16": L.MV_TOK | L.MV_TOK16})
    if D == 256 and e in (2, 4):
        v.update({"toksplit2": L.MV_TOK | L.MV_TOK16 | L.MV_TOKSPLIT2,
                  "toksplit4": L.MV_TOK | L.MV_TOK16 | L.MV_TOKSPLIT4})
    return v


@pytest.mark.parametrize("fam", ["wc", "init"])
@pytest.mark.parametrize("D,e", cases.MHC_CASES)
def test_mhc_bf16_fixture_every_variant(gpu_device, fam, D, e):
    """Each fused kernel FORCED (whatever the token-count policy would pick) on the reference's mHC
    fixture, held to MHC_BF16_BOUND vs the reference fp64 run -- so a kernel the policy selects only
    at large T still meets the reference, not only the HIP chain.  Per-variant errors go to
    gpurun_out/parity/mhc_variants_<fam>_D<D>_e<e>.json (summary: profiles/r05/parity/)."""
    from hv_amd import ManifoldHyperConnection, ops
    g = golden(f"mhc_{fam}_D{D}_e{e}")
    gb = golden(f"mhc_{fam}_D{D}_e{e}_bf16ref")
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=True)
    W.load_formula_weights(m, fam)
    m = m.to(gpu_device).eval()
    x = cases.mhc_input(D, e).to(gpu_device).to(torch.bfloat16)
    rec = {"ref_bf16_vs_f64": float(gb["err_vs_f64"]), "bound": MHC_BF16_BOUND}
    for name, v in _mhc_variants(D, e).items():
        with torch.no_grad():
            ops.launch_counts(reset=True)
            if v is None:
                with run_options(use_fused_mhc=False):
                    y = m.forward_tokens(x)
            else:
                with run_options(mhc_variant=v):
                    y = m.forward_tokens(x)
            fused = ops.launch_counts()["mhc_fused"]
        assert fused == (0 if v is None else 1), (name, fused)
        err = rel_l2(y.float().cpu().numpy(), g["y64"])
        rec[name] = {"hip_bf16_vs_f64": err, "ratio_to_ref_bf16": err / rec["ref_bf16_vs_f64"]}
        assert err <= MHC_BF16_BOUND, (name, err)
    record_parity(f"mhc_variants_{fam}_D{D}_e{e}", rec)


@pytest.mark.parametrize("fam", ["wc", "init"])
@pytest.mark.parametrize("D,e,T", cases.MHC_LARGE_CASES)
def test_mhc_bf16_large_T_reference(gpu_device, fam, D, e, T):
    """The automatic kernel policy at the token counts that select each large-T kernel
    ((256, 2): token-tile 32 at 25,601, split-hidden at 102,401; (128, 4): split-hidden; (256, 4):
    the chain) against the reference's fp64 run (row subsample of fixture mhc_<fam>_D_e_T)."""
    from hv_amd import ManifoldHyperConnection, _lib, ops
    g = golden(f"mhc_{fam}_D{D}_e{e}_T{T}")
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=True)
    W.load_formula_weights(m, fam)
    m = m.to(gpu_device).eval()
    x = cases.mhc_input_large(D, e, T).to(gpu_device).to(torch.bfloat16)
    expect = {(256, 2, 25601): _lib.MV_TOK, (256, 2, 102401): _lib.MV_SPLIT256, (128, 4, 25601): 0,
              (256, 4, 25601): None}[(D, e, T)]
    v = ops._mhc_variant(D, T, None, D * e)
    if expect is None:
        assert not ops.mhc_fused_supported(D, D * e, torch.bfloat16, T=T)
    else:
        assert v == expect, hex(v)
    with torch.no_grad():
        ops.launch_counts(reset=True)
        y = m(x)
        assert ops.launch_counts()["mhc_fused"] == (0 if expect is None else 1)
    rows = torch.from_numpy(g["rows"]).to(gpu_device)
    err = rel_l2(y[rows].float().cpu().numpy(), g["y64"])
    record_parity(f"mhc_large_{fam}_D{D}_e{e}_T{T}", {"variant": v, "hip_bf16_vs_f64": err, "bound": MHC_BF16_BOUND})
    assert err <= MHC_BF16_BOUND, err


@pytest.mark.parametrize("D,e,T,with_res", [(32, 4, 64, False), (32, 4, 1000, False), (64, 4, 64, False),
                                             (64, 4, 777, False), (128, 4, 200, False), (256, 2, 401, False),
                                             (256, 2, 130, True)])
def test_mhc_fused_kernel_matches_unfused_chain(gpu_device, D, e, T, with_res):
    """hv_mhc_fused (one launch, on-chip intermediates) vs the six-launch chain, both bf16."""
    from hv_amd import ManifoldHyperConnection, _lib
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=True)
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    g = torch.Generator().manual_seed(T)
    x = torch.randn(T, D, generator=g).to(torch.bfloat16).to(gpu_device)
    res = torch.randn(T, D, generator=g).to(torch.bfloat16).to(gpu_device) if with_res else None
    with torch.no_grad():
        with run_options(mhc_variant=_lib.MV_WIDE):
            y1 = m.forward_tokens(x, residual=res).float().cpu().numpy()
        with run_options(use_fused_mhc=False):
            y0 = m.forward_tokens(x, residual=res).float().cpu().numpy()
    assert rel_l2(y1, y0) < 1e-2
    assert np.abs(y1 - y0).max() < 0.1


@pytest.mark.parametrize("tile", [16, 32, "split2", "split4"])
@pytest.mark.parametrize("D,e,T,with_res", [(256, 2, 401, False), (256, 2, 401, True), (256, 2, 6416, True),
                                             (256, 2, 130, False), (256, 2, 7, True), (128, 4, 1000, False),
                                             (128, 4, 6400, True), (256, 4, 1600, True), (256, 4, 77, False)])
def test_mhc_tok_kernel_matches_unfused_chain(gpu_device, tile, D, e, T, with_res):
    """Token-tile fused kernel (HV_MV_TOK, csrc/hv_mhc_tok.hip: 16 / 32 tokens per workgroup,
    weights streamed L2 -> LDS transposer -> MFMA) vs the unfused bf16 chain, ragged T included.
    Hd = 1024 always runs 16-token tiles.  split2 / split4: (256, 512) 16-token tiles shared by
    2 / 4 workgroups (HV_MV_TOKSPLIT*, partial y reduced by the last to finish)."""
    from hv_amd import ManifoldHyperConnection, _lib
    if isinstance(tile, str) and D != 256:
        pytest.skip("hidden split: D = 256 only")
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=True)
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    g = torch.Generator().manual_seed(T + D)
    x = torch.randn(T, D, generator=g).to(torch.bfloat16).to(gpu_device)
    res = torch.randn(T, D, generator=g).to(torch.bfloat16).to(gpu_device) if with_res else None
    v = _lib.MV_TOK | (_lib.MV_TOK16 if tile != 32 else 0)
    v |= {"split2": _lib.MV_TOKSPLIT2, "split4": _lib.MV_TOKSPLIT4,
          }.get(tile, 0)
    from hv_amd import ops
    with torch.no_grad():
        ops.launch_counts(reset=True)
        with run_options(mhc_variant=v):
            y1 = m.forward_tokens(x, residual=res).float().cpu().numpy()
            if isinstance(tile, str):       # deterministic (fixed part order), and the counters reset
                y1b = m.forward_tokens(x, residual=res).float().cpu().numpy()
                assert np.array_equal(y1, y1b)
        assert ops.launch_counts()["mhc_fused"] == (2 if isinstance(tile, str) else 1)
        with run_options(use_fused_mhc=False):
            y0 = m.forward_tokens(x, residual=res).float().cpu().numpy()
    assert rel_l2(y1, y0) < 1e-2
    assert np.abs(y1 - y0).max() < 0.1


@pytest.mark.parametrize("T", [401, 6416, 33])
def test_mhc_tok_group_equals_single_launches(gpu_device, T):
    """hv_mhc_fused_group: q / k / v (three sites on one x) in ONE launch give the same bits as
    three single launches of the token-tile kernel, and the attention block takes that path."""
    from hv_amd import ManifoldHyperConnection, _lib, ops
    from hv_amd.runtime import HVOptions, RunCtx, use_ctx
    ms = []
    for i in range(3):
        m = ManifoldHyperConnection(256, expansion_rate=2)
        W.load_formula_weights(m, "wc" if i != 1 else "init")
        ms.append(m.to(gpu_device).eval())
    x = torch.randn(T, 256, generator=torch.Generator().manual_seed(T)).to(torch.bfloat16).to(gpu_device)
    with torch.no_grad():
        for v in (_lib.MV_TOK, _lib.MV_TOK | _lib.MV_TOK16, _lib.MV_TOK | _lib.MV_TOK16 | _lib.MV_TOKSPLIT2,
                  _lib.MV_TOK | _lib.MV_TOK16 | _lib.MV_TOKSPLIT4):
            with use_ctx(RunCtx(dtype=torch.bfloat16, opts=HVOptions(mhc_variant=v))):
                plans = [m.plan() for m in ms]
                outs = ops.mhc_fused_group(x, plans, v)
                singles = [ops.mhc_fused(x, p.b1, p.c1, p.w2, p.bias2, p.wct, p.g_post, p.b_post, variant=v)
                           for p in plans]
            for a, b in zip(outs, singles):
                assert torch.equal(a, b)


def test_convmhc_and_blocks_fp32(gpu_device):
    from hv_amd import ConvMHCLayer, ResidualMHCLayer, TransformerEncoderBlock
    for (cin, cout, k, s, HW) in [(3, 32, 3, 2, 32), (64, 64, 3, 1, 16), (64, 128, 3, 2, 16)]:
        g = golden(f"convmhc_{cin}_{cout}_s{s}")
        m = ConvMHCLayer(cin, cout, kernel_size=k, stride=s)
        m.hv_precision = "fp32"
        W.load_formula_weights(m, "wc")
        m = m.to(gpu_device).eval()
        y = m(torch.from_numpy(g["x"]).to(gpu_device)).float().cpu().numpy()
        np.testing.assert_allclose(y, g["y"], rtol=0, atol=1e-3)
    g = golden("residual_128")
    m = ResidualMHCLayer(128, num_blocks=2, expansion_rate=4, bottleneck=True)
    m.hv_precision = "fp32"
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    np.testing.assert_allclose(m(torch.from_numpy(g["x"]).to(gpu_device)).cpu().numpy(), g["y"], rtol=0, atol=1e-3)
    g = golden("encblock_256_n50")
    m = TransformerEncoderBlock(embed_dim=256, num_heads=8)
    m.hv_precision = "fp32"
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    np.testing.assert_allclose(m(torch.from_numpy(g["x"]).to(gpu_device)).cpu().numpy(), g["y"], rtol=0, atol=1e-3)


# ------------------------------------------------------------------------------ full model
def _build(tag, fam, precision, device):
    from hv_amd import HybridVisionSystem
    m = HybridVisionSystem(dict(MODEL_CFG[tag], precision=precision))
    m.load_state_dict(formula_state_dict(tag, fam))
    return m.to(device).eval()


def _check_fp32(out, g, sub):
    for s in range(3):
        step = sub if s == 0 else 1
        pr = out["predictions"][f"scale_{s}"][:, :, ::step].cpu().numpy()
        np.testing.assert_allclose(pr, g[f"pred{s}_f64"], rtol=0, atol=1e-3)
        np.testing.assert_allclose(pr, g[f"pred{s}"], rtol=0, atol=2e-3)
        bx = out["decoded"][f"scale_{s}"]["boxes"][:, :, ::step].cpu().numpy()
        np.testing.assert_allclose(bx, g[f"boxes{s}"], rtol=1e-3, atol=1e-3)
        ci = out["decoded"][f"scale_{s}"]["class_indices"].cpu().numpy()
        sure = g[f"margin{s}"] >= 1e-4
        assert (ci[sure] == g[f"cls{s}_f64"][sure]).all(), f"class index mismatch at scale {s}"
    np.testing.assert_allclose(out["final_features"].cpu().numpy(), g["final_features_f64"], rtol=0, atol=1e-4)


@pytest.mark.parametrize("tag,tiny,fam,S,B,sub", cases.MODEL_CASES)
def test_model_fp32_matches_reference(gpu_device, tag, tiny, fam, S, B, sub):
    g = golden(f"model_{tag}")
    m = _build("tiny" if tiny else "base", fam, "fp32", gpu_device)
    x = cases.model_input(B, S).to(gpu_device)
    first = m(x, task="detection")["predictions"]["scale_2"].clone()   # discovers convs/linears
    out = m(x, task="detection")                                      # fully grouped prep
    assert torch.equal(first, out["predictions"]["scale_2"])
    _check_fp32(out, g, sub)
    assert set(out) >= {"backbone_features", "vit_features", "fused_features", "predictions", "decoded",
                        "final_features"}


@pytest.mark.parametrize("tag,tiny,fam,S,B,sub", [c for c in cases.MODEL_CASES if c[2] == "wc"])
def test_model_bf16_agreement(gpu_device, tag, tiny, fam, S, B, sub):
    g = golden(f"model_{tag}")
    m = _build("tiny" if tiny else "base", fam, "bf16", gpu_device)
    x = cases.model_input(B, S).to(gpu_device)
    first = m(x, task="detection")["predictions"]["scale_2"].clone()
    out = m(x, task="detection")
    assert torch.equal(first, out["predictions"]["scale_2"])
    agree = []
    for s in range(3):
        step = sub if s == 0 else 1
        pr = out["predictions"][f"scale_{s}"][:, :, ::step].cpu().numpy()
        assert rel_l2(pr, g[f"pred{s}_f64"]) < 0.1
        ci = out["decoded"][f"scale_{s}"]["class_indices"].cpu().numpy()
        sure = g[f"margin{s}"] >= 1e-2
        if sure.any():
            agree.append((ci[sure] == g[f"cls{s}_f64"][sure]).mean())
    assert agree and min(agree) > 0.9, agree


@pytest.mark.parametrize("S,B,fixture,nref", [(640, 16, "base_wc_640_b2", 2), (1024, 8, "base_wc_1024_b1", 1)])
def test_timed_step_graph_matches_reference(gpu_device, S, B, fixture, nref):
    """The exact object bench.py times -- base model, bf16, hipGraph replay of the whole forward
    (grouped Sinkhorn + coefficient prep + token path) -- at config B (640², B=16) and at config
    D's per-GPU shape (1024², B=8), where the big-grid kernels are selected (256x256 ping-pong
    GEMM, LDS-DMA tiles, fused mHC, MFMA attention over 401 / 1025 tokens).  Checked:
      * the graph replay equals the eager bf16 forward bit for bit, and the kernel families
        above actually ran (host launch counters, include/hv_tuning.h);
      * the first `nref` images (the reference fixture's input) agree with the reference's fp64
        run at the bf16 contract of test_model_bf16_agreement (rel-L2 < 0.1 on logits, >= 90%
        class agreement on cells with top-1/top-2 margin >= 1e-2);
      * at 640 they are ALSO held to the reference's own bf16 numerics (fixture
        model_base_wc_640_b2_bf16ref: the reference under CUDA autocast's bf16 policy, S8):
        logits (vs fp64), boxes (vs the reference fp32 run) and final features no worse than
        the reference's own bf16 error (ratio <= 0.5; measured 0.24-0.27, final features 0.09),
        class agreement no
        lower;
      * the fp32 HIP path on the same batch meets the fp32 contract on those images (atol 1e-3),
        and on EVERY image of the batch the bf16 step stays near the fp32 step: logits rel-L2
        < 0.1, final features < 0.05, boxes per scale < 1.5x the measured worst.  Measured
        (round-3 build, both configs, profiles/r03/parity/): logits 0.062-0.071, final 0.010,
        boxes 0.017 / 0.188 / 0.283 at scales 0/1/2 -- a box side is anchor * exp(t_wh), so its
        relative error IS the absolute logit error, which grows with |t| on the coarse scales.
      * every measured figure (per-scale worst rel-L2 over the batch, class agreement on the
        fixture images) is written to gpurun_out/parity/timed_step_<S>.json (profiles/r03/)."""
    from hv_amd import ops
    g = golden(f"model_{fixture}")
    sub = int(g["sub"])
    x = torch.cat([cases.model_input(nref, S),
                   torch.randn(B - nref, 3, S, S, generator=torch.Generator().manual_seed(2))]).to(gpu_device)
    m16 = _build("base", "wc", "bf16", gpu_device)
    with torch.no_grad():
        m16(x)                                            # discovers convs / linears
        ops.launch_counts(reset=True)
        eager = m16(x)
        counts = ops.launch_counts(reset=True)
        e_pred = {k: v.clone() for k, v in eager["predictions"].items()}
        e_final = eager["final_features"].clone()
        del eager
        runner = m16.capture(x)
        out = runner(x)
        torch.cuda.synchronize()
        for k in e_pred:
            assert torch.equal(out["predictions"][k], e_pred[k]), k
        assert torch.equal(out["final_features"], e_final)
        b16 = {"pred": {k: v.float().cpu().numpy() for k, v in out["predictions"].items()},
               "boxes": {k: v["boxes"].cpu().numpy() for k, v in out["decoded"].items()},
               "cls": {k: v["class_indices"].cpu().numpy() for k, v in out["decoded"].items()},
               "final": out["final_features"].cpu().numpy()}
        del runner, out, m16, e_pred, e_final
    torch.cuda.empty_cache()
    print("launch counts per forward:", counts)
    for fam in ("gemm_pp256", "mhc_fused", "attn_mfma", "sinkhorn_group"):
        assert counts[fam] > 0, (fam, counts)
    assert counts["glds_128x128"] + counts["glds_64x128"] + counts["glds_64x64"] + counts["glds_128x64"] > 0
    assert counts["attn_scalar"] == 0
    agree, anchor = [], {}
    gb = golden(f"model_{fixture}_bf16ref") if S == 640 else None
    for s in range(3):
        step = sub if s == 0 else 1
        pr = b16["pred"][f"scale_{s}"][:nref, :, ::step]
        e_log = rel_l2(pr, g[f"pred{s}_f64"])
        assert e_log < 0.1, s
        e_box = rel_l2(b16["boxes"][f"scale_{s}"][:nref, :, ::step], g[f"boxes{s}"])
        if gb is not None:
            # S8 anchor: the reference under its own autocast policy on the same images
            r_log, r_box = float(gb[f"pred{s}_err_vs_f64"]), float(gb[f"boxes{s}_err_vs_f32"])
            anchor[f"scale_{s}"] = {"logits_hip": round(e_log, 5), "logits_ref_bf16": round(r_log, 5),
                                    "logits_ratio": round(e_log / r_log, 4), "boxes_hip": round(e_box, 5),
                                    "boxes_ref_bf16": round(r_box, 5), "boxes_ratio": round(e_box / r_box, 4)}
            assert e_log <= 0.5 * r_log and e_box <= 0.5 * r_box, (s, anchor[f"scale_{s}"])
        ci = b16["cls"][f"scale_{s}"][:nref]
        sure = g[f"margin{s}"] >= 1e-2
        if sure.any():
            agree.append((ci[sure] == g[f"cls{s}_f64"][sure]).mean())
    assert agree and min(agree) > 0.9, agree
    rec = {"config": f"base {S}x{S} B={B} bf16 hipGraph replay", "fixture": fixture,
           "class_agreement_vs_ref_f64_margin_1e-2": [round(float(a), 5) for a in agree]}
    if gb is not None:
        e_fin = rel_l2(b16["final"][:nref], g["final_features_f64"])
        r_fin = float(gb["final_err_vs_f64"])
        anchor["final_features"] = {"hip": round(e_fin, 5), "ref_bf16": round(r_fin, 5), "ratio": round(e_fin / r_fin, 4)}
        anchor["class_agreement_ref_bf16"] = [round(float(a), 5) for a in gb["class_agreement_margin_1e-2"]]
        anchor["bound"] = "HIP bf16 error <= 0.5x the reference's own bf16 error (S8) on every output"
        rec["vs_reference_bf16"] = anchor
        assert e_fin <= 0.5 * r_fin, anchor
        assert min(agree) >= min(gb["class_agreement_margin_1e-2"]), (agree, anchor)
    m32 = _build("base", "wc", "fp32", gpu_device)
    with torch.no_grad():
        m32(x)
        o32 = m32(x)
        torch.cuda.synchronize()
    ref_g = {k: g[k][:nref] for k in g.files if k[:4] in ("pred", "boxe", "marg", "cls0", "cls1", "cls2")}
    ref_g.update({"final_features_f64": g["final_features_f64"][:nref]})
    sub_out = {"predictions": {k: v[:nref] for k, v in o32["predictions"].items()},
               "decoded": {k: {kk: vv[:nref] for kk, vv in v.items()} for k, v in o32["decoded"].items()},
               "final_features": o32["final_features"][:nref]}
    _check_fp32(sub_out, ref_g, sub)
    worst = {}
    for s in range(3):
        k = f"scale_{s}"
        p32 = o32["predictions"][k].cpu().numpy()
        bx32 = o32["decoded"][k]["boxes"].cpu().numpy()
        for i in range(B):
            worst[f"logits{s}"] = max(worst.get(f"logits{s}", 0), rel_l2(b16["pred"][k][i], p32[i]))
            worst[f"boxes{s}"] = max(worst.get(f"boxes{s}", 0), rel_l2(b16["boxes"][k][i], bx32[i]))
    f32 = o32["final_features"].cpu().numpy()
    worst["final"] = max(rel_l2(b16["final"][i], f32[i]) for i in range(B))
    rec["worst_image_rel_l2_bf16_graph_vs_fp32_hip"] = {k: round(float(v), 5) for k, v in worst.items()}
    rec["bounds"] = {"logits": 0.1, "final": 0.05, "boxes0": 0.026, "boxes1": 0.28, "boxes2": 0.42}
    record_parity(f"timed_step_{S}", rec)
    assert max(v for k, v in worst.items() if k.startswith("logits")) < 0.1, worst
    assert worst["final"] < 0.05, worst
    for s_, bound in enumerate((0.026, 0.28, 0.42)):      # 1.5x the measured worst per scale (r03)
        assert worst[f"boxes{s_}"] < bound, worst


def test_streaming_640_b1_frozen_graph_and_pipeline(gpu_device):
    """Config E's timed objects at their real shape: base model, bf16, 640x640, batch 1,
    coefficients frozen, hipGraph replay (scripts/inference.py:224-291 -> engine.infer,
    src/inference/engine.py:251-317).
      (1) The frozen B=1 GraphRunner (bench.py's `latency` leg) on image 0 of the reference
          fixture model_base_wc_640_b2: the bf16 contract against the reference's fp64 run
          (logits rel-L2 < 0.1, >= 90% class agreement on margin >= 1e-2 cells); the fp32 HIP
          forward of the same image meets the fp32 contract (atol 1e-3, bit-exact margin-filtered
          class indices); the graph equals the eager frozen forward bit for bit.
      (2) StreamingPipeline (1280x720 uint8 BGR frame -> Pillow-exact resize -> graphed forward
          -> graphed hv_nms, what bench.py's `streaming` leg times) returns exactly the detections
          of the reference post_process (restated in oracle/hv_oracle.py, pinned by the nms_*
          fixtures) run on the decode of the same bf16 frozen forward, bit for bit; and the fp32
          forward's 25 strongest detections on the same preprocessed frame are found in it (a box
          with IoU >= 0.5; label agreement recorded).
    The measured figures go to gpurun_out/parity/streaming_640_b1.json."""
    from hv_amd import ops
    from hv_amd.engine import StreamingPipeline
    from oracle import hv_oracle as O
    g = golden("model_base_wc_640_b2")
    sub = int(g["sub"])
    x = cases.model_input(2, 640)[:1].contiguous().to(gpu_device)
    rec = {"config": "base 640x640 B=1 bf16, frozen coefficients, hipGraph replay"}
    m16 = _build("base", "wc", "bf16", gpu_device).freeze()
    with torch.no_grad():
        eager = m16(x)
        e_pred = {k: v.clone() for k, v in eager["predictions"].items()}
        del eager
        runner = m16.capture(x)
        out = runner(x)
        torch.cuda.synchronize()
        for k in e_pred:
            assert torch.equal(out["predictions"][k], e_pred[k]), k
        b16 = {k: v.float().cpu().numpy() for k, v in out["predictions"].items()}
        c16 = {k: v["class_indices"].cpu().numpy() for k, v in out["decoded"].items()}
        del runner, out
    agree, rels = [], []
    for s in range(3):
        step = sub if s == 0 else 1
        pr = b16[f"scale_{s}"][:, :, ::step]
        rels.append(rel_l2(pr, g[f"pred{s}_f64"][:1]))
        ci = c16[f"scale_{s}"]
        sure = g[f"margin{s}"][:1] >= 1e-2
        if sure.any():
            agree.append(float((ci[sure] == g[f"cls{s}_f64"][:1][sure]).mean()))
    rec["graph_vs_ref_f64"] = {"logits_rel_l2": [round(r, 5) for r in rels], "class_agreement_margin_1e-2": agree}
    assert max(rels) < 0.1, rels
    assert agree and min(agree) > 0.9, agree
    m32 = _build("base", "wc", "fp32", gpu_device)
    with torch.no_grad():
        o32 = m32(x)
    ref_g = {k: g[k][:1] for k in g.files if k[:4] in ("pred", "boxe", "marg", "cls0", "cls1", "cls2")}
    ref_g["final_features_f64"] = g["final_features_f64"][:1]
    _check_fp32(o32, ref_g, sub)
    rec["bf16_vs_fp32_logits_rel_l2"] = [round(rel_l2(b16[f"scale_{s}"], o32["predictions"][f"scale_{s}"].cpu().numpy()), 5)
                                         for s in range(3)]
    # (2) the streaming pipeline on camera frames
    conf, iou, md = 0.25, 0.45, 100
    pipe = StreamingPipeline(m16, (720, 1280), (640, 640), conf_threshold=conf, iou_threshold=iou, max_detections=md)
    matched_all, n_all, same_label, counts, cands = 0, 0, 0, [], []
    for i, fr in enumerate(cases.camera_frames(60, 2, 720, 1280)):
        got = pipe(fr)
        with torch.no_grad():
            fd = torch.from_numpy(fr[None]).to(gpu_device)
            xin = ops.preprocess(fd, 640, 640, bgr=True, dtype=torch.bfloat16, nhwc=True, resample="pil")
            dec16 = m16(xin)["decoded"]                  # the pipeline's own composition, eager
            ref = O.post_process({k: {n: v[n].cpu() for n in ("boxes", "class_scores", "class_indices")}
                                  for k, v in dec16.items()}, conf, iou, md)[0]
            det32 = m32.detect(ops.preprocess(fd, 640, 640, resample="pil"), conf + 0.05, iou, md)[0]
        counts.append(len(got["scores"]))
        # candidates per scale above the threshold, and how many of them share a score (the tie
        # order the exact sort reproduces)
        cs = {k: v["class_scores"].reshape(-1) for k, v in sorted(dec16.items())}
        cands.append({k: {"candidates": int((v > conf).sum()),
                          "tied": int(v[v > conf].numel() - torch.unique(v[v > conf]).numel())}
                      for k, v in cs.items()})
        assert len(got["scores"]) == ref["scores"].numel() > 0, (i, len(got["scores"]), ref["scores"].numel())
        np.testing.assert_array_equal(got["scores"], ref["scores"].numpy())
        np.testing.assert_array_equal(got["labels"], ref["labels"].numpy())
        np.testing.assert_array_equal(got["boxes"], ref["boxes"].numpy())
        # the fp32 forward's strongest detections (top 25 by score: below that the max_det cut and
        # the near-uniform class scores of a random-init model reorder freely) found in the bf16
        # pipeline's output: a box with IoU >= 0.5 (any label), and whether its label agrees
        top = det32["scores"].cpu().argsort(descending=True)[:25]
        b32, l32 = det32["boxes"].cpu()[top], det32["labels"].cpu()[top]
        gb, gl = torch.from_numpy(got["boxes"]), torch.from_numpy(got["labels"])
        for j in range(b32.shape[0]):
            ious = O._iou(b32[j:j + 1], gb)
            if ious.numel() and ious.max().item() >= 0.5:
                matched_all += 1
                same_label += int(gl[int(ious.argmax())] == l32[j])
        n_all += b32.shape[0]
    assert pipe.recaptures == 0
    frac = matched_all / max(n_all, 1)
    rec["pipeline"] = {"frames": 2, "detections_per_frame": counts, "candidates_per_scale": cands,
                       "fp32_top_detections": n_all,
                       "fp32_top_matched_by_bf16_box_iou_0.5": round(frac, 4),
                       "label_agreement_of_matched": round(same_label / max(matched_all, 1), 4)}
    record_parity("streaming_640_b1", rec)
    assert n_all == 0 or frac >= 0.7, rec["pipeline"]     # measured 0.86 (label agreement 0.95)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_graph_capture_replays_the_eager_forward(gpu_device, precision):
    """The hipGraph-captured step (Sinkhorn + prep + token path) equals the eager forward."""
    m = _build("tiny", "wc", precision, gpu_device)
    x = cases.model_input(2, 224).to(gpu_device)
    with torch.no_grad():
        ref = m(x)
        runner = m.capture(x)
        out = runner(x)
        for s in range(3):
            assert torch.equal(out["predictions"][f"scale_{s}"], ref["predictions"][f"scale_{s}"])
        assert torch.equal(out["final_features"], ref["final_features"])
        x2 = x.flip(-1).contiguous()
        out2 = runner(x2)["predictions"]["scale_0"].clone()
        assert torch.equal(out2, m(x2)["predictions"]["scale_0"])


def test_inference_engine_api(gpu_device):
    """InferenceEngine (reference src/inference/engine.py) over the HIP model: infer on a uint8
    BGR frame, the graph-replay streaming path, infer_batch splitting, stats."""
    import numpy as np
    from inference.engine import InferenceConfig, InferenceEngine
    m = _build("tiny", "wc", "fp32", gpu_device)
    cfg = InferenceConfig(device=str(gpu_device), use_half_precision=False, warmup_iterations=1,
                          input_height=128, input_width=128, use_graphs=True)
    eng = InferenceEngine(cfg, m)
    frame = np.random.default_rng(0).integers(0, 255, (96, 160, 3), dtype=np.uint8)
    r = eng.infer(frame)
    assert r["batch_size"] == 1 and r["outputs"]["predictions"]["scale_0"].shape[0] == 1
    m.freeze(False)
    direct = m(eng._to_tensor(frame)[None], task="detection")["predictions"]["scale_0"]
    assert torch.allclose(r["outputs"]["predictions"]["scale_0"], direct, atol=1e-5)
    rs = eng.infer_batch([frame, frame[:, ::-1]])
    assert len(rs) == 2 and rs[1]["outputs"]["predictions"]["scale_0"].shape[0] == 1
    assert eng.get_performance_stats()["total_inferences"] == 1


def test_model_deterministic_and_frozen_cache(gpu_device):
    m = _build("tiny", "wc", "fp32", gpu_device)
    x = cases.model_input(2, 224).to(gpu_device)
    a = m(x)["predictions"]["scale_2"].clone()
    m.freeze()
    b = m(x)["predictions"]["scale_2"].clone()
    c = m(x)["predictions"]["scale_2"].clone()
    assert torch.equal(a, b) and torch.equal(b, c)


@pytest.mark.parametrize("D,T", [(32, 1000), (64, 777), (128, 300)])
def test_mhc_fused_workgroup_shapes_bitwise_equal(gpu_device, D, T):
    """The 4-wave (default) and 8-wave workgroup shapes of hv_mhc_fused give identical bits:
    every wave computes its own tokens end to end, only the barrier grouping differs."""
    from hv_amd import ManifoldHyperConnection, _lib
    m = ManifoldHyperConnection(D, expansion_rate=4, use_mixed_precision=True)
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    x = torch.randn(T, D, generator=torch.Generator().manual_seed(T)).to(torch.bfloat16).to(gpu_device)
    with torch.no_grad():
        with run_options(mhc_variant=_lib.MV_ONE_GROUP8):
            y8 = m.forward_tokens(x).cpu()
        # D=128: the per-wave 4-wave kernel (default is split-hidden)
        with run_options(mhc_variant=_lib.MV_PERWAVE128 if D == 128 else 0):
            y4 = m.forward_tokens(x).cpu()
    assert torch.equal(y4, y8)


@pytest.mark.parametrize("D,T,with_res", [(32, 1000, False), (32, 777, True), (64, 777, False), (64, 4097, True),
                                           (64, 100, True)])
def test_mhc_fused_pipelined_bitwise_equal(gpu_device, D, T, with_res):
    """The software-pipelined per-wave kernel (3-stage weight ring, GEMM1+GELU of chunk c+1 beside
    GEMM2 of chunk c, Wc^T resident for GEMM3) computes exactly the per-wave kernel's arithmetic:
    bitwise equal to it, with and without the unmerged fragment reads, ragged T, residual."""
    from hv_amd import ManifoldHyperConnection, _lib
    m = ManifoldHyperConnection(D, expansion_rate=4, use_mixed_precision=True)
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    g = torch.Generator().manual_seed(T + D)
    x = torch.randn(T, D, generator=g).to(torch.bfloat16).to(gpu_device)
    res = torch.randn(T, D, generator=g).to(torch.bfloat16).to(gpu_device) if with_res else None
    with torch.no_grad():
        ys = {}
        for v in (_lib.MV_PERWAVE, _lib.MV_PIPE, _lib.MV_PIPE_NOMERGE, 0):
            with run_options(mhc_variant=v):
                ys[v] = m.forward_tokens(x, residual=res).cpu()
    for v in (_lib.MV_PIPE, _lib.MV_PIPE_NOMERGE, 0):
        assert torch.equal(ys[v], ys[_lib.MV_PERWAVE]), v


def test_graph_survives_option_change(gpu_device):
    """A GraphRunner keeps the buffers its graph reads outside the graph pool (the grouped
    Sinkhorn / coefficient-prep program of the capture's RunCtx): set_options() after a capture
    rebuilds the model's caches, and the first runner must still replay correctly."""
    from hv_amd import _lib
    m = _build("tiny", "wc", "bf16", gpu_device)
    x = torch.randn(2, 3, 128, 128, generator=torch.Generator().manual_seed(9)).to(gpu_device)
    with torch.no_grad():
        m.set_options(mhc_variant=_lib.MV_PERWAVE)
        ref = {k: v.clone() for k, v in m(x)["predictions"].items()}
        ra = m.capture(x)
        m.set_options(mhc_variant=_lib.MV_PIPE)
        rb = m.capture(x)
        torch.cuda.empty_cache()
        a = ra(x, owned=True)["predictions"]
        b = rb(x, owned=True)["predictions"]
        torch.cuda.synchronize()
    for k in ref:
        assert torch.equal(a[k], ref[k]), k
        assert torch.equal(b[k], ref[k]), k


def test_graph_capture_concurrent_with_eager_forwards(gpu_device):
    """The engine's worker pool (reference src/inference/engine.py:389-471, 4 workers :577,611-615)
    may run eager forwards while another thread captures: the runner pins the RunCtx ITS capture
    forward ran under (forward_eval returns it; nothing per call is stored on the module), so a
    concurrent forward cannot make it pin a foreign context; the capture runs in thread-local
    capture mode, so the other thread's launches and allocations do not invalidate it.  After the other thread's contexts are dropped and the
    cache freed, the replay still equals the eager forward bit for bit."""
    import threading
    from hv_amd import _lib
    m = _build("tiny", "wc", "bf16", gpu_device)
    x = torch.randn(2, 3, 128, 128, generator=torch.Generator().manual_seed(11)).to(gpu_device)
    with torch.no_grad():
        ref = {k: v.clone() for k, v in m(x)["predictions"].items()}
    stop, errors, seen = threading.Event(), [], []

    def worker():
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s), torch.no_grad():
                while not stop.is_set():
                    out, ctx = m.forward_eval(x)
                    seen.append(id(ctx))
                    s.synchronize()
                    del out, ctx
        except Exception as e:                     # noqa: BLE001  (reported by the main thread)
            errors.append(repr(e))

    t = threading.Thread(target=worker)
    t.start()
    try:
        with torch.no_grad():
            runner = m.capture(x)
    finally:
        stop.set()
        t.join(timeout=60)
    assert not t.is_alive() and not errors, errors
    assert seen and runner.ctx is not None and runner.ctx.plans
    with torch.no_grad():
        m.set_options(mhc_variant=_lib.MV_PIPE)       # drops the model's caches
        torch.cuda.empty_cache()
        out = runner(x, owned=True)["predictions"]
        torch.cuda.synchronize()
    for k in ref:
        assert torch.equal(out[k], ref[k]), k


def test_model_pipelined_mhc_bitwise_equal(gpu_device):
    """In the base model at 640^2 (stem / stage-1 fused sites at T = 409,600 / 102,400 tokens per
    4 images): the pipelined per-wave fused mHC kernel leaves the whole forward bitwise unchanged,
    eager and as a captured graph."""
    from hv_amd import _lib
    m = _build("base", "wc", "bf16", gpu_device)
    x = torch.randn(4, 3, 640, 640, generator=torch.Generator().manual_seed(5)).to(gpu_device)
    with torch.no_grad():
        m.set_options(mhc_variant=_lib.MV_PERWAVE)
        a = {k: v.clone() for k, v in m(x)["predictions"].items()}
        m.set_options(mhc_variant=_lib.MV_PIPE_NOMERGE)
        b = {k: v.clone() for k, v in m(x)["predictions"].items()}
        runner = m.capture(x)
        c = runner(x, owned=True)["predictions"]
        torch.cuda.synchronize()
    for k in a:
        assert torch.equal(a[k], b[k]), k
        assert torch.equal(a[k], c[k]), k


@pytest.mark.parametrize("T,with_res", [(64, False), (200, True), (1000, False), (6417, True)])
def test_mhc_fused_split_hidden_matches_unfused(gpu_device, T, with_res):
    """The split-hidden D=128 kernel (the default: hidden dimension across 4 waves, split-K
    GEMM3 reduced in LDS) vs the unfused six-launch chain and the per-wave fused kernel (bf16),
    ragged T, residual; deterministic (two runs bitwise equal)."""
    from hv_amd import ManifoldHyperConnection, _lib
    m = ManifoldHyperConnection(128, expansion_rate=4, use_mixed_precision=True)
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    g = torch.Generator().manual_seed(T)
    x = torch.randn(T, 128, generator=g).to(torch.bfloat16).to(gpu_device)
    res = torch.randn(T, 128, generator=g).to(torch.bfloat16).to(gpu_device) if with_res else None
    with torch.no_grad():
        with run_options():
            y3 = m.forward_tokens(x, residual=res).float().cpu()
            y3b = m.forward_tokens(x, residual=res).float().cpu()
        with run_options(mhc_variant=_lib.MV_ONE_GROUP8):
            y2 = m.forward_tokens(x, residual=res).float().cpu()
        with run_options(use_fused_mhc=False):
            y0 = m.forward_tokens(x, residual=res).float().cpu()
    assert torch.equal(y3, y3b)
    assert rel_l2(y3.numpy(), y0.numpy()) < 1e-2 and (y3 - y0).abs().max() < 0.1
    assert rel_l2(y3.numpy(), y2.numpy()) < 1e-2


@pytest.mark.parametrize("D,e,T,with_res", [(256, 2, 64, False), (256, 2, 401, True), (256, 2, 6416, False),
                                             (256, 2, 25601, True), (128, 4, 6417, True)])
def test_mhc_fused_split_hidden_d256_and_splitw(gpu_device, D, e, T, with_res):
    """The split-hidden kernel at D = 256 (Hd = 512: the ViT / FPN / head sites; one 4-wave group
    of 64 tokens per workgroup, GEMM3 in eight 32-column parts, two x chunks per quarter wave)
    and its split-wait form (variant 12: the chunk loop leaves the W2 half of chunk c+2 in
    flight) vs the unfused chain (bf16): ragged T, residual; the split-wait form is bitwise equal
    to the plain one (same arithmetic, other waits) and both are deterministic."""
    from hv_amd import ManifoldHyperConnection, _lib, ops
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=True)
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    g = torch.Generator().manual_seed(T + D)
    x = torch.randn(T, D, generator=g).to(torch.bfloat16).to(gpu_device)
    res = torch.randn(T, D, generator=g).to(torch.bfloat16).to(gpu_device) if with_res else None
    # forced: the automatic policy takes the token-tile kernel at these D = 128 token counts
    v = _lib.MV_SPLIT256 if D == 256 else _lib.MV_WIDE
    with torch.no_grad():
        with run_options(mhc_variant=v):
            ops.launch_counts(reset=True)
            y1 = m.forward_tokens(x, residual=res).float().cpu()
            assert ops.launch_counts()["mhc_fused"] == 1
            y1b = m.forward_tokens(x, residual=res).float().cpu()
        with run_options(mhc_variant=v | _lib.MV_SPLITW):
            y2 = m.forward_tokens(x, residual=res).float().cpu()
        with run_options(use_fused_mhc=False):
            y0 = m.forward_tokens(x, residual=res).float().cpu()
    assert torch.equal(y1, y1b)
    assert torch.equal(y1, y2)
    assert rel_l2(y1.numpy(), y0.numpy()) < 1e-2 and (y1 - y0).abs().max() < 0.1


# ------------------------------------------------------------------------------ call-site surface (§8b)
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_attention_cross_mask_weights_match_reference(gpu_device, precision):
    """MultiHeadManifoldAttention(query, key, value, key_padding_mask, need_weights) -- the
    general call form of manifold_layers.py:386-434 -- against the reference's own outputs."""
    from hv_amd import MultiHeadManifoldAttention
    g = golden("attn_cross_mask")
    m = MultiHeadManifoldAttention(256, num_heads=8)
    for mod in (m.q_proj, m.k_proj, m.v_proj, m.out_proj):
        mod.hv_precision = precision
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    q, kv, mask = (torch.from_numpy(g[k]).to(gpu_device) for k in ("q", "kv", "mask"))
    out, w = m(q, kv, kv, key_padding_mask=mask, need_weights=True)
    out_n, w_n = m(q, kv, kv)
    out_self, _ = m(q, q, q)
    assert w_n is None and w.shape == (2, 8, 7, 11)
    if precision == "fp32":
        np.testing.assert_allclose(out.cpu().numpy(), g["out"], rtol=0, atol=1e-3)
        np.testing.assert_allclose(w.cpu().numpy(), g["weights"], rtol=0, atol=1e-5)
        np.testing.assert_allclose(out_self.cpu().numpy(), g["out_self"], rtol=0, atol=1e-3)
    else:
        assert rel_l2(out.float().cpu().numpy(), g["out"]) < 5e-2
        assert rel_l2(w.cpu().numpy(), g["weights"]) < 5e-2
        assert rel_l2(out_self.float().cpu().numpy(), g["out_self"]) < 5e-2
    assert (w.cpu()[0, :, :, ::3] == 0).all() and (w.cpu()[1, :, :, 8:] == 0).all()
    # every key masked: softmax over -inf gives NaN in the reference, and here
    full = torch.ones(2, 11, dtype=torch.bool, device=gpu_device)
    o_nan, w_nan = m(q, kv, kv, key_padding_mask=full, need_weights=True)
    assert torch.isnan(w_nan).all()


def test_vit_return_features_and_extract(gpu_device):
    """VisionTransformerEncoder.forward(return_features=True) -> (output, [embedding, block
    outputs...]) and extract_features (vit_encoder_decoder.py:277-333)."""
    from hv_amd import VisionTransformerEncoder
    from oracle import hv_oracle as O
    enc = VisionTransformerEncoder(image_size=16, patch_size=1, in_channels=64, embed_dim=256, depth=2,
                                   num_heads=8, num_classes=10)
    enc.hv_precision = "fp32"
    for mod in enc.modules():
        if hasattr(mod, "hv_precision"):
            mod.hv_precision = "fp32"
    W.load_formula_weights(enc, "wc")
    enc = enc.to(gpu_device).eval()
    x = torch.randn(2, 64, 6, 6, generator=torch.Generator().manual_seed(3)).to(gpu_device)
    out, feats = enc(x, return_features=True)
    assert out.shape == (2, 10) and len(feats) == 3 and all(f.shape == (2, 37, 256) for f in feats)
    torch.testing.assert_close(out, enc(x), rtol=0, atol=1e-5)     # enc(x): CLS-only last block
    cls = enc.extract_features(x)
    sd = {k: v.detach().cpu() for k, v in enc.state_dict().items()}
    ref_tok = O.rmsnorm(feats[-1].float().cpu(), sd["norm.scale"])[:, 0]
    np.testing.assert_allclose(cls.float().cpu().numpy(), ref_tok.numpy(), rtol=0, atol=1e-4)
    head = torch.nn.functional.linear(ref_tok, sd["head.weight"], sd["head.bias"])
    np.testing.assert_allclose(out.float().cpu().numpy(), head.numpy(), rtol=0, atol=1e-4)


def test_forward_emits_detections(gpu_device):
    """outputs['detections'] (read at scripts/inference.py:121, mhc_trainer.py:246): per scale
    [B, A, H, W, 5+C] = (xyxy box, objectness, class probabilities), the per-scale layout of
    DetectionPostprocessor._extract_predictions (postprocessing.py:234-244)."""
    m = _build("tiny", "wc", "fp32", gpu_device)
    x = cases.model_input(2, 224).to(gpu_device)
    out = m(x)
    assert set(out["detections"]) == {"small_scale", "medium_scale", "large_scale"}
    for s, key in enumerate(("small_scale", "medium_scale", "large_scale")):
        d = out["detections"][key]
        dec = out["decoded"][f"scale_{s}"]
        assert d.shape[:-1] == dec["boxes"].shape[:-1] and d.shape[-1] == 85
        assert torch.equal(d[..., :4], dec["boxes"])
        assert torch.equal(d[..., 4:5], dec["objectness"])
        torch.testing.assert_close(d[..., 5:] * d[..., 4:5], dec["scores"], rtol=1e-6, atol=1e-7)
        cls = torch.sigmoid(out["predictions"][f"scale_{s}"][..., 5:])
        torch.testing.assert_close(d[..., 5:], cls, rtol=1e-5, atol=1e-6)


def test_engine_owned_outputs_recapture_and_stability(gpu_device):
    """Streaming engine semantics: infer() results are owned (a later frame does not overwrite
    an earlier result), a parameter change after the graph was captured (frozen coefficients)
    is picked up by re-capturing, and every result carries the lazy stability metrics."""
    from inference.engine import InferenceConfig, InferenceEngine
    m = _build("tiny", "wc", "fp32", gpu_device)
    cfg = InferenceConfig(device=str(gpu_device), use_half_precision=False, warmup_iterations=1,
                          input_height=128, input_width=128, use_graphs=True)
    eng = InferenceEngine(cfg, m)
    g = torch.Generator().manual_seed(5)
    f1, f2 = (torch.randn(1, 3, 128, 128, generator=g).to(gpu_device) for _ in range(2))
    r1 = eng.infer(f1)
    keep = r1["outputs"]["predictions"]["scale_1"].clone()
    r2 = eng.infer(f2)
    assert torch.equal(r1["outputs"]["predictions"]["scale_1"], keep)
    assert not torch.equal(r2["outputs"]["predictions"]["scale_1"], keep)
    assert r1["outputs"]["predictions"]["scale_1"].data_ptr() != r2["outputs"]["predictions"]["scale_1"].data_ptr()
    st = r2["stability_metrics"]
    assert any(k.endswith("max_eigenvalue") for k in st) and len(st) > 0
    # in-place weight update (load_state_dict copies into the same storage)
    sd = {k: (v * 1.5 if k.endswith("pred_conv.weight") else v) for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    r3 = eng.infer(f2)
    assert eng._runner.recaptures == 1
    m.freeze(False)
    direct = m(f2)["predictions"]["scale_1"]
    torch.testing.assert_close(r3["outputs"]["predictions"]["scale_1"], direct, rtol=0, atol=1e-5)
    assert not torch.equal(r3["outputs"]["predictions"]["scale_1"], r2["outputs"]["predictions"]["scale_1"])


def test_graph_runner_recaptures_before_replay_on_storage_changes(gpu_device):
    """GraphRunner checks runtime.VersionWatch BEFORE it replays: a `.data` swap of a parameter
    (the old storage is freed), a rebound Sinkhorn history buffer (storage the graph WRITES) and
    a `_buffers[...]` rebind as `.to()` does it (no registration hook) each trigger a re-capture,
    the result equals the eager forward on the new storage, and the graph writes the new history
    buffer."""
    m = _build("tiny", "wc", "fp32", gpu_device)
    x = cases.model_input(2, 224).to(gpu_device)
    mods = dict(m.named_modules())
    with torch.no_grad():
        runner = m.capture(x)
        runner(x)
        assert runner.recaptures == 0

        def check(n):
            out = runner(x)["predictions"]["scale_1"].clone()
            assert runner.recaptures == n
            assert torch.equal(out, m(x)["predictions"]["scale_1"])
            runner(x)                                   # nothing changed: no further capture
            assert runner.recaptures == n
        conv = mods["detection_head.pred_heads.1.pred_conv"]
        conv.bias.data = conv.bias.data * 1.3 + 0.1     # new storage, old one freed
        torch.cuda.empty_cache()
        check(1)
        sk = mods["detection_head.pred_heads.1.mhc_enhance.sinkhorn"]
        sk.convergence_history = torch.full_like(sk.convergence_history, -7.0)   # rebound output buffer
        check(2)
        assert (sk.convergence_history != -7.0).all()  # the re-captured graph wrote the new buffer
        bn = mods["backbone.stem.1.bn"]
        bn._buffers["running_mean"] = bn.running_mean + 0.05                       # .to()-style rebind
        check(3)


def test_streaming_pipeline_matches_eager_path(gpu_device):
    """Config E's pipeline (StreamingPipeline: uint8 camera frame -> Pillow-exact preprocessing
    -> graphed forward -> graphed NMS -> host) returns exactly the detections of the eager path
    on the same frame (ops.preprocess -> model.detect), keeps returning correct results across
    frames, and re-captures after an in-place weight change."""
    from hv_amd import ops
    from inference.engine import StreamingPipeline
    m = _build("tiny", "wc", "fp32", gpu_device)
    frames = [cases.camera_frames(40 + i, 1, 96, 160)[0] for i in range(3)]
    pipe = StreamingPipeline(m, (96, 160), (128, 128), conf_threshold=0.05, iou_threshold=0.45, max_detections=50)

    def eager(fr):
        x = ops.preprocess(torch.from_numpy(fr[None]).to(gpu_device), 128, 128, resample="pil")
        return m.detect(x, 0.05, 0.45, 50)[0]
    for fr in frames + frames[:1]:
        got = pipe(fr)
        ref = eager(fr)
        assert len(got["scores"]) == ref["scores"].numel() > 0
        np.testing.assert_array_equal(got["scores"], ref["scores"].cpu().numpy())
        np.testing.assert_array_equal(got["labels"], ref["labels"].cpu().numpy())
        np.testing.assert_array_equal(got["boxes"], ref["boxes"].cpu().numpy())
    sd = {k: (v * 1.3 if k.endswith("pred_conv.bias") else v) for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    got = pipe(frames[1])
    assert pipe.recaptures == 1
    m.freeze(False)
    ref = eager(frames[1])
    np.testing.assert_array_equal(got["scores"], ref["scores"].cpu().numpy())


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_vit_shortcuts_match_plain_path(gpu_device, precision):
    """The inference-path restructurings of the encoder are exact: the CLS-only last block
    (only the CLS row survives, vit_encoder_decoder.py:308-311), the q/k/v projections on
    three streams and the grouped q/k/v GEMM1 give the plain path's vit features (fp32: 1e-5; bf16: same GEMM kernels on
    fewer rows -> rounding-level)."""
    m = _build("base", "wc", precision, gpu_device)
    x = cases.model_input(2, 224).to(gpu_device)
    outs = {}
    for cls_only, par, grp in ((True, True, False), (False, False, False), (True, False, False),
                               (True, False, True)):
        m.set_options(cls_only_last_block=cls_only, parallel_qkv=par, group_qkv=grp)   # per model
        with torch.no_grad():
            o = m(x)
        outs[(cls_only, par, grp)] = (o["vit_features"].float().cpu(), o["predictions"]["scale_2"].cpu())
    ref_v, ref_p = outs[(False, False, False)]
    tol = 1e-5 if precision == "fp32" else 2e-2
    for key, (v, p) in outs.items():
        assert (v - ref_v).abs().max().item() <= tol * max(1.0, ref_v.abs().max().item()), key
    assert torch.equal(outs[(True, True, False)][0], outs[(True, False, False)][0])   # streams change no bits


def test_device_tables_hold_every_pointer(gpu_device):
    """hv_amd/tables.py on the live programs (verdict r5 item 7): after an eval forward (prep
    program + its Sinkhorn group), a post_process (NMS plan) and a training step (grouped training
    prep, its Sinkhorn group, the optimizer table), every pointer in every recorded device table
    lies in a tensor the owning program holds."""
    from hv_amd import HybridVisionSystem, ops, tables
    from hv_amd.targets import synthetic_targets
    from hv_amd.trainer import HVTrainer
    m = HybridVisionSystem(dict(num_blocks=[1, 1, 1, 1], vit_depth=1, sk_iters=5, verbose=False))
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    x = torch.randn(2, 3, 96, 96, device=gpu_device)
    with torch.no_grad():
        out = m(x)
    prog = m._sk_cache["program"]
    plan = ops.NmsPlan(out["decoded"], 0.05, 0.5, 50)
    plan.run()
    m.train()
    tr = HVTrainer(m, lr=1e-3, monitor_every=0)
    tr.step(x, [t.to(gpu_device) for t in synthetic_targets(2, 96, seed=3)])
    torch.cuda.synchronize()
    entry = m.__dict__["_train_prep_cache"]["pool"][0]
    owners = {"prep program": prog, "prep sinkhorn": prog.sk, "nms plan": plan, "train prep": entry["prep"],
              "train sinkhorn": entry["sk"], "optimizer": tr.opt}
    for what, o in owners.items():
        assert tables._TABLES in o.__dict__, what
        assert tables.unheld_pointers(o) == [], what


def test_prep_overlap_equals_serial_prep(gpu_device):
    """HVOptions.prep_overlap (the Sinkhorn group + mHC coefficient prep on a side stream beside the
    weight prep and the first layers; default from batch 8): the eager forward and a captured
    graph's replay give bit-identical outputs with and without it."""
    from hv_amd import HybridVisionSystem
    m = HybridVisionSystem(dict(num_blocks=[1, 1, 1, 1], vit_depth=2, sk_iters=5, verbose=False))
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    x = torch.randn(8, 3, 96, 96, generator=torch.Generator().manual_seed(4)).to(gpu_device)
    outs = {}
    for on in (False, True):
        m.set_options(prep_overlap=on, prep_overlap_min_batch=1 << 30)
        with torch.no_grad():
            eager = {k: v.clone() for k, v in m(x)["predictions"].items()}
            runner = m.capture(x)
            g = {k: v.clone() for k, v in runner.replay()["predictions"].items()}
        torch.cuda.synchronize()
        outs[on] = (eager, g)
        del runner
    for s in outs[False][0]:
        assert torch.equal(outs[False][0][s], outs[True][0][s]), s
        assert torch.equal(outs[False][1][s], outs[True][1][s]), s
        assert torch.equal(outs[True][0][s], outs[True][1][s]), s
