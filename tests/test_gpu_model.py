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

from conftest import MODEL_CFG, formula_state_dict, golden
from oracle import cases
from oracle import weights as W

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


# ------------------------------------------------------------------------------ mHC layer
@pytest.mark.parametrize("fam", ["wc", "init"])
@pytest.mark.parametrize("D,e", cases.MHC_CASES)
def test_mhc_fp32_matches_reference(gpu_device, fam, D, e):
    from hv_amd import ManifoldHyperConnection
    from hv_amd import manifold as MF
    g = golden(f"mhc_{fam}_D{D}_e{e}")
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=False)
    W.load_formula_weights(m, fam)
    m = m.to(gpu_device).eval()
    x = cases.mhc_input(D, e).to(gpu_device)
    for fold in (True, False):
        old = MF.FOLD_MAX_D
        MF.FOLD_MAX_D = 4096 if fold else 0
        try:
            y = m(x).cpu().numpy()
        finally:
            MF.FOLD_MAX_D = old
        np.testing.assert_allclose(y, g["y64"], rtol=0, atol=1e-3)
        np.testing.assert_allclose(y, g["y"], rtol=0, atol=1e-3)


@pytest.mark.parametrize("D,e", cases.MHC_CASES)
def test_mhc_bf16_agreement(gpu_device, D, e):
    from hv_amd import ManifoldHyperConnection
    g = golden(f"mhc_wc_D{D}_e{e}")
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=True)
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    y = m(cases.mhc_input(D, e).to(gpu_device)).float().cpu().numpy()
    # bf16 activations, fp32 coefficients; centred coefficients keep this at the bf16 level
    assert rel_l2(y, g["y64"]) < 5e-2


@pytest.mark.parametrize("D,e,T,with_res", [(32, 4, 64, False), (32, 4, 1000, False), (64, 4, 64, False),
                                             (64, 4, 777, False), (128, 4, 200, False), (256, 2, 401, False),
                                             (256, 2, 130, True)])
def test_mhc_fused_kernel_matches_unfused_chain(gpu_device, D, e, T, with_res):
    """hv_mhc_fused (one launch, on-chip intermediates) vs the six-launch chain, both bf16."""
    from hv_amd import ManifoldHyperConnection
    from hv_amd import manifold as MF
    from hv_amd.runtime import RunCtx, use_ctx
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=True)
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    g = torch.Generator().manual_seed(T)
    x = torch.randn(T, D, generator=g).to(torch.bfloat16).to(gpu_device)
    res = torch.randn(T, D, generator=g).to(torch.bfloat16).to(gpu_device) if with_res else None
    from hv_amd import _lib
    _lib.lib().hv_mhc_fused_enable_wide(1)
    with torch.no_grad(), use_ctx(RunCtx(dtype=torch.bfloat16)):
        MF.USE_FUSED = True
        y1 = m.forward_tokens(x, residual=res).float().cpu().numpy()
        MF.USE_FUSED = False
        try:
            y0 = m.forward_tokens(x, residual=res).float().cpu().numpy()
        finally:
            MF.USE_FUSED = True
            _lib.lib().hv_mhc_fused_enable_wide(0)
    assert rel_l2(y1, y0) < 1e-2
    assert np.abs(y1 - y0).max() < 0.1


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
    import ctypes
    from hv_amd import ManifoldHyperConnection, _lib
    from hv_amd.runtime import RunCtx, use_ctx
    lib = _lib.lib()
    lib.hv_mhc_fused_set_variant.argtypes = [ctypes.c_int]
    m = ManifoldHyperConnection(D, expansion_rate=4, use_mixed_precision=True)
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).eval()
    x = torch.randn(T, D, generator=torch.Generator().manual_seed(T)).to(torch.bfloat16).to(gpu_device)
    with torch.no_grad(), use_ctx(RunCtx(dtype=torch.bfloat16)):
        try:
            lib.hv_mhc_fused_set_variant(2)
            y8 = m.forward_tokens(x).cpu()
        finally:
            lib.hv_mhc_fused_set_variant(0)
        y4 = m.forward_tokens(x).cpu()
    assert torch.equal(y4, y8)
