"""Pin the CPU oracle (oracle/hv_oracle.py) against the reference's own outputs
(tests/golden, produced by oracle/gen_golden.py from the reference with shims S1-S7).

CPU only.  These tests are what makes the oracle trustworthy as the GPU parity checker.
"""
import numpy as np
import pytest
import torch

from conftest import formula_state_dict, golden
from oracle import cases, hv_oracle as O, weights as W


@pytest.mark.parametrize("fam", ["wc", "init"])
@pytest.mark.parametrize("D,it", cases.SK_CASES)
def test_sinkhorn_oracle_matches_reference(fam, D, it):
    g = golden(f"sk_{fam}_D{D}_it{it}")
    raw = cases.sinkhorn_raw(D, it, fam)
    hist = torch.zeros(it)
    M = O.sinkhorn(raw, it, history=hist)
    idx = [0, 1, D // 2, D - 1]
    np.testing.assert_allclose(M[idx].numpy(), g["rows"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(M.sum(0).numpy(), g["col_sums"], rtol=1e-5)
    np.testing.assert_allclose(hist.numpy(), g["history"], rtol=1e-4, atol=1e-7)
    if "M" in g.files:
        np.testing.assert_allclose(M.numpy(), g["M"], rtol=1e-5, atol=1e-8)


def test_sinkhorn_oracle_batched_reference_cases():
    for name, it in (("sk_batched_4x8x8", 20), ("sk_batched_2x5x7", 10)):
        g = golden(name)
        hist = torch.zeros(it)
        M = O.sinkhorn(torch.from_numpy(g["raw"]), it, history=hist)
        np.testing.assert_allclose(M.numpy(), g["M"], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(hist.numpy(), g["history"], rtol=1e-4, atol=1e-7)


def _mhc_sd(D, e, fam):
    shapes = {
        "H_pre_raw": (D, D * e), "H_post_raw": (D * e, D), "H_res_raw": (D, D),
        "mlp.0.weight": (2 * D * e, D * e), "mlp.0.bias": (2 * D * e,),
        "mlp.3.weight": (D * e, 2 * D * e), "mlp.3.bias": (D * e,),
        "norm_pre.weight": (D,), "norm_pre.bias": (D,),
        "norm_post.weight": (D,), "norm_post.bias": (D,),
    }
    return {k: W.make_tensor(k, s, fam) for k, s in shapes.items()}


@pytest.mark.parametrize("fam", ["wc", "init"])
@pytest.mark.parametrize("D,e", cases.MHC_CASES)
def test_mhc_oracle_matches_reference(fam, D, e):
    g = golden(f"mhc_{fam}_D{D}_e{e}")
    sd = _mhc_sd(D, e, fam)
    y = O.mhc(sd, "", cases.mhc_input(D, e), 20)
    np.testing.assert_allclose(y.numpy(), g["y"], rtol=0, atol=2e-4)
    # against the float64 reference run as well
    sd64 = O.cast_state_dict(sd, torch.float64)
    y64 = O.mhc(sd64, "", cases.mhc_input(D, e).double(), 20)
    np.testing.assert_allclose(y64.float().numpy(), g["y64"], rtol=0, atol=2e-5)


@pytest.mark.parametrize("fam", ["wc", "init"])
@pytest.mark.parametrize("D,e,T", cases.MHC_LARGE_CASES)
def test_mhc_oracle_matches_reference_large_T(fam, D, e, T):
    """The large-T fixtures (the kernel-policy thresholds): the regenerated input matches the
    one the reference ran on (checksums), and the oracle's fp64 chain on the stored row subsample
    reproduces the reference's fp64 rows (the chain is per token)."""
    g = golden(f"mhc_{fam}_D{D}_e{e}_T{T}")
    x = cases.mhc_input_large(D, e, T)
    assert int(g["T"]) == T
    assert float(x.double().sum()) == float(g["x_sum"]) and float(x.double().abs().sum()) == float(g["x_abs_sum"])
    rows = torch.from_numpy(g["rows"])
    assert torch.equal(rows, cases.mhc_large_rows(T))
    sd64 = O.cast_state_dict(_mhc_sd(D, e, fam), torch.float64)
    y64 = O.mhc(sd64, "", x[rows].double(), 20)
    np.testing.assert_allclose(y64.float().numpy(), g["y64"], rtol=0, atol=2e-5)


def _module_sd(names_shapes, fam):
    return {n: W.make_tensor(n, s, fam) for n, s in names_shapes}


def test_convmhc_blocks_match_reference():
    for (cin, cout, k, s, HW) in [(3, 32, 3, 2, 32), (64, 64, 3, 1, 16), (64, 128, 3, 2, 16)]:
        g = golden(f"convmhc_{cin}_{cout}_s{s}")
        shapes = _convmhc_shapes("", cin, cout, k)
        sd = _module_sd(shapes, "wc")
        y = O.conv_mhc_layer(sd, "", torch.from_numpy(g["x"]), cin, cout, k, s, 20)
        np.testing.assert_allclose(y.numpy(), g["y"], rtol=0, atol=5e-4)


def _mhc_shapes(p, D, e):
    return [(p + k, s) for k, s in [
        ("H_pre_raw", (D, D * e)), ("H_post_raw", (D * e, D)), ("H_res_raw", (D, D)),
        ("mlp.0.weight", (2 * D * e, D * e)), ("mlp.0.bias", (2 * D * e,)),
        ("mlp.3.weight", (D * e, 2 * D * e)), ("mlp.3.bias", (D * e,)),
        ("norm_pre.weight", (D,)), ("norm_pre.bias", (D,)),
        ("norm_post.weight", (D,)), ("norm_post.bias", (D,))]]


def _convmhc_shapes(p, cin, cout, k):
    sh = [(p + "conv.weight", (cout, cin, k, k)), (p + "bn.weight", (cout,)),
          (p + "bn.bias", (cout,)), (p + "bn.running_mean", (cout,)), (p + "bn.running_var", (cout,))]
    sh += _mhc_shapes(p + "mhc.", cout, 4)
    if cout >= 32:
        sh += [(p + "channel_attention.1.weight", (cout // 4, cout, 1, 1)),
               (p + "channel_attention.1.bias", (cout // 4,)),
               (p + "channel_attention.3.weight", (cout, cout // 4, 1, 1)),
               (p + "channel_attention.3.bias", (cout,))]
    return sh


def test_residual_block_matches_reference():
    g = golden("residual_128")
    c = 128
    sh = (_convmhc_shapes("blocks.0.", c, c // 2, 1) + _convmhc_shapes("blocks.1.", c // 2, c, 3)
          + _convmhc_shapes("projection.", c, c, 1))
    sd = _module_sd(sh, "wc")
    y = O.residual_mhc_layer(sd, "", torch.from_numpy(g["x"]), c, 20)
    np.testing.assert_allclose(y.numpy(), g["y"], rtol=0, atol=5e-4)


def test_encoder_block_matches_reference():
    g = golden("encblock_256_n50")
    D = 256
    sh = []
    for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
        sh += _mhc_shapes(f"attention.{n}.", D, 2)
    sh += _mhc_shapes("residual_mhc1.", D, 2) + _mhc_shapes("residual_mhc2.", D, 2)
    sh += [("norm1.scale", (D,)), ("norm2.scale", (D,)), ("mlp.0.weight", (4 * D, D)),
           ("mlp.0.bias", (4 * D,)), ("mlp.3.weight", (D, 4 * D)), ("mlp.3.bias", (D,))]
    sd = _module_sd(sh, "wc")
    y = O.encoder_block(sd, "", torch.from_numpy(g["x"]), 20)
    np.testing.assert_allclose(y.numpy(), g["y"], rtol=0, atol=5e-4)


def _attn_sd(fam="wc"):
    sh = []
    for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
        sh += _mhc_shapes(f"{n}.", 256, 2)
    return _module_sd(sh, fam)


def test_attention_cross_mask_weights_match_reference():
    """MultiHeadManifoldAttention with cross-attention, a key padding mask and need_weights
    (manifold_layers.py:386-434) -- the reference's own outputs (tests/golden/attn_cross_mask)."""
    g = golden("attn_cross_mask")
    sd = _attn_sd()
    q, kv, mask = (torch.from_numpy(g[k]) for k in ("q", "kv", "mask"))
    out, w = O.attention_general(sd, "", q, kv, kv, 20, 8, mask)
    np.testing.assert_allclose(out.numpy(), g["out"], rtol=0, atol=5e-4)
    np.testing.assert_allclose(w.numpy(), g["weights"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(O.attention(sd, "", q, 20).numpy(), g["out_self"], rtol=0, atol=5e-4)


def test_decode_matches_reference():
    g = golden("decode_s1")
    out = O.decode(torch.from_numpy(g["pred"]), O.anchor_wh(1))
    np.testing.assert_allclose(out["boxes"].numpy(), g["boxes"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(out["scores"].numpy(), g["scores"], rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(out["class_indices"].numpy(), g["class_indices"])


@pytest.mark.parametrize("tag,tiny,fam,S,B,sub", cases.MODEL_CASES[:3])
def test_model_oracle_matches_reference(tag, tiny, fam, S, B, sub):
    _check_model(tag, tiny, fam, S, B, sub)


@pytest.mark.slow
@pytest.mark.parametrize("tag,tiny,fam,S,B,sub", cases.MODEL_CASES[3:])
def test_model_oracle_matches_reference_large(tag, tiny, fam, S, B, sub):
    _check_model(tag, tiny, fam, S, B, sub)


def _check_model(tag, tiny, fam, S, B, sub):
    g = golden(f"model_{tag}")
    sd = formula_state_dict("tiny" if tiny else "base", fam)
    cfg = O.TINY if tiny else O.BASE
    with torch.no_grad():
        out = O.system_forward(sd, cases.model_input(B, S), cfg)
    for s in range(3):
        step = sub if s == 0 else 1
        pr = out["predictions"][f"scale_{s}"][:, :, ::step].numpy()
        # the oracle vs the reference, both fp32 on CPU: bounded by the reference's own
        # fp32-vs-fp64 error (up to 6.9e-4 from thread count alone)
        np.testing.assert_allclose(pr, g[f"pred{s}"], rtol=0, atol=2e-3)
        np.testing.assert_allclose(pr, g[f"pred{s}_f64"], rtol=0, atol=2e-3)
        ci = out["decoded"][f"scale_{s}"]["class_indices"].numpy()
        sure = g[f"margin{s}"] >= 1e-4
        assert (ci[sure] == g[f"cls{s}_f64"][sure]).all()
    np.testing.assert_allclose(out["final_features"].numpy(), g["final_features_f64"], rtol=0, atol=1e-4)


@pytest.mark.parametrize("tag,tiny,S,B,tseed", cases.TRAIN_CASES)
def test_train_step_oracle_matches_reference(tag, tiny, S, B, tseed):
    """Row T: the oracle's training-mode forward (BN batch statistics), YOLOLoss and autograd
    against the reference itself (tests/golden/train_<tag>: oracle/gen_golden.py G5), both in
    float64 -- fp64 leaves ~1e-10 of the model's ~1e6 rounding amplification, so the match is
    tight even where fp32 runs of the same model disagree by percents (base 224)."""
    import json
    import math
    import os
    import sys
    from conftest import GOLDEN, PKG
    if PKG not in sys.path:
        sys.path.insert(0, PKG)
    from hv_amd.targets import synthetic_targets
    g = golden(f"train_{tag}")
    kind = "tiny" if tiny else "base"
    names = json.load(open(os.path.join(GOLDEN, f"train_{kind}_param_names.json")))
    sd = {k: (v.double().requires_grad_(True) if v.is_floating_point() else v)
          for k, v in formula_state_dict(kind, "wc").items()}
    assert (int(g["B"]), int(g["S"])) == (B, S)
    x = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(1)).double()
    tg = [t.double() for t in synthetic_targets(B, S, seed=tseed)]
    with O.train_mode():
        out = O.system_forward(sd, x, O.TINY if tiny else O.BASE)
    loss = O.yolo_loss(out["predictions"], tg)
    loss["total_loss"].backward()
    assert abs(loss["total_loss"].item() / float(g["total_loss_f64"]) - 1) < 1e-6  # fixture stored as fp32
    for k in ("coord_loss", "obj_loss", "noobj_loss", "cls_loss"):
        assert abs(loss[k] - float(g[k + "_f64"])) <= 1e-6 * max(1.0, abs(float(g[k + "_f64"])))
    for s in range(3):
        np.testing.assert_allclose(out["predictions"][f"scale_{s}"].detach().numpy(), g[f"pred{s}_f64"],
                                   rtol=0, atol=1e-5)
    gn = g["grad_norm_f64"]
    gp = g["grad_probe_f64"] if "grad_probe_f64" in g.files else None
    gmax = float(gn.max())
    for i, n in enumerate(names):
        mine = sd[n].grad
        if gn[i] < 0:
            assert mine is None or float(mine.abs().max()) == 0.0, n
            continue
        assert abs(float(mine.norm()) - gn[i]) <= 1e-6 * max(gn[i], 1e-3) + 1e-9 * gmax, (n, float(mine.norm()), gn[i])
        if gp is not None:
            pr = float(mine.flatten() @ cases.grad_probe(n, mine.numel())) / math.sqrt(mine.numel())
            assert abs(pr - gp[i]) <= 1e-6 * max(gn[i], 1e-3) + 1e-9 * gmax, (n, pr, gp[i])
    for key in g.files:
        if key.startswith("g:") and key.endswith("_f64"):
            n = key[2:-4]
            np.testing.assert_allclose(sd[n].grad.numpy(), g[key], rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_post_process_oracle_matches_reference(seed):
    """§8f-1: the oracle's post_process/NMS vs the reference's (tests/golden/nms_*)."""
    g = golden(f"nms_{seed}")
    res = O.post_process(cases.nms_case(seed), float(g["conf"]), float(g["iou"]), int(g["max_det"]))
    for b, r in enumerate(res):
        np.testing.assert_array_equal(r["labels"].numpy(), g[f"labels{b}"])
        np.testing.assert_allclose(r["scores"].numpy(), g[f"scores{b}"], rtol=0, atol=0)
        np.testing.assert_allclose(r["boxes"].reshape(-1, 4).numpy(), g[f"boxes{b}"], rtol=0, atol=0)


@pytest.mark.parametrize("seed", range(6))
def test_std_sort_restatement_matches_torch_sort(seed):
    """oracle/std_sort.py (libstdc++ introsort over (value, index), descending) reproduces the
    reference's torch.sort(descending=True).indices exactly -- tie order included -- on inputs
    with heavy ties (the NMS sort, yolo_head.py:700)."""
    from oracle.std_sort import std_sort_desc
    g = torch.Generator().manual_seed(seed)
    for _ in range(20):
        n = int(torch.randint(1, 2500, (1,), generator=g))
        k = int(torch.randint(1, 60, (1,), generator=g))
        v = torch.randint(0, k, (n,), generator=g).float() / k
        assert std_sort_desc(v.tolist()) == torch.sort(v, descending=True).indices.tolist()
    v = torch.round(torch.rand(20000, generator=g) * 3000) / 3000
    assert std_sort_desc(v.tolist()) == torch.sort(v, descending=True).indices.tolist()


@pytest.mark.parametrize("case", cases.NMS_LARGE_CASES, ids=[c[0] for c in cases.NMS_LARGE_CASES])
def test_post_process_oracle_matches_reference_large(case):
    """§8f-1 at detection-grid sizes: > 8,192 candidates per scale (640^2 / 1024^2 grids at conf
    0.01) and max_det up to 5,000 -- the oracle vs the reference (tests/golden/nms_large_*)."""
    tag, seed, B, grids, conf, iou, mx, spread = case
    g = golden(f"nms_large_{tag}")
    res = O.post_process(cases.nms_case(seed, B=B, grids=grids, spread=spread), conf, iou, mx)
    for b, r in enumerate(res):
        np.testing.assert_array_equal(r["labels"].numpy(), g[f"labels{b}"])
        np.testing.assert_array_equal(r["scores"].numpy(), g[f"scores{b}"])
        np.testing.assert_array_equal(r["boxes"].reshape(-1, 4).numpy(), g[f"boxes{b}"])


@pytest.mark.parametrize("case", [c[0] for c in cases.PIL_CASES])
def test_preprocess_oracle_matches_pillow(case):
    """oracle/preproc.py (numpy restatement of Pillow's Resample.c) against Pillow's own output
    for the reference's default preprocessing resize -- bit-exact."""
    from oracle import preproc as P
    g = golden(f"preproc_pil_{case}")
    n, h, w = (int(v) for v in g["in_hw"])
    oh, ow = (int(v) for v in g["out_hw"])
    bgr = cases.camera_frames(int(g["seed"]), n, h, w)
    rgb, _ = P.preprocess_frames(bgr, oh, ow)
    np.testing.assert_array_equal(rgb, g["resized_rgb"])


@pytest.mark.parametrize("D,fam", cases.STAB_CASES)
def test_stability_monitor_oracle_matches_reference(D, fam):
    """a4: the oracle's _monitor_stability restatement (fp64) vs the reference's fp32 run
    (tests/golden/stab_*: eigvalsh eigenvalues, signal ratio, sum errors)."""
    g = golden(f"stab_{fam}_D{D}")
    H = torch.from_numpy(g["H"]) if "H" in g.files else O.sinkhorn(cases.sinkhorn_raw(D, 20, fam), 20)
    x_in, x_out = cases.stab_inputs(D, fam)
    r = O.monitor_stability(H, x_in, x_out)
    # the reference's eigvalsh runs in fp32 (LAPACK ssyevd): |err| ~ n * eps32 * ||H||
    np.testing.assert_allclose(r["eigenvalues"].numpy(), g["eigenvalues"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(float(r["signal_ratio"]), float(g["signal_ratio"]), rtol=1e-5)
    np.testing.assert_allclose(float(g["history0"]), float(g["signal_ratio"]), rtol=1e-6)
    for k in ("row_sum_error", "col_sum_error"):
        np.testing.assert_allclose(float(r[k]), float(g[k]), rtol=0, atol=2e-6)


@pytest.mark.parametrize("fam", ["wc", "init"])
@pytest.mark.parametrize("D,e", [c for c in cases.MHC_CASES if c[0] <= 512])
def test_autocast_emulation_reproduces_reference_bf16(fam, D, e):
    """S8 (oracle/autocast_emu.py): the oracle's mHC restatement run under the emulated CUDA
    autocast bf16 policy reproduces the reference's own bf16 output (fixture *_bf16ref, written
    by the reference's ManifoldHyperConnection under the same policy) -- the bf16 anchors the GPU
    tests multiply are the reference's numerics, not an artefact of where the casts sit -- and the
    recorded error anchor is what that output's distance from fp64 is."""
    from oracle.autocast_emu import CudaAutocastBF16
    g = golden(f"mhc_{fam}_D{D}_e{e}")
    gb = golden(f"mhc_{fam}_D{D}_e{e}_bf16ref")
    sd = _mhc_sd(D, e, fam)
    x = cases.mhc_input(D, e)
    with torch.no_grad(), CudaAutocastBF16() as mode:
        y = O.mhc(sd, "", x, 20).float()
    assert mode.counts["lower"] >= 4 and mode.counts["fp32"] >= 2
    ref = torch.from_numpy(gb["y"])
    assert float((y - ref).norm() / ref.norm()) < 2e-2
    y64 = torch.from_numpy(g["y64"]).double()
    err = float((ref.double() - y64).norm() / y64.norm())
    np.testing.assert_allclose(err, float(gb["err_vs_f64"]), rtol=1e-6)


def test_autocast_emulation_policy():
    """The emulated CUDA autocast bf16 policy: GEMM-class ops compute in bf16, LayerNorm /
    softmax / reductions in fp32, the rest keeps its input dtype; autograd sees the casts."""
    from oracle.autocast_emu import CudaAutocastBF16
    lin = torch.nn.Linear(8, 8)
    x = torch.randn(4, 8, requires_grad=True)
    with CudaAutocastBF16():
        h = lin(x)
        z = torch.nn.functional.layer_norm(h, (8,))
        s = torch.softmax(h, -1)
        a = torch.nn.functional.gelu(h)
        loss = (z.sum() + s.sum() + a.float().sum())
    assert h.dtype == torch.bfloat16 and a.dtype == torch.bfloat16
    assert z.dtype == torch.float32 and s.dtype == torch.float32
    loss.backward()
    assert x.grad.dtype == torch.float32 and lin.weight.grad.dtype == torch.float32
