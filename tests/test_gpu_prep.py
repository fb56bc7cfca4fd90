"""Grouped parameter preparation (hv_mhc_prep_group / hv_wprep_group via prep.PrepProgram)
against the independent per-site path (manifold.build_plan, ops.conv_weight_prep/bn_fold)."""
import pytest
import torch
import torch.nn as nn

from oracle import weights as W

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_mhc_prep_group_matches_per_site(gpu_device, dtype):
    from hv_amd import ManifoldHyperConnection, ops
    from hv_amd import manifold as MF
    from hv_amd.prep import PrepProgram
    from hv_amd.runtime import RunCtx
    mods = [ManifoldHyperConnection(D, expansion_rate=e) for D, e in
            [(32, 4), (64, 4), (256, 2), (256, 4), (96, 2), (320, 2), (512, 4), (1792, 2)]]
    for m in mods:
        W.load_formula_weights(m, "wc")
        m.to(gpu_device).eval()
    ctx = RunCtx(dtype=dtype)
    prog = PrepProgram(mods, dtype, gpu_device, fold_max_d=1024)
    prog.run(ctx)
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    for m in mods:
        p = ctx.plans[id(m)]
        h, hist = ops.sinkhorn(m.H_res_raw, m.sinkhorn.num_iterations)
        assert torch.equal(m.sinkhorn.convergence_history, hist)
        q = MF.build_plan(m, h, dtype, fold_max_d=1024)
        assert p.fold == q.fold == (m.input_dim <= 1024)
        assert rel(p.b1, q.b1) < tol, (m.input_dim, rel(p.b1, q.b1))
        assert rel(p.c1, q.c1) < 1e-5
        assert rel(p.wct, q.wct) < 1e-6
        assert rel(p.w2, q.w2) == 0
        if not p.fold:
            assert rel(p.w1, q.w1) == 0


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_weight_prep_group_matches_per_layer(gpu_device, dtype):
    from hv_amd import ops
    from hv_amd.prep import PrepProgram
    from hv_amd.runtime import RunCtx
    from hv_amd import ManifoldHyperConnection
    g = torch.Generator().manual_seed(5)
    m = ManifoldHyperConnection(32, expansion_rate=4).to(gpu_device).eval()
    convs = []
    # cin % 64 == 0 takes the LDS-staged reorder (1x1 and 3x3), the others the element loop
    for cin, cout, k, bias, with_bn in [(3, 32, 3, False, True), (64, 128, 1, True, False), (96, 40, 3, True, True),
                                        (128, 24, 3, False, True), (192, 17, 3, True, False)]:
        c = nn.Conv2d(cin, cout, k, padding=k // 2, bias=bias)
        bn = nn.BatchNorm2d(cout) if with_bn else None
        with torch.no_grad():
            c.weight.copy_(torch.randn(c.weight.shape, generator=g))
            if bias:
                c.bias.copy_(torch.randn(cout, generator=g))
            if bn is not None:
                bn.weight.copy_(torch.rand(cout, generator=g) + 0.5)
                bn.bias.copy_(torch.randn(cout, generator=g))
                bn.running_mean.copy_(torch.randn(cout, generator=g))
                bn.running_var.copy_(torch.rand(cout, generator=g) + 0.2)
                bn = bn.to(gpu_device).eval()
        convs.append((c.to(gpu_device), bn))
    lin = nn.Linear(96, 48).to(gpu_device)
    prog = PrepProgram([m], dtype, gpu_device, fold_max_d=1024)
    for c, bn in convs:
        prog.add_conv(c, bn)
    prog.add_linear(lin)
    ctx = RunCtx(dtype=dtype)
    prog.run(ctx)
    for c, bn in convs:
        w, s, b = ctx.plans[("conv", id(c))]
        if bn is not None:
            s0, b0 = ops.bn_fold(c.out_channels, gpu_device, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                 c.bias, bn.eps)
            assert torch.equal(s, s0) and torch.equal(b, b0)
        else:
            assert s is None and torch.equal(b, c.bias.detach())
        w0 = ops.conv_weight_prep(c.weight, dtype)
        assert w.shape == w0.shape and w.stride() == w0.stride()
        assert torch.equal(w, w0)
        pad = w.as_strided((w.shape[0], w.stride(0)), (w.stride(0), 1))[:, w.shape[1]:]
        assert (pad == 0).all()
    wl, bl = ctx.plans[("linear", id(lin))]
    assert torch.equal(wl, ops.cast(lin.weight.detach(), dtype)) and torch.equal(bl, lin.bias.detach())
