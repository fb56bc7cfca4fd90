"""GPU parity of the training-step kernels against plain PyTorch fp32
references of the same ops (torch autograd on the CPU), against the reference's own
gradient fixtures (tests/golden sk_*/mhc_*: autograd of the imported reference), and the
full tiny-model training step against autograd of the oracle restatement."""
from typing import Optional

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden
from oracle import cases

pytestmark = pytest.mark.gpu

DT = {"fp32": torch.float32, "bf16": torch.bfloat16}


def rel(a, b) -> float:
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def OT():
    from hv_amd import ops_train
    return ops_train


TOL = {"fp32": 1e-5, "bf16": 1.5e-2}


# ------------------------------------------------------------------ GEMMs
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("P,N1,N2", [(64, 32, 32), (1000, 64, 136), (4096, 256, 512), (70001, 32, 128),
                                     (333, 512, 24)])
def test_wgrad_dense(gpu_device, prec, P, N1, N2):
    g = torch.Generator().manual_seed(P + N1)
    a = torch.randn(P, N1, generator=g)
    b = torch.randn(P, N2, generator=g)
    dt = DT[prec]
    ad, bd = a.to(dt), b.to(dt)
    out = OT().wgrad(ad.to(gpu_device), bd.to(gpu_device))
    ref = ad.float().t() @ bd.float()
    assert rel(out, ref) < (1e-5 if prec == "fp32" else 1e-5 * 10)


def test_wgrad_accumulate(gpu_device):
    a = torch.randn(512, 64)
    b = torch.randn(512, 32)
    c0 = torch.randn(64, 32)
    out = c0.clone().to(gpu_device)
    OT().wgrad(a.to(gpu_device), b.to(gpu_device), out=out, accumulate=True)
    assert rel(out, c0 + a.t() @ b) < 1e-5


def _wgrad_variant(v, fn):
    from hv_amd.runtime import HVOptions, set_train_state
    set_train_state(HVOptions(wgrad_variant=v))
    try:
        return fn()
    finally:
        set_train_state()


@pytest.mark.parametrize("kind", ["dense", "conv_stem"])
def test_wgrad_many_splits_and_variants(gpu_device, kind):
    """Small outputs over many pixels (one or two tiles): the plan splits the pixels up to 256 ways
    and sums the partials with the many-split reduction; HV_WV_K64 (64-row LDS stages) is bitwise
    the default; HV_WV_CAP64 (the round-4 plan, <= 64 splits) agrees within fp32 rounding."""
    T = OT()
    g = torch.Generator().manual_seed(11)
    if kind == "dense":
        a = torch.randn(200003, 128, generator=g).to(torch.bfloat16)
        b = torch.randn(200003, 64, generator=g).to(torch.bfloat16)
        ad, bd = a.to(gpu_device), b.to(gpu_device)
        run = lambda: T.wgrad(ad, bd)                                  # noqa: E731
        ref = a.float().t() @ b.float()
    else:                                              # the stem conv: Cin = 3, scalar im2col
        x = torch.randn(2, 3, 320, 320, generator=g).to(torch.bfloat16).float()
        dy = torch.randn(2, 32, 160, 160, generator=g).to(torch.bfloat16).float()
        ref = torch.nn.grad.conv2d_weight(x, (32, 3, 3, 3), dy, 2, 1)
        xd = x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(gpu_device)
        dyd = dy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(gpu_device)
        run = lambda: T.conv_grad_reorder(T.conv_wgrad(dyd, xd, 3, 2, 1), 32, 3, 3)   # noqa: E731
    out = {v: _wgrad_variant(v, run).clone() for v in (0, 1, 2)}
    assert torch.equal(out[0], out[1])
    for v in (0, 2):
        assert rel(out[v], ref) < 1e-5
    assert torch.equal(out[0], _wgrad_variant(0, run))                 # deterministic


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("cin,cout,k,s,hw", [(32, 64, 3, 1, 16), (64, 128, 3, 2, 16), (64, 32, 1, 1, 12),
                                             (3, 32, 3, 2, 32), (256, 256, 3, 1, 10), (128, 64, 3, 2, 15)])
def test_conv_wgrad_dgrad(gpu_device, prec, cin, cout, k, s, hw):
    from hv_amd import ops
    T = OT()
    dt = DT[prec]
    g = torch.Generator().manual_seed(cin * 7 + cout)
    x = torch.randn(2, cin, hw, hw, generator=g).to(dt).float()
    w = (torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5).to(dt).float()
    p = k // 2
    y = F.conv2d(x, w, None, s, p)
    dy = torch.randn(y.shape, generator=g).to(dt).float()
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w, dy, s, p)
    dw_ref = torch.nn.grad.conv2d_weight(x, w.shape, dy, s, p)
    xd = x.permute(0, 2, 3, 1).contiguous().to(dt).to(gpu_device)
    dyd = dy.permute(0, 2, 3, 1).contiguous().to(dt).to(gpu_device)
    dw = T.conv_grad_reorder(T.conv_wgrad(dyd, xd, k, s, p), cout, cin, k)
    tol = 1e-5 if prec == "fp32" else 1e-2
    assert rel(dw, dw_ref) < tol
    if cin % 8 == 0 or prec == "fp32":
        wd = w.to(gpu_device)
        flip = s == 1
        wt = T.dgrad_weight(wd, dt, flip)
        dx = T.conv_dgrad(dyd, wt, k, s, p, (hw, hw), flipped=flip)
        assert rel(dx.float().permute(0, 3, 1, 2), dx_ref) < tol


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("act", ["gelu", "silu", "relu", "leaky"])
def test_gemm_train_modes(gpu_device, prec, act):
    """mode 1 stores the pre-activation and applies act + dropout; mode 2 applies the
    derivative and the SAME mask (regenerated from the seed)."""
    T = OT()
    dt = DT[prec]
    g = torch.Generator().manual_seed(3)
    M, N, K = 300, 128, 96
    a = torch.randn(M, K, generator=g).to(dt)
    b = (torch.randn(N, K, generator=g) / K ** 0.5).to(dt)
    bias = torch.randn(N, generator=g)
    ad, bd = a.to(gpu_device), b.to(gpu_device)
    pre = torch.empty(M, N, device=gpu_device, dtype=dt)
    p = 0.25
    y = T.gemm_train(ad, bd, mode=1, act=act, aux=pre, bias=bias.to(gpu_device), drop_p=p, seed=1234)
    pre_ref = a.float() @ b.float().t() + bias
    assert rel(pre.float(), pre_ref) < TOL[prec]
    fa = {"gelu": F.gelu, "silu": F.silu, "relu": F.relu, "leaky": lambda t: F.leaky_relu(t, 0.1)}[act]
    yc = y.float().cpu()
    act_ref = fa(pre.float().cpu())
    kept = yc != 0
    frac = 1 - kept.float().mean().item()
    assert abs(frac - p) < 0.03 or act == "relu"
    np.testing.assert_allclose(yc[kept].numpy(), (act_ref / (1 - p))[kept].numpy(), rtol=2e-2, atol=2e-2)
    # mode 2 with the same seed reproduces the mask: dpre = dh * keep/(1-p) * act'(pre)
    dh = torch.randn(M, K, generator=g).to(dt)
    w2 = (torch.randn(N, K, generator=g) / K ** 0.5).to(dt)
    dpre = T.gemm_train(dh.to(gpu_device), w2.to(gpu_device), mode=2, act=act, aux=pre, drop_p=p, seed=1234)
    z = pre.float().cpu().requires_grad_(True)
    (fa(z) * (dh.float() @ w2.float().t())).sum().backward()
    ref = z.grad * (kept.float() / (1 - p))
    assert rel(dpre.float(), ref) < (1e-4 if prec == "fp32" else 2e-2)
    # the elementwise kernel uses the same mask convention
    dpre2 = T.act_backward((dh.to(gpu_device) @ w2.to(gpu_device).t()).to(dt).contiguous(), pre, act, p, 1234)
    assert rel(dpre2.float(), ref) < (1e-4 if prec == "fp32" else 2e-2)


# ------------------------------------------------------------------ norms
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("act", ["silu", "relu", "leaky"])
def test_batchnorm_train(gpu_device, prec, act):
    T = OT()
    dt = DT[prec]
    g = torch.Generator().manual_seed(5)
    n, h, w, c = 4, 9, 7, 48
    x = (torch.randn(n, h, w, c, generator=g) * 2 + 0.5).to(dt)
    gamma = torch.rand(c, generator=g) + 0.5
    beta = torch.randn(c, generator=g)
    rm, rv = torch.zeros(c), torch.ones(c)
    xd = x.to(gpu_device)
    rmd, rvd = rm.clone().to(gpu_device), rv.clone().to(gpu_device)
    mean, rstd = T.bn_stats(xd, 1e-5, 0.1, rmd, rvd)
    y = T.bn_apply(xd, mean, rstd, gamma.to(gpu_device), beta.to(gpu_device), act)
    xr = x.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    fa = {"silu": F.silu, "relu": F.relu, "leaky": lambda t: F.leaky_relu(t, 0.1)}[act]
    yr = fa(F.batch_norm(xr, rm, rv, gr, br, True, 0.1, 1e-5))
    assert rel(y.float().permute(0, 3, 1, 2), yr.detach()) < TOL[prec]
    assert rel(rmd, rm) < 1e-5 and rel(rvd, rv) < 1e-5
    dy = torch.randn(n, c, h, w, generator=g).to(dt).float()
    (yr * dy).sum().backward()
    dx, dg, db = T.bn_backward(xd, dy.permute(0, 2, 3, 1).contiguous().to(dt).to(gpu_device), mean, rstd,
                               gamma.to(gpu_device), beta.to(gpu_device), act)
    assert rel(dx.float().permute(0, 3, 1, 2), xr.grad) < (1e-4 if prec == "fp32" else 3e-2)
    assert rel(dg, gr.grad) < (1e-4 if prec == "fp32" else 2e-2)
    assert rel(db, br.grad) < (1e-4 if prec == "fp32" else 2e-2)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("cols", [32, 256, 1792])
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_rownorm_train_backward(gpu_device, mode, cols, prec):
    T = OT()
    dt = DT[prec]
    g = torch.Generator().manual_seed(cols + mode)
    rows = 77
    x = (torch.randn(rows, cols, generator=g) * 3 + 1).to(dt)
    gamma = torch.rand(cols, generator=g) + 0.5
    beta = torch.randn(cols, generator=g)
    p = 0.2
    y, mean, rstd = T.rownorm_train(mode, x.to(gpu_device), 1e-5, gamma.to(gpu_device),
                                    beta.to(gpu_device) if mode == 0 else None, p, 99)
    xr = x.float().clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    brr = beta.clone().requires_grad_(True)
    if mode == 0:
        yr = F.layer_norm(xr, (cols,), gr, brr, 1e-5)
    else:
        yr = xr / torch.sqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * gr
    keep = (y.float().cpu() != 0).float()
    assert abs(1 - keep.mean().item() - p) < 0.05
    yr_d = yr * keep / (1 - p)
    assert rel(y.float(), yr_d.detach()) < TOL[prec]
    dy = torch.randn(rows, cols, generator=g).to(dt).float()
    (yr_d * dy).sum().backward()
    dx, dg, db = T.rownorm_backward(mode, x.to(gpu_device), dy.to(dt).to(gpu_device), mean, rstd,
                                    gamma.to(gpu_device), p, 99, dx_dtype=torch.float32)
    assert rel(dx, xr.grad) < (1e-4 if prec == "fp32" else 3e-2)
    assert rel(dg, gr.grad) < (1e-4 if prec == "fp32" else 3e-2)
    if mode == 0:
        assert rel(db, brr.grad) < (1e-4 if prec == "fp32" else 3e-2)


# ------------------------------------------------------------------ Sinkhorn backward
@pytest.mark.parametrize("fam", ["wc", "init"])
@pytest.mark.parametrize("D,it", cases.SK_CASES)
def test_sinkhorn_backward_matches_reference_fixture(gpu_device, fam, D, it):
    from hv_amd import ops
    from hv_amd.train_fn import SinkhornGroupFn
    gld = golden(f"sk_{fam}_D{D}_it{it}")
    raw = cases.sinkhorn_raw(D, it, fam).to(gpu_device).requires_grad_(True)
    grp = ops.SinkhornGroup([raw.detach()], [it], gpu_device)
    (M,) = SinkhornGroupFn.apply(grp, None, raw)
    G = torch.randn(D, D, generator=cases.gen_seed(D, it, 3)).to(gpu_device)
    (M * G).sum().backward()
    gr = raw.grad.cpu()
    idx = [0, 1, D // 2, D - 1]
    ref = torch.from_numpy(gld["grad_rows"])
    assert rel(gr[idx], ref) < 1e-3, rel(gr[idx], ref)
    if "grad" in gld.files:
        assert rel(gr, torch.from_numpy(gld["grad"])) < 1e-3


def test_sinkhorn_backward_grouped_equals_single(gpu_device):
    from hv_amd import ops
    from hv_amd.train_fn import SinkhornGroupFn
    Ds, its = (32, 64, 256, 1792), (20, 5, 20, 20)
    raws = [cases.sinkhorn_raw(D, 20, "wc").to(gpu_device).requires_grad_(True) for D in Ds]
    Gs = [torch.randn(D, D, device=gpu_device) for D in Ds]
    grp = ops.SinkhornGroup([r.detach() for r in raws], list(its), gpu_device)
    outs = SinkhornGroupFn.apply(grp, None, *raws)
    sum((o * G).sum() for o, G in zip(outs, Gs)).backward()
    grouped = [r.grad.clone() for r in raws]
    for r, it, G, gg in zip(raws, its, Gs, grouped):
        r2 = r.detach().clone().requires_grad_(True)
        g1 = ops.SinkhornGroup([r2.detach()], [it], gpu_device)
        (o,) = SinkhornGroupFn.apply(g1, None, r2)
        (o * G).sum().backward()
        assert torch.equal(r2.grad, gg)


# ------------------------------------------------------------------ mHC
@pytest.mark.parametrize("fam", ["wc", "init"])
@pytest.mark.parametrize("D,e", cases.MHC_CASES)
def test_mhc_backward_matches_reference_fixture(gpu_device, fam, D, e):
    """Gradients of x and H_res_raw (through the Sinkhorn) vs autograd of the reference."""
    from hv_amd import ManifoldHyperConnection
    from oracle import weights as W
    gld = golden(f"mhc_{fam}_D{D}_e{e}")
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=False)
    W.load_formula_weights(m, fam)
    m = m.to(gpu_device).train()
    for d in (m.mlp[2], m.mlp[5], m.dropout):
        d.p = 0.0
    x = cases.mhc_input(D, e).to(gpu_device).requires_grad_(True)
    y = m(x)
    np.testing.assert_allclose(y.detach().cpu().numpy(), gld["y64"], rtol=0, atol=1e-3)
    G = torch.randn(64, D, generator=cases.gen_seed(D, e, 12)).to(gpu_device)
    (y * G).sum().backward()
    assert rel(x.grad, torch.from_numpy(gld["gx"])) < 2e-3
    gh = m.H_res_raw.grad.cpu()
    ref = torch.from_numpy(gld["g_hres"])
    assert rel(gh[: ref.shape[0]], ref) < 5e-3
    assert abs(m.H_pre_raw.grad.abs().sum().item() / float(gld["g_hpre_sum"]) - 1) < 5e-3
    assert abs(m.mlp[0].weight.grad.abs().sum().item() / float(gld["g_w1_sum"]) - 1) < 5e-3


@pytest.mark.parametrize("D,e", [(32, 4), (64, 4), (256, 2), (512, 2)])
def test_mhc_all_param_grads_vs_oracle(gpu_device, D, e):
    """Every parameter gradient of the training mHC vs torch autograd of the oracle (fp64)."""
    from hv_amd import ManifoldHyperConnection
    from oracle import hv_oracle as O
    from oracle import weights as W
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=False)
    W.load_formula_weights(m, "wc")
    sd = {k: v.detach().double().clone().requires_grad_(True) for k, v in m.state_dict().items()
          if v.is_floating_point()}
    m = m.to(gpu_device).train()
    for d in (m.mlp[2], m.mlp[5], m.dropout):
        d.p = 0.0
    x = cases.mhc_input(D, e)
    G = torch.randn(64, D, generator=cases.gen_seed(D, e, 12))
    y = m(x.to(gpu_device))
    (y * G.to(gpu_device)).sum().backward()
    yo = O.mhc(sd, "", x.double(), m.sinkhorn.num_iterations)
    (yo * G.double()).sum().backward()
    for name, p in m.named_parameters():
        ref = sd[name].grad
        assert ref is not None
        assert rel(p.grad, ref) < 2e-3, (name, rel(p.grad, ref))


@pytest.mark.parametrize("D,e,T", [(64, 4, 2000), (256, 2, 600)])
def test_mhc_bf16_train_agreement(gpu_device, D, e, T):
    from hv_amd import ManifoldHyperConnection
    from oracle import weights as W
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=False)
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device).train()
    for d in (m.mlp[2], m.mlp[5], m.dropout):
        d.p = 0.0
    x = torch.randn(T, D, device=gpu_device)
    G = torch.randn(T, D, device=gpu_device)
    y = m(x.clone().requires_grad_(True))
    (y * G).sum().backward()
    ref = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad()
    m.use_mixed_precision = True
    m.hv_precision = "bf16"
    xb = x.to(torch.bfloat16).requires_grad_(True)
    yb = m(xb)
    (yb.float() * G).sum().backward()
    assert rel(yb.float(), y.detach()) < 3e-2
    for n, p in m.named_parameters():
        assert rel(p.grad, ref[n]) < 0.1, (n, rel(p.grad, ref[n]))


# ------------------------------------------------------------------ attention / SE / misc
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_attention_train_backward(gpu_device, prec):
    T = OT()
    dt = DT[prec]
    n, L, H, hd = 2, 50, 8, 32
    g = torch.Generator().manual_seed(11)
    q, k, v, do = (torch.randn(n, L, H * hd, generator=g).to(dt) for _ in range(4))
    o, lse = T.attention_train(q.to(gpu_device), k.to(gpu_device), v.to(gpu_device), H, 0.0, 0)
    qr, kr, vr = (t.float().view(n, L, H, hd).transpose(1, 2).clone().requires_grad_(True) for t in (q, k, v))
    att = torch.softmax(qr @ kr.transpose(-1, -2) * hd ** -0.5, -1)
    orf = (att @ vr).transpose(1, 2).reshape(n, L, H * hd)
    assert rel(o.float(), orf.detach()) < TOL[prec]
    (orf * do.float()).sum().backward()
    dq, dk, dv = T.attention_backward(q.to(gpu_device), k.to(gpu_device), v.to(gpu_device), o,
                                      do.to(gpu_device), lse, H, 0.0, 0)
    for a, r in ((dq, qr.grad), (dk, kr.grad), (dv, vr.grad)):
        assert rel(a.float(), r.transpose(1, 2).reshape(n, L, H * hd)) < (1e-4 if prec == "fp32" else 3e-2)


@pytest.mark.parametrize("L,p", [(1, 0.0), (17, 0.1), (50, 0.0), (401, 0.1), (130, 0.3)])
def test_attention_train_mfma_matches_scalar(gpu_device, L, p):
    """The bf16 matrix-core attention (forward with lse + dropout, key-parallel dK/dV and
    query-parallel dQ backward) against the scalar kernels on the same inputs and the same
    dropout seed: identical masks (keep(i, j) regenerated from (seed, element)), so the outputs
    and gradients agree to bf16 rounding; L = 401 is the ViT at 640²."""
    T = OT()
    n, H, hd = 2, 8, 32
    g = torch.Generator().manual_seed(L)
    q, k, v, do = (torch.randn(n, L, H * hd, generator=g).to(torch.bfloat16).to(gpu_device) for _ in range(4))
    res = {}
    for mfma in (True, False):
        T.ATTN_MFMA = mfma
        try:
            o, lse = T.attention_train(q, k, v, H, p, 1234)
            dq, dk, dv = T.attention_backward(q, k, v, o, do, lse, H, p, 1234)
        finally:
            T.ATTN_MFMA = True
        res[mfma] = (o, lse, dq, dk, dv)
    assert (res[True][1] - res[False][1]).abs().max().item() < 2e-3           # lse
    for a, b_ in zip(res[True][:1] + res[True][2:], res[False][:1] + res[False][2:]):
        if b_.abs().max().item() == 0:      # L = 1: softmax of one key is 1, dS = 0 exactly; rounding only
            assert a.float().abs().max().item() < 1e-2
        else:
            assert rel(a.float(), b_.float()) < 2e-2
    dv = res[True][4].float()
    assert abs((dv * v.float()).sum().item() - (do.float() * res[True][0].float()).sum().item()) \
        < 2e-2 * max(1.0, abs((do.float() * res[True][0].float()).sum().item()))


def test_attention_dropout_consistent(gpu_device):
    """With dropout the backward must see the forward's mask: check dv = (P*mask)^T do."""
    T = OT()
    n, L, H, hd = 1, 40, 8, 32
    q, k, v = (torch.randn(n, L, H * hd, device=gpu_device) for _ in range(3))
    p = 0.3
    o, lse = T.attention_train(q, k, v, H, p, 77)
    do = torch.randn_like(o)
    dq, dk, dv = T.attention_backward(q, k, v, o, do, lse, H, p, 77)
    # dv . v == do . o  (both equal sum_ij P_ij m_ij (do_i . v_j))
    lhs = (dv * v).sum().item()
    rhs = (do * o).sum().item()
    assert abs(lhs - rhs) < 1e-3 * max(1.0, abs(rhs))


def test_se_gate_backward(gpu_device):
    from hv_amd.train_fn import SEGateFn
    g = torch.Generator().manual_seed(2)
    n, h, w, c, cr = 3, 6, 5, 64, 16
    y = torch.randn(n, h, w, c, generator=g)
    idn = torch.randn(n, h, w, c, generator=g)
    w1, b1 = torch.randn(cr, c, 1, 1, generator=g) * 0.2, torch.randn(cr, generator=g) * 0.1
    w2, b2 = torch.randn(c, cr, 1, 1, generator=g) * 0.2, torch.randn(c, generator=g) * 0.1
    dout = torch.randn(n, h, w, c, generator=g)
    ts = [t.clone().to(gpu_device).requires_grad_(True) for t in (y, idn, w1, b1, w2, b2)]
    out = SEGateFn.apply(*ts)
    (out * dout.to(gpu_device)).sum().backward()
    rs = [t.clone().requires_grad_(True) for t in (y, idn, w1, b1, w2, b2)]
    yy = rs[0].permute(0, 3, 1, 2)
    gt = F.adaptive_avg_pool2d(yy, 1)
    gt = torch.sigmoid(F.conv2d(F.silu(F.conv2d(gt, rs[2], rs[3])), rs[4], rs[5]))
    ref = (yy * gt).permute(0, 2, 3, 1) + rs[1]
    assert rel(out, ref.detach()) < 1e-5
    (ref * dout).sum().backward()
    for a, r in zip(ts, rs):
        assert rel(a.grad, r.grad) < 1e-4


def test_pool_upsample_tokens_backward(gpu_device):
    T = OT()
    x = torch.randn(2, 8, 6, 16)
    dy = torch.randn(2, 4, 3, 16)
    xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    F.max_pool2d(xr, 2, 2).backward(dy.permute(0, 3, 1, 2))
    dx = T.maxpool2x2_backward(x.to(gpu_device), dy.to(gpu_device))
    assert rel(dx.permute(0, 3, 1, 2), xr.grad) < 1e-6
    big = torch.randn(2, 8, 6, 16)
    db = T.upsample_backward(big.to(gpu_device), 4, 3)
    small = torch.zeros(2, 16, 4, 3, requires_grad=True)
    F.interpolate(small, size=(8, 6), mode="nearest").backward(big.permute(0, 3, 1, 2))
    assert rel(db.permute(0, 3, 1, 2), small.grad) < 1e-6
    tok = torch.randn(2, 5, 8)
    cls, pos = torch.randn(8), torch.randn(6, 8)
    z = T.vit_assemble(tok.to(gpu_device), cls.to(gpu_device), pos.to(gpu_device))
    zr = torch.cat([cls.expand(2, 1, 8), tok], 1) + pos
    assert rel(z, zr) < 1e-6
    dz = torch.randn(2, 6, 8)
    dx, dcls, dpos = T.vit_assemble_backward(dz.to(gpu_device))
    assert rel(dx, dz[:, 1:]) < 1e-6 and rel(dcls, dz[:, 0].sum(0)) < 1e-6 and rel(dpos, dz.sum(0)) < 1e-6


# ------------------------------------------------------------------ loss / optimizer
@pytest.mark.parametrize("empty_scale", [False, True])
def test_yolo_loss_matches_oracle(gpu_device, empty_scale):
    from hv_amd.targets import synthetic_targets
    from oracle import hv_oracle as O
    T = OT()
    B, S, A = 2, 128, 3
    tg = synthetic_targets(B, S, seed=5)
    if empty_scale:
        tg[2].zero_()
    g = torch.Generator().manual_seed(9)
    preds, lgs = {}, []
    for s, t in enumerate(tg):
        h, w = t.shape[2], t.shape[3]
        p = torch.randn(B, A, h, w, 85, generator=g)
        preds[f"scale_{s}"] = p.clone().requires_grad_(True)
        lgs.append(p.permute(0, 2, 3, 1, 4).reshape(B, h, w, A * 85).contiguous())
    ref = O.yolo_loss(preds, tg)
    ref["total_loss"].backward()
    total = 0.0
    for s, (lg, t) in enumerate(zip(lgs, tg)):
        sums, dl = T.yolo_loss(lg.to(gpu_device), t.to(gpu_device), A, (5.0, 1.0, 0.5, 1.0))
        total += sums[4].item()
        B_, h, w, _ = lg.shape
        gr = preds[f"scale_{s}"].grad
        if gr is None:                       # scale without objects: the reference skips it
            assert dl.abs().max().item() == 0 and sums[4].item() == 0
            continue
        dref = gr.permute(0, 2, 3, 1, 4).reshape(B_, h, w, -1)
        assert rel(dl, dref) < 1e-5
    assert abs(total - ref["total_loss"].item()) < 1e-4 * abs(ref["total_loss"].item())


def test_fused_adamw_and_clipping_match_torch(gpu_device):
    from hv_amd.trainer import FusedAdamW, mhc_group
    torch.manual_seed(0)
    named = [("a.mhc.w", torch.randn(1000)), ("b.H_res_raw", torch.randn(33, 7)), ("c.conv.weight", torch.randn(4097)),
             ("d.bias", torch.randn(5))]
    mine = [(n, t.clone().to(gpu_device).requires_grad_(True)) for n, t in named]
    ref = [(n, t.clone().requires_grad_(True)) for n, t in named]
    opt = FusedAdamW(mine, lr=1e-2, weight_decay=1e-2, max_norms=(0.5, 1.0))
    topt = torch.optim.AdamW([p for _, p in ref], lr=1e-2, weight_decay=1e-2, eps=1e-8)
    for step in range(3):
        gs = [torch.randn_like(t) * (3.0 if i % 2 else 0.1) for i, (_, t) in enumerate(named)]
        for (_, p), gr in zip(mine, gs):
            p.grad = gr.clone().to(gpu_device)
        for (_, p), gr in zip(ref, gs):
            p.grad = gr.clone()
        opt.step(clip=True)
        for grp in (0, 1):
            torch.nn.utils.clip_grad_norm_([p for n, p in ref if mhc_group(n) == grp], 0.5 if grp == 0 else 1.0)
        topt.step()
    for (_, a), (_, b) in zip(mine, ref):
        assert rel(a.detach(), b.detach()) < 1e-5


# ------------------------------------------------------------------ full model
def _tiny_model(gpu_device, precision="fp32"):
    from hv_amd import HybridVisionSystem
    from oracle import weights as W
    m = HybridVisionSystem(dict(num_blocks=[1, 1, 1, 1], vit_depth=1, sk_iters=5, verbose=False,
                                precision=precision))
    W.load_formula_weights(m, "wc")
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(gpu_device).train()
    for mod in m.modules():
        if isinstance(mod, (torch.nn.Dropout, torch.nn.Dropout2d)):
            mod.p = 0.0
    return m, sd


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_grouped_train_prep_matches_per_site(gpu_device, precision):
    """The grouped training coefficient prep (train_prep.TrainPrep: prep group + ONE transpose group
    launch for all sites) gives the loss and every parameter gradient of the per-site preparation
    (model.hv_train_group_prep = False), dropout off: bitwise-close in fp32 (the same fp32 products,
    other launch boundaries), within bf16 rounding of the fold GEMM in bf16.  Two forwards before one
    backward (`model(x1) + model(x2)`, reference autograd semantics) give the per-site gradients too:
    the second forward takes a second buffer set from the pool instead of overwriting the first's."""
    from hv_amd.targets import synthetic_targets
    res = {}
    for grouped in (True, False):
        m, _ = _tiny_model(gpu_device, precision)
        m.hv_train_group_prep = grouped
        B, S = 2, 64
        x = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(3)).to(gpu_device)
        tg = [t.to(gpu_device) for t in synthetic_targets(B, S, seed=4)]
        out = m(x, targets=tg, compute_loss=True)
        out["loss"]["total_loss"].backward()
        torch.cuda.synchronize()
        res[grouped] = (float(out["loss"]["total_loss"]),
                        {n: p.grad.detach().float().cpu() for n, p in m.named_parameters() if p.grad is not None})
    (l1, g1), (l0, g0) = res[True], res[False]
    tol = 1e-5 if precision == "fp32" else 2e-2
    assert abs(l1 - l0) <= tol * abs(l0), (l1, l0)
    assert g1.keys() == g0.keys()
    for n in g0:
        d = (g1[n] - g0[n]).norm().item()
        assert d <= tol * g0[n].norm().item() + 1e-6, (n, d, g0[n].norm().item())
    two = {}
    for grouped in (True, False):
        m, _ = _tiny_model(gpu_device, precision)
        m.hv_train_group_prep = grouped
        x1 = torch.randn(2, 3, 64, 64, generator=torch.Generator().manual_seed(3)).to(gpu_device)
        x2 = torch.randn(2, 3, 64, 64, generator=torch.Generator().manual_seed(5)).to(gpu_device)
        tg = [t.to(gpu_device) for t in synthetic_targets(2, 64, seed=4)]
        loss = m(x1, targets=tg, compute_loss=True)["loss"]["total_loss"] + \
            m(x2, targets=tg, compute_loss=True)["loss"]["total_loss"]
        loss.backward()
        torch.cuda.synchronize()
        two[grouped] = {n: p.grad.detach().float().cpu() for n, p in m.named_parameters() if p.grad is not None}
        pool = m.__dict__["_train_prep_cache"]["pool"]
        assert len(pool) == 2 and all(e["busy"] == 0 for e in pool)
        # a forward whose graph is dropped without a backward frees its set again
        m(x1, targets=tg, compute_loss=True)
        m(x2, targets=tg, compute_loss=True)
        assert len(pool) == 2 and all(e["busy"] == 0 for e in pool)
    for n in two[False]:
        d = (two[True][n] - two[False][n]).norm().item()
        assert d <= tol * two[False][n].norm().item() + 1e-6, (n, d)


def test_tiny_train_step_grads_match_oracle(gpu_device):
    """Loss and every parameter gradient of one tiny-config training step (BN batch stats,
    dropout off) vs autograd of the oracle in fp64.  This configuration is ill-conditioned
    (BatchNorm over 8 values at stage 4): the oracle's OWN fp32 gradients sit ~1% (median)
    from its fp64 ones, so each parameter must be within 3x the oracle-fp32 error (+1e-3)."""
    from hv_amd.targets import synthetic_targets
    from oracle import hv_oracle as O
    m, sd = _tiny_model(gpu_device)
    B, S = 2, 64
    x = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(1))
    tg = synthetic_targets(B, S, seed=3)
    out = m(x.to(gpu_device), targets=[t.to(gpu_device) for t in tg], compute_loss=True)
    out["loss"]["total_loss"].backward()
    grads = {}
    for dt in (torch.float64, torch.float32):
        sdo = {k: (v.to(dt).requires_grad_(True) if v.is_floating_point() else v) for k, v in sd.items()}
        with O.train_mode():
            ref = O.system_forward(sdo, x.to(dt), O.TINY)
        lref = O.yolo_loss(ref["predictions"], [t.to(dt) for t in tg])
        lref["total_loss"].backward()
        grads[dt] = {k: v.grad for k, v in sdo.items() if v.is_floating_point()}
        if dt == torch.float64:
            assert abs(out["loss"]["total_loss"].item() / lref["total_loss"].item() - 1) < 1e-4
            for s in range(3):
                a = out["predictions"][f"scale_{s}"].detach().cpu()
                assert (a - ref["predictions"][f"scale_{s}"].detach()).abs().max().item() < 1e-3
    bad = []
    gmax = max(g.norm().item() for g in grads[torch.float64].values() if g is not None)
    for name, p in m.named_parameters():
        r = grads[torch.float64][name]
        if r is None:
            assert p.grad is None or p.grad.abs().max().item() < 1e-6, name
            continue
        if r.norm().item() < 1e-7 * gmax:
            # structurally zero (conv bias before BatchNorm, a bias shared by every key of a
            # softmax): only rounding noise is left -- it must stay at the noise level
            assert p.grad.norm().item() < 1e-5 * gmax, name
            continue
        r32 = grads[torch.float32][name].double()
        mine = p.grad.double().cpu()
        e_ref = (r32 - r).norm().item()
        e = (mine - r).norm().item()
        if e > 3 * e_ref + 1e-3 * r.norm().item() + 1e-9:
            bad.append((name, e / (r.norm().item() + 1e-30), e_ref / (r.norm().item() + 1e-30)))
    assert not bad, bad[:10]


def test_base_train_step_matches_reference_fixture(gpu_device):
    """Config C's model (base, 353.8M params, reference architecture) through one fp32
    training step at 224 B=2 against the reference itself (tests/golden/train_base_224_b2,
    dropout 0, BN batch statistics).  This forward is ill-conditioned in train mode: rounding
    grows layer by layer from stage 3 on (the reference's own fp32 run is 9% rel-L2 from its
    fp64 run on the head logits, and its fp32 gradient norms sit a median 4% from fp64), so
    the HIP fp32 step is held to the reference fp32 run's OWN error, statistically:
      * loss and per-scale predictions within 3x the reference fp32 error (+1e-3);
      * median and 90th percentile of the per-parameter gradient errors (norm, and a fixed
        random projection of the gradient) within 3x the reference fp32 ones (+1e-3);
      * no single parameter beyond 10x max(its own reference fp32 error, the median one):
        a missing or wrong gradient term (an O(1) error) fails here;
      * parameters whose fp64 gradient is structurally zero stay at the rounding level, and
        parameters the reference leaves without gradient get none."""
    import json
    import math
    import os
    from conftest import GOLDEN, formula_state_dict, golden
    from hv_amd import HybridVisionSystem
    from hv_amd.targets import synthetic_targets
    from oracle import cases
    g = golden("train_base_224_b2")
    names = json.load(open(os.path.join(GOLDEN, "train_base_param_names.json")))
    m = HybridVisionSystem(dict(verbose=False, precision="fp32"))
    m.load_state_dict(formula_state_dict("base", "wc"))
    m = m.to(gpu_device).train()
    for mod in m.modules():
        if isinstance(mod, (torch.nn.Dropout, torch.nn.Dropout2d)):
            mod.p = 0.0
    B, S = int(g["B"]), int(g["S"])
    x = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(1)).to(gpu_device)
    tg = [t.to(gpu_device) for t in synthetic_targets(B, S, seed=int(g["target_seed"]))]
    out = m(x, targets=tg, compute_loss=True)
    out["loss"]["total_loss"].backward()
    torch.cuda.synchronize()
    l64, l32 = float(g["total_loss_f64"]), float(g["total_loss"])
    lm = out["loss"]["total_loss"].item()
    assert abs(lm / l64 - 1) <= 3 * abs(l32 / l64 - 1) + 1e-3, (lm, l32, l64)
    for s in range(3):
        p64 = g[f"pred{s}_f64"].astype(np.float64)
        e_ref = np.linalg.norm(g[f"pred{s}"] - p64) / np.linalg.norm(p64)
        mine = out["predictions"][f"scale_{s}"].detach().cpu().double().numpy()
        e = np.linalg.norm(mine - p64) / np.linalg.norm(p64)
        assert e <= 3 * e_ref + 1e-3, (s, e, e_ref)
    params = dict(m.named_parameters())
    n64, n32 = g["grad_norm_f64"], g["grad_norm"]
    p64, p32 = g["grad_probe_f64"], g["grad_probe"]
    gmax = float(n64.max())
    e_mine, e_ref, idx = [], [], []
    for i, n in enumerate(names):
        gr = params[n].grad
        if n64[i] < 0:
            assert gr is None or float(gr.abs().max()) == 0.0, n
            continue
        gr = gr.detach().double().cpu().flatten()
        nm = float(gr.norm())
        if n64[i] < 1e-9 * gmax:                    # structurally zero (bias before BN / LN shift)
            assert nm < 1e-8 * gmax, (n, nm)
            continue
        pm = float(gr @ cases.grad_probe(n, gr.numel())) / math.sqrt(gr.numel())
        e_mine.append(max(abs(nm - n64[i]), abs(pm - p64[i])) / n64[i])
        e_ref.append(max(abs(n32[i] - n64[i]), abs(p32[i] - p64[i])) / n64[i])
        idx.append(n)
    e_mine, e_ref = np.array(e_mine), np.array(e_ref)
    med_ref, p90_ref = np.median(e_ref), np.percentile(e_ref, 90)
    print(f"grad err median {np.median(e_mine):.3e} (ref fp32 {med_ref:.3e}), "
          f"p90 {np.percentile(e_mine, 90):.3e} (ref {p90_ref:.3e}), max {e_mine.max():.3e} (ref {e_ref.max():.3e})")
    assert np.median(e_mine) <= 3 * med_ref + 1e-3
    assert np.percentile(e_mine, 90) <= 3 * p90_ref + 1e-3
    bad = [(idx[i], e_mine[i], e_ref[i]) for i in range(len(idx)) if e_mine[i] > 10 * max(e_ref[i], med_ref)]
    assert not bad, bad[:10]


def _group_norms(named_norms):
    """Gradient norm per (top-level module, clip group): sqrt of the summed squared per-parameter
    norms; the clip groups are the trainer's (mhc_trainer.py:342-383: mHC parameters / others)."""
    from hv_amd.trainer import mhc_group
    acc = {}
    for n, v in named_norms:
        key = f"{n.split('.')[0]}/{'mhc' if mhc_group(n) == 0 else 'other'}"
        acc[key] = acc.get(key, 0.0) + float(v) ** 2
    return {k: v ** 0.5 for k, v in acc.items()}


def _base_train_step(gpu_device, precision, B, S, seed_x, target_seed):
    from conftest import formula_state_dict
    from hv_amd import HybridVisionSystem
    from hv_amd.targets import synthetic_targets
    m = HybridVisionSystem(dict(verbose=False, precision=precision))
    m.load_state_dict(formula_state_dict("base", "wc"))
    m = m.to(gpu_device).train()
    for mod in m.modules():
        if isinstance(mod, (torch.nn.Dropout, torch.nn.Dropout2d)):
            mod.p = 0.0
    x = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(seed_x)).to(gpu_device)
    tg = [t.to(gpu_device) for t in synthetic_targets(B, S, seed=target_seed)]
    out = m(x, targets=tg, compute_loss=True)
    out["loss"]["total_loss"].backward()
    torch.cuda.synchronize()
    loss = {k: float(v) for k, v in out["loss"].items() if torch.is_tensor(v) and v.numel() == 1}
    preds = {k: v.detach().float().cpu().numpy() for k, v in out["predictions"].items()}
    norms, finite = [], True
    for n, p in m.named_parameters():
        if p.grad is not None:
            finite &= bool(torch.isfinite(p.grad).all())
            norms.append((n, p.grad.detach().double().norm().item()))
    del out, m
    torch.cuda.empty_cache()
    return loss, preds, dict(norms), finite


# The ViT gradient groups are the one place the HIP bf16 step is noisier than the reference's own
# bf16 (medians over 9 batches at 224: 1.7x; over 5 at 640: 2.8-3.6x; every other group 0.45-1.3x).
# Bisected on the GPU (tools/vit_grad_probe.py bisect640, profiles/r06/parity/vit_bisect.txt): the
# attention core, the blocks' MLP Linears and the q / k / v outputs all in fp32 together only take
# the 640 median from 0.36 to 0.31 (the reference: 0.10), the fp32 residual stream and the
# softmax-consistent Delta of the attention backward (both kept: they are autocast's precision)
# move it by < 0.01.  No single op carries it; these two groups keep a 4x bound.
VIT_GROUP_BOUND = {"vit_encoder/other": 4.0, "vit_encoder/mhc": 4.0}


def _anchor_check(mine: dict, ref: dict, what: str, per_group: float = 1.5, mean: float = 1.5,
                  wide: Optional[dict] = None):
    """Per-group errors held to the reference's own bf16 errors (S8): each group within
    `per_group` x its reference error (`wide` overrides it per group; floor 1e-2: near-exact
    groups would otherwise test rounding), and the mean over groups within `mean` x the reference
    mean.  Both sides are medians over input batches where the caller has several (the groups
    are chaotic at init: one batch's ViT group 0.04, another's 0.79, on one build)."""
    wide = wide or {}
    bad = {k: (mine[k], ref[k]) for k in ref
           if mine.get(k, 1.0) > wide.get(k, per_group) * max(ref[k], 1e-2)}
    assert not bad, (what, bad)
    m_mean = float(np.mean([mine[k] for k in ref]))
    r_mean = float(np.mean(list(ref.values())))
    assert m_mean <= mean * r_mean, (what, m_mean, r_mean)
    return {"hip_mean": m_mean, "ref_bf16_mean": r_mean,
            "max_ratio": max(mine[k] / max(ref[k], 1e-2) for k in ref)}


def test_base_train_step_bf16_matches_reference_and_fp32(gpu_device):
    """Config C's object in its own precision: the base model's bf16 training step (bf16
    activations / GEMMs, fp32 parameters, coefficients and reductions -- the reference's autocast
    contract, manifold_layers.py:186,248, mhc_trainer.py:241; loss yolo_head.py:374-465), held to
    the REFERENCE's OWN bf16 error (S8: the reference run under CUDA autocast's bf16 op policy,
    oracle/autocast_emu.py, fixtures *_bf16ref / train_base_640_b2_ref):
      (1) 224x224 B=2 vs the reference's fp64 run (fixture train_base_224_b2): total loss within
          3x the reference-bf16 loss error; per (top-level module, clip group) gradient norm --
          the quantities the trainer's per-group clipping (mhc_trainer.py:342-383) acts on --
          within 1.5x the reference-bf16 group error, mean over groups within 1.5x, both sides the
          MEDIAN over three input batches (x seeds 1, 2, 3; fixtures train_base_224_b2 and
          train_base_224_b2_seeds: the reference in fp64 and under the bf16 policy per batch);
          head logits within 1.25x the reference-bf16 logits error;
      (2) 640x640 B=2 (config C's resolution), HIP bf16 vs HIP fp32 on the same batch, against the
          reference's bf16-vs-fp32 on the same batches (x seeds 7-11, targets seed 11; fixtures
          train_base_640_b2_ref and train_base_640_b2_seeds): gradient groups as medians over the
          five batches on both sides, loss / logits on the fixture batch, plus finiteness of every
          gradient.
    Train-mode logits at init are NOT a usable bf16 observable: BatchNorm batch statistics over
    B=2 amplify rounding, and the reference's own bf16 logits are 0.89-0.96 rel-L2 from its
    fp64 / fp32 runs (measured on the fixtures) -- the loss and gradient groups are."""
    import json
    import os
    from conftest import GOLDEN, golden, record_parity
    g = golden("train_base_224_b2")
    gb = golden("train_base_224_b2_bf16ref")
    names = json.load(open(os.path.join(GOLDEN, "train_base_param_names.json")))
    B, S = int(g["B"]), int(g["S"])
    loss16, p16, n16, fin16 = _base_train_step(gpu_device, "bf16", B, S, 1, int(g["target_seed"]))
    assert fin16
    ref64 = _group_norms([(n, v) for n, v in zip(names, g["grad_norm_f64"]) if v >= 0])
    refb = _group_norms([(n, v) for n, v in zip(names, gb["grad_norm"]) if v >= 0])
    mine = _group_norms(n16.items())
    l64 = float(g["total_loss_f64"])
    med = lambda ds: {k: float(np.median([d[k] for d in ds])) for k in ds[0]}   # noqa: E731
    # group errors per input batch: x seed 1 (the fixture), 2 and 3 (train_base_224_b2_seeds)
    gs = golden("train_base_224_b2_seeds")
    e_seed = [{k: abs(mine.get(k, 0.0) / v - 1) for k, v in ref64.items() if v > 0}]
    r_seed = [{k: abs(refb[k] / v - 1) for k, v in ref64.items() if v > 0}]
    for xs in cases.TRAIN224_SEEDS:
        _, _, n16s, fin = _base_train_step(gpu_device, "bf16", B, S, xs, int(g["target_seed"]))
        assert fin
        r64s = _group_norms([(n, v) for n, v in zip(names, gs[f"grad_norm_f64_s{xs}"]) if v >= 0])
        rbs = _group_norms([(n, v) for n, v in zip(names, gs[f"grad_norm_bf16_s{xs}"]) if v >= 0])
        mines = _group_norms(n16s.items())
        e_seed.append({k: abs(mines.get(k, 0.0) / v - 1) for k, v in r64s.items() if v > 0})
        r_seed.append({k: abs(rbs[k] / v - 1) for k, v in r64s.items() if v > 0})
    e_groups, r_groups = med(e_seed), med(r_seed)
    e_log = {s: float(np.linalg.norm(p16[f"scale_{s}"] - g[f"pred{s}_f64"]) / np.linalg.norm(g[f"pred{s}_f64"]))
             for s in range(3)}
    r_log = {s: float(gb[f"pred{s}_err_vs_f64"]) for s in range(3)}
    rec = {"224_b2_vs_ref_f64": {"loss_rel": abs(loss16["total_loss"] / l64 - 1),
                                 "ref_bf16_loss_rel": abs(float(gb["total_loss"]) / l64 - 1),
                                 "x_seeds": [1] + list(cases.TRAIN224_SEEDS),
                                 "statistic": f"median over the {1 + len(cases.TRAIN224_SEEDS)} batches",
                                 "group_norm_rel": e_groups, "ref_bf16_group_norm_rel": r_groups,
                                 "group_norm_rel_per_seed": e_seed, "ref_bf16_group_norm_rel_per_seed": r_seed,
                                 "logits_rel_l2": e_log, "ref_bf16_logits_rel_l2": r_log}}
    r1 = rec["224_b2_vs_ref_f64"]
    # (2) config C's resolution: bf16 vs fp32 HIP on the same batch, against the reference's own
    # on the same batches.  A gradient group's bf16 error at init is a heavy-tailed function of
    # where the roundings fall (one batch's ViT group measured 0.04, another 0.79 on the same
    # build; the reference's own per-batch values spread as widely), so both sides are medians
    # over several batches
    gr = golden("train_base_640_b2_ref")
    gr2 = golden("train_base_640_b2_seeds")
    seeds640 = (7,) + tuple(cases.TRAIN640_SEEDS)
    runs, ref_runs = [], []
    for xs in seeds640:
        loss32, p32, n32, fin32 = _base_train_step(gpu_device, "fp32", 2, 640, xs, 11)
        loss16b, p16b, n16b, fin16b = _base_train_step(gpu_device, "bf16", 2, 640, xs, 11)
        assert fin32 and fin16b
        g32, g16 = _group_norms(n32.items()), _group_norms(n16b.items())
        assert set(g16) == set(g32)
        runs.append(({k: abs(g16.get(k, 0.0) / v - 1) for k, v in g32.items() if v > 0},
                     {k: abs(loss16b[k] / loss32[k] - 1) for k in loss32 if abs(loss32[k]) > 1e-6},
                     {k: float(np.linalg.norm(p16b[k] - p32[k]) / np.linalg.norm(p32[k])) for k in p32}))
        sfx = "" if xs == 7 else f"_s{xs}"
        src = gr if xs == 7 else gr2
        rf32 = _group_norms([(n, v) for n, v in zip(names, src["grad_norm_f32" + sfx]) if v >= 0])
        rf16 = _group_norms([(n, v) for n, v in zip(names, src["grad_norm_bf16" + sfx]) if v >= 0])
        ref_runs.append({k: abs(rf16[k] / v - 1) for k, v in rf32.items() if v > 0})
    e2 = med([r[0] for r in runs])
    r2g = med(ref_runs)
    rec["640_b2_bf16_vs_fp32"] = {
        "x_seeds": list(seeds640), "statistic": f"median over the {len(seeds640)} batches, both sides",
        "loss_rel": med([r[1] for r in runs]),
        "ref_bf16_loss_rel": abs(float(gr["total_loss_bf16"]) / float(gr["total_loss_f32"]) - 1),
        "group_norm_rel": e2, "ref_bf16_group_norm_rel": r2g,
        "ref_bf16_group_norm_rel_per_seed": ref_runs,
        "group_norm_rel_per_seed": [r[0] for r in runs],
        "logits_rel_l2": med([r[2] for r in runs]),
        "ref_bf16_logits_rel_l2": [float(v) for v in gr["logits_rel_l2_bf16_vs_f32"]]}
    r2 = rec["640_b2_bf16_vs_fp32"]
    record_parity("train_bf16_base", rec)          # on file before any bound is checked
    r1["groups"] = _anchor_check(e_groups, r_groups, "224 groups", wide=VIT_GROUP_BOUND)
    r2["groups"] = _anchor_check(e2, r2g, "640 groups", wide=VIT_GROUP_BOUND)
    record_parity("train_bf16_base", rec)
    assert r1["loss_rel"] <= 3.0 * r1["ref_bf16_loss_rel"], r1
    for s in range(3):
        assert e_log[s] <= 1.25 * r_log[s], (s, e_log, r_log)
    assert r2["loss_rel"]["total_loss"] <= 3.0 * r2["ref_bf16_loss_rel"], r2
    for s in range(3):
        assert r2["logits_rel_l2"][f"scale_{s}"] <= 1.25 * r2["ref_bf16_logits_rel_l2"][s], r2


def test_large_1024_train_step_bf16_vs_fp32(gpu_device):
    """Config D's training leg at its per-GPU shape (1024x1024, B=8 -- bench.py's `large`
    training line): the bf16 step against the fp32 HIP step on the same batch.  No reference
    run exists at this size (the CPU reference needs ~1 h per precision), so the anchors are the
    reference's own bf16-vs-fp32 errors at config C's 640 B=2 (fixture train_base_640_b2_ref,
    S8): total loss within 3x, per-group gradient norms within 3x (mean 2x); every gradient
    finite; the loss components all present and positive."""
    from conftest import golden, record_parity
    import json
    import os
    from conftest import GOLDEN
    names = json.load(open(os.path.join(GOLDEN, "train_base_param_names.json")))
    gr = golden("train_base_640_b2_ref")
    loss32, _, n32, fin32 = _base_train_step(gpu_device, "fp32", 8, 1024, 5, 13)
    loss16, _, n16, fin16 = _base_train_step(gpu_device, "bf16", 8, 1024, 5, 13)
    assert fin32 and fin16
    g32, g16 = _group_norms(n32.items()), _group_norms(n16.items())
    rf32 = _group_norms([(n, v) for n, v in zip(names, gr["grad_norm_f32"]) if v >= 0])
    rf16 = _group_norms([(n, v) for n, v in zip(names, gr["grad_norm_bf16"]) if v >= 0])
    e = {k: abs(g16.get(k, 0.0) / v - 1) for k, v in g32.items() if v > 0}
    r = {k: abs(rf16[k] / v - 1) for k, v in rf32.items() if v > 0}
    rec = {"config": "base 1024x1024 B=8 train step, bf16 vs fp32 HIP",
           "loss_bf16": loss16, "loss_fp32": loss32,
           "loss_rel": abs(loss16["total_loss"] / loss32["total_loss"] - 1),
           "ref640_bf16_loss_rel": abs(float(gr["total_loss_bf16"]) / float(gr["total_loss_f32"]) - 1),
           "group_norm_rel": e, "ref640_bf16_group_norm_rel": r}
    rec["groups"] = _anchor_check(e, r, "1024 groups", per_group=3.0, mean=2.0)   # across resolutions
    record_parity("train_bf16_large_1024", rec)
    for k in ("coord_loss", "obj_loss", "noobj_loss", "cls_loss", "total_loss"):
        assert loss16[k] > 0 and np.isfinite(loss16[k]), (k, loss16)
    assert rec["loss_rel"] <= 3.0 * rec["ref640_bf16_loss_rel"], rec


def test_tiny_train_step_bf16_runs_and_agrees(gpu_device):
    """bf16 activations through the whole training step.  The model's gradient at init is so
    ill-conditioned that the oracle's own fp32 gradients are ~1% (median) away from fp64
    (see test above) -- bf16 rounding (2^16 x larger) leaves no per-parameter agreement to
    test at model level, so this checks finiteness and the loss; per-op bf16 gradients are
    pinned by the kernel/layer tests above (e.g. test_mhc_bf16_train_agreement)."""
    from hv_amd.targets import synthetic_targets
    m32, _ = _tiny_model(gpu_device, "fp32")
    m16, _ = _tiny_model(gpu_device, "bf16")
    B, S = 2, 64
    x = torch.randn(B, 3, S, S, device=gpu_device)
    tg = [t.to(gpu_device) for t in synthetic_targets(B, S, seed=3)]
    l32 = m32(x, targets=tg, compute_loss=True)["loss"]["total_loss"]
    l32.backward()
    l16 = m16(x, targets=tg, compute_loss=True)["loss"]["total_loss"]
    l16.backward()
    assert abs(l16.item() / l32.item() - 1) < 0.15
    for p in m16.parameters():
        if p.grad is not None:
            assert torch.isfinite(p.grad).all()


def test_fused_adamw_per_parameter_steps_match_torch(gpu_device):
    """A parameter without gradient for the first steps keeps its own step count: its AdamW
    bias correction 1 - beta^t uses that count (torch.optim.AdamW state['step']), not the
    optimizer's global step; the state_dict reports the same counts as torch."""
    from hv_amd.trainer import FusedAdamW
    torch.manual_seed(1)
    named = [("a.conv.weight", torch.randn(300)), ("b.bias", torch.randn(7)), ("c.mhc.H_res_raw", torch.randn(5, 5))]
    mine = [(n, t.clone().to(gpu_device).requires_grad_(True)) for n, t in named]
    ref = [(n, t.clone().requires_grad_(True)) for n, t in named]
    opt = FusedAdamW(mine, lr=1e-2, weight_decay=1e-2)
    topt = torch.optim.AdamW([p for _, p in ref], lr=1e-2, weight_decay=1e-2, eps=1e-8)
    for step in range(5):
        active = (True, step >= 2, step % 2 == 0)
        for i, ((_, p), (_, q)) in enumerate(zip(mine, ref)):
            gr = torch.randn_like(q)
            p.grad = gr.clone().to(gpu_device)
            q.grad = gr.clone() if active[i] else None
        opt.step(clip=False, active=active)
        topt.step()
    for (n, a), (_, b) in zip(mine, ref):
        assert rel(a.detach(), b.detach()) < 1e-5, n
    tsd, msd = topt.state_dict()["state"], opt.state_dict()["state"]
    assert set(tsd) == set(msd)
    for i in tsd:
        assert float(tsd[i]["step"]) == float(msd[i]["step"]), i


def test_trainer_step_reduces_loss(gpu_device):
    from hv_amd.targets import synthetic_targets
    from hv_amd.trainer import HVTrainer
    m, _ = _tiny_model(gpu_device, "bf16")
    tr = HVTrainer(m, lr=1e-3)
    B, S = 2, 64
    x = torch.randn(B, 3, S, S, device=gpu_device)
    tg = [t.to(gpu_device) for t in synthetic_targets(B, S, seed=3)]
    losses = [tr.step(x, tg)["total_loss"].item() for _ in range(6)]
    assert all(np.isfinite(losses))
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_trainer_graph_step_equals_eager(gpu_device, precision):
    """HVTrainer(graph=True): step 1 eager, step 2 captured into a hipGraph and replayed, later
    steps replays (monitor steps eager) -- forward, YOLOLoss, backward (Sinkhorn autograd
    included), gradient flush, clipping and AdamW.  With dropout off, every step leaves the
    parameters, the optimizer moments and the BN statistics BITWISE equal to the eager trainer's
    on the same batches (the graph replays exactly the launches an eager step issues)."""
    from hv_amd.targets import synthetic_targets
    from hv_amd.trainer import HVTrainer
    ma, _ = _tiny_model(gpu_device, precision)
    mb, _ = _tiny_model(gpu_device, precision)
    ta = HVTrainer(ma, lr=1e-3, monitor_every=4)
    tb = HVTrainer(mb, lr=1e-3, monitor_every=4, graph=True)
    B, S = 2, 96
    gen = torch.Generator().manual_seed(5)
    for step in range(6):
        x = torch.randn(B, 3, S, S, generator=gen).to(gpu_device)
        tg = [t.to(gpu_device) for t in synthetic_targets(B, S, seed=20 + step)]
        la = {k: float(v) for k, v in ta.step(x, tg).items()}
        lb = {k: float(v) for k, v in tb.step(x, tg).items()}
        torch.cuda.synchronize()
        assert la == lb, (step, la, lb)
        for (n, pa), (_, pb) in zip(ma.named_parameters(), mb.named_parameters()):
            assert torch.equal(pa, pb), (step, n)
        for (n, ba), (_, bb) in zip(ma.named_buffers(), mb.named_buffers()):
            if "running" in n or "num_batches" in n:
                assert torch.equal(ba, bb), (step, n)
        for a, b in zip(ta.opt.exp_avg_sq, tb.opt.exp_avg_sq):
            assert torch.equal(a, b)
    assert tb.captures == 1 and tb.replays == 4          # steps 2-4 and 6; 1 (warm-up) and 5 (monitor) eager
    assert ta.opt.param_steps == tb.opt.param_steps


def test_trainer_graph_dropout_masks_change_per_replay(gpu_device):
    """With dropout on, the replayed graph draws NEW masks every step (the dropout kernels add
    the device seed-offset word the graph advances), so two replays on the same batch with lr = 0
    (parameters unchanged) give different losses -- and identical ones with dropout off."""
    from hv_amd import HybridVisionSystem
    from hv_amd.targets import synthetic_targets
    from hv_amd.trainer import HVTrainer, SEED_STRIDE
    from oracle import weights as W
    B, S = 2, 96
    x = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(3)).to(gpu_device)
    tg = [t.to(gpu_device) for t in synthetic_targets(B, S, seed=4)]
    res = {}
    for drop in (True, False):
        m = HybridVisionSystem(dict(num_blocks=[1, 1, 1, 1], vit_depth=1, sk_iters=5, verbose=False))
        W.load_formula_weights(m, "wc")
        m = m.to(gpu_device).train()
        if not drop:
            for mod in m.modules():
                if isinstance(mod, (torch.nn.Dropout, torch.nn.Dropout2d)):
                    mod.p = 0.0
        tr = HVTrainer(m, lr=0.0, weight_decay=0.0, monitor_every=0, graph=True)
        off0 = int(tr.seed_offset.item())
        losses = [float(tr.step(x, tg)["total_loss"]) for _ in range(4)]
        assert tr.replays == 3
        assert int(tr.seed_offset.item()) == (off0 + 4 * SEED_STRIDE + 2 ** 31) % 2 ** 32 - 2 ** 31
        res[drop] = losses
    assert res[True][2] != res[True][3] and res[True][1] != res[True][2]
    assert res[False][1] == res[False][2] == res[False][3]


def test_trainer_graph_hyperparameters_without_recapture(gpu_device):
    """AdamW reads lr / betas / eps / weight decay from the optimizer's DEVICE array, refreshed
    before every replay: a scheduler changing lr every step (mhc_trainer.py:275) keeps replaying
    ONE captured graph, and the replayed steps equal the eager trainer's under the same schedule
    bit for bit; lr = wd = 0 after a change leaves the parameters bit-identical (a stale replay
    would not).  The clip norms and the model's kernel variants are baked in: changing them
    re-captures.  step_count counts steps, not captures."""
    from hv_amd.targets import synthetic_targets
    from hv_amd.trainer import HVTrainer
    ma, _ = _tiny_model(gpu_device, "bf16")
    mb, _ = _tiny_model(gpu_device, "bf16")
    ta = HVTrainer(ma, lr=1e-3, monitor_every=0)
    tb = HVTrainer(mb, lr=1e-3, monitor_every=0, graph=True)
    B, S = 2, 96
    x = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(9)).to(gpu_device)
    tg = [t.to(gpu_device) for t in synthetic_targets(B, S, seed=9)]
    for step in range(6):
        lr = 1e-3 * (0.5 + 0.5 * np.cos(np.pi * step / 6))     # cosine schedule, new value per step
        for t in (ta, tb):
            t.opt.lr = lr
            t.opt.wd = 1e-4 * (1 + step)
            t.step(x, tg)
        torch.cuda.synchronize()
        for (n, pa), (_, pb) in zip(ma.named_parameters(), mb.named_parameters()):
            assert torch.equal(pa, pb), (step, n)
    assert tb.captures == 1 and tb.replays == 5 and tb.opt.step_count == 6
    tb.opt.lr, tb.opt.wd = 0.0, 0.0
    before = [p.detach().clone() for p in mb.parameters()]
    tb.step(x, tg)
    torch.cuda.synchronize()
    assert tb.captures == 1 and tb.opt.step_count == 7
    for a, p in zip(before, mb.parameters()):
        assert torch.equal(a, p)
    tb.opt.max_norms[0] = 0.25
    tb.step(x, tg)
    assert tb.captures == 2
    mb.set_options(use_fused_mhc=False)
    tb.step(x, tg)
    assert tb.captures == 3 and tb.opt.step_count == 9


def test_trainer_skips_parameters_without_gradient(gpu_device):
    """final_fusion / output_projection feed no loss term, so their gradients stay None in the
    reference and torch.optim / ManifoldAwareOptimizer (optimizer.py:144) skip them: no weight
    decay, no moment update.  They must stay bit-identical through HVTrainer steps."""
    from hv_amd.targets import synthetic_targets
    from hv_amd.trainer import HVTrainer
    m, _ = _tiny_model(gpu_device, "bf16")
    tr = HVTrainer(m, lr=1e-3, weight_decay=0.1)
    frozen = {n: p.detach().clone() for n, p in m.named_parameters()
              if n.startswith(("final_fusion.", "output_projection."))}
    used = m.detection_head.pred_heads[0].pred_conv.weight.detach().clone()
    B, S = 2, 64
    x = torch.randn(B, 3, S, S, device=gpu_device)
    tg = [t.to(gpu_device) for t in synthetic_targets(B, S, seed=3)]
    for _ in range(2):
        tr.step(x, tg)
    torch.cuda.synchronize()
    for n, p in m.named_parameters():
        if n in frozen:
            assert torch.equal(p.detach(), frozen[n]), n
    assert not torch.equal(m.detection_head.pred_heads[0].pred_conv.weight.detach(), used)
    names = [n for n, _ in tr.opt.named]
    assert all(tr.opt.param_steps[names.index(n)] == 0 for n in frozen)


def test_final_features_trainable_and_no_grad_train_mode(gpu_device):
    """final_features stays in the autograd graph (hybrid_vision.py:369-402): a loss on it
    reaches final_fusion, output_projection and the FPN; and a train-mode forward under
    torch.no_grad (BN recalibration) still uses batch statistics and updates running stats."""
    m, _ = _tiny_model(gpu_device, "fp32")
    x = torch.randn(2, 3, 64, 64, device=gpu_device)
    out = m(x)
    out["final_features"].pow(2).sum().backward()
    for p in (m.final_fusion.H_pre_raw, m.final_fusion.H_res_raw, m.output_projection[4].weight,
              m.feature_fusion.output_convs[0].weight):
        assert p.grad is not None and p.grad.abs().max().item() > 0
    assert m.detection_head.pred_heads[0].pred_conv.weight.grad is None   # not on this loss's path
    bn = next(mod for mod in m.modules() if isinstance(mod, torch.nn.BatchNorm2d))
    before = bn.running_mean.clone()
    with torch.no_grad():
        m(x)
    torch.cuda.synchronize()
    assert not torch.equal(bn.running_mean, before)


def test_module_level_training_api(gpu_device):
    """The drop-in modules train on their own (reference test style, test_models.py:130-187):
    finite outputs, gradients reach every parameter that influences the output, and the
    training-mode stability monitor fills the reference buffers."""
    from hv_amd import ConvMHCLayer, ManifoldHyperConnection, TransformerEncoderBlock
    torch.manual_seed(0)
    m = ManifoldHyperConnection(64, expansion_rate=4).to(gpu_device).train()
    x = torch.randn(2, 10, 64, device=gpu_device, requires_grad=True)
    y = m(x)
    y.float().pow(2).mean().backward()
    assert torch.isfinite(x.grad).all()
    gn = torch.nn.utils.clip_grad_norm_(m.parameters(), 1e9)
    assert torch.isfinite(gn) and gn < 100
    met = m.get_stability_metrics()
    assert "signal_ratio" in met and met["max_eigenvalue"] <= 1.0 + 1e-3
    c = ConvMHCLayer(32, 32, 3, 1).to(gpu_device).train()
    xi = torch.randn(2, 32, 16, 16, device=gpu_device, requires_grad=True)
    c(xi).float().sum().backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in c.parameters())
    blk = TransformerEncoderBlock(256, 8).to(gpu_device).train()
    t = torch.randn(2, 17, 256, device=gpu_device, requires_grad=True)
    blk(t).float().sum().backward()
    assert torch.isfinite(t.grad).all()


@pytest.mark.parametrize("M,N,K,act,ln", [(300, 136, 128, "gelu", False), (1000, 256, 256, "silu", True),
                                          (777, 96, 64, "leaky", False), (1300, 1100, 1024, "gelu", False)])
def test_gemm_train_staged_epilogue_bitwise(gpu_device, M, N, K, act, ln):
    """The LDS-staged training epilogue (the default; variant GV_FLAT_TRAIN = fragment layout) writes exactly the
    bits of the fragment-layout one: pre-activation, dropout(act) output (mode 1) and the
    gradient through act + dropout with a residual (mode 2), incl. the LayerNorm-after-product
    variant and ragged M / N."""
    from hv_amd import _lib, ops
    T = OT()
    g = torch.Generator().manual_seed(M + N)
    a = torch.randn(M, K, generator=g).to(torch.bfloat16).to(gpu_device)
    b = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(gpu_device)
    bias = torch.randn(N, generator=g).to(gpu_device)
    res = torch.randn(M, N, generator=g).to(torch.bfloat16).to(gpu_device)
    kw = {}
    if ln:
        mean, rstd = ops.row_stats(a, 1e-5)
        kw = dict(a_mean=mean, a_rstd=rstd, b_colsum=b.float().sum(1))
    outs = {}
    from conftest import gemm_variant
    # staged (default) / fragment-layout epilogue, and the 256x256 ping-pong kernel with the
    # training epilogues (GV_TILE_256 forces it; the automatic choice takes it for long K and wide N)
    # ("nopf": the gradient epilogue loading each pass's aux rows after the previous pass's
    # stores instead of one pass ahead, HV_GV_TRAIN_NOPF)
    for key, v in (("staged", 0), ("flat", _lib.GV_FLAT_TRAIN), ("pp256", _lib.GV_TILE_256),
                   ("nopf", _lib.GV_TRAIN_NOPF)):
        if key == "pp256" and K % 64:
            continue
        with gemm_variant(v):
            pre = torch.empty(M, N, device=gpu_device, dtype=torch.bfloat16)
            y = T.gemm_train(a, b, mode=1, act=act, aux=pre, bias=bias, drop_p=0.2, seed=5, **kw)
            dpre = T.gemm_train(a, b, mode=2, act=act, aux=pre, drop_p=0.2, seed=5, residual=res)
            dpre0 = T.gemm_train(a, b, mode=2, act=act, aux=pre, drop_p=0.2, seed=5)
            outs[key] = (pre, y, dpre, dpre0)
    for key in outs:
        for x0, x1 in zip(outs["staged"], outs[key]):
            assert torch.equal(x0, x1), key


@pytest.mark.parametrize("M,N,K,tile", [(300, 136, 128, 0), (1000, 256, 256, 0), (777, 96, 64, 0), (4100, 1024, 512, 0),
                                        (1000, 256, 256, 1), (1000, 256, 256, 3), (200, 64, 128, 4)])
def test_gemm_train_epilogue_colsum(gpu_device, M, N, K, tile):
    """gemm_train(mode 2, colsum=): the bias gradient summed in the gradient epilogue
    (hv_gemm_desc.colsum_part, per 64-row block, reduced by hv_colsum_final) equals the column
    sums of the stored output, for every training tile shape (forced 128x128 / 128x64 / 64x64,
    automatic 64x128) and ragged M / N; C itself is bitwise the colsum-free launch's; a variant
    whose kernel cannot sum (GV_TRAIN_NOPF) falls back to the separate pass."""
    from hv_amd import _lib
    T = OT()
    g = torch.Generator().manual_seed(M + N + tile)
    a = torch.randn(M, K, generator=g).to(torch.bfloat16).to(gpu_device)
    b = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(gpu_device)
    pre = torch.randn(M, N, generator=g).to(torch.bfloat16).to(gpu_device)
    from conftest import gemm_variant
    for v in (tile, _lib.GV_TRAIN_NOPF):
        with gemm_variant(v):
            db = torch.full((N,), float("nan"), device=gpu_device)
            d0 = T.gemm_train(a, b, mode=2, act="gelu", aux=pre, drop_p=0.2, seed=5)
            d1 = T.gemm_train(a, b, mode=2, act="gelu", aux=pre, drop_p=0.2, seed=5, colsum=db)
        assert torch.equal(d0, d1)
        ref = T.colsum(d1)
        assert torch.allclose(db, ref, rtol=1e-5, atol=1e-4 * ref.abs().max().item()), (v, (db - ref).abs().max())


def test_dropout_seed_offset_word(gpu_device):
    """hv_kernels.h seed_offset: every dropout kernel (GEMM training epilogue, row norm,
    elementwise dropout / activation backward, MFMA attention forward + backward) uses
    seed + *seed_offset -- bitwise the same masks as passing that sum as the seed."""
    from hv_amd.runtime import set_train_state
    T = OT()
    g = torch.Generator().manual_seed(8)
    bf = torch.bfloat16
    a = torch.randn(200, 64, generator=g).to(bf).to(gpu_device)
    b = (torch.randn(96, 64, generator=g) / 8).to(bf).to(gpu_device)
    x = torch.randn(70, 256, generator=g).to(bf).to(gpu_device)
    q, k, v = (torch.randn(2, 50, 256, generator=g).to(bf).to(gpu_device) for _ in range(3))
    off = torch.tensor([123457], dtype=torch.int32, device=gpu_device)
    s0 = 1000

    def run(seed):
        pre = torch.empty(200, 96, device=gpu_device, dtype=bf)
        out = [T.gemm_train(a, b, mode=1, act="gelu", aux=pre, drop_p=0.3, seed=seed)]
        out.append(T.gemm_train(a, b, mode=2, act="gelu", aux=pre, drop_p=0.3, seed=seed))
        out.append(T.rownorm_train(0, x, 1e-5, None, None, 0.3, seed)[0])
        out.append(T.dropout(x, 0.3, seed))
        out.append(T.act_backward(x, x, "gelu", 0.3, seed))
        o, lse = T.attention_train(q, k, v, 8, 0.2, seed)
        out += [o, *T.attention_backward(q, k, v, o, o, lse, 8, 0.2, seed)]
        return out

    set_train_state(seed_offset=off)
    try:
        with_off = run(s0)
    finally:
        set_train_state()
    plain = run(s0 + 123457)
    other = run(s0)
    for i, (u, w) in enumerate(zip(with_off, plain)):
        assert torch.equal(u, w), i
    assert not torch.equal(with_off[3], other[3])


def test_trainer_manifold_regularization_matches_reference_formula(gpu_device):
    """HVTrainer(manifold_weight=w) / model.hv_manifold_weight: total_loss = detection + w * reg
    with the reference trainer's regulariser (mhc_trainer.py:248-255,299-340): mean over the mHC
    sites of mean|rowsum(H)-1| + mean|colsum(H)-1| + 0.1 mean relu(eigvalsh(H)-1), H =
    SK(H_res_raw).
      * the formula (hv_amd.train_model.manifold_regularization) on matrices FAR from doubly
        stochastic (so rounding does not decide the |.| signs), value and gradient, vs fp64 autograd
        of the reference expression on the CPU;
      * in the model: the reported manifold_loss equals the formula on the oracle's fp64 Sinkhorn of
        every site up to fp32 rounding of the row / column sums (the projections are column-exact:
        the term is ~1e-5, at the rounding level of a 1792-element fp32 sum), total_loss -
        detection == w * manifold_loss, and the term adds a finite, nonzero gradient to the
        H_res_raw parameters only."""
    import torch.nn.functional as Fn
    from hv_amd.targets import synthetic_targets
    from hv_amd.train_model import manifold_regularization
    from oracle import hv_oracle as O

    def ref_formula(hs):
        terms = [(h.sum(1) - 1).abs().mean() + (h.sum(0) - 1).abs().mean() +
                 0.1 * Fn.relu(torch.linalg.eigvalsh(h) - 1).mean() for h in hs]
        return torch.stack(terms).mean()

    g = torch.Generator().manual_seed(4)
    hs = [(torch.rand(n, n, generator=g) * 2.5 / n).double() for n in (8, 32, 100)]
    hs[1] = hs[1] + torch.eye(32, dtype=torch.float64) * 0.8          # eigenvalues above 1 too
    mine = [h.float().to(gpu_device).requires_grad_(True) for h in hs]
    val = manifold_regularization({i: h for i, h in enumerate(mine)})
    val.backward()
    refs = [h.clone().requires_grad_(True) for h in hs]
    rv = ref_formula(refs)
    rv.backward()
    assert abs(val.item() / rv.item() - 1) < 1e-5
    for a, b in zip(mine, refs):
        assert (a.grad.double().cpu() - b.grad).norm() <= 1e-5 * b.grad.norm()

    B, S, w = 2, 64, 0.5
    x = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(1)).to(gpu_device)
    tg = [t.to(gpu_device) for t in synthetic_targets(B, S, seed=3)]
    res = {}
    for weight in (0.0, w):
        m, _ = _tiny_model(gpu_device)
        m.hv_manifold_weight = weight
        out = m(x, targets=tg, compute_loss=True)
        out["loss"]["total_loss"].backward()
        torch.cuda.synchronize()
        res[weight] = (m, {k: float(v) for k, v in out["loss"].items() if torch.is_tensor(v) and v.numel() == 1})
    m0, l0 = res[0.0]
    m1, l1 = res[w]
    with torch.no_grad():
        hs = [O.sinkhorn(mm.H_res_raw.detach().double().cpu(), mm.sinkhorn.num_iterations)
              for mm in m1.modules() if hasattr(mm, "H_res_raw")]
        reg = ref_formula(hs).item()
    assert abs(l1["manifold_loss"] - reg) < 5e-7, (l1["manifold_loss"], reg)
    assert abs((l1["total_loss"] - l0["total_loss"]) - w * l1["manifold_loss"]) < 1e-5 * max(1.0, abs(l0["total_loss"]))
    named0 = dict(m0.named_parameters())
    moved = 0
    for n, p1 in m1.named_parameters():
        g0 = named0[n].grad
        if p1.grad is None:                          # a parameter neither loss reaches
            assert g0 is None, n
            continue
        if g0 is None:                               # reached by the regulariser only (final_fusion)
            assert n.endswith("H_res_raw"), n
            g0 = torch.zeros_like(p1.grad)
        extra = p1.grad - g0
        assert torch.isfinite(extra).all(), n
        if n.endswith("H_res_raw"):
            moved += int(extra.abs().max().item() > 0)
        else:
            assert extra.abs().max().item() <= 1e-6 * max(1.0, g0.abs().max().item()), n
    assert moved > 0
