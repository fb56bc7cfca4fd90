"""torch.ops.hv.* (SURVEY §8b): the C-ABI launchers as PyTorch dispatcher operators.  Each op
matches the module path that the parity tests pin (same kernels), its autograd matches the
module's training autograd, and the ops are visible to torch.compile / torch.export (fake
kernels: no graph break, exported graph holds the hv ops)."""
import pytest
import torch

from oracle import cases
from oracle import weights as W

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _mhc_args(m):
    return (m.H_pre_raw, m.H_post_raw, m.H_res_raw, m.norm_pre.weight, m.norm_pre.bias, m.mlp[0].weight,
            m.mlp[0].bias, m.mlp[3].weight, m.mlp[3].bias, m.norm_post.weight, m.norm_post.bias)


@pytest.mark.parametrize("D,e,prec", [(64, 4, "fp32"), (256, 2, "fp32"), (128, 4, "bf16")])
def test_hv_mhc_op_forward_and_autograd(gpu_device, D, e, prec):
    import hv_amd  # noqa: F401  (registers the ops)
    from hv_amd import ManifoldHyperConnection
    dt = torch.float32 if prec == "fp32" else torch.bfloat16
    m = ManifoldHyperConnection(D, expansion_rate=e, use_mixed_precision=prec == "bf16", dropout_rate=0.0)
    W.load_formula_weights(m, "wc")
    m = m.to(gpu_device)
    x = cases.mhc_input(D, e).to(gpu_device).to(dt)
    m.eval()
    with torch.no_grad():
        ref = m(x)
        y = torch.ops.hv.mhc(x, *_mhc_args(m), m.sinkhorn.num_iterations)
    assert torch.equal(y, ref)                    # same plan, same kernels as the module forward
    # autograd: the op's backward vs the module's training autograd (dropout 0)
    m.train()
    m.monitor_every = 0
    xa = x.clone().requires_grad_(True)
    g = torch.randn(x.shape, generator=torch.Generator().manual_seed(D)).to(gpu_device).to(dt)
    m.zero_grad()
    m(xa).backward(g)
    ref_grads = [xa.grad.clone()] + [p.grad.clone() for p in _mhc_args(m)]
    xb = x.clone().requires_grad_(True)
    params = [p.detach().clone().requires_grad_(True) for p in _mhc_args(m)]
    y = torch.ops.hv.mhc(xb, *params, m.sinkhorn.num_iterations)
    y.backward(g)
    mine = [xb.grad] + [p.grad for p in params]
    tol = 1e-4 if prec == "fp32" else 2e-2
    for i, (a, b) in enumerate(zip(mine, ref_grads)):
        assert rel(a, b) < tol, (i, rel(a, b))


def test_hv_small_ops_forward_and_autograd(gpu_device):
    import hv_amd  # noqa: F401
    from hv_amd import ops
    from hv_amd import train_fn as TF
    g = torch.Generator().manual_seed(3)
    dev = gpu_device
    # sinkhorn: forward == ops.sinkhorn, backward == the grouped reverse sweep
    raw = cases.sinkhorn_raw(64, 20, "wc").to(dev).requires_grad_(True)
    M, h = torch.ops.hv.sinkhorn(raw, 20, 1e-8, 1.0)
    M0, h0 = ops.sinkhorn(raw.detach(), 20)
    assert torch.equal(M, M0.squeeze(0)) and torch.equal(h, h0[:20])
    G = torch.randn(64, 64, generator=g).to(dev)
    (M * G).sum().backward()
    grp = ops.SinkhornGroup([raw.detach()], [20], dev)
    grp.run()
    assert torch.allclose(raw.grad, grp.backward([G])[0], rtol=0, atol=0)
    # linear / layernorm / rmsnorm / attention vs torch fp32 autograd
    x = torch.randn(37, 64, generator=g).to(dev).requires_grad_(True)
    w = (torch.randn(48, 64, generator=g) / 8).to(dev).requires_grad_(True)
    b = torch.randn(48, generator=g).to(dev).requires_grad_(True)
    for act, tf in (("gelu", torch.nn.functional.gelu), ("relu", torch.relu)):
        y = torch.ops.hv.linear(x, w, b, act)
        xr, wr, br = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
        yr = tf(xr @ wr.T + br)
        assert rel(y, yr) < 1e-4
        gy = torch.randn(y.shape, generator=g).to(dev)
        ga = torch.autograd.grad(y, (x, w, b), gy)
        gr = torch.autograd.grad(yr, (xr, wr, br), gy)
        for a_, r_ in zip(ga, gr):
            assert rel(a_, r_) < 1e-4
    gam, bet = torch.randn(64, generator=g).to(dev).requires_grad_(True), torch.randn(64, generator=g).to(dev).requires_grad_(True)
    y = torch.ops.hv.layernorm(x, gam, bet, 1e-5)
    xr, gr_, br_ = (t.detach().clone().requires_grad_(True) for t in (x, gam, bet))
    yr = torch.nn.functional.layer_norm(xr, (64,), gr_, br_, 1e-5)
    assert rel(y, yr) < 1e-5
    gy = torch.randn(y.shape, generator=g).to(dev)
    for a_, r_ in zip(torch.autograd.grad(y, (x, gam, bet), gy), torch.autograd.grad(yr, (xr, gr_, br_), gy)):
        assert rel(a_, r_) < 1e-4
    sc = torch.rand(64, generator=g).to(dev).requires_grad_(True)
    y = torch.ops.hv.rmsnorm(x, sc, 1e-8)
    xr, sr = x.detach().clone().requires_grad_(True), sc.detach().clone().requires_grad_(True)
    yr = xr / torch.sqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-8) * sr
    assert rel(y, yr) < 1e-5
    for a_, r_ in zip(torch.autograd.grad(y, (x, sc), gy), torch.autograd.grad(yr, (xr, sr), gy)):
        assert rel(a_, r_) < 1e-4
    q, k, v = (torch.randn(2, 50, 256, generator=g).to(dev).requires_grad_(True) for _ in range(3))
    o = torch.ops.hv.attention(q, k, v, 8)
    qr, kr, vr = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    sp = lambda t: t.view(2, 50, 8, 32).transpose(1, 2)          # noqa: E731
    orf = torch.softmax(sp(qr) @ sp(kr).transpose(-1, -2) * 32 ** -0.5, -1) @ sp(vr)
    orf = orf.transpose(1, 2).reshape(2, 50, 256)
    assert rel(o, orf) < 1e-4
    go = torch.randn(o.shape, generator=g).to(dev)
    for a_, r_ in zip(torch.autograd.grad(o, (q, k, v), go), torch.autograd.grad(orf, (qr, kr, vr), go)):
        assert rel(a_, r_) < 1e-4
    # SE gate (NHWC) vs the training Function
    yy = torch.randn(2, 6, 6, 32, generator=g).to(dev).requires_grad_(True)
    ws = [(torch.randn(8, 32, 1, 1, generator=g) / 6).to(dev), torch.randn(8, generator=g).to(dev),
          (torch.randn(32, 8, 1, 1, generator=g) / 3).to(dev), torch.randn(32, generator=g).to(dev)]
    out = torch.ops.hv.se_gate(yy, None, *ws)
    yr = yy.detach().clone().requires_grad_(True)
    outr = TF.SEGateFn.apply(yr, None, *ws)
    assert torch.equal(out, outr)
    gz = torch.randn(out.shape, generator=g).to(dev)
    assert torch.equal(torch.autograd.grad(out, yy, gz)[0], torch.autograd.grad(outr, yr, gz)[0])


def test_hv_conv_decode_nms_ops_match_module_path(gpu_device):
    import hv_amd  # noqa: F401
    from hv_amd import ops
    g = torch.Generator().manual_seed(5)
    dev = gpu_device
    x = torch.randn(2, 9, 9, 16, generator=g).to(dev)
    w = (torch.randn(24, 16, 3, 3, generator=g) / 12).to(dev)
    bw, bb = torch.rand(24, generator=g).to(dev) + 0.5, torch.randn(24, generator=g).to(dev)
    mu, var = torch.randn(24, generator=g).to(dev), torch.rand(24, generator=g).to(dev) + 0.5
    y = torch.ops.hv.conv_bn_act(x, w, None, bw, bb, mu, var, 2, 1, "silu", 1e-5)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w, None, 2, 1)
    ref = torch.nn.functional.batch_norm(ref, mu, var, bw, bb, False, 0.0, 1e-5)
    ref = torch.nn.functional.silu(ref).permute(0, 2, 3, 1)
    assert rel(y, ref) < 1e-4
    logits = torch.randn(2, 5, 5, 255, generator=g).to(dev)
    awh = torch.rand(3, 2, generator=g).to(dev)
    outs = torch.ops.hv.yolo_decode(logits, 3, 80, awh)
    d, _ = ops.yolo_decode(logits, 3, 80, awh)
    for t, key in zip(outs, ("raw_predictions", "boxes", "scores", "class_scores", "class_indices", "objectness")):
        assert torch.equal(t, d[key]), key
    dec = {k: {n: t.to(dev) for n, t in v.items()} for k, v in cases.nms_case(3).items()}
    keys = sorted(dec)
    got = torch.ops.hv.nms([dec[k]["boxes"] for k in keys], [dec[k]["class_scores"] for k in keys],
                           [dec[k]["class_indices"] for k in keys], 0.5, 0.5, 100)
    ref = ops.nms_batched(dec, 0.5, 0.5, 100)
    for a_, b_ in zip(got, ref):
        assert torch.equal(a_, b_)


def test_hv_ops_visible_to_compile_and_export(gpu_device):
    """fullgraph torch.compile (aot_eager: no codegen) and torch.export trace through the hv
    ops via their fake kernels; the exported program holds them and reproduces the eager
    result."""
    import hv_amd  # noqa: F401
    from hv_amd import ManifoldHyperConnection

    class Block(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.mhc = ManifoldHyperConnection(64, expansion_rate=4, use_mixed_precision=False)
            self.scale = torch.nn.Parameter(torch.ones(64))

        def forward(self, x):
            m = self.mhc
            y = torch.ops.hv.mhc(x, *_mhc_args(m), 20)
            return torch.ops.hv.rmsnorm(y + x, self.scale, 1e-8)

    blk = Block().to(gpu_device).eval()
    x = torch.randn(40, 64, generator=torch.Generator().manual_seed(1)).to(gpu_device)
    with torch.no_grad():
        eager = blk(x)
        comp = torch.compile(blk, backend="aot_eager", fullgraph=True)(x)
        assert torch.equal(comp, eager)
        ep = torch.export.export(blk, (x,))
    names = {str(n.target) for n in ep.graph.nodes if n.op == "call_function"}
    assert any("hv.mhc" in s for s in names) and any("hv.rmsnorm" in s for s in names), names
    with torch.no_grad():
        assert torch.equal(ep.module()(x), eager)
