"""GPU parity of the individual HIP kernels (through the libhvs C ABI) against plain PyTorch
fp32 references of the same op computed on the CPU, and against the oracle fixtures."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import gemm_variant, golden, run_options
from oracle import cases

pytestmark = pytest.mark.gpu

DT = {"fp32": torch.float32, "bf16": torch.bfloat16}
# bf16 operands are rounded to 8 significant bits; tolerance relative to the output scale
TOL = {"fp32": 2e-5, "bf16": 2e-2}


def _ops():
    from hv_amd import ops
    return ops


def rel_err(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


# ------------------------------------------------------------------------------ Sinkhorn
@pytest.mark.parametrize("fam", ["wc", "init"])
@pytest.mark.parametrize("D,it", cases.SK_CASES)
def test_sinkhorn_matches_reference_fixture(gpu_device, fam, D, it):
    ops = _ops()
    g = golden(f"sk_{fam}_D{D}_it{it}")
    raw = cases.sinkhorn_raw(D, it, fam).to(gpu_device)
    M, hist = ops.sinkhorn(raw, it)
    M = M.cpu()
    idx = [0, 1, D // 2, D - 1]
    np.testing.assert_allclose(M[idx].numpy(), g["rows"], rtol=2e-5, atol=1e-7)
    np.testing.assert_allclose(M.sum(0).numpy(), g["col_sums"], rtol=2e-5)
    np.testing.assert_allclose(M.sum(1).numpy(), g["row_sums"], rtol=2e-5)
    # history = |mean_i r_i - 1| with r_i ~ 1: the subtraction exposes the mean's own rounding
    # (a few fp32 ulps of 1.0 = 1.2e-7 each, summation-order dependent) at full size
    np.testing.assert_allclose(hist.cpu().numpy(), g["history"], rtol=1e-3, atol=5e-7)
    if "M" in g.files:
        np.testing.assert_allclose(M.numpy(), g["M"], rtol=2e-5, atol=1e-8)


def test_sinkhorn_batched_reference_cases(gpu_device):
    ops = _ops()
    for name, it in (("sk_batched_4x8x8", 20), ("sk_batched_2x5x7", 10)):
        g = golden(name)
        M, hist = ops.sinkhorn(torch.from_numpy(g["raw"]).to(gpu_device), it)
        np.testing.assert_allclose(M.cpu().numpy(), g["M"], rtol=2e-5, atol=1e-7)
        np.testing.assert_allclose(hist.cpu().numpy(), g["history"], rtol=1e-3, atol=2e-7)


def test_sinkhorn_grouped_equals_single(gpu_device):
    """All mHC sites share one launch set: grouped results must equal one-at-a-time runs."""
    ops = _ops()
    raws = [cases.sinkhorn_raw(D, 20, "wc").to(gpu_device) for D in (32, 64, 256, 512, 1792)]
    grp = ops.SinkhornGroup(raws, [20, 5, 20, 20, 20], gpu_device)
    outs = [o.clone() for o in grp.run(raws)]
    for r, it, o in zip(raws, [20, 5, 20, 20, 20], outs):
        M, _ = ops.sinkhorn(r, it)
        assert torch.equal(M, o[0])


def test_sinkhorn_many_iterations_falls_back_to_grouped_passes(gpu_device):
    """More iterations than the single-workgroup kernel's LDS history holds
    (hv_sinkhorn_small_max_iters): the whole group runs through the grouped passes -- any
    iteration count works, as in the reference -- and a small entry with few iterations in the
    same group is unaffected; matrices and histories vs the oracle in fp64."""
    import math
    ops = _ops()
    from hv_amd import _lib, SinkhornKnoppProjection
    from oracle import hv_oracle as O
    it = _lib.lib().hv_sinkhorn_small_max_iters() + 24
    raws = [cases.sinkhorn_raw(D, 20, "wc") for D in (48, 64, 300)]
    iters = [it, 5, it]
    grp = ops.SinkhornGroup([r.to(gpu_device) for r in raws], iters, gpu_device)
    outs = [o.clone().cpu() for o in grp.run()]
    for r, n, o, h in zip(raws, iters, outs, grp.hists):
        hist = torch.zeros(n, dtype=torch.float64)
        ref = O.sinkhorn(r.double(), n, history=hist)
        assert (o[0].double() - ref).abs().max().item() < 1e-5 * max(1.0, ref.abs().max().item()), n
        np.testing.assert_allclose(h[:n].cpu().numpy(), hist.numpy(), rtol=1e-3, atol=2e-6)
    sk = SinkhornKnoppProjection(num_iterations=150).to(gpu_device)       # module level, D=64
    M = sk(cases.sinkhorn_raw(64, 20, "init").to(gpu_device)).cpu()
    assert math.isclose(float(M.sum(0).mean()), 1.0, rel_tol=1e-4)


def test_sinkhorn_reference_properties(gpu_device):
    """test_models.py:33-56 / :85-100: doubly stochastic within rtol 1e-4, deterministic."""
    from hv_amd import SinkhornKnoppProjection
    sk = SinkhornKnoppProjection(num_iterations=20).to(gpu_device)
    x = torch.randn(4, 8, 8, generator=torch.Generator().manual_seed(0)).to(gpu_device)
    p = sk(x)
    assert torch.all(p >= 0)
    rs, cs = p.sum(2), p.sum(1)
    assert torch.allclose(rs, torch.ones_like(rs), rtol=1e-4)
    assert torch.allclose(cs, torch.ones_like(cs), rtol=1e-4)
    assert torch.equal(sk(x), p)
    _, h = sk(x, return_history=True)
    assert len(h["row_sums"]) == 20 and abs(h["final_col_error"]) < 1e-4


# ------------------------------------------------------------------------------ GEMM
GEMM_SHAPES = [(1, 64, 32), (7, 33, 40), (64, 256, 128), (130, 200, 96), (300, 64, 1024), (1000, 512, 256),
               (257, 1000, 64)]


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
def test_gemm_epilogue_vs_torch(gpu_device, prec, M, N, K):
    ops = _ops()
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    a = torch.randn(M, K, generator=g)
    b = torch.randn(N, K, generator=g) / K ** 0.5
    bias = torch.randn(N, generator=g)
    scale = torch.rand(N, generator=g) + 0.5
    res = torch.randn(M, N, generator=g)
    dt = DT[prec]
    ad, bd = a.to(dt), b.to(dt)
    ref = F.gelu((ad.float() @ bd.float().T) * 0.5 * scale + bias) + res
    out = ops.gemm(ad.to(gpu_device), bd.to(gpu_device), bias=bias.to(gpu_device), scale=scale.to(gpu_device),
                   act="gelu", alpha=0.5, residual=res.to(gpu_device), out_dtype=torch.float32)
    assert rel_err(out, ref) < TOL[prec]


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_gemm_ln_prologue_and_concat(gpu_device, prec):
    ops = _ops()
    dt = DT[prec]
    g = torch.Generator().manual_seed(5)
    T, D, H, N = 200, 64, 96, 48
    x = (torch.randn(T, D, generator=g) * 3 + 1).to(dt)
    h = torch.randn(T, H, generator=g).to(dt)
    b = (torch.randn(N, D, generator=g) / 8).to(dt)
    bc = (torch.randn(N, D + H, generator=g) / 8).to(dt)
    xd = x.to(gpu_device)
    mean, rstd = ops.row_stats(xd, 1e-5)
    z = F.layer_norm(x.float(), (D,), eps=1e-5)
    out = ops.gemm(xd, b.to(gpu_device), a_mean=mean, a_rstd=rstd, out_dtype=torch.float32)
    assert rel_err(out, z.to(dt).float() @ b.float().T) < TOL[prec]
    out2 = ops.gemm(xd, bc.to(gpu_device), a2=h.to(gpu_device), out_dtype=torch.float32)
    assert rel_err(out2, torch.cat([x, h], 1).float() @ bc.float().T) < TOL[prec]


@pytest.mark.parametrize("T,D,N", [(200, 64, 96), (1000, 256, 1024), (77, 128, 40)])
def test_gemm_ln_epilogue_equals_prologue(gpu_device, T, D, N):
    """LDS-DMA kernel with the LayerNorm applied after the product, rstd (x.b - mean colsum(b)),
    against the LN-on-load register-staged path and a torch reference (bf16 operands)."""
    ops = _ops()
    g = torch.Generator().manual_seed(T + D)
    x = (torch.randn(T, D, generator=g) * 2 + 3).to(torch.bfloat16).to(gpu_device)   # large mean
    b = (torch.randn(N, D, generator=g) / 8).to(torch.bfloat16).to(gpu_device)
    bias = torch.randn(N, generator=g).to(gpu_device)
    mean, rstd = ops.row_stats(x, 1e-5)
    cs = b.float().sum(1).contiguous()
    epi = ops.gemm(x, b, bias=bias, act="gelu", a_mean=mean, a_rstd=rstd, b_colsum=cs, out_dtype=torch.float32)
    pro = ops.gemm(x, b, bias=bias, act="gelu", a_mean=mean, a_rstd=rstd, out_dtype=torch.float32)
    z = F.layer_norm(x.float().cpu(), (D,), eps=1e-5)
    ref = F.gelu(z @ b.float().cpu().T + bias.cpu())
    assert rel_err(epi, ref) < 1e-4            # exact operand: better than the bf16-rounded z of `pro`
    assert rel_err(pro, ref) < TOL["bf16"]


@pytest.mark.parametrize("M,N,K,kind", [(401, 512, 1024, "plain"), (401, 1024, 256 + 768, "ln"),
                                         (401, 256, 768, "cat"), (16, 1792, 1792, "plain"),
                                         (16, 7168, 1792, "resmod"), (400, 1024, 2304, "conv")])
def test_gemm_splitk_vs_unsplit(gpu_device, M, N, K, kind):
    """Split-K (small output grids: ops._splitk engages for < 192 64x64 tiles, bf16) against the
    register-staged un-split kernel and a CPU fp32 torch reference: same epilogue (LN after the
    product, scale, bias, GELU, residual / row-modulo residual, concat-K, implicit-GEMM conv);
    only the summation order differs.  Also checks the split actually engaged and that it is
    deterministic (bitwise across runs)."""
    ops = _ops()
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(M + N + K)
    dev = gpu_device
    kw = {}
    if kind == "conv":
        x = torch.randn(1, 20, 20, 256, generator=g).to(dt).to(dev)
        w = (torch.randn(N, 2304, generator=g) / 48).to(dt).to(dev)
        kw = dict(scale=(torch.rand(N, generator=g) + 0.5).to(dev), bias=torch.randn(N, generator=g).to(dev),
                  act="silu")
        run = lambda: ops.conv2d(x, w, 3, 1, 1, **kw)                      # noqa: E731
    else:
        a = (torch.randn(M, K if kind != "cat" else 256, generator=g) * (3 if kind == "ln" else 1) + 1).to(dt).to(dev)
        b = (torch.randn(N, K, generator=g) / K ** 0.5).to(dt).to(dev)
        kw = dict(bias=torch.randn(N, generator=g).to(dev), act="gelu")
        if kind == "ln":
            mean, rstd = ops.row_stats(a, 1e-5)
            kw.update(a_mean=mean, a_rstd=rstd, b_colsum=b.float().sum(1).contiguous())
        if kind == "cat":
            kw["a2"] = torch.randn(M, K - 256, generator=g).to(dt).to(dev)
        if kind == "resmod":
            kw.update(residual=torch.randn(4, N, generator=g).to(dt).to(dev), residual_mod=4)
            kw.pop("act")
        run = lambda: ops.gemm(a, b, **kw)                                   # noqa: E731
    with run_options(splitk=True):                          # opt-in path (off by default)
        ops.launch_counts(reset=True)
        out = run()
        counts = ops.launch_counts(reset=True)
        assert counts["gemm_splitk"] == 1, counts           # the split path ran
        assert torch.equal(run(), out)                      # deterministic
    ref = run()                                             # same LDS-DMA kernel family, un-split
    d = (out.float() - ref.float()).abs()
    assert d.max().item() <= 2 ** -6 * max(1.0, ref.float().abs().max().item()), d.max().item()
    assert rel_err(out.float(), ref.float()) < 4e-3
    if kind == "plain":                                     # and vs CPU fp32 torch
        cpu = F.gelu(a.float().cpu() @ b.float().cpu().T + kw["bias"].cpu())
        assert rel_err(out.float().cpu(), cpu) < TOL["bf16"]


def test_gemm_residual_mod(gpu_device):
    ops = _ops()
    a = torch.randn(6 * 10, 32)
    b = torch.randn(16, 32)
    pos = torch.randn(10, 16)
    out = ops.gemm(a.to(gpu_device), b.to(gpu_device), residual=pos.to(gpu_device), residual_mod=10)
    ref = a @ b.T + pos.repeat(6, 1)
    assert rel_err(out, ref) < 1e-5


@pytest.mark.parametrize("M,N,K,conv", [(4096, 512, 1024, False), (333, 1000, 576, False),
                                         (2 * 40 * 40, 256, 9 * 64, True), (2 * 20 * 20, 96, 9 * 128, True)])
def test_gemm_lds_dma_path_equals_register_path(gpu_device, M, N, K, conv):
    """The global_load_lds kernel (K % 64 == 0, bf16) against the register-staged kernel."""
    ops = _ops()
    from hv_amd import _lib
    g = torch.Generator().manual_seed(M + N)
    if conv:
        c = K // 9
        hw = int(round((M // 2) ** 0.5))
        x = torch.randn(2, hw, hw, c, generator=g).to(torch.bfloat16).to(gpu_device)
        w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(gpu_device)
        run = lambda: ops.conv2d(x, w, 3, 1, 1, out_dtype=torch.float32)  # noqa: E731
        ref = F.conv2d(x.float().cpu().permute(0, 3, 1, 2), w.float().cpu().view(N, 3, 3, c).permute(0, 3, 1, 2),
                       None, 1, 1).permute(0, 2, 3, 1)
    else:
        a = torch.randn(M, K, generator=g).to(torch.bfloat16).to(gpu_device)
        b = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(gpu_device)
        bias = torch.randn(N, generator=g).to(gpu_device)
        run = lambda: ops.gemm(a, b, bias=bias, act="relu", out_dtype=torch.float32)  # noqa: E731
        ref = F.relu(a.float().cpu() @ b.float().cpu().T + bias.cpu())
    fast = run()
    with gemm_variant(_lib.GV_REGSTAGE):
        slow = run()
    assert rel_err(fast, slow) < 1e-5
    assert rel_err(fast, ref) < 1e-4


@pytest.mark.parametrize("kind,M,N,K", [("plain", 401, 512, 2048), ("plain", 333, 96, 1024), ("ln", 400, 2048, 1024),
                                         ("cat", 400, 512, 2560), ("conv", 400, 1024, 9 * 512), ("conv", 400, 200, 9 * 256)])
def test_gemm_small_m_long_k_tile_vs_register_path(gpu_device, kind, M, N, K):
    """The 32x64 LDS-DMA tile the automatic policy takes for small-M, long-K inference GEMMs (a
    grid of < 256 64x64 tiles with K >= 1,024: the B=1 frame's 20x20 convs and D = 512 / 1024 mHC
    chains) against the register-staged kernel: plain / LN-after-product / concat-K / implicit
    3x3 conv, ragged M and N."""
    ops = _ops()
    from hv_amd import _lib
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(M * 7 + N + K)
    dev = gpu_device
    if kind == "conv":
        c = K // 9
        x = torch.randn(1, 20, 20, c, generator=g).to(dt).to(dev)
        w = (torch.randn(N, K, generator=g) / K ** 0.5).to(dt).to(dev)
        kw = dict(scale=(torch.rand(N, generator=g) + 0.5).to(dev), bias=torch.randn(N, generator=g).to(dev), act="silu")
        run = lambda: ops.conv2d(x, w, 3, 1, 1, **kw)                          # noqa: E731
    else:
        a = (torch.randn(M, K if kind != "cat" else 512, generator=g) * (3 if kind == "ln" else 1) + 1).to(dt).to(dev)
        b = (torch.randn(N, K, generator=g) / K ** 0.5).to(dt).to(dev)
        kw = dict(bias=torch.randn(N, generator=g).to(dev), act="gelu")
        if kind == "ln":
            mean, rstd = ops.row_stats(a, 1e-5)
            kw.update(a_mean=mean, a_rstd=rstd, b_colsum=b.float().sum(1).contiguous())
        if kind == "cat":
            kw["a2"] = torch.randn(M, K - 512, generator=g).to(dt).to(dev)
        run = lambda: ops.gemm(a, b, **kw)                                       # noqa: E731
    fast = run()
    with gemm_variant(_lib.GV_REGSTAGE):
        slow = run()
    d = (fast.float() - slow.float()).abs()
    assert d.max().item() <= 2 ** -6 * max(1.0, slow.float().abs().max().item()), d.max().item()
    assert rel_err(fast.float(), slow.float()) < 4e-3
    assert torch.equal(run(), fast)                                              # deterministic


SMALLK_CASES = [  # (kind, M, N, K): 1-8 k-tiles, ragged M / N (scalar store tail), every epilogue form
    ("plain", 4096, 512, 64), ("plain", 1000, 777, 128), ("ln_gelu", 1500, 1024, 256), ("gelu_res", 2048, 768, 512),
    ("res32_mod", 1200, 640, 256), ("scale_f32", 700, 384, 192), ("conv1x1", 2 * 40 * 40, 256, 128),
    ("ln_gelu", 8192, 1024, 256), ("ln_gelu", 6416, 3072, 256), ("conv1x1", 2 * 56 * 56, 512, 256),
    # bf16 output, no residual, N % 128 in 64..127: edge column tiles whose waves differ in
    # "full" (the early next-tile DMA must stay workgroup-uniform); M % 4 != 0 under LN
    ("ln_gelu", 1501, 320, 256), ("bf16", 4096, 448, 128), ("ln_gelu", 26003, 448, 256),
    ("bf16", 20000, 320, 192)]


@pytest.mark.parametrize("kind,M,N,K", SMALLK_CASES)
def test_gemm_smallk_equals_ring(gpu_device, kind, M, N, K):
    """The persistent small-K kernel (hv_gemm_sk.hip: N-permuted B rows, register epilogue with
    16-byte stores, next tile's first k-tile prefetched across the epilogue) against the 128x128
    LDS-DMA ring kernel: same per-element k order and epilogue arithmetic -> bit-identical; plus
    a CPU fp32 check.  The 8192x1024x256 case (512 tiles) must take it without forcing."""
    ops = _ops()
    from hv_amd import _lib
    g = torch.Generator().manual_seed(M * 3 + N + K)
    bf = torch.bfloat16
    a = torch.randn(M, K, generator=g).to(bf).to(gpu_device)
    b = (torch.randn(N, K, generator=g) / K ** 0.5).to(bf).to(gpu_device)
    bias = torch.randn(N, generator=g).to(gpu_device)
    af, bfl = a.float().cpu(), b.float().cpu()
    if kind == "plain":
        run = lambda: ops.gemm(a, b, bias=bias, out_dtype=torch.float32)  # noqa: E731
        ref = af @ bfl.T + bias.cpu()
    elif kind == "bf16":
        run = lambda: ops.gemm(a, b, bias=bias, act="gelu")  # noqa: E731
        ref = F.gelu(af @ bfl.T + bias.cpu())
    elif kind == "ln_gelu":
        mean = af.mean(1)
        rstd = 1.0 / torch.sqrt(af.var(1, unbiased=False) + 1e-5)
        cs = bfl.sum(1)
        run = lambda: ops.gemm(a, b, bias=bias, act="gelu", a_mean=mean.to(gpu_device),  # noqa: E731
                               a_rstd=rstd.to(gpu_device), b_colsum=cs.to(gpu_device))
        ref = F.gelu(((af - mean[:, None]) * rstd[:, None]) @ bfl.T + bias.cpu())
    elif kind == "gelu_res":
        res = torch.randn(M, N, generator=g).to(bf).to(gpu_device)
        run = lambda: ops.gemm(a, b, bias=bias, act="gelu", residual=res)  # noqa: E731
        ref = F.gelu(af @ bfl.T + bias.cpu()) + res.float().cpu()
    elif kind == "res32_mod":
        res = torch.randn(400, N, generator=g).to(gpu_device)
        run = lambda: ops.gemm(a, b, act="silu", residual=res, residual_mod=400, out_dtype=torch.float32)  # noqa: E731
        ref = F.silu(af @ bfl.T) + res.cpu().repeat(3, 1)
    elif kind == "scale_f32":
        sc = torch.rand(N, generator=g).to(gpu_device) + 0.5
        run = lambda: ops.gemm(a, b, bias=bias, scale=sc, alpha=0.75, act="relu", out_dtype=torch.float32)  # noqa: E731
        ref = F.relu((af @ bfl.T) * 0.75 * sc.cpu() + bias.cpu())
    else:  # 1x1 convolution over NHWC pixels
        hw = int(round((M // 2) ** 0.5))
        x = a.view(2, hw, hw, K)
        run = lambda: ops.conv2d(x, b, 1, 1, 0, out_dtype=torch.float32)  # noqa: E731
        ref = af @ bfl.T
    with gemm_variant(_lib.GV_TILE_SMALLK):
        ops.launch_counts(reset=True)
        fast = run()
        assert ops.launch_counts()["gemm_smallk"] == 1
    with gemm_variant(_lib.GV_TILE_128x128):
        ring = run()
    if M * N >= 8192 * 1024:
        ops.launch_counts(reset=True)
        auto = run()
        assert ops.launch_counts()["gemm_smallk"] == 1
        assert torch.equal(auto, fast)
    # the B-resident column-stationary form (K 192 / 256, no residual; 3- and 4-stage A rings)
    res_forms = []
    for v in (_lib.GV_SK_RES3, _lib.GV_SK_RES4):
        with gemm_variant(_lib.GV_TILE_SMALLK | v):
            res_forms.append(run())
    torch.cuda.synchronize()
    assert torch.equal(fast.reshape(ring.shape), ring), \
        f"max |diff| {(fast.float().reshape(ring.shape) - ring.float()).abs().max().item()}"
    for r in res_forms:
        assert torch.equal(r.reshape(ring.shape), ring), \
            f"B-resident: max |diff| {(r.float().reshape(ring.shape) - ring.float()).abs().max().item()}"
    tol = 2e-2 if fast.dtype == torch.bfloat16 else 1e-4
    assert rel_err(fast.reshape(ref.shape), ref) < tol


PP256_CASES = [  # (kind, M, N, K): ragged M/N, 1-3 K-tiles (prologue/tail vmcnt branches), long K
    ("plain", 4096, 512, 1024), ("plain", 1000, 520, 640), ("plain", 300, 260, 64), ("plain", 513, 300, 128),
    ("plain", 700, 777, 192), ("gelu_res", 2048, 768, 2048), ("ln", 1500, 1024, 256), ("concat", 1024, 512, 768),
    ("conv", 2 * 40 * 40, 256, 9 * 64), ("conv", 2 * 20 * 20, 300, 9 * 128)]


@pytest.mark.parametrize("kind,M,N,K", PP256_CASES)
def test_gemm_pingpong256_equals_default(gpu_device, kind, M, N, K):
    """The 256x256 ping-pong LDS-DMA kernel (variant GV_BIG_ALWAYS forces it) and the 8-stage
    64x64 ring (GV_DEEP8) against the default tiles: same per-element k order, so bit-identical
    outputs; plus a CPU fp32 check."""
    ops = _ops()
    from hv_amd import _lib
    g = torch.Generator().manual_seed(M * 7 + N + K)
    bf = torch.bfloat16
    if kind == "conv":
        c = K // 9
        hw = int(round((M // 2) ** 0.5))
        x = torch.randn(2, hw, hw, c, generator=g).to(bf).to(gpu_device)
        w = (torch.randn(N, K, generator=g) / K ** 0.5).to(bf).to(gpu_device)
        run = lambda: ops.conv2d(x, w, 3, 1, 1, out_dtype=torch.float32)  # noqa: E731
        ref = F.conv2d(x.float().cpu().permute(0, 3, 1, 2), w.float().cpu().view(N, 3, 3, c).permute(0, 3, 1, 2),
                       None, 1, 1).permute(0, 2, 3, 1)
    else:
        a = torch.randn(M, K, generator=g).to(bf).to(gpu_device)
        b = (torch.randn(N, K, generator=g) / K ** 0.5).to(bf).to(gpu_device)
        bias = torch.randn(N, generator=g).to(gpu_device)
        af, bfl = a.float().cpu(), b.float().cpu()
        if kind == "plain":
            run = lambda: ops.gemm(a, b, bias=bias, out_dtype=torch.float32)  # noqa: E731
            ref = af @ bfl.T + bias.cpu()
        elif kind == "gelu_res":
            res = torch.randn(M, N, generator=g).to(bf).to(gpu_device)
            run = lambda: ops.gemm(a, b, bias=bias, act="gelu", residual=res)  # noqa: E731
            ref = F.gelu(af @ bfl.T + bias.cpu()) + res.float().cpu()
        elif kind == "ln":
            mean = af.mean(1)
            rstd = 1.0 / torch.sqrt(af.var(1, unbiased=False) + 1e-5)
            cs = bfl.sum(1)
            run = lambda: ops.gemm(a, b, bias=bias, a_mean=mean.to(gpu_device), a_rstd=rstd.to(gpu_device),  # noqa: E731
                                   b_colsum=cs.to(gpu_device), out_dtype=torch.float32)
            ref = ((af - mean[:, None]) * rstd[:, None]) @ bfl.T + bias.cpu()
        else:  # K-concatenated operand [a | a2]
            k1 = 256
            a1, a2 = a[:, :k1].contiguous(), a[:, k1:].contiguous()
            run = lambda: ops.gemm(a1, b, a2=a2, out_dtype=torch.float32)  # noqa: E731
            ref = af @ bfl.T
    outs = {}
    for staged in (1, 0):                       # LDS-staged coalesced epilogue vs fragment-layout stores
        flat = 0 if staged else _lib.GV_FLAT_EPI
        for deep in (1, 0):                     # 3/4-buffer LDS-DMA rings vs 2 buffers
            with gemm_variant(flat | _lib.GV_NO_BIG | (0 if deep else _lib.GV_SHALLOW)):
                outs["base", staged, deep] = run()
        with gemm_variant(flat | _lib.GV_BIG_ALWAYS):
            outs["pp", staged] = run()
        # 64x64 tiles on the 8-stage ring (fewer K-tiles than stages included: K = 64 .. 192)
        with gemm_variant(flat | _lib.GV_TILE_64x64 | _lib.GV_DEEP8):
            outs["deep8", staged] = run()
    torch.cuda.synchronize()
    pp, base = outs["pp", 1], outs["base", 0, 0]
    for key, o in outs.items():
        assert torch.equal(o, base), f"{key}: max |diff| {(o.float() - base.float()).abs().max().item()}"
    assert rel_err(pp, ref) < (2e-2 if pp.dtype == bf else 1e-4)


@pytest.mark.parametrize("cin,cout,s,hw", [(32, 64, 1, 40), (32, 32, 2, 33), (16, 8, 1, 9), (40, 24, 1, 15)])
def test_conv_ktail_lds_dma_vs_register_path(gpu_device, cin, cout, s, hw):
    """3x3 convs with K = 9*cin not a multiple of 64 on the LDS-DMA kernel (zero-line K tail)
    against the register-staged kernel and torch."""
    ops = _ops()
    from hv_amd import _lib
    g = torch.Generator().manual_seed(cin * 100 + cout + hw)
    x = torch.randn(2, hw, hw, cin, generator=g).to(torch.bfloat16).to(gpu_device)
    w = (torch.randn(cout, 9 * cin, generator=g) / (9 * cin) ** 0.5).to(torch.bfloat16).to(gpu_device)
    bias = torch.randn(cout, generator=g).to(gpu_device)
    run = lambda: ops.conv2d(x, w, 3, s, 1, bias=bias, act="silu", out_dtype=torch.float32)  # noqa: E731
    with gemm_variant(_lib.GV_CONV_KTAIL):
        fast = run()
    slow = run()
    ref = F.silu(F.conv2d(x.float().cpu().permute(0, 3, 1, 2), w.float().cpu().view(cout, 3, 3, cin).permute(0, 3, 1, 2),
                          bias.cpu(), s, 1)).permute(0, 2, 3, 1)
    assert rel_err(fast, slow) < 1e-5
    assert rel_err(fast, ref) < 1e-4


CONV_CASES = [(3, 32, 3, 2, 1, 33), (32, 32, 3, 1, 1, 20), (32, 64, 3, 2, 1, 17), (64, 32, 1, 1, 0, 9),
              (128, 96, 3, 1, 1, 7), (16, 8, 3, 1, 1, 5)]


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("cin,cout,k,s,p,hw", CONV_CASES)
def test_conv_implicit_gemm_vs_torch(gpu_device, prec, cin, cout, k, s, p, hw):
    ops = _ops()
    dt = DT[prec]
    g = torch.Generator().manual_seed(cin * 100 + cout + k + s)
    x = torch.randn(2, cin, hw, hw + 3, generator=g).to(dt).float()
    w = (torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5).to(dt).float()
    sc, bi = torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g)
    ref = F.silu(F.conv2d(x, w, None, s, p) * sc.view(1, -1, 1, 1) + bi.view(1, -1, 1, 1))
    xd = ops.nchw_to_nhwc(x.to(gpu_device), dt)
    wd = ops.conv_weight_prep(w.to(gpu_device), dt)
    out = ops.conv2d(xd, wd, k, s, p, scale=sc.to(gpu_device), bias=bi.to(gpu_device), act="silu",
                     out_dtype=torch.float32)
    assert rel_err(out.permute(0, 3, 1, 2), ref) < TOL[prec]


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("cout,s,h,w", [(32, 2, 33, 36), (32, 2, 640, 640), (64, 1, 17, 9), (32, 1, 1, 1)])
def test_conv_stem_direct_vs_torch_and_gemm(gpu_device, prec, cout, s, h, w):
    """hv_conv_stem (NCHW fp32 image, 3 channels) vs CPU fp32 torch conv+affine+SiLU of the
    storage-rounded operands, and vs the implicit-GEMM conv of the same operands (summation
    order is the only difference)."""
    ops = _ops()
    dt = DT[prec]
    n = 1 if h >= 640 else 2
    g = torch.Generator().manual_seed(cout + s + h)
    x = torch.randn(n, 3, h, w, generator=g)
    wt = torch.randn(cout, 3, 3, 3, generator=g) / 27 ** 0.5
    sc, bi = torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g)
    wd = ops.conv_weight_prep(wt.to(gpu_device), dt)
    out = ops.conv_stem(x.to(gpu_device), wd, 3, s, 1, dt, scale=sc.to(gpu_device), bias=bi.to(gpu_device),
                        act="silu")
    assert out is not None and out.dtype == dt
    xr, wr = x.to(dt).float(), wt.to(dt).float()
    if h < 640:
        ref = F.silu(F.conv2d(xr, wr, None, s, 1) * sc.view(1, -1, 1, 1) + bi.view(1, -1, 1, 1))
        assert rel_err(out.float().permute(0, 3, 1, 2), ref) < TOL[prec]
    xh = ops.nchw_to_nhwc(x.to(gpu_device), dt)
    out_h = ops.conv_stem(xh, wd, 3, s, 1, dt, scale=sc.to(gpu_device), bias=bi.to(gpu_device), act="silu",
                          nhwc=True)
    assert torch.equal(out_h, out)                      # NHWC input == NCHW fp32 input, bit for bit
    gem = ops.conv2d(xh, wd, 3, s, 1, scale=sc.to(gpu_device), bias=bi.to(gpu_device), act="silu")
    d = (out.float() - gem.float()).abs().max().item()
    assert d <= (2e-5 if prec == "fp32" else 2 ** -7 * max(1.0, gem.float().abs().max().item())), d


@pytest.mark.parametrize("n,c", [(1, 1024), (3, 64), (16, 512), (17, 128), (2, 2048)])
def test_se_mlp_batched_vs_torch(gpu_device, n, c):
    """hv_se_mlp2: batched two-stage SE MLP (n <= 16) and the per-image kernel (n > 16) vs CPU
    fp32 torch (vision_backbone.py:77-83: sigmoid(W2 silu(W1 p + b1) + b2))."""
    ops = _ops()
    cr = c // 4
    g = torch.Generator().manual_seed(n * 31 + c)
    w1, b1 = torch.randn(cr, c, 1, 1, generator=g) / c ** 0.5, torch.randn(cr, generator=g)
    w2, b2 = torch.randn(c, cr, 1, 1, generator=g) / cr ** 0.5, torch.randn(c, generator=g)
    pooled = torch.randn(n, c, generator=g)
    gt = ops.se_mlp(pooled.to(gpu_device), w1.to(gpu_device), b1.to(gpu_device), w2.to(gpu_device), b2.to(gpu_device))
    ref = torch.sigmoid(F.linear(F.silu(F.linear(pooled, w1.view(cr, c), b1)), w2.view(c, cr), b2))
    assert rel_err(gt, ref) < 1e-5


@pytest.mark.parametrize("n,h,c,dt", [(1, 80, 64, torch.bfloat16), (3, 40, 128, torch.bfloat16),
                                      (16, 20, 256, torch.bfloat16), (5, 13, 32, torch.float32),
                                      (2, 10, 1024, torch.float32), (1, 320, 32, torch.bfloat16)])
def test_se_gate_matches_mean_then_mlp_bitwise(gpu_device, n, h, c, dt):
    """hv_se_gate (pool chunk sums + MLP finishing the mean) is bitwise hv_channel_mean followed by
    hv_se_mlp2, on both MLP forms (n <= 4 batched, n > 4 per image), repeatably, and agrees with CPU
    fp32 torch of vision_backbone.py:77-83 on the same rounded input."""
    ops = _ops()
    cr = max(c // 16, 4)
    g = torch.Generator().manual_seed(n * 131 + h + c)
    x = torch.randn(n, h, h, c, generator=g).to(dt)
    w1, b1 = torch.randn(cr, c, generator=g) / c ** 0.5, torch.randn(cr, generator=g)
    w2, b2 = torch.randn(c, cr, generator=g) / cr ** 0.5, torch.randn(c, generator=g)
    xd, ws = x.to(gpu_device), [t.to(gpu_device) for t in (w1, b1, w2, b2)]
    fused = ops.se_gate(xd, *ws)
    pair = ops.se_mlp(ops.channel_mean(xd), *ws)
    again = ops.se_gate(xd, *ws)
    torch.cuda.synchronize()
    assert torch.equal(fused, pair)
    assert torch.equal(fused, again)
    ref = torch.sigmoid(F.linear(F.silu(F.linear(x.float().mean((1, 2)), w1, b1)), w2, b2))
    assert rel_err(fused, ref) < 1e-5


@pytest.mark.parametrize("cout,h,w", [(32, 20, 23), (64, 7, 70), (32, 320, 320), (64, 9, 130)])
def test_conv3x3_c32_halo_kernel_vs_torch_and_regstage(gpu_device, cout, h, w):
    """The halo-tiled MFMA conv (hv_stem.hip, bf16 3x3 s1 p1, Cin 32, Cout 32/64: stem[1], stem[2])
    vs CPU fp32 torch and vs the register-staged implicit GEMM on the same bf16 operands."""
    from hv_amd import _lib
    ops = _ops()
    dt = torch.bfloat16
    n = 1 if h >= 320 else 2
    g = torch.Generator().manual_seed(cout * 7 + h + w)
    x = torch.randn(n, 32, h, w, generator=g).to(dt).float()
    wt = (torch.randn(cout, 32, 3, 3, generator=g) / 288 ** 0.5).to(dt).float()
    sc, bi = torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g)
    xd = ops.nchw_to_nhwc(x.to(gpu_device), dt)
    wd = ops.conv_weight_prep(wt.to(gpu_device), dt)
    kw = dict(scale=sc.to(gpu_device), bias=bi.to(gpu_device), act="silu")
    out = ops.conv2d(xd, wd, 3, 1, 1, **kw)
    with gemm_variant(_lib.GV_REGSTAGE):
        reg = ops.conv2d(xd, wd, 3, 1, 1, **kw)
    d = (out.float() - reg.float()).abs()
    assert d.max().item() <= 2 ** -7 * max(1.0, reg.float().abs().max().item())
    assert (d > 0).float().mean().item() < 0.02            # equal up to rare 1-ulp roundings
    if h < 320:
        ref = F.silu(F.conv2d(x, wt, None, 1, 1) * sc.view(1, -1, 1, 1) + bi.view(1, -1, 1, 1))
        assert rel_err(out.float().permute(0, 3, 1, 2), ref) < TOL["bf16"]


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("n,h,w,c", [(2, 8, 6, 64), (1, 320, 320, 64), (3, 5, 7, 8)])
def test_scale_maxpool_equals_scale_then_pool(gpu_device, prec, n, h, w, c):
    """maxpool2x2(x, gate) == maxpool2x2(scale_residual(x, gate)) bit for bit (gate > 0)."""
    ops = _ops()
    dt = DT[prec]
    g = torch.Generator().manual_seed(h * w + c)
    x = torch.randn(n, h, w, c, generator=g).to(dt).to(gpu_device)
    gate = torch.sigmoid(torch.randn(n, c, generator=g)).to(gpu_device)
    fused = ops.maxpool2x2(x, gate)
    ref = ops.maxpool2x2(ops.scale_residual(x, gate, None))
    assert torch.equal(fused, ref)
    plain = ops.maxpool2x2(x)
    assert torch.equal(plain.cpu(), F.max_pool2d(x.float().cpu().permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1).to(dt))


# ------------------------------------------------------------------------------ pointwise / norms
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_norms_and_pointwise_vs_torch(gpu_device, prec):
    ops = _ops()
    dt = DT[prec]
    tol = TOL[prec]
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 12, 10, 64, generator=g).to(dt)
    xd = x.to(gpu_device)
    gam, bet = torch.rand(64, generator=g) + 0.5, torch.randn(64, generator=g)
    y = ops.layernorm(xd.view(-1, 64).float().contiguous(), gam.to(gpu_device), bet.to(gpu_device), 1e-5)
    assert rel_err(y, F.layer_norm(x.float().view(-1, 64), (64,), gam, bet, 1e-5)) < 1e-5
    sc = torch.rand(64, generator=g) + 0.5
    r = ops.rmsnorm(xd, sc.to(gpu_device))
    xf = x.float()
    assert rel_err(r, xf / torch.sqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-8) * sc) < tol
    mp = ops.maxpool2x2(xd)
    assert rel_err(mp, F.max_pool2d(xf.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)) < tol
    cm = ops.channel_mean(xd)
    assert rel_err(cm, xf.mean(dim=(1, 2))) < 1e-5
    for (n, hw, c) in [(3, 2500, 32), (2, 1030, 1024), (1, 77, 2048 if dt == torch.bfloat16 else 1024), (2, 9, 40)]:
        xc = torch.randn(n, hw, c, generator=g).to(dt)
        got = ops.channel_mean(xc.to(gpu_device))
        assert rel_err(got, xc.float().mean(dim=1)) < 1e-5, (n, hw, c)
    b = torch.randn(2, 6, 5, 64, generator=g).to(dt)
    up = ops.upsample_add(xd, b.to(gpu_device))
    ref = xf + F.interpolate(b.float().permute(0, 3, 1, 2), size=(12, 10), mode="nearest").permute(0, 2, 3, 1)
    assert rel_err(up, ref) < tol
    gate = torch.rand(2, 64, generator=g)
    sr = ops.scale_residual(xd, gate.to(gpu_device), xd)
    assert rel_err(sr, xf * gate.view(2, 1, 1, 64) + xf) < tol
    w1, b1 = torch.randn(16, 64, 1, 1, generator=g) / 8, torch.randn(16, generator=g)
    w2, b2 = torch.randn(64, 16, 1, 1, generator=g) / 4, torch.randn(64, generator=g)
    pooled = torch.randn(2, 64, generator=g)
    gt = ops.se_mlp(pooled.to(gpu_device), w1.to(gpu_device), b1.to(gpu_device), w2.to(gpu_device), b2.to(gpu_device))
    ref = torch.sigmoid(F.linear(F.silu(F.linear(pooled, w1.view(16, 64), b1)), w2.view(64, 16), b2))
    assert rel_err(gt, ref) < 1e-5
    t = torch.randn(3 * 7, 64, generator=g).to(dt)
    assert torch.equal(ops.gather_rows(t.to(gpu_device), 7).cpu(), t.view(3, 7, 64)[:, 0])
    v = torch.randn(2, 64, generator=g)
    assert rel_err(ops.add_rowvec(xd, v.to(gpu_device)), xf + v.view(2, 1, 1, 64)) < tol
    pe = torch.randn(256, 32, generator=g)
    for lout in (49, 400, 1024, 256):
        ref = F.interpolate(pe.T.unsqueeze(0), size=(lout,), mode="linear").squeeze(0).T
        assert rel_err(ops.interp_linear(pe.to(gpu_device), lout), ref) < 1e-6


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("L", [1, 33, 50, 257, 401, 1025])
def test_attention_vs_torch(gpu_device, prec, L):
    ops = _ops()
    dt = DT[prec]
    g = torch.Generator().manual_seed(L)
    q, k, v = (torch.randn(2, L, 256, generator=g).to(dt) for _ in range(3))
    o = ops.attention(q.to(gpu_device), k.to(gpu_device), v.to(gpu_device), 8)
    qh, kh, vh = (t.float().view(2, L, 8, 32).transpose(1, 2) for t in (q, k, v))
    ref = (torch.softmax(qh @ kh.transpose(-1, -2) * 32 ** -0.5, -1) @ vh).transpose(1, 2).reshape(2, L, 256)
    assert rel_err(o, ref) < TOL[prec]


def test_decode_matches_reference_fixture(gpu_device):
    ops = _ops()
    g = golden("decode_s1")
    pred = torch.from_numpy(g["pred"])                     # [2, 3, 7, 9, 85]
    from oracle import hv_oracle as O
    lg = pred.permute(0, 2, 3, 1, 4).reshape(2, 7, 9, 3 * 85).contiguous()
    dec, pr = ops.yolo_decode(lg.to(gpu_device), 3, 80, O.anchor_wh(1).float().to(gpu_device))
    np.testing.assert_array_equal(pr.cpu().numpy(), g["pred"])
    np.testing.assert_allclose(dec["boxes"].cpu().numpy(), g["boxes"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(dec["scores"].cpu().numpy(), g["scores"], rtol=1e-5, atol=1e-7)
    np.testing.assert_array_equal(dec["class_indices"].cpu().numpy(), g["class_indices"])


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_gpu_post_process_matches_reference_fixture(gpu_device, seed):
    """§8f-1: hv_nms (two launches per batch) vs the reference's post_process (tests/golden/nms_*)."""
    from hv_amd.detect import YOLODetectionHead
    g = golden(f"nms_{seed}")
    dec = {k: {n: t.to(gpu_device) for n, t in v.items()} for k, v in cases.nms_case(seed).items()}
    head = YOLODetectionHead([16, 16, 16], num_classes=80)
    res = head.post_process(dec, float(g["conf"]), float(g["iou"]), int(g["max_det"]))
    for b, r in enumerate(res):
        np.testing.assert_array_equal(r["labels"].cpu().numpy(), g[f"labels{b}"])
        np.testing.assert_array_equal(r["scores"].cpu().numpy(), g[f"scores{b}"])
        np.testing.assert_array_equal(r["boxes"].reshape(-1, 4).cpu().numpy(), g[f"boxes{b}"])


@pytest.mark.parametrize("case", cases.NMS_LARGE_CASES, ids=[c[0] for c in cases.NMS_LARGE_CASES])
def test_gpu_post_process_large_matches_reference_fixture(gpu_device, case):
    """§8f-1 past the LDS capacity: > 8,192 candidates per (image, scale) (640^2 / 1024^2 grids at
    conf 0.01: up to 47,209), max_det 1,500 / 5,000 (cross-scale pass > 8,192 survivors) --
    boxes, scores and labels bit-exact vs the reference post_process (tests/golden/nms_large_*),
    and the same detections on a second run (no atomic-order dependence)."""
    from hv_amd import ops
    tag, seed, B, grids, conf, iou, mx, spread = case
    g = golden(f"nms_large_{tag}")
    assert int(np.max(g["max_candidates"])) > 8192
    dec = {k: {n: t.to(gpu_device) for n, t in v.items()}
           for k, v in cases.nms_case(seed, B=B, grids=grids, spread=spread).items()}
    boxes, scores, labels, count = (t.clone() for t in ops.nms_batched(dec, conf, iou, mx))
    again = ops.nms_batched(dec, conf, iou, mx)
    for a, b2 in zip((boxes, scores, labels, count), again):
        assert torch.equal(a, b2)
    for b in range(B):
        n = int(count[b])
        assert n == len(g[f"scores{b}"])
        np.testing.assert_array_equal(scores[b, :n].cpu().numpy(), g[f"scores{b}"])
        np.testing.assert_array_equal(labels[b, :n].cpu().numpy(), g[f"labels{b}"])
        np.testing.assert_array_equal(boxes[b, :n].cpu().numpy(), g[f"boxes{b}"])
        assert not scores[b, n:].any() and not boxes[b, n:].any()


@pytest.mark.parametrize("n,levels", [(1, 1), (16, 3), (17, 2), (300, 7), (5000, 40), (70000, 300),
                                      (3000, 0), (900, 0)])
def test_gpu_sort_desc_exact_matches_std_sort(gpu_device, n, levels):
    """hv_sort_desc_exact == the reference's CPU torch.sort(descending=True).indices (libstdc++
    introsort: tie order included) on heavily tied values (levels > 0) and on distinct values
    (levels = 0: the spent-budget segments take the parallel rank sort); with the depth limit
    forced to 0 / 1 / 3 it matches oracle/std_sort.py's restatement through the heap-sort fallback
    too."""
    from hv_amd import ops
    from oracle.std_sort import std_sort_desc
    g = torch.Generator().manual_seed(n)
    if levels == 0:
        v = torch.randperm(n, generator=g).float() / n + 0.5
    else:
        v = (torch.randint(0, levels, (n,), generator=g).float() / levels) * torch.rand(1, generator=g)
    got = ops.sort_desc_exact(v.to(gpu_device)).cpu()
    assert torch.equal(got, torch.sort(v, descending=True).indices)
    if n <= 5000:
        for d in (0, 1, 3):
            got = ops.sort_desc_exact(v.to(gpu_device), depth_limit=d).cpu().tolist()
            assert got == std_sort_desc(v.tolist(), depth_limit=d), d


def test_gpu_post_process_ties_match_oracle(gpu_device):
    """Scores on a coarse grid (hundreds of ties per scale, > 8,192 candidates at scale 0) with
    clustered boxes: which of two tied boxes survives, and the output order, follow the
    reference's unstable CPU sort (oracle = the reference's own torch.sort call)."""
    from oracle import hv_oracle as O
    from hv_amd import ops
    dec = cases.nms_case(31, B=2, grids=((80, 80), (40, 40), (20, 20)))
    for v in dec.values():
        v["class_scores"] = torch.round(v["class_scores"] * 200) / 200
    for conf, iou, mx in ((0.01, 0.5, 100), (0.3, 0.7, 3000)):
        ref = O.post_process(dec, conf, iou, mx)
        dd = {k: {n: t.to(gpu_device) for n, t in v.items()} for k, v in dec.items()}
        boxes, scores, labels, count = ops.nms_batched(dd, conf, iou, mx)
        for b in range(2):
            n = int(count[b])
            assert n == len(ref[b]["scores"])
            np.testing.assert_array_equal(scores[b, :n].cpu().numpy(), ref[b]["scores"].numpy())
            np.testing.assert_array_equal(labels[b, :n].cpu().numpy(), ref[b]["labels"].numpy())
            np.testing.assert_array_equal(boxes[b, :n].cpu().numpy(), ref[b]["boxes"].reshape(-1, 4).numpy())


def test_gpu_nms_large_matches_oracle(gpu_device):
    """640x640-sized grids (19200 + 4800 + 1200 cells, many candidates) vs the oracle."""
    from oracle import hv_oracle as O
    from hv_amd import ops
    dec = cases.nms_case(9, B=2, grids=((80, 80), (40, 40), (20, 20)), frac_above=0.9)  # ~7% above 0.5
    ref = O.post_process(dec, 0.5, 0.5, 100)
    dd = {k: {n: t.to(gpu_device) for n, t in v.items()} for k, v in dec.items()}
    boxes, scores, labels, count = ops.nms_batched(dd, 0.5, 0.5, 100)
    for b in range(2):
        n = int(count[b])
        assert n == len(ref[b]["scores"])
        np.testing.assert_array_equal(scores[b, :n].cpu().numpy(), ref[b]["scores"].numpy())
        np.testing.assert_array_equal(labels[b, :n].cpu().numpy(), ref[b]["labels"].numpy())
        np.testing.assert_array_equal(boxes[b, :n].cpu().numpy(), ref[b]["boxes"].reshape(-1, 4).numpy())


@pytest.mark.parametrize("h,w,oh,ow", [(480, 640, 640, 640), (720, 1280, 640, 640), (64, 64, 64, 64), (300, 200, 416, 416)])
def test_gpu_preprocess_matches_torch(gpu_device, h, w, oh, ow):
    """§8f-2, the kornia path (K.Resize bilinear = F.interpolate, preprocessing.py:148-152):
    uint8 BGR frames -> resize (bilinear, align_corners=False) -> /255 -> ImageNet norm."""
    from hv_amd import ops
    g = torch.Generator().manual_seed(h * w)
    frames = torch.randint(0, 256, (2, h, w, 3), generator=g, dtype=torch.uint8)
    t = frames.flip(-1).permute(0, 3, 1, 2).float() / 255.0
    t = F.interpolate(t, size=(oh, ow), mode="bilinear", align_corners=False)
    ref = (t - torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)) / torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    out = ops.preprocess(frames.to(gpu_device), oh, ow, resample="bilinear")
    assert (out.cpu() - ref).abs().max().item() < 2e-5
    nh = ops.preprocess(frames.to(gpu_device), oh, ow, dtype=torch.bfloat16, nhwc=True, resample="bilinear")
    assert nh.permute(0, 2, 3, 1).is_contiguous()
    assert (nh.float().cpu() - ref).abs().max().item() < 2e-2
    h16 = ops.preprocess(frames.to(gpu_device), oh, ow, dtype=torch.float16, resample="bilinear")
    assert (h16.float().cpu() - ref).abs().max().item() < 5e-3


@pytest.mark.parametrize("n,h,w", [(1, 1, 1), (3, 5, 11), (2, 20, 20)])
def test_decode_argmax_first_index_on_ties(gpu_device, n, h, w):
    """hv_yolo_decode's class index/score equal the first-index argmax / max of the scores it
    returns, with heavy ties (logits on a coarse grid) and partial 8-cell wave groups."""
    ops = _ops()
    from oracle import hv_oracle as O
    g = torch.Generator().manual_seed(n * 100 + h)
    lg = (torch.randint(-3, 4, (n, h, w, 3 * 85), generator=g).float() * 0.5).to(gpu_device)
    dec, pr = ops.yolo_decode(lg, 3, 80, O.anchor_wh(1).float().to(gpu_device))
    sc = dec["scores"].float().cpu().reshape(-1, 80)
    ci = dec["class_indices"].cpu().reshape(-1)
    assert torch.equal(ci, torch.argmax(sc, dim=1))
    cs = dec["class_scores"].float().cpu().reshape(-1) if "class_scores" in dec else None
    if cs is not None:
        assert torch.equal(cs, sc.max(dim=1).values)
    assert torch.equal(pr.cpu().reshape(-1), lg.reshape(n, h, w, 3, 85).permute(0, 3, 1, 2, 4).cpu().reshape(-1))


@pytest.mark.parametrize("case", ["720x1280_640", "480x640_640", "300x200_416", "37x53_29x71", "64x64_64", "1x1_3x5"])
def test_gpu_preprocess_pil_bit_exact(gpu_device, case):
    """§8f-2, the reference's default preprocessing (torchvision Resize on a PIL image =
    Pillow Image.resize(BILINEAR); kornia is not in requirements.txt): the resized uint8 image
    must equal Pillow's BIT FOR BIT (tests/golden/preproc_pil_*, made by Pillow itself), and
    the normalised tensor must equal torchvision's ToTensor + Normalize in fp32 exactly."""
    from hv_amd import ops
    from oracle import cases
    g = golden(f"preproc_pil_{case}")
    bgr = torch.from_numpy(cases.camera_frames(int(g["seed"]), *[int(v) for v in g["in_hw"]]))
    oh, ow = (int(v) for v in g["out_hw"])
    rgb_u8 = torch.from_numpy(g["resized_rgb"])                       # [n, oh, ow, 3] from Pillow
    ref = (rgb_u8.permute(0, 3, 1, 2).float().div(255) - torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)) \
        / torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    out = ops.preprocess(bgr.to(gpu_device), oh, ow, resample="pil")
    assert torch.equal(out.cpu(), ref)
    nh = ops.preprocess(bgr.to(gpu_device), oh, ow, dtype=torch.bfloat16, nhwc=True, resample="pil")
    assert torch.equal(nh.cpu(), ref.to(torch.bfloat16))


@pytest.mark.parametrize("n", [0, 5, 2048, 5000])
def test_write_bytes_eager_and_captured(gpu_device, n):
    """hv_write_bytes (ops.upload_bytes inside a capture): host bytes reach the device through
    kernel arguments, stream-ordered; captured, the graph replays the bytes recorded at capture
    even after the host buffer is overwritten."""
    from hv_amd import ops
    rng = np.random.default_rng(n)
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    t = ops.upload_bytes(data, gpu_device)
    torch.cuda.synchronize()
    assert bytes(t.cpu().numpy().tobytes()) == data
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    buf = bytearray(data)
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            tc = ops.upload_bytes(bytes(buf), gpu_device)
            out = tc.to(torch.int32) + 1
    for i in range(len(buf)):
        buf[i] = 0
    g.replay()
    torch.cuda.synchronize()
    assert bytes(tc.cpu().numpy().tobytes()) == data
    assert torch.equal(out.cpu(), torch.frombuffer(bytearray(data), dtype=torch.uint8).to(torch.int32) + 1) if n else True
