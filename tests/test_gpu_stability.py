"""a4 on the GPU: the stability monitor (reference src/models/manifold_layers.py:282-316) through
hv_symeig_group / hv_stability_stats, against the reference fixtures (tests/golden/stab_*, the
reference's own fp32 run) and the fp64 oracle on the same fp32 matrices."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import cases, hv_oracle as O

pytestmark = pytest.mark.gpu


def _H(D, fam):
    g = golden(f"stab_{fam}_D{D}")
    H = torch.from_numpy(g["H"]) if "H" in g.files else O.sinkhorn(cases.sinkhorn_raw(D, 20, fam), 20)
    return g, H.float().contiguous()


def test_symeig_group_matches_reference_and_oracle(gpu_device):
    """Every STAB case (n = 1 .. 1792, mixed sizes) in ONE grouped launch sequence."""
    from hv_amd import ops
    recs = [(D, fam) + _H(D, fam) for D, fam in cases.STAB_CASES]
    mats = [H.to(gpu_device) for *_, H in recs]
    outs = ops.symeig_group(mats)
    torch.cuda.synchronize()
    for (D, fam, g, H), ev in zip(recs, outs):
        ev = ev.cpu().double()
        ref64 = O.monitor_stability(H, torch.ones(1, D), torch.ones(1, D))["eigenvalues"]
        # fp64 tridiagonalisation + bisection to 1e-10, rounded to fp32
        np.testing.assert_allclose(ev.numpy(), ref64.numpy(), rtol=0, atol=1e-6, err_msg=f"D={D} {fam} vs fp64")
        # the reference's own fp32 eigvalsh
        np.testing.assert_allclose(ev.numpy(), g["eigenvalues"], rtol=0, atol=2e-5, err_msg=f"D={D} {fam} vs ref")
        # doubly stochastic symmetric part: the top eigenvalue is 1 (eigenvector = ones)
        assert abs(ev[-1].item() - 1.0) < 1e-5
        assert bool((ev[1:] >= ev[:-1]).all())


@pytest.mark.parametrize("kind", ["diag", "identity", "tridiag", "lowrank", "clustered"])
def test_symeig_edge_cases(gpu_device, kind):
    """Already-tridiagonal columns (zero reflectors), repeated eigenvalues, rank deficiency."""
    from hv_amd import ops
    n = 97
    g = torch.Generator().manual_seed(5)
    if kind == "diag":
        H = torch.diag(torch.randn(n, generator=g))
    elif kind == "identity":
        H = torch.eye(n)
    elif kind == "tridiag":
        H = torch.diag(torch.randn(n, generator=g)) + torch.diag(torch.randn(n - 1, generator=g), 1)
    elif kind == "lowrank":
        u = torch.randn(n, 3, generator=g)
        H = u @ u.T
    else:
        q, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
        lam = torch.tensor([1.0] * 40 + [1.0 + 1e-7] * 30 + [-2.0] * 27, dtype=torch.float64)
        H = ((q * lam) @ q.T).float()
    (ev,) = ops.symeig_group([H.contiguous().to(gpu_device)])
    ref = torch.linalg.eigvalsh(((H.double() + H.double().T) / 2))
    np.testing.assert_allclose(ev.cpu().double().numpy(), ref.numpy(), rtol=0,
                               atol=1e-6 * max(1.0, ref.abs().max().item()))


@pytest.mark.parametrize("D,fam", [c for c in cases.STAB_CASES if c[0] >= 8])
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_stability_stats_match_reference(gpu_device, D, fam, dt):
    from hv_amd import ops
    g, H = _H(D, fam)
    x_in, x_out = cases.stab_inputs(D, fam)
    dtype = torch.float32 if dt == "fp32" else torch.bfloat16
    hist = torch.zeros(1000, device=gpu_device)
    st = ops.stability_stats(x_in.to(gpu_device, dtype), x_out.to(gpu_device, dtype), H.to(gpu_device), hist, 7)
    st = st.cpu()
    r = O.monitor_stability(H, x_in.to(dtype).float(), x_out.to(dtype).float())
    tol = 1e-5 if dt == "fp32" else 1e-5       # bf16: the oracle sees the same rounded inputs
    np.testing.assert_allclose(st[0].item(), r["signal_ratio"].item(), rtol=tol)
    assert hist[7].item() == st[0].item()
    np.testing.assert_allclose(st[1].item(), r["row_sum_error"].item(), atol=2e-6)
    np.testing.assert_allclose(st[2].item(), r["col_sum_error"].item(), atol=2e-6)
    if dt == "fp32":
        np.testing.assert_allclose(st[0].item(), float(g["signal_ratio"]), rtol=1e-5)


def test_module_monitor_matches_oracle(gpu_device):
    """ManifoldHyperConnection in train mode: the buffers the reference fills (eigenvalues,
    signal_ratio_history) and get_stability_metrics, against the oracle on the module's own H_res."""
    from hv_amd import ManifoldHyperConnection
    torch.manual_seed(0)
    m = ManifoldHyperConnection(128, expansion_rate=2).to(gpu_device).train()
    x = torch.randn(3, 20, 128, device=gpu_device)
    y = m(x)
    met = m.get_stability_metrics()
    with torch.no_grad():
        H = m.sinkhorn(m.H_res_raw).detach().cpu().float()
    xb = x.to(m.dtype).float().cpu().reshape(-1, 128)      # the module monitors its compute-dtype input
    r = O.monitor_stability(H, xb, y.detach().float().cpu().reshape(-1, 128))
    np.testing.assert_allclose(m.eigenvalues.cpu().double().numpy(), r["eigenvalues"].numpy(), atol=1e-5)
    np.testing.assert_allclose(met["max_eigenvalue"], r["eigenvalues"].max().item(), atol=1e-5)
    np.testing.assert_allclose(m.signal_ratio_history[0].item(), r["signal_ratio"].item(), rtol=1e-4)
    assert m.signal_ratio_idx == 1
