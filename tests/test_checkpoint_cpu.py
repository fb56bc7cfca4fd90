"""§8f-4 checkpoint compatibility (CPU): the model's state_dict has exactly the reference's
layout (names, shapes, dtypes recorded from the reference itself in tests/golden/state_dict_*.json),
and optimizer state round-trips between the fused AdamW and torch.optim.AdamW."""
import json
import os

import torch

from conftest import GOLDEN, MODEL_CFG


def test_state_dict_layout_matches_reference():
    from hv_amd import HybridVisionSystem
    for tag in ("tiny", "base"):
        lay = json.load(open(os.path.join(GOLDEN, f"state_dict_{tag}.json")))
        m = HybridVisionSystem(dict(MODEL_CFG[tag]))
        sd = m.state_dict()
        assert [k for k, _, _ in lay] == list(sd.keys())
        for k, shape, dt in lay:
            assert list(sd[k].shape) == shape, k
            assert str(sd[k].dtype).replace("torch.", "") == dt, k


def test_optimizer_state_roundtrip_with_torch_adamw(tmp_path):
    from hv_amd.trainer import FusedAdamW
    torch.manual_seed(0)
    named = [("a.mhc.w", torch.randn(10, requires_grad=True)), ("b.conv.weight", torch.randn(3, 4, requires_grad=True))]
    opt = FusedAdamW(named, lr=2e-3, weight_decay=1e-2)
    for t in opt.exp_avg + opt.exp_avg_sq:
        t.copy_(torch.rand_like(t))
    opt.step_count = 7
    opt.param_steps = [7, 7]
    ref = torch.optim.AdamW([p for _, p in named], lr=1.0)
    ref.load_state_dict(opt.state_dict())
    sd = ref.state_dict()
    assert sd["param_groups"][0]["lr"] == 2e-3 and float(sd["state"][0]["step"]) == 7
    opt2 = FusedAdamW(named)
    opt2.load_state_dict(sd)
    assert opt2.step_count == 7 and opt2.lr == 2e-3 and opt2.wd == 1e-2
    for a, b in zip(opt.exp_avg + opt.exp_avg_sq, opt2.exp_avg + opt2.exp_avg_sq):
        assert torch.equal(a, b)


def test_checkpoint_file_roundtrip(tmp_path):
    from hv_amd import HybridVisionSystem
    from hv_amd.trainer import load_checkpoint, save_checkpoint
    torch.manual_seed(0)
    m = HybridVisionSystem(dict(MODEL_CFG["tiny"]))
    path = str(tmp_path / "ck.pt")
    save_checkpoint(path, m, epoch=3, global_step=42)
    torch.manual_seed(1)
    m2 = HybridVisionSystem(dict(MODEL_CFG["tiny"]))
    ck = load_checkpoint(path, m2)
    assert ck["epoch"] == 3 and ck["global_step"] == 42
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
    assert set(ck) >= {"epoch", "global_step", "model_state_dict", "optimizer_state_dict", "scheduler_state_dict",
                       "scaler_state_dict", "config", "history", "best_val_loss", "experiment_name", "timestamp"}


def test_checkpoint_loads_into_reference_trainer_state_types(tmp_path):
    """The reference trainer's load_checkpoint (mhc_trainer.py:641-647) feeds the optimizer,
    scheduler and scaler states to torch objects: the scaler state must be accepted by an
    enabled GradScaler and the param group must carry the reference optimizer's own keys
    (optimizer.py:55-70, read by its step() at :125)."""
    from hv_amd.trainer import FusedAdamW, save_checkpoint
    torch.manual_seed(0)
    named = [("a.mhc.w", torch.randn(10, requires_grad=True)), ("b.conv.weight", torch.randn(3, 4, requires_grad=True))]
    opt = FusedAdamW(named)
    opt.param_steps = [3, 0]                         # b never received a gradient
    sd = opt.state_dict()
    assert list(sd["state"]) == [0]
    g = sd["param_groups"][0]
    assert g["manifold_update_freq"] == 100 and g["mhc_params"]["project_iterations"] == 20

    class _T:
        pass
    tr = _T()
    tr.opt = opt
    m = torch.nn.Linear(2, 2)
    path = str(tmp_path / "ck.pt")
    save_checkpoint(path, m, tr)
    ck = torch.load(path, weights_only=True)
    sc = torch.amp.GradScaler("cpu", enabled=True)
    sc.load_state_dict(ck["scaler_state_dict"])
    assert sc.get_scale() == 65536.0
    ref = torch.optim.AdamW([p for _, p in named], lr=1.0)
    ref.load_state_dict(ck["optimizer_state_dict"])
    assert ref.param_groups[0]["manifold_update_freq"] == 100
