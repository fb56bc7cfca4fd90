"""Pointer lifetime of the device tables (hv_amd/tables.py, verdict r5 item 7): every pointer a
persistent program writes into a device table must lie in a tensor the program itself holds --
a buffer referenced only by a raw table pointer is freed and reused by the caching allocator
(round 5's `k_pg4` fault).  Programs are built from CPU tensors here (the table builders only
call host-side size queries); the GPU suite walks the live programs of a forward and a training
step (tests/test_gpu_model.py / test_gpu_train.py)."""
import gc

import torch

from conftest import MODEL_CFG  # noqa: F401  (sys.path set-up)


def _tiny_mhc_modules():
    from hv_amd import HybridVisionSystem
    m = HybridVisionSystem(dict(num_blocks=[1, 1, 1, 1], vit_depth=1, sk_iters=5, verbose=False))
    return m, m._mhc_modules


def test_train_prep_holds_every_table_pointer():
    """TrainPrep's prep and transpose tables point only at buffers it holds; dropping what it
    keeps (e.g. removing `TrainPrep._keep`) is reported -- the check that would have caught the
    round-5 `k_pg4` fault before a GPU ran it."""
    from hv_amd import tables
    from hv_amd.train_prep import TrainPrep
    _, mods = _tiny_mhc_modules()
    h_res = [torch.full((m.input_dim, m.input_dim), 1.0 / m.input_dim) for m in mods]
    prep = TrainPrep(mods, h_res, torch.float32)
    assert set(prep.__dict__[tables._TABLES]) == {"mhc_prep", "transpose"}
    assert tables.unheld_pointers(prep) == []
    n_cs = len(prep._keep)
    prep._keep.clear()
    gc.collect()
    bad = tables.unheld_pointers(prep)
    assert {f for _, _, f, _ in bad} == {"cs"} and len(bad) == n_cs
    prep2 = TrainPrep(mods, h_res, torch.float32)
    prep2.h_res = []                       # the Sinkhorn outputs are read through the table too
    assert {f for _, _, f, _ in tables.unheld_pointers(prep2)} == {"h_res"}


def test_optimizer_table_holds_params_grads_and_moments():
    from hv_amd import tables
    from hv_amd.trainer import FusedAdamW
    lin = torch.nn.Linear(8, 4)
    for p in lin.parameters():
        p.grad = torch.zeros_like(p)
    opt = FusedAdamW(list(lin.named_parameters()))
    opt._build()
    assert tables.unheld_pointers(opt) == []
    opt.exp_avg = []                       # moments dropped: their pointers are now unheld
    gc.collect()
    assert {f for _, _, f, _ in tables.unheld_pointers(opt)} == {"exp_avg"}


def test_table_walker_reads_nested_structs():
    """SinkhornBwdEntry nests a SinkhornEntry: its pointers are walked too."""
    from hv_amd import _lib as L
    from hv_amd import tables
    ents = (L.SinkhornBwdEntry * 2)()
    ents[1].fwd.out = 0x1000
    ents[1].draw = 0x2000
    assert sorted(tables.table_pointers(ents)) == [(1, "draw", 0x2000), (1, "fwd.out", 0x1000)]
