"""CPU-side checks: the C-ABI library loads and exports every entry point declared in
include/hv_kernels.h (drop-in ABI) and include/hv_tuning.h (A/B knobs, launch counters); the host module surface mirrors the reference (state_dict layout,
constructor call forms); the product path refuses to run without the HIP path."""
import json
import os
import re

import pytest
import torch

from conftest import GOLDEN, MODEL_CFG, ROOT


def _declared():
    src = "".join(open(os.path.join(ROOT, "include", h)).read() for h in ("hv_kernels.h", "hv_tuning.h"))
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|size_t|void|const char\s*\*)\s*(hv_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_declared_symbol():
    from hv_amd import _lib
    lib = _lib.lib()
    declared = _declared()
    assert len(declared) >= 25
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert set(declared) == set(_lib.EXPORTED), set(declared) ^ set(_lib.EXPORTED)
    assert lib.hv_abi_version() == _lib.ABI_VERSION == 4


def test_library_built_from_this_tree():
    """Build provenance: the loaded libhvs.so carries the hash of the sources it was compiled
    from (Makefile HV_SRC_HASH); it equals the hash of the sources in this tree."""
    from hv_amd import _lib
    assert _lib.source_hash() is not None
    assert _lib.build_id() == _lib.source_hash()


def test_no_gpu_calls_needed_for_size_queries():
    from hv_amd import _lib
    lib = _lib.lib()
    assert lib.hv_sinkhorn_work_floats(1, 8, 8, 5) > 0
    assert lib.hv_channel_mean_work_floats(2, 4096, 64) == 2 * (4096 // ((256 // 16) * 8)) * 64


@pytest.mark.parametrize("tag", ["tiny", "base"])
def test_state_dict_layout_matches_reference(tag):
    from hv_amd import HybridVisionSystem
    m = HybridVisionSystem(MODEL_CFG[tag])
    lay = json.load(open(os.path.join(GOLDEN, f"state_dict_{tag}.json")))
    mine = [(k, list(v.shape), str(v.dtype).replace("torch.", "")) for k, v in m.state_dict().items()]
    assert mine == [tuple(x) for x in lay] or mine == [list(x) for x in lay] or \
        [tuple(a) for a in mine] == [tuple(a) for a in lay]


def test_call_site_constructor_forms():
    from models.hybrid_vision import HybridVisionSystem   # drop-in path (scripts/train.py:27)
    m = HybridVisionSystem(config={"use_vit": True, "verbose": False, "num_blocks": [1, 1, 1, 1],
                                   "vit_depth": 1}, num_classes=80, use_vit=True, use_rag=False)
    assert m.num_classes == 80 and m.use_vit
    counts = m.get_parameter_count()
    assert counts["total"] == sum(p.numel() for p in m.parameters())
    with pytest.raises(NotImplementedError):
        HybridVisionSystem({"use_rag": True})


def test_product_path_refuses_cpu():
    from hv_amd import HybridVisionSystem, ManifoldHyperConnection
    m = ManifoldHyperConnection(32, expansion_rate=4).eval()
    with pytest.raises(RuntimeError, match="HIP path only"):
        m(torch.randn(4, 32))
    s = HybridVisionSystem(MODEL_CFG["tiny"]).eval()
    with pytest.raises(RuntimeError, match="HIP path only"):
        s(torch.randn(1, 3, 64, 64))


def test_oracle_not_imported_by_product():
    pkg = os.path.join(ROOT, "humanoid-vision-system_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith(".py"):
                txt = open(os.path.join(dp, f)).read()
                assert "oracle" not in re.sub(r'""".*?"""', "", txt, flags=re.S).replace("# ", ""), f


def test_pil_resample_tables_match_oracle():
    """The host-side table builder of hv_preprocess_pil (Pillow Resample.c coefficients, no GPU
    needed) equals the oracle's restatement, which is pinned bit-exactly against Pillow."""
    import numpy as np
    from hv_amd import _lib
    from oracle import cases
    from oracle import preproc as P
    lib = _lib.lib()
    for _, _, h, w, oh, ow, _ in cases.PIL_CASES + [("", 1, 720, 1280, 416, 416, 0), ("", 1, 1080, 1920, 640, 640, 0)]:
        n = lib.hv_pil_table_ints(h, w, oh, ow)
        tab = torch.empty(n, dtype=torch.int32)
        assert lib.hv_pil_resample_tables(h, w, oh, ow, tab.data_ptr()) == 0
        t = tab.numpy().astype(np.int64)
        hb, hk = P.coeffs(w, ow)
        vb, vk = P.coeffs(h, oh)
        assert (t[0], t[1]) == (hk.shape[1], vk.shape[1])
        o = 2
        for arr in (hb, hk, vb, vk):
            np.testing.assert_array_equal(t[o:o + arr.size], arr.reshape(-1))
            o += arr.size
        assert o == n


def test_no_process_global_kernel_switches():
    """Kernel-variant selection is per call (hv_gemm_desc.variant / hv_mhc_fused_args.variant,
    runtime.HVOptions per model): the library exports no global setters and the package keeps no
    module-level switches."""
    from hv_amd import _lib, manifold, vit, ops, detect, backbone
    lib = _lib.lib()
    for name in ("hv_gemm_set_path", "hv_gemm_set_big_tile", "hv_gemm_set_force_tile", "hv_gemm_set_smallk",
                 "hv_mhc_fused_set_variant", "hv_mhc_fused_enable_wide"):
        assert not hasattr(lib, name), name
    for mod, names in ((manifold, ("FOLD_MAX_D", "USE_FUSED", "PARALLEL_QKV", "GROUP_QKV")),
                       (vit, ("CLS_ONLY_LAST_BLOCK",)), (ops, ("SPLITK_ON",)),
                       (detect, ("_PREP_OVERLAP",)), (backbone, ("_DIRECT_STEM",))):
        for n in names:
            assert not hasattr(mod, n), (mod.__name__, n)


def test_version_watch_sees_every_storage_change():
    """runtime.VersionWatch (the graph / frozen-coefficient staleness check): in-place updates,
    `.data` swaps, buffer re-registration, `_buffers[...]` rebinding (what `.to()` does, no hook)
    and a rebound OUTPUT buffer (one the forward writes, e.g. a Sinkhorn history) all change the
    snapshot; writing into an output buffer in place does not."""
    import torch.nn as nn
    from hv_amd.runtime import VersionWatch

    class Leaf(nn.Module):
        def __init__(self):
            super().__init__()
            self.w = nn.Parameter(torch.randn(4))
            self.register_buffer("running_mean", torch.zeros(4))
            self.register_buffer("convergence_history", torch.zeros(3))

    root = nn.Sequential(Leaf(), Leaf())
    vw = VersionWatch(root)
    s0 = vw.snapshot()
    assert vw.snapshot() == s0
    root[1].convergence_history.add_(1.0)               # the forward writes its history: no change
    assert vw.snapshot() == s0
    def inplace():
        with torch.no_grad():
            root[0].w.mul_(2.0)
    steps = [inplace,                                                             # optimizer-style in place
             lambda: setattr(root[0].w, "data", root[0].w.data.clone()),          # .data swap
             lambda: root[1].running_mean.add_(1.0),                              # input buffer in place
             lambda: setattr(root[1], "running_mean", torch.ones(4)),             # re-registration
             lambda: root[0]._buffers.__setitem__("running_mean", torch.ones(4)), # .to()-style rebind
             lambda: setattr(root[1], "convergence_history", torch.zeros(3)),     # output buffer rebound
             lambda: root[0]._buffers.__setitem__("convergence_history", torch.zeros(3))]
    prev = s0
    keep = []
    for i, step in enumerate(steps):
        keep.append([b for m in root for b in m._buffers.values()])   # old storage stays alive: fresh pointers
        step()
        cur = vw.snapshot()
        assert cur != prev, f"step {i} not detected"
        prev = cur


@pytest.mark.parametrize("tag", ["tiny", "base"])
def test_seeded_construction_matches_reference(tag):
    """torch.manual_seed(0); HybridVisionSystem({}) draws the same random numbers in the same
    order as the reference constructors (torch.randn(...) * alpha for H_pre/H_post/H_res before
    the Xavier re-init, manifold_layers.py:149-157,194-196; the default nn.Linear / nn.Conv2d
    inits; hybrid_vision.py:183-197's re-inits), so a seeded fresh model equals the
    reference's: fixture tests/golden/seeded_init_<tag>.npz (oracle/gen_golden.py --only seeded)
    holds the first 8 / last 4 values and the fp64 sum / sum of squares of every entry."""
    import numpy as np
    from hv_amd import HybridVisionSystem
    g = np.load(os.path.join(GOLDEN, f"seeded_init_{tag}.npz"))
    names = [k for k, _, _ in json.load(open(os.path.join(GOLDEN, f"state_dict_{tag}.json")))]
    torch.manual_seed(0)
    m = HybridVisionSystem(dict(MODEL_CFG[tag]))
    sd = m.state_dict()
    bad = []
    for i, n in enumerate(names):
        v = sd[n].detach().reshape(-1).double()
        k = min(8, v.numel())
        head_ok = np.array_equal(v[:k].float().numpy(), g["head"][i, :k])
        tail_ok = np.array_equal(v[-min(4, v.numel()):].float().numpy(), g["tail"][i, :min(4, v.numel())]) \
            if v.numel() else True
        s1, s2 = float(v.sum()), float((v * v).sum())
        sums_ok = abs(s1 - g["s1"][i]) <= 1e-9 * max(1.0, abs(g["s2"][i]) ** 0.5 * v.numel() ** 0.5) and \
            abs(s2 - g["s2"][i]) <= 1e-9 * max(1.0, abs(g["s2"][i]))
        if not (head_ok and tail_ok and sums_ok):
            bad.append(n)
    assert not bad, (len(bad), bad[:10])


def test_hv_dispatcher_ops_have_fake_kernels():
    """torch.ops.hv.* (hv_amd/library.py) are registered with fake kernels: shape propagation
    under FakeTensorMode works on a machine without a GPU (what torch.compile / torch.export
    run before any kernel)."""
    from torch._subclasses.fake_tensor import FakeTensorMode
    import hv_amd
    assert set(hv_amd.library.OPS) <= set(dir(torch.ops.hv))
    with FakeTensorMode():
        f = lambda *s, dt=torch.float32: torch.empty(*s, device="cuda", dtype=dt)   # noqa: E731
        D, Hd = 64, 256
        x = f(100, D, dt=torch.bfloat16)
        assert torch.ops.hv.mhc(x, f(D, Hd), f(Hd, D), f(D, D), f(D), f(D), f(2 * Hd, Hd), f(2 * Hd), f(Hd, 2 * Hd),
                                f(Hd), f(D), f(D), 20).shape == (100, D)
        M, h = torch.ops.hv.sinkhorn(f(3, 16, 16), 7, 1e-8, 1.0)
        assert M.shape == (3, 16, 16) and h.shape == (7,)
        assert torch.ops.hv.linear(x, f(96, D), None, "gelu").shape == (100, 96)
        assert torch.ops.hv.conv_bn_act(f(2, 40, 40, 32, dt=torch.bfloat16), f(64, 32, 3, 3), None, f(64), f(64),
                                        f(64), f(64), 2, 1, "silu", 1e-5).shape == (2, 20, 20, 64)
        assert torch.ops.hv.attention(f(2, 9, 256), f(2, 9, 256), f(2, 9, 256), 8).shape == (2, 9, 256)
        outs = torch.ops.hv.yolo_decode(f(2, 8, 8, 255), 3, 80, f(3, 2))
        assert [tuple(t.shape) for t in outs] == [(2, 3, 8, 8, 85), (2, 3, 8, 8, 4), (2, 3, 8, 8, 80), (2, 3, 8, 8),
                                                  (2, 3, 8, 8), (2, 3, 8, 8, 1)]
        assert outs[4].dtype == torch.int64
        b, s, l, c = torch.ops.hv.nms([f(2, 3, 8, 8, 4)], [f(2, 3, 8, 8)], [f(2, 3, 8, 8, dt=torch.int64)], 0.5, 0.5, 50)
        assert b.shape == (2, 50, 4) and l.dtype == torch.int64 and c.shape == (2,)
