"""Shared pytest configuration: markers, import paths, golden-fixture helpers."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "humanoid-vision-system_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: full-size model cases")
    # bisection knob: HV_TEST_GEMM_VARIANT=<HV_GV_* bits> runs every test's default options with
    # that GEMM variant (training steps included -- they read runtime.DEFAULT_OPTIONS)
    if os.environ.get("HV_TEST_GEMM_VARIANT"):
        from hv_amd import runtime
        runtime.DEFAULT_OPTIONS = runtime.HVOptions(gemm_variant=int(os.environ["HV_TEST_GEMM_VARIANT"], 0))


def golden(name: str):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def formula_state_dict(tag: str, fam: str):
    """Reference-layout state dict (tests/golden/state_dict_<tag>.json) filled from the weight
    formula (oracle/weights.py) -- no reference import needed."""
    import json
    import torch
    from oracle import weights as W
    lay = json.load(open(os.path.join(GOLDEN, f"state_dict_{tag}.json")))
    sd = {}
    for name, shape, dt in lay:
        t = W.make_tensor(name, tuple(shape), fam)
        if t is None:
            if name.endswith("anchors"):
                t = torch.from_numpy(np.load(os.path.join(GOLDEN, "anchors.npy")))
            else:
                t = torch.zeros(shape, dtype=getattr(torch, dt))
        sd[name] = t
    return sd


def record_parity(name: str, values: dict) -> None:
    """Persist a parity test's measured agreement (rel-L2, class agreement, ...) as
    gpurun_out/parity/<name>.json -- the GPU box merges gpurun_out/ back, and the round's
    records are copied to profiles/ -- so the numbers behind each tolerance stay on file."""
    import json
    d = os.path.join(ROOT, "gpurun_out", "parity")
    try:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name + ".json"), "w") as f:
            json.dump(values, f, indent=1, sort_keys=True)
    except OSError:
        pass
    print(f"parity record {name}: {values}")


def run_options(dtype=None, **kw):
    """Context manager: run the enclosed HIP ops under per-call options (runtime.HVOptions --
    kernel variants, restructurings) instead of the defaults; nothing process-global changes."""
    import torch
    from hv_amd.runtime import HVOptions, RunCtx, use_ctx
    return use_ctx(RunCtx(dtype=dtype or torch.bfloat16, opts=HVOptions(**kw)))


def gemm_variant(v: int):
    """Pin the GEMM kernel variant (HV_GV_* bits, hv_amd._lib.GV_*) of the enclosed launches."""
    return run_options(gemm_variant=v)


MODEL_CFG = {"tiny": dict(num_blocks=[1, 1, 1, 1], vit_depth=1, sk_iters=5, verbose=False),
             "base": dict(verbose=False)}
