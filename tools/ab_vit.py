"""A/B of inference-path switches on the bench workload (base 640², B=16, bf16, graph replay):
alternating captures, 20 timed replays each, several rounds.  usage: python tools/ab_vit.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem  # noqa: E402
from hv_amd import manifold as MF  # noqa: E402
from hv_amd import detect as DT  # noqa: E402
from hv_amd import ops as OPS  # noqa: E402
from hv_amd import vit as VT  # noqa: E402

SWITCHES = {
    "base": lambda: None,
    "parallel_qkv": lambda: setattr(MF, "PARALLEL_QKV", True),
    "no_cls_only": lambda: setattr(VT, "CLS_ONLY_LAST_BLOCK", False),
    "no_group_qkv": lambda: setattr(MF, "GROUP_QKV", False),
    "sk_split": lambda: setattr(OPS, "SINKHORN_SPLIT", True),
    "prep_overlap": lambda: setattr(DT, "_PREP_OVERLAP", True),
}


def reset():
    MF.PARALLEL_QKV = False
    MF.GROUP_QKV = True
    VT.CLS_ONLY_LAST_BLOCK = True
    OPS.SINKHORN_SPLIT = False
    DT._PREP_OVERLAP = False


def main():
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else list(SWITCHES)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = HybridVisionSystem({"image_size": 640, "verbose": False}).to(dev).eval()
    x = torch.randn(16, 3, 640, 640, device=dev)
    res = {n: [] for n in names}
    with torch.no_grad():
        for rnd in range(3):
            for n in names:
                reset()
                SWITCHES[n]()
                m(x)
                r = m.capture(x)
                for _ in range(3):
                    r.replay()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(20):
                    r.replay()
                torch.cuda.synchronize()
                res[n].append((time.perf_counter() - t0) / 20 * 1e3)
                del r
                torch.cuda.empty_cache()
            print(f"round {rnd}: " + "  ".join(f"{n} {res[n][-1]:.3f}" for n in names), flush=True)
    reset()
    for n in names:
        print(f"{n:20s} min {min(res[n]):.3f} ms  mean {sum(res[n]) / len(res[n]):.3f} ms")


if __name__ == "__main__":
    main()
