"""Per-parameter bf16 gradient errors of one training-step group (verdict r5 item 1): the base
model's 224 B=2 bf16 step vs the reference's fp64 gradient norms (fixture train_base_224_b2), beside
the reference's OWN bf16 error (train_base_224_b2_bf16ref).  Prints every parameter of the group
sorted by its share of the group-norm error, and the fp32 HIP step's error for comparison.

    python tools/vit_grad_probe.py [group-prefix, default vit_encoder] > gpurun_out/vit_grad_probe.txt
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "humanoid-vision-system_amd"))

from conftest import GOLDEN, golden  # noqa: E402
from test_gpu_train import _base_train_step  # noqa: E402
from hv_amd.trainer import mhc_group  # noqa: E402


def main():
    prefix = sys.argv[1] if len(sys.argv) > 1 else "vit_encoder"
    dev = torch.device("cuda:0")
    g = golden("train_base_224_b2")
    gb = golden("train_base_224_b2_bf16ref")
    names = json.load(open(os.path.join(GOLDEN, "train_base_param_names.json")))
    ref64 = {n: float(v) for n, v in zip(names, g["grad_norm_f64"]) if v >= 0}
    refb = {n: float(v) for n, v in zip(names, gb["grad_norm"]) if v >= 0}
    B, S = int(g["B"]), int(g["S"])
    runs = {}
    for prec in ("bf16", "fp32"):
        _, _, norms, fin = _base_train_step(dev, prec, B, S, 1, int(g["target_seed"]))
        runs[prec] = norms
        print(f"{prec}: finite={fin}")
    rows = []
    for n in names:
        if not n.startswith(prefix) or n not in ref64:
            continue
        grp = "mhc" if mhc_group(n) == 0 else "other"
        r = ref64[n]
        rows.append((grp, n, r, runs["bf16"].get(n, 0.0), runs["fp32"].get(n, 0.0), refb.get(n, 0.0)))
    for grp in ("other", "mhc"):
        sel = [x for x in rows if x[0] == grp]
        G = np.sqrt(sum(x[2] ** 2 for x in sel))
        Gh = np.sqrt(sum(x[3] ** 2 for x in sel))
        Gb = np.sqrt(sum(x[5] ** 2 for x in sel))
        print(f"\n== {prefix}/{grp}: group norm f64 {G:.6g}  hip-bf16 {Gh:.6g} (rel {abs(Gh / G - 1):.4f})  "
              f"ref-bf16 {Gb:.6g} (rel {abs(Gb / G - 1):.4f})")
        # share of the squared-norm difference each parameter carries
        tot = sum(abs(x[3] ** 2 - x[2] ** 2) for x in sel) or 1.0
        sel.sort(key=lambda x: -abs(x[3] ** 2 - x[2] ** 2))
        print(f"{'param':60s} {'norm_f64':>11s} {'hip16_rel':>10s} {'hip32_rel':>10s} {'ref16_rel':>10s} {'share':>7s}")
        for _, n, r, h, h32, rb in sel[:40]:
            print(f"{n:60s} {r:11.4e} {h / r - 1 if r else 0:10.4f} {h32 / r - 1 if r else 0:10.4f} "
                  f"{rb / r - 1 if r else 0:10.4f} {abs(h ** 2 - r ** 2) / tot:7.3f}")


if __name__ == "__main__":
    main()
