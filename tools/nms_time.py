"""hv_nms on the streaming leg's real input: the base model's decoded outputs of one 640x640 frame
(random-init weights, as bench.py's streaming leg), conf 0.25 / IoU 0.45 / max_det 100.  Prints the
candidate count and the number of tied scores per scale, and the NmsPlan.run time (HIP events,
median of 50)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import HybridVisionSystem, ops  # noqa: E402

torch.manual_seed(0)
m = HybridVisionSystem({"image_size": 640, "verbose": False}).cuda().eval()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
x = torch.randn(B, 3, 640, 640, device="cuda")
with torch.no_grad():
    dec = m(x)["decoded"]
for k in sorted(dec):
    s = dec[k]["class_scores"].reshape(B, -1)[0]
    c = s[s > 0.25]
    u = torch.unique(c)
    print(f"{k}: cells {s.numel()} candidates {c.numel()} distinct scores {u.numel()}")
plan = ops.NmsPlan(dec, 0.25, 0.45, 100)
ts = []
for _ in range(50):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    plan.run()
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
ts.sort()
print(f"NmsPlan.run: median {ts[len(ts) // 2] * 1e3:.1f} us, min {ts[0] * 1e3:.1f} us; kept {plan.count.tolist()}")
# the same call against the oracle (CPU restatement of post_process with std::sort's tie order)
from oracle import hv_oracle as O  # noqa: E402
ref = O.post_process({k: {n: v[n][:1].cpu() for n in ("boxes", "class_scores", "class_indices")}
                      for k, v in dec.items()}, 0.25, 0.45, 100)[0]
k0 = int(plan.count[0])
same = (k0 == ref["scores"].numel() and torch.equal(plan.scores[0, :k0].cpu(), ref["scores"])
        and torch.equal(plan.boxes[0, :k0].cpu(), ref["boxes"]) and torch.equal(plan.labels[0, :k0].cpu(), ref["labels"]))
print(f"image 0 equals the oracle: {same}")
