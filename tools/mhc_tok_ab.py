"""Token-tile fused mHC (HV_MV_TOK, csrc/hv_mhc_tok.hip) per launch against the unfused chain and
the chunk-streaming fused kernels, at in-model token counts; plus the grouped q/k/v launch against
three single launches.  usage: python tools/mhc_tok_ab.py [D:T:e ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "humanoid-vision-system_amd")]
import torch  # noqa: E402
from hv_amd import ManifoldHyperConnection, _lib, ops  # noqa: E402
from hv_amd import manifold as MF  # noqa: E402
from hv_amd.runtime import HVOptions, RunCtx, use_ctx  # noqa: E402

shapes = [tuple(int(v) for v in s.split(":")) for s in sys.argv[1:]] or \
    [(256, 401, 2), (256, 1604, 2), (256, 6416, 2), (256, 25600, 2), (128, 6400, 4), (128, 25600, 4),
     (256, 1600, 4), (256, 6400, 4)]


def timed(fn, n=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


T_ = _lib.MV_TOK
CASES = {"unfused": HVOptions(use_fused_mhc=False, mhc_tok=False),
         "fused_old": HVOptions(mhc_tok=False, mhc256_min_tokens=0),
         "tok32": HVOptions(mhc_variant=T_),
         "tok16": HVOptions(mhc_variant=T_ | _lib.MV_TOK16),
         "toks2": HVOptions(mhc_variant=T_ | _lib.MV_TOK16 | _lib.MV_TOKSPLIT2),
         "toks4": HVOptions(mhc_variant=T_ | _lib.MV_TOK16 | _lib.MV_TOKSPLIT4)}

for D, T, ex in shapes:
    Hd = ex * D
    m = ManifoldHyperConnection(D, expansion_rate=ex).cuda().eval()
    x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    r = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    p = m.plan()
    fl = 2.0 * T * (D * 2 * Hd + 2 * Hd * Hd + (Hd + D) * D)
    res = {}
    with torch.no_grad():
        with use_ctx(RunCtx(dtype=torch.bfloat16, opts=CASES["unfused"])):
            ref = MF.mhc_apply(x, p, r).float()
        for k, o in CASES.items():
            if k.startswith("tok") and not ops.mhc_fused_supported(D, Hd, torch.bfloat16, variant=o.mhc_variant):
                continue
            with use_ctx(RunCtx(dtype=torch.bfloat16, opts=o)):
                y = MF.mhc_apply(x, p, r).float()
                err = ((y - ref).norm() / ref.norm()).item()
                t = min(timed(lambda: MF.mhc_apply(x, p, r)) for _ in range(3))
            res[k] = t
            print(f"mhc D={D:4d} Hd={Hd:5d} T={T:7d} {k:9s}: {t * 1e3:8.1f} us {fl / t / 1e9:7.1f} TF/s  "
                  f"rel err vs unfused {err:.2e}", flush=True)
        # grouped q / k / v (same x, three sites) vs three single launches
        if ops.mhc_fused_supported(D, Hd, torch.bfloat16, variant=T_):
            ms = [ManifoldHyperConnection(D, expansion_rate=ex).cuda().eval() for _ in range(3)]
            ps = [mm.plan() for mm in ms]
            for tag, v in (("tok32", T_), ("tok16", T_ | _lib.MV_TOK16), ("toks2", T_ | _lib.MV_TOK16 | _lib.MV_TOKSPLIT2),
                           ("toks4", T_ | _lib.MV_TOK16 | _lib.MV_TOKSPLIT4)):
                if not ops.mhc_fused_supported(D, Hd, torch.bfloat16, variant=v):
                    continue
                outs = ops.mhc_fused_group(x, ps, v)
                with use_ctx(RunCtx(dtype=torch.bfloat16, opts=HVOptions(mhc_variant=v))):
                    singles = [MF.mhc_apply(x, pp) for pp in ps]
                    same = all(torch.equal(a, b) for a, b in zip(outs, singles))
                    t1 = min(timed(lambda: [MF.mhc_apply(x, pp) for pp in ps]) for _ in range(3))
                tg = min(timed(lambda: ops.mhc_fused_group(x, ps, v)) for _ in range(3))
                print(f"qkv D={D:4d} T={T:7d} {tag}: group {tg * 1e3:8.1f} us vs 3 singles {t1 * 1e3:8.1f} us "
                      f"(bitwise equal {same})", flush=True)
