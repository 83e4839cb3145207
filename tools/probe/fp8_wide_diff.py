"""Where the wide fp8 chunk kernel's FTRL state differs from the 4-value kernel's: per mismatching element,
the row's occurrence count in the step, the column, both values (one local step, k=128 fp8 FTRL)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fast_tffm_amd.data.synthetic import CriteoSynth  # noqa: E402
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig  # noqa: E402
from fast_tffm_amd.ops import kernels as K  # noqa: E402

V, B = 60_000, 8192
gen = CriteoSynth(V, seed=13, device="cuda")
b = gen.batch(B)
cnt = torch.bincount(b.ids.long(), minlength=V)


def run(var, sr):
    if var:
        os.environ["FM_HIP_VARIANT"] = var
    else:
        os.environ.pop("FM_HIP_VARIANT", None)
    o = K.OptConfig("ftrl", lr=0.05, l1=0.01, l2=0.01, beta=1.0)
    cfg = FMConfig(vocabulary_size=V, factor_num=128, loss_type="logistic", batch_size=B, init_value_range=0.05,
                   seed=3, opt=o, dtype=K.FP8, factor_lambda=0.001, bias_lambda=0.001, stochastic_rounding=sr)
    m = FactorizationMachine(cfg, device="cuda")
    m.train_step(b)
    torch.cuda.synchronize()
    t = m.table
    out = (t.v.clone(), t.s0v.clone(), t.s1v.clone())
    m.close()
    return out


for sr, va, vb in ((False, None, None), (False, "fp8narrow", "fp8narrow"), (True, None, "fp8narrow"),
                   (False, None, "fp8narrow")):
    print(f"== {va} vs {vb}")
    a, n = run(va, sr), run(vb, sr)
    for name, x, y in zip(("v", "s0v", "s1v"), a, n):
        bits = torch.uint8 if x.dtype == K.FP8 else torch.int16
        d = x.view(bits) != y.view(bits)
        idx = d.nonzero()
        print(f"sr={sr} {name}: {idx.shape[0]} mismatches", flush=True)
        for r, c in idx[:12].tolist():
            print(f"   row {r} col {c} count {int(cnt[r])}  a {float(x[r, c].float()):.9e}  "
                  f"b {float(y[r, c].float()):.9e}")
        if idx.shape[0]:
            rows = idx[:, 0].unique()
            print("   occurrence counts of mismatching rows:",
                  torch.bincount(cnt[rows].clamp(max=40)).nonzero().flatten().tolist())
