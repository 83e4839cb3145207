"""Phase breakdown of the MFMA fp8 forward (build variant "mfprof"; FM_HIP_VARIANT=mfprof):
headline shape (V = 10M, B = 131072, Criteo-shaped binary batch), 20 forwards."""
import os
import torch

from fast_tffm_amd.data.synthetic import CriteoSynth
from fast_tffm_amd.models.table import FMTable
from fast_tffm_amd.ops import kernels as K, native

assert os.environ.get("FM_HIP_VARIANT") == "mfprof"
V, B = 10_000_000, 131072
t = FMTable(V, 128, dtype=K.FP8, device="cuda", seed=1, init_range=0.01)
b = CriteoSynth(V, seed=2, device="cuda").batch(B)
ids = b.ids.to(torch.int32)
h = native.hip()
for it in range(25):
    if it == 5:
        torch.cuda.synchronize()
        h.mf_prof()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
    K.fm_forward(b.offsets, ids, None, t.v, t.w, t.Kp, labels=b.labels, weights=b.weights, loss="logistic",
                 want_reg=True, max_feats=b.max_feats)
ev1.record()
torch.cuda.synchronize()
p = h.mf_prof()
tot = sum(p[:5])
names = ["indices", "tails", "row pass", "K-loop", "epilogue"]
print(f"forward {ev0.elapsed_time(ev1) / 20 * 1000:.1f} us/call; tiles {p[5] // 20}/call; "
      f"per tile {tot / max(p[5], 1):.0f} clocks")
for n, c in zip(names, p[:5]):
    print(f"  {n:10s} {100 * c / tot:5.1f}%  {c / max(p[5], 1):8.0f} clocks/tile")
