"""Host cost of the plan chain's Python + binding calls (no device sync inside the loops): per-call
median microseconds of K.dedup at the bench shape, of the workspace-size query it runs per call, and of
the other plan-start calls.  usage: PYTHONPATH=. python tools/probe/host_dedup.py"""
import time

import torch

from fast_tffm_amd.data.synthetic import CriteoSynth
from fast_tffm_amd.ops import kernels as K
from fast_tffm_amd.ops import native


def med(fn, n=60):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
        if len(ts) % 20 == 0:
            torch.cuda.synchronize()
    ts.sort()
    return ts[len(ts) // 2] * 1e6


b = CriteoSynth(125_000_000, seed=3, device="cuda").batch(131072)
n = b.nnz
rows = b.ids.to(torch.int32)
ws = K.DedupWorkspace(n, rows.device, 32)
keys = torch.empty(n, dtype=torch.int32, device="cuda")
sb = K.slot_bits_for(b.B, b.max_feats)
h = native.hip()
torch.cuda.synchronize()
print(f"n={n}")
print(f"dedup_workspace_bytes (sort size queries)   {med(lambda: h.dedup_workspace_bytes(n)):8.1f} us")
print(f"K.dedup local (gen_codes)                   "
      f"{med(lambda: K.dedup(rows, ws=ws, key_bits=27, gen_codes=True, ex_shift=sb, offsets=b.offsets)):8.1f} us")
def shard_dedup():
    return K.dedup(keys, ws=ws, key_bits=27, gen_codes=True, ex_shift=sb, offsets=b.offsets, want_inv=False,
                   shard_ids=rows, shard=(1, 125_000_000))


print(f"K.dedup shard (gen_codes + shard_ids)       {med(shard_dedup):8.1f} us")
dd = K.dedup(rows, ws=ws, key_bits=27)
both = torch.empty((2, 1, 1), dtype=torch.int64, device="cuda")
print(f"K.owner_counts                              "
      f"{med(lambda: K.owner_counts(dd, 125_000_000, 1, out=both[0, :, 0], out2=both[1, :, 0])):8.1f} us")
def pinned_copy():
    torch.empty(both.shape, dtype=torch.int64, pin_memory=True).copy_(both, non_blocking=True)
    torch.cuda.Event().record()


print(f"torch.empty pinned + copy_ + event          {med(pinned_copy):8.1f} us")
torch.cuda.synchronize()
