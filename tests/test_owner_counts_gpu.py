"""owner_counts (hip/shard.hip: one wave per owner, 64-way search over the sorted unique keys)
against a plain PyTorch bincount of key // Rps; U from the device, keys past U ignored.
Reference: the per-owner id counts of the sharded lookup, tffm/fm_model.py:72-90 (partition
of the unique ids by owner before the embedding all-to-all)."""
import types

import pytest
import torch

from fast_tffm_amd.ops import kernels as K

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W,Rps,U", [(1, 1000, 0), (1, 1000, 1), (1, 125_000_000, 400_000), (2, 5000, 64),
                                     (3, 5000, 65), (8, 100_000, 378_000), (8, 1000, 4096), (16, 40, 300),
                                     (7, 1 << 20, 100_003)])
def test_owner_counts_matches_bincount(W, Rps, U):
    g = torch.Generator().manual_seed(W * 1000 + U)
    total = W * Rps
    if U:
        keys = torch.unique(torch.randint(0, total, (U * 2,), generator=g, dtype=torch.int64))[:U]
    else:
        keys = torch.empty(0, dtype=torch.int64)
    U = keys.numel()
    # skewed owners too: empty shards must count 0
    buf = torch.full((U + 37,), total - 1, dtype=torch.int64)  # junk past U must be ignored
    buf[:U] = keys
    dd = types.SimpleNamespace(uniq=buf.to(torch.int32).cuda(),
                               num_unique=torch.tensor([U], dtype=torch.int32, device="cuda"))
    got = K.owner_counts(dd, Rps, W).cpu()
    want = torch.bincount(torch.div(keys, Rps, rounding_mode="floor"), minlength=W)
    assert torch.equal(got, want), (got, want)


def test_owner_counts_empty_middle_shards():
    W, Rps = 8, 1000
    keys = torch.tensor([5, 6, 7, 3000, 3001, 7999], dtype=torch.int64)
    dd = types.SimpleNamespace(uniq=keys.to(torch.int32).cuda(),
                               num_unique=torch.tensor([keys.numel()], dtype=torch.int32, device="cuda"))
    got = K.owner_counts(dd, Rps, W).cpu().tolist()
    assert got == [3, 0, 0, 2, 0, 0, 0, 1]
