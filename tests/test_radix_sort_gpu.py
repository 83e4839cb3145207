"""In-tree radix sort (hip/radix_sort.hip) against torch's stable sort, bitwise, and the dedup plan
built on it against the rocPRIM-sorted plan, bitwise (the two backends must give the same stable
order: the plan fixes the backward's summation order)."""

import pytest
import torch

from fast_tffm_amd.data.synthetic import CriteoSynth
from fast_tffm_amd.ops import kernels as K

pytestmark = pytest.mark.gpu


def _keys(n: int, bits: int, seed: int) -> torch.Tensor:
    g = torch.Generator(device="cuda").manual_seed(seed)
    hi = 2 ** min(bits, 31)
    hot = torch.randint(0, hi, (2048,), generator=g, device="cuda")
    pick = (torch.rand(n, generator=g, device="cuda") ** 3 * 2048).long().clamp_max(2047)
    cold = torch.randint(0, hi, (n,), generator=g, device="cuda")
    return torch.where(torch.rand(n, generator=g, device="cuda") < 0.85, hot[pick], cold).to(torch.int32)


@pytest.mark.parametrize("n,bits", [(1, 8), (1000, 8), (8191, 16), (8193, 18), (100_000, 24), (1_000_003, 27),
                                    (300_000, 31)])
def test_radix_sort_matches_stable_sort(n, bits):
    k = _keys(n, bits, seed=n + bits)
    v = torch.arange(n, dtype=torch.int32, device="cuda")
    ko, vo = K.radix_sort(k, v, key_bits=bits)
    ref_k, ref_i = torch.sort(k.long(), stable=True)
    assert torch.equal(ko.long(), ref_k)
    assert torch.equal(vo.long(), ref_i)


def test_radix_sort_ignores_bits_above_end_bit():
    n = 50_000
    k = _keys(n, 20, seed=3)
    k_hi = k | (torch.randint(0, 8, (n,), device="cuda", dtype=torch.int32) << 20)  # junk above bit 20
    v = torch.arange(n, dtype=torch.int32, device="cuda")
    _, vo = K.radix_sort(k_hi, v, key_bits=20)
    _, ref_i = torch.sort(k.long(), stable=True)
    assert torch.equal(vo.long(), ref_i)


@pytest.mark.parametrize("V", [20_000, 10_000_000])
def test_dedup_plan_bitwise_equal_across_sort_backends(V):
    b = CriteoSynth(V, seed=5, device="cuda").batch(16384)
    rows = b.ids.to(torch.int32)
    bits = max(1, (V - 1).bit_length())
    sb = K.slot_bits_for(b.B, b.max_feats)
    outs = []
    for algo in ("rocprim", "fm"):
        was = K.set_sort_algo(algo)
        try:
            ws = K.DedupWorkspace(rows.numel(), rows.device, 32)
            ex = K.csr_rows(b.offsets, out=ws.ex_of_occ[: b.nnz], nnz=b.nnz, slot_bits=sb)
            dd = K.dedup(rows, ws=ws, key_bits=bits, ex_of_occ=ex, ex_shift=sb, offsets=b.offsets)
            torch.cuda.synchronize()
            n = rows.numel()
            U = int(dd.counts[0])
            C = int(dd.counts[1])
            outs.append([dd.skeys[:n].clone(), dd.perm[:n].clone(), dd.uniq[:U].clone(), dd.seg_start[:U + 1].clone(),
                         dd.seg_chunk[:U + 1].clone(), dd.chunk_start[:C + 1].clone(), dd.chunk_seg[:C].clone(),
                         dd.chunk_key[:C].clone(), dd.counts[:3].clone()])
        finally:
            K.set_sort_algo(was)
    for a, c in zip(*outs):
        assert torch.equal(a, c)
