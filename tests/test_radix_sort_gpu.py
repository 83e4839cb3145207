"""In-tree onesweep radix sort (hip/radix_sort.hip) against torch's stable sort, bitwise (up to a
Criteo-sized batch: ~620 tiles resolving their prefixes by look-back at once), and the dedup plan
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
                                    (300_000, 31), (200_000, 32), (5_111_808, 24)])
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


def _plan(dd, n):
    torch.cuda.synchronize()
    U, C = int(dd.counts[0]), int(dd.counts[1])
    return [dd.skeys[:n].clone(), dd.perm[:n].clone(), dd.uniq[:U].clone(), dd.seg_start[:U + 1].clone(),
            dd.seg_chunk[:U + 1].clone(), dd.chunk_start[:C + 1].clone(), dd.chunk_seg[:C].clone(),
            dd.chunk_key[:C].clone(), dd.counts[:3].clone()]


def _offsets(B: int, short: bool, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    # short: empty and 1-2-feature examples (the code generator's example window has to move)
    lens = torch.randint(0, 3, (B,), generator=g) if short else torch.randint(20, 60, (B,), generator=g)
    offs = torch.zeros(B + 1, dtype=torch.int32)
    offs[1:] = torch.cumsum(lens, 0)
    return offs.cuda()


@pytest.mark.parametrize("algo", ["fm", "rocprim"])
@pytest.mark.parametrize("short,shift", [(False, 6), (True, 3), (False, 0)])
def test_dedup_generated_codes_match_csr_rows(algo, short, shift):
    """gen_codes (csr_rows folded into the sort's first pass) == csr_rows + dedup, bitwise."""
    offsets = _offsets(150_000 if short else 20_000, short, seed=7 + shift)
    n = int(offsets[-1])
    rows = _keys(n, 20, seed=11)
    was = K.set_sort_algo(algo)
    try:
        ws1 = K.DedupWorkspace(n, rows.device, 32)
        ex = K.csr_rows(offsets, out=ws1.ex_of_occ[:n], nnz=n, slot_bits=shift)
        ref = _plan(K.dedup(rows, ws=ws1, key_bits=20, ex_of_occ=ex, ex_shift=shift,
                            offsets=offsets if shift else None), n)
        ws2 = K.DedupWorkspace(n, rows.device, 32)
        got = _plan(K.dedup(rows, ws=ws2, key_bits=20, gen_codes=True, ex_shift=shift, offsets=offsets), n)
    finally:
        K.set_sort_algo(was)
    for a, c in zip(ref, got):
        assert torch.equal(a, c)


@pytest.mark.parametrize("algo", ["fm", "rocprim"])
@pytest.mark.parametrize("misalign", [0, 1])
def test_dedup_fused_shard_keys(algo, misalign):
    """shard_ids (the sharded-key map folded into the sort's histogram) == shard_keys + dedup, bitwise."""
    n, W, Rps = 300_001, 8, 2 ** 20
    base = torch.randint(0, W * Rps, (n + 1,), device="cuda", dtype=torch.int32)
    ids = base[misalign:misalign + n]   # (misalign: 4-byte offset -> the scalar load path)
    bits = (W * Rps - 1).bit_length()
    was = K.set_sort_algo(algo)
    try:
        keys_ref = K.shard_keys(ids, W, Rps, torch.empty(n, dtype=torch.int32, device="cuda"))
        ref = _plan(K.dedup(keys_ref, ws=K.DedupWorkspace(n, ids.device, 32), key_bits=bits), n)
        buf = torch.full((n + 1,), -1, dtype=torch.int32, device="cuda")[misalign:misalign + n]
        got = _plan(K.dedup(buf, ws=K.DedupWorkspace(n, ids.device, 32), key_bits=bits, shard_ids=ids,
                            shard=(W, Rps)), n)
    finally:
        K.set_sort_algo(was)
    assert torch.equal(buf, keys_ref)
    for a, c in zip(ref, got):
        assert torch.equal(a, c)


def test_lookback_failure_is_loud():
    """A look-back that hits its spin bound (injected: spin cap < 0) must not pass silently: the
    dedup's counts[7] makes DedupOut.sync raise, and the sticky device word makes
    check_device_errors raise (the bench / trainer reporting points); cleared, the next plan is fine."""
    from fast_tffm_amd.ops import native

    h = native.hip()
    was = K.set_sort_algo("fm")
    keys = _keys(100_000, 24, seed=5)
    K.dedup(keys.clone(), key_bits=24).sync()  # (first use: the sort's self-check runs outside the injection)
    K.check_device_errors()  # (clean start)
    try:
        h.set_sort_spin_cap(-1)
        dd = K.dedup(keys.clone(), key_bits=24)
        with pytest.raises(RuntimeError, match="spin bound"):
            dd.sync()
        with pytest.raises(RuntimeError, match="radix sort"):
            K.check_device_errors()
        K.check_device_errors()  # cleared by the raising check
    finally:
        h.set_sort_spin_cap(1 << 20)
        K.set_sort_algo(was)
    dd = K.dedup(keys.clone(), key_bits=24)
    assert dd.sync() == int(torch.unique(keys).numel())
    K.check_device_errors()


def test_radix_sort_rejects_oversized_n():
    """n >= 2^30 would overflow the 30-bit look-back prefixes: the launcher refuses it (no launch)."""
    from fast_tffm_amd.ops import native

    h = native.hip()
    t = torch.empty(1, dtype=torch.int32, device="cuda")
    with pytest.raises(RuntimeError, match="code -5"):
        h.radix_sort(keys=t.data_ptr(), vals=t.data_ptr(), kout=t.data_ptr(), vout=t.data_ptr(), n=(1 << 30) + 1,
                     end_bit=32, ws=t.data_ptr(), ws_bytes=1 << 62, stream=torch.cuda.current_stream().cuda_stream)
