"""Raw-mode loader output into caller-owned slots (the GPU tokenizer's page-locked buffers):
the same line bytes and offsets as heap batches, slot reuse through release(), and a heap
fallback for a batch larger than its slot.  CPU only (plain host buffers stand in for pinned
ones: the loader only needs writable memory)."""

import numpy as np
import torch

from fast_tffm_amd.data.synthetic import write_libsvm
from fast_tffm_amd.ops import native


def _args(files, B):
    return dict(files=files, weight_files=[], batch_size=B, vocab_size=5000, hash_feature_id=False, shuffle=True,
                num_epochs=2, seed=3, threads=2, rank=0, world=1, queue_size=2)


def _heap_batches(files, B):
    L = native.cpu().TextLoader(start_epoch=0, skip_batches=0, raw=True, **_args(files, B))
    out = []
    while (it := L.next()) is not None:
        out.append((bytes(it[0]), it[1].copy(), it[3], it[4]))
    L.close()
    return out


def test_slot_batches_equal_heap_batches(tmp_path):
    files = []
    for i in range(2):
        p = str(tmp_path / f"d{i}")
        write_libsvm(p, 700, shape="criteo", vocab_size=5000, seed=i)
        files.append(p)
    B = 128
    want = _heap_batches(files, B)
    slots = [(torch.empty(B * 1024, dtype=torch.uint8), torch.empty(B + 1, dtype=torch.int64)) for _ in range(3)]
    spec = [[b.data_ptr(), b.numel(), ls.data_ptr(), ls.numel()] for b, ls in slots]
    L = native.cpu().TextLoader(start_epoch=0, skip_batches=0, raw=True, raw_slots=spec, **_args(files, B))
    got, used = [], set()
    while (it := L.next()) is not None:
        assert isinstance(it[0], int)
        s, nbytes, nlines = it[0], it[1], it[2]
        used.add(s)
        got.append((bytes(slots[s][0][:nbytes].numpy()), slots[s][1][: nlines + 1].numpy().copy(), it[4], it[5]))
        L.release(s)
    L.close()
    assert len(got) == len(want) and used <= {0, 1, 2}
    for (gb, gl, ge, gc), (wb, wl, we, wc) in zip(got, want):
        assert gb == wb and np.array_equal(gl, wl) and (ge, gc) == (we, wc)


def test_batch_larger_than_its_slot_uses_the_heap(tmp_path):
    p = str(tmp_path / "d")
    write_libsvm(p, 300, shape="criteo", vocab_size=5000, seed=5)
    B = 64
    want = _heap_batches([p], B)
    tiny = [(torch.empty(256, dtype=torch.uint8), torch.empty(B + 1, dtype=torch.int64))]
    spec = [[b.data_ptr(), b.numel(), ls.data_ptr(), ls.numel()] for b, ls in tiny]
    L = native.cpu().TextLoader(start_epoch=0, skip_batches=0, raw=True, raw_slots=spec, **_args([p], B))
    got = []
    while (it := L.next()) is not None:
        assert not isinstance(it[0], int)  # every batch exceeds 256 bytes: heap path, slot returned
        got.append((bytes(it[0]), it[1].copy()))
    L.close()
    assert [g[0] for g in got] == [w[0] for w in want]
