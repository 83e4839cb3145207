"""Diagnostic: error of the VALU and MFMA fp8 forwards against fp64 (pred and r1), in units of the
terms' magnitude (tests/test_fwd_mfma_gpu.py helpers)."""
import sys
import torch

sys.path.insert(0, "tests")
from test_fwd_mfma_gpu import _table, _fwd, _magnitudes  # noqa: E402
from fast_tffm_amd.data.synthetic import random_batch  # noqa: E402

for spread in (0, 4, 17):
    t = _table(6000, seed=11)
    if spread == 0:   # every row at one scale
        t.set_v(None, torch.randn((6000, 128), device="cuda") * 0.05)
    elif spread == 4:
        g = torch.Generator(device="cuda").manual_seed(3)
        mag = torch.exp2(torch.randint(-4, 1, (6000, 1), generator=g, device="cuda").float())
        t.set_v(None, torch.randn((6000, 128), generator=g, device="cuda") * mag)
    b = random_batch(1000, 6000, max_feats=40, min_feats=0, seed=1, device="cuda", with_vals=False)
    mag, col = _magnitudes(t, b)
    p = t.reference_rows().double()
    ex = torch.repeat_interleave(torch.arange(b.B, device="cuda"), (b.offsets[1:] - b.offsets[:-1]).long(),
                                 output_size=b.ids.numel())
    s1 = torch.zeros((b.B, 128), dtype=torch.float64, device="cuda").index_add(0, ex, p[b.ids.long(), 1:])
    for name, on in (("valu", False), ("mfma", True)):
        o = _fwd(t, b, on)
        # pred error vs a fp64 pred from the same stored rows
        lin = torch.zeros(b.B, dtype=torch.float64, device="cuda").index_add(0, ex, p[b.ids.long(), 0])
        s2 = torch.zeros(b.B, dtype=torch.float64, device="cuda").index_add(0, ex, (p[b.ids.long(), 1:] ** 2).sum(1))
        ref = lin + 0.5 * ((s1 * s1).sum(1) - s2)
        ep = ((o.pred.double() - ref).abs() / mag.clamp_min(1e-30)).max().item()
        er = ((o.r1.double() - s1).abs() - 2.0 ** -8 * s1.abs()).clamp_min(0)
        er = (er / col.clamp_min(1e-30)).max().item()
        print(f"spread {spread:2d} {name}: max |pred err|/mag = {ep:.3e}  max r1 excess err/colabs = {er:.3e}")
