"""Long-horizon precision parity of the low-precision tables.

A planted FM teacher (k=8, hashed Zipf-popular ids over 24 fields) labels Criteo-shaped
examples; students with fp32, bf16 + stochastic rounding and fp8 (e4m3 + per-row scale)
+ stochastic rounding tables train 400 steps on the same batch sequence, and their
held-out logloss must agree with the fp32 student's within 0.5% (relative).  The fp32
student must also beat the label-prior baseline clearly (the comparison is between models
that actually learned something).  fp32 is the reference's precision
(tffm/fm_model.py:269-284); the low-precision tables keep fp32 arithmetic and accumulation,
bf16 tables fp32 optimizer state, fp8 tables bf16 optimizer state with stochastic rounding
(ops/kernels.py state_dtype).  Adagrad (the reference optimizer) and FTRL (BASELINE config 5) both.
"""

import math

import pytest
import torch

from fast_tffm_amd.data.batch import Batch
from fast_tffm_amd.data.synthetic import CriteoSynth
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

pytestmark = pytest.mark.gpu

V, B, STEPS, NTRAIN, NHELD = 50_000, 4096, 400, 48, 8
FIELDS = [12, 40, 100, 300, 800, 2000, 5000, 9000] * 3  # 24 fields, small to mid cardinality


def _teacher_data(dev):
    g = torch.Generator(device=dev).manual_seed(77)
    w = torch.randn(V, generator=g, device=dev) * 0.6
    v = torch.randn(V, 8, generator=g, device=dev) * 0.35
    synth = CriteoSynth(V, fields=FIELDS, alpha=1.05, seed=99, device=dev)
    out = []
    for _ in range(NTRAIN + NHELD):
        b = synth.batch(B)
        ids = b.ids.long().view(B, len(FIELDS))
        s1 = v[ids].sum(1)
        score = w[ids].sum(1) + 0.5 * (s1.pow(2) - v[ids].pow(2).sum(1)).sum(1) - 1.0
        labels = (torch.rand(B, generator=g, device=dev) < torch.sigmoid(score)).float()
        out.append(Batch(labels, b.offsets, b.ids, None, None, b.nnz, max_feats=b.max_feats,
                         offsets_host=b.offsets_host))
    return out[:NTRAIN], out[NTRAIN:]


@pytest.fixture(scope="module")
def data():
    return _teacher_data(torch.device("cuda:0"))


def _train(dtype, opt, data):
    train, held = data
    cfg = FMConfig(vocabulary_size=V, factor_num=16, loss_type="logistic", batch_size=B, init_value_range=0.01,
                   seed=5, dtype=dtype, opt=opt, stochastic_rounding=True)
    m = FactorizationMachine(cfg, device="cuda:0")
    for i in range(STEPS):
        m.train_step(train[i % NTRAIN], train[(i + 1) % NTRAIN])
    loss = sum(m.eval_loss(b) for b in held) / len(held)
    m.close()
    return loss


@pytest.mark.parametrize("opt", [K.OptConfig("adagrad", lr=0.3), K.OptConfig("ftrl", lr=0.3, l1=0.001, l2=0.001)],
                         ids=["adagrad", "ftrl"])
def test_low_precision_tables_match_fp32_heldout_logloss(data, opt):
    held = data[1]
    p = sum(float(b.labels.mean()) for b in held) / len(held)
    prior = -(p * math.log(p) + (1 - p) * math.log(1 - p))
    ref = _train(torch.float32, opt, data)
    # the students learn the teacher's signal (CPU fp32: 0.611 / 0.621 against a 0.676 prior)
    assert ref < 0.95 * prior, (ref, prior)
    for dtype in (torch.bfloat16, K.FP8):
        got = _train(dtype, opt, data)
        print(f"[parity] {opt.name} {str(dtype).replace('torch.', '')}: held-out logloss {got:.5f} "
              f"vs fp32 {ref:.5f} (rel {(got - ref) / ref:+.2e}; prior {prior:.5f})")
        assert abs(got - ref) / ref < 5e-3, (str(dtype), got, ref, prior)
