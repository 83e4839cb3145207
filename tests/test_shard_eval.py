"""Row-sharded executor: evaluation between pipelined training steps, and the
single-communicator mode.

* ``forward()`` (validation / predict) called while a depth-2 lookahead pipeline
  holds plans in every training slot must not touch those plans' buffers: the
  table after training is bitwise identical to a run without the forward
  (regression: an eval plan used to reuse the next-but-one batch's slot and
  overwrite its dedup in place);
* ``FM_SINGLE_COMM=1`` (every collective on one communicator, program order)
  trains bitwise identically to the default two-communicator pipeline;
* a caller that trains another batch than the ``next_batch`` / ``next2`` it promised gets the
  plans of the promised batches dropped (regression: the pipeline ran out of plan slots) and
  trains bitwise like a run whose lookahead matched.

CPU, gloo, world 2 (reference C3/C4/C6 sites: /root/reference/run_tffm.py:181-226).
"""

import os

import torch
import torch.multiprocessing as mp

from fast_tffm_amd.data.synthetic import random_batch
from fast_tffm_amd.models.fm import FactorizationMachine, FMConfig
from fast_tffm_amd.ops import kernels as K

V, KF, B, STEPS, WORLD = 1499, 8, 32, 6, 2


def _free_port() -> int:
    from ports import free_port

    return free_port()


def _worker(rank, world, port, variant, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if variant == "single_comm":
        os.environ["FM_SINGLE_COMM"] = "1"
    from fast_tffm_amd.parallel import dist as fmdist

    ctx = fmdist.init_distributed(backend="gloo", rank=rank, world=world, device="cpu")
    cfg = FMConfig(vocabulary_size=V, factor_num=KF, loss_type="logistic", factor_lambda=0.01, batch_size=B,
                   init_value_range=0.1, seed=5, mode="shard", threads=1,
                   opt=K.OptConfig("adagrad", lr=0.1, initial_accumulator=0.1))
    m = FactorizationMachine(cfg, device="cpu", dist=ctx)
    assert m._exchange.comm_mode == ("single" if variant == "single_comm" else "dual")
    bs = [random_batch(B, V, max_feats=12, seed=100 * s + rank) for s in range(STEPS)]
    vb = random_batch(B, V, max_feats=12, seed=7777 + rank)
    losses, evals = [], []
    order = [0, 1, 2, 4, 3, 5] if variant in ("deviate", "reorder") else list(range(STEPS))
    for s in range(STEPS):
        if variant == "deviate":  # promises the natural order, trains ``order``
            nb = bs[s + 1] if s + 1 < STEPS else None
            nb2 = bs[s + 2] if s + 2 < STEPS else None
        else:
            nb = bs[order[s + 1]] if s + 1 < STEPS else None
            nb2 = bs[order[s + 2]] if s + 2 < STEPS else None
        losses.append(m.train_step(bs[order[s]], nb, nb2).mean_loss())
        if variant == "eval" and s in (1, 3):
            evals.append(m.eval_loss(vb))  # every training slot is busy here
    torch.save({"rows": m.table.reference_rows(), "acc": m.table.s0v.clone(), "losses": torch.tensor(losses),
                "evals": torch.tensor(evals)}, os.path.join(out_dir, f"{variant}{rank}.pt"))
    fmdist.shutdown()


def _run(tmp_path, variant):
    port = _free_port()
    mp.spawn(_worker, args=(WORLD, port, variant, str(tmp_path)), nprocs=WORLD, join=True)
    return [torch.load(os.path.join(tmp_path, f"{variant}{r}.pt"), weights_only=True) for r in range(WORLD)]


def test_forward_between_lookahead_steps_leaves_training_unchanged(tmp_path):
    plain = _run(tmp_path, "plain")
    ev = _run(tmp_path, "eval")
    for a, b in zip(plain, ev):
        assert torch.equal(a["losses"], b["losses"])
        assert torch.equal(a["rows"], b["rows"])
        assert torch.equal(a["acc"], b["acc"])
        assert b["evals"].numel() == 2 and torch.isfinite(b["evals"]).all()


def test_single_communicator_mode_is_exact(tmp_path):
    dual = _run(tmp_path, "plain")
    single = _run(tmp_path, "single_comm")
    for a, b in zip(dual, single):
        assert torch.equal(a["losses"], b["losses"])
        assert torch.equal(a["rows"], b["rows"])


def test_broken_lookahead_promise_drops_pending_plans(tmp_path):
    ref = _run(tmp_path, "reorder")
    dev = _run(tmp_path, "deviate")
    for a, b in zip(ref, dev):
        assert torch.equal(a["losses"], b["losses"])
        assert torch.equal(a["rows"], b["rows"])
        assert torch.equal(a["acc"], b["acc"])
