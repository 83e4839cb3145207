"""End-to-end: run.py train / predict / generate on (a slice of) the reference's sample data.

The reference has no integration tests; these cover the CLI
contract: stdout lines, checkpoint + auto-resume, validation early stop,
``<file>_score`` outputs and the serving export signature.
"""

import contextlib
import io
import os
import re

import numpy as np
import pytest

from fast_tffm_amd import cli
from fast_tffm_amd.config import load_config
from fast_tffm_amd.serving import ServingModel
from fast_tffm_amd.utils import checkpoint as ckpt


def _copy_head(src, dst, n):
    with open(src, "rb") as f, open(dst, "wb") as g:
        for i, line in enumerate(f):
            if i >= n:
                break
            g.write(line)


@pytest.fixture()
def workdir(tmp_path, ref_data_dir):
    d = tmp_path / "data"
    d.mkdir()
    for i in range(2):
        _copy_head(os.path.join(ref_data_dir, f"train_{i}"), d / f"train_{i}", 3000)
        _copy_head(os.path.join(ref_data_dir, f"weight_{i}"), d / f"weight_{i}", 3000)
    _copy_head(os.path.join(ref_data_dir, "test_0"), d / "test_0", 1500)
    return tmp_path


def _write_cfg(workdir, **over):
    vals = dict(loss_type="logistic", batch_size=1000, epoch_num=2, save_steps=3, extra_train="",
                log_dir=str(workdir / "log"), factor_num=8, extra_general="", device="cpu")
    vals.update(over)
    text = f"""[General]
vocabulary_size = 200000
vocabulary_block_num = 4
factor_num = {vals['factor_num']}
hash_feature_id = False
log_dir = {vals['log_dir']}
save_summaries_steps = 1
device = {vals['device']}
{vals['extra_general']}

[Train]
batch_size = {vals['batch_size']}
init_value_range = 0.01
factor_lambda = 0.0001
bias_lambda = 0.0001
epoch_num = {vals['epoch_num']}
learning_rate = 0.05
adagrad.initial_accumulator = 0.1
save_steps = {vals['save_steps']}
loss_type = {vals['loss_type']}
train_files = {workdir}/data/train_*
weight_files = {workdir}/data/weight_*
{vals['extra_train']}

[Predict]
predict_files = {workdir}/data/test_0
"""
    p = workdir / "run.cfg"
    p.write_text(text)
    return str(p)


def _run(argv):
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = cli.main(argv)
    return rc, buf.getvalue()


def test_config_parity_and_echo(workdir):
    cfg_path = _write_cfg(workdir)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        c = load_config(cfg_path)
    out = buf.getvalue()
    assert out.startswith("Config: ")
    assert "  vocabulary_size = 200000" in out and "  adagrad.initial_accumulator = 0.1" in out
    assert c.vocabulary_size == 200000 and c.factor_num == 8 and c.batch_size == 1000
    assert c.adagrad_init_accumulator == 0.1 and c.loss_type == "logistic"
    assert len(c.train_files) == 2 and len(c.weight_files) == 2 and c.predict_files


def test_reference_sample_cfg_loads():
    p = "/root/reference/sample.cfg"
    if not os.path.exists(p):
        pytest.skip("reference sample.cfg not available")
    c = load_config(p, echo=False)
    assert (c.vocabulary_size, c.vocabulary_block_num, c.factor_num) == (800000, 10, 100)
    assert (c.batch_size, c.num_epochs, c.save_steps, c.loss_type) == (50000, 20, 10, "mse")
    assert len(c.train_files) == 5 and len(c.weight_files) == 5  # resolved next to the cfg


@pytest.mark.parametrize("global_bias", [False, True])
def test_train_predict_generate(workdir, global_bias):
    cfg_path = _write_cfg(workdir, extra_general="global_bias = true" if global_bias else "")
    rc, out = _run(["train", cfg_path, "--max-steps", "5"])
    assert rc == 0
    assert "======== train ========" in out
    losses = [float(m) for m in re.findall(r"-- Global Step: \d+; Avg loss: ([0-9.]+);", out)]
    assert len(losses) == 5
    assert "Average speed: " in out and "Model saved to " in out
    log = workdir / "log"
    assert ckpt.latest_checkpoint(str(log)).endswith("model.ckpt-5")
    assert (log / "metrics.jsonl").exists()

    # auto-resume: restores step 5 and the reader position; 2 epochs x 6000 lines / 1000 = 12 steps in all
    rc, out2 = _run(["train", cfg_path])
    assert "Restored checkpoint" in out2
    steps2 = [int(m) for m in re.findall(r"-- Global Step: (\d+);", out2)]
    assert steps2 == list(range(6, 13))
    losses += [float(m) for m in re.findall(r"-- Global Step: \d+; Avg loss: ([0-9.]+);", out2)]
    assert np.mean(losses[-3:]) < np.mean(losses[:3])
    assert ckpt.latest_checkpoint(str(log)).endswith("model.ckpt-12")

    rc, out3 = _run(["predict", cfg_path])
    assert rc == 0 and "Done. Scores saved" in out3
    scores = np.loadtxt(workdir / "data" / "test_0_score")
    assert scores.shape == (1500,) and np.isfinite(scores).all()

    export = workdir / "export"
    rc, out4 = _run(["generate", cfg_path, "--export_path", str(export)])
    assert rc == 0 and "Done exporting!" in out4
    sm = ServingModel.load(str(export), device="cpu")
    lines = open(workdir / "data" / "test_0").read().splitlines()[:50]
    feats = [" ".join(t if ":" in t else t + ":1" for t in ln.split()[1:]) for ln in lines]
    np.testing.assert_allclose(sm.predict(np.array(feats)), scores[:50], rtol=1e-5, atol=1e-6)
    # the TF SavedModel of the reference's serving graph (saved_model.pb + variables bundle),
    # evaluated by the independent numpy graph interpreter, gives the same scores
    from fast_tffm_amd.utils import saved_model as tfsm

    info = tfsm.read_saved_model(str(export))
    assert info["tags"] == ["serve"] and info["saver"]["restore_op_name"] == "save/restore_all"
    sig = info["signatures"]["serving_default"]
    assert sig["method_name"] == "tensorflow/serving/predict"
    assert set(sig["inputs"]) == {"data_lines"} and set(sig["outputs"]) == {"scores"}
    np.testing.assert_allclose(tfsm.run_graph(str(export), feats), scores[:50], rtol=1e-5, atol=1e-5)
    # export path must be new
    with pytest.raises(FileExistsError):
        _run(["generate", cfg_path, "--export_path", str(export)])


def test_validation_early_stop(workdir):
    extra = f"validation_files = {workdir}/data/test_0\ntolerance = 100.0"
    cfg_path = _write_cfg(workdir, extra_train=extra, log_dir=str(workdir / "log_es"))
    rc, out = _run(["train", cfg_path])
    assert "Preloading validation data..." in out
    assert re.search(r"validation loss at step 3: [0-9.]+", out)
    assert "Loss on validation data set is below tolerance. Training completed." in out
    assert "-- Global Step: 4;" not in out


def test_predict_requires_log_dir(workdir, monkeypatch):
    cfg_path = _write_cfg(workdir)
    text = open(cfg_path).read().replace(f"log_dir = {workdir}/log\n", "")
    open(cfg_path, "w").write(text)
    codes = []
    monkeypatch.setattr(os, "_exit", lambda c: (_ for _ in ()).throw(SystemExit(c)))
    with pytest.raises(SystemExit) as e:
        _run(["predict", cfg_path])
    assert e.value.code == 1


def test_dist_ps_role_exits(workdir):
    rc, out = _run(["train", _write_cfg(workdir), "--dist", "ps", "0", "localhost:1", "localhost:2"])
    assert rc == 0 and "not needed" in out


def test_trace_file_written(workdir):
    cfg_path = _write_cfg(workdir, log_dir=str(workdir / "log_tr"))
    trace = str(workdir / "timeline")
    rc, out = _run(["train", cfg_path, "-t", trace, "-m"])
    assert os.path.exists(trace + ".json")
    assert "speed:" in out and "example_queue:" in out
    # shuffle_queue is the loader's real window fill (reference run_tffm.py:52-63), not a constant:
    # the window holds between min_after_dequeue + B and capacity (4.5 B) lines while full, less
    # while the epoch's tail drains
    fills = [float(x) for x in re.findall(r"shuffle_queue: ([0-9.]+)%", out)]
    assert fills and all(0.0 <= f <= 100.0 for f in fills)
    assert len(set(fills)) > 1 or fills[0] < 100.0


@pytest.fixture()
def synth_workdir(tmp_path):
    """Criteo-shaped synthetic train / weight / test files (no reference data needed: GPU boxes)."""
    from fast_tffm_amd.data.synthetic import write_libsvm

    d = tmp_path / "data"
    d.mkdir()
    for i in range(2):
        write_libsvm(str(d / f"train_{i}"), 3000, shape="criteo", vocab_size=200_000, seed=i,
                     weights_path=str(d / f"weight_{i}"))
    write_libsvm(str(d / "test_0"), 1500, shape="criteo", vocab_size=200_000, seed=9)
    return tmp_path


@pytest.mark.gpu
@pytest.mark.parametrize("gpu_parse", [False, True], ids=["cpu_parser", "gpu_tokenizer"])
def test_train_and_resume_on_gpu(synth_workdir, gpu_parse):
    """run.py train on the GPU with the file-fed input path (native loader + the C++ device
    feeder: CPU parser or GPU tokenizer), stopped after 5 steps and auto-resumed to the end."""
    workdir = synth_workdir
    cfg_path = _write_cfg(workdir, device="cuda", extra_train="gpu_parse = true" if gpu_parse else "")
    rc, out = _run(["train", cfg_path, "--max-steps", "5"])
    assert rc == 0
    losses = [float(m) for m in re.findall(r"-- Global Step: \d+; Avg loss: ([0-9.]+);", out)]
    assert len(losses) == 5
    rc, out2 = _run(["train", cfg_path])
    assert rc == 0 and "Restored checkpoint" in out2
    steps2 = [int(m) for m in re.findall(r"-- Global Step: (\d+);", out2)]
    assert steps2 == list(range(6, 13))
    losses += [float(m) for m in re.findall(r"-- Global Step: \d+; Avg loss: ([0-9.]+);", out2)]
    assert np.isfinite(losses).all() and np.mean(losses[-3:]) < np.mean(losses[:3])
