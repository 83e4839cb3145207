#!/usr/bin/env python3
"""End-to-end ``run.py train`` throughput on the reference's sample workload shape
(sample.cfg: vocabulary 800k, factor_num 100, batch 50000, Adagrad, weighted mse,
text files + weight files), reporting the reference's own metric line
``Average speed: ... ex/s`` (run_tffm.py:79-81) for each input path:
native C++ loader with the CPU parser, with the GPU tokenizer, binary .fmb caches and
HBM-resident .fmb caches -- plus the trainer's steady-state speed (epochs 2+: excludes
process start-up, reader warm-up and the first pass over the files).

usage: python tools/bench_train_e2e.py [--lines 500000] [--files 4] [--epochs 6]
"""

import argparse
import os
import re
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fast_tffm_amd.data.synthetic import write_libsvm  # noqa: E402

CFG = """[General]
vocabulary_size = 800000
vocabulary_block_num = 10
factor_num = 100
hash_feature_id = False
save_summaries_steps = 1000000
[Train]
batch_size = {batch}
init_value_range = 0.01
factor_lambda = 0
bias_lambda = 0
epoch_num = {epochs}
learning_rate = 0.01
adagrad.initial_accumulator = 0.1
save_steps = 1000000
loss_type = mse
train_files = {train}
{weights}
parse_threads = {threads}
gpu_parse = {gpu}
device_cache = {dcache}
log_steps = 40
[Predict]
predict_files =
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=500_000)
    ap.add_argument("--files", type=int, default=4)
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--batch", type=int, default=50_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dir", default="/tmp/fm_e2e")
    ap.add_argument("--paths", default="false,true,fmb,fmb_hbm",
                    help="comma list: false (CPU parser), true (GPU tokenizer), fmb, fmb_hbm")
    a = ap.parse_args()
    data = os.path.join(a.dir, "data")
    os.makedirs(data, exist_ok=True)
    src, wsrc = os.path.join(data, "train_0"), os.path.join(data, "weight_0")
    if not os.path.exists(src):
        t = time.time()
        write_libsvm(src, a.lines, shape="criteo", vocab_size=800_000, seed=0, weights_path=wsrc)
        print(f"wrote {a.lines} lines in {time.time() - t:.1f}s", flush=True)
    for i in range(1, a.files):  # same lines, distinct files (the shuffle window mixes them)
        for s, d in ((src, f"train_{i}"), (wsrc, f"weight_{i}")):
            if not os.path.exists(os.path.join(data, d)):
                shutil.copy(s, os.path.join(data, d))
    text = dict(train=f"{data}/train_*", weights=f"weight_files = {data}/weight_*")
    paths = a.paths.split(",")
    if "fmb_hbm" in paths and "fmb" not in paths:
        paths.insert(paths.index("fmb_hbm"), "fmb")  # (the caches are converted by the fmb run)
    for gpu in paths:
        cfg = os.path.join(a.dir, f"e2e_{gpu}.cfg")
        fmb = gpu.startswith("fmb")
        src = text if not fmb else dict(train=f"{a.dir}/fmb/*.fmb", weights="")
        with open(cfg, "w") as f:
            f.write(CFG.format(batch=a.batch, epochs=a.epochs, threads=a.threads, gpu="false" if fmb else gpu,
                               dcache="true" if gpu == "fmb_hbm" else "false", **src))
        if gpu == "fmb":
            t = time.time()
            r = subprocess.run([sys.executable, os.path.join(ROOT, "run.py"), "convert",
                                os.path.join(a.dir, "e2e_false.cfg"), "--out", os.path.join(a.dir, "fmb")],
                               capture_output=True, text=True)
            if r.returncode != 0:
                print(r.stdout[-2000:], r.stderr[-3000:])
                sys.exit(r.returncode)
            print(f"run.py convert: {time.time() - t:.1f}s (incl. start-up)", flush=True)
        shutil.rmtree(os.path.join(a.dir, f"log_{gpu}"), ignore_errors=True)  # no auto-resume of an old run
        t = time.time()
        r = subprocess.run([sys.executable, os.path.join(ROOT, "run.py"), "train", cfg,
                            "--log-dir", os.path.join(a.dir, f"log_{gpu}")], capture_output=True, text=True)
        if r.returncode != 0:
            print(r.stdout[-2000:], r.stderr[-3000:])
            sys.exit(r.returncode)
        m = re.search(r"Average speed:\s+([0-9.eE+]+)", r.stdout)
        ms = re.search(r"Steady-state speed \(epochs 2\+\):\s+([0-9.eE+]+)", r.stdout)
        steps = len(re.findall(r"Global Step", r.stdout))
        name = {"fmb": "binary .fmb caches (host assembly)",
                "fmb_hbm": "binary .fmb caches resident in HBM"}.get(gpu, f"gpu_parse={gpu}")
        name += f" [{a.threads} threads]"
        steady = f"{float(ms.group(1)):.4g}" if ms else "n/a"
        losses = re.findall(r"Global Step: (\d+); Avg loss: ([0-9.eE+-]+);", r.stdout)
        if losses:  # (the same shuffle and seed on every path: the same batches, the same loss)
            name += f" last loss {losses[-1][1]} (step {losses[-1][0]})"
        print(f"{name}: Average speed {float(m.group(1)):.4g} ex/s, steady state (epochs 2+) {steady} ex/s "
              f"({a.files * a.lines * a.epochs} examples, wall {time.time() - t:.1f}s incl. start-up)", flush=True)


if __name__ == "__main__":
    main()
