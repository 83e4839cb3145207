"""Command line: ``python run.py {train,predict,generate,convert,import_tf,export_tf} CONFIG [options]``.

Same arguments as the reference's run_tffm.py (run_tffm.py:124-162):
  task {train,predict,generate}, config_file,
  --dist JOB_NAME TASK_INDEX PS_HOSTS WORKER_HOSTS, --protocol, --wait-for-workers N,
  -t/--trace FILE, -m/--monitor, --export_path DIR.
Extensions: --device {auto,cpu,cuda}, --mode {auto,local,shard,dp,dp_dense},
--max-steps N, --log-dir DIR (overrides [General] log_dir), and the task
``convert CONFIG --out DIR``: parse the config's train files (+ weight files) once
into binary CSR caches (``DIR/<name>.fmb``, data/bincache.py) that ``train``
reads at memory speed when ``train_files`` points at them.  Checkpoint migration:
``import_tf CONFIG --tf_checkpoint DIR|PREFIX`` loads a TensorFlow checkpoint in the
reference's variable layout (``vocab_block_{i}`` + ``/Adagrad`` slots + ``global_step``)
and writes it as this package's checkpoint into ``log_dir`` (``train`` resumes from it,
``predict`` / ``generate`` use it); ``export_tf CONFIG --export_path DIR`` writes the
latest checkpoint of ``log_dir`` back as such a TF checkpoint.

Distributed runs: launch one process per GPU with torchrun (RANK/WORLD_SIZE/
MASTER_ADDR from the environment), or keep the reference's ``--dist worker i
PS_HOSTS W1,W2,...`` form (rank i of len(WORKERS), rendezvous at the first
worker host).  ``--dist ps ...`` processes are not needed (the table lives in
the workers' HBM) and exit immediately.
"""

from __future__ import annotations

import argparse
import os
import sys


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="run.py", description="MI355X-native distributed factorization machine")
    p.add_argument("task", choices=["train", "predict", "generate", "convert", "import_tf", "export_tf"])
    p.add_argument("config_file", type=str)
    p.add_argument("--dist", nargs=4, metavar=("JOB_NAME", "TASK_INDEX", "PS_HOSTS", "WORKER_HOSTS"), default=None,
                   help="For distributed training or prediction")
    p.add_argument("--protocol", default="grpc",
                   help="kept for compatibility; the transport is RCCL (GPU) / gloo (CPU)")
    p.add_argument("--wait-for-workers", type=int,
                   help="Minimal workers started before training (the rendezvous waits for all of them)")
    p.add_argument("-t", "--trace", metavar="OUTPUT_FILE_NAME",
                   help="Stores runtime stats of the first steps as a chrome-trace timeline file")
    p.add_argument("-m", "--monitor", action="store_true", help="Prints execution speed to screen")
    p.add_argument("--export_path", help="Specifies the location to which the model is to be exported.")
    p.add_argument("--device", default=None, choices=["auto", "cpu", "cuda"])
    p.add_argument("--mode", default=None, choices=["auto", "local", "shard", "dp", "dp_dense"])
    p.add_argument("--max-steps", type=int, default=None)
    p.add_argument("--log-dir", default=None)
    p.add_argument("--out", default=None, help="convert: output directory of the .fmb caches")
    p.add_argument("--tf_checkpoint", default=None,
                   help="import_tf: TF checkpoint directory (its 'checkpoint' file names the newest) or prefix")
    return p


def main(argv: list[str] | None = None) -> int:
    args = build_parser().parse_args(argv)
    from .config import load_config
    from .parallel import dist as fmdist

    dist_info = fmdist.parse_dist_args(args.dist)
    if dist_info.get("role") == "ps":
        print("Parameter-server processes are not needed: every worker holds a shard of the table in its own "
              "GPU memory. Exiting.")
        return 0

    cfg = load_config(args.config_file)
    if args.log_dir is not None:
        cfg.log_dir = args.log_dir
    if args.device is not None:
        cfg.device = args.device
    if args.mode is not None:
        cfg.mode = args.mode
    if args.max_steps is not None:
        cfg.max_steps = args.max_steps
    if dist_info.get("world", int(os.environ.get("WORLD_SIZE", "1"))) > 1 or cfg.mode not in ("auto", "local"):
        # multi-rank step: compute, lookahead and RCCL streams need their own hardware
        # queues (HIP's default 4 makes them share and serialize); before HIP starts
        fmdist.ensure_hw_queues()

    if args.task == "predict" and cfg.log_dir is None:
        print("Missing log directory. Must include a checkpoint file.")
        os._exit(1)
    if args.task == "generate":
        if args.export_path is None:
            print("Export path is not specified. Use --export_path.")
            os._exit(2)
        from .serving import export_model
        from .utils.checkpoint import latest_checkpoint

        path = latest_checkpoint(cfg.log_dir)
        if path is None:
            print(f"No checkpoint found in {cfg.log_dir}.")
            return 1
        print("Exporting trained model to", args.export_path)
        export_model(path, args.export_path, vocabulary_block_num=cfg.vocabulary_block_num,
                     hash_feature_id=cfg.hash_feature_id, loss_type=cfg.loss_type)
        print("Done exporting!")
        return 0

    if args.task == "convert":
        if args.out is None:
            print("Output directory is not specified. Use --out.")
            return 2
        from .data.bincache import convert_files

        for path, st in convert_files(cfg.train_files, cfg.weight_files or None, args.out, cfg.vocabulary_size,
                                      cfg.hash_feature_id, cfg.parse_threads):
            print(f"{path}: {st['examples']} examples, {st['nnz']} features"
                  f"{' (+ weights)' if cfg.weight_files else ''}", flush=True)
        print(f"Done converting. Set train_files = {os.path.join(args.out, '*.fmb')} and no weight_files to train "
              "from the caches.")
        return 0

    if args.task in ("import_tf", "export_tf"):
        return _migrate(args, cfg)

    ctx = None
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if dist_info.get("role") == "worker" or world_env > 1:
        dev = None if cfg.device == "auto" else cfg.device
        ctx = fmdist.init_distributed(rank=dist_info.get("rank"), world=dist_info.get("world"),
                                      master_addr=dist_info.get("master_addr"),
                                      master_port=dist_info.get("master_port"), device=dev)
        if args.wait_for_workers is not None and ctx.rank == 0:
            print(f"All {ctx.world} workers joined (wait-for-workers={args.wait_for_workers}).")
    from .trainer import Trainer

    tr = Trainer(cfg, ctx, monitor=args.monitor, trace=args.trace)
    try:
        if args.task == "train":
            tr.train()
        else:
            tr.predict()
    finally:
        tr.close()
        if ctx is not None:
            fmdist.shutdown()
    return 0


def _tf_prefix(path: str) -> str:
    """A TF checkpoint prefix from a directory (via its ``checkpoint`` state file) or a prefix."""
    import re

    if os.path.isdir(path):
        state = os.path.join(path, "checkpoint")
        if not os.path.exists(state):
            raise FileNotFoundError(f"no 'checkpoint' state file in {path}")
        with open(state) as f:
            m = re.search(r'^model_checkpoint_path:\s*"(.*)"', f.read(), re.M)
        if m is None:
            raise ValueError(f"{state} names no model_checkpoint_path")
        p = m.group(1)
        return p if os.path.isabs(p) else os.path.join(path, p)
    return path


def _migrate(args, cfg) -> int:
    from .utils import checkpoint as ckpt

    if cfg.log_dir is None:
        print("Missing log directory.")
        return 1
    if args.task == "export_tf":
        if args.export_path is None:
            print("Export path is not specified. Use --export_path.")
            return 2
        path = ckpt.latest_checkpoint(cfg.log_dir)
        if path is None:
            print(f"No checkpoint found in {cfg.log_dir}.")
            return 1
        prefix = ckpt.export_tf_checkpoint(path, args.export_path, cfg.vocabulary_block_num)
        print(f"TensorFlow checkpoint written to {prefix}")
        return 0
    if args.tf_checkpoint is None:
        print("TF checkpoint is not specified. Use --tf_checkpoint.")
        return 2
    from .trainer import Trainer

    prefix = _tf_prefix(args.tf_checkpoint)
    tr = Trainer(cfg, None)
    step = ckpt.import_tf_checkpoint(tr.model, prefix, cfg.vocabulary_block_num)
    path = ckpt.save_checkpoint(tr.model, cfg.log_dir, step)
    print(f"Imported {prefix} (global_step {step}) into {path}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
