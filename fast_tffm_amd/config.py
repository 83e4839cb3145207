"""INI configuration, key-for-key compatible with the reference's sample.cfg.

Reference loader: ``Model._get_config`` (tffm/fm_model.py:367-475) with the
Python-2 ``ConfigParser``; every value read is echoed as ``  key = value`` under
a ``Config:`` header; comma lists are stripped, globbed and sorted.

Decisions on reference quirks:
* ``hash_feature_id`` is read by the reference but never passed to the parser
  (fm_model.py:400-401 vs :69-71); here it is wired through, as README.md:50
  promises.
* ``save_steps`` is "optional" but used unconditionally (int(None) crashes the
  reference): here it defaults to 100.
* weight/validation file count checks compare the *expanded* file lists, not
  the pattern counts (fm_model.py:447, :467).
* ``predict_files`` is truly optional (the reference crashes on None, :472-475).
* ``model_file`` is read and kept, unused, like the reference (:405-407).

Extensions (new keys, all optional):
  [General]     seed, device = auto|cpu|cuda,
                global_bias = true|false (learned b0; its gradient is all-reduced over ranks),
                dtype = fp32|bf16|fp8 (fp8: OCP e4m3 + per-row scale, GPU)
  [Train]       optimizer = adagrad|ftrl|sgd, ftrl.l1, ftrl.l2, ftrl.beta,
                ftrl.initial_accumulator, parse_threads, loader = native|python, gpu_parse = true|false,
                device_cache = auto|true|false, stochastic_rounding = true|false,
                shuffle = true|false,
                max_steps, dedup_chunk, log_steps
  [Distributed] mode = auto|local|shard|dp|dp_dense, grad_reduce = sum|mean,
                comm_dtype = auto|fp32|bf16 (row-sharded wire rows; auto = table storage dtype),
                microbatches = 1|2|... (row-sharded step parts overlapping the exchange; default 1),
                prefetch_rows = auto|on|off (exchange the next step's rows early, re-send updated ones),
                overlap_grads = auto|on|off (split backward; first half's gradients sent while the rest runs;
                                auto = on with one microbatch),
                staleness = 0|1 (row-sharded step: 0 = synchronous; 1 = bounded staleness, the reference's
                                asynchronous updates made deterministic: step t reads every row with the
                                gradients of steps <= t-2 applied, step t-1's exchange + apply overlap it)
"""

from __future__ import annotations

import configparser
import glob
import os
from dataclasses import dataclass, field

GENERAL, TRAIN, PREDICT, DISTRIBUTED = "General", "Train", "Predict", "Distributed"


_TABLE_DTYPES = ("fp32", "bf16", "fp8")  # -> torch.float32 / bfloat16 / float8_e4m3fn

class ConfigError(ValueError):
    pass


def _expand(patterns: list[str], base_dir: str | None = None) -> list[str]:
    out: list[str] = []
    for p in patterns:
        hits = glob.glob(p)
        if not hits and base_dir and not os.path.isabs(p):
            hits = glob.glob(os.path.join(base_dir, p))
        out.extend(hits)
    return sorted(out)


@dataclass
class FMRunConfig:
    # [General]
    vocabulary_size: int = 8000000
    vocabulary_block_num: int = 100
    factor_num: int = 10
    hash_feature_id: bool = False
    log_dir: str | None = None
    model_file: str | None = None
    save_summaries_steps: int = 100
    seed: int = 0
    dtype: str = "fp32"
    device: str = "auto"
    # [Train]
    batch_size: int = 50000
    init_value_range: float = 0.01
    factor_lambda: float = 0.0
    bias_lambda: float = 0.0
    num_epochs: int = 10
    learning_rate: float = 0.01
    adagrad_init_accumulator: float = 0.1
    loss_type: str = "mse"
    save_steps: int = 100
    queue_size: int = 10000
    shuffle_threads: int = 1
    train_files: list[str] = field(default_factory=list)
    weight_files: list[str] = field(default_factory=list)
    validation_data_files: list[str] = field(default_factory=list)
    validation_weight_files: list[str] = field(default_factory=list)
    tolerance: float | None = None
    optimizer: str = "adagrad"
    ftrl_l1: float = 0.0
    ftrl_l2: float = 0.0
    ftrl_beta: float = 0.0
    ftrl_initial_accumulator: float = 0.1
    parse_threads: int = 4
    loader: str = "native"      # native (C++ loader thread) | python
    gpu_parse: bool = False     # native loader: tokenize on the GPU (hip/parse.hip)
    device_cache: str = "auto"  # .fmb train files: keep them in HBM, gather batches on the device
                                # (auto: when they take <= 40% of the free device memory)
    stochastic_rounding: bool = True  # bf16 / fp8 tables: stochastically rounded updates
    shuffle: bool = True
    max_steps: int | None = None
    dedup_chunk: int = 32
    global_bias: bool = False
    log_steps: int = 1
    # [Predict]
    predict_files: list[str] = field(default_factory=list)
    # [Distributed]
    mode: str = "auto"
    grad_reduce: str = "sum"
    comm_dtype: str = "auto"
    microbatches: int = 0
    prefetch_rows: str = "auto"
    overlap_grads: str = "auto"
    staleness: int = 0
    config_file: str | None = None

    # ------------------------------------------------------------------
    def fm_config(self):
        """The model/step configuration (models.fm.FMConfig)."""
        import torch

        from .models.fm import FMConfig
        from .ops.kernels import OptConfig

        if self.optimizer == "ftrl":
            opt = OptConfig("ftrl", lr=self.learning_rate, l1=self.ftrl_l1, l2=self.ftrl_l2, beta=self.ftrl_beta,
                            initial_accumulator=self.ftrl_initial_accumulator)
        else:
            opt = OptConfig(self.optimizer, lr=self.learning_rate, initial_accumulator=self.adagrad_init_accumulator)
        return FMConfig(vocabulary_size=self.vocabulary_size, factor_num=self.factor_num, loss_type=self.loss_type,
                        factor_lambda=self.factor_lambda, bias_lambda=self.bias_lambda, batch_size=self.batch_size,
                        init_value_range=self.init_value_range, seed=self.seed,
                        dtype={"fp32": torch.float32, "bf16": torch.bfloat16,
                               "fp8": torch.float8_e4m3fn}[self.dtype], opt=opt, mode=self.mode,
                        grad_reduce=self.grad_reduce, comm_dtype=self.comm_dtype, microbatches=self.microbatches,
                        prefetch_rows=self.prefetch_rows,
                        overlap_grads=self.overlap_grads, staleness=self.staleness,
                        stochastic_rounding=self.stochastic_rounding, dedup_chunk=self.dedup_chunk,
                        global_bias=self.global_bias)


def load_config(config_file: str, *, echo: bool = True, printer=print) -> FMRunConfig:
    if not os.path.exists(config_file):
        raise ConfigError(f"config file not found: {config_file}")
    cp = configparser.ConfigParser(inline_comment_prefixes=(";",), strict=False)
    cp.read(config_file)
    base_dir = os.path.dirname(os.path.abspath(config_file))
    c = FMRunConfig(config_file=config_file)

    def read(section: str, option: str, required: bool = True):
        if not cp.has_option(section, option):
            if required:
                raise ConfigError("%s is undefined." % option)
            return None
        value = cp.get(section, option)
        if echo:
            printer("  {0} = {1}".format(option, value))
        return value

    def read_list(section: str, option: str, required: bool = True):
        v = read(section, option, required)
        if v is None:
            return None
        return [s.strip() for s in v.split(",") if s.strip()]

    def opt(section, option, conv, default):
        v = read(section, option, required=False)
        return default if v is None else conv(v)

    def to_bool(v: str) -> bool:
        return v.strip().lower() == "true"

    if echo:
        printer("Config: ")
    c.vocabulary_size = int(read(GENERAL, "vocabulary_size"))
    c.vocabulary_block_num = int(read(GENERAL, "vocabulary_block_num"))
    c.factor_num = int(read(GENERAL, "factor_num"))
    c.hash_feature_id = to_bool(read(GENERAL, "hash_feature_id"))
    c.log_dir = read(GENERAL, "log_dir", required=False)
    c.model_file = read(GENERAL, "model_file", required=False)
    c.save_summaries_steps = opt(GENERAL, "save_summaries_steps", int, c.save_summaries_steps)
    c.seed = opt(GENERAL, "seed", int, c.seed)
    c.global_bias = opt(GENERAL, "global_bias", to_bool, c.global_bias)
    c.dtype = opt(GENERAL, "dtype", lambda s: s.strip().lower(), c.dtype)
    c.device = opt(GENERAL, "device", lambda s: s.strip().lower(), c.device)

    c.batch_size = int(read(TRAIN, "batch_size"))
    c.init_value_range = float(read(TRAIN, "init_value_range"))
    c.factor_lambda = float(read(TRAIN, "factor_lambda"))
    c.bias_lambda = float(read(TRAIN, "bias_lambda"))
    c.num_epochs = int(read(TRAIN, "epoch_num"))
    c.learning_rate = float(read(TRAIN, "learning_rate"))
    c.adagrad_init_accumulator = float(read(TRAIN, "adagrad.initial_accumulator"))
    c.loss_type = read(TRAIN, "loss_type").strip().lower()
    c.save_steps = opt(TRAIN, "save_steps", int, c.save_steps)
    c.queue_size = opt(TRAIN, "queue_size", int, c.queue_size)
    c.shuffle_threads = opt(TRAIN, "shuffle_threads", int, c.shuffle_threads)
    c.optimizer = opt(TRAIN, "optimizer", lambda s: s.strip().lower(), c.optimizer)
    c.ftrl_l1 = opt(TRAIN, "ftrl.l1", float, c.ftrl_l1)
    c.ftrl_l2 = opt(TRAIN, "ftrl.l2", float, c.ftrl_l2)
    c.ftrl_beta = opt(TRAIN, "ftrl.beta", float, c.ftrl_beta)
    c.ftrl_initial_accumulator = opt(TRAIN, "ftrl.initial_accumulator", float, c.ftrl_initial_accumulator)
    c.parse_threads = opt(TRAIN, "parse_threads", int, c.parse_threads)
    c.loader = opt(TRAIN, "loader", lambda s: s.strip().lower(), c.loader)
    c.gpu_parse = opt(TRAIN, "gpu_parse", lambda s: s.strip().lower() == "true", c.gpu_parse)
    c.device_cache = opt(TRAIN, "device_cache", lambda s: s.strip().lower(), c.device_cache)
    if c.device_cache not in ("auto", "true", "false"):
        raise ConfigError(f"[Train] device_cache must be auto, true or false, got {c.device_cache}")
    c.stochastic_rounding = opt(TRAIN, "stochastic_rounding", lambda s: s.strip().lower() == "true",
                                c.stochastic_rounding)
    if c.loader not in ("native", "python"):
        raise ConfigError(f"[Train] loader must be native or python, got {c.loader}")
    c.shuffle = opt(TRAIN, "shuffle", to_bool, c.shuffle)
    c.max_steps = opt(TRAIN, "max_steps", int, c.max_steps)
    c.dedup_chunk = opt(TRAIN, "dedup_chunk", int, c.dedup_chunk)
    c.log_steps = opt(TRAIN, "log_steps", int, c.log_steps)

    if c.loss_type not in ("logistic", "mse"):
        raise ConfigError("loss_type must be 'logistic' or 'mse', got %r" % c.loss_type)
    if c.optimizer not in ("adagrad", "ftrl", "sgd"):
        raise ConfigError("optimizer must be adagrad|ftrl|sgd, got %r" % c.optimizer)
    if c.dtype not in _TABLE_DTYPES:
        raise ConfigError("dtype must be fp32|bf16|fp8, got %r" % c.dtype)

    c.train_files = _expand(read_list(TRAIN, "train_files"), base_dir)
    wf = read_list(TRAIN, "weight_files", required=False)
    if wf is not None:
        c.weight_files = _expand(wf, base_dir)
        if len(c.train_files) != len(c.weight_files):
            raise ConfigError("The numbers of train files and weight files do not match.")

    vf = read_list(TRAIN, "validation_files", required=False)
    if vf is not None:
        c.validation_data_files = _expand(vf, base_dir)
        c.tolerance = float(read(TRAIN, "tolerance"))
    vwf = read_list(TRAIN, "validation_weight_files", required=False)
    if vwf is not None:
        c.validation_weight_files = _expand(vwf, base_dir)
        if len(c.validation_data_files) != len(c.validation_weight_files):
            raise ConfigError("The numbers of validation data files and validation weight files do not match.")

    pf = read_list(PREDICT, "predict_files", required=False)
    if pf is not None:
        c.predict_files = _expand(pf, base_dir)

    c.mode = opt(DISTRIBUTED, "mode", lambda s: s.strip().lower(), c.mode)
    c.grad_reduce = opt(DISTRIBUTED, "grad_reduce", lambda s: s.strip().lower(), c.grad_reduce)
    c.comm_dtype = opt(DISTRIBUTED, "comm_dtype", lambda s: s.strip().lower(), c.comm_dtype)
    c.microbatches = opt(DISTRIBUTED, "microbatches", int, c.microbatches)
    c.prefetch_rows = opt(DISTRIBUTED, "prefetch_rows", lambda s: s.strip().lower(), c.prefetch_rows)
    c.overlap_grads = opt(DISTRIBUTED, "overlap_grads", lambda s: s.strip().lower(), c.overlap_grads)
    c.staleness = opt(DISTRIBUTED, "staleness", int, c.staleness)
    if c.comm_dtype not in ("auto", "storage", "fp32", "bf16"):
        raise ConfigError(f"[Distributed] comm_dtype must be auto, fp32 or bf16, got {c.comm_dtype}")
    if c.staleness not in (0, 1):
        raise ConfigError(f"[Distributed] staleness must be 0 or 1, got {c.staleness}")
    return c
