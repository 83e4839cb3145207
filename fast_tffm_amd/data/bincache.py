"""Binary CSR caches (``.fmb``): libsvm text parsed once, trained on at memory speed.

The format and the converter are native (``csrc/cpu/bincsr.{h,cpp}``); the native
loader (``csrc/cpu/loader.cpp``, binary mode) reads them with the text path's exact
epoch / shuffle-window / rank-sharding / resume semantics, so for the same seed a
cache yields the batches its text file would.  Rationale: SURVEY.md §7.3 "Input
throughput" -- the reference's per-line FmParser (cc/fm_parser_op.cc:58-109) bounds
file-fed training far below the GPU step rate.

    python run.py convert CONFIG --out DIR       # DIR/<train file name>.fmb per train file
    python -m fast_tffm_amd.data.bincache --vocab V [--hash] [--weights W ...] --out DIR FILE ...
"""

from __future__ import annotations

import argparse
import os
import sys

from ..ops import native

SUFFIX = ".fmb"


def is_bin_file(path: str) -> bool:
    return bool(native.cpu().is_bin_file(path))


def convert(text_path: str, out_path: str, vocab_size: int, hash_feature_id: bool = False,
            weight_path: str | None = None, threads: int = 4, chunk_lines: int = 1 << 20) -> dict:
    """Parse one text file (+ its weight file) into ``out_path``; returns its stats."""
    return dict(native.cpu().convert_to_bin(text_path, weight_path or "", out_path, int(vocab_size),
                                            bool(hash_feature_id), int(threads), int(chunk_lines)))


def convert_files(files: list[str], weight_files: list[str] | None, out_dir: str, vocab_size: int,
                  hash_feature_id: bool = False, threads: int = 4):
    """Convert every file into ``out_dir/<basename>.fmb`` (names must be unique); yields (path, stats)."""
    if weight_files and len(weight_files) != len(files):
        raise ValueError("The numbers of train files and weight files do not match.")
    names = [os.path.basename(f) for f in files]
    if len(set(names)) != len(names):
        raise ValueError("train files must have distinct base names to share one cache directory")
    os.makedirs(out_dir, exist_ok=True)
    for i, f in enumerate(files):
        out = os.path.join(out_dir, os.path.basename(f) + SUFFIX)
        yield out, convert(f, out, vocab_size, hash_feature_id, weight_files[i] if weight_files else None, threads)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="convert libsvm text files to binary CSR caches (.fmb)")
    ap.add_argument("files", nargs="+")
    ap.add_argument("--weights", nargs="*", default=None, help="weight files, one per text file")
    ap.add_argument("--vocab", type=int, required=True, help="vocabulary_size of the model")
    ap.add_argument("--hash", action="store_true", help="hash_feature_id = True")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 4)
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)
    for path, st in convert_files(a.files, a.weights, a.out, a.vocab, a.hash, a.threads):
        print(f"{path}: {st['examples']} examples, {st['nnz']} features", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
