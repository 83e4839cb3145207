#!/usr/bin/env python3
"""Write synthetic libsvm sample data in the reference's layout (data/train_{i},
data/weight_{i}, data/test_{i}).

usage: python tools/make_sample_data.py [--out data] [--shape criteo|a1a] [--train 5] [--lines 10000]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fast_tffm_amd.data.synthetic import write_libsvm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", default="data")
ap.add_argument("--shape", default="criteo", choices=["criteo", "a1a"])
ap.add_argument("--train", type=int, default=5)
ap.add_argument("--test", type=int, default=2)
ap.add_argument("--lines", type=int, default=10000)
ap.add_argument("--vocab", type=int, default=1_000_000)
ap.add_argument("--values", action="store_true", help="write id:value tokens")
a = ap.parse_args()
os.makedirs(a.out, exist_ok=True)
for i in range(a.train):
    write_libsvm(os.path.join(a.out, f"train_{i}"), a.lines, shape=a.shape, vocab_size=a.vocab, seed=i,
                 weights_path=os.path.join(a.out, f"weight_{i}"), with_values=a.values)
for i in range(a.test):
    write_libsvm(os.path.join(a.out, f"test_{i}"), a.lines // 2, shape=a.shape, vocab_size=a.vocab, seed=100 + i,
                 with_values=a.values)
print(f"wrote {a.train} train / {a.test} test files ({a.shape}) to {a.out}")
