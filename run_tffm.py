#!/usr/bin/env python3
"""Reference-compatible entry point name (run_tffm.py).

Usage: python run_tffm.py {train,predict,generate} CONFIG [--dist ...] [-t FILE] [-m] [--export_path DIR]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from fast_tffm_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
