"""Host-side sanitizer run of the C++ libsvm parser.

GPU AddressSanitizer is not available on the MI355X pool; the host parser is
built standalone with ``-fsanitize=address,undefined`` and driven by
tests/native/parser_fuzz.cpp (grammar cases + 20k random mutations, 1 and 4
threads).  Any sanitizer report aborts the driver with a non-zero status.
"""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "fast_tffm_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.timeout(300)
def test_parser_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "parser_fuzz")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-pthread", "-fopenmp", "-I", CSRC,
           os.path.join(ROOT, "tests", "native", "parser_fuzz.cpp"), os.path.join(CSRC, "cpu", "parser.cpp"),
           "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "parser_fuzz: ok" in r.stdout
