"""B2 (reference CMakeLists.txt:50-61): the CMake build stamps the same content hash as
build_native.py, so the hash-checked loader (ops/native.py) accepts a CMake-built module.
Configure only (seconds); the compile is the same hipcc / g++ invocation build_native runs."""

import os
import shutil
import subprocess

import pytest

from fast_tffm_amd import build_native as bn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("cmake") is None or shutil.which("ninja") is None, reason="cmake / ninja missing")
def test_cmake_stamps_build_native_hashes(tmp_path):
    r = subprocess.run(["cmake", "-S", ROOT, "-B", str(tmp_path), "-G", "Ninja"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    ninja = (tmp_path / "build.ninja").read_text()
    assert f'FM_BUILD_HASH=\\"{bn.cpu_hash()}\\"' in ninja
    assert f'FM_BUILD_HASH=\\"{bn.hip_hash()}\\"' in ninja
