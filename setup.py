"""setuptools entry: ``python setup.py build_ext --inplace`` builds both native
modules in-tree (fast_tffm_amd/_native/) through fast_tffm_amd/build_native.py
(hipcc --offload-arch=gfx950 for the HIP module, g++ -fopenmp for the host
module); ``pip install .`` packages them.  Parity with the reference's
setup.py build (reference setup.py:88-201), without its nvcc monkey-patching:
the HIP module is one explicit hipcc invocation.  CMakeLists.txt is the
equivalent CMake build (reference CMakeLists.txt)."""

import os
import sys

from setuptools import Extension, find_packages, setup
from setuptools.command.build_ext import build_ext

ROOT = os.path.dirname(os.path.abspath(__file__))


class BuildNative(build_ext):
    """Delegates to build_native (hipcc / g++); the Extension entries only name the outputs."""

    def build_extensions(self):
        sys.path.insert(0, ROOT)
        from fast_tffm_amd import build_native

        built = build_native.build_all(force=bool(self.force))
        if not self.inplace:  # copy into the build tree for wheels / installs
            import shutil

            dst = os.path.join(self.build_lib, "fast_tffm_amd", "_native")
            os.makedirs(dst, exist_ok=True)
            for p in built:
                shutil.copy2(p, dst)


setup(
    name="fast_tffm_amd",
    version="0.1.0",
    description="MI355X-native distributed factorization machine trainer (HIP/gfx950 + RCCL)",
    packages=find_packages(include=["fast_tffm_amd", "fast_tffm_amd.*"]),
    package_data={"fast_tffm_amd": ["csrc/*.h", "csrc/cpu/*", "csrc/hip/*", "_native/*.so"]},
    ext_modules=[Extension("fast_tffm_amd._native._fm_cpu", sources=[]),
                 Extension("fast_tffm_amd._native._fm_hip", sources=[])],
    cmdclass={"build_ext": BuildNative},
    python_requires=">=3.10",
    install_requires=["torch", "numpy", "safetensors"],
    entry_points={"console_scripts": ["fast-tffm-amd=fast_tffm_amd.cli:main"]},
)
