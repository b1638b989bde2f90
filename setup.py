"""Build the native runtime extension in-tree:  python setup.py build_ext --inplace

The extension is plain C++ (compiled by the host compiler) that links the HIP runtime and
PyTorch's c10_hip directly — no hipify step, no CUDA sources.
"""
import os
from setuptools import setup, find_packages
from torch.utils.cpp_extension import BuildExtension, CppExtension

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

ext = CppExtension(
    "tilelang._tl_runtime",
    ["csrc/tl_runtime.cpp"],
    include_dirs=[os.path.join(ROCM, "include")],
    define_macros=[("__HIP_PLATFORM_AMD__", "1"), ("USE_ROCM", "1")],
    library_dirs=[os.path.join(ROCM, "lib")],
    libraries=["amdhip64", "c10_hip"],
    extra_compile_args=["-O2", "-std=c++17", "-Wno-unused-function"],
)

setup(
    name="tilelang-mi355x",
    version="0.1.7+mi355x",
    packages=find_packages(include=["tilelang", "tilelang.*"]),
    package_data={"tilelang": ["include/tl/*.h"]},
    ext_modules=[ext],
    cmdclass={"build_ext": BuildExtension.with_options(use_ninja=False)},
)
