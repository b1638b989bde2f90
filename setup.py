"""Build the native runtime extension in-tree:  python setup.py build_ext --inplace

The extension is plain C++ (compiled by the host compiler) that links the HIP runtime and
PyTorch's c10_hip directly — no hipify step, no CUDA sources.
"""
import os
import pybind11
from setuptools import Extension, setup, find_packages
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

# host-only compiler core (fragment algebra, LDS model, arena planner, hierarchical layouts)
# (plain pybind11, no torch linkage: the compiler runs without loading the torch/HIP runtime)
core = Extension(
    "tilelang._tl_core",
    ["csrc/core/bindings.cc", "csrc/core/fragment.cc", "csrc/core/lds.cc", "csrc/core/hier.cc"],
    include_dirs=[pybind11.get_include()],
    language="c++",
    extra_compile_args=["-O2", "-std=c++17", "-fvisibility=hidden"],
)

setup(
    name="tilelang-mi355x",
    version="0.1.7+mi355x",
    packages=find_packages(include=["tilelang", "tilelang.*"]),
    package_data={"tilelang": ["include/tl/*.h"]},
    ext_modules=[ext, core],
    cmdclass={"build_ext": BuildExtension.with_options(use_ninja=False)},
)
