from .callback import (register_cuda_postproc, register_hip_postproc, register_hip_compile,  # noqa: F401
                       register_hip_postproc_callback, register_hip_compile_callback)
