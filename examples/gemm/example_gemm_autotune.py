"""Carver-driven GEMM autotuning (reference: examples/gemm/example_gemm_autotune.py).

``MatmulTemplate(...).with_arch(CDNA())`` ranks MFMA tilings for MI355X analytically (LDS budget
of 160 KiB, wave64 partitions, 256-CU wave quantisation, the HBM/L2 traffic of each tile); the top
hints become configs for ``AutoTuner``, which compiles them in parallel, checks each against the
PyTorch reference and times them (cold-cache ``do_bench``).  ``--with_roller 0`` tunes a fixed grid.
"""
import argparse
import itertools

import tilelang
import tilelang.language as T
from tilelang.autotuner import AutoTuner
from tilelang.carver.arch import CDNA
from tilelang.carver.template import MatmulTemplate


def ref_program(A, B):
    return A @ B.T


def get_configs(M, N, K, with_roller=True, topk=12):
    if with_roller:
        hints = MatmulTemplate(M=M, N=N, K=K, in_dtype="float16", out_dtype="float16",
                               accum_dtype="float").with_arch(CDNA("hip")).recommend_hints(topk=topk)
        if not hints:
            raise ValueError("the carver returned no MFMA tilings")
        configs = []
        for h in hints:
            c = h.to_config()
            configs.append(dict(block_M=c["block_M"], block_N=c["block_N"], block_K=c.get("block_K", 64),
                                num_stages=c.get("num_stages", 2), thread_num=c["threads"], enable_rasteration=True))
        return configs
    grid = itertools.product([128, 256], [128, 256], [32, 64], [2, 3], [256, 512], [True])
    return [dict(block_M=a, block_N=b, block_K=c, num_stages=d, thread_num=e, enable_rasteration=f)
            for a, b, c, d, e, f in grid]


def kernel(M, N, K, block_M=128, block_N=128, block_K=64, num_stages=2, thread_num=256, enable_rasteration=True,
           dtype="float16", accum_dtype="float"):

    @T.prim_func
    def matmul(A: T.Tensor((M, K), dtype), B: T.Tensor((N, K), dtype), C: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=thread_num) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            B_shared = T.alloc_shared((block_N, block_K), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            T.use_swizzle(panel_size=8, enable=enable_rasteration)
            T.clear(C_local)
            for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=num_stages):
                T.copy(A[by * block_M, k * block_K], A_shared)
                T.copy(B[bx * block_N, k * block_K], B_shared)
                T.gemm(A_shared, B_shared, C_local, transpose_B=True)
            T.copy(C_local, C[by * block_M, bx * block_N])

    return matmul


def autotune(M, N, K, with_roller=True, topk=12, warmup=5, rep=20):
    def factory(**cfg):
        return tilelang.compile(kernel(M, N, K, **cfg), out_idx=[-1])

    tuner = AutoTuner.from_kernel(factory, get_configs(M, N, K, with_roller, topk))
    tuner.set_profile_args(ref_prog=ref_program, rtol=1e-2, atol=1e-2)
    return tuner.run(warmup=warmup, rep=rep)


def main(M=4096, N=4096, K=4096, with_roller=True):
    res = autotune(M, N, K, with_roller)
    print(f"best config: {res.config}")
    print(f"best latency: {res.latency:.4f} ms, {2 * M * N * K / res.latency * 1e-9:.1f} TFLOPS")
    if res.ref_latency:
        print(f"reference (torch/hipBLASLt): {res.ref_latency:.4f} ms")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=4096)
    p.add_argument("--n", type=int, default=4096)
    p.add_argument("--k", type=int, default=4096)
    p.add_argument("--with_roller", type=int, default=1)
    a = p.parse_args()
    main(a.m, a.n, a.k, bool(a.with_roller))
