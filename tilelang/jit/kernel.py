"""``JITKernel``: a compiled tilelang kernel callable on torch tensors.

Reference: ``tilelang/jit/kernel.py:31-758`` (compile + adapter + profiler +
source export) and the Cython adapter (``jit/adapter/cython``).  Execution goes
through the native runtime ``tilelang._tl_runtime.Kernel`` (C++: argument
validation, dynamic-shape binding, output allocation, ``hipModuleLaunchKernel`` on
the current stream).
"""
from __future__ import annotations

import threading
from pathlib import Path
from typing import List, Optional, Union

from ..engine.lower import lower, CompiledArtifact
from ..ir import dtypes as _dt
from ..ir import stmt as S
from ..ir.buffer import Buffer
from ..ir.expr import BinOp, IntImm, Var, as_int
from ..utils.target import Target, determine_target
from ..contrib import hipcc
from .. import cache as _cache

_OP = {"+": 2, "-": 3, "*": 4, "//": 5, "/": 5, "%": 6, "min": 8, "max": 9}


def _prog(e, symtab) -> List[int]:
    if isinstance(e, int):
        return [0, e]
    if isinstance(e, IntImm):
        return [0, e.value]
    if isinstance(e, Var):
        if e not in symtab:
            raise ValueError(f"grid expression uses {e.name}, which is neither a tensor shape symbol nor an int "
                             f"scalar parameter")
        return [1, symtab[e]]
    if isinstance(e, BinOp) and e.op in _OP:
        return _prog(e.a, symtab) + _prog(e.b, symtab) + [_OP[e.op]]
    from ..ir.expr import Cast
    if isinstance(e, Cast):
        return _prog(e.value, symtab)
    raise ValueError(f"unsupported grid expression {e}")


_SCALAR_TYPES = {}


def _scalar_type_code(dtype) -> int:
    import torch
    from .. import _native
    key = str(dtype)
    if key not in _SCALAR_TYPES:
        _SCALAR_TYPES[key] = _native.runtime().scalar_type_of(torch.empty(0, dtype=_dt.to_torch(dtype)))
    return _SCALAR_TYPES[key]


def _linear_in(e, n):
    """(a, b) with ``e == a * n + b`` proved on the IR: only ``+``, ``-``, ``*`` by a constant and
    casts are walked; ``min``/``max``/``//``/``%`` or anything else is not affine -> None."""
    from ..ir.expr import BinOp, Cast, as_int
    c = as_int(e)
    if c is not None:
        return (0, c)
    if e is n:
        return (1, 0)
    if isinstance(e, Cast):
        return _linear_in(e.value, n)
    if isinstance(e, BinOp) and e.op in ("+", "-"):
        la, lb = _linear_in(e.a, n), _linear_in(e.b, n)
        if la is None or lb is None:
            return None
        sg = 1 if e.op == "+" else -1
        return (la[0] + sg * lb[0], la[1] + sg * lb[1])
    if isinstance(e, BinOp) and e.op == "*":
        ca, cb = as_int(e.a), as_int(e.b)
        if cb is not None:
            la = _linear_in(e.a, n)
            return None if la is None else (la[0] * cb, la[1] * cb)
        if ca is not None:
            lb = _linear_in(e.b, n)
            return None if lb is None else (lb[0] * ca, lb[1] * ca)
    return None


def _affine_of(e, symtab):
    """(symbol id, a, b) when ``e`` is ``a * n + b`` (a > 0) in one shape symbol ``n``, else None.
    Proved structurally (``_linear_in``): sampling a few points accepted ``T.min(n, 64)`` or
    ``n + n // 8`` as ``n``, and the launcher would then size outputs with the wrong formula."""
    from ..ir.expr import free_vars
    fv = [v for v in free_vars(e)]
    if len(fv) != 1 or fv[0] not in symtab:
        return None
    ab = _linear_in(e, fv[0])
    if ab is None or ab[0] <= 0:
        return None
    return (symtab[fv[0]], ab[0], ab[1])


class JITKernel:

    def __init__(self, func: S.PrimFunc = None, out_idx: Union[List[int], int, None] = None, target="auto",
                 target_host=None, execution_backend: str = "native", verbose: bool = False,
                 pass_configs: Optional[dict] = None, compile_flags: Optional[List[str]] = None,
                 from_database: bool = False, artifact: Optional[CompiledArtifact] = None, code=None):
        self.func = func
        self.verbose = verbose
        self.pass_configs = dict(pass_configs or {})
        self.compile_flags = list(compile_flags or [])
        self.execution_backend = execution_backend
        self.target = determine_target(target)
        self._rt = None
        self._lock = threading.Lock()
        self.config = None
        self.latency = None
        self.ref_latency = None
        self._launch = None       # launcher specs restored from the disk cache
        self._residency_ok = set()
        self.from_disk_cache = False
        key = None
        if artifact is None:
            from ..cache import kernel_cache
            key = kernel_cache.kernel_key(func, self.target, out_idx, self.pass_configs, self.compile_flags)
            # the layout dump is a side effect of lowering: never serve such a compile from the cache
            visual = bool(dict(self.pass_configs or {}).get("tl.layout_visualization_enable"))
            hit = None if visual else kernel_cache.load(key)
            if hit is not None:
                is_cpu, kernels, code, self._launch = hit
                tgt = Target("cpu", "host", getattr(self.target, "mesh", None)) if is_cpu and \
                    self.target.kind != "cpu" else self.target
                artifact = CompiledArtifact(func, tgt, kernels, is_cpu)
                self.from_disk_cache = True
                key = None
            else:
                artifact = lower(func, self.target, pass_configs=self.pass_configs)
        self.artifact = artifact
        self.target = artifact.target
        nparams = len(func.params)
        if out_idx is None:
            out_idx = []
        elif isinstance(out_idx, int):
            out_idx = [out_idx]
        self.out_idx = sorted(i % nparams for i in out_idx)
        for i in self.out_idx:
            if not isinstance(func.params[i], Buffer):
                raise ValueError(f"out_idx {i} refers to a scalar parameter")
        self.code = code if code is not None else self._compile()
        if key is not None:
            from ..cache import kernel_cache
            kernel_cache.save(key, self)

    # -- compilation -------------------------------------------------------------------
    def _compile(self):
        """One code object (gfx950) or shared object (cpu) per device kernel of the program."""
        a = self.artifact
        out = []
        hip_flags = self.hip_flags()
        for dk in a.kernels:
            if a.is_cpu:
                out.append(_cache.compile_cpu_cached(dk.source, self.compile_flags, self.verbose))
            else:
                out.append(_cache.compile_hip_cached(dk.source, hip_flags, self.verbose))
        return out

    def hip_flags(self) -> List[str]:
        """hipcc flags of this kernel's gfx950 compile: the user's plus what the pass configs imply."""
        flags = list(self.compile_flags)
        if self.pass_configs.get("tl.gemm_fold_default_guard") is False:
            flags.append("-DTL_GEMM_FOLD_DEFAULT_GUARD=0")
        if self.pass_configs.get("tl.no_nans"):
            # the kernel promises no NaN values: fmaxf on MFMA results then needs no canonicalising
            # v_max_f32 x, x per operand (the softmax row max of the attention kernels that set it)
            flags.append("-fno-honor-nans")
        return flags

    def _param_specs(self, dk, with_outputs: bool):
        symtab = {}
        for p in dk.params:
            if p["kind"] == "dyn":
                symtab[p["var"]] = len(symtab)
        for p in dk.params:
            if p["kind"] == "scalar" and p["var"].dtype.is_int:
                symtab[p["var"]] = len(symtab)
        specs = []
        for i, p in enumerate(dk.params):
            d = dict(kind={"buffer": 0, "scalar": 1, "dyn": 2}.get(p["kind"], 1), name=p["name"], scalar_type=0,
                     nbytes=8, is_float=False, shape=[], strides=[], is_output=False, sym=-1, max_elems=0)
            if p["kind"] == "buffer":
                b: Buffer = p["buffer"]
                if b.name in getattr(dk, "narrow_index", ()):
                    d["max_elems"] = 1 << 31  # compiled with 32-bit offsets: refuse larger tensors
                d["scalar_type"] = _scalar_type_code(b.dtype)
                d["is_output"] = with_outputs and (b.param_index in self.out_idx)
                for s in b.shape:
                    v = as_int(s)
                    if v is not None:
                        d["shape"].append((True, v))
                    elif isinstance(s, Var) and s in symtab:
                        d["shape"].append((False, symtab[s]))
                    else:
                        aff = _affine_of(s, symtab)
                        if aff is None:
                            raise ValueError(f"unsupported dynamic shape expression {s} for {b.name} (an extent "
                                             "must be a * n + b in one symbol n)")
                        d["shape"].append((False, ) + aff)
                if b.strides is not None:
                    for s in b.strides:
                        v = as_int(s)
                        d["strides"].append((True, v) if v is not None else (False, symtab[s]))
            elif p["kind"] == "scalar":
                v = p["var"]
                d["nbytes"] = max(1, v.dtype.bits // 8)
                d["is_float"] = v.dtype.is_float
                d["scalar_type"] = _scalar_type_code(v.dtype)  # host check of the Python value's type
                d["sym"] = symtab.get(v, -1)
            elif p["kind"] == "dyn":
                v = p["var"]
                d["nbytes"] = max(1, v.dtype.bits // 8)
                d["sym"] = symtab[v]
            else:  # extra (runtime-provided) params, e.g. mesh pointers
                d["kind"] = 1
                d["nbytes"] = p.get("nbytes", 8)
                d["is_float"] = False
            specs.append(d)
        grid = [_prog(g, symtab) for g in dk.grid]
        return specs, len(symtab), grid

    @property
    def runtimes(self):
        if self._rt is None:
            with self._lock:
                if self._rt is None:
                    from .. import _native
                    rt = _native.runtime()
                    a = self.artifact
                    rts = []
                    for i, (dk, code) in enumerate(zip(a.kernels, self.code)):
                        specs, nsyms, grid = self._launch[i] if self._launch is not None else \
                            self._param_specs(dk, with_outputs=(i == 0))
                        blob = code.encode() if isinstance(code, str) else code
                        k = rt.Kernel(blob, dk.name, a.is_cpu, specs, nsyms, grid, [int(b) for b in dk.block],
                                      int(dk.lds_bytes), dk.name)
                        if getattr(dk, "cooperative", False) and not a.is_cpu:
                            k.set_cooperative(True)
                        rts.append(k)
                    self._rt = rts
        return self._rt

    @property
    def runtime(self):
        return self.runtimes[0]

    # -- execution -----------------------------------------------------------------------
    def __call__(self, *args, **kwargs):
        if kwargs:
            names = [p.name for i, p in enumerate(self.func.params) if i not in self.out_idx]
            full = list(args)
            for n in names[len(args):]:
                if n in kwargs:
                    full.append(kwargs[n])
            args = tuple(full)
        from ..runtime import errors as _errors
        _errors.poll()  # a bounded device wait of an earlier launch timed out: raise it here
        rts = self.runtimes
        kernels = self.artifact.kernels
        is_cpu = self.artifact.is_cpu
        mesh_ctx = None
        if any(dk.mesh is not None for dk in kernels):
            from ..parallel.mesh import current_mesh, MeshError
            mesh_ctx = current_mesh()
            if mesh_ctx is None:
                raise MeshError(f"{self.artifact.kernel_name} uses T.comm / current_core but no mesh is active: call "
                                f"tilelang.parallel.init_mesh() (one process per GPU) or run it inside "
                                f"VirtualMesh.run()")

        keep = []  # per-launch workspaces stay referenced until every launch is issued
        watch = []  # (error word, label, decoder) read back behind the launches

        def _margs(dk):
            out = mesh_ctx.launch_args(dk.mesh) if dk.mesh is not None else []
            if dk.mesh is not None and not is_cpu:
                watch.append((mesh_ctx.err, f"{dk.name} (mesh rank {mesh_ctx.rank})", mesh_ctx.error_decoder))
            if getattr(dk, "cooperative", False) and not is_cpu:
                import torch
                dev = next((a.device for a in args if isinstance(a, torch.Tensor) and a.is_cuda), None)
                dev = dev if dev is not None else torch.device("cuda", torch.cuda.current_device())
                # barrier state of THIS launch (tl/common.h sync_grid): zeroed on the launch stream
                ws = torch.zeros(4, dtype=torch.int32, device=dev)
                err = _errors.device_word(dev)
                keep.append(ws)
                watch.append((err, dk.name, None))
                out = out + [ws.data_ptr(), err.data_ptr()]
            return out

        if mesh_ctx is not None and not self.artifact.is_cpu:
            key = (id(mesh_ctx), mesh_ctx.ranks_on_device)
            if key not in self._residency_ok:
                for r, dk in zip(rts, kernels):
                    if dk.mesh is not None:
                        mesh_ctx.check_residency(dk.name, int(dk.mesh["nblocks"]), int(r.max_resident_blocks()))
                self._residency_ok.add(key)

        out = rts[0](*args, *_margs(kernels[0]))
        if len(rts) == 1:
            for w, label, dec in watch:
                _errors.record(w, label, dec)
            return out
        # later kernels of the program see the outputs of the first as ordinary arguments
        outs = list(out) if isinstance(out, tuple) else ([out] if out is not None else [])
        full, ai, oi = [], 0, 0
        for i, p in enumerate(self.func.params):
            if i in self.out_idx:
                full.append(outs[oi])
                oi += 1
            else:
                full.append(args[ai])
                ai += 1
        for r, dk in zip(rts[1:], kernels[1:]):
            r(*full, *_margs(dk))
        for w, label, dec in watch:
            _errors.record(w, label, dec)
        return out

    @classmethod
    def from_database(cls, func: S.PrimFunc, out_idx=None, target="auto", pass_configs=None, compile_flags=None,
                      **_):
        """The cached kernel for this program/options, or None when the disk cache has no entry
        (reference ``JITKernel.from_database``, ``tilelang/jit/kernel.py:142-183``)."""
        from ..cache import kernel_cache
        tgt = determine_target(target)
        key = kernel_cache.kernel_key(func, tgt, out_idx, dict(pass_configs or {}), list(compile_flags or []))
        if kernel_cache.load(key) is None:
            return None
        return cls(func, out_idx=out_idx, target=tgt, pass_configs=pass_configs, compile_flags=compile_flags)

    def set_validation(self, enabled: bool):
        for r in self.runtimes:
            r.set_validate(enabled)

    # -- introspection (reference API) -----------------------------------------------------
    def get_kernel_source(self) -> str:
        return self.artifact.kernel_source

    def get_host_source(self) -> str:
        a = self.artifact
        lines = [f"// native launcher: hipModuleLaunchKernel({a.kernel_name}, grid={a.grid}, block={a.block}, "
                 f"lds={a.lds_bytes}B)"]
        for p in a.params:
            lines.append(f"//   {p['kind']:6s} {p['name']} {p.get('dtype', '')}")
        return "\n".join(lines)

    def show_source(self, which: str = "kernel"):
        print(self.get_kernel_source() if which == "kernel" else self.get_host_source())

    def get_assembly(self) -> str:
        if self.artifact.is_cpu:
            return ""
        return hipcc.compile_hip(self.artifact.kernel_source, options=self.hip_flags(), asm=True).decode()

    def export_sources(self, directory: str):
        Path(directory).mkdir(parents=True, exist_ok=True)
        (Path(directory) / "kernel.hip").write_text(self.get_kernel_source())
        (Path(directory) / "host.txt").write_text(self.get_host_source())

    def export_library(self, path: str):
        if self.artifact.is_cpu:
            import shutil
            shutil.copy(self.code[0], path)
        else:
            Path(path).write_bytes(self.code[0])

    def get_profiler(self, tensor_supply_type=None):
        from ..profiler import Profiler
        from ..utils.tensor import TensorSupplyType
        return Profiler(self, tensor_supply_type or TensorSupplyType.Auto)

    @property
    def params(self):
        return self.func.params

    @property
    def kernel_source(self):
        return self.artifact.kernel_source

    def update_tuner_result(self, latency, config, ref_latency=None):
        self.latency, self.config, self.ref_latency = latency, config, ref_latency
        return self

    def __repr__(self):
        return f"JITKernel({self.artifact.kernel_name}, target={self.target})"
