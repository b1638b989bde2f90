"""gfx950 HIP C++ emitter (and the CPU C++ emitter used by the plumbing target).

Reference: ``src/target/codegen_hip.cc`` (``CodeGenTileLangHIP``: ``extern "C"
__global__`` with ``__launch_bounds__``, dynamic LDS, MFMA intrinsics) and
``src/target/codegen_cpp.cc`` / ``codegen_c_host.cc`` for CPU.  Unlike the
reference there is no separate host stub: the kernel is launched by the native
runtime (``csrc/tl_runtime.cpp``) through ``hipModuleLaunchKernel`` with a packed
argument array, and CPU kernels are called through a generated ``tl_entry(void**)``.
"""
from __future__ import annotations

import math
import re
from typing import Dict, List

from ..ir import stmt as S
from ..ir import lowered as L
from ..ir import dtypes as _dt
from ..ir.buffer import Buffer
from ..ir.expr import (BinOp, BufferLoad, Call, Cast, FloatImm, IntImm, PrimExpr, Select, StringImm, UnOp, Var,
                       is_nonneg, as_int, free_vars)

_MATH = {
    "exp", "exp2", "exp10", "log", "log2", "log10", "log1p", "expm1", "sqrt", "rsqrt", "rcp", "sin", "cos", "tan",
    "asin", "acos", "atan", "sinh", "cosh", "tanh", "erf", "floor", "ceil", "trunc", "round", "nearbyint", "sigmoid",
    "abs", "pow", "fmod", "atan2", "fma", "isnan", "isinf", "isfinite", "fast_exp", "fast_exp2", "fast_exp10",
    "fast_log", "fast_log2", "fast_log10", "fast_sin", "fast_cos", "fast_tan"
}

_C_KEYWORDS = {"int", "float", "double", "char", "long", "short", "void", "for", "if", "else", "while", "do",
               "return", "break", "continue", "switch", "case", "default", "auto", "const", "static", "signed",
               "unsigned", "struct", "union", "enum", "typedef", "goto", "sizeof", "volatile", "register", "extern",
               "inline", "new", "delete", "class", "template", "this", "half", "bool", "true", "false", "min", "max",
               "abs", "exp", "log", "tid", "lane", "wave", "tl", "smem", "tl_smem"}



# T.atomic_*(memory_order=...) -> clang __ATOMIC_* (same numbering as the reference's ids)
_MEMORY_ORDER_C = {"relaxed": "__ATOMIC_RELAXED", "consume": "__ATOMIC_CONSUME", "acquire": "__ATOMIC_ACQUIRE",
                   "release": "__ATOMIC_RELEASE", "acq_rel": "__ATOMIC_ACQ_REL", "seq_cst": "__ATOMIC_SEQ_CST"}

class CodeGenError(Exception):
    pass


class KernelSource:
    """Result of code generation."""

    def __init__(self):
        self.source = ""
        self.kernel_name = ""
        self.params: List[dict] = []      # runtime argument spec
        self.grid: List[PrimExpr] = []
        self.block: List[int] = []
        self.lds_bytes = 0
        self.is_cpu = False
        self.dyn_vars: List[Var] = []


class CodeGen:

    def __init__(self, func: S.PrimFunc, kernel: S.KernelStmt, target, lds_offsets: Dict[Buffer, int],
                 lds_total: int, pass_cfg=None):
        self.func = func
        self.kernel = kernel
        self.target = target
        self.is_cpu = kernel.is_cpu or getattr(target, "kind", "hip") == "cpu"
        self.lds_offsets = lds_offsets
        self.lds_total = lds_total
        self.lines: List[str] = []
        self.ind = 1
        self.names: Dict[int, str] = {}
        self.used_names = set()
        self.pass_cfg = pass_cfg or {}
        self.fast_math = bool(self.pass_cfg.get("tl.enable_fast_math", False))
        self.pack_f32 = bool(self.pass_cfg.get("tl.pack_f32", False))
        self.param_ptr: Dict[Buffer, str] = {}

    # -- names ------------------------------------------------------------------------
    def name_of(self, obj, base: str) -> str:
        k = id(obj)
        if k in self.names:
            return self.names[k]
        base = re.sub(r"[^A-Za-z0-9_]", "_", base) or "v"
        if base[0].isdigit():
            base = "v" + base
        if base in _C_KEYWORDS:
            base = base + "_"
        name = base
        i = 1
        while name in self.used_names:
            name = f"{base}_{i}"
            i += 1
        self.used_names.add(name)
        self.names[k] = name
        self._keep = getattr(self, "_keep", [])
        self._keep.append(obj)
        return name

    def buf_name(self, b: Buffer) -> str:
        base = getattr(b, "reinterpret", None)
        if base is not None:  # dtype view of a tensor: the same address as another element type
            return f"(({self.ctype(b.dtype)}*)({self.buf_name(base)}))"
        return self.name_of(b, b.name)

    # -- expressions ---------------------------------------------------------------------
    def ctype(self, dt) -> str:
        return _dt.cpu_type(dt) if self.is_cpu else _dt.hip_type(dt)

    def e(self, x) -> str:
        if isinstance(x, bool):
            return "true" if x else "false"
        if isinstance(x, int):
            return str(x)
        if isinstance(x, str):
            return x
        if isinstance(x, IntImm):
            dt = x.dtype
            if dt.is_bool:
                return "true" if x.value else "false"
            if dt.name == "int64":
                return f"{x.value}LL"
            if dt.name in ("uint32", ):
                return f"{x.value}u"
            if dt.name == "uint64":
                return f"{x.value}ULL"
            if dt.name == "int32":
                return str(x.value) if x.value >= -2**31 + 1 else f"({x.value + 1} - 1)"
            return f"(({self.ctype(dt)}){x.value})"
        if isinstance(x, FloatImm):
            return self.float_lit(x.value, x.dtype)
        if isinstance(x, StringImm):
            return '"' + x.value.replace('"', '\\"') + '"'
        if isinstance(x, Var):
            return self.name_of(x, x.name)
        if isinstance(x, L.BufferPtr):
            return f"(&{self.buf_ref(x.buffer)}[{self.e(x.offset)}])"
        if isinstance(x, BinOp):
            return self.binop(x)
        if isinstance(x, UnOp):
            return f"({x.op}{self.e(x.a)})"
        if isinstance(x, Cast):
            return self.cast(x.value, x.dtype)
        if isinstance(x, Select):
            return f"({self.e(x.cond)} ? {self.e(x.t)} : {self.e(x.f)})"
        if isinstance(x, BufferLoad):
            return f"{self.buf_ref(x.buffer)}[{self.e(x.indices[0])}]"
        if isinstance(x, Call):
            return self.call(x)
        raise CodeGenError(f"cannot emit expression {type(x).__name__}: {x}")

    def float_lit(self, v: float, dt) -> str:
        if math.isinf(v):
            s = ("-" if v < 0 else "") + ("__builtin_huge_valf()" if dt.bits <= 32 else "__builtin_huge_val()")
        elif math.isnan(v):
            s = "__builtin_nanf(\"\")"
        else:
            s = repr(float(v))
            if "e" not in s and "." not in s:
                s += ".0"
            if dt.bits <= 32:
                s += "f"
        if dt.name in ("float32", "float64"):
            return s if not s.startswith("-") else f"({s})"
        return self.cast_str(s, _dt.float32, dt)

    def cast_str(self, s: str, src, dst) -> str:
        if dst.is_fp8 and not self.is_cpu:
            return f"{self.ctype(dst)}((float)({s}))"
        if src.is_fp8 and not self.is_cpu:
            return f"(({self.ctype(dst)})(float)({s}))"
        if self.is_cpu and (dst.name in ("float16", "bfloat16") or src.name in ("float16", "bfloat16")):
            if dst.name in ("float16", "bfloat16"):
                return f"{self.ctype(dst)}((float)({s}))"
            return f"(({self.ctype(dst)})(float)({s}))"
        if dst.is_bool:
            return f"(bool)({s})"
        return f"(({self.ctype(dst)})({s}))"

    def cast(self, v, dt) -> str:
        return self.cast_str(self.e(v), v.dtype, dt)

    def binop(self, x: BinOp) -> str:
        a, b = self.e(x.a), self.e(x.b)
        op = x.op
        if op in ("min", "max"):
            if x.dtype.is_float and x.dtype.bits == 32:
                return f"__builtin_f{op}f({a}, {b})"
            return f"tl::{op}_({a}, {b})"
        if op == "//":
            if x.dtype.is_float:
                return f"floorf({a} / {b})" if not self.is_cpu else f"std::floor({a} / {b})"
            if is_nonneg(x.a) and is_nonneg(x.b):
                return f"({a} / {b})"
            return f"tl::floordiv({a}, {b})"
        if op == "%":
            if x.dtype.is_float:
                return f"fmodf({a}, {b})"
            if is_nonneg(x.a) and is_nonneg(x.b):
                return f"({a} % {b})"
            return f"tl::floormod({a}, {b})"
        if op in ("&&", "||"):
            return f"({a} {op} {b})"
        if op == "/" and self.fast_math and not self.is_cpu and x.dtype.is_float and x.dtype.bits == 32:
            # fast math: a * v_rcp_f32(b) (1 ulp) instead of the IEEE division sequence
            # (v_div_scale / v_div_fmas / v_div_fixup, ~10 instructions) -- nvcc -use_fast_math's
            # __fdividef; e.g. the SwiGLU x / (1 + exp(-x)) epilogue of the MoE up projection
            return f"({a} * __builtin_amdgcn_rcpf({b}))"
        return f"({a} {op} {b})"

    def _nt(self, buf) -> bool:
        """Streamed-once global buffer (``T.copy(..., eviction_policy="evict_first")``): non-temporal
        vector accesses (``global_load/store ... nt``) on the GPU."""
        return not self.is_cpu and buf.scope == "global" and getattr(buf, "nontemporal", False)

    def call(self, x: Call) -> str:
        op = x.op
        args = x.args
        if op in _MATH:
            if self.fast_math and op in ("exp", "log", "exp2", "log2", "sin", "cos") and \
                    x.dtype.name == "float32":
                op = "fast_" + op
            return f"tl::{op}({', '.join(self.e(a) for a in args)})"
        if op == "extern":
            name = args[0].value if isinstance(args[0], StringImm) else args[0]
            return f"{name}({', '.join(self.e(a) for a in args[1:])})"
        if op == "tl.lane_id":
            return "tl::lane_id()" if not self.is_cpu else "0"
        if op == "tl.wave_id":
            return "tl::wave_id()" if not self.is_cpu else "0"
        if op in ("tl.shfl_xor", "tl.shfl_down", "tl.shfl_up", "tl.shfl") and not self.is_cpu:
            fn = op.split(".")[1]
            return f"tl::{fn}({', '.join(self.e(a) for a in args)})"
        if op.startswith("tl.wave_reduce_") or op in ("tl.shfl_xor", "tl.shfl_down", "tl.shfl_up", "tl.shfl"):
            if self.is_cpu:
                # the CPU target runs one thread per block: there is no wave to reduce over
                raise CodeGenError(f"T.{op[3:]}: wave-level reductions / shuffles need the 64 lanes of a "
                                   "gfx950 wave; the CPU target (one thread per block) cannot emulate them")
        if op.startswith("tl.wave_reduce_"):
            return f"tl::{op[3:]}({self.e(args[0])})"
        if op.startswith("tl.atomic_"):
            kind = op[len("tl.atomic_"):]
            mo = x.attrs.get("memory_order")
            targ = f"<{_MEMORY_ORDER_C[mo]}>" if mo else ""
            if kind in ("add", "max", "min", "addx2", "addx4", "store"):
                rest = ", ".join(self.e(a) for a in args[1:])
                return f"tl::atomic_{kind}{targ}(&{self.e(args[0])}, {rest})"
            if kind == "load":
                return f"tl::atomic_load{targ}(&{self.e(args[0])})"
        if op == "tl.clock":
            return "clock64()" if not self.is_cpu else "0"
        if op == "tl.ballot":
            return f"__ballot({self.e(args[0])})"
        if op == "tl.dp4a":
            return f"__builtin_amdgcn_sdot4({self.e(args[0])}, {self.e(args[1])}, {self.e(args[2])}, false)"
        if op == "tl.reinterpret":
            return f"__builtin_bit_cast({self.ctype(x.dtype)}, {self.e(args[0])})"
        if op == "tl.pack_b16":
            return (f"((uint32_t)__builtin_bit_cast(uint16_t, {self.e(args[0])}) | "
                    f"((uint32_t)__builtin_bit_cast(uint16_t, {self.e(args[1])}) << 16))")
        if op == "tl.address_of":
            return f"(&{self.e(args[0])})"
        if op == "tl.mesh_rank":
            v = self.kernel.attrs.get("mesh_rank_var")
            if v is None:
                raise CodeGenError("T.comm.current_core() used in a kernel without mesh parameters")
            return self.e(v)
        if op == "tl.sync_threads":
            return "tl::sync_threads()" if self.is_cpu else "__syncthreads()"
        if op == "tl.fence":
            return "tl::fence_agent()"
        if op == "tl.sync_warp":
            return "tl::sync_warp()"
        if op == "tl.sync_grid":
            if self.is_cpu:
                return "tl::sync_grid()"
            ex = {x["name"]: x for x in self.kernel.attrs.get("extra_params", [])}
            if "tl_gsync_ws" not in ex:
                raise CodeGenError("T.sync_grid in a kernel without its grid-barrier workspace parameters")
            ws = self.name_of(ex["tl_gsync_ws"]["var"], "tl_gsync_ws")
            err = self.name_of(ex["tl_dev_err"]["var"], "tl_dev_err")
            return f"tl::sync_grid({ws}, {err})"
        if op == "tl.unswitch":
            c = self.e(args[0])
            if not self.is_cpu and not self._uniform_cond(args[0]):
                raise CodeGenError(f"T.Pipelined(alt_cond={args[0]}): the condition must be the same for every lane "
                                   "of a wave (block indices, scalar parameters, the wave index or a thread "
                                   "expression constant over each wave); it becomes one scalar branch")
            return f"({c})" if self.is_cpu else f"__builtin_amdgcn_readfirstlane((int)({c}))"
        if op == "tl.setprio":
            return "(void)0" if self.is_cpu else f"__builtin_amdgcn_s_setprio({int(args[0].value)})"
        raise CodeGenError(f"unknown intrinsic {op}")

    def buf_ref(self, b: Buffer) -> str:
        return self.buf_name(b)

    # -- statements -----------------------------------------------------------------------
    def w(self, line: str):
        self.lines.append("  " * self.ind + line)

    def s(self, st):
        if st is None:
            return
        if isinstance(st, S.SeqStmt):
            scoped = getattr(st, "scoped", False)
            if scoped:
                self.w("{")
                self.ind += 1
            stmts = st.stmts
            i = 0
            while i < len(stmts):
                if i + 1 < len(stmts) and self.pack_f32 and not self.is_cpu and \
                        self._emit_pk_pair(stmts[i], stmts[i + 1]):
                    i += 2
                    continue
                self.s(stmts[i])
                i += 1
            if scoped:
                self.ind -= 1
                self.w("}")
        elif isinstance(st, S.ForStmt):
            v = self.e(st.var)
            mn, ext = st.min, st.extent
            end = mn + ext
            if st.annotations.get("unroll_factor"):
                self.w(f"#pragma unroll {int(st.annotations['unroll_factor'])}")
            elif st.kind == "unroll" or (as_int(ext) is not None and as_int(ext) <= 8 and st.kind != "serial"):
                self.w("#pragma unroll")
            step = as_int(st.annotations.get("step", 1)) or 1
            inc = f"++{v}" if step == 1 else f"{v} += {step}"
            self.w(f"for (int {v} = {self.e(mn)}; {v} < {self.e(end)}; {inc}) {{")
            self.ind += 1
            self.s(st.body)
            self.ind -= 1
            self.w("}")
        elif isinstance(st, S.WhileStmt):
            self.w(f"while ({self.e(st.cond)}) {{")
            self.ind += 1
            self.s(st.body)
            self.ind -= 1
            self.w("}")
        elif isinstance(st, S.IfStmt):
            if not self.is_cpu and self._wave_uniform(st.cond):
                # a condition on the thread index that is constant within every wave (e.g. wave
                # >= 4 written as tid >= 256): evaluated per lane it is a VGPR compare and an
                # exec-mask branch, so s_setprio / other scalar instructions inside run in EVERY
                # wave (guide T5); readfirstlane makes it a scalar branch
                self.w(f"if (__builtin_amdgcn_readfirstlane((int)({self.e(st.cond)}))) {{")
            else:
                self.w(f"if ({self.e(st.cond)}) {{")
            self.ind += 1
            self.s(st.then_body)
            self.ind -= 1
            if st.else_body is not None:
                self.w("} else {")
                self.ind += 1
                self.s(st.else_body)
                self.ind -= 1
            self.w("}")
        elif isinstance(st, S.StoreStmt):
            b = st.buffer
            self.w(f"{self.buf_ref(b)}[{self.e(st.indices[0])}] = {self.e(st.value)};")
        elif isinstance(st, S.LetStmt):
            self.w(f"const {self.ctype(st.var.dtype)} {self.e(st.var)} = {self.e(st.value)};")
        elif isinstance(st, S.EvaluateStmt):
            self.w(f"{self.e(st.expr)};")
        elif isinstance(st, S.AllocStmt):
            self.alloc(st.buffer)
        elif isinstance(st, S.BreakStmt):
            self.w("break;")
        elif isinstance(st, S.ContinueStmt):
            self.w("continue;")
        elif isinstance(st, S.AssertStmt):
            if not self.is_cpu:
                self.w(f'tl::device_assert({self.e(st.cond)}, "{st.msg}");')
            else:
                self.w(f'if (!({self.e(st.cond)})) {{ return; }}')
        elif isinstance(st, S.AttrStmt):
            self.s(st.body)
        elif isinstance(st, S.RawStmt):
            for ln in st.code.splitlines():
                self.w(ln)
        elif isinstance(st, L.CallStmt):
            t = f"<{', '.join(st.targs)}>" if st.targs else ""
            self.w(f"{st.name}{t}({', '.join(self.e(a) for a in st.args)});")
        elif isinstance(st, L.VecStoreStmt):
            b = st.buffer
            n = len(st.values)
            ct = self.ctype(b.dtype)
            vals = ", ".join(self.e(v) for v in st.values)
            dst = f"&{self.buf_ref(b)}[{self.e(st.index)}]"
            fn = "store_vec_nt" if self._nt(b) else "store_vec"
            self.w(f"{{ {ct} _v[{n}] = {{{vals}}}; tl::{fn}<{ct}, {n}>({dst}, _v); }}")
        elif isinstance(st, L.VecLoadStmt):
            ct = self.ctype(st.src.dtype)
            dst = f"*reinterpret_cast<{ct}(*)[{st.n}]>(&{self.buf_ref(st.dst)}[{st.dst_index}])"
            fn = "load_vec_nt" if self._nt(st.src) else "load_vec"
            self.w(f"tl::{fn}<{ct}, {st.n}>({dst}, &{self.buf_ref(st.src)}[{self.e(st.src_index)}]);")
        elif isinstance(st, L.CopyBytesStmt):
            self.w(f"tl::copy_bytes<{st.nbytes}>(&{self.buf_ref(st.dst)}[{self.e(st.dst_index)}], "
                   f"&{self.buf_ref(st.src)}[{self.e(st.src_index)}]);")
        elif isinstance(st, L.CommentStmt):
            self.w(f"// {st.text}")
        elif isinstance(st, L.PtrDeclStmt):
            ct = self.ctype(st.buffer.dtype)
            self.w(f"{ct}* {self.buf_name(st.buffer)} = reinterpret_cast<{ct}*>({self.e(st.ptr)});")
        elif isinstance(st, L.ObjDeclStmt):
            self.w(f"{st.ctype} {self.e(st.var)};")
        elif isinstance(st, L.AutoLetStmt):
            self.w(f"const auto {self.e(st.var)} = {self.e(st.value)};")
        elif isinstance(st, S.KernelStmt):
            raise CodeGenError("nested kernel")
        elif isinstance(st, S.TileOpStmt):
            raise CodeGenError(f"unlowered tile op {st.op.kind}")
        else:
            raise CodeGenError(f"cannot emit {type(st).__name__}")

    # -- packed fp32 pairs ----------------------------------------------------------------------
    def _emit_pk_pair(self, a, b) -> bool:
        """``x[2m] = f(.., y[2m], ..); x[2m+1] = f(.., y[2m+1], ..)`` on fp32 registers (unrolled
        fragment loops) as ONE ``tl::floatx2`` expression: mul / add / sub (and the fma the
        compiler contracts them into) issue as ``v_pk_mul_f32`` / ``v_pk_add_f32`` /
        ``v_pk_fma_f32``, two lanes' worth per VALU slot.  Only + - * of same-index register
        pairs, thread-invariant scalars and constants; anything else keeps the scalar form.
        Opt-in (pass config ``tl.pack_f32``): beside MFMAs a packed f32 op costs MORE than the two
        scalar ones it replaces (MI355X_MICROARCH 'price of one filler': +22-26 cycles per gap), so
        it pays only in VALU-bound code with no matrix work to hide under (measured neutral on the
        attention forward, profiles/r4/fa_v4.log)."""
        if not (isinstance(a, S.StoreStmt) and isinstance(b, S.StoreStmt) and a.buffer is b.buffer):
            return False
        buf = a.buffer
        if buf.scope != "local" or str(buf.dtype) not in ("float32", "float") or len(a.indices) != 1:
            return False
        ia, ib = as_int(a.indices[0]), as_int(b.indices[0])
        if ia is None or ib != ia + 1 or ia % 2:
            return False
        vexpr = self._pk_expr(a.value, b.value, buf)
        if vexpr is None or not vexpr[1]:
            return False
        ref = self.buf_ref(buf)
        self.w(f"{{ const tl::floatx2 _pk = {vexpr[0]}; {ref}[{ia}] = _pk.x; {ref}[{ia + 1}] = _pk.y; }}")
        return True

    def _pk_expr(self, x, y, dst):
        """(C expression, is_vector) of the element pair (x, y), or None.  ``dst``: the stored
        buffer (a splatted scalar must not read it: the second store would see the first's value)."""
        if isinstance(x, BufferLoad) and isinstance(y, BufferLoad) and x.buffer is y.buffer and \
                x.buffer.scope == "local" and str(x.buffer.dtype) in ("float32", "float") and len(x.indices) == 1:
            i0, i1 = as_int(x.indices[0]), as_int(y.indices[0])
            if i0 is not None and i1 == i0 + 1 and i0 % 2 == 0:
                r = self.buf_ref(x.buffer)
                return f"tl::floatx2{{{r}[{i0}], {r}[{i1}]}}", True
        if isinstance(x, BinOp) and isinstance(y, BinOp) and x.op == y.op and x.op in ("+", "-", "*") and \
                str(x.dtype) in ("float32", "float"):
            l, r = self._pk_expr(x.a, y.a, dst), self._pk_expr(x.b, y.b, dst)
            if l is None or r is None:
                return None
            return f"({l[0]} {x.op} {r[0]})", l[1] or r[1]
        # the same scalar on both sides (a constant, or a per-row value both elements share)
        if str(getattr(x, "dtype", "")) in ("float32", "float") and not _has_local_call(x) and not _reads(x, dst):
            ex, ey = self.e(x), self.e(y)
            if ex == ey:
                return f"(float)({ex})", False
        return None

    def alloc(self, b: Buffer):
        ct = self.ctype(b.dtype)
        name = self.buf_name(b)
        if b.scope == "shared":
            if self.is_cpu:
                self.w(f"static thread_local {ct} {name}[{int(b.shape[0])}];")
                return
            off = self.lds_offsets[b]
            self.w(f"{ct}* {name} = reinterpret_cast<{ct}*>(tl_smem + {off});")
        elif b.scope in ("local", "var", "fragment"):
            n = as_int(b.numel())
            if n is None:
                raise CodeGenError(f"local buffer {b.name} needs a static size")
            init = ""
            if b.init_value is not None and False:
                init = ""
            self.w(f"{ct} {name}[{n}];")
        else:
            raise CodeGenError(f"cannot allocate {b.scope} buffer {b.name} inside a kernel")

    # -- kernel ------------------------------------------------------------------------------
    def generate(self, name: str) -> KernelSource:
        ks = KernelSource()
        ks.is_cpu = self.is_cpu
        k = self.kernel
        kname = self.name_of(k, name)
        ks.kernel_name = kname
        params = []
        sig = []
        # parameters: buffers and scalars of the PrimFunc, then dynamic shape symbols
        flat = k.attrs.get("flat", {})
        dyn_vars = []
        seen = set()
        for p in self.func.params:
            if isinstance(p, Buffer):
                for s in list(p.shape) + list(p.strides or []):
                    if isinstance(s, PrimExpr):
                        for v in free_vars(s):
                            if id(v) not in seen and not any(v is q for q in self.func.params):
                                seen.add(id(v))
                                dyn_vars.append(v)
        for p in self.func.params:
            if isinstance(p, Buffer):
                fb = flat.get(p)
                target_buf = fb if fb is not None else p
                pname = self.name_of(target_buf, p.name)
                if fb is not None:
                    self.names[id(p)] = pname
                ct = self.ctype(p.dtype)
                sig.append(f"{ct}* __restrict__ {pname}")
                params.append(dict(kind="buffer", name=p.name, dtype=p.dtype.name, shape=list(p.shape),
                                   strides=p.strides, buffer=p))
            else:
                sig.append(f"{self.ctype(p.dtype)} {self.name_of(p, p.name)}")
                params.append(dict(kind="scalar", name=p.name, dtype=p.dtype.name, var=p))
        for v in dyn_vars:
            sig.append(f"{self.ctype(v.dtype)} {self.name_of(v, v.name)}")
            params.append(dict(kind="dyn", name=v.name, dtype=v.dtype.name, var=v))
        for extra in k.attrs.get("extra_params", []):
            sig.append(f"{extra['ctype']} {self.name_of(extra['var'], extra['name'])}")
            params.append(extra)
        ks.params = params
        ks.dyn_vars = dyn_vars
        ks.grid = list(k.grid)
        ks.block = list(k.threads)
        ks.lds_bytes = self.lds_total
        self.ind = 1
        body_lines_start = len(self.lines)
        self.preamble(k)
        self.s(k.body)
        body = self.lines[body_lines_start:]
        hdr = []
        if self.is_cpu:
            hdr.append('#include "tl/cpu.h"')
        else:
            hdr.append('#include "tl/tl.h"')
        for src in self.func.attrs.get("import_source", []):
            hdr.append(src)
        if k.prelude:
            hdr.append(k.prelude)
        nthreads = k.num_threads
        out = hdr + [""]
        if self.is_cpu and any("tl::sync_grid()" in ln for ln in body):
            # grid-wide barrier on the CPU target: every block is a host thread (their shared
            # tiles are thread_local) meeting at tl::sync_grid(); block ids unpacked x-fastest
            out.append(f'extern "C" void {kname}({", ".join(sig)}) {{')
            gs = [self.e(g) for g in k.grid]
            total = " * ".join(f"({g})" for g in gs) or "1"
            out.append(f"  const int tl_nblocks = {total};")
            out.append("  tl::GridBarrier tl_gbar(tl_nblocks);")
            out.append("  std::vector<std::thread> tl_threads;")
            out.append("  for (int tl_b = 0; tl_b < tl_nblocks; ++tl_b) {")
            out.append("    tl_threads.emplace_back([&, tl_b]() {")
            out.append("      tl::cur_grid_barrier() = &tl_gbar;")
            stride = "1"
            for v, g in zip(k.block_vars, gs):
                vn = self.name_of(v, v.name)
                out.append(f"      const int {vn} = (tl_b / ({stride})) % ({g});")
                stride = f"({stride}) * ({g})"
            out += ["    " + ln for ln in body]
            out.append("    });")
            out.append("  }")
            out.append("  for (auto& t : tl_threads) t.join();")
            out.append("}")
            unpack = []
            for i, p in enumerate(params):
                ty = sig[i].rsplit(" ", 1)[0].replace("__restrict__", "").strip()
                unpack.append(f"*reinterpret_cast<{ty}*>(args[{i}])")
            out.append(f'extern "C" void tl_entry(void** args) {{ {kname}({", ".join(unpack)}); }}')
        elif self.is_cpu:
            out.append(f'extern "C" void {kname}({", ".join(sig)}) {{')
            # grid loops
            depth = 0
            for i, (v, g) in enumerate(zip(k.block_vars, k.grid)):
                vn = self.name_of(v, v.name)
                out.append("  " * (1 + depth) + f"for (int {vn} = 0; {vn} < {self.e(g)}; ++{vn}) {{")
                depth += 1
            out += ["  " * depth + ln for ln in body]
            for _ in range(depth):
                depth -= 1
                out.append("  " * (1 + depth) + "}")
            out.append("}")
            # generic entry point
            unpack = []
            for i, p in enumerate(params):
                decl = sig[i]
                ty = decl.rsplit(" ", 1)[0].replace("__restrict__", "").strip()
                unpack.append(f"*reinterpret_cast<{ty}*>(args[{i}])")
            out.append(f'extern "C" void tl_entry(void** args) {{ {kname}({", ".join(unpack)}); }}')
        else:
            wpe = max(1, min(8, 2048 // max(nthreads, 64) // 4 if nthreads else 1))
            lb = f"__launch_bounds__({nthreads})"
            if self.pass_cfg.get("tl.min_waves_per_eu"):
                lb = f"__launch_bounds__({nthreads}, {int(self.pass_cfg['tl.min_waves_per_eu'])})"
            out.append(f'extern "C" __global__ void {lb} {kname}({", ".join(sig)}) {{')
            if self.lds_total:
                out.append(f"  __shared__ __attribute__((aligned(1024))) char tl_smem[{self.lds_total}];")
            out += body
            out.append("}")
        ks.source = "\n".join(out) + "\n"
        return ks

    def _uniform_cond(self, cond) -> bool:
        """True if ``cond`` provably takes one value per wave: it depends only on block indices,
        scalar kernel parameters and the wave index, plus thread indices in a wave-constant way
        (checked by evaluation).  Loop variables and let-bound values are rejected: a register
        value need not be uniform."""
        from ..ir.expr import free_vars, substitute, IntImm
        k = self.kernel
        uniform = set(map(id, k.block_vars))
        uniform |= {id(p) for p in getattr(self.func, "params", []) if isinstance(p, Var)}
        if k.attrs.get("wave") is not None:
            uniform.add(id(k.attrs["wave"]))
        fv = free_vars(cond)
        rest = [v for v in fv if id(v) not in uniform]
        if not rest:
            return True
        sub = substitute(cond, {v: IntImm(0) for v in fv if id(v) in uniform})
        return self._wave_uniform(sub)

    def _wave_uniform(self, cond) -> bool:
        """True if ``cond`` depends on thread indices only and takes one value per wave64 (checked
        by evaluation over the workgroup's threads)."""
        from ..ir.expr import EvalError, evaluate, free_vars
        k = self.kernel
        tvars = list(k.thread_vars or [])
        tid = k.attrs.get("tid")
        wave = k.attrs.get("wave")
        lane = k.attrs.get("lane")
        fv = free_vars(cond)
        if not fv:
            return False
        dims = [int(t) for t in (k.threads or [1])]
        n = 1
        for d in dims:
            n *= d
        if n % 64 or n > 1024:
            return False

        def env_of(t):
            env = {}
            rem = t
            for v, d in zip(tvars, dims):
                env[v] = rem % d
                rem //= d
            if tid is not None:
                env[tid] = t
            if wave is not None:
                env[wave] = t // 64
            if lane is not None:
                env[lane] = t % 64
            return env

        known = set(map(id, tvars)) | {id(x) for x in (tid, wave, lane) if x is not None}
        if any(id(v) not in known for v in fv):
            return False
        if all(v is wave for v in fv):
            return False  # already scalar (readfirstlane'd wave index)
        try:
            for w0 in range(0, n, 64):
                first = bool(evaluate(cond, env_of(w0)))
                if any(bool(evaluate(cond, env_of(t))) != first for t in range(w0 + 1, w0 + 64)):
                    return False
        except EvalError:
            return False
        return True

    def preamble(self, k: S.KernelStmt):
        tid = k.attrs.get("tid")
        if self.is_cpu:
            if tid is not None:
                self.w(f"const int {self.e(tid)} = 0;")
            for v in k.thread_vars:
                self.w(f"const int {self.e(v)} = 0;")
            if k.attrs.get("lane") is not None:
                self.w(f"const int {self.e(k.attrs['lane'])} = 0;")
            if k.attrs.get("wave") is not None:
                self.w(f"const int {self.e(k.attrs['wave'])} = 0;")
            return
        dims = ["x", "y", "z"]
        for v, d in zip(k.thread_vars, dims):
            self.w(f"const int {self.e(v)} = threadIdx.{d};")
        if tid is not None:
            if len(k.threads) == 1:
                self.w(f"const int {self.e(tid)} = threadIdx.x;")
            else:
                t = "threadIdx.x"
                mul = k.threads[0]
                for i in range(1, len(k.threads)):
                    t += f" + threadIdx.{dims[i]} * {mul}"
                    mul *= k.threads[i]
                self.w(f"const int {self.e(tid)} = {t};")
        if k.attrs.get("lane") is not None:
            self.w(f"const int {self.e(k.attrs['lane'])} = {self.e(tid)} & 63;")
        if k.attrs.get("wave") is not None:
            self.w(f"const int {self.e(k.attrs['wave'])} = __builtin_amdgcn_readfirstlane({self.e(tid)} >> 6);")
        sw = self.func.attrs.get("use_swizzle")
        if sw and len(k.block_vars) >= 2:
            panel = int(sw.get("panel_size", 8))
            order = sw.get("order", "row")
            bxn, byn = self.e(k.block_vars[0]), self.e(k.block_vars[1])
            self.w("int tl_bid = blockIdx.x + blockIdx.y * gridDim.x;")
            self.w("tl_bid = tl::xcd_remap(tl_bid, gridDim.x * gridDim.y);")
            self.w(f"int {bxn}, {byn};")
            fn = "rasterize_row" if order == "row" else "rasterize_col"
            self.w(f"tl::{fn}<{panel}>(tl_bid, gridDim.x, gridDim.y, {bxn}, {byn});")
            for v, d in list(zip(k.block_vars, dims))[2:]:
                self.w(f"const int {self.e(v)} = blockIdx.{d};")
        else:
            for v, d in zip(k.block_vars, dims):
                self.w(f"const int {self.e(v)} = blockIdx.{d};")
        for b in self.func.params:
            pass


def generate(func, kernel, target, lds_offsets, lds_total, name, pass_cfg=None) -> KernelSource:
    return CodeGen(func, kernel, target, lds_offsets, lds_total, pass_cfg).generate(name)


def _reads(e, buf) -> bool:
    from ..ir.expr import post_order
    return any(isinstance(n, BufferLoad) and n.buffer is buf for n in post_order(e))


def _has_local_call(e) -> bool:
    """Calls (possibly impure or costly) anywhere in ``e``: such a scalar is not splatted."""
    from ..ir.expr import post_order
    return any(isinstance(n, Call) for n in post_order(e))
