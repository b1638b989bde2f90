"""Data types of the tile IR.

The reference re-exports TVM's ``DataType`` strings (``"float16"``, ``"float"``,
``"float8_e4m3"``...) through ``tilelang/language/v2/dtypes.py``.  Here a DType
is a tiny immutable record that also knows its HIP (gfx950) and CPU C++
spelling and the matching ``torch.dtype``.

gfx950 uses OCP fp8 (``e4m3fn`` / ``e5m2``), not the MI300 ``fnuz`` encodings
the reference's AMD path assumes (``src/tl_templates/hip/hip_fp8.h:5-10``);
``float8_e4m3fnuz`` is accepted as a spelling but rejected at codegen time.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class DType:
    name: str          # canonical name, e.g. "float16"
    kind: str          # "float" | "int" | "uint" | "bool" | "handle"
    bits: int
    lanes: int = 1

    # -- classification -------------------------------------------------
    @property
    def is_float(self) -> bool:
        return self.kind == "float"

    @property
    def is_int(self) -> bool:
        return self.kind in ("int", "uint")

    @property
    def is_bool(self) -> bool:
        return self.kind == "bool"

    @property
    def is_fp8(self) -> bool:
        return self.kind == "float" and self.bits == 8

    @property
    def is_low_float(self) -> bool:
        return self.kind == "float" and self.bits < 32

    @property
    def bytes(self) -> int:
        return max(1, self.bits // 8) * self.lanes

    def with_lanes(self, lanes: int) -> "DType":
        return DType(self.name, self.kind, self.bits, lanes)

    def __str__(self) -> str:  # noqa: D401
        return self.name if self.lanes == 1 else f"{self.name}x{self.lanes}"

    def __repr__(self) -> str:
        return f"T.{self.name}"

    def __eq__(self, other) -> bool:
        if isinstance(other, str):
            try:
                other = as_dtype(other)
            except Exception:  # noqa: BLE001
                return False
        if not isinstance(other, DType):
            return False
        return self.name == other.name and self.lanes == other.lanes

    def __hash__(self) -> int:
        return hash((self.name, self.lanes))

    # allow ``T.float16(1.5)`` style constant construction
    def __call__(self, value=None):
        from .expr import const, Var
        if value is None:
            return Var("v", self)
        return const(value, self)

    def torch(self):
        """The matching ``torch.dtype``."""
        return to_torch(self)

    # ``T.float32.max()`` helpers used by some programs
    def max(self):
        from .expr import const
        return const(max_value(self), self)

    def min(self):
        from .expr import const
        return const(min_value(self), self)


_TABLE = {}


def _reg(name, kind, bits, *aliases):
    dt = DType(name, kind, bits)
    _TABLE[name] = dt
    for a in aliases:
        _TABLE[a] = dt
    return dt


float16 = _reg("float16", "float", 16, "half", "fp16", "f16")
bfloat16 = _reg("bfloat16", "float", 16, "bf16")
float32 = _reg("float32", "float", 32, "float", "fp32", "f32")
float64 = _reg("float64", "float", 64, "double", "fp64")
float8_e4m3fn = _reg("float8_e4m3fn", "float", 8, "float8_e4m3", "e4m3", "fp8_e4m3")
float8_e5m2 = _reg("float8_e5m2", "float", 8, "e5m2", "fp8_e5m2")
float8_e4m3fnuz = _reg("float8_e4m3fnuz", "float", 8)
float8_e5m2fnuz = _reg("float8_e5m2fnuz", "float", 8)
float8_e8m0fnu = _reg("float8_e8m0fnu", "float", 8, "e8m0")
float4_e2m1fn = _reg("float4_e2m1fn", "float", 4, "fp4")
float4_e2m1fn_x2 = _reg("float4_e2m1fn_x2", "float", 8, "fp4x2")  # two e2m1 per byte (low nibble first)
int8 = _reg("int8", "int", 8)
int16 = _reg("int16", "int", 16)
int32 = _reg("int32", "int", 32, "int")
int64 = _reg("int64", "int", 64)
uint8 = _reg("uint8", "uint", 8)
uint16 = _reg("uint16", "uint", 16)
uint32 = _reg("uint32", "uint", 32)
uint64 = _reg("uint64", "uint", 64)
boolean = _reg("bool", "bool", 8)
handle = _reg("handle", "handle", 64)
void = _reg("void", "handle", 0)


NAMES = _TABLE


def as_dtype(x) -> DType:
    """Normalise anything dtype-like (str, DType, torch.dtype) to a DType."""
    if isinstance(x, DType):
        return x
    if isinstance(x, str):
        if x in _TABLE:
            return _TABLE[x]
        # vector spelling "float16x8"
        for base in sorted(_TABLE, key=len, reverse=True):
            if x.startswith(base + "x") and x[len(base) + 1:].isdigit():
                return _TABLE[base].with_lanes(int(x[len(base) + 1:]))
        raise ValueError(f"unknown dtype {x!r}")
    try:
        import torch
        if isinstance(x, torch.dtype):
            return from_torch(x)
    except ImportError:  # pragma: no cover
        pass
    if x is int:
        return int32
    if x is float:
        return float32
    if x is bool:
        return boolean
    raise TypeError(f"cannot convert {x!r} to a dtype")


_TORCH_NAMES = {
    "float16": "float16",
    "bfloat16": "bfloat16",
    "float32": "float32",
    "float64": "float64",
    "float8_e4m3fn": "float8_e4m3fn",
    "float8_e5m2": "float8_e5m2",
    "float8_e4m3fnuz": "float8_e4m3fnuz",
    "float8_e5m2fnuz": "float8_e5m2fnuz",
    "float8_e8m0fnu": "float8_e8m0fnu",
    "float4_e2m1fn_x2": "float4_e2m1fn_x2",
    "int8": "int8",
    "int16": "int16",
    "int32": "int32",
    "int64": "int64",
    "uint8": "uint8",
    "uint16": "uint16",
    "uint32": "uint32",
    "uint64": "uint64",
    "bool": "bool",
}


def to_torch(dt):
    import torch
    dt = as_dtype(dt)
    name = _TORCH_NAMES.get(dt.name)
    if name is None or not hasattr(torch, name):
        if dt.name in ("float4_e2m1fn", "float4_e2m1fn_x2"):
            return torch.uint8
        raise TypeError(f"dtype {dt} has no torch equivalent")
    return getattr(torch, name)


def from_torch(tdt) -> DType:
    s = str(tdt).replace("torch.", "")
    if s == "float":
        s = "float32"
    if s == "half":
        s = "float16"
    return as_dtype(s)


# C++ spellings used by the HIP emitter (see include/tl/common.h)
_HIP_NAMES = {
    "float16": "half_t",
    "bfloat16": "bfloat16_t",
    "float32": "float",
    "float64": "double",
    "float8_e4m3fn": "fp8_e4_t",
    "float8_e5m2": "fp8_e5_t",
    "float8_e8m0fnu": "uint8_t",
    "float4_e2m1fn": "uint8_t",
    "float4_e2m1fn_x2": "uint8_t",
    "int8": "int8_t",
    "int16": "int16_t",
    "int32": "int",
    "int64": "int64_t",
    "uint8": "uint8_t",
    "uint16": "uint16_t",
    "uint32": "uint32_t",
    "uint64": "uint64_t",
    "bool": "bool",
    "handle": "void*",
    "void": "void",
}

# CPU C++ spellings (include/tl/cpu.h)
_CPU_NAMES = dict(_HIP_NAMES)
_CPU_NAMES.update({"float16": "half_t", "bfloat16": "bfloat16_t", "float8_e4m3fn": "fp8_e4_t",
                   "float8_e5m2": "fp8_e5_t"})


def hip_type(dt) -> str:
    dt = as_dtype(dt)
    if dt.name in ("float8_e4m3fnuz", "float8_e5m2fnuz"):
        raise TypeError("gfx950 uses OCP fp8 (float8_e4m3fn / float8_e5m2); fnuz types are MI300-only")
    base = _HIP_NAMES[dt.name]
    if dt.lanes == 1:
        return base
    return f"tl::vec<{base}, {dt.lanes}>"


def cpu_type(dt) -> str:
    dt = as_dtype(dt)
    return _CPU_NAMES[dt.name]


def max_value(dt):
    dt = as_dtype(dt)
    if dt.is_float:
        return {
            "float16": 65504.0,
            "bfloat16": 3.3895313892515355e38,
            "float32": 3.4028234663852886e38,
            "float64": 1.7976931348623157e308,
            "float8_e4m3fn": 448.0,
            "float8_e5m2": 57344.0,
        }.get(dt.name, float("inf"))
    if dt.kind == "int":
        return 2**(dt.bits - 1) - 1
    if dt.kind == "uint":
        return 2**dt.bits - 1
    return 1


def min_value(dt):
    dt = as_dtype(dt)
    if dt.is_float:
        return -max_value(dt)
    if dt.kind == "int":
        return -(2**(dt.bits - 1))
    return 0


def promote(a: DType, b: DType) -> DType:
    """Binary-op result type: the wider float wins, floats beat ints."""
    if a == b:
        return a
    if a.is_float and not b.is_float:
        return a
    if b.is_float and not a.is_float:
        return b
    if a.is_float and b.is_float:
        if a.bits != b.bits:
            return a if a.bits > b.bits else b
        return float32  # e.g. fp16 op bf16
    if a.is_bool:
        return b
    if b.is_bool:
        return a
    return a if a.bits >= b.bits else b


__all__ = [
    "DType", "as_dtype", "to_torch", "from_torch", "hip_type", "cpu_type", "promote", "max_value",
    "min_value", "float16", "bfloat16", "float32", "float64", "float8_e4m3fn", "float8_e5m2",
    "float8_e4m3fnuz", "float8_e5m2fnuz", "float8_e8m0fnu", "float4_e2m1fn", "int8", "int16",
    "int32", "int64", "uint8", "uint16", "uint32", "uint64", "boolean", "handle", "void"
]
