"""The tile IR: expressions, buffers, statements, tile operators, printer."""
from . import dtypes
from .dtypes import DType, as_dtype
from .expr import (PrimExpr, IntImm, FloatImm, StringImm, Var, BinOp, UnOp, Cast, Select, Call, BufferLoad,
                   const, convert, cast, call, select, substitute, evaluate, structural_equal, as_int)
from .buffer import Buffer, BufferRegion, to_region
from .stmt import (Stmt, SeqStmt, ForStmt, WhileStmt, IfStmt, StoreStmt, EvaluateStmt, LetStmt, AllocStmt,
                   TileOpStmt, BreakStmt, ContinueStmt, AssertStmt, AttrStmt, RawStmt, KernelStmt, PrimFunc)
from . import tileop
from .printer import expr_str, stmt_str, func_str

__all__ = [
    "dtypes", "DType", "as_dtype", "PrimExpr", "IntImm", "FloatImm", "StringImm", "Var", "BinOp", "UnOp",
    "Cast", "Select", "Call", "BufferLoad", "const", "convert", "cast", "call", "select", "substitute",
    "evaluate", "structural_equal", "as_int", "Buffer", "BufferRegion", "to_region", "Stmt", "SeqStmt",
    "ForStmt", "WhileStmt", "IfStmt", "StoreStmt", "EvaluateStmt", "LetStmt", "AllocStmt", "TileOpStmt",
    "BreakStmt", "ContinueStmt", "AssertStmt", "AttrStmt", "RawStmt", "KernelStmt", "PrimFunc", "tileop",
    "expr_str", "stmt_str", "func_str"
]
