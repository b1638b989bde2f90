"""gfx950 LDS bank-conflict model.

Encodes the per-instruction lane groups and bank functions measured on MI355X
(``MI355X_MICROARCH.md`` §LDS): a wave64 access is serviced in fixed lane
groups, one LDS cycle per group when conflict-free; each extra distinct dword
address on a bank inside a group costs one more cycle; identical addresses
broadcast.  Used to *choose* LDS swizzles (``layout/mfma.py``) and to report
expected ``SQ_LDS_BANK_CONFLICT`` cycles next to the rocprof counter.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

_B128_GROUPS = [
    list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
    list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
    list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
    list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64)),
]

# instruction -> (lane groups, bytes per lane, bank modulus)
INSTRUCTIONS: Dict[str, tuple] = {
    "ds_read_b32": ([list(range(0, 32)), list(range(32, 64))], 4, 32),
    "ds_read_b64": ([list(range(0, 32)), list(range(32, 64))], 8, 64),
    "ds_read_b128": (_B128_GROUPS, 16, 64),
    "ds_read_b64_tr_b16": ([list(range(0, 32)), list(range(32, 64))], 8, 64),
    "ds_write_b32": ([list(range(0, 32)), list(range(32, 64))], 4, 32),
    "ds_write_b64": ([list(range(i, i + 16)) for i in range(0, 64, 16)], 8, 32),
    "ds_write_b128": ([list(range(i, i + 8)) for i in range(0, 64, 8)], 16, 32),
}


def instruction_cycles(instr: str, byte_addrs: Sequence[int]) -> int:
    """LDS-array cycles one wave-instruction costs (conflict-free == number of groups).
    Evaluated by the native model (``tilelang._tl_core.lds_instruction_cycles``, csrc/core/lds.cc)."""
    from .._native import core
    return core().lds_instruction_cycles(instr, [-1 if a is None else int(a) for a in byte_addrs])


def instruction_cycles_py(instr: str, byte_addrs: Sequence[int]) -> int:
    """Pure-Python twin of the native model (kept as the executable specification for tests)."""
    groups, width, mod = INSTRUCTIONS[instr]
    total = 0
    for g in groups:
        banks: Dict[int, set] = {}
        for lane in g:
            a = byte_addrs[lane]
            if a is None:
                continue
            for w in range(width // 4):
                dword = a // 4 + w
                banks.setdefault(dword % mod, set()).add(dword)
        total += max((len(s) for s in banks.values()), default=1)
    return total


def conflict_cycles(instr: str, byte_addrs: Sequence[int]) -> int:
    """Extra cycles beyond the conflict-free cost (what SQ_LDS_BANK_CONFLICT counts)."""
    groups, _, _ = INSTRUCTIONS[instr]
    return instruction_cycles(instr, byte_addrs) - len(groups)


def pattern_cost(instr: str, patterns: List[Sequence[int]]) -> int:
    return sum(instruction_cycles(instr, p) for p in patterns)
