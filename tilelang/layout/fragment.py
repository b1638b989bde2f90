"""Fragment layouts: how a logical tile is distributed over a block's lanes.

Reference: ``src/layout/layout.{h,cc}`` (``FragmentNode``: forward_thread +
forward_index + replicate_size, Inverse/Repeat/Replicate/CondenseReplicateVar)
and the Python mirror ``tilelang/layout/fragment.py``.

Representation used here (MI355X-first, not a TVM iter-map): every fragment is
a *mixed-radix digit permutation*.  Each logical dimension is split into digits
(size, stride); every digit is placed either in the **thread** number or in the
per-thread **local** (register) index; extra thread digits that are bound to no
logical digit are **replication** digits.  All CDNA4 MFMA operand/accumulator
layouts, their k-permuted variants, reduction results and the default
vectorised layouts are of this form, so forward *and* inverse maps are exact
closed-form expressions (``//``, ``%``, ``*``) that clang folds per unrolled
register index.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple



@dataclass(frozen=True)
class Digit:
    dim: int       # logical dimension (-1 for a replication digit)
    stride: int    # weight of this digit inside its logical dimension
    size: int

    def __repr__(self):
        if self.dim < 0:
            return f"rep{self.size}"
        return f"d{self.dim}[{self.size}x{self.stride}]"


def _mixed(digs: Sequence[Digit], values: Sequence):
    """Compose a mixed-radix number (most significant digit first)."""
    acc = 0
    for d, v in zip(digs, values):
        acc = acc * d.size + v
    return acc


class Fragment:
    """A thread/register distribution of a logical tile.

    ``thread_digits``: most-significant first, their mixed-radix value is the thread id.
    ``local_digits``:  most-significant first, their mixed-radix value is the register index.
    """

    def __init__(self, shape: Sequence[int], thread_digits: Sequence[Digit], local_digits: Sequence[Digit],
                 name: str = "frag", thread_offset: int = 0):
        self.shape = [int(s) for s in shape]
        self.thread_digits = list(thread_digits)
        self.local_digits = list(local_digits)
        self.name = name
        self.thread_offset = thread_offset   # for BindThreadRange-style offsets
        self._validate()

    # -- sizes -------------------------------------------------------------------
    @property
    def num_threads(self) -> int:
        n = 1
        for d in self.thread_digits:
            n *= d.size
        return n

    @property
    def local_size(self) -> int:
        n = 1
        for d in self.local_digits:
            n *= d.size
        return n

    @property
    def replicate_size(self) -> int:
        n = 1
        for d in self.thread_digits:
            if d.dim < 0:
                n *= d.size
        return n

    def _validate(self):
        # every logical dim must be exactly covered by its digits
        for dim, ext in enumerate(self.shape):
            digs = sorted([d for d in self.thread_digits + self.local_digits if d.dim == dim], key=lambda d: d.stride)
            acc = 1
            for d in digs:
                if d.stride != acc:
                    raise ValueError(f"{self.name}: digits of dim {dim} do not tile it: {digs}")
                acc *= d.size
            if acc != ext:
                raise ValueError(f"{self.name}: digits of dim {dim} cover {acc}, extent is {ext}")

    def reshape(self, new_shape: Sequence[int]) -> "Fragment":
        """The same thread / register assignment of the same elements, indexed by a row-major
        reshape of the tile (``T.reshape`` / ``T.view`` of a fragment).  Each digit keeps its
        place in the thread or register number; a digit that straddles a boundary of the new
        shape is split in two (high part more significant), so the register index of every
        element is unchanged and the view shares the source's registers."""
        new_shape = [int(s) for s in new_shape]
        total = 1
        for s in self.shape:
            total *= s
        nt = 1
        for s in new_shape:
            nt *= s
        if nt != total:
            raise ValueError(f"{self.name}: cannot reshape {self.shape} to {new_shape}")

        def inner(shape, d):
            r = 1
            for s in shape[d + 1:]:
                r *= s
            return r

        def convert(d: Digit) -> List[Digit]:
            if d.dim < 0:
                return [d]
            lin, size = d.stride * inner(self.shape, d.dim), d.size
            parts = []  # least significant first
            while size > 1:
                nd = max(i for i in range(len(new_shape)) if inner(new_shape, i) <= lin)
                inn = inner(new_shape, nd)
                if lin % inn:
                    raise ValueError(f"{self.name}: digit {d} does not map onto {new_shape}")
                st = lin // inn
                room = new_shape[nd] // st
                take = min(room, size)
                if size % take or new_shape[nd] % st:
                    raise ValueError(f"{self.name}: digit {d} does not map onto {new_shape}")
                parts.append(Digit(nd, st, take))
                lin *= take
                size //= take
            return list(reversed(parts)) or [Digit(0 if not new_shape else len(new_shape) - 1, 1, 1)]

        td = [x for d in self.thread_digits for x in convert(d)]
        ld = [x for d in self.local_digits for x in convert(d)]
        # size-1 placeholder digits would break the tiling check: drop them
        td = [x for x in td if x.size > 1 or x.dim < 0]
        ld = [x for x in ld if x.size > 1]
        return Fragment(new_shape, td, ld, self.name + "_reshape", self.thread_offset)

    # -- maps --------------------------------------------------------------------
    def _digit_values(self, idx):
        vals = {}
        for d in self.thread_digits + self.local_digits:
            if d.dim < 0:
                continue
            x = idx[d.dim]
            v = (x // d.stride) % d.size if d.size != self.shape[d.dim] or d.stride != 1 else x
            if isinstance(x, int):
                v = (x // d.stride) % d.size
            vals[d] = v
        return vals

    def forward_thread(self, *idx, rep=0):
        """Thread owning logical element ``idx`` (replica ``rep``)."""
        idx = list(idx)
        vals = self._digit_values(idx)
        rep_digits = [d for d in self.thread_digits if d.dim < 0]
        rep_vals = {}
        r = rep
        for d in reversed(rep_digits):
            rep_vals[id(d)] = r % d.size if not isinstance(r, int) or True else r
            r = r // d.size
        acc = 0
        for d in self.thread_digits:
            v = rep_vals[id(d)] if d.dim < 0 else vals[d]
            acc = acc * d.size + v
        return acc + self.thread_offset

    def forward_index(self, *idx):
        idx = list(idx)
        vals = self._digit_values(idx)
        acc = 0
        for d in self.local_digits:
            acc = acc * d.size + vals[d]
        return acc

    def inverse(self, thread, local) -> List:
        """Logical index held by ``thread`` in register ``local`` (ints or exprs)."""
        thread = thread - self.thread_offset if self.thread_offset else thread
        vals = {}
        t = thread
        for d in reversed(self.thread_digits):
            if d.size == 1:
                v = 0
            else:
                v = t % d.size
                t = t // d.size
            vals[id(d)] = v
        l = local
        for d in reversed(self.local_digits):
            if d.size == 1:
                v = 0
            else:
                v = l % d.size
                l = l // d.size
            vals[id(d)] = v
        idx = [0] * len(self.shape)
        for d in self.thread_digits + self.local_digits:
            if d.dim < 0:
                continue
            v = vals[id(d)]
            term = v * d.stride if d.stride != 1 else v
            idx[d.dim] = term if (isinstance(idx[d.dim], int) and idx[d.dim] == 0) else idx[d.dim] + term
        return idx

    # -- native engine ---------------------------------------------------------------
    @property
    def native(self):
        """The C++ twin (``tilelang._tl_core.Fragment``) used for whole-layout numeric work."""
        nf = self.__dict__.get("_native_frag")
        if nf is None:
            from .._native import core
            nf = core().Fragment(self.shape, [(d.dim, d.stride, d.size) for d in self.thread_digits],
                                 [(d.dim, d.stride, d.size) for d in self.local_digits], self.thread_offset)
            self.__dict__["_native_frag"] = nf
        return nf

    # -- structure queries ---------------------------------------------------------
    def signature(self) -> Tuple:
        return (tuple(self.shape), tuple(self.thread_digits), tuple(self.local_digits), self.thread_offset)

    def is_equal(self, other: "Fragment") -> bool:
        if other is None:
            return False
        if self.signature() == other.signature():
            return True
        if self.shape != other.shape or self.num_threads != other.num_threads or \
                self.local_size != other.local_size:
            return False
        # numeric comparison (digit structure may differ but the map be identical)
        return self.native.equals(other.native)

    def table(self) -> Dict[Tuple[int, ...], List[Tuple[int, int]]]:
        """logical idx -> list of (thread, local) (replicas)."""
        out = {}
        flat = self.native.table()
        nd = len(self.shape)
        L = self.local_size
        for t in range(self.num_threads):
            for r in range(L):
                o = (t * L + r) * nd
                out.setdefault(tuple(flat[o:o + nd]), []).append((t + self.thread_offset, r))
        return out

    def thread_local_map(self, thread: int) -> Dict[Tuple[int, ...], int]:
        """For one thread: logical idx -> local index."""
        if isinstance(thread, int):
            return self.native.thread_local_map(thread)
        return {tuple(self.inverse(thread, r)): r for r in range(self.local_size)}

    def inner_vector_width(self, dim: Optional[int] = None) -> int:
        """Number of consecutive registers that hold consecutive elements of the innermost dim."""
        if not self.local_digits:
            return 1
        last = self.local_digits[-1]
        if dim is None:
            dim = len(self.shape) - 1
        if last.dim == dim and last.stride == 1:
            return last.size
        return 1

    def __repr__(self):
        return (f"Fragment({self.name}, shape={self.shape}, thread={self.thread_digits}, "
                f"local={self.local_digits})")

    # reference-API conveniences --------------------------------------------------
    def get_thread_size(self):
        return self.num_threads

    def get_input_shape(self):
        return list(self.shape)

    def map_forward_thread(self, *idx):
        return self.forward_thread(*idx)

    def map_forward_index(self, *idx):
        return self.forward_index(*idx)

    def replicate(self, n: int) -> "Fragment":
        """Replicate the whole fragment ``n`` times over more threads (outer replication digit)."""
        return Fragment(self.shape, [Digit(-1, 1, n)] + self.thread_digits, self.local_digits, self.name + "_rep")

    def repeat(self, repeats: Sequence[int], repeat_on_thread: bool = False) -> "Fragment":
        """Tile the fragment ``repeats[d]`` times along each dim (on registers or threads)."""
        new_shape = [s * r for s, r in zip(self.shape, repeats)]
        td, ld = list(self.thread_digits), list(self.local_digits)
        outer = []
        for dim, (s, r) in enumerate(zip(self.shape, repeats)):
            if r > 1:
                outer.append(Digit(dim, s, r))
        if repeat_on_thread:
            td = outer + td
        else:
            ld = outer + ld
        return Fragment(new_shape, td, ld, self.name + "_repeat")

    def condense_rep_var(self) -> "Fragment":
        return Fragment(self.shape, [d for d in self.thread_digits if d.dim >= 0], self.local_digits, self.name)


# ---------------------------------------------------------------------------
# constructors
# ---------------------------------------------------------------------------


def _split_dim(dim: int, extent: int, factors: Sequence[int]) -> List[Digit]:
    """Split a dimension into digits with the given sizes (most significant first)."""
    digs = []
    stride = extent
    for f in factors:
        stride //= f
        digs.append(Digit(dim, stride, f))
    return digs


def make_linear_fragment(shape: Sequence[int], num_threads: int, vec: int = 1, name="linear") -> Fragment:
    """Default fragment: row-major elements, ``vec`` consecutive elements per thread per step,
    threads over the flattened tile, remaining repeats in registers.  Falls back to
    replication when the tile has fewer elements than threads."""
    shape = [int(s) for s in shape]
    total = 1
    for s in shape:
        total *= s
    vec = max(1, vec)
    while vec > 1 and (shape[-1] % vec != 0 or total // vec < 1):
        vec //= 2
    # decompose the flattened index (outer, thread, vec) over the dims
    slots = total // vec
    t_used = min(num_threads, slots)
    while slots % t_used != 0:
        t_used -= 1
    rep = num_threads // t_used if num_threads % t_used == 0 else None
    if rep is None:
        raise ValueError(f"cannot distribute {shape} over {num_threads} threads")
    outer = slots // t_used
    # flattened factors, most significant first: outer, t_used, vec
    factors = [("l", outer), ("t", t_used), ("l", vec)]
    # assign each factor to digits over dims (row-major flatten)
    digits_t, digits_l = [], []
    remaining = list(shape)  # remaining extent of each dim (from most significant side)
    dim = 0
    # convert to a per-dim decomposition by walking factors from least significant
    rev = list(reversed(factors))
    cur_dim = len(shape) - 1
    cur_stride = 1
    placed = []
    for kind, f in rev:
        while f > 1:
            if cur_dim < 0:
                raise ValueError("fragment factor overflow")
            avail = shape[cur_dim] // cur_stride
            if avail == 1:
                cur_dim -= 1
                cur_stride = 1
                continue
            take = _gcd_pow(f, avail)
            if take == 1:
                return _greedy_fragment(shape, num_threads, vec, name)
            placed.append((kind, Digit(cur_dim, cur_stride, take)))
            cur_stride *= take
            f //= take
            if cur_stride == shape[cur_dim]:
                cur_dim -= 1
                cur_stride = 1
    # most significant first
    placed.reverse()
    digits_t = [d for k, d in placed if k == "t"]
    digits_l = [d for k, d in placed if k == "l"]
    if rep > 1:
        digits_t = [Digit(-1, 1, rep)] + digits_t
    # dims of extent 1 need no digits
    return Fragment(shape, digits_t or [Digit(-1, 1, num_threads)] if not digits_t else digits_t, digits_l, name)


def _greedy_fragment(shape, num_threads: int, vec: int, name: str) -> Fragment:
    """Fallback of make_linear_fragment for extents the row-major split cannot tile (a thread
    factor straddling a non-power-of-two dim, e.g. [32, 576] over 128 threads): ``vec`` on the
    innermost dim, then the threads take the largest factors they can from the innermost dims
    outward, and whatever a dim has left over goes to registers."""
    import math
    t_left = num_threads
    td, ld_inner, ld_outer = [], [], []
    for dim in range(len(shape) - 1, -1, -1):
        ext, stride = shape[dim], 1
        if dim == len(shape) - 1 and vec > 1:
            ld_inner.append(Digit(dim, 1, vec))
            stride = vec
        avail = ext // stride
        take = math.gcd(t_left, avail)
        if take > 1:
            td.insert(0, Digit(dim, stride, take))
            stride *= take
            t_left //= take
        if ext // stride > 1:
            ld_outer.insert(0, Digit(dim, stride, ext // stride))
    if t_left > 1:
        td.insert(0, Digit(-1, 1, t_left))  # fewer elements than threads: replicate
    return Fragment(shape, td, ld_outer + ld_inner, name)


def _gcd_pow(a: int, b: int) -> int:
    import math
    return math.gcd(a, b)


def make_replicated_fragment(shape: Sequence[int], num_threads: int, name="replicated") -> Fragment:
    """Every thread holds the whole tile (e.g. small per-row statistics used by all lanes)."""
    shape = [int(s) for s in shape]
    local = []
    for dim, s in enumerate(shape):
        if s > 1:
            local.append(Digit(dim, 1, s))
    return Fragment(shape, [Digit(-1, 1, num_threads)], local, name)


def fragment_from_table(shape, num_threads, fn_thread, fn_index, replicate=1, name="user") -> Fragment:
    """Build a digit fragment from reference-style forward functions by probing.

    Supports layouts whose forward maps are mixed-radix digit placements (every
    layout the reference builds for CDNA is); raises otherwise.
    """
    shape = [int(s) for s in shape]
    import itertools
    # probe each dim's power-of-two digits
    digits_t = []
    digits_l = []
    for dim, ext in enumerate(shape):
        stride = 1
        while stride < ext:
            idx0 = [0] * len(shape)
            idx1 = list(idx0)
            idx1[dim] = stride
            t0, t1 = fn_thread(*idx0), fn_thread(*idx1)
            l0, l1 = fn_index(*idx0), fn_index(*idx1)
            size = 2
            while stride * size < ext and ext % (stride * size * 2) == 0:
                idx2 = list(idx0)
                idx2[dim] = stride * size
                if (fn_thread(*idx2) - t0) == (t1 - t0) * size and (fn_index(*idx2) - l0) == (l1 - l0) * size:
                    size *= 2
                else:
                    break
            if ext % (stride * size) != 0:
                size = ext // stride
            d = Digit(dim, stride, size)
            if t1 != t0:
                digits_t.append((t1 - t0, d))
            else:
                digits_l.append((l1 - l0, d))
            stride *= size
    digits_t.sort(key=lambda x: -x[0])
    digits_l.sort(key=lambda x: -x[0])
    td = [d for _, d in digits_t]
    ld = [d for _, d in digits_l]
    if replicate > 1:
        td = [Digit(-1, 1, replicate)] + td
    f = Fragment(shape, td, ld, name)
    # verify
    for idx in itertools.islice(itertools.product(*[range(s) for s in shape]), 4096):
        if f.forward_thread(*idx) != fn_thread(*idx) or f.forward_index(*idx) != fn_index(*idx):
            raise ValueError(f"layout {name} is not a mixed-radix digit layout; unsupported on this backend")
    return f
