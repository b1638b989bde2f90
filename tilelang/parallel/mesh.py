"""Device mesh runtime: a 2-D mesh of MI355X GPUs (one process per GPU) or a virtual mesh.

Reference: the fork's mesh model (``tilelang/language/comm.py``, ``src/op/comm.cc``, the
Sunmmio driver's 4x4 default ``tilelang/carver/arch/driver/sunmmio_driver.py:8-11``) treats a
"core" as one node of an ``nrow x ncol`` mesh.  On MI355X a core is one GPU of the node; the
8 GPUs are fully connected by xGMI, so e.g. a 2x4 mesh has a dedicated link between every pair.

This module owns everything a T.comm kernel needs at run time:

* the mesh shape used when tracing (``get_device_mesh_config`` / ``device_mesh_config``),
* a ``MeshContext`` per rank: rank id, row/column process groups for host collectives
  (RCCL over xGMI via ``torch.distributed``), and the **symmetric workspace**: every rank
  allocates the same number of bytes, exports it (``hipIpcGetMemHandle``) and opens all
  peers' exports, giving a device table ``ws[nranks]`` of peer pointers that kernels store
  into directly (``include/tl/mesh.h``),
* launch epochs (tags that make the flag protocol reusable without resetting memory) and
  the device error word (bounded spins record timeouts there instead of hanging).

Contexts:
  ``init_mesh()``          one process per GPU under torchrun (``nccl`` backend = RCCL), or
                           CPU processes under ``gloo`` (workspaces are /dev/shm mappings);
  ``VirtualMesh(r, c)``    all ranks in one process — threads on the CPU target, one HIP
                           stream per rank on a single GPU — for tests and debugging.
"""
from __future__ import annotations

import contextlib
import mmap
import os
import threading
import uuid
from typing import List, Optional, Tuple

_override: Optional[Tuple[int, int]] = None
_global_ctx: Optional["MeshContext"] = None
_tls = threading.local()

DEFAULT_MESH = (4, 4)  # reference default (Sunmmio driver); an active context always wins
EPOCH_LIMIT = (1 << 20) - 1


def _parse(s: str) -> Tuple[int, int]:
    s = s.lower().replace("*", "x")
    r, c = s.split("x")
    return int(r), int(c)


def get_device_mesh_config() -> Tuple[int, int]:
    """Mesh shape ``(nrow, ncol)`` used by ``T.comm`` / ``T.MeshTensor`` while tracing.

    Priority: the active mesh context > ``set_device_mesh_config`` > ``TILELANG_DEVICE_MESH``
    (e.g. ``2x4``) > the reference default 4x4."""
    ctx = current_mesh()
    if ctx is not None:
        return ctx.shape
    if _override is not None:
        return _override
    env = os.environ.get("TILELANG_DEVICE_MESH")
    if env:
        return _parse(env)
    return DEFAULT_MESH


def set_device_mesh_config(nrow: Optional[int], ncol: Optional[int] = None):
    global _override
    if nrow is None:
        _override = None
        return
    if ncol is None:
        nrow, ncol = nrow
    if nrow < 1 or ncol < 1:
        raise ValueError(f"invalid mesh shape {nrow}x{ncol}")
    _override = (int(nrow), int(ncol))


@contextlib.contextmanager
def device_mesh_config(nrow: int, ncol: int):
    """``with device_mesh_config(2, 4): ...`` — trace kernels for a 2x4 mesh."""
    global _override
    old = _override
    set_device_mesh_config(nrow, ncol)
    try:
        yield (nrow, ncol)
    finally:
        _override = old


def default_mesh_shape(world: int) -> Tuple[int, int]:
    """Most square factorisation with nrow <= ncol (8 -> 2x4, 4 -> 2x2, 2 -> 1x2)."""
    r = int(world ** 0.5)
    while r > 1 and world % r:
        r -= 1
    return r, world // r


def current_mesh() -> Optional["MeshContext"]:
    ctx = getattr(_tls, "ctx", None)
    return ctx if ctx is not None else _global_ctx


# ---------------------------------------------------------------------------------------
# contexts
# ---------------------------------------------------------------------------------------


class MeshError(RuntimeError):
    pass


class MeshContext:
    """Per-rank mesh state.  Subclasses provide workspace allocation and host collectives."""

    def __init__(self, nrow: int, ncol: int, rank: int, device):
        import torch
        self.nrow, self.ncol = int(nrow), int(ncol)
        self.rank = int(rank)
        if not 0 <= self.rank < self.nrow * self.ncol:
            raise ValueError(f"rank {rank} outside a {nrow}x{ncol} mesh")
        self.device = torch.device(device)
        self.epoch = 0
        self.ws_bytes = 0
        self.ws_table = None      # int64 tensor [nranks] of workspace pointers (on self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        # mesh ranks whose kernels share this GPU (co-residency budget, see check_residency)
        self.ranks_on_device = 1

    # -- geometry ---------------------------------------------------------------------
    @property
    def shape(self) -> Tuple[int, int]:
        return (self.nrow, self.ncol)

    @property
    def world(self) -> int:
        return self.nrow * self.ncol

    @property
    def row(self) -> int:
        return self.rank // self.ncol

    @property
    def col(self) -> int:
        return self.rank % self.ncol

    def core(self) -> Tuple[int, int]:
        return (self.row, self.col)

    def group_ranks(self, direction: str) -> List[int]:
        d = direction.lower()
        if d in ("h", "horizontal"):
            return [self.row * self.ncol + j for j in range(self.ncol)]
        if d in ("v", "vertical"):
            return [i * self.ncol + self.col for i in range(self.nrow)]
        if d in ("a", "all"):
            return list(range(self.world))
        raise ValueError(f"invalid direction {direction}")

    # -- kernel launch support ---------------------------------------------------------------
    def ensure_workspace(self, nbytes: int):
        raise NotImplementedError

    def next_epoch(self) -> int:
        self.epoch += 1
        if self.epoch > EPOCH_LIMIT:
            self._reset_workspace()
            self.epoch = 1
        return self.epoch

    def _reset_workspace(self):
        raise NotImplementedError

    def launch_args(self, mesh_meta: dict) -> list:
        """Trailing kernel arguments (rank, ws table, epoch, err) for one launch."""
        if tuple(mesh_meta["shape"]) != self.shape:
            raise MeshError(f"kernel was traced for a {mesh_meta['shape'][0]}x{mesh_meta['shape'][1]} mesh but the "
                            f"active mesh is {self.nrow}x{self.ncol}")
        if mesh_meta["ws_bytes"] > self.ws_bytes:
            self.ensure_workspace(mesh_meta["ws_bytes"])
        ws = self.ws_table.data_ptr() if self.ws_table is not None else 0
        return [self.rank, ws, self.next_epoch(), self.err.data_ptr()]

    def check_residency(self, label: str, nblocks: int, resident: int):
        """Cross-GPU waits inside a T.comm kernel assume every block of every rank is running: a
        block waiting on a peer block that was never scheduled (because the grid exceeds what the
        GPU holds at once) would wait forever.  Refuse such launches up front."""
        need = nblocks * self.ranks_on_device
        if need > resident:
            raise MeshError(f"{label}: T.comm kernel with {nblocks} blocks x {self.ranks_on_device} rank(s) "
                            f"on this GPU "
                            f"needs {need} co-resident workgroups but the GPU holds {resident}; use a persistent grid "
                            f"(T.Persistent / a loop over tiles inside fewer blocks)")

    def error_decoder(self, label, e):
        """MeshError for the bits of the device error word (tl/mesh.h spin codes)."""
        what = []
        if e & 1:
            what.append("waiting for a receiver to free its slot")
        if e & 2:
            what.append("waiting for data from a sender")
        if e & 4:
            what.append("waiting at a mesh barrier")
        msg = f"{label}: timed out " + ", ".join(what) + " (a peer did not run the same kernel sequence)" \
            if what else f"{label}:"
        if e & 16:
            msg += " routing overflow: a token's expert ids are not distinct or out of range (rows dropped)"
        return MeshError(msg)

    def check(self):
        """Raise if any bounded wait of a mesh kernel on this rank timed out."""
        import torch
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
            from ..runtime import errors
            errors.poll()  # launches recorded by JITKernel raise through the monitor first
        e = int(self.err.item())
        if e:
            self.err.zero_()
            raise self.error_decoder(f"mesh rank {self.rank}", e)

    @contextlib.contextmanager
    def activate(self):
        old = getattr(_tls, "ctx", None)
        _tls.ctx = self
        try:
            yield self
        finally:
            _tls.ctx = old

    # host collectives are provided by subclasses (see tilelang.parallel.collectives)
    def __repr__(self):
        return f"{type(self).__name__}(rank={self.rank}, mesh={self.nrow}x{self.ncol}, device={self.device})"


class _ShmBuffer:
    """A named /dev/shm mapping (CPU process meshes)."""

    def __init__(self, name: str, nbytes: int, create: bool):
        import numpy as np
        import torch
        self.path = f"/dev/shm/{name}"
        self.nbytes = nbytes
        if create:
            fd = os.open(self.path, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o600)
            os.ftruncate(fd, nbytes)
        else:
            fd = os.open(self.path, os.O_RDWR)
        self.mm = mmap.mmap(fd, nbytes)
        os.close(fd)
        self.arr = np.frombuffer(self.mm, dtype=np.uint8)
        self.tensor = torch.from_numpy(self.arr)

    def ptr(self) -> int:
        return self.tensor.data_ptr()

    def close(self, unlink: bool):
        self.tensor = None
        self.arr = None
        try:
            self.mm.close()
        except BufferError:
            pass
        if unlink:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


class ProcessMesh(MeshContext):
    """One process per rank under ``torch.distributed`` (``nccl`` = RCCL on ROCm, or ``gloo``
    for CPU meshes).  Row/column groups back the host collectives; the symmetric workspace
    is shared through HIP IPC (GPU) or /dev/shm (CPU)."""

    def __init__(self, nrow: int, ncol: int, device=None, ws_flags: Optional[int] = None):
        import torch
        import torch.distributed as dist
        if not dist.is_initialized():
            raise MeshError("torch.distributed is not initialised; call init_mesh() or dist.init_process_group")
        world = dist.get_world_size()
        if nrow * ncol != world:
            raise MeshError(f"mesh {nrow}x{ncol} needs {nrow * ncol} ranks, world size is {world}")
        rank = dist.get_rank()
        if device is None:
            if dist.get_backend() == "nccl":
                local = os.environ.get("LOCAL_RANK", rank % max(1, torch.cuda.device_count()))
                device = torch.device("cuda", int(local))
            else:
                device = torch.device("cpu")
        super().__init__(nrow, ncol, rank, device)
        if self.device.type == "cuda":
            # ranks that picked the same GPU share its workgroup slots
            devs = [None] * world
            dist.all_gather_object(devs, (os.uname().nodename, self.device.index))
            self.ranks_on_device = sum(1 for d in devs if d == devs[rank])
        # workspace memory class (runtime ws_alloc): 2 = fine-grained, coherent at system scope
        # (the default the device protocols are written for), 1 = uncached, 0 = coarse-grained
        # hipMalloc (A/B only); TL_MESH_WS_FLAGS overrides
        self.ws_flags = int(os.environ.get("TL_MESH_WS_FLAGS", "2")) if ws_flags is None else int(ws_flags)
        self.world_group = dist.group.WORLD
        # every rank creates every row and column group in the same order (new_group is collective)
        self.row_groups = [dist.new_group([r * ncol + c for c in range(ncol)]) for r in range(nrow)]
        self.col_groups = [dist.new_group([r * ncol + c for r in range(nrow)]) for c in range(ncol)]
        self._own = None          # own allocation (ptr or _ShmBuffer)
        self._peers = []          # opened peer mappings
        self._gen = 0
        tok = [uuid.uuid4().hex[:12] if rank == 0 else None]
        dist.broadcast_object_list(tok, src=0)
        self._uid = tok[0]

    def _peer_preflight(self):
        """Collective, once: every pair of distinct GPUs that the mesh's ranks use must have peer
        access (hipDeviceCanAccessPeer over xGMI); fail fast with the pair instead of a kernel
        that faults or times out on its first remote store."""
        if self.__dict__.get("_peer_ok"):
            return
        import torch
        import torch.distributed as dist
        devs = [None] * self.world
        dist.all_gather_object(devs, (os.uname().nodename, self.device.index))
        mine = devs[self.rank]
        bad = []
        for r, d in enumerate(devs):
            if d[0] != mine[0]:
                bad.append((r, "on another node (IPC workspaces need one node)"))
            elif d[1] != mine[1] and not torch.cuda.can_device_access_peer(mine[1], d[1]):
                bad.append((r, f"GPU {mine[1]} cannot access GPU {d[1]} (hipDeviceCanAccessPeer)"))
        flag = torch.tensor([len(bad)], dtype=torch.int32, device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if bad:
            raise MeshError(f"mesh rank {self.rank}: no peer access to rank " +
                            "; rank ".join(f"{r}: {why}" for r, why in bad))
        if int(flag.item()):
            raise MeshError(f"mesh rank {self.rank}: a peer rank reported missing peer access (see its error)")
        self._peer_ok = True

    def group(self, direction: str):
        d = direction.lower()
        if d in ("h", "horizontal"):
            return self.row_groups[self.row]
        if d in ("v", "vertical"):
            return self.col_groups[self.col]
        return self.world_group

    # -- symmetric workspace --------------------------------------------------------------
    def ensure_workspace(self, nbytes: int):
        """Collective: every rank reaches the same launch, so growth happens in lock step."""
        import torch
        import torch.distributed as dist
        if nbytes <= self.ws_bytes:
            return
        nbytes = max(int(nbytes), 2 * self.ws_bytes, 1 << 20)
        nbytes = (nbytes + (1 << 20) - 1) & ~((1 << 20) - 1)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dist.barrier()
        self._release()
        self._gen += 1
        ptrs = []
        if self.device.type == "cuda":
            self._peer_preflight()
            from .. import _native
            rt = _native.runtime()
            dev = self.device.index
            own = rt.ws_alloc(nbytes, dev, self.ws_flags)
            handle = rt.ipc_get_handle(own, dev)
            handles = [None] * self.world
            dist.all_gather_object(handles, handle)
            for r, h in enumerate(handles):
                if r == self.rank:
                    ptrs.append(own)
                else:
                    p = rt.ipc_open_handle(h, dev)
                    self._peers.append(p)
                    ptrs.append(p)
            self._own = own
        else:
            name = f"tl_mesh_{self._uid}_{self._gen}_{self.rank}"
            own = _ShmBuffer(name, nbytes, create=True)
            dist.barrier()
            for r in range(self.world):
                if r == self.rank:
                    ptrs.append(own.ptr())
                else:
                    b = _ShmBuffer(f"tl_mesh_{self._uid}_{self._gen}_{r}", nbytes, create=False)
                    self._peers.append(b)
                    ptrs.append(b.ptr())
            self._own = own
        self.ws_table = torch.tensor(ptrs, dtype=torch.int64, device=self.device)
        self.ws_bytes = nbytes
        self.epoch = 0
        dist.barrier()

    def _release(self):
        if self._own is None:
            return
        if self.device.type == "cuda":
            from .. import _native
            rt = _native.runtime()
            for p in self._peers:
                rt.ipc_close_handle(p, self.device.index)
            rt.ws_free(self._own, self.device.index)
        else:
            for b in self._peers:
                b.close(unlink=False)
            self._own.close(unlink=True)
        self._own, self._peers, self.ws_table, self.ws_bytes = None, [], None, 0

    def _reset_workspace(self):
        import torch.distributed as dist
        n = self.ws_bytes
        self._release()
        dist.barrier()
        self.ensure_workspace(n)

    # -- named symmetric buffers (device-driven exchanges outside T.comm, e.g. ops/ep.py) -----
    def symmetric_buffer(self, key: str, nbytes: int) -> "SymmetricBuffer":
        """Collective: a zeroed device buffer of ``nbytes`` on every rank, IPC-opened by every
        peer (the ``T.comm`` workspace stays separate).  Cached by ``key``; a larger request
        re-allocates it (all ranks must request the same size at the same point)."""
        import torch
        import torch.distributed as dist
        bufs = self.__dict__.setdefault("_sym", {})
        b = bufs.get(key)
        if b is not None and b.nbytes >= nbytes:
            return b
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dist.barrier()
        if b is not None:
            b.release()
        if self.device.type != "cuda":
            # CPU process mesh: a zeroed /dev/shm mapping per rank, opened by every peer (the
            # CPU build of the device protocols, tl/ep_cpu.h, runs on these)
            self._gen += 1
            tag = f"tl_sym_{self._uid}_{self._gen}"
            own = _ShmBuffer(f"{tag}_{self.rank}", int(nbytes), create=True)
            dist.barrier()
            peers = [_ShmBuffer(f"{tag}_{r}", int(nbytes), create=False) for r in range(self.world) if r != self.rank]
            it = iter(peers)
            ptrs = [own.ptr() if r == self.rank else next(it).ptr() for r in range(self.world)]
            b = _ShmSymmetricBuffer(self, own, peers, ptrs, int(nbytes))
            bufs[key] = b
            dist.barrier()
            return b
        self._peer_preflight()
        from .. import _native
        rt = _native.runtime()
        dev = self.device.index
        own = rt.ws_alloc(int(nbytes), dev, self.ws_flags)
        handles = [None] * self.world
        dist.all_gather_object(handles, rt.ipc_get_handle(own, dev))
        ptrs, peers = [], []
        for r, h in enumerate(handles):
            if r == self.rank:
                ptrs.append(own)
            else:
                q = rt.ipc_open_handle(h, dev)
                peers.append(q)
                ptrs.append(q)
        b = SymmetricBuffer(self, own, peers, ptrs, int(nbytes))
        bufs[key] = b
        dist.barrier()
        return b

    def close(self):
        import torch
        import torch.distributed as dist
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dist.barrier()
        for b in self.__dict__.pop("_sym", {}).values():
            b.release()
        self._release()


class _ShmSymmetricBuffer:
    """``SymmetricBuffer`` of a CPU process mesh: /dev/shm mappings instead of IPC handles."""

    def __init__(self, mesh, own, peers, ptrs, nbytes: int):
        import torch
        self.mesh, self.own, self.peers, self.nbytes = mesh, own, list(peers), nbytes
        self.ptrs = list(ptrs)
        self.local = own.tensor
        self.table = torch.tensor(self.ptrs, dtype=torch.int64)

    def view(self, offset: int, shape, dtype):
        import math
        import torch
        n = math.prod(shape) * torch.empty((), dtype=dtype).element_size()
        if offset % 16 or offset + n > self.nbytes:
            raise ValueError(f"view [{offset}, {offset + n}) outside the {self.nbytes}-byte buffer or misaligned")
        return self.local[offset:offset + n].view(dtype).view(*shape)

    def release(self):
        if self.own is None:
            return
        self.local = None
        for q in self.peers:
            q.close(unlink=False)
        self.own.close(unlink=True)
        self.own, self.peers = None, []


class SymmetricBuffer:
    """One rank's view of a symmetric IPC buffer: ``local`` (uint8 tensor over this rank's
    allocation) and ``table`` (int64 device tensor of every rank's base address as mapped in
    this process, indexed by rank)."""

    def __init__(self, mesh, own: int, peers, ptrs, nbytes: int):
        import torch
        from .. import _native
        self.mesh, self.own, self.peers, self.nbytes = mesh, own, list(peers), nbytes
        self.ptrs = list(ptrs)
        dev = mesh.device.index
        self.local = _native.runtime().tensor_from_ptr(own, nbytes, dev)
        self.table = torch.tensor(self.ptrs, dtype=torch.int64, device=mesh.device)

    def view(self, offset: int, shape, dtype):
        """A typed tensor over [offset, offset + prod(shape) * itemsize) of the local buffer."""
        import math
        import torch
        n = math.prod(shape) * torch.empty((), dtype=dtype).element_size()
        if offset % 16 or offset + n > self.nbytes:
            raise ValueError(f"view [{offset}, {offset + n}) outside the {self.nbytes}-byte buffer or misaligned")
        return self.local[offset:offset + n].view(dtype).view(*shape)

    def release(self):
        if self.own is None:
            return
        from .. import _native
        rt = _native.runtime()
        dev = self.mesh.device.index
        self.local = None
        for q in self.peers:
            rt.ipc_close_handle(q, dev)
        rt.ws_free(self.own, dev)
        self.own, self.peers = None, []


class VirtualRank(MeshContext):
    """One rank of a ``VirtualMesh`` (all ranks live in this process)."""

    def __init__(self, mesh: "VirtualMesh", rank: int):
        super().__init__(mesh.nrow, mesh.ncol, rank, mesh.device)
        self.mesh = mesh
        self.stream = None

    def ensure_workspace(self, nbytes: int):
        if nbytes > self.mesh.capacity:
            raise MeshError(f"kernel needs a {nbytes}-byte mesh workspace; create the VirtualMesh with "
                            f"workspace_bytes >= {nbytes}")
        self.ws_table = self.mesh.ws_table
        self.ws_bytes = self.mesh.capacity

    def _reset_workspace(self):
        raise MeshError("virtual mesh epoch overflow; create a new VirtualMesh")


class VirtualMesh:
    """All ranks of an ``nrow x ncol`` mesh in one process.

    CPU target: ``run(fn)`` calls ``fn(rank_ctx)`` for every rank in its own thread (the
    native runtime releases the GIL while a CPU kernel spins on its peers).
    GPU: ``run(fn)`` calls ``fn`` for every rank in turn, each under its own HIP stream, then
    synchronises — the per-rank kernels run concurrently on the one device (keep the grids
    small enough to be co-resident and the mesh within the process's hardware queues)."""

    def __init__(self, nrow: int, ncol: int, device="cpu", workspace_bytes: int = 64 << 20):
        import torch
        self.nrow, self.ncol = int(nrow), int(ncol)
        self.device = torch.device(device)
        self.capacity = int(workspace_bytes)
        self.buffers = [torch.zeros(self.capacity, dtype=torch.uint8, device=self.device)
                        for _ in range(self.nrow * self.ncol)]
        self.ws_table = torch.tensor([b.data_ptr() for b in self.buffers], dtype=torch.int64, device=self.device)
        self.ranks = [VirtualRank(self, r) for r in range(self.nrow * self.ncol)]
        for r in self.ranks:
            r.ranks_on_device = len(self.ranks)  # all virtual ranks run on the one device
        self._coll = _VirtualCollectives(self.nrow * self.ncol)
        for r in self.ranks:
            r.collectives = self._coll
        if self.device.type == "cuda":
            for r in self.ranks:
                r.stream = torch.cuda.Stream(self.device)

    @property
    def shape(self):
        return (self.nrow, self.ncol)

    def run(self, fn, *args, **kwargs) -> list:
        import torch
        results = [None] * len(self.ranks)
        if self.device.type == "cuda":
            cur = torch.cuda.current_stream(self.device)
            for r in self.ranks:
                r.stream.wait_stream(cur)
            for r in self.ranks:
                with torch.cuda.stream(r.stream), r.activate():
                    results[r.rank] = fn(r, *args, **kwargs)
            for r in self.ranks:
                cur.wait_stream(r.stream)
            torch.cuda.synchronize(self.device)
            return results
        errors = []

        def body(r):
            try:
                with r.activate():
                    results[r.rank] = fn(r, *args, **kwargs)
            except BaseException as e:  # noqa: BLE001
                errors.append((r.rank, e))
                self._coll.abort()

        ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in self.ranks]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errors:
            errors.sort(key=lambda x: x[0])
            raise errors[0][1]
        return results

    def check(self):
        for r in self.ranks:
            r.check()


class _VirtualCollectives:
    """Rendezvous used by host collectives of a VirtualMesh (threads exchange tensors)."""

    def __init__(self, n: int):
        self.n = n
        self.barrier = threading.Barrier(n)
        self.lock = threading.Lock()
        self.slots = {}

    def abort(self):
        self.barrier.abort()

    def exchange(self, key, rank: int, value):
        """Every rank deposits ``value``; returns the list of all ranks' values."""
        with self.lock:
            self.slots.setdefault(key, {})[rank] = value
        self.barrier.wait()
        vals = self.slots[key]
        out = [vals.get(r) for r in range(self.n)]
        self.barrier.wait()
        with self.lock:
            self.slots.pop(key, None)
        return out


# ---------------------------------------------------------------------------------------
# process-mesh entry points
# ---------------------------------------------------------------------------------------


def init_mesh(nrow: Optional[int] = None, ncol: Optional[int] = None, backend: Optional[str] = None,
              ws_flags: Optional[int] = None, device=None) -> ProcessMesh:
    """Initialise ``torch.distributed`` from the torchrun environment if needed (``nccl``
    = RCCL when a GPU is visible, else ``gloo``) and make this rank's ``ProcessMesh`` the
    active context.  The default shape is the most square factorisation of the world."""
    import torch
    import torch.distributed as dist
    global _global_ctx
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
        dist.init_process_group(backend=backend)
    world = dist.get_world_size()
    if nrow is None and ncol is None:
        nrow, ncol = default_mesh_shape(world)
    elif nrow is None:
        nrow = world // ncol
    elif ncol is None:
        ncol = world // nrow
    ctx = ProcessMesh(nrow, ncol, device=device, ws_flags=ws_flags)
    _global_ctx = ctx
    return ctx


def shutdown_mesh():
    global _global_ctx
    if _global_ctx is not None:
        _global_ctx.close()
        _global_ctx = None


def set_mesh(ctx: Optional[MeshContext]):
    global _global_ctx
    _global_ctx = ctx
