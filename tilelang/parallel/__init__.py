"""Mesh parallelism on MI355X: device mesh contexts, T.comm lowering, host collectives.

* ``mesh``        — mesh shape for tracing, ``ProcessMesh`` (one process per GPU, RCCL groups,
                    IPC symmetric workspaces), ``VirtualMesh`` (all ranks in one process)
* ``comm_lower``  — T.comm tile ops -> device-initiated xGMI transfers (include/tl/mesh.h)
* ``comm_plan``   — the reference's 2-D routing schedule of each op (inspection/parity)
* ``collectives`` — tensor-level broadcast/put/all_gather/all_reduce/... over mesh rows/cols
* ``sharding``    — MeshTensor shard/unshard following MeshShardingPolicy
"""
from .mesh import (  # noqa: F401
    DEFAULT_MESH, MeshContext, MeshError, ProcessMesh, VirtualMesh, VirtualRank, current_mesh, default_mesh_shape,
    device_mesh_config, get_device_mesh_config, init_mesh, set_device_mesh_config, set_mesh, shutdown_mesh,
)
