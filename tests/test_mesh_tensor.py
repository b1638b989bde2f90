"""MeshTensor sharding arithmetic (test vectors from the reference's
testing/python/language/test_tilelang_language_mesh_tensor.py)."""
import math

import pytest

import tilelang.language as T
from tilelang.language.annot import MeshTensorAnnot, MeshShardingPolicy, MeshReplicationType, TensorAnnot


@pytest.mark.parametrize("shape, nrows, ncols", [((100, 200, 300), 2, 2), ((64, 128), 4, 1), ((10, 20, 30, 40), 8, 8)])
def test_replicate_all(shape, nrows, ncols):
    p = MeshShardingPolicy(replicate=MeshReplicationType.ALL)
    assert MeshTensorAnnot._get_sharded_shape(shape, p, nrows, ncols) == shape


@pytest.mark.parametrize("shape, d, nrows, ncols", [((100, 200, 300), 1, 2, 2), ((100, 203, 300), 1, 2, 2),
                                                    ((128, 256, 512), 0, 4, 4), ((128, 256, 512), 2, 2, 8)])
def test_cross_mesh_dim(shape, d, nrows, ncols):
    exp = list(shape)
    exp[d] = math.ceil(shape[d] / (nrows * ncols))
    assert MeshTensorAnnot._get_sharded_shape(shape, MeshShardingPolicy(cross_mesh_dim=d), nrows, ncols) == tuple(exp)


def test_invalid_cross_mesh_dim():
    with pytest.raises(ValueError, match="Invalid cross_mesh_dim"):
        MeshTensorAnnot._get_sharded_shape((100, 200), MeshShardingPolicy(cross_mesh_dim=2), 2, 2)


@pytest.mark.parametrize("shape, y, nrows, ncols", [((100, 200, 300), 0, 4, 4), ((103, 200, 300), 0, 4, 4)])
def test_replicate_row(shape, y, nrows, ncols):
    exp = list(shape)
    exp[y] = math.ceil(shape[y] / nrows)
    p = MeshShardingPolicy(y=y, replicate=MeshReplicationType.ROW)
    assert MeshTensorAnnot._get_sharded_shape(shape, p, nrows, ncols) == tuple(exp)


@pytest.mark.parametrize("policy, msg", [
    (MeshShardingPolicy(x=1, y=0, replicate=MeshReplicationType.ROW),
     "Cannot shard on x-axis when replicating on rows"),
    (MeshShardingPolicy(y=3, replicate=MeshReplicationType.ROW), "Invalid y-split dimension"),
    (MeshShardingPolicy(x=1, y=0, replicate=MeshReplicationType.COLUMN), "Cannot shard on y-axis"),
])
def test_invalid_policies(policy, msg):
    with pytest.raises(ValueError, match=msg):
        MeshTensorAnnot._get_sharded_shape((100, 200, 300), policy, 4, 4)


def test_none_replication_splits_both():
    p = MeshShardingPolicy(y=0, x=1)
    assert MeshTensorAnnot._get_sharded_shape((128, 256), p, 4, 2) == (32, 128)


@pytest.mark.parametrize("shape, cfg, policy, hdims, hgroups, hstrides, exp_hdims, exp_hstrides", [
    ((128, 256), (2, 4), MeshShardingPolicy(y=0, x=1), (128, 256), ((0, 1), (1, 2)), (256, 1), (64, 64), (64, 1)),
    ((128, 128), (2, 2), MeshShardingPolicy(y=0, x=1), (2, 4, 16, 2, 4, 16), ((0, 3), (3, 6)),
     (8192, 1024, 16, 4096, 256, 1), (1, 4, 16, 1, 4, 16), (4096, 1024, 16, 4096, 256, 1)),
    ((128, 128), (2, 2), MeshShardingPolicy(y=0, replicate=MeshReplicationType.ROW), (4, 32, 4, 32),
     ((0, 2), (2, 4)), (1024, 1, 4096, 32), (2, 32, 4, 32), (1024, 1, 2048, 32)),
    ((128, 128), (2, 2), MeshShardingPolicy(cross_mesh_dim=0), (4, 32, 128), ((0, 2), (2, 3)), (32, 1, 4096),
     (1, 32, 128), (32, 1, 32)),
])
def test_hierarchical_sharding(shape, cfg, policy, hdims, hgroups, hstrides, exp_hdims, exp_hstrides):
    t = MeshTensorAnnot()(shape, policy, cfg, hierarchical_dims=hdims, hierarchical_strides=hstrides,
                          hierarchical_groups=hgroups)
    assert t.meta_data["sharded_hdims"] == exp_hdims
    assert t.meta_data["sharded_hstrides"] == exp_hstrides


def test_tensor_meta_attr_on_prim_func():
    cfg = (2, 4)
    A_t = T.MeshTensor((128, 256), T.MeshShardingPolicy(y=0, x=1), cfg, dtype="float32")

    @T.prim_func
    def kernel(A: A_t):
        with T.Kernel(1, threads=64):
            pass

    assert kernel.params[0].shape == [64, 64]
    meta = kernel.attrs["tensor_meta"]["A"]
    assert meta["global_shape"] == (128, 256)
    assert meta["sharded_hdims"] == (64, 64)
    assert TensorAnnot._construct_strides((64, 64)) == meta["sharded_hstrides"]
