"""SeerAttention block-sparse attention (reference examples/seer_attention/test_block_sparse_attn_tilelang.py)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "examples", "seer_attention"))
import block_sparse_attn_tilelang as seer  # noqa: E402


def test_seer_cpu():
    seer.test_topk_sparse_attention("cpu", "cpu")
    seer.test_topk_sparse_attention_qlen_lt_klen("cpu", "cpu")


@pytest.mark.gpu
def test_seer_gpu():
    seer.test_topk_sparse_attention()
    seer.test_topk_sparse_attention_qlen_lt_klen()
