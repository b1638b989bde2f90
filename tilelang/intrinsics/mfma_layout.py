"""Lane maps of the gfx950 16x16 MFMA tiles (reference: tilelang/intrinsics/mfma_layout.py).

Standard (unswapped) operand order, wave64, ``K_PER`` = consecutive k per lane (8 for
16x16x32 f16/bf16, 16 for 16x16x64 int8):

    A operand: lane l holds A[i = l % 16][k = K_PER * (l // 16) + j],  j < K_PER
    B operand: lane l holds B[k = K_PER * (l // 16) + j][n = l % 16]
    C / D    : lane l holds C[i = 4 * (l // 16) + v][n = l % 16],       v < 4
"""


def k_per_lane(dtype: str) -> int:
    return 16 if dtype in ("int8", "uint8") else 8


def a_coord(lane, j, k_per):
    """(row, k) of element j of lane's A fragment."""
    return lane % 16, k_per * (lane // 16) + j


def b_coord(lane, j, k_per):
    """(k, col) of element j of lane's B fragment."""
    return k_per * (lane // 16) + j, lane % 16


def c_coord(lane, v):
    """(row, col) of accumulator register v of lane."""
    return 4 * (lane // 16) + v, lane % 16
