"""Plot the gfx950 MFMA operand / accumulator fragments (reference:
examples/plot_layout/fragment_mfma_load_a.py, which builds CDNA3 16x16x16 load layouts).

gfx950 tiles (wave64): ``v_mfma_f32_16x16x32_{f16,bf16}`` A operand: lane l holds
A[l % 16][8 * (l // 16) + j], j < 8; int8 ``16x16x64``: 16 consecutive k per lane; the 16x16
accumulator: lane l holds C[4 * (l // 16) + v][l % 16].  ``make_mfma_load_base_layout`` builds
those maps as ``Fragment`` objects; ``plot_layout`` renders thread/register grids (txt, svg)."""
import argparse

from tilelang.intrinsics.mfma_layout import a_coord, b_coord, c_coord, k_per_lane
from tilelang.layout import Fragment
from tilelang.tools.plot_layout import layout_text, plot_layout


def _fragment_from_map(rows, cols, owner):
    """Fragment over [rows, cols] from a (row, col) -> (lane, reg) table (reference-style
    ``Fragment(shape, forward_fn=...)``: converted to the compiler's digit form)."""
    return Fragment([rows, cols], forward_fn=lambda i, j: owner[(int(i), int(j))], num_threads=64)


def make_mfma_load_base_layout(dtype="float16", matrix="A", k_dim=None):
    """Fragment of one 16 x k_dim MFMA operand (A: [16, k], B: [k, 16])."""
    kp = k_per_lane(dtype)
    k_dim = k_dim or 4 * kp
    owner = {}
    for lane in range(64):
        for j in range(kp):
            r, c = a_coord(lane, j, kp) if matrix == "A" else b_coord(lane, j, kp)
            owner[(r, c)] = (lane, j)
    shape = (16, k_dim) if matrix == "A" else (k_dim, 16)
    return _fragment_from_map(shape[0], shape[1], owner)


def make_mfma_store_layout():
    owner = {}
    for lane in range(64):
        for v in range(4):
            owner[c_coord(lane, v)] = (lane, v)
    return _fragment_from_map(16, 16, owner)


def main(save_dir="./tmp", formats="txt,svg"):
    for name, frag in (("mfma_16x16x32_f16_A", make_mfma_load_base_layout("float16", "A")),
                       ("mfma_16x16x32_f16_B", make_mfma_load_base_layout("float16", "B")),
                       ("mfma_16x16x64_i8_A", make_mfma_load_base_layout("int8", "A")),
                       ("mfma_16x16_C", make_mfma_store_layout())):
        print(f"== {name}")
        print(layout_text(frag, max_rows=16, max_cols=16))
        plot_layout(frag, save_dir, name, formats)


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--save_dir", default="./tmp")
    a = p.parse_args()
    main(a.save_dir)
