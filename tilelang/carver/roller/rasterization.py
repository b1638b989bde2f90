"""Block rasterisation plans (reference ``tilelang/carver/roller/rasterization.py``).

On MI355X a plan maps to ``T.use_swizzle(panel_size, order)``, which also spreads consecutive
tiles over the 8 XCDs (each XCD has its own 4 MiB L2)."""
from __future__ import annotations


class Rasterization:
    panel_width_ = None

    def get_code(self):
        """The DSL statement that applies the plan (empty: launch order as is)."""
        return []

    @property
    def panel_width(self):
        return self.panel_width_


def l2_panel_width(M: int, N: int, K: int, bm: int, bn: int, eb: int, l2_bytes: int = 4 << 20, xcds: int = 8,
                   cus: int = 256, k_window: int = 256) -> int:
    """Panel width (tile rows per panel) for one XCD's L2.

    Blocks are dealt round-robin over the XCDs, so each XCD runs cus / xcds consecutive tiles of the
    swizzled order at a time; a panel of ``w`` tile rows holds them as w rows x (per_xcd / w)
    columns, which stream w A row panels (bm rows) and per_xcd / w B column panels (bn rows)
    through the L2 side by side.  The power of two minimising those rows (the HBM / Infinity-Cache
    fetches per K step) whose ``k_window`` K-slice of every row fits the L2 is returned (ties: the
    wider panel); at least 1, at most the number of tile rows.  256x256 tiles, 32 per XCD: 8
    (measured: panel 2 / 4 / 8 / 16 within 1 % of each other at 4096^3, profiles/r4/gemm_panel_ab.log)."""
    tiles_m = max(1, -(-M // bm))
    per_xcd = max(1, cus // xcds)
    best, best_rows = 1, None
    w = 1
    while w <= min(tiles_m, per_xcd):
        rows = w * bm + max(1, per_xcd // w) * bn
        if rows * min(K, k_window) * eb <= l2_bytes and (best_rows is None or rows <= best_rows):
            best, best_rows = w, rows
        w *= 2
    return best


class NoRasterization(Rasterization):

    def __repr__(self):
        return "<NoRasterization>"


class Rasterization2DRow(Rasterization):

    def __init__(self, panel_width=8):
        self.panel_width_ = panel_width

    def __repr__(self):
        return f"<Rasterization2DRow({self.panel_width_})>"

    def swizzle_args(self):
        return dict(panel_size=self.panel_width_, order="row")

    def get_code(self):
        return [f"T.use_swizzle(panel_size={self.panel_width_}, order=\"row\")"]


class Rasterization2DColumn(Rasterization):

    def __init__(self, panel_width=8):
        self.panel_width_ = panel_width

    def __repr__(self):
        return f"<Rasterization2DColumn({self.panel_width_})>"

    def swizzle_args(self):
        return dict(panel_size=self.panel_width_, order="column")

    def get_code(self):
        return [f"T.use_swizzle(panel_size={self.panel_width_}, order=\"column\")"]
