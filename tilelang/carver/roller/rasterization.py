"""Block rasterisation plans (reference ``tilelang/carver/roller/rasterization.py``).

On MI355X a plan maps to ``T.use_swizzle(panel_size, order)``, which also spreads consecutive
tiles over the 8 XCDs (each XCD has its own 4 MiB L2)."""
from __future__ import annotations


class Rasterization:
    panel_width_ = None

    def get_code(self):
        return []

    @property
    def panel_width(self):
        return self.panel_width_


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


class Rasterization2DColumn(Rasterization):

    def __init__(self, panel_width=8):
        self.panel_width_ = panel_width

    def __repr__(self):
        return f"<Rasterization2DColumn({self.panel_width_})>"

    def swizzle_args(self):
        return dict(panel_size=self.panel_width_, order="column")
