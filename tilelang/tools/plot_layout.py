"""Render fragment layouts (reference ``tilelang/tools/plot_layout.py``).

``plot_layout(frag)`` draws the (thread, register) owner of every element of a 2-D fragment.
Without matplotlib it writes a text grid ("T<thread>:R<reg>") and an SVG, which is what the
MFMA layouts of this backend are easiest to inspect with.
"""
from __future__ import annotations

import os
from typing import Optional

from ..layout.fragment import Fragment


def layout_grid(frag: Fragment):
    """rows x cols list of (thread, register) of replica 0."""
    if len(frag.shape) != 2:
        raise ValueError("plot_layout draws 2-D fragments")
    R, C = frag.shape
    grid = [[None] * C for _ in range(R)]
    for (i, j), owners in frag.table().items():
        grid[i][j] = min(owners)
    return grid


def layout_text(frag: Fragment, max_rows: int = 32, max_cols: int = 32) -> str:
    grid = layout_grid(frag)
    lines = []
    for row in grid[:max_rows]:
        lines.append(" ".join(f"T{t:<3d}R{r:<2d}" for t, r in row[:max_cols]))
    return "\n".join(lines)


def _color(t: int) -> str:
    h = (t * 47) % 360
    return f"hsl({h},70%,75%)"


def layout_svg(frag: Fragment, cell: int = 28) -> str:
    grid = layout_grid(frag)
    R, C = len(grid), len(grid[0])
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{C * cell}" height="{R * cell}" font-size="8">']
    for i, row in enumerate(grid):
        for j, (t, r) in enumerate(row):
            x, y = j * cell, i * cell
            out.append(f'<rect x="{x}" y="{y}" width="{cell}" height="{cell}" fill="{_color(t)}" stroke="#333"/>')
            out.append(f'<text x="{x + 2}" y="{y + 11}">T{t}</text><text x="{x + 2}" y="{y + 22}">R{r}</text>')
    out.append("</svg>")
    return "\n".join(out)


def plot_layout(frag: Fragment, save_directory: str = "./tmp", name: str = "layout", formats: str = "txt,svg",
                verbose: bool = False) -> Optional[str]:
    os.makedirs(save_directory, exist_ok=True)
    paths = []
    fm = [f.strip() for f in formats.split(",") if f.strip()]
    if "txt" in fm:
        p = os.path.join(save_directory, f"{name}.txt")
        with open(p, "w") as f:
            f.write(layout_text(frag, 10**9, 10**9) + "\n")
        paths.append(p)
    if "svg" in fm:
        p = os.path.join(save_directory, f"{name}.svg")
        with open(p, "w") as f:
            f.write(layout_svg(frag))
        paths.append(p)
    if "png" in fm or "pdf" in fm:
        try:
            import matplotlib  # noqa: F401
            import matplotlib.pyplot as plt
        except ImportError:
            if verbose:
                print("matplotlib not available; wrote txt/svg only")
        else:
            grid = layout_grid(frag)
            fig, ax = plt.subplots(figsize=(len(grid[0]) * 0.5, len(grid) * 0.5))
            ax.imshow([[t for t, _ in row] for row in grid], cmap="tab20")
            for i, row in enumerate(grid):
                for j, (t, r) in enumerate(row):
                    ax.text(j, i, f"T{t}\nR{r}", ha="center", va="center", fontsize=5)
            for ext in ("png", "pdf"):
                if ext in fm:
                    p = os.path.join(save_directory, f"{name}.{ext}")
                    fig.savefig(p)
                    paths.append(p)
            plt.close(fig)
    if verbose:
        print("\n".join(paths))
    return paths[0] if paths else None
