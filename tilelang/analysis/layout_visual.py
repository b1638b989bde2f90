"""Layout visualisation pass (reference ``tilelang/analysis/layout_visual.py:84``, enabled with
``pass_configs={"tl.layout_visualization_enable": True, "tl.layout_visualization_formats": ...}``).

After layout inference every fragment's (thread, register) map and every shared tile's LDS
swizzle is written out: one ``<kernel>.layouts.txt`` summary plus, per 2-D fragment, the
element grids of ``tilelang.tools.plot_layout`` in the requested formats (txt / svg / png / pdf).
The directory is ``$TILELANG_LAYOUT_DIR`` or ``./tilelang_layouts``."""
from __future__ import annotations

import os
from typing import List

from ..layout.fragment import Fragment


def layout_dir() -> str:
    return os.environ.get("TILELANG_LAYOUT_DIR", os.path.join(os.getcwd(), "tilelang_layouts"))


def dump_layouts(kernel_name: str, li, formats: str = "txt") -> List[str]:
    from ..tools.plot_layout import plot_layout
    fm = "txt,svg,png,pdf" if "all" in formats else formats
    d = layout_dir()
    os.makedirs(d, exist_ok=True)
    paths = []
    lines = [f"# layouts of {kernel_name}"]
    for b, lay in li.frag.items():
        lines.append(f"fragment {b.name} {list(b.shape)} {b.dtype}: {lay!r}")
        if isinstance(lay, Fragment) and len(lay.shape) == 2:
            p = plot_layout(lay, d, f"{kernel_name}.{b.name}", fm)
            if p:
                paths.append(p)
    for b in getattr(li, "shared_buffers", []) or []:
        lines.append(f"shared {b.name} {list(b.shape)} {b.dtype}: {getattr(b, 'layout', None)!r}")
    summary = os.path.join(d, f"{kernel_name}.layouts.txt")
    with open(summary, "w") as f:
        f.write("\n".join(lines) + "\n")
    paths.insert(0, summary)
    return paths
