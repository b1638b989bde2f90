// tl/swizzle.h — block-index remapping for L2 locality on MI355X.
//
// Reference: src/tl_templates/hip/threadblock_swizzle.h (rasterization2DRow/Column<panel>).
// MI355X has 8 XCDs with private 4 MiB L2s and the dispatcher deals consecutive workgroups
// round-robin over them (blocks b and b+8 share an XCD).  xcd_remap() first makes each XCD
// own a contiguous chunk of the launch (bijective for any grid size, guide §5 "XCD swizzle
// must be bijective"), then the panel rasterisation makes neighbouring tiles of that chunk
// share A rows / B columns.  Purely a performance mapping: correctness never depends on it.
#pragma once

namespace tl {

TL_DEVICE int xcd_remap(int bid, int nblocks) {
  constexpr int NXCD = 8;
  if (nblocks < NXCD) return bid;
  const int q = nblocks / NXCD, r = nblocks % NXCD;
  const int xcd = bid % NXCD, k = bid / NXCD;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

// Map a linear block id onto (bx, by) of a grid_x x grid_y tile grid, panel-major:
// groups of PANEL rows (by) are walked column-by-column so consecutive ids reuse B columns.
template <int PANEL> TL_DEVICE void rasterize_row(int id, int grid_x, int grid_y, int& bx, int& by) {
  const int panel_span = PANEL * grid_x;
  const int panel = id / panel_span;
  const int first_row = panel * PANEL;
  const int rows = (grid_y - first_row) < PANEL ? (grid_y - first_row) : PANEL;
  const int in_panel = id % panel_span;
  by = first_row + in_panel % rows;
  bx = in_panel / rows;
}

template <int PANEL> TL_DEVICE void rasterize_col(int id, int grid_x, int grid_y, int& bx, int& by) {
  const int panel_span = PANEL * grid_y;
  const int panel = id / panel_span;
  const int first_col = panel * PANEL;
  const int cols = (grid_x - first_col) < PANEL ? (grid_x - first_col) : PANEL;
  const int in_panel = id % panel_span;
  bx = first_col + in_panel % cols;
  by = in_panel / cols;
}

}  // namespace tl
