// tl/copy.h — global<->LDS data movement for gfx950.
//
// The reference's HIP cp_async_gs<16> is a plain synchronous vector copy
// (src/tl_templates/hip/copy.h:76-81).  gfx950 has real asynchronous global->LDS DMA:
// global_load_lds_dwordx4 writes 16 bytes per lane to LDS at  M0 + 16*lane  without a VGPR
// round trip; completion is tracked on the vector-memory counter (s_waitcnt vmcnt).
// The LDS destination is lane-linear per wave-instruction (1 KiB), so swizzled LDS images
// are produced by permuting the per-lane *global* source address (guide rule 21).
#pragma once

namespace tl {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) char lds_char_t;

// One wave-instruction of LDS-DMA: every lane loads 16 B from gsrc; the wave writes
// 1 KiB contiguously starting at lds_dst (which must be wave-uniform and 16-B aligned).
TL_DEVICE void glds16(const void* gsrc, void* lds_dst) {
  __builtin_amdgcn_global_load_lds(gsrc, (lds_void_t*)(lds_dst), 16, 0, 0);
}
TL_DEVICE void glds4(const void* gsrc, void* lds_dst) {
  __builtin_amdgcn_global_load_lds(gsrc, (lds_void_t*)(lds_dst), 4, 0, 0);
}

// Non-temporal variant (aux=2: nt) for streamed-once operands (decode weights).
TL_DEVICE void glds16_nt(const void* gsrc, void* lds_dst) {
  __builtin_amdgcn_global_load_lds(gsrc, (lds_void_t*)(lds_dst), 16, 0, 2);
}

// Buffer-resource based LDS-DMA with hardware out-of-bounds zero fill: lanes whose byte
// offset is >= num_bytes write zeros to LDS.  Used for ragged tiles.
TL_DEVICE __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t num_bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)num_bytes, 0x00020000);
}
TL_DEVICE void buffer_lds16(__amdgpu_buffer_rsrc_t rsrc, uint32_t voffset, void* lds_dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_t*)(lds_dst), 16, voffset, 0, 0, 0);
}
// 4 bytes per lane (small tiles: one instruction per wave, see transform/pipeline.py
// _small_dma_plan); lane l writes lds_dst + 4 l
TL_DEVICE void buffer_lds4(__amdgpu_buffer_rsrc_t rsrc, uint32_t voffset, void* lds_dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_t*)(lds_dst), 4, voffset, 0, 0, 0);
}

}  // namespace tl
