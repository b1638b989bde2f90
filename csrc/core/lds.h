// lds.h — gfx950 LDS bank model, swizzle search and arena planning (see lds.cc).
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace tlcore {

struct LdsInstr {
  std::vector<std::vector<int>> groups;  // lanes serviced together (one LDS cycle when conflict-free)
  int width;                             // bytes per lane
  int modulus;                           // banks seen by the instruction
};

const LdsInstr& lds_instr(const std::string& name);

// LDS-array cycles one wave instruction costs; byte_addrs[64], negative = inactive lane
int64_t instruction_cycles(const LdsInstr& ins, const int64_t* byte_addrs);

// modelled cycles of every candidate chunk-XOR swizzle (list of (row_bit, chunk_bit)) for the
// access patterns rows_cols [P][64][2] of a [*, cols] tile of elem_bytes elements
std::vector<int64_t> swizzle_costs(const std::string& instr, const std::vector<int64_t>& rows_cols, int64_t npat,
                                   int64_t cols, int64_t elem_bytes,
                                   const std::vector<std::vector<std::pair<int, int>>>& candidates);

struct ArenaPlan {
  std::vector<int64_t> offsets;
  int64_t total;
};

// place buffers (byte sizes, live ranges [first, last] over top-level statements) in one
// dynamic-LDS arena; reuse = share space between buffers with disjoint live ranges
ArenaPlan plan_arena(const std::vector<int64_t>& sizes, const std::vector<int64_t>& first,
                     const std::vector<int64_t>& last, int64_t align, bool reuse, int64_t limit);

}  // namespace tlcore
