// hier.h — hierarchical (multi-level mixed-radix) layouts and their mesh sharding.
//
// Reference: src/layout/hierarchical_layout.cc:19-98 (offset = sum_i h_i * hstride_i, each
// logical dim decomposed over hdims[g0:g1], most significant first) and the MeshTensor
// hierarchical sharding of tilelang/language/v2/annot.py:612-655.
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

namespace tlcore {

class HierLayout {
 public:
  HierLayout(std::vector<int64_t> hdims, std::vector<int64_t> hstrides, std::vector<std::pair<int, int>> hgroups);
  int64_t offset(const std::vector<int64_t>& idx) const;
  std::vector<int64_t> logical_to_hierarchical(const std::vector<int64_t>& idx) const;
  std::vector<int64_t> hierarchical_to_logical(const std::vector<int64_t>& h) const;
  std::vector<int64_t> offset_to_logical(int64_t off) const;
  std::vector<int64_t> offsets() const;  // every logical element, row-major
  bool is_bijective() const;

 private:
  std::vector<int64_t> hdims_, hstrides_, shape_;
  std::vector<std::pair<int, int>> hgroups_;
};

// hdims after splitting logical dim `dim` into `parts` shards on its most significant digit
std::vector<int64_t> shard_hier(const std::vector<int64_t>& hdims, const std::vector<std::pair<int, int>>& hgroups,
                                int dim, int64_t parts);

}  // namespace tlcore
