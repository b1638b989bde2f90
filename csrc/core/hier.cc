// hier.cc — hierarchical layouts (see hier.h).
#include "hier.h"

#include <algorithm>
#include <numeric>
#include <stdexcept>
#include <string>

namespace tlcore {

HierLayout::HierLayout(std::vector<int64_t> hdims, std::vector<int64_t> hstrides,
                       std::vector<std::pair<int, int>> hgroups)
    : hdims_(std::move(hdims)), hstrides_(std::move(hstrides)), hgroups_(std::move(hgroups)) {
  if (hdims_.size() != hstrides_.size()) throw std::invalid_argument("hdims and hstrides must have the same length");
  std::vector<int> covered;
  for (auto& g : hgroups_) {
    if (!(0 <= g.first && g.first <= g.second && g.second <= (int)hdims_.size()))
      throw std::invalid_argument("invalid hierarchical group");
    int64_t n = 1;
    for (int i = g.first; i < g.second; ++i) {
      n *= hdims_[i];
      covered.push_back(i);
    }
    shape_.push_back(n);
  }
  std::sort(covered.begin(), covered.end());
  std::vector<int> all(hdims_.size());
  std::iota(all.begin(), all.end(), 0);
  if (covered != all) throw std::invalid_argument("hierarchical groups must partition the hierarchical dims");
}

std::vector<int64_t> HierLayout::logical_to_hierarchical(const std::vector<int64_t>& idx) const {
  if (idx.size() != shape_.size()) throw std::invalid_argument("index rank mismatch");
  std::vector<int64_t> h(hdims_.size(), 0);
  for (size_t d = 0; d < hgroups_.size(); ++d) {
    int64_t x = idx[d];
    for (int i = hgroups_[d].second - 1; i >= hgroups_[d].first; --i) {
      h[i] = x % hdims_[i];
      x /= hdims_[i];
    }
  }
  return h;
}

std::vector<int64_t> HierLayout::hierarchical_to_logical(const std::vector<int64_t>& h) const {
  std::vector<int64_t> out;
  for (auto& g : hgroups_) {
    int64_t x = 0;
    for (int i = g.first; i < g.second; ++i) x = x * hdims_[i] + h[i];
    out.push_back(x);
  }
  return out;
}

int64_t HierLayout::offset(const std::vector<int64_t>& idx) const {
  auto h = logical_to_hierarchical(idx);
  int64_t off = 0;
  for (size_t i = 0; i < h.size(); ++i) off += h[i] * hstrides_[i];
  return off;
}

std::vector<int64_t> HierLayout::offset_to_logical(int64_t off) const {
  std::vector<size_t> order(hdims_.size());
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return hstrides_[a] > hstrides_[b]; });
  std::vector<int64_t> h(hdims_.size(), 0);
  for (size_t i : order) {
    h[i] = off / hstrides_[i];
    off %= hstrides_[i];
  }
  return hierarchical_to_logical(h);
}

std::vector<int64_t> HierLayout::offsets() const {
  int64_t n = 1;
  for (auto s : shape_) n *= s;
  std::vector<int64_t> out((size_t)n), idx(shape_.size(), 0);
  for (int64_t e = 0; e < n; ++e) {
    int64_t x = e;
    for (int d = (int)shape_.size() - 1; d >= 0; --d) {
      idx[d] = x % shape_[d];
      x /= shape_[d];
    }
    out[(size_t)e] = offset(idx);
  }
  return out;
}

bool HierLayout::is_bijective() const {
  auto o = offsets();
  std::sort(o.begin(), o.end());
  for (size_t i = 0; i < o.size(); ++i)
    if (o[i] != (int64_t)i) return false;
  return true;
}

std::vector<int64_t> shard_hier(const std::vector<int64_t>& hdims, const std::vector<std::pair<int, int>>& hgroups,
                                int dim, int64_t parts) {
  std::vector<int64_t> out = hdims;
  if (parts == 1) return out;
  if (dim < 0 || dim >= (int)hgroups.size()) throw std::invalid_argument("shard dim out of range");
  int start = hgroups[dim].first, end = hgroups[dim].second;
  if (start >= end) return out;
  if (hdims[start] % parts != 0)
    throw std::invalid_argument("The most significant hierarchical dimension (" + std::to_string(hdims[start]) +
                                ") of logical dimension " + std::to_string(dim) +
                                " is not divisible by the shard factor (" + std::to_string(parts) + ").");
  out[start] = hdims[start] / parts;
  return out;
}

}  // namespace tlcore
