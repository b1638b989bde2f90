// fragment.cc — numeric engine of the digit Fragment algebra (see fragment.h).
#include "fragment.h"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace tlcore {

Fragment::Fragment(std::vector<int64_t> shape, std::vector<Digit> thread, std::vector<Digit> local,
                   int64_t thread_offset)
    : shape_(std::move(shape)), thread_(std::move(thread)), local_(std::move(local)), thread_offset_(thread_offset) {
  nthreads_ = 1;
  for (auto& d : thread_) nthreads_ *= d.size;
  nlocal_ = 1;
  for (auto& d : local_) nlocal_ *= d.size;
  validate();
}

void Fragment::validate() const {
  for (int dim = 0; dim < (int)shape_.size(); ++dim) {
    std::vector<Digit> ds;
    for (auto& d : thread_)
      if (d.dim == dim) ds.push_back(d);
    for (auto& d : local_)
      if (d.dim == dim) ds.push_back(d);
    std::sort(ds.begin(), ds.end(), [](const Digit& a, const Digit& b) { return a.stride < b.stride; });
    int64_t acc = 1;
    for (auto& d : ds) {
      if (d.stride != acc)
        throw std::invalid_argument("fragment digits of dim " + std::to_string(dim) + " do not tile it");
      acc *= d.size;
    }
    if (acc != shape_[dim])
      throw std::invalid_argument("fragment digits of dim " + std::to_string(dim) + " cover " + std::to_string(acc) +
                                  ", extent is " + std::to_string(shape_[dim]));
  }
}

void Fragment::inverse(int64_t t, int64_t r, int64_t* out) const {
  for (size_t i = 0; i < shape_.size(); ++i) out[i] = 0;
  t -= thread_offset_;
  for (auto it = thread_.rbegin(); it != thread_.rend(); ++it) {
    int64_t v = t % it->size;
    t /= it->size;
    if (it->dim >= 0) out[it->dim] += v * it->stride;
  }
  for (auto it = local_.rbegin(); it != local_.rend(); ++it) {
    int64_t v = r % it->size;
    r /= it->size;
    if (it->dim >= 0) out[it->dim] += v * it->stride;
  }
}

int64_t Fragment::forward_thread(const int64_t* idx, int64_t rep) const {
  int64_t acc = 0;
  std::vector<int64_t> reps;
  for (auto& d : thread_)
    if (d.dim < 0) reps.push_back(d.size);
  std::vector<int64_t> rv(reps.size());
  for (int i = (int)reps.size() - 1; i >= 0; --i) {
    rv[i] = rep % reps[i];
    rep /= reps[i];
  }
  size_t ri = 0;
  for (auto& d : thread_) {
    int64_t v = d.dim < 0 ? rv[ri++] : (idx[d.dim] / d.stride) % d.size;
    acc = acc * d.size + v;
  }
  return acc + thread_offset_;
}

int64_t Fragment::forward_index(const int64_t* idx) const {
  int64_t acc = 0;
  for (auto& d : local_) acc = acc * d.size + (idx[d.dim] / d.stride) % d.size;
  return acc;
}

int64_t Fragment::register_of(int64_t t, const int64_t* idx) const {
  for (int i = 0; i < (int)shape_.size(); ++i)
    if (idx[i] < 0 || idx[i] >= shape_[i]) return -1;
  // thread digits of t must match the element's digits
  int64_t tt = t - thread_offset_;
  if (tt < 0 || tt >= nthreads_) return -1;
  for (auto it = thread_.rbegin(); it != thread_.rend(); ++it) {
    int64_t v = tt % it->size;
    tt /= it->size;
    if (it->dim >= 0 && (idx[it->dim] / it->stride) % it->size != v) return -1;
  }
  return forward_index(idx);
}

std::vector<int64_t> Fragment::table() const {
  const int nd = (int)shape_.size();
  std::vector<int64_t> out((size_t)(nthreads_ * nlocal_ * nd));
  for (int64_t t = 0; t < nthreads_; ++t)
    for (int64_t r = 0; r < nlocal_; ++r) inverse(t + thread_offset_, r, &out[(size_t)((t * nlocal_ + r) * nd)]);
  return out;
}

bool Fragment::equals(const Fragment& o) const {
  if (shape_ != o.shape_ || nthreads_ != o.nthreads_ || nlocal_ != o.nlocal_) return false;
  return table() == o.table();
}

int64_t Fragment::resolve_affine(const Fragment& buf, const std::vector<int64_t>& A, const std::vector<int64_t>& b,
                                 int64_t r) const {
  const int nd = (int)shape_.size();
  const int bd = buf.ndim();
  if ((int)A.size() != bd * nd || (int)b.size() != bd) throw std::invalid_argument("resolve_affine: bad map shape");
  std::vector<int64_t> li(nd), bi(bd);
  int64_t result = -3;
  for (int64_t t = 0; t < nthreads_; ++t) {
    inverse(t + thread_offset_, r, li.data());
    for (int i = 0; i < bd; ++i) {
      int64_t v = b[i];
      for (int j = 0; j < nd; ++j) v += A[i * nd + j] * li[j];
      bi[i] = v;
    }
    int64_t reg = buf.register_of(t + thread_offset_, bi.data());
    if (reg < 0) return -1;
    if (result == -3) result = reg;
    else if (result != reg) return -2;
  }
  return result;
}

std::vector<int64_t> reduce_owners(const Fragment& src, const Fragment& dst, int dim, bool squeeze, int64_t T) {
  const int sn = src.ndim(), dn = dst.ndim();
  const int64_t SL = src.local_size(), DL = dst.local_size();
  std::vector<int64_t> owner((size_t)SL, -1);
  std::vector<int64_t> idx((size_t)sn), didx((size_t)std::max(dn, 1)), dtab((size_t)(DL * std::max(dn, 1)));
  for (int64_t t = 0; t < T; ++t) {
    for (int64_t q = 0; q < DL; ++q) dst.inverse(t, q, &dtab[(size_t)(q * dn)]);
    for (int64_t r = 0; r < SL; ++r) {
      src.inverse(t, r, idx.data());
      int k = 0;
      for (int i = 0; i < sn; ++i) {
        if (i == dim) {
          if (squeeze) didx[(size_t)k++] = 0;
        } else {
          didx[(size_t)k++] = idx[(size_t)i];
        }
      }
      int64_t li = -1;
      for (int64_t q = 0; q < DL && li < 0; ++q) {
        bool eq = true;
        for (int i = 0; i < dn && eq; ++i) eq = dtab[(size_t)(q * dn + i)] == didx[(size_t)i];
        if (eq) li = q;
      }
      if (li < 0) return {};
      if (owner[(size_t)r] < 0) owner[(size_t)r] = li;
      else if (owner[(size_t)r] != li) return {};
    }
  }
  return owner;
}

}  // namespace tlcore
