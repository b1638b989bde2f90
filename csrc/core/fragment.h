// fragment.h — the digit-permutation Fragment algebra of the tilelang compiler core.
//
// Reference counterpart: src/layout/layout.{h,cc} (FragmentNode: forward_thread, forward_index,
// replicate, Inverse, DetectInjective) which the reference evaluates through TVM's
// iter-affine-map machinery.  Here a fragment is a *mixed-radix digit permutation*: every
// logical dim is split into digits (size, stride); each digit sits either in the thread number
// or in the per-thread register index; thread digits bound to no logical dim are replication.
// All CDNA4 MFMA operand/accumulator layouts, reductions and vectorised default layouts have this
// form, so forward and inverse maps are exact and cheap -- this file holds the numeric engine
// (whole-layout tables, ownership/uniformity proofs over every lane of the block) that layout
// inference and tile-op lowering run thousands of times per kernel.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace tlcore {

struct Digit {
  int dim;         // logical dim, -1 = replication
  int64_t stride;  // weight of the digit inside its dim
  int64_t size;
};

class Fragment {
 public:
  Fragment(std::vector<int64_t> shape, std::vector<Digit> thread, std::vector<Digit> local, int64_t thread_offset = 0);

  int64_t num_threads() const { return nthreads_; }
  int64_t local_size() const { return nlocal_; }
  int ndim() const { return (int)shape_.size(); }
  const std::vector<int64_t>& shape() const { return shape_; }

  // logical index held by thread t in register r (replicas map to the same element)
  void inverse(int64_t t, int64_t r, int64_t* out) const;
  // (thread of replica 0, register) owning a logical element
  int64_t forward_thread(const int64_t* idx, int64_t rep = 0) const;
  int64_t forward_index(const int64_t* idx) const;
  // does thread t own element idx?  returns its register or -1
  int64_t register_of(int64_t t, const int64_t* idx) const;

  // [T * L * ndim] logical indices, row-major over (thread, register)
  std::vector<int64_t> table() const;
  bool equals(const Fragment& o) const;

  // Register of `buf` that holds buf[A @ loop_idx + b] for register r of this (loop) layout,
  // proven uniform over every thread; -1 = some thread does not own the element, -2 = the
  // register differs between threads.  A is [buf.ndim x ndim] row-major.
  int64_t resolve_affine(const Fragment& buf, const std::vector<int64_t>& A, const std::vector<int64_t>& b,
                         int64_t r) const;

 private:
  std::vector<int64_t> shape_;
  std::vector<Digit> thread_, local_;
  int64_t thread_offset_;
  int64_t nthreads_, nlocal_;
  void validate() const;
};

// Reduction grouping of tile_op lowering (lower_tile_op._reduce_groups): for every register r of
// `src`, the register of `dst` that every thread 0..T-1 holding src element idx (idx with `dim`
// set to 0 when `squeeze`, else removed) owns; empty when some thread does not own that element
// or two threads disagree (the layouts are not reduce-compatible).
std::vector<int64_t> reduce_owners(const Fragment& src, const Fragment& dst, int dim, bool squeeze, int64_t T);

}  // namespace tlcore
