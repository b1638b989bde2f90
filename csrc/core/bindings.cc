// bindings.cc — pybind11 module tilelang._tl_core: the native compiler core used by the Python
// passes (layout inference, tile-op lowering, LDS planning, swizzle selection, hierarchical
// layouts).  Pure host C++: it builds and runs without a GPU.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>

#include "fragment.h"
#include "hier.h"
#include "lds.h"

namespace py = pybind11;
using namespace tlcore;

namespace {

std::vector<Digit> to_digits(const std::vector<std::tuple<int, int64_t, int64_t>>& v) {
  std::vector<Digit> out;
  out.reserve(v.size());
  for (auto& t : v) out.push_back({std::get<0>(t), std::get<1>(t), std::get<2>(t)});
  return out;
}

py::tuple as_tuple(const int64_t* p, int n) {
  py::tuple t(n);
  for (int i = 0; i < n; ++i) t[i] = py::int_(p[i]);
  return t;
}

}  // namespace

PYBIND11_MODULE(_tl_core, m) {
  m.doc() = "tilelang native compiler core (fragment algebra, LDS model, arena planner, hierarchical layouts)";

  py::class_<Fragment>(m, "Fragment")
      .def(py::init([](std::vector<int64_t> shape, const std::vector<std::tuple<int, int64_t, int64_t>>& td,
                       const std::vector<std::tuple<int, int64_t, int64_t>>& ld, int64_t thread_offset) {
             return Fragment(std::move(shape), to_digits(td), to_digits(ld), thread_offset);
           }),
           py::arg("shape"), py::arg("thread_digits"), py::arg("local_digits"), py::arg("thread_offset") = 0)
      .def_property_readonly("num_threads", &Fragment::num_threads)
      .def_property_readonly("local_size", &Fragment::local_size)
      .def("inverse",
           [](const Fragment& f, int64_t t, int64_t r) {
             std::vector<int64_t> out(f.ndim());
             f.inverse(t, r, out.data());
             return as_tuple(out.data(), f.ndim());
           })
      .def("forward_thread",
           [](const Fragment& f, std::vector<int64_t> idx, int64_t rep) { return f.forward_thread(idx.data(), rep); },
           py::arg("idx"), py::arg("rep") = 0)
      .def("forward_index", [](const Fragment& f, std::vector<int64_t> idx) { return f.forward_index(idx.data()); })
      .def("table", &Fragment::table, "flat [T * L * ndim] logical indices over (thread, register)")
      .def("thread_local_map",
           [](const Fragment& f, int64_t t) {
             py::dict d;
             std::vector<int64_t> idx(f.ndim());
             for (int64_t r = 0; r < f.local_size(); ++r) {
               f.inverse(t, r, idx.data());
               d[as_tuple(idx.data(), f.ndim())] = py::int_(r);
             }
             return d;
           })
      .def("equals", &Fragment::equals)
      .def("resolve_affine", &Fragment::resolve_affine, py::arg("buf"), py::arg("A"), py::arg("b"), py::arg("r"),
           "register of `buf` holding buf[A @ idx + b] for register r of this loop layout on every thread "
           "(-1 not owned, -2 non-uniform)");

  m.def("reduce_owners", &reduce_owners, py::arg("src"), py::arg("dst"), py::arg("dim"), py::arg("squeeze"),
        py::arg("T"), "dst register of every src register for a tile reduction over `dim` (empty = incompatible)");
  m.def("lds_instruction_cycles", [](const std::string& instr, const std::vector<int64_t>& addrs) {
    if (addrs.size() != 64) throw std::invalid_argument("need 64 lane addresses");
    return instruction_cycles(lds_instr(instr), addrs.data());
  });
  m.def("swizzle_costs", &swizzle_costs, py::arg("instr"), py::arg("rows_cols"), py::arg("npat"), py::arg("cols"),
        py::arg("elem_bytes"), py::arg("candidates"));
  m.def(
      "plan_arena",
      [](const std::vector<int64_t>& sizes, const std::vector<int64_t>& first, const std::vector<int64_t>& last,
         int64_t align, bool reuse, int64_t limit) {
        ArenaPlan p = plan_arena(sizes, first, last, align, reuse, limit);
        return py::make_tuple(p.offsets, p.total);
      },
      py::arg("sizes"), py::arg("first"), py::arg("last"), py::arg("align"), py::arg("reuse"), py::arg("limit"));

  py::class_<HierLayout>(m, "HierarchicalLayout")
      .def(py::init<std::vector<int64_t>, std::vector<int64_t>, std::vector<std::pair<int, int>>>())
      .def("offset", &HierLayout::offset)
      .def("logical_to_hierarchical", &HierLayout::logical_to_hierarchical)
      .def("hierarchical_to_logical", &HierLayout::hierarchical_to_logical)
      .def("offset_to_logical", &HierLayout::offset_to_logical)
      .def("offsets", &HierLayout::offsets, "offset of every logical element, row-major")
      .def("is_bijective", &HierLayout::is_bijective);
  m.def("shard_hier", &shard_hier, py::arg("hdims"), py::arg("hgroups"), py::arg("dim"), py::arg("parts"),
        "split logical dim `dim` of a hierarchical layout into `parts` shards over its most significant "
        "hierarchical digits; returns the per-shard hdims");
}
