// pybind11 bindings of the native (host) runtime: the paged KV-block manager
// and the per-step scheduler helpers. Built with g++ only (no torch), so the
// CPU-side engine logic is native and importable on a machine without a GPU.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "block_manager.h"
#include "step_builder.h"

namespace py = pybind11;
using die::BlockManager;

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "MI355X inference engine native runtime (block manager, step builder)";
  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, int, bool, double>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("prefix_caching") = true, py::arg("ttl_s") = -1.0)
      .def_property_readonly("num_blocks", &BlockManager::num_blocks)
      .def_property_readonly("block_size", &BlockManager::block_size)
      .def("num_free", &BlockManager::num_free)
      .def("num_cached", &BlockManager::num_cached)
      .def("num_available", &BlockManager::num_available)
      .def("num_used", &BlockManager::num_used)
      .def("can_allocate", &BlockManager::can_allocate)
      .def("refcount", &BlockManager::refcount)
      .def("allocate", &BlockManager::allocate)
      .def("incref", &BlockManager::incref)
      .def("free", &BlockManager::free)
      .def("lookup", &BlockManager::lookup)
      .def("match_prefix", &BlockManager::match_prefix)
      .def("register_block", &BlockManager::register_block)
      .def("forget", &BlockManager::forget)
      .def("evict_expired", &BlockManager::evict_expired)
      .def("reset_prefix_cache", &BlockManager::reset_prefix_cache)
      .def_static("hash_blocks", &BlockManager::hash_blocks, py::arg("tokens"), py::arg("block_size"),
                  py::arg("parent") = 0, py::arg("salt") = 0)
      .def("stats", [](const BlockManager& b) {
        auto s = b.stats();
        py::dict d;
        d["num_blocks"] = s.num_blocks;
        d["block_size"] = s.block_size;
        d["free"] = s.free;
        d["cached"] = s.cached;
        d["used"] = s.used;
        d["indexed"] = s.indexed;
        d["allocations"] = s.allocations;
        d["evictions"] = s.evictions;
        d["ttl_evictions"] = s.ttl_evictions;
        d["prefix_hit_blocks"] = s.hit_blocks;
        d["prefix_queried_blocks"] = s.queried_blocks;
        return d;
      });

  m.def("build_decode_inputs", &die::build_decode_inputs,
        "Fill pinned int buffers for a decode step (positions, slot mapping, context lengths, block tables).");
  m.def("build_prefill_inputs", &die::build_prefill_inputs,
        "Fill pinned int buffers for a prefill step (token ids, positions, slots, cu_seqlens, context lengths, "
        "block tables).");
}
