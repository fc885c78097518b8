// pybind11 module `_runtime`: Python binding of the native paged-KV block manager
// (core in block_manager.h).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "block_manager.h"

namespace py = pybind11;
using dllm::BlockManager;

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "distributed_llm_amd native serving runtime (paged-KV block manager)";
  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, int, bool, int>(), py::arg("num_blocks"), py::arg("block_size") = 16,
           py::arg("prefix_cache") = true, py::arg("placement") = 2)
      .def_property_readonly("block_size", &BlockManager::block_size)
      .def_property_readonly("num_blocks", &BlockManager::num_blocks)
      .def("num_free_blocks", &BlockManager::num_free_blocks)
      .def("num_cached_blocks", &BlockManager::num_cached_blocks)
      .def("has_seq", &BlockManager::has_seq)
      .def("can_allocate", &BlockManager::can_allocate)
      .def("allocate", &BlockManager::allocate)
      .def("append_token", &BlockManager::append_token)
      .def("slots", &BlockManager::slots)
      .def("commit_append", &BlockManager::commit_append)
      .def("set_last_tokens", &BlockManager::set_last_tokens)
      .def("commit", &BlockManager::commit)
      .def("block_table", &BlockManager::block_table)
      .def("seq_len", &BlockManager::seq_len)
      .def("committed", &BlockManager::committed)
      .def("free", &BlockManager::free)
      .def("reset", &BlockManager::reset)
      .def("stats", [](const BlockManager& b) {
        py::dict d;
        for (const auto& kv : b.stats()) d[kv.first.c_str()] = kv.second;
        return d;
      })
      .def("check_invariants", &BlockManager::check_invariants);
}
