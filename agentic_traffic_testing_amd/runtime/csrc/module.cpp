// pybind11 module of the native serving runtime: paged-KV block manager / batch builder
// (block_manager.cpp) and the TP step-metadata shared-memory channel (shm_channel.cpp).
#include <pybind11/pybind11.h>

namespace py = pybind11;

#ifndef ATTA_BUILD_HASH
#define ATTA_BUILD_HASH "unknown"
#endif

void register_block_manager(py::module_& m);
void register_shm_channel(py::module_& m);

PYBIND11_MODULE(_atta_runtime, m) {
  m.doc() = "Native serving runtime for agentic_traffic_testing_amd";
  // sha of the sources this binary was built from (ops/build.py runtime_source_hash)
  m.attr("BUILD_HASH") = ATTA_BUILD_HASH;
  register_block_manager(m);
  register_shm_channel(m);
}
