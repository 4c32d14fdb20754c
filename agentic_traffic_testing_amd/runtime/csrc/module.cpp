// pybind11 module of the native serving runtime: paged-KV block manager / batch builder
// (block_manager.cpp) and the TP step-metadata shared-memory channel (shm_channel.cpp).
#include <pybind11/pybind11.h>

namespace py = pybind11;

void register_block_manager(py::module_& m);
void register_shm_channel(py::module_& m);

PYBIND11_MODULE(_atta_runtime, m) {
  m.doc() = "Native serving runtime for agentic_traffic_testing_amd";
  register_block_manager(m);
  register_shm_channel(m);
}
