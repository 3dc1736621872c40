// Python module for the native layer: simulator context + HIP/CDNA4 kernels.
#include <pybind11/pybind11.h>

namespace py = pybind11;

namespace gsc {
void register_sim(py::module_& m);
void register_ops(py::module_& m);
}  // namespace gsc

PYBIND11_MODULE(_native, m) {
  m.doc() = "gsc_amd native layer (gfx950): batched coord-sim + GNN/MLP/optimizer kernels";
  gsc::register_sim(m);
  gsc::register_ops(m);
}
