// Registry of HIP op launchers exposed to Python (filled as kernels are added).
#include <pybind11/pybind11.h>
namespace py = pybind11;
namespace gsc {
void register_ops(py::module_& m) { (void)m; }
}  // namespace gsc
