// Registry of HIP op launchers exposed to Python.
#include <pybind11/pybind11.h>
namespace py = pybind11;
namespace gsc {
void register_explore(py::module_& m);
void register_gnn(py::module_& m);
void register_optim(py::module_& m);
void register_mlp(py::module_& m);
void register_streams(py::module_& m);
void register_replay(py::module_& m);
void register_gnn_lw(py::module_& m);
void register_actor_proj(py::module_& m);
void register_sparse_act(py::module_& m);
void register_ops(py::module_& m) {
  register_explore(m);
  register_gnn(m);
  register_optim(m);
  register_mlp(m);
  register_streams(m);
  register_replay(m);
  register_gnn_lw(m);
  register_actor_proj(m);
  register_sparse_act(m);
}
}  // namespace gsc
