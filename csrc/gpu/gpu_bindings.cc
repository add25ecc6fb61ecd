#include <pybind11/pybind11.h>

#include "gpu/gpu_api.h"

namespace py = pybind11;

void register_gpu_bindings(PyObject* module) {
  py::module_ m = py::reinterpret_borrow<py::module_>(module);
  (void)m;
}
