// Host-side API of the GPU runtime (csrc/gpu/*.hip.cc, csrc/kernels/*.hip).
#pragma once
#include <Python.h>

void register_gpu_bindings(PyObject* module);
