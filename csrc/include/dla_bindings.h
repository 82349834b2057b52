// Shared declarations between the binding translation units.
#pragma once
#include <torch/extension.h>
#include <hip/hip_runtime.h>

namespace dla {
int dtype_code(const at::Tensor& t);
hipStream_t current_stream(const at::Tensor& t);

void bind_ops(pybind11::module& m);
void bind_nn(pybind11::module& m);
void bind_comm(pybind11::module& m);
}  // namespace dla
