// Bindings for the model hot-path kernels (normalisation / activation / GEMM).
#include <torch/extension.h>

#include "dla_bindings.h"

namespace dla {

void bind_nn(pybind11::module& m) { (void)m; }

}  // namespace dla
