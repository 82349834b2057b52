// Python module entry point: distributed_learning_amd._C
#include "dla_bindings.h"

PYBIND11_MODULE(_C, m) {
  m.doc() = "distributed_learning_amd native extension (gfx950 HIP kernels + RCCL comm engine)";
  m.attr("arch") = "gfx950";
  dla::bind_ops(m);
  dla::bind_nn(m);
  dla::bind_comm(m);
}
