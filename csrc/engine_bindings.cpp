// torch.ops.tpamd.* registrations for the fused conv/GEMM engine kernels.
#include <torch/library.h>
#include <ATen/ATen.h>
#include "tp_launchers.h"

void register_engine_ops_def(torch::Library& m) {}
void register_engine_ops_impl(torch::Library& m) {}
