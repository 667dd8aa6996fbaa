// Non-collective device kernels exposed to Python (layout transforms for the
// TP collects, fused epilogues, MFMA GEMM).  Each op is registered on the
// `_device` module by register_ops().
#pragma once

#include <pybind11/pybind11.h>

namespace ccmpi {
namespace dev {

void register_ops(pybind11::module_& m);

}  // namespace dev
}  // namespace ccmpi
