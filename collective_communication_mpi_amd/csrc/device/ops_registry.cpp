// Collects every op family's pybind registration.
#include "ops.hpp"

namespace ccmpi {
namespace dev {

void register_layout_ops(pybind11::module_& m);
void register_gemm_ops(pybind11::module_& m);
void register_attn_ops(pybind11::module_& m);
void register_head_ops(pybind11::module_& m);
void register_wgrad_ops(pybind11::module_& m);
void register_swiglu_ops(pybind11::module_& m);

void register_ops(pybind11::module_& m) {
  register_layout_ops(m);
  register_gemm_ops(m);
  register_attn_ops(m);
  register_head_ops(m);
  register_wgrad_ops(m);
  register_swiglu_ops(m);
}

}  // namespace dev
}  // namespace ccmpi
