// Host AdamW for FSDP CPU offload (the 405B chapter's `--cpu-offload on`).
//
// With offload the parameter, gradient and optimizer-state shards live in pinned host memory
// and the update runs on the CPU while the GPU is idle between steps.  This kernel streams the
// four buffers once with OpenMP threads; bf16 is widened/narrowed with integer shifts in
// 16-element blocks so the compiler vectorises the f32 math (AVX2/AVX-512 under
// -march=x86-64-v3).  Same update order as the GPU kernel / torch fused AdamW.
#include <ATen/ATen.h>
#include <torch/library.h>

#include "cpu/adamw_host.h"

namespace dtg {
namespace {

using host::adamw_host;

void adamw_cpu_(const at::Tensor& p, const at::Tensor& g, const at::Tensor& m, const at::Tensor& v, double lr,
                double beta1, double beta2, double eps, double wd, int64_t step, double grad_scale) {
  TORCH_CHECK(p.device().is_cpu() && g.device().is_cpu() && m.device().is_cpu() && v.device().is_cpu(),
              "adamw_cpu_: all buffers must be host tensors");
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous(),
              "adamw_cpu_: buffers must be contiguous");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adamw_cpu_: size mismatch");
  const float bc1 = 1.0 - std::pow(beta1, (double)step);
  const float bc2s = std::sqrt(1.0 - std::pow(beta2, (double)step));
  auto isbf = [](const at::Tensor& t) { return t.scalar_type() == at::kBFloat16; };
  auto isf = [](const at::Tensor& t) { return t.scalar_type() == at::kFloat; };
  TORCH_CHECK((isbf(p) || isf(p)) && (isbf(g) || isf(g)) && (isbf(m) || isf(m)) && m.scalar_type() == v.scalar_type(),
              "adamw_cpu_: bf16/f32 only");
#define DTG_HOST_ADAM(PT, GT, ST)                                                                              \
  adamw_host<PT, GT, ST>(reinterpret_cast<PT*>(p.data_ptr()), reinterpret_cast<const GT*>(g.data_ptr()),     \
                         reinterpret_cast<ST*>(m.data_ptr()), reinterpret_cast<ST*>(v.data_ptr()), n, lr, beta1, \
                         beta2, eps, wd, bc1, bc2s, grad_scale)
  if (isbf(p) && isbf(g) && isbf(m)) DTG_HOST_ADAM(uint16_t, uint16_t, uint16_t);
  else if (isbf(p) && isbf(g)) DTG_HOST_ADAM(uint16_t, uint16_t, float);
  else if (isbf(p) && isbf(m)) DTG_HOST_ADAM(uint16_t, float, uint16_t);
  else if (isbf(p)) DTG_HOST_ADAM(uint16_t, float, float);
  else if (isbf(g) && isbf(m)) DTG_HOST_ADAM(float, uint16_t, uint16_t);
  else if (isbf(g)) DTG_HOST_ADAM(float, uint16_t, float);
  else if (isbf(m)) DTG_HOST_ADAM(float, float, uint16_t);
  else DTG_HOST_ADAM(float, float, float);
#undef DTG_HOST_ADAM
}

}  // namespace

TORCH_LIBRARY_IMPL(dtg, CPU, m) { m.impl("adamw_cpu_", &adamw_cpu_); }

}  // namespace dtg
