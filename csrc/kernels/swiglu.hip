// SwiGLU on the fused gate|up projection output.
//
//   gu = x @ [W_gate; W_up]^T   ->  [T, 2I]  (gate = gu[:, :I], up = gu[:, I:])
//   h  = silu(gate) * up        ->  [T, I]
//
// One fused GEMM replaces the two HF Linear calls; this kernel reads gu once and writes h
// once (forward) and reads dh + gu once to write dgu (backward).  f32 math, one rounding.
#include "common.h"

namespace dtg {

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

__global__ void swiglu_fwd_kernel(const uint16_t* __restrict__ gu, int64_t gu_stride,
                                  uint16_t* __restrict__ h, int64_t T, int I) {
  const int chunks = I >> 3;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= T * chunks) return;
  const int64_t t = gid / chunks;
  const int c = (gid % chunks) * 8;
  float g[8], u[8], o[8];
  load8(gu + t * gu_stride + c, g);
  load8(gu + t * gu_stride + I + c, u);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = g[j] * sigmoidf_(g[j]) * u[j];
  store8(h + t * I + c, o);
}

__global__ void swiglu_bwd_kernel(const uint16_t* __restrict__ dh, const uint16_t* __restrict__ gu,
                                  int64_t gu_stride, uint16_t* __restrict__ dgu, int64_t T, int I) {
  const int chunks = I >> 3;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= T * chunks) return;
  const int64_t t = gid / chunks;
  const int c = (gid % chunks) * 8;
  float g[8], u[8], d[8], dg[8], du[8];
  load8(gu + t * gu_stride + c, g);
  load8(gu + t * gu_stride + I + c, u);
  load8(dh + t * I + c, d);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float s = sigmoidf_(g[j]);
    const float silu = g[j] * s;
    du[j] = d[j] * silu;
    dg[j] = d[j] * u[j] * s * (1.f + g[j] * (1.f - s));
  }
  store8(dgu + t * 2 * I + c, dg);
  store8(dgu + t * 2 * I + I + c, du);
}

at::Tensor swiglu_fwd(const at::Tensor& gu) {
  DTG_CHECK_CUDA_BF16(gu);
  DTG_CHECK(gu.dim() == 2 && gu.stride(1) == 1 && gu.stride(0) % 8 == 0 && gu.size(1) % 16 == 0,
            "swiglu: gu must be [T, 2I] with I % 8 == 0");
  const int64_t T = gu.size(0);
  const int I = gu.size(1) / 2;
  const c10::DeviceGuard g(gu.device());
  auto h = at::empty({T, I}, gu.options());
  const int64_t n = T * (I / 8);
  if (n == 0) return h;
  swiglu_fwd_kernel<<<(n + 255) / 256, 256, 0, stream()>>>(bf16_ptr(gu), gu.stride(0),
                                                           bf16_mut(h), T, I);
  DTG_LAUNCH_CHECK();
  return h;
}

at::Tensor swiglu_bwd(const at::Tensor& dh_, const at::Tensor& gu) {
  auto dh = dh_.contiguous();
  DTG_CHECK_CUDA_BF16(gu);
  DTG_CHECK_CUDA_BF16(dh);
  const int64_t T = gu.size(0);
  const int I = gu.size(1) / 2;
  DTG_CHECK(dh.size(0) == T && dh.size(1) == I, "swiglu_bwd: shape mismatch");
  const c10::DeviceGuard g(gu.device());
  auto dgu = at::empty({T, 2 * I}, gu.options());
  const int64_t n = T * (I / 8);
  if (n == 0) return dgu;
  swiglu_bwd_kernel<<<(n + 255) / 256, 256, 0, stream()>>>(bf16_ptr(dh), bf16_ptr(gu),
                                                           gu.stride(0), bf16_mut(dgu), T, I);
  DTG_LAUNCH_CHECK();
  return dgu;
}

TORCH_LIBRARY_IMPL(dtg, CUDA, m) {
  m.impl("swiglu_fwd", &swiglu_fwd);
  m.impl("swiglu_bwd", &swiglu_bwd);
}

}  // namespace dtg
