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

// Backward that also emits the operands of the MLP's weight-gradient GEMMs in K-contiguous
// (token-minor) layout, so hipBLASLt runs them as "TN" without separate transpose passes:
//   dgu  [T, 2I]   (row-major, for dX = dgu @ W_gu)
//   dguT [2I, T]   (for dW_gu = dguT @ X)
//   hT   [I, T]    (h = silu(g) * u recomputed from gu, for dW_down = dY^T @ h)
// One workgroup owns a TT-token x TF-feature tile: 16-byte row loads of g, u, dh (TF x 2-byte
// segments of TT token rows); the three transposed tiles are staged through LDS (pitch TF + 2
// halfwords) and stored as 16-byte columns (TT x 2-byte segments of TF feature rows).
// 64 x 128 is the measured best of the 64/128 x 64/128 tiles and of a register-blocked 8 x 8
// form (-2.1 ms per 8B step against 64 x 64, profiles/r3/s32; 4.64 vs 4.52 TB/s against the
// register-blocked one, profiles/r5/transpose/); the others were removed in round 6.  Staging the
// three outputs one after another through a single 16.6 KB buffer doubled the occupancy (6
// instead of 3 waves per SIMD) and changed nothing: 5.53 vs 5.50 TB/s, step 581.0 vs 580.7 ms
// (profiles/r6/swiglu_seq/).
constexpr int kSgTT = 64, kSgTF = 128;

template <int TT, int TF>
__global__ __launch_bounds__(256) void swiglu_bwd_t_kernel(
    const uint16_t* __restrict__ dh, const uint16_t* __restrict__ gu, int64_t gu_stride,
    uint16_t* __restrict__ dgu, uint16_t* __restrict__ dguT, uint16_t* __restrict__ hT, int64_t T, int I) {
  static_assert(TT == 64 && TF == 128, "tile");
  constexpr int kPitch = TF + 2;
  constexpr int kVF = TF / 8;                 // 16-byte vectors per token row of the tile
  constexpr int kRowsPerPass = 256 / kVF;     // token rows per phase-1 pass
  constexpr int kVT = TT / 8;                 // 16-byte vectors per transposed row segment
  constexpr int kOutPerPass = 256 / kVT;      // feature rows per phase-2 pass
  extern __shared__ uint16_t smem[];
  uint16_t* s_dg = smem;
  uint16_t* s_du = smem + TT * kPitch;
  uint16_t* s_h = smem + 2 * TT * kPitch;
  const int64_t t0 = (int64_t)blockIdx.y * TT;
  const int c0 = (int)blockIdx.x * TF;
  const int tid = threadIdx.x;
  // all loads of the tile first (3 x TT*TF/2048 vectors per lane in flight), then the math
  constexpr int kNP = TT / kRowsPerPass;
  u16x8 rg[kNP], ru[kNP], rd[kNP];
#pragma unroll
  for (int i = 0; i < kNP; ++i) {
    const int lt = tid / kVF + kRowsPerPass * i;
    const int lc = (tid % kVF) * 8;
    const int64_t t = t0 + lt;
    const int c = c0 + lc;
    if (t < T && c < I) {
      rg[i] = *reinterpret_cast<const u16x8*>(gu + t * gu_stride + c);
      ru[i] = *reinterpret_cast<const u16x8*>(gu + t * gu_stride + I + c);
      rd[i] = *reinterpret_cast<const u16x8*>(dh + t * I + c);
    }
  }
#pragma unroll
  for (int i = 0; i < kNP; ++i) {
    const int lt = tid / kVF + kRowsPerPass * i;
    const int lc = (tid % kVF) * 8;
    const int64_t t = t0 + lt;
    const int c = c0 + lc;
    u16x8 vdg = {0, 0, 0, 0, 0, 0, 0, 0}, vdu = vdg, vh = vdg;
    if (t < T && c < I) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float g = bf2f(rg[i][j]), u = bf2f(ru[i][j]), d = bf2f(rd[i][j]);
        const float sg = sigmoidf_(g);
        const float silu = g * sg;
        vdu[j] = f2bf(d * silu);
        vdg[j] = f2bf(d * u * sg * (1.f + g * (1.f - sg)));
        vh[j] = f2bf(silu * u);
      }
      *reinterpret_cast<u16x8*>(dgu + t * 2 * I + c) = vdg;
      *reinterpret_cast<u16x8*>(dgu + t * 2 * I + I + c) = vdu;
    }
    uint32_t* a = reinterpret_cast<uint32_t*>(s_dg + lt * kPitch + lc);
    uint32_t* b = reinterpret_cast<uint32_t*>(s_du + lt * kPitch + lc);
    uint32_t* h = reinterpret_cast<uint32_t*>(s_h + lt * kPitch + lc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] = (uint32_t)vdg[2 * j] | ((uint32_t)vdg[2 * j + 1] << 16);
      b[j] = (uint32_t)vdu[2 * j] | ((uint32_t)vdu[2 * j + 1] << 16);
      h[j] = (uint32_t)vh[2 * j] | ((uint32_t)vh[2 * j + 1] << 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < TF / kOutPerPass; ++i) {
    const int oc = tid / kVT + kOutPerPass * i;  // feature within the tile -> output row
    const int ot = (tid % kVT) * 8;              // first token of this 8-token vector
    const int c = c0 + oc;
    const int64_t t = t0 + ot;
    if (c >= I || t >= T) continue;
    u16x8 a, b, h;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = s_dg[(ot + j) * kPitch + oc];
      b[j] = s_du[(ot + j) * kPitch + oc];
      h[j] = s_h[(ot + j) * kPitch + oc];
    }
    *reinterpret_cast<u16x8*>(dguT + (int64_t)c * T + t) = a;
    *reinterpret_cast<u16x8*>(dguT + (int64_t)(I + c) * T + t) = b;
    *reinterpret_cast<u16x8*>(hT + (int64_t)c * T + t) = h;
  }
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> swiglu_bwd_t(const at::Tensor& dh_, const at::Tensor& gu) {
  auto dh = dh_.contiguous();
  DTG_CHECK_CUDA_BF16(gu);
  DTG_CHECK_CUDA_BF16(dh);
  DTG_CHECK(gu.dim() == 2 && gu.stride(1) == 1 && gu.stride(0) % 8 == 0, "swiglu_bwd_t: gu must be [T, 2I] row-major");
  const int64_t T = gu.size(0);
  const int I = gu.size(1) / 2;
  DTG_CHECK(T % 8 == 0 && I % 8 == 0, "swiglu_bwd_t: T and I must be multiples of 8");
  DTG_CHECK(dh.size(0) == T && dh.size(1) == I, "swiglu_bwd_t: shape mismatch");
  const c10::DeviceGuard g(gu.device());
  auto dgu = at::empty({T, 2 * I}, gu.options());
  auto dguT = at::empty({2 * I, T}, gu.options());
  auto hT = at::empty({I, T}, gu.options());
  if (T == 0 || I == 0) return {dgu, dguT, hT};
  const size_t lds = 3 * (size_t)kSgTT * (kSgTF + 2) * sizeof(uint16_t);
  swiglu_bwd_t_kernel<kSgTT, kSgTF><<<tile_grid((T + kSgTT - 1) / kSgTT, (I + kSgTF - 1) / kSgTF), 256, lds, stream()>>>(
      bf16_ptr(dh), bf16_ptr(gu), gu.stride(0), bf16_mut(dgu), bf16_mut(dguT), bf16_mut(hT), T, I);
  DTG_LAUNCH_CHECK();
  return {dgu, dguT, hT};
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
  m.impl("swiglu_bwd_t", &swiglu_bwd_t);
}

}  // namespace dtg
