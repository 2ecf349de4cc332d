// SwiGLU on the fused gate|up projection output.
//
//   gu = x @ [W_gate; W_up]^T   ->  [T, 2I]  (gate = gu[:, :I], up = gu[:, I:])
//   h  = silu(gate) * up        ->  [T, I]
//
// One fused GEMM replaces the two HF Linear calls; this kernel reads gu once and writes h
// once (forward) and reads dh + gu once to write dgu (backward).  f32 math, one rounding.
#include <cstdlib>

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
// One workgroup owns a 64-token x 64-feature tile: 16-byte row loads of g, u, dh; the three
// transposed tiles are staged through LDS (pitch 66 halfwords) and stored as 16-byte columns.
namespace {
constexpr int kSgTile = 64;  // features per workgroup
constexpr int kSgPitch = kSgTile + 2;
}  // namespace

// TT tokens x 64 features per workgroup.  TT = 64 stores the transposed tiles as 128-byte
// row segments, TT = 128 as 256-byte segments (twice the LDS: 3 x 128 x 66 halfwords).
template <int TT>
__global__ __launch_bounds__(256) void swiglu_bwd_t_kernel(
    const uint16_t* __restrict__ dh, const uint16_t* __restrict__ gu, int64_t gu_stride,
    uint16_t* __restrict__ dgu, uint16_t* __restrict__ dguT, uint16_t* __restrict__ hT, int64_t T, int I, int gc) {
  static_assert(TT == 64 || TT == 128, "token tile");
  __shared__ uint16_t s_dg[TT * kSgPitch];
  __shared__ uint16_t s_du[TT * kSgPitch];
  __shared__ uint16_t s_h[TT * kSgPitch];
  int64_t rt, ct;
  tile_coords(gc, (T + TT - 1) / TT, (I + kSgTile - 1) / kSgTile, rt, ct);
  const int64_t t0 = rt * TT;
  const int c0 = (int)ct * kSgTile;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < TT / 32; ++i) {
    const int lt = (tid >> 3) + 32 * i;
    const int lc = (tid & 7) * 8;
    const int64_t t = t0 + lt;
    const int c = c0 + lc;
    float g[8], u[8], d[8];
    u16x8 vdg = {0, 0, 0, 0, 0, 0, 0, 0}, vdu = vdg, vh = vdg;
    if (t < T && c < I) {
      load8(gu + t * gu_stride + c, g);
      load8(gu + t * gu_stride + I + c, u);
      load8(dh + t * I + c, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float sg = sigmoidf_(g[j]);
        const float silu = g[j] * sg;
        vdu[j] = f2bf(d[j] * silu);
        vdg[j] = f2bf(d[j] * u[j] * sg * (1.f + g[j] * (1.f - sg)));
        vh[j] = f2bf(silu * u[j]);
      }
      *reinterpret_cast<u16x8*>(dgu + t * 2 * I + c) = vdg;
      *reinterpret_cast<u16x8*>(dgu + t * 2 * I + I + c) = vdu;
    }
    uint32_t* a = reinterpret_cast<uint32_t*>(s_dg + lt * kSgPitch + lc);
    uint32_t* b = reinterpret_cast<uint32_t*>(s_du + lt * kSgPitch + lc);
    uint32_t* h = reinterpret_cast<uint32_t*>(s_h + lt * kSgPitch + lc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] = (uint32_t)vdg[2 * j] | ((uint32_t)vdg[2 * j + 1] << 16);
      b[j] = (uint32_t)vdu[2 * j] | ((uint32_t)vdu[2 * j + 1] << 16);
      h[j] = (uint32_t)vh[2 * j] | ((uint32_t)vh[2 * j + 1] << 16);
    }
  }
  __syncthreads();
  constexpr int kVecPerRow = TT / 8;          // 16-byte vectors per transposed row segment
  constexpr int kRowsPerIter = 256 / kVecPerRow;
#pragma unroll
  for (int i = 0; i < kSgTile / kRowsPerIter; ++i) {
    const int oc = tid / kVecPerRow + kRowsPerIter * i;  // feature within the tile -> output row
    const int ot = (tid % kVecPerRow) * 8;               // first token of this 8-token vector
    const int c = c0 + oc;
    const int64_t t = t0 + ot;
    if (c >= I || t >= T) continue;
    u16x8 a, b, h;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = s_dg[(ot + j) * kSgPitch + oc];
      b[j] = s_du[(ot + j) * kSgPitch + oc];
      h[j] = s_h[(ot + j) * kSgPitch + oc];
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
  // DTG_SWIGLU_TT=64|128: token tile (A/B knob; see the kernel comment)
  const char* tt_env = std::getenv("DTG_SWIGLU_TT");  // read per call: tests switch it in-process
  const int tt = (tt_env && std::atoi(tt_env) == 128) ? 128 : 64;
  const int gc = tile_group_env(kDefaultTileGroup);
  const dim3 grid = tile_grid(gc, (T + tt - 1) / tt, (I + kSgTile - 1) / kSgTile);
  if (tt == 128)
    swiglu_bwd_t_kernel<128><<<grid, 256, 0, stream()>>>(bf16_ptr(dh), bf16_ptr(gu), gu.stride(0), bf16_mut(dgu),
                                                         bf16_mut(dguT), bf16_mut(hT), T, I, gc);
  else
    swiglu_bwd_t_kernel<64><<<grid, 256, 0, stream()>>>(bf16_ptr(dh), bf16_ptr(gu), gu.stride(0), bf16_mut(dgu),
                                                        bf16_mut(dguT), bf16_mut(hT), T, I, gc);
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
