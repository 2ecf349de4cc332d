// SwiGLU on the fused gate|up projection output.
//
//   gu = x @ [W_gate; W_up]^T   ->  [T, 2I]  (gate = gu[:, :I], up = gu[:, I:])
//   h  = silu(gate) * up        ->  [T, I]
//
// One fused GEMM replaces the two HF Linear calls; this kernel reads gu once and writes h
// once (forward) and reads dh + gu once to write dgu (backward).  f32 math, one rounding.
#include <cstdlib>
#include <cstring>

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
// halfwords) and stored as 16-byte columns (TT x 2-byte segments of TF feature rows).  Segment
// length is what the tile shape buys: 128-byte segments (64 x 64) leave HBM well short of its
// streaming rate, 256-byte ones recover most of it (the adamw_t_ tile measurements, r3_s07).
template <int TT, int TF>
__global__ __launch_bounds__(256) void swiglu_bwd_t_kernel(
    const uint16_t* __restrict__ dh, const uint16_t* __restrict__ gu, int64_t gu_stride,
    uint16_t* __restrict__ dgu, uint16_t* __restrict__ dguT, uint16_t* __restrict__ hT, int64_t T, int I, int gc) {
  static_assert((TT == 64 || TT == 128) && (TF == 64 || TF == 128), "tile");
  constexpr int kPitch = TF + 2;
  constexpr int kVF = TF / 8;                 // 16-byte vectors per token row of the tile
  constexpr int kRowsPerPass = 256 / kVF;     // token rows per phase-1 pass
  constexpr int kVT = TT / 8;                 // 16-byte vectors per transposed row segment
  constexpr int kOutPerPass = 256 / kVT;      // feature rows per phase-2 pass
  extern __shared__ uint16_t smem[];
  uint16_t* s_dg = smem;
  uint16_t* s_du = smem + TT * kPitch;
  uint16_t* s_h = smem + 2 * TT * kPitch;
  int64_t rt, ct;
  tile_coords(gc, (T + TT - 1) / TT, (I + TF - 1) / TF, rt, ct);
  const int64_t t0 = rt * TT;
  const int c0 = (int)ct * TF;
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

// Register-blocked form (DTG_SWIGLU_TILE=reg): no LDS.  Every lane owns an 8-token x 8-feature
// block -- 16-B row loads of g, u and dh, f32 math, 16-B row stores of dg and du, then the three
// transposed outputs through an in-register 8 x 8 transpose (transpose8x8) as 16-B column stores.
// A wave's 64 lanes cover 64 tokens x 64 features (8 lanes per 128 contiguous bytes of every row
// they load or store); 4 waves per workgroup cover 128 x 128.
__global__ __launch_bounds__(256) void swiglu_bwd_t_reg_kernel(
    const uint16_t* __restrict__ dh, const uint16_t* __restrict__ gu, int64_t gu_stride,
    uint16_t* __restrict__ dgu, uint16_t* __restrict__ dguT, uint16_t* __restrict__ hT, int64_t T, int I, int gc) {
  int64_t rt, ct;
  tile_coords(gc, (T + 127) / 128, (I + 127) / 128, rt, ct);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t t0 = rt * 128 + (w >> 1) * 64 + (lane >> 3) * 8;  // first token of this lane's block
  const int c0 = (int)ct * 128 + (w & 1) * 64 + (lane & 7) * 8;    // and first feature
  if (t0 >= T || c0 >= I) return;  // T and I are multiples of 8: a block is wholly in or out
  u16x8 vg[8], vu[8], vd[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint16_t* row = gu + (t0 + i) * gu_stride + c0;
    vg[i] = *reinterpret_cast<const u16x8*>(row);
    vu[i] = *reinterpret_cast<const u16x8*>(row + I);
    vd[i] = *reinterpret_cast<const u16x8*>(dh + (t0 + i) * I + c0);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    u16x8 dg, du, h;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float g = bf2f(vg[i][j]), u = bf2f(vu[i][j]), d = bf2f(vd[i][j]);
      const float sg = sigmoidf_(g);
      const float silu = g * sg;
      du[j] = f2bf(d * silu);
      dg[j] = f2bf(d * u * sg * (1.f + g * (1.f - sg)));
      h[j] = f2bf(silu * u);
    }
    uint16_t* o = dgu + (t0 + i) * 2 * I + c0;
    *reinterpret_cast<u16x8*>(o) = dg;
    *reinterpret_cast<u16x8*>(o + I) = du;
    vg[i] = dg;  // the inputs of row i are dead: reuse their registers for the outputs
    vu[i] = du;
    vd[i] = h;
  }
  transpose8x8(vg);
  transpose8x8(vu);
  transpose8x8(vd);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    *reinterpret_cast<u16x8*>(dguT + (int64_t)(c0 + j) * T + t0) = vg[j];
    *reinterpret_cast<u16x8*>(dguT + (int64_t)(I + c0 + j) * T + t0) = vu[j];
    *reinterpret_cast<u16x8*>(hT + (int64_t)(c0 + j) * T + t0) = vd[j];
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
  // DTG_SWIGLU_TILE = TTxTF (64x64 | 64x128 | 128x64 | 128x128): token x feature tile (A/B knob;
  // read per call so tests and benchmarks switch it in-process)
  // Default 64 x 128: -2.1 ms per 8B step against 64 x 64, three alternating same-box pairs
  // (profiles/r3_s32; the parser had dropped "64x128" before, so round 3's first A/B never ran it).
  const char* te = std::getenv("DTG_SWIGLU_TILE");
  int tt = 64, tf = 128;
  if (te) {
    if (!std::strcmp(te, "64x64")) tt = 64, tf = 64;
    else if (!std::strcmp(te, "64x128")) tt = 64, tf = 128;
    else if (!std::strcmp(te, "128x64")) tt = 128, tf = 64;
    else if (!std::strcmp(te, "128x128")) tt = 128, tf = 128;
  }
  const int gc = tile_group_env(kDefaultTileGroup);
  if (te && !std::strcmp(te, "reg")) {
    swiglu_bwd_t_reg_kernel<<<tile_grid(gc, (T + 127) / 128, (I + 127) / 128), 256, 0, stream()>>>(
        bf16_ptr(dh), bf16_ptr(gu), gu.stride(0), bf16_mut(dgu), bf16_mut(dguT), bf16_mut(hT), T, I, gc);
    DTG_LAUNCH_CHECK();
    return {dgu, dguT, hT};
  }
  const dim3 grid = tile_grid(gc, (T + tt - 1) / tt, (I + tf - 1) / tf);
  const size_t lds = 3 * (size_t)tt * (tf + 2) * sizeof(uint16_t);
#define DTG_SG_LAUNCH(TT_, TF_)                                                                            \
  do {                                                                                                     \
    auto fn = swiglu_bwd_t_kernel<TT_, TF_>;                                                               \
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
    fn<<<grid, 256, lds, stream()>>>(bf16_ptr(dh), bf16_ptr(gu), gu.stride(0), bf16_mut(dgu), bf16_mut(dguT),  \
                                     bf16_mut(hT), T, I, gc);                                              \
  } while (0)
  if (tt == 64 && tf == 64) DTG_SG_LAUNCH(64, 64);
  else if (tt == 64) DTG_SG_LAUNCH(64, 128);
  else if (tf == 64) DTG_SG_LAUNCH(128, 64);
  else DTG_SG_LAUNCH(128, 128);
#undef DTG_SG_LAUNCH
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
