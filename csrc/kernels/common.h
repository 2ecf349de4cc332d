// Shared device helpers for the gfx950 (CDNA4) kernels of this framework.
//
// Conventions
//  * bf16 tensors are handled as raw 16-bit words (uint16_t) in global memory and
//    widened to f32 in registers; every kernel accumulates in f32.
//  * Memory-bound kernels move 16 B per lane (8 x bf16) per access (CDNA guide G13).
//  * Wave size is 64 and is hard-coded (gfx950 has no wave32 mode for compute).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

namespace dtg {

constexpr int kWave = 64;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

// Round-to-nearest-even f32 -> bf16; hipcc lowers the cast to v_cvt_pk_bf16_f32 on gfx950
// (NaN stays NaN, unlike integer-trick rounding: MI355X microarch "Correctness boundaries").
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ void load8(const uint16_t* p, float* out) {
  u16x8 v = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = bf2f(v[i]);
}

__device__ __forceinline__ void store8(uint16_t* p, const float* in) {
  u16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = f2bf(in[i]);
  *reinterpret_cast<u16x8*>(p) = v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `scratch` must hold blockDim.x/64 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}

__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, scratch[i]);
  return r;
}

inline hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

inline const uint16_t* bf16_ptr(const at::Tensor& t) {
  return reinterpret_cast<const uint16_t*>(t.data_ptr());
}
inline uint16_t* bf16_mut(const at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

#define DTG_CHECK(cond, ...) TORCH_CHECK(cond, "dtg: ", __VA_ARGS__)
#define DTG_CHECK_CUDA_BF16(t)                                                     \
  DTG_CHECK((t).is_cuda() && (t).scalar_type() == at::kBFloat16, #t " must be a bf16 GPU tensor")
#define DTG_LAUNCH_CHECK() C10_HIP_KERNEL_LAUNCH_CHECK()

// 8 x 8 transpose of 16-bit values held in registers: v[i] = row i on entry, column i on exit.
// Three butterfly stages (elements, pairs, quads); only the first needs byte permutes, the other
// two move whole dwords.
__device__ __forceinline__ void transpose8x8(u16x8 (&v)[8]) {
  u16x8 t[8], u[8];
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    t[i] = __builtin_shufflevector(v[i], v[i + 1], 0, 8, 2, 10, 4, 12, 6, 14);
    t[i + 1] = __builtin_shufflevector(v[i], v[i + 1], 1, 9, 3, 11, 5, 13, 7, 15);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = (k & 1) + 4 * (k >> 1);  // 0, 1, 4, 5
    u[i] = __builtin_shufflevector(t[i], t[i + 2], 0, 1, 8, 9, 4, 5, 12, 13);
    u[i + 2] = __builtin_shufflevector(t[i], t[i + 2], 2, 3, 10, 11, 6, 7, 14, 15);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = __builtin_shufflevector(u[i], u[i + 4], 0, 1, 2, 3, 8, 9, 10, 11);
    v[i + 4] = __builtin_shufflevector(u[i], u[i + 4], 4, 5, 6, 7, 12, 13, 14, 15);
  }
}

// Grid of the tile-transposing streaming kernels: blockIdx.x = column tile (fastest, so the
// workgroups resident at one time read neighbouring segments of the same source rows),
// blockIdx.y = row tile.  A banded 1-D tile walk (column tiles grouped so that the transposed
// output rows are written in long runs) gained 4-8 % on a lone [T, 28672] transpose, was mixed
// on the SwiGLU backward and moved the 8B step < 0.5 % (profiles/r1/s62_tile_order_ab.md); it
// was removed in round 6 with the other opt-in tilings.
inline dim3 tile_grid(int64_t n_row_tiles, int64_t n_col_tiles) {
  DTG_CHECK(n_row_tiles <= 65535 && n_col_tiles < (int64_t(1) << 31), "tile grid: too many tiles");
  return dim3((unsigned)n_col_tiles, (unsigned)n_row_tiles);
}

}  // namespace dtg
