// bf16 2-D transpose through LDS: out[c, r] = x[r, c]  (x: [R, C] with row stride ldx).
//
// Why it exists: hipBLASLt's MFMA kernels run 25-40 % faster when both GEMM operands are
// K-contiguous ("TN").  A Linear layer's weight gradient dW = dY^T X reduces over the token
// dimension, which is the *strided* dimension of both row-major activations, and its input
// gradient dX = dY W reads W along its strided dimension.  Transposing dY / X / W into
// K-contiguous copies costs one streaming read + write each, far less than the GEMM time it
// buys back on the big layers (tools/bench_gemm_layouts.py, profiles/).
//
// Tile: 64 rows x 64 columns (8 KB) per 256-thread workgroup.  Loads and stores are 16 B per
// lane (8 bf16) along the contiguous dimension of each side; the LDS tile is padded by one
// dword per row so the column-wise LDS gathers of the store phase spread over the banks.
#include "common.h"

namespace dtg {

namespace {
constexpr int kTile = 64;
constexpr int kPitch = kTile + 2;  // halfwords per LDS row (33 dwords: odd -> conflict-free columns)
}  // namespace

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const uint16_t* __restrict__ x, int64_t ldx,
                                                             uint16_t* __restrict__ out, int64_t R, int64_t C) {
  __shared__ uint16_t tile[kTile * kPitch];
  const int64_t r0 = (int64_t)blockIdx.y * kTile;
  const int64_t c0 = (int64_t)blockIdx.x * kTile;
  const int tid = threadIdx.x;
  // Load phase: 64 rows x 8 vectors of 8; thread -> (row = tid / 8 + 32 * i, vec = tid % 8).
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int lr = (tid >> 3) + 32 * i;
    const int lc = (tid & 7) * 8;
    const int64_t r = r0 + lr, c = c0 + lc;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r < R && c < C) v = *reinterpret_cast<const u16x8*>(x + r * ldx + c);
    uint32_t* dst = reinterpret_cast<uint32_t*>(tile + lr * kPitch + lc);
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[j] = (uint32_t)v[2 * j] | ((uint32_t)v[2 * j + 1] << 16);
  }
  __syncthreads();
  // Store phase: output row = input column (64 of them), 8 vectors of 8 input rows each.
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int oc = (tid >> 3) + 32 * i;   // input column within the tile
    const int orr = (tid & 7) * 8;        // first input row of this vector
    const int64_t c = c0 + oc, r = r0 + orr;
    u16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = tile[(orr + j) * kPitch + oc];
    if (c < C && r < R) *reinterpret_cast<u16x8*>(out + c * R + r) = v;
  }
}

at::Tensor transpose2d(const at::Tensor& x) {
  DTG_CHECK_CUDA_BF16(x);
  DTG_CHECK(x.dim() == 2 && x.stride(1) == 1, "transpose2d: x must be 2-D with unit column stride");
  const int64_t R = x.size(0), C = x.size(1);
  DTG_CHECK(R % 8 == 0 && C % 8 == 0 && x.stride(0) % 8 == 0,
            "transpose2d: both dims and the row stride must be multiples of 8 (16-byte vectors)");
  DTG_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "transpose2d: x must be 16-byte aligned");
  const c10::DeviceGuard g(x.device());
  auto out = at::empty({C, R}, x.options());
  if (R == 0 || C == 0) return out;
  const dim3 grid((C + kTile - 1) / kTile, (R + kTile - 1) / kTile);
  DTG_CHECK(grid.y <= 65535, "transpose2d: too many rows");
  transpose_bf16_kernel<<<grid, 256, 0, stream()>>>(bf16_ptr(x), x.stride(0), bf16_mut(out), R, C);
  DTG_LAUNCH_CHECK();
  return out;
}

TORCH_LIBRARY_IMPL(dtg, CUDA, m) { m.impl("transpose2d", &transpose2d); }

}  // namespace dtg
