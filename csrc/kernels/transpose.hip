// bf16 2-D transpose: out[c, r] = x[r, c]  (x: [R, C] with row stride ldx).
//
// Why it exists: hipBLASLt's MFMA kernels run 25-40 % faster when both GEMM operands are
// K-contiguous ("TN").  A Linear layer's weight gradient dW = dY^T X reduces over the token
// dimension, which is the *strided* dimension of both row-major activations, and its input
// gradient dX = dY W reads W along its strided dimension.  Transposing dY / X / W into
// K-contiguous copies costs one streaming read + write each, far less than the GEMM time it
// buys back on the big layers (tools/bench_gemm_layouts.py, profiles/).
#include "common.h"

namespace dtg {

// Register-blocked: no LDS, no barrier.  Every lane moves one 8 x 8 block -- eight 16-B row
// loads, an in-register transpose (transpose8x8), eight 16-B column stores -- and a wave's 64
// lanes cover a 64 x 64 tile (4 waves: 128 x 128 per workgroup).  Eight lanes read 128
// contiguous bytes of one input row per load instruction, and eight lanes write 128 contiguous
// bytes of one output row per store instruction.  Against the LDS-tiled kernels it replaced
// (64 x 64 and 128 x 128 tiles, removed in round 6): +2 % on [T, 4096], +12 % on [T, 28672]
// (profiles/r5/transpose/).
__global__ __launch_bounds__(256) void transpose_bf16_reg_kernel(const uint16_t* __restrict__ x, int64_t ldx,
                                                                 uint16_t* __restrict__ out, int64_t R, int64_t C) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.y * 128 + (w >> 1) * 64 + (lane >> 3) * 8;  // this lane's first input row
  const int64_t c = (int64_t)blockIdx.x * 128 + (w & 1) * 64 + (lane & 7) * 8;    // and first input column
  if (r >= R || c >= C) return;  // R and C are multiples of 8: a block is wholly in or out
  u16x8 v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const u16x8*>(x + (r + i) * ldx + c);
  transpose8x8(v);
#pragma unroll
  for (int j = 0; j < 8; ++j) *reinterpret_cast<u16x8*>(out + (c + j) * R + r) = v[j];
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
  transpose_bf16_reg_kernel<<<tile_grid((R + 127) / 128, (C + 127) / 128), 256, 0, stream()>>>(
      bf16_ptr(x), x.stride(0), bf16_mut(out), R, C);
  DTG_LAUNCH_CHECK();
  return out;
}

// Many matrices of one flat buffer in ONE launch: out[dst_off + c * R + r] = x[src_off + r * C + c]
// for every row (src_off, R, C, dst_off, tile0) of `mats` (int64 [n, 5], on the GPU), in 64 x 64
// tiles numbered from tile0.  ZeRO's replicated weights land by bucket (the parameter all-gather);
// one launch per bucket writes the W^T copies the backward's dX GEMMs read (parallel/
// data_parallel.py), instead of one launch per matrix inside the backward.
struct TMat {
  int64_t src, rows, cols, dst, tile0;
};

__global__ __launch_bounds__(256) void transpose_mats_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ out,
                                                             const TMat* __restrict__ mats, int nmats) {
  constexpr int TR = 64, TC = 64, P = TC + 2, LV = TR * TC / 8 / 256, VPR = TC / 8, VPC = TR / 8;
  __shared__ uint16_t tile[TR * P];
  const int64_t t = blockIdx.x;
  int lo = 0, hi = nmats - 1;  // the matrix whose tile range holds t
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (mats[mid].tile0 <= t) lo = mid; else hi = mid - 1;
  }
  const TMat m = mats[lo];
  const int64_t lt = t - m.tile0, ctiles = (m.cols + TC - 1) / TC;
  const int64_t r0 = (lt / ctiles) * TR, c0 = (lt % ctiles) * TC;
  const uint16_t* src = x + m.src;
  uint16_t* dst = out + m.dst;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < LV; ++i) {
    const int id = tid + 256 * i;
    const int lr = id / VPR, lc = (id % VPR) * 8;
    const int64_t r = r0 + lr, c = c0 + lc;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r < m.rows && c < m.cols) v = *reinterpret_cast<const u16x8*>(src + r * m.cols + c);
    uint32_t* d = reinterpret_cast<uint32_t*>(tile + lr * P + lc);
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = (uint32_t)v[2 * j] | ((uint32_t)v[2 * j + 1] << 16);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < LV; ++i) {
    const int id = tid + 256 * i;
    const int oc = id / VPC, orr = (id % VPC) * 8;
    const int64_t c = c0 + oc, r = r0 + orr;
    u16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = tile[(orr + j) * P + oc];
    if (c < m.cols && r < m.rows) *reinterpret_cast<u16x8*>(dst + c * m.rows + r) = v;
  }
}

void transpose_mats_(const at::Tensor& x, const at::Tensor& out, const at::Tensor& mats, const at::Tensor& mats_host,
                     int64_t ntiles) {
  DTG_CHECK_CUDA_BF16(x);
  DTG_CHECK_CUDA_BF16(out);
  DTG_CHECK(x.is_contiguous() && out.is_contiguous(), "transpose_mats_: flat buffers must be contiguous");
  DTG_CHECK(mats.is_cuda() && mats.scalar_type() == at::kLong && mats.dim() == 2 && mats.size(1) == 5 &&
                mats.is_contiguous(), "transpose_mats_: mats must be int64 [n, 5] on the GPU");
  DTG_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
            "transpose_mats_: buffers must be 16-byte aligned");
  const int nm = (int)mats.size(0);
  if (nm == 0 || ntiles == 0) return;
  // Host-side bounds check of the descriptors (a bad offset would fault on the GPU), on the
  // caller's host copy of them: no device -> host copy in the hot path.
  DTG_CHECK(mats_host.device().is_cpu() && mats_host.scalar_type() == at::kLong && mats_host.is_contiguous() &&
                mats_host.sizes() == mats.sizes(), "transpose_mats_: mats_host must be the CPU copy of mats");
  const int64_t* d = mats_host.data_ptr<int64_t>();
  int64_t tiles = 0;
  for (int i = 0; i < nm; ++i) {
    const int64_t so = d[5 * i], R = d[5 * i + 1], C = d[5 * i + 2], dof = d[5 * i + 3], t0 = d[5 * i + 4];
    DTG_CHECK(R % 8 == 0 && C % 8 == 0 && so % 8 == 0 && dof % 8 == 0, "transpose_mats_: matrix ", i,
              " needs dims / offsets that are multiples of 8");
    DTG_CHECK(so >= 0 && so + R * C <= x.numel() && dof >= 0 && dof + R * C <= out.numel(),
              "transpose_mats_: matrix ", i, " out of range");
    DTG_CHECK(t0 == tiles, "transpose_mats_: tile0 of matrix ", i, " must follow the previous matrix");
    tiles += ((R + 63) / 64) * ((C + 63) / 64);
  }
  DTG_CHECK(tiles == ntiles, "transpose_mats_: ntiles does not match the descriptors");
  const c10::DeviceGuard g(x.device());
  transpose_mats_kernel<<<dim3((unsigned)ntiles), 256, 0, stream()>>>(
      bf16_ptr(x), bf16_mut(out), reinterpret_cast<const TMat*>(mats.data_ptr<int64_t>()), nm);
  DTG_LAUNCH_CHECK();
}

TORCH_LIBRARY_IMPL(dtg, CUDA, m) {
  m.impl("transpose2d", &transpose2d);
  m.impl("transpose_mats_", &transpose_mats_);
}

}  // namespace dtg
