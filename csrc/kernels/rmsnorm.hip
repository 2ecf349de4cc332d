// RMSNorm (+ fused residual add) forward/backward for gfx950.
//
// Semantics follow the Llama RMSNorm the reference trains through HF transformers
// (SURVEY §2.6 K7): statistics in f32, the normalised activation rounded to the input
// dtype, then multiplied by the weight:  y = bf16(w * bf16(x * rsqrt(mean(x^2) + eps))).
// The fused variant first forms h = bf16(x + residual) (the decoder's residual add,
// SURVEY K11) and normalises h, so one HBM pass replaces two.
//
// Layout: one 256-thread workgroup per row; each lane owns PER 16-byte chunks of the row
// (8 bf16 each) and keeps them in registers between the reduction and the write.  The
// backward writes per-workgroup f32 partials of dw that a second kernel column-reduces
// (no atomics, bitwise reproducible).
#include "common.h"

namespace dtg {

constexpr int kNormThreads = 256;

template <int PER, bool ADD>
__global__ __launch_bounds__(kNormThreads) void rmsnorm_fwd_kernel(
    const uint16_t* __restrict__ x, int64_t x_stride, const uint16_t* __restrict__ res,
    int64_t res_stride, const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
    uint16_t* __restrict__ h_out, float* __restrict__ rstd_out, int H, float eps) {
  __shared__ float scratch[kNormThreads / 64];
  const int row = blockIdx.x;
  const int nch = H >> 3;
  const uint16_t* xr = x + row * x_stride;
  float v[PER][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = threadIdx.x + i * kNormThreads;
    if (c < nch) {
      load8(xr + c * 8, v[i]);
      if constexpr (ADD) {
        float r[8];
        load8(res + row * res_stride + c * 8, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(v[i][j] + r[j]));  // bf16 residual add
        store8(h_out + (int64_t)row * H + c * 8, v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum(ss, scratch);
  const float rstd = rsqrtf(ss / H + eps);
  if (threadIdx.x == 0) rstd_out[row] = rstd;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = threadIdx.x + i * kNormThreads;
    if (c < nch) {
      float wv[8], o[8];
      load8(w + c * 8, wv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = wv[j] * bf2f(f2bf(v[i][j] * rstd));
      store8(y + (int64_t)row * H + c * 8, o);
    }
  }
}

// dx = rstd * (g - n * mean(g * n)),  g = dy * w,  n = x * rstd  (+ dres if given)
// dw_partial[block][col] = sum over this block's rows of dy * bf16(n)
// Rows are software-pipelined: the next row's x / dy / dres vectors are loaded (as raw 16-byte
// words) before the current row's block reduction, so every lane keeps its loads in flight
// across the two barriers of block_sum instead of issuing them after it.
template <int PER, bool DRES>
__global__ __launch_bounds__(kNormThreads) void rmsnorm_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, int64_t x_stride,
    const uint16_t* __restrict__ w, const float* __restrict__ rstd_in,
    const uint16_t* __restrict__ dres, uint16_t* __restrict__ dx, float* __restrict__ dw_part,
    int T, int H, int rows_per_block) {
  __shared__ float scratch[kNormThreads / 64];
  const int nch = H >> 3;
  float dwacc[PER][8];
  float wv[PER][8];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = threadIdx.x + i * kNormThreads;
#pragma unroll
    for (int j = 0; j < 8; ++j) dwacc[i][j] = wv[i][j] = 0.f;
    // Lanes past the row (H not a multiple of 8 * 256, e.g. 3072 for Llama-3.2-3B) keep w = 0:
    // their g = dy * w enters the row's dot product, and an uninitialised register there held
    // NaN/inf often enough to turn whole rows of dx into NaN (rime chapter, profiles/r2_s47).
    if (c < nch) load8(w + c * 8, wv[i]);
  }
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(T, r0 + rows_per_block);
  const u16x8 z{0, 0, 0, 0, 0, 0, 0, 0};
  u16x8 nx[PER], nd[PER], nr[PER];
  auto fetch = [&](int row) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * kNormThreads;
      const bool ok = c < nch && row < r1;
      nx[i] = ok ? *reinterpret_cast<const u16x8*>(x + row * x_stride + c * 8) : z;
      nd[i] = ok ? *reinterpret_cast<const u16x8*>(dy + (int64_t)row * H + c * 8) : z;
      if constexpr (DRES) nr[i] = ok ? *reinterpret_cast<const u16x8*>(dres + (int64_t)row * H + c * 8) : z;
    }
  };
  if (r0 < r1) fetch(r0);
  for (int row = r0; row < r1; ++row) {
    const float rstd = rstd_in[row];
    u16x8 cr[PER];
    float xv[PER][8], g[PER][8];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if constexpr (DRES) cr[i] = nr[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xv[i][j] = bf2f(nx[i][j]);
        const float d = bf2f(nd[i][j]);
        const float n = xv[i][j] * rstd;
        g[i][j] = d * wv[i][j];
        dot += g[i][j] * n;
        dwacc[i][j] += d * bf2f(f2bf(n));
      }
    }
    fetch(row + 1);  // in flight across the reduction below
    dot = block_sum(dot, scratch) / H;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * kNormThreads;
      if (c < nch) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          o[j] = rstd * (g[i][j] - xv[i][j] * rstd * dot);
          if constexpr (DRES) o[j] += bf2f(cr[i][j]);
        }
        store8(dx + (int64_t)row * H + c * 8, o);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = threadIdx.x + i * kNormThreads;
    if (c < nch) {
      float4* dst = reinterpret_cast<float4*>(dw_part + (int64_t)blockIdx.x * H + c * 8);
      dst[0] = make_float4(dwacc[i][0], dwacc[i][1], dwacc[i][2], dwacc[i][3]);
      dst[1] = make_float4(dwacc[i][4], dwacc[i][5], dwacc[i][6], dwacc[i][7]);
    }
  }
}

// Column sums of an [nrows, H] f32 matrix -> bf16 [H].  A workgroup owns 32 columns; its 8
// row-groups of 32 lanes read 128-B row segments (coalesced) and are combined through LDS,
// so the reduction spreads over H/32 workgroups instead of H serial threads.
// Column sums of the [nrows, H] f32 partials, fixed summation order (deterministic).  16 columns
// x 16 row groups per workgroup: H / 16 workgroups (256 at H = 4096, one per CU) each walking
// nrows / 16 rows -- the 32-column form had half the chip idle and twice the dependent-load depth.
constexpr int kColsumCols = 16;
__global__ __launch_bounds__(256) void colsum_to_bf16_kernel(const float* __restrict__ part, int nrows, int H,
                                                             uint16_t* __restrict__ out) {
  constexpr int G = 256 / kColsumCols;
  __shared__ float red[G][kColsumCols + 1];
  const int lane = threadIdx.x % kColsumCols, grp = threadIdx.x / kColsumCols;
  const int c = blockIdx.x * kColsumCols + lane;
  float s = 0.f;
  if (c < H)
    for (int r = grp; r < nrows; r += G) s += part[(int64_t)r * H + c];
  red[grp][lane] = s;
  __syncthreads();
  if (grp == 0 && c < H) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g) t += red[g][lane];
    out[c] = f2bf(t);
  }
}

static int pick_per(int H) {
  const int nch = H / 8;
  const int per = (nch + kNormThreads - 1) / kNormThreads;
  if (per <= 1) return 1;
  if (per <= 2) return 2;
  if (per <= 4) return 4;
  if (per <= 8) return 8;
  return -1;
}

#define DTG_PER_DISPATCH(per, ...)                   \
  switch (per) {                                     \
    case 1: { constexpr int P = 1; __VA_ARGS__; break; } \
    case 2: { constexpr int P = 2; __VA_ARGS__; break; } \
    case 4: { constexpr int P = 4; __VA_ARGS__; break; } \
    case 8: { constexpr int P = 8; __VA_ARGS__; break; } \
    default: DTG_CHECK(false, "rmsnorm: unsupported hidden size"); \
  }

static void check_rows(const at::Tensor& t, const char* name) {
  DTG_CHECK_CUDA_BF16(t);
  DTG_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.stride(0) % 8 == 0, name,
            " must be 2-D with unit inner stride and 16-byte aligned rows");
}

std::tuple<at::Tensor, at::Tensor> rmsnorm_fwd(const at::Tensor& x, const at::Tensor& w,
                                               double eps) {
  check_rows(x, "x");
  DTG_CHECK_CUDA_BF16(w);
  const int T = x.size(0), H = x.size(1);
  DTG_CHECK(H % 8 == 0 && w.numel() == H && w.is_contiguous(), "rmsnorm: bad weight/hidden");
  const c10::DeviceGuard g(x.device());
  auto y = at::empty({T, H}, x.options());
  auto rstd = at::empty({T}, x.options().dtype(at::kFloat));
  if (T == 0) return {y, rstd};
  const int per = pick_per(H);
  DTG_PER_DISPATCH(per, rmsnorm_fwd_kernel<P, false><<<T, kNormThreads, 0, stream()>>>(
                            bf16_ptr(x), x.stride(0), nullptr, 0, bf16_ptr(w), bf16_mut(y),
                            nullptr, rstd.data_ptr<float>(), H, (float)eps));
  DTG_LAUNCH_CHECK();
  return {y, rstd};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> add_rmsnorm_fwd(const at::Tensor& x,
                                                               const at::Tensor& res,
                                                               const at::Tensor& w, double eps) {
  check_rows(x, "x");
  check_rows(res, "residual");
  DTG_CHECK_CUDA_BF16(w);
  const int T = x.size(0), H = x.size(1);
  DTG_CHECK(res.size(0) == T && res.size(1) == H, "add_rmsnorm: shape mismatch");
  DTG_CHECK(H % 8 == 0 && w.numel() == H && w.is_contiguous(), "rmsnorm: bad weight/hidden");
  const c10::DeviceGuard g(x.device());
  auto y = at::empty({T, H}, x.options());
  auto h = at::empty({T, H}, x.options());
  auto rstd = at::empty({T}, x.options().dtype(at::kFloat));
  if (T == 0) return {y, h, rstd};
  const int per = pick_per(H);
  DTG_PER_DISPATCH(per, rmsnorm_fwd_kernel<P, true><<<T, kNormThreads, 0, stream()>>>(
                            bf16_ptr(x), x.stride(0), bf16_ptr(res), res.stride(0), bf16_ptr(w),
                            bf16_mut(y), bf16_mut(h), rstd.data_ptr<float>(), H, (float)eps));
  DTG_LAUNCH_CHECK();
  return {y, h, rstd};
}

std::tuple<at::Tensor, at::Tensor> rmsnorm_bwd(const at::Tensor& dy_, const at::Tensor& x,
                                               const at::Tensor& w, const at::Tensor& rstd,
                                               const c10::optional<at::Tensor>& dres_) {
  auto dy = dy_.contiguous();
  check_rows(x, "x");
  DTG_CHECK_CUDA_BF16(dy);
  const int T = x.size(0), H = x.size(1);
  DTG_CHECK(dy.size(0) == T && dy.size(1) == H, "rmsnorm_bwd: dy shape");
  DTG_CHECK(rstd.scalar_type() == at::kFloat && rstd.numel() == T, "rmsnorm_bwd: rstd");
  const c10::DeviceGuard g(x.device());
  auto dx = at::empty({T, H}, x.options());
  auto dw = at::empty({H}, w.options());
  if (T == 0) { dw.zero_(); return {dx, dw}; }
  // ~2 workgroups per CU worth of blocks keeps the partial-dw matrix (and colsum) small; the
  // kernel's row pipelining provides the memory-level parallelism (2048 blocks measured
  // 103 us + 84 us colsum vs 128 + 18 at 512 unpipelined, Llama-8B shape).
  const int nblk = std::min(T, 512);
  const int rpb = (T + nblk - 1) / nblk;
  const int nb = (T + rpb - 1) / rpb;
  auto part = at::empty({nb, H}, x.options().dtype(at::kFloat));
  at::Tensor dres;
  const bool has_dres = dres_.has_value() && dres_->defined();
  if (has_dres) {
    dres = dres_->contiguous();
    DTG_CHECK_CUDA_BF16(dres);
  }
  const int per = pick_per(H);
  if (has_dres) {
    DTG_PER_DISPATCH(per, rmsnorm_bwd_kernel<P, true><<<nb, kNormThreads, 0, stream()>>>(
                              bf16_ptr(dy), bf16_ptr(x), x.stride(0), bf16_ptr(w),
                              rstd.data_ptr<float>(), bf16_ptr(dres), bf16_mut(dx),
                              part.data_ptr<float>(), T, H, rpb));
  } else {
    DTG_PER_DISPATCH(per, rmsnorm_bwd_kernel<P, false><<<nb, kNormThreads, 0, stream()>>>(
                              bf16_ptr(dy), bf16_ptr(x), x.stride(0), bf16_ptr(w),
                              rstd.data_ptr<float>(), nullptr, bf16_mut(dx),
                              part.data_ptr<float>(), T, H, rpb));
  }
  DTG_LAUNCH_CHECK();
  colsum_to_bf16_kernel<<<(H + kColsumCols - 1) / kColsumCols, 256, 0, stream()>>>(part.data_ptr<float>(), nb, H,
                                                                                    bf16_mut(dw));
  DTG_LAUNCH_CHECK();
  return {dx, dw};
}

TORCH_LIBRARY_IMPL(dtg, CUDA, m) {
  m.impl("rmsnorm_fwd", &rmsnorm_fwd);
  m.impl("add_rmsnorm_fwd", &add_rmsnorm_fwd);
  m.impl("rmsnorm_bwd", &rmsnorm_bwd);
}

}  // namespace dtg
