// Fused AdamW over flat parameter shards.
//
// The framework keeps every rank's trainable state in a few flat buffers (one per dtype
// group: parameters, gradients, exp_avg, exp_avg_sq), so one launch updates the whole shard
// with 16-byte vector accesses; there is no per-tensor metadata walk.
//
// Update order matches torch's fused AdamW (the reference's `AdamW(fused=True)`):
//   p   *= 1 - lr * wd
//   m    = m + (g - m) * (1 - beta1)
//   v    = v * beta2 + (1 - beta2) * g * g
//   p   -= (lr / (1 - beta1^t)) * m / (sqrt(v) / sqrt(1 - beta2^t) + eps)
// computed in f32 from whatever storage dtype the buffers use (bf16 "pure bf16" training as
// in the reference, or f32 states / an f32 master copy).
#include <type_traits>

#include "common.h"

namespace dtg {

template <typename T>
__device__ __forceinline__ float ld(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ld<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
template <>
__device__ __forceinline__ float ld<float>(const float* p, int64_t i) { return p[i]; }
template <typename T>
__device__ __forceinline__ void st(T* p, int64_t i, float v);
template <>
__device__ __forceinline__ void st<uint16_t>(uint16_t* p, int64_t i, float v) { p[i] = f2bf(v); }
template <>
__device__ __forceinline__ void st<float>(float* p, int64_t i, float v) { p[i] = v; }

struct AdamHyper {
  float lr, beta1, beta2, eps, wd, bc1, bc2_sqrt, grad_scale;
};

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float* o);
template <>
__device__ __forceinline__ void ld8<uint16_t>(const uint16_t* p, float* o) { load8(p, o); }
template <>
__device__ __forceinline__ void ld8<float>(const float* p, float* o) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float* v);
template <>
__device__ __forceinline__ void st8<uint16_t>(uint16_t* p, const float* v) { store8(p, v); }
template <>
__device__ __forceinline__ void st8<float>(float* p, const float* v) {
  reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
}

__device__ __forceinline__ void adam_elem(float& pv, float gv, float& mv, float& vv, const AdamHyper& h,
                                          float step_size, float decay) {
  // No FMA contraction: every kernel that inlines this (adamw_, adamw_t_) must round the same
  // way, so the optimizer choice never changes a bit of the trained weights.
#pragma clang fp contract(off)
  pv *= decay;
  mv = mv + (gv - mv) * (1.f - h.beta1);
  vv = vv * h.beta2 + (1.f - h.beta2) * gv * gv;
  pv -= step_size * mv / (sqrtf(vv) / h.bc2_sqrt + h.eps);
}

// Vector body: 8 elements per lane per iteration with 16/32-byte accesses (requires n % 8 == 0
// and 16-byte aligned buffers, which the flat stores guarantee); scalar kernel otherwise.
// `dev_hyper` (optional, f32 [3] = lr, 1 - beta1^t, sqrt(1 - beta2^t)) overrides the launch
// arguments: a HIP-graph-captured step replays the same kernel arguments every time, so the
// step-dependent values live in device memory the host rewrites before each replay.
template <typename GT, typename ST, bool MASTER, bool VEC, int U = 2>
__global__ __launch_bounds__(256) void adamw_kernel(uint16_t* __restrict__ p, float* __restrict__ master,
                                                    const GT* __restrict__ g, ST* __restrict__ m,
                                                    ST* __restrict__ v, int64_t n, AdamHyper h,
                                                    const float* __restrict__ dev_hyper) {
  if (dev_hyper != nullptr) {
    h.lr = dev_hyper[0];
    h.bc1 = dev_hyper[1];
    h.bc2_sqrt = dev_hyper[2];
  }
  const float step_size = h.lr / h.bc1;
  const float decay = 1.f - h.lr * h.wd;
  if constexpr (VEC) {
    // U 8-element vectors per lane per iteration (each one grid-stride away from the last):
    // 4U 16-byte loads in flight per lane before the first use, which is what lifts this purely
    // streaming kernel toward HBM bandwidth (4 in flight left it latency-bound).
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 8;
    int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
    for (; i + (U - 1) * stride < n; i += U * stride) {
      float pv[U][8], gv[U][8], mv[U][8], vv[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t k = i + u * stride;
        if (MASTER) ld8<float>(master + k, pv[u]); else load8(p + k, pv[u]);
        ld8<GT>(g + k, gv[u]);
        ld8<ST>(m + k, mv[u]);
        ld8<ST>(v + k, vv[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t k = i + u * stride;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          adam_elem(pv[u][j], gv[u][j] * h.grad_scale, mv[u][j], vv[u][j], h, step_size, decay);
        st8<ST>(m + k, mv[u]);
        st8<ST>(v + k, vv[u]);
        if (MASTER) st8<float>(master + k, pv[u]);
        store8(p + k, pv[u]);
      }
    }
    for (; i < n; i += stride) {
      float pv[8], gv[8], mv[8], vv[8];
      if (MASTER) ld8<float>(master + i, pv); else load8(p + i, pv);
      ld8<GT>(g + i, gv);
      ld8<ST>(m + i, mv);
      ld8<ST>(v + i, vv);
#pragma unroll
      for (int j = 0; j < 8; ++j) adam_elem(pv[j], gv[j] * h.grad_scale, mv[j], vv[j], h, step_size, decay);
      st8<ST>(m + i, mv);
      st8<ST>(v + i, vv);
      if (MASTER) st8<float>(master + i, pv);
      store8(p + i, pv);
    }
  } else {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      float pv = MASTER ? master[i] : bf2f(p[i]);
      float mv = ld<ST>(m, i), vv = ld<ST>(v, i);
      adam_elem(pv, ld<GT>(g, i) * h.grad_scale, mv, vv, h, step_size, decay);
      st<ST>(m, i, mv);
      st<ST>(v, i, vv);
      if (MASTER) master[i] = pv;
      p[i] = f2bf(pv);
    }
  }
}

void adamw_(const at::Tensor& p, const c10::optional<at::Tensor>& master, const at::Tensor& g,
            const at::Tensor& m, const at::Tensor& v, double lr, double beta1, double beta2,
            double eps, double wd, int64_t step, double grad_scale, const c10::optional<at::Tensor>& hyper) {
  DTG_CHECK_CUDA_BF16(p);
  DTG_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous(),
            "adamw_: buffers must be contiguous");
  const int64_t n = p.numel();
  DTG_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adamw_: size mismatch");
  DTG_CHECK(m.scalar_type() == v.scalar_type(), "adamw_: exp_avg/exp_avg_sq dtype mismatch");
  DTG_CHECK(step >= 1, "adamw_: step must be >= 1");
  const bool has_master = master.has_value() && master->defined();
  const float* hp = nullptr;
  if (hyper.has_value() && hyper->defined()) {
    DTG_CHECK(hyper->is_cuda() && hyper->scalar_type() == at::kFloat && hyper->numel() >= 3 && hyper->is_contiguous(),
              "adamw_: hyper must be a contiguous f32 GPU tensor [lr, 1-beta1^t, sqrt(1-beta2^t)]");
    hp = hyper->data_ptr<float>();
  }
  if (has_master)
    DTG_CHECK(master->scalar_type() == at::kFloat && master->numel() == n && master->is_contiguous(),
              "adamw_: master must be contiguous f32");
  if (n == 0) return;
  const c10::DeviceGuard gd(p.device());
  AdamHyper h;
  h.lr = lr;
  h.beta1 = beta1;
  h.beta2 = beta2;
  h.eps = eps;
  h.wd = wd;
  h.bc1 = 1.0 - std::pow(beta1, (double)step);
  h.bc2_sqrt = std::sqrt(1.0 - std::pow(beta2, (double)step));
  h.grad_scale = grad_scale;
  const int threads = 256;
  const int64_t want = (n + threads * 8 - 1) / (threads * 8);
  // 2 vectors per lane per iteration, up to 16 workgroups per CU: unroll 2 / 4 x 4-32 workgroups
  // per CU span 5.04-5.41 TB/s, 16 and 32 within 2 % (profiles/r3/s08/kernels.log); the knobs
  // were removed in round 6
  constexpr int unroll = 2, wg_per_cu = 16;
  const int blocks = (int)std::min<int64_t>(want, 256 * wg_per_cu);
  float* mp = has_master ? master->data_ptr<float>() : nullptr;
  const bool gb = g.scalar_type() == at::kBFloat16;
  const bool sb = m.scalar_type() == at::kBFloat16;
  DTG_CHECK(gb || g.scalar_type() == at::kFloat, "adamw_: grad must be bf16 or f32");
  DTG_CHECK(sb || m.scalar_type() == at::kFloat, "adamw_: states must be bf16 or f32");
  auto aligned = [](const at::Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; };
  const bool vec = (n % 8 == 0) && aligned(p) && aligned(g) && aligned(m) && aligned(v) &&
                   (!has_master || aligned(*master));
#define DTG_ADAM_LAUNCH(GT, ST, MASTER)                                                      \
  do { if (vec) adamw_kernel<GT, ST, MASTER, true, unroll><<<blocks, threads, 0, stream()>>>(       \
      bf16_mut(p), mp, reinterpret_cast<const GT*>(g.data_ptr()), reinterpret_cast<ST*>(m.data_ptr()), \
      reinterpret_cast<ST*>(v.data_ptr()), n, h, hp);                                       \
  else adamw_kernel<GT, ST, MASTER, false><<<blocks, threads, 0, stream()>>>(               \
      bf16_mut(p), mp, reinterpret_cast<const GT*>(g.data_ptr()), reinterpret_cast<ST*>(m.data_ptr()), \
      reinterpret_cast<ST*>(v.data_ptr()), n, h, hp); } while (0)
  if (has_master) {
    if (gb && sb) DTG_ADAM_LAUNCH(uint16_t, uint16_t, true);
    else if (gb) DTG_ADAM_LAUNCH(uint16_t, float, true);
    else if (sb) DTG_ADAM_LAUNCH(float, uint16_t, true);
    else DTG_ADAM_LAUNCH(float, float, true);
  } else {
    if (gb && sb) DTG_ADAM_LAUNCH(uint16_t, uint16_t, false);
    else if (gb) DTG_ADAM_LAUNCH(uint16_t, float, false);
    else if (sb) DTG_ADAM_LAUNCH(float, uint16_t, false);
    else DTG_ADAM_LAUNCH(float, float, false);
  }
#undef DTG_ADAM_LAUNCH
  DTG_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// AdamW that also refreshes the transposed copy of every weight matrix (single / DDP engines).
//
// hipBLASLt's backward dX = dY W runs at TN speed only with W^T (K-contiguous); weights change
// once per step, so instead of transposing every weight in every backward (one read + one write
// of W per step), this kernel writes W^T while the updated W is still in registers: the read is
// saved, the write moves here.  The flat buffer is described as a list of matrices (2-D params;
// 1-D params as [1, n] rows with no transposed copy); the grid walks 64 x TC tiles of all of
// them, one tile per workgroup (TC = 64 | 128 | 256 columns; the engines use 256).  An LDS-staged
// form (update row-wise, park the tile in LDS, write its columns as W^T rows) ran 5.54 TB/s at
// its best tile against this kernel's 5.98 (profiles/r5/transpose/) and was removed in round 6.
// ------------------------------------------------------------------------------------------
struct MatDesc {
  int64_t off, rows, cols, toff, tile0;  // toff < 0: no transposed copy
};

constexpr int kAtRows = 64;

// Eight raw elements of a buffer, converted to f32 only when the update runs (bf16 vectors stay
// packed in 4 VGPRs while their loads are in flight).
template <typename T>
struct Raw8;
template <>
struct Raw8<uint16_t> {
  u16x8 v;
  __device__ __forceinline__ void load(const uint16_t* p) { v = *reinterpret_cast<const u16x8*>(p); }
  __device__ __forceinline__ float operator[](int j) const { return bf2f(v[j]); }
};
template <>
struct Raw8<float> {
  f32x4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = reinterpret_cast<const f32x4*>(p)[0];
    b = reinterpret_cast<const f32x4*>(p)[1];
  }
  __device__ __forceinline__ float operator[](int j) const { return j < 4 ? a[j] : b[j - 4]; }
};

// Register-blocked: no LDS, no barriers.  One 64 x TC tile per workgroup of TC threads (TC / 64
// waves); every lane owns an 8 x 8 block: eight 16-B row vectors of p, g, m, v in, the update in f32, p / m / v rows out,
// and -- for a matrix with a transposed copy -- the updated block through an in-register 8 x 8
// transpose (transpose8x8) to eight 16-B rows of W^T.  Eight lanes cover 128 contiguous bytes of
// every row they load or store.  Matrices with a W^T have rows and columns that are multiples of
// 8 (the engine's descriptor builder), so their blocks are whole; the W^T-less rows (norm
// weights, odd vocabularies) may end mid-block and are bounds-checked per row.
template <typename ST, bool MASTER, int TC>
__global__ __launch_bounds__(TC) void adamw_t_reg_kernel(uint16_t* __restrict__ p, float* __restrict__ master,
                                                         const uint16_t* __restrict__ g, ST* __restrict__ m,
                                                         ST* __restrict__ v, uint16_t* __restrict__ pt,
                                                         const MatDesc* __restrict__ mats, int nmats, AdamHyper h,
                                                         const float* __restrict__ dev_hyper) {
  if (dev_hyper != nullptr) {
    h.lr = dev_hyper[0];
    h.bc1 = dev_hyper[1];
    h.bc2_sqrt = dev_hyper[2];
  }
  const float step_size = h.lr / h.bc1;
  const float decay = 1.f - h.lr * h.wd;
  const int64_t t = blockIdx.x;
  int lo = 0, hi = nmats - 1;  // the matrix whose tiles include t
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (mats[mid].tile0 <= t) lo = mid; else hi = mid - 1;
  }
  const MatDesc md = mats[lo];
  const int64_t lt = t - md.tile0;
  const int64_t ntc = (md.cols + TC - 1) / TC;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r = (lt / ntc) * kAtRows + (lane >> 3) * 8;
  const int64_t c = (lt % ntc) * TC + 64 * w + (lane & 7) * 8;
  if (r >= md.rows || c >= md.cols) return;
  const int nr = md.rows - r < 8 ? (int)(md.rows - r) : 8;  // 8 except at a W^T-less row end
  using PT = typename std::conditional<MASTER, float, uint16_t>::type;
  Raw8<PT> pr[8];
  Raw8<uint16_t> gr[8];
  Raw8<ST> mr[8], vr[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i < nr) {
      const int64_t k = md.off + (r + i) * md.cols + c;
      if constexpr (MASTER) pr[i].load(master + k); else pr[i].load(p + k);
      gr[i].load(g + k);
      mr[i].load(m + k);
      vr[i].load(v + k);
    }
  }
  u16x8 pb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i < nr) {
      const int64_t k = md.off + (r + i) * md.cols + c;
      float pv[8], mv[8], vv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pv[j] = pr[i][j];
        mv[j] = mr[i][j];
        vv[j] = vr[i][j];
        adam_elem(pv[j], gr[i][j] * h.grad_scale, mv[j], vv[j], h, step_size, decay);
      }
      st8<ST>(m + k, mv);
      st8<ST>(v + k, vv);
      if (MASTER) st8<float>(master + k, pv);
#pragma unroll
      for (int j = 0; j < 8; ++j) pb[i][j] = f2bf(pv[j]);
      *reinterpret_cast<u16x8*>(p + k) = pb[i];
    }
  }
  if (md.toff >= 0) {  // whole 8 x 8 blocks (rows and columns are multiples of 8)
    transpose8x8(pb);
#pragma unroll
    for (int j = 0; j < 8; ++j) *reinterpret_cast<u16x8*>(pt + md.toff + (c + j) * md.rows + r) = pb[j];
  }
}

void adamw_t_(const at::Tensor& p, const c10::optional<at::Tensor>& master, const at::Tensor& g, const at::Tensor& m,
              const at::Tensor& v, const at::Tensor& pt, const at::Tensor& mats, int64_t ntiles, double lr,
              double beta1, double beta2, double eps, double wd, int64_t step, double grad_scale,
              const c10::optional<at::Tensor>& hyper, int64_t tile_cols) {
  DTG_CHECK_CUDA_BF16(p);
  DTG_CHECK_CUDA_BF16(pt);
  DTG_CHECK(g.scalar_type() == at::kBFloat16, "adamw_t_: grads must be bf16");
  DTG_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous() && pt.is_contiguous(),
            "adamw_t_: buffers must be contiguous");
  DTG_CHECK(tile_cols == 64 || tile_cols == 128 || tile_cols == 256, "adamw_t_: tile_cols must be 64, 128 or 256");
  const int64_t n = p.numel();
  DTG_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adamw_t_: size mismatch");
  DTG_CHECK(m.scalar_type() == v.scalar_type(), "adamw_t_: exp_avg/exp_avg_sq dtype mismatch");
  DTG_CHECK(step >= 1, "adamw_t_: step must be >= 1");
  DTG_CHECK(mats.is_cuda() && mats.scalar_type() == at::kLong && mats.dim() == 2 && mats.size(1) == 5 &&
                mats.is_contiguous(), "adamw_t_: mats must be int64 [n, 5] on the GPU");
  auto aligned = [](const at::Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; };
  DTG_CHECK(aligned(p) && aligned(g) && aligned(m) && aligned(v) && aligned(pt), "adamw_t_: 16-byte aligned buffers");
  const bool has_master = master.has_value() && master->defined();
  if (has_master)
    DTG_CHECK(master->scalar_type() == at::kFloat && master->numel() == n && master->is_contiguous() &&
              aligned(*master), "adamw_t_: master must be contiguous f32");
  const float* hp = nullptr;
  if (hyper.has_value() && hyper->defined()) {
    DTG_CHECK(hyper->is_cuda() && hyper->scalar_type() == at::kFloat && hyper->numel() >= 3 && hyper->is_contiguous(),
              "adamw_t_: hyper must be a contiguous f32 GPU tensor");
    hp = hyper->data_ptr<float>();
  }
  const int nm = (int)mats.size(0);
  if (nm == 0 || ntiles == 0) return;
  const c10::DeviceGuard gd(p.device());
  AdamHyper h;
  h.lr = lr;
  h.beta1 = beta1;
  h.beta2 = beta2;
  h.eps = eps;
  h.wd = wd;
  h.bc1 = 1.0 - std::pow(beta1, (double)step);
  h.bc2_sqrt = std::sqrt(1.0 - std::pow(beta2, (double)step));
  h.grad_scale = grad_scale;
  float* mp = has_master ? master->data_ptr<float>() : nullptr;
  const auto* md = reinterpret_cast<const MatDesc*>(mats.data_ptr<int64_t>());
  const auto* gp = reinterpret_cast<const uint16_t*>(g.data_ptr());
  uint16_t* ptp = bf16_mut(pt);
  const bool sb = m.scalar_type() == at::kBFloat16;
  DTG_CHECK(sb || m.scalar_type() == at::kFloat, "adamw_t_: states must be bf16 or f32");
  DTG_CHECK(ntiles < (int64_t(1) << 31), "adamw_t_: too many tiles");
#define DTG_ADAMT_REG(ST, MASTER, TC)                                                                       \
  adamw_t_reg_kernel<ST, MASTER, TC><<<(unsigned)ntiles, TC, 0, stream()>>>(                                \
      bf16_mut(p), mp, gp, reinterpret_cast<ST*>(m.data_ptr()), reinterpret_cast<ST*>(v.data_ptr()), ptp, md, nm, \
      h, hp)
#define DTG_ADAMT_REG_TC(ST, MASTER)                                 \
  do {                                                                \
    if (tile_cols == 64) DTG_ADAMT_REG(ST, MASTER, 64);               \
    else if (tile_cols == 128) DTG_ADAMT_REG(ST, MASTER, 128);        \
    else DTG_ADAMT_REG(ST, MASTER, 256);                              \
  } while (0)
  if (has_master) {
    if (sb) DTG_ADAMT_REG_TC(uint16_t, true); else DTG_ADAMT_REG_TC(float, true);
  } else {
    if (sb) DTG_ADAMT_REG_TC(uint16_t, false); else DTG_ADAMT_REG_TC(float, false);
  }
#undef DTG_ADAMT_REG_TC
#undef DTG_ADAMT_REG
  DTG_LAUNCH_CHECK();
}

TORCH_LIBRARY_IMPL(dtg, CUDA, m) {
  m.impl("adamw_", &adamw_);
  m.impl("adamw_t_", &adamw_t_);
}

}  // namespace dtg
