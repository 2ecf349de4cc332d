// Causal-LM cross entropy over a chunk of logits, with the softmax gradient written in
// place.
//
// The model's loss head computes logits chunk by chunk with one hipBLASLt GEMM, then calls
// `ce_fwd_bwd_` which (1) reduces max/sum-exp per row with an online softmax, (2) returns the
// per-row loss lse - x[label] and (3) overwrites the chunk with
// (softmax - onehot(label)) * grad_scale, so the [T, V] f32 logits of HF's ForCausalLMLoss
// are never materialised and no second pass over logits is needed in backward.
// Rows whose label == ignore_index contribute 0 loss and 0 gradient (HF semantics).
//
// Vocab-parallel (tensor-parallel lm_head): `ce_stats` returns the local
// (max, sum-exp, target logit) per row, the caller all-reduces them over the TP group, and
// `ce_grad_` writes the local gradient slice from the global log-sum-exp.
//
// Rows of odd length (V = 50257, 156939) are handled with a scalar head/tail around a
// 16-byte-vector body, so no padding of the vocabulary is required.
#include "common.h"

namespace dtg {

constexpr int kCeThreads = 512;

struct RowSpan {
  int head, nvec, tail_start;
};

__device__ __forceinline__ RowSpan row_span(const uint16_t* row, int V) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(row);
  int head = ((16 - (a & 15)) & 15) >> 1;
  if (head > V) head = V;
  const int nvec = (V - head) >> 3;
  return {head, nvec, head + nvec * 8};
}

__device__ __forceinline__ void online_add(float x, float& m, float& s) {
  if (x > m) {
    s = s * __expf(m - x) + 1.f;
    m = x;
  } else {
    s += __expf(x - m);
  }
}

// Per-row max and sum(exp(x - max)) over this row, reduced over the block.
__device__ __forceinline__ void row_stats(const uint16_t* row, int V, float* scratch, float& m_out,
                                          float& s_out) {
  const RowSpan sp = row_span(row, V);
  float m = -INFINITY, s = 0.f;
  for (int i = threadIdx.x; i < sp.head; i += blockDim.x) online_add(bf2f(row[i]), m, s);
  for (int i = sp.tail_start + threadIdx.x; i < V; i += blockDim.x) online_add(bf2f(row[i]), m, s);
  const uint16_t* body = row + sp.head;
  for (int v = threadIdx.x; v < sp.nvec; v += blockDim.x) {
    float x[8];
    load8(body + v * 8, x);
    float vm = x[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) vm = fmaxf(vm, x[j]);
    if (vm > m) {
      s *= __expf(m - vm);
      m = vm;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(x[j] - m);
  }
  const float gm = block_max(m, scratch);
  float sc = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  __syncthreads();
  const float gs = block_sum(sc, scratch);
  m_out = gm;
  s_out = gs;
}

// grad = (exp(x - lse) - [col == label]) * scale, in place; label is relative to this row slice.
__device__ __forceinline__ void row_grad(uint16_t* row, int V, float lse, int64_t label, float scale) {
  const RowSpan sp = row_span(row, V);
  for (int i = threadIdx.x; i < sp.head; i += blockDim.x) {
    float g = __expf(bf2f(row[i]) - lse) - (i == label ? 1.f : 0.f);
    row[i] = f2bf(g * scale);
  }
  for (int i = sp.tail_start + threadIdx.x; i < V; i += blockDim.x) {
    float g = __expf(bf2f(row[i]) - lse) - (i == label ? 1.f : 0.f);
    row[i] = f2bf(g * scale);
  }
  uint16_t* body = row + sp.head;
  for (int v = threadIdx.x; v < sp.nvec; v += blockDim.x) {
    float x[8];
    load8(body + v * 8, x);
    const int64_t c0 = sp.head + v * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (__expf(x[j] - lse) - (c0 + j == label ? 1.f : 0.f)) * scale;
    store8(body + v * 8, x);
  }
}

__device__ __forceinline__ void row_zero(uint16_t* row, int V) {
  for (int i = threadIdx.x; i < V; i += blockDim.x) row[i] = 0;
}

__global__ __launch_bounds__(kCeThreads) void ce_fused_kernel(uint16_t* __restrict__ logits,
                                                              int64_t ld, int V,
                                                              const int64_t* __restrict__ labels,
                                                              int64_t ignore_index, float scale,
                                                              bool compute_grad,
                                                              float* __restrict__ loss) {
  __shared__ float scratch[kCeThreads / 64];
  __shared__ float xl;
  uint16_t* row = logits + blockIdx.x * ld;
  const int64_t label = labels[blockIdx.x];
  const bool valid = label != ignore_index;
  if (threadIdx.x == 0) xl = (valid && label >= 0 && label < V) ? bf2f(row[label]) : 0.f;
  float m, s;
  row_stats(row, V, scratch, m, s);
  const float lse = m + __logf(s);
  if (threadIdx.x == 0) loss[blockIdx.x] = valid ? (lse - xl) : 0.f;
  if (!compute_grad) return;
  if (valid) row_grad(row, V, lse, label, scale);
  else row_zero(row, V);
}

__global__ __launch_bounds__(kCeThreads) void ce_stats_kernel(const uint16_t* __restrict__ logits,
                                                              int64_t ld, int V,
                                                              const int64_t* __restrict__ labels,
                                                              int64_t vstart, float* __restrict__ m_out,
                                                              float* __restrict__ s_out,
                                                              float* __restrict__ xl_out) {
  __shared__ float scratch[kCeThreads / 64];
  const uint16_t* row = logits + blockIdx.x * ld;
  const int64_t l = labels[blockIdx.x] - vstart;
  float m, s;
  row_stats(row, V, scratch, m, s);
  if (threadIdx.x == 0) {
    m_out[blockIdx.x] = m;
    s_out[blockIdx.x] = s;
    xl_out[blockIdx.x] = (l >= 0 && l < V) ? bf2f(row[l]) : 0.f;
  }
}

__global__ __launch_bounds__(kCeThreads) void ce_grad_kernel(uint16_t* __restrict__ logits, int64_t ld,
                                                             int V, const int64_t* __restrict__ labels,
                                                             const float* __restrict__ lse,
                                                             int64_t vstart, int64_t ignore_index,
                                                             float scale) {
  uint16_t* row = logits + blockIdx.x * ld;
  const int64_t label = labels[blockIdx.x];
  if (label == ignore_index) {
    row_zero(row, V);
    return;
  }
  row_grad(row, V, lse[blockIdx.x], label - vstart, scale);
}

static void check_logits(const at::Tensor& logits, const at::Tensor& labels) {
  DTG_CHECK_CUDA_BF16(logits);
  DTG_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "ce: logits must be [t, V] row-major");
  DTG_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous() &&
                labels.numel() == logits.size(0),
            "ce: labels must be contiguous int64 [t]");
}

at::Tensor ce_fwd_bwd_(const at::Tensor& logits, const at::Tensor& labels, int64_t ignore_index,
                       double grad_scale, bool compute_grad) {
  check_logits(logits, labels);
  const c10::DeviceGuard g(logits.device());
  const int64_t t = logits.size(0);
  auto loss = at::empty({t}, logits.options().dtype(at::kFloat));
  if (t == 0) return loss;
  ce_fused_kernel<<<t, kCeThreads, 0, stream()>>>(bf16_mut(logits), logits.stride(0),
                                                  logits.size(1), labels.data_ptr<int64_t>(),
                                                  ignore_index, (float)grad_scale, compute_grad,
                                                  loss.data_ptr<float>());
  DTG_LAUNCH_CHECK();
  return loss;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> ce_stats(const at::Tensor& logits,
                                                        const at::Tensor& labels, int64_t vstart) {
  check_logits(logits, labels);
  const c10::DeviceGuard g(logits.device());
  const int64_t t = logits.size(0);
  auto opts = logits.options().dtype(at::kFloat);
  auto m = at::empty({t}, opts), s = at::empty({t}, opts), xl = at::empty({t}, opts);
  if (t == 0) return {m, s, xl};
  ce_stats_kernel<<<t, kCeThreads, 0, stream()>>>(bf16_ptr(logits), logits.stride(0),
                                                  logits.size(1), labels.data_ptr<int64_t>(), vstart,
                                                  m.data_ptr<float>(), s.data_ptr<float>(),
                                                  xl.data_ptr<float>());
  DTG_LAUNCH_CHECK();
  return {m, s, xl};
}

void ce_grad_(const at::Tensor& logits, const at::Tensor& labels, const at::Tensor& lse,
              int64_t vstart, int64_t ignore_index, double grad_scale) {
  check_logits(logits, labels);
  DTG_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == logits.size(0),
            "ce_grad_: lse must be f32 [t]");
  const c10::DeviceGuard g(logits.device());
  const int64_t t = logits.size(0);
  if (t == 0) return;
  ce_grad_kernel<<<t, kCeThreads, 0, stream()>>>(bf16_mut(logits), logits.stride(0), logits.size(1),
                                                 labels.data_ptr<int64_t>(), lse.data_ptr<float>(),
                                                 vstart, ignore_index, (float)grad_scale);
  DTG_LAUNCH_CHECK();
}

TORCH_LIBRARY_IMPL(dtg, CUDA, m) {
  m.impl("ce_fwd_bwd_", &ce_fwd_bwd_);
  m.impl("ce_stats", &ce_stats);
  m.impl("ce_grad_", &ce_grad_);
}

}  // namespace dtg
