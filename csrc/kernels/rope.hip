// Rotary position embedding applied in place to the q and k heads of a fused QKV
// activation [T, (Hq + 2*Hkv) * D].
//
// HF Llama semantics: q' = q*cos + rotate_half(q)*sin with rotate_half(x) = [-x2, x1],
// cos/sin = cat(freqs, freqs) evaluated at position_ids.  The tables here hold the D/2
// distinct frequencies in f32 ([max_pos, D/2]); the kernel rotates pairs (i, i + D/2) in
// f32 and rounds once.  `inverse` rotates by -theta, which is exactly the backward of the
// forward rotation (the Jacobian is orthogonal), so the same kernel serves both passes.
//
// Positions come from a per-token int64 vector, so packed sequences whose position ids
// restart at every EOS need no special path.
#include "common.h"

namespace dtg {

// One thread per (token, head, 8-pair group): two 16-B loads of x and two 32-B table loads.
template <int D>
__global__ void rope_kernel(uint16_t* __restrict__ qkv, int64_t row_stride, int nheads,
                            const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                            const int64_t* __restrict__ pos, int64_t T, bool inverse) {
  constexpr int HALF = D / 2;
  constexpr int GROUPS = HALF / 8;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = T * nheads * GROUPS;
  if (gid >= total) return;
  const int grp = gid % GROUPS;
  const int64_t th = gid / GROUPS;
  const int head = th % nheads;
  const int64_t tok = th / nheads;
  const int64_t p = pos[tok];
  uint16_t* base = qkv + tok * row_stride + (int64_t)head * D + grp * 8;
  float x1[8], x2[8];
  load8(base, x1);
  load8(base + HALF, x2);
  const float4* cp = reinterpret_cast<const float4*>(cos_t + p * HALF + grp * 8);
  const float4* sp = reinterpret_cast<const float4*>(sin_t + p * HALF + grp * 8);
  float4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
  float c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  float s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  if (inverse) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = -s[j];
  }
  float o1[8], o2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    o1[j] = x1[j] * c[j] - x2[j] * s[j];
    o2[j] = x2[j] * c[j] + x1[j] * s[j];
  }
  store8(base, o1);
  store8(base + HALF, o2);
}

// Raw-pointer launch for other translation units (the flash-attention backward's split dK path).
void rope_rows_launch(uint16_t* x, int64_t row_stride, int nheads, int head_dim, const float* cos_t,
                      const float* sin_t, const int64_t* pos, int64_t T, bool inverse, hipStream_t st) {
  const int threads = 256;
  if (T == 0) return;
  if (head_dim == 128) {
    const int64_t total = T * nheads * (64 / 8);
    rope_kernel<128><<<(total + threads - 1) / threads, threads, 0, st>>>(x, row_stride, nheads, cos_t, sin_t, pos, T,
                                                                          inverse);
  } else {
    DTG_CHECK(head_dim == 64, "rope: head_dim must be 64 or 128");
    const int64_t total = T * nheads * (32 / 8);
    rope_kernel<64><<<(total + threads - 1) / threads, threads, 0, st>>>(x, row_stride, nheads, cos_t, sin_t, pos, T,
                                                                         inverse);
  }
  DTG_LAUNCH_CHECK();
}

void rope_(const at::Tensor& qkv, const at::Tensor& cos_t, const at::Tensor& sin_t,
           const at::Tensor& pos, int64_t nheads, int64_t head_dim, bool inverse) {
  DTG_CHECK_CUDA_BF16(qkv);
  DTG_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1 && qkv.stride(0) % 8 == 0,
            "rope: qkv must be [T, C] with 16-B aligned rows");
  DTG_CHECK(qkv.size(1) >= nheads * head_dim, "rope: not enough columns for the rotated heads");
  DTG_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat &&
                cos_t.is_contiguous() && sin_t.is_contiguous() && cos_t.size(1) == head_dim / 2,
            "rope: tables must be contiguous f32 [max_pos, D/2]");
  DTG_CHECK(pos.scalar_type() == at::kLong && pos.is_contiguous() && pos.numel() == qkv.size(0),
            "rope: position ids must be int64 [T]");
  const int64_t T = qkv.size(0);
  if (T == 0) return;
  const c10::DeviceGuard g(qkv.device());
  const int threads = 256;
  if (head_dim == 128) {
    const int64_t total = T * nheads * (64 / 8);
    rope_kernel<128><<<(total + threads - 1) / threads, threads, 0, stream()>>>(
        bf16_mut(qkv), qkv.stride(0), nheads, cos_t.data_ptr<float>(), sin_t.data_ptr<float>(),
        pos.data_ptr<int64_t>(), T, inverse);
  } else if (head_dim == 64) {
    const int64_t total = T * nheads * (32 / 8);
    rope_kernel<64><<<(total + threads - 1) / threads, threads, 0, stream()>>>(
        bf16_mut(qkv), qkv.stride(0), nheads, cos_t.data_ptr<float>(), sin_t.data_ptr<float>(),
        pos.data_ptr<int64_t>(), T, inverse);
  } else {
    DTG_CHECK(false, "rope: head_dim must be 64 or 128");
  }
  DTG_LAUNCH_CHECK();
}

TORCH_LIBRARY_IMPL(dtg, CUDA, m) { m.impl("rope_", &rope_); }

}  // namespace dtg
