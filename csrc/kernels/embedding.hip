// Deterministic embedding backward: dE[id] += sum of dY rows whose token is id.
//
// ATen's index_add_ on bf16 accumulates with atomics: the summation order of repeated tokens
// changes from run to run and every add rounds to bf16.  Here the token ids are sorted once
// (stable device radix sort, no host sync) and one wave owns each distinct id: it sums that
// id's dY rows in sorted (= token) order in f32 and adds the total to the table row once.  The
// result is bitwise reproducible, which is what lets the RCCL world-1 engine tests compare
// engines bit for bit and what `--determinism on` promises (related-topics/determinism).
//
// Work: dY is read once (T x H bf16) plus one read-modify-write of each touched table row.
// A wave that does not start a run of equal ids exits immediately.
#include "common.h"

namespace dtg {

// One wave per sorted position; 8 bf16 columns per lane, 512 columns per pass.
__global__ __launch_bounds__(256) void embedding_bwd_kernel(uint16_t* __restrict__ out, int64_t out_stride,
                                                            const uint16_t* __restrict__ dy, int64_t dy_stride,
                                                            const int64_t* __restrict__ sorted,
                                                            const int64_t* __restrict__ order, int64_t T, int H) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= T) return;
  const int64_t id = sorted[i];
  if (i > 0 && sorted[i - 1] == id) return;  // not the first of its run
  int64_t end = i + 1;
  while (end < T && sorted[end] == id) ++end;
  uint16_t* orow = out + id * out_stride;
  for (int c0 = lane * 8; c0 < H; c0 += 512) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int64_t j = i; j < end; ++j) {
      float x[8];
      load8(dy + order[j] * dy_stride + c0, x);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += x[e];
    }
    float o[8];
    load8(orow + c0, o);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] += acc[e];
    store8(orow + c0, o);
  }
}

void embedding_bwd_(const at::Tensor& out, const at::Tensor& ids, const at::Tensor& dy) {
  DTG_CHECK_CUDA_BF16(out);
  DTG_CHECK_CUDA_BF16(dy);
  DTG_CHECK(ids.scalar_type() == at::kLong && ids.is_cuda(), "embedding_bwd_: ids must be int64 on the GPU");
  DTG_CHECK(out.dim() == 2 && dy.dim() == 2 && out.size(1) == dy.size(1) && out.stride(1) == 1 &&
                dy.stride(1) == 1 && out.stride(0) % 8 == 0 && dy.stride(0) % 8 == 0 && dy.size(1) % 8 == 0,
            "embedding_bwd_: out [V, H] / dy [T, H] with unit column stride, 16-B aligned rows, H % 8 == 0");
  const int64_t T = dy.size(0);
  DTG_CHECK(ids.numel() == T, "embedding_bwd_: one id per dy row");
  if (T == 0) return;
  const c10::DeviceGuard g(out.device());
  auto flat = ids.reshape({-1});
  auto [sorted, order] = at::sort(flat, /*stable=*/true, /*dim=*/0, /*descending=*/false);
  const int64_t blocks = (T + 3) / 4;
  hipLaunchKernelGGL(embedding_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, stream(), bf16_mut(out),
                     out.stride(0), bf16_ptr(dy), dy.stride(0), sorted.data_ptr<int64_t>(),
                     order.data_ptr<int64_t>(), T, (int)dy.size(1));
  DTG_LAUNCH_CHECK();
}

TORCH_LIBRARY_IMPL(dtg, CUDA, m) { m.impl("embedding_bwd_", &embedding_bwd_); }

}  // namespace dtg
