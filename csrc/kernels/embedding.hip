// Deterministic embedding backward: dE[id] += sum of dY rows whose token is id.
//
// ATen's index_add_ on bf16 accumulates with atomics: the summation order of repeated tokens
// changes from run to run and every add rounds to bf16.  Here the token ids are sorted once
// (stable device radix sort, no host sync) and every table row is written by exactly one wave
// with an f32 sum in a fixed order, so the result is bitwise reproducible -- what lets the RCCL
// world-1 engine tests compare engines bit for bit and what `--determinism on` promises
// (related-topics/determinism).
//
// Work is split by CHUNKS of the sorted positions, not by runs of equal ids: one wave per
// (chunk of kChunk positions, 512-column slice).  A run of one id can be thousands of rows long
// (a frequent token in real text; under vocab-parallel TP the out-of-shard tokens), and the first
// form of this kernel -- one wave per run -- spent ~100 ms on such a run at TP = 8.  Now:
//   pass 1: each wave sums every run segment inside its chunk.  A segment that is a whole run is
//           added to its table row directly (its only writer).  A segment of a run that crosses
//           the chunk's edges goes to a per-chunk f32 partial slot instead: slot 0 for the
//           chunk's first segment if the run began in an earlier chunk, slot 1 for its last
//           segment if the run begins here and continues.
//   pass 2: the chunk where a crossing run begins adds its slot 1 and the slot 0 of every
//           following chunk the run covers, in chunk order, to the table row.
// Ids outside [0, V) are skipped (vocab-parallel embedding marks out-of-shard tokens with -1).
#include "common.h"

namespace dtg {

constexpr int kChunk = 32;     // sorted positions per wave
constexpr int kColsPerWave = 512;  // 64 lanes x 8 bf16 columns

__device__ __forceinline__ void add_row(uint16_t* orow, int c, const float* acc) {
  float o[8];
  load8(orow + c, o);
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] += acc[e];
  store8(orow + c, o);
}

__global__ __launch_bounds__(256) void embedding_bwd_chunks_kernel(
    uint16_t* __restrict__ out, int64_t out_stride, int64_t V, const uint16_t* __restrict__ dy, int64_t dy_stride,
    const int64_t* __restrict__ sorted, const int64_t* __restrict__ order, int64_t T, int H,
    float* __restrict__ partial) {
  const int nslices = (H + kColsPerWave - 1) / kColsPerWave;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t chunk = w / nslices;
  const int c = (int)(w % nslices) * kColsPerWave + (threadIdx.x & 63) * 8;
  const int64_t p0 = chunk * kChunk;
  if (p0 >= T) return;
  const int64_t p1 = min(p0 + kChunk, T);
  const bool cols = c < H;
  int64_t a = p0;
  while (a < p1) {
    const int64_t id = sorted[a];
    int64_t b = a + 1;
    while (b < p1 && sorted[b] == id) ++b;
    const bool valid = id >= 0 && id < V;
    if (valid && cols) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int64_t j = a; j < b; ++j) {
        float x[8];
        load8(dy + order[j] * dy_stride + c, x);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += x[e];
      }
      const bool before = a == p0 && a > 0 && sorted[a - 1] == id;
      const bool after = b == p1 && b < T && sorted[b] == id;
      if (!before && !after) {
        add_row(out + id * out_stride, c, acc);
      } else {
        float* slot = partial + ((chunk * 2 + (before ? 0 : 1)) * (int64_t)H + c);
        *reinterpret_cast<float4*>(slot) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        *reinterpret_cast<float4*>(slot + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
      }
    }
    a = b;
  }
}

__global__ __launch_bounds__(256) void embedding_bwd_merge_kernel(
    uint16_t* __restrict__ out, int64_t out_stride, int64_t V, const int64_t* __restrict__ sorted, int64_t T, int H,
    const float* __restrict__ partial) {
  const int nslices = (H + kColsPerWave - 1) / kColsPerWave;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t chunk = w / nslices;
  const int c = (int)(w % nslices) * kColsPerWave + (threadIdx.x & 63) * 8;
  const int64_t p0 = chunk * kChunk;
  if (p0 >= T || c >= H) return;
  const int64_t p1 = min(p0 + kChunk, T);
  const int64_t id = sorted[p1 - 1];
  if (id < 0 || id >= V || p1 >= T || sorted[p1] != id) return;  // last run of the chunk ends here
  // the run began in an earlier chunk: that chunk owns it (its slot 1 holds the run's head)
  if (sorted[p0] == id && p0 > 0 && sorted[p0 - 1] == id) return;
  float acc[8];
  const float* s = partial + (chunk * 2 + 1) * (int64_t)H + c;
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = s[e];
  for (int64_t k = chunk + 1; k * kChunk < T; ++k) {  // chunks the run reaches into, in order
    const float* t = partial + (k * 2) * (int64_t)H + c;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += t[e];
    const int64_t e1 = min((k + 1) * kChunk, T);
    if (e1 >= T || sorted[e1] != id) break;  // the run ends inside chunk k
  }
  add_row(out + id * out_stride, c, acc);
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
  const int H = (int)dy.size(1);
  const int64_t nchunks = (T + kChunk - 1) / kChunk;
  const int64_t nslices = (H + kColsPerWave - 1) / kColsPerWave;
  // every slot a pass-2 wave reads was written by pass 1 (slot 1 of the run's first chunk, slot 0
  // of each chunk it covers), so the scratch needs no zero fill
  auto partial = at::empty({nchunks * 2, (int64_t)H}, dy.options().dtype(at::kFloat));
  const int64_t waves = nchunks * nslices;
  const unsigned blocks = (unsigned)((waves + 3) / 4);
  hipLaunchKernelGGL(embedding_bwd_chunks_kernel, dim3(blocks), dim3(256), 0, stream(), bf16_mut(out), out.stride(0),
                     out.size(0), bf16_ptr(dy), dy.stride(0), sorted.data_ptr<int64_t>(), order.data_ptr<int64_t>(), T,
                     H, partial.data_ptr<float>());
  DTG_LAUNCH_CHECK();
  hipLaunchKernelGGL(embedding_bwd_merge_kernel, dim3(blocks), dim3(256), 0, stream(), bf16_mut(out), out.stride(0),
                     out.size(0), sorted.data_ptr<int64_t>(), T, H, partial.data_ptr<float>());
  DTG_LAUNCH_CHECK();
}

TORCH_LIBRARY_IMPL(dtg, CUDA, m) { m.impl("embedding_bwd_", &embedding_bwd_); }

}  // namespace dtg
