// Flash-style causal attention, forward and backward, for gfx950 (replaces
// the flash-attn / SDPA dependencies N2, N3 of the reference).
//
// Supports GQA (Hq a multiple of Hkv), head_dim 64/128, causal sliding windows (Mistral; a
// separate WIN instantiation, so the plain causal kernels are unchanged), and variable-length
// packed sequences through `cu_seqlens` (the rime packed path: documents restart their position
// ids at each EOS) -- a dense [B, S] batch is just cu_seqlens = arange(B+1)*S.
// Layout: token-major q [T, Hq, D], k/v [T, Hkv, D] with an arbitrary token stride, so q, k
// and v are read straight out of the fused QKV projection output with no copies.
//
// MFMA mapping (v_mfma_f32_32x32x16_bf16, CDNA guide §3):
//  * Forward computes S^T = K Q^T so a lane owns one query column (online-softmax state is
//    per lane; the row reduction is 31 f32 max + one cross-half shuffle), then
//    O^T += V^T P^T with P^T taken straight from the S^T accumulator registers (the k order
//    inside a 16-step is permuted; V^T fragments are fetched in the same permuted order with
//    ds_read_b64_tr_b16, T10).  The running max is rescaled lazily (only when it grows by more
//    than 2^8, T13), so most tiles skip the O rescale.
//  * Backward is split in two kernels that both recompute P (seven MFMA products per tile
//    instead of five) so that no partial sum crosses workgroups: no f32 dQ atomics, whose
//    chip-wide rate bounds the one-kernel form at these shapes, and dQ is bitwise reproducible.
//    bwd_dq_kernel is query-stationary with the forward's structure; bwd_dkdv_kernel is
//    key-stationary with this wave's K and V rows held in registers, so only Q/dO slices stream
//    through LDS.
//  * Tiles live in LDS as 16-byte-chunk XOR-swizzled images (T10 image (b)); ds_read_b128 row
//    reads and transposed reads share one copy, and every lane's LDS offsets are computed once
//    (the swizzle depends on the low 4 row bits only, so tile/step offsets are immediates).
//  * Global -> register staging goes through buffer descriptors: rows past the end of a
//    sequence read as zeros from the range check, with no per-row branches.
#include "common.h"

#include <ATen/hip/HIPGeneratorImpl.h>
#include <ATen/hip/PhiloxUtils.cuh>
#include <ATen/core/DistributionsHelper.h>

#include <climits>
#include <cstdlib>
#include <type_traits>

#include <cmath>

namespace dtg {

// csrc/kernels/rope.hip
void rope_rows_launch(uint16_t* x, int64_t row_stride, int nheads, int head_dim, const float* cos_t,
                      const float* sin_t, const int64_t* pos, int64_t T, bool inverse, hipStream_t st);

namespace fa {

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kRescaleThreshold = 8.f;  // log2 units: P values stay below 2^8

// Byte offset of 16-byte chunk `ch` of row `row` in a [rows][W] bf16 LDS image.
template <int W>
__device__ __forceinline__ int off(int row, int ch) {
  constexpr int NCH = W / 8;
  static_assert(NCH == 8 || NCH == 16, "head_dim 64 or 128");
  int sw;
  if constexpr (NCH == 16) sw = ((row & 3) << 2) | ((row >> 2) & 3);
  else sw = ((row & 1) << 2) | ((row >> 1) & 3);
  return row * (W * 2) + 16 * (ch ^ sw);
}

__device__ __forceinline__ i16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(p));
}

// Transposed fragment (MFMA row index = a tile column, k index running down the rows) from
// the two precomputed lane addresses of tr_offsets.  Must run with all 64 lanes active.
__device__ __forceinline__ bf16x8 tr_frag_at(const char* pa, const char* pb) {
  const i16x4 a = tr_read(pa);
  const i16x4 b = tr_read(pb);
  // Whole-vector concatenation: per-element extraction of the tr-read result miscompiles on
  // ROCm 7.2 (hipcc duplicates the low dword; caught by tests/native/probe_fragments.hip).
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const i16x8 ab = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, ab);
}

// Lane offsets of the transposed fragment for output column tile d (columns 32d..32d+31) and
// k rows {4h+q .. +3} (A half) and {4h+q+8 ..} (B half) of a 16-row step; add 16*step*rowbytes.
template <int W>
__device__ __forceinline__ void tr_offsets(int d, int& oa, int& ob) {
  const int lane = threadIdx.x & 63;
  const int i = lane & 15, g = lane >> 4;
  const int q = i >> 2, p = i & 3;
  const int ch = ((32 * d + 16 * (g & 1)) >> 3) + (p >> 1);
  const int half = 8 * (p & 1);
  const int row = 4 * (g >> 1) + q;
  oa = off<W>(row, ch) + half;
  ob = off<W>(row + 8, ch) + half;
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 lds_frag(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

// Pack accumulator registers 8s .. 8s+7 into a bf16 operand fragment.
__device__ __forceinline__ bf16x8 pack8(const f32x16& x, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = static_cast<__bf16>(x[8 * s + j]);
  return r;
}

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Reductions of x over the lane pair (l, l ^ 32): v_permlane32_swap(x, x) leaves x[l & 31] and
// x[32 + (l & 31)] in its two results on every lane (VALU only; __shfl_xor compiles to
// ds_bpermute_b32, whose LDS round trip sits on the softmax's dependency chain).  max and +
// are commutative, so the result is bitwise the shuffle form's.
__device__ __forceinline__ float pair_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Scheduling hints (T19) for a region of n MFMAs fed by n*rpm LDS reads: keep `ahead` reads in
// flight in front of the MFMA chain instead of hipcc's read -> wait -> MFMA serialisation.
constexpr int kSchedMfma = 0x008, kSchedDsRead = 0x100;
template <int N, int RPM, int AHEAD>
__device__ __forceinline__ void pipeline_reads() {
  __builtin_amdgcn_sched_group_barrier(kSchedDsRead, AHEAD * RPM, 0);
#pragma unroll
  for (int i = 0; i < N - AHEAD; ++i) {
    __builtin_amdgcn_sched_group_barrier(kSchedMfma, 1, 0);
    __builtin_amdgcn_sched_group_barrier(kSchedDsRead, RPM, 0);
  }
  __builtin_amdgcn_sched_group_barrier(kSchedMfma, AHEAD, 0);
}

// Forward: wave priority around the MFMA phases -- the wave issuing a GEMM block outranks its
// SIMD partner, which meanwhile runs its softmax on the VALU.  Round 6's bounded attention
// attempt (profiles/r6/attention/): forward +1.5 % at the 8B shape, +2.7 % at S 8192, rime
// neutral; the same around the dQ kernel's MFMA phases was neutral and is not used.
__device__ __forceinline__ void prio_hi() { __builtin_amdgcn_s_setprio(1); }
__device__ __forceinline__ void prio_lo() { __builtin_amdgcn_s_setprio(0); }

// Row of accumulator register `reg` for lane half h (32x32 C/D map).
__device__ __forceinline__ int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }
// The lane-independent part: acc_row(reg, h) == acc_row0(reg) + 4h, a compile-time constant, so
// a mask test against a row becomes one compare with a per-lane threshold.
constexpr int acc_row0(int reg) { return (reg & 3) + 8 * (reg >> 2); }

// Attention-probability dropout (GPT-2's attn_pdrop), regenerated in the backward
// instead of stored.  The keep decision of (query q, key k) -- sequence-relative indices of
// sequence s0 = cu[seq], query head hd -- is byte (k & 3) of word (q & 3) of
//     Philox4x32-10(counter = {k & ~3, s0 + (q & ~3), hd, offset lo}, key = {seed lo, seed hi ^ offset hi})
// compared with thr = round(keep * 256): kept iff byte < thr, so the keep probability is exactly
// thr / 256 and kept probabilities are scaled by 256 / thr (unbiased).  One Philox call covers a
// 4 x 4 (query, key) block, which matches both accumulator layouts: a forward / dQ lane owns one
// query and runs of 4 consecutive keys (one word per call), a dK/dV lane one key and runs of 4
// consecutive queries (one byte of each word).  The CPU reference (dtg.ops._cpu) implements the
// same function, so the tests check the kernels' masks bit for bit.
struct DropCfg {
  uint32_t k0, k1, off;  // seed (low, high word), per-call offset
  int thr;               // keep iff random byte < thr (0..256)
  float scale;           // 256 / thr
  // Device words {seed lo, seed hi, offset lo, offset hi} (an int64 [2] tensor) that override
  // k0 / k1 / off when set: the forward's draw from torch's CUDA generator, written by
  // drop_rng_kernel on the stream, read back by the backward.  Under HIP-graph capture the
  // generator hands out device pointers refreshed before every replay, so each replay of a
  // captured step draws a new mask (the values baked into a kernel argument would repeat it).
  const uint32_t* rng;
};

// The kernel's effective dropout key / offset (wave-uniform loads of dc.rng when set).
__device__ __forceinline__ DropCfg resolve_drop(const DropCfg& in) {
  DropCfg d = in;
  if (d.rng != nullptr) {
    d.k0 = d.rng[0];
    d.k1 = d.rng[1] ^ d.rng[3];  // the offset's high word keys the generator (no wrap at 2^32)
    d.off = d.rng[2];
  }
  return d;
}

__device__ __forceinline__ void philox4x32_10(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint32_t lo0 = 0xD2511F53u * c[0], hi0 = __umulhi(0xD2511F53u, c[0]);
    const uint32_t lo1 = 0xCD9E8D57u * c[2], hi1 = __umulhi(0xCD9E8D57u, c[2]);
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
  }
}

// Forward / dQ layout: lane query q, registers 4g + e = keys key0 + 8g + 4h + e.  Zeroes the
// dropped entries of x (one 32-key half) and returns nothing else; keep*scale is applied by the
// caller where it folds into a constant.
__device__ __forceinline__ void drop_row_half(const DropCfg& dc, int s0, int q, int head, int key0, int h,
                                              f32x16& x) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    uint32_t c[4] = {(uint32_t)(key0 + 8 * g + 4 * h), (uint32_t)(s0 + (q & ~3)), (uint32_t)head, dc.off};
    philox4x32_10(c, dc.k0, dc.k1);
    const int ws = q & 3;
    const uint32_t wd = ws == 0 ? c[0] : ws == 1 ? c[1] : ws == 2 ? c[2] : c[3];
#pragma unroll
    for (int e = 0; e < 4; ++e) x[4 * g + e] = (int)((wd >> (8 * e)) & 255u) < dc.thr ? x[4 * g + e] : 0.f;
  }
}

// Buffer descriptor over `bytes` bytes at p, built from provably wave-uniform values (T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, int bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo),
                                           (short)0, n, 0x00020000);
}

// Register-staged copy of R rows x W bf16 (token stride `stride`) into a swizzled LDS image.
// Rows at or past `nvalid` are outside the descriptor's range and read as zeros.
template <int R, int W, int NT>
struct Stager {
  static constexpr int NCH = W / 8;
  static constexpr int PER = (R * NCH) / NT;
  static constexpr int RSTEP = NT / NCH;  // rows between a thread's consecutive chunks
  static_assert((R * NCH) % NT == 0 && NT % NCH == 0 && RSTEP % 16 == 0, "tile split");
  u16x8 regs[PER];
  __device__ __forceinline__ void load(const uint16_t* base, int64_t stride, int nvalid) {
    const int row0 = threadIdx.x / NCH, ch = threadIdx.x % NCH;
    const int bytes = nvalid > 0 ? static_cast<int>((nvalid - 1) * stride * 2 + W * 2) : 0;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(base, bytes);
    const int s2 = static_cast<int>(stride) * 2;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int voff = (row0 + i * RSTEP) * s2 + ch * 16;
      regs[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0));
    }
  }
  __device__ __forceinline__ void store(char* tile) const {
    const int o = off<W>(threadIdx.x / NCH, threadIdx.x % NCH);
#pragma unroll
    for (int i = 0; i < PER; ++i) *reinterpret_cast<u16x8*>(tile + o + i * RSTEP * W * 2) = regs[i];
  }
};

// One lane's 16-byte slices of a row: elements [16c + 8h, +8) for c < D/16 (zero if !ok).
template <int NC>
__device__ __forceinline__ void load_row_frags(const uint16_t* row, bool ok, int h, bf16x8* out) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const u16x8 z{0, 0, 0, 0, 0, 0, 0, 0};
    const u16x8 v = ok ? *reinterpret_cast<const u16x8*>(row + 16 * c + 8 * h) : z;
    out[c] = __builtin_bit_cast(bf16x8, v);
  }
}

// Grid order.  Workgroups are dispatched x-fastest and handed to the 8 XCDs round-robin, so
//  * the block index goes in z (slowest) with the heaviest causal blocks first across ALL
//    (head, sequence) pairs -- the tail of the launch is then made of the lightest blocks;
//  * the head index x is permuted so that the query heads of one GQA group (which read the same
//    K/V) land on the same XCD and share its L2: head = (x % hkv) * group + x / hkv.
__device__ __forceinline__ int grid_head(int x, int hq, int hkv) {
  const int group = hq / hkv;
  return (x % hkv) * group + x / hkv;
}

// Row-per-lane epilogue of a transposed 32x32 accumulator (lane = output row, registers =
// columns 32d + 8g + 4h + e) widened per CDNA guide T21: v_permlane32_swap pairs column groups
// (2j, 2j+1) so that lanes 0-31 hold 16 contiguous bytes of group 2j and lanes 32-63 those of
// group 2j+1 -- 8 dwordx4 stores per lane instead of 16 dwordx2 (the store tail is issue-bound).
// Must run with all 64 lanes active; `ok` only masks the stores.
template <int ND>
__device__ __forceinline__ void store_rows_wide(const f32x16* acc, float scale, uint16_t* row, bool ok) {
  const int h = (threadIdx.x & 63) >> 5;
#pragma unroll
  for (int d = 0; d < ND; ++d) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      uint32_t w[4];  // packed bf16 pairs: w[0..1] group 2j, w[2..3] group 2j+1
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int base = 4 * (2 * j + u);
        w[2 * u + 0] = (uint32_t)f2bf(acc[d][base + 0] * scale) | ((uint32_t)f2bf(acc[d][base + 1] * scale) << 16);
        w[2 * u + 1] = (uint32_t)f2bf(acc[d][base + 2] * scale) | ((uint32_t)f2bf(acc[d][base + 3] * scale) << 16);
      }
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const auto r = __builtin_amdgcn_permlane32_swap(w[x], w[2 + x], false, false);
        w[x] = r[0];
        w[2 + x] = r[1];
      }
      if (ok) *reinterpret_cast<uint4*>(row + 32 * d + 16 * j + 8 * h) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

// Keys of query sequence `seq`: by default the sequence's own tokens (self-attention over
// cu_seqlens).  With explicit per-sequence key ranges (kstart/klen: context parallelism, where a
// local query chunk attends to a prefix of the gathered full row) the causal mask is
// bottom-right aligned as in FlashAttention-2 varlen: query i of a sequence of len_q queries
// attends to keys <= i + (len_k - len_q).
struct KeyRange {
  int start, len, off;
};
__device__ __forceinline__ KeyRange key_range(const int* kstart, const int* klen, int seq, int s0, int seqlen) {
  if (kstart == nullptr) return KeyRange{s0, seqlen, 0};
  const int n = klen[seq];
  return KeyRange{kstart[seq], n, n - seqlen};
}

struct FwdParams {
  const uint16_t *q, *k, *v;
  int64_t sq, sk, sv;  // token strides (elements)
  uint16_t* o;         // [T, Hq, D] contiguous
  float* lse;          // [Hq, T]
  const int* cu;       // [nseq + 1]
  int64_t T;
  int hq, hkv;
  float c2;  // softmax scale * log2(e)
  long long* stamps;  // diagnostic path only (flash_attn_fwd_stamped): 6 words per workgroup
  const int *kstart, *klen;  // optional per-sequence key ranges (see KeyRange)
  int window;  // causal sliding window (Mistral): query i sees keys in (i + off - window, i + off]; 0 = none
  DropCfg drop;  // DROP instantiations only
};

// In-kernel timeline stamps (CDNA guide §7 'In-kernel stamps'): constant-rate 100 MHz clock,
// one lane per workgroup, plus the hardware wave id / XCC id of the workgroup's wave 0.
__device__ __forceinline__ void fa_stamp(long long* st, int slot, int k) {
  if (st != nullptr && threadIdx.x == 0) {
    st[slot * 6 + k] = (long long)__builtin_amdgcn_s_memrealtime();
    if (k == 0) {
      st[slot * 6 + 4] = (long long)__builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_REG_HW_ID
      st[slot * 6 + 5] = (long long)__builtin_amdgcn_s_getreg(20 | (31 << 11));  // HW_REG_XCC_ID
    }
  }
}

constexpr int kFwdBQ = 128;  // query rows per work item (4 waves x 32)
constexpr int kFwdBK = 64;   // keys per K/V tile

// WIN: sliding-window instantiation (only launched with P.window > 0); without it every window
// term folds to a compile-time 0 and the kernel is the plain causal one.
template <int D, bool CAUSAL, bool WIN = false, bool DROP = false>
__global__ __launch_bounds__(256, 2) void fwd_kernel(FwdParams P) {
  [[maybe_unused]] const DropCfg dcfg = DROP ? resolve_drop(P.drop) : P.drop;
  constexpr int RB = 2 * D;
  constexpr int TILE = kFwdBK * RB;
  constexpr int NC = D / 16;  // k-steps over head_dim
  constexpr int ND = D / 32;  // 32-wide d tiles of the output
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [K0 | V0 | K1 | V1]

  fa_stamp(P.stamps, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), 0);
  const int seq = blockIdx.y, head = grid_head(blockIdx.x, P.hq, P.hkv);
  const int s0 = P.cu[seq];
  const int seqlen = P.cu[seq + 1] - s0;
  const int qb = CAUSAL ? (gridDim.z - 1 - blockIdx.z) : blockIdx.z;  // heavy blocks first
  const int q0 = qb * kFwdBQ;
  if (q0 >= seqlen) return;
  const KeyRange kr = key_range(P.kstart, P.klen, seq, s0, seqlen);
  const int klen = kr.len, koff_c = kr.off;  // causal: query i attends keys <= i + koff_c
  const int kvh = head / (P.hq / P.hkv);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int qrow = q0 + 32 * w + r;  // this lane's query (sequence-relative)

  bf16x8 qf[NC];  // Q^T fragments for all k-steps
  // Q rows arrive as whole 256-B lines (the K/V stager's coalesced buffer loads) and are turned
  // into fragments through LDS (fragment-shaped loads straight to registers, 32 rows x 32 B per
  // instruction, were slower: profiles/r3).
  Stager<kFwdBQ, D, 256> sq;
  sq.load(P.q + (int64_t)(s0 + q0) * P.sq + (int64_t)head * D, P.sq, seqlen - q0);
  int koff[NC], toa[ND], tob[ND];
#pragma unroll
  for (int c = 0; c < NC; ++c) koff[c] = off<D>(r, 2 * c + h);
#pragma unroll
  for (int d = 0; d < ND; ++d) tr_offsets<D>(d, toa[d], tob[d]);

  const int kv_end = CAUSAL ? min(klen, q0 + kFwdBQ + koff_c) : klen;
  const int ntiles = (kv_end + kFwdBK - 1) / kFwdBK;
  // sliding window: the first key any query of this block sees is q0 + koff_c - window + 1
  const int win = (CAUSAL && WIN) ? P.window : 0;
  const int t_begin = win > 0 ? max(0, q0 + koff_c - win + 1) / kFwdBK : 0;
  const uint16_t* kbase = P.k + (int64_t)kr.start * P.sk + (int64_t)kvh * D;
  const uint16_t* vbase = P.v + (int64_t)kr.start * P.sv + (int64_t)kvh * D;

  f32x16 acc[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) acc[i] = f32x16{};
  float m = -INFINITY, l = 0.f;

  Stager<kFwdBK, D, 256> sk, sv;
  sk.load(kbase + (int64_t)t_begin * kFwdBK * P.sk, P.sk, klen - t_begin * kFwdBK);
  sv.load(vbase + (int64_t)t_begin * kFwdBK * P.sv, P.sv, klen - t_begin * kFwdBK);
  sq.store(smem + 2 * TILE);  // the second K/V buffer is free until tile 0 ends
  sk.store(smem);
  sv.store(smem + TILE);
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NC; ++c) qf[c] = lds_frag(smem + 2 * TILE + 32 * w * RB + koff[c]);
  __syncthreads();  // every wave holds its Q before tile 0 restages that buffer
  fa_stamp(P.stamps, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), 1);

  const int wave_q0 = q0 + 32 * w, wave_qmax = wave_q0 + 31;
  // Tile loop unrolled by two so the double-buffer offsets are compile-time immediates.
  auto tile_step = [&](int t, auto buf) {
    constexpr int B = decltype(buf)::value;
    const int kt0 = t * kFwdBK;
    const bool more = t + 1 < ntiles;
    if (more) {
      const int nk = kt0 + kFwdBK;
      sk.load(kbase + (int64_t)nk * P.sk, P.sk, klen - nk);
      sv.load(vbase + (int64_t)nk * P.sv, P.sv, klen - nk);
    }
    const char* K = smem + B * 2 * TILE;
    const char* V = K + TILE;
    // wave-uniform skip of tiles above the diagonal (or entirely before every query's window)
    if ((!CAUSAL || kt0 <= wave_qmax + koff_c) && (win == 0 || kt0 + kFwdBK - 1 >= wave_q0 + koff_c - win + 1)) {
      f32x16 s[2];
      __builtin_amdgcn_sched_barrier(0);
      prio_hi();
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        bf16x8 kf[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) kf[c] = lds_frag(K + kt * 32 * RB + koff[c]);
        s[kt] = f32x16{};
#pragma unroll
        for (int c = 0; c < NC; ++c) s[kt] = mfma(kf[c], qf[c], s[kt]);
      }
      pipeline_reads<2 * NC, 1, 4>();
      __builtin_amdgcn_sched_barrier(0);
      prio_lo();
      if ((CAUSAL && kt0 + kFwdBK - 1 > wave_q0 + koff_c) || kt0 + kFwdBK > klen ||
          (win > 0 && kt0 < wave_qmax + koff_c - win + 1)) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          // key = kt0 + 32 kt + acc_row is masked when key > min(qrow + koff_c, klen - 1), or
          // (sliding window) key < qrow + koff_c - win + 1
          const int lim = (CAUSAL ? min(qrow + koff_c, klen - 1) : klen - 1) - (kt0 + 32 * kt + 4 * h);
          const int llim = win > 0 ? qrow + koff_c - win + 1 - (kt0 + 32 * kt + 4 * h) : INT_MIN;
#pragma unroll
          for (int i = 0; i < 16; ++i)
            s[kt][i] = (acc_row0(i) > lim || acc_row0(i) < llim) ? -INFINITY : s[kt][i];
        }
      }
      // (Four independent partial max / sum chains instead of one 32-deep chain measured no gain
      // at the 8B shape and -2 % on rime, profiles/r4/s17: hipcc packs the partial sums into
      // v_pk_add_f32, and the other wave on the SIMD already fills the chain's latency.)
      float mx = s[0][0];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[kt][i]);
      }
      mx = pair_max(mx) * P.c2;
      if (__builtin_amdgcn_ballot_w64(mx > m + kRescaleThreshold) != 0) {
        const float mn = fmaxf(m, mx);
        const float alpha = (mn == -INFINITY) ? 1.f : fexp2(m - mn);
        l *= alpha;
#pragma unroll
        for (int d = 0; d < ND; ++d) acc[d] *= alpha;
        m = mn;
      }
      const float mu = (m == -INFINITY) ? 0.f : m;
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = fexp2(__builtin_fmaf(s[kt][i], P.c2, -mu));
          s[kt][i] = p;
          rs += p;
        }
      }
      l += rs;  // the softmax normaliser counts every probability, dropped or not
      if constexpr (DROP) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) drop_row_half(dcfg, s0, qrow, head, kt0 + 32 * kt, h, s[kt]);
      }
      bf16x8 pf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) pf[j] = pack8(s[j >> 1], j & 1);
      __builtin_amdgcn_sched_barrier(0);
      prio_hi();
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // 16-key steps
        const char* vb = V + 16 * j * RB;
        bf16x8 vt[ND];
#pragma unroll
        for (int d = 0; d < ND; ++d) vt[d] = tr_frag_at(vb + toa[d], vb + tob[d]);
#pragma unroll
        for (int d = 0; d < ND; ++d) acc[d] = mfma(vt[d], pf[j], acc[d]);
      }
      pipeline_reads<4 * ND, 2, 3>();
      __builtin_amdgcn_sched_barrier(0);
      prio_lo();
    }
    if (more) {
      char* nb = smem + (1 - B) * 2 * TILE;
      sk.store(nb);
      sv.store(nb + TILE);
    }
    __syncthreads();
  };
  int t = t_begin;
  for (; t + 1 < ntiles; t += 2) {
    tile_step(t, std::integral_constant<int, 0>{});
    tile_step(t + 1, std::integral_constant<int, 1>{});
  }
  if (t < ntiles) tile_step(t, std::integral_constant<int, 0>{});
  fa_stamp(P.stamps, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), 2);

  const float lt = pair_sum(l);
  const float inv = (lt > 0.f ? 1.f / lt : 0.f) * (DROP ? P.drop.scale : 1.f);
  uint16_t* op = P.o + ((int64_t)(s0 + min(qrow, seqlen - 1)) * P.hq + head) * D;
  store_rows_wide<ND>(acc, inv, op, qrow < seqlen);
  if (qrow < seqlen && h == 0)
    P.lse[(int64_t)head * P.T + s0 + qrow] = (lt > 0.f) ? (m + log2f(lt)) * kLn2 : -INFINITY;
  if (P.stamps != nullptr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    fa_stamp(P.stamps, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), 3);
  }
}

struct BwdParams {
  const uint16_t *q, *k, *v, *dout, *o;
  int64_t sq, sk, sv;  // token strides of q, k, v (dout and o are contiguous [T, Hq, D])
  const float* lse;    // [Hq, T]
  float* delta;        // [Hq, T]: written by bwd_dq_kernel, read by bwd_dkdv_kernel
  uint16_t *dq, *dk, *dv;  // [T, H, D] views
  int64_t sdq, sdk, sdv;   // token strides of dq, dk, dv
  const int* cu;
  int64_t T;
  int hq, hkv;
  float scale, c2;
  const int *kstart, *klen;  // optional per-sequence key ranges (see KeyRange)
  int window;                // causal sliding window, as FwdParams::window
  // dK/dV with the query items of each key block split over `nsplit` workgroups (grids too small
  // for the chip: one KV head per TP rank): f32 partials [nsplit, T, Hkv, D], summed in split
  // order by bwd_kv_combine_kernel (deterministic).  nsplit <= 1: bf16 dK / dV written directly.
  float *dk_part, *dv_part;
  int nsplit;
  DropCfg drop;  // DROP instantiations only
  // Optional RoPE backward fused into the dQ / dK epilogues (flash_attn_bwd_qkv_rope): f32
  // tables [max_pos, D/2] and int64 position ids [T]; null = none.
  const float *rope_cos, *rope_sin;
  const int64_t* rope_pos;
};

// Inverse rotary rotation of a row-per-lane accumulator (lane = row, registers = columns
// 32d + 8g + 4h + e) in place, in f32 before the single bf16 rounding of the store: the backward
// of q' = q cos + rotate_half(q) sin, i.e. (x1, x2) -> (x1 cos + x2 sin, x2 cos - x1 sin) for the
// column pairs (i, i + D/2), which live in tiles d and d + ND/2 of the same register.  Same
// semantics as rope_kernel(inverse = true), one rounding fewer.
template <int ND>
__device__ __forceinline__ void rope_inv_rows(f32x16* acc, const float* cos_t, const float* sin_t, int64_t p) {
  constexpr int HT = ND / 2;     // tiles in the first half
  constexpr int HALF = 16 * ND;  // D / 2
  const int h = (threadIdx.x & 63) >> 5;
  const float* cp = cos_t + p * HALF;
  const float* sp = sin_t + p * HALF;
#pragma unroll
  for (int d = 0; d < HT; ++d) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int i = 32 * d + 8 * g + 4 * h;
      const float4 c = *reinterpret_cast<const float4*>(cp + i);
      const float4 sn = *reinterpret_cast<const float4*>(sp + i);
      const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * g + e;
        const float x1 = acc[d][r], x2 = acc[d + HT][r];
        acc[d][r] = x1 * cc[e] + x2 * ss[e];
        acc[d + HT][r] = x2 * cc[e] - x1 * ss[e];
      }
    }
  }
}

constexpr int kDqBQ = 128;  // query rows per workgroup (4 waves x 32)
constexpr int kDqBK = 64;   // keys per K/V tile
constexpr int kKvBK = 128;  // keys per workgroup (4 waves x 32)
constexpr int kKvBQ = 32;   // query rows per item

// dQ = scale * sum_keys dS K, query-stationary (the forward's structure).  Also writes
// delta = rowsum(dO * O) for its rows, which bwd_dkdv_kernel (launched after it) reads.
template <int D, bool CAUSAL, int OCC, bool WIN = false, bool DROP = false>
__global__ __launch_bounds__(256, OCC) void bwd_dq_kernel(BwdParams P) {
  [[maybe_unused]] const DropCfg dcfg = DROP ? resolve_drop(P.drop) : P.drop;
  constexpr int RB = 2 * D;
  constexpr int TILE = kDqBK * RB;
  constexpr int NC = D / 16;
  constexpr int ND = D / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [K0 | V0 | K1 | V1]

  const int seq = blockIdx.y, head = grid_head(blockIdx.x, P.hq, P.hkv);
  const int s0 = P.cu[seq];
  const int seqlen = P.cu[seq + 1] - s0;
  const int qb = CAUSAL ? (gridDim.z - 1 - blockIdx.z) : blockIdx.z;  // heavy blocks first
  const int q0 = qb * kDqBQ;
  if (q0 >= seqlen) return;
  const KeyRange kr = key_range(P.kstart, P.klen, seq, s0, seqlen);
  const int klen = kr.len, koff_c = kr.off;
  const int kvh = head / (P.hq / P.hkv);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int qrow = q0 + 32 * w + r;
  const bool qok = qrow < seqlen;
  const int64_t t_row = s0 + (qok ? qrow : seqlen - 1);

  int koff[NC], toa[ND], tob[ND];
#pragma unroll
  for (int c = 0; c < NC; ++c) koff[c] = off<D>(r, 2 * c + h);
#pragma unroll
  for (int d = 0; d < ND; ++d) tr_offsets<D>(d, toa[d], tob[d]);

  const int kv_end = CAUSAL ? min(klen, q0 + kDqBQ + koff_c) : klen;
  const int ntiles = (kv_end + kDqBK - 1) / kDqBK;
  const int win = (CAUSAL && WIN) ? P.window : 0;  // sliding window: first key of this block's queries
  const int t_begin = win > 0 ? max(0, q0 + koff_c - win + 1) / kDqBK : 0;
  const uint16_t* kbase = P.k + (int64_t)kr.start * P.sk + (int64_t)kvh * D;
  const uint16_t* vbase = P.v + (int64_t)kr.start * P.sv + (int64_t)kvh * D;

  // Prologue: Q, dO and O rows arrive as whole lines (coalesced, range-checked buffer loads:
  // rows past the end read zeros), delta = rowsum(dO * O) is reduced in that layout, and Q / dO
  // reach their MFMA fragments through LDS (both K/V buffer pairs are free until tile 0 is
  // staged) -- instead of three sets of fragment-shaped loads (32 rows x 32 B per instruction).
  constexpr int QIMG = kDqBQ * RB;
  static_assert(2 * QIMG <= 4 * TILE, "Q + dO images must fit the K/V buffers");
  float* rowd = reinterpret_cast<float*>(smem + 4 * TILE);  // [kDqBQ] delta per row
  bf16x8 qf[NC], dof[NC];
  float delta;
  Stager<kDqBK, D, 256> sk, sv;
  {
    Stager<kDqBQ, D, 256> sq, sdo, so;
    const int64_t srow = (int64_t)(s0 + q0);
    sq.load(P.q + srow * P.sq + (int64_t)head * D, P.sq, seqlen - q0);
    sdo.load(P.dout + (srow * P.hq + head) * D, (int64_t)P.hq * D, seqlen - q0);
    so.load(P.o + (srow * P.hq + head) * D, (int64_t)P.hq * D, seqlen - q0);
    sk.load(kbase + (int64_t)t_begin * kDqBK * P.sk, P.sk, klen - t_begin * kDqBK);
    sv.load(vbase + (int64_t)t_begin * kDqBK * P.sv, P.sv, klen - t_begin * kDqBK);
    {
      constexpr int NCH = D / 8, RSTEP = 256 / NCH, PER = kDqBQ / RSTEP;
      const int row0 = threadIdx.x / NCH, ch = threadIdx.x % NCH;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        float part = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) part += bf2f(sdo.regs[i][j]) * bf2f(so.regs[i][j]);
#pragma unroll
        for (int x = 1; x < NCH; x <<= 1) part += __shfl_xor(part, x, 64);  // the row's NCH lanes
        if (ch == 0) rowd[row0 + i * RSTEP] = part;
      }
    }
    sq.store(smem);
    sdo.store(smem + QIMG);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      qf[c] = lds_frag(smem + 32 * w * RB + koff[c]);
      dof[c] = lds_frag(smem + QIMG + 32 * w * RB + koff[c]);
    }
    delta = rowd[32 * w + r];
    __syncthreads();  // every wave holds its fragments before tile 0 overwrites the images
  }
  if (qok && h == 0) P.delta[(int64_t)head * P.T + s0 + qrow] = delta;
  const float lse2 = qok ? P.lse[(int64_t)head * P.T + s0 + qrow] * kLog2e : 0.f;

  f32x16 acc[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) acc[i] = f32x16{};

  sk.store(smem);
  sv.store(smem + TILE);
  __syncthreads();

  const int wave_q0 = q0 + 32 * w, wave_qmax = wave_q0 + 31;
  // The three pieces of a 32-key half: S / dP MFMAs, softmax -> dS fragments, dQ MFMAs.
  auto sd_mfma = [&](const char* K, const char* V, int kt, f32x16& s, f32x16& dp) {
    bf16x8 f[NC], g[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) f[c] = lds_frag(K + kt * 32 * RB + koff[c]);
#pragma unroll
    for (int c = 0; c < NC; ++c) s = mfma(f[c], qf[c], s);
#pragma unroll
    for (int c = 0; c < NC; ++c) g[c] = lds_frag(V + kt * 32 * RB + koff[c]);
#pragma unroll
    for (int c = 0; c < NC; ++c) dp = mfma(g[c], dof[c], dp);
  };
  // Does any element of the 32-key half at key0 need the causal / length / window mask?
  auto half_masked = [&](int key0) {
    return (CAUSAL && key0 + 31 > wave_q0 + koff_c) || key0 + 32 > klen ||
           (win > 0 && key0 < wave_qmax + koff_c - win + 1);
  };
  auto softmax_ds = [&](int key0, f32x16& s, const f32x16& dp, bf16x8* dsf) {
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = fexp2(__builtin_fmaf(s[i], P.c2, -lse2));
    if (half_masked(key0)) {
      const int lim = (CAUSAL ? min(qrow + koff_c, klen - 1) : klen - 1) - (key0 + 4 * h);
      const int llim = win > 0 ? qrow + koff_c - win + 1 - (key0 + 4 * h) : INT_MIN;
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = (acc_row0(i) > lim || acc_row0(i) < llim) ? 0.f : s[i];
    }
    if constexpr (DROP) {  // dS = P o (M dP_dropped / keep - delta); delta = rowsum(dO o O) still holds
      f32x16 z = dp;
      drop_row_half(dcfg, s0, qrow, head, key0, h, z);
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] *= z[i] * dcfg.scale - delta;
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] *= dp[i] - delta;  // dS^T / scale
    }
    dsf[0] = pack8(s, 0);
    dsf[1] = pack8(s, 1);
  };
  auto dq_mfma = [&](const char* K, int kt, const bf16x8* dsf) {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const char* kb = K + (32 * kt + 16 * st) * RB;
      bf16x8 kt_[ND];
#pragma unroll
      for (int d = 0; d < ND; ++d) kt_[d] = tr_frag_at(kb + toa[d], kb + tob[d]);
#pragma unroll
      for (int d = 0; d < ND; ++d) acc[d] = mfma(kt_[d], dsf[st], acc[d]);
    }
  };
  // Wave-uniform: a 32-key half entirely above the diagonal, past the end, or before every
  // query's sliding window contributes nothing.
  auto half_live = [&](int key0) {
    return !((CAUSAL && key0 > wave_qmax + koff_c) || key0 >= klen) &&
           !(win > 0 && key0 + 31 < wave_q0 + koff_c - win + 1);
  };
  // Tile loop unrolled by two so the double-buffer offsets are compile-time immediates.
  auto tile_step = [&](int t, auto buf) {
    constexpr int B = decltype(buf)::value;
    const int kt0 = t * kDqBK;
    const bool more = t + 1 < ntiles;
    if (more) {
      const int nk = kt0 + kDqBK;
      sk.load(kbase + (int64_t)nk * P.sk, P.sk, klen - nk);
      sv.load(vbase + (int64_t)nk * P.sv, P.sv, klen - nk);
    }
    const char* K = smem + B * 2 * TILE;
    const char* V = K + TILE;
    const bool live0 = half_live(kt0), live1 = half_live(kt0 + 32);
    {  // (a software-pipelined body -- half 1's S / dP under half 0's softmax -- measured no
       // faster, bitwise equal: profiles/r3_s09)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        if (!(kt == 0 ? live0 : live1)) continue;
        f32x16 s = f32x16{}, dp = f32x16{};
        __builtin_amdgcn_sched_barrier(0);
        sd_mfma(K, V, kt, s, dp);
        pipeline_reads<2 * NC, 1, 4>();
        __builtin_amdgcn_sched_barrier(0);
        bf16x8 dsf[2];
        softmax_ds(kt0 + 32 * kt, s, dp, dsf);
        __builtin_amdgcn_sched_barrier(0);
        dq_mfma(K, kt, dsf);
        pipeline_reads<2 * ND, 2, 3>();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (more) {
      char* nb = smem + (1 - B) * 2 * TILE;
      sk.store(nb);
      sv.store(nb + TILE);
    }
    __syncthreads();
  };
  int t = t_begin;
  for (; t + 1 < ntiles; t += 2) {
    tile_step(t, std::integral_constant<int, 0>{});
    tile_step(t + 1, std::integral_constant<int, 1>{});
  }
  if (t < ntiles) tile_step(t, std::integral_constant<int, 0>{});

  if (P.rope_cos != nullptr) rope_inv_rows<ND>(acc, P.rope_cos, P.rope_sin, P.rope_pos[s0 + min(qrow, seqlen - 1)]);
  store_rows_wide<ND>(acc, P.scale, P.dq + (int64_t)(s0 + min(qrow, seqlen - 1)) * P.sdq + (int64_t)head * D, qok);
}

// dK, dV, key-stationary: 4 waves x 32 keys, one wave per SIMD with the dK/dV accumulators in
// AGPRs; this lane's K and V rows live in VGPRs (they are the B operands of S = Q K^T and
// dP = dO V^T), and the workgroup sweeps (query head, 32-row slice) items with Q/dO
// double-buffered in LDS.  S and dP start from the row constants
// (-lse/scale, -delta) so p = exp2(c2 S') and dS = p dP' need no per-element subtraction;
// only the causal diagonal is masked (padded query rows carry Q = dO = 0 and contribute 0).
// D = 128 at one wave per SIMD: every value stays in registers (306 of them with 32-row items,
// 408 with the default 64-row items).  Forced to two waves the allocator spills ~50 dwords per
// lane to scratch and the kernel runs at half speed (profiles/r3_s20).
// QB: query rows per item, 32 or 64.  QB = 64 runs each item as two 32-row halves in a software
// pipeline (S/dP MFMAs of half 1 under the softmax VALU of half 0, dK/dV MFMAs of half 0 under
// the softmax of half 1): at one wave per SIMD there is no partner wave to fill the matrix pipe
// while a wave does its VALU, so the overlap has to come from the wave's own instruction stream.
template <int D, bool CAUSAL, int PF, bool WIN = false, int QB = kKvBQ, bool DROP = false>
__global__ __launch_bounds__(256, D == 128 ? 1 : 2) void bwd_dkdv_kernel(BwdParams P) {
  [[maybe_unused]] const DropCfg dcfg = DROP ? resolve_drop(P.drop) : P.drop;
  static_assert(QB == 32 || QB == 64, "query rows per item");
  constexpr int RB = 2 * D;
  constexpr int NC = D / 16;
  constexpr int ND = D / 32;
  constexpr int SLICE = QB * RB;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [Q0 | dO0 | Q1 | dO1 | rowc]
  char* qd = smem;
  float* rowc = reinterpret_cast<float*>(qd + 4 * SLICE);      // [2][-lse/scale x QB, -delta x QB]

  const int seq = blockIdx.y, kvh = blockIdx.x;
  const int s0 = P.cu[seq];
  const int seqlen = P.cu[seq + 1] - s0;
  const KeyRange kr = key_range(P.kstart, P.klen, seq, s0, seqlen);
  const int klen = kr.len, koff_c = kr.off;  // query q attends key k iff k <= q + koff_c
  const int nsplit = P.nsplit > 1 ? P.nsplit : 1;
  const int split = blockIdx.z % nsplit;
  const int kb = (blockIdx.z / nsplit) * kKvBK;  // z = 0 first: the heaviest causal key blocks
  if (kb >= klen) return;
  const int group = P.hq / P.hkv;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int wkey0 = kb + 32 * w;
  const int key = wkey0 + r;

  bf16x8 kf[NC], vf[NC];
  {
    const bool ok = key < klen;
    const int64_t t = kr.start + (ok ? key : klen - 1);
    load_row_frags<NC>(P.k + t * P.sk + (int64_t)kvh * D, ok, h, kf);
    load_row_frags<NC>(P.v + t * P.sv + (int64_t)kvh * D, ok, h, vf);
  }
  int roff[NC], toa[ND], tob[ND];
#pragma unroll
  for (int c = 0; c < NC; ++c) roff[c] = off<D>(r, 2 * c + h);
#pragma unroll
  for (int d = 0; d < ND; ++d) tr_offsets<D>(d, toa[d], tob[d]);

  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    dk[i] = f32x16{};
    dv[i] = f32x16{};
  }

  const int first_slice = CAUSAL ? (max(0, kb - koff_c) / QB) : 0;
  const int win = (CAUSAL && WIN) ? P.window : 0;  // sliding window: the last query that sees this block
  const int end_slice = win > 0 ? min((seqlen + QB - 1) / QB, (kb + kKvBK - 1 - koff_c + win - 1) / QB + 1)
                                : (seqlen + QB - 1) / QB;
  const int per_head = max(0, end_slice - first_slice);
  const int nitems = per_head * group;
  const float inv_scale = 1.f / P.scale;

  // Register-staged items: with PF = 2, item j is loaded into set j % 2 two items ahead of its
  // use, so its global loads have a whole item of compute to land in (PF = 1: one set, loads
  // issued one item ahead and waited for at the end of the current item).
  struct Item {
    Stager<QB, D, 256> q, dout;
    uint32_t lse, dlt;  // raw f32 bits of this lane's row (threadIdx.x & (QB - 1))
  };
  Item ia, ib;
  auto load_item = [&](Item& X, int it) {
    const int hqi = kvh * group + it / per_head;
    const int qs = (first_slice + it % per_head) * QB;
    const int nv = seqlen - qs;
    X.q.load(P.q + (int64_t)(s0 + qs) * P.sq + (int64_t)hqi * D, P.sq, nv);
    X.dout.load(P.dout + ((int64_t)(s0 + qs) * P.hq + hqi) * D, (int64_t)P.hq * D, nv);
    // The rows' lse / delta through range-checked buffer loads (rows past the sequence end read
    // 0), issued by every lane, kept raw and combined only in store_item.  A lane-divergent load
    // (or math on it here) made hipcc put an s_waitcnt vmcnt(0) right behind it -- which also
    // waits for the Q/dO prefetch just issued, exposing its whole latency in every item.  The
    // volatile bit (aux bit 31) keeps the loads from being sunk into store_item's branch.
    const int nrow = min(QB, seqlen - qs);
    const int64_t ro = (int64_t)hqi * P.T + s0 + qs;
    const int vo = (threadIdx.x & (QB - 1)) * 4;
    X.lse = __builtin_amdgcn_raw_buffer_load_b32(make_rsrc(P.lse + ro, nrow * 4), vo, 0, (int)(1u << 31));
    X.dlt = __builtin_amdgcn_raw_buffer_load_b32(make_rsrc(P.delta + ro, nrow * 4), vo, 0, (int)(1u << 31));
  };
  auto store_item = [&](const Item& X, int buf) {
    X.q.store(qd + buf * 2 * SLICE);
    X.dout.store(qd + buf * 2 * SLICE + SLICE);
    if (threadIdx.x < 2 * QB) {  // threads 0..QB-1: -lse/scale, QB..2QB-1: -delta of row threadIdx.x & (QB - 1)
      const float l = __builtin_bit_cast(float, X.lse), dl = __builtin_bit_cast(float, X.dlt);
      rowc[buf * 2 * QB + threadIdx.x] = (threadIdx.x & QB) ? -dl : -l * inv_scale;
    }
  };
  // Dropout in the key-stationary layout (DROP): s holds P, dp holds dO.V^T (started from 0, not
  // -delta), cnd the rows' -delta; afterwards s = the dropped, rescaled probabilities (dV's
  // operand) and dp = dS / scale.
  auto drop_cols = [&](int qsu, int hqi, f32x16& s, f32x16& dp, const float* cnd) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint32_t c[4] = {(uint32_t)(key & ~3), (uint32_t)(s0 + qsu + 8 * g + 4 * h), (uint32_t)hqi, dcfg.off};
      philox4x32_10(c, dcfg.k0, dcfg.k1);
      const int sh = 8 * (key & 3);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * g + e;
        const bool keep = (int)((c[e] >> sh) & 255u) < dcfg.thr;
        const float p = s[i];
        dp[i] = p * ((keep ? dp[i] * dcfg.scale : 0.f) + cnd[acc_row(i, h)]);
        s[i] = keep ? p * dcfg.scale : 0.f;
      }
    }
  };
  auto compute = [&](int it, int buf) {
    const int qs = (first_slice + it % per_head) * QB;
    // No skip of the (at most 3 per head) slices whose queries all precede this wave's keys:
    // a branch around the dK/dV updates makes hipcc carry the accumulators through VGPR copies
    // every item; the mask zeroes those slices' contributions instead.
    {
      const char* Ql = qd + buf * 2 * SLICE;
      const char* dOl = Ql + SLICE;
      const float* c0 = rowc + buf * 2 * QB;
      f32x16 s, dp;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s[i] = c0[acc_row(i, h)];
        dp[i] = DROP ? 0.f : c0[QB + acc_row(i, h)];
      }
      __builtin_amdgcn_sched_barrier(0);
      {
        bf16x8 f[NC], g[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) f[c] = lds_frag(Ql + roff[c]);
#pragma unroll
        for (int c = 0; c < NC; ++c) s = mfma(f[c], kf[c], s);
#pragma unroll
        for (int c = 0; c < NC; ++c) g[c] = lds_frag(dOl + roff[c]);
#pragma unroll
        for (int c = 0; c < NC; ++c) dp = mfma(g[c], vf[c], dp);
      }
      pipeline_reads<2 * NC, 1, 4>();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = fexp2(s[i] * P.c2);
      if ((CAUSAL && wkey0 + 31 > qs + koff_c) || (win > 0 && qs + kKvBQ - 1 > wkey0 - koff_c + win - 1)) {
        const int lim = key - koff_c - qs - 4 * h;  // query row qs + acc_row < key - koff_c is masked
        // sliding window: query row qs + acc_row > key - koff_c + win - 1 is masked
        const int ulim = win > 0 ? key - koff_c + win - 1 - qs - 4 * h : INT_MAX;
#pragma unroll
        for (int i = 0; i < 16; ++i) s[i] = (acc_row0(i) < lim || acc_row0(i) > ulim) ? 0.f : s[i];
      }
      if constexpr (DROP) {
        drop_cols(qs, kvh * group + it / per_head, s, dp, c0 + QB);
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) dp[i] *= s[i];  // dS / scale
      }
      const bf16x8 pf[2] = {pack8(s, 0), pack8(s, 1)};
      const bf16x8 dsf[2] = {pack8(dp, 0), pack8(dp, 1)};
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const char* ob = dOl + 16 * st * RB;
        const char* qb = Ql + 16 * st * RB;
        bf16x8 a[ND], b[ND];
#pragma unroll
        for (int d = 0; d < ND; ++d) a[d] = tr_frag_at(ob + toa[d], ob + tob[d]);
#pragma unroll
        for (int d = 0; d < ND; ++d) dv[d] = mfma(a[d], pf[st], dv[d]);
#pragma unroll
        for (int d = 0; d < ND; ++d) b[d] = tr_frag_at(qb + toa[d], qb + tob[d]);
#pragma unroll
        for (int d = 0; d < ND; ++d) dk[d] = mfma(b[d], dsf[st], dk[d]);
      }
      pipeline_reads<4 * ND, 2, 3>();
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // QB = 64: halves u = 0, 1 (rows qs + 32u).  Masking is branch-free (a select per element) so
  // the halves' MFMA and VALU phases stay in one basic block the scheduler can interleave.
  auto sd_mfma = [&](const char* Ql, const char* dOl, f32x16& s, f32x16& dp) {
    bf16x8 f[NC], g[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) f[c] = lds_frag(Ql + roff[c]);
#pragma unroll
    for (int c = 0; c < NC; ++c) s = mfma(f[c], kf[c], s);
#pragma unroll
    for (int c = 0; c < NC; ++c) g[c] = lds_frag(dOl + roff[c]);
#pragma unroll
    for (int c = 0; c < NC; ++c) dp = mfma(g[c], vf[c], dp);
  };
  auto softmax_half = [&](int qsu, int hqi, const float* cnd, f32x16& s, f32x16& dp, bf16x8 (&pf)[2],
                          bf16x8 (&dsf)[2]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = fexp2(s[i] * P.c2);
    // causal: the mask runs on every half (branch-free).  Skipping it on halves that need none
    // (a wave-uniform branch) measured 1 % slower at the 8B shape and 3 % on packed rime rows
    // (profiles/r4/s17): the branch splits the halves' basic block and with it the schedule.
    if constexpr (CAUSAL) {
      const int lim = key - koff_c - qsu - 4 * h;  // query row qsu + acc_row < key - koff_c is masked
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = acc_row0(i) < lim ? 0.f : s[i];
    }
    if constexpr (DROP) {
      drop_cols(qsu, hqi, s, dp, cnd);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) dp[i] *= s[i];
    }
    pf[0] = pack8(s, 0);
    pf[1] = pack8(s, 1);
    dsf[0] = pack8(dp, 0);
    dsf[1] = pack8(dp, 1);
  };
  auto kv_mfma = [&](const char* Ql, const char* dOl, const bf16x8 (&pf)[2], const bf16x8 (&dsf)[2]) {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const char* ob = dOl + 16 * st * RB;
      const char* qb = Ql + 16 * st * RB;
      bf16x8 a[ND], b[ND];
#pragma unroll
      for (int d = 0; d < ND; ++d) a[d] = tr_frag_at(ob + toa[d], ob + tob[d]);
#pragma unroll
      for (int d = 0; d < ND; ++d) dv[d] = mfma(a[d], pf[st], dv[d]);
#pragma unroll
      for (int d = 0; d < ND; ++d) b[d] = tr_frag_at(qb + toa[d], qb + tob[d]);
#pragma unroll
      for (int d = 0; d < ND; ++d) dk[d] = mfma(b[d], dsf[st], dk[d]);
    }
  };
  auto compute64 = [&](int it, int buf) {
    const int qs = (first_slice + it % per_head) * QB;
    const char* Ql = qd + buf * 2 * SLICE;
    const char* dOl = Ql + SLICE;
    const float* c0 = rowc + buf * 2 * QB;
    f32x16 s0, dp0, s1, dp1;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      s0[i] = c0[acc_row(i, h)];
      dp0[i] = DROP ? 0.f : c0[QB + acc_row(i, h)];
      s1[i] = c0[32 + acc_row(i, h)];
      dp1[i] = DROP ? 0.f : c0[QB + 32 + acc_row(i, h)];
    }
    __builtin_amdgcn_sched_barrier(0);
    sd_mfma(Ql, dOl, s0, dp0);
    pipeline_reads<2 * NC, 1, 4>();
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 pf0[2], dsf0[2], pf1[2], dsf1[2];
    sd_mfma(Ql + 32 * RB, dOl + 32 * RB, s1, dp1);  // || softmax of half 0
    const int hqi = kvh * group + it / per_head;
    softmax_half(qs, hqi, c0 + QB, s0, dp0, pf0, dsf0);
    __builtin_amdgcn_sched_barrier(0);
    kv_mfma(Ql, dOl, pf0, dsf0);  // || softmax of half 1
    softmax_half(qs + 32, hqi, c0 + QB + 32, s1, dp1, pf1, dsf1);
    __builtin_amdgcn_sched_barrier(0);
    kv_mfma(Ql + 32 * RB, dOl + 32 * RB, pf1, dsf1);
    pipeline_reads<4 * ND, 2, 3>();
    __builtin_amdgcn_sched_barrier(0);
  };

  auto run_item = [&](int it, int buf) {
    if constexpr (QB == 64) compute64(it, buf);
    else compute(it, buf);
  };

  // Settle this lane's K/V fragment loads before the item loop, on every path into it.  Left
  // pending, hipcc's wait-count analysis carried them around the loop's back edge and put an
  // s_waitcnt vmcnt(1) / vmcnt(0) in front of the first S MFMA of every item -- a wait on the
  // Q/dO loads just issued for a later item (ISA: llvm-objdump of bwd_dkdv_kernel).  The wait
  // is the builtin (vmcnt(0); expcnt, lgkmcnt unconstrained), which the wait-count pass sees.
  // The earlier form, an empty asm with "+v" operands on the fragments, pinned them to VGPRs
  // there; the allocator then homed them in AGPRs and copied 44 AGPR -> AGPR registers every
  // item (v_accvgpr_mov; 695 -> 648 loop instructions without them).
  __builtin_amdgcn_s_waitcnt(0x0f70);

  static_assert(PF == 1 || QB == 32, "two-item prefetch only with 32-row items");
  if constexpr (PF == 2) {
    // Prefetch loads are issued unconditionally (a finished tail re-reads its last item): with
    // a branch around them hipcc's wait counting must assume they may be absent and drains
    // every outstanding load at the next store, i.e. the prefetch stops being two items deep.
    load_item(ia, 0);
    load_item(ib, min(1, nitems - 1));
    store_item(ia, 0);
    __syncthreads();
    auto step = [&](int it, auto par) {
      constexpr int S = decltype(par)::value;  // == it % 2: LDS buffer of item it
      Item& cur = S == 0 ? ia : ib;            // item it: already in LDS, its registers are free
      Item& nxt = S == 0 ? ib : ia;            // item it + 1, loaded one step ago
      load_item(cur, min(it + 2, nitems - 1));
      compute(it, S);
      if (it + 1 < nitems) store_item(nxt, S ^ 1);
      __syncthreads();
    };
    int it = 0;
    for (; it + 1 < nitems; it += 2) {
      step(it, std::integral_constant<int, 0>{});
      step(it + 1, std::integral_constant<int, 1>{});
    }
    if (it < nitems) step(it, std::integral_constant<int, 0>{});
  } else {
    // this workgroup's share of the key block's items (all of them unless split)
    const int it0 = (int)((int64_t)split * nitems / nsplit), it1 = (int)((int64_t)(split + 1) * nitems / nsplit);
    if (it0 < it1) {
      load_item(ia, it0);
      store_item(ia, it0 & 1);
    }
    __syncthreads();
    for (int it = it0; it < it1; ++it) {
      const int buf = it & 1;
      const bool more = it + 1 < it1;
      if (more) load_item(ia, it + 1);
      run_item(it, buf);
      if (more) store_item(ia, buf ^ 1);
      __syncthreads();
    }
  }

  const int64_t krow = kr.start + min(key, klen - 1);
  if (nsplit > 1) {  // f32 partials (lane = key row; registers = columns 32d + 8g + 4h + e)
    if (key < klen) {
      const int64_t o = (((int64_t)split * P.T + krow) * P.hkv + kvh) * D + 4 * h;
      float* pk = P.dk_part + o;
      float* pv = P.dv_part + o;
#pragma unroll
      for (int d = 0; d < ND; ++d) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          *reinterpret_cast<f32x4*>(pk + 32 * d + 8 * g) = f32x4{dk[d][4 * g], dk[d][4 * g + 1], dk[d][4 * g + 2], dk[d][4 * g + 3]};
          *reinterpret_cast<f32x4*>(pv + 32 * d + 8 * g) = f32x4{dv[d][4 * g], dv[d][4 * g + 1], dv[d][4 * g + 2], dv[d][4 * g + 3]};
        }
      }
    }
    return;
  }
  if (P.rope_cos != nullptr) rope_inv_rows<ND>(dk, P.rope_cos, P.rope_sin, P.rope_pos[krow]);
  store_rows_wide<ND>(dk, P.scale, P.dk + krow * P.sdk + (int64_t)kvh * D, key < klen);
  store_rows_wide<ND>(dv, 1.f, P.dv + krow * P.sdv + (int64_t)kvh * D, key < klen);
}

// dK = scale * sum_s dk_part[s], dV = sum_s dv_part[s] in split order, to bf16 [T, Hkv, D] views
// (token strides sdk / sdv).  One lane per 8 consecutive elements of a (token, head) row.
template <int D>
__global__ __launch_bounds__(256) void bwd_kv_combine_kernel(const float* __restrict__ dk_part,
                                                             const float* __restrict__ dv_part, int nsplit,
                                                             int64_t T, int hkv, float scale, uint16_t* __restrict__ dk,
                                                             int64_t sdk, uint16_t* __restrict__ dv, int64_t sdv) {
  constexpr int V = D / 8;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // vector index
  const int64_t rows = T * hkv;
  if (i >= rows * V) return;
  const int64_t row = i / V;
  const int c = (int)(i % V) * 8;
  const int64_t t = row / hkv;
  const int hh = (int)(row % hkv);
  float a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = b[j] = 0.f;
  for (int sp = 0; sp < nsplit; ++sp) {
    const int64_t o = ((int64_t)sp * rows + row) * D + c;
    const f32x4 k0 = *reinterpret_cast<const f32x4*>(dk_part + o), k1 = *reinterpret_cast<const f32x4*>(dk_part + o + 4);
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(dv_part + o), v1 = *reinterpret_cast<const f32x4*>(dv_part + o + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] += k0[j];
      a[4 + j] += k1[j];
      b[j] += v0[j];
      b[4 + j] += v1[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] *= scale;
  store8(dk + t * sdk + (int64_t)hh * D + c, a);
  store8(dv + t * sdv + (int64_t)hh * D + c, b);
}

}  // namespace fa

// p -> keep threshold / scale (fa::DropCfg), and the Philox key / offset of this call.
static fa::DropCfg make_drop(double p, int64_t seed, int64_t offset) {
  DTG_CHECK(p >= 0.0 && p < 1.0, "flash_attn dropout: p must be in [0, 1)");
  fa::DropCfg d{};
  d.k0 = (uint32_t)((uint64_t)seed & 0xffffffffu);
  d.k1 = (uint32_t)((uint64_t)seed >> 32) ^ (uint32_t)((uint64_t)offset >> 32);
  d.off = (uint32_t)((uint64_t)offset & 0xffffffffu);
  d.thr = (int)std::lround((1.0 - p) * 256.0);
  d.thr = std::max(1, std::min(256, d.thr));
  d.scale = 256.f / (float)d.thr;
  return d;
}

// Launch tuning of the backward kernels, read ONCE from the environment when the extension loads
// (DTG_FA_KV_SPLIT = N: dK/dV query-item split, 0 = auto; DTG_FA_KV_QB = 32 | 64: dK/dV query
// rows per item; DTG_FA_OCC = 1 | 2: dQ waves per SIMD at head_dim 128; DTG_FA_KV_PF = 1 | 2:
// dK/dV items staged ahead) -- never per launch.  Tests and A/B tools change them in-process with
// the `flash_attn_tuning` op (dtg.ops.fa_tuning).
struct Tuning {
  int kv_split, kv_qb, dq_occ, kv_pf;
};
static int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return (e != nullptr && e[0] != 0) ? std::atoi(e) : dflt;
}
static Tuning& tuning_slot() {
  static Tuning t{std::max(0, env_int("DTG_FA_KV_SPLIT", 0)), env_int("DTG_FA_KV_QB", 64) == 32 ? 32 : 64,
                  env_int("DTG_FA_OCC", 1) == 2 ? 2 : 1, env_int("DTG_FA_KV_PF", 1) == 2 ? 2 : 1};
  return t;
}
static const Tuning& tuning() { return tuning_slot(); }
static const bool kTuningLoaded = (tuning_slot(), true);  // at library load

// (kv_split, kv_qb) -> the previous values; a negative argument leaves that knob unchanged.
std::vector<int64_t> flash_attn_tuning(const at::Tensor& like, int64_t kv_split, int64_t kv_qb) {
  (void)like;
  (void)kTuningLoaded;
  Tuning& t = tuning_slot();
  std::vector<int64_t> old{t.kv_split, t.kv_qb};
  if (kv_split >= 0) t.kv_split = (int)kv_split;
  if (kv_qb >= 0) {
    DTG_CHECK(kv_qb == 32 || kv_qb == 64, "flash_attn_tuning: kv_qb must be 32 or 64");
    t.kv_qb = (int)kv_qb;
  }
  return old;
}

// Dynamic LDS above 64 KiB must be opted into per kernel (MI355X: 160 KiB per CU).
static void set_lds_limit(const void* fn, size_t bytes) {
  if (bytes > 65536) C10_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
}

static void check_qkv(const at::Tensor& t, const char* name, int64_t heads, int64_t d) {
  DTG_CHECK_CUDA_BF16(t);
  DTG_CHECK(t.dim() == 3 && t.size(1) == heads && t.size(2) == d && t.stride(2) == 1 &&
                t.stride(1) == d && t.stride(0) % 8 == 0,
            name, " must be [T, H, D] with contiguous heads and 16-B aligned token stride");
}

// Optional per-sequence key ranges (k_start / k_len int32 [nseq]): checked, or nullptr pointers.
static void key_range_ptrs(const at::Tensor* k_start, const at::Tensor* k_len, int nseq, const int** ks,
                           const int** kl) {
  *ks = *kl = nullptr;
  if (k_start == nullptr) return;
  for (const at::Tensor* t : {k_start, k_len})
    DTG_CHECK(t->scalar_type() == at::kInt && t->is_cuda() && t->is_contiguous() && t->numel() == nseq,
              "flash_attn: k_start / k_len must be int32 [nseq] on the GPU");
  *ks = k_start->data_ptr<int>();
  *kl = k_len->data_ptr<int>();
}

static std::tuple<at::Tensor, at::Tensor> flash_attn_fwd_impl(const at::Tensor& q, const at::Tensor& k,
                                                              const at::Tensor& v, const at::Tensor& cu_seqlens,
                                                              int64_t max_seqlen, double scale, bool causal,
                                                              at::Tensor* stamps, const at::Tensor* k_start = nullptr,
                                                              const at::Tensor* k_len = nullptr, int64_t window = 0,
                                                              const fa::DropCfg* drop = nullptr) {
  const int64_t T = q.size(0), hq = q.size(1), D = q.size(2), hkv = k.size(1);
  check_qkv(q, "q", hq, D);
  check_qkv(k, "k", hkv, D);
  check_qkv(v, "v", hkv, D);
  DTG_CHECK(v.size(0) == k.size(0) && (k_start != nullptr || k.size(0) == T), "flash_attn: q/k/v token counts differ");
  DTG_CHECK(hq % hkv == 0, "flash_attn: Hq must be a multiple of Hkv");
  DTG_CHECK(D == 64 || D == 128, "flash_attn: head_dim must be 64 or 128");
  DTG_CHECK(cu_seqlens.scalar_type() == at::kInt && cu_seqlens.is_cuda() && cu_seqlens.is_contiguous(),
            "flash_attn: cu_seqlens must be int32 on the GPU");
  const c10::DeviceGuard g(q.device());
  auto o = at::empty({T, hq, D}, q.options());
  auto lse = at::empty({hq, T}, q.options().dtype(at::kFloat));
  const int nseq = cu_seqlens.numel() - 1;
  if (T == 0 || nseq <= 0 || max_seqlen <= 0) return {o, lse};
  DTG_CHECK(nseq <= 65535, "flash_attn: at most 65535 sequences per call");
  const int nqb = (int)((max_seqlen + fa::kFwdBQ - 1) / fa::kFwdBQ);
  fa::FwdParams P{bf16_ptr(q), bf16_ptr(k), bf16_ptr(v), q.stride(0), k.stride(0), v.stride(0),
                  bf16_mut(o), lse.data_ptr<float>(), cu_seqlens.data_ptr<int>(), T, (int)hq, (int)hkv,
                  (float)(scale * fa::kLog2e), nullptr, nullptr, nullptr, 0};
  key_range_ptrs(k_start, k_len, nseq, &P.kstart, &P.klen);
  DTG_CHECK(window >= 0 && window < (1ll << 30), "flash_attn: window must be >= 0 (0 = full causal)");
  P.window = causal ? (int)window : 0;
  dim3 grid(hq, nseq, nqb);
  if (stamps != nullptr) {
    *stamps = at::zeros({(int64_t)grid.x * grid.y * grid.z, 6}, q.options().dtype(at::kLong));
    P.stamps = reinterpret_cast<long long*>(stamps->data_ptr<int64_t>());
  }
  const size_t lds = 4 * fa::kFwdBK * D * 2;
#define DTG_FWD(DD, C, ...)                                                               \
  do { set_lds_limit((const void*)&fa::fwd_kernel<DD, C, ##__VA_ARGS__>, lds);               \
       hipLaunchKernelGGL((fa::fwd_kernel<DD, C, ##__VA_ARGS__>), grid, dim3(256), lds, stream(), P); } while (0)
  if (drop != nullptr) {  // attention dropout: the default variant's DROP instantiation
    DTG_CHECK(P.window == 0 && P.kstart == nullptr, "flash_attn dropout: no sliding window / key ranges");
    P.drop = *drop;
    if (D == 128) { if (causal) DTG_FWD(128, true, false, true); else DTG_FWD(128, false, false, true); }
    else { if (causal) DTG_FWD(64, true, false, true); else DTG_FWD(64, false, false, true); }
  } else if (P.window > 0) {  // sliding window (causal only): the WIN instantiation
    if (D == 128) DTG_FWD(128, true, true); else DTG_FWD(64, true, true);
  } else if (D == 128) { if (causal) DTG_FWD(128, true); else DTG_FWD(128, false); }
  else { if (causal) DTG_FWD(64, true); else DTG_FWD(64, false); }
#undef DTG_FWD
  DTG_LAUNCH_CHECK();
  return {o, lse};
}

std::tuple<at::Tensor, at::Tensor> flash_attn_fwd(const at::Tensor& q, const at::Tensor& k,
                                                  const at::Tensor& v, const at::Tensor& cu_seqlens,
                                                  int64_t max_seqlen, double scale, bool causal, int64_t window) {
  return flash_attn_fwd_impl(q, k, v, cu_seqlens, max_seqlen, scale, causal, nullptr, nullptr, nullptr, window);
}

// Diagnostic: the same launch with per-workgroup timeline stamps [start, prologue done, tile
// loop done, stores complete, HW_ID, XCC_ID] (tools/fa_timeline.py).
std::tuple<at::Tensor, at::Tensor, at::Tensor> flash_attn_fwd_stamped(const at::Tensor& q, const at::Tensor& k,
                                                                      const at::Tensor& v,
                                                                      const at::Tensor& cu_seqlens,
                                                                      int64_t max_seqlen, double scale, bool causal) {
  at::Tensor st;
  auto [o, lse] = flash_attn_fwd_impl(q, k, v, cu_seqlens, max_seqlen, scale, causal, &st);
  return {o, lse, st};
}

static void launch_bwd_dq(const fa::BwdParams& P, int64_t D, bool causal, int64_t max_seqlen, int64_t hq, int nseq,
                          hipStream_t st, bool drop = false);
static void launch_bwd_dkdv(fa::BwdParams P, int64_t D, bool causal, int64_t max_seqlen_k, int64_t hkv,
                            int nseq, hipStream_t st, const at::Tensor& dk_t, const at::Tensor& dv_t, bool drop = false);

// Shared backward driver: outputs are [T, H, D] views (contiguous heads, any token stride).
struct RopeTabs {
  const at::Tensor *cos, *sin, *pos;
};

static void flash_attn_bwd_impl(const at::Tensor& dout_, const at::Tensor& q, const at::Tensor& k,
                                const at::Tensor& v, const at::Tensor& o, const at::Tensor& lse,
                                const at::Tensor& cu_seqlens, int64_t max_seqlen, double scale,
                                bool causal, const at::Tensor& dq, const at::Tensor& dk,
                                const at::Tensor& dv, const at::Tensor* k_start = nullptr,
                                const at::Tensor* k_len = nullptr, int64_t max_seqlen_k = -1,
                                int64_t window = 0, const fa::DropCfg* drop = nullptr,
                                const RopeTabs* rope = nullptr) {
  auto dout = dout_.contiguous();
  const int64_t T = q.size(0), hq = q.size(1), D = q.size(2), hkv = k.size(1);
  check_qkv(q, "q", hq, D);
  check_qkv(k, "k", hkv, D);
  check_qkv(v, "v", hkv, D);
  check_qkv(dq, "dq", hq, D);
  check_qkv(dk, "dk", hkv, D);
  check_qkv(dv, "dv", hkv, D);
  DTG_CHECK_CUDA_BF16(dout);
  DTG_CHECK(o.is_contiguous() && dout.sizes() == o.sizes() && o.size(0) == T, "flash_attn_bwd: o/dout");
  DTG_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.size(0) == hq && lse.size(1) == T,
            "flash_attn_bwd: lse must be f32 [Hq, T]");
  DTG_CHECK(D == 64 || D == 128, "flash_attn: head_dim must be 64 or 128");
  DTG_CHECK(cu_seqlens.scalar_type() == at::kInt && cu_seqlens.is_cuda() && cu_seqlens.is_contiguous(),
            "flash_attn: cu_seqlens must be int32 on the GPU");
  const c10::DeviceGuard g(q.device());
  auto opts = q.options();
  const int nseq = cu_seqlens.numel() - 1;
  // Contract: cu_seqlens covers every token (cu[-1] == T, checked by the Python wrapper), so
  // every row of dq/dk/dv is written by the kernels below -- no zero-fill pass.
  if (T == 0 || nseq <= 0 || max_seqlen <= 0) {
    dq.zero_();
    dk.zero_();
    dv.zero_();
    return;
  }
  DTG_CHECK(nseq <= 65535, "flash_attn: at most 65535 sequences per call");
  auto delta = at::empty({hq, T}, opts.dtype(at::kFloat));
  fa::BwdParams P{bf16_ptr(q), bf16_ptr(k), bf16_ptr(v), bf16_ptr(dout), bf16_ptr(o), q.stride(0), k.stride(0),
                  v.stride(0), lse.data_ptr<float>(), delta.data_ptr<float>(), bf16_mut(dq), bf16_mut(dk),
                  bf16_mut(dv), dq.stride(0), dk.stride(0), dv.stride(0), cu_seqlens.data_ptr<int>(), T, (int)hq,
                  (int)hkv, (float)scale, (float)(scale * fa::kLog2e), nullptr, nullptr, 0};
  key_range_ptrs(k_start, k_len, nseq, &P.kstart, &P.klen);
  DTG_CHECK(window >= 0 && window < (1ll << 30), "flash_attn: window must be >= 0 (0 = full causal)");
  P.window = causal ? (int)window : 0;
  if (max_seqlen_k < 0) max_seqlen_k = max_seqlen;
  if (rope != nullptr) {
    const at::Tensor &ct = *rope->cos, &stb = *rope->sin, &pt = *rope->pos;
    DTG_CHECK(ct.is_cuda() && ct.scalar_type() == at::kFloat && stb.scalar_type() == at::kFloat && ct.is_contiguous() &&
                  stb.is_contiguous() && ct.dim() == 2 && ct.size(1) == D / 2 && stb.sizes() == ct.sizes(),
              "flash_attn rope: tables must be contiguous f32 [max_pos, D/2] on the GPU");
    DTG_CHECK(pt.is_cuda() && pt.scalar_type() == at::kLong && pt.is_contiguous() && pt.numel() == T,
              "flash_attn rope: position ids must be int64 [T] on the GPU");
    DTG_CHECK(P.kstart == nullptr && drop == nullptr, "flash_attn rope: self-attention without dropout only");
    P.rope_cos = ct.data_ptr<float>();
    P.rope_sin = stb.data_ptr<float>();
    P.rope_pos = pt.data_ptr<int64_t>();
  }
  if (drop != nullptr) {
    DTG_CHECK(P.window == 0 && P.kstart == nullptr, "flash_attn dropout: no sliding window / key ranges");
    P.drop = *drop;
    launch_bwd_dq(P, D, causal, max_seqlen, hq, nseq, stream(), true);
    launch_bwd_dkdv(P, D, causal, max_seqlen_k, hkv, nseq, stream(), dk, dv, true);
    return;
  }
  // (A concurrent form -- dQ on a side stream while dK/dV runs -- was slower at every shape:
  // the pair contends for LDS bandwidth and L2, profiles/r3_s04; removed in round 6.)
  launch_bwd_dq(P, D, causal, max_seqlen, hq, nseq, stream());
  launch_bwd_dkdv(P, D, causal, max_seqlen_k, hkv, nseq, stream(), dk, dv);
}

static void launch_bwd_dq(const fa::BwdParams& P, int64_t D, bool causal, int64_t max_seqlen, int64_t hq, int nseq,
                          hipStream_t st, bool drop) {
  const int occ = tuning().dq_occ;
  {
    dim3 grid(hq, nseq, (max_seqlen + fa::kDqBQ - 1) / fa::kDqBQ);
    const size_t lds = 4 * fa::kDqBK * D * 2 + fa::kDqBQ * 4;  // + the per-row delta
#define DTG_BWD_DQ(DD, C, O, ...)                                                         \
  do { set_lds_limit((const void*)&fa::bwd_dq_kernel<DD, C, O, ##__VA_ARGS__>, lds);         \
       hipLaunchKernelGGL((fa::bwd_dq_kernel<DD, C, O, ##__VA_ARGS__>), grid, dim3(256), lds, st, P); } while (0)
    if (drop) {  // attention dropout (no window, delta computed here)
      if (D == 128) { if (causal) DTG_BWD_DQ(128, true, 1, false, true); else DTG_BWD_DQ(128, false, 1, false, true); }
      else { if (causal) DTG_BWD_DQ(64, true, 2, false, true); else DTG_BWD_DQ(64, false, 2, false, true); }
    } else if (P.window > 0) {  // sliding window (causal only)
      if (D == 128) DTG_BWD_DQ(128, true, 1, true); else DTG_BWD_DQ(64, true, 2, true);
    } else if (D == 128) {
      if (occ == 2) { if (causal) DTG_BWD_DQ(128, true, 2); else DTG_BWD_DQ(128, false, 2); }
      else { if (causal) DTG_BWD_DQ(128, true, 1); else DTG_BWD_DQ(128, false, 1); }
    } else { if (causal) DTG_BWD_DQ(64, true, 2); else DTG_BWD_DQ(64, false, 2); }
#undef DTG_BWD_DQ
    DTG_LAUNCH_CHECK();
  }
}

static void launch_bwd_dkdv(fa::BwdParams P, int64_t D, bool causal, int64_t max_seqlen_k, int64_t hkv,
                            int nseq, hipStream_t st, const at::Tensor& dk_t, const at::Tensor& dv_t, bool drop) {
  // Items the dK/dV kernel stages ahead (DTG_FA_KV_PF=1|2).  Equal on MI355X once the kernel's
  // false vmcnt waits were gone (bwd 0.767 vs 0.768 ms at the 8B shape, profiles/r1_s51_*), so
  // the single-set form with fewer registers is the default.
  const Tuning tn = tuning();
  const int kv_pf = tn.kv_pf;
  // Split the query items of each key block over several workgroups when the grid cannot fill
  // the chip (e.g. TP = 8: one KV head per rank -> 16 x 8 workgroups for 256 CUs): aim for
  // >= 2 workgroups per CU.  Tuning::kv_split = N forces N (1 = off).
  const int nkb = (int)((max_seqlen_k + fa::kKvBK - 1) / fa::kKvBK);
  const int64_t wgs = (int64_t)hkv * nseq * nkb;
  const int kv_pf_eff = drop ? 1 : kv_pf;  // dropout: the single-set, 64-row-item instantiation
  int nsplit = 1;
  if (tn.kv_split > 0) nsplit = std::min(8, tn.kv_split);
  else if (wgs > 0 && wgs < 512) nsplit = (int)std::min<int64_t>(4, (512 + wgs - 1) / wgs);
  at::Tensor dk_part, dv_part;
  if (nsplit > 1 && P.kstart == nullptr && P.window == 0 && kv_pf_eff == 1) {
    dk_part = at::empty({nsplit, P.T, hkv, D}, dk_t.options().dtype(at::kFloat));
    dv_part = at::empty({nsplit, P.T, hkv, D}, dk_t.options().dtype(at::kFloat));
    P.dk_part = dk_part.data_ptr<float>();
    P.dv_part = dv_part.data_ptr<float>();
    P.nsplit = nsplit;
  } else {
    nsplit = 1;
    P.nsplit = 1;
  }
  {
    dim3 grid(hkv, nseq, nkb * nsplit);
    // Tuning::kv_qb = 32 | 64: query rows per item.  64 (the two-half software pipeline) is the
    // default: backward 2-4 % faster on every benchmarked shape, -1.9 ms per 8B step
    // (profiles/r3_s39).  Sliding windows and the two-item prefetch keep 32.
    const int qb = drop || (tn.kv_qb != 32 && P.window == 0 && kv_pf == 1) ? 64 : 32;
    const size_t lds = 4 * (size_t)qb * D * 2 + 2 * 2 * qb * 4;
#define DTG_BWD_KV(DD, C, PF, ...)                                                        \
  do { set_lds_limit((const void*)&fa::bwd_dkdv_kernel<DD, C, PF, ##__VA_ARGS__>, lds);      \
       hipLaunchKernelGGL((fa::bwd_dkdv_kernel<DD, C, PF, ##__VA_ARGS__>), grid, dim3(256), lds, st, P); } while (0)
    if (drop) {
      if (D == 128) { if (causal) DTG_BWD_KV(128, true, 1, false, 64, true); else DTG_BWD_KV(128, false, 1, false, 64, true); }
      else { if (causal) DTG_BWD_KV(64, true, 1, false, 64, true); else DTG_BWD_KV(64, false, 1, false, 64, true); }
    } else if (P.window > 0) {  // sliding window (causal only)
      if (D == 128) DTG_BWD_KV(128, true, 1, true); else DTG_BWD_KV(64, true, 1, true);
    } else if (kv_pf == 2) {
      if (D == 128) { if (causal) DTG_BWD_KV(128, true, 2); else DTG_BWD_KV(128, false, 2); }
      else { if (causal) DTG_BWD_KV(64, true, 2); else DTG_BWD_KV(64, false, 2); }
    } else if (qb == 64) {
      if (D == 128) { if (causal) DTG_BWD_KV(128, true, 1, false, 64); else DTG_BWD_KV(128, false, 1, false, 64); }
      else { if (causal) DTG_BWD_KV(64, true, 1, false, 64); else DTG_BWD_KV(64, false, 1, false, 64); }
    } else {
      if (D == 128) { if (causal) DTG_BWD_KV(128, true, 1); else DTG_BWD_KV(128, false, 1); }
      else { if (causal) DTG_BWD_KV(64, true, 1); else DTG_BWD_KV(64, false, 1); }
    }
#undef DTG_BWD_KV
    DTG_LAUNCH_CHECK();
  }
  if (nsplit > 1) {
    const int64_t nv = P.T * hkv * (D / 8);
    if (D == 128)
      fa::bwd_kv_combine_kernel<128><<<(nv + 255) / 256, 256, 0, st>>>(P.dk_part, P.dv_part, nsplit, P.T, (int)hkv,
                                                                      P.scale, P.dk, P.sdk, P.dv, P.sdv);
    else
      fa::bwd_kv_combine_kernel<64><<<(nv + 255) / 256, 256, 0, st>>>(P.dk_part, P.dv_part, nsplit, P.T, (int)hkv,
                                                                     P.scale, P.dk, P.sdk, P.dv, P.sdv);
    DTG_LAUNCH_CHECK();
    // the split kernel's epilogue writes f32 partials: the fused RoPE backward runs on the
    // combined dK instead
    if (P.rope_cos != nullptr) rope_rows_launch(P.dk, P.sdk, (int)hkv, (int)D, P.rope_cos, P.rope_sin, P.rope_pos, P.T, true, st);
  }
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> flash_attn_bwd(
    const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
    const at::Tensor& o, const at::Tensor& lse, const at::Tensor& cu_seqlens, int64_t max_seqlen,
    double scale, bool causal, int64_t window) {
  auto dq = at::empty(q.sizes(), q.options());
  auto dk = at::empty(k.sizes(), k.options());
  auto dv = at::empty(v.sizes(), v.options());
  flash_attn_bwd_impl(dout, q, k, v, o, lse, cu_seqlens, max_seqlen, scale, causal, dq, dk, dv, nullptr, nullptr, -1,
                      window);
  return {dq, dk, dv};
}

// q, k, v are head slices of one fused [T, (nq + 2 nkv) * D] projection output; the gradient
// comes back in the same fused layout so the QKV GEMM backward consumes it directly.
at::Tensor flash_attn_bwd_qkv(const at::Tensor& dout, const at::Tensor& qkv, int64_t nq, int64_t nkv,
                              int64_t head_dim, const at::Tensor& o, const at::Tensor& lse,
                              const at::Tensor& cu_seqlens, int64_t max_seqlen, double scale, bool causal,
                              int64_t window) {
  DTG_CHECK_CUDA_BF16(qkv);
  const int64_t T = qkv.size(0), D = head_dim;
  DTG_CHECK(qkv.dim() == 2 && qkv.size(1) == (nq + 2 * nkv) * D && qkv.stride(1) == 1,
            "flash_attn_bwd_qkv: qkv must be [T, (nq + 2 nkv) * D]");
  auto dqkv = at::empty({T, (nq + 2 * nkv) * D}, qkv.options());
  auto view3 = [&](const at::Tensor& t, int64_t h0, int64_t nh) {
    return t.as_strided({T, nh, D}, {t.stride(0), D, 1}, t.storage_offset() + h0 * D);
  };
  flash_attn_bwd_impl(dout, view3(qkv, 0, nq), view3(qkv, nq, nkv), view3(qkv, nq + nkv, nkv), o, lse,
                      cu_seqlens, max_seqlen, scale, causal, view3(dqkv, 0, nq), view3(dqkv, nq, nkv),
                      view3(dqkv, nq + nkv, nkv), nullptr, nullptr, -1, window);
  return dqkv;
}

// flash_attn_bwd_qkv with the RoPE backward of the q and k heads fused into the dQ / dK
// epilogues (replaces rope_(dqkv, cos, sin, pos, nq + nkv, D, inverse = true) after it).
at::Tensor flash_attn_bwd_qkv_rope(const at::Tensor& dout, const at::Tensor& qkv, int64_t nq, int64_t nkv,
                                   int64_t head_dim, const at::Tensor& o, const at::Tensor& lse,
                                   const at::Tensor& cu_seqlens, int64_t max_seqlen, double scale, bool causal,
                                   const at::Tensor& cos_t, const at::Tensor& sin_t, const at::Tensor& pos,
                                   int64_t window) {
  DTG_CHECK_CUDA_BF16(qkv);
  const int64_t T = qkv.size(0), D = head_dim;
  DTG_CHECK(qkv.dim() == 2 && qkv.size(1) == (nq + 2 * nkv) * D && qkv.stride(1) == 1,
            "flash_attn_bwd_qkv_rope: qkv must be [T, (nq + 2 nkv) * D]");
  auto dqkv = at::empty({T, (nq + 2 * nkv) * D}, qkv.options());
  auto view3 = [&](const at::Tensor& t, int64_t h0, int64_t nh) {
    return t.as_strided({T, nh, D}, {t.stride(0), D, 1}, t.storage_offset() + h0 * D);
  };
  const RopeTabs rt{&cos_t, &sin_t, &pos};
  flash_attn_bwd_impl(dout, view3(qkv, 0, nq), view3(qkv, nq, nkv), view3(qkv, nq + nkv, nkv), o, lse,
                      cu_seqlens, max_seqlen, scale, causal, view3(dqkv, 0, nq), view3(dqkv, nq, nkv),
                      view3(dqkv, nq + nkv, nkv), nullptr, nullptr, -1, window, nullptr, &rt);
  return dqkv;
}

// FlashAttention-2-style varlen over explicit per-sequence key ranges (context parallelism).
std::tuple<at::Tensor, at::Tensor> flash_attn_varlen_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                                         const at::Tensor& cu_seqlens_q, const at::Tensor& k_start,
                                                         const at::Tensor& k_len, int64_t max_seqlen_q,
                                                         int64_t max_seqlen_k, double scale, bool causal) {
  (void)max_seqlen_k;  // the forward grid spans query blocks only
  return flash_attn_fwd_impl(q, k, v, cu_seqlens_q, max_seqlen_q, scale, causal, nullptr, &k_start, &k_len);
}

// Key ranges must be disjoint; keys outside every range get zero dK / dV.
std::tuple<at::Tensor, at::Tensor, at::Tensor> flash_attn_varlen_bwd(
    const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& o,
    const at::Tensor& lse, const at::Tensor& cu_seqlens_q, const at::Tensor& k_start, const at::Tensor& k_len,
    int64_t max_seqlen_q, int64_t max_seqlen_k, double scale, bool causal) {
  auto dq = at::empty(q.sizes(), q.options());
  auto dk = at::zeros(k.sizes(), k.options());
  auto dv = at::zeros(v.sizes(), v.options());
  flash_attn_bwd_impl(dout, q, k, v, o, lse, cu_seqlens_q, max_seqlen_q, scale, causal, dq, dk, dv, &k_start, &k_len,
                      max_seqlen_k);
  return {dq, dk, dv};
}

// Attention-probability dropout (GPT-2 attn_pdrop): p and the Philox key / offset of this call as
// an int64 [2] device tensor {seed, offset} (dtg::philox_rng draws it from torch's CUDA generator,
// graph-safe); the backward regenerates the same keep mask from the same tensor (see fa::DropCfg).
static fa::DropCfg make_drop_dev(double p, const at::Tensor& rng, const at::Tensor& like) {
  DTG_CHECK(rng.is_cuda() && rng.scalar_type() == at::kLong && rng.numel() == 2 && rng.is_contiguous() &&
                rng.device() == like.device(),
            "flash_attn dropout: rng must be a contiguous int64 [2] tensor {seed, offset} on the inputs' device");
  fa::DropCfg d = make_drop(p, 0, 0);
  d.rng = reinterpret_cast<const uint32_t*>(rng.data_ptr<int64_t>());
  return d;
}

std::tuple<at::Tensor, at::Tensor> flash_attn_fwd_drop(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                                       const at::Tensor& cu_seqlens, int64_t max_seqlen, double scale,
                                                       bool causal, double p, const at::Tensor& rng) {
  const fa::DropCfg d = make_drop_dev(p, rng, q);
  return flash_attn_fwd_impl(q, k, v, cu_seqlens, max_seqlen, scale, causal, nullptr, nullptr, nullptr, 0, &d);
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> flash_attn_bwd_drop(
    const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& o,
    const at::Tensor& lse, const at::Tensor& cu_seqlens, int64_t max_seqlen, double scale, bool causal, double p,
    const at::Tensor& rng) {
  const fa::DropCfg d = make_drop_dev(p, rng, q);
  auto dq = at::empty(q.sizes(), q.options());
  auto dk = at::empty(k.sizes(), k.options());
  auto dv = at::empty(v.sizes(), v.options());
  flash_attn_bwd_impl(dout, q, k, v, o, lse, cu_seqlens, max_seqlen, scale, causal, dq, dk, dv, nullptr, nullptr, -1, 0,
                      &d);
  return {dq, dk, dv};
}

at::Tensor flash_attn_bwd_qkv_drop(const at::Tensor& dout, const at::Tensor& qkv, int64_t nq, int64_t nkv,
                                   int64_t head_dim, const at::Tensor& o, const at::Tensor& lse,
                                   const at::Tensor& cu_seqlens, int64_t max_seqlen, double scale, bool causal,
                                   double p, const at::Tensor& rng) {
  DTG_CHECK_CUDA_BF16(qkv);
  const fa::DropCfg d = make_drop_dev(p, rng, qkv);
  const int64_t T = qkv.size(0), D = head_dim;
  DTG_CHECK(qkv.dim() == 2 && qkv.size(1) == (nq + 2 * nkv) * D && qkv.stride(1) == 1,
            "flash_attn_bwd_qkv_drop: qkv must be [T, (nq + 2 nkv) * D]");
  auto dqkv = at::empty({T, (nq + 2 * nkv) * D}, qkv.options());
  auto view3 = [&](const at::Tensor& t, int64_t h0, int64_t nh) {
    return t.as_strided({T, nh, D}, {t.stride(0), D, 1}, t.storage_offset() + h0 * D);
  };
  flash_attn_bwd_impl(dout, view3(qkv, 0, nq), view3(qkv, nq, nkv), view3(qkv, nq + nkv, nkv), o, lse, cu_seqlens,
                      max_seqlen, scale, causal, view3(dqkv, 0, nq), view3(dqkv, nq, nkv), view3(dqkv, nq + nkv, nkv),
                      nullptr, nullptr, -1, 0, &d);
  return dqkv;
}

// {seed, offset} of one dropout call from torch's CUDA generator for `like`'s device, written into
// a fresh int64 [2] device tensor by a one-lane kernel on the current stream.  Outside capture the
// generator hands out values; under HIP-graph capture it hands out pointers to its seed and to an
// offset it advances before every replay, so the captured unpack yields a new offset each replay.
__global__ void philox_rng_kernel(at::PhiloxCudaState st, int64_t* out) {
  if (threadIdx.x == 0) {
    const auto so = at::cuda::philox::unpack(st);
    out[0] = static_cast<int64_t>(std::get<0>(so));
    out[1] = static_cast<int64_t>(std::get<1>(so));
  }
}

at::Tensor philox_rng(const at::Tensor& like, int64_t increment) {
  DTG_CHECK(like.is_cuda(), "philox_rng: needs a GPU tensor");
  const c10::DeviceGuard g(like.device());
  auto gen = at::get_generator_or_default<at::CUDAGeneratorImpl>(
      std::nullopt, at::cuda::detail::getDefaultCUDAGenerator(like.device().index()));
  at::PhiloxCudaState st;
  {
    std::lock_guard<std::mutex> lock(gen->mutex_);
    st = gen->philox_cuda_state(static_cast<uint64_t>(std::max<int64_t>(4, increment)));
  }
  auto out = at::empty({2}, like.options().dtype(at::kLong));
  philox_rng_kernel<<<1, 64, 0, stream()>>>(st, out.data_ptr<int64_t>());
  DTG_LAUNCH_CHECK();
  return out;
}

TORCH_LIBRARY_IMPL(dtg, CUDA, m) {
  m.impl("flash_attn_fwd_drop", &flash_attn_fwd_drop);
  m.impl("flash_attn_bwd_drop", &flash_attn_bwd_drop);
  m.impl("flash_attn_bwd_qkv_drop", &flash_attn_bwd_qkv_drop);
  m.impl("philox_rng", &philox_rng);
  m.impl("flash_attn_varlen_fwd", &flash_attn_varlen_fwd);
  m.impl("flash_attn_varlen_bwd", &flash_attn_varlen_bwd);
  m.impl("flash_attn_fwd", &flash_attn_fwd);
  m.impl("flash_attn_fwd_stamped", &flash_attn_fwd_stamped);
  m.impl("flash_attn_bwd", &flash_attn_bwd);
  m.impl("flash_attn_bwd_qkv", &flash_attn_bwd_qkv);
  m.impl("flash_attn_bwd_qkv_rope", &flash_attn_bwd_qkv_rope);
  m.impl("flash_attn_tuning", &flash_attn_tuning);
}

}  // namespace dtg
