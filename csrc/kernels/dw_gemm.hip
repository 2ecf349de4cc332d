// Weight-gradient GEMM with both operands token-major: C[M, N] = A^T B (+ C), A = dY [K, M],
// B = X [K, N], K = tokens.  (SURVEY K-list: the Linear backward; VERDICT r3 "next round" #6.)
//
// Why it exists: a Linear layer's dW = dY^T X reduces over the token dimension, which is the
// STRIDED dimension of both row-major activations.  hipBLASLt runs this "NT" layout 25-40 %
// slower than the K-contiguous "TN" one (csrc/kernels/transpose.hip), so the default backward
// transposes dY and X first (12.7 ms/step of transposes at the 8B shape, plus the transposed
// writes of swiglu_bwd_t; profiles/r3/s46/step_roofline.md).  gfx950 reads an MN-major LDS
// tile straight into MFMA operand order with ds_read_b64_tr_b16, so this kernel consumes the
// token-major tiles as they are: no transpose pass, no transposed copies.
//
// Structure (one 256 x 256 output tile per 512-thread workgroup, 8 waves as 2 (M) x 4 (N),
// 128 x 64 outputs per wave = 4 x 2 accumulators of v_mfma_f32_32x32x16_bf16):
//  * K-tiles of 64 token rows.  Each K-tile of A and of B is a [64][256] bf16 image (512-B
//    rows, 32 KB) filled by global_load_lds_dwordx4 -- LDS-DMA, no VGPR staging -- two stages
//    (128 KB of the 160 KB LDS), the load of tile t+1 in flight while tile t is consumed;
//  * the image is XOR-swizzled in 64-B units by (row & 3) (written through a pre-swizzled
//    global SOURCE address: the DMA's LDS destination is lane-linear), so one tr-read's
//    half-wave (4 rows x 64 B) covers all 64 banks once;
//  * operand fragments by two ds_read_b64_tr_b16 each (k-order {4h..4h+3, 8+4h..}: the same
//    permutation on both operands, so the dot product is unchanged);
//  * raw s_barrier + explicit counted waits (a __syncthreads() would drain the DMA in flight);
//    all LDS in one __shared__ array (a second object makes hipcc wait vmcnt(0) per ds_read);
//  * workgroup -> tile map: XCD-bijective remap, then bands of GM tile rows so the 32
//    workgroups resident on one XCD share A and B panels in its L2.
//  * epilogue: f32 accumulators -> C (bf16 or f32), optionally C += (addmm_ semantics).
#include "common.h"

#include <type_traits>

namespace dtg {
namespace dwg {

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int ROWB = 512;                 // bytes per k-row of a tile image (BM == BN == 256)
constexpr int TILE_BYTES = BK * ROWB;     // 32 KB per operand per stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;
constexpr int LDS_BYTES = 2 * STAGE_BYTES;  // 128 KB
constexpr int GM = 4;                     // tile rows per band of the workgroup order

// Byte offset of logical 16-byte chunk `ch` (0..31) of k-row `row` in a tile image.
__device__ __forceinline__ int img_off(int row, int ch) { return row * ROWB + 16 * (ch ^ ((row & 3) << 2)); }

__device__ __forceinline__ bf16x8 tr_frag(const char* base, int oa) {
  const i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + oa));
  const i16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + oa + 8 * ROWB));
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const i16x8 ab = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, ab);
}

// Lane offset (k-step 0) of the transposed fragment of columns cb .. cb+31 of an image.
__device__ __forceinline__ int frag_off(int cb) {
  const int lane = threadIdx.x & 63;
  const int i = lane & 15, g = lane >> 4;
  const int q = i >> 2, p = i & 3;
  const int ch = ((cb + 16 * (g & 1)) >> 3) + (p >> 1);
  return img_off(4 * (g >> 1) + q, ch) + 8 * (p & 1);
}

// One 16-byte-per-lane LDS-DMA: lane l's 16 bytes from `gsrc` land at LDS byte lds_dst + 16 l.
// Inline asm, so that hipcc does not see an LDS write in flight: with the builtin it waits
// vmcnt(0) before the first ds_read of every K-tile (it cannot tell the staged buffer from the
// one being read) and the prefetch never overlaps the MFMAs.  The waits are counted by hand.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

// Issue the LDS-DMA of one K-tile (rows k0 .. k0+63, columns c0 .. c0+255) of a token-major
// operand into the image at `img`: 32 wave-instructions of 1 KB (two k-rows), 4 per wave.
__device__ __forceinline__ void stage(const uint16_t* __restrict__ src, int64_t ld, int64_t k0, int64_t c0,
                                      uint32_t img) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = 4 * w + i;
    const int row = 2 * j + (lane >> 5);
    const int lc = (lane & 31) ^ ((row & 3) << 2);  // logical chunk this lane's 16 B belong to
    const uint16_t* g = src + (k0 + row) * ld + c0 + 8 * lc;
    glds16(g, __builtin_amdgcn_readfirstlane(img + 1024 * j));
  }
}

__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Workgroup id -> (tile row, tile col): XCD-bijective remap (consecutive ids land on one XCD),
// then bands of GM tile rows walked column by column.
__device__ __forceinline__ void tile_of(int tm_n, int tn_n, int& tm, int& tn) {
  const int nwg = tm_n * tn_n, orig = blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int per_band = GM * tn_n;
  const int band = wgid / per_band;
  const int first = band * GM;
  const int rows = tm_n - first < GM ? tm_n - first : GM;
  const int in = wgid - band * per_band;
  tm = first + in % rows;
  tn = in / rows;
}

// acc[mt][nt][r] = C[m0 + 128 wr + 32 mt + row(r)][n0 + 64 wc + 32 nt + (lane & 31)]
template <bool OUT_F32, bool ACCUM>
__device__ __forceinline__ void store_tile(const f32x16 (&acc)[4][2], void* __restrict__ C, int64_t ldc, int64_t m0,
                                           int64_t n0, int wr, int wc) {
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5, col = lane & 31;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + 128 * wr + 32 * mt + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t n = n0 + 64 * wc + 32 * nt + col;
        float v = acc[mt][nt][r];
        if constexpr (OUT_F32) {
          float* c = reinterpret_cast<float*>(C) + m * ldc + n;
          if constexpr (ACCUM) v += *c;
          *c = v;
        } else {
          uint16_t* c = reinterpret_cast<uint16_t*>(C) + m * ldc + n;
          if constexpr (ACCUM) v += bf2f(*c);
          *c = f2bf(v);
        }
      }
}

template <bool OUT_F32, bool ACCUM>
__global__ __launch_bounds__(512) void dw_gemm_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                      const uint16_t* __restrict__ B, int64_t ldb,
                                                      void* __restrict__ C, int64_t ldc, int M, int N, int K) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  int tm, tn;
  tile_of(M / BM, N / BN, tm, tn);
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 2, wc = w & 3;  // 2 (M) x 4 (N)

  int oa[4], ob[2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) oa[mt] = frag_off(128 * wr + 32 * mt);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) ob[nt] = frag_off(64 * wc + 32 * nt);

  f32x16 acc[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;

  const int nk = K / BK;
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem);
  stage(A, lda, 0, m0, lds0);
  stage(B, ldb, 0, n0, lds0 + TILE_BYTES);
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * STAGE_BYTES;
    if (t + 1 < nk) {
      const uint32_t nxt = lds0 + ((t + 1) & 1) * STAGE_BYTES;
      stage(A, lda, (int64_t)(t + 1) * BK, m0, nxt);
      stage(B, ldb, (int64_t)(t + 1) * BK, n0, nxt + TILE_BYTES);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this wave's DMA of tile t has landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier();  // ... and every wave's
    const char* ia = cur;
    const char* ib = cur + TILE_BYTES;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 fa[4], fb[2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) fb[nt] = tr_frag(ib + 16 * s * ROWB, ob[nt]);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) fa[mt] = tr_frag(ia + 16 * s * ROWB, oa[mt]);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma(fa[mt], fb[nt], acc[mt][nt]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier();  // every wave is done reading `cur`: the next DMA may refill it
  }

  store_tile<OUT_F32, ACCUM>(acc, C, ldc, m0, n0, wr, wc);
}

// Variant 2: the same tile, images and fragments, pipelined by k-step ("phase") instead of by
// K-tile.  A K-tile's 64 rows are four quarters of 16 rows (A 8 KB + B 8 KB, one LDS-DMA
// wave-instruction of each per wave).  Phase (t, s), s = 0..3:
//   1. read the fragments of k-step s of tile t (retired by the previous phase's wait+barrier);
//   2. issue the DMA of quarter s of tile t+1 into the other buffer (its rows were last read
//      four phases ago, before that phase's barrier);
//   3. s_waitcnt vmcnt(6): this wave's DMA of the quarter the NEXT phase reads has landed (three
//      quarters stay in flight);
//   4. barrier (every wave's has), lgkmcnt(0), 8 MFMAs of k-step s.
// The fragment reads of a phase issue behind the previous phase's MFMAs, so the matrix pipe
// never waits on LDS at a K-tile seam (variant 1 drains it twice per K-tile).
__device__ __forceinline__ void stage_quarter(const uint16_t* __restrict__ src, int64_t ld, int64_t k0, int64_t c0,
                                              uint32_t img, int q) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = 8 * q + w;  // wave-instruction j of the tile: rows 2j, 2j + 1
  const int row = 2 * j + (lane >> 5);
  const int lc = (lane & 31) ^ ((row & 3) << 2);
  glds16(src + (k0 + row) * ld + c0 + 8 * lc, __builtin_amdgcn_readfirstlane(img + 1024 * j));
}

// PP (variant 3): the 8-phase GEMM template's ping-pong on top -- two barriers per phase
// (reads + DMA | barrier | MFMAs at raised priority | barrier) and the M-half wave group wr = 1
// one barrier behind wr = 0, so on every SIMD (waves w and w + 4) one wave issues its MFMAs
// while the other reads its fragments.  Data hazards are still covered: a quarter is retired
// (vmcnt + barrier) two barriers before any wave of either group reads it, and a buffer row is
// refilled >= 6 barriers after its last read completed.
template <bool OUT_F32, bool ACCUM, bool PP>
__global__ __launch_bounds__(512) void dw_gemm_v2_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                         const uint16_t* __restrict__ B, int64_t ldb,
                                                         void* __restrict__ C, int64_t ldc, int M, int N, int K) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  int tm, tn;
  tile_of(M / BM, N / BN, tm, tn);
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int w = threadIdx.x >> 6;
  const int wr = w >> 2, wc = w & 3;

  int oa[4], ob[2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) oa[mt] = frag_off(128 * wr + 32 * mt);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) ob[nt] = frag_off(64 * wc + 32 * nt);

  f32x16 acc[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;

  const int nk = K / BK;
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    stage_quarter(A, lda, 0, m0, lds0, q);
    stage_quarter(B, ldb, 0, n0, lds0 + TILE_BYTES, q);
  }
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // quarter 0 of tile 0
  barrier();
  if (PP && wr == 1) barrier();  // the stagger (wave-uniform branch)
  for (int t = 0; t < nk; ++t) {
    const char* ia = smem + (t & 1) * STAGE_BYTES;
    const char* ib = ia + TILE_BYTES;
    const uint32_t nxt = lds0 + ((t + 1) & 1) * STAGE_BYTES;
    const bool more = t + 1 < nk;
    const int64_t k1 = (int64_t)(t + 1) * BK;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 fa[4], fb[2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) fb[nt] = tr_frag(ib + 16 * s * ROWB, ob[nt]);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) fa[mt] = tr_frag(ia + 16 * s * ROWB, oa[mt]);
      if (more) {
        stage_quarter(A, lda, k1, m0, nxt, s);
        stage_quarter(B, ldb, k1, n0, nxt + TILE_BYTES, s);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (PP) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma(fa[mt], fb[nt], acc[mt][nt]);
      if constexpr (PP) {
        __builtin_amdgcn_s_setprio(0);
        barrier();
      }
    }
  }
  if (PP && wr == 0) barrier();  // equal barrier counts for both groups
  store_tile<OUT_F32, ACCUM>(acc, C, ldc, m0, n0, wr, wc);
}

// Variant 4: variant 2's k-step pipeline on a deep ring.  The 160 KB LDS holds 10 quarter
// slots (A 8 KB + B 8 KB each); quarter Q (global k-rows 16Q .. 16Q+15) lives in slot Q % 10 and
// its DMA is issued 8 phases before it is read, so 7 quarters stay in flight across every
// barrier (vmcnt(14)) instead of 3 -- the counters of variant 2 (profiles/r4/s13: 25-33 % of wave
// cycles in s_waitcnt, matrix pipe 58 % busy) say HBM/L2 latency is not covered.  The DMA uses
// the saddr form: a wave-uniform 64-bit base in SGPRs (advanced per quarter) plus a per-lane
// 32-bit offset computed once, instead of 64-bit per-lane address arithmetic per instruction.
// Hazards: slot (Q + 8) % 10 was last read in phase Q - 2, whose reads every wave retired
// (lgkmcnt(0)) before barrier Q - 1, which precedes the refill in phase Q; quarter Q + 1 is
// retired by every wave's vmcnt before barrier Q and read after it.
constexpr int QBYTES = 16 * ROWB;  // slot: A quarter, then B quarter

__device__ __forceinline__ void glds16_s(uint32_t voff, const void* sbase, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds_dst)
               : "memory");
}

__device__ __forceinline__ const uint16_t* uniform_ptr(const uint16_t* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  return reinterpret_cast<const uint16_t*>((static_cast<uint64_t>(hi) << 32) | lo);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// KS k-steps (quarters) per phase and barrier; AHEAD quarters in flight; ring of
// AHEAD + 2 KS slots (the refill of phase p targets the slots read in phase p - 2).
template <bool OUT_F32, bool ACCUM, int KS, int AHEAD>
__global__ __launch_bounds__(512) void dw_gemm_v4_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                         const uint16_t* __restrict__ B, int64_t ldb,
                                                         void* __restrict__ C, int64_t ldc, int M, int N, int K) {
  constexpr int RING = AHEAD + 2 * KS;
  static_assert(RING * 2 * QBYTES <= 160 * 1024, "LDS");
  static_assert(AHEAD % KS == 0, "whole phases in flight");
  __shared__ __attribute__((aligned(1024))) char smem[RING * 2 * QBYTES];
  int tm, tn;
  tile_of(M / BM, N / BN, tm, tn);
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;

  int oa[4], ob[2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) oa[mt] = frag_off(128 * wr + 32 * mt);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) ob[nt] = frag_off(64 * wc + 32 * nt);

  // this lane's 16 bytes of its wave's DMA instruction of a quarter: quarter row 2w + (lane >> 5)
  const int qrow = 2 * w + (lane >> 5);
  const int lc = (lane & 31) ^ ((qrow & 3) << 2);
  const uint32_t va = (uint32_t)(qrow * lda * 2 + lc * 16);
  const uint32_t vb = (uint32_t)(qrow * ldb * 2 + lc * 16);
  const uint16_t* abase = A + m0;  // + 16 Q lda per quarter
  const uint16_t* bbase = B + n0;
  const int64_t astep = 16 * lda, bstep = 16 * ldb;
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem);
  auto issue = [&](int q) {
    const uint32_t slot = lds0 + (uint32_t)(q % RING) * (2 * QBYTES) + 1024 * w;
    glds16_s(va, uniform_ptr(abase + (int64_t)q * astep), __builtin_amdgcn_readfirstlane(slot));
    glds16_s(vb, uniform_ptr(bbase + (int64_t)q * bstep), __builtin_amdgcn_readfirstlane(slot + QBYTES));
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;

  const int nq = K / 16;  // a multiple of 4 (K % 64 == 0), so of KS
  const int pre = nq < AHEAD ? nq : AHEAD;
  for (int q = 0; q < pre; ++q) issue(q);
  if (nq > AHEAD) wait_vm<2 * (AHEAD - KS)>();  // the first phase's quarters have landed
  else wait_vm<0>();
  barrier();
  auto phase = [&](int q, auto steady) {
    bf16x8 fa[KS][4], fb[KS][2];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const char* ia = smem + ((q + k) % RING) * (2 * QBYTES);
      const char* ib = ia + QBYTES;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) fb[k][nt] = tr_frag(ib, ob[nt]);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) fa[k][mt] = tr_frag(ia, oa[mt]);
    }
    if constexpr (decltype(steady)::value) {
#pragma unroll
      for (int k = 0; k < KS; ++k) issue(q + AHEAD + k);
      wait_vm<2 * (AHEAD - KS)>();  // the next phase's quarters have landed
    } else {
      wait_vm<0>();
    }
    barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma(fa[k][mt], fb[k][nt], acc[mt][nt]);
  };
  // branch-free steady state (unrolled by two phases so the next phase's reads can issue behind
  // this phase's MFMAs), then the drain of the last AHEAD quarters
  const int steady_end = nq - AHEAD > 0 ? nq - AHEAD : 0;  // a multiple of KS
  int q = 0;
  for (; q + KS < steady_end; q += 2 * KS) {
    phase(q, std::true_type{});
    phase(q + KS, std::true_type{});
  }
  for (; q < steady_end; q += KS) phase(q, std::true_type{});
  for (; q < nq; q += KS) phase(q, std::false_type{});
  store_tile<OUT_F32, ACCUM>(acc, C, ldc, m0, n0, wr, wc);
}

// Variants 6-9 (4 waves x 128 x 128 with AGPR accumulators on the ring; hipBLASLt's register-
// staged structure one / two K-tiles ahead) measured slower than 5 (MFMA busy 0.42-0.53,
// profiles/r4/s16, s20) and were removed; their source is in the git history of this file.

}  // namespace dwg

// c (=|+=) a^T @ b;  a: [K, M], b: [K, N] (token-major, unit column stride), c: [M, N].
// Shapes must be tile multiples (M, N % 256, K % 64); callers fall back to hipBLASLt otherwise.
void dw_gemm_(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c, bool accumulate) {
  DTG_CHECK_CUDA_BF16(a);
  DTG_CHECK_CUDA_BF16(b);
  DTG_CHECK(c.is_cuda() && (c.scalar_type() == at::kBFloat16 || c.scalar_type() == at::kFloat),
            "dw_gemm_: c must be a bf16 or f32 GPU tensor");
  DTG_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "dw_gemm_: 2-D operands");
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1);
  DTG_CHECK(b.size(0) == K && c.size(0) == M && c.size(1) == N, "dw_gemm_: shape mismatch");
  DTG_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && c.stride(1) == 1, "dw_gemm_: unit column stride required");
  DTG_CHECK(M % dwg::BM == 0 && N % dwg::BN == 0 && K % dwg::BK == 0 && K > 0,
            "dw_gemm_: M, N must be multiples of 256 and K of 64 (got ", M, ", ", N, ", ", K, ")");
  DTG_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 &&
                reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0,
            "dw_gemm_: operands must be 16-byte aligned rows");
  DTG_CHECK(K < (int64_t(1) << 31) && M * N < (int64_t(1) << 40), "dw_gemm_: too large");
  // per-lane / scalar byte offsets within one K-tile (64 rows) are 32-bit in the ring and
  // register-staged variants
  DTG_CHECK(a.stride(0) < (int64_t(1) << 24) && b.stride(0) < (int64_t(1) << 24), "dw_gemm_: row pitch too large");
  const int64_t tiles = (M / dwg::BM) * (N / dwg::BN);
  DTG_CHECK(tiles < (int64_t(1) << 31), "dw_gemm_: too many tiles");
  const c10::DeviceGuard g(a.device());
  const dim3 grid((unsigned)tiles), block(512);
  const bool f32 = c.scalar_type() == at::kFloat;
  // DTG_DWG_VARIANT = 1 (K-tile pipeline) | 2 (k-step pipeline) | 3 (k-step + ping-pong) | 4 (k-step,
  // 10-slot ring, 8 quarters ahead) | 5 (2 k-steps per barrier, 6 quarters ahead)
  // (6-9: removed after measurement); read per call
  const char* ve = std::getenv("DTG_DWG_VARIANT");
  const int variant = ve ? std::atoi(ve) : 5;  // the fastest measured (profiles/r4/s15, s16)
#define DTG_DWG_LAUNCH(F, ACC)                                                                                    \
  do {                                                                                                            \
    if (variant == 1)                                                                                             \
      dwg::dw_gemm_kernel<F, ACC><<<grid, block, 0, stream()>>>(bf16_ptr(a), a.stride(0), bf16_ptr(b), b.stride(0), \
                                                                c.data_ptr(), c.stride(0), (int)M, (int)N, (int)K); \
    else if (variant == 4)                                                                                        \
      dwg::dw_gemm_v4_kernel<F, ACC, 1, 8><<<grid, block, 0, stream()>>>(bf16_ptr(a), a.stride(0), bf16_ptr(b),    \
                                                                         b.stride(0), c.data_ptr(), c.stride(0),   \
                                                                         (int)M, (int)N, (int)K);                  \
    else if (variant == 5)                                                                                        \
      dwg::dw_gemm_v4_kernel<F, ACC, 2, 6><<<grid, block, 0, stream()>>>(bf16_ptr(a), a.stride(0), bf16_ptr(b),    \
                                                                         b.stride(0), c.data_ptr(), c.stride(0),   \
                                                                         (int)M, (int)N, (int)K);                  \
    else if (variant == 3)                                                                                        \
      dwg::dw_gemm_v2_kernel<F, ACC, true><<<grid, block, 0, stream()>>>(bf16_ptr(a), a.stride(0), bf16_ptr(b),    \
                                                                         b.stride(0), c.data_ptr(), c.stride(0),   \
                                                                         (int)M, (int)N, (int)K);                  \
    else                                                                                                          \
      dwg::dw_gemm_v2_kernel<F, ACC, false><<<grid, block, 0, stream()>>>(bf16_ptr(a), a.stride(0), bf16_ptr(b),   \
                                                                          b.stride(0), c.data_ptr(), c.stride(0),  \
                                                                          (int)M, (int)N, (int)K);                 \
  } while (0)
  if (f32) {
    if (accumulate) DTG_DWG_LAUNCH(true, true); else DTG_DWG_LAUNCH(true, false);
  } else {
    if (accumulate) DTG_DWG_LAUNCH(false, true); else DTG_DWG_LAUNCH(false, false);
  }
#undef DTG_DWG_LAUNCH
  DTG_LAUNCH_CHECK();
}

TORCH_LIBRARY_IMPL(dtg, CUDA, m) { m.impl("dw_gemm_", &dw_gemm_); }

}  // namespace dtg
