// Flash-style causal attention, forward and backward, for gfx950 (replaces
// the flash-attn / SDPA dependencies N2, N3 of the reference).
//
// Supports GQA (Hq a multiple of Hkv), head_dim 64/128, and variable-length packed
// sequences through `cu_seqlens` (the rime packed path: documents restart their position
// ids at each EOS) -- a dense [B, S] batch is just cu_seqlens = arange(B+1)*S.
// Layout: token-major q [T, Hq, D], k/v [T, Hkv, D] with an arbitrary token stride, so q, k
// and v are read straight out of the fused QKV projection output with no copies.
//
// MFMA mapping (v_mfma_f32_32x32x16_bf16, CDNA guide §3):
//  * Forward computes S^T = K Q^T so a lane owns one query column (online-softmax state is
//    per lane; the row reduction is 31 f32 max + one cross-half shuffle), then
//    O^T += V^T P^T with P^T taken straight from the S^T accumulator registers (the k order
//    inside a 16-step is permuted; V^T fragments are fetched in the same permuted order with
//    ds_read_b64_tr_b16, T10).
//  * Backward keeps the key on the lane: S and dP accumulators are the B operands of the
//    dV^T and dK^T products; dS crosses LDS once (stored transposed) for dQ, which is summed
//    across key blocks with f32 atomics in the full-rate two-128-B-rows shape (Guideline 12).
//  * All K/V/Q/dO tiles live in LDS as 16-byte-chunk XOR-swizzled images (T10 image (b)), so
//    ds_read_b128 row reads and transposed reads share one copy.
#include "common.h"

#include <cstdlib>

namespace dtg {
namespace fa {

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// Byte offset of 16-byte chunk `ch` of row `row` in a [rows][W] bf16 LDS image.
template <int W>
__device__ __forceinline__ int off(int row, int ch) {
  constexpr int NCH = W / 8;
  int sw;
  if constexpr (NCH >= 16) sw = ((row & 3) << 2) | ((row >> 2) & 3);
  else if constexpr (NCH == 8) sw = ((row & 1) << 2) | ((row >> 1) & 3);
  else sw = row & (NCH - 1);
  return row * (W * 2) + 16 * (ch ^ sw);
}

// A/B fragment whose MFMA row index is the tile row and whose k index runs along the row:
// lane (r, h) gets tile[row][8*chunk .. +7].
template <int W>
__device__ __forceinline__ bf16x8 row_frag(const char* tile, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(tile + off<W>(row, ch));
}

__device__ __forceinline__ i16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(p));
}

// Fragment whose MFMA row index is a tile COLUMN (col0 + lane%32) and whose k index runs down
// the tile rows: elements 0..3 come from rows rowA..rowA+3, elements 4..7 from rowB..rowB+3.
// Must be executed by all 64 lanes (EXEC all ones, T10).
template <int W>
__device__ __forceinline__ bf16x8 tr_frag(const char* tile, int rowA, int rowB, int col0) {
  const int lane = threadIdx.x & 63;
  const int i = lane & 15, g = lane >> 4;
  const int q = i >> 2, p = i & 3;
  const int colbase = col0 + 16 * (g & 1);
  const int ch = (colbase >> 3) + (p >> 1);
  const int half = 8 * (p & 1);
  const i16x4 a = tr_read(tile + off<W>(rowA + q, ch) + half);
  const i16x4 b = tr_read(tile + off<W>(rowB + q, ch) + half);
  // Whole-vector concatenation: per-element extraction of the tr-read result miscompiles on
  // ROCm 7.2 (hipcc duplicates the low dword; caught by tests/native/probe_fragments.hip).
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const i16x8 ab = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, ab);
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Pack accumulator registers 8s .. 8s+7 into a bf16 operand fragment.
__device__ __forceinline__ bf16x8 pack8(const f32x16& x, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = static_cast<__bf16>(x[8 * s + j]);
  return r;
}

// Row of accumulator register `reg` for lane half h (32x32 C/D map).
__device__ __forceinline__ int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

struct FwdParams {
  const uint16_t *q, *k, *v;
  int64_t sq, sk, sv;  // token strides (elements)
  uint16_t* o;         // [T, Hq, D] contiguous
  float* lse;          // [Hq, T]
  const int* cu;       // [nseq + 1]
  int64_t T;
  int hq, hkv;
  float c2;  // softmax scale * log2(e)
};

constexpr int kFwdBQ = 128;  // query rows per workgroup (4 waves x 32)
constexpr int kFwdBK = 64;   // keys per K/V tile

// Register-staged copy of R rows x W bf16 from global into a swizzled LDS image.
template <int R, int W, int NT>
struct Stager {
  static constexpr int NCH = W / 8;
  static constexpr int PER = (R * NCH) / NT;
  static_assert((R * NCH) % NT == 0, "tile must split evenly over the threads");
  u16x8 regs[PER];
  __device__ __forceinline__ void load(const uint16_t* base, int64_t stride, int nvalid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = threadIdx.x + i * NT;
      const int row = idx / NCH, ch = idx % NCH;
      if (row < nvalid) regs[i] = *reinterpret_cast<const u16x8*>(base + row * stride + ch * 8);
      else regs[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  __device__ __forceinline__ void store(char* tile) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = threadIdx.x + i * NT;
      const int row = idx / NCH, ch = idx % NCH;
      *reinterpret_cast<u16x8*>(tile + off<W>(row, ch)) = regs[i];
    }
  }
};

template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void fwd_kernel(FwdParams P) {
  constexpr int TILE_BYTES = kFwdBK * D * 2;
  constexpr int NC = D / 16;  // k-steps over head_dim
  constexpr int ND = D / 32;  // 32-wide d tiles of the output
  extern __shared__ __attribute__((aligned(16))) char smem[];
  auto kbuf = [&](int i) { return smem + i * 2 * TILE_BYTES; };
  auto vbuf = [&](int i) { return smem + i * 2 * TILE_BYTES + TILE_BYTES; };

  const int seq = blockIdx.z, head = blockIdx.y;
  const int s0 = P.cu[seq];
  const int seqlen = P.cu[seq + 1] - s0;
  const int qb = CAUSAL ? (gridDim.x - 1 - blockIdx.x) : blockIdx.x;  // heavy blocks first
  const int q0 = qb * kFwdBQ;
  if (q0 >= seqlen) return;
  const int kvh = head / (P.hq / P.hkv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int qrow = q0 + 32 * w + r;  // this lane's query (sequence-relative)

  // Q^T fragments for all k-steps, straight from global into registers.
  bf16x8 qf[NC];
  {
    const bool ok = qrow < seqlen;
    const uint16_t* qp = P.q + (int64_t)(s0 + (ok ? qrow : 0)) * P.sq + (int64_t)head * D + 8 * h;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      u16x8 v = ok ? *reinterpret_cast<const u16x8*>(qp + 16 * c) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      qf[c] = __builtin_bit_cast(bf16x8, v);
    }
  }

  const int kv_end = CAUSAL ? min(seqlen, q0 + kFwdBQ) : seqlen;
  const int ntiles = (kv_end + kFwdBK - 1) / kFwdBK;
  const uint16_t* kbase = P.k + (int64_t)s0 * P.sk + (int64_t)kvh * D;
  const uint16_t* vbase = P.v + (int64_t)s0 * P.sv + (int64_t)kvh * D;

  f32x16 acc[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) acc[i] = f32x16{};
  float m = -INFINITY, l = 0.f;

  Stager<kFwdBK, D, 256> sk, sv;
  sk.load(kbase, P.sk, seqlen);
  sv.load(vbase, P.sv, seqlen);
  sk.store(kbuf(0));
  sv.store(vbuf(0));
  __syncthreads();

  const int wave_qmax = q0 + 32 * w + 31;
  for (int t = 0; t < ntiles; ++t) {
    const int kt0 = t * kFwdBK;
    const bool more = t + 1 < ntiles;
    if (more) {
      const int nk = kt0 + kFwdBK;
      sk.load(kbase + (int64_t)nk * P.sk, P.sk, seqlen - nk);
      sv.load(vbase + (int64_t)nk * P.sv, P.sv, seqlen - nk);
    }
    const char* K = kbuf(t & 1);
    const char* V = vbuf(t & 1);
    // Wave-uniform skip of tiles entirely above this wave's causal diagonal.
    const bool active = !CAUSAL || kt0 <= wave_qmax;
    if (active) {
      f32x16 s[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt] = f32x16{};
#pragma unroll
        for (int c = 0; c < NC; ++c) s[kt] = mfma(row_frag<D>(K, kt * 32 + r, 2 * c + h), qf[c], s[kt]);
      }
      const bool need_mask = (CAUSAL && kt0 + kFwdBK - 1 > q0 + 32 * w) || (kt0 + kFwdBK > seqlen);
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float x = s[kt][i] * P.c2;
          if (need_mask) {
            const int key = kt0 + kt * 32 + acc_row(i, h);
            if (key >= seqlen || (CAUSAL && key > qrow)) x = -INFINITY;
          }
          s[kt][i] = x;
          mx = fmaxf(mx, x);
        }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m, mx);
      const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
      const float alpha = exp2f(m - m_use);
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = exp2f(s[kt][i] - m_use);
          s[kt][i] = p;
          rs += p;
        }
      }
      l = l * alpha + rs;
      m = m_new;
#pragma unroll
      for (int d = 0; d < ND; ++d) acc[d] *= alpha;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 pf = pack8(s[kt], st);
          const int ra = kt * 32 + 16 * st + 4 * h;
#pragma unroll
          for (int d = 0; d < ND; ++d) acc[d] = mfma(tr_frag<D>(V, ra, ra + 8, 32 * d), pf, acc[d]);
        }
      }
    }
    if (more) {
      sk.store(kbuf((t + 1) & 1));
      sv.store(vbuf((t + 1) & 1));
    }
    __syncthreads();
  }

  const float lt = l + __shfl_xor(l, 32, 64);
  if (qrow < seqlen) {
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    uint16_t* op = P.o + ((int64_t)(s0 + qrow) * P.hq + head) * D;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        ushort4 v;
        v.x = f2bf(acc[d][4 * g4 + 0] * inv);
        v.y = f2bf(acc[d][4 * g4 + 1] * inv);
        v.z = f2bf(acc[d][4 * g4 + 2] * inv);
        v.w = f2bf(acc[d][4 * g4 + 3] * inv);
        *reinterpret_cast<ushort4*>(op + 32 * d + 8 * g4 + 4 * h) = v;
      }
    }
    if (h == 0) P.lse[(int64_t)head * P.T + s0 + qrow] = (lt > 0.f) ? (m + log2f(lt)) * kLn2 : -INFINITY;
  }
}

// delta[h][t] = sum_d dO[t][h][d] * O[t][h][d]   (one wave per (t, h) row)
template <int D>
__global__ void bwd_pre_kernel(const uint16_t* __restrict__ o, const uint16_t* __restrict__ dout,
                               float* __restrict__ delta, int64_t T, int hq) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T * hq) return;
  constexpr int PERL = D / 64;  // elements per lane
  const uint16_t* op = o + row * D + lane * PERL;
  const uint16_t* dp = dout + row * D + lane * PERL;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < PERL; ++j) s += bf2f(op[j]) * bf2f(dp[j]);
  s = wave_sum(s);
  if (lane == 0) {
    const int64_t t = row / hq;
    const int hh = row % hq;
    delta[(int64_t)hh * T + t] = s;
  }
}

struct BwdParams {
  const uint16_t *q, *k, *v, *dout;
  int64_t sq, sk, sv;  // token strides of q, k, v (dout is contiguous [T, Hq, D])
  const float *lse, *delta;
  float* dq;           // [T, Hq, D] f32 accumulator
  uint16_t *dk, *dv;   // [T, Hkv, D] views
  int64_t sdk, sdv;    // token strides of dk, dv
  const int* cu;
  int64_t T;
  int hq, hkv;
  float scale, c2;
};

constexpr int kBwdBK = 128;  // keys per workgroup (4 waves x 32)
constexpr int kBwdBQ = 32;   // query rows per slice

template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, D == 128 ? 1 : 2) void bwd_kernel(BwdParams P) {
  constexpr int NC = D / 16;
  constexpr int ND = D / 32;
  constexpr int SLICE = kBwdBQ * D * 2;           // bytes of one Q (or dO) slice image
  constexpr int KBYTES = kBwdBK * D * 2;
  constexpr int DSBYTES = kBwdBK * kBwdBQ * 2;    // dS^T image [128 keys][32 q]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Kl = smem;
  auto qbuf = [&](int i) { return smem + KBYTES + i * 2 * SLICE; };
  auto dobuf = [&](int i) { return smem + KBYTES + i * 2 * SLICE + SLICE; };
  char* dSl = smem + KBYTES + 4 * SLICE;
  float* rowc = reinterpret_cast<float*>(smem + KBYTES + 4 * SLICE + DSBYTES);  // [2][2][32]

  const int seq = blockIdx.z, kvh = blockIdx.y;
  const int s0 = P.cu[seq];
  const int seqlen = P.cu[seq + 1] - s0;
  const int kb = blockIdx.x * kBwdBK;
  if (kb >= seqlen) return;
  const int group = P.hq / P.hkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int key = kb + 32 * w + r;  // this lane's key (sequence-relative)

  // K block -> LDS (used by S and dQ); V rows for this lane's key -> registers (dP B operand).
  {
    Stager<kBwdBK, D, 256> stk;
    stk.load(P.k + (int64_t)(s0 + kb) * P.sk + (int64_t)kvh * D, P.sk, seqlen - kb);
    stk.store(Kl);
  }
  bf16x8 vf[NC];
  {
    const bool ok = key < seqlen;
    const uint16_t* vp = P.v + (int64_t)(s0 + (ok ? key : 0)) * P.sv + (int64_t)kvh * D + 8 * h;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      u16x8 t = ok ? *reinterpret_cast<const u16x8*>(vp + 16 * c) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      vf[c] = __builtin_bit_cast(bf16x8, t);
    }
  }

  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    dk[i] = f32x16{};
    dv[i] = f32x16{};
  }

  const int first_slice = CAUSAL ? (kb / kBwdBQ) : 0;
  const int nslices_q = (seqlen + kBwdBQ - 1) / kBwdBQ;
  const int per_head = nslices_q - first_slice;
  const int nitems = per_head * group;

  auto item_rows = [&](int it, int& hqi, int& qs) {
    hqi = kvh * group + it / per_head;
    qs = (first_slice + it % per_head) * kBwdBQ;
  };

  Stager<kBwdBQ, D, 256> sq, sdo;
  float rc = 0.f;  // lse2 / delta prefetch for threads 0..63
  auto load_item = [&](int it) {
    int hqi, qs;
    item_rows(it, hqi, qs);
    const int nv = seqlen - qs;
    sq.load(P.q + (int64_t)(s0 + qs) * P.sq + (int64_t)hqi * D, P.sq, nv);
    sdo.load(P.dout + ((int64_t)(s0 + qs) * P.hq + hqi) * D, (int64_t)P.hq * D, nv);
    if (threadIdx.x < 64) {
      const int qi = qs + (threadIdx.x & 31);
      const bool ok = qi < seqlen;
      if (threadIdx.x < 32) rc = ok ? P.lse[(int64_t)hqi * P.T + s0 + qi] * kLog2e : 0.f;
      else rc = ok ? P.delta[(int64_t)hqi * P.T + s0 + qi] : 0.f;
    }
  };
  auto store_item = [&](int buf) {
    sq.store(qbuf(buf));
    sdo.store(dobuf(buf));
    if (threadIdx.x < 64) rowc[buf * 64 + threadIdx.x] = rc;
  };

  if (nitems > 0) {
    load_item(0);
    store_item(0);
  }
  __syncthreads();

  for (int it = 0; it < nitems; ++it) {
    const int buf = it & 1;
    const bool more = it + 1 < nitems;
    if (more) load_item(it + 1);
    int hqi, qs;
    item_rows(it, hqi, qs);
    const char* Ql = qbuf(buf);
    const char* dOl = dobuf(buf);
    const float* lse2 = rowc + buf * 64;
    const float* dlt = lse2 + 32;

    f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      s = mfma(row_frag<D>(Ql, r, 2 * c + h), row_frag<D>(Kl, 32 * w + r, 2 * c + h), s);
      dp = mfma(row_frag<D>(dOl, r, 2 * c + h), vf[c], dp);
    }
    // P and dS (key on the lane, query rows in the registers).
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qr = acc_row(i, h);
      const int qi = qs + qr;
      const bool valid = (qi < seqlen) && (key < seqlen) && (!CAUSAL || key <= qi);
      const float p = valid ? exp2f(s[i] * P.c2 - lse2[qr]) : 0.f;
      s[i] = p;
      dp[i] = p * (dp[i] - dlt[qr]) * P.scale;
    }
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const bf16x8 pf = pack8(s, st);
      const bf16x8 dsf = pack8(dp, st);
      const int ra = 16 * st + 4 * h;
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        dv[d] = mfma(tr_frag<D>(dOl, ra, ra + 8, 32 * d), pf, dv[d]);
        dk[d] = mfma(tr_frag<D>(Ql, ra, ra + 8, 32 * d), dsf, dk[d]);
      }
    }
    // dS^T -> LDS image [128 keys][32 q]: this lane's key row, 4 groups of 4 queries.
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      ushort4 v;
      v.x = f2bf(dp[4 * g4 + 0]);
      v.y = f2bf(dp[4 * g4 + 1]);
      v.z = f2bf(dp[4 * g4 + 2]);
      v.w = f2bf(dp[4 * g4 + 3]);
      *reinterpret_cast<ushort4*>(dSl + off<kBwdBQ>(32 * w + r, g4) + 8 * h) = v;
    }
    __syncthreads();
    // dQ[q][d] = sum_key dS[q][key] K[key][d]; wave -> (d tile, key range).
    {
      constexpr int KSPLIT = 4 / ND;  // waves sharing one d tile split the keys
      const int dt = w % ND;
      const int kpart = w / ND;
      constexpr int KPER = kBwdBK / KSPLIT;
      f32x16 q = f32x16{};
#pragma unroll
      for (int st = 0; st < KPER / 16; ++st) {
        const int k0 = kpart * KPER + 16 * st + 8 * h;
        q = mfma(tr_frag<kBwdBQ>(dSl, k0, k0 + 4, 0), tr_frag<D>(Kl, k0, k0 + 4, 32 * dt), q);
      }
      float* dqp = P.dq + (int64_t)(s0 + qs) * P.hq * D + (int64_t)hqi * D + 32 * dt + r;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qr = acc_row(i, h);
        if (qs + qr < seqlen) atomicAdd(dqp + (int64_t)qr * P.hq * D, q[i]);
      }
    }
    if (more) store_item(buf ^ 1);
    __syncthreads();
  }

  if (key < seqlen) {
    uint16_t* dkp = P.dk + (int64_t)(s0 + key) * P.sdk + (int64_t)kvh * D;
    uint16_t* dvp = P.dv + (int64_t)(s0 + key) * P.sdv + (int64_t)kvh * D;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        ushort4 a, b;
        a.x = f2bf(dk[d][4 * g4 + 0]); a.y = f2bf(dk[d][4 * g4 + 1]);
        a.z = f2bf(dk[d][4 * g4 + 2]); a.w = f2bf(dk[d][4 * g4 + 3]);
        b.x = f2bf(dv[d][4 * g4 + 0]); b.y = f2bf(dv[d][4 * g4 + 1]);
        b.z = f2bf(dv[d][4 * g4 + 2]); b.w = f2bf(dv[d][4 * g4 + 3]);
        *reinterpret_cast<ushort4*>(dkp + 32 * d + 8 * g4 + 4 * h) = a;
        *reinterpret_cast<ushort4*>(dvp + 32 * d + 8 * g4 + 4 * h) = b;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Backward v2: 8 waves share one 256-key block (32 keys per wave, dK^T/dV^T in registers) and
// sweep 64-row query items.  Per item: phase 1 computes S, dP (key on the lane), P, dS and the
// dV^T/dK^T products and stores dS^T to LDS; phase 2 computes this item's dQ partial over all
// 256 keys (one 32x32 tile per wave) and adds it with f32 atomics.  Compared with v1 the K/V
// block and the Q/dO staging are shared by twice the waves (2 waves per SIMD instead of 1) and
// the dQ atomic traffic per FLOP halves (256- instead of 128-key blocks).
constexpr int kB2K = 256;  // keys per workgroup (8 waves x 32)
constexpr int kB2Q = 64;   // query rows per item (2 x 32-row sub-tiles)
constexpr int kB2Threads = 512;

template <int D, bool CAUSAL>
__global__ __launch_bounds__(kB2Threads, 2) void bwd2_kernel(BwdParams P) {
  constexpr int NC = D / 16;
  constexpr int ND = D / 32;
  constexpr int KBYTES = kB2K * D * 2;
  constexpr int QBYTES = kB2Q * D * 2;
  constexpr int DSBYTES = kB2K * kB2Q * 2;  // dS^T image [256 keys][64 q]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Kl = smem;
  char* Ql = smem + KBYTES;
  char* dOl = Ql + QBYTES;
  char* dSl = dOl + QBYTES;
  float* rowc = reinterpret_cast<float*>(dSl + DSBYTES);  // lse2[64], delta[64]

  const int seq = blockIdx.z, kvh = blockIdx.y;
  const int s0 = P.cu[seq];
  const int seqlen = P.cu[seq + 1] - s0;
  const int kb = blockIdx.x * kB2K;
  if (kb >= seqlen) return;
  const int group = P.hq / P.hkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int key = kb + 32 * w + r;

  {
    Stager<kB2K, D, kB2Threads> stk;
    stk.load(P.k + (int64_t)(s0 + kb) * P.sk + (int64_t)kvh * D, P.sk, seqlen - kb);
    stk.store(Kl);
  }
  bf16x8 vf[NC];
  {
    const bool ok = key < seqlen;
    const uint16_t* vp = P.v + (int64_t)(s0 + (ok ? key : 0)) * P.sv + (int64_t)kvh * D + 8 * h;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      u16x8 t = ok ? *reinterpret_cast<const u16x8*>(vp + 16 * c) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      vf[c] = __builtin_bit_cast(bf16x8, t);
    }
  }
  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    dk[i] = f32x16{};
    dv[i] = f32x16{};
  }

  const int first_slice = CAUSAL ? (kb / kB2Q) : 0;
  const int nslices = (seqlen + kB2Q - 1) / kB2Q;
  const int per_head = nslices - first_slice;
  const int nitems = per_head * group;
  auto item = [&](int it, int& hqi, int& qs) {
    hqi = kvh * group + it / per_head;
    qs = (first_slice + it % per_head) * kB2Q;
  };

  Stager<kB2Q, D, kB2Threads> sq, sdo;
  float rc = 0.f;
  auto load_item = [&](int it) {
    int hqi, qs;
    item(it, hqi, qs);
    const int nv = seqlen - qs;
    sq.load(P.q + (int64_t)(s0 + qs) * P.sq + (int64_t)hqi * D, P.sq, nv);
    sdo.load(P.dout + ((int64_t)(s0 + qs) * P.hq + hqi) * D, (int64_t)P.hq * D, nv);
    if (threadIdx.x < 128) {
      const int qi = qs + (threadIdx.x & 63);
      const bool ok = qi < seqlen;
      if (threadIdx.x < 64) rc = ok ? P.lse[(int64_t)hqi * P.T + s0 + qi] * kLog2e : 0.f;
      else rc = ok ? P.delta[(int64_t)hqi * P.T + s0 + qi] : 0.f;
    }
  };
  auto store_item = [&]() {
    sq.store(Ql);
    sdo.store(dOl);
    if (threadIdx.x < 128) rowc[threadIdx.x] = rc;
  };

  if (nitems > 0) {
    load_item(0);
    store_item();
  }
  __syncthreads();

  // dQ tile assignment: tiles = 2 q-subtiles x ND d-tiles; waves beyond split the keys.
  constexpr int TILES = 2 * ND;
  constexpr int KSPLIT = 8 / TILES;
  constexpr int KPER = kB2K / KSPLIT;
  const int tile = w % TILES, kpart = w / TILES;
  const int tq = tile / ND, tdt = tile % ND;

  for (int it = 0; it < nitems; ++it) {
    const bool more = it + 1 < nitems;
    if (more) load_item(it + 1);
    int hqi, qs;
    item(it, hqi, qs);
    // ---------------- phase 1: per 32-row sub-tile, key on the lane (not unrolled: keeps one
    // sub-tile's S/dP live at a time)
#pragma unroll 1
    for (int qt = 0; qt < 2; ++qt) {
      const int qrow0 = qs + 32 * qt;
      const bool skip = CAUSAL && (qrow0 + 31 < kb + 32 * w);  // all queries before all keys
      f32x16 s = f32x16{}, dp = f32x16{};
      if (!skip) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          s = mfma(row_frag<D>(Ql, 32 * qt + r, 2 * c + h), row_frag<D>(Kl, 32 * w + r, 2 * c + h), s);
          dp = mfma(row_frag<D>(dOl, 32 * qt + r, 2 * c + h), vf[c], dp);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int qr = 32 * qt + acc_row(i, h);
          const int qi = qs + qr;
          const bool valid = (qi < seqlen) && (key < seqlen) && (!CAUSAL || key <= qi);
          const float p = valid ? exp2f(s[i] * P.c2 - rowc[qr]) : 0.f;
          s[i] = p;
          dp[i] = p * (dp[i] - rowc[64 + qr]) * P.scale;
        }
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 pf = pack8(s, st);
          const bf16x8 dsf = pack8(dp, st);
          const int ra = 32 * qt + 16 * st + 4 * h;
#pragma unroll
          for (int d = 0; d < ND; ++d) {
            dv[d] = mfma(tr_frag<D>(dOl, ra, ra + 8, 32 * d), pf, dv[d]);
            dk[d] = mfma(tr_frag<D>(Ql, ra, ra + 8, 32 * d), dsf, dk[d]);
          }
        }
      }
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        ushort4 v;
        v.x = f2bf(dp[4 * g4 + 0]);
        v.y = f2bf(dp[4 * g4 + 1]);
        v.z = f2bf(dp[4 * g4 + 2]);
        v.w = f2bf(dp[4 * g4 + 3]);
        *reinterpret_cast<ushort4*>(dSl + off<kB2Q>(32 * w + r, 4 * qt + g4) + 8 * h) = v;
      }
    }
    __syncthreads();
    // ---------------- phase 2: next item's Q/dO go to LDS while this item's dQ is summed
    if (more) store_item();
    {
      f32x16 q = f32x16{};
#pragma unroll
      for (int st = 0; st < KPER / 16; ++st) {
        const int k0 = kpart * KPER + 16 * st + 8 * h;
        q = mfma(tr_frag<kB2Q>(dSl, k0, k0 + 4, 32 * tq), tr_frag<D>(Kl, k0, k0 + 4, 32 * tdt), q);
      }
      const int qbase = qs + 32 * tq;
      float* dqp = P.dq + (int64_t)(s0 + qbase) * P.hq * D + (int64_t)hqi * D + 32 * tdt + r;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qr = acc_row(i, h);
        if (qbase + qr < seqlen) atomicAdd(dqp + (int64_t)qr * P.hq * D, q[i]);
      }
    }
    __syncthreads();
  }

  if (key < seqlen) {
    uint16_t* dkp = P.dk + (int64_t)(s0 + key) * P.sdk + (int64_t)kvh * D;
    uint16_t* dvp = P.dv + (int64_t)(s0 + key) * P.sdv + (int64_t)kvh * D;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        ushort4 a, b;
        a.x = f2bf(dk[d][4 * g4 + 0]); a.y = f2bf(dk[d][4 * g4 + 1]);
        a.z = f2bf(dk[d][4 * g4 + 2]); a.w = f2bf(dk[d][4 * g4 + 3]);
        b.x = f2bf(dv[d][4 * g4 + 0]); b.y = f2bf(dv[d][4 * g4 + 1]);
        b.z = f2bf(dv[d][4 * g4 + 2]); b.w = f2bf(dv[d][4 * g4 + 3]);
        *reinterpret_cast<ushort4*>(dkp + 32 * d + 8 * g4 + 4 * h) = a;
        *reinterpret_cast<ushort4*>(dvp + 32 * d + 8 * g4 + 4 * h) = b;
      }
    }
  }
}

// dq f32 [T, W] (contiguous) -> bf16 destination rows with token stride `ld` (W % 8 == 0).
__global__ void f32_to_bf16_rows_kernel(const float* __restrict__ in, uint16_t* __restrict__ out,
                                        int64_t T, int W, int64_t ld) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= T * W) return;
  const int64_t t = i / W;
  const int c = i % W;
  const float4 a = reinterpret_cast<const float4*>(in + i)[0];
  const float4 b = reinterpret_cast<const float4*>(in + i)[1];
  float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  store8(out + t * ld + c, v);
}

}  // namespace fa

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

std::tuple<at::Tensor, at::Tensor> flash_attn_fwd(const at::Tensor& q, const at::Tensor& k,
                                                  const at::Tensor& v, const at::Tensor& cu_seqlens,
                                                  int64_t max_seqlen, double scale, bool causal) {
  const int64_t T = q.size(0), hq = q.size(1), D = q.size(2), hkv = k.size(1);
  check_qkv(q, "q", hq, D);
  check_qkv(k, "k", hkv, D);
  check_qkv(v, "v", hkv, D);
  DTG_CHECK(k.size(0) == T && v.size(0) == T, "flash_attn: q/k/v token counts differ");
  DTG_CHECK(hq % hkv == 0, "flash_attn: Hq must be a multiple of Hkv");
  DTG_CHECK(D == 64 || D == 128, "flash_attn: head_dim must be 64 or 128");
  DTG_CHECK(cu_seqlens.scalar_type() == at::kInt && cu_seqlens.is_cuda() && cu_seqlens.is_contiguous(),
            "flash_attn: cu_seqlens must be int32 on the GPU");
  const c10::DeviceGuard g(q.device());
  auto o = at::empty({T, hq, D}, q.options());
  auto lse = at::empty({hq, T}, q.options().dtype(at::kFloat));
  const int nseq = cu_seqlens.numel() - 1;
  if (T == 0 || nseq <= 0 || max_seqlen <= 0) return {o, lse};
  fa::FwdParams P{bf16_ptr(q), bf16_ptr(k), bf16_ptr(v), q.stride(0), k.stride(0), v.stride(0),
                  bf16_mut(o), lse.data_ptr<float>(), cu_seqlens.data_ptr<int>(), T, (int)hq, (int)hkv,
                  (float)(scale * fa::kLog2e)};
  dim3 grid((max_seqlen + fa::kFwdBQ - 1) / fa::kFwdBQ, hq, nseq);
  const size_t lds = 4 * fa::kFwdBK * D * 2;
#define DTG_FWD(DD, C)                                                                    \
  do { set_lds_limit((const void*)&fa::fwd_kernel<DD, C>, lds);                              \
       hipLaunchKernelGGL((fa::fwd_kernel<DD, C>), grid, dim3(256), lds, stream(), P); } while (0)
  if (D == 128) { if (causal) DTG_FWD(128, true); else DTG_FWD(128, false); }
  else { if (causal) DTG_FWD(64, true); else DTG_FWD(64, false); }
#undef DTG_FWD
  DTG_LAUNCH_CHECK();
  return {o, lse};
}

// Shared backward driver: outputs are [T, H, D] views (contiguous heads, any token stride).
static void flash_attn_bwd_impl(const at::Tensor& dout_, const at::Tensor& q, const at::Tensor& k,
                                const at::Tensor& v, const at::Tensor& o, const at::Tensor& lse,
                                const at::Tensor& cu_seqlens, int64_t max_seqlen, double scale,
                                bool causal, const at::Tensor& dq, const at::Tensor& dk,
                                const at::Tensor& dv) {
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
  auto dq32 = at::zeros({T, hq, D}, opts.dtype(at::kFloat));
  auto delta = at::empty({hq, T}, opts.dtype(at::kFloat));
  {
    const int64_t rows = T * hq;
    const int blocks = (rows + 3) / 4;
    if (D == 128) fa::bwd_pre_kernel<128><<<blocks, 256, 0, stream()>>>(bf16_ptr(o), bf16_ptr(dout), delta.data_ptr<float>(), T, hq);
    else fa::bwd_pre_kernel<64><<<blocks, 256, 0, stream()>>>(bf16_ptr(o), bf16_ptr(dout), delta.data_ptr<float>(), T, hq);
    DTG_LAUNCH_CHECK();
  }
  fa::BwdParams P{bf16_ptr(q), bf16_ptr(k), bf16_ptr(v), bf16_ptr(dout), q.stride(0), k.stride(0),
                  v.stride(0), lse.data_ptr<float>(), delta.data_ptr<float>(), dq32.data_ptr<float>(),
                  bf16_mut(dk), bf16_mut(dv), dk.stride(0), dv.stride(0), cu_seqlens.data_ptr<int>(), T,
                  (int)hq, (int)hkv, (float)scale, (float)(scale * fa::kLog2e)};
  // v1 (4 waves x 32 keys, 1 wave/SIMD) is the default; DTG_FA_BWD=2 selects the experimental
  // 8-wave variant (register-bound at head_dim 128: spills, see profiles/).
  static const bool use_v1 = [] {
    const char* e = std::getenv("DTG_FA_BWD");
    return !(e != nullptr && e[0] == '2');
  }();
  if (use_v1) {
    dim3 grid((max_seqlen + fa::kBwdBK - 1) / fa::kBwdBK, hkv, nseq);
    const size_t lds = fa::kBwdBK * D * 2 + 4 * fa::kBwdBQ * D * 2 + fa::kBwdBK * fa::kBwdBQ * 2 + 2 * 64 * 4;
#define DTG_BWD(DD, C)                                                                    \
  do { set_lds_limit((const void*)&fa::bwd_kernel<DD, C>, lds);                              \
       hipLaunchKernelGGL((fa::bwd_kernel<DD, C>), grid, dim3(256), lds, stream(), P); } while (0)
    if (D == 128) { if (causal) DTG_BWD(128, true); else DTG_BWD(128, false); }
    else { if (causal) DTG_BWD(64, true); else DTG_BWD(64, false); }
#undef DTG_BWD
  } else {
    dim3 grid((max_seqlen + fa::kB2K - 1) / fa::kB2K, hkv, nseq);
    const size_t lds = fa::kB2K * D * 2 + 2 * fa::kB2Q * D * 2 + fa::kB2K * fa::kB2Q * 2 + 128 * 4;
#define DTG_BWD2(DD, C)                                                                   \
  do { set_lds_limit((const void*)&fa::bwd2_kernel<DD, C>, lds);                             \
       hipLaunchKernelGGL((fa::bwd2_kernel<DD, C>), grid, dim3(fa::kB2Threads), lds, stream(), P); } while (0)
    if (D == 128) { if (causal) DTG_BWD2(128, true); else DTG_BWD2(128, false); }
    else { if (causal) DTG_BWD2(64, true); else DTG_BWD2(64, false); }
#undef DTG_BWD2
  }
  DTG_LAUNCH_CHECK();
  const int W = hq * D;
  const int64_t n = T * W;
  fa::f32_to_bf16_rows_kernel<<<(n / 8 + 255) / 256, 256, 0, stream()>>>(dq32.data_ptr<float>(), bf16_mut(dq),
                                                                          T, W, dq.stride(0));
  DTG_LAUNCH_CHECK();
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> flash_attn_bwd(
    const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
    const at::Tensor& o, const at::Tensor& lse, const at::Tensor& cu_seqlens, int64_t max_seqlen,
    double scale, bool causal) {
  auto dq = at::empty(q.sizes(), q.options());
  auto dk = at::empty(k.sizes(), k.options());
  auto dv = at::empty(v.sizes(), v.options());
  flash_attn_bwd_impl(dout, q, k, v, o, lse, cu_seqlens, max_seqlen, scale, causal, dq, dk, dv);
  return {dq, dk, dv};
}

// q, k, v are head slices of one fused [T, (nq + 2 nkv) * D] projection output; the gradient
// comes back in the same fused layout so the QKV GEMM backward consumes it directly.
at::Tensor flash_attn_bwd_qkv(const at::Tensor& dout, const at::Tensor& qkv, int64_t nq, int64_t nkv,
                              int64_t head_dim, const at::Tensor& o, const at::Tensor& lse,
                              const at::Tensor& cu_seqlens, int64_t max_seqlen, double scale, bool causal) {
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
                      view3(dqkv, nq + nkv, nkv));
  return dqkv;
}

TORCH_LIBRARY_IMPL(dtg, CUDA, m) {
  m.impl("flash_attn_fwd", &flash_attn_fwd);
  m.impl("flash_attn_bwd", &flash_attn_bwd);
  m.impl("flash_attn_bwd_qkv", &flash_attn_bwd_qkv);
}

}  // namespace dtg
