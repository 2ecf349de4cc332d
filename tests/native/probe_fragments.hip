// Probe of the gfx950 operand/accumulator maps the attention kernels rely on
// (v_mfma_f32_32x32x16_bf16 A/B/C maps, ds_read_b64_tr_b16 via the swizzled LDS image).
// Prints PASS/FAIL per check; run by tests/test_native_probes.py on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cmath>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

template <int W>
__device__ int off(int row, int ch) {
  constexpr int NCH = W / 8;
  int sw;
  if constexpr (NCH >= 16) sw = ((row & 3) << 2) | ((row >> 2) & 3);
  else if constexpr (NCH == 8) sw = ((row & 1) << 2) | ((row >> 1) & 3);
  else sw = row & (NCH - 1);
  return row * (W * 2) + 16 * (ch ^ sw);
}

// 1) tr read: tile[r][c] = r*128 + c (as raw 16-bit ints); each lane writes what it got.
__global__ void tr_probe(short* out, int rowA, int rowB, int col0) {
  __shared__ __attribute__((aligned(16))) char tile[64 * 256];
  for (int i = threadIdx.x; i < 64 * 128; i += 64) {
    int r = i / 128, c = i % 128;
    *reinterpret_cast<short*>(tile + off<128>(r, c / 8) + 2 * (c % 8)) = (short)(r * 128 + c);
  }
  __syncthreads();
  const int lane = threadIdx.x;
  const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3, h = lane >> 5;
  const int colbase = col0 + 16 * (g & 1);
  const int ch = (colbase >> 3) + (p >> 1);
  const int half = 8 * (p & 1);
  i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(tile + off<128>(rowA + 4 * h + q, ch) + half));
  i16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(tile + off<128>(rowB + 4 * h + q, ch) + half));
  for (int j = 0; j < 4; ++j) { out[lane * 8 + j] = a[j]; out[lane * 8 + 4 + j] = b[j]; }
}

// 2) MFMA map: A[i][k] = float data, B[k][j]; lane fragments built per the documented maps.
__global__ void mfma_probe(const float* A, const float* B, float* C) {
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)A[r * 16 + 8 * h + j];
    b[j] = (__bf16)B[(8 * h + j) * 32 + r];
  }
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  for (int reg = 0; reg < 16; ++reg) {
    int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
    C[row * 32 + r] = acc[reg];
  }
}


// 3) accumulator as operand: S^T = K Q^T (32 keys x 32 q, K-dim 16), then O^T = V^T S^T with
//    S^T packed from the accumulator (permuted k) and V^T read from a swizzled LDS image with
//    the transposed read, exactly as the attention forward does it.
__global__ void acc_operand_probe(const float* K, const float* Q, const float* V, float* O, const float* S, int mode) {
  __shared__ __attribute__((aligned(16))) char tile[32 * 256];
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  for (int i = lane; i < 32 * 128; i += 64) {
    int row = i / 128, c = i % 128;
    __bf16 v = (__bf16)V[row * 128 + c];
    *reinterpret_cast<__bf16*>(tile + off<128>(row, c / 8) + 2 * (c % 8)) = v;
  }
  __syncthreads();
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)K[r * 16 + 8 * h + j]; b[j] = (__bf16)Q[r * 16 + 8 * h + j]; }
  f32x16 s = {};
  s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, s, 0, 0, 0);  // S^T[key][q]
  for (int dt = 0; dt < 4; ++dt) {
    f32x16 acc = {};
    for (int st = 0; st < 2; ++st) {
      bf16x8 pf;
      for (int j = 0; j < 8; ++j) {
        const int key = 16 * st + 8 * (j >> 2) + 4 * h + (j & 3);
        pf[j] = (mode & 2) ? (__bf16)S[key * 32 + r] : (__bf16)s[8 * st + j];
      }
      const int ra = 16 * st + 4 * h, rb = ra + 8;
      const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
      const int colbase = 32 * dt + 16 * (g & 1);
      const int ch = (colbase >> 3) + (p >> 1);
      const int half = 8 * (p & 1);
      i16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(tile + off<128>(ra + q, ch) + half));
      i16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(tile + off<128>(rb + q, ch) + half));
      typedef short i16x8 __attribute__((ext_vector_type(8)));
      bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
      if (mode & 1)
        for (int j = 0; j < 8; ++j) {
          const int key = 16 * st + 8 * (j >> 2) + 4 * h + (j & 3);
          vf[j] = (__bf16)V[key * 128 + 32 * dt + r];
        }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, acc, 0, 0, 0);
    }
    for (int reg = 0; reg < 16; ++reg) {
      int d = 32 * dt + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      O[d * 32 + r] = acc[reg];  // O^T[d][q]
    }
  }
}

int main() {
  int fails = 0;
  // tr probe
  short* d;
  (void)hipMalloc(&d, 64 * 8 * 2);
  int rowA = 16, rowB = 24, col0 = 32;
  tr_probe<<<1, 64>>>(d, rowA, rowB, col0);
  std::vector<short> o(64 * 8);
  (void)hipMemcpy(o.data(), d, o.size() * 2, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int lane = 0; lane < 64; ++lane) {
    int r = lane & 31, h = lane >> 5;
    for (int j = 0; j < 8; ++j) {
      int row = (j < 4 ? rowA : rowB) + 4 * h + (j & 3);
      int col = col0 + r;
      short want = row * 128 + col;
      if (o[lane * 8 + j] != want) {
        if (bad < 8) printf("tr lane %d elem %d got r%d c%d want r%d c%d\n", lane, j, o[lane * 8 + j] / 128, o[lane * 8 + j] % 128, row, col);
        ++bad;
      }
    }
  }
  printf("tr_read_b64_tr_b16 map: %s (%d bad)\n", bad ? "FAIL" : "PASS", bad);
  fails += bad != 0;
  // mfma probe with asymmetric data
  std::vector<float> A(32 * 16), B(16 * 32), C(32 * 32), R(32 * 32, 0.f);
  for (int i = 0; i < 32; ++i) for (int k = 0; k < 16; ++k) A[i * 16 + k] = (float)((i * 3 + k * 7) % 11 - 5);
  for (int k = 0; k < 16; ++k) for (int j = 0; j < 32; ++j) B[k * 32 + j] = (float)((k * 5 + j * 2) % 13 - 6);
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) for (int k = 0; k < 16; ++k) R[i * 32 + j] += A[i * 16 + k] * B[k * 32 + j];
  float *dA, *dB, *dC;
  (void)hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dC, C.size() * 4);
  (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  mfma_probe<<<1, 64>>>(dA, dB, dC);
  (void)hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
  bad = 0;
  for (int i = 0; i < 32 * 32; ++i) if (std::fabs(C[i] - R[i]) > 1e-3) { if (bad < 4) printf("mfma C[%d][%d] got %f want %f\n", i / 32, i % 32, C[i], R[i]); ++bad; }
  printf("mfma_f32_32x32x16_bf16 maps: %s (%d bad)\n", bad ? "FAIL" : "PASS", bad);
  fails += bad != 0;

  {
    std::vector<float> K(32 * 16), Q(32 * 16), V(32 * 128), O(128 * 32), R(128 * 32, 0.f), S(32 * 32, 0.f);
    for (int i = 0; i < 32 * 16; ++i) { K[i] = (float)((i * 7) % 3 - 1); Q[i] = (float)((i * 5 + 1) % 3 - 1); }
    for (int i = 0; i < 32 * 128; ++i) V[i] = (float)((i * 11 + 3) % 7 - 3);
    for (int key = 0; key < 32; ++key) for (int q = 0; q < 32; ++q) for (int k = 0; k < 16; ++k) S[key * 32 + q] += K[key * 16 + k] * Q[q * 16 + k];
    for (int d = 0; d < 128; ++d) for (int q = 0; q < 32; ++q) for (int key = 0; key < 32; ++key) R[d * 32 + q] += V[key * 128 + d] * S[key * 32 + q];
    float *dK, *dQ, *dV, *dO, *dS;
    (void)hipMalloc(&dS, S.size() * 4);
    (void)hipMemcpy(dS, S.data(), S.size() * 4, hipMemcpyHostToDevice);
    (void)hipMalloc(&dK, K.size() * 4); (void)hipMalloc(&dQ, Q.size() * 4); (void)hipMalloc(&dV, V.size() * 4); (void)hipMalloc(&dO, O.size() * 4);
    (void)hipMemcpy(dK, K.data(), K.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dQ, Q.data(), Q.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dV, V.data(), V.size() * 4, hipMemcpyHostToDevice);
    for (int mode = 3; mode >= 0; --mode) {
      acc_operand_probe<<<1, 64>>>(dK, dQ, dV, dO, dS, mode);
      (void)hipMemcpy(O.data(), dO, O.size() * 4, hipMemcpyDeviceToHost);
      int bad3 = 0;
      for (int i = 0; i < 128 * 32; ++i) if (std::fabs(O[i] - R[i]) > 1e-3) { if (bad3 < 3) printf("accop mode %d O^T[%d][%d] got %f want %f\n", mode, i / 32, i % 32, O[i], R[i]); ++bad3; }
      printf("PV mode %d (V %s, P %s): %s (%d bad)\n", mode, (mode & 1) ? "global" : "tr-read", (mode & 2) ? "global" : "accumulator", bad3 ? "FAIL" : "PASS", bad3);
      fails += bad3 != 0;
    }
  }
  return fails ? 1 : 0;
}
