// Power-aware GEMM solution selection for hipBLASLt on MI355X.
//
// Why: MI355X runs its MFMA pipes under a board power limit.  With random bf16 operands a
// sustained GEMM settles at ~1.5 PF/s while the same GEMM on zeros reaches ~2.1 PF/s
// (profiles/r1_s24_gemm_ceiling_random_vs_zeros.jsonl): the clock is set by power, not by the
// kernel.  PyTorch TunableOp ranks solutions with a few short timed calls, i.e. at whatever
// clock the chip has at that instant, which favours kernels that are fastest at boost clock.
// During training the GEMMs run back to back for hundreds of milliseconds, so what matters is
// the throughput at the power limit -- where a solution that moves fewer bytes through the
// register file per FLOP (e.g. 32x32 MFMA tiles instead of 16x16) can sustain a higher clock.
//
// This tool times every hipBLASLt solution of one problem (TunableOp's "tn_M_N_K_ld_A_B_C"
// spelling) with a short burst, then re-times the best candidates -- plus the library's
// heuristic default and the best 32x32-MFMA solutions -- under sustained back-to-back load,
// round-robin so clock drift hits every candidate alike.  It prints one JSON line per
// candidate.  Caveat: this binary links the system hipBLASLt (/opt/rocm), while PyTorch runs
// its own bundled copy, whose solution indices differ (TunableOp's Gemm_Hipblaslt_618xxx vs
// 439xxx here, profiles/r3_s14): rank solutions here, but pin them through TunableOp itself
// (tools/tune_gemms.py --retune [--rotating-mb]).
//
//   hipcc -O2 --offload-arch=gfx950 tools/gemm_sustained.cpp -lhipblaslt -o build/gemm_sustained
//   build/gemm_sustained tn_28672_16384_4096_ld_4096_4096_28672 [secs_per_round=0.4] [top=12]
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK_HIP(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)
#define CK_BL(x)                                                                   \
  do {                                                                             \
    hipblasStatus_t s_ = (x);                                                      \
    if (s_ != HIPBLAS_STATUS_SUCCESS) {                                            \
      std::fprintf(stderr, "hipBLASLt error %d at %s:%d\n", (int)s_, __FILE__, __LINE__); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

// N(0,1)-like bf16 fill from a counter hash (Irwin-Hall of 4 uniforms), no host round trip.
__global__ void fill_randn_bf16(uint16_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    float s = 0.f;
    for (int j = 0; j < 4; ++j) {
      h ^= h >> 16;
      h *= 0x7feb352du;
      h ^= h >> 15;
      h *= 0x846ca68bu;
      h ^= h >> 16;
      s += (h & 0xffffff) * (1.f / 16777216.f);
    }
    const float v = (s - 2.f) * 1.7320508f;  // unit variance
    uint32_t b;
    std::memcpy(&b, &v, 4);
    p[i] = (uint16_t)((b + 0x7fff + ((b >> 16) & 1)) >> 16);
  }
}

struct Cand {
  hipblasLtMatmulAlgo_t algo;
  int index;
  std::string kernel;
  size_t ws;
  double short_ms = 1e30;
  std::vector<double> sustained;
  bool is_default = false;
};

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s tn_M_N_K_ld_LDA_LDB_LDC [secs_per_round] [top]\n", argv[0]);
    return 2;
  }
  const std::string spec = argv[1];
  const double secs = argc > 2 ? std::atof(argv[2]) : 0.4;
  const int top = argc > 3 ? std::atoi(argv[3]) : 12;
  char ta, tb;
  long m, n, k, lda, ldb, ldc;
  if (std::sscanf(spec.c_str(), "%c%c_%ld_%ld_%ld_ld_%ld_%ld_%ld", &ta, &tb, &m, &n, &k, &lda, &ldb, &ldc) != 8) {
    std::fprintf(stderr, "bad spec %s\n", spec.c_str());
    return 2;
  }
  const hipblasOperation_t opA = ta == 't' ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  const hipblasOperation_t opB = tb == 't' ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  // column-major storage extents (BLAS convention, as TunableOp records them)
  const long ar = ta == 'n' ? m : k, ac = ta == 'n' ? k : m;
  const long br = tb == 'n' ? k : n, bc = tb == 'n' ? n : k;
  const size_t na = (size_t)lda * ac, nb = (size_t)ldb * bc, nc = (size_t)ldc * n;
  uint16_t *A, *B, *C;
  CK_HIP(hipMalloc(&A, na * 2));
  CK_HIP(hipMalloc(&B, nb * 2));
  CK_HIP(hipMalloc(&C, nc * 2));
  fill_randn_bf16<<<4096, 256>>>(A, na, 1u);
  fill_randn_bf16<<<4096, 256>>>(B, nb, 2u);
  CK_HIP(hipMemset(C, 0, nc * 2));
  const size_t ws_max = 256ull << 20;
  void* ws;
  CK_HIP(hipMalloc(&ws, ws_max));
  hipStream_t st;
  CK_HIP(hipStreamCreate(&st));

  hipblasLtHandle_t h;
  CK_BL(hipblasLtCreate(&h));
  hipblasLtMatmulDesc_t desc;
  CK_BL(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  CK_BL(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA)));
  CK_BL(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB)));
  hipblasLtMatrixLayout_t la, lb, lc;
  CK_BL(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, ar, ac, lda));
  CK_BL(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, br, bc, ldb));
  CK_BL(hipblasLtMatrixLayoutCreate(&lc, HIP_R_16BF, m, n, ldc));
  const float alpha = 1.f, beta = 0.f;

  std::vector<hipblasLtMatmulHeuristicResult_t> all;
  CK_BL(hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, opA, opB, HIP_R_16BF, HIP_R_16BF,
                                   HIP_R_16BF, HIP_R_16BF, HIPBLAS_COMPUTE_32F, all));
  std::vector<Cand> cands;
  for (auto& r : all) {
    size_t wsz = 0;
    if (hipblaslt_ext::matmulIsAlgoSupported(h, desc, &alpha, la, lb, &beta, lc, lc, r.algo, wsz) !=
        HIPBLAS_STATUS_SUCCESS || wsz > ws_max)
      continue;
    Cand c;
    c.algo = r.algo;
    c.index = hipblaslt_ext::getIndexFromAlgo(r.algo);
    c.kernel = hipblaslt_ext::getKernelNameFromAlgo(h, r.algo);
    c.ws = wsz;
    cands.push_back(c);
  }
  // the library's own pick (what TunableOp records as "Default")
  {
    hipblasLtMatmulPreference_t pref;
    CK_BL(hipblasLtMatmulPreferenceCreate(&pref));
    CK_BL(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws_max, sizeof(ws_max)));
    hipblasLtMatmulHeuristicResult_t hr[1];
    int got = 0;
    if (hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, lc, lc, pref, 1, hr, &got) == HIPBLAS_STATUS_SUCCESS && got) {
      const int di = hipblaslt_ext::getIndexFromAlgo(hr[0].algo);
      for (auto& c : cands)
        if (c.index == di) c.is_default = true;
    }
    hipblasLtMatmulPreferenceDestroy(pref);
  }
  std::fprintf(stderr, "[gemm_sustained] %s: %zu supported solutions of %zu\n", spec.c_str(), cands.size(), all.size());
  const double flop = 2.0 * m * n * k;
  auto run = [&](Cand& c, int iters) {
    for (int i = 0; i < iters; ++i)
      CK_BL(hipblasLtMatmul(h, desc, &alpha, A, la, B, lb, &beta, C, lc, C, lc, &c.algo, ws, c.ws, st));
  };
  hipEvent_t e0, e1;
  CK_HIP(hipEventCreate(&e0));
  CK_HIP(hipEventCreate(&e1));
  // phase 1: short bursts (what a quick tuner sees)
  for (auto& c : cands) {
    run(c, 2);
    CK_HIP(hipEventRecord(e0, st));
    run(c, 5);
    CK_HIP(hipEventRecord(e1, st));
    CK_HIP(hipEventSynchronize(e1));
    float ms;
    CK_HIP(hipEventElapsedTime(&ms, e0, e1));
    c.short_ms = ms / 5;
  }
  std::sort(cands.begin(), cands.end(), [](const Cand& a, const Cand& b) { return a.short_ms < b.short_ms; });
  std::vector<Cand*> fin;
  for (int i = 0; i < (int)cands.size() && (int)fin.size() < top; ++i) fin.push_back(&cands[i]);
  int n32 = 0;
  for (auto& c : cands) {
    const bool mi32 = c.kernel.find("MI32x32") != std::string::npos;
    const bool in = std::find(fin.begin(), fin.end(), &c) != fin.end();
    if (in) continue;
    if (c.is_default || (mi32 && n32 < 4)) {
      fin.push_back(&c);
      n32 += mi32;
    }
  }
  // phase 2: sustained, round-robin over the finalists, 3 rounds
  const double est_ms = std::max(0.05, fin.empty() ? 1.0 : fin[0]->short_ms);
  for (int round = 0; round < 3; ++round) {
    for (Cand* c : fin) {
      const int iters = std::max(20, (int)(secs * 1000.0 / std::max(est_ms, c->short_ms)));
      run(*c, iters / 2);  // settle the clock under this kernel's load
      CK_HIP(hipEventRecord(e0, st));
      run(*c, iters);
      CK_HIP(hipEventRecord(e1, st));
      CK_HIP(hipEventSynchronize(e1));
      float ms;
      CK_HIP(hipEventElapsedTime(&ms, e0, e1));
      c->sustained.push_back(ms / iters);
    }
    std::fprintf(stderr, "[gemm_sustained] round %d done\n", round);
  }
  for (Cand* c : fin) {
    std::vector<double> s = c->sustained;
    std::sort(s.begin(), s.end());
    const double med = s[s.size() / 2];
    std::printf("{\"spec\": \"%s\", \"index\": %d, \"default\": %s, \"short_ms\": %.4f, \"sustained_ms\": %.4f, "
                "\"short_TF\": %.1f, \"sustained_TF\": %.1f, \"kernel\": \"%s\"}\n",
                spec.c_str(), c->index, c->is_default ? "true" : "false", c->short_ms, med, flop / c->short_ms / 1e9,
                flop / med / 1e9, c->kernel.c_str());
  }
  std::fflush(stdout);
  hipblasLtDestroy(h);
  return 0;
}
