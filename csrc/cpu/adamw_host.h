// Torch-independent core of the host AdamW (csrc/cpu/adamw_cpu.cpp): bf16 <-> f32 conversions
// and the OpenMP update loops over raw pointers.  Kept in a header so the same code is also
// compiled into the sanitizer harness (tests/native/sanitize_adamw_host.cpp, built with
// -fsanitize=address,undefined and run by tests/test_native_sanitizers_cpu.py).
//
// Three implementations of ONE arithmetic definition, selected at run time (or forced with
// DTG_HOST_ADAMW_ISA=scalar|avx2|avx512):
//   avx512  16 f32 lanes: bf16 widened by vpmovzxwd + shift, narrowed by integer
//           round-to-nearest-even + NaN quieting + vpmovdw (bit-exact with f2bf below; the
//           hardware VCVTNEPS2BF16 is NOT used because it flushes f32 denormals to zero)
//   avx2    8 lanes, same integer conversions
//   scalar  the reference loop
// Every operation is written out with explicit fused multiply-adds where the update has them
// and separate multiplies/adds elsewhere, so no compiler contraction choice (-ffp-contract)
// can make the paths disagree: they are bit-identical to each other and to the GPU kernel's
// contraction of the same formula (csrc/kernels/adamw.hip):
//   p  = p * (1 - lr*wd)
//   m  = fma(g - m, 1 - b1, m)
//   v  = fma(v, b2, ((1 - b2) * g) * g)
//   p  = p - (lr/bc1 * m) / (sqrt(v) / bc2s + eps)
// Threads take contiguous ranges (hardware prefetchers see one stream per buffer per thread).
#pragma once

#include <immintrin.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace dtg {
namespace host {

inline float bf2f(uint16_t v) {
  uint32_t u = static_cast<uint32_t>(v) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

inline uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

template <typename T>
inline float ld(const T* p, int64_t i);
template <>
inline float ld<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
template <>
inline float ld<float>(const float* p, int64_t i) { return p[i]; }
template <typename T>
inline void st(T* p, int64_t i, float v);
template <>
inline void st<uint16_t>(uint16_t* p, int64_t i, float v) { p[i] = f2bf(v); }
template <>
inline void st<float>(float* p, int64_t i, float v) { p[i] = v; }

struct AdamConsts {
  float step_size, decay, c1, b2, c2, bc2s, eps, gs;
};

inline AdamConsts make_consts(float lr, float b1, float b2, float eps, float wd, float bc1, float bc2s, float gs) {
  return AdamConsts{lr / bc1, 1.f - lr * wd, 1.f - b1, b2, 1.f - b2, bc2s, eps, gs};
}

// One element; every rounding step is its own statement (see the header comment).
inline void adam_scalar(float& p, float graw, float& m, float& v, const AdamConsts& k) {
  const float g = graw * k.gs;
  p = p * k.decay;
  const float d = g - m;
  m = std::fma(d, k.c1, m);
  const float cg = k.c2 * g;
  const float gg = cg * g;
  v = std::fma(v, k.b2, gg);
  float s = std::sqrt(v);
  s = s / k.bc2s;
  const float den = s + k.eps;
  float u = k.step_size * m;
  u = u / den;
  p = p - u;
}

template <typename PT, typename GT, typename ST>
inline void adam_range_scalar(PT* p, const GT* g, ST* m, ST* v, int64_t lo, int64_t hi, const AdamConsts& k) {
  for (int64_t i = lo; i < hi; ++i) {
    float pv = ld<PT>(p, i), mv = ld<ST>(m, i), vv = ld<ST>(v, i);
    adam_scalar(pv, ld<GT>(g, i), mv, vv, k);
    st<PT>(p, i, pv);
    st<ST>(m, i, mv);
    st<ST>(v, i, vv);
  }
}

// ------------------------------------------------------------------------------- AVX-512
#define DTG_AVX512 __attribute__((target("avx512f")))
#define DTG_AVX2 __attribute__((target("avx2,fma")))

DTG_AVX512 inline __m512 ld16(const uint16_t* p) {
  const __m256i h = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p));
  return _mm512_castsi512_ps(_mm512_slli_epi32(_mm512_cvtepu16_epi32(h), 16));
}
DTG_AVX512 inline __m512 ld16(const float* p) { return _mm512_loadu_ps(p); }
DTG_AVX512 inline void st16(uint16_t* p, __m512 x) {
  const __m512i u = _mm512_castps_si512(x);
  const __m512i hi = _mm512_srli_epi32(u, 16);
  const __m512i lsb = _mm512_and_si512(hi, _mm512_set1_epi32(1));
  __m512i r = _mm512_srli_epi32(_mm512_add_epi32(_mm512_add_epi32(u, _mm512_set1_epi32(0x7fff)), lsb), 16);
  const __mmask16 nan =
      _mm512_cmpgt_epu32_mask(_mm512_and_si512(u, _mm512_set1_epi32(0x7fffffff)), _mm512_set1_epi32(0x7f800000));
  r = _mm512_mask_mov_epi32(r, nan, _mm512_or_si512(hi, _mm512_set1_epi32(0x40)));
  _mm256_storeu_si256(reinterpret_cast<__m256i*>(p), _mm512_cvtepi32_epi16(r));
}
DTG_AVX512 inline void st16(float* p, __m512 x) { _mm512_storeu_ps(p, x); }

template <typename PT, typename GT, typename ST>
DTG_AVX512 void adam_range_avx512(PT* p, const GT* g, ST* m, ST* v, int64_t lo, int64_t hi, const AdamConsts& k) {
  const __m512 gs = _mm512_set1_ps(k.gs), decay = _mm512_set1_ps(k.decay), c1 = _mm512_set1_ps(k.c1),
               b2 = _mm512_set1_ps(k.b2), c2 = _mm512_set1_ps(k.c2), bc2s = _mm512_set1_ps(k.bc2s),
               eps = _mm512_set1_ps(k.eps), step = _mm512_set1_ps(k.step_size);
  int64_t i = lo;
  for (; i + 16 <= hi; i += 16) {
    const __m512 gv = _mm512_mul_ps(ld16(g + i), gs);
    __m512 pv = _mm512_mul_ps(ld16(p + i), decay);
    __m512 mv = ld16(m + i);
    __m512 vv = ld16(v + i);
    mv = _mm512_fmadd_ps(_mm512_sub_ps(gv, mv), c1, mv);
    vv = _mm512_fmadd_ps(vv, b2, _mm512_mul_ps(_mm512_mul_ps(c2, gv), gv));
    const __m512 den = _mm512_add_ps(_mm512_div_ps(_mm512_sqrt_ps(vv), bc2s), eps);
    pv = _mm512_sub_ps(pv, _mm512_div_ps(_mm512_mul_ps(step, mv), den));
    st16(p + i, pv);
    st16(m + i, mv);
    st16(v + i, vv);
  }
  adam_range_scalar(p, g, m, v, i, hi, k);
}

// --------------------------------------------------------------------------------- AVX2
DTG_AVX2 inline __m256 ld8(const uint16_t* p) {
  const __m128i h = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
  return _mm256_castsi256_ps(_mm256_slli_epi32(_mm256_cvtepu16_epi32(h), 16));
}
DTG_AVX2 inline __m256 ld8(const float* p) { return _mm256_loadu_ps(p); }
DTG_AVX2 inline void st8(uint16_t* p, __m256 x) {
  const __m256i u = _mm256_castps_si256(x);
  const __m256i hi = _mm256_srli_epi32(u, 16);
  const __m256i lsb = _mm256_and_si256(hi, _mm256_set1_epi32(1));
  __m256i r = _mm256_srli_epi32(_mm256_add_epi32(_mm256_add_epi32(u, _mm256_set1_epi32(0x7fff)), lsb), 16);
  // |u| as a signed int is >= 0, so the signed compare is the unsigned one here
  const __m256i nan = _mm256_cmpgt_epi32(_mm256_and_si256(u, _mm256_set1_epi32(0x7fffffff)),
                                         _mm256_set1_epi32(0x7f800000));
  r = _mm256_blendv_epi8(r, _mm256_or_si256(hi, _mm256_set1_epi32(0x40)), nan);
  const __m128i packed = _mm_packus_epi32(_mm256_castsi256_si128(r), _mm256_extracti128_si256(r, 1));
  _mm_storeu_si128(reinterpret_cast<__m128i*>(p), packed);
}
DTG_AVX2 inline void st8(float* p, __m256 x) { _mm256_storeu_ps(p, x); }

template <typename PT, typename GT, typename ST>
DTG_AVX2 void adam_range_avx2(PT* p, const GT* g, ST* m, ST* v, int64_t lo, int64_t hi, const AdamConsts& k) {
  const __m256 gs = _mm256_set1_ps(k.gs), decay = _mm256_set1_ps(k.decay), c1 = _mm256_set1_ps(k.c1),
               b2 = _mm256_set1_ps(k.b2), c2 = _mm256_set1_ps(k.c2), bc2s = _mm256_set1_ps(k.bc2s),
               eps = _mm256_set1_ps(k.eps), step = _mm256_set1_ps(k.step_size);
  int64_t i = lo;
  for (; i + 8 <= hi; i += 8) {
    const __m256 gv = _mm256_mul_ps(ld8(g + i), gs);
    __m256 pv = _mm256_mul_ps(ld8(p + i), decay);
    __m256 mv = ld8(m + i);
    __m256 vv = ld8(v + i);
    mv = _mm256_fmadd_ps(_mm256_sub_ps(gv, mv), c1, mv);
    vv = _mm256_fmadd_ps(vv, b2, _mm256_mul_ps(_mm256_mul_ps(c2, gv), gv));
    const __m256 den = _mm256_add_ps(_mm256_div_ps(_mm256_sqrt_ps(vv), bc2s), eps);
    pv = _mm256_sub_ps(pv, _mm256_div_ps(_mm256_mul_ps(step, mv), den));
    st8(p + i, pv);
    st8(m + i, mv);
    st8(v + i, vv);
  }
  adam_range_scalar(p, g, m, v, i, hi, k);
}

// ----------------------------------------------------------------------------- dispatch
enum class Isa { kScalar = 0, kAvx2 = 1, kAvx512 = 2 };

inline Isa detect_isa() {
  Isa best = Isa::kScalar;
#if defined(__x86_64__)
  __builtin_cpu_init();
  if (__builtin_cpu_supports("avx512f")) best = Isa::kAvx512;
  else if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) best = Isa::kAvx2;
#endif
  if (const char* e = std::getenv("DTG_HOST_ADAMW_ISA")) {
    Isa want = best;
    if (!std::strcmp(e, "scalar")) want = Isa::kScalar;
    else if (!std::strcmp(e, "avx2")) want = Isa::kAvx2;
    else if (!std::strcmp(e, "avx512")) want = Isa::kAvx512;
    if (static_cast<int>(want) <= static_cast<int>(best)) best = want;  // never above the CPU
  }
  return best;
}

// Re-read per call so tests can switch paths inside one process.
inline Isa host_isa() { return detect_isa(); }

template <typename PT, typename GT, typename ST>
void adamw_host(PT* p, const GT* g, ST* m, ST* v, int64_t n, float lr, float b1, float b2, float eps, float wd,
                float bc1, float bc2s, float gs) {
  const AdamConsts k = make_consts(lr, b1, b2, eps, wd, bc1, bc2s, gs);
  const Isa isa = host_isa();
  constexpr int64_t kGrain = 64;  // thread ranges start on 64-element (128-B bf16) boundaries
#pragma omp parallel
  {
#ifdef _OPENMP
    const int64_t nt = omp_get_num_threads(), t = omp_get_thread_num();
#else
    const int64_t nt = 1, t = 0;
#endif
    const int64_t units = (n + kGrain - 1) / kGrain;
    const int64_t lo = std::min(n, (units * t / nt) * kGrain);
    const int64_t hi = std::min(n, (units * (t + 1) / nt) * kGrain);
    if (lo < hi) {
      if (isa == Isa::kAvx512) adam_range_avx512(p, g, m, v, lo, hi, k);
      else if (isa == Isa::kAvx2) adam_range_avx2(p, g, m, v, lo, hi, k);
      else adam_range_scalar(p, g, m, v, lo, hi, k);
    }
  }
}

}  // namespace host
}  // namespace dtg
