// Torch-independent core of the host AdamW (csrc/cpu/adamw_cpu.cpp): bf16 <-> f32 conversions
// and the OpenMP update loop over raw pointers.  Kept in a header so the same code is also
// compiled into the sanitizer harness (tests/native/sanitize_adamw_host.cpp, built with
// -fsanitize=address,undefined and run by tests/test_native_sanitizers_cpu.py).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>

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

template <typename PT, typename GT, typename ST>
void adamw_host(PT* p, const GT* g, ST* m, ST* v, int64_t n, float lr, float b1, float b2, float eps, float wd,
                float bc1, float bc2s, float gs) {
  const float step_size = lr / bc1, decay = 1.f - lr * wd;
  constexpr int64_t BLK = 16;
  const int64_t nblk = (n + BLK - 1) / BLK;
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < nblk; ++b) {
    const int64_t s = b * BLK, e = std::min(n, s + BLK);
    float pv[BLK], gv[BLK], mv[BLK], vv[BLK];
    const int64_t cnt = e - s;
    for (int64_t j = 0; j < cnt; ++j) {
      pv[j] = ld<PT>(p, s + j);
      gv[j] = ld<GT>(g, s + j) * gs;
      mv[j] = ld<ST>(m, s + j);
      vv[j] = ld<ST>(v, s + j);
    }
#pragma omp simd
    for (int64_t j = 0; j < cnt; ++j) {
      pv[j] *= decay;
      mv[j] = mv[j] + (gv[j] - mv[j]) * (1.f - b1);
      vv[j] = vv[j] * b2 + (1.f - b2) * gv[j] * gv[j];
      pv[j] -= step_size * mv[j] / (std::sqrt(vv[j]) / bc2s + eps);
    }
    for (int64_t j = 0; j < cnt; ++j) {
      st<PT>(p, s + j, pv[j]);
      st<ST>(m, s + j, mv[j]);
      st<ST>(v, s + j, vv[j]);
    }
  }
}

}  // namespace host
}  // namespace dtg
