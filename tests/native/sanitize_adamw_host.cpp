// Sanitizer harness for the host AdamW core (csrc/cpu/adamw_host.h), SURVEY §5.2.
// Built with -fsanitize=address,undefined -fopenmp by tests/test_native_sanitizers_cpu.py:
// out-of-bounds accesses in the 16-element blocking (odd tails), uninitialised reads and UB in
// the bf16 conversions abort the run.  Also checks the update against a double-precision
// scalar reference.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <vector>

#include "cpu/adamw_host.h"

using dtg::host::adamw_host;
using dtg::host::bf2f;
using dtg::host::f2bf;

static int check(int64_t n, int step) {
  // exact-size heap buffers so any read/write past n is an ASan error
  std::unique_ptr<float[]> p(new float[n]), m(new float[n]), v(new float[n]), g(new float[n]);
  std::unique_ptr<uint16_t[]> pb(new uint16_t[n]), gb(new uint16_t[n]), mb(new uint16_t[n]), vb(new uint16_t[n]);
  std::vector<double> rp(n), rm(n), rv(n);
  uint32_t seed = 12345u + (uint32_t)n;
  auto rnd = [&] { seed = seed * 1664525u + 1013904223u; return ((seed >> 8) & 0xffff) / 32768.0f - 1.0f; };
  for (int64_t i = 0; i < n; ++i) {
    p[i] = rnd();
    g[i] = rnd();
    m[i] = 0.1f * rnd();
    v[i] = 0.01f * std::fabs(rnd());
    pb[i] = f2bf(p[i]); gb[i] = f2bf(g[i]); mb[i] = f2bf(m[i]); vb[i] = f2bf(v[i]);
    rp[i] = p[i]; rm[i] = m[i]; rv[i] = v[i];
  }
  const float lr = 1e-3f, b1 = 0.9f, b2 = 0.999f, eps = 1e-8f, wd = 0.01f, gs = 0.5f;
  const double bc1 = 1.0 - std::pow((double)b1, step), bc2s = std::sqrt(1.0 - std::pow((double)b2, step));
  adamw_host<float, float, float>(p.get(), g.get(), m.get(), v.get(), n, lr, b1, b2, eps, wd, (float)bc1, (float)bc2s, gs);
  adamw_host<uint16_t, uint16_t, uint16_t>(pb.get(), gb.get(), mb.get(), vb.get(), n, lr, b1, b2, eps, wd,
                                           (float)bc1, (float)bc2s, gs);
  int bad = 0;
  for (int64_t i = 0; i < n; ++i) {
    const double gg = (double)g[i] * gs;
    rp[i] *= 1.0 - (double)lr * wd;
    rm[i] = rm[i] + (gg - rm[i]) * (1.0 - b1);
    rv[i] = rv[i] * b2 + (1.0 - b2) * gg * gg;
    rp[i] -= (lr / bc1) * rm[i] / (std::sqrt(rv[i]) / bc2s + eps);
    if (std::fabs(p[i] - rp[i]) > 1e-5 * (1 + std::fabs(rp[i]))) ++bad;
    if (std::fabs(bf2f(pb[i]) - rp[i]) > 2e-2 * (1 + std::fabs(rp[i]))) ++bad;
  }
  std::printf("n=%lld step=%d mismatches=%d\n", (long long)n, step, bad);
  return bad;
}

int main() {
  int bad = 0;
  for (int64_t n : {1LL, 15LL, 16LL, 17LL, 1000LL, 4097LL, 100003LL}) bad += check(n, n % 7 + 1);
  // NaN propagation through the bf16 conversion (quiet NaN, no UB)
  const uint16_t q = f2bf(std::nanf(""));
  if (!std::isnan(bf2f(q))) ++bad;
  std::printf(bad ? "FAIL\n" : "OK\n");
  return bad ? 1 : 0;
}
