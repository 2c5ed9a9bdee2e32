// tpe_sample.hpp -- candidate sampling shared by the scoring kernels.
//
// GMM1 / LGMM1 draws (hyperopt/tpe.py:79-106, 229-257): component by inverse
// CDF of the below mixture's weights, then N(mu, sigma) by Box-Muller, with
// the reference's acceptance test low <= y < high.  Draw `a` of candidate `g`
// is Philox4x32-10 at counter (g, a, "SAMP") under the label key, so every
// kernel that draws candidate g sees the same value.
#pragma once

#include "tpe_common.hpp"

namespace tpe {
namespace {
constexpr int kBS = 256;       // block size of the candidate kernels
constexpr int kStage = 64;     // below-mixture components staged in LDS for sampling
constexpr uint32_t kMaxAttempts = 256;
constexpr uint32_t kStreamSample = 0x53414D50u;  // "SAMP"

__device__ __forceinline__ tpe_best empty_best() { return tpe_best{0.0, -1, 0.0, 0}; }

// first j with cdf[j] > u  (numpy multinomial / inverse CDF)
__device__ __forceinline__ int upper_bound(const double* cdf, int n, double u) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cdf[mid] > u) hi = mid; else lo = mid + 1;
  }
  return lo;
}

struct Mix {  // sampler view of the below mixture (LDS or global)
  const double* cdf;
  const double* mu;
  const double* sg;
  int n;
};

// stage the below mixture for sampling; returns the view (call by all threads)
__device__ __forceinline__ Mix stage_mix(const tpe_seg& S, const double* wcdf, const double* mu,
                                         const double* sigma, double* s_cdf, double* s_mu,
                                         double* s_sg) {
  const int n = S.n_obs + 1;
  if (n > kStage) return Mix{wcdf + S.comp_off, mu + S.comp_off, sigma + S.comp_off, n};
  for (int k = threadIdx.x; k < n; k += kBS) {
    s_cdf[k] = wcdf[S.comp_off + k];
    s_mu[k] = mu[S.comp_off + k];
    s_sg[k] = sigma[S.comp_off + k];
  }
  __syncthreads();
  return Mix{s_cdf, s_mu, s_sg, n};
}

// One draw from the (possibly truncated) below mixture: returns the value in
// the mixture's own space (x for GMM1, log x for LGMM1).  Same accepted
// distribution as the reference's rejection loop (component ~ w, then
// N(mu, sigma), accept low <= y < high).
__device__ __forceinline__ double draw64(const Mix& M, uint64_t key, int64_t g, bool lo_on,
                                         bool hi_on, double lo, double hi) {
  double y = 0.0;
  for (uint32_t a = 0; a < kMaxAttempts; ++a) {
    const U4 r = draw_words(key, g, a, kStreamSample);
    const double u = (double)r.x * 0x1.0p-32 * M.cdf[M.n - 1];
    const int j = upper_bound(M.cdf, M.n, u);
    y = M.mu[j] + M.sg[j] * normal_f64(r.y, r.z, r.w);
    if ((!lo_on || lo <= y) && (!hi_on || y < hi)) return y;
  }
  // acceptance below ~1e-77: keep the last draw, clamped into the support
  if (lo_on && y < lo) y = lo;
  if (hi_on && !(y < hi)) y = nextafter(hi, -INFINITY);
  return y;
}

__device__ __forceinline__ float draw32(const Mix& M, uint64_t key, int64_t g, bool lo_on,
                                        bool hi_on, float lo, float hi) {
  float y = 0.0f;
  for (uint32_t a = 0; a < kMaxAttempts; ++a) {
    const U4 r = draw_words(key, g, a, kStreamSample);
    const double u = (double)r.x * 0x1.0p-32 * M.cdf[M.n - 1];
    const int j = upper_bound(M.cdf, M.n, u);
    y = (float)M.mu[j] + (float)M.sg[j] * normal_f32(r.y, r.z);
    if ((!lo_on || lo <= y) && (!hi_on || y < hi)) return y;
  }
  if (lo_on && y < lo) y = lo;
  if (hi_on && !(y < hi)) y = nextafterf(hi, -INFINITY);
  return y;
}

}  // namespace
}  // namespace tpe
