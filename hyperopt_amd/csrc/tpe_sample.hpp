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
constexpr int kGuide = 256;    // guide-table buckets (top 8 bits of the word)

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
  const uint32_t* thr;  // staged: component k takes words < thr[k] (fp32 draws)
  const uint8_t* guide; // staged: first k with thr[k] > b * 2^24 for bucket b
  const float* mu32;
  const float* sg32;
  int n;
};

struct MixLds {  // LDS image of a below mixture of <= kStage components
  double cdf[kStage], mu[kStage], sg[kStage];
  uint32_t thr[kStage];
  float mu32[kStage], sg32[kStage];
  uint8_t guide[kGuide];
};

// stage the below mixture for sampling; returns the view (call by all threads).
// thr[k] = ceil(cdf[k] / cdf[n-1] * 2^32): a 32-bit word w selects the first k
// with w < thr[k] -- the same component as cdf[k] > w * 2^-32 * cdf[n-1].
// guide[b] (Chen & Asau guide table) is where that search starts for words of
// bucket b = w >> 24; most buckets hold no threshold, so the walk is one
// comparison.
__device__ __forceinline__ Mix stage_mix(const tpe_seg& S, const double* wcdf, const double* mu,
                                         const double* sigma, MixLds& L) {
  const int n = S.n_obs + 1;
  if (n > kStage)
    return Mix{wcdf + S.comp_off, mu + S.comp_off, sigma + S.comp_off, nullptr, nullptr,
               nullptr, nullptr, n};
  const double total = wcdf[S.comp_off + n - 1];
  for (int k = threadIdx.x; k < n; k += kBS) {
    const double c = wcdf[S.comp_off + k], m = mu[S.comp_off + k], g = sigma[S.comp_off + k];
    L.cdf[k] = c;
    L.mu[k] = m;
    L.sg[k] = g;
    L.mu32[k] = (float)m;
    L.sg32[k] = (float)g;
    const double t = ceil(c / total * 4294967296.0);
    L.thr[k] = (t >= 4294967295.0) ? 0xFFFFFFFFu : (t > 0.0 ? (uint32_t)t : 0u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kGuide; b += kBS) {
    const uint32_t w = (uint32_t)b << 24;
    int lo = 0, hi = n - 1;  // first k with thr[k] > w (n-1 if none)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (w < L.thr[mid]) hi = mid; else lo = mid + 1;
    }
    L.guide[b] = (uint8_t)lo;
  }
  __syncthreads();
  return Mix{L.cdf, L.mu, L.sg, L.thr, L.guide, L.mu32, L.sg32, n};
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

// fp32 draws come in pairs: attempt `a` of candidates 2m and 2m+1 is ONE
// Philox call at counter (m, a): word x picks 2m's component, word w picks
// 2m+1's, and (y, z) give the Box-Muller pair (cos -> 2m, sin -> 2m+1).
// Candidate g's value therefore depends on g alone, whichever kernel draws it.
__device__ __forceinline__ int comp_of(const Mix& M, uint32_t word) {
  if (M.thr) {  // block-uniform: staged mixture, guide table + 32-bit walk
    int k = M.guide[word >> 24];
    while (k < M.n - 1 && word >= M.thr[k]) ++k;
    return k;
  }
  const double u = (double)word * 0x1.0p-32 * M.cdf[M.n - 1];
  return upper_bound(M.cdf, M.n, u);
}
__device__ __forceinline__ float mu32_of(const Mix& M, int j) {
  return M.mu32 ? M.mu32[j] : (float)M.mu[j];
}
__device__ __forceinline__ float sg32_of(const Mix& M, int j) {
  return M.sg32 ? M.sg32[j] : (float)M.sg[j];
}

__device__ __forceinline__ void attempt32_pair(const Mix& M, uint64_t key, int64_t m, uint32_t a,
                                               float& y0, float& y1) {
  const U4 r = draw_words(key, m, a, kStreamSample);
  const int j0 = comp_of(M, r.x), j1 = comp_of(M, r.w);
  float z0, z1;
  normal_pair_f32(r.y, r.z, z0, z1);
  y0 = fmaf(sg32_of(M, j0), z0, mu32_of(M, j0));
  y1 = fmaf(sg32_of(M, j1), z1, mu32_of(M, j1));
}

// attempt `a` of candidate `g` alone (same value as attempt32_pair's half)
__device__ __forceinline__ float attempt32(const Mix& M, uint64_t key, int64_t g, uint32_t a) {
  const U4 r = draw_words(key, g >> 1, a, kStreamSample);
  const int j = comp_of(M, (g & 1) ? r.w : r.x);
  const float u1 = 1.0f - u01_f32(r.y);
  const float u2 = (float)(r.z >> 8) * 0x1.0p-24f;
  const float rr = __builtin_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
  const float z = rr * ((g & 1) ? __builtin_amdgcn_sinf(u2) : __builtin_amdgcn_cosf(u2));
  return fmaf(sg32_of(M, j), z, mu32_of(M, j));
}

__device__ __forceinline__ bool accept32(float y, bool lo_on, bool hi_on, float lo, float hi) {
  return (!lo_on || lo <= y) && (!hi_on || y < hi);
}

// after kMaxAttempts rejections (acceptance below ~1e-77): clamp into the support
__device__ __forceinline__ float clamp32(float y, bool lo_on, bool hi_on, float lo, float hi) {
  if (lo_on && y < lo) y = lo;
  if (hi_on && !(y < hi)) y = nextafterf(hi, -INFINITY);
  return y;
}

__device__ __forceinline__ float draw32(const Mix& M, uint64_t key, int64_t g, bool lo_on,
                                        bool hi_on, float lo, float hi) {
  float y = 0.0f;
  for (uint32_t a = 0; a < kMaxAttempts; ++a) {
    y = attempt32(M, key, g, a);
    if (accept32(y, lo_on, hi_on, lo, hi)) return y;
  }
  return clamp32(y, lo_on, hi_on, lo, hi);
}

// R consecutive candidates g0 .. g0+R-1 per thread (g0 even), n of them
// valid, each exactly as draw32 draws it (to_x: LGMM1 values as exp(y), as
// draw32's callers store them; otherwise the mixture coordinate y).  Every lane walks its own queue of
// candidate pairs: one Philox call per attempt serves both candidates of a
// pair, and a rejection costs that lane one more step instead of stalling the
// whole wave for a full draw.  Results go through `stage` (R*kBS floats of
// LDS; each thread reads back only its own slots).
template <int R>
__device__ __forceinline__ void draw32_pairs(const Mix& M, uint64_t key, int64_t g0, int n,
                                             bool lo_on, bool hi_on, float lo, float hi,
                                             bool to_x, float* stage, float (&x)[R]) {
  static_assert(R % 2 == 0, "pairs");
  const int tid = threadIdx.x;
  int p = 0;
  uint32_t att = 0;
  bool d0 = false, d1 = false;
  while (true) {
    const bool act = p < R / 2 && 2 * p < n;
    if (!__any(act)) break;
    if (act) {
      float y0, y1;
      attempt32_pair(M, key, (g0 >> 1) + p, att, y0, y1);
      const bool last = att + 1 >= kMaxAttempts;
      const bool has1 = 2 * p + 1 < n;
      if (!d0) {
        const bool ok = accept32(y0, lo_on, hi_on, lo, hi);
        if (ok || last) {
          if (!ok) y0 = clamp32(y0, lo_on, hi_on, lo, hi);
          stage[(2 * p) * kBS + tid] = to_x ? __expf(y0) : y0;
          d0 = true;
        }
      }
      if (has1 && !d1) {
        const bool ok = accept32(y1, lo_on, hi_on, lo, hi);
        if (ok || last) {
          if (!ok) y1 = clamp32(y1, lo_on, hi_on, lo, hi);
          stage[(2 * p + 1) * kBS + tid] = to_x ? __expf(y1) : y1;
          d1 = true;
        }
      }
      if (d0 && (d1 || !has1)) {
        ++p;
        att = 0;
        d0 = d1 = false;
      } else {
        ++att;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < R; ++k) x[k] = (k < n) ? stage[k * kBS + tid] : 1.0f;
}

}  // namespace
}  // namespace tpe
