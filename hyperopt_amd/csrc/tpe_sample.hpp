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
  const uint2* gd;      // staged: guide entry of bucket b (see stage_mix)
  const float2* ms32;   // staged: (mu, sigma) in fp32
  int n;
};

struct MixLds {  // LDS image of a below mixture of <= kStage components
  double cdf[kStage], mu[kStage], sg[kStage];
  uint32_t thr[kStage];
  float2 ms32[kStage];
  uint2 gd[kGuide];
};

// stage the below mixture for sampling; returns the view (call by all threads).
// thr[k] = ceil(cdf[k] / cdf[n-1] * 2^32): a 32-bit word w selects the first k
// with w < thr[k] -- the same component as cdf[k] > w * 2^-32 * cdf[n-1].
// Guide table (Chen & Asau) over buckets b = w >> 24: g = the first k with
// thr[k] > b * 2^24 is the smallest component a word of the bucket can take.
// Entry gd[b] = {thr[g], g | step << 8 | multi << 9}: step = (g < n-1), and
// the component is g + step * (w >= thr[g]) unless a second threshold falls
// inside the bucket (multi), where the walk over thr[] finishes the search.
__device__ __forceinline__ Mix stage_mix(const tpe_seg& S, const double* wcdf, const double* mu,
                                         const double* sigma, MixLds& L) {
  const int n = S.n_obs + 1;
  if (n > kStage)
    return Mix{wcdf + S.comp_off, mu + S.comp_off, sigma + S.comp_off, nullptr, nullptr,
               nullptr, n};
  const double total = wcdf[S.comp_off + n - 1];
  for (int k = threadIdx.x; k < n; k += kBS) {
    const double c = wcdf[S.comp_off + k], m = mu[S.comp_off + k], g = sigma[S.comp_off + k];
    L.cdf[k] = c;
    L.mu[k] = m;
    L.sg[k] = g;
    L.ms32[k] = make_float2((float)m, (float)g);
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
    const uint32_t top = w | 0xFFFFFFu;  // largest word of the bucket
    const uint32_t step = lo < n - 1 ? 1u : 0u;
    const uint32_t multi = (lo + 1 < n - 1 && L.thr[lo + 1] <= top) ? 1u : 0u;
    L.gd[b] = make_uint2(L.thr[lo], (uint32_t)lo | step << 8 | multi << 9);
  }
  __syncthreads();
  return Mix{L.cdf, L.mu, L.sg, L.thr, L.gd, L.ms32, n};
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
  if (M.thr) {  // block-uniform: staged mixture, one guide entry (+ rare walk)
    const uint2 e = M.gd[word >> 24];
    int k = (int)(e.y & 0xFFu) + ((word >= e.x) ? (int)((e.y >> 8) & 1u) : 0);
    if (e.y & 0x200u)
      while (k < M.n - 1 && word >= M.thr[k]) ++k;
    return k;
  }
  const double u = (double)word * 0x1.0p-32 * M.cdf[M.n - 1];
  return upper_bound(M.cdf, M.n, u);
}
__device__ __forceinline__ float2 ms32_of(const Mix& M, int j) {  // (mu, sigma)
  return M.ms32 ? M.ms32[j] : make_float2((float)M.mu[j], (float)M.sg[j]);
}

__device__ __forceinline__ void attempt32_pair(const Mix& M, uint64_t key, int64_t m, uint32_t a,
                                               float& y0, float& y1) {
#ifdef TPE_DIAG_NO_PHILOX  // diagnostic builds only (tools/diag_variants.sh)
  const uint32_t hsh = (uint32_t)m * 0x9E3779B9u ^ a * 0x85EBCA6Bu ^ (uint32_t)key;
  const U4 r{hsh, hsh * 0xC2B2AE35u, hsh ^ 0x27D4EB2Fu, hsh * 0x165667B1u};
#else
  const U4 r = draw_words(key, m, a, kStreamSample);
#endif
#ifdef TPE_DIAG_NO_COMP
  const int j0 = (int)(r.x & 7), j1 = (int)(r.w & 7);
#else
  const int j0 = comp_of(M, r.x), j1 = comp_of(M, r.w);
#endif
  float z0, z1;
#ifdef TPE_DIAG_NO_BM
  z0 = (float)(int)r.y * 0x1.0p-31f;
  z1 = (float)(int)r.z * 0x1.0p-31f;
#else
  normal_pair_f32(r.y, r.z, z0, z1);
#endif
  const float2 c0 = ms32_of(M, j0), c1 = ms32_of(M, j1);
  y0 = fmaf(c0.y, z0, c0.x);
  y1 = fmaf(c1.y, z1, c1.x);
}

// attempt `a` of candidate `g` alone (same value as attempt32_pair's half)
__device__ __forceinline__ float attempt32(const Mix& M, uint64_t key, int64_t g, uint32_t a) {
  const U4 r = draw_words(key, g >> 1, a, kStreamSample);
  const int j = comp_of(M, (g & 1) ? r.w : r.x);
  const float u1 = 1.0f - u01_f32(r.y);
  const float u2 = (float)(r.z >> 8) * 0x1.0p-24f;
  const float rr = __builtin_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
  const float z = rr * ((g & 1) ? __builtin_amdgcn_sinf(u2) : __builtin_amdgcn_cosf(u2));
  const float2 c = ms32_of(M, j);
  return fmaf(c.y, z, c.x);
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

// R consecutive candidates g0 .. g0+R-1 per thread, n of them valid, each
// exactly as draw32 draws it (to_x: LGMM1 values as exp(y), as draw32's
// callers store them; otherwise the mixture coordinate y).
// Attempt 0 of every pair is drawn unrolled into registers (one Philox call
// serves both candidates of a pair).  An odd g0 (a shard that starts inside a
// pair -- g0 is cand_base + an even offset, so the test is job-uniform)
// draws attempt 0 of each candidate alone instead: same values, since
// attempt32(g) is the half of attempt32_pair(g >> 1) that g owns.  Bounded
// labels then retry their
// rejected candidates one at a time, each lane walking its own queue (a
// rejection costs that lane one more step instead of stalling the wave for a
// whole draw); the retried values come back through `wstage`, the calling
// wave's own R*64 floats of LDS (slot r of lane l at r*64 + l).
template <int R>
__device__ __forceinline__ void draw32_pairs(const Mix& M, uint64_t key, int64_t g0, int n,
                                             bool lo_on, bool hi_on, float lo, float hi,
                                             bool to_x, float* wstage, float (&x)[R]) {
  static_assert(R % 2 == 0 && R <= 32, "pairs, one mask bit per candidate");
  // pair m = (g0 >> 1) + p holds candidates 2m (cos half) and 2m+1 (sin
  // half).  Aligned: x[2p], x[2p+1] = pair p.  Odd g0: x[2p] is pair p's
  // sin half and x[2p-1] pair p's cos half; x[R-1] needs one more pair.
  // Selects, not a second unrolled draw loop: the register footprint (and
  // so the occupancy of the scorer) stays that of the aligned loop.
  const bool odd = (g0 & 1) != 0;
#pragma unroll
  for (int p = 0; p < R / 2; ++p) {
    float c, s;
    attempt32_pair(M, key, (g0 >> 1) + p, 0u, c, s);
    x[2 * p] = odd ? s : c;
    x[2 * p + 1] = s;  // odd: replaced by the next pair's cos half
    if (p > 0 && odd) x[2 * p - 1] = c;
  }
  if (odd) {
    float c, s;
    attempt32_pair(M, key, (g0 >> 1) + R / 2, 0u, c, s);
    x[R - 1] = c;
  }
  uint32_t rej = 0;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (!accept32(x[r], lo_on, hi_on, lo, hi)) rej |= 1u << r;
  rej &= n >= R ? ~0u : (n <= 0 ? 0u : (1u << n) - 1u);
#ifdef TPE_DIAG_NO_RETRY  // diagnostic builds only: rejected draws clamped, no retries
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (rej & (1u << r)) x[r] = clamp32(x[r], lo_on, hi_on, lo, hi);
  rej = 0;
#endif
  if (__any(rej != 0)) {
    float* st = wstage + lane_id();
    uint32_t todo = rej, att = 1;
    while (__any(todo != 0)) {
      if (todo) {
        const int r = __builtin_ctz(todo);
        float y = attempt32(M, key, g0 + r, att);
        const bool ok = accept32(y, lo_on, hi_on, lo, hi);
        if (ok || att + 1 >= kMaxAttempts) {
          if (!ok) y = clamp32(y, lo_on, hi_on, lo, hi);
          st[r * kWave] = y;
          todo &= todo - 1;
          att = 1;
        } else {
          ++att;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (rej & (1u << r)) x[r] = st[r * kWave];
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (to_x) x[r] = __expf(x[r]);
    if (r >= n) x[r] = 1.0f;
  }
}

}  // namespace
}  // namespace tpe
