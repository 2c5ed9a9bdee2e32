// tpe_sample.hpp -- candidate sampling shared by the scoring kernels.
//
// GMM1 / LGMM1 draws (hyperopt/tpe.py:79-106, 229-257): component by inverse
// CDF of the below mixture's weights, then N(mu, sigma) by Box-Muller, with
// the reference's acceptance test low <= y < high.  Every draw is a function
// of (label key, global candidate index, attempt) through Philox4x32-10, so
// every kernel that draws candidate g sees the same value; the fp64 and fp32
// streams differ (draw64 / attempt32_*).
#pragma once

#include "tpe_common.hpp"

namespace tpe {
namespace {
constexpr int kBS = 256;       // block size of the candidate kernels
constexpr int kStage = 64;     // below-mixture components staged in LDS for sampling
constexpr uint32_t kMaxAttempts = 256;
constexpr uint32_t kStreamSample = 0x53414D50u;  // "SAMP"
constexpr uint32_t kStreamRetry = 0x52455452u;   // "RETR": fp32 retries
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
  const float4* cw;     // staged: {mu, sigma, bits of thr[k-1], 1 / (thr[k] - thr[k-1])}
  int n;
};

struct MixLds {  // LDS image of a below mixture of <= kStage components
  double cdf[kStage], mu[kStage], sg[kStage];
  uint32_t thr[kStage];
  float4 cw[kStage];
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
// cw[k] also carries the end thr[k] and inverse width of component k's word
// interval [thr[k-1], thr[k]) so the fp32 sampler can read the word's
// position inside it (comp_res).
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
  for (int k = threadIdx.x; k < n; k += kBS) {
    const uint32_t lo = k ? L.thr[k - 1] : 0u, width = L.thr[k] - lo;
    L.cw[k] = make_float4((float)L.mu[k], (float)L.sg[k], __uint_as_float(L.thr[k]),
                          width ? 1.0f / (float)width : 0.0f);
  }
  __syncthreads();
  return Mix{L.cdf, L.mu, L.sg, L.thr, L.gd, L.cw, n};
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

// fp32 draws.  Attempt 0 of candidates 4m .. 4m+3 is ONE Philox call at
// counter (m, 0): word k picks candidate 4m+k's component by inverse CDF, and
// the word's position inside that component's interval -- a uniform of its
// own, independent of which component it picked -- feeds Box-Muller: the
// residuals of words 0 / 1 give radius / angle of the pair (4m, 4m+1) (cos ->
// 4m, sin -> 4m+1), words 2 / 3 those of (4m+2, 4m+3).  Four candidates per
// call, so the sampler spends half as many Philox rounds (quarter-rate
// v_mad_u64_u32) per candidate as a pair-per-call scheme.  Retries (bounded
// labels) take two attempts per call at counter (g, c) in a stream of their
// own (retry32).  Candidate g's value depends on g alone, whichever kernel
// draws it.
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

// component (mu, sigma) of `word` and the word's upper residual t in (0, 1]:
// the distance from the word to the top of its component's interval, over the
// interval's width -- uniform on the interval's grid whatever the component,
// and never 0, so Box-Muller takes log(t) directly (no 1 - u, no clamp).
// The staged test is per word on purpose: splitting the samplers into staged
// and global instantiations lets the scheduler hoist the four words' LDS
// reads and costs ~35 VGPRs, which lost more (occupancy) than the branches.
__device__ __forceinline__ void comp_res(const Mix& M, uint32_t word, float& mu, float& sg,
                                         float& res) {
#ifdef TPE_DIAG_NO_COMP  // diagnostic builds only (tools/diag_variants.sh)
  const float4 c = M.cw ? M.cw[word & 7] : make_float4(0.0f, 1.0f, 0.0f, 0x1.0p-32f);
  mu = c.x;
  sg = c.y;
  res = (float)(~word) * 0x1.0p-32f + 0x1.0p-32f;
#else
  if (M.cw) {
    const float4 c = M.cw[comp_of(M, word)];
    mu = c.x;
    sg = c.y;
    res = (float)(__float_as_uint(c.z) - word) * c.w;  // c.z: the interval's end
  } else {
    const double total = M.cdf[M.n - 1];
    const double u = (double)word * 0x1.0p-32 * total;
    const int k = upper_bound(M.cdf, M.n, u);
    const double lo = k ? M.cdf[k - 1] : 0.0, wk = M.cdf[k] - lo;
    res = wk > 0.0 ? (float)((M.cdf[k] - u) / wk) : 1.0f;
    mu = (float)M.mu[k];
    sg = (float)M.sg[k];
  }
#endif
}

// Box-Muller pair from two upper residuals: radius from ta (clamped to
// >= 2^-24, so the radius stays < 5.77), angle from tb (in turns)
__device__ __forceinline__ void bm_pair(float ta, float tb, float& z0, float& z1) {
#ifdef TPE_DIAG_NO_BM
  z0 = ta - 0.5f;
  z1 = tb - 0.5f;
#else
  // v_sqrt_f32 (1 ulp) without the correctly-rounded expansion: the argument
  // is 0 or a normal number in [2.4e-7, 33.3]
  const float r =
      __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(fmaxf(ta, 0x1.0p-24f)));
  z0 = r * __builtin_amdgcn_cosf(tb);
  z1 = r * __builtin_amdgcn_sinf(tb);
#endif
}

__device__ __forceinline__ U4 quad_words(uint64_t key, int64_t m) {
#ifdef TPE_DIAG_NO_PHILOX  // diagnostic builds only
  const uint32_t hsh = (uint32_t)m * 0x9E3779B9u ^ (uint32_t)key;
  return U4{hsh, hsh * 0xC2B2AE35u, hsh ^ 0x27D4EB2Fu, hsh * 0x165667B1u};
#else
  return draw_words(key, m, 0u, kStreamSample);
#endif
}

// attempt 0 of candidates 4m .. 4m+3
__device__ __forceinline__ void attempt32_quad(const Mix& M, uint64_t key, int64_t m, float& y0,
                                               float& y1, float& y2, float& y3) {
  const U4 r = quad_words(key, m);
  float mu0, sg0, r0, mu1, sg1, r1, mu2, sg2, r2, mu3, sg3, r3;
  comp_res(M, r.x, mu0, sg0, r0);
  comp_res(M, r.y, mu1, sg1, r1);
  comp_res(M, r.z, mu2, sg2, r2);
  comp_res(M, r.w, mu3, sg3, r3);
  float z0, z1, z2, z3;
  bm_pair(r0, r1, z0, z1);
  bm_pair(r2, r3, z2, z3);
  y0 = fmaf(sg0, z0, mu0);
  y1 = fmaf(sg1, z1, mu1);
  y2 = fmaf(sg2, z2, mu2);
  y3 = fmaf(sg3, z3, mu3);
}

// attempt 0 of candidate g alone (its share of attempt32_quad at m = g >> 2)
__device__ __forceinline__ float attempt32_first(const Mix& M, uint64_t key, int64_t g) {
  const U4 r = quad_words(key, g >> 2);
  const bool hi_pair = (g & 2) != 0, second = (g & 1) != 0;
  float mua, sga, ra, mub, sgb, rb;
  comp_res(M, hi_pair ? r.z : r.x, mua, sga, ra);
  comp_res(M, hi_pair ? r.w : r.y, mub, sgb, rb);
  float z0, z1;
  bm_pair(ra, rb, z0, z1);
  return second ? fmaf(sgb, z1, mub) : fmaf(sga, z0, mua);
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

// Retries of candidate g (bounded labels, attempt 0 rejected): call c >= 1
// of the retry stream, at counter (g, c), gives attempts 2c-1 and 2c -- words
// 0 / 1 pick their components, the two words' residuals are the Box-Muller
// pair's radius / angle -- and the first accepted one is the draw.  Two
// attempts per call: at C3's ~7% rejection a rejected candidate needs a
// second call 0.5% of the time, and a wave's retry pass costs one Philox,
// two component lookups and one Box-Muller pair instead of four lookups and
// two pairs.  After kMaxRetryCalls calls (acceptance below ~1e-77) the last
// attempt is clamped.
constexpr uint32_t kMaxRetryCalls = kMaxAttempts / 2;

__device__ __forceinline__ float retry32(const Mix& M, uint64_t key, int64_t g, bool lo_on,
                                         bool hi_on, float lo, float hi) {
  float y = 0.0f;
  for (uint32_t c = 1; c <= kMaxRetryCalls; ++c) {
    const U4 r = draw_words(key, g, c, kStreamRetry);
    float mu0, sg0, r0, mu1, sg1, r1;
    comp_res(M, r.x, mu0, sg0, r0);
    comp_res(M, r.y, mu1, sg1, r1);
    float z0, z1;
    bm_pair(r0, r1, z0, z1);
    const float y0 = fmaf(sg0, z0, mu0), y1 = fmaf(sg1, z1, mu1);
    const bool a0 = accept32(y0, lo_on, hi_on, lo, hi);
    y = a0 ? y0 : y1;
    if (a0 || accept32(y1, lo_on, hi_on, lo, hi)) return y;
  }
  return clamp32(y, lo_on, hi_on, lo, hi);
}

__device__ __forceinline__ float draw32(const Mix& M, uint64_t key, int64_t g, bool lo_on,
                                        bool hi_on, float lo, float hi) {
  const float y = attempt32_first(M, key, g);
  if (accept32(y, lo_on, hi_on, lo, hi)) return y;
  return retry32(M, key, g, lo_on, hi_on, lo, hi);
}

// R consecutive candidates g0 .. g0+R-1 per thread, n of them valid, each
// exactly as draw32 draws it (to_x: LGMM1 values as exp(y), as draw32's
// callers store them; otherwise the mixture coordinate y).  Attempt 0 is
// drawn unrolled into registers, one Philox call per four candidates.  A
// start inside a call (g0 not a multiple of 4 -- only at a shard boundary;
// g0 is cand_base + a multiple of R, so the test is job-uniform) draws
// attempt 0 one candidate at a time in a rolled loop through `wstage`, which
// keeps the register footprint of the aligned loop.
// Bounded labels then retry their rejected candidates (retry32, as draw32).
// ~7% of C3's bounded draws are rejected, so a wave holds ~70 of them but its
// busiest lane ~4: the wave's rejections are listed in `wlist` (kRetryList
// entries per wave, a prefix sum of the lanes' counts places them) and worked
// off 64 at a time, one per lane, so the wave waits ~2 retry calls instead of
// its busiest lane's ~4; rejections past the list (a rare wave) retry in
// their own lane.  Retried values come back
// through `wstage`, the wave's R*64 floats of LDS (slot r of lane l at
// r*64 + l).
constexpr int kRetryList = 256;  // listed rejections per wave (uint16 entries)

template <int R>
__device__ __forceinline__ void draw32_pairs(const Mix& M, uint64_t key, int64_t g0, int n,
                                             bool lo_on, bool hi_on, float lo, float hi,
                                             bool to_x, float* wstage, uint16_t* wlist,
                                             float (&x)[R]) {
  static_assert(R % 4 == 0 && R <= 32, "quads, one mask bit per candidate");
  const int lane = lane_id();
  float* st = wstage + lane;
  if ((g0 & 3) == 0) {
#pragma unroll
    for (int q = 0; q < R / 4; ++q)
      attempt32_quad(M, key, (g0 >> 2) + q, x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
  } else {
#pragma unroll 1
    for (int r = 0; r < R; ++r) st[r * kWave] = attempt32_first(M, key, g0 + r);
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = st[r * kWave];
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
  auto retry = [&](int64_t g) __attribute__((always_inline)) -> float {
    return retry32(M, key, g, lo_on, hi_on, lo, hi);
  };
  if (__any(rej != 0)) {
    // list the wave's rejections: exclusive prefix of the lanes' counts
    const int cnt = __popc(rej);
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const int o = __shfl_up(incl, off, kWave);
      if (lane >= off) incl += o;
    }
    const int total = min(__shfl(incl, kWave - 1, kWave), kRetryList);
    int pos = incl - cnt;
    uint32_t left = 0;  // this lane's rejections past the list
    for (uint32_t m = rej; m; m &= m - 1) {
      const int r = __builtin_ctz(m);
      if (pos < kRetryList)
        wlist[pos] = (uint16_t)((lane << 5) | r);
      else
        left |= 1u << r;
      ++pos;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int b = 0; b < total; b += kWave) {
      const int e = b + lane;
      const int ent = e < total ? (int)wlist[e] : 0;
      const int owner = ent >> 5, r = ent & 31;
      const int64_t go = __shfl(g0, owner, kWave);  // every lane takes part
      if (e < total) wstage[r * kWave + owner] = retry(go + r);
    }
    while (left) {
      const int r = __builtin_ctz(left);
      left &= left - 1;
      st[r * kWave] = retry(g0 + r);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
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

// ---------------------------------------------------------------------------
// Lean fp32 sampler (round 5): the same stream as attempt32_quad / draw32 /
// draw32_pairs -- bit for bit -- with the component lookup cut to one guide
// read, one compare and one select per word.  For below mixtures of at most
// kStage components (tpe.suggest's are at most 26: n_below <= the LF cap 25,
// tpe.py:633-636, plus the prior); the scorers keep the generic path for
// larger ones.  The guide entry of bucket b = w >> 24 is
//   {thr[g], byte offset of cw[g], byte offset of cw[g + step], multi}
// (g, step, multi as in stage_mix), so a word's component record is
// cw[w >= thr[g] ? g + step : g] -- no bit fields, no uniform flags in
// VGPRs; a bucket holding a second threshold (multi) walks thr[] as comp_of
// does, tested once per Philox call for its four words.
// ---------------------------------------------------------------------------
struct LeanMix {
  uint4 gd[kGuide];
  float4 cw[kStage];  // {mu, sigma, bits of thr[k], 1 / (thr[k] - thr[k-1])}, as MixLds::cw
  uint32_t thr[kStage];
};

// stage a below mixture of n <= kStage components (call by all threads)
__device__ __forceinline__ void stage_lean(const tpe_seg& S, const double* wcdf, const double* mu,
                                           const double* sigma, LeanMix& L) {
  const int n = S.n_obs + 1;
  const double total = wcdf[S.comp_off + n - 1];
  for (int k = threadIdx.x; k < n; k += kBS) {
    const double t = ceil(wcdf[S.comp_off + k] / total * 4294967296.0);
    L.thr[k] = (t >= 4294967295.0) ? 0xFFFFFFFFu : (t > 0.0 ? (uint32_t)t : 0u);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < n; k += kBS) {
    const uint32_t lo = k ? L.thr[k - 1] : 0u, width = L.thr[k] - lo;
    L.cw[k] = make_float4((float)mu[S.comp_off + k], (float)sigma[S.comp_off + k],
                          __uint_as_float(L.thr[k]), width ? 1.0f / (float)width : 0.0f);
  }
  for (int b = threadIdx.x; b < kGuide; b += kBS) {
    const uint32_t w = (uint32_t)b << 24;
    int lo = 0, hi = n - 1;  // first k with thr[k] > w (n-1 if none)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (w < L.thr[mid]) hi = mid; else lo = mid + 1;
    }
    const uint32_t top = w | 0xFFFFFFu;
    const int step = lo < n - 1 ? 1 : 0;
    const uint32_t multi = (lo + 1 < n - 1 && L.thr[lo + 1] <= top) ? 1u : 0u;
    L.gd[b] = make_uint4(L.thr[lo], (uint32_t)lo * 16u, (uint32_t)(lo + step) * 16u, multi);
  }
  __syncthreads();
}

__device__ __forceinline__ const float4& lean_cw(const LeanMix& L, uint32_t off) {
  return *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(L.cw) + off);
}
// the rare walk of a multi bucket (comp_of's), from the selected component
__device__ __forceinline__ uint32_t lean_walk(const LeanMix& L, int n, uint32_t w,
                                                        uint32_t off) {
  int k = (int)(off >> 4);
  while (k < n - 1 && w >= L.thr[k]) ++k;
  return (uint32_t)k << 4;
}
__device__ __forceinline__ uint32_t lean_sel(const uint4& e, uint32_t w) {
  return w >= e.x ? e.z : e.y;
}
// word -> (mu, sigma, upper residual), as comp_res
__device__ __forceinline__ void lean_res(const LeanMix& L, uint32_t off, uint32_t w, float& mu,
                                         float& sg, float& res) {
  const float4 c = lean_cw(L, off);
  mu = c.x;
  sg = c.y;
  res = (float)(__float_as_uint(c.z) - w) * c.w;
}

// attempt 0 of candidates 4m .. 4m+3 (attempt32_quad)
__device__ __forceinline__ void lean_quad(const LeanMix& L, int n, uint32_t k0, uint32_t k1,
                                          int64_t m, float& y0, float& y1, float& y2, float& y3) {
  const U4 r = philox(U4{(uint32_t)m, (uint32_t)((uint64_t)m >> 32), 0u, kStreamSample}, k0, k1);
  const uint4 e0 = L.gd[r.x >> 24], e1 = L.gd[r.y >> 24], e2 = L.gd[r.z >> 24],
              e3 = L.gd[r.w >> 24];
  uint32_t o0 = lean_sel(e0, r.x), o1 = lean_sel(e1, r.y), o2 = lean_sel(e2, r.z),
           o3 = lean_sel(e3, r.w);
  if (__builtin_expect((e0.w | e1.w | e2.w | e3.w) != 0u, 0)) {
    if (e0.w) o0 = lean_walk(L, n, r.x, o0);
    if (e1.w) o1 = lean_walk(L, n, r.y, o1);
    if (e2.w) o2 = lean_walk(L, n, r.z, o2);
    if (e3.w) o3 = lean_walk(L, n, r.w, o3);
  }
  float mu0, sg0, r0, mu1, sg1, r1, mu2, sg2, r2, mu3, sg3, r3;
  lean_res(L, o0, r.x, mu0, sg0, r0);
  lean_res(L, o1, r.y, mu1, sg1, r1);
  lean_res(L, o2, r.z, mu2, sg2, r2);
  lean_res(L, o3, r.w, mu3, sg3, r3);
  float z0, z1, z2, z3;
  bm_pair(r0, r1, z0, z1);
  bm_pair(r2, r3, z2, z3);
  y0 = fmaf(sg0, z0, mu0);
  y1 = fmaf(sg1, z1, mu1);
  y2 = fmaf(sg2, z2, mu2);
  y3 = fmaf(sg3, z3, mu3);
}

__device__ __forceinline__ uint32_t lean_comp(const LeanMix& L, int n, uint32_t w) {
  const uint4 e = L.gd[w >> 24];
  const uint32_t o = lean_sel(e, w);
  return e.w ? lean_walk(L, n, w, o) : o;
}

// attempt 0 of candidate g alone (attempt32_first)
__device__ __forceinline__ float lean_first(const LeanMix& L, int n, uint64_t key, int64_t g) {
  const U4 r = draw_words(key, g >> 2, 0u, kStreamSample);
  const bool hi_pair = (g & 2) != 0, second = (g & 1) != 0;
  const uint32_t wa = hi_pair ? r.z : r.x, wb = hi_pair ? r.w : r.y;
  float mua, sga, ra, mub, sgb, rb;
  lean_res(L, lean_comp(L, n, wa), wa, mua, sga, ra);
  lean_res(L, lean_comp(L, n, wb), wb, mub, sgb, rb);
  float z0, z1;
  bm_pair(ra, rb, z0, z1);
  return second ? fmaf(sgb, z1, mub) : fmaf(sga, z0, mua);
}

// retries of candidate g (retry32)
__device__ __forceinline__ float lean_retry(const LeanMix& L, int n, uint64_t key,
                                                      int64_t g, bool lo_on, bool hi_on, float lo,
                                                      float hi) {
  float y = 0.0f;
  for (uint32_t c = 1; c <= kMaxRetryCalls; ++c) {
    const U4 r = draw_words(key, g, c, kStreamRetry);
    float mu0, sg0, r0, mu1, sg1, r1;
    lean_res(L, lean_comp(L, n, r.x), r.x, mu0, sg0, r0);
    lean_res(L, lean_comp(L, n, r.y), r.y, mu1, sg1, r1);
    float z0, z1;
    bm_pair(r0, r1, z0, z1);
    const float y0 = fmaf(sg0, z0, mu0), y1 = fmaf(sg1, z1, mu1);
    const bool a0 = accept32(y0, lo_on, hi_on, lo, hi);
    y = a0 ? y0 : y1;
    if (a0 || accept32(y1, lo_on, hi_on, lo, hi)) return y;
  }
  return clamp32(y, lo_on, hi_on, lo, hi);
}

// candidate g exactly as draw32 draws it
__device__ __forceinline__ float lean_draw1(const LeanMix& L, int n, uint64_t key, int64_t g,
                                            bool lo_on, bool hi_on, float lo, float hi) {
  const float y = lean_first(L, n, key, g);
  if (accept32(y, lo_on, hi_on, lo, hi)) return y;
  return lean_retry(L, n, key, g, lo_on, hi_on, lo, hi);
}

// R consecutive candidates g0 .. per thread (draw32_pairs' stream, its retry
// list) into the wave's stage: candidate r of lane l at wstage[r * 64 + l]
// (the draws never sit in VGPRs: the scorer reads them back one at a time,
// which keeps it under 80 VGPRs without spills).  BOUNDED = false: a label
// without bounds (nothing is rejected).  Slots r >= n hold draws past the
// job's end (not candidates; never retried).
template <int R, bool BOUNDED>
__device__ __forceinline__ void lean_draw(const LeanMix& L, int nmix, uint64_t key, int64_t g0,
                                          int n, bool lo_on, bool hi_on, float lo, float hi,
                                          float* wstage, uint16_t* wlist) {
  static_assert(R % 4 == 0 && R <= 32, "quads, one mask bit per candidate");
  const int lane = lane_id();
  float* st = wstage + lane;
  const uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
  const float lo_e = lo_on ? lo : -INFINITY, hi_e = hi_on ? hi : INFINITY;
  uint32_t rej = 0;
  auto put = [&](int r, float y) __attribute__((always_inline)) {
    st[r * kWave] = y;  // (slots r >= n are drawn too and never read as candidates)
    if (BOUNDED) rej |= (lo_e <= y && y < hi_e) ? 0u : (1u << r);
  };
  if ((g0 & 3) == 0) {
#pragma unroll
    for (int q = 0; q < R / 4; ++q) {
      float y0, y1, y2, y3;
      lean_quad(L, nmix, k0, k1, (g0 >> 2) + q, y0, y1, y2, y3);
      put(4 * q, y0);
      put(4 * q + 1, y1);
      put(4 * q + 2, y2);
      put(4 * q + 3, y3);
    }
  } else {
#pragma unroll 1
    for (int r = 0; r < R; ++r) {
      const float y = lean_first(L, nmix, key, g0 + r);
      st[r * kWave] = y;
      if (BOUNDED && !(lo_e <= y && y < hi_e)) rej |= 1u << r;
    }
  }
  if (!BOUNDED) return;
  rej &= n >= R ? ~0u : (n <= 0 ? 0u : (1u << n) - 1u);
#ifdef TPE_DIAG_NO_RETRY  // diagnostic builds only: rejected draws clamped, no retries
  for (int r = 0; r < R; ++r)
    if (rej & (1u << r)) st[r * kWave] = clamp32(st[r * kWave], lo_on, hi_on, lo, hi);
  rej = 0;
#endif
  if (__any(rej != 0)) {
    // the wave's rejections listed and retried 64 at a time (draw32_pairs)
    const int cnt = __popc(rej);
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const int o = __shfl_up(incl, off, kWave);
      if (lane >= off) incl += o;
    }
    const int total = min(__shfl(incl, kWave - 1, kWave), kRetryList);
    int pos = incl - cnt;
    uint32_t left = 0;
    for (uint32_t m = rej; m; m &= m - 1) {
      const int r = __builtin_ctz(m);
      if (pos < kRetryList)
        wlist[pos] = (uint16_t)((lane << 5) | r);
      else
        left |= 1u << r;
      ++pos;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int b = 0; b < total; b += kWave) {
      const int e = b + lane;
      const int ent = e < total ? (int)wlist[e] : 0;
      const int owner = ent >> 5, r = ent & 31;
      const int64_t go = __shfl(g0, owner, kWave);
      if (e < total)
        wstage[r * kWave + owner] = lean_retry(L, nmix, key, go + r, lo_on, hi_on, lo, hi);
    }
    while (left) {
      const int r = __builtin_ctz(left);
      left &= left - 1;
      st[r * kWave] = lean_retry(L, nmix, key, g0 + r, lo_on, hi_on, lo, hi);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

}  // namespace
}  // namespace tpe
