// tpe_fit.hip -- Parzen posterior fit and categorical pseudocount posteriors.
//
// Replaces hyperopt/tpe.py:399-467 (adaptive_parzen_normal), the observation
// transforms of the ap_*_sampler functions (tpe.py:484-572) and the
// categorical posteriors (tpe.py:578-615 with pyll/base.py:1053-1060).
//
// Layout (HBM): every label contributes two segments (below / above).  The
// observation pool is one fp64 array, segments index it by offset; the
// fitted mixtures land in SoA fp64 pools (w, mu, sigma, wcdf) plus two
// scoring-ready AoS coefficient pools (double4 / float4 per component) that
// the scoring kernels stream through LDS.
//
// Sort: the mixture is sorted by mean with ties kept in observation (tid)
// order -- a stable sort.  Each element's destination is its rank
// #{j : x_j < x_i or (x_j == x_i and j < i)}, counted over LDS tiles; the
// prior is inserted at searchsorted(x, prior_mu, 'left') (tpe.py:427), or by
// the len==1 rule of tpe.py:414-421.
#include <algorithm>
#include <stdarg.h>
#include <stdio.h>

#include "tpe_common.hpp"

namespace tpe {

namespace {
constexpr int kFitBS = 256;
constexpr int kRankTile = 2048;  // fp64 elements per LDS tile (16 KB)

__global__ __launch_bounds__(kFitBS) void k_fit_transform(const double* __restrict__ obs,
                                                          double* __restrict__ xf,
                                                          const tpe_seg* __restrict__ segs) {
  const tpe_seg& S = segs[blockIdx.y];
  const int64_t i = (int64_t)blockIdx.x * kFitBS + threadIdx.x;
  if (i >= S.n_obs) return;
  double v = obs[S.obs_off + i];
  if (S.transform == TPE_OBS_LOG) {
    // np.maximum(obs, floor) keeps NaN; floor=-inf means "no clamp"
    if (v < S.floor) v = S.floor;
    v = log(v);
  }
  xf[S.obs_off + i] = v;
}

__global__ __launch_bounds__(kFitBS) void k_fit_rank(const double* __restrict__ xf,
                                                     tpe_seg* __restrict__ segs,
                                                     double* __restrict__ w,
                                                     double* __restrict__ mu) {
  __shared__ double tile[kRankTile];
  __shared__ int red[kFitBS / kWave];
  tpe_seg* S = segs + blockIdx.y;
  const int n = S->n_obs;
  if ((int64_t)blockIdx.x * kFitBS >= (n > 0 ? n : 1)) return;  // block-uniform
  const int64_t ooff = S->obs_off, coff = S->comp_off;
  const double pmu = S->prior_mu;
  const int i = blockIdx.x * kFitBS + threadIdx.x;
  const double v = (i < n) ? xf[ooff + i] : 0.0;

  int rank = 0, below_prior = 0;
  for (int t0 = 0; t0 < n; t0 += kRankTile) {
    const int m = min(kRankTile, n - t0);
    __syncthreads();
    for (int j = threadIdx.x; j < m; j += kFitBS) tile[j] = xf[ooff + t0 + j];
    __syncthreads();
    for (int j = threadIdx.x; j < m; j += kFitBS) below_prior += tile[j] < pmu;
    if (i < n) {
      // tiles entirely before / after i need one comparison per element
      if (t0 + m <= i) {
        for (int j = 0; j < m; ++j) rank += tile[j] <= v;
      } else if (t0 > i) {
        for (int j = 0; j < m; ++j) rank += tile[j] < v;
      } else {
        for (int j = 0; j < m; ++j) {
          const double u = tile[j];
          rank += (u < v) | ((u == v) & (t0 + j < i));
        }
      }
    }
  }
  int prior_pos;
  if (n >= 2) {
    prior_pos = block_sum<kFitBS, int>(below_prior, red);
  } else if (n == 1) {
    prior_pos = (pmu < xf[ooff]) ? 0 : 1;  // tpe.py:414-421
  } else {
    prior_pos = 0;
  }
  if (i < n) {
    const int pos = rank + (rank >= prior_pos ? 1 : 0);
    mu[coff + pos] = v;
    w[coff + pos] = lf_weight(i, n, S->lf);  // ramp follows tid order (tpe.py:441-447)
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    mu[coff + prior_pos] = pmu;
    w[coff + prior_pos] = S->prior_weight;
    S->prior_pos = prior_pos;
  }
}

// bandwidths, clipping, normalisation, truncation mass and scoring coefficients
__global__ __launch_bounds__(kFitBS) void k_fit_finalize(tpe_seg* __restrict__ segs,
                                                         double* __restrict__ w,
                                                         const double* __restrict__ mu,
                                                         double* __restrict__ sigma,
                                                         double* __restrict__ wcdf,
                                                         double* __restrict__ coef64,
                                                         float* __restrict__ coef32,
                                                         float* __restrict__ coef32n,
                                                         float* __restrict__ wide32,
                                                         float* __restrict__ pm,
                                                         float* __restrict__ sm) {
  __shared__ double redd[kFitBS / kWave];
  tpe_seg* S = segs + blockIdx.x;
  const int n = S->n_obs, nc = n + 1, pos = S->prior_pos;
  const int64_t off = S->comp_off;
  const double ps = S->prior_sigma;
  const double lo_clip = ps / fmin(100.0, 1.0 + (double)nc);  // tpe.py:455
  const double hi_clip = ps / 1.0;

  // 1) weights: normalise (tpe.py:465)
  double part = 0.0;
  for (int k = threadIdx.x; k < nc; k += kFitBS) part += w[off + k];
  const double wsum = block_sum<kFitBS, double>(part, redd);
  for (int k = threadIdx.x; k < nc; k += kFitBS) w[off + k] = w[off + k] / wsum;

  // 2) bandwidths (tpe.py:410-439, 457-459)
  for (int k = threadIdx.x; k < nc; k += kFitBS) {
    double s;
    if (n == 0) {
      s = ps;
    } else if (n == 1) {
      s = (k == pos) ? ps : ps * 0.5;
    } else if (k == 0) {
      s = mu[off + 1] - mu[off];
    } else if (k == nc - 1) {
      s = mu[off + nc - 1] - mu[off + nc - 2];
    } else {
      s = fmax(mu[off + k] - mu[off + k - 1], mu[off + k + 1] - mu[off + k]);
    }
    s = fmin(fmax(s, lo_clip), hi_clip);
    if (k == pos) s = ps;
    sigma[off + k] = s;
  }
  __syncthreads();

  // 3) truncation mass p_accept (tpe.py:145-150)
  double pacc = 1.0;
  if (S->bounded) {
    double acc = 0.0;
    for (int k = threadIdx.x; k < nc; k += kFitBS) {
      const double m = mu[off + k], s = sigma[off + k];
      acc += w[off + k] * (normal_cdf(S->high, m, s) - normal_cdf(S->low, m, s));
    }
    pacc = block_sum<kFitBS, double>(acc, redd);
  }

  // 4) fp64 scoring coefficients {mu, 1/sigma', log-coef, w}
  //    GMM1 (tpe.py:152-158):  lc = log(w / sqrt(2 pi sigma^2) / p_accept)
  //    LGMM1 (tpe.py:284-287, 208-217): lc = log(w) - log(max(sigma,EPS) sqrt(2 pi));
  //    no p_accept (reference quirk)
  double lmax = -INFINITY;
  for (int k = threadIdx.x; k < nc; k += kFitBS) {
    const double m = mu[off + k], s = sigma[off + k], wk = w[off + k];
    double lc, inv;
    if (S->family == TPE_LGMM1) {
      const double sp = fmax(s, kEps);
      lc = log(wk) - log(sp * 2.5066282746310002);
      inv = 1.0 / sp;
    } else {
      const double z = sqrt(kTwoPi * (s * s));
      lc = log(wk / z / pacc);
      inv = 1.0 / fmax(s, kEps);
    }
    double* c = coef64 + 4 * (off + k);
    c[0] = m;
    c[1] = inv;
    c[2] = lc;
    c[3] = wk;
    lmax = fmax(lmax, lc * kLog2e);
  }
  const double cmax = block_max<kFitBS, double>(lmax, redd);

  // 5) fp32 coefficients in log2 units around a float-exact centre:
  //    t = xc*a + b,  v = c - t^2,  term = 2^v  (v <= 0, offset cmax)
  const double center = (double)(float)S->prior_mu;
  const double sq = 0.8493218002880191;  // sqrt(0.5 * log2(e))
  for (int k = threadIdx.x; k < nc; k += kFitBS) {
    const double* c = coef64 + 4 * (off + k);
    const double a = c[1] * sq;
    float* f = coef32 + 4 * (off + k);
    f[0] = (float)a;
    f[1] = (float)(-(c[0] - center) * a);
    f[2] = (float)(c[2] * kLog2e - cmax);
    f[3] = 0.0f;
  }

  // 6) cumulative weights for the sampler: each thread scans one contiguous
  //    chunk, thread 0 scans the chunk totals, chunks add their offset
  __shared__ double chunk_tot[kFitBS];
  const int per = (nc + kFitBS - 1) / kFitBS;
  const int k0 = threadIdx.x * per, k1 = min(nc, k0 + per);
  double run = 0.0;
  for (int k = k0; k < k1; ++k) {
    run += w[off + k];
    wcdf[off + k] = run;
  }
  chunk_tot[threadIdx.x] = run;
  __syncthreads();
  if (threadIdx.x == 0) {
    double acc = 0.0;
    for (int t = 0; t < kFitBS; ++t) {
      const double c = chunk_tot[t];
      chunk_tot[t] = acc;
      acc += c;
    }
    S->p_accept = pacc;
    S->cmax = cmax;
    S->center = center;
  }
  __syncthreads();
  const double base = chunk_tot[threadIdx.x];
  if (base != 0.0)
    for (int k = k0; k < k1; ++k) wcdf[off + k] += base;

  // 7) pruning data for the sorted fp32 path.  In log2 units relative to
  //    cmax, every candidate y of the support has log2(sum) >= v_prior(y) >=
  //    lglob (bounded: the prior term at the farther end of [low, high];
  //    unbounded: at 6 prior sigmas -- blocks beyond fall back to all
  //    components).  Component k's term is below 2^(lglob - 40), i.e.
  //    negligible at fp32 resolution even summed over 1e4 terms, once
  //    |y - mu_k| > r_k = sqrt(c_k - lglob + 40) / a_k.  Wide components (the
  //    prior and sigma >= prior_sigma/4) are always evaluated from a compact
  //    list; narrow ones through a [k_lo, k_hi] window found with the prefix
  //    max of mu + r (pm) and the suffix min of mu - r (sm).
  const double ap = coef64[4 * (off + pos) + 1] * sq;
  const double cp = coef64[4 * (off + pos) + 2] * kLog2e - cmax;
  double lglob;
  if (S->bounded) {
    const double dl = S->low - S->prior_mu, dh = S->high - S->prior_mu;
    lglob = cp - ap * ap * fmax(dl * dl, dh * dh);
  } else {
    lglob = cp - ap * ap * 36.0 * ps * ps;
  }
  const double thr = lglob - 40.0;
  for (int k = threadIdx.x; k < nc; k += kFitBS) {
    const float4 f = reinterpret_cast<const float4*>(coef32)[off + k];
    const bool wide = (k == pos) || (sigma[off + k] >= 0.25 * ps);
    float4 g = f;
    if (wide) g.z = -INFINITY;
    reinterpret_cast<float4*>(coef32n)[off + k] = g;
    const double m = mu[off + k];
    if (wide) {
      pm[off + k] = -INFINITY;
      sm[off + k] = INFINITY;
    } else {
      const double r = sqrt(fmax(f.z - thr, 0.0)) / (double)f.x * 1.001 + 1e-6 * fabs(m) + 1e-30;
      pm[off + k] = (float)(m + r);
      sm[off + k] = (float)(m - r);
    }
  }
  __syncthreads();
  __shared__ float chunk_f[kFitBS];
  __shared__ int chunk_n[kFitBS];
  // prefix max (pm), chunked
  float run_max = -INFINITY;
  int n_wide_local = 0;
  for (int k = k0; k < k1; ++k) {
    run_max = fmaxf(run_max, pm[off + k]);
    pm[off + k] = run_max;
    n_wide_local += (k == pos) || (sigma[off + k] >= 0.25 * ps);
  }
  chunk_f[threadIdx.x] = run_max;
  chunk_n[threadIdx.x] = n_wide_local;
  __syncthreads();
  if (threadIdx.x == 0) {
    float acc = -INFINITY;
    int nacc = 0;
    for (int t = 0; t < kFitBS; ++t) {
      const float c = chunk_f[t];
      chunk_f[t] = acc;
      acc = fmaxf(acc, c);
      const int cn = chunk_n[t];
      chunk_n[t] = nacc;
      nacc += cn;
    }
    S->lglob = lglob;
    S->n_wide = nacc;
  }
  __syncthreads();
  {
    const float before = chunk_f[threadIdx.x];
    for (int k = k0; k < k1; ++k) pm[off + k] = fmaxf(pm[off + k], before);
    int wpos = chunk_n[threadIdx.x];
    for (int k = k0; k < k1; ++k)
      if ((k == pos) || (sigma[off + k] >= 0.25 * ps))
        reinterpret_cast<float4*>(wide32)[off + (wpos++)] =
            reinterpret_cast<const float4*>(coef32)[off + k];
  }
  __syncthreads();
  // suffix min (sm), chunked
  float run_min = INFINITY;
  for (int k = k1 - 1; k >= k0; --k) {
    run_min = fminf(run_min, sm[off + k]);
    sm[off + k] = run_min;
  }
  chunk_f[threadIdx.x] = run_min;
  __syncthreads();
  if (threadIdx.x == 0) {
    float acc = INFINITY;
    for (int t = kFitBS - 1; t >= 0; --t) {
      const float c = chunk_f[t];
      chunk_f[t] = acc;
      acc = fminf(acc, c);
    }
  }
  __syncthreads();
  {
    const float after = chunk_f[threadIdx.x];
    for (int k = k0; k < k1; ++k) sm[off + k] = fminf(sm[off + k], after);
  }
}

// ---------------------------------------------------------------------------
// categorical posteriors
// ---------------------------------------------------------------------------
// numpy's pairwise_sum for float64 (n <= 8192: one buffer), so
// `pseudocounts / np.sum(pseudocounts)` is reproduced bit for bit.
__device__ double np_pw_leaf(const double* a, int64_t n) {
  if (n < 8) {
    double r = 0.0;
    for (int64_t i = 0; i < n; ++i) r += a[i];
    return r;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int64_t i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

__device__ double np_pairwise_sum(const double* a, int64_t n) {
  if (n <= 128) return np_pw_leaf(a, n);
  struct Frame {
    int64_t s, n;
    double left;
    int st;
  } stk[48];
  int sp = 0;
  stk[0] = Frame{0, n, 0.0, 0};
  double ret = 0.0;
  while (sp >= 0) {
    Frame& f = stk[sp];
    if (f.n <= 128) {
      ret = np_pw_leaf(a + f.s, f.n);
      --sp;
      continue;
    }
    int64_t n2 = f.n / 2;
    n2 -= n2 % 8;
    if (f.st == 0) {
      f.st = 1;
      stk[sp + 1] = Frame{f.s, n2, 0.0, 0};
      ++sp;
    } else if (f.st == 1) {
      f.left = ret;
      f.st = 2;
      stk[sp + 1] = Frame{f.s + n2, f.n - n2, 0.0, 0};
      ++sp;
    } else {
      ret = f.left + ret;
      --sp;
    }
  }
  return ret;
}

constexpr int kCatBS = 256;
constexpr int kCatWaves = kCatBS / kWave;

// Weighted counts, one wave per (segment, category): the wave scans the
// observations 64 at a time, ballots the matches, and adds their LF weights
// in observation order -- exactly np.bincount's sequential sum
// (pyll/base.py:1053-1060), but the dependent fp64 chain is only as long as
// the category's own count.
__global__ __launch_bounds__(kCatBS) void k_cat_counts(const int64_t* __restrict__ obs,
                                                       const tpe_cat_seg* __restrict__ segs,
                                                       double* __restrict__ p) {
  const tpe_cat_seg& S = segs[blockIdx.y];
  const int k = blockIdx.x * kCatWaves + threadIdx.x / kWave;
  if (k >= S.n_cat) return;  // wave-uniform
  const int n = S.n_obs, lane = lane_id();
  // linear-forgetting ramp (np.linspace(1/N, 1, N-LF), tpe.py:380-392)
  const bool ramp = S.lf > 0 && S.lf < n;
  const int64_t num = n - S.lf;
  const double start = 1.0 / (double)n;
  const double step = (ramp && num > 1) ? (1.0 - start) / (double)(num - 1) : 0.0;
  double cnt = 0.0;
  constexpr int kDepth = 8;  // tiles of 64 observations loaded per step
  for (int t0 = 0; t0 < n; t0 += kDepth * kWave) {
    int64_t cur[kDepth];
#pragma unroll
    for (int b = 0; b < kDepth; ++b) {
      const int i = t0 + b * kWave + lane;
      cur[b] = i < n ? obs[S.obs_off + i] : -1;
    }
#pragma unroll
    for (int b = 0; b < kDepth; ++b) {
      uint64_t m = __ballot(cur[b] == (int64_t)k);
      while (m) {  // wave-uniform, in observation order
        const int64_t i = t0 + b * kWave + __builtin_ctzll(m);
        m &= m - 1;
        double wt = 1.0;
        if (ramp && i < num) {
          if (num == 1) wt = start;
          else if (i == num - 1) wt = 1.0;
          else wt = __dadd_rn(__dmul_rn((double)i, step), start);
        }
        cnt = __dadd_rn(cnt, wt);
      }
    }
  }
  if (lane == 0) {
    double pseudo;
    if (S.mode == 0) {
      pseudo = cnt + S.prior_weight;  // tpe.py:589
    } else {
      const double pk = p[S.prior_p_off + k];
      pseudo = cnt + (double)S.n_cat * (S.prior_weight * pk);  // tpe.py:603
    }
    p[S.p_off + k] = pseudo;
  }
}

// normalise (numpy pairwise sum), log p (categorical_lpdf, tpe.py:60-73) and
// the cumulative p of the inverse-CDF sampler; one block per segment
__global__ __launch_bounds__(kCatBS) void k_cat_finalize(const tpe_cat_seg* __restrict__ segs,
                                                         double* __restrict__ p,
                                                         double* __restrict__ logp,
                                                         double* __restrict__ cdf) {
  const tpe_cat_seg& S = segs[blockIdx.x];
  const int K = S.n_cat;
  __shared__ double total;
  if (threadIdx.x == 0) total = np_pairwise_sum(p + S.p_off, K);
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += kCatBS) {
    const double pk = p[S.p_off + k] / total;
    p[S.p_off + k] = pk;
    logp[S.p_off + k] = log(pk);
  }
  __syncthreads();
  __shared__ double chunk_tot[kCatBS];
  const int per = (K + kCatBS - 1) / kCatBS;
  const int k0 = threadIdx.x * per, k1 = min(K, k0 + per);
  double run = 0.0;
  for (int k = k0; k < k1; ++k) {
    run += p[S.p_off + k];
    cdf[S.p_off + k] = run;
  }
  chunk_tot[threadIdx.x] = run;
  __syncthreads();
  if (threadIdx.x == 0) {
    double acc = 0.0;
    for (int t = 0; t < kCatBS; ++t) {
      const double c = chunk_tot[t];
      chunk_tot[t] = acc;
      acc += c;
    }
  }
  __syncthreads();
  const double base = chunk_tot[threadIdx.x];
  if (base != 0.0)
    for (int k = k0; k < k1; ++k) cdf[S.p_off + k] += base;
}
}  // namespace

}  // namespace tpe

using namespace tpe;

extern "C" int tpe_parzen_fit(const double* obs, double* xf, tpe_seg* segs, int n_seg,
                              int max_obs, double* w, double* mu, double* sigma, double* wcdf,
                              double* coef64, float* coef32, float* coef32n, float* wide32,
                              float* pm, float* sm, void* stream) {
  if (n_seg < 0 || max_obs < 0) {
    set_error("tpe_parzen_fit: n_seg=%d max_obs=%d", n_seg, max_obs);
    return TPE_E_ARG;
  }
  if (n_seg == 0) return TPE_OK;
  if (!segs || !w || !mu || !sigma || !wcdf || !coef64 || !coef32 || !coef32n || !wide32 ||
      !pm || !sm || (max_obs > 0 && (!obs || !xf))) {
    set_error("tpe_parzen_fit: null pointer");
    return TPE_E_ARG;
  }
  if (n_seg > 65535) {
    set_error("tpe_parzen_fit: n_seg %d > 65535", n_seg);
    return TPE_E_UNSUPPORTED;
  }
  hipStream_t st = (hipStream_t)stream;
  const int gx = (max(max_obs, 1) + kFitBS - 1) / kFitBS;
  if (max_obs > 0) {
    hipLaunchKernelGGL(k_fit_transform, dim3(gx, n_seg), dim3(kFitBS), 0, st, obs, xf, segs);
  }
  hipLaunchKernelGGL(k_fit_rank, dim3(gx, n_seg), dim3(kFitBS), 0, st, xf, segs, w, mu);
  hipLaunchKernelGGL(k_fit_finalize, dim3(n_seg), dim3(kFitBS), 0, st, segs, w, mu, sigma, wcdf,
                     coef64, coef32, coef32n, wide32, pm, sm);
  return check_launch("tpe_parzen_fit");
}

extern "C" int tpe_cat_posterior(const int64_t* obs, const tpe_cat_seg* segs, int n_seg,
                                 int max_cat, double* p_pool, double* logp_pool,
                                 double* cdf_pool, void* stream) {
  if (n_seg < 0 || (n_seg > 0 && (!segs || !p_pool || !logp_pool || !cdf_pool))) {
    set_error("tpe_cat_posterior: bad arguments");
    return TPE_E_ARG;
  }
  if (n_seg == 0) return TPE_OK;
  if (n_seg > 65535 || max_cat < 0) {
    set_error("tpe_cat_posterior: n_seg=%d max_cat=%d", n_seg, max_cat);
    return TPE_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  const int gx = (std::max(max_cat, 1) + kCatWaves - 1) / kCatWaves;
  hipLaunchKernelGGL(k_cat_counts, dim3(gx, n_seg), dim3(kCatBS), 0, st, obs, segs, p_pool);
  hipLaunchKernelGGL(k_cat_finalize, dim3(n_seg), dim3(kCatBS), 0, st, segs, p_pool, logp_pool,
                     cdf_pool);
  return check_launch("tpe_cat_posterior");
}
