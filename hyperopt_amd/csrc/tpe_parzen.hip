// tpe_parzen.hip -- Parzen posterior fit (adaptive_parzen_normal) for many
// segments at once.
//
// Replaces hyperopt/tpe.py:399-467 (adaptive_parzen_normal) and the
// observation transforms of the ap_*_sampler functions (tpe.py:484-572).
// Every label contributes two segments (below / above); the observation pool
// is one fp64 array indexed by segment offsets, and the fitted mixtures land
// in SoA fp64 pools (w, mu, sigma, wcdf) plus scoring-ready AoS coefficient
// pools (double4 / float4 per component).
//
// Pipeline (one launch each, every launch spread over many blocks per
// segment so a 10k-observation segment is not one CU's serial work):
//   K1 k_fit_tilesort  transform (log for LGMM1 priors) and sort each 2048-
//                      observation tile by (value, index) -- bitonic in LDS;
//   K2 k_fit_rank      stable rank of every observation = its position in its
//                      tile + binary-search counts in the other sorted tiles
//                      (earlier tiles: values <= v, later tiles: < v); the
//                      prior goes in at searchsorted(x, prior_mu, 'left')
//                      (tpe.py:427) or by the len==1 rule (tpe.py:414-421);
//                      the LF ramp follows tid order (tpe.py:441-447);
//   K3 k_fit_comp      bandwidths with the clip (tpe.py:430-459), per-tile
//                      sums of the weights and of w * (Phi(high) - Phi(low));
//   K4 k_fit_coef      normalised weights (tpe.py:465), p_accept
//                      (tpe.py:145-150), fp64 coefficients, cumulative
//                      weights for the sampler, per-tile max of log-coef;
//   K5 k_fit_coef32    fp32 log2-domain coefficients offset by the max;
//   K6 k_fit_prune     (only for the sorted scorer) reach windows + wide list.
#include <algorithm>

#include "tpe_common.hpp"

namespace tpe {
namespace {
constexpr int kFitBS = 256;
constexpr int kSortTile = 2048;  // observations sorted per LDS tile
constexpr double kSqrt2Pi = 2.5066282746310002;

// scratch layout (tpe_fit_scratch_bytes): xf | sort keys | sort perm | tile partials
struct FitScratch {
  double* xf;
  uint64_t* key;
  int32_t* perm;
  double* part;  // per segment: kPartStride doubles per component tile
};
constexpr int kPartStride = 4;  // {sum w, sum w*dPhi, max lc*log2e, -}

__host__ __device__ __forceinline__ int64_t align_up(int64_t x, int64_t a) {
  return (x + a - 1) / a * a;
}
__host__ __device__ __forceinline__ int64_t comp_tiles(int max_obs) {
  return (max_obs + 1 + kFitBS - 1) / kFitBS;
}
__host__ __device__ __forceinline__ FitScratch carve(void* base, int n_seg, int max_obs,
                                                     int64_t n_obs_total) {
  char* p = static_cast<char*>(base);
  FitScratch s;
  s.xf = reinterpret_cast<double*>(p);
  p += align_up(8 * std::max<int64_t>(n_obs_total, 1), 256);
  s.key = reinterpret_cast<uint64_t*>(p);
  p += align_up(8 * std::max<int64_t>(n_obs_total, 1), 256);
  s.perm = reinterpret_cast<int32_t*>(p);
  p += align_up(4 * std::max<int64_t>(n_obs_total, 1), 256);
  s.part = reinterpret_cast<double*>(p);
  (void)n_seg;
  (void)max_obs;
  return s;
}
__host__ __device__ __forceinline__ int64_t scratch_bytes(int n_seg, int max_obs,
                                                          int64_t n_obs_total) {
  const int64_t n = std::max<int64_t>(n_obs_total, 1);
  return align_up(8 * n, 256) * 2 + align_up(4 * n, 256) +
         8 * (int64_t)n_seg * comp_tiles(max_obs) * kPartStride;
}

// number of entries < key (lower) / <= key (upper) in sorted a[0, n)
__device__ __forceinline__ int count_lt(const uint64_t* a, int n, uint64_t key) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int count_le(const uint64_t* a, int n, uint64_t key) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] <= key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// K1: transform + tile sort, one 1024-thread block per 2048-observation tile
// (a pair per thread per bitonic stage: the sort is barrier/latency-bound, so
// more waves per tile, not fewer instructions, is what shortens it)
constexpr int kSortBS = 1024;
__global__ __launch_bounds__(kSortBS) void k_fit_tilesort(const double* __restrict__ obs,
                                                         const tpe_seg* __restrict__ segs,
                                                         FitScratch sc) {
  __shared__ uint64_t skey[kSortTile];
  __shared__ uint16_t sidx[kSortTile];
  const tpe_seg& S = segs[blockIdx.y];
  const int n = S.n_obs;
  const int t0 = blockIdx.x * kSortTile;
  if (t0 >= n) return;  // block-uniform
  const int m = min(kSortTile, n - t0);
  int N = 2;
  while (N < m) N <<= 1;
  const int64_t ooff = S.obs_off;
  for (int e = threadIdx.x; e < N; e += kSortBS) {
    if (e < m) {
      double v = obs[ooff + t0 + e];
      if (S.transform == TPE_OBS_LOG) {
        // np.maximum(obs, floor) keeps NaN; floor=-inf means "no clamp"
        if (v < S.floor) v = S.floor;
        v = log(v);
      }
      sc.xf[ooff + t0 + e] = v;
      skey[e] = order_key(v);
      sidx[e] = (uint16_t)e;
    } else {
      skey[e] = ~0ull;
      sidx[e] = 0xFFFF;
    }
  }
  __syncthreads();
  for (int k = 2; k <= N; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int e = threadIdx.x; e < N / 2; e += kSortBS) {
        const int i = ((e & ~(j - 1)) << 1) | (e & (j - 1));
        const int l = i + j;
        const uint64_t ka = skey[i], kb = skey[l];
        const uint16_t ia = sidx[i], ib = sidx[l];
        const bool gt = (ka > kb) || (ka == kb && ia > ib);
        if (gt == ((i & k) == 0)) {
          skey[i] = kb;
          skey[l] = ka;
          sidx[i] = ib;
          sidx[l] = ia;
        }
      }
      __syncthreads();
    }
  }
  for (int e = threadIdx.x; e < m; e += kSortBS) {
    sc.key[ooff + t0 + e] = skey[e];
    sc.perm[ooff + t0 + e] = t0 + sidx[e];
  }
}

// K2: stable ranks, prior insertion, mu and LF weights in sorted order.
// LDS: the segment's sorted tiles are first copied into LDS (segments of up
// to kRankLds observations, launches of up to 1024 blocks), so the ~4 x 11
// dependent probes of a rank hit LDS instead of L2: 23 -> 16 us at an 8-way
// label share, but 31 -> 57 us for a whole C3 level (4000 blocks each
// copying 80 KB), hence the block-count gate at the launch.
constexpr int kRankLds = 12288;  // keys staged per block (96 KB)

template <bool LDS>
__global__ __launch_bounds__(kFitBS) void k_fit_rank(tpe_seg* __restrict__ segs, FitScratch sc,
                                                     double* __restrict__ w,
                                                     double* __restrict__ mu) {
  extern __shared__ uint64_t s_keys[];
  tpe_seg* S = segs + blockIdx.y;
  const int n = S->n_obs;
  const int q = blockIdx.x * kFitBS + threadIdx.x;
  if ((int64_t)blockIdx.x * kFitBS >= (n > 0 ? n : 1)) return;  // block-uniform
  const int64_t ooff = S->obs_off, coff = S->comp_off;
  const double pmu = S->prior_mu;
  const int nt = (n + kSortTile - 1) / kSortTile;
  const uint64_t* key = sc.key + ooff;
  if constexpr (LDS) {
    // eight loads in flight per thread, then the stores
    for (int e0 = 0; e0 < n; e0 += 8 * kFitBS) {
      uint64_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * kFitBS + threadIdx.x;
        v[u] = e < n ? key[e] : 0ull;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * kFitBS + threadIdx.x;
        if (e < n) s_keys[e] = v[u];
      }
    }
    __syncthreads();
    key = s_keys;
  }
  // the prior's insertion point (keys < prior) and this observation's stable
  // rank, searched together tile by tile (two independent chains per step)
  const bool two = n >= 2;
  const uint64_t kp = two ? order_key(pmu) : 0ull;
  const int t = q / kSortTile, p = q - t * kSortTile;
  const bool mine = q < n;
  const uint64_t kq = mine ? key[q] : 0ull;
  int prior_pos = 0, rank = p;
  for (int tt = 0; tt < nt; ++tt) {
    const uint64_t* a = key + tt * kSortTile;
    const int mm = min(kSortTile, n - tt * kSortTile);
    const bool search = mine && tt != t, le = tt < t;
    int plo = 0, phi = two ? mm : 0, rlo = 0, rhi = search ? mm : 0;
    while (plo < phi || rlo < rhi) {
      if (plo < phi) {
        const int mid = (plo + phi) >> 1;
        if (a[mid] < kp) plo = mid + 1; else phi = mid;
      }
      if (rlo < rhi) {
        const int mid = (rlo + rhi) >> 1;
        const uint64_t v = a[mid];
        if (le ? v <= kq : v < kq) rlo = mid + 1; else rhi = mid;
      }
    }
    prior_pos += plo;
    rank += rlo;
  }
  if (n == 1) prior_pos = (pmu < sc.xf[ooff]) ? 0 : 1;  // tpe.py:414-421
  if (mine) {
    const int gi = sc.perm[ooff + q];
    const int pos = rank + (rank >= prior_pos ? 1 : 0);
    mu[coff + pos] = sc.xf[ooff + gi];
    w[coff + pos] = lf_weight(gi, n, S->lf);  // ramp follows tid order (tpe.py:441-447)
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    mu[coff + prior_pos] = pmu;
    w[coff + prior_pos] = S->prior_weight;
    S->prior_pos = prior_pos;
  }
}

// K3: bandwidths (tpe.py:410-439, 454-459) + per-tile weight sums
__global__ __launch_bounds__(kFitBS) void k_fit_comp(const tpe_seg* __restrict__ segs,
                                                     FitScratch sc, const double* __restrict__ w,
                                                     const double* __restrict__ mu,
                                                     double* __restrict__ sigma) {
  __shared__ double red[kFitBS / kWave];
  const tpe_seg& S = segs[blockIdx.y];
  const int n = S.n_obs, nc = n + 1, pos = S.prior_pos;
  if (blockIdx.x * kFitBS >= nc) return;  // block-uniform
  const int k = blockIdx.x * kFitBS + threadIdx.x;
  const int64_t off = S.comp_off;
  const double ps = S.prior_sigma;
  double wk = 0.0, dphi = 0.0;
  if (k < nc) {
    double s;
    if (S.given) {  // an explicit mixture: its sigmas as given (tpe_mixture_prepare)
      s = sigma[off + k];
    } else if (n == 0) {
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
    if (!S.given) {
      const double lo_clip = ps / fmin(100.0, 1.0 + (double)nc);  // tpe.py:455
      s = fmin(fmax(s, lo_clip), ps);
      if (k == pos) s = ps;
      sigma[off + k] = s;
    }
    wk = w[off + k];
    if (S.bounded) {
      const double m = mu[off + k];
      dphi = normal_cdf(S.high, m, s) - normal_cdf(S.low, m, s);
    }
  }
  const double sw = block_sum<kFitBS, double>(wk, red);
  const double spa = block_sum<kFitBS, double>(wk * dphi, red);
  if (threadIdx.x == 0) {
    double* P = sc.part + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * kPartStride;
    P[0] = sw;
    P[1] = spa;
  }
}

// K4: normalised weights, p_accept, fp64 coefficients, cumulative weights
__global__ __launch_bounds__(kFitBS) void k_fit_coef(tpe_seg* __restrict__ segs, FitScratch sc,
                                                     double* __restrict__ w,
                                                     const double* __restrict__ mu,
                                                     const double* __restrict__ sigma,
                                                     double* __restrict__ wcdf,
                                                     double* __restrict__ coef64) {
  __shared__ double red[kFitBS / kWave];
  __shared__ double wscan[kFitBS / kWave];
  tpe_seg* S = segs + blockIdx.y;
  const int nc = S->n_obs + 1;
  const int tiles = (nc + kFitBS - 1) / kFitBS;
  if ((int)blockIdx.x >= tiles) return;  // block-uniform
  const double* P = sc.part + (int64_t)blockIdx.y * gridDim.x * kPartStride;
  // every block re-reduces the (few) tile partials in the same order
  double a = 0.0, b = 0.0, before = 0.0;
  for (int t = threadIdx.x; t < tiles; t += kFitBS) {
    a += P[t * kPartStride];
    b += P[t * kPartStride + 1];
    if (t < (int)blockIdx.x) before += P[t * kPartStride];
  }
  const double wsum = block_sum<kFitBS, double>(a, red);
  const double pacc = S->bounded ? block_sum<kFitBS, double>(b, red) / wsum : 1.0;
  const double base = block_sum<kFitBS, double>(before, red);
  const int k = blockIdx.x * kFitBS + threadIdx.x;
  const int64_t off = S->comp_off;
  double wr = 0.0, lmax = -INFINITY;
  if (k < nc) {
    wr = w[off + k];
    const double wk = wr / wsum;
    w[off + k] = wk;
    const double m = mu[off + k], s = sigma[off + k];
    double lc, inv;
    if (S->family == TPE_LGMM1) {
      // LGMM1_lpdf: log(w) - log(max(sigma,EPS) sqrt(2 pi)); no p_accept (tpe.py:284-287)
      const double sp = fmax(s, kEps);
      lc = log(wk) - log(sp * kSqrt2Pi);
      inv = 1.0 / sp;
    } else {
      // GMM1_lpdf: log(w / sqrt(2 pi sigma^2) / p_accept) (tpe.py:152-158)
      const double z = sqrt(kTwoPi * (s * s));
      lc = log(wk / z / pacc);
      inv = 1.0 / fmax(s, kEps);
    }
    double* c = coef64 + 4 * (off + k);
    c[0] = m;
    c[1] = inv;
    c[2] = lc;
    c[3] = wk;
    lmax = lc * kLog2e;
  }
  // inclusive scan of the raw weights inside the tile -> cumulative weights
  const int lane = lane_id(), wid = threadIdx.x / kWave;
  double v = wr;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const double u = __shfl_up(v, o, kWave);
    if (lane >= o) v += u;
  }
  if (lane == kWave - 1) wscan[wid] = v;
  __syncthreads();
  for (int q = 0; q < wid; ++q) v += wscan[q];
  if (k < nc) wcdf[off + k] = (base + v) / wsum;
  const double tmax = block_max<kFitBS, double>(lmax, red);
  if (threadIdx.x == 0) {
    sc.part[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * kPartStride + 2] = tmax;
    if (blockIdx.x == 0) S->p_accept = pacc;
  }
}

// K5: fp32 coefficients in log2 units around a float-exact centre:
//     t = xc*a + b,  v = c - t^2,  term = 2^v  (v <= 0, offset cmax)
__global__ __launch_bounds__(kFitBS) void k_fit_coef32(tpe_seg* __restrict__ segs, FitScratch sc,
                                                       const double* __restrict__ coef64,
                                                       float* __restrict__ coef32) {
  __shared__ double red[kFitBS / kWave];
  tpe_seg* S = segs + blockIdx.y;
  const int nc = S->n_obs + 1;
  const int tiles = (nc + kFitBS - 1) / kFitBS;
  if ((int)blockIdx.x >= tiles) return;
  const double* P = sc.part + (int64_t)blockIdx.y * gridDim.x * kPartStride;
  double mx = -INFINITY;
  for (int t = threadIdx.x; t < tiles; t += kFitBS) mx = fmax(mx, P[t * kPartStride + 2]);
  const double cmax = block_max<kFitBS, double>(mx, red);
  const double center = (double)(float)S->prior_mu;
  const double sq = 0.8493218002880191;  // sqrt(0.5 * log2(e))
  const int k = blockIdx.x * kFitBS + threadIdx.x;
  const int64_t off = S->comp_off;
  if (k < nc) {
    const double* c = coef64 + 4 * (off + k);
    const double a = c[1] * sq;
    float* f = coef32 + 4 * (off + k);
    f[0] = (float)a;
    f[1] = (float)(-(c[0] - center) * a);
    f[2] = (float)(c[2] * kLog2e - cmax);
    f[3] = 0.0f;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    S->cmax = cmax;
    S->center = center;
  }
}

// K6 (sorted scorer only): pruning data.  In log2 units relative to cmax,
// every candidate y of the support has log2(sum) >= v_prior(y) >= lglob
// (bounded: the prior term at the farther end of [low, high]; unbounded: at
// 6 prior sigmas -- blocks beyond fall back to all components).  Component
// k's term is below 2^(lglob - 40), i.e. negligible at fp32 resolution even
// summed over 1e4 terms, once |y - mu_k| > r_k = sqrt(c_k - lglob + 40) / a_k.
// Wide components (the prior and sigma >= prior_sigma/4) are always evaluated
// from a compact list; narrow ones through a [k_lo, k_hi] window found with
// the prefix max of mu + r (pm) and the suffix min of mu - r (sm).
__global__ __launch_bounds__(kFitBS) void k_fit_prune(tpe_seg* __restrict__ segs,
                                                      const double* __restrict__ mu,
                                                      const double* __restrict__ sigma,
                                                      const double* __restrict__ coef64,
                                                      const float* __restrict__ coef32,
                                                      float* __restrict__ coef32n,
                                                      float* __restrict__ wide32,
                                                      float* __restrict__ pm,
                                                      float* __restrict__ sm) {
  __shared__ float chunk_f[kFitBS];
  __shared__ int chunk_n[kFitBS];
  tpe_seg* S = segs + blockIdx.x;
  const int n = S->n_obs, nc = n + 1, pos = S->prior_pos;
  const int64_t off = S->comp_off;
  const double ps = S->prior_sigma, cmax = S->cmax;
  const double sq = 0.8493218002880191;
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
  const int per = (nc + kFitBS - 1) / kFitBS;
  const int k0 = threadIdx.x * per, k1 = min(nc, k0 + per);
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
  const float after = chunk_f[threadIdx.x];
  for (int k = k0; k < k1; ++k) sm[off + k] = fminf(sm[off + k], after);
}
}  // namespace

// K3-K5 over mixtures whose means and raw weights are in place (prior_pos
// set): shared with tpe_fit_sorted (tpe_sorted.hip), whose compaction
// replaces K1-K2.  part: n_seg * fit_part_doubles(max_obs) doubles.
int64_t fit_part_doubles(int max_obs) { return comp_tiles(max_obs) * kPartStride; }
void fit_tail(tpe_seg* segs, int n_seg, int max_obs, double* part, double* w, const double* mu,
              double* sigma, double* wcdf, double* coef64, float* coef32, hipStream_t st) {
  const FitScratch sc{nullptr, nullptr, nullptr, part};
  const int gc = (int)comp_tiles(max_obs);
  hipLaunchKernelGGL(k_fit_comp, dim3(gc, n_seg), dim3(kFitBS), 0, st, segs, sc, w, mu, sigma);
  hipLaunchKernelGGL(k_fit_coef, dim3(gc, n_seg), dim3(kFitBS), 0, st, segs, sc, w, mu, sigma,
                     wcdf, coef64);
  hipLaunchKernelGGL(k_fit_coef32, dim3(gc, n_seg), dim3(kFitBS), 0, st, segs, sc, coef64,
                     coef32);
}
}  // namespace tpe

using namespace tpe;

extern "C" int64_t tpe_fit_scratch_bytes(int n_seg, int max_obs, int64_t n_obs_total) {
  if (n_seg < 0 || max_obs < 0 || n_obs_total < 0) return -1;
  return scratch_bytes(n_seg, max_obs, n_obs_total);
}

extern "C" int tpe_parzen_fit(const double* obs, void* scratch, tpe_seg* segs, int n_seg,
                              int max_obs, int64_t n_obs_total, double* w, double* mu,
                              double* sigma, double* wcdf, double* coef64, float* coef32,
                              float* coef32n, float* wide32, float* pm, float* sm,
                              void* stream) {
  if (n_seg < 0 || max_obs < 0 || n_obs_total < 0) {
    set_error("tpe_parzen_fit: n_seg=%d max_obs=%d n_obs_total=%lld", n_seg, max_obs,
              (long long)n_obs_total);
    return TPE_E_ARG;
  }
  if (n_seg == 0) return TPE_OK;
  if (!segs || !scratch || !w || !mu || !sigma || !wcdf || !coef64 || !coef32 ||
      (max_obs > 0 && !obs)) {
    set_error("tpe_parzen_fit: null pointer");
    return TPE_E_ARG;
  }
  const bool prune = coef32n || wide32 || pm || sm;
  if (prune && !(coef32n && wide32 && pm && sm)) {
    set_error("tpe_parzen_fit: coef32n, wide32, pm and sm go together");
    return TPE_E_ARG;
  }
  if (n_seg > 65535 || max_obs >= (1 << 30)) {
    set_error("tpe_parzen_fit: n_seg %d / max_obs %d out of range", n_seg, max_obs);
    return TPE_E_UNSUPPORTED;
  }
  hipStream_t st = (hipStream_t)stream;
  const FitScratch sc = carve(scratch, n_seg, max_obs, n_obs_total);
  if (max_obs > 0) {
    const int gs = (max_obs + kSortTile - 1) / kSortTile;
    hipLaunchKernelGGL(k_fit_tilesort, dim3(gs, n_seg), dim3(kSortBS), 0, st, obs, segs, sc);
  }
  const int gr = (std::max(max_obs, 1) + kFitBS - 1) / kFitBS;
  // staged ranks need > 64 KB of dynamic LDS: opt in once (gfx950 has 160 KB)
  static const bool rank_lds = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&k_fit_rank<true>),
      hipFuncAttributeMaxDynamicSharedMemorySize, 8 * kRankLds) == hipSuccess;
  // staging costs every block a copy of its segment's keys: it pays while
  // the launch leaves the GPU half-idle (a rank's share of labels), not when
  // thousands of blocks already hide the L2 latency (a whole C3 level)
  if (rank_lds && max_obs <= kRankLds && (int64_t)gr * n_seg <= 1024)
    hipLaunchKernelGGL(k_fit_rank<true>, dim3(gr, n_seg), dim3(kFitBS),
                       (size_t)8 * std::max(max_obs, 1), st, segs, sc, w, mu);
  else
    hipLaunchKernelGGL(k_fit_rank<false>, dim3(gr, n_seg), dim3(kFitBS), 0, st, segs, sc, w, mu);
  fit_tail(segs, n_seg, max_obs, sc.part, w, mu, sigma, wcdf, coef64, coef32, st);
  if (prune)
    hipLaunchKernelGGL(k_fit_prune, dim3(n_seg), dim3(kFitBS), 0, st, segs, mu, sigma, coef64,
                       coef32, coef32n, wide32, pm, sm);
  return check_launch("tpe_parzen_fit");
}

extern "C" int64_t tpe_mixture_scratch_bytes(int n_seg, int max_comp) {
  if (n_seg < 0 || max_comp < 1) return -1;
  return 8 * (int64_t)std::max(n_seg, 1) * fit_part_doubles(max_comp - 1);
}

extern "C" int tpe_mixture_prepare(tpe_seg* segs, int n_seg, int max_comp, void* scratch,
                                   double* w, const double* mu, double* sigma, double* wcdf,
                                   double* coef64, float* coef32, void* stream) {
  if (n_seg < 0 || max_comp < 1 || n_seg > 65535 || max_comp >= (1 << 30)) {
    set_error("tpe_mixture_prepare: n_seg=%d max_comp=%d", n_seg, max_comp);
    return TPE_E_ARG;
  }
  if (n_seg == 0) return TPE_OK;
  if (!segs || !scratch || !w || !mu || !sigma || !wcdf || !coef64 || !coef32) {
    set_error("tpe_mixture_prepare: null pointer");
    return TPE_E_ARG;
  }
  fit_tail(segs, n_seg, max_comp - 1, static_cast<double*>(scratch), w, mu, sigma, wcdf, coef64,
           coef32, (hipStream_t)stream);
  return check_launch("tpe_mixture_prepare");
}
