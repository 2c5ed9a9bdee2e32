// tpe_fit.hip -- categorical pseudocount posteriors.
//
// Replaces the categorical posteriors of hyperopt/tpe.py:578-615 (randint /
// categorical / pchoice) with pyll/base.py:1053-1060 (bincount).  The Parzen
// fit of continuous labels is tpe_parzen.hip.
#include <algorithm>
#include <stdarg.h>
#include <stdio.h>

#include "tpe_common.hpp"

namespace tpe {

namespace {
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
  };
  // (one thread sums; its explicit stack lives in LDS, not in scratch: a
  // private array here gave the calling kernel 1.5 KB of scratch per lane)
  __shared__ Frame stk[48];
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

// Weighted counts, one wave per (segment, category): np.bincount's sum
// (pyll/base.py:1053-1060) adds the LF weights of a category's observations
// sequentially in observation order, so the fp64 chain itself cannot be
// split.  The wave scans 64 observations per step, ballots the matches, and
// every matching lane writes its weight (computed in parallel) into the
// wave's LDS list at its rank; when the list fills, lane 0 folds it into the
// running count in list order -- the only serial work left is one fp64 add
// per match.
constexpr int kCatList = 512;  // weights buffered per wave before a fold

__global__ __launch_bounds__(kCatBS) void k_cat_counts(const int64_t* __restrict__ obs,
                                                       const tpe_cat_seg* __restrict__ segs,
                                                       double* __restrict__ p) {
  __shared__ double s_list[kCatWaves][kCatList];
  const tpe_cat_seg& S = segs[blockIdx.y];
  const int k = blockIdx.x * kCatWaves + threadIdx.x / kWave;
  if (k >= S.n_cat) return;  // wave-uniform
  double* list = s_list[threadIdx.x / kWave];
  const int n = S.n_obs, lane = lane_id();
  // linear-forgetting ramp (np.linspace(1/N, 1, N-LF), tpe.py:380-392)
  const bool ramp = S.lf > 0 && S.lf < n;
  const int64_t num = n - S.lf;
  const double start = 1.0 / (double)n;
  const double step = (ramp && num > 1) ? (1.0 - start) / (double)(num - 1) : 0.0;
  const uint64_t lt = (1ull << lane) - 1ull;
  double cnt = 0.0;
  int filled = 0;
  auto fold = [&]() {
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      // kFoldB weights read together (one LDS latency per batch, not per add),
      // then added in list order: the fp64 add chain is the only serial part
      constexpr int kFoldB = 32;
      int j = 0;
      for (; j + kFoldB <= filled; j += kFoldB) {
        double v[kFoldB];
#pragma unroll
        for (int i = 0; i < kFoldB; ++i) v[i] = list[j + i];
#pragma unroll
        for (int i = 0; i < kFoldB; ++i) cnt = __dadd_rn(cnt, v[i]);
      }
      for (; j < filled; ++j) cnt = __dadd_rn(cnt, list[j]);
    }
    filled = 0;
    __builtin_amdgcn_wave_barrier();
  };
  constexpr int kDepth = 32;  // tiles of 64 observations in flight per step (latency-bound scan)
  for (int t0 = 0; t0 < n; t0 += kDepth * kWave) {
    int64_t cur[kDepth];
#pragma unroll
    for (int b = 0; b < kDepth; ++b) {
      const int i = t0 + b * kWave + lane;
      cur[b] = i < n ? obs[S.obs_off + i] : -1;
    }
#pragma unroll
    for (int b = 0; b < kDepth; ++b) {
      const bool hit = cur[b] == (int64_t)k;
      const uint64_t m = __ballot(hit);
      if (m == 0) continue;  // wave-uniform
      if (filled + kWave > kCatList) fold();
      if (hit) {
        const int64_t i = t0 + b * kWave + lane;
        double wt = 1.0;
        if (ramp && i < num) {
          if (num == 1) wt = start;
          else if (i == num - 1) wt = 1.0;
          else wt = __dadd_rn(__dmul_rn((double)i, step), start);
        }
        list[filled + __popcll(m & lt)] = wt;
      }
      filled += __popcll(m);
    }
  }
  fold();
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
