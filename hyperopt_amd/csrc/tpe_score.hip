// tpe_score.hip -- candidate sampling, EI scoring and argmax for TPE.
//
// Replaces, per label:
//   GMM1 / LGMM1 sampling          hyperopt/tpe.py:79-106, 229-257
//   categorical sampling           hyperopt/pyll/stochastic.py:119-158
//   GMM1_lpdf / LGMM1_lpdf         hyperopt/tpe.py:117-180, 265-307 (+ logsum_rows :260-262)
//   categorical_lpdf               hyperopt/tpe.py:60-73
//   broadcast_best (argmax)        hyperopt/tpe.py:649-658
//
// Continuous, unquantized labels (the N x M hot loop):
//   grid = (candidate chunks, labels); a block owns kBS*R candidates held in
//   registers (R per thread), sampled with Philox from the below mixture (or
//   read, for injected candidates), and streams each mixture's components
//   through one LDS tile (float4 {a,b,c,-} / double4 {mu,1/sigma,logcoef,w}),
//   read back as wave-wide broadcasts.  fp32 terms are evaluated as
//       t = xc*a + b ;  v = c - t*t ;  sum += 2^v        (one v_exp_f32 / pair)
//   with the log2 coefficients pre-offset by the mixture's max, so no running
//   max is needed; a wave whose prior term shows the sum could leave the
//   normal range (v_prior < -100) takes the exact online log-sum-exp instead.
//   fp64 (parity mode) always runs the exact online log-sum-exp.
//   The argmax is fused: per-thread -> wave butterfly -> block -> partials ->
//   one reduce block per label.  Nothing per-candidate touches HBM unless the
//   caller asks for the per-candidate outputs.
//
// Quantized labels (lattice path): candidate values are k*q, so each distinct
// value is scored once in fp64 with the reference's erf-pair sum and the
// argmax keeps the first candidate index of the best value.
#include <algorithm>

#include "tpe_common.hpp"
#include "tpe_sample.hpp"

namespace tpe {

namespace {
constexpr int kR32 = 8;
constexpr int kR64 = 4;
constexpr int kTile32 = 1024;  // float4 components per tile (16 KB)
constexpr int kTile64 = 512;   // double4 components per tile (16 KB)
#ifndef TPE_LATR
#define TPE_LATR 16
#endif
constexpr int kLatR = TPE_LATR;  // lattice sampler: candidates per thread
constexpr int kLatLds = 4096;  // lattice slots deduplicated in LDS per block
constexpr float kFastFloor = -100.0f;            // log2 units below the mixture max
constexpr float kLn2f = 0.6931471805599453f;

// ---------------------------------------------------------------------------
// mixture log-density at R candidates, fp32 (log2-domain, offset by cmax)
// ---------------------------------------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int R>
struct Lse32 {
  float xc[R], s[R], m[R];
  bool fast;
};

// centre the candidates and decide the wave's mode: the fast path (fixed
// offset, one v_exp_f32 per pair) is exact whenever the prior component's
// term keeps the sum in the normal fp32 range for every lane of the wave
template <int R>
__device__ __forceinline__ void lse32_begin(Lse32<R>& L, const float4* __restrict__ coef,
                                            const tpe_seg& S, const float (&y)[R]) {
  const float cen = (float)S.center;
  const float4 cp = coef[S.prior_pos];
  bool ok = true;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    L.xc[r] = y[r] - cen;
    const float t = fmaf(L.xc[r], cp.x, cp.y);
    ok = ok && (fmaf(-t, t, cp.z) >= kFastFloor);
    L.s[r] = 0.0f;
    L.m[r] = -INFINITY;
  }
  L.fast = __all(ok);
}

// accumulate the mm components staged in `tile` (block-uniform mm)
template <int R>
__device__ __forceinline__ void lse32_tile(Lse32<R>& L, const float4* tile, int mm) {
  if (L.fast) {
    // packed fp32: two candidates per v_pk_fma_f32 (the microbenchmark in
    // tools/valu_microbench.hip: 15.8 vs 18.9 cycles per 64 pairs)
    static_assert(R % 2 == 0, "R must be even");
    f32x2 xc2[R / 2], acc[R / 2];
#pragma unroll
    for (int p = 0; p < R / 2; ++p) {
      xc2[p] = f32x2{L.xc[2 * p], L.xc[2 * p + 1]};
      acc[p] = f32x2{0.0f, 0.0f};
    }
#pragma unroll 4
    for (int k = 0; k < mm; ++k) {
      const float4 c = tile[k];
      const f32x2 a2 = f32x2{c.x, c.x}, b2 = f32x2{c.y, c.y}, c2 = f32x2{c.z, c.z};
#pragma unroll
      for (int p = 0; p < R / 2; ++p) {
        const f32x2 t = __builtin_elementwise_fma(xc2[p], a2, b2);
        const f32x2 v = __builtin_elementwise_fma(-t, t, c2);
        acc[p] += f32x2{__builtin_amdgcn_exp2f(v.x), __builtin_amdgcn_exp2f(v.y)};
      }
    }
#pragma unroll
    for (int p = 0; p < R / 2; ++p) {
      L.s[2 * p] += acc[p].x;
      L.s[2 * p + 1] += acc[p].y;
    }
  } else {
    for (int k = 0; k < mm; ++k) {
      const float4 c = tile[k];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float t = fmaf(L.xc[r], c.x, c.y);
        const float v = fmaf(-t, t, c.z);
        if (v > L.m[r]) {
          L.s[r] = L.s[r] * __builtin_amdgcn_exp2f(L.m[r] - v) + 1.0f;
          L.m[r] = v;
        } else if (c.z > -INFINITY) {  // masked (wide) components add nothing
          L.s[r] += __builtin_amdgcn_exp2f(v - L.m[r]);
        }
      }
    }
  }
}

// accumulate components [k0, k1) of `coef` (block-uniform bounds; syncs)
template <int R>
__device__ __forceinline__ void lse32_accum(Lse32<R>& L, const float4* __restrict__ coef, int k0,
                                            int k1, float4* tile) {
  for (int t0 = k0; t0 < k1; t0 += kTile32) {
    const int mm = min(kTile32, k1 - t0);
    __syncthreads();
    for (int j = threadIdx.x; j < mm; j += kBS) tile[j] = coef[t0 + j];
    __syncthreads();
    lse32_tile(L, tile, mm);
  }
}

// largest / smallest term of component c over centred candidates [xlo, xhi]
// (t = xc*a + b is increasing in xc, v = c - t^2)
__device__ __forceinline__ float term_max(const float4 c, float xlo, float xhi) {
  const float tl = fmaf(xlo, c.x, c.y), th = fmaf(xhi, c.x, c.y);
  const float t2 = (tl <= 0.0f && th >= 0.0f) ? 0.0f : fminf(tl * tl, th * th);
  return c.z - t2;
}
__device__ __forceinline__ float term_min(const float4 c, float xlo, float xhi) {
  const float tl = fmaf(xlo, c.x, c.y), th = fmaf(xhi, c.x, c.y);
  return c.z - fmaxf(tl * tl, th * th);
}

// like lse32_accum, but only components whose largest term over the block's
// candidates reaches `thr` are staged (compacted, in index order) and summed.
// Returns the number of components summed (block-uniform).
template <int R>
__device__ __forceinline__ int lse32_accum_pruned(Lse32<R>& L, const float4* __restrict__ coef,
                                                  int k0, int k1, float4* tile, int* cnt,
                                                  float xlo, float xhi, float thr) {
  constexpr int kQ = kTile32 / kBS, kW = kBS / kWave;
  const int wid = threadIdx.x / kWave;
  const unsigned lane = lane_id();
  const uint64_t below_me = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int used = 0;
  for (int t0 = k0; t0 < k1; t0 += kTile32) {
    const int mm = min(kTile32, k1 - t0);
    float4 c[kQ];
    bool keep[kQ];
    uint64_t bal[kQ];
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const int j = q * kBS + threadIdx.x;
      keep[q] = false;
      if (j < mm) {
        c[q] = coef[t0 + j];
        keep[q] = term_max(c[q], xlo, xhi) >= thr;
      }
      bal[q] = __ballot(keep[q]);
    }
    __syncthreads();  // previous tile consumed, cnt free
    if (lane == 0)
#pragma unroll
      for (int q = 0; q < kQ; ++q) cnt[q * kW + wid] = __popcll(bal[q]);
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      int mine = 0;
#pragma unroll
      for (int w = 0; w < kW; ++w) {
        const int n = cnt[q * kW + w];
        if (w < wid) mine += n;
        tot += n;
      }
      if (keep[q]) tile[pre + mine + __popcll(bal[q] & below_me)] = c[q];
      pre = tot;
    }
    __syncthreads();
    lse32_tile(L, tile, tot);
    used += tot;
  }
  return used;
}

template <int R>
__device__ __forceinline__ void lse32_end(const Lse32<R>& L, const tpe_seg& S, float (&out)[R]) {
  const float C = (float)S.cmax;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float l2 = __builtin_amdgcn_logf(L.s[r]);  // log2
    out[r] = (L.fast ? (l2 + C) : (L.m[r] + l2 + C)) * kLn2f;
  }
}

template <int R>
__device__ __forceinline__ void lse32(const float4* __restrict__ coef, const tpe_seg& S,
                                      const float (&y)[R], float (&out)[R], float4* tile) {
  Lse32<R> L;
  lse32_begin(L, coef, S, y);
  lse32_accum(L, coef, 0, S.n_obs + 1, tile);
  lse32_end(L, S, out);
}

// exact online log-sum-exp, fp64 (parity mode)
template <int R>
__device__ __forceinline__ void lse64(const double4* __restrict__ coef, const tpe_seg& S,
                                      const double (&y)[R], double (&out)[R], double4* tile) {
  const int nc = S.n_obs + 1;
  double s[R], m[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    s[r] = 0.0;
    m[r] = -INFINITY;
  }
  for (int t0 = 0; t0 < nc; t0 += kTile64) {
    const int mm = min(kTile64, nc - t0);
    __syncthreads();
    for (int j = threadIdx.x; j < mm; j += kBS) tile[j] = coef[t0 + j];
    __syncthreads();
    for (int k = 0; k < mm; ++k) {
      const double4 c = tile[k];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double t = (y[r] - c.x) * c.y;
        const double v = -0.5 * (t * t) + c.z;
        // one exp per pair on every lane: a branch per lane would run the
        // (software) fp64 exp twice whenever the wave diverges.  Same values
        // as s*exp(m-v)+1 (new max) / s+exp(v-m), NaN included.
        const bool up = v > m[r];
        const double e = exp(up ? m[r] - v : v - m[r]);
        s[r] = up ? s[r] * e + 1.0 : s[r] + e;
        m[r] = up ? v : m[r];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) out[r] = log(s[r]) + m[r];
}

// ---------------------------------------------------------------------------
// continuous, unquantized: sample/read + score + argmax
// ---------------------------------------------------------------------------
template <bool INJ>
__global__ __launch_bounds__(kBS) void k_score32(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const double* __restrict__ mu, const double* __restrict__ sigma,
    const double* __restrict__ wcdf, const float4* __restrict__ coef32,
    const double* __restrict__ cand, double* __restrict__ out_bl, double* __restrict__ out_al,
    double* __restrict__ out_x, tpe_best* __restrict__ partial) {
  __shared__ float4 tile[kTile32];
  __shared__ MixLds s_mix;
  __shared__ BestT red[kBS / kWave];
  const tpe_job J = jobs[blockIdx.y];
  tpe_best* P = partial + (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  const int64_t base = (int64_t)blockIdx.x * (kBS * kR32);
  if (base >= J.n_cand) {
    if (threadIdx.x == 0) *P = empty_best();
    return;
  }
  const tpe_seg SB = segs[J.below], SA = segs[J.above];
  const bool lgmm = J.family == TPE_LGMM1;
  const bool lo_on = J.flags & TPE_F_LOW, hi_on = J.flags & TPE_F_HIGH;
  // x: the given value (INJ) or the fp32 draw in the mixture's coordinate
  // (log x for LGMM1, whose value is exp(y) evaluated in fp64: log(value) is
  // then y itself, see cand_value in tpe_table.hip)
  float x[kR32], y[kR32];
  if (INJ) {
#pragma unroll
    for (int r = 0; r < kR32; ++r) {
      const int64_t li = base + r * kBS + threadIdx.x;
      x[r] = li < J.n_cand ? (float)cand[J.cand_off + li] : 1.0f;
    }
  } else {
    const Mix M = stage_mix(SB, wcdf, mu, sigma, s_mix);
#pragma unroll
    for (int r = 0; r < kR32; ++r) {
      const int64_t li = base + r * kBS + threadIdx.x;
      x[r] = li < J.n_cand ? draw32(M, J.key, J.cand_base + li, lo_on, hi_on, (float)J.low,
                                    (float)J.high)
                           : 1.0f;
    }
  }
#pragma unroll
  for (int r = 0; r < kR32; ++r) {
    const int64_t li = base + r * kBS + threadIdx.x;
    if (li < J.n_cand)
      y[r] = (lgmm && INJ) ? __logf(x[r]) : x[r];
    else
      y[r] = (float)SA.center;  // inactive lanes sit on the prior mean
  }
  float lb[kR32], la[kR32];
  lse32<kR32>(coef32 + SB.comp_off, SB, y, lb, tile);
  lse32<kR32>(coef32 + SA.comp_off, SA, y, la, tile);
  BestT b{0.0, -1, 0.0};
#pragma unroll
  for (int r = 0; r < kR32; ++r) {
    const int64_t li = base + r * kBS + threadIdx.x;
    if (li >= J.n_cand) continue;
    double bl = lb[r], al = la[r];
    if (lgmm) {  // lognormal_lpdf's -log(x) (tpe.py:214-216)
      bl -= (double)y[r];
      al -= (double)y[r];
    }
    const double v = (lgmm && !INJ) ? exp((double)x[r]) : (double)x[r];
    const int64_t o = J.out_off + li;
    if (out_bl) out_bl[o] = bl;
    if (out_al) out_al[o] = al;
    if (out_x) out_x[o] = v;
    best_update(b, bl - al, J.cand_base + li, v);
  }
  b = block_best<kBS>(b, red);
  if (threadIdx.x == 0) *P = tpe_best{b.score, b.index, b.value, 0};
}

template <bool INJ>
__global__ __launch_bounds__(kBS) void k_score64(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const double* __restrict__ mu, const double* __restrict__ sigma,
    const double* __restrict__ wcdf, const double4* __restrict__ coef64,
    const double* __restrict__ cand, double* __restrict__ out_bl, double* __restrict__ out_al,
    double* __restrict__ out_x, tpe_best* __restrict__ partial) {
  __shared__ double4 tile[kTile64];
  __shared__ MixLds s_mix;
  __shared__ BestT red[kBS / kWave];
  const tpe_job J = jobs[blockIdx.y];
  tpe_best* P = partial + (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  const int64_t base = (int64_t)blockIdx.x * (kBS * kR64);
  if (base >= J.n_cand) {
    if (threadIdx.x == 0) *P = empty_best();
    return;
  }
  const tpe_seg SB = segs[J.below], SA = segs[J.above];
  const bool lgmm = J.family == TPE_LGMM1;
  const bool lo_on = J.flags & TPE_F_LOW, hi_on = J.flags & TPE_F_HIGH;
  double x[kR64], y[kR64];
  if (INJ) {
#pragma unroll
    for (int r = 0; r < kR64; ++r) {
      const int64_t li = base + r * kBS + threadIdx.x;
      x[r] = li < J.n_cand ? cand[J.cand_off + li] : 1.0;
    }
  } else {
    const Mix M = stage_mix(SB, wcdf, mu, sigma, s_mix);
#pragma unroll
    for (int r = 0; r < kR64; ++r) {
      const int64_t li = base + r * kBS + threadIdx.x;
      double v = 1.0;
      if (li < J.n_cand) {
        v = draw64(M, J.key, J.cand_base + li, lo_on, hi_on, J.low, J.high);
        if (lgmm) v = exp(v);
      }
      x[r] = v;
    }
  }
#pragma unroll
  for (int r = 0; r < kR64; ++r) {
    const int64_t li = base + r * kBS + threadIdx.x;
    y[r] = li < J.n_cand ? (lgmm ? log(x[r]) : x[r]) : SA.prior_mu;
  }
  double lb[kR64], la[kR64];
  lse64<kR64>(coef64 + SB.comp_off, SB, y, lb, tile);
  lse64<kR64>(coef64 + SA.comp_off, SA, y, la, tile);
  BestT b{0.0, -1, 0.0};
#pragma unroll
  for (int r = 0; r < kR64; ++r) {
    const int64_t li = base + r * kBS + threadIdx.x;
    if (li >= J.n_cand) continue;
    double bl = lb[r], al = la[r];
    if (lgmm) {
      bl -= y[r];
      al -= y[r];
    }
    const int64_t o = J.out_off + li;
    if (out_bl) out_bl[o] = bl;
    if (out_al) out_al[o] = al;
    if (out_x) out_x[o] = x[r];
    best_update(b, bl - al, J.cand_base + li, x[r]);
  }
  b = block_best<kBS>(b, red);
  if (threadIdx.x == 0) *P = tpe_best{b.score, b.index, b.value, 0};
}

// one block per job: combine its partials
__global__ __launch_bounds__(kBS) void k_reduce(const tpe_job* __restrict__ jobs,
                                                const tpe_best* __restrict__ partial, int64_t nper,
                                                tpe_best* __restrict__ best) {
  __shared__ BestT red[kBS / kWave];
  BestT b = thread_best<kBS>(partial + (int64_t)blockIdx.x * nper, nper);
  b = block_best<kBS>(b, red);
  if (threadIdx.x == 0) best[blockIdx.x] = tpe_best{b.score, b.index, b.value, jobs[blockIdx.x].n_cand};
}

// ---------------------------------------------------------------------------
// continuous, unquantized, sorted + pruned (fp32)
// ---------------------------------------------------------------------------
constexpr int kNB = 512;                 // value bins per label
constexpr int kSortR = 16;               // candidates per thread in count / scatter
constexpr int kSortPer = kBS * kSortR;   // candidates per count / scatter block (4096)

__device__ __forceinline__ int bin_of(float y, float lo, float scale) {
  float t = (y - lo) * scale;
  t = fminf(fmaxf(t, 0.0f), (float)(kNB - 1));  // NaN -> 0
  return (int)t;
}

// the candidate exactly as k_score32<false> draws it, in the mixture's
// coordinate (log x for LGMM1: its value is exp(y) in fp64)
__device__ __forceinline__ float cand32(const Mix& M, const tpe_job& J, int64_t li, bool lo_on,
                                        bool hi_on) {
  return draw32(M, J.key, J.cand_base + li, lo_on, hi_on, (float)J.low, (float)J.high);
}

// K1: draw every candidate once (kept in `gen`, generation order, coalesced)
// and count them per (block, value bin)
__global__ __launch_bounds__(kBS) void k_sort_count(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const double* __restrict__ mu, const double* __restrict__ sigma,
    const double* __restrict__ wcdf, uint32_t* __restrict__ counts, float* __restrict__ gen) {
  __shared__ uint32_t h[kNB];
  __shared__ MixLds s_mix;
  const tpe_job J = jobs[blockIdx.y];
  const int64_t base = (int64_t)blockIdx.x * kSortPer;
  if (base >= J.n_cand) return;
  for (int i = threadIdx.x; i < kNB; i += kBS) h[i] = 0u;
  const Mix M = stage_mix(segs[J.below], wcdf, mu, sigma, s_mix);
  __syncthreads();
  const bool lo_on = J.flags & TPE_F_LOW, hi_on = J.flags & TPE_F_HIGH;
  const float lo = (float)J.bin_lo, scale = (float)(kNB / (J.bin_hi - J.bin_lo));
  for (int r = 0; r < kSortR; ++r) {
    const int64_t li = base + r * kBS + threadIdx.x;
    if (li >= J.n_cand) break;
    const float y = cand32(M, J, li, lo_on, hi_on);
    gen[J.sort_off + li] = y;
    atomicAdd(&h[bin_of(y, lo, scale)], 1u);
  }
  __syncthreads();
  uint32_t* row = counts + 2 * J.cnt_off + (int64_t)blockIdx.x * kNB;
  for (int i = threadIdx.x; i < kNB; i += kBS) row[i] = h[i];
}

// K2: per job, global start of every (block, bin) run in (bin, block) order;
// counts keep their values (row b at 2*cnt_off), offsets go to the second half
// K2: exclusive offsets of every (block, bin) run in bin-major order.  The
// count matrix is cut into chunks of kScanChunk blocks: column sums per chunk
// (K2a), one scan over (bin, chunk) per job (K2b), offsets per chunk (K2c).
constexpr int kScanChunk = 32;

__device__ __forceinline__ int64_t sort_nblk(const tpe_job& J) {
  return (J.n_cand + kSortPer - 1) / kSortPer;
}

__global__ __launch_bounds__(kNB) void k_sort_colsum(const tpe_job* __restrict__ jobs,
                                                     uint32_t* __restrict__ counts) {
  const tpe_job J = jobs[blockIdx.y];
  const int64_t nblk = sort_nblk(J);
  const int64_t b0 = (int64_t)blockIdx.x * kScanChunk;
  if (b0 >= nblk) return;
  const int64_t b1 = min(nblk, b0 + kScanChunk);
  const uint32_t* C = counts + 2 * J.cnt_off;
  uint32_t* S = counts + 2 * J.cnt_off + 2 * nblk * kNB;
  uint32_t t = 0;
#pragma unroll 8
  for (int64_t b = b0; b < b1; ++b) t += C[b * kNB + threadIdx.x];
  S[blockIdx.x * kNB + threadIdx.x] = t;
}

__global__ __launch_bounds__(kNB) void k_sort_scan(const tpe_job* __restrict__ jobs,
                                                   uint32_t* __restrict__ counts) {
  __shared__ uint32_t tot[kNB];
  const tpe_job J = jobs[blockIdx.x];
  const int64_t nblk = sort_nblk(J);
  const int nch = (int)((nblk + kScanChunk - 1) / kScanChunk);
  uint32_t* S = counts + 2 * J.cnt_off + 2 * nblk * kNB;
  const int bin = threadIdx.x;
  uint32_t t = 0;
  for (int c = 0; c < nch; ++c) t += S[c * kNB + bin];
  tot[bin] = t;
  __syncthreads();
  // inclusive Hillis-Steele scan over bins
  for (int d = 1; d < kNB; d <<= 1) {
    const uint32_t v = bin >= d ? tot[bin - d] : 0u;
    __syncthreads();
    tot[bin] += v;
    __syncthreads();
  }
  uint32_t run = tot[bin] - t;  // exclusive
  for (int c = 0; c < nch; ++c) {
    const uint32_t v = S[c * kNB + bin];
    S[c * kNB + bin] = run;
    run += v;
  }
}

__global__ __launch_bounds__(kNB) void k_sort_offsets(const tpe_job* __restrict__ jobs,
                                                      uint32_t* __restrict__ counts) {
  const tpe_job J = jobs[blockIdx.y];
  const int64_t nblk = sort_nblk(J);
  const int64_t b0 = (int64_t)blockIdx.x * kScanChunk;
  if (b0 >= nblk) return;
  const int64_t b1 = min(nblk, b0 + kScanChunk);
  const uint32_t* C = counts + 2 * J.cnt_off;
  uint32_t* O = counts + 2 * J.cnt_off + nblk * kNB;
  const uint32_t* S = counts + 2 * J.cnt_off + 2 * nblk * kNB;
  uint32_t run = S[blockIdx.x * kNB + threadIdx.x];
  for (int64_t b = b0; b < b1; ++b) {
    O[b * kNB + threadIdx.x] = run;
    run += C[b * kNB + threadIdx.x];
  }
}

// K3: bucket the block's candidates in LDS by bin, then write each bin's run
// contiguously to its global slot range (coalesced runs instead of scattered
// 4-byte stores)
__global__ __launch_bounds__(kBS) void k_sort_scatter(const tpe_job* __restrict__ jobs,
                                                      const uint32_t* __restrict__ counts,
                                                      const float* __restrict__ gen,
                                                      float* __restrict__ sorted_x,
                                                      uint32_t* __restrict__ sorted_i) {
  __shared__ uint32_t lstart[kNB], cur[kNB], goff[kNB];
  __shared__ float sx[kSortPer];
  __shared__ uint32_t si[kSortPer];
  __shared__ uint16_t sb[kSortPer];
  __shared__ uint32_t part[kBS];
  const tpe_job J = jobs[blockIdx.y];
  const int64_t base = (int64_t)blockIdx.x * kSortPer;
  if (base >= J.n_cand) return;
  const int64_t nblk = (J.n_cand + kSortPer - 1) / kSortPer;
  const uint32_t* C = counts + 2 * J.cnt_off + (int64_t)blockIdx.x * kNB;
  const uint32_t* O = counts + 2 * J.cnt_off + nblk * kNB + (int64_t)blockIdx.x * kNB;
  // local exclusive scan of this block's bin counts (kNB = 2 * kBS)
  const uint32_t c0 = C[2 * threadIdx.x], c1 = C[2 * threadIdx.x + 1];
  part[threadIdx.x] = c0 + c1;
  goff[2 * threadIdx.x] = O[2 * threadIdx.x];
  goff[2 * threadIdx.x + 1] = O[2 * threadIdx.x + 1];
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int t = 0; t < kBS; ++t) {
      const uint32_t c = part[t];
      part[t] = acc;
      acc += c;
    }
  }
  __syncthreads();
  lstart[2 * threadIdx.x] = cur[2 * threadIdx.x] = part[threadIdx.x];
  lstart[2 * threadIdx.x + 1] = cur[2 * threadIdx.x + 1] = part[threadIdx.x] + c0;
  __syncthreads();
  const float lo = (float)J.bin_lo, scale = (float)(kNB / (J.bin_hi - J.bin_lo));
  const int n = (int)min((int64_t)kSortPer, J.n_cand - base);
  for (int r = 0; r < kSortR; ++r) {
    const int e = r * kBS + threadIdx.x;
    if (e >= n) break;
    const float x = gen[J.sort_off + base + e];  // (the mixture coordinate)
    const int b = bin_of(x, lo, scale);
    const uint32_t lp = atomicAdd(&cur[b], 1u);
    sx[lp] = x;
    si[lp] = (uint32_t)(base + e);
    sb[lp] = (uint16_t)b;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < n; e += kBS) {
    const int b = sb[e];
    const uint32_t g = goff[b] + (uint32_t)(e - lstart[b]);
    sorted_x[J.sort_off + g] = sx[e];
    sorted_i[J.sort_off + g] = si[e];
  }
}

// first k with a[k] > v (a non-decreasing)
__device__ __forceinline__ int first_greater(const float* a, int n, float v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] > v) hi = mid; else lo = mid + 1;
  }
  return lo;
}

__global__ __launch_bounds__(kBS) void k_score_sorted(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const float4* __restrict__ coef32, const float4* __restrict__ coef32n,
    const float4* __restrict__ wide32, const float* __restrict__ pm,
    const float* __restrict__ sm, const float* __restrict__ sorted_x,
    const uint32_t* __restrict__ sorted_i, tpe_best* __restrict__ partial,
    unsigned long long* __restrict__ pairs) {
  __shared__ float4 tile[kTile32];
  __shared__ BestT red[kBS / kWave];
  __shared__ float fred[3][kBS / kWave];
  __shared__ int win[2];
  __shared__ float yr[2];
  __shared__ int cnt[kTile32 / kWave];
  __shared__ float lred[2][kBS / kWave];
  const tpe_job J = jobs[blockIdx.y];
  tpe_best* P = partial + (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  const int64_t base = (int64_t)blockIdx.x * (kBS * kR32);
  if (base >= J.n_cand) {
    if (threadIdx.x == 0) *P = empty_best();
    return;
  }
  const tpe_seg SB = segs[J.below], SA = segs[J.above];
  const bool lgmm = J.family == TPE_LGMM1;
  float x[kR32], y[kR32];
  uint32_t li[kR32];
  float ymin = INFINITY, ymax = -INFINITY, vmin = INFINITY;
  const float4 cp = coef32[SA.comp_off + SA.prior_pos];
  const float cen = (float)SA.center;
  int nvalid = 0;
#pragma unroll
  for (int r = 0; r < kR32; ++r) {
    const int64_t p = base + r * kBS + threadIdx.x;
    if (p < J.n_cand) {
      x[r] = sorted_x[J.sort_off + p];  // the mixture coordinate
      li[r] = sorted_i[J.sort_off + p];
      y[r] = x[r];
      ymin = fminf(ymin, y[r]);
      ymax = fmaxf(ymax, y[r]);
      const float t = fmaf(y[r] - cen, cp.x, cp.y);
      vmin = fminf(vmin, fmaf(-t, t, cp.z));
      ++nvalid;
    } else {
      x[r] = 1.0f;
      li[r] = 0;
      y[r] = cen;
    }
  }
  // block reductions: y range and the smallest prior term
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    ymin = fminf(ymin, __shfl_xor(ymin, off, kWave));
    ymax = fmaxf(ymax, __shfl_xor(ymax, off, kWave));
    vmin = fminf(vmin, __shfl_xor(vmin, off, kWave));
  }
  const int wid = threadIdx.x / kWave;
  if (lane_id() == 0) {
    fred[0][wid] = ymin;
    fred[1][wid] = ymax;
    fred[2][wid] = vmin;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = fred[0][0], b = fred[1][0], c = fred[2][0];
    for (int k = 1; k < kBS / kWave; ++k) {
      a = fminf(a, fred[0][k]);
      b = fmaxf(b, fred[1][k]);
      c = fminf(c, fred[2][k]);
    }
    const int nc = SA.n_obs + 1;
    yr[0] = a;
    yr[1] = b;
    if (c >= (float)SA.lglob) {
      const float* PM = pm + SA.comp_off;
      const float* SMn = sm + SA.comp_off;
      win[0] = first_greater(PM, nc, a);           // first k with mu+r > ymin
      win[1] = first_greater(SMn, nc, b) - 1;      // last k with mu-r < ymax... (sm < b)
    } else {
      win[0] = -1;  // far-out block: every component, unmasked
      win[1] = nc - 1;
    }
  }
  __syncthreads();
  const int k_lo = win[0], k_hi = win[1];

  float lb[kR32], la[kR32];
  lse32<kR32>(coef32 + SB.comp_off, SB, y, lb, tile);
  Lse32<kR32> L;
  lse32_begin(L, coef32 + SA.comp_off, SA, y);
  int64_t evaluated;
  if (k_lo < 0) {
    lse32_accum(L, coef32 + SA.comp_off, 0, SA.n_obs + 1, tile);
    evaluated = SA.n_obs + 1;
  } else {
    // Block threshold.  Every candidate of the block has log2(sum) >= Lb =
    // log2(sum_k 2^min_block(v_k)) over the window + wide components.  A
    // component whose largest term over the block is below Lb - margin adds
    // less than 2^-margin of the sum; with margin = log2(n) + 20 all dropped
    // components together change the sum by < 2^-20 (relative).  Components
    // outside the window were already below 2^(lglob - 40) (tpe_fit.hip).
    const float xlo = yr[0] - cen, xhi = yr[1] - cen;
    float m = -INFINITY, sacc = 0.0f;
    auto add = [&](const float4 cc) {
      const float v = term_min(cc, xlo, xhi);
      if (v > m) {
        sacc = sacc * __builtin_amdgcn_exp2f(m - v) + 1.0f;
        m = v;
      } else if (v > -INFINITY) {
        sacc += __builtin_amdgcn_exp2f(v - m);
      }
    };
    for (int k = k_lo + (int)threadIdx.x; k <= k_hi; k += kBS) add(coef32n[SA.comp_off + k]);
    for (int k = threadIdx.x; k < SA.n_wide; k += kBS) add(wide32[SA.comp_off + k]);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const float mo = __shfl_xor(m, off, kWave), so = __shfl_xor(sacc, off, kWave);
      const float mn = fmaxf(m, mo);
      sacc = (mn == -INFINITY) ? 0.0f
                               : sacc * __builtin_amdgcn_exp2f(m - mn) + so * __builtin_amdgcn_exp2f(mo - mn);
      m = mn;
    }
    if (lane_id() == 0) {
      lred[0][wid] = m;
      lred[1][wid] = sacc;
    }
    __syncthreads();
    float mb = -INFINITY;
    for (int w = 0; w < kBS / kWave; ++w) mb = fmaxf(mb, lred[0][w]);
    float sb = 0.0f;
    for (int w = 0; w < kBS / kWave; ++w)
      if (lred[0][w] > -INFINITY) sb += lred[1][w] * __builtin_amdgcn_exp2f(lred[0][w] - mb);
    const float margin = __builtin_amdgcn_logf((float)(SA.n_obs + 1)) + 20.0f;
    const float thr = (mb > -INFINITY) ? mb + __builtin_amdgcn_logf(sb) - margin : -INFINITY;
    evaluated = 0;
    if (k_hi >= k_lo)
      evaluated = lse32_accum_pruned(L, coef32n + SA.comp_off, k_lo, k_hi + 1, tile, cnt, xlo,
                                     xhi, thr);
    lse32_accum(L, wide32 + SA.comp_off, 0, SA.n_wide, tile);
    evaluated += SA.n_wide;
  }
  lse32_end(L, SA, la);

  BestT b{0.0, -1, 0.0};
#pragma unroll
  for (int r = 0; r < kR32; ++r) {
    const int64_t p = base + r * kBS + threadIdx.x;
    if (p >= J.n_cand) continue;
    double bl = lb[r], al = la[r];
    if (lgmm) {  // lognormal_lpdf's -log(x) (tpe.py:214-216): log of exp(y) is y
      bl -= (double)y[r];
      al -= (double)y[r];
    }
    best_update(b, bl - al, J.cand_base + (int64_t)li[r],
                lgmm ? exp((double)x[r]) : (double)x[r]);
  }
  b = block_best<kBS>(b, red);
  if (threadIdx.x == 0) {
    *P = tpe_best{b.score, b.index, b.value, 0};
    if (pairs) {
      const int64_t n = min((int64_t)(kBS * kR32), J.n_cand - base);
      atomicAdd(pairs, (unsigned long long)(n * (evaluated + SB.n_obs + 1)));
    }
  }
  (void)nvalid;
}

// ---------------------------------------------------------------------------
// quantized labels
// ---------------------------------------------------------------------------
// POW2: every job draws in fp32 (TPE_F_DRAW32) with q a power of two and at
// most kLatLds lattice slots (C3's quniform labels) -- slots come from rintf
// in fp32 and the kernel carries no fp64 slot code (fewer registers); the
// general instantiation handles the rest.  lfirst is dynamic LDS sized by the
// host to the largest lattice of the launch (up to kLatLds slots).
__host__ __device__ __forceinline__ bool lattice_pow2(const tpe_job& j) {
  int qe;
  return (j.flags & TPE_F_DRAW32) && frexp(j.q, &qe) == 0.5 && qe > -100 && qe < 100 &&
         j.lat_n <= kLatLds;
}

__device__ __forceinline__ void score_slots(const tpe_job* __restrict__ jobs,
                                            const tpe_seg* __restrict__ segs,
                                            const double* __restrict__ w,
                                            const double* __restrict__ mu,
                                            const double* __restrict__ sigma,
                                            tpe_best* __restrict__ partial, int job, int64_t sb,
                                            int64_t nper, double* sh,
                                            const double* __restrict__ P,
                                            const double* __restrict__ Sm);
constexpr int kSlotsPerBlock = kBS / kWave;  // score_slots: lattice slots per block

// Candidates [start, min(n_cand, limit)) of every job (start a multiple of the
// kBS * kLatR tile); need (nullable): only the jobs whose flag is set.
// slot_n > 0 (tpe_lattice_suggest's first launch): the grid's first
// slot_n * n_jobs blocks score the lattice slots instead (score_slots; the
// slot scores do not depend on the draws, so they share the launch)
template <bool POW2>
#ifndef TPE_LAT_WPE  // diagnostic builds: waves-per-EU target of the lattice sampler
#define TPE_LAT_WPE 4     // (power-of-two candidate counts: 128 VGPRs, no spill)
#endif
__global__ __launch_bounds__(kBS) __attribute__((amdgpu_waves_per_eu(POW2 ? TPE_LAT_WPE : 1))) void k_lattice_sample(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const double* __restrict__ mu, const double* __restrict__ sigma,
    const double* __restrict__ wcdf, unsigned long long* __restrict__ slot_first,
    int32_t* __restrict__ err, int n_tiles, int n_jobs, int64_t start, int64_t limit,
    const int32_t* __restrict__ need, const double* __restrict__ w,
    tpe_best* __restrict__ slot_part, int slot_n, const double* __restrict__ qP,
    const double* __restrict__ qS) {
  extern __shared__ uint32_t lfirst[];
  __shared__ MixLds s_mix;
  __shared__ alignas(16) float s_stage[kLatR * kBS];  // (also the slot blocks' fp64 scratch)
  __shared__ uint16_t s_list[(kBS / kWave) * kRetryList];
  const int64_t spj = slot_n;  // slot blocks per job (score_slots)
  const int64_t slot_blocks = spj * n_jobs;
  if ((int64_t)blockIdx.x < slot_blocks) {  // block-uniform
    const int job = (int)(blockIdx.x / spj);
    const int64_t sb = (int64_t)blockIdx.x - (int64_t)job * spj;
    score_slots(jobs, segs, w, mu, sigma, slot_part, job, sb, slot_n,
                reinterpret_cast<double*>(s_stage), qP, qS);
    return;
  }
  const unsigned bid = (unsigned)((int64_t)blockIdx.x - slot_blocks);
  // one (job, tile) work item
  auto tile = [&](int job, int64_t base) __attribute__((always_inline)) {
    const tpe_job J = jobs[job];
    const int64_t n_lim = min(J.n_cand, limit);
    if (base >= n_lim || base < start) return;
    const tpe_seg SB = segs[J.below];
    const bool lgmm = J.family == TPE_LGMM1;
    const bool lo_on = J.flags & TPE_F_LOW, hi_on = J.flags & TPE_F_HIGH;
    // the first kLatLds slots of the lattice are deduplicated in LDS (for the
    // wide lattices of unbounded labels that is where the mass sits); slots
    // beyond go to the global marks directly, each read before its atomic
    const int n_loc = (int)min((int64_t)kLatLds, J.lat_n);
    for (int s = threadIdx.x; s < n_loc; s += kBS) lfirst[s] = 0xFFFFFFFFu;
    const Mix M = stage_mix(SB, wcdf, mu, sigma, s_mix);
    __syncthreads();
    if constexpr (POW2) {
      // kLatR consecutive candidates per thread (draw32_pairs); q a power of two:
      // x * (1/q) is exact in fp32, so rintf gives np.round(x / q) (tpe.py:106)
      // exactly and the slot needs no fp64 work
      const int64_t t0 = base + (int64_t)threadIdx.x * kLatR;
      const int nv = (int)max((int64_t)0, min((int64_t)kLatR, n_lim - t0));
      float x[kLatR];
      draw32_pairs<kLatR>(M, J.key, J.cand_base + t0, nv, lo_on, hi_on, (float)J.low,
                          (float)J.high, lgmm, s_stage + (threadIdx.x / kWave) * (kLatR * kWave), s_list + (threadIdx.x / kWave) * kRetryList,
                          x);
      const float inv_q32 = (float)(1.0 / J.q);
      const int kmin = (int)J.lat_kmin, nl = (int)J.lat_n;
#pragma unroll
      for (int r = 0; r < kLatR; ++r) {
        if (r >= nv) continue;
        const float t = rintf(x[r] * inv_q32);
        const int slot = (fabsf(t) < 2147483648.0f) ? (int)t - kmin : -1;
        if (slot < 0 || slot >= nl) {
          atomicOr(err, 2);
          continue;
        }
        // most draws land on slots already holding a smaller index: a plain read
        // first keeps the atomics (and their same-address serialisation) rare
        const uint32_t rel = (uint32_t)(t0 + r - base);
#ifdef TPE_DIAG_NO_MARK  // diagnostic builds only: slots computed, not marked
        if (rel == 0xFFFFFFFFu) lfirst[slot] = rel;
#else
        if (rel < lfirst[slot]) atomicMin(&lfirst[slot], rel);
#endif
      }
    } else {
      // np.round(x / q) (tpe.py:106) without a division per draw: t = x * (1/q) is
      // within 3.4e-16 |t| of fl(x / q), so rint(t) == rint(fl(x / q)) unless
      // fl(x / q) sits that close to a half-integer -- those few redo the division
      const double inv_q = 1.0 / J.q;
      auto mark = [&](double v, int64_t li) {
        const double t = v * inv_q;
        double k = rint(t);
        if (fabs(fabs(t - k) - 0.5) <= 8e-16 * fabs(t)) k = rint(v / J.q);
        const int64_t slot = (int64_t)k - J.lat_kmin;
        if (slot < 0 || slot >= J.lat_n) {
          atomicOr(err, 2);
          return;
        }
        if (slot < n_loc) {
          const uint32_t rel = (uint32_t)(li - base);
          if (rel < lfirst[slot]) atomicMin(&lfirst[slot], rel);
        } else {
          unsigned long long* dst = &slot_first[J.lat_off + slot];
          const unsigned long long g = (unsigned long long)(J.cand_base + li);
          if (g < __hip_atomic_load(dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(dst, g);
        }
      };
      if (J.flags & TPE_F_DRAW32) {
        const int64_t t0 = base + (int64_t)threadIdx.x * kLatR;
        const int nv = (int)max((int64_t)0, min((int64_t)kLatR, n_lim - t0));
        float x[kLatR];
        draw32_pairs<kLatR>(M, J.key, J.cand_base + t0, nv, lo_on, hi_on, (float)J.low,
                            (float)J.high, lgmm, s_stage + (threadIdx.x / kWave) * (kLatR * kWave), s_list + (threadIdx.x / kWave) * kRetryList,
                            x);
#pragma unroll
        for (int r = 0; r < kLatR; ++r)
          if (r < nv) mark((double)x[r], t0 + r);
      } else {
        for (int r = 0; r < kLatR; ++r) {
          const int64_t li = base + r * kBS + threadIdx.x;
          if (li >= n_lim) break;
          double v = draw64(M, J.key, J.cand_base + li, lo_on, hi_on, J.low, J.high);
          if (lgmm) v = exp(v);
          mark(v, li);
        }
      }
    }
    __syncthreads();
    // blocks run roughly in index order, so the global slot mostly holds a
    // smaller index already: an agent-scope load first keeps the (cross-XCD)
    // atomics to the blocks that improve a slot
#ifdef TPE_DIAG_NO_FLUSH  // diagnostic builds only: block results dropped
    if (n_loc > 0x7FFFFFF0)
#endif
    for (int s = threadIdx.x; s < n_loc; s += kBS) {
      const uint32_t f = lfirst[s];
      if (f == 0xFFFFFFFFu) continue;
      unsigned long long* dst = &slot_first[J.lat_off + s];
      const unsigned long long g = (unsigned long long)(J.cand_base + base + f);
      if (g < __hip_atomic_load(dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(dst, g);
    }
  };  // tile
  const int64_t tb = (int64_t)kBS * kLatR;
  if (!need) {
    // XCD-aware work order (as k_score_table): each XCD sweeps a contiguous
    // eighth of the (job, tile) list, so a job's first-index atomics stay in
    // few XCDs' L2s
    const int64_t W = (int64_t)n_tiles * n_jobs, per = (W + 7) / 8;
    const int64_t wi = (int64_t)(bid & 7) * per + (bid >> 3);
    if (wi >= W) return;
    const int job = (int)(wi / n_tiles);
    tile(job, (wi - (int64_t)job * n_tiles) * tb);
  } else {
    // the conditional rest of the streams: a grid-stride loop over the tiles
    // of the jobs whose flag is set, so a launch whose jobs are all settled is
    // a small grid that reads the flags and exits (a one-tile-per-block grid
    // of ~10^4 such blocks cost ~80 us of dispatch)
    for (int job = 0; job < n_jobs; ++job) {
      if (!need[job]) continue;  // block-uniform
      for (int64_t t = bid; t < n_tiles; t += (int64_t)gridDim.x - slot_blocks) {
        __syncthreads();  // the previous tile's LDS reads are done
        tile(job, t * tb);
      }
    }
  }
}

__global__ __launch_bounds__(kBS) void k_lattice_compact(
    const tpe_job* __restrict__ jobs, const unsigned long long* __restrict__ slot_first,
    double* __restrict__ vals, int64_t* __restrict__ firsts,
    unsigned long long* __restrict__ counts) {
  const tpe_job J = jobs[blockIdx.y];
  const int64_t s = (int64_t)blockIdx.x * kBS + threadIdx.x;
  if (s >= J.lat_n) return;
  const unsigned long long f = slot_first[J.lat_off + s];
  if (f == ~0ull) return;
  const unsigned long long pos = atomicAdd(&counts[blockIdx.y], 1ull);
  vals[J.lat_off + pos] = (double)(J.lat_kmin + s) * J.q;  // np.round(x/q) * q
  firsts[J.lat_off + pos] = (int64_t)f;
}

// Component windows of the quantized log-mass (round 5).  A component whose
// two erf arguments are both beyond +-6.5 contributes exactly 0 (qlpdf skips
// it), i.e. unless mu - b < ub and mu + b > lb, b = 6.5 max(sqrt2 sigma, EPS).
// The means are sorted, so with P[k] = max_{j<=k} (mu_j + b_j) and
// S[k] = min_{j>=k} (mu_j - b_j) (both non-decreasing; k_qreach) every
// component that can contribute lies in [first k with P[k] > lb, last k with
// S[k] < ub] -- found by a block-wide search -- and qlpdf loops over that
// window only.  Each thread still visits its own components in the same
// order and skips the same ones, so the sums are bit-identical to the full
// loop's.  A NaN mean or sigma gives P = +inf / S = -inf from there on, which
// keeps NaN components (sorted last) inside every window.
constexpr int kQB = 256;  // k_qreach block: one per segment (small: it runs beside the table build)
constexpr int kQPer = 8;   // components per thread per pass (all its loads issued together)
__device__ __forceinline__ double qreach_b(double s) { return 6.5 * fmax(__dmul_rn(kSqrt2, s), kEps); }

// inclusive block scans over the threads' values in thread order: max from
// the front (prefix) or min from the back (suffix); wave DPP / shuffles, then
// the waves' totals through LDS
__device__ __forceinline__ double block_prefix_max(double v, double* sw) {
  const int lane = lane_id(), wid = threadIdx.x / kWave;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const double u = __shfl_up(v, o, kWave);
    if (lane >= o) v = fmax(v, u);
  }
  __syncthreads();
  if (lane == kWave - 1) sw[wid] = v;
  __syncthreads();
  for (int w = 0; w < wid; ++w) v = fmax(v, sw[w]);
  return v;
}
__device__ __forceinline__ double block_suffix_min(double v, double* sw) {
  const int lane = lane_id(), wid = threadIdx.x / kWave;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const double u = __shfl_down(v, o, kWave);
    if (lane + o < kWave) v = fmin(v, u);
  }
  __syncthreads();
  if (lane == 0) sw[wid] = v;
  __syncthreads();
  for (int w = wid + 1; w < kQB / kWave; ++w) v = fmin(v, sw[w]);
  return v;
}

// One block per (job, mixture, direction): blockIdx.x = 4 job + 2 dir + mix,
// dir 0 the prefix max P from the front, dir 1 the suffix min S from the
// back; the next pass's loads are issued before this pass's scan (the block
// walks ~50 passes of 2 048 components at C5's 10^5: each otherwise waited
// one load round trip)
__global__ __launch_bounds__(kQB) void k_qreach(const tpe_job* __restrict__ jobs,
                                               const tpe_seg* __restrict__ segs,
                                               const double* __restrict__ mu,
                                               const double* __restrict__ sigma,
                                               double* __restrict__ P, double* __restrict__ Sm) {
  __shared__ double sw[kQB / kWave];
  const tpe_job J = jobs[blockIdx.x >> 2];
  const bool suffix = (blockIdx.x >> 1) & 1;
  const tpe_seg S = segs[(blockIdx.x & 1) ? J.above : J.below];
  const int nc = S.n_obs + 1;
  const double* m = mu + S.comp_off;
  const double* g = sigma + S.comp_off;
  constexpr int kPass = kQB * kQPer;
  const int npass = (nc + kPass - 1) / kPass;
  // thread t's raw loads of components base + t * kQPer + i
  auto load = [&](int base, double (&mk)[kQPer], double (&gk)[kQPer]) __attribute__((always_inline)) {
    const int a = base + (int)threadIdx.x * kQPer;
#pragma unroll
    for (int i = 0; i < kQPer; ++i) {
      const int k = a + i;
      mk[i] = k < nc ? m[k] : 0.0;
      gk[i] = k < nc ? g[k] : 0.0;
    }
  };
  // (hi = mu + b for the prefix, lo = mu - b for the suffix; NaN -> +inf / -inf)
  auto value = [&](int k, double mk, double gk) -> double {
    const double r = qreach_b(gk);
    const bool ok = mk == mk && r == r;
    if (!suffix) return k >= nc ? -INFINITY : (ok ? mk + r : INFINITY);
    return k >= nc ? INFINITY : (ok ? mk - r : -INFINITY);
  };
  double nm[kQPer], ng[kQPer];
  load(suffix ? (npass - 1) * kPass : 0, nm, ng);
  double carry = suffix ? INFINITY : -INFINITY;  // the earlier passes' max / later passes' min
  for (int q = 0; q < npass; ++q) {  // block-uniform
    const int ps = suffix ? npass - 1 - q : q;
    const int base = ps * kPass;
    const int a = base + (int)threadIdx.x * kQPer;
    double v[kQPer];
#pragma unroll
    for (int i = 0; i < kQPer; ++i) v[i] = value(a + i, nm[i], ng[i]);
    if (q + 1 < npass) load((suffix ? ps - 1 : ps + 1) * kPass, nm, ng);  // (in flight)
    if (!suffix) {
#pragma unroll
      for (int i = 1; i < kQPer; ++i) v[i] = fmax(v[i], v[i - 1]);
      const double incl = block_prefix_max(v[kQPer - 1], sw);
      double before = __shfl_up(incl, 1, kWave);  // max over the threads before this one
      if (lane_id() == 0) {
        before = -INFINITY;
        for (int w = 0; w < (int)threadIdx.x / kWave; ++w) before = fmax(before, sw[w]);
      }
      before = fmax(before, carry);
#pragma unroll
      for (int i = 0; i < kQPer; ++i)
        if (a + i < nc) P[S.comp_off + a + i] = fmax(before, v[i]);
      for (int w = 0; w < kQB / kWave; ++w) carry = fmax(carry, sw[w]);  // (the pass's total)
    } else {
#pragma unroll
      for (int i = kQPer - 2; i >= 0; --i) v[i] = fmin(v[i], v[i + 1]);
      const double incl = block_suffix_min(v[0], sw);
      double after = __shfl_down(incl, 1, kWave);  // min over the threads after this one
      if (lane_id() == kWave - 1) {
        after = INFINITY;
        for (int w = (int)threadIdx.x / kWave + 1; w < kQB / kWave; ++w) after = fmin(after, sw[w]);
      }
      after = fmin(after, carry);
#pragma unroll
      for (int i = 0; i < kQPer; ++i)
        if (a + i < nc) Sm[S.comp_off + a + i] = fmin(after, v[i]);
      for (int w = 0; w < kQB / kWave; ++w) carry = fmin(carry, sw[w]);  // (the pass's total)
    }
    __syncthreads();
  }
}

// normal_cdf(x, m, s) (GMM1) or lognormal_cdf_logx(x = log of the bound, m,
// s) (LGMM1) with one erf: the two share z = (x - m) / max(sqrt2 s, EPS) and
// differ only in how erf(z) is combined (numpy's order for each: 0.5 * (1 +
// e), tpe.py:109-114; 0.5 + 0.5 * e, tpe.py:186-205) -- one inlined erf per
// bound instead of one per family and bound (register pressure)
__device__ __forceinline__ double qcdf(bool lg, double x, double m, double s) {
  const double bottom = fmax(__dmul_rn(kSqrt2, s), kEps);
  const double e = erf((x - m) / bottom);
  return lg ? __dadd_rn(0.5, __dmul_rn(0.5, e)) : __dmul_rn(0.5, __dadd_rn(1.0, e));
}

// how many leading k in [0, n) satisfy pred (pred holds on a prefix): a
// wave-wide search, kWave probes per round (three rounds for n <= 2^18); call
// by the whole wave (n wave-uniform)
template <typename F>
__device__ __forceinline__ int wave_prefix_count(int n, F pred) {
  int lo = 0, len = n;
  const int t = lane_id();
  while (len > 0) {  // wave-uniform
    const int stride = (len + kWave - 1) / kWave;
    const int nprobe = (len + stride - 1) / stride;
    const int p = lo + min((t + 1) * stride, len) - 1;
    // pred holds on a prefix, so the lanes whose probe holds are a prefix too
    const int c = __popcll(__ballot(t < nprobe && pred(p)));
    if (c == nprobe) return lo + len;
    lo += c * stride;
    len = min(stride, len - c * stride) - 1;  // (probe c failed: the boundary is before it)
  }
  return lo;
}

// quantized mixture log-mass of one value, one WAVE, lanes stride components
// (lane l takes components k = l mod 64, in order).  tpe.py:159-174 (GMM1) and
// :288-305 (LGMM1): sum_k w_k*cdf(ub) - w_k*cdf(lb), then log(prob) -
// log(p_accept).  P / Sm (nullable): k_qreach's arrays -- the loop then
// covers the value's component window only, entered at the full loop's pass
// that holds the window's first component, so every lane visits the same
// components in the same order and skips the same ones: the same sums, bit
// for bit.  The lanes' partial sums meet in one fixed butterfly.  Round 6: a
// wave per value instead of a 256-thread block (C4's ~370-component windows
// left a block's threads one or two components each, behind eight block-wide
// barriers per value).  Every lane returns the value.
__device__ __forceinline__ double qlpdf(const tpe_job& J, const tpe_seg& S,
                                        const double* __restrict__ w,
                                        const double* __restrict__ mu,
                                        const double* __restrict__ sigma, double x,
                                        int32_t* err,
                                        const double* __restrict__ P = nullptr,
                                        const double* __restrict__ Sm = nullptr) {
  const bool lg = J.family == TPE_LGMM1;
  const double hq = J.q / 2.0;
  double ub = x + hq, lb = x - hq;
  if (J.flags & TPE_F_HIGH) ub = fmin(ub, lg ? exp(J.high) : J.high);
  if (J.flags & TPE_F_LOW) lb = fmax(lb, lg ? exp(J.low) : J.low);
  double lub = 0.0, llb = 0.0;
  const int lane = lane_id();
  if (lg) {
    lb = fmax(0.0, lb);
    if (ub < 0.0 && lane == 0 && err) atomicOr(err, 1);  // tpe.py:196-197
    lub = log(ub < kEps ? kEps : ub);
    llb = log(lb < kEps ? kEps : lb);
  }
  const int nc = S.n_obs + 1;
  double acc = 0.0;
  const double xu = lg ? lub : ub, xl = lg ? llb : lb;
  // kQU components per lane per pass, their loads issued together
  constexpr int kQU = 4;
  constexpr int kPassQ = kQU * kWave;
  int kbeg = 0, kend = nc;
  const double dl = 1e-9 * (1.0 + fabs(xl) + fabs(xu));  // (covers the fp64 rounding of mu +- b)
  const double wa = xl - dl, wb = xu + dl;
  if (P && wa == wa && wb == wb) {  // wave-uniform
    kbeg = wave_prefix_count(nc, [&](int k) { return P[S.comp_off + k] <= wa; });
    kend = max(kbeg, wave_prefix_count(nc, [&](int k) { return Sm[S.comp_off + k] < wb; }));
  }
  for (int k0 = kbeg / kPassQ * kPassQ + lane; k0 < kend; k0 += kPassQ) {
    double mq[kQU], sq[kQU];
#pragma unroll
    for (int u = 0; u < kQU; ++u) {
      const int k = k0 + u * kWave;
      const bool in = k >= kbeg && k < kend;
      mq[u] = in ? mu[S.comp_off + k] : INFINITY;
      sq[u] = in ? sigma[S.comp_off + k] : 1.0;
    }
#pragma unroll
    for (int u = 0; u < kQU; ++u) {
      const double m = mq[u], s = sq[u];
      // both erf arguments beyond +-6.5 (erf exactly +-1 in fp64): the two cdf
      // values are equal and the term w*cu - w*cl is exactly 0 -- skip it
      // (padding: m = +inf is skipped)
      const double b65 = 6.5 * fmax(__dmul_rn(kSqrt2, s), kEps);
      if (xl - m >= b65 || xu - m <= -b65 || m == INFINITY) continue;
      const double wk = w[S.comp_off + k0 + u * kWave];
      const double cu = qcdf(lg, xu, m, s), cl = qcdf(lg, xl, m, s);
      acc += __dsub_rn(__dmul_rn(wk, cu), __dmul_rn(wk, cl));  // two-stage, as tpe.py:171-173
    }
  }
#pragma unroll
  for (int o = kWave / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, kWave);
  return log(acc) - log(S.p_accept);
}

// how many leading k in [0, n) satisfy pred (pred holds on a prefix): a
// block-wide search, kBS probes per round (three rounds for n <= 2^24)
template <typename F>
__device__ __forceinline__ int prefix_count(int n, F pred) {
  int lo = 0, len = n;
  while (len > 0) {  // block-uniform
    const int stride = (len + kBS - 1) / kBS;
    const int nprobe = (len + stride - 1) / stride;
    const int t = threadIdx.x;
    const int p = lo + min((t + 1) * stride, len) - 1;
    const int c = __syncthreads_count(t < nprobe && pred(p));
    if (c == nprobe) return lo + len;
    lo += c * stride;
    len = min(stride, len - c * stride) - 1;  // (probe c failed: the boundary is before it)
  }
  return lo;
}

// The same log-mass with the whole BLOCK on one value (threads stride the
// components, k = t mod 256; block-wide window search and sum): for mixtures
// of more than kQBig components (C3's 10^4, C5's 10^5), whose windows give a wave
// thousands of CDF pairs.  Its own bits (another lane map), chosen per
// mixture size alone (qlpdf_big), so every kernel scoring a value picks the
// same variant.
__device__ __forceinline__ double qlpdf_block(const tpe_job& J, const tpe_seg& S,
                                        const double* __restrict__ w,
                                        const double* __restrict__ mu,
                                        const double* __restrict__ sigma, double x,
                                        int32_t* err, double* sh,
                                        const double* __restrict__ P = nullptr,
                                        const double* __restrict__ Sm = nullptr) {
  const bool lg = J.family == TPE_LGMM1;
  const double hq = J.q / 2.0;
  double ub = x + hq, lb = x - hq;
  if (J.flags & TPE_F_HIGH) ub = fmin(ub, lg ? exp(J.high) : J.high);
  if (J.flags & TPE_F_LOW) lb = fmax(lb, lg ? exp(J.low) : J.low);
  double lub = 0.0, llb = 0.0;
  if (lg) {
    lb = fmax(0.0, lb);
    if (ub < 0.0 && threadIdx.x == 0 && err) atomicOr(err, 1);  // tpe.py:196-197
    lub = log(ub < kEps ? kEps : ub);
    llb = log(lb < kEps ? kEps : lb);
  }
  const int nc = S.n_obs + 1;
  double acc = 0.0;
  const double xu = lg ? lub : ub, xl = lg ? llb : lb;
  // kQU components per thread per pass, their loads issued together (the
  // skip test is cheap; a serial load -> test chain per component is what
  // bounded this loop)
  constexpr int kQU = 4;
  int kbeg = 0, kend = nc;
  const double dl = 1e-9 * (1.0 + fabs(xl) + fabs(xu));  // (covers the fp64 rounding of mu +- b)
  const double wa = xl - dl, wb = xu + dl;
  if (P && wa == wa && wb == wb) {  // block-uniform
    kbeg = prefix_count(nc, [&](int k) { return P[S.comp_off + k] <= wa; });
    kend = max(kbeg, prefix_count(nc, [&](int k) { return Sm[S.comp_off + k] < wb; }));
  }
  // the full loop's thread-to-component map, entered at the window's first pass
  for (int k0 = kbeg / (kQU * kBS) * (kQU * kBS) + threadIdx.x; k0 < kend; k0 += kQU * kBS) {
    double mq[kQU], sq[kQU];
#pragma unroll
    for (int u = 0; u < kQU; ++u) {
      const int k = k0 + u * kBS;
      const bool in = k >= kbeg && k < kend;
      mq[u] = in ? mu[S.comp_off + k] : INFINITY;
      sq[u] = in ? sigma[S.comp_off + k] : 1.0;
    }
#pragma unroll
    for (int u = 0; u < kQU; ++u) {
      const double m = mq[u], s = sq[u];
      // both erf arguments beyond +-6.5 (erf exactly +-1 in fp64): the two cdf
      // values are equal and the term w*cu - w*cl is exactly 0 -- skip it
      // (padding: m = +inf is skipped)
      const double b65 = 6.5 * fmax(__dmul_rn(kSqrt2, s), kEps);
      if (xl - m >= b65 || xu - m <= -b65 || m == INFINITY) continue;
      const double wk = w[S.comp_off + k0 + u * kBS];
      const double cu = qcdf(lg, xu, m, s), cl = qcdf(lg, xl, m, s);
      acc += __dsub_rn(__dmul_rn(wk, cu), __dmul_rn(wk, cl));  // two-stage, as tpe.py:171-173
    }
  }
  acc = block_sum<kBS, double>(acc, sh);
  return log(acc) - log(S.p_accept);
}

// mixtures above this many components take the block-wide log-mass
constexpr int kQBig = 4096;
__device__ __forceinline__ bool qlpdf_big(const tpe_seg& SB, const tpe_seg& SA) {
  return max(SB.n_obs, SA.n_obs) + 1 > kQBig;
}

// one wave per value (kQW values per 256-thread block): the wave shares the
// value's component CDF pairs
constexpr int kQW = kBS / kWave;

// grid (nper, n_jobs), nper = the partial entries per job (>= every job's
// count): a job of small mixtures scores value pos = kQW blockIdx.x + wave,
// one of large ones (qlpdf_big) value blockIdx.x with the whole block
__global__ __launch_bounds__(kBS) void k_score_q(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const double* __restrict__ w, const double* __restrict__ mu,
    const double* __restrict__ sigma, const double* __restrict__ vals,
    const int64_t* __restrict__ firsts, const unsigned long long* __restrict__ counts,
    double* __restrict__ out_bl, double* __restrict__ out_al, tpe_best* __restrict__ partial,
    int32_t* __restrict__ err, const double* __restrict__ qP, const double* __restrict__ qS,
    int64_t nper) {
  __shared__ double sh[kBS / kWave];
  const tpe_job J = jobs[blockIdx.y];
  const tpe_seg SB = segs[J.below], SA = segs[J.above];
  const int64_t cnt = counts ? (int64_t)counts[blockIdx.y] : J.n_cand;
  const int64_t voff = counts ? J.lat_off : J.cand_off;
  auto put = [&](int64_t pos, double bl, double al, double v) __attribute__((always_inline)) {
    const int64_t idx = firsts ? firsts[J.lat_off + pos] : J.cand_base + pos;
    if (out_bl) out_bl[J.out_off + pos] = bl;
    if (out_al) out_al[J.out_off + pos] = al;
    partial[(int64_t)blockIdx.y * nper + pos] = tpe_best{bl - al, idx, v, 0};
  };
  if (qlpdf_big(SB, SA)) {  // block-uniform: block b scores value b with every thread
    const int64_t pos = blockIdx.x;
    if (pos >= nper) return;
    if (pos >= cnt) {
      if (threadIdx.x == 0) partial[(int64_t)blockIdx.y * nper + pos] = empty_best();
      return;
    }
    const double v = vals[voff + pos];
    const double bl = qlpdf_block(J, SB, w, mu, sigma, v, err, sh, qP, qS);
    const double al = qlpdf_block(J, SA, w, mu, sigma, v, err, sh, qP, qS);
    if (threadIdx.x == 0) put(pos, bl, al, v);
    return;
  }
  // otherwise block b < nper / kQW scores values kQW b .. one per wave (the
  // grid has a block per value for the large-mixture jobs; the rest exit)
  const int64_t pos = (int64_t)blockIdx.x * kQW + threadIdx.x / kWave;
  if (pos >= nper) return;  // wave-uniform
  const bool lead = lane_id() == 0;
  if (pos >= cnt) {  // wave-uniform
    if (lead) partial[(int64_t)blockIdx.y * nper + pos] = empty_best();
    return;
  }
  const double v = vals[voff + pos];
  const double bl = qlpdf(J, SB, w, mu, sigma, v, err, qP, qS);
  const double al = qlpdf(J, SA, w, mu, sigma, v, err, qP, qS);
  if (lead) put(pos, bl, al, v);
}

// Prefix-first lattice argmax (tpe_lattice_suggest).  A lattice value's score
// does not depend on where it is drawn, and the reference's winner is the
// best-scoring value that occurs in the stream, at its first occurrence
// (np.argmax: first index of the maximum).  So after the first `prefix`
// candidates the winner is settled unless some value not yet seen scores
// strictly higher (or is NaN while the best seen is not): a value first seen
// later has a larger index and loses every tie.  score_slots scores every
// slot of the lattice (seen or not), k_lattice_decide takes the argmax over
// the seen ones and flags the jobs where an unseen slot could still win; only
// those draw the rest of their stream (the sampler with `need`) and decide
// again over everything seen.  (The slots are scored by extra blocks of the
// prefix's sampling launch, k_lattice_sample.)
// Slot block sb of job `job` (slot_n blocks per job): slots
// kSlotsPerBlock sb .. one per wave, or (mixtures past kQBig, qlpdf_big)
// slot sb with the whole block; the blocks past a job's slots exit.  sh:
// kBS / kWave doubles of LDS.  Call by the whole block.
__device__ __forceinline__ void score_slots(const tpe_job* __restrict__ jobs,
                                            const tpe_seg* __restrict__ segs,
                                            const double* __restrict__ w,
                                            const double* __restrict__ mu,
                                            const double* __restrict__ sigma,
                                            tpe_best* __restrict__ partial, int job, int64_t sb,
                                            int64_t nper, double* sh, const double* __restrict__ P,
                                            const double* __restrict__ Sm) {
  const tpe_job J = jobs[job];
  const tpe_seg SB = segs[J.below], SA = segs[J.above];
  // every slot is scored, drawn or not: a slot below 0 (the bracket under a
  // qloguniform / qlognormal lattice, never drawn) must not raise the
  // reference's negative-argument error (tpe.py:196-197) -- a drawn value
  // x = round(exp(y)/q)*q >= 0 never has ub = x + q/2 < 0, so no err here
  auto value = [&](int64_t s) { return (double)(J.lat_kmin + s) * J.q; };  // as k_lattice_compact
  if (qlpdf_big(SB, SA)) {  // block-uniform: slot sb with every thread
    const int64_t s = sb;
    if (s >= J.lat_n || s >= nper) return;
    const double v = value(s);
    const double bl = qlpdf_block(J, SB, w, mu, sigma, v, nullptr, sh, P, Sm);
    const double al = qlpdf_block(J, SA, w, mu, sigma, v, nullptr, sh, P, Sm);
    if (threadIdx.x == 0) partial[(int64_t)job * nper + s] = tpe_best{bl - al, -1, v, 0};
    return;
  }
  const int64_t s = sb * kSlotsPerBlock + threadIdx.x / kWave;
  if (s >= J.lat_n || s >= nper) return;  // wave-uniform
  const double v = value(s);
  const double bl = qlpdf(J, SB, w, mu, sigma, v, nullptr, P, Sm);
  const double al = qlpdf(J, SA, w, mu, sigma, v, nullptr, P, Sm);
  if (lane_id() == 0) partial[(int64_t)job * nper + s] = tpe_best{bl - al, -1, v, 0};
}

// Can the sampler put a draw on slot s at all?  Only unseen slots that could
// win ask; a "yes" costs the rest of the stream, a wrong "no" would cost
// parity, so the test is a superset: some below component's draw range
// (mean +- 5.8 sigma for fp32 Box-Muller draws, 8.7 for fp64 ones, widened
// for fp32 rounding) meets the slot's rounding bin, and the bin meets the
// bounds -- or holds a bound, where the sampler's last-resort clamp lands.
// (The lattice brackets the bounds with a slot on each side that no draw
// reaches; their probability mass is negative or 0/0, their score NaN.)
__device__ __forceinline__ bool slot_reachable(const tpe_job& J, const tpe_seg& SB,
                                               const double* __restrict__ mu,
                                               const double* __restrict__ sigma, int64_t s) {
  const double k = (double)(J.lat_kmin + s);
  double lo = (k - 0.5) * J.q, hi = (k + 0.5) * J.q;  // the bin of np.round(x / q) == k
  if (J.family == TPE_LGMM1) {  // the sampler's coordinate: log x
    if (!(hi > 0.0)) return false;
    lo = lo > 0.0 ? log(lo) : -INFINITY;
    hi = log(hi);
  }
  const double m = 1e-6 * (fabs(lo) + fabs(hi)) + 1e-300;
  lo -= m;
  hi += m;
  const bool lo_on = J.flags & TPE_F_LOW, hi_on = J.flags & TPE_F_HIGH;
  if (lo_on && hi < J.low) return false;
  if (hi_on && lo > J.high) return false;
  if ((lo_on && lo <= J.low && J.low <= hi) || (hi_on && lo <= J.high && J.high <= hi))
    return true;
  const double z = (J.flags & TPE_F_DRAW32) ? 5.8 : 8.7;
  for (int c = 0; c <= SB.n_obs; ++c) {
    const double mc = mu[SB.comp_off + c], r = z * sigma[SB.comp_off + c];
    const double mm = 1e-6 * (fabs(mc) + r);
    if (mc - r - mm <= hi && lo <= mc + r + mm) return true;
  }
  return false;
}

// one block per job; seen-ness and first indices from slot_first.  pass 0:
// best over the seen slots, need = an unseen, reachable slot could win (jobs
// whose whole stream was the prefix never need more); pass 1 (need jobs
// only): best over every slot seen in the whole stream
__global__ __launch_bounds__(kBS) void k_lattice_decide(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const double* __restrict__ mu, const double* __restrict__ sigma,
    const tpe_best* __restrict__ partial, int64_t nper,
    const unsigned long long* __restrict__ slot_first, int64_t prefix, int pass,
    int32_t* __restrict__ need, tpe_best* __restrict__ best) {
  __shared__ BestT red[kBS / kWave];
  const int j = blockIdx.x;
  if (pass == 1 && !need[j]) return;  // block-uniform
  const tpe_job J = jobs[j];
  const tpe_best* P = partial + (int64_t)j * nper;
  const unsigned long long* F = slot_first + J.lat_off;
  BestT b{0.0, -1, 0.0};
  for (int64_t s = threadIdx.x; s < J.lat_n; s += kBS) {
    const unsigned long long f = F[s];
    if (f != ~0ull) best_update(b, P[s].score, (int64_t)f, P[s].value);
  }
  b = block_best<kBS>(b, red);
  int open = 0;
  if (pass == 0 && J.n_cand > prefix) {
    for (int64_t s = threadIdx.x; s < J.lat_n && !open; s += kBS)
      open = F[s] == ~0ull && better(P[s].score, INT64_MAX, b.score, b.index) &&
             slot_reachable(J, segs[J.below], mu, sigma, s);
    open = __syncthreads_or(open);
  }
  if (threadIdx.x == 0) {
    best[j] = tpe_best{b.score, b.index, b.value, J.n_cand};
    if (pass == 0) need[j] = open;
  }
}

// ---------------------------------------------------------------------------
// categorical labels
// ---------------------------------------------------------------------------
constexpr int kRC = 16;      // categorical candidates per thread
constexpr int kCatKey = 256;  // categories of the rank-key fast path (8-bit category field)

// Categorical draws (randint / categorical priors sampled from the below
// posterior, tpe.py:575-610): candidate g takes word (g & 3) of the Philox call
// at counter (g >> 2, attempt 0) -- four candidates per call -- and its
// category is the first k with word < thr[k], thr[k] = ceil(cdf[k] / cdf[K-1]
// * 2^32): the inverse CDF at 2^-32 resolution, the same rule as the
// continuous samplers' component choice.
__device__ __forceinline__ uint32_t cat_thr(const double* cdf, int K, int k) {
  const double t = ceil(cdf[k] / cdf[K - 1] * 4294967296.0);
  return (t >= 4294967295.0) ? 0xFFFFFFFFu : (t > 0.0 ? (uint32_t)t : 0u);
}
__device__ __forceinline__ int cat_search(const double* cdf, int K, uint32_t w) {
  int lo = 0, hi = K - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (w < cat_thr(cdf, K, mid)) hi = mid; else lo = mid + 1;
  }
  return lo;
}

// injected candidates (given category indices): per-candidate lookup + argmax
__global__ __launch_bounds__(kBS) void k_score_cat_inj(
    const tpe_job* __restrict__ jobs, const tpe_cat_seg* __restrict__ csegs,
    const double* __restrict__ logp, const double* __restrict__ cand,
    double* __restrict__ out_bl, double* __restrict__ out_al, double* __restrict__ out_x,
    tpe_best* __restrict__ partial) {
  __shared__ BestT red[kBS / kWave];
  const tpe_job J = jobs[blockIdx.y];
  tpe_best* P = partial + (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  const int64_t base = (int64_t)blockIdx.x * (kBS * kRC);
  if (base >= J.n_cand) {
    if (threadIdx.x == 0) *P = empty_best();
    return;
  }
  const tpe_cat_seg CB = csegs[J.below], CA = csegs[J.above];
  const int K = CB.n_cat;
  const double* lb = logp + CB.p_off;
  const double* la = logp + CA.p_off;
  BestT b{0.0, -1, 0.0};
  for (int r = 0; r < kRC; ++r) {
    const int64_t li = base + r * kBS + threadIdx.x;
    if (li >= J.n_cand) break;
    const int64_t k = (int64_t)cand[J.cand_off + li];
    double bl = NAN, al = NAN;
    if (k >= 0 && k < K) {
      bl = lb[k];
      al = la[k];
    }
    const int64_t o = J.out_off + li;
    if (out_bl) out_bl[o] = bl;
    if (out_al) out_al[o] = al;
    if (out_x) out_x[o] = (double)k;
    best_update(b, bl - al, J.cand_base + li, (double)k);
  }
  b = block_best<kBS>(b, red);
  if (threadIdx.x == 0) *P = tpe_best{b.score, b.index, b.value, 0};
}

// sampled candidates.  The score depends on the category alone, so every
// category gets a rank (number of categories that beat it under np.argmax
// rules: NaN first, then larger score; equal scores share a rank) and a
// candidate's argmax key is rank << 48 | index << 8 | category: the smallest
// key is the reference's winner (best score, first index).  K <= KR: the
// thresholds sit in registers; KR < K <= kCatKey: binary search over the cdf
// (thresholds formed on the fly, same values); K > kCatKey: per-candidate
// fp64 argmax.  (The host picks KR from tpe_job.lat_n, the category count.)
__device__ __forceinline__ uint32_t word_of(const U4& q, int sel) {
  return sel == 0 ? q.x : sel == 1 ? q.y : sel == 2 ? q.z : q.w;
}

// Candidates [lo + blockIdx.x * kBS * kRC, ...) of job blockIdx.y; the
// block's winner goes to partial[job * nper + blockIdx.x].  need (nullable):
// jobs whose flag is 0 are skipped (the prefix-first path's second pass).
template <int KR>
__global__ __launch_bounds__(kBS) void k_score_cat(
    const tpe_job* __restrict__ jobs, const tpe_cat_seg* __restrict__ csegs,
    const double* __restrict__ logp, const double* __restrict__ cdf,
    double* __restrict__ out_bl, double* __restrict__ out_al, double* __restrict__ out_x,
    tpe_best* __restrict__ partial, int64_t lo, int64_t nper, const int32_t* __restrict__ need) {
  __shared__ double s_sc[kCatKey];
  __shared__ uint64_t s_key[kCatKey];
  __shared__ uint32_t s_thr[KR];
  __shared__ uint64_t red[kBS / kWave];
  if (need && !need[blockIdx.y]) return;  // block-uniform
  const tpe_job J = jobs[blockIdx.y];
  tpe_best* P = partial + (int64_t)blockIdx.y * nper + blockIdx.x;
  const int64_t base = lo + (int64_t)blockIdx.x * (kBS * kRC);
  if (base >= J.n_cand) {
    if (threadIdx.x == 0) *P = empty_best();
    return;
  }
  const tpe_cat_seg CB = csegs[J.below], CA = csegs[J.above];
  const int K = CB.n_cat;
  const double* lb = logp + CB.p_off;
  const double* la = logp + CA.p_off;
  const double* cb = cdf + CB.p_off;
  const int64_t t0 = base + (int64_t)threadIdx.x * kRC;
  const bool outs = out_bl || out_al || out_x;
  auto put = [&](int64_t li, int k) __attribute__((always_inline)) {
    if (outs) {
      const int64_t o = J.out_off + li;
      if (out_bl) out_bl[o] = lb[k];
      if (out_al) out_al[o] = la[k];
      if (out_x) out_x[o] = (double)k;
    }
  };
  if (K > kCatKey) {  // block-uniform: many categories, plain fp64 argmax
    BestT b{0.0, -1, 0.0};
    for (int r = 0; r < kRC; ++r) {
      const int64_t li = t0 + r;
      if (li >= J.n_cand) break;
      const int64_t g = J.cand_base + li;
      const int k = cat_search(cb, K, word_of(draw_words(J.key, g >> 2, 0, kStreamSample),
                                              (int)(g & 3)));
      put(li, k);
      best_update(b, lb[k] - la[k], g, (double)k);
    }
    b = block_best<kBS>(b, reinterpret_cast<BestT*>(s_sc));
    if (threadIdx.x == 0) *P = tpe_best{b.score, b.index, b.value, 0};
    return;
  }
  for (int k = threadIdx.x; k < K; k += kBS) {
    s_sc[k] = lb[k] - la[k];
    if (k < KR) s_thr[k] = cat_thr(cb, K, k);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += kBS) {
    const double sk = s_sc[k];
    uint32_t rank = 0;
    for (int j = 0; j < K; ++j) {
      const double sj = s_sc[j];
      rank += (sj != sj) ? (sk == sk) : (sk == sk && sj > sk);
    }
    s_key[k] = ((uint64_t)rank << 48) | (uint64_t)k;
  }
  __syncthreads();
  const bool in_regs = K <= KR;  // block-uniform
  uint32_t thr[KR - 1];
#pragma unroll
  for (int j = 0; j + 1 < KR; ++j) thr[j] = (in_regs && j + 1 < K) ? s_thr[j] : 0xFFFFFFFFu;
  auto category = [&](uint32_t w) __attribute__((always_inline)) -> int {
    if (in_regs) {
      int k = 0;
#pragma unroll
      for (int j = 0; j + 1 < KR; ++j) k += (w >= thr[j]) ? 1 : 0;
      return min(k, K - 1);
    }
    return cat_search(cb, K, w);
  };
  uint64_t best = ~0ull;
  auto take = [&](int64_t li, uint32_t w) __attribute__((always_inline)) {
    const int k = category(w);
    const int64_t g = J.cand_base + li;
    best = min(best, s_key[k] | ((uint64_t)g << 8));
    put(li, k);
  };
  const int64_t g0 = J.cand_base + t0;
  if ((g0 & 3) == 0 && t0 + kRC <= J.n_cand) {  // four candidates per Philox call
#pragma unroll
    for (int c = 0; c < kRC / 4; ++c) {
      const U4 r = draw_words(J.key, (g0 >> 2) + c, 0, kStreamSample);
      take(t0 + 4 * c + 0, r.x);
      take(t0 + 4 * c + 1, r.y);
      take(t0 + 4 * c + 2, r.z);
      take(t0 + 4 * c + 3, r.w);
    }
  } else {  // unaligned base or the job's last candidates: one call per candidate
    for (int r = 0; r < kRC; ++r) {
      const int64_t li = t0 + r;
      if (li >= J.n_cand) break;
      const int64_t g = J.cand_base + li;
      take(li, word_of(draw_words(J.key, g >> 2, 0, kStreamSample), (int)(g & 3)));
    }
  }
  // block min of the keys
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const uint64_t o = __shfl_xor(best, off, kWave);
    best = min(best, o);
  }
  if (lane_id() == 0) red[threadIdx.x / kWave] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t b = red[0];
#pragma unroll
    for (int w = 1; w < kBS / kWave; ++w) b = min(b, red[w]);
    if (b == ~0ull) {
      *P = empty_best();
    } else {
      const int k = (int)(b & 0xFF);
      const int64_t g = (int64_t)((b >> 8) & ((1ull << 40) - 1));
      *P = tpe_best{s_sc[k], g, (double)k, 0};
    }
  }
}

// The prefix-first decision for categorical jobs (tpe_categorical_suggest).
// Pass 0: the winner of the first `prefix` candidates (partials [0, n1)); a
// later candidate can only beat it with a strictly better score (its index is
// larger), i.e. with a category that scores better -- and every such category
// is absent from the prefix (else it would have won there).  need[j] = 1 when
// one of them can be drawn at all (a non-empty inverse-CDF interval) and the
// stream is longer than the prefix.  Pass 1 (jobs with need): the rest's
// partials [0, n2) folded into best[j].
__global__ __launch_bounds__(kBS) void k_cat_decide(
    const tpe_job* __restrict__ jobs, const tpe_cat_seg* __restrict__ csegs,
    const double* __restrict__ logp, const double* __restrict__ cdf,
    const tpe_best* __restrict__ partial, int64_t nper, int64_t n_use, int64_t prefix, int pass,
    int32_t* __restrict__ need, tpe_best* __restrict__ best) {
  __shared__ BestT red[kBS / kWave];
  const int j = blockIdx.x;
  if (pass == 1 && !need[j]) return;  // block-uniform
  const tpe_job J = jobs[j];
  const tpe_best* P = partial + (int64_t)j * nper;
  BestT b{0.0, -1, 0.0};
  if (pass == 1 && threadIdx.x == 0) b = BestT{best[j].score, best[j].index, best[j].value};
  for (int64_t i = threadIdx.x; i < n_use; i += kBS) best_update(b, P[i].score, P[i].index, P[i].value);
  b = block_best<kBS>(b, red);
  int open = 0;
  if (pass == 0 && J.n_cand > prefix) {
    const tpe_cat_seg CB = csegs[J.below], CA = csegs[J.above];
    const int K = CB.n_cat;
    for (int k = threadIdx.x; k < K && !open; k += kBS) {
      const double sk = logp[CB.p_off + k] - logp[CA.p_off + k];
      // category k takes the words [thr[k-1], thr[k]) (thr[-1] = 0, the last one
      // up to 2^32)
      const uint64_t t0 = k > 0 ? cat_thr(cdf + CB.p_off, K, k - 1) : 0ull;
      const uint64_t t1 = k < K - 1 ? (uint64_t)cat_thr(cdf + CB.p_off, K, k) : (1ull << 32);
      open = better(sk, INT64_MAX, b.score, b.index) && t1 > t0;
    }
    open = __syncthreads_or(open);
  }
  if (threadIdx.x == 0) {
    best[j] = tpe_best{b.score, b.index, b.value, J.n_cand};
    if (pass == 0) need[j] = open;
  }
}

// ---------------------------------------------------------------------------
// sampler only
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kBS) void k_sample(const tpe_job* __restrict__ jobs,
                                                const tpe_seg* __restrict__ segs,
                                                const double* __restrict__ mu,
                                                const double* __restrict__ sigma,
                                                const double* __restrict__ wcdf,
                                                double* __restrict__ out_x) {
  __shared__ MixLds s_mix;
  __shared__ float s_stage[kLatR * kBS];
  __shared__ uint16_t s_list[(kBS / kWave) * kRetryList];
  const tpe_job J = jobs[blockIdx.y];
  const int64_t base = (int64_t)blockIdx.x * (kBS * kLatR);
  if (base >= J.n_cand) return;
  const Mix M = stage_mix(segs[J.below], wcdf, mu, sigma, s_mix);
  const bool lgmm = J.family == TPE_LGMM1;
  const bool lo_on = J.flags & TPE_F_LOW, hi_on = J.flags & TPE_F_HIGH;
  if (sizeof(T) == 4) {
    // the fp32 stream exactly as the scorers draw it: kLatR consecutive
    // candidates per thread through draw32_pairs (the table scorer's and the
    // DRAW32 lattice sampler's code); LGMM1 values as exp(y) in fp64 for
    // unquantized labels (the scorers' values), __expf(y) for quantized ones
    // (the lattice sampler's slots)
    const bool quant = J.flags & TPE_F_QUANT;
    const int64_t t0 = base + (int64_t)threadIdx.x * kLatR;
    const int nv = (int)max((int64_t)0, min((int64_t)kLatR, J.n_cand - t0));
    float x[kLatR];
    draw32_pairs<kLatR>(M, J.key, J.cand_base + t0, nv, lo_on, hi_on, (float)J.low,
                        (float)J.high, lgmm && quant,
                        s_stage + (threadIdx.x / kWave) * (kLatR * kWave),
                        s_list + (threadIdx.x / kWave) * kRetryList, x);
#pragma unroll
    for (int r = 0; r < kLatR; ++r) {
      if (r >= nv) continue;
      double v = (lgmm && !quant) ? exp((double)x[r]) : (double)x[r];
      if (quant) v = rint(v / J.q) * J.q;
      out_x[J.out_off + t0 + r] = v;
    }
    return;
  }
  for (int r = 0; r < kLatR; ++r) {
    const int64_t li = base + r * kBS + threadIdx.x;
    if (li >= J.n_cand) break;
    double v = draw64(M, J.key, J.cand_base + li, lo_on, hi_on, J.low, J.high);
    if (lgmm) v = exp(v);
    if (J.flags & TPE_F_QUANT) v = rint(v / J.q) * J.q;
    out_x[J.out_off + li] = v;
  }
}

__global__ void k_combine(const tpe_best* __restrict__ sets, int n_sets, int n_labels,
                          tpe_best* __restrict__ out) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n_labels) return;
  tpe_best b = sets[l];
  int64_t n = b.n_scored;
  bool inexact = n < 0;  // a set whose exact decision is still owed (band overflow)
  for (int s = 1; s < n_sets; ++s) {
    const tpe_best o = sets[(int64_t)s * n_labels + l];
    n += o.n_scored;
    inexact = inexact || o.n_scored < 0;
    if (better(o.score, o.index, b.score, b.index)) b = o;
  }
  b.n_scored = inexact ? -1 : n;  // -1 travels: every rank sees the label is owed
  out[l] = b;
}

int64_t max_blocks(const tpe_job* hj, int n, int64_t per_block, int want_quant) {
  int64_t g = 1;
  for (int i = 0; i < n; ++i) {
    const bool q = (hj[i].flags & TPE_F_QUANT) != 0;
    if (want_quant >= 0 && q != (bool)want_quant) continue;
    g = std::max(g, (hj[i].n_cand + per_block - 1) / per_block);
  }
  return g;
}

bool check_jobs(const char* fn, const tpe_job* hj, int n) {
  if (n < 0 || n > 65535) {
    set_error("%s: n_jobs=%d outside [0, 65535]", fn, n);
    return false;
  }
  if (n > 0 && !hj) {
    set_error("%s: host_jobs is NULL", fn);
    return false;
  }
  for (int i = 0; i < n; ++i)
    if (hj[i].n_cand < 0) {
      set_error("%s: job %d has n_cand < 0", fn, i);
      return false;
    }
  return true;
}
}  // namespace
}  // namespace tpe

using namespace tpe;

extern "C" int64_t tpe_score_partials(const tpe_job* host_jobs, int n_jobs) {
  // the larger of the fp32 and fp64 grids
  return (int64_t)n_jobs * max_blocks(host_jobs, n_jobs, kBS * kR64, -1);
}

extern "C" int tpe_score_continuous(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                                    const tpe_seg* segs, const double* w, const double* mu,
                                    const double* sigma, const double* wcdf,
                                    const double* coef64, const float* coef32,
                                    const double* cand, int precision, double* out_bl,
                                    double* out_al, double* out_x, tpe_best* partial,
                                    int64_t n_partial, tpe_best* best, void* stream) {
  (void)w;
  if (!check_jobs("tpe_score_continuous", host_jobs, n_jobs)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  if (precision != 32 && precision != 64) {
    set_error("tpe_score_continuous: precision must be 32 or 64, got %d", precision);
    return TPE_E_ARG;
  }
  bool inj = false;
  for (int i = 0; i < n_jobs; ++i) {
    if (host_jobs[i].family == TPE_CAT || (host_jobs[i].flags & TPE_F_QUANT)) {
      set_error("tpe_score_continuous: job %d is not an unquantized GMM1/LGMM1 job", i);
      return TPE_E_ARG;
    }
    const bool ji = (host_jobs[i].flags & TPE_F_INJECTED) != 0;
    if (i > 0 && ji != inj) {
      set_error("tpe_score_continuous: mixed injected / sampled jobs in one call");
      return TPE_E_ARG;
    }
    inj = ji;
  }
  if (!jobs || !segs || !mu || !sigma || !wcdf || !partial || !best || (inj && !cand) ||
      (precision == 32 ? !coef32 : !coef64)) {
    set_error("tpe_score_continuous: null pointer");
    return TPE_E_ARG;
  }
  const int R = precision == 32 ? kR32 : kR64;
  const int64_t gx = max_blocks(host_jobs, n_jobs, (int64_t)kBS * R, -1);
  if (gx * n_jobs > n_partial) {
    set_error("tpe_score_continuous: partial workspace %lld < %lld", (long long)n_partial,
              (long long)(gx * n_jobs));
    return TPE_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)gx, (unsigned)n_jobs);
  if (precision == 32) {
    const float4* c = reinterpret_cast<const float4*>(coef32);
    if (inj)
      hipLaunchKernelGGL(k_score32<true>, grid, dim3(kBS), 0, st, jobs, segs, mu, sigma, wcdf, c,
                         cand, out_bl, out_al, out_x, partial);
    else
      hipLaunchKernelGGL(k_score32<false>, grid, dim3(kBS), 0, st, jobs, segs, mu, sigma, wcdf,
                         c, cand, out_bl, out_al, out_x, partial);
  } else {
    const double4* c = reinterpret_cast<const double4*>(coef64);
    if (inj)
      hipLaunchKernelGGL(k_score64<true>, grid, dim3(kBS), 0, st, jobs, segs, mu, sigma, wcdf, c,
                         cand, out_bl, out_al, out_x, partial);
    else
      hipLaunchKernelGGL(k_score64<false>, grid, dim3(kBS), 0, st, jobs, segs, mu, sigma, wcdf,
                         c, cand, out_bl, out_al, out_x, partial);
  }
  hipLaunchKernelGGL(k_reduce, dim3(n_jobs), dim3(kBS), 0, st, jobs, partial, gx, best);
  return check_launch("tpe_score_continuous");
}

// k_lattice_sample over candidates [start, min(n_cand, limit)) of every job
// (of the jobs with need[j] set, when need is given); false (error set) when
// the grid is too large
static bool launch_lattice_sample(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                                  const tpe_seg* segs, const double* mu, const double* sigma,
                                  const double* wcdf, uint64_t* slot_first, int32_t* err,
                                  int64_t start, int64_t limit, const int32_t* need,
                                  hipStream_t st, const char* who, const double* w = nullptr,
                                  tpe_best* slot_part = nullptr, int64_t slot_n = 0,
                                  const double* qP = nullptr, const double* qS = nullptr) {
  int64_t gx = 1;
  for (int i = 0; i < n_jobs; ++i) {
    const int64_t n = std::min(host_jobs[i].n_cand, limit);
    gx = std::max(gx, (n + (int64_t)kBS * kLatR - 1) / ((int64_t)kBS * kLatR));
  }
  const int64_t per = (gx * n_jobs + 7) / 8;
  const int64_t sblocks = need ? 0 : slot_n * n_jobs;  // slot scoring rides on the prefix launch
  if (gx > INT32_MAX || 8 * per + sblocks > INT32_MAX || slot_n > INT32_MAX) {
    set_error("%s: %lld work items", who, (long long)(gx * n_jobs));
    return false;
  }
  bool pow2 = true;
  int64_t n_loc = 1;
  for (int i = 0; i < n_jobs; ++i) {
    pow2 = pow2 && lattice_pow2(host_jobs[i]);
    n_loc = std::max(n_loc, std::min((int64_t)kLatLds, host_jobs[i].lat_n));
  }
  const size_t lds = (size_t)n_loc * sizeof(uint32_t);
  unsigned long long* sf = (unsigned long long*)slot_first;
  // with need: a grid-stride grid (k_lattice_sample): two blocks per CU
  const unsigned grid =
      need ? (unsigned)std::min<int64_t>(8 * per, 512) : (unsigned)(8 * per + sblocks);
  const int sn = need ? 0 : (int)slot_n;
  if (pow2)
    hipLaunchKernelGGL(k_lattice_sample<true>, dim3(grid), dim3(kBS), lds, st, jobs, segs, mu,
                       sigma, wcdf, sf, err, (int)gx, n_jobs, start, limit, need, w, slot_part,
                       sn, qP, qS);
  else
    hipLaunchKernelGGL(k_lattice_sample<false>, dim3(grid), dim3(kBS), lds, st, jobs, segs, mu,
                       sigma, wcdf, sf, err, (int)gx, n_jobs, start, limit, need, w, slot_part,
                       sn, qP, qS);
  return true;
}

extern "C" int tpe_lattice_sample(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                                  const tpe_seg* segs, const double* mu, const double* sigma,
                                  const double* wcdf, uint64_t* slot_first, int32_t* err,
                                  void* stream) {
  if (!check_jobs("tpe_lattice_sample", host_jobs, n_jobs)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  if (!jobs || !segs || !mu || !sigma || !wcdf || !slot_first || !err) {
    set_error("tpe_lattice_sample: null pointer");
    return TPE_E_ARG;
  }
  int64_t end = 0;
  for (int i = 0; i < n_jobs; ++i) {
    const tpe_job& j = host_jobs[i];
    if (!(j.flags & TPE_F_QUANT) || j.family == TPE_CAT || !(j.q > 0) || j.lat_n <= 0) {
      set_error("tpe_lattice_sample: job %d is not a quantized job with a lattice", i);
      return TPE_E_ARG;
    }
    end = std::max(end, j.lat_off + j.lat_n);
  }
  hipStream_t st = (hipStream_t)stream;
  bool ready = true;
  for (int i = 0; i < n_jobs; ++i) ready = ready && (host_jobs[i].flags & TPE_F_LATTICE_READY);
  if (!ready && hipMemsetAsync(slot_first, 0xFF, (size_t)end * sizeof(uint64_t), st) != hipSuccess)
    return check_launch("tpe_lattice_sample memset");
  if (!launch_lattice_sample(jobs, host_jobs, n_jobs, segs, mu, sigma, wcdf, slot_first, err, 0,
                             INT64_MAX, nullptr, st, "tpe_lattice_sample"))
    return TPE_E_UNSUPPORTED;
  return check_launch("tpe_lattice_sample");
}

extern "C" int tpe_lattice_suggest(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                                   const tpe_seg* segs, const double* w, const double* mu,
                                   const double* sigma, const double* wcdf, uint64_t* slot_first,
                                   int64_t prefix, tpe_best* partial, int64_t n_partial,
                                   int32_t* need, tpe_best* best, int32_t* err, double* reach_hi,
                                   double* reach_lo, void* stream) {
  if (!check_jobs("tpe_lattice_suggest", host_jobs, n_jobs)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  if (!jobs || !segs || !w || !mu || !sigma || !wcdf || !slot_first || !partial || !need ||
      !best || !err) {
    set_error("tpe_lattice_suggest: null pointer");
    return TPE_E_ARG;
  }
  if (prefix <= 0 || prefix % ((int64_t)kBS * kLatR) != 0) {
    set_error("tpe_lattice_suggest: prefix %lld is not a positive multiple of %d",
              (long long)prefix, kBS * kLatR);
    return TPE_E_ARG;
  }
  int64_t end = 0, max_n = 1;
  for (int i = 0; i < n_jobs; ++i) {
    const tpe_job& j = host_jobs[i];
    if (!(j.flags & TPE_F_QUANT) || j.family == TPE_CAT || !(j.q > 0) || j.lat_n <= 0 ||
        (j.flags & TPE_F_INJECTED)) {
      set_error("tpe_lattice_suggest: job %d is not a sampled quantized job with a lattice", i);
      return TPE_E_ARG;
    }
    end = std::max(end, j.lat_off + j.lat_n);
    max_n = std::max(max_n, j.lat_n);
  }
  if (max_n > INT32_MAX || max_n * n_jobs > n_partial) {
    set_error("tpe_lattice_suggest: partial workspace %lld < %lld slots", (long long)n_partial,
              (long long)(max_n * n_jobs));
    return TPE_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  bool ready = true;
  for (int i = 0; i < n_jobs; ++i) ready = ready && (host_jobs[i].flags & TPE_F_LATTICE_READY);
  if (!ready && hipMemsetAsync(slot_first, 0xFF, (size_t)end * sizeof(uint64_t), st) != hipSuccess)
    return check_launch("tpe_lattice_suggest memset");
  unsigned long long* sf = (unsigned long long*)slot_first;
  const bool win = reach_hi && reach_lo;  // the slots' component windows (k_qreach)
  if (win)
    hipLaunchKernelGGL(k_qreach, dim3(4 * n_jobs), dim3(kQB), 0, st, jobs, segs, mu, sigma,
                       reach_hi, reach_lo);
  if (!launch_lattice_sample(jobs, host_jobs, n_jobs, segs, mu, sigma, wcdf, slot_first, err, 0,
                             prefix, nullptr, st, "tpe_lattice_suggest", w, partial, max_n,
                             win ? reach_hi : nullptr, win ? reach_lo : nullptr))
    return TPE_E_UNSUPPORTED;
  hipLaunchKernelGGL(k_lattice_decide, dim3(n_jobs), dim3(kBS), 0, st, jobs, segs, mu, sigma,
                     partial, max_n, sf, prefix, 0, need, best);
  bool more = false;
  for (int i = 0; i < n_jobs; ++i) more = more || host_jobs[i].n_cand > prefix;
  if (more) {  // the rest of the streams that need it (blocks of the others exit at once)
    if (!launch_lattice_sample(jobs, host_jobs, n_jobs, segs, mu, sigma, wcdf, slot_first, err,
                               prefix, INT64_MAX, need, st, "tpe_lattice_suggest"))
      return TPE_E_UNSUPPORTED;
    hipLaunchKernelGGL(k_lattice_decide, dim3(n_jobs), dim3(kBS), 0, st, jobs, segs, mu, sigma,
                       partial, max_n, sf, prefix, 1, need, best);
  }
  return check_launch("tpe_lattice_suggest");
}

extern "C" int tpe_lattice_compact(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                                   const uint64_t* slot_first, double* vals, int64_t* firsts,
                                   int64_t* counts, void* stream) {
  if (!check_jobs("tpe_lattice_compact", host_jobs, n_jobs)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  if (!jobs || !slot_first || !vals || !firsts || !counts) {
    set_error("tpe_lattice_compact: null pointer");
    return TPE_E_ARG;
  }
  int64_t maxn = 1;
  bool ready = true;
  for (int i = 0; i < n_jobs; ++i) {
    maxn = std::max(maxn, host_jobs[i].lat_n);
    ready = ready && (host_jobs[i].flags & TPE_F_LATTICE_READY);
  }
  hipStream_t st = (hipStream_t)stream;
  if (!ready && hipMemsetAsync(counts, 0, (size_t)n_jobs * sizeof(int64_t), st) != hipSuccess)
    return check_launch("tpe_lattice_compact memset");
  hipLaunchKernelGGL(k_lattice_compact, dim3((unsigned)((maxn + kBS - 1) / kBS), (unsigned)n_jobs),
                     dim3(kBS), 0, st, jobs, (const unsigned long long*)slot_first, vals, firsts,
                     (unsigned long long*)counts);
  return check_launch("tpe_lattice_compact");
}

extern "C" int64_t tpe_quantized_partials(const tpe_job* host_jobs, int n_jobs, int64_t max_vals) {
  (void)host_jobs;
  return (int64_t)n_jobs * std::max((int64_t)1, max_vals);  // one entry per value
}

extern "C" int tpe_score_quantized(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                                   const tpe_seg* segs, const double* w, const double* mu,
                                   const double* sigma, const double* vals,
                                   const int64_t* firsts, const int64_t* counts, int64_t max_vals,
                                   double* out_bl, double* out_al, tpe_best* partial,
                                   int64_t n_partial, tpe_best* best, int32_t* err,
                                   double* reach_hi, double* reach_lo, void* stream) {
  if (!check_jobs("tpe_score_quantized", host_jobs, n_jobs)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  if (!jobs || !segs || !w || !mu || !sigma || !vals || !partial || !best || !err ||
      ((firsts == nullptr) != (counts == nullptr))) {
    set_error("tpe_score_quantized: null pointer (firsts and counts go together)");
    return TPE_E_ARG;
  }
  for (int i = 0; i < n_jobs; ++i)
    if (!(host_jobs[i].flags & TPE_F_QUANT) || !(host_jobs[i].q > 0) ||
        host_jobs[i].family == TPE_CAT) {
      set_error("tpe_score_quantized: job %d is not quantized", i);
      return TPE_E_ARG;
    }
  const int64_t gx = std::max((int64_t)1, max_vals);  // partial entries per job
  if (gx * n_jobs > n_partial) {
    set_error("tpe_score_quantized: partial workspace too small");
    return TPE_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  const bool win = reach_hi && reach_lo;  // the values' component windows (k_qreach)
  if (win)
    hipLaunchKernelGGL(k_qreach, dim3(4 * n_jobs), dim3(kQB), 0, st, jobs, segs, mu, sigma,
                       reach_hi, reach_lo);
  hipLaunchKernelGGL(k_score_q, dim3((unsigned)gx, (unsigned)n_jobs),
                     dim3(kBS), 0, st, jobs, segs, w, mu, sigma, vals, firsts,
                     (const unsigned long long*)counts, out_bl, out_al, partial, err,
                     win ? reach_hi : nullptr, win ? reach_lo : nullptr, gx);
  hipLaunchKernelGGL(k_reduce, dim3(n_jobs), dim3(kBS), 0, st, jobs, partial, gx, best);
  return check_launch("tpe_score_quantized");
}

extern "C" int64_t tpe_categorical_partials(const tpe_job* host_jobs, int n_jobs) {
  return (int64_t)n_jobs * max_blocks(host_jobs, n_jobs, kBS * kRC, -1);
}

extern "C" int tpe_score_categorical(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                                     const tpe_cat_seg* csegs, const double* logp_pool,
                                     const double* cdf_pool, const double* cand,
                                     double* out_bl, double* out_al, double* out_x,
                                     tpe_best* partial, int64_t n_partial, tpe_best* best,
                                     void* stream) {
  if (!check_jobs("tpe_score_categorical", host_jobs, n_jobs)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  bool inj = false;
  for (int i = 0; i < n_jobs; ++i) {
    if (host_jobs[i].family != TPE_CAT) {
      set_error("tpe_score_categorical: job %d is not categorical", i);
      return TPE_E_ARG;
    }
    const bool ji = (host_jobs[i].flags & TPE_F_INJECTED) != 0;
    if (i > 0 && ji != inj) {
      set_error("tpe_score_categorical: mixed injected / sampled jobs in one call");
      return TPE_E_ARG;
    }
    inj = ji;
  }
  if (!jobs || !csegs || !logp_pool || !cdf_pool || !partial || !best || (inj && !cand)) {
    set_error("tpe_score_categorical: null pointer");
    return TPE_E_ARG;
  }
  const int64_t gx = max_blocks(host_jobs, n_jobs, (int64_t)kBS * kRC, -1);
  if (gx * n_jobs > n_partial) {
    set_error("tpe_score_categorical: partial workspace too small");
    return TPE_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)gx, (unsigned)n_jobs);
  int kmax = 1;  // category counts (tpe_job.lat_n of categorical jobs; 0 = unknown)
  for (int i = 0; i < n_jobs; ++i)
    kmax = std::max(kmax, host_jobs[i].lat_n > 0 ? (int)host_jobs[i].lat_n : kCatKey);
  if (inj)
    hipLaunchKernelGGL(k_score_cat_inj, grid, dim3(kBS), 0, st, jobs, csegs, logp_pool, cand,
                       out_bl, out_al, out_x, partial);
  else if (kmax <= 4)
    hipLaunchKernelGGL(k_score_cat<4>, grid, dim3(kBS), 0, st, jobs, csegs, logp_pool, cdf_pool,
                       out_bl, out_al, out_x, partial, (int64_t)0, gx, nullptr);
  else if (kmax <= 8)
    hipLaunchKernelGGL(k_score_cat<8>, grid, dim3(kBS), 0, st, jobs, csegs, logp_pool, cdf_pool,
                       out_bl, out_al, out_x, partial, (int64_t)0, gx, nullptr);
  else
    hipLaunchKernelGGL(k_score_cat<16>, grid, dim3(kBS), 0, st, jobs, csegs, logp_pool, cdf_pool,
                       out_bl, out_al, out_x, partial, (int64_t)0, gx, nullptr);
  hipLaunchKernelGGL(k_reduce, dim3(n_jobs), dim3(kBS), 0, st, jobs, partial, gx, best);
  return check_launch("tpe_score_categorical");
}

// prefix-first categorical argmax (the suggest path; see k_cat_decide)
static void launch_cat(int kmax, dim3 grid, hipStream_t st, const tpe_job* jobs,
                       const tpe_cat_seg* csegs, const double* logp, const double* cdf,
                       tpe_best* partial, int64_t lo, int64_t nper, const int32_t* need) {
  if (kmax <= 4)
    hipLaunchKernelGGL(k_score_cat<4>, grid, dim3(kBS), 0, st, jobs, csegs, logp, cdf, nullptr,
                       nullptr, nullptr, partial, lo, nper, need);
  else if (kmax <= 8)
    hipLaunchKernelGGL(k_score_cat<8>, grid, dim3(kBS), 0, st, jobs, csegs, logp, cdf, nullptr,
                       nullptr, nullptr, partial, lo, nper, need);
  else
    hipLaunchKernelGGL(k_score_cat<16>, grid, dim3(kBS), 0, st, jobs, csegs, logp, cdf, nullptr,
                       nullptr, nullptr, partial, lo, nper, need);
}

extern "C" int tpe_categorical_suggest(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                                       const tpe_cat_seg* csegs, const double* logp_pool,
                                       const double* cdf_pool, int64_t prefix, tpe_best* partial,
                                       int64_t n_partial, int32_t* need, tpe_best* best,
                                       void* stream) {
  if (!check_jobs("tpe_categorical_suggest", host_jobs, n_jobs)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  for (int i = 0; i < n_jobs; ++i)
    if (host_jobs[i].family != TPE_CAT || (host_jobs[i].flags & TPE_F_INJECTED)) {
      set_error("tpe_categorical_suggest: job %d is not a sampled categorical job", i);
      return TPE_E_ARG;
    }
  if (!jobs || !csegs || !logp_pool || !cdf_pool || !partial || !need || !best) {
    set_error("tpe_categorical_suggest: null pointer");
    return TPE_E_ARG;
  }
  constexpr int64_t kT = (int64_t)kBS * kRC;
  if (prefix <= 0 || prefix % kT != 0) {
    set_error("tpe_categorical_suggest: prefix %lld is not a positive multiple of %lld",
              (long long)prefix, (long long)kT);
    return TPE_E_ARG;
  }
  const int64_t gx = max_blocks(host_jobs, n_jobs, kT, -1);
  if (gx * n_jobs > n_partial) {
    set_error("tpe_categorical_suggest: partial workspace %lld < %lld", (long long)n_partial,
              (long long)(gx * n_jobs));
    return TPE_E_ARG;
  }
  int kmax = 1;
  for (int i = 0; i < n_jobs; ++i)
    kmax = std::max(kmax, host_jobs[i].lat_n > 0 ? (int)host_jobs[i].lat_n : kCatKey);
  hipStream_t st = (hipStream_t)stream;
  const int64_t g1 = std::min(gx, prefix / kT);  // prefix blocks per job
  launch_cat(kmax, dim3((unsigned)g1, (unsigned)n_jobs), st, jobs, csegs, logp_pool, cdf_pool,
             partial, 0, gx, nullptr);
  hipLaunchKernelGGL(k_cat_decide, dim3(n_jobs), dim3(kBS), 0, st, jobs, csegs, logp_pool,
                     cdf_pool, partial, gx, g1, prefix, 0, need, best);
  if (gx > g1) {  // the rest of the streams that need it (blocks of the others exit at once)
    launch_cat(kmax, dim3((unsigned)(gx - g1), (unsigned)n_jobs), st, jobs, csegs, logp_pool,
               cdf_pool, partial, prefix, gx, need);
    hipLaunchKernelGGL(k_cat_decide, dim3(n_jobs), dim3(kBS), 0, st, jobs, csegs, logp_pool,
                       cdf_pool, partial, gx, gx - g1, prefix, 1, need, best);
  }
  return check_launch("tpe_categorical_suggest");
}

extern "C" int tpe_sample(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                          const tpe_seg* segs, const double* mu, const double* sigma,
                          const double* wcdf, int precision, double* out_x, void* stream) {
  if (!check_jobs("tpe_sample", host_jobs, n_jobs)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  if (!jobs || !segs || !mu || !sigma || !wcdf || !out_x || (precision != 32 && precision != 64)) {
    set_error("tpe_sample: bad arguments");
    return TPE_E_ARG;
  }
  for (int i = 0; i < n_jobs; ++i)
    if (host_jobs[i].family == TPE_CAT) {
      set_error("tpe_sample: categorical jobs are sampled by tpe_score_categorical");
      return TPE_E_ARG;
    }
  const int64_t gx = max_blocks(host_jobs, n_jobs, (int64_t)kBS * kLatR, -1);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)gx, (unsigned)n_jobs);
  if (precision == 32)
    hipLaunchKernelGGL(k_sample<float>, grid, dim3(kBS), 0, st, jobs, segs, mu, sigma, wcdf, out_x);
  else
    hipLaunchKernelGGL(k_sample<double>, grid, dim3(kBS), 0, st, jobs, segs, mu, sigma, wcdf,
                       out_x);
  return check_launch("tpe_sample");
}

extern "C" int tpe_best_combine(const tpe_best* sets, int n_sets, int n_labels, tpe_best* out,
                                void* stream) {
  if (n_sets <= 0 || n_labels < 0 || (n_labels > 0 && (!sets || !out))) {
    set_error("tpe_best_combine: bad arguments");
    return TPE_E_ARG;
  }
  if (n_labels == 0) return TPE_OK;
  hipLaunchKernelGGL(k_combine, dim3((n_labels + kBS - 1) / kBS), dim3(kBS), 0,
                     (hipStream_t)stream, sets, n_sets, n_labels, out);
  return check_launch("tpe_best_combine");
}

extern "C" int64_t tpe_sort_layout(int64_t n_cand, int64_t* sorted_slots) {
  // u32 words used = 2 x the returned value: the count matrix (blocks x
  // bins), the run offsets (same shape), then per-chunk column sums
  if (sorted_slots) *sorted_slots = n_cand;
  const int64_t nblk = (n_cand + kSortPer - 1) / kSortPer;
  const int64_t nch = (nblk + kScanChunk - 1) / kScanChunk;
  return nblk * (int64_t)kNB + (nch * (int64_t)kNB + 1) / 2;
}

static bool check_sorted_jobs(const char* fn, const tpe_job* host_jobs, int n_jobs) {
  if (!check_jobs(fn, host_jobs, n_jobs)) return false;
  for (int i = 0; i < n_jobs; ++i) {
    const tpe_job& j = host_jobs[i];
    if (j.family == TPE_CAT || (j.flags & (TPE_F_QUANT | TPE_F_INJECTED))) {
      set_error("%s: job %d is not a sampled unquantized GMM1/LGMM1 job", fn, i);
      return false;
    }
    if (!(j.bin_hi > j.bin_lo) || j.n_cand > 0xFFFFFFFFll) {
      set_error("%s: job %d has an empty bin range or > 2^32 candidates", fn, i);
      return false;
    }
  }
  return true;
}

extern "C" int tpe_sort_candidates(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                                   const tpe_seg* segs, const double* mu, const double* sigma,
                                   const double* wcdf, uint32_t* counts, float* gen,
                                   float* sorted_x, uint32_t* sorted_i, void* stream) {
  if (!check_sorted_jobs("tpe_sort_candidates", host_jobs, n_jobs)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  if (!jobs || !segs || !mu || !sigma || !wcdf || !counts || !gen || !sorted_x || !sorted_i) {
    set_error("tpe_sort_candidates: null pointer");
    return TPE_E_ARG;
  }
  const int64_t gs = max_blocks(host_jobs, n_jobs, (int64_t)kSortPer, -1);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_sort_count, dim3((unsigned)gs, (unsigned)n_jobs), dim3(kBS), 0, st, jobs,
                     segs, mu, sigma, wcdf, counts, gen);
  const int64_t gch = (gs + kScanChunk - 1) / kScanChunk;
  hipLaunchKernelGGL(k_sort_colsum, dim3((unsigned)gch, (unsigned)n_jobs), dim3(kNB), 0, st, jobs,
                     counts);
  hipLaunchKernelGGL(k_sort_scan, dim3(n_jobs), dim3(kNB), 0, st, jobs, counts);
  hipLaunchKernelGGL(k_sort_offsets, dim3((unsigned)gch, (unsigned)n_jobs), dim3(kNB), 0, st, jobs,
                     counts);
  hipLaunchKernelGGL(k_sort_scatter, dim3((unsigned)gs, (unsigned)n_jobs), dim3(kBS), 0, st, jobs,
                     counts, gen, sorted_x, sorted_i);
  return check_launch("tpe_sort_candidates");
}

extern "C" int tpe_score_sorted(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                                const tpe_seg* segs, const float* coef32, const float* coef32n,
                                const float* wide32, const float* pm, const float* sm,
                                const float* sorted_x, const uint32_t* sorted_i,
                                tpe_best* partial, int64_t n_partial, tpe_best* best,
                                uint64_t* pairs, void* stream) {
  if (!check_sorted_jobs("tpe_score_sorted", host_jobs, n_jobs)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  if (!jobs || !segs || !coef32 || !coef32n || !wide32 || !pm || !sm || !sorted_x ||
      !sorted_i || !partial || !best) {
    set_error("tpe_score_sorted: null pointer");
    return TPE_E_ARG;
  }
  const int64_t gx = max_blocks(host_jobs, n_jobs, (int64_t)kBS * kR32, -1);
  if (gx * n_jobs > n_partial) {
    set_error("tpe_score_sorted: partial workspace too small");
    return TPE_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_score_sorted, dim3((unsigned)gx, (unsigned)n_jobs), dim3(kBS), 0, st, jobs,
                     segs, reinterpret_cast<const float4*>(coef32),
                     reinterpret_cast<const float4*>(coef32n),
                     reinterpret_cast<const float4*>(wide32), pm, sm, sorted_x, sorted_i, partial,
                     (unsigned long long*)pairs);
  hipLaunchKernelGGL(k_reduce, dim3(n_jobs), dim3(kBS), 0, st, jobs, partial, gx, best);
  return check_launch("tpe_score_sorted");
}
