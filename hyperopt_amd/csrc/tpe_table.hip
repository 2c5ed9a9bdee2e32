// tpe_table.hip -- cell-table scoring of unquantized continuous labels.
//
// Computes the same per-candidate quantities as GMM1_lpdf / LGMM1_lpdf
// (hyperopt/tpe.py:117-180, 265-307, logsum_rows :260-262) and the argmax of
// broadcast_best (tpe.py:649-658), for candidates sampled from the below
// posterior (tpe.py:79-106, 229-257) -- but without a component loop per
// candidate.
//
// Expansion.  In the scoring coordinate y (x for GMM1, log x for LGMM1) a
// mixture's density is S(y) = sum_j exp(l_j(y)),
//     l_j(y) = lc_j - 0.5 ((y - mu_j) inv_j)^2        (coef64: {mu, inv, lc, w}).
// The candidate range is cut into nb cells of half-width h.  Around a cell
// centre y0, with u = (y - y0)/h in [-1, 1],
//     l_j(y0 + h u) = l_j(y0) + A_j u + B_j u^2,
//     A_j = -h (y0 - mu_j) inv_j^2,   B_j = -0.5 h^2 inv_j^2,
// and exp(A u + B u^2) = sum_n c_n u^n with c_0 = 1, c_1 = A,
// (n+1) c_{n+1} = A c_n + 2B c_{n-1}.  So on the cell
//     S(y) = exp(m) * sum_{n<kP} P_n u^n,  P_n = sum_j exp(l_j(y0) - m) c_n^(j),
// a degree-8 polynomial per cell and mixture: the per-candidate work is two
// Horner evaluations and two logs, independent of the number of components.
//
// Error.  Every term is positive, so the relative error of S is at most the
// worst relative error of one component's truncated series.  |c_n| is at most
// the coefficient c~_n of exp(|A|u + |B|u^2) (same recurrence, all terms
// positive), so for |u| <= 1.05 the truncation error is at most
// e^{a+b} sum_{n>=9} c~_n 1.05^n (a = 1.05|A|, b = 1.05^2|B|); over
// 9|A| + 65|B| <= 5.8 its maximum is 4.3e-7.  P_0..P_5 are stored in fp32 and
// P_6..P_8 in fp16 (|P_n| <= e^{a+b} c~_n P_0, P_0 >= 1): the rounding adds at
// most 1.4e-7; the scorer evaluates that fp16 tail in fp16 arithmetic, which
// adds at most 4.4e-7 (tools/table_bounds.py 9 evaluates the three maxima).
// Components whose largest term anywhere in the candidate range is below
// exp(-25)/M of the prior component's smallest term there (a lower bound of S
// everywhere) are left out (together < 1.4e-11 of S); the rest are found per
// cell through reach windows over the sorted means.
// The plan step chooses h so that every component that can be included in
// any cell satisfies the bound; if the cell budget (job.tbl_cap) forces a
// larger h, failing cells are flagged and their candidates take the exact
// fp32 log-sum-exp over all components.  Candidates outside the grid
// (injected values, rounding at the edges) take the exact path too.
//
// Layout.  One tpe_table per job plus a 128-B slot per cell: the job's region
// holds tbl_cap 64-B cells (four 16-B chunks, the scorer's whole gather), then
// tbl_cap (m_below, m_above) fp32 pairs (per-candidate outputs only):
//     floats [2n], [2n+1]: below / above P_n, n < 6                  chunks 0-2
//     dword 12 + (n - 6): fp16 {below P_n (low half), above P_n}, n = 6..8
//     [15] m_below - m_above (the score offset); NaN marks a cell that failed
//          the bound                                                  chunk 3
// The cell centre is not stored: both sides form it from the cell index
// (cell_centre).  The pairs (below P_n, above P_n) sit in adjacent registers
// for packed-FP32 Horner.
#include <algorithm>
#include <type_traits>

#include "tpe_common.hpp"
#include "tpe_sample.hpp"

namespace tpe {
namespace {
constexpr int kP = 9;                // expansion terms per cell and mixture
constexpr int kP32 = 6;              // of which stored in fp32 (the rest in fp16)
constexpr int kCellF = 16;           // floats per cell (64 B: four 16-B chunks)
constexpr int kSlotB = 128;          // bytes per cell slot of a job's region (cells + m pairs)
constexpr int kChunks = 4;           // 16-B chunks of a cell the scorer reads
constexpr double kRhoLim = 5.8;      // admissible 9|A| + 65|B|
#ifndef TPE_SCORE_WPE  // waves per SIMD the fast scorer is compiled for (its VGPR budget;
#define TPE_SCORE_WPE 4  // its 32 KB draw stage per block allows four blocks per CU anyway)
#endif
#ifndef TPE_TAU_TABLE
#define TPE_TAU_TABLE 17.0
#endif
constexpr double kTauExtra = TPE_TAU_TABLE;  // exclusion margin (nats) on top of log(M)
constexpr double kDrawZ = 5.8;       // |z| of an fp32 Box-Muller draw is < 5.77
constexpr double kDrawZ64 = 8.7;     // |z| of an fp64 Box-Muller draw (53-bit uniforms) is < 8.6
constexpr double kTauExact = 40.0;   // margin of the pruned exact fp64 scorer: e^-40 < 5e-18
constexpr float kULim = 1.05f;       // |u| accepted by the scorer (fp32 cell-centre rounding)
#ifndef TPE_TR
#define TPE_TR 16
#endif
constexpr int kTR = TPE_TR;          // candidates per thread and tile in the scorer
#ifndef TPE_TILES
#define TPE_TILES 1
#endif
constexpr int kTiles = TPE_TILES;    // tiles (kBS * kTR candidates) per scorer block
constexpr int64_t kTile = (int64_t)kBS * kTR;
#ifndef TPE_TRF
#define TPE_TRF 32
#endif
constexpr int kTRF = TPE_TRF;        // candidates per thread in the fast scorer (tpe_score_table_fast;
                                     // 32: its per-block setup and band tail over 8192 candidates --
                                     // 0.288 -> 0.272 ms per C3 level against 16, one-box A/B)
constexpr int64_t kTileF = (int64_t)kBS * kTRF;  // its tile: one band tile per scorer block
#ifndef TPE_BUILD_BLOCKS
#define TPE_BUILD_BLOCKS 384
#endif
// build blocks per job (grid-stride over cells).  384, not 512: a C3 uniform
// label has ~180 quads (one per block) and a normal label ~625 block rounds,
// so 512 launched ~330 idle blocks per uniform job and left the normal jobs'
// second round uneven; table-build group 0.229 -> 0.214 ms per C3 level,
// C5 unchanged (1.74 -> 1.68-1.73 ms), two-round A/B on one box (late round 5)
constexpr int kBuildBlocks = TPE_BUILD_BLOCKS;
constexpr int kCoopCells = 4096;     // labels with at most this many cells build a quad per block
constexpr float kLn2T = 0.6931471805599453f;

__device__ __forceinline__ double4 ld4(const double* coef64, int64_t k) {
  return reinterpret_cast<const double4*>(coef64)[k];
}

// s = h*inv such that 9 s (z + s) + 32.5 s^2 <= kRhoLim (|y0-mu| inv <= z + s)
__device__ __forceinline__ double admissible_s(double z) {
  return (-9.0 * z + sqrt(81.0 * z * z + 166.0 * kRhoLim)) / 83.0;
}

// inclusive block scans over threadIdx order (256 threads); `sh` holds one
// entry per wave.  Every thread gets its own inclusive result.
__device__ __forceinline__ double block_scan_max(double v, double* sh) {
  const int lane = lane_id(), wid = threadIdx.x / kWave;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const double o = __shfl_up(v, off, kWave);
    if (lane >= off) v = fmax(v, o);
  }
  __syncthreads();
  if (lane == kWave - 1) sh[wid] = v;
  __syncthreads();
  for (int w = 0; w < wid; ++w) v = fmax(v, sh[w]);
  return v;
}
__device__ __forceinline__ int block_scan_sum(int v, int* sh) {
  const int lane = lane_id(), wid = threadIdx.x / kWave;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int o = __shfl_up(v, off, kWave);
    if (lane >= off) v += o;
  }
  __syncthreads();
  if (lane == kWave - 1) sh[wid] = v;
  __syncthreads();
  for (int w = 0; w < wid; ++w) v += sh[w];
  return v;
}

// ---------------------------------------------------------------------------
// plan: coordinate range, admissible half-width, reach windows, wide list.
// Two launches over (component tiles, 2 * n_jobs) -- y = 2*job + half, half 0
// the below mixture, 1 the above: P1 does every component's reach / bound and
// the tile-local scans, P2 applies the other tiles' carries.
// ---------------------------------------------------------------------------
constexpr int kPlanStride = 4;  // per tile: {max reach_hi, min reach_lo, #wide, min h}

// range of the scoring coordinate (where the below sampler can put a
// candidate: mu +- 5.8 sigma per component, clipped to the bounds) and the
// global lower bound T of a term that can matter (the prior's smallest term
// over the range, minus log(M) + kTauExtra); identical in every block
// draw_z: |z| bound of the sampler's normals (kDrawZ for fp32 draws, kDrawZ64
// for fp64 ones); tau: the exclusion margin (kTauExtra for the table,
// kTauExact for the pruned exact fp64 scorer)
__device__ __forceinline__ void plan_range(const tpe_job& J, const tpe_seg& SB, const tpe_seg& S,
                                           const double* __restrict__ mu,
                                           const double* __restrict__ sigma,
                                           const double* __restrict__ coef64, double* red,
                                           double draw_z, double tau, double& a, double& b,
                                           double& T) {
  a = INFINITY;
  b = -INFINITY;
  for (int k = threadIdx.x; k < SB.n_obs + 1; k += kBS) {
    const double m = mu[SB.comp_off + k], sg = sigma[SB.comp_off + k];
    a = fmin(a, m - draw_z * sg);
    b = fmax(b, m + draw_z * sg);
  }
  a = -block_max<kBS, double>(-a, red);
  b = block_max<kBS, double>(b, red);
  if (J.flags & TPE_F_INJECTED) {
    a = fmax(a, J.bin_lo);
    b = fmin(b, J.bin_hi);
  }
  if (J.flags & TPE_F_LOW) a = fmax(a, J.low);
  if (J.flags & TPE_F_HIGH) b = fmin(b, J.high);
  if (!(isfinite(a) && isfinite(b) && b >= a)) {
    // empty or degenerate: one cell at a finite point, candidates off it are exact
    const double c = isfinite(a) ? a : (isfinite(b) ? b : SB.prior_mu);
    a = b = c;
  }
  const double4 cp = ld4(coef64, S.comp_off + S.prior_pos);
  const double far = fmax(fabs(a - cp.x), fabs(b - cp.x)) * cp.y;
  T = cp.z - 0.5 * far * far - (log((double)(S.n_obs + 1)) + tau);
}

// wide components (the prior, and any with sigma >= prior_sigma / 4) are not
// windowed but listed; decided from the coefficient's 1/sigma everywhere
// (plan and build agree by construction)
__device__ __forceinline__ bool is_wide(const tpe_seg& S, int k, double inv) {
  return (k == S.prior_pos) || (inv <= 4.0 / S.prior_sigma);
}

// component k of mixture S: wide flag, reach interval, admissible half-width
__device__ __forceinline__ void plan_comp(const tpe_seg& S, const double* __restrict__ sigma,
                                          const double* __restrict__ coef64, double T, int k,
                                          bool& wide, double& hr, double& lr, double& hk) {
  const double4 c = ld4(coef64, S.comp_off + k);
  const double d = c.z - T;
  const double z = d > 0.0 ? sqrt(2.0 * d) : 0.0;
  hk = d > 0.0 ? admissible_s(z) / c.y : INFINITY;
  wide = is_wide(S, k, c.y);
  const double r = z / c.y * (1.0 + 1e-9) + 1e-12 * fabs(c.x);
  hr = wide ? -INFINITY : c.x + r;
  lr = wide ? INFINITY : c.x - r;
}

__global__ __launch_bounds__(kBS) void k_table_plan1(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const double* __restrict__ mu, const double* __restrict__ sigma,
    const double* __restrict__ coef64, double* __restrict__ reach_hi,
    double* __restrict__ reach_lo, double* __restrict__ part, tpe_table* __restrict__ tables,
    double draw_z, double tau) {
  __shared__ double red[kBS / kWave];
  __shared__ double scan_d[kBS / kWave];
  const int job = blockIdx.y >> 1, half = blockIdx.y & 1;
  const tpe_job J = jobs[job];
  const tpe_seg SB = segs[J.below];
  const tpe_seg S = segs[half ? J.above : J.below];
  const int nc = S.n_obs + 1;
  if ((int)blockIdx.x * kBS >= nc) return;  // block-uniform
  double a, b, T;
  plan_range(J, SB, S, mu, sigma, coef64, red, draw_z, tau, a, b, T);
  const int k = blockIdx.x * kBS + threadIdx.x;
  bool wide = true;
  double hr = -INFINITY, lr = INFINITY, hk = INFINITY;
  if (k < nc) plan_comp(S, sigma, coef64, T, k, wide, hr, lr, hk);
  hr = block_scan_max(hr, scan_d);  // tile-local prefix max
  if (k < nc) reach_hi[S.comp_off + k] = hr;
  // tile-local suffix min: thread t handles element tile_end - t
  const int tend = min(nc, (int)(blockIdx.x + 1) * kBS) - 1;
  const int kr = tend - (int)threadIdx.x;
  bool wr;
  double hr2, lr2 = INFINITY, hk2;
  if (kr >= (int)blockIdx.x * kBS) plan_comp(S, sigma, coef64, T, kr, wr, hr2, lr2, hk2);
  lr2 = -block_scan_max(-lr2, scan_d);
  if (kr >= (int)blockIdx.x * kBS) reach_lo[S.comp_off + kr] = lr2;
  const double tmax = block_max<kBS, double>(hr, red);
  const double tmin = -block_max<kBS, double>(-lr2, red);
  const double nw = block_sum<kBS, double>((k < nc && wide) ? 1.0 : 0.0, red);
  const double hmin = -block_max<kBS, double>(-hk, red);
  if (threadIdx.x == 0) {
    double* P = part + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * kPlanStride;
    P[0] = tmax;
    P[1] = tmin;
    P[2] = nw;
    P[3] = hmin;
    if (blockIdx.x == 0) {
      if (half == 0) {
        tables[job].lo = a;
        tables[job].hi = b;
        tables[job].T_below = T;
      } else {
        tables[job].T_above = T;
      }
    }
  }
}

__global__ __launch_bounds__(kBS) void k_table_plan2(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const double* __restrict__ mu, const double* __restrict__ sigma,
    const double* __restrict__ coef64, double* __restrict__ reach_hi,
    double* __restrict__ reach_lo, int32_t* __restrict__ wide_idx,
    const double* __restrict__ part, tpe_table* __restrict__ tables) {
  __shared__ double red[kBS / kWave];
  __shared__ int scan_n[kBS / kWave];
  const int job = blockIdx.y >> 1, half = blockIdx.y & 1;
  const tpe_job J = jobs[job];
  const tpe_seg S = segs[half ? J.above : J.below];
  const int nc = S.n_obs + 1;
  const int tiles = (nc + kBS - 1) / kBS;
  const int t = blockIdx.x;
  if (t >= tiles) return;  // block-uniform
  const double* P = part + (int64_t)blockIdx.y * gridDim.x * kPlanStride;
  double chi = -INFINITY, clo = INFINITY, woff = 0.0, hmin = INFINITY, nw = 0.0;
  for (int q = threadIdx.x; q < tiles; q += kBS) {
    if (q < t) {
      chi = fmax(chi, P[q * kPlanStride]);
      woff += P[q * kPlanStride + 2];
    }
    if (q > t) clo = fmin(clo, P[q * kPlanStride + 1]);
    hmin = fmin(hmin, P[q * kPlanStride + 3]);
    nw += P[q * kPlanStride + 2];
  }
  chi = block_max<kBS, double>(chi, red);
  clo = -block_max<kBS, double>(-clo, red);
  const int wbase = (int)block_sum<kBS, double>(woff, red);
  hmin = -block_max<kBS, double>(-hmin, red);
  const int ntot = (int)block_sum<kBS, double>(nw, red);
  const int k = t * kBS + threadIdx.x;
  bool wide = false;
  if (k < nc) {
    reach_hi[S.comp_off + k] = fmax(reach_hi[S.comp_off + k], chi);
    reach_lo[S.comp_off + k] = fmin(reach_lo[S.comp_off + k], clo);
    wide = is_wide(S, k, ld4(coef64, S.comp_off + k).y);
  }
  const int incl = block_scan_sum(wide ? 1 : 0, scan_n);
  if (wide) wide_idx[S.comp_off + wbase + incl - 1] = k;
  if (t == 0 && threadIdx.x == 0) {
    if (half == 0) {
      tables[job].h_below = hmin;
      tables[job].n_wide_below = ntot;
      // raised by k_table_build (build_items, build_ab) and k_table_score
      // (eps_cubic) with atomics: zeroed here, one launch before
      tables[job].build_items = 0;
      tables[job].build_ab = 0.0f;
      tables[job].eps_cubic = 0.0f;
    } else {
      tables[job].h_above = hmin;
      tables[job].n_wide_above = ntot;
    }
  }
}

// cell geometry from the plan (identical in every thread that asks)
struct Grid {
  double origin, h;
  int nb;
};

// centre of cell c in fp32 from the fp32 origin and half-width (the build
// expands around exactly this point; the scorer recomputes it from the cell
// index with the same two operations)
__device__ __forceinline__ float cell_centre(float origin, float h, int c) {
  return fmaf((float)(2 * c + 1), h, origin);
}
__device__ __forceinline__ Grid grid_of(const tpe_table& Tb, int64_t cap) {
  const double span = Tb.hi - Tb.lo;
  double hn = fmin(Tb.h_below, Tb.h_above);
  if (!(hn > 0.0) || !isfinite(hn)) hn = fmax(span, 1.0);
  Grid g;
  if (!(span > 0.0)) {
    g.nb = 1;
    g.h = hn;
    g.origin = Tb.lo - hn;
    return g;
  }
  double n = ceil(span / (2.0 * hn));
  if (!(n <= (double)cap)) n = (double)cap;
  g.nb = (int)fmax(1.0, n);
  g.h = span / (2.0 * g.nb);
  g.origin = Tb.lo;
  return g;
}

// first k with a[k] >= v / last k with a[k] <= v  (a non-decreasing)
__device__ __forceinline__ int first_ge(const double* a, int n, double v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] >= v) hi = mid; else lo = mid + 1;
  }
  return lo;
}
__device__ __forceinline__ int last_le(const double* a, int n, double v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] > v) hi = mid; else lo = mid + 1;
  }
  return lo - 1;
}

// e^x as fp32 for x <= 0 with a relative error <= 2^-22 + 2^-25 (v_exp_f32
// on the fractional part of x log2 e, formed in fp64): the build's rescale and
// merge factors (mix_eps counts two roundings per factor)
__device__ __forceinline__ float exp_acc(double x) {
  const double t = x * kLog2e;
  const double n = floor(t);
  return ldexpf(__builtin_amdgcn_exp2f((float)(t - n)), (int)n);
}
__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, kWave));
  return v;
}

// Wave reductions without the LDS crossbar (all 64 lanes active): DPP within
// each 16-lane row (quad perms, half-row and row mirrors leave the row total
// in every lane of the row), then the four row totals by readlane.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL,
                                                            0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF,
                                                         true);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f<kDppXor1>(v);
  v += dpp_f<kDppXor2>(v);
  v += dpp_f<kDppHalfMirror>(v);
  v += dpp_f<kDppMirror>(v);
  const int b = __builtin_bit_cast(int, v);
  return (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16))) +
         (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48)));
}
// The nine P_n sums of a wave at once (transposed butterfly).  Per DPP stage
// each lane keeps half of its live values and adds its partner's copy of
// them: stage 1 pairs lane i with 15-i of its row (row mirror, bit 3 chooses
// the half), stage 2 with 7-i of its half-row (half mirror, bit 2), stages 3
// and 4 with i^2 and i^1 (quad perms); a stage's partner always holds the same
// subset as the lane, because the mirrors come first.  After four stages lane
// p of each row holds its row's sum of P_rev4(p) (rev4: the 4-bit reversal);
// (row_sum9_transposed: the build sums each row on its own, one cell per
// row): 9 exchange-adds instead of the 9 x 4 of one DPP sum per term.
template <int CTRL, int M>
__device__ __forceinline__ void fold_stage(double (&w)[16], bool hi) {
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const double keep = hi ? w[2 * j + 1] : w[2 * j], send = hi ? w[2 * j] : w[2 * j + 1];
    w[j] = keep + dpp_d<CTRL>(send);
  }
}
__device__ __forceinline__ int rev4(int p) {
  return ((p & 1) << 3) | ((p & 2) << 1) | ((p & 4) >> 1) | ((p & 8) >> 3);
}

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// The two reach windows of the span [ylo, yhi] (a run of cells) at once: four
// searches of wave_first's kind in one pass, one per 16-lane group -- g = 0 /
// 2: the first k of the below / above mixture with reach_hi[k] >= ylo, g = 1 /
// 3: the first k with reach_lo[k] > yhi (the window ends one before it).  16-ary narrowing:
// 10^4 components take 4 dependent probes, for all four searches together
// instead of 3 for each.  Every lane gets all four answers.
struct Windows {
  int lo_b, end_b, lo_a, end_a;
};
__device__ __forceinline__ Windows cell_windows(const tpe_seg& SB, const tpe_seg& SA,
                                                const double* __restrict__ reach_hi,
                                                const double* __restrict__ reach_lo, double ylo,
                                                double yhi) {
  const int lane = lane_id(), g = lane >> 4, l = lane & 15;
  const tpe_seg& S = g < 2 ? SB : SA;
  const bool gt = g & 1;
  const double* a = (gt ? reach_lo : reach_hi) + S.comp_off;
  const double v = gt ? yhi : ylo;
  int lo = 0, hi = S.n_obs + 1;  // answer in [lo, hi]
  while (__any(lo < hi)) {
    const bool active = lo < hi;
    const int stride = (hi - lo + 15) / 16;
    const int idx = lo + l * stride;
    bool p = true;  // probes past the end qualify
    if (active && idx < hi) p = gt ? (a[idx] > v) : (a[idx] >= v);
    const uint32_t m = (uint32_t)(__ballot(p) >> (g * 16)) & 0xFFFFu;
    const int f = m ? __builtin_ctz(m) : 16;
    if (active) {
      if (f == 0) {
        hi = lo;  // a[lo] qualifies
      } else {
        const int nlo = lo + (f - 1) * stride + 1;
        hi = min(lo + f * stride, hi);
        lo = nlo;
      }
    }
  }
  return Windows{__builtin_amdgcn_readlane(lo, 0), __builtin_amdgcn_readlane(lo, 16),
                 __builtin_amdgcn_readlane(lo, 32), __builtin_amdgcn_readlane(lo, 48)};
}

// Row-level reduction (each 16-lane DPP row on its own): the nine P_n sums
// of the row, lane p holding the sum of P_rev4(p) (wave_sum9_transposed
// without the cross-row steps).
__device__ __forceinline__ double row_sum9_transposed(const double (&P)[9]) {
  const int lane = lane_id();
  double w[16];
#pragma unroll
  for (int n = 0; n < 16; ++n) w[n] = n < 9 ? P[n] : 0.0;
  fold_stage<kDppMirror, 5>(w, (lane >> 3) & 1);      // 9 live -> 5
  w[5] = 0.0;
  fold_stage<kDppHalfMirror, 3>(w, (lane >> 2) & 1);  // -> 3
  w[3] = 0.0;
  fold_stage<kDppXor2, 2>(w, (lane >> 1) & 1);        // -> 2
  fold_stage<kDppXor1, 1>(w, lane & 1);               // -> 1
  return w[0];
}

// One wave builds one mixture's expansion on four consecutive cells, one per
// 16-lane row (y0: the row's cell centre); returns the row's failed flag.
// k_lo .. k_hi: the reach window of the four cells' span (cell_windows) --
// a superset of each cell's own, whose components the exclusion test below
// drops -- then the wide list; every row walks the same items.
struct BuildLds {  // the block's four waves' partial expansions of one mixture
  int m[kBS / kWave][4];         // per wave and row: its scale (a power of two's exponent)
  double p[kBS / kWave][kWave];  // per wave and lane: its row's sum of P_rev4(lane & 15)
  int bad[kBS / kWave][4];
};
__device__ __forceinline__ int row_max_i(int v) {  // max over the lane's 16-lane DPP row
  v = max(v, __builtin_amdgcn_mov_dpp(v, kDppXor1, 0xF, 0xF, true));
  v = max(v, __builtin_amdgcn_mov_dpp(v, kDppXor2, 0xF, 0xF, true));
  v = max(v, __builtin_amdgcn_mov_dpp(v, kDppHalfMirror, 0xF, 0xF, true));
  v = max(v, __builtin_amdgcn_mov_dpp(v, kDppMirror, 0xF, 0xF, true));
  return v;
}
constexpr int kNoScale = -100000;  // a lane that has summed nothing yet
__device__ __forceinline__ bool build_mix(const tpe_seg& S, const double* __restrict__ coef64,
                                          int k_lo, int k_hi,
                                          const int32_t* __restrict__ wide_idx, int n_wide,
                                          double T, double y0, double h, float* cell, bool store,
                                          int mix, double& m_out, BuildLds& X, bool coop,
                                          int& itm) {
  // coop (block-uniform): the block's four waves build the same four cells
  // and split the items; otherwise every wave builds its own four cells
  constexpr int kNW = kBS / kWave;
  const int wv = coop ? (int)threadIdx.x / kWave : 0;
  const int stride = coop ? 16 * kNW : 16;
  const int64_t off = S.comp_off;
  const int nwin = max(0, k_hi - k_lo + 1);
  const int items = nwin + n_wide;
  itm = max(itm, items);  // (the error bound's summation depth, mix_eps)
  const int lane = lane_id(), l = lane & 15, row = lane >> 4;
  // component of work item `it` (window first, then the wide list)
  auto comp = [&](int it) -> int {
    return it < nwin ? k_lo + it : wide_idx[off + (it - nwin)];
  };
  const float hf = (float)h, Tf = (float)T;
  // One pass over the items.  Each lane keeps its own scale 2^sl (sl an
  // integer, raised when a term would exceed 2^8 of it) and rescales its
  // partial sums by exact powers of two; the row's lanes (and the block's
  // waves, coop) meet at the largest scale the same way, and the cell's sums
  // are finally normalised by the power of two that puts P_0 in [1, 2) --
  // every rescaling exact, P_0 >= 1 as the storage bound assumes.  The
  // exponent is formed in fp64, the series and the per-component tests in
  // fp32.  P_0..P_3 are summed in fp64 (a sum of ~10^2 fp32 terms per lane
  // would carry ~10^2 roundings into mix_eps), P_4..P_8 in fp32: at most 2 %
  // of the terms' absolute sum lies there (tools/table_bounds.py), so their
  // rounding costs mix_eps K 2^-24 0.0198.  The next item's coefficients are
  // loaded before this item's work.
  constexpr int kP64 = 4;
  double P[kP64];
  float Q[kP - kP64];
#pragma unroll
  for (int n = 0; n < kP64; ++n) P[n] = 0.0;
#pragma unroll
  for (int n = 0; n < kP - kP64; ++n) Q[n] = 0.0f;
  auto acc = [&](int n, float t) __attribute__((always_inline)) {
    if (n < kP64)
      P[n] += (double)t;
    else
      Q[n - kP64] += t;
  };
  auto rescale = [&](int d) __attribute__((always_inline)) {  // multiply the sums by 2^d
#pragma unroll
    for (int n = 0; n < kP64; ++n) P[n] = ldexp(P[n], d);
#pragma unroll
    for (int n = 0; n < kP - kP64; ++n) Q[n] = ldexpf(Q[n], d);
  };
  int sl = kNoScale;
  bool bad = false;
  int it = wv * 16 + l;  // the block's four waves split the items, 16 lanes per cell each
  int k = it < items ? comp(it) : 0;
  double4 c = it < items ? ld4(coef64, off + k) : make_double4(0.0, 0.0, 0.0, 0.0);
  for (; it < items; it += stride) {
    const int itn = it + stride;
    const int kn = itn < items ? comp(itn) : 0;
    const double4 cn = itn < items ? ld4(coef64, off + kn) : c;
    // window items that are wide come from the list instead; an item below
    // the plan's floor on the whole cell is left out (branch-free: an
    // excluded item adds zero terms)
    const bool skip = it < nwin && is_wide(S, k, c.y);
    const double dy = y0 - c.x;
    const float dyf = (float)dy, inv = (float)c.y;
    const float zn = fmaxf(fabsf(dyf) - hf, 0.0f) * inv;
    const bool inc = !skip && ((float)c.z - 0.5f * zn * zn >= Tf);
    const double zc = dy * c.y;
    const double t2 = (c.z - 0.5 * zc * zc) * kLog2e;  // log2 of the term at the centre
    const bool up = inc && t2 > (double)(sl + 8);
    if (__any(up)) {
      if (up) {
        const int ns = (int)ceil(t2);
        rescale(max(sl - ns, -1100));
        sl = ns;
      }
    }
    const float hi2 = hf * inv * inv;
    const float Af = inc ? -dyf * hi2 : 0.0f, B2 = inc ? -hf * hi2 : 0.0f;  // A and 2B
    bad = bad || (9.0f * fabsf(Af) + 32.5f * fabsf(B2) > (float)(kRhoLim * (1.0 + 1e-5)));
    // the term 2^(t2 - sl) = 2^n 2^f, n = floor(t2 - sl) exact and f in [0, 1)
    // rounded once to fp32: a relative error <= ln2 2^-24 (+ v_exp_f32's),
    // whatever the term's size
    const double xs = t2 - (double)sl, xn = floor(xs);
    const float e = inc ? ldexpf(__builtin_amdgcn_exp2f((float)(xs - xn)), (int)xn) : 0.0f;
    float cm = 0.0f, cc = e;  // e * c_n
    acc(0, e);
#pragma unroll
    for (int n = 0; n + 1 < kP; ++n) {
      const float cnx = fmaf(Af, cc, B2 * cm) * (1.0f / (float)(n + 1));
      acc(n + 1, cnx);
      cm = cc;
      cc = cnx;
    }
    k = kn;
    c = cn;
  }
  // the row's lanes at the row's largest scale (exact); then the block's
  // waves at theirs (coop)
  int sr = row_max_i(sl);
  rescale(max(sl - sr, -1100));
  static_assert(kP == 9, "row_sum9_transposed folds nine terms");
  double Pall[kP];
#pragma unroll
  for (int n = 0; n < kP; ++n) Pall[n] = n < kP64 ? P[n] : (double)Q[n - kP64];
  double tot = row_sum9_transposed(Pall);  // lane p of the row: the row's total of P_rev4(p)
  bad = ((__ballot(bad) >> (lane & ~15)) & 0xFFFFull) != 0;
  bool anybad = bad;
  if (coop) {
    if (l == 0) {
      X.bad[wv][row] = bad;
      X.m[wv][row] = sr;
    }
    X.p[wv][lane] = tot;
    __syncthreads();
    int sb = X.m[0][row];
#pragma unroll
    for (int w = 1; w < kNW; ++w) sb = max(sb, X.m[w][row]);
    tot = 0.0;
    anybad = false;
    for (int w = 0; w < kNW; ++w) {
      tot += ldexp(X.p[w][lane], max(X.m[w][row] - sb, -1100));
      anybad = anybad || X.bad[w][row];
    }
    sr = sb;
    __syncthreads();  // (X is reused by the next call)
  }
  // normalise: P_0 (the row's lane 0) in [1, 2)
  const double p0 = __shfl(tot, lane & ~15, kWave);
  int e0 = 0;
  if (p0 > 0.0) {
    (void)frexp(p0, &e0);  // p0 = f 2^e0, f in [0.5, 1)
    e0 -= 1;
    tot = ldexp(tot, -e0);
  }
  const int n = rev4(l);
  if (store && wv == 0 && n < kP) {
    if (n < kP32)
      cell[2 * n + mix] = (float)tot;
    else
      reinterpret_cast<_Float16*>(cell + 2 * kP32)[2 * (n - kP32) + mix] = (_Float16)(float)tot;
  }
  m_out = (p0 > 0.0) ? (double)(sr + e0) * kLn2 : -INFINITY;
  return anybad;
}

// ---------------------------------------------------------------------------
// score cells.  The argmax needs only the score
//     f(u) = (m_b - m_a) + log P_b(u) - log P_a(u)
// per candidate, and on a cell f is far smoother than either mixture (a
// difference of two log-densities, sampled at half-widths of ~0.06 of the
// narrowest bandwidth): a cubic interpolant at four Chebyshev nodes of
// [-1.05, 1.05] reproduces it to ~1e-7 on C3's histories.
// k_table_score gives each cell kScoreLanes = 8 lanes: lanes 0-3 evaluate f
// at the nodes from the cell's STORED coefficients (fp32 Horner, the log of
// the ratio as exponent + v_log_f32 of the mantissa); the nodes' values are
// broadcast, every lane forms the same cubic (fp64 divided differences) and
// rounds it to fp32.  Then the cubic's error is BOUNDED, not sampled: lane i
// takes the sub-interval of [-1.0501, 1.0501] centred at c_i (half-width
// r = 1.0501 / 8) and encloses
//     e(c_i + t) = f^(c_i + t) - q(c_i + t),   |t| <= r,
// f^ = off + ln P^_b - ln P^_a being the score of the stored polynomials
// (exact reals).  Per mixture: the Taylor coefficients T_k of P^ at c_i (a
// Horner shift), a_k = T_k / T_0, the log series ln P^(c+t) = ln T_0 +
// sum_k l_k t^k with l_k = a_k - (1/k) sum_{j<k} j l_j a_{k-j} (exact up to
// fp64 rounding) for k <= kLogD, and the rest bounded by the majorant
// -ln(1 - w~(t)), w~ = sum |a_k| t^k: its coefficients m_k >= |l_k| (same
// recurrence on |a_k|, all terms positive), summed for kLogD < k <= kLogM,
// and past kLogM by Cauchy's estimate on the radius 4r (m_k (4r)^k <=
// -ln(1 - w~(4r)) <= ln 2 when w~(4r) <= 1/2; otherwise the cell is flagged).
// So |e| <= |E_0| + sum_{k<=kLogD} |E_k| r^k + rem_b + rem_a + rounding, E_k
// the coefficients of the difference polynomial; the cell's bound is the
// largest of its lanes'.  A cell whose bound exceeds kFitTol (or whose P is
// not positive, or whose cubic is not finite) is flagged (NaN c0) and its
// candidates take the two-polynomial cell.  The job's tpe_table gets
//   slope     = max |c1| + 2.11 |c2| + 3.31 |c3|  (>= |q'(u)| on |u| <= 1.0501)
//   eps_cubic = max over unflagged cells of  fit + 2^-21 sum_k |c_k| 1.0501^k
//               + 4.5 2^-24 slope_cell + 2^-24 |off| (1 + 1e-4)
// (the cubic's fp32 Horner beyond its 2^-22 |s| part, u's fp32 rounding, the
// fp32 score offset) and eps_mix, the per-mixture polynomial bound
// (mix_eps).  16 B per cell, after the job's cells and m pairs in its
// 128-B-per-cell region.
// ---------------------------------------------------------------------------
constexpr double kFitTol = 1.0e-6;   // cubic-vs-polynomial bound allowed (nats)
constexpr int kScoreLanes = 8;       // lanes per cell: 4 nodes, 8 sub-intervals
constexpr int kScoreCellsPerBlock = kBS / kScoreLanes;
#ifndef TPE_SCORE_BLOCKS
#define TPE_SCORE_BLOCKS 160
#endif
// per job (grid-stride over cells).  160, not 256: a C3 normal label's ~10 000
// cells are ~313 block rounds (two even rounds instead of 1.2), a uniform
// label's 710 cells need 23 blocks; build group -5 us per C3 level, C5
// unchanged (three one-box A/Bs, late round 5)
constexpr int kScoreBlocks = TPE_SCORE_BLOCKS;
constexpr double kUFit = 1.0501;     // |u| the bounds cover (u's fp32 rounding: <= 1.05 (1 + 5 2^-24))
constexpr int kLogD = 7;             // log-series terms carried exactly
constexpr int kLogM = 12;            // majorant terms summed (then Cauchy's tail)
constexpr double kU32 = 0x1.0p-24;   // fp32 unit roundoff
// max of a + b = 1.0501|A| + 1.1028|B| over the admissible set 9|A| + 65|B| <=
// 5.8 (1 + 2e-5) (the build's test with its fp32 slack): at |A| = 0.64446
constexpr double kAbMax = 0.6768;

// Per-mixture relative error bound of a stored cell polynomial against its
// mixture, |P^(u) - S(y) e^-m| <= eps_mix S(y) e^-m on |u| <= kUFit, from the
// build's worst case over the job's cells (DESIGN.md 3.1 derives each term):
// items = most components one cell summed, coop = the cooperative build (64
// lanes per row), ab = max 1.0501|A| + 1.1028|B| of a summed component (also
// >= a + 2b).  Terms relative to a component's value carry e^ab (its
// majorant over its value at u); those of the P_n sums carry E2 = e^2ab.
__host__ __device__ inline double mix_eps(int items, bool coop, double ab) {
  const double u = kU32, ud = 0x1.0p-53;
  const int stride = coop ? 64 : 16;
  const int K = (items + stride - 1) / stride + 5 + (coop ? 5 : 0);  // fp64 adds into one P_n
  const double E1 = exp(ab), E2 = E1 * E1;
  return 4.4e-7                         // series truncation (tools/table_bounds.py)
         + 1.0e-10                      // components below the exclusion floor
         + 0.6932 * u + 1e-13           // each term's exponent: its fraction rounded to fp32
         + 0x1.0p-22                    // v_exp_f32 (checked exhaustively, tpe_check_transcendentals)
         + 5.5 * u * ab                 // A, B rounded to fp32
         + 4.0 * u * ab * E2            // the fp32 series recurrence (4 roundings per step)
         + u * E2                       // P_0..P_5 stored in fp32
         + (K + 1) * u * 0.0198 * 1.0001  // P_4..P_8 summed in fp32 (tools/table_bounds.py)
         + 1.5e-7 + 0x1.0p-25 * 4.2 * E1  // P_6..P_8 in fp16 (+ subnormal spacing)
         + (K + 8) * 2.0 * ud * E2;     // fp64 sums, rescale and merge factors of the P_n
}

// The LGMM1 candidate drawn as y (fp32) is returned as x = exp(y) in fp64
// (cand_value), and the reference scores log(x) (tpe.py:284-287 via
// lognormal_lpdf, :208-217), which differs from y by the two roundings:
// |log(exp(y)) - y| <= 2^-51 (1 + |y|).  In cell units (|y| <= max(|lo|, |hi|)
// on the grid) that is a shift of u by at most this; the error bounds add it
// times the slope (the cubic's, or |P'| of the two-polynomial cell), so the
// band holds the winner of the scores at log(x).  0 for GMM1.
__host__ __device__ inline float lgmm_du(const tpe_job& J, const tpe_table& T) {
  if (J.family != TPE_LGMM1 || !(T.h > 0.0)) return 0.0f;
  const double ym = fmax(fabs(T.lo), fabs(T.hi)) + 2.0 * T.h;
  return (float)(0x1.0p-51 * (1.0 + ym) / T.h * 1.01);
}

__device__ __forceinline__ const float4* score_cells_of(const char* region, int64_t cap) {
  return reinterpret_cast<const float4*>(region + ((cap * (int64_t)(kCellF * 4 + 8) + 15) & ~15ll));
}

// one mixture's stored coefficients as doubles (exact)
__device__ __forceinline__ void cell_coefs(const float* cell, int mix, double (&p)[kP]) {
  const _Float16* tail = reinterpret_cast<const _Float16*>(cell + 2 * kP32);
#pragma unroll
  for (int n = 0; n < kP32; ++n) p[n] = (double)cell[2 * n + mix];
#pragma unroll
  for (int n = kP32; n < kP; ++n) p[n] = (double)(float)tail[2 * (n - kP32) + mix];
}

// ln P^(c + t) = lnT0 + sum_{k=1..kLogD} l[k] t^k + R, |R| <= rem on |t| <= r;
// false when P^(c) <= 0 or the majorant's radius check fails
__device__ __forceinline__ bool log_taylor(const double (&p)[kP], double c, double r, double& lnT0,
                                           double (&l)[kLogD + 1], double& rem) {
  double T[kP];
#pragma unroll
  for (int n = 0; n < kP; ++n) T[n] = p[n];
#pragma unroll
  for (int i = 0; i < kP - 1; ++i)
#pragma unroll
    for (int j = kP - 2; j >= i; --j) T[j] = fma(c, T[j + 1], T[j]);
  if (!(T[0] > 0.0) || !isfinite(T[0])) return false;
  lnT0 = log(T[0]);
  const double inv0 = 1.0 / T[0];
  double a[kP];
  a[0] = 1.0;
#pragma unroll
  for (int k = 1; k < kP; ++k) a[k] = T[k] * inv0;
  l[0] = 0.0;
#pragma unroll
  for (int k = 1; k <= kLogD; ++k) {
    double s = 0.0;
#pragma unroll
    for (int j = 1; j < k; ++j) s = fma((double)j * l[j], a[k - j], s);
    l[k] = a[k] - s * (1.0 / (double)k);
  }
  // majorant of the log series (fp32: a bound, inflated by 1e-3 below)
  float aa[kP], m[kLogM + 1];
  float w4 = 0.0f, rr = 1.0f;
  const float r4 = (float)(4.0 * r);
#pragma unroll
  for (int k = 1; k < kP; ++k) {
    aa[k] = (float)fabs(a[k]);
    rr *= r4;
    w4 = fmaf(aa[k], rr, w4);
  }
  w4 *= 1.001f;
  if (!(w4 <= 0.5f)) return false;
  float tail = 0.0f, rk = 1.0f, jm[kLogM + 1];  // jm[j] = j m_j
  const float rf = (float)r;
#pragma unroll
  for (int k = 1; k <= kLogM; ++k) {
    // m_k = |a_k| + (1/k) sum_j j m_j |a_{k-j}| (fp32 rounding inside the
    // 1e-3 inflation below)
    float s = 0.0f;
#pragma unroll
    for (int j = 1; j < k; ++j)
      if (k - j < kP) s = fmaf(jm[j], aa[k - j], s);
    const float mk = fmaf(s, 1.0f / (float)k, k < kP ? aa[k] : 0.0f);
    m[k] = mk;
    jm[k] = (float)k * mk;
    rk *= rf;
    if (k > kLogD) tail = fmaf(mk, rk, tail);
  }
  // past kLogM: m_k (4r)^k <= ln 2, so sum_{k > kLogM} m_k r^k <= ln2 4^-(M+1) / (3/4)
  rem = (double)tail * 1.001 + 0.6931471805599453 * ldexp(1.0, -2 * (kLogM + 1)) / 0.75;
  return true;
}

#ifndef TPE_TSCORE_WPE  // diagnostic builds: waves-per-EU target of the cubics kernel
#define TPE_TSCORE_WPE 4
#endif
__global__ __launch_bounds__(kBS) __attribute__((amdgpu_waves_per_eu(TPE_TSCORE_WPE))) void k_table_score(const tpe_job* __restrict__ jobs,
                                                     tpe_table* __restrict__ tables,
                                                     float* __restrict__ cells,
                                                     unsigned long long* __restrict__ stats) {
  __shared__ float fred[kBS / kWave];
  const tpe_job J = jobs[blockIdx.y];
  const tpe_table Tb = tables[blockIdx.y];
  const int nb = Tb.nb;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // the per-mixture bound from the build's worst case (k_table_build's atomics)
    tables[blockIdx.y].build_ab = (float)kAbMax;
    tables[blockIdx.y].eps_mix =
        (float)(mix_eps(Tb.build_items, nb <= kCoopCells, kAbMax) * (1.0 + 1e-6));
  }
  char* region = reinterpret_cast<char*>(cells) + J.tbl_off * kSlotB;
  float4* outs = const_cast<float4*>(score_cells_of(region, J.tbl_cap));
  const int sub = threadIdx.x / kScoreLanes, l = threadIdx.x % kScoreLanes;
  const int gbase = lane_id() & ~(kScoreLanes - 1);  // first lane of this cell's group
  constexpr double kU = (double)kULim;
  const double nd0 = kU * 0.92387953251128674, nd1 = kU * 0.38268343236508978, nd2 = -nd1,
               nd3 = -nd0;
  const double un = l == 0 ? nd0 : l == 1 ? nd1 : l == 2 ? nd2 : nd3;  // (lanes >= 4: unused)
  const double i10 = 1.0 / (nd1 - nd0), i21 = 1.0 / (nd2 - nd1), i32 = 1.0 / (nd3 - nd2),
               i20 = 1.0 / (nd2 - nd0), i31 = 1.0 / (nd3 - nd1), i30 = 1.0 / (nd3 - nd0);
  const float uf = (float)un;
  // LGMM1: the exact score is taken at log(exp(y)) of the returned value, not
  // at y (cand_value) -- a shift of u by at most du_lg (lgmm_du)
  const float du_lg = lgmm_du(J, Tb);
  constexpr double r = kUFit / kScoreLanes;
  const double cI = -kUFit + (2 * l + 1) * r;  // this lane's sub-interval centre
  float slope = 0.0f, epsc = 0.0f;  // over this thread's unflagged cells (lane 0 of a group)
  // group-uniform trip count: every lane of a group runs the shuffles
  for (int64_t c = (int64_t)blockIdx.x * kScoreCellsPerBlock + sub; c < nb;
       c += (int64_t)gridDim.x * kScoreCellsPerBlock) {
    const float* cell = reinterpret_cast<const float*>(region) + c * kCellF;
    const double off = (double)cell[15];
    const _Float16* tail = reinterpret_cast<const _Float16*>(cell + 2 * kP32);
    float pb = 0.0f, pa = 0.0f;
#pragma unroll
    for (int n = kP - 1; n >= kP32; --n) {
      pb = fmaf(pb, uf, (float)tail[2 * (n - kP32)]);
      pa = fmaf(pa, uf, (float)tail[2 * (n - kP32) + 1]);
    }
#pragma unroll
    for (int n = kP32 - 1; n >= 0; --n) {
      pb = fmaf(pb, uf, cell[2 * n]);
      pa = fmaf(pa, uf, cell[2 * n + 1]);
    }
    const bool ok_pt = (pb > 0.0f) && (pa > 0.0f) && isfinite(pb) && isfinite(pa);
    // log(pb / pa) = ln2 * (e + log2(m)), m = the ratio's mantissa in [0.5, 1)
    int e = 0;
    const float mt = ok_pt ? frexpf(pb / pa, &e) : 1.0f;
    const double f = off + kLn2 * ((double)e + (double)__builtin_amdgcn_logf(mt));
    const double f0 = __shfl(f, gbase + 0, kWave), f1 = __shfl(f, gbase + 1, kWave),
                 f2 = __shfl(f, gbase + 2, kWave), f3 = __shfl(f, gbase + 3, kWave);
    const bool nodes_ok = ((__ballot(!ok_pt) >> gbase) & 0xFull) == 0;
    // Newton divided differences -> monomial coefficients of the cubic (the
    // node spacings' reciprocals are constants: multiplies, not fp64
    // divisions -- q is an approximation whose own error the bound below
    // measures, so its last bits are free)
    const double d01 = (f1 - f0) * i10, d12 = (f2 - f1) * i21, d23 = (f3 - f2) * i32;
    const double d012 = (d12 - d01) * i20, d123 = (d23 - d12) * i31;
    const double d0123 = (d123 - d012) * i30;
    const double c3 = d0123;
    const double c2 = d012 - d0123 * (nd0 + nd1 + nd2);
    const double c1 = d01 - d012 * (nd0 + nd1) + d0123 * (nd0 * nd1 + nd0 * nd2 + nd1 * nd2);
    const double c0 = f0 - d01 * nd0 + d012 * nd0 * nd1 - d0123 * nd0 * nd1 * nd2;
    const float4 q = make_float4((float)c0, (float)c1, (float)c2, (float)c3);
    // the bound of |f^ - q| on this lane's sub-interval
    const double q0 = q.x, q1 = q.y, q2 = q.z, q3 = q.w;
    bool fail = !nodes_ok || !(off == off) || !isfinite(q0) || !isfinite(q1) || !isfinite(q2) ||
                !isfinite(q3);
    double bound = INFINITY;
    if (!fail) {
      double pbv[kP], pav[kP], lb[kLogD + 1], la[kLogD + 1], lnb = 0.0, lna = 0.0, rb = 0.0,
             ra = 0.0;
      cell_coefs(cell, 0, pbv);
      cell_coefs(cell, 1, pav);
      const bool okb = log_taylor(pbv, cI, r, lnb, lb, rb);
      const bool oka = log_taylor(pav, cI, r, lna, la, ra);
      if (okb && oka) {
        // the cubic's Taylor coefficients at cI
        const double qc = ((q3 * cI + q2) * cI + q1) * cI + q0;
        const double qk[4] = {qc, (3.0 * q3 * cI + 2.0 * q2) * cI + q1, 3.0 * q3 * cI + q2, q3};
        const double E0 = off + lnb - lna - qc;
        double sum = fabs(E0), rk = 1.0;
#pragma unroll
        for (int k = 1; k <= kLogD; ++k) {
          rk *= r;
          const double Ek = lb[k] - la[k] - (k < 4 ? qk[k] : 0.0);
          sum = fma(fabs(Ek), rk, sum);
        }
        // fp64 rounding of the whole computation (magnitudes ~|off| + |ln T0|)
        const double slack = 1e-13 * (1.0 + fabs(off) + fabs(lnb) + fabs(lna) + fabs(qc));
        bound = sum + rb + ra + slack;
      }
    }
    // the cell's bound: the largest of its 8 lanes'
    float bmax = (float)(bound * (1.0 + 1e-6));
#pragma unroll
    for (int o = 1; o < kScoreLanes; o <<= 1) bmax = fmaxf(bmax, __shfl_xor(bmax, o, kWave));
    if (!(bmax == bmax)) bmax = INFINITY;
    fail = fail || !(bmax <= (float)kFitTol);
    const bool bad = ((__ballot(fail) >> gbase) & ((1ull << kScoreLanes) - 1)) != 0;
    if (l == 0) {
      outs[c] = bad ? make_float4(__int_as_float(0x7FC00000), 0.0f, 0.0f, 0.0f) : q;
      if (bad && stats) atomicAdd(stats + 2, 1ull);
      if (!bad) {
        // |q'(u)| <= |c1| + 2|c2||u| + 3|c3|u^2 on |u| <= 1.0501
        const float sl = fabsf(q.y) + 2.11f * fabsf(q.z) + 3.31f * fabsf(q.w);
        slope = fmaxf(slope, sl);
        const float ev = 0x1.0p-21f * (1.0501f * fabsf(q.y) + 1.1028f * fabsf(q.z) +
                                        1.1581f * fabsf(q.w));
        const float ec = bmax + ev + (4.5f * 0x1.0p-24f + du_lg) * sl +
                         0x1.0p-24f * 1.0001f * (float)fabs(off);
        epsc = fmaxf(epsc, ec * 1.0001f);
      }
    }
  }
  slope = block_max<kBS, float>(slope, fred);
  epsc = block_max<kBS, float>(epsc, fred);
  // non-negative floats order as their bits
  if (threadIdx.x == 0 && slope > 0.0f)
    atomicMax(reinterpret_cast<unsigned int*>(&tables[blockIdx.y].slope), __float_as_uint(slope));
  if (threadIdx.x == 0 && epsc > 0.0f)
    atomicMax(reinterpret_cast<unsigned int*>(&tables[blockIdx.y].eps_cubic),
              __float_as_uint(epsc));
}

#ifndef TPE_BUILD_WPE  // diagnostic builds: waves-per-EU target of the build kernel
#define TPE_BUILD_WPE 1
#endif
__global__ __launch_bounds__(kBS) __attribute__((amdgpu_waves_per_eu(TPE_BUILD_WPE))) void k_table_build(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const double* __restrict__ sigma, const double* __restrict__ coef64,
    const double* __restrict__ reach_hi, const double* __restrict__ reach_lo,
    const int32_t* __restrict__ wide_idx, tpe_table* __restrict__ tables,
    float* __restrict__ cells, unsigned long long* __restrict__ stats) {
  const tpe_job J = jobs[blockIdx.y];
  const tpe_table Tb = tables[blockIdx.y];
  const Grid g = grid_of(Tb, J.tbl_cap);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    tpe_table* W = tables + blockIdx.y;
    W->origin = g.origin;
    W->h = g.h;
    W->inv_h = (float)(1.0 / g.h);
    W->inv_w = (float)(0.5 / g.h);
    W->nb = g.nb;
    W->slope = 0.0f;  // raised by k_table_score (the next launch)
  }
  const tpe_seg SB = segs[J.below], SA = segs[J.above];
  const int wid = threadIdx.x / kWave, row = lane_id() >> 4;
  float* region = cells + J.tbl_off * (kSlotB / 4);
  __shared__ BuildLds X;
  // four consecutive cells (a "quad", one per 16-lane row) per wave; a label
  // with few cells (wide windows: many components per cell) gives each quad
  // the whole block, whose four waves split the components -- so it still
  // spreads over many waves when it is one of a rank's few labels
  const bool coop = g.nb <= kCoopCells;  // block-uniform
  const int64_t q0 = coop ? blockIdx.x : (int64_t)blockIdx.x * (kBS / kWave) + wid;
  const int64_t qs = coop ? gridDim.x : (int64_t)gridDim.x * (kBS / kWave);
  int itm = 0;       // most items a cell of this wave summed
  for (int64_t q = q0; 4 * q < g.nb; q += qs) {
    const int c0 = (int)(4 * q), c1 = min(c0 + 3, g.nb - 1);
    const int c = c0 + row;
    const bool mine = c < g.nb;
    const double y0 = (double)cell_centre((float)g.origin, (float)g.h, min(c, c1));
    const double ylo = (double)cell_centre((float)g.origin, (float)g.h, c0) - g.h;
    const double yhi = (double)cell_centre((float)g.origin, (float)g.h, c1) + g.h;
    float* out = region + (int64_t)min(c, c1) * kCellF;
    double mb, ma;
    const Windows w = cell_windows(SB, SA, reach_hi, reach_lo, ylo, yhi);
    const bool bb = build_mix(SB, coef64, w.lo_b, w.end_b - 1, wide_idx, Tb.n_wide_below,
                              Tb.T_below, y0, g.h, out, mine, 0, mb, X, coop, itm);
    const bool ba = build_mix(SA, coef64, w.lo_a, w.end_a - 1, wide_idx, Tb.n_wide_above,
                              Tb.T_above, y0, g.h, out, mine, 1, ma, X, coop, itm);
    if ((!coop || wid == 0) && (lane_id() & 15) == 0 && mine) {
      // dword 15: the score offset m_below - m_above, NaN marks a failed cell
      out[15] = (bb || ba) ? __int_as_float(0x7FC00000) : (float)(mb - ma);
      float* mp = region + (int64_t)J.tbl_cap * kCellF + 2 * c;  // (m_below, m_above)
      mp[0] = (float)mb;
      mp[1] = (float)ma;
      if ((bb || ba) && stats) atomicAdd(stats + 1, 1ull);
    }
  }
  // the job's worst case for the polynomial bound (mix_eps, k_table_score):
  // one atomic per wave (itm is wave-uniform)
  if (lane_id() == 0 && itm > 0) atomicMax(&tables[blockIdx.y].build_items, itm);
}

// ---------------------------------------------------------------------------
// scoring
// ---------------------------------------------------------------------------
typedef float f4 __attribute__((ext_vector_type(4)));  // native vector (no memcpy copies)

// f(integral_constant<int, R>) for R = B .. E-1, unrolled at compile time
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// both mixtures' degree-8 polynomials at u: q0..q2 = fp32 pairs
// (b_2k, a_2k, b_2k+1, a_2k+1), q3 = fp16 pairs {b_n | a_n} for n = 6..8 (and
// the score offset in q3.w).  The fp16 tail P_6 + u(P_7 + u P_8) is evaluated
// in packed fp16 (v_pk_fma_f16, both mixtures per instruction; its rounding is
// bounded in tools/table_bounds.py), the fp32 steps are packed FMAs
// (v_pk_fma_f32) on adjacent registers
typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void horner9x2(const f4 q0, const f4 q1, const f4 q2, const f4 q3,
                                          float u, float& pb, float& pa) {
  static_assert(kP == 9 && kP32 == 6, "six fp32 and three fp16 terms");
  const h2_t c6 = __builtin_bit_cast(h2_t, q3.x), c7 = __builtin_bit_cast(h2_t, q3.y),
             c8 = __builtin_bit_cast(h2_t, q3.z);
  const _Float16 uh = (_Float16)u;
  const h2_t uu = {uh, uh};
  h2_t t = __builtin_elementwise_fma(c8, uu, c7);
  t = __builtin_elementwise_fma(t, uu, c6);
  float b = (float)t.x, a = (float)t.y;
#define TPE_H2(cb, ca) b = fmaf(b, u, cb); a = fmaf(a, u, ca);
  TPE_H2(q2.z, q2.w) TPE_H2(q2.x, q2.y) TPE_H2(q1.z, q1.w) TPE_H2(q1.x, q1.y)
  TPE_H2(q0.z, q0.w) TPE_H2(q0.x, q0.y)
#undef TPE_H2
  pb = b;
  pa = a;
}

// exact fp32 log-sum-exp over every component (natural log), the dense
// kernel's arithmetic: t = xc*a + b, v = c - t^2 in log2 units offset by cmax
__device__ __forceinline__ float lse_exact32(const float4* __restrict__ coef, const tpe_seg& S, float y) {
  const float xc = y - (float)S.center;
  float m = -INFINITY, s = 0.0f;
#pragma unroll 8
  for (int k = 0; k < S.n_obs + 1; ++k) {
    const float4 c = coef[k];
    const float t = fmaf(xc, c.x, c.y);
    const float v = fmaf(-t, t, c.z);
    if (v > m) {
      s = s * __builtin_amdgcn_exp2f(m - v) + 1.0f;
      m = v;
    } else {
      s += __builtin_amdgcn_exp2f(v - m);
    }
  }
  return (m + __builtin_amdgcn_logf(s) + (float)S.cmax) * kLn2T;
}

// The same log-sum-exp with the whole wave on one candidate (y wave-uniform,
// every lane active): lane l sums components l, l + 64, ... online, then the
// 64 partial sums are merged at the wave's maximum.  A per-lane serial sum over
// 10^4 components is ~10^5 instructions in one lane -- a tail of ~100 us for
// the wave that holds such a candidate.  Rounding: <= M/64 + 8 sequential
// steps per term, inside the bound taken for the serial sum (kEpsLse).
__device__ __forceinline__ float lse_wave32(const float4* __restrict__ coef, const tpe_seg& S,
                                            float y) {
  const float xc = y - (float)S.center;
  float m = -INFINITY, s = 0.0f;
  for (int k = lane_id(); k < S.n_obs + 1; k += kWave) {
    const float4 c = coef[k];
    const float t = fmaf(xc, c.x, c.y);
    const float v = fmaf(-t, t, c.z);
    if (v > m) {
      s = s * __builtin_amdgcn_exp2f(m - v) + 1.0f;
      m = v;
    } else {
      s += __builtin_amdgcn_exp2f(v - m);
    }
  }
  float M = m;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) M = fmaxf(M, __shfl_xor(M, o, kWave));
  float t = (m == -INFINITY) ? 0.0f : s * __builtin_amdgcn_exp2f(m - M);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o, kWave);
  return (M + __builtin_amdgcn_logf(t) + (float)S.cmax) * kLn2T;
}

template <bool INJ>
__global__ __launch_bounds__(kBS) void k_score_table(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const double* __restrict__ mu, const double* __restrict__ sigma,
    const double* __restrict__ wcdf, const float4* __restrict__ coef32,
    const tpe_table* __restrict__ tables, const float* __restrict__ cells,
    const double* __restrict__ cand, double* __restrict__ out_bl, double* __restrict__ out_al,
    double* __restrict__ out_x, tpe_best* __restrict__ partial,
    unsigned long long* __restrict__ stats, int n_tiles, int n_jobs) {
  __shared__ MixLds s_mix;
  // per wave: 4 DMA slabs of 64 x 16 B, the gather's LDS image; also the
  // sampler's staging buffer before scoring
  __shared__ float4 s_rows[(kBS / kWave) * kWave * kChunks];
  __shared__ uint16_t s_list[(kBS / kWave) * kRetryList];
  __shared__ BestT red[kBS / kWave];
  __shared__ int nred[kBS / kWave];
  static_assert(kTR * kWave * sizeof(float) <= kWave * kChunks * sizeof(float4), "staging alias");
  // XCD-aware work order: consecutive blocks land on consecutive XCDs (block
  // b on XCD b % 8), so block b takes work item (b % 8) * per + b / 8 of the
  // (job, tile) list -- each XCD sweeps one contiguous eighth of it and its
  // L2 holds the cell tables of ~1/8 of the labels instead of all of them
  int job, bx;
  {
    const int64_t W = (int64_t)n_tiles * n_jobs, per = (W + 7) / 8;
    const int64_t w = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (w >= W) return;  // padding block (the grid is 8 * per)
    job = (int)(w / n_tiles);
    bx = (int)(w - (int64_t)job * n_tiles);
  }
  const tpe_job J = jobs[job];
  tpe_best* P = partial + (int64_t)job * n_tiles + bx;
  const int64_t base0 = (int64_t)bx * kTiles * kTile;
  if (base0 >= J.n_cand) {
    if (threadIdx.x == 0) *P = empty_best();
    return;
  }
  const tpe_seg SB = segs[J.below], SA = segs[J.above];
  const tpe_table Tb = tables[job];
  const bool lgmm = J.family == TPE_LGMM1;
  const bool lo_on = J.flags & TPE_F_LOW, hi_on = J.flags & TPE_F_HIGH;
  const bool log_in = INJ && lgmm, exp_out = !INJ && lgmm;
  const float g0 = (float)Tb.origin, inv_w = Tb.inv_w, inv_h = Tb.inv_h;
  const int nb = Tb.nb;
  // the job's cell table: a uniform base + 32-bit byte offsets (saddr loads)
  const char* cbase = reinterpret_cast<const char*>(cells) + J.tbl_off * kSlotB;
  const float* mpairs = reinterpret_cast<const float*>(cbase) + J.tbl_cap * kCellF;
  const float h32 = (float)Tb.h;
  const int lane = lane_id(), gi = lane & (kChunks - 1), gbase = lane & ~(kChunks - 1);
  // wave-uniform (scalar) base of the wave's LDS region: the DMA destinations need no
  // per-instruction readfirstlane
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  float4* rows = s_rows + wave * (kWave * kChunks);
  const bool outs = out_bl || out_al || out_x;
  Mix M{};
#ifndef TPE_DIAG_SKIP_SAMPLE
  if (!INJ) M = stage_mix(SB, wcdf, mu, sigma, s_mix);  // once per block
#endif
  BestT run{0.0, -1, 0.0};
  int n_exact = 0;
  // the block's tiles in index order; a thread owns kTR consecutive candidates
  // of each (pairs share a Philox call)
  for (int tile = 0; tile < kTiles; ++tile) {
    const int64_t base = base0 + tile * kTile;
    if (base >= J.n_cand) break;
    if (tile > 0) __syncthreads();  // the previous tile's slabs / stash are done
    const int64_t t0 = base + (int64_t)threadIdx.x * kTR;
    // x[r]: the candidate in the scoring coordinate y for sampled jobs (log x for
    // LGMM1; the value exp(y) is formed only for outputs and the winner), the
    // given value for injected ones
    float x[kTR];
    if (INJ) {
#pragma unroll
      for (int r = 0; r < kTR; ++r) x[r] = t0 + r < J.n_cand ? (float)cand[J.cand_off + t0 + r] : 1.0f;
    } else {
#ifdef TPE_DIAG_SKIP_SAMPLE  // diagnostic builds only (tools/diag_variants.sh)
      const float w = 2.0f * (float)Tb.h * (float)Tb.nb;
#pragma unroll
      for (int r = 0; r < kTR; ++r)
        x[r] = (float)Tb.origin + w * __builtin_amdgcn_fractf((float)(t0 + r) * 0.6180339887f);
#else
      const int nv = (int)max((int64_t)0, min((int64_t)kTR, J.n_cand - t0));
      draw32_pairs<kTR>(M, J.key, J.cand_base + t0, nv, lo_on, hi_on, (float)J.low,
                        (float)J.high, false, reinterpret_cast<float*>(rows), s_list + (threadIdx.x / kWave) * kRetryList, x);
#endif
    }
    // per-thread argmax in fp32 over the thread's candidates r = 0..kTR-1
    // (np.argmax rules: larger score, NaN wins, ties -> smaller r)
    float bs = -INFINITY, by = 0.0f;
    int br = -1;
    uint32_t exact_mask = 0;
    auto outputs = [&](float lb, float la, float y, int r) {
      double bl = lb, al = la;
      if (lgmm) {  // lognormal_lpdf's -log(x) (tpe.py:214-216): in both, not in the score
        bl -= (double)y;
        al -= (double)y;
      }
      const int64_t o = J.out_off + t0 + r;
      if (out_bl) out_bl[o] = bl;
      if (out_al) out_al[o] = al;
      if (out_x) out_x[o] = exp_out ? exp((double)y) : (double)y;
    };
    const int nvalid = (int)max((int64_t)0, min((int64_t)kTR, J.n_cand - t0));
    // cell of every candidate of the thread (byte offset in the job's table)
    float yv[kTR];
    uint32_t co[kTR];
#pragma unroll
    for (int r = 0; r < kTR; ++r) {
      yv[r] = log_in ? __logf(x[r]) : x[r];
      const float t = (yv[r] - g0) * inv_w;
      int c = (t >= 0.0f) ? (int)t : 0;  // NaN -> 0
      co[r] = (uint32_t)min(c, nb - 1) * (kCellF * 4);
    }
    // Cooperative gather by LDS-DMA: lane gi of each 4-lane group fetches one
    // 16-B chunk of every group member's 64-B cell (global_load_lds_dwordx4),
    // so a wave-instruction touches 16 cells instead of 64 and the data lands
    // in LDS without passing through VGPRs.  Slab j holds member j's cells:
    // lane (g, gi) brings chunk gi^j, so lane (g, j) reads its chunk k from
    // slab j, slot 4g + (k^j) -- conflict-free ds_read_b128.  Candidate r+1's
    // DMA is issued as soon as candidate r's chunks are in registers, and runs
    // under r's polynomial work.
    typedef __attribute__((address_space(3))) void* lds_vp;
    typedef const __attribute__((address_space(1))) void* glb_vp;
    auto fetch = [&](int r) __attribute__((always_inline)) {
      auto one = [&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        // member j's cell offset: a quad-perm broadcast inside the 4-lane group
        const uint32_t cj = (uint32_t)__builtin_amdgcn_mov_dpp(
            (int)co[r], j | (j << 2) | (j << 4) | (j << 6), 0xF, 0xF, true);
        __builtin_amdgcn_global_load_lds((glb_vp)(cbase + (cj + ((gi ^ j) * 16))),
                                         (lds_vp)(rows + j * kWave), 16, 0, 0);
      };
      static_for<0, kChunks>(one);
    };
    const f4* slab = reinterpret_cast<const f4*>(rows) + gi * kWave;
    auto score = [&](auto rc) __attribute__((always_inline)) {
      constexpr int r = decltype(rc)::value;
      const float y = yv[r];
      // candidate r's DMA has landed (the compiler does not order LDS-DMA
      // writes before later ds_reads by itself)
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      static_assert(kChunks == 4, "the reads below take chunks 0..3");
      const f4 q0 = slab[gbase | gi], q1 = slab[gbase | (1 ^ gi)], q2 = slab[gbase | (2 ^ gi)],
               q3 = slab[gbase | (3 ^ gi)];
      // the reads must land before the next candidate's DMA overwrites the slabs
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      if constexpr (r + 1 < kTR) fetch(r + 1);
      const int cell = (int)(co[r] / (kCellF * 4));
      const float u = (y - cell_centre(g0, h32, cell)) * inv_h;
      float pb, pa;
      horner9x2(q0, q1, q2, q3, u, pb, pa);
      const float dlog = (__builtin_amdgcn_logf(pb) - __builtin_amdgcn_logf(pa)) * kLn2T;
      const bool valid = r < nvalid;
      // q3.w: m_below - m_above, NaN for a cell that failed the bound
      const bool ok = (q3.w == q3.w) && (fabsf(u) <= kULim) && (pb > 0.0f) && (pa > 0.0f);
      exact_mask |= (valid && !ok) ? (1u << r) : 0u;
      if (valid && ok) {
        if (outs)
          outputs(mpairs[2 * cell] + __builtin_amdgcn_logf(pb) * kLn2T,
                  mpairs[2 * cell + 1] + __builtin_amdgcn_logf(pa) * kLn2T, y, r);
        // table scores are finite: strict > keeps the first of equal scores
        const float sc = q3.w + dlog;
        const bool take = sc > bs;
        bs = take ? sc : bs;
        by = take ? (INJ ? x[r] : y) : by;
        br = take ? r : br;
      }
    };
#ifdef TPE_DIAG_SKIP_SCORE  // diagnostic builds only: the sampler alone
#pragma unroll
    for (int r = 0; r < kTR; ++r)
      if (t0 + r < J.n_cand && yv[r] > bs) {
        bs = yv[r];
        by = yv[r];
        br = r;
      }
#else
    fetch(0);
    static_for<0, kTR>(score);
#endif
    // exact fp32 log-sum-exp for the (rare) candidates the table does not cover;
    // their values wait in the lane's own LDS row
    if (__any(exact_mask != 0)) {
      float* stash = reinterpret_cast<float*>(rows + lane * (kTR / 4));
#pragma unroll
      for (int r = 0; r < kTR; ++r)
        if (exact_mask & (1u << r)) stash[r] = x[r];
      __builtin_amdgcn_wave_barrier();
      while (exact_mask) {
        const int r = __builtin_ctz(exact_mask);
        exact_mask &= exact_mask - 1;
        const float xv = stash[r];
        const float y = log_in ? __logf(xv) : xv;
        const float lb = lse_exact32(coef32 + SB.comp_off, SB, y);
        const float la = lse_exact32(coef32 + SA.comp_off, SA, y);
        if (outs) outputs(lb, la, y, r);
        const float sc = lb - la;
        const bool na = sc != sc, nb_ = bs != bs;
        const bool take =
            (br < 0) || (na ? (!nb_ || r < br) : (!nb_ && (sc > bs || (sc == bs && r < br))));
        if (take) {
          bs = sc;
          br = r;
          by = INJ ? xv : y;
        }
        ++n_exact;
      }
    }
    // the winner's value (by: the given value, or y of a sampled candidate --
    // exp(y) in fp64 for LGMM1, the value every fp32 scorer gives)
    const double bx = exp_out ? exp((double)by) : (double)by;
    if (br >= 0) best_update(run, (double)bs, J.cand_base + t0 + br, bx);
  }  // tiles
  const BestT best = block_best<kBS>(run, red);
  if (stats) {
    const int ne = block_sum<kBS, int>(n_exact, nred);
    if (threadIdx.x == 0 && ne) atomicAdd(stats, (unsigned long long)ne);
  }
  if (threadIdx.x == 0) *P = tpe_best{best.score, best.index, best.value, 0};
}

// fp32 score error bound of the fast path.  A candidate
// scored by its cell's cubic has
//     |s32 - s64| <= eps_cubic + 2.0001 eps_mix + 2^-22 |s32|
// (tpe_table: eps_cubic bounds the cubic against the stored polynomials, its
// fp32 evaluation beyond the |s| part, u's rounding and the fp32 offset;
// eps_mix the stored polynomial against its mixture, whose log then moves by
// at most eps_mix / (1 - eps_mix)).  A candidate of the two-polynomial cell
// carries its own bound (eps_2poly); one of the exact fp32 log-sum-exp
// fallback is always re-scored in fp64 (its hi is +inf).
constexpr float kEpsRel = 0x1.0p-22f;  // >= gamma_3 of the cubic's three fp32 FMAs

// outward rounding of a round-to-nearest fp32 result x (|exact - x| <= ulp/2
// <= 2^-24 |x|): up(x) >= exact >= dn(x) (the fma adds at least one ulp; the
// 1e-30 covers x = 0)
__device__ __forceinline__ float up(float x) { return fmaf(fabsf(x), 0x1.0p-23f, x) + 1e-30f; }
__device__ __forceinline__ float dn(float x) { return fmaf(-fabsf(x), 0x1.0p-23f, x) - 1e-30f; }
constexpr float kEtaLog2 = 0x1.0p-22f;  // v_log_f32 error, absolute or relative to |log2 p| (checked exhaustively)

// order-preserving float -> uint32 code (larger float, larger code; code 0 is
// below every float: "no value yet")
__device__ __forceinline__ uint32_t ord_enc(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord_dec(uint32_t e) {
  if (e == 0u) return -INFINITY;
  return __uint_as_float((e & 0x80000000u) ? (e & 0x7FFFFFFFu) : ~e);
}

// the value of an unquantized candidate drawn as y in fp32: y (GMM1) or
// exp(y) evaluated in fp64 (LGMM1)
__device__ __forceinline__ double cand_value(float y, bool lgmm) {
  return lgmm ? exp((double)y) : (double)y;
}
// the coordinate its exact fp64 score is taken at: the returned value (GMM1)
// or log of it (LGMM1: the reference scores log(x) of the value it returns,
// tpe.py:284-287 / lognormal_lpdf :208-217) -- within lgmm_du of y in cell units
__device__ __forceinline__ double score_coord(float y, bool lgmm) {
  return lgmm ? log(cand_value(y, true)) : (double)y;
}

// relative error bound of one mixture's two-polynomial value p (fp32 Horner
// from the fp16 tail, horner9x2) at u against the stored polynomial at the
// exact u: gamma_6 times the absolute polynomial, the fp16 tail's rounding
// (u to fp16, two fp16 FMAs, subnormal spacing), and u's fp32 rounding times
// a bound of |P'|; +inf when it is not below p
__device__ __forceinline__ float poly_rel_err(const float (&P)[kP], float u, float p, float du) {
  const float au = fabsf(u);
  float pabs = 0.0f, pd = 0.0f;
#pragma unroll
  for (int n = kP - 1; n >= 0; --n) {
    pabs = fmaf(pabs, au, fabsf(P[n]));
    if (n >= 1) pd = fmaf(pd, 1.0501f, (float)n * fabsf(P[n]));
  }
  const float dt = 0x1.0p-9f * 1.16f * (fabsf(P[6]) + fabsf(P[7]) + fabsf(P[8])) + 0x1.0p-23f;
  const float dp = (6.1f * 0x1.0p-24f * pabs + 1.35f * dt + du * pd) * 1.001f;
  return dp < p ? dp / (p - dp) : INFINITY;
}

// bound of |s - s64| for a two-polynomial score s = off + (lb2 - la2) ln2,
// beyond the polynomials' own 2.0001 eps_mix
__device__ __forceinline__ float eps_2poly(const f4 q0, const f4 q1, const f4 q2, const f4 q3,
                                           float u, float pb, float pa, float lb2, float la2,
                                           float s, float du) {
  float Pb[kP], Pa[kP];
  const float c[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
#pragma unroll
  for (int n = 0; n < kP32; ++n) {
    Pb[n] = c[2 * n];
    Pa[n] = c[2 * n + 1];
  }
  const h2_t t6 = __builtin_bit_cast(h2_t, q3.x), t7 = __builtin_bit_cast(h2_t, q3.y),
             t8 = __builtin_bit_cast(h2_t, q3.z);
  Pb[6] = (float)t6.x; Pa[6] = (float)t6.y;
  Pb[7] = (float)t7.x; Pa[7] = (float)t7.y;
  Pb[8] = (float)t8.x; Pa[8] = (float)t8.y;
  const float rb = poly_rel_err(Pb, u, pb, du), ra = poly_rel_err(Pa, u, pa, du);
  const float off = fabsf(q3.w);
  return (0x1.0p-24f * off + rb + ra +
          kLn2T * kEtaLog2 * (fmaxf(1.0f, fabsf(lb2)) + fmaxf(1.0f, fabsf(la2))) +
          0x1.0p-21f * (fabsf(s) + off + kLn2T * (fabsf(lb2) + fabsf(la2)))) * 1.001f;
}

// Band tiles: every scorer block (tile of kTile candidates) writes a header
// {lo, hi_max, n} into band_ctl and its band entries into its own kTileSlots
// slots -- plain stores, no atomics (one returning atomic per block on a job
// word contended when a job's ~10^3 blocks ran together).  lo = the tile's
// best lower bound s - eps (a lower bound of G), hi_max = its largest upper
// bound (+inf with a NaN or log-sum-exp candidate), entries = its candidates
// with s + eps >= lo (a superset of the band's: G >= lo); a tile with more
// than kTileSlots such candidates writes n = kTileFull and no entries.
constexpr int kTileSlots = 256;  // (a plateau of near-equal scores puts ~60 of a tile's 4096
                                  // candidates in the band; 256 keeps such levels exact without
                                  // the whole-stream fp64 fallback)
constexpr uint32_t kTileFull = 0xFFFFFFFFu;
constexpr int kHdrWords = 4;  // per tile: lo, hi_max (float bits), n, unused

// Fast path for sampled candidates (the suggest path: no per-candidate
// log-densities asked for).  Same draws as k_score_table (draw32_pairs), same
// cell index; the score comes from the cell's 16-B cubic (k_table_score):
// one global_load_dwordx4 per candidate instead of a 64-B gather, and three
// FMAs instead of two degree-8 polynomials and two logs.  Loads run four
// candidates ahead.  Candidates on a flagged score cell (or off the grid)
// take the two-polynomial cell, then the exact log-sum-exp, after the loop.
// out_score / out_x / out_eps (nullable, tests): per-candidate fp32 score,
// value and the bound eps the band used (+inf: always re-scored).
template <bool HOOKS>  // HOOKS: the per-candidate test outputs (out_score / out_x / out_eps)
__global__ __launch_bounds__(kBS) __attribute__((amdgpu_waves_per_eu(TPE_SCORE_WPE))) void k_score_table_fast(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const double* __restrict__ mu, const double* __restrict__ sigma,
    const double* __restrict__ wcdf, const float4* __restrict__ coef32,
    const tpe_table* __restrict__ tables, const float* __restrict__ cells,
    tpe_band* __restrict__ band, uint32_t* __restrict__ band_ctl,
    double* __restrict__ out_score, double* __restrict__ out_x, double* __restrict__ out_eps,
    tpe_best* __restrict__ partial, unsigned long long* __restrict__ stats, int n_tiles,
    int n_jobs, int tile_cap) {
  __shared__ LeanMix s_lean;
  // retry staging, then each lane's scores (slot r of lane l at r * 64 + l)
  __shared__ float s_stage[(kBS / kWave) * kTRF * kWave];
  __shared__ uint16_t s_list[(kBS / kWave) * kRetryList];
  __shared__ uint64_t s_key[kBS / kWave];
  __shared__ float s_wy[kBS / kWave];
  __shared__ float s_lo[kBS / kWave], s_hi[kBS / kWave];
  __shared__ int s_cnt[kBS / kWave];
  __shared__ int s_n;
  int job, bx;
  {  // XCD-aware work order (see k_score_table)
    const int64_t W = (int64_t)n_tiles * n_jobs, per = (W + 7) / 8;
    const int64_t w = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (w >= W) return;
    job = (int)(w / n_tiles);
    bx = (int)(w - (int64_t)job * n_tiles);
  }
  const tpe_job J = jobs[job];
  tpe_best* P = partial + (int64_t)job * n_tiles + bx;
  uint32_t* hdr = band_ctl + ((int64_t)job * n_tiles + bx) * kHdrWords;
  const int64_t base = (int64_t)bx * kTileF;
  if (base >= J.n_cand) {
    if (threadIdx.x == 0) {
      *P = empty_best();
      hdr[0] = __float_as_uint(-INFINITY);
      hdr[1] = __float_as_uint(-INFINITY);
      hdr[2] = 0u;
    }
    return;
  }
  const tpe_seg SB = segs[J.below], SA = segs[J.above];
  const tpe_table Tb = tables[job];
  const bool lgmm = J.family == TPE_LGMM1;
  const bool lo_on = J.flags & TPE_F_LOW, hi_on = J.flags & TPE_F_HIGH;
  const float g0 = (float)Tb.origin, inv_w = Tb.inv_w, inv_h = Tb.inv_h, h32 = (float)Tb.h;
  const int nb = Tb.nb;
  const char* region = reinterpret_cast<const char*>(cells) + J.tbl_off * kSlotB;
  const float4* sc = score_cells_of(region, J.tbl_cap);
  const int lane = lane_id();
  float* stage = s_stage + (threadIdx.x / kWave) * (kTRF * kWave);
  // the below mixture: staged for the lean sampler (tpe.suggest: always --
  // at most 26 components) or read from global memory (draw32_pairs)
  const int nmix = SB.n_obs + 1;
  const bool lean = nmix <= kStage;  // block-uniform
  const Mix M{wcdf + SB.comp_off, mu + SB.comp_off, sigma + SB.comp_off, nullptr, nullptr,
              nullptr, nmix};
  const int64_t t0 = base + (int64_t)threadIdx.x * kTRF;
  const int nvalid = (int)max((int64_t)0, min((int64_t)kTRF, J.n_cand - t0));
  const float lo32 = (float)J.low, hi32 = (float)J.high;
  uint16_t* wlist = s_list + (threadIdx.x / kWave) * kRetryList;
  // the candidates, in the scoring coordinate y (log x for LGMM1), into the
  // wave's stage (slot r of lane l at r * 64 + l)
  if (lean) {
    stage_lean(SB, wcdf, mu, sigma, s_lean);
    if (lo_on || hi_on)
      lean_draw<kTRF, true>(s_lean, nmix, J.key, J.cand_base + t0, nvalid, lo_on, hi_on, lo32,
                           hi32, stage, wlist);
    else
      lean_draw<kTRF, false>(s_lean, nmix, J.key, J.cand_base + t0, nvalid, false, false, lo32,
                            hi32, stage, wlist);
  } else {
    // a below mixture past the LDS staging (explicit observation lists, never
    // tpe.suggest's): one candidate at a time, the same stream (draw32)
#pragma unroll 1
    for (int r = 0; r < kTRF; ++r)
      stage[r * kWave + lane] =
          r < nvalid ? draw32(M, J.key, J.cand_base + t0 + r, lo_on, hi_on, lo32, hi32) : 1.0f;
  }
  // candidate g again, exactly as drawn above (the tile winner's and the band
  // entries' values: x[] need not live through the tail)
  auto redraw = [&](int64_t g) __attribute__((always_inline)) -> float {
    return lean ? lean_draw1(s_lean, nmix, J.key, g, lo_on, hi_on, lo32, hi32)
                : draw32(M, J.key, g, lo_on, hi_on, lo32, hi32);
  };
  const float nbm1 = (float)(nb - 1);
  // the cell of y: trunc of (y - origin) / 2h clamped to [0, nb - 1] (NaN -> 0)
  auto cell_of = [&](float y) __attribute__((always_inline)) -> int {
    return (int)__builtin_amdgcn_fmed3f((y - g0) * inv_w, 0.0f, nbm1);
  };
  auto cubic_at = [&](int c) __attribute__((always_inline)) -> float4 {
    return *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(sc) +
                                            ((uint32_t)c << 4));
  };
  float bs = -INFINITY, by = 0.0f;
  int br = -1;
  uint32_t fb = 0;  // candidates the score cells do not cover
  // FULL: every slot of the thread valid (all but a job's last tile).  y is
  // read back from the stage four candidates ahead of its score, together
  // with its cell's cubic; the slot then takes the score (or, for a fallback
  // candidate, keeps y).  Branch-free: slots past the job's end are scored
  // like the rest and masked out of the argmax and the fallback mask.
  auto score_all = [&](auto full_tag) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(full_tag)::value;
    float yq[4];
    float4 q[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      yq[r] = stage[r * kWave + lane];
      q[r] = cubic_at(cell_of(yq[r]));
    }
#pragma unroll
    for (int r = 0; r < kTRF; ++r) {
      const float y = yq[r & 3];
      const int c = cell_of(y);
      const float4 k = q[r & 3];
      if (r + 4 < kTRF) {
        yq[r & 3] = stage[(r + 4) * kWave + lane];
        q[r & 3] = cubic_at(cell_of(yq[r & 3]));
      }
#ifdef TPE_DIAG_SKIP_SCORE  // diagnostic builds only: the sampler alone (the draw is its score)
      const float s = y + 0.0f * (float)c + 0.0f * k.x;
      const bool ok = true;
#else
      const float u = (y - cell_centre(g0, h32, c)) * inv_h;
      const float s = fmaf(fmaf(fmaf(k.w, u, k.z), u, k.y), u, k.x);
      const bool ok = (s == s) && (fabsf(u) <= kULim);
#endif
      fb |= ok ? 0u : (1u << r);
      // finite scores: strict > keeps the first of equal scores (np.argmax)
      const float sv = (ok && (FULL || r < nvalid)) ? s : -INFINITY;
      const bool take = sv > bs;
      br = take ? r : br;
      by = take ? y : by;
      bs = fmaxf(bs, sv);
      // kept for the band (a fallback candidate keeps its y for the fallback pass)
      stage[r * kWave + lane] = ok ? s : y;
      if (HOOKS && out_score && ok && r < nvalid) out_score[J.out_off + t0 + r] = (double)s;
      if (HOOKS && out_x && r < nvalid) out_x[J.out_off + t0 + r] = cand_value(y, lgmm);
    }
    if (!FULL) fb &= nvalid <= 0 ? 0u : (1u << nvalid) - 1u;
  };
  if (nvalid == kTRF)
    score_all(std::true_type{});
  else
    score_all(std::false_type{});
  // the lane's best cubic-scored candidate (its bounds are monotone in s)
  const float bs_cubic = bs;
  const float ea = (Tb.eps_cubic + 2.0001f * Tb.eps_mix) * 1.000001f;  // (covers its rounding)
  // eps(s) = ea + 2^-22 |s| of a cubic-scored candidate; bounds s -/+ eps are
  // rounded outwards (up / dn)
  auto eps_of = [&](float v) __attribute__((always_inline)) -> float {
    return fmaf(kEpsRel, fabsf(v), ea) * 1.000001f;
  };
  float lo_fb = -INFINITY, hi_fb = -INFINITY;  // the lane's fallback candidates' bounds
  int n_fb = 0;
  uint32_t lsem = 0;  // candidates scored by the exact fp32 log-sum-exp
  const uint32_t fbm = fb;
  if (__any(fb != 0)) {
    // fallback: the two-polynomial cell, else the exact fp32 log-sum-exp;
    // the lane's candidates wait in its own column of the wave's stage, and
    // their UPPER BOUNDS (two-polynomial) or scores (log-sum-exp) replace
    // them there
    // (the fallback candidates' y were staged by their own lanes above; the
    // log-sum-exp below reads other lanes' columns)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const f4* cell4 = reinterpret_cast<const f4*>(region);
    auto fold = [&](int r, float s, float y, float keep) __attribute__((always_inline)) {
      stage[r * kWave + lane] = keep;
      if (HOOKS && out_score) out_score[J.out_off + t0 + r] = (double)s;
      const bool na = s != s, nbn = bs != bs;
      const bool take =
          (br < 0) || (na ? (!nbn || r < br) : (!nbn && (s > bs || (s == bs && r < br))));
      if (take) {
        bs = s;
        br = r;
        by = y;
      }
      ++n_fb;
    };
    while (fb) {
      const int r = __builtin_ctz(fb);
      fb &= fb - 1;
      const float y = stage[r * kWave + lane];
      const int c = cell_of(y);
      const float u = (y - cell_centre(g0, h32, c)) * inv_h;
      const f4 q0 = cell4[4 * c], q1 = cell4[4 * c + 1], q2 = cell4[4 * c + 2],
               q3 = cell4[4 * c + 3];
      float pb, pa;
      horner9x2(q0, q1, q2, q3, u, pb, pa);
      bool done = false;
      if ((q3.w == q3.w) && (fabsf(u) <= kULim) && (pb > 0.0f) && (pa > 0.0f) &&
          isfinite(pb) && isfinite(pa)) {
        const float lb2 = __builtin_amdgcn_logf(pb), la2 = __builtin_amdgcn_logf(pa);
        const float s = q3.w + (lb2 - la2) * kLn2T;
        const float e2 = eps_2poly(q0, q1, q2, q3, u, pb, pa, lb2, la2, s,
                                   4.5f * 0x1.0p-24f + lgmm_du(J, Tb)) +
                         2.0001f * Tb.eps_mix;
        if (s == s && e2 < INFINITY) {
          const float hi = up(s + e2);
          fold(r, s, y, hi);
          lo_fb = fmaxf(lo_fb, dn(s - e2));
          hi_fb = fmaxf(hi_fb, hi);
          if (HOOKS && out_eps) out_eps[J.out_off + t0 + r] = (double)hi - (double)s;
          done = true;
        }
      }
      if (!done) lsem |= 1u << r;  // the exact log-sum-exp, below, the wave together
    }
    // the exact fp32 log-sum-exp over every component, one candidate at a
    // time with the whole wave (its y still waits in the stage); always in
    // the band (hi = +inf: its bound is not tracked)
    uint32_t ex = lsem;
    for (;;) {
      const uint64_t lanes = __ballot(ex != 0);
      if (!lanes) break;
      const int L = __builtin_ctzll(lanes);
      const int r = __shfl(ex ? __builtin_ctz(ex) : 0, L, kWave);
      const float y = stage[r * kWave + L];
      const float s = lse_wave32(coef32 + SB.comp_off, SB, y) -
                      lse_wave32(coef32 + SA.comp_off, SA, y);
      if (lane == L) {
        fold(r, s, y, INFINITY);
        hi_fb = INFINITY;
        if (HOOKS && out_eps) out_eps[J.out_off + t0 + r] = INFINITY;
        ex &= ex - 1;
      }
    }
  }
  // the lane's best lower bound and largest upper bound
  float lo_t = lo_fb, hi_t = hi_fb;
  if (bs_cubic > -INFINITY) {
    const float e = eps_of(bs_cubic);
    lo_t = fmaxf(lo_t, dn(bs_cubic - e));
    hi_t = fmaxf(hi_t, up(bs_cubic + e));
  }
  // one LDS round: the tile's fp32 winner, lo and hi_max (and the fallback
  // count).  np.argmax's order in integers: the wave's largest score order
  // code (NaN canonical: above every number; -0 as +0; 0: no candidate),
  // then the first lane holding it -- lanes are in index order and a lane's
  // own best is its first -- whose key (code, complement of the tile-local
  // index) and y go to LDS; thread 0 forms the block winner's value once.
  const int wid = threadIdx.x / kWave;
  {
    const float a = wave_max_f(lo_t), b = wave_max_f(hi_t);
    uint32_t code = 0u;
    if (br >= 0) code = ord_enc((bs != bs) ? __uint_as_float(0x7FC00000u) : bs + 0.0f);
    uint32_t wc = code;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) wc = max(wc, (uint32_t)__shfl_xor((int)wc, o, kWave));
    const uint64_t own = __ballot(code == wc && wc != 0u);
    if (own != 0ull && lane == (int)__builtin_ctzll(own)) {
      s_key[wid] = ((uint64_t)wc << 32) | (uint64_t)(~(uint32_t)(threadIdx.x * kTRF + br));
      s_wy[wid] = by;
    } else if (own == 0ull && lane == 0) {
      s_key[wid] = 0ull;
    }
    int nf = n_fb;
    if (stats) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) nf += __shfl_xor(nf, o, kWave);
    }
    if (lane == 0) {
      s_lo[wid] = a;
      s_hi[wid] = b;
      s_cnt[wid] = nf;
    }
    if (threadIdx.x == 0) s_n = 0;
  }
  __syncthreads();
  float lo_blk = s_lo[0], hi_blk = s_hi[0];
  if (threadIdx.x == 0) {
    uint64_t k = s_key[0];
    int kw = 0, ne = s_cnt[0];
#pragma unroll
    for (int w = 1; w < kBS / kWave; ++w) {
      if (s_key[w] > k) {
        k = s_key[w];
        kw = w;
      }
      ne += s_cnt[w];
    }
    *P = k == 0ull ? empty_best()
                   : tpe_best{(double)ord_dec((uint32_t)(k >> 32)),
                              J.cand_base + base + (int64_t)(~(uint32_t)k),
                              cand_value(s_wy[kw], lgmm), 0};
    if (stats && ne) atomicAdd(stats, (unsigned long long)ne);
  }
#pragma unroll
  for (int w = 1; w < kBS / kWave; ++w) {
    lo_blk = fmaxf(lo_blk, s_lo[w]);
    hi_blk = fmaxf(hi_blk, s_hi[w]);
  }
  if (HOOKS && out_eps) {  // (test hook) the bound of every cubic-scored candidate
#pragma unroll
    for (int r = 0; r < kTRF; ++r)
      if (r < nvalid && !((fbm >> r) & 1u)) {
        const float v = stage[r * kWave + lane];
        out_eps[J.out_off + t0 + r] = (double)up(v + eps_of(v)) - (double)v;
      }
  }
#ifdef TPE_DIAG_NO_BAND  // diagnostic builds only: the fp32 winner alone
  return;
#endif
  // ---- the band tile: its candidates with hi >= lo_blk (NaN hi included);
  // only a lane whose largest upper bound reaches lo_blk holds any.  A
  // cubic-scored candidate's hi = up(s + eps(s)) is monotone in s, so it is
  // tested as s >= s_thr, s_thr = a value below every s with hi >= lo_blk
  // (s + eps(s) < lo_blk whenever s < s_thr: eps(s) <= ea' + 2^-22 |s|, the
  // 2^-20 |lo_blk| slack covers the outward roundings); its hi is formed
  // only for the entries written.  Fallback candidates carry their hi in the
  // stage (two-polynomial) or are always in (log-sum-exp: +inf).
  const float s_thr = lo_blk - fmaf(0x1.0p-20f, fabsf(lo_blk), ea * 1.0001f) - 1e-30f;
  uint32_t em = 0;
  if (!(hi_t < lo_blk)) {
#pragma unroll
    for (int r = 0; r < kTRF; ++r) {
      if (r < nvalid) {
        const float v = stage[r * kWave + lane];
        const bool in = ((fbm >> r) & 1u) ? (((lsem >> r) & 1u) || !(v < lo_blk)) : !(v < s_thr);
        if (in) em |= 1u << r;
      }
    }
  }
  const int cnt = __popc(em);
  const int pos0 = cnt ? atomicAdd(&s_n, cnt) : 0;  // (LDS; the entries' order is free)
  __syncthreads();
  const int total = s_n;
  if (total <= tile_cap && em) {
    tpe_band* B = band + ((int64_t)job * n_tiles + bx) * kTileSlots;
    int pos = pos0;
    // over the lane's entries only (usually one: its own best, whose value
    // it holds; any other entry is drawn again -- exactly as above -- so the
    // draws need not live through the tail)
    for (uint32_t m = em; m; m &= m - 1) {
      const int r = __builtin_ctz(m);
      const float yv = r == br ? by : redraw(J.cand_base + t0 + r);
      const float v = stage[r * kWave + lane];
      const float hi = ((lsem >> r) & 1u) ? INFINITY : ((fbm >> r) & 1u) ? v : up(v + eps_of(v));
      B[pos] = tpe_band{J.cand_base + t0 + r, yv, hi};
      ++pos;
    }
  }
  if (threadIdx.x == 0) {
    hdr[0] = __float_as_uint(lo_blk);
    hdr[1] = __float_as_uint(hi_blk == hi_blk ? hi_blk : INFINITY);
    hdr[2] = total <= tile_cap ? (uint32_t)total : kTileFull;
  }
}

// ---------------------------------------------------------------------------
// exact re-score of the band: one kernel (k_band), kBandBlocks blocks per job
// ---------------------------------------------------------------------------
// Every survivor's two log-densities are summed in fp64 over EVERY component
// (within e^-45 of the sum) -- GMM1_lpdf / LGMM1_lpdf's sums (tpe.py:117-180,
// 265-307; LGMM1's -log x cancels in the score) -- and its score is a
// function of its y alone, whatever the sharding of the candidates, within
// fp64 rounding of the reference's.  Two ways, per job:
//  * few survivors (<= kBandSurv; a peaked score): directly -- the components
//    split into kBandBlocks chunks, one block each, every survivor's partial
//    log-sum-exp per chunk (per thread an online sum in a fixed order, then a
//    fixed reduction tree), the chunks combined in order by the job's last
//    block;
//  * many (a flat score: thousands within the band, in a few cells): per
//    table cell holding survivors, both mixtures expanded around the cell
//    centre to degree kBandD (band_expand; components whose series would
//    converge slowly summed term by term), the cells dealt to the job's
//    blocks; survivors off the grid or past the kBandCells listed take the
//    direct sum (band_direct).
// Steps of every block:
//  1. G = max over the job's tiles of their lo; a tile whose entries did not
//     fit (kTileFull) with hi_max >= G makes the job "overflowed": block 0
//     gives the fp32 winner with n_scored = -1 (the caller re-scores the job
//     exactly).
//  2. The survivors -- entries with hi >= G of the tiles with hi_max >= G, in
//     flat entry order, the same in every block.  The exact winner i* is
//     among them: lo_k <= s64_k <= s64_i* <= hi_i* for every k, so hi_i* >=
//     G, and i* is in its tile's entries (hi_i* >= G >= that tile's lo);
//     every other candidate has s64 <= hi < G <= s64_i*.
//  3. The block's share of the sums (above).
//  4. The last block of the job to finish takes np.argmax over the
//     survivors (largest score, then smallest index, NaN first): best[j] =
//     {fp64 score, index, value, n_cand}, and re-arms the counter.
#ifndef TPE_BAND_BLOCKS  // diagnostic builds: k_band blocks per job
#define TPE_BAND_BLOCKS 16
#endif
constexpr int kBandBlocks = TPE_BAND_BLOCKS;  // blocks per job
constexpr int kBandSurv = 128;       // survivors a job may score directly
#ifndef TPE_BAND_DIRECT
#define TPE_BAND_DIRECT 128
#endif
constexpr int kBandDirect = TPE_BAND_DIRECT;  // ... and always does; more take the cell
                                              // expansions where the cells can hold them.
// (16 made drop-in bands of 30-130 survivors cheaper, but a rank's share of
// a label can then take the other path than the whole label and score the
// same candidate with other fp64 bits: the winners must not depend on the
// rank count -- test_gpu_shard.py -- so a job's path keeps to 128.)
#ifndef TPE_SURV_BATCH
#define TPE_SURV_BATCH 8
#endif
constexpr int kSurvBatch = TPE_SURV_BATCH;  // survivors summed together per pass
constexpr int kDirStage = 256;       // a block's component chunk staged in LDS when it fits
                                     // (a multiple of kBX: the per-thread order is unchanged;
                                     // small: k_band shares CUs with the side stream's launches)
#ifndef TPE_BAND_BX
#define TPE_BAND_BX 256
#endif
constexpr int kBX = TPE_BAND_BX;     // k_band block
constexpr int kBandTiles = 4096;     // tiles of a job the kernel's LDS prefix holds (2^24 candidates;
                                     // a larger job takes the exact fallback)
constexpr int kTilesPT = kBandTiles / kBX;  // tile headers per thread (prefix pass)
constexpr int kBandD = 20;           // expansion degree
constexpr double kBandTau = 45.0;    // exclusion margin (nats) on top of log(M)
constexpr double kBandRho = 1.5;     // admissible 1.05 |A| + 1.1025 |B|
constexpr int kBandCells = 64;       // cells expanded per job (sorted; the rest: direct)
constexpr int kBandBits = 32768;     // cell bitmap (LDS)

#ifndef TPE_BAND_DIR
#define TPE_BAND_DIR 16
#endif
constexpr int kChunkDir = TPE_BAND_DIR;  // slow components listed per (cell, chunk, mixture)
                                          // (a full list sends the cell's survivors to the
                                          // direct sum over every component)
struct BandMix {  // one mixture's expansion on one cell (or one chunk of its components)
  double P[kBandD + 1];
  double m;
  int n_dir;  // slow components listed; -1: more than fit (the job takes the exact fallback)
  int pad;
  int dir[kChunkDir];
};
#ifndef TPE_BAND_EPT
#define TPE_BAND_EPT 8
#endif
#ifndef TPE_BAND_U
#define TPE_BAND_U 2
#endif
constexpr int kEPT = TPE_BAND_EPT;   // band entries per thread per window (k_band)
constexpr int kExpU = TPE_BAND_U;    // band_expand: component loads in flight per thread
constexpr int kBandSurvMax = 65536;  // survivors a job may have (more: the exact fallback)
struct BandWork {  // per job (tpe_band_bytes)
  double part[kBandBlocks][kBandSurv][4];         // direct: per chunk and survivor {m, s} b, a
  BandMix cpart[kBandCells][kBandBlocks][2];      // cells: per cell, chunk and mixture
  float sy[kBandSurvMax];                         // the survivors (flat entry order): y ...
  int64_t sidx[kBandSurvMax];                     // ... and candidate index
  int cells[kBandCells];                          // the listed cells (ascending)
  int ns, ncell, over, direct;                    // survivors, cells, job overflowed, path
  long long tmark[16];                            // (TPE_BAND_TIMING diagnostic builds)
  BestT win[kBandBlocks];                         // k_band_final's per-block winners (k_band_pick)
  unsigned int done;                              // (unused)
  unsigned int pad[3];
};

// One step of the online log-sum-exp (s >= 1 at scale m) that needs no exp
// and changes nothing in the result's bits: a term below e^-37 of the
// scale adds < 2^-53 <= ulp(s)/2 to s (s is left as it is, as the rounded
// add would); a term above e^60 of it makes s * e^(m - v) < 2^-53 for any
// s < 1e10 (s = 1 + that rounds to 1).  NaN differences fall through.
__device__ __forceinline__ bool lse_skip(double& m, double& s, double v) {
  const double d = v - m;
  if (d < -37.0) return true;
  if (d > 60.0) {
    s = 1.0;
    m = v;
    return true;
  }
  return false;
}

// (m, s): e^m s; combined in a fixed order
__device__ __forceinline__ void lse_merge(double& m, double& s, double m2, double s2) {
  if (m2 == -INFINITY) return;
  if (m2 > m) {
    s = s * exp(m - m2) + s2;
    m = m2;
  } else {
    s += s2 * exp(m2 - m);
  }
}

// expansion of mixture S on the cell (y0, h) into E (LDS); all threads.
// One pass over the components, U loads in flight per thread; each thread
// keeps its own scale (raised when a term would exceed e^8 of it) and the
// threads are merged at the end (fixed order: deterministic).  A component's
// series exp(A u + B u^2) converges like rho^n / n!, rho = 1.05|A| +
// 1.1025|B|: with rho <= kBandRho the tail past degree 20 is < 1.1e-16 of
// its term (1.5^21 / 21!; a component the table admitted has rho <= 0.68:
// < 4e-23); components with a larger rho are summed term by term.
// Components whose largest term on the cell is below e^-45 / M of the prior
// component's smallest one there are left out (< e^-45 of the sum).
template <int BX, int U>
__device__ void band_expand(const tpe_seg& S, const double* __restrict__ coef64, double y0,
                            double h, BandMix& E, double* dred, int k_begin, int k_end) {
  const int nc = S.n_obs + 1;  // (the floor is the whole mixture's)
  const int64_t off = S.comp_off;
  const double4 cp = ld4(coef64, off + S.prior_pos);
  const double far = (fabs(y0 - cp.x) + 1.05 * h) * cp.y;
  const double T = cp.z - 0.5 * far * far - (log((double)nc) + kBandTau);
  if (threadIdx.x == 0) E.n_dir = 0;
  __syncthreads();
  double P[kBandD + 1];
#pragma unroll
  for (int n = 0; n <= kBandD; ++n) P[n] = 0.0;
  double ml = -INFINITY;
  for (int k0 = k_begin; k0 < k_end; k0 += U * BX) {
    double4 cs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u * BX + (int)threadIdx.x;
      cs[u] = k < k_end ? ld4(coef64, off + k) : make_double4(0.0, 0.0, -INFINITY, 0.0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double4 c = cs[u];
      const double zn = fmax(fabs(y0 - c.x) - 1.05 * h, 0.0) * c.y;
      if (!(c.z - 0.5 * zn * zn >= T)) continue;  // (padding: lc = -inf)
      const double hi2 = h * c.y * c.y;
      const double A = -(y0 - c.x) * hi2, B = -0.5 * h * hi2;
      if (1.05 * fabs(A) + 1.1025 * fabs(B) > kBandRho) {
        const int p = atomicAdd(&E.n_dir, 1);
        if (p < kChunkDir) E.dir[p] = k0 + u * BX + (int)threadIdx.x;
        continue;
      }
      const double z0 = (y0 - c.x) * c.y;
      const double v = c.z - 0.5 * z0 * z0;
      if (v > ml + 8.0) {  // new scale: rescale this thread's sums
        const double r = (ml == -INFINITY) ? 0.0 : exp(ml - v);
#pragma unroll
        for (int n = 0; n <= kBandD; ++n) P[n] *= r;
        ml = v;
      }
      double cm = 0.0, cc = exp(v - ml);  // e * c_n
      P[0] += cc;
#pragma unroll
      for (int n = 0; n < kBandD; ++n) {
        const double cn = fma(A, cc, 2.0 * B * cm) * (1.0 / (double)(n + 1));
        P[n + 1] += cn;
        cm = cc;
        cc = cn;
      }
    }
  }
  const double m = block_max<BX, double>(ml, dred);
  {
    const double r = (ml == -INFINITY) ? 0.0 : exp(ml - m);
#pragma unroll
    for (int n = 0; n <= kBandD; ++n) P[n] *= r;
  }
  // block sums of the kBandD + 1 terms (fixed order: deterministic)
  // (every term's butterfly stepped together: their LDS exchanges overlap)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    double t[kBandD + 1];
#pragma unroll
    for (int n = 0; n <= kBandD; ++n) t[n] = __shfl_xor(P[n], o, kWave);
#pragma unroll
    for (int n = 0; n <= kBandD; ++n) P[n] += t[n];
  }
  __syncthreads();  // (E.n_dir complete; dred free)
  const int wid = threadIdx.x / kWave;
  if (lane_id() == 0) {
#pragma unroll
    for (int n = 0; n <= kBandD; ++n) dred[wid * (kBandD + 1) + n] = P[n];
  }
  __syncthreads();
  if (threadIdx.x <= kBandD) {
    double t = 0.0;
    for (int w = 0; w < BX / kWave; ++w) t += dred[w * (kBandD + 1) + threadIdx.x];
    E.P[threadIdx.x] = t;
  }
  if (threadIdx.x == 0) {
    E.m = m;
    if (E.n_dir > kChunkDir) E.n_dir = -1;
  }
  __syncthreads();
}

// log of the mixture at y from its cell expansion (u = (y - y0) / h)
__device__ __forceinline__ double band_eval(const BandMix& E, const int* dir, int nd,
                                            const double* __restrict__ coef64, int64_t off,
                                            double u, double y) {
  double p = E.P[kBandD];
#pragma unroll
  for (int n = kBandD - 1; n >= 0; --n) p = fma(p, u, E.P[n]);
  for (int i = 0; i < nd; ++i) {
    const double4 c = ld4(coef64, off + dir[i]);
    const double t = (y - c.x) * c.y;
    p += exp(c.z - 0.5 * t * t - E.m);
  }
  return log(p) + E.m;
}

// log of the mixture at y summed directly over every component (online
// log-sum-exp, k_score64's arithmetic)
__device__ __forceinline__ double band_direct(const tpe_seg& S, const double* __restrict__ coef64,
                                              double y) {
  double mo = -INFINITY, so = 0.0;
  for (int k = 0; k < S.n_obs + 1; ++k) {
    const double4 c = ld4(coef64, S.comp_off + k);
    const double t = (y - c.x) * c.y;
    const double v = -0.5 * (t * t) + c.z;
    if (lse_skip(mo, so, v)) continue;
    const bool up = v > mo;
    const double e = exp(up ? mo - v : v - mo);
    so = up ? so * e + 1.0 : so + e;
    mo = up ? v : mo;
  }
  return log(so) + mo;
}

// the fp32 cell of a band candidate (as the scorer forms it); -2: off the
// grid (the direct sum)
__device__ __forceinline__ int band_cell(const tpe_table& Tb, float y) {
  const float g0 = (float)Tb.origin, h32 = (float)Tb.h;
  const float t = (y - g0) * Tb.inv_w;
  int c = (t >= 0.0f) ? (int)t : 0;
  c = min(c, Tb.nb - 1);
  const double u = ((double)y - (double)cell_centre(g0, h32, c)) / Tb.h;
  return (fabs(u) <= (double)kULim && y == y) ? c : -2;
}

__global__ __launch_bounds__(kBX) void k_band(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const double* __restrict__ coef64, const tpe_table* __restrict__ tables,
    const tpe_band* __restrict__ band, const uint32_t* __restrict__ band_ctl,
    const tpe_best* __restrict__ partial, int n_tiles, tpe_best* __restrict__ best,
    BandWork* __restrict__ work) {
  constexpr int kNW = kBX / kWave;
  __shared__ BestT red[kNW];
  __shared__ int s_end[kBandTiles];  // inclusive prefix of the tiles' counted entries
  __shared__ uint32_t s_bits[kBandBits / 32];
  __shared__ int s_cell[kBandCells];
  __shared__ float s_y[kBandSurv];
  __shared__ int64_t s_idx[kBandSurv];
  __shared__ int s_wt[kNW];
  __shared__ float s_g[kNW];
  __shared__ double s_red[kNW][kSurvBatch][2];
  __shared__ double dred[kNW * (kBandD + 1)];
  __shared__ BandMix s_eb;
  __shared__ int s_over, s_off;
  __shared__ int s_tile[kEPT * kBX];
  __shared__ int s_wm[kNW];
  __shared__ double4 s_cst[kDirStage];  // direct path: the block's chunk of one mixture
  const int j = blockIdx.y, kb = blockIdx.x;
  const int lane = lane_id(), wid = threadIdx.x / kWave;
  const tpe_job J = jobs[j];
  const uint32_t* H = band_ctl + (int64_t)j * n_tiles * kHdrWords;
  const tpe_band* Bj = band + (int64_t)j * n_tiles * kTileSlots;
  // exclusive block scan of one int per thread (wave scan + wave totals)
  auto block_excl = [&](int v, int& total) -> int {
    int incl = v;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int w = __shfl_up(incl, o, kWave);
      if (lane >= o) incl += w;
    }
    __syncthreads();
    if (lane == kWave - 1) s_wt[wid] = incl;
    __syncthreads();
    int pos = incl - v;
    total = 0;
#pragma unroll
    for (int w = 0; w < kNW; ++w) {
      pos += w < wid ? s_wt[w] : 0;
      total += s_wt[w];
    }
    return pos;
  };
#ifdef TPE_BAND_TIMING
#define TMARK(i) \
  if (blockIdx.x == 0 && threadIdx.x == 0) work[blockIdx.y].tmark[i] = wall_clock64();
#else
#define TMARK(i)
#endif
  TMARK(0)
  // ---- 1. G, overflow, the tiles' counts ----
  float g = -INFINITY;
  for (int t = threadIdx.x; t < n_tiles; t += kBX) g = fmaxf(g, __uint_as_float(H[t * kHdrWords]));
  g = wave_max_f(g);
  if (lane == 0) s_g[wid] = g;
  if (threadIdx.x == 0) s_over = n_tiles > kBandTiles;
  for (int w = threadIdx.x; w < kBandBits / 32; w += kBX) s_bits[w] = 0u;
  __syncthreads();
  float G = s_g[0];
#pragma unroll
  for (int w = 1; w < kNW; ++w) G = fmaxf(G, s_g[w]);
  // the relevant tiles' counts in LDS, then their inclusive prefix in place
  for (int t = threadIdx.x; t < kBandTiles; t += kBX) {
    int c = 0;
    if (t < n_tiles) {
      const float hm = __uint_as_float(H[t * kHdrWords + 1]);
      const uint32_t n = H[t * kHdrWords + 2];
      if (!(hm < G) && n != 0u) {
        if (n == kTileFull) s_over = 1;
        else c = (int)n;
      }
    }
    s_end[t] = c;
  }
  __syncthreads();
  int tot = 0;
  for (int i = 0; i < kTilesPT; ++i) tot += s_end[threadIdx.x * kTilesPT + i];
  int n_ent = 0;
  int run = block_excl(tot, n_ent);
  for (int i = 0; i < kTilesPT; ++i) {
    run += s_end[threadIdx.x * kTilesPT + i];
    s_end[threadIdx.x * kTilesPT + i] = run;
  }
  __syncthreads();
  if (s_over) {  // the fp32 winner; the caller re-scores the job exactly
    if (kb == 0) {
      BestT b32 = thread_best<kBX>(partial + (int64_t)j * n_tiles, n_tiles);
      b32 = block_best<kBX>(b32, red);
      if (threadIdx.x == 0) {
        best[j] = tpe_best{b32.score, b32.index, b32.value, -1};
        work[j].over = 1;  // (k_band_final / k_band_pick leave the job alone)
      }
    }
    return;
  }
  const int nt = min(n_tiles, kBandTiles);
  const tpe_table Tb = tables[j];
  // every entry once, kEPT consecutive ones per thread loaded together;
  // fn(entry, flat position) for the survivors, every thread taking part.
  // A window's flat positions find their tile without a search: each tile
  // marks its first position in the window with its id, and a running max
  // over the window (thread, then wave and block prefix) fills the rest.
  constexpr int kWin = kEPT * kBX;
  auto for_survivors = [&](auto&& fn) {
    for (int f0 = 0; f0 < n_ent; f0 += kWin) {
      for (int i = threadIdx.x; i < kWin; i += kBX) s_tile[i] = -1;
      __syncthreads();
      for (int t = threadIdx.x; t < nt; t += kBX) {
        const int st = t > 0 ? s_end[t - 1] : 0, en = s_end[t];
        if (en > st && en > f0 && st < f0 + kWin) s_tile[max(st, f0) - f0] = t;
      }
      __syncthreads();
      int tl[kEPT];
      int run = -1;
#pragma unroll
      for (int u = 0; u < kEPT; ++u) {
        run = max(run, s_tile[threadIdx.x * kEPT + u]);
        tl[u] = run;
      }
      int incl = run;  // inclusive max-scan over the wave, then the waves before
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const int w = __shfl_up(incl, o, kWave);
        if (lane >= o) incl = max(incl, w);
      }
      int carry = __shfl_up(incl, 1, kWave);
      if (lane == 0) carry = -1;
      if (lane == kWave - 1) s_wm[wid] = incl;
      __syncthreads();
#pragma unroll
      for (int w = 0; w < kNW; ++w) carry = w < wid ? max(carry, s_wm[w]) : carry;
      tpe_band E[kEPT];
#pragma unroll
      for (int u = 0; u < kEPT; ++u) {
        const int f = f0 + threadIdx.x * kEPT + u;
        E[u].hi = -INFINITY;
        if (f < n_ent) {
          const int t = max(tl[u], carry);
          const int e = f - (t > 0 ? s_end[t - 1] : 0);
          E[u] = Bj[(int64_t)t * kTileSlots + e];
        }
      }
      uint32_t keep = 0;
#pragma unroll
      for (int u = 0; u < kEPT; ++u)
        if (f0 + threadIdx.x * kEPT + u < n_ent && !(E[u].hi < G)) keep |= 1u << u;
      fn(E, keep);
    }
  };
  TMARK(1)
  // ---- 2. the survivors: their number and cells; block 0 lists them (flat
  // entry order) for k_band_final ----
  BandWork& W = work[j];
  int ns = 0;
  if (threadIdx.x == 0) s_off = 0;
  for_survivors([&](const tpe_band (&E)[kEPT], uint32_t keep) {
    int total = 0;
    int pos = ns + block_excl(__popc(keep), total);
#pragma unroll
    for (int u = 0; u < kEPT; ++u) {
      if ((keep >> u) & 1u) {
        if (pos < kBandSurv) {
          s_y[pos] = E[u].y;
          s_idx[pos] = E[u].index;
        }
        if (kb == 0 && pos < kBandSurvMax) {
          W.sy[pos] = E[u].y;
          W.sidx[pos] = E[u].index;
        }
        ++pos;
        const int c = band_cell(Tb, E[u].y);
        // (read first: a band's thousands of survivors share a few cells,
        // and same-word LDS atomics serialise)
        if (c >= 0 && c < kBandBits) {
          if (!(s_bits[c >> 5] & (1u << (c & 31)))) atomicOr(&s_bits[c >> 5], 1u << (c & 31));
        } else {
          s_off = 1;
        }
      }
    }
    ns += total;
  });
  __syncthreads();
  // the listed cells (ascending)
  constexpr int kPer = kBandBits / 32 / kBX;  // bitmap words per thread
  int ncell = 0;
  {
    int c = 0;
#pragma unroll
    for (int i = 0; i < kPer; ++i) c += __popc(s_bits[threadIdx.x * kPer + i]);
    int pos = block_excl(c, ncell);
    for (int i = 0; i < kPer && pos < kBandCells; ++i) {
      uint32_t b = s_bits[threadIdx.x * kPer + i];
      while (b && pos < kBandCells) {
        const int cell = (threadIdx.x * kPer + i) * 32 + __builtin_ctz(b);
        s_cell[pos] = cell;
        if (kb == 0) W.cells[pos] = cell;
        ++pos;
        b &= b - 1;
      }
    }
  }
  __syncthreads();
  TMARK(2)
  // the path: a few survivors are summed directly; more take the cell
  // expansions (their cost does not grow with the survivors: ~12 us against
  // ~5 us per 8 direct survivors), up to kBandSurv directly when the cells
  // cannot hold them (too many, or survivors off the grid); else the exact
  // fallback
  const bool cells_ok = ncell <= kBandCells && !s_off && ns <= kBandSurvMax;
  const bool direct = ns <= kBandDirect || (ns <= kBandSurv && !cells_ok);
  const bool over = !direct && !cells_ok;
  if (kb == 0 && threadIdx.x == 0) {
    W.ns = ns;
    W.ncell = min(ncell, kBandCells);
    W.over = over;
    W.direct = direct;
  }
  if (over) {
    // many survivors, off the grid or over too many cells: the exact fallback
    if (kb == 0) {
      BestT b32 = thread_best<kBX>(partial + (int64_t)j * n_tiles, n_tiles);
      b32 = block_best<kBX>(b32, red);
      if (threadIdx.x == 0) best[j] = tpe_best{b32.score, b32.index, b32.value, -1};
    }
    return;
  }
  const tpe_seg SB = segs[J.below], SA = segs[J.above];
  const bool lgmm = J.family == TPE_LGMM1;
  if (direct) {
    // ---- 3a. direct: this block's component chunk, for every survivor ----
    for (int mix = 0; mix < 2; ++mix) {
      const tpe_seg& S = mix ? SA : SB;
      const int nc = S.n_obs + 1;
      const int per = (nc + kBandBlocks - 1) / kBandBlocks;
      const int k0 = kb * per, k1 = min(nc, k0 + per);
      const double4* C = reinterpret_cast<const double4*>(coef64) + S.comp_off;
      // the chunk in LDS once (every batch of survivors re-reads it; each
      // thread's components and their order are the global loop's)
      const bool staged = k1 - k0 <= kDirStage;
      if (staged) {
        for (int k = k0 + (int)threadIdx.x; k < k1; k += kBX) s_cst[k - k0] = C[k];
        __syncthreads();
      }
      TMARK(8 + 3 * mix)
      for (int b0 = 0; b0 < ns; b0 += kSurvBatch) {
        const int nbat = min(kSurvBatch, ns - b0);  // (block-uniform: the batch's real survivors)
        double m[kSurvBatch], sm[kSurvBatch], y[kSurvBatch];
#pragma unroll
        for (int i = 0; i < kSurvBatch; ++i) {
          m[i] = -INFINITY;
          sm[i] = 0.0;
          y[i] = score_coord(s_y[min(b0 + i, ns - 1)], lgmm);
        }
        auto acc = [&](const double4 c) {
#pragma unroll
          for (int i = 0; i < kSurvBatch; ++i) {
            if (i >= nbat) continue;  // (a short batch: no work for its empty slots)
            const double t = (y[i] - c.x) * c.y;
            const double v = -0.5 * (t * t) + c.z;  // (log coefficient c.z: GMM1_lpdf's terms)
            if (lse_skip(m[i], sm[i], v)) continue;
            const bool upv = v > m[i];
            const double e = exp(upv ? m[i] - v : v - m[i]);
            sm[i] = upv ? sm[i] * e + 1.0 : sm[i] + e;
            m[i] = upv ? v : m[i];
          }
        };
        if (staged) {
          for (int k = k0 + (int)threadIdx.x; k < k1; k += kBX) acc(s_cst[k - k0]);
        } else {
          for (int k = k0 + (int)threadIdx.x; k < k1; k += kBX) acc(C[k]);
        }
        if (b0 == 0) { TMARK(9 + 3 * mix) }
        // fixed reduction tree: the wave's largest scale (DPP max), each lane's
        // sum brought to it once, a plain wave sum; then the block's waves in
        // order (lse_merge)
        // (wave_max_d / wave_sum_d's butterflies, the batch's survivors
        // stepped together so their LDS exchanges overlap: same bits)
        double mw[kSurvBatch], v[kSurvBatch];
#pragma unroll
        for (int i = 0; i < kSurvBatch; ++i) mw[i] = m[i];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
          double t[kSurvBatch];
#pragma unroll
          for (int i = 0; i < kSurvBatch; ++i) t[i] = __shfl_xor(mw[i], off, kWave);
#pragma unroll
          for (int i = 0; i < kSurvBatch; ++i) mw[i] = fmax(mw[i], t[i]);
        }
#pragma unroll
        for (int i = 0; i < kSurvBatch; ++i)
          v[i] = (m[i] == -INFINITY) ? 0.0 : sm[i] * exp(m[i] - mw[i]);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
          double t[kSurvBatch];
#pragma unroll
          for (int i = 0; i < kSurvBatch; ++i) t[i] = __shfl_xor(v[i], off, kWave);
#pragma unroll
          for (int i = 0; i < kSurvBatch; ++i) v[i] += t[i];
        }
        if (lane == 0) {
#pragma unroll
          for (int i = 0; i < kSurvBatch; ++i) {
            s_red[wid][i][0] = mw[i];
            s_red[wid][i][1] = v[i];
          }
        }
        __syncthreads();
        if (threadIdx.x < kSurvBatch && b0 + (int)threadIdx.x < ns) {
          const int i = threadIdx.x;
          double mm = s_red[0][i][0], ss = s_red[0][i][1];
          for (int w = 1; w < kNW; ++w) lse_merge(mm, ss, s_red[w][i][0], s_red[w][i][1]);
          W.part[kb][b0 + i][2 * mix] = mm;
          W.part[kb][b0 + i][2 * mix + 1] = ss;
        }
        __syncthreads();  // (s_red reused; s_cst free after the last batch)
        if (b0 == 0) { TMARK(10 + 3 * mix) }
      }
    }
  } else {
    // ---- 3b. cells: (cell, chunk) units, kBandBlocks of them when the cells
    // are fewer (each cell's components in nch chunks), else one cell each;
    // block kb takes units kb, kb + kBandBlocks, ... (k_band_final merges
    // a cell's chunks in order) ----
    const float g0 = (float)Tb.origin, h32 = (float)Tb.h;
    const int nch = max(1, kBandBlocks / max(ncell, 1));
    for (int unit = kb; unit < ncell * nch; unit += kBandBlocks) {
      const int k = unit / nch, ch = unit % nch;
      const double y0 = (double)cell_centre(g0, h32, s_cell[k]);
      for (int mix = 0; mix < 2; ++mix) {
        const tpe_seg& S = mix ? SA : SB;
        const int nc = S.n_obs + 1;
        const int per = (nc + nch - 1) / nch;
        const int k0 = min(nc, ch * per), k1 = min(nc, k0 + per);
        band_expand<kBX, kExpU>(S, coef64, y0, Tb.h, s_eb, dred, k0, k1);
        BandMix& Q = W.cpart[k][ch][mix];
        if (threadIdx.x <= kBandD) Q.P[threadIdx.x] = s_eb.P[threadIdx.x];
        if (threadIdx.x == 0) {
          Q.m = s_eb.m;
          Q.n_dir = s_eb.n_dir;
        }
        if (threadIdx.x < kChunkDir) Q.dir[threadIdx.x] = s_eb.dir[threadIdx.x];
        __syncthreads();  // (s_eb reused)
      }
    }
  }
  TMARK(3)
}

// The band's decision (after k_band), kFinBlocks blocks per job, each
// scoring a share of the job's survivors: direct -- a survivor's kBandBlocks
// chunk partial sums merged on 16 lanes (the largest scale by a max
// butterfly, the chunks' sums brought to it and added by a fixed butterfly);
// cells -- each listed cell's chunk expansions merged in chunk order (into
// LDS; every block the same) and evaluated at the block's survivors.  Each
// block leaves its np.argmax in W.win[kb]; k_band_pick folds them into
// best[j] = {fp64 score, index, value, n_cand}.  (One block per job scored a
// C3 band of ~4 000 survivors in ~16 us on one CU: fp64-rate bound; a
// last-block hand-off inside the kernel cost 10-17 us in round 3.)
#ifndef TPE_BAND_FX
#define TPE_BAND_FX 512
#endif
#ifndef TPE_BAND_FINB
#define TPE_BAND_FINB 8
#endif
constexpr int kFX = TPE_BAND_FX;         // k_band_final block
constexpr int kFinBlocks = TPE_BAND_FINB;  // k_band_final blocks per job (<= kBandBlocks: W.win)
constexpr int kFStage = 512;   // survivors staged in LDS per round (k_band_final, cells; small:
                               // the kernel shares CUs with the side stream's big launches)
static_assert(kFinBlocks <= kBandBlocks && kFinBlocks <= kWave, "W.win holds the blocks' winners");
__global__ __launch_bounds__(kFX) void k_band_final(const tpe_job* __restrict__ jobs,
                                                    const tpe_seg* __restrict__ segs,
                                                    const double* __restrict__ coef64,
                                                    const tpe_table* __restrict__ tables,
                                                    BandWork* __restrict__ work) {
  constexpr int kNW = kFX / kWave;
  __shared__ BestT red[kNW];
  __shared__ double s_P[kBandCells][2][kBandD + 2];  // merged expansions: P_0..P_20, m
  __shared__ double s_tmp[kBandCells][2][kBandD + 2];  // per (cell, chunk) unit: its P and m
  __shared__ int s_nd[kBandCells][2];
  __shared__ int s_ndu[kBandCells][2];             // per (cell, chunk) unit: slow components ...
  __shared__ int s_dir[kBandCells][2][kChunkDir];  // ... and their indices (units <= kBandCells)
  __shared__ int s_cells[kBandCells];
  __shared__ float s_sy[kFStage];
  __shared__ int64_t s_si[kFStage];
  const int j = blockIdx.y, kb = blockIdx.x;
  BandWork& W = work[j];
  if (kb == 0) { TMARK(4) }
  if (W.over) return;  // (k_band gave the fp32 winner with n_scored = -1)
  const tpe_job J = jobs[j];
  const int ns = W.ns, ncell = W.ncell;
  const int nch = max(1, kBandBlocks / max(ncell, 1));  // (k_band's chunks per cell)
  const bool lgmm = J.family == TPE_LGMM1;
  const tpe_seg SB = segs[J.below], SA = segs[J.above];
  const tpe_table Tb = tables[j];
  BestT bx{0.0, -1, 0.0};
  if (W.direct) {
    // one survivor per 16 lanes, lane c holding chunk c's partials
    constexpr int kSPB = kFX / kBandBlocks;  // survivors per block pass
    static_assert(kBandBlocks == 16, "16-lane groups");
    const int c = threadIdx.x % kBandBlocks;
    for (int i = kb * kSPB + (int)threadIdx.x / kBandBlocks; i < ns; i += kFinBlocks * kSPB) {
      const double4 q = *reinterpret_cast<const double4*>(W.part[c][i]);
      double mb = q.x, ma = q.z;
#pragma unroll
      for (int o = kBandBlocks / 2; o >= 1; o >>= 1) {
        const double tb = __shfl_xor(mb, o, kWave), ta = __shfl_xor(ma, o, kWave);
        mb = fmax(mb, tb);
        ma = fmax(ma, ta);
      }
      double sb = q.x == -INFINITY ? 0.0 : q.y * exp(q.x - mb);
      double sa = q.z == -INFINITY ? 0.0 : q.w * exp(q.z - ma);
#pragma unroll
      for (int o = kBandBlocks / 2; o >= 1; o >>= 1) {
        const double tb = __shfl_xor(sb, o, kWave), ta = __shfl_xor(sa, o, kWave);
        sb += tb;
        sa += ta;
      }
      if (c == 0) best_update(bx, (log(sb) + mb) - (log(sa) + ma), W.sidx[i],
                              cand_value(W.sy[i], lgmm));
    }
  } else {
    // merge: the chunks' expansions (P_0..P_20 and m per (cell, chunk,
    // mixture)) staged in LDS with all their global reads in flight at once,
    // then thread t takes (cell, mixture, term) items: every term summed over
    // the chunks in order at the cell's largest scale
    for (int t = threadIdx.x; t < ncell * nch * 2 * (kBandD + 2); t += kFX) {
      const int n = t % (kBandD + 2), r = t / (kBandD + 2), u = r >> 1, mix = r & 1;
      const BandMix& q = W.cpart[u / nch][u % nch][mix];
      s_tmp[u][mix][n] = n <= kBandD ? q.P[n] : q.m;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < ncell * 2 * (kBandD + 1); t += kFX) {
      const int k = t / (2 * (kBandD + 1)), r = t % (2 * (kBandD + 1));
      const int mix = r / (kBandD + 1), n = r % (kBandD + 1);
      double mm = -INFINITY;
      for (int c = 0; c < nch; ++c) mm = fmax(mm, s_tmp[k * nch + c][mix][kBandD + 1]);
      double acc = 0.0;
      for (int c = 0; c < nch; ++c) {
        const double qm = s_tmp[k * nch + c][mix][kBandD + 1];
        acc += qm == -INFINITY ? 0.0 : s_tmp[k * nch + c][mix][n] * exp(qm - mm);
      }
      s_P[k][mix][n] = acc;
      if (n == 0) s_P[k][mix][kBandD + 1] = mm;
    }
    // the slow-component lists (one thread per cell and mixture); -1: a
    // chunk's list overflowed (that cell's survivors take the direct sum)
    for (int t = threadIdx.x; t < ncell * nch * 2; t += kFX) {
      const int u = t >> 1, mix = t & 1;
      s_ndu[u][mix] = W.cpart[u / nch][u % nch][mix].n_dir;
    }
    for (int t = threadIdx.x; t < ncell * nch * 2 * kChunkDir; t += kFX) {
      const int d = t % kChunkDir, r = t / kChunkDir, u = r >> 1, mix = r & 1;
      s_dir[u][mix][d] = W.cpart[u / nch][u % nch][mix].dir[d];
    }
    __syncthreads();
    // each list in component order (k_band lists them in atomic order): the
    // slow components are then summed in a fixed order, run to run
    for (int t = threadIdx.x; t < ncell * nch * 2; t += kFX) {
      const int u = t >> 1, mix = t & 1, nd = s_ndu[u][mix];
      int* L = s_dir[u][mix];
      for (int a = 1; a < nd; ++a) {
        const int v = L[a];
        int b = a - 1;
        while (b >= 0 && L[b] > v) {
          L[b + 1] = L[b];
          --b;
        }
        L[b + 1] = v;
      }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < ncell * 2; t += kFX) {
      const int k = t >> 1, mix = t & 1;
      int nd = 0;
      for (int c = 0; c < nch; ++c) {
        const int q = s_ndu[k * nch + c][mix];
        nd = (nd < 0 || q < 0) ? -1 : nd + q;
      }
      s_nd[k][mix] = nd;
    }
    for (int t = threadIdx.x; t < ncell; t += kFX) s_cells[t] = W.cells[t];
    __syncthreads();
    if (kb == 0) { TMARK(5) }
    const float g0 = (float)Tb.origin, h32 = (float)Tb.h;
    // this block's survivors, in rounds of kFStage staged in LDS by
    // coalesced loads all in flight at once
    const int per = (ns + kFinBlocks - 1) / kFinBlocks;
    const int i0 = min(ns, kb * per), i1 = min(ns, i0 + per);
    for (int r0 = i0; r0 < i1; r0 += kFStage) {
      const int rn = min(kFStage, i1 - r0);
      __syncthreads();  // (the previous round's reads of s_sy / s_si done)
      for (int t = threadIdx.x; t < rn; t += kFX) {
        s_sy[t] = W.sy[r0 + t];
        s_si[t] = W.sidx[r0 + t];
      }
      __syncthreads();
      for (int t = threadIdx.x; t < rn; t += kFX) {
        const float yf = s_sy[t];
        const int c = band_cell(Tb, yf);
        int lo = 0, hi = ncell;  // its listed position (k_band listed every survivor's cell)
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (s_cells[mid] < c) lo = mid + 1; else hi = mid;
        }
        const int k = lo;
        const double y = score_coord(yf, lgmm);
        const double u = (y - (double)cell_centre(g0, h32, c)) / Tb.h;
        auto horner = [&](int mix) {
          double p = s_P[k][mix][kBandD];
#pragma unroll
          for (int n = kBandD - 1; n >= 0; --n) p = fma(p, u, s_P[k][mix][n]);
          return p;
        };
        // log of the mixture from its expansion value p, plus its slow
        // components term by term; the direct sum when a chunk's list overflowed
        auto finish = [&](int mix, const tpe_seg& S, double p) -> double {
          const int ndt = s_nd[k][mix];
          if (ndt < 0) return band_direct(S, coef64, y);
          const double m = s_P[k][mix][kBandD + 1];
          if (ndt > 0) {
            for (int cc = 0; cc < nch; ++cc) {
              const int un = k * nch + cc, nd = s_ndu[un][mix];
              for (int d = 0; d < nd; ++d) {
                const double4 cf = ld4(coef64, S.comp_off + s_dir[un][mix][d]);
                const double t = (y - cf.x) * cf.y;
                p += exp(cf.z - 0.5 * t * t - m);
              }
            }
          }
          return log(p) + m;
        };
        const double pb = horner(0), pa = horner(1);
        const double lb = finish(0, SB, pb);
        const double la = finish(1, SA, pa);
        best_update(bx, lb - la, s_si[t], cand_value(yf, lgmm));
      }
    }
  }
  if (kb == 0) { TMARK(6) }
  bx = block_best<kFX>(bx, red);
  if (threadIdx.x == 0) W.win[kb] = bx;
}

// The job's winner from its k_band_final blocks' (one wave per job).
__global__ __launch_bounds__(kWave) void k_band_pick(const tpe_job* __restrict__ jobs,
                                                     tpe_best* __restrict__ best,
                                                     BandWork* __restrict__ work) {
  const int j = blockIdx.x, lane = threadIdx.x;
  BandWork& W = work[j];
  if (W.over) return;
  BestT b{0.0, -1, 0.0};
  if (lane < kFinBlocks) b = W.win[lane];
  b = wave_best(b);
  if (lane == 0) {
    best[j] = tpe_best{b.score, b.index, b.value, jobs[j].n_cand};
#ifdef TPE_BAND_TIMING
    W.tmark[7] = wall_clock64();
#endif
  }
}

// ---------------------------------------------------------------------------
// exact fp64 scoring with component pruning (the parity mode at large M)
// ---------------------------------------------------------------------------
// The plan (k_table_plan1/2 with margin kTauExact) gives every mixture a
// floor T: a component whose term stays below T over the whole candidate
// range can add at most e^-40 of the prior component's term, itself a lower
// bound of the sum (exactly the table's exclusion rule with a wider margin),
// and reach windows over the sorted means.  A candidate sums, in fp64 with
// the online log-sum-exp of k_score64, the components of its reach window
// plus the wide list -- ~2 sigma_min / (range / M) components instead of M --
// and every component when it lies off the planned range.
//
// Coherence: a block sorts its kP64N candidates by coordinate in LDS (bitonic)
// and each wave scores runs of 64 consecutive ones, looping over the union of
// its lanes' windows with wave-uniform (scalar) component loads; a lane adds
// only the components of its own window, so a candidate's sum -- terms, order
// and offset -- is a function of its coordinate alone, whatever its
// neighbours.  The offset is the mixture's largest log-coefficient (every
// term <= 1, one exp per pair); a sum below 2^-900 (or a candidate off the
// range, or NaN) is redone with the online log-sum-exp over all components.
#ifndef TPE_R64P  // diagnostic builds: candidates per thread of k_score_pruned64
#define TPE_R64P 8   // (2 048 sorted together: a wave's 64 span half the range of 4: fp64 C3 -10 %)
#endif
constexpr int kR64P = TPE_R64P;          // candidates per thread
constexpr int kP64N = kBS * kR64P;       // candidates per block (sorted together)

// exp(v) for the pruned sum's terms (v <= 0 or NaN; 0 below -745.2): n =
// rint(32 v / ln2), r = v - n ln2/32 (Cody-Waite, the high part's 32 bits
// keep n ln2_hi exact), exp(r) by its degree-6 Taylor polynomial (|r| <=
// ln2/64: truncation < 2^-57), times 2^((n mod 32)/32) from a 32-entry table
// (correctly rounded) and 2^(n div 32) -- ~1 ulp, the library exp's accuracy,
// with 13 instead of 17 dependent fp64 steps and no overflow branch (round 6,
// with 2 048 candidates per block: fp64 C3 level 256 -> 217 ms, same-box A/B)
__constant__ double kExp2Tab[32] = {
    0x1.0000000000000p+0, 0x1.059b0d3158574p+0, 0x1.0b5586cf9890fp+0, 0x1.11301d0125b51p+0,
    0x1.172b83c7d517bp+0, 0x1.1d4873168b9aap+0, 0x1.2387a6e756238p+0, 0x1.29e9df51fdee1p+0,
    0x1.306fe0a31b715p+0, 0x1.371a7373aa9cbp+0, 0x1.3dea64c123422p+0, 0x1.44e086061892dp+0,
    0x1.4bfdad5362a27p+0, 0x1.5342b569d4f82p+0, 0x1.5ab07dd485429p+0, 0x1.6247eb03a5585p+0,
    0x1.6a09e667f3bcdp+0, 0x1.71f75e8ec5f74p+0, 0x1.7a11473eb0187p+0, 0x1.82589994cce13p+0,
    0x1.8ace5422aa0dbp+0, 0x1.93737b0cdc5e5p+0, 0x1.9c49182a3f090p+0, 0x1.a5503b23e255dp+0,
    0x1.ae89f995ad3adp+0, 0x1.b7f76f2fb5e47p+0, 0x1.c199bdd85529cp+0, 0x1.cb720dcef9069p+0,
    0x1.d5818dcfba487p+0, 0x1.dfc97337b9b5fp+0, 0x1.ea4afa2a490dap+0, 0x1.f50765b6e4540p+0};
__device__ __forceinline__ double exp_neg64(double v, const double* __restrict__ tab) {
  const double n = rint(v * 0x1.71547652b82fep+5);
  double r = fma(-n, 0x1.62e42fee00000p-6, v);
  r = fma(-n, 0x1.a39ef35793c76p-38, r);
  double p = fma(r, 1.0 / 720.0, 1.0 / 120.0);
  p = fma(r, p, 1.0 / 24.0);
  p = fma(r, p, 1.0 / 6.0);
  p = fma(r, p, 0.5);
  p = fma(r, p, 1.0);
  p = fma(r, p, 1.0);
  const int ni = (int)fmax(n, -40000.0);  // (NaN: the polynomial is NaN already)
  const double e = ldexp(tab[ni & 31] * p, ni >> 5);
  return v < -745.2 ? 0.0 : e;
}

__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = min(v, __shfl_xor(v, off, kWave));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = max(v, __shfl_xor(v, off, kWave));
  return __builtin_amdgcn_readfirstlane(v);
}

// largest log-coefficient of mixture S (every thread gets it)
__device__ __forceinline__ double lc_max(const tpe_seg& S, const double* __restrict__ coef64,
                                         double* red) {
  double m = -INFINITY;
  for (int k = threadIdx.x; k < S.n_obs + 1; k += kBS) m = fmax(m, coef64[4 * (S.comp_off + k) + 2]);
  return block_max<kBS, double>(m, red);
}

// log of mixture S at y for lane-active candidates (see above); call by the
// whole wave
__device__ __forceinline__ double lse64_pruned(const tpe_seg& S, const double* __restrict__ coef64,
                                               const double* __restrict__ rh,
                                               const double* __restrict__ rl,
                                               const int32_t* __restrict__ wide, int n_wide,
                                               double m, bool act, bool inr, double y,
                                               double4* stage, const double* etab) {
  const int nc = S.n_obs + 1;
  const int64_t off = S.comp_off;
  int k_lo = nc, k_hi = -1;
  if (act && inr) {
    k_lo = first_ge(rh + off, nc, y);
    k_hi = last_le(rl + off, nc, y);
  }
  const int ulo = wave_min_i(k_lo), uhi = wave_max_i(k_hi);
  double s = 0.0;
  // the union window in chunks of 64 components: one coalesced load per lane
  // into the wave's LDS slice (the wide flag folded in as w = 0), then every
  // lane reads the chunk's components in order by LDS broadcast -- the same
  // terms added in the same order as a loop over the window with a scalar
  // load per component (round 6: that loop waited on two dependent scalar
  // loads per component), so the sums are the same bits
  // (staged: x = mu, y = 1/sigma, z = log-coefficient - m, or -inf for a
  // component of the wide list -- its term is then exactly 0, and the wide
  // loop below adds it; the lane's own window as one unsigned compare)
  const int lane = lane_id();
  // (k_hi < k_lo, no window: a base no k reaches; uint32 arithmetic wraps)
  const uint32_t wlo = k_hi < k_lo ? 0x80000000u : (uint32_t)k_lo;
  const uint32_t wspan = k_hi < k_lo ? 0u : (uint32_t)(k_hi - k_lo);
  for (int kb = ulo; kb <= uhi; kb += kWave) {  // wave-uniform
    const int kk = kb + lane;
    double4 c = make_double4(0.0, 0.0, -INFINITY, 0.0);
    if (kk <= uhi) {
      c = ld4(coef64, off + kk);
      c.z = is_wide(S, kk, c.y) ? -INFINITY : c.z - m;
    }
    stage[lane] = c;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int n = min(kWave, uhi - kb + 1);
#pragma unroll 2
    for (int j = 0; j < n; ++j) {
      const double4 cj = stage[j];
      const double t = (y - cj.x) * cj.y;
      const double e = exp_neg64(fma(-0.5 * t, t, cj.z), etab);
      s += ((uint32_t)(kb + j) - wlo <= wspan) ? e : 0.0;
    }
    __builtin_amdgcn_wave_barrier();  // (the chunk read before the next one is staged)
  }
  if (__any(act && inr)) {
    for (int i = 0; i < n_wide; ++i) {
      const double4 c = ld4(coef64, off + wide[off + i]);
      const double t = (y - c.x) * c.y;
      s += exp(fma(-0.5 * t, t, c.z - m));
    }
  }
  double r = log(s) + m;
  const bool slow = act && !(inr && s >= 0x1p-900);
  if (__any(slow)) {
    // one exp per pair on every lane (as k_score64): same values as
    // s*exp(m-v)+1 (new max) / s+exp(v-m), NaN included
    double mo = -INFINITY, so = 0.0;
    for (int k = 0; k < nc; ++k) {
      const double4 c = ld4(coef64, off + k);
      const double t = (y - c.x) * c.y;
      const double v = -0.5 * (t * t) + c.z;
      const bool up = v > mo;
      const double e = exp(up ? mo - v : v - mo);
      so = up ? so * e + 1.0 : so + e;
      mo = up ? v : mo;
    }
    if (slow) r = log(so) + mo;
  }
  return r;
}

// ascending bitonic sort of kP64N (key, index) pairs in LDS, ties by index
__device__ __forceinline__ void sort_block(double* key, uint16_t* idx) {
  for (int k = 2; k <= kP64N; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int h = 0; h < kP64N / 2 / kBS; ++h) {
        const int p = h * kBS + threadIdx.x;
        const int i = ((p & ~(j - 1)) << 1) | (p & (j - 1)), l = i + j;
        const double a = key[i], b = key[l];
        const uint16_t ia = idx[i], ib = idx[l];
        const bool gt = a > b || (!(a < b) && ia > ib);
        if (gt == ((i & k) == 0)) {
          key[i] = b;
          key[l] = a;
          idx[i] = ib;
          idx[l] = ia;
        }
      }
      __syncthreads();
    }
  }
}

template <bool INJ>
__global__ __launch_bounds__(kBS) void k_score_pruned64(
    const tpe_job* __restrict__ jobs, const tpe_seg* __restrict__ segs,
    const double* __restrict__ mu, const double* __restrict__ sigma,
    const double* __restrict__ wcdf, const double* __restrict__ coef64,
    const double* __restrict__ reach_hi, const double* __restrict__ reach_lo,
    const int32_t* __restrict__ wide_idx, const tpe_table* __restrict__ tables,
    const double* __restrict__ cand, double* __restrict__ out_bl, double* __restrict__ out_al,
    double* __restrict__ out_x, tpe_best* __restrict__ partial) {
  __shared__ MixLds s_mix;
  __shared__ BestT red[kBS / kWave];
  __shared__ double dred[kBS / kWave];
  __shared__ double s_key[kP64N], s_x[kP64N];
  __shared__ uint16_t s_idx[kP64N];
  __shared__ double4 s_win[kBS / kWave][kWave];  // each wave's chunk of its union window
  __shared__ double s_etab[32];
  if (threadIdx.x < 32) s_etab[threadIdx.x] = kExp2Tab[threadIdx.x];  // (before the sort's barriers)
  const tpe_job J = jobs[blockIdx.y];
  tpe_best* P = partial + (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kP64N;
  if (base >= J.n_cand) {
    if (threadIdx.x == 0) *P = empty_best();
    return;
  }
  const int n_here = (int)min((int64_t)kP64N, J.n_cand - base);
  const tpe_seg SB = segs[J.below], SA = segs[J.above];
  const tpe_table Tb = tables[blockIdx.y];
  const bool lgmm = J.family == TPE_LGMM1;
  const bool lo_on = J.flags & TPE_F_LOW, hi_on = J.flags & TPE_F_HIGH;
  Mix M{};
  if (!INJ) M = stage_mix(SB, wcdf, mu, sigma, s_mix);
  for (int r = 0; r < kR64P; ++r) {
    const int i = r * kBS + threadIdx.x;
    double x = 0.0, y = INFINITY;
    if (i < n_here) {
      const int64_t li = base + i;
      if (INJ) {
        x = cand[J.cand_off + li];
        y = lgmm ? log(x) : x;
      } else if (J.flags & TPE_F_DRAW32) {
        // the table path's fp32 stream (the exact re-score of an overflowed band)
        const float y32 = draw32(M, J.key, J.cand_base + li, lo_on, hi_on, (float)J.low,
                                 (float)J.high);
        x = cand_value(y32, lgmm);
        y = score_coord(y32, lgmm);  // (LGMM1: log of the returned value, as INJ)
      } else {
        x = draw64(M, J.key, J.cand_base + li, lo_on, hi_on, J.low, J.high);
        if (lgmm) x = exp(x);
        y = lgmm ? log(x) : x;
      }
    }
    s_key[i] = y;
    s_x[i] = x;
    s_idx[i] = (uint16_t)i;
  }
  const double mb = lc_max(SB, coef64, dred), ma = lc_max(SA, coef64, dred);
  __syncthreads();
  sort_block(s_key, s_idx);
  BestT b{0.0, -1, 0.0};
  const int wid = threadIdx.x / kWave;
  for (int r = 0; r < kR64P; ++r) {
    const int p = (wid * kR64P + r) * kWave + lane_id();
    const int i = s_idx[p];
    const bool act = i < n_here;
    const double y = s_key[p], x = s_x[i];
    const bool inr = y >= Tb.lo && y <= Tb.hi;
    double bl = lse64_pruned(SB, coef64, reach_hi, reach_lo, wide_idx, Tb.n_wide_below, mb, act,
                             inr, y, s_win[wid], s_etab);
    double al = lse64_pruned(SA, coef64, reach_hi, reach_lo, wide_idx, Tb.n_wide_above, ma, act,
                             inr, y, s_win[wid], s_etab);
    if (!act) continue;
    if (lgmm) {  // lognormal_lpdf's -log(x) (tpe.py:214-216)
      bl -= y;
      al -= y;
    }
    const int64_t li = base + i;
    const int64_t o = J.out_off + li;
    if (out_bl) out_bl[o] = bl;
    if (out_al) out_al[o] = al;
    if (out_x) out_x[o] = x;
    best_update(b, bl - al, J.cand_base + li, x);
  }
  b = block_best<kBS>(b, red);
  if (threadIdx.x == 0) *P = tpe_best{b.score, b.index, b.value, 0};
}

__global__ __launch_bounds__(kBS) void k_reduce_t(const tpe_job* __restrict__ jobs,
                                                  const tpe_best* __restrict__ partial,
                                                  int64_t nper, tpe_best* __restrict__ best) {
  __shared__ BestT red[kBS / kWave];
  BestT b = thread_best<kBS>(partial + (int64_t)blockIdx.x * nper, nper);
  b = block_best<kBS>(b, red);
  if (threadIdx.x == 0)
    best[blockIdx.x] = tpe_best{b.score, b.index, b.value, jobs[blockIdx.x].n_cand};
}

// scorer blocks (tiles) per job of the fast path: the partial layout
int64_t tpe_table_fast_tiles(const tpe_job* hj, int n) {
  int64_t gx = 1;
  for (int i = 0; i < n; ++i) gx = std::max(gx, (hj[i].n_cand + kTileF - 1) / kTileF);
  return gx;
}

bool check_table_jobs(const char* fn, const tpe_job* hj, int n, bool* inj) {
  if (n < 0 || n > 65535 || (n > 0 && !hj)) {
    set_error("%s: bad job list (n_jobs=%d)", fn, n);
    return false;
  }
  for (int i = 0; i < n; ++i) {
    const tpe_job& j = hj[i];
    if (j.family == TPE_CAT || (j.flags & TPE_F_QUANT) || j.n_cand < 0) {
      set_error("%s: job %d is not an unquantized GMM1/LGMM1 job", fn, i);
      return false;
    }
    if (j.tbl_cap < 1 || j.tbl_off < 0) {
      set_error("%s: job %d has no cell table (tbl_cap=%lld)", fn, i, (long long)j.tbl_cap);
      return false;
    }
    const bool ji = (j.flags & TPE_F_INJECTED) != 0;
    if (i > 0 && ji != *inj) {
      set_error("%s: mixed injected / sampled jobs in one call", fn);
      return false;
    }
    *inj = ji;
  }
  return true;
}
}  // namespace
}  // namespace tpe

using namespace tpe;

extern "C" int64_t tpe_table_scratch_bytes(int n_jobs, int max_comp) {
  if (n_jobs < 0 || max_comp < 0) return -1;
  const int64_t tiles = std::max(1, (max_comp + kBS - 1) / kBS);
  return 8 * (int64_t)kPlanStride * tiles * 2 * std::max(n_jobs, 1);
}

extern "C" int tpe_table_build(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                               const tpe_seg* segs, const double* mu, const double* sigma,
                               const double* coef64, int max_comp, double* reach_hi,
                               double* reach_lo, int32_t* wide_idx, double* scratch,
                               tpe_table* tables, float* cells, uint64_t* stats, void* stream) {
  bool inj = false;
  if (!check_table_jobs("tpe_table_build", host_jobs, n_jobs, &inj)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  if (!jobs || !segs || !mu || !sigma || !coef64 || !reach_hi || !reach_lo || !wide_idx ||
      !scratch || !tables || !cells) {
    set_error("tpe_table_build: null pointer");
    return TPE_E_ARG;
  }
  if (max_comp < 1 || n_jobs > 32767) {
    set_error("tpe_table_build: max_comp=%d n_jobs=%d", max_comp, n_jobs);
    return TPE_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  const dim3 pg((max_comp + kBS - 1) / kBS, 2 * n_jobs);
  hipLaunchKernelGGL(k_table_plan1, pg, dim3(kBS), 0, st, jobs, segs, mu, sigma, coef64, reach_hi,
                     reach_lo, scratch, tables, kDrawZ, kTauExtra);
  hipLaunchKernelGGL(k_table_plan2, pg, dim3(kBS), 0, st, jobs, segs, mu, sigma, coef64, reach_hi,
                     reach_lo, wide_idx, scratch, tables);
  hipLaunchKernelGGL(k_table_build, dim3(kBuildBlocks, n_jobs), dim3(kBS), 0, st, jobs, segs,
                     sigma, coef64, reach_hi, reach_lo, wide_idx, tables, cells,
                     (unsigned long long*)stats);
  int64_t cap = 1;
  for (int i = 0; i < n_jobs; ++i) cap = std::max(cap, host_jobs[i].tbl_cap);
  const int64_t sblocks =
      std::min<int64_t>(kScoreBlocks, (cap + kScoreCellsPerBlock - 1) / kScoreCellsPerBlock);
  hipLaunchKernelGGL(k_table_score, dim3((unsigned)sblocks, n_jobs), dim3(kBS), 0, st, jobs, tables,
                     cells, (unsigned long long*)stats);
  return check_launch("tpe_table_build");
}

extern "C" int tpe_score_table(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                               const tpe_seg* segs, const double* mu, const double* sigma,
                               const double* wcdf, const float* coef32, const tpe_table* tables,
                               const float* cells, const double* cand, double* out_bl,
                               double* out_al, double* out_x, tpe_best* partial,
                               int64_t n_partial, tpe_best* best, uint64_t* stats,
                               void* stream) {
  bool inj = false;
  if (!check_table_jobs("tpe_score_table", host_jobs, n_jobs, &inj)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  if (!jobs || !segs || !mu || !sigma || !wcdf || !coef32 || !tables || !cells || !partial ||
      !best || (inj && !cand)) {
    set_error("tpe_score_table: null pointer");
    return TPE_E_ARG;
  }
  int64_t gx = 1;
  for (int i = 0; i < n_jobs; ++i)
    gx = std::max(gx, (host_jobs[i].n_cand + kTiles * kTile - 1) / (kTiles * kTile));
  if (gx * n_jobs > n_partial) {
    set_error("tpe_score_table: partial workspace %lld < %lld", (long long)n_partial,
              (long long)(gx * n_jobs));
    return TPE_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  // one block per (job, tile) work item, padded to a multiple of the 8 XCDs
  // (the kernel maps blocks to work items XCD by XCD)
  const int64_t per = (gx * n_jobs + 7) / 8;
  if (gx > INT32_MAX || 8 * per > INT32_MAX) {
    set_error("tpe_score_table: %lld work items", (long long)(gx * n_jobs));
    return TPE_E_UNSUPPORTED;
  }
  const dim3 grid((unsigned)(8 * per));
  const float4* c = reinterpret_cast<const float4*>(coef32);
  unsigned long long* s = (unsigned long long*)stats;
  if (inj)
    hipLaunchKernelGGL(k_score_table<true>, grid, dim3(kBS), 0, st, jobs, segs, mu, sigma, wcdf,
                       c, tables, cells, cand, out_bl, out_al, out_x, partial, s, (int)gx,
                       n_jobs);
  else
#ifndef TPE_DIAG_EXTRA_LDS  // diagnostic builds: dynamic LDS padding to lower occupancy
#define TPE_DIAG_EXTRA_LDS 0
#endif
    hipLaunchKernelGGL(k_score_table<false>, grid, dim3(kBS), TPE_DIAG_EXTRA_LDS, st, jobs, segs, mu, sigma, wcdf,
                       c, tables, cells, cand, out_bl, out_al, out_x, partial, s, (int)gx,
                       n_jobs);
  hipLaunchKernelGGL(k_reduce_t, dim3(n_jobs), dim3(kBS), 0, st, jobs, partial, gx, best);
  return check_launch("tpe_score_table");
}

extern "C" int64_t tpe_band_bytes(const tpe_job* host_jobs, int n_jobs, int64_t* ctl_bytes,
                                  int64_t* work_bytes) {
  if (n_jobs < 0 || (n_jobs > 0 && !host_jobs)) return -1;
  const int64_t tiles = n_jobs > 0 ? tpe_table_fast_tiles(host_jobs, n_jobs) * n_jobs : 1;
  if (ctl_bytes) *ctl_bytes = tiles * kHdrWords * (int64_t)sizeof(uint32_t);
  if (work_bytes) *work_bytes = (int64_t)sizeof(BandWork) * std::max(n_jobs, 1);
  return tiles * kTileSlots * (int64_t)sizeof(tpe_band);
}

extern "C" int tpe_score_table_fast(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                                    const tpe_seg* segs, const double* mu, const double* sigma,
                                    const double* wcdf, const float* coef32,
                                    const tpe_table* tables, const float* cells, tpe_band* band,
                                    uint32_t* band_ctl, double* out_score, double* out_x,
                                    double* out_eps, tpe_best* partial, int64_t n_partial,
                                    int tile_cap, uint64_t* stats, void* stream) {
  bool inj = false;
  if (!check_table_jobs("tpe_score_table_fast", host_jobs, n_jobs, &inj)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  if (inj) {
    set_error("tpe_score_table_fast: sampled jobs only (injected candidates: tpe_score_table)");
    return TPE_E_ARG;
  }
  if (!jobs || !segs || !mu || !sigma || !wcdf || !coef32 || !tables || !cells || !band ||
      !band_ctl || !partial) {
    set_error("tpe_score_table_fast: null pointer");
    return TPE_E_ARG;
  }
  if (tile_cap < 0 || tile_cap > kTileSlots) {
    set_error("tpe_score_table_fast: tile_cap=%d (0..%d)", tile_cap, kTileSlots);
    return TPE_E_ARG;
  }
  const int64_t gx = tpe_table_fast_tiles(host_jobs, n_jobs);
  if (gx * n_jobs > n_partial) {
    set_error("tpe_score_table_fast: partial workspace %lld < %lld", (long long)n_partial,
              (long long)(gx * n_jobs));
    return TPE_E_ARG;
  }
  const int64_t per = (gx * n_jobs + 7) / 8;
  if (gx > INT32_MAX || 8 * per > INT32_MAX) {
    set_error("tpe_score_table_fast: %lld work items", (long long)(gx * n_jobs));
    return TPE_E_UNSUPPORTED;
  }
  hipStream_t st = (hipStream_t)stream;
  if (out_score || out_x || out_eps)
    hipLaunchKernelGGL(k_score_table_fast<true>, dim3((unsigned)(8 * per)), dim3(kBS), 0, st, jobs,
                       segs, mu, sigma, wcdf, reinterpret_cast<const float4*>(coef32), tables,
                       cells, band, band_ctl, out_score, out_x, out_eps, partial,
                       (unsigned long long*)stats, (int)gx, n_jobs, tile_cap);
  else
    hipLaunchKernelGGL(k_score_table_fast<false>, dim3((unsigned)(8 * per)), dim3(kBS), 0, st, jobs,
                       segs, mu, sigma, wcdf, reinterpret_cast<const float4*>(coef32), tables,
                       cells, band, band_ctl, out_score, out_x, out_eps, partial,
                       (unsigned long long*)stats, (int)gx, n_jobs, tile_cap);
  return check_launch("tpe_score_table_fast");
}

extern "C" int tpe_band_rescore(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                                const tpe_seg* segs, const double* coef64,
                                const tpe_table* tables, const tpe_band* band,
                                const uint32_t* band_ctl, const tpe_best* partial,
                                int64_t n_partial, tpe_best* best, void* work, void* stream) {
  bool inj = false;
  if (!check_table_jobs("tpe_band_rescore", host_jobs, n_jobs, &inj)) return TPE_E_ARG;
  if (n_jobs == 0) return TPE_OK;
  if (inj) {
    set_error("tpe_band_rescore: sampled jobs only");
    return TPE_E_ARG;
  }
  if (!jobs || !segs || !coef64 || !tables || !band || !band_ctl || !partial || !best || !work) {
    set_error("tpe_band_rescore: null pointer");
    return TPE_E_ARG;
  }
  const int64_t gx = tpe_table_fast_tiles(host_jobs, n_jobs);
  if (gx * n_jobs > n_partial) {
    set_error("tpe_band_rescore: partial workspace %lld < %lld", (long long)n_partial,
              (long long)(gx * n_jobs));
    return TPE_E_ARG;
  }
  hipLaunchKernelGGL(k_band, dim3(kBandBlocks, n_jobs), dim3(kBX), 0, (hipStream_t)stream, jobs,
                     segs, coef64, tables, band, band_ctl, partial, (int)gx, best,
                     static_cast<BandWork*>(work));
  hipLaunchKernelGGL(k_band_final, dim3(kFinBlocks, n_jobs), dim3(kFX), 0, (hipStream_t)stream,
                     jobs, segs, coef64, tables, static_cast<BandWork*>(work));
  hipLaunchKernelGGL(k_band_pick, dim3(n_jobs), dim3(kWave), 0, (hipStream_t)stream, jobs, best,
                     static_cast<BandWork*>(work));
  return check_launch("tpe_band_rescore");
}

extern "C" int64_t tpe_pruned64_partials(const tpe_job* host_jobs, int n_jobs) {
  int64_t gx = 1;
  for (int i = 0; i < n_jobs; ++i)
    gx = std::max(gx, (host_jobs[i].n_cand + kBS * kR64P - 1) / (kBS * kR64P));
  return gx * n_jobs;
}

extern "C" int tpe_score_pruned64(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                                  const tpe_seg* segs, const double* mu, const double* sigma,
                                  const double* wcdf, const double* coef64, int max_comp,
                                  double* reach_hi, double* reach_lo, int32_t* wide_idx,
                                  double* scratch, tpe_table* tables, const double* cand,
                                  double* out_bl, double* out_al, double* out_x,
                                  tpe_best* partial, int64_t n_partial, tpe_best* best,
                                  void* stream) {
  if (n_jobs < 0 || n_jobs > 32767 || (n_jobs > 0 && !host_jobs)) {
    set_error("tpe_score_pruned64: bad job list (n_jobs=%d)", n_jobs);
    return TPE_E_ARG;
  }
  bool inj = false;
  for (int i = 0; i < n_jobs; ++i) {
    const tpe_job& j = host_jobs[i];
    if (j.family == TPE_CAT || (j.flags & TPE_F_QUANT) || j.n_cand < 0) {
      set_error("tpe_score_pruned64: job %d is not an unquantized GMM1/LGMM1 job", i);
      return TPE_E_ARG;
    }
    const bool ji = (j.flags & TPE_F_INJECTED) != 0;
    if (i > 0 && ji != inj) {
      set_error("tpe_score_pruned64: mixed injected / sampled jobs in one call");
      return TPE_E_ARG;
    }
    inj = ji;
  }
  if (n_jobs == 0) return TPE_OK;
  if (!jobs || !segs || !mu || !sigma || !wcdf || !coef64 || !reach_hi || !reach_lo ||
      !wide_idx || !scratch || !tables || !partial || !best || (inj && !cand) || max_comp < 1) {
    set_error("tpe_score_pruned64: null pointer or max_comp < 1");
    return TPE_E_ARG;
  }
  const int64_t gx = tpe_pruned64_partials(host_jobs, n_jobs) / n_jobs;
  if (gx * n_jobs > n_partial) {
    set_error("tpe_score_pruned64: partial workspace %lld < %lld", (long long)n_partial,
              (long long)(gx * n_jobs));
    return TPE_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  const dim3 pg((max_comp + kBS - 1) / kBS, 2 * n_jobs);
  hipLaunchKernelGGL(k_table_plan1, pg, dim3(kBS), 0, st, jobs, segs, mu, sigma, coef64, reach_hi,
                     reach_lo, scratch, tables, kDrawZ64, kTauExact);
  hipLaunchKernelGGL(k_table_plan2, pg, dim3(kBS), 0, st, jobs, segs, mu, sigma, coef64, reach_hi,
                     reach_lo, wide_idx, scratch, tables);
  const dim3 grid((unsigned)gx, (unsigned)n_jobs);
  if (inj)
    hipLaunchKernelGGL(k_score_pruned64<true>, grid, dim3(kBS), 0, st, jobs, segs, mu, sigma, wcdf,
                       coef64, reach_hi, reach_lo, wide_idx, tables, cand, out_bl, out_al, out_x,
                       partial);
  else
    hipLaunchKernelGGL(k_score_pruned64<false>, grid, dim3(kBS), 0, st, jobs, segs, mu, sigma,
                       wcdf, coef64, reach_hi, reach_lo, wide_idx, tables, cand, out_bl, out_al,
                       out_x, partial);
  hipLaunchKernelGGL(k_reduce_t, dim3(n_jobs), dim3(kBS), 0, st, jobs, partial, gx, best);
  return check_launch("tpe_score_pruned64");
}

extern "C" int64_t tpe_table_partials(const tpe_job* host_jobs, int n_jobs) {
  int64_t gx = 1;
  for (int i = 0; i < n_jobs; ++i)
    gx = std::max(gx, (host_jobs[i].n_cand + kTiles * kTile - 1) / (kTiles * kTile));
  return gx * n_jobs;
}
