// tpe_common.hpp -- device helpers shared by the TPE kernels (gfx950 / CDNA4).
//
// Wave64 everywhere: reductions use 64-lane butterflies, block sizes are
// multiples of 64.  Nothing here is CUDA-shaped; there is one code path.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/tpe_hip.h"

namespace tpe {

constexpr double kEps = 1e-12;  // hyperopt/tpe.py:32
constexpr int kWave = 64;
constexpr double kSqrt2 = 1.4142135623730951;
constexpr double kTwoPi = 6.283185307179586;  // 2 * np.pi, as the reference forms it
constexpr double kLog2e = 1.4426950408889634;
constexpr double kLn2 = 0.6931471805599453;

// ---------------------------------------------------------------------------
// host-side error reporting
// ---------------------------------------------------------------------------
void set_error(const char* fmt, ...);
int check_launch(const char* what);
void defer_launch_checks(bool on);

// ---------------------------------------------------------------------------
// Philox4x32-10 (counter-based; one call = 4 independent 32-bit words)
// ---------------------------------------------------------------------------
struct U4 {
  uint32_t x, y, z, w;
};

#ifndef TPE_PHILOX_ROUNDS  // diagnostic builds only (tools/diag_variants.sh): 10 in the product
#define TPE_PHILOX_ROUNDS 10
#endif
__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < TPE_PHILOX_ROUNDS; ++r) {
    // 64-bit products: one v_mad_u64_u32 per multiply gives both halves
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    // three-input XORs: one v_bitop3_b32 each (gfx950; 0x96 = a ^ b ^ c)
    c = U4{(uint32_t)__builtin_amdgcn_bitop3_b32(hi1, c.y, k0, 0x96), lo1,
           (uint32_t)__builtin_amdgcn_bitop3_b32(hi0, c.w, k1, 0x96), lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// draw `attempt` of candidate `idx` for a label keyed by `key`
__device__ __forceinline__ U4 draw_words(uint64_t key, int64_t idx, uint32_t attempt,
                                         uint32_t stream) {
  return philox(U4{(uint32_t)idx, (uint32_t)((uint64_t)idx >> 32), attempt, stream},
                (uint32_t)key, (uint32_t)(key >> 32));
}

// uniforms: [0,1) with 53 / 24 random bits
__device__ __forceinline__ double u01_f64(uint32_t a, uint32_t b) {
  const uint64_t m = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
  return (double)m * 0x1.0p-53;
}
__device__ __forceinline__ float u01_f32(uint32_t a) { return (float)(a >> 8) * 0x1.0p-24f; }

// standard normal by Box-Muller (one of the pair); |z| <= 8.6 (fp64), 5.8 (fp32)
__device__ __forceinline__ double normal_f64(uint32_t a, uint32_t b, uint32_t c) {
  const double u1 = 1.0 - u01_f64(a, b);  // (0, 1]
  const double u2 = (double)c * 0x1.0p-32;
  return sqrt(-2.0 * log(u1)) * cospi(2.0 * u2);
}
// both Box-Muller normals of one (a, b) pair
__device__ __forceinline__ void normal_pair_f32(uint32_t a, uint32_t b, float& z0, float& z1) {
  const float u1 = 1.0f - u01_f32(a);  // (0, 1]
  const float u2 = (float)(b >> 8) * 0x1.0p-24f;
  const float r = __builtin_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
  z0 = r * __builtin_amdgcn_cosf(u2);
  z1 = r * __builtin_amdgcn_sinf(u2);
}

// ---------------------------------------------------------------------------
// argmax with np.argmax semantics: larger score wins, ties -> smaller index,
// NaN counts as the maximum (first NaN wins).  index < 0 marks "empty".
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ bool better(double sa, int64_t ia, double sb, int64_t ib) {
  if (ib < 0) return ia >= 0;
  if (ia < 0) return false;
  const bool na = sa != sa, nb = sb != sb;
  if (na || nb) return (na && nb) ? ia < ib : na;
  if (sa != sb) return sa > sb;
  return ia < ib;
}

struct BestT {
  double score;
  int64_t index;
  double value;
};

__device__ __forceinline__ void best_update(BestT& b, double s, int64_t i, double v) {
  if (better(s, i, b.score, b.index)) {
    b.score = s;
    b.index = i;
    b.value = v;
  }
}

__device__ __forceinline__ BestT wave_best(BestT b) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    BestT o;
    o.score = __shfl_xor(b.score, off, kWave);
    o.index = __shfl_xor(b.index, off, kWave);
    o.value = __shfl_xor(b.value, off, kWave);
    if (better(o.score, o.index, b.score, b.index)) b = o;
  }
  return b;
}

// this thread's np.argmax over P[tid], P[tid + BS], ... (< nper), eight loads
// in flight at a time (a job's partials are thousands of 32-B records: one
// load per dependent step left the reduce latency-bound)
template <int BS>
__device__ __forceinline__ BestT thread_best(const tpe_best* __restrict__ P, int64_t nper) {
  BestT b{0.0, -1, 0.0};
  int64_t i = threadIdx.x;
  constexpr int kU = 8;
  for (; i + (kU - 1) * BS < nper; i += kU * BS) {
    tpe_best p[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) p[u] = P[i + u * BS];
#pragma unroll
    for (int u = 0; u < kU; ++u) best_update(b, p[u].score, p[u].index, p[u].value);
  }
  for (; i < nper; i += BS) {
    const tpe_best p = P[i];
    best_update(b, p.score, p.index, p.value);
  }
  return b;
}

// block-wide argmax; result valid in every thread. `sh` holds >= nwaves BestT.
template <int BS>
__device__ __forceinline__ BestT block_best(BestT b, BestT* sh) {
  b = wave_best(b);
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  __syncthreads();
  if (lane == 0) sh[wid] = b;
  __syncthreads();
  BestT r = sh[0];
#pragma unroll
  for (int k = 1; k < BS / kWave; ++k)
    if (better(sh[k].score, sh[k].index, r.score, r.index)) r = sh[k];
  return r;
}

template <int BS, typename T>
__device__ __forceinline__ T block_sum(T v, T* sh) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  T r = sh[0];
#pragma unroll
  for (int k = 1; k < BS / kWave; ++k) r += sh[k];
  return r;
}

template <int BS, typename T>
__device__ __forceinline__ T block_max(T v, T* sh) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, kWave));
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  T r = sh[0];
#pragma unroll
  for (int k = 1; k < BS / kWave; ++k) r = fmax(r, sh[k]);
  return r;
}

// ---------------------------------------------------------------------------
// numpy-exact arithmetic helpers (no FMA contraction where numpy has none)
// ---------------------------------------------------------------------------
// np.linspace(1/N, 1, N-LF) element i, then ones(LF): tpe.py:380-392
__device__ __forceinline__ double lf_weight(int64_t i, int64_t n, int32_t lf) {
  if (!(lf > 0 && lf < n)) return 1.0;
  const int64_t num = n - lf;
  if (i >= num) return 1.0;
  const double start = 1.0 / (double)n;
  if (num == 1) return start;
  if (i == num - 1) return 1.0;
  const double step = (1.0 - start) / (double)(num - 1);
  return __dadd_rn(__dmul_rn((double)i, step), start);
}

// normal_cdf: 0.5 * (1 + erf((x - mu) / max(sqrt(2) * sigma, EPS)))  tpe.py:109-114
__device__ __forceinline__ double normal_cdf(double x, double mu, double sigma) {
  const double bottom = fmax(__dmul_rn(kSqrt2, sigma), kEps);
  const double z = (x - mu) / bottom;
  return __dmul_rn(0.5, __dadd_rn(1.0, erf(z)));
}

// lognormal_cdf on a precomputed log(max(x, EPS)):  0.5 + 0.5 * erf(z)  tpe.py:186-205
__device__ __forceinline__ double lognormal_cdf_logx(double logx, double mu, double sigma) {
  const double bottom = fmax(__dmul_rn(kSqrt2, sigma), kEps);
  const double z = (logx - mu) / bottom;
  return __dadd_rn(0.5, __dmul_rn(0.5, erf(z)));
}

// total order of (value) used by the fit's sorts: ascending, -0.0 == +0.0, NaN
// last (np.sort / np.argsort put NaN last)
__device__ __forceinline__ uint64_t order_key(double v) {
  if (v != v) return ~0ull - 1;
  if (v == 0.0) v = 0.0;
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | (1ull << 63));
}

// the fit's observation transform (ap_*_sampler, tpe.py:506-572): log of
// np.maximum(obs, floor) for the log-domain priors (NaN stays NaN)
__device__ __forceinline__ double obs_transform(double v, int transform, double floor) {
  if (transform == TPE_OBS_LOG) {
    if (v < floor) v = floor;
    v = log(v);
  }
  return v;
}

// float -> ordered position inside a 64-lane wave's work split
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// the fit's bandwidth / coefficient launches (tpe_parzen.hip), shared by
// tpe_parzen_fit and tpe_fit_sorted
int64_t fit_part_doubles(int max_obs);
void fit_tail(tpe_seg* segs, int n_seg, int max_obs, double* part, double* w, const double* mu,
              double* sigma, double* wcdf, double* coef64, float* coef32, hipStream_t st);

}  // namespace tpe
