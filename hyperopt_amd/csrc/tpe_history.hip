// tpe_history.hip -- observation lists gathered from an HBM-resident history.
//
// The reference rebuilds every label's below/above observation lists from the
// Trials documents on every suggest (miscs_to_idxs_vals, base.py:200-214, and
// ap_split_trials, tpe.py:623-646: the lists keep tid order).  Here the history
// is a label-major matrix resident in HBM -- vals[col * ld + row] and an
// active flag per (label, row) -- appended to as trials complete.  A suggest
// step uploads only the per-row below flag (the n_below best losses) and this
// kernel compacts, for every (label, half) descriptor, the rows that are
// active for the label and on the requested side of the split, in row (tid)
// order, into the fp64 observation pool of the Parzen fit or the int64 pool
// of the categorical posterior.  A descriptor never writes more than its
// `count` elements; finding a different number sets bit 4 of *err.
#include "tpe_common.hpp"

namespace tpe {
namespace {
constexpr int kGBS = 1024;
constexpr int kGWaves = kGBS / kWave;
constexpr int kGT = 16;                 // 1024-row tiles per pass (16 384 rows)
constexpr int kGSlots = kGT * kGWaves;  // (tile, wave) counts scanned per pass

// Compacts one descriptor's rows (block-wide, in position order).  A pass
// covers kGT tiles: every thread first loads its kGT rows' flags and values
// (the global loads of the whole pass in flight at once -- the kernel is
// latency-bound, one block per descriptor), the waves' per-tile counts go to
// LDS, one block-wide exclusive scan over the (tile, wave) slots gives every
// wave its offsets, then the writes: three barriers per pass instead of three
// per tile.
__device__ __forceinline__ void gather_one(const double* __restrict__ V,
                                           const uint8_t* __restrict__ A,
                                           const int32_t* __restrict__ rows, int64_t n_rows,
                                           const uint8_t* __restrict__ is_below,
                                           const tpe_gather& G, double* __restrict__ out_f,
                                           int64_t* __restrict__ out_i, int32_t* __restrict__ err,
                                           int* wsum, int64_t& carry_s) {
  const uint8_t side = G.below ? 1 : 0;
  const int lane = lane_id(), wid = threadIdx.x / kWave;
  const uint64_t lt = (1ull << lane) - 1ull;
  if (threadIdx.x == 0) carry_s = 0;
  for (int64_t p0 = 0; p0 < n_rows; p0 += (int64_t)kGT * kGBS) {
    bool take[kGT];
    double v[kGT];
#pragma unroll
    for (int t = 0; t < kGT; ++t) {
      const int64_t i = p0 + (int64_t)t * kGBS + threadIdx.x;
      take[t] = false;
      v[t] = 0.0;
      if (i < n_rows) {
        const int64_t r = rows ? (int64_t)rows[i] : i;
        take[t] = A[r] && (is_below[i] == side);
        if (take[t]) v[t] = V[r];
      }
    }
    int before[kGT];
#pragma unroll
    for (int t = 0; t < kGT; ++t) {
      const uint64_t bal = __ballot(take[t]);
      before[t] = __popcll(bal & lt);
      if (lane == 0) wsum[t * kGWaves + wid] = __popcll(bal);
    }
    __syncthreads();
    // exclusive scan of the kGSlots counts (slot order = tile-major, then
    // wave = row order), one slot per thread
    int c = threadIdx.x < kGSlots ? wsum[threadIdx.x] : 0;
    int incl = c;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const int o = __shfl_up(incl, off, kWave);
      if (lane >= off) incl += o;
    }
    __syncthreads();
    if (threadIdx.x < kGSlots && lane == kWave - 1) wsum[kGSlots + wid] = incl;  // wave totals
    __syncthreads();
    int wave_base = 0;
    for (int q = 0; q < wid && q < kGSlots / kWave; ++q) wave_base += wsum[kGSlots + q];
    const int64_t carry = carry_s;
    if (threadIdx.x < kGSlots) wsum[threadIdx.x] = wave_base + incl - c;  // exclusive
    int total = 0;
    for (int q = 0; q < kGSlots / kWave; ++q) total += wsum[kGSlots + q];
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kGT; ++t) {
      const int64_t pos = carry + wsum[t * kGWaves + wid] + before[t];
      if (take[t] && pos < G.count) {
        if (G.to_int)
          out_i[G.dst_off + pos] = (int64_t)v[t] - G.offset;
        else
          out_f[G.dst_off + pos] = v[t];
      }
    }
    __syncthreads();  // everyone has read carry_s / wsum
    if (threadIdx.x == 0) carry_s = carry + total;
    __syncthreads();
  }
  if (threadIdx.x == 0 && carry_s != G.count && err) atomicOr(err, 4);
}

__global__ __launch_bounds__(kGBS) void k_gather_obs(const double* __restrict__ vals,
                                                     const uint8_t* __restrict__ active,
                                                     int64_t ld, const int32_t* __restrict__ rows,
                                                     int64_t n_rows,
                                                     const uint8_t* __restrict__ is_below,
                                                     const tpe_gather* __restrict__ gs,
                                                     double* __restrict__ out_f,
                                                     int64_t* __restrict__ out_i,
                                                     int32_t* __restrict__ err) {
  __shared__ int wsum[kGSlots + kGSlots / kWave];
  __shared__ int64_t carry_s;
  const tpe_gather G = gs[blockIdx.x];
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  gather_one(vals + (int64_t)G.col * ld, active + (int64_t)G.col * ld, rows, n_rows, is_below, G,
             out_f, out_i, err, wsum, carry_s);
}

// one block per descriptor; descriptor g reads history hs[g.hist]
__global__ __launch_bounds__(kGBS) void k_gather_obs_multi(const tpe_history* __restrict__ hs,
                                                           const uint8_t* __restrict__ aux,
                                                           const tpe_gather* __restrict__ gs,
                                                           double* __restrict__ out_f,
                                                           int64_t* __restrict__ out_i,
                                                           int32_t* __restrict__ err) {
  __shared__ int wsum[kGSlots + kGSlots / kWave];
  __shared__ int64_t carry_s;
  const tpe_gather G = gs[blockIdx.x];
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  const tpe_history H = hs[G.hist];
  const int32_t* rows =
      H.rows_off >= 0 ? reinterpret_cast<const int32_t*>(aux + H.rows_off) : nullptr;
  gather_one(H.vals + (int64_t)G.col * H.ld, H.active + (int64_t)G.col * H.ld, rows, H.n_rows,
             aux + H.isb_off, G, out_f, out_i, err, wsum, carry_s);
}
// appended rows: stage = vals (n_labels x k fp64, label-major) then the
// active flags (n_labels x k bytes), scattered into columns r0..r0+k-1
__global__ __launch_bounds__(256) void k_history_append(const uint8_t* __restrict__ stage,
                                                        int n_labels, int64_t k,
                                                        double* __restrict__ vals,
                                                        uint8_t* __restrict__ active, int64_t ld,
                                                        int64_t r0) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)n_labels * k) return;
  const int64_t l = t / k, j = t % k;
  const double* sv = reinterpret_cast<const double*>(stage);
  const uint8_t* sa = stage + (int64_t)n_labels * k * 8;
  vals[l * ld + r0 + j] = sv[t];
  active[l * ld + r0 + j] = sa[t];
}
}  // namespace
}  // namespace tpe

using namespace tpe;

extern "C" int tpe_history_append(const void* stage, int n_labels, int64_t k, double* vals,
                                  uint8_t* active, int64_t ld, int64_t r0, void* stream) {
  if (n_labels < 0 || k < 0 || r0 < 0 || ld < r0 + k ||
      ((int64_t)n_labels * k > 0 && (!stage || !vals || !active))) {
    set_error("tpe_history_append: bad arguments");
    return TPE_E_ARG;
  }
  const int64_t n = (int64_t)n_labels * k;
  if (n == 0) return TPE_OK;
  hipLaunchKernelGGL(k_history_append, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, static_cast<const uint8_t*>(stage), n_labels, k, vals,
                     active, ld, r0);
  return check_launch("tpe_history_append");
}

extern "C" int tpe_gather_obs(const double* vals, const uint8_t* active, int64_t ld,
                              const int32_t* rows, int64_t n_rows, const uint8_t* is_below,
                              const tpe_gather* gathers, const tpe_gather* host_gathers,
                              int n_gathers, double* obs_f64, int64_t* obs_i64, int32_t* err,
                              void* stream) {
  if (n_gathers < 0 || n_gathers > 65535 || n_rows < 0 || ld < 0) {
    set_error("tpe_gather_obs: n_gathers=%d n_rows=%lld ld=%lld", n_gathers,
              (long long)n_rows, (long long)ld);
    return TPE_E_ARG;
  }
  if (n_gathers == 0) return TPE_OK;
  if (!vals || !active || !gathers || !host_gathers || (n_rows > 0 && !is_below)) {
    set_error("tpe_gather_obs: null pointer");
    return TPE_E_ARG;
  }
  for (int i = 0; i < n_gathers; ++i) {
    const tpe_gather& g = host_gathers[i];
    if (g.col < 0 || g.dst_off < 0 || g.count < 0 || (g.to_int ? !obs_i64 : !obs_f64)) {
      set_error("tpe_gather_obs: gather %d has a bad column / offset / count / output pool", i);
      return TPE_E_ARG;
    }
  }
  hipLaunchKernelGGL(k_gather_obs, dim3(n_gathers), dim3(kGBS), 0, (hipStream_t)stream, vals,
                     active, ld, rows, n_rows, is_below, gathers, obs_f64, obs_i64, err);
  return check_launch("tpe_gather_obs");
}

extern "C" int tpe_gather_obs_multi(const tpe_history* hists, const tpe_history* host_hists,
                                    int n_hists, const void* aux, const tpe_gather* gathers,
                                    const tpe_gather* host_gathers, int n_gathers,
                                    double* obs_f64, int64_t* obs_i64, int32_t* err,
                                    void* stream) {
  if (n_gathers < 0 || n_gathers > 2147483647 || n_hists < 0) {
    set_error("tpe_gather_obs_multi: n_gathers=%d n_hists=%d", n_gathers, n_hists);
    return TPE_E_ARG;
  }
  if (n_gathers == 0) return TPE_OK;
  if (!hists || !host_hists || !aux || !gathers || !host_gathers || n_hists == 0) {
    set_error("tpe_gather_obs_multi: null pointer or no history");
    return TPE_E_ARG;
  }
  for (int h = 0; h < n_hists; ++h) {
    const tpe_history& H = host_hists[h];
    if (!H.vals || !H.active || H.ld < 0 || H.n_cols < 0 || H.n_rows < 0 || H.isb_off < 0 ||
        (H.rows_off < 0 && H.n_rows > H.ld)) {
      set_error("tpe_gather_obs_multi: history %d has a bad pointer / size / offset", h);
      return TPE_E_ARG;
    }
  }
  for (int i = 0; i < n_gathers; ++i) {
    const tpe_gather& g = host_gathers[i];
    if (g.hist < 0 || g.hist >= n_hists || g.col < 0 || g.col >= host_hists[g.hist].n_cols ||
        g.dst_off < 0 || g.count < 0 || (g.to_int ? !obs_i64 : !obs_f64)) {
      set_error("tpe_gather_obs_multi: gather %d has a bad history / column / offset / count "
                "/ output pool", i);
      return TPE_E_ARG;
    }
  }
  hipLaunchKernelGGL(k_gather_obs_multi, dim3((unsigned)n_gathers), dim3(kGBS), 0,
                     (hipStream_t)stream, hists, (const uint8_t*)aux, gathers, obs_f64, obs_i64,
                     err);
  return check_launch("tpe_gather_obs_multi");
}
