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

__global__ __launch_bounds__(kGBS) void k_gather_obs(const double* __restrict__ vals,
                                                     const uint8_t* __restrict__ active,
                                                     int64_t ld, const int32_t* __restrict__ rows,
                                                     int64_t n_rows,
                                                     const uint8_t* __restrict__ is_below,
                                                     const tpe_gather* __restrict__ gs,
                                                     double* __restrict__ out_f,
                                                     int64_t* __restrict__ out_i,
                                                     int32_t* __restrict__ err) {
  __shared__ int wsum[kGWaves];
  __shared__ int64_t carry_s;
  const tpe_gather G = gs[blockIdx.x];
  const double* V = vals + (int64_t)G.col * ld;
  const uint8_t* A = active + (int64_t)G.col * ld;
  const uint8_t side = G.below ? 1 : 0;
  const int lane = lane_id(), wid = threadIdx.x / kWave;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  for (int64_t t0 = 0; t0 < n_rows; t0 += kGBS) {
    const int64_t i = t0 + threadIdx.x;
    bool take = false;
    int64_t r = 0;
    if (i < n_rows) {
      r = rows ? (int64_t)rows[i] : i;
      take = A[r] && (is_below[i] == side);
    }
    const uint64_t bal = __ballot(take);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wid] = __popcll(bal);
    __syncthreads();
    int64_t pos = carry_s;
    int tile = 0;
    for (int q = 0; q < kGWaves; ++q) {
      const int c = wsum[q];
      if (q < wid) pos += c;
      tile += c;
    }
    pos += before;
    if (take && pos < G.count) {
      const double v = V[r];
      if (G.to_int)
        out_i[G.dst_off + pos] = (int64_t)v - G.offset;
      else
        out_f[G.dst_off + pos] = v;
    }
    __syncthreads();  // everyone has read carry_s / wsum
    if (threadIdx.x == 0) carry_s += tile;
    __syncthreads();
  }
  if (threadIdx.x == 0 && carry_s != G.count && err) atomicOr(err, 4);
}
}  // namespace
}  // namespace tpe

using namespace tpe;

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
