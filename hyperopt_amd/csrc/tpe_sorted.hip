// tpe_sorted.hip -- the Parzen fit from a sorted, HBM-resident history.
//
// adaptive_parzen_normal (hyperopt/tpe.py:399-467) sorts each label's below /
// above observations on every suggest.  Both sets are subsets of the label's
// whole history, and a stable sort of a subset is the whole history's stable
// order with the other rows removed.  So the history keeps, per label column,
// its rows sorted by (transformed value, row) -- updated when trials are
// appended (tpe_history_order: the new rows sorted in LDS, then merged into
// the existing order, O(T) per append instead of O(T log T) per suggest) --
// and a suggest's fit (tpe_fit_sorted) is one compaction block per segment,
// then the fit's bandwidth / coefficient launches:
//
//   1. rows in row (tid) order: which belong to the segment (active for the
//      label, on its side of the split), each one's position in the segment's
//      tid-ordered list (the linear-forgetting ramp follows it, tpe.py:441-447)
//      and how many lie below the prior mean (its searchsorted 'left' slot,
//      tpe.py:427; the len == 1 rule of tpe.py:414-421);
//   2. the column's sorted order compacted to the segment: means and ramp
//      weights in sorted order, the prior inserted at its slot;
//   3. bandwidths and clip (tpe.py:430-459), normalisation, p_accept
//      (tpe.py:145-150), fp64 / fp32 coefficients and cumulative weights:
//      the multi-kernel fit's own launches (fit_tail, tpe_parzen.hip), many
//      blocks per segment, so both fits give the same bits.
//
// Rows are ordered by (key(transform(v)), row): row order is tid order for an
// identity row list, and ties keep tid order -- np.argsort(kind="stable") of
// the reference's list (tie semantics).
#include <algorithm>

#include "tpe_common.hpp"

namespace tpe {
namespace {
constexpr int kSB = 1024;            // block size of every kernel here
constexpr int kSWaves = kSB / kWave;
constexpr int kNew = 2048;           // new rows sorted per tpe_history_order call
constexpr int kRowsPT = 12;          // rows per thread per compaction pass
constexpr int kPass = kRowsPT * kSB; // rows per compaction pass
constexpr int kSlots = kRowsPT * kSWaves;

__device__ __forceinline__ uint64_t row_key(const double* __restrict__ V, int64_t row,
                                            const tpe_colspec& C) {
  return order_key(obs_transform(V[row], C.transform, C.floor));
}

// ---- order maintenance -----------------------------------------------------
// K1: the new rows [n_old, n_old + k) of every spec's column, sorted by
// (key, row) in LDS (bitonic over the next power of two)
__global__ __launch_bounds__(kSB) void k_order_sort_new(const double* __restrict__ vals,
                                                        int64_t ld,
                                                        const tpe_colspec* __restrict__ specs,
                                                        int64_t n_old, int k,
                                                        uint64_t* __restrict__ new_keys,
                                                        int32_t* __restrict__ new_rows) {
  __shared__ uint64_t skey[kNew];
  __shared__ uint16_t sidx[kNew];
  const tpe_colspec C = specs[blockIdx.x];
  const double* V = vals + (int64_t)C.col * ld;
  int N = 2;
  while (N < k) N <<= 1;
  for (int e = threadIdx.x; e < N; e += kSB) {
    skey[e] = e < k ? row_key(V, n_old + e, C) : ~0ull;
    sidx[e] = (uint16_t)e;
  }
  __syncthreads();
  for (int s = 2; s <= N; s <<= 1) {
    for (int j = s >> 1; j > 0; j >>= 1) {
      for (int e = threadIdx.x; e < N / 2; e += kSB) {
        const int i = ((e & ~(j - 1)) << 1) | (e & (j - 1)), l = i + j;
        const uint64_t ka = skey[i], kb = skey[l];
        const uint16_t ia = sidx[i], ib = sidx[l];
        const bool gt = (ka > kb) || (ka == kb && ia > ib);
        if (gt == ((i & s) == 0)) {
          skey[i] = kb;
          skey[l] = ka;
          sidx[i] = ib;
          sidx[l] = ia;
        }
      }
      __syncthreads();
    }
  }
  uint64_t* K = new_keys + (int64_t)blockIdx.x * kNew;
  int32_t* R = new_rows + (int64_t)blockIdx.x * kNew;
  for (int e = threadIdx.x; e < k; e += kSB) {
    K[e] = skey[e];
    R[e] = (int32_t)(n_old + sidx[e]);
  }
}

// K2: merge -- an old entry at i goes to i + #(new keys < its key), a new one
// at j to j + #(old keys <= its key): old rows precede new rows (smaller row
// ids) on equal keys, so the merged order is again by (key, row)
__global__ __launch_bounds__(256) void k_order_merge(const double* __restrict__ vals, int64_t ld,
                                                     const tpe_colspec* __restrict__ specs,
                                                     const int32_t* __restrict__ order,
                                                     int64_t n_old, int k,
                                                     const uint64_t* __restrict__ new_keys,
                                                     const int32_t* __restrict__ new_rows,
                                                     int32_t* __restrict__ merged) {
  const tpe_colspec C = specs[blockIdx.y];
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = n_old + k;
  if (e >= n) return;
  const double* V = vals + (int64_t)C.col * ld;
  const int32_t* O = order + (int64_t)C.col * ld;
  const uint64_t* K = new_keys + (int64_t)blockIdx.y * kNew;
  int32_t* M = merged + (int64_t)blockIdx.y * n;
  if (e < n_old) {
    const int32_t row = O[e];
    const uint64_t key = row_key(V, row, C);
    int lo = 0, hi = k;  // #(new keys < key)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (K[mid] < key) lo = mid + 1; else hi = mid;
    }
    M[e + lo] = row;
  } else {
    const int j = (int)(e - n_old);
    const uint64_t key = K[j];
    int64_t lo = 0, hi = n_old;  // #(old keys <= key)
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (row_key(V, O[mid], C) <= key) lo = mid + 1; else hi = mid;
    }
    M[j + lo] = new_rows[(int64_t)blockIdx.y * kNew + j];
  }
}

// K3: the merged orders back into the history's order matrix
__global__ __launch_bounds__(256) void k_order_copy(const tpe_colspec* __restrict__ specs,
                                                    const int32_t* __restrict__ merged, int64_t n,
                                                    int64_t ld, int32_t* __restrict__ order) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < n) order[(int64_t)specs[blockIdx.y].col * ld + e] = merged[(int64_t)blockIdx.y * n + e];
}

// ---- the fit ------------------------------------------------------------------
// Block-wide stream compaction over items [0, n) in item order, kRowsPT items
// per thread per pass.  The loads of a pass are issued together, in two
// dependent rounds: first(i) (e.g. the order entry), then second(first) (the
// row's fields); take(L) says whether the item is kept, emit(i, rank, L) gets
// its rank among the kept items.  Returns the number kept.
struct RowLoad {
  int32_t row;
  uint8_t act, side;
  double v;
  int32_t gi;
};
template <class First, class Second, class Take, class Emit>
__device__ int64_t block_compact(int64_t n, First first, Second second, Take take, Emit emit,
                                 int* wsum, int64_t* carry_s) {
  const int lane = lane_id(), wid = threadIdx.x / kWave;
  const uint64_t lt = (1ull << lane) - 1ull;
  if (threadIdx.x == 0) *carry_s = 0;
  __syncthreads();
  for (int64_t p0 = 0; p0 < n; p0 += kPass) {
    int32_t f[kRowsPT];
#pragma unroll
    for (int t = 0; t < kRowsPT; ++t) {
      const int64_t i = p0 + (int64_t)t * kSB + threadIdx.x;
      f[t] = i < n ? first(i) : 0;
    }
    RowLoad L[kRowsPT];
#pragma unroll
    for (int t = 0; t < kRowsPT; ++t) {
      const int64_t i = p0 + (int64_t)t * kSB + threadIdx.x;
      L[t] = i < n ? second(f[t]) : RowLoad{0, 0, 2, 0.0, 0};
    }
    bool tk[kRowsPT];
    int before[kRowsPT];
#pragma unroll
    for (int t = 0; t < kRowsPT; ++t) {
      const int64_t i = p0 + (int64_t)t * kSB + threadIdx.x;
      tk[t] = i < n && take(L[t]);
      const uint64_t bal = __ballot(tk[t]);
      before[t] = __popcll(bal & lt);
      if (lane == 0) wsum[t * kSWaves + wid] = __popcll(bal);
    }
    __syncthreads();
    // exclusive scan of the kSlots (tile, wave) counts, slot order = item order
    const int c = threadIdx.x < kSlots ? wsum[threadIdx.x] : 0;
    int incl = c;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const int o = __shfl_up(incl, off, kWave);
      if (lane >= off) incl += o;
    }
    __syncthreads();
    if (threadIdx.x < kSlots && lane == kWave - 1) wsum[kSlots + wid] = incl;
    __syncthreads();
    int wave_base = 0;
    for (int q = 0; q < wid && q < kSlots / kWave; ++q) wave_base += wsum[kSlots + q];
    const int64_t carry = *carry_s;
    if (threadIdx.x < kSlots) wsum[threadIdx.x] = wave_base + incl - c;
    int total = 0;
    for (int q = 0; q < kSlots / kWave; ++q) total += wsum[kSlots + q];
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kRowsPT; ++t)
      if (tk[t]) emit(p0 + (int64_t)t * kSB + threadIdx.x,
                      carry + wsum[t * kSWaves + wid] + before[t], L[t]);
    __syncthreads();
    if (threadIdx.x == 0) *carry_s = carry + total;
    __syncthreads();
  }
  return *carry_s;
}

__global__ __launch_bounds__(kSB) void k_fit_sorted(
    const double* __restrict__ vals, const uint8_t* __restrict__ active, int64_t ld,
    const int32_t* __restrict__ order, int64_t n_rows, const uint8_t* __restrict__ is_below,
    const tpe_gather* __restrict__ gathers, tpe_seg* __restrict__ segs,
    int32_t* __restrict__ gi_scr, double* __restrict__ w, double* __restrict__ mu,
    int32_t* __restrict__ err) {
  __shared__ int wsum[kSlots + kSlots / kWave];
  __shared__ int64_t carry_s;
  __shared__ int s_lt;
  __shared__ double s_x0;
  tpe_seg* S = segs + blockIdx.x;
  const tpe_gather G = gathers[blockIdx.x];
  const int64_t col = G.col;
  const uint8_t side = G.below ? 1 : 0;
  const double* V = vals + col * ld;
  const uint8_t* A = active + col * ld;
  const int32_t* O = order + col * ld;
  int32_t* GI = gi_scr + (int64_t)blockIdx.x * n_rows;
  const int transform = S->transform;
  const double floor_ = S->floor, pmu = S->prior_mu;
  const uint64_t kp = order_key(pmu);
  const int64_t coff = S->comp_off;
  if (threadIdx.x == 0) {
    s_lt = 0;
    s_x0 = 0.0;
  }
  // 1. rows in tid order: position in the segment's list, count below the prior
  int lt = 0;
  const int64_t n = block_compact(
      n_rows, [&](int64_t r) { return (int32_t)r; },
      [&](int32_t r) { return RowLoad{r, A[r], is_below[r], V[r], 0}; },
      [&](const RowLoad& L) {
        const bool t = L.act && L.side == side;
        lt += (t && order_key(obs_transform(L.v, transform, floor_)) < kp) ? 1 : 0;
        return t;
      },
      [&](int64_t r, int64_t rank, const RowLoad& L) {
        GI[r] = (int32_t)rank;
        if (rank == 0) s_x0 = obs_transform(L.v, transform, floor_);
      },
      wsum, &carry_s);
  atomicAdd(&s_lt, lt);
  if (n != G.count) {  // the segment was sized for another count: nothing written
    if (threadIdx.x == 0 && err) atomicOr(err, 4);
    return;
  }
  __syncthreads();
  const int nn = (int)n, lf = S->lf;
  // the prior's slot: searchsorted(obs, prior_mu, 'left') (tpe.py:427), or the
  // len == 1 rule (tpe.py:414-421)
  const int prior_pos = n >= 2 ? s_lt : (n == 1 ? ((pmu < s_x0) ? 0 : 1) : 0);
  // 2. the column's sorted order compacted to the segment
  block_compact(
      n_rows, [&](int64_t e) { return O[e]; },
      [&](int32_t row) { return RowLoad{row, A[row], is_below[row], V[row], GI[row]}; },
      [&](const RowLoad& L) { return L.act && L.side == side; },
      [&](int64_t e, int64_t p, const RowLoad& L) {
        const int64_t pos = p + (p >= prior_pos ? 1 : 0);
        mu[coff + pos] = obs_transform(L.v, transform, floor_);
        w[coff + pos] = lf_weight(L.gi, nn, lf);  // ramp in tid order (tpe.py:441-447)
      },
      wsum, &carry_s);
  if (threadIdx.x == 0) {
    mu[coff + prior_pos] = pmu;
    w[coff + prior_pos] = S->prior_weight;
    S->prior_pos = prior_pos;
  }
}
}  // namespace
}  // namespace tpe

using namespace tpe;

extern "C" int64_t tpe_history_order_scratch_bytes(int n_specs, int64_t n_rows) {
  if (n_specs < 0 || n_rows < 0) return -1;
  return (int64_t)n_specs * ((int64_t)kNew * 12 + 4 * std::max<int64_t>(n_rows, 1)) + 256;
}

extern "C" int tpe_history_order(const double* vals, int64_t ld, const tpe_colspec* specs,
                                 const tpe_colspec* host_specs, int n_specs, int64_t n_old,
                                 int64_t n_new, int32_t* order, void* scratch, void* stream) {
  if (n_specs < 0 || n_specs > 65535 || n_old < 0 || n_new < 0 || n_new > kNew ||
      n_old + n_new > ld || n_old + n_new > INT32_MAX) {
    set_error("tpe_history_order: n_specs=%d n_old=%lld n_new=%lld ld=%lld (at most %d new rows "
              "per call)", n_specs, (long long)n_old, (long long)n_new, (long long)ld, kNew);
    return TPE_E_ARG;
  }
  if (n_specs == 0 || n_new == 0) return TPE_OK;
  if (!vals || !specs || !host_specs || !order || !scratch) {
    set_error("tpe_history_order: null pointer");
    return TPE_E_ARG;
  }
  for (int i = 0; i < n_specs; ++i)
    if (host_specs[i].col < 0 || (host_specs[i].transform != TPE_OBS_IDENTITY &&
                                  host_specs[i].transform != TPE_OBS_LOG)) {
      set_error("tpe_history_order: spec %d has a bad column / transform", i);
      return TPE_E_ARG;
    }
  char* p = static_cast<char*>(scratch);
  uint64_t* keys = reinterpret_cast<uint64_t*>(p);
  int32_t* rows = reinterpret_cast<int32_t*>(p + (int64_t)n_specs * kNew * 8);
  int32_t* merged = reinterpret_cast<int32_t*>(p + (int64_t)n_specs * kNew * 12);
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = n_old + n_new;
  const dim3 g((unsigned)((n + 255) / 256), (unsigned)n_specs);
  hipLaunchKernelGGL(k_order_sort_new, dim3(n_specs), dim3(kSB), 0, st, vals, ld, specs, n_old,
                     (int)n_new, keys, rows);
  hipLaunchKernelGGL(k_order_merge, g, dim3(256), 0, st, vals, ld, specs, order, n_old,
                     (int)n_new, keys, rows, merged);
  hipLaunchKernelGGL(k_order_copy, g, dim3(256), 0, st, specs, merged, n, ld, order);
  return check_launch("tpe_history_order");
}

// scratch: the per-row list positions (int32 per segment and row), then the
// fit tail's tile partials (counts are <= n_rows)
static int64_t gi_bytes(int n_seg, int64_t n_rows) {
  return (4 * (int64_t)std::max(n_seg, 1) * std::max<int64_t>(n_rows, 1) + 255) / 256 * 256;
}
extern "C" int64_t tpe_fit_sorted_scratch_bytes(int n_seg, int64_t n_rows) {
  if (n_seg < 0 || n_rows < 0 || n_rows > INT32_MAX) return -1;
  return gi_bytes(n_seg, n_rows) +
         8 * (int64_t)std::max(n_seg, 1) * fit_part_doubles((int)n_rows);
}

extern "C" int tpe_fit_sorted(const double* vals, const uint8_t* active, int64_t ld,
                              const int32_t* order, int64_t n_rows, const uint8_t* is_below,
                              const tpe_gather* gathers, const tpe_gather* host_gathers,
                              tpe_seg* segs, int n_seg, void* scratch, double* w, double* mu,
                              double* sigma, double* wcdf, double* coef64, float* coef32,
                              int32_t* err, void* stream) {
  if (n_seg < 0 || n_seg > 65535 || n_rows < 0 || n_rows > ld || n_rows > INT32_MAX) {
    set_error("tpe_fit_sorted: n_seg=%d n_rows=%lld ld=%lld", n_seg, (long long)n_rows,
              (long long)ld);
    return TPE_E_ARG;
  }
  if (n_seg == 0) return TPE_OK;
  if (!vals || !active || !order || !is_below || !gathers || !host_gathers || !segs ||
      !scratch || !w || !mu || !sigma || !wcdf || !coef64 || !coef32) {
    set_error("tpe_fit_sorted: null pointer");
    return TPE_E_ARG;
  }
  for (int i = 0; i < n_seg; ++i) {
    const tpe_gather& g = host_gathers[i];
    if (g.col < 0 || g.to_int || g.count < 0 || g.count > n_rows) {
      set_error("tpe_fit_sorted: segment %d: column %d, count %lld (at most n_rows = %lld "
                "observations)", i, g.col, (long long)g.count, (long long)n_rows);
      return TPE_E_ARG;
    }
  }
  int max_obs = 0;
  for (int i = 0; i < n_seg; ++i) max_obs = std::max(max_obs, (int)host_gathers[i].count);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_fit_sorted, dim3(n_seg), dim3(kSB), 0, st, vals, active, ld, order, n_rows,
                     is_below, gathers, segs, reinterpret_cast<int32_t*>(scratch), w, mu, err);
  double* part = reinterpret_cast<double*>(static_cast<char*>(scratch) + gi_bytes(n_seg, n_rows));
  fit_tail(segs, n_seg, max_obs, part, w, mu, sigma, wcdf, coef64, coef32, st);
  return check_launch("tpe_fit_sorted");
}
