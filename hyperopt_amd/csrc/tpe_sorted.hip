// tpe_sorted.hip -- the Parzen fit from a sorted, HBM-resident history.
//
// adaptive_parzen_normal (hyperopt/tpe.py:399-467) sorts each label's below /
// above observations on every suggest.  Both sets are subsets of the label's
// whole history, and a stable sort of a subset is the whole history's stable
// order with the other rows removed.  So the history keeps, per label column,
// its rows sorted by (transformed value, row) -- updated when trials are
// appended (tpe_history_order: the new rows sorted in LDS, then merged into
// the existing order, O(T) per append instead of O(T log T) per suggest) --
// and a suggest's fit (tpe_fit_sorted) is a chunked compaction (two
// launches over (chunk, segment) blocks), then the fit's bandwidth /
// coefficient launches:
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
#include <cstdlib>

#include "tpe_common.hpp"

namespace tpe {
namespace {
constexpr int kSB = 1024;            // block size of every kernel here
constexpr int kNew = 2048;           // new rows sorted per tpe_history_order call

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
// ---- the fit: chunked compaction ---------------------------------------------
// Rows (tid order) and order entries (sorted order) are cut into chunks of
// kChunk; every (chunk, segment) pair is a 256-thread block, so a segment's
// random gathers through its column's order (the rows' flags, values and list
// positions) are spread over many CUs instead of one CU's load pipeline.
// Two launches: counts per chunk with every row's rank among its chunk's
// members, then the sorted-order emit (means and ramp weights), which adds
// the row's chunk base (an exclusive prefix of the chunk counts, formed in
// LDS by every block) to the rank it gathers; each block re-reduces the few
// counts of the chunks before it (fixed order).
constexpr int kCB = 256;                 // block size of the compaction kernels
constexpr int kCR = 4;                   // items per thread
constexpr int kChunk = kCB * kCR;        // items per chunk (item u * kCB + t of a chunk)
constexpr int kCnt = 4;                  // per (segment, chunk): members tid / lt / first row / members sorted

struct SegView {
  const double* V;
  const uint8_t* A;
  const int32_t* O;
  uint8_t side;
  int transform;
  double floor_;
  uint64_t kp;
};
__device__ __forceinline__ SegView seg_view(const double* vals, const uint8_t* active,
                                            const int32_t* order, int64_t ld,
                                            const tpe_gather& G, const tpe_seg& S) {
  const int64_t col = G.col;
  return SegView{vals + col * ld, active + col * ld, order + col * ld,
                 (uint8_t)(G.below ? 1 : 0), S.transform, S.floor, order_key(S.prior_mu)};
}

// exclusive ranks of the kept items of a chunk (item order u * kCB + t) and
// the chunk's total; sh: >= kCR * kCB / kWave ints
__device__ __forceinline__ int chunk_ranks(const bool (&tk)[kCR], int (&rank)[kCR], int* sh) {
  constexpr int kNW = kCB / kWave;
  const int lane = lane_id(), wid = threadIdx.x / kWave;
  const uint64_t lt = (1ull << lane) - 1ull;
  int before[kCR];
#pragma unroll
  for (int u = 0; u < kCR; ++u) {
    const uint64_t bal = __ballot(tk[u]);
    before[u] = __popcll(bal & lt);
    if (lane == 0) sh[u * kNW + wid] = __popcll(bal);
  }
  __syncthreads();
  int total = 0, mine[kCR];
#pragma unroll
  for (int u = 0; u < kCR; ++u) mine[u] = 0;
  for (int q = 0; q < kCR * kNW; ++q) {  // 16 slot counts, slot order = item order
    const int c = sh[q];
#pragma unroll
    for (int u = 0; u < kCR; ++u) mine[u] += (q < u * kNW + wid) ? c : 0;
    total += c;
  }
#pragma unroll
  for (int u = 0; u < kCR; ++u) rank[u] = mine[u] + before[u];
  __syncthreads();  // sh reused
  return total;
}

// K1: per (chunk, segment): members in the tid-order chunk, how many of them
// lie below the prior mean, the first member row; members in the sorted
// chunk; and every row's word: its rank among the chunk's members (-1 for a
// non-member) -- the chunk's base is added where the word is read (K3)
__global__ __launch_bounds__(kCB) void k_fit_count(
    const double* __restrict__ vals, const uint8_t* __restrict__ active, int64_t ld,
    const int32_t* __restrict__ order, int64_t n_rows, const uint8_t* __restrict__ is_below,
    const tpe_gather* __restrict__ gathers, const tpe_seg* __restrict__ segs,
    int32_t* __restrict__ cnt, int32_t* __restrict__ gi_scr) {
  __shared__ int sh[kCR * (kCB / kWave)];
  static_assert(kCR >= 4, "four block reductions share sh");
  const int sg = blockIdx.y;
  const SegView Q = seg_view(vals, active, order, ld, gathers[sg], segs[sg]);
  const int64_t c0 = (int64_t)blockIdx.x * kChunk;
  int32_t rows[kCR];
#pragma unroll
  for (int u = 0; u < kCR; ++u) {
    const int64_t e = c0 + u * kCB + threadIdx.x;
    rows[u] = e < n_rows ? Q.O[e] : -1;
  }
  int n1 = 0, nlt = 0, n2 = 0, first = INT32_MAX;
  bool tk[kCR];
#pragma unroll
  for (int u = 0; u < kCR; ++u) {
    const int64_t r = c0 + u * kCB + threadIdx.x;
    tk[u] = r < n_rows && Q.A[r] && is_below[r] == Q.side;
    if (tk[u]) {
      ++n1;
      nlt += order_key(obs_transform(Q.V[r], Q.transform, Q.floor_)) < Q.kp ? 1 : 0;
      first = min(first, (int)r);
    }
    const int32_t row = rows[u];
    if (row >= 0 && Q.A[row] && is_below[row] == Q.side) ++n2;
  }
  int rk[kCR];
  chunk_ranks(tk, rk, sh);
  int32_t* GI = gi_scr + (int64_t)sg * n_rows;
#pragma unroll
  for (int u = 0; u < kCR; ++u) {
    const int64_t r = c0 + u * kCB + threadIdx.x;
    if (r < n_rows) GI[r] = tk[u] ? rk[u] : -1;
  }
  n1 = block_sum<kCB, int>(n1, sh);
  nlt = block_sum<kCB, int>(nlt, sh + kCB / kWave);
  n2 = block_sum<kCB, int>(n2, sh + 2 * (kCB / kWave));
  first = -block_max<kCB, int>(-first, sh + 3 * (kCB / kWave));
  if (threadIdx.x == 0) {
    int32_t* C = cnt + ((int64_t)sg * gridDim.x + blockIdx.x) * kCnt;
    C[0] = n1;
    C[1] = nlt;
    C[2] = first;
    C[3] = n2;
  }
}

// exclusive block scan of one int per thread (sh: >= kCB / kWave ints,
// reusable after the call); total: the block's sum
__device__ __forceinline__ int block_excl_sum(int v, int* sh, int& total) {
  constexpr int kNW = kCB / kWave;
  const int lane = lane_id(), wid = threadIdx.x / kWave;
  int incl = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int x = __shfl_up(incl, o, kWave);
    if (lane >= o) incl += x;
  }
  __syncthreads();
  if (lane == kWave - 1) sh[wid] = incl;
  __syncthreads();
  int pos = incl - v;
  total = 0;
#pragma unroll
  for (int w = 0; w < kNW; ++w) {
    pos += w < wid ? sh[w] : 0;
    total += sh[w];
  }
  __syncthreads();
  return pos;
}

// columns of up to kPreChunks chunks (4M rows) take the chunk bases from LDS
// in K3; longer ones globalize the words first (K2)
constexpr int kPreChunks = 4096;

// sum of field f over chunks [0, c) (all threads; fixed order)
__device__ __forceinline__ int64_t chunks_before(const int32_t* C, int c, int f, int64_t* sh) {
  int64_t v = 0;
  for (int q = threadIdx.x; q < c; q += kCB) v += C[q * kCnt + f];
  return block_sum<kCB, int64_t>(v, sh);
}

// K2 (columns of more than kPreChunks chunks only): the chunk's base added
// to its members' words in place, so K3 reads global list positions
__global__ __launch_bounds__(kCB) void k_fit_globalize(int64_t n_rows,
                                                       const int32_t* __restrict__ cnt,
                                                       int32_t* __restrict__ gi_scr) {
  __shared__ int64_t sh64[kCB / kWave];
  const int sg = blockIdx.y;
  const int32_t* C = cnt + (int64_t)sg * gridDim.x * kCnt;
  const int64_t base = chunks_before(C, blockIdx.x, 0, sh64);
  const int64_t c0 = (int64_t)blockIdx.x * kChunk;
  int32_t* GI = gi_scr + (int64_t)sg * n_rows;
#pragma unroll
  for (int u = 0; u < kCR; ++u) {
    const int64_t r = c0 + u * kCB + threadIdx.x;
    if (r < n_rows) {
      const int32_t g = GI[r];
      if (g >= 0) GI[r] = (int32_t)(base + g);
    }
  }
}

// K3: sorted-order emit -- means and ramp weights in sorted order, the prior
// at its slot: searchsorted(obs, prior_mu, 'left') (tpe.py:427), or the
// len == 1 rule (tpe.py:414-421).  A count other than gathers[sg].count sets
// bit 4 of *err and writes nothing.
template <bool LOCAL>  // LOCAL: the words are chunk-local ranks (K2 skipped)
__global__ __launch_bounds__(kCB) void k_fit_emit_sorted(
    const double* __restrict__ vals, const uint8_t* __restrict__ active, int64_t ld,
    const int32_t* __restrict__ order, int64_t n_rows, const uint8_t* __restrict__ is_below,
    const tpe_gather* __restrict__ gathers, tpe_seg* __restrict__ segs,
    const int32_t* __restrict__ cnt, const int32_t* __restrict__ gi_scr,
    double* __restrict__ w, double* __restrict__ mu, int32_t* __restrict__ err) {
  __shared__ int sh[kCR * (kCB / kWave)];
  __shared__ int64_t sh64[kCB / kWave];
  __shared__ int32_t s_pre[LOCAL ? kPreChunks : 1];  // tid chunks' member bases
  const int sg = blockIdx.y;
  tpe_seg* S = segs + sg;
  const tpe_gather G = gathers[sg];
  const SegView Q = seg_view(vals, active, order, ld, G, *S);
  const int nch = gridDim.x;
  const int32_t* C = cnt + (int64_t)sg * nch * kCnt;
  const int64_t n = chunks_before(C, nch, 0, sh64);
  if (n != G.count) {  // the segment was sized for another count: nothing written
    if (blockIdx.x == 0 && threadIdx.x == 0 && err) atomicOr(err, 4);
    return;
  }
  const int64_t n_lt = chunks_before(C, nch, 1, sh64);
  const int64_t base = chunks_before(C, blockIdx.x, 3, sh64);
  if constexpr (LOCAL) {  // exclusive prefix of the tid chunks' member counts
    int carry = 0;
    for (int q0 = 0; q0 < nch; q0 += kCB) {
      const int q = q0 + (int)threadIdx.x;
      const int c = q < nch ? C[q * kCnt] : 0;
      int total;
      const int ex = block_excl_sum(c, sh, total);
      if (q < nch) s_pre[q] = carry + ex;
      carry += total;
    }
    __syncthreads();
  }
  int prior_pos = 0;
  if (n >= 2) {
    prior_pos = (int)n_lt;
  } else if (n == 1) {
    int first = INT32_MAX;
    for (int q = 0; q < nch; ++q) first = min(first, C[q * kCnt + 2]);
    const double x0 = obs_transform(Q.V[first], Q.transform, Q.floor_);
    prior_pos = (S->prior_mu < x0) ? 0 : 1;
  }
  const int64_t c0 = (int64_t)blockIdx.x * kChunk;
  int32_t rows[kCR];
#pragma unroll
  for (int u = 0; u < kCR; ++u) {
    const int64_t e = c0 + u * kCB + threadIdx.x;
    rows[u] = e < n_rows ? Q.O[e] : -1;
  }
  bool tk[kCR];
  double v[kCR];
  int32_t gi[kCR];
#pragma unroll
  for (int u = 0; u < kCR; ++u) {
    const int32_t row = rows[u];
    const bool in = row >= 0;
    v[u] = in ? Q.V[row] : 0.0;
    gi[u] = in ? gi_scr[(int64_t)sg * n_rows + row] : -1;  // -1: not a member
    tk[u] = gi[u] >= 0;
    if (LOCAL && tk[u]) gi[u] += s_pre[row / kChunk];
  }
  int rk[kCR];
  chunk_ranks(tk, rk, sh);
  const int64_t coff = S->comp_off;
  const int nn = (int)n, lf = S->lf;
#pragma unroll
  for (int u = 0; u < kCR; ++u) {
    if (!tk[u]) continue;
    const int64_t p = base + rk[u];
    const int64_t pos = p + (p >= prior_pos ? 1 : 0);
    mu[coff + pos] = obs_transform(v[u], Q.transform, Q.floor_);
    w[coff + pos] = lf_weight(gi[u], nn, lf);  // ramp in tid order (tpe.py:441-447)
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    mu[coff + prior_pos] = S->prior_mu;
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

// scratch: the per-row list positions (int32 per segment and row), the chunk
// counts, then the fit tail's tile partials (counts are <= n_rows)
static int64_t gi_bytes(int n_seg, int64_t n_rows) {
  return (4 * (int64_t)std::max(n_seg, 1) * std::max<int64_t>(n_rows, 1) + 255) / 256 * 256;
}
static int64_t n_chunks(int64_t n_rows) { return std::max<int64_t>(1, (n_rows + kChunk - 1) / kChunk); }
static int64_t cnt_bytes(int n_seg, int64_t n_rows) {
  return (4 * kCnt * (int64_t)std::max(n_seg, 1) * n_chunks(n_rows) + 255) / 256 * 256;
}
extern "C" int64_t tpe_fit_sorted_scratch_bytes(int n_seg, int64_t n_rows) {
  if (n_seg < 0 || n_rows < 0 || n_rows > INT32_MAX) return -1;
  return gi_bytes(n_seg, n_rows) + cnt_bytes(n_seg, n_rows) +
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
  char* p = static_cast<char*>(scratch);
  int32_t* gi = reinterpret_cast<int32_t*>(p);
  int32_t* cnt = reinterpret_cast<int32_t*>(p + gi_bytes(n_seg, n_rows));
  double* part = reinterpret_cast<double*>(p + gi_bytes(n_seg, n_rows) + cnt_bytes(n_seg, n_rows));
  const dim3 grid((unsigned)n_chunks(n_rows), (unsigned)n_seg);
  hipLaunchKernelGGL(k_fit_count, grid, dim3(kCB), 0, st, vals, active, ld, order, n_rows,
                     is_below, gathers, segs, cnt, gi);
  // TPE_FIT_GLOBALIZE=1 (tests): the long-column path at any size
  const char* gl = getenv("TPE_FIT_GLOBALIZE");
  if (n_chunks(n_rows) <= kPreChunks && !(gl && gl[0] == '1')) {
    hipLaunchKernelGGL(k_fit_emit_sorted<true>, grid, dim3(kCB), 0, st, vals, active, ld, order,
                       n_rows, is_below, gathers, segs, cnt, gi, w, mu, err);
  } else {
    hipLaunchKernelGGL(k_fit_globalize, grid, dim3(kCB), 0, st, n_rows, cnt, gi);
    hipLaunchKernelGGL(k_fit_emit_sorted<false>, grid, dim3(kCB), 0, st, vals, active, ld, order,
                       n_rows, is_below, gathers, segs, cnt, gi, w, mu, err);
  }
  fit_tail(segs, n_seg, max_obs, part, w, mu, sigma, wcdf, coef64, coef32, st);
  return check_launch("tpe_fit_sorted");
}
