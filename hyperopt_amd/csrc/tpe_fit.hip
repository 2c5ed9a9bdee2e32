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
// sequentially in observation order, fl(..fl(fl(c + w0) + w1)..), and the
// result must be that chain's bits.  The wave scans 64 observations per
// step, ballots the matches, and every matching lane writes its weight
// (computed in parallel) into the wave's LDS list at its rank; a full list
// is folded into the running count by seq_fold below -- the same bits as the
// serial chain, in a few wave-wide passes instead of one fp64 add latency
// per match (a 60 000-match category: ~0.45 ms serially).
constexpr int kCatList = 1024;  // weights buffered per wave before a fold

// The sequential fp64 sum S_{k+1} = fl(S_k + w_k) over list[0, n), wave-
// parallel and bit-exact (every lane returns it).  While S stays in one
// binade [2^e, 2^(e+1)) its values are A * u (u = 2^(e-52), A < 2^53 an
// integer) and each step adds d_k * u with d_k = w_k / u rounded to an
// integer -- nearest, ties to the even A_{k+1} (IEEE round-to-nearest-even
// on the binade's grid).  d_k is a shift of w_k's mantissa except at a tie
// (remainder exactly u/2), where it depends on the parity of A_k; parities
// compose as maps P -> a P ^ c (a tie: P -> 0, else P -> P ^ (d_k & 1)), so
// one wave scan of those maps and one of the d_k give every A_k.  The first
// step whose A would reach 2^53 (the next binade, where the grid is 2u), or
// whose w_k is at least 2^(e+1), is taken by the hardware add from its exact
// predecessor, and the pass repeats from the step after it.  Passes: one
// per list plus one per binade crossed.  (Checked against the serial chain
// on LF ramps, dyadic tie-heavy weights and 24-decade ranges:
// tests/test_seq_fold.py restates it on the host; the GPU tests compare the
// counts with np.bincount's.)
// wave scans by DPP (row shifts, then the row broadcasts of 15 and 31):
// lanes whose source is outside the wave keep `old`, the scan's identity
template <int CTRL, int ROWM>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t old, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWM, 0xF, false);
}
template <int CTRL, int ROWM>
__device__ __forceinline__ void scan_step_u64(uint64_t& v) {
  const uint32_t lo = dpp_u32<CTRL, ROWM>(0u, (uint32_t)v);
  const uint32_t hi = dpp_u32<CTRL, ROWM>(0u, (uint32_t)(v >> 32));
  v += ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_incl_sum_u64(uint64_t v) {
  scan_step_u64<0x111, 0xF>(v);  // row_shr:1
  scan_step_u64<0x112, 0xF>(v);  // row_shr:2
  scan_step_u64<0x114, 0xF>(v);  // row_shr:4
  scan_step_u64<0x118, 0xF>(v);  // row_shr:8
  scan_step_u64<0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3
  scan_step_u64<0x143, 0xC>(v);  // row_bcast:31 -> rows 2, 3
  return v;
}
// parity maps P -> a P ^ c packed as a | c << 1; y (earlier) then x
__device__ __forceinline__ uint32_t map_then(uint32_t y, uint32_t x) {
  const uint32_t a2 = x & 1u, c2 = (x >> 1) & 1u;
  return (a2 & y & 1u) | ((((a2 & (y >> 1)) ^ c2) & 1u) << 1);
}
template <int CTRL, int ROWM>
__device__ __forceinline__ void scan_step_map(uint32_t& x) {
  x = map_then(dpp_u32<CTRL, ROWM>(1u, x), x);  // (1: the identity map)
}

// The same sum by lane 0 alone (list reads batched; every lane returns it):
// one dependent fp64 add per entry, cheaper than seq_fold's passes while the
// sum is small and crosses a binade every few entries (the first ~4k of a
// chain: a pass per crossing)
constexpr int kSerialHits = 4096;
__device__ double serial_fold(double S, const double* list, int n, int lane) {
  if (lane == 0) {
    constexpr int kB = 8;
    int j = 0;
    for (; j + kB <= n; j += kB) {
      double v[kB];
#pragma unroll
      for (int i = 0; i < kB; ++i) v[i] = list[j + i];
#pragma unroll
      for (int i = 0; i < kB; ++i) S = __dadd_rn(S, v[i]);
    }
    for (; j < n; ++j) S = __dadd_rn(S, list[j]);
  }
  return __shfl(S, 0, kWave);
}
// list[0, n) into S, the first entries of a chain (done < kSerialHits)
// serially, the rest by seq_fold
template <int kSE>
__device__ double fold_list(double S, const double* list, int n, int64_t& done, int lane);

// one entry's d (w / u rounded on the binade of biased exponent es, ties
// left for the parity scan: bit j of tie), or bit j of huge (w >= 2^(e+1))
__device__ __forceinline__ uint64_t fold_step(double w, int es, bool on, uint32_t& tie,
                                              uint32_t& huge, int j) {
  if (!on) return 0;
  constexpr uint64_t kFrac = (1ull << 52) - 1;
  const uint64_t wb = (uint64_t)__double_as_longlong(w);
  const int ew = (int)((wb >> 52) & 0x7ff);
  const uint64_t M = (wb & kFrac) | (ew ? (1ull << 52) : 0ull);
  const int sh = es - max(ew, 1);
  if (sh < 0) {
    huge |= 1u << j;
    return 0;
  }
  if (sh == 0) return M;
  if (sh >= 64) return 0;
  const uint64_t rem = M & ((1ull << sh) - 1), half = 1ull << (sh - 1);
  if (rem == half) tie |= 1u << j;
  return (M >> sh) + (rem > half ? 1ull : 0ull);
}

template <int kSE>
__device__ double seq_fold(double S, const double* list, int n, int lane) {
  double v[kSE];
#pragma unroll
  for (int j = 0; j < kSE; ++j) {
    const int i = lane * kSE + j;
    v[j] = i < n ? list[i] : 0.0;
  }
  constexpr uint64_t kFrac = (1ull << 52) - 1, kTop = 1ull << 53;
  int r0 = 0;
  while (r0 < n) {  // (wave-uniform)
    const uint64_t sb = (uint64_t)__double_as_longlong(S);
    const int es = (int)((sb >> 52) & 0x7ff);
    if (S == 0.0 || es == 0) {  // 0 + w = w; a subnormal sum (never on the LF ramp): one add
      S = __dadd_rn(S, list[r0]);
      ++r0;
      continue;
    }
    const uint64_t A = (sb & kFrac) | (1ull << 52);
    uint64_t d[kSE];
    uint32_t tie = 0, huge = 0;
#pragma unroll
    for (int j = 0; j < kSE; ++j) {
      const int i = lane * kSE + j;
      d[j] = fold_step(v[j], es, i >= r0 && i < n, tie, huge, j);
    }
    // parity maps (bit 0: a, bit 1: c), composed over the lane, then an
    // inclusive wave scan (later o earlier: a = a2 a1, c = a2 c1 ^ c2)
    uint32_t a = 1, c = 0;
#pragma unroll
    for (int j = 0; j < kSE; ++j) {
      if ((tie >> j) & 1u) {
        a = 0;
        c = 0;
      } else {
        c ^= (uint32_t)(d[j] & 1ull);
      }
    }
    uint32_t x = a | (c << 1);
    scan_step_map<0x111, 0xF>(x);
    scan_step_map<0x112, 0xF>(x);
    scan_step_map<0x114, 0xF>(x);
    scan_step_map<0x118, 0xF>(x);
    scan_step_map<0x142, 0xA>(x);
    scan_step_map<0x143, 0xC>(x);
    const uint32_t ex = dpp_u32<0x138, 0xF>(1u, x);  // wave_shr:1 (lane 0: the identity)
    uint32_t P = ((ex & 1u) & (uint32_t)(A & 1ull)) ^ (ex >> 1);
    uint64_t tot = 0;
#pragma unroll
    for (int j = 0; j < kSE; ++j) {
      if ((tie >> j) & 1u) {
        d[j] += (P + d[j]) & 1ull;  // ties to the even A_{k+1}
        P = 0;
      } else {
        P ^= (uint32_t)(d[j] & 1ull);
      }
      tot += d[j];
    }
    const uint64_t incl = wave_incl_sum_u64(tot);
    // the first step leaving the binade
    uint64_t cum = incl - tot;
    int jc = -1;
#pragma unroll
    for (int j = 0; j < kSE; ++j) {
      if (jc < 0) {
        if (((huge >> j) & 1u) || A + cum + d[j] >= kTop) jc = j;
        else cum += d[j];
      }
    }
    const uint64_t bal = __ballot(jc >= 0);
    auto lane_u64 = [](uint64_t v, int l) {
      return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    };
    if (bal == 0) {
      const uint64_t Dt = lane_u64(incl, kWave - 1);
      S = ldexp((double)(A + Dt), es - 1075);
      r0 = n;
    } else {
      const int L = __ffsll((unsigned long long)bal) - 1;
      const int g = L * kSE + __builtin_amdgcn_readlane(jc, L);
      const uint64_t Dx = lane_u64(cum, L);
      S = __dadd_rn(ldexp((double)(A + Dx), es - 1075), list[g]);
      r0 = g + 1;
    }
  }
  return S;
}

template <int kSE>
__device__ double fold_list(double S, const double* list, int n, int64_t& done, int lane) {
  int f = 0;
  if (done < kSerialHits) {
    f = (int)std::min<int64_t>(n, kSerialHits - done);
    S = serial_fold(S, list, f, lane);
  }
  constexpr int kN = kSE * kWave;
  for (; f < n; f += kN) S = seq_fold<kSE>(S, list + f, min(kN, n - f), lane);
  done += n;
  return S;
}

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
  int64_t folded = 0;
  auto fold = [&]() {
    __builtin_amdgcn_wave_barrier();
    cnt = fold_list<8>(cnt, list, filled, folded, lane);
    filled = 0;
    __builtin_amdgcn_wave_barrier();
  };
  // kDepth tiles of 64 observations per step, the next step's loads issued
  // before this step's matches are listed (a latency-bound scan); the list
  // holds a whole step, so it is folded only between steps
  constexpr int kDepth = 16;
  static_assert(kDepth * kWave <= kCatList, "a step's matches fit the list");
  const int64_t* O = obs + S.obs_off;
  int64_t nxt[kDepth];
#pragma unroll
  for (int b = 0; b < kDepth; ++b) {
    const int i = b * kWave + lane;
    nxt[b] = i < n ? O[i] : -1;
  }
  for (int t0 = 0; t0 < n; t0 += kDepth * kWave) {
    int64_t cur[kDepth];
#pragma unroll
    for (int b = 0; b < kDepth; ++b) {
      cur[b] = nxt[b];
      const int i = t0 + (kDepth + b) * kWave + lane;
      nxt[b] = i < n ? O[i] : -1;
    }
    if (filled + kDepth * kWave > kCatList) fold();
#pragma unroll
    for (int b = 0; b < kDepth; ++b) {
      const bool hit = cur[b] == (int64_t)k;
      const uint64_t m = __ballot(hit);
      if (m == 0) continue;  // wave-uniform
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

// The same counts read straight from the HBM history (the gathered lists'
// work folded in): one 1024-thread block per (segment, category) walks the
// rows in windows of kCHW (row order = tid order, as tpe_gather_obs lists
// them), a row being an observation of the segment when the label is active
// there and the row is on the segment's side of the split.  Waves 1-15 scan:
// one scan of the packed (observations << 16 | matches) counts per (tile,
// wave) gives every observation its position in the segment -- its LF
// weight -- and every match its rank in the window, the window's match
// weights going to LDS in order; wave 0 folds (seq_fold) the previous
// window's weights meanwhile, from the other of two LDS buffers (the fold of
// a long chain is a serial-latency walk; the scan is load latency: they
// overlap).  A segment whose observation count differs from S.n_obs sets
// bit 4 of *err (tpe_gather_obs' rule).
constexpr int kCHB = 1024;             // block
constexpr int kCHScan = kCHB / kWave - 1;  // scanning waves (wave 0 folds)
constexpr int kCHT = 8;                // rows per scanning thread per window
constexpr int kCHW = kCHScan * kWave * kCHT;  // rows per window (7 680)
constexpr int kCHSlots = kCHT * kCHScan;      // (tile, wave) counts per window
constexpr int kCHSE = 8;               // seq_fold entries per lane (512 per pass; wider
                                       // passes measured slower: 16 +25 %, 32 +65 %)
static_assert(kCHSlots <= 2 * kWave, "the slot scan: two slots per lane of one wave");
static_assert(kCHW < (1 << 16), "packed 16-bit counts");

__global__ __launch_bounds__(kCHB) void k_cat_counts_hist(
    const double* __restrict__ vals, const uint8_t* __restrict__ active, int64_t ld,
    const int32_t* __restrict__ rows, int64_t n_rows, const uint8_t* __restrict__ is_below,
    const tpe_gather* __restrict__ gathers, const tpe_cat_seg* __restrict__ segs,
    double* __restrict__ p, int32_t* __restrict__ err) {
  __shared__ double s_w[2][kCHW];
  __shared__ uint32_t s_slot[2 * kWave];
  __shared__ uint32_t s_tot[2];  // per buffer: the window's packed totals
  const tpe_cat_seg S = segs[blockIdx.y];
  const int k = blockIdx.x;
  if (k >= S.n_cat) return;  // (block-uniform)
  const tpe_gather G = gathers[blockIdx.y];
  const double* __restrict__ V = vals + (int64_t)G.col * ld;
  const uint8_t* __restrict__ Ac = active + (int64_t)G.col * ld;
  const uint8_t side = G.below ? 1 : 0;
  const int lane = lane_id(), wid = threadIdx.x / kWave;
  const int sw = wid - 1;                   // scanning wave index (waves 1..)
  const int st = threadIdx.x - kWave;       // scanning thread index
  const uint64_t lt = (1ull << lane) - 1ull;
  const int n = S.n_obs;
  const bool ramp = S.lf > 0 && S.lf < n;
  const int64_t num = n - S.lf;
  const double start = 1.0 / (double)n;
  const double step = (ramp && num > 1) ? (1.0 - start) / (double)(num - 1) : 0.0;
  double cnt = 0.0;     // (wave 0)
  int64_t folded = 0;  // (wave 0) matches folded so far
  int64_t carry = 0;   // (scanners) observations before the window
  const int64_t n_win = (n_rows + kCHW - 1) / kCHW;
  for (int64_t it = 0; it <= n_win; ++it) {  // (block-uniform; the last round only folds)
    const int buf = (int)(it & 1);
    const bool scan = it < n_win;
    bool mem[kCHT], hit[kCHT];
    uint32_t pre[kCHT];
    // ---- phase 0: scanners load and ballot window `it`; wave 0 folds window it - 1
    if (wid > 0 && scan) {
      const int64_t p0 = it * kCHW;
#pragma unroll
      for (int t = 0; t < kCHT; ++t) {
        const int64_t i = p0 + (int64_t)t * (kCHScan * kWave) + st;
        mem[t] = hit[t] = false;
        if (i < n_rows) {
          const int64_t r = rows ? (int64_t)rows[i] : i;
          const bool a = Ac[r] != 0;
          const double v = V[r];  // (read unconditionally: one latency, not two)
          mem[t] = a && is_below[i] == side;
          hit[t] = mem[t] && (int64_t)v - G.offset == (int64_t)k;
        }
      }
#pragma unroll
      for (int t = 0; t < kCHT; ++t) {
        const uint64_t bm = __ballot(mem[t]), bh = __ballot(hit[t]);
        pre[t] = ((uint32_t)__popcll(bm & lt) << 16) | (uint32_t)__popcll(bh & lt);
        if (lane == 0) s_slot[t * kCHScan + sw] = ((uint32_t)__popcll(bm) << 16) |
                                                  (uint32_t)__popcll(bh);
      }
    }
    if (wid == 0 && it > 0) {
      const int nh = (int)(s_tot[buf ^ 1] & 0xffffu);
#ifdef TPE_DIAG_CAT_NOFOLD  // (diagnostic builds: the scan alone)
      if (nh > 0) cnt += s_w[buf ^ 1][nh - 1];
#else
      cnt = fold_list<kCHSE>(cnt, s_w[buf ^ 1], nh, folded, lane);
#endif
    }
    __syncthreads();
    if (!scan) break;
    // ---- phase 1: exclusive scan of the slots (tile-major, then wave: row
    // order) on wave 1, two slots per lane
    if (wid == 1) {
      const uint32_t c0 = 2 * lane < kCHSlots ? s_slot[2 * lane] : 0u;
      const uint32_t c1 = 2 * lane + 1 < kCHSlots ? s_slot[2 * lane + 1] : 0u;
      uint32_t incl = c0 + c1;
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, o, kWave);
        if (lane >= o) incl += y;
      }
      const uint32_t ex = incl - (c0 + c1);
      if (2 * lane < kCHSlots) s_slot[2 * lane] = ex;
      if (2 * lane + 1 < kCHSlots) s_slot[2 * lane + 1] = ex + c0;
      if (lane == kWave - 1) s_tot[buf] = incl;
    }
    __syncthreads();
    // ---- phase 2: the window's match weights into s_w[buf], in order
    if (wid > 0) {
#pragma unroll
      for (int t = 0; t < kCHT; ++t) {
        if (hit[t]) {
          const uint32_t ex = s_slot[t * kCHScan + sw] + pre[t];
          const int64_t pos = carry + (int64_t)(ex >> 16);
          double wt = 1.0;
          if (ramp && pos < num) {
            if (num == 1) wt = start;
            else if (pos == num - 1) wt = 1.0;
            else wt = __dadd_rn(__dmul_rn((double)pos, step), start);
          }
          s_w[buf][ex & 0xffffu] = wt;
        }
      }
      carry += (int64_t)(s_tot[buf] >> 16);
    }
    __syncthreads();  // (s_slot reused; s_w[buf] complete for the fold)
  }
  if (threadIdx.x == kWave) {  // (a scanner holds the observation count)
    if (carry != (int64_t)n && err) atomicOr(err, 4);
  }
  if (threadIdx.x == 0) {
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

// Long histories (n_rows >= kCathMinRows, at most kCathMaxCat categories):
// the single block per (segment, category) above walks every row itself --
// 13 windows of 7 680 rows at 100k rows, ~115 us of scanning alone (C5's
// categorical levels).  Chunked instead, the same bits:
//   k_cath_count  one block per (4096-row chunk, segment): the chunk's members
//                 and matches per category (ballots);
//   k_cath_emit   one block per (chunk, segment): every member's position in
//                 the segment (chunk base + wave base + rank in the tile) gives
//                 its LF weight, every match its place in its category's list,
//                 in row order -- the lists the single-block kernel folds;
//   k_cath_fold   one wave per (segment, category): the list folded in order
//                 (fold_list: the serial chain's bits), staged through LDS.
constexpr int kCathMinRows = 32768;
constexpr int kCathMaxCat = 32;
constexpr int kCC = 4096;                 // rows per chunk
constexpr int kCathBS = 256;              // k_cath_count / k_cath_emit block
constexpr int kCathW = kCathBS / kWave;   // waves per chunk block
constexpr int kCathRPW = kCC / kCathW;    // rows per wave (1024)
constexpr int kCathT = kCathRPW / kWave;  // tiles of 64 rows per wave (16)
constexpr int kCathStride = 1 + kCathMaxCat;  // counts per (segment, chunk): members, matches

__host__ __device__ inline int64_t cath_chunks(int64_t n_rows) { return (n_rows + kCC - 1) / kCC; }
__host__ __device__ inline int64_t cath_count_bytes(int n_seg, int64_t n_rows) {
  return ((int64_t)4 * n_seg * cath_chunks(n_rows) * kCathStride + 255) & ~(int64_t)255;
}

// row i of the walk: a member of the segment (active label, the segment's
// side of the split) and its category (-1: none of 0..n_cat-1)
__device__ __forceinline__ void cath_row(const double* __restrict__ V,
                                         const uint8_t* __restrict__ Ac,
                                         const int32_t* __restrict__ rows,
                                         const uint8_t* __restrict__ is_below, int64_t i,
                                         int64_t n_rows, uint8_t side, int64_t offset, int n_cat,
                                         bool& mem, int& cat) {
  mem = false;
  cat = -1;
  if (i < n_rows) {
    const int64_t r = rows ? (int64_t)rows[i] : i;
    const bool a = Ac[r] != 0;
    const double v = V[r];
    mem = a && is_below[i] == side;
    const int64_t cv = (int64_t)v - offset;  // (k_cat_counts_hist's test)
    if (mem && cv >= 0 && cv < (int64_t)n_cat) cat = (int)cv;
  }
}

__global__ __launch_bounds__(kCathBS) void k_cath_count(
    const double* __restrict__ vals, const uint8_t* __restrict__ active, int64_t ld,
    const int32_t* __restrict__ rows, int64_t n_rows, const uint8_t* __restrict__ is_below,
    const tpe_gather* __restrict__ gathers, const tpe_cat_seg* __restrict__ segs,
    uint32_t* __restrict__ cnt) {
  __shared__ uint32_t s_c[kCathW][kCathStride];
  const int seg = blockIdx.y, c = blockIdx.x;
  const tpe_cat_seg S = segs[seg];
  const tpe_gather G = gathers[seg];
  const double* __restrict__ V = vals + (int64_t)G.col * ld;
  const uint8_t* __restrict__ Ac = active + (int64_t)G.col * ld;
  const uint8_t side = G.below ? 1 : 0;
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const int K = S.n_cat;
  bool mem[kCathT];
  int cat[kCathT];
  const int64_t r0 = (int64_t)c * kCC + (int64_t)w * kCathRPW;
#pragma unroll
  for (int t = 0; t < kCathT; ++t)
    cath_row(V, Ac, rows, is_below, r0 + t * kWave + lane, n_rows, side, G.offset, K, mem[t],
             cat[t]);
  uint32_t nm = 0;
#pragma unroll
  for (int t = 0; t < kCathT; ++t) nm += (uint32_t)__popcll(__ballot(mem[t]));
  if (lane == 0) s_c[w][0] = nm;
  for (int k = 0; k < K; ++k) {  // (block-uniform)
    uint32_t nk = 0;
#pragma unroll
    for (int t = 0; t < kCathT; ++t) nk += (uint32_t)__popcll(__ballot(cat[t] == k));
    if (lane == 0) s_c[w][1 + k] = nk;
  }
  __syncthreads();
  uint32_t* out = cnt + ((int64_t)seg * gridDim.x + c) * kCathStride;
  for (int j = threadIdx.x; j < 1 + K; j += kCathBS) {
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < kCathW; ++q) v += s_c[q][j];
    out[j] = v;
  }
}

__global__ __launch_bounds__(kCathBS) void k_cath_emit(
    const double* __restrict__ vals, const uint8_t* __restrict__ active, int64_t ld,
    const int32_t* __restrict__ rows, int64_t n_rows, const uint8_t* __restrict__ is_below,
    const tpe_gather* __restrict__ gathers, const tpe_cat_seg* __restrict__ segs,
    const uint32_t* __restrict__ cnt, double* __restrict__ lists) {
  __shared__ uint32_t s_w[kCathW][kCathStride];   // per wave: members, matches
  __shared__ int64_t s_pre[kCathStride];          // chunks before this one
  __shared__ int64_t s_tot[kCathStride];          // the whole segment
  __shared__ int64_t s_cur[kCathW][kCathStride];  // per wave: next member position, list slots
  const int seg = blockIdx.y, c = blockIdx.x, nch = gridDim.x;
  const tpe_cat_seg S = segs[seg];
  const tpe_gather G = gathers[seg];
  const double* __restrict__ V = vals + (int64_t)G.col * ld;
  const uint8_t* __restrict__ Ac = active + (int64_t)G.col * ld;
  const uint8_t side = G.below ? 1 : 0;
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const uint64_t lt = (1ull << lane) - 1ull;
  const int K = S.n_cat;
  bool mem[kCathT];
  int cat[kCathT];
  const int64_t r0 = (int64_t)c * kCC + (int64_t)w * kCathRPW;
#pragma unroll
  for (int t = 0; t < kCathT; ++t)
    cath_row(V, Ac, rows, is_below, r0 + t * kWave + lane, n_rows, side, G.offset, K, mem[t],
             cat[t]);
  // this wave's members and matches
  uint32_t nm = 0;
#pragma unroll
  for (int t = 0; t < kCathT; ++t) nm += (uint32_t)__popcll(__ballot(mem[t]));
  if (lane == 0) s_w[w][0] = nm;
  for (int k = 0; k < K; ++k) {
    uint32_t nk = 0;
#pragma unroll
    for (int t = 0; t < kCathT; ++t) nk += (uint32_t)__popcll(__ballot(cat[t] == k));
    if (lane == 0) s_w[w][1 + k] = nk;
  }
  // the chunks before this one, and the segment's totals per category
  const uint32_t* C = cnt + (int64_t)seg * nch * kCathStride;
  for (int j = threadIdx.x; j < 1 + K; j += kCathBS) {
    int64_t pre = 0, tot = 0;
#pragma unroll 8
    for (int q = 0; q < nch; ++q) {  // (eight loads in flight)
      const int64_t v = C[(int64_t)q * kCathStride + j];
      pre += q < c ? v : 0;
      tot += v;
    }
    s_pre[j] = pre;
    s_tot[j] = tot;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // per wave: its first member position and list slots
    int64_t m = s_pre[0];
    int64_t koff[kCathMaxCat];
    int64_t acc = (int64_t)seg * n_rows;  // (segment seg's lists start at seg * n_rows)
    for (int k = 0; k < K; ++k) {
      koff[k] = acc + s_pre[1 + k];
      acc += s_tot[1 + k];
    }
    for (int q = 0; q < kCathW; ++q) {
      s_cur[q][0] = m;
      m += s_w[q][0];
      for (int k = 0; k < K; ++k) {
        s_cur[q][1 + k] = koff[k];
        koff[k] += s_w[q][1 + k];
      }
    }
  }
  __syncthreads();
  // the wave's tiles in row order: member positions -> LF weights -> list slots
  const int n = S.n_obs;
  const bool ramp = S.lf > 0 && S.lf < n;
  const int64_t num = n - S.lf;
  const double start = 1.0 / (double)n;
  const double step = (ramp && num > 1) ? (1.0 - start) / (double)(num - 1) : 0.0;
  int64_t mpos = s_cur[w][0];
#pragma unroll
  for (int t = 0; t < kCathT; ++t) {
    const uint64_t mb = __ballot(mem[t]);
    const int64_t pos = mpos + __popcll(mb & lt);
    mpos += __popcll(mb);
    int64_t slot = -1;
    for (int k = 0; k < K; ++k) {  // (block-uniform)
      const uint64_t kb = __ballot(cat[t] == k);
      if (kb == 0) continue;  // (wave-uniform)
      const int64_t base = s_cur[w][1 + k];
      if (cat[t] == k) slot = base + __popcll(kb & lt);
      if (lane == 0) s_cur[w][1 + k] = base + __popcll(kb);
      __builtin_amdgcn_wave_barrier();
    }
    if (slot >= 0) {
      double wt = 1.0;
      if (ramp && pos < num) {
        if (num == 1) wt = start;
        else if (pos == num - 1) wt = 1.0;
        else wt = __dadd_rn(__dmul_rn((double)pos, step), start);
      }
      lists[slot] = wt;
    }
  }
}

// seq_fold across a whole block (kFW waves): the same binade-grid steps, the
// parity maps and the integer increments scanned over the block (wave scans,
// then the waves' totals through LDS), so one pass covers kSE * 64 * kFW
// entries -- a long chain's ~50k weights take ~15 passes instead of ~100
// (a pass is a latency-bound chain of dependent steps, not throughput).
// Every thread returns the same S (block-uniform control).
#ifndef TPE_FOLD_WAVES  // diagnostic builds: k_cath_fold's waves and entries per lane
#define TPE_FOLD_WAVES 8
#endif
#ifndef TPE_FOLD_SE
#define TPE_FOLD_SE 8
#endif
constexpr int kFW = TPE_FOLD_WAVES;   // waves of k_cath_fold
constexpr int kFB = kFW * kWave;      // its block
constexpr int kFSE = TPE_FOLD_SE;     // entries per lane per pass
constexpr int kFoldN = kFSE * kFB;    // entries per pass / per staged chunk (4 096)
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int o) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o, kWave);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o, kWave);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}
struct FoldX {
  uint32_t wmap[kFW];        // each wave's composed parity map (inclusive)
  uint64_t wsum[kFW];        // each wave's increment total
  int64_t wcross[kFW];       // each wave's first leaving entry (-1: none) ...
  uint64_t wcum[kFW];        // ... and the increments before it
  double S;                  // (the serial prefix's result, broadcast)
};
__device__ double block_seq_fold(double S, const double* list, int n, FoldX& X) {
  constexpr int kSE = kFSE;
  const int lane = lane_id(), wid = threadIdx.x / kWave;
  double v[kSE];
#pragma unroll
  for (int j = 0; j < kSE; ++j) {
    const int i = threadIdx.x * kSE + j;
    v[j] = i < n ? list[i] : 0.0;
  }
  constexpr uint64_t kFrac = (1ull << 52) - 1, kTop = 1ull << 53;
  int r0 = 0;
  while (r0 < n) {  // (block-uniform)
    const uint64_t sb = (uint64_t)__double_as_longlong(S);
    const int es = (int)((sb >> 52) & 0x7ff);
    if (S == 0.0 || es == 0) {
      S = __dadd_rn(S, list[r0]);
      ++r0;
      continue;
    }
    const uint64_t A = (sb & kFrac) | (1ull << 52);
    uint64_t d[kSE];
    uint32_t tie = 0, huge = 0;
#pragma unroll
    for (int j = 0; j < kSE; ++j) {
      const int i = threadIdx.x * kSE + j;
      d[j] = fold_step(v[j], es, i >= r0 && i < n, tie, huge, j);
    }
    uint32_t a = 1, c = 0;
#pragma unroll
    for (int j = 0; j < kSE; ++j) {
      if ((tie >> j) & 1u) {
        a = 0;
        c = 0;
      } else {
        c ^= (uint32_t)(d[j] & 1ull);
      }
    }
    uint32_t x = a | (c << 1);
    scan_step_map<0x111, 0xF>(x);
    scan_step_map<0x112, 0xF>(x);
    scan_step_map<0x114, 0xF>(x);
    scan_step_map<0x118, 0xF>(x);
    scan_step_map<0x142, 0xA>(x);
    scan_step_map<0x143, 0xC>(x);
    const uint32_t ex = dpp_u32<0x138, 0xF>(1u, x);  // the wave's lanes before this one
    if (lane == kWave - 1) X.wmap[wid] = x;
    __syncthreads();
    // the waves before this one, composed in order: lane q < wid holds wave
    // q's map (the others the identity), an ordered scan over 16 lanes
    uint32_t pre = (lane < kFW && lane < wid) ? X.wmap[lane] : 1u;
#pragma unroll
    for (int o = 1; o < kFW; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)pre, o, kWave);
      pre = lane >= o ? map_then(y, pre) : pre;
    }
    pre = (uint32_t)__builtin_amdgcn_readlane((int)pre, kFW - 1);
    const uint32_t in = map_then(pre, ex);
    uint32_t P = ((in & 1u) & (uint32_t)(A & 1ull)) ^ (in >> 1);
    uint64_t tot = 0;
#pragma unroll
    for (int j = 0; j < kSE; ++j) {
      if ((tie >> j) & 1u) {
        d[j] += (P + d[j]) & 1ull;  // ties to the even A_{k+1}
        P = 0;
      } else {
        P ^= (uint32_t)(d[j] & 1ull);
      }
      tot += d[j];
    }
    const uint64_t incl = wave_incl_sum_u64(tot);
    if (lane == kWave - 1) X.wsum[wid] = incl;
    __syncthreads();
    // the waves' increment totals: before this wave, and all of them
    const uint64_t wsl = lane < kFW ? X.wsum[lane] : 0ull;
    uint64_t base = lane < wid ? wsl : 0ull, all = wsl;
#pragma unroll
    for (int o = 1; o < kFW; o <<= 1) {  // (lanes 0..15 reduce; lane 0's sums broadcast)
      base += shfl_xor_u64(base, o);
      all += shfl_xor_u64(all, o);
    }
    base = readlane_u64(base, 0);
    all = readlane_u64(all, 0);
    uint64_t cum = base + incl - tot;
    int jc = -1;
#pragma unroll
    for (int j = 0; j < kSE; ++j) {
      if (jc < 0) {
        if (((huge >> j) & 1u) || A + cum + d[j] >= kTop) jc = j;
        else cum += d[j];
      }
    }
    const uint64_t bal = __ballot(jc >= 0);
    if (lane == 0) {
      if (bal == 0) {
        X.wcross[wid] = -1;
      } else {
        const int L = __ffsll((unsigned long long)bal) - 1;
        X.wcross[wid] = (int64_t)(wid * kWave + L) * kSE + __builtin_amdgcn_readlane(jc, L);
        X.wcum[wid] =
            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(cum >> 32), L) << 32) |
            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cum, L);
      }
    }
    __syncthreads();
    const uint64_t cb = __ballot(lane < kFW && X.wcross[lane < kFW ? lane : 0] >= 0);
    const int qc = cb ? __ffsll((unsigned long long)cb) - 1 : -1;  // the first wave leaving
    if (qc < 0) {
      S = ldexp((double)(A + all), es - 1075);
      r0 = n;
    } else {
      const int g = (int)X.wcross[qc];
      S = __dadd_rn(ldexp((double)(A + X.wcum[qc]), es - 1075), list[g]);
      r0 = g + 1;
    }
    __syncthreads();  // (X is rewritten by the next pass)
  }
  return S;
}

__global__ __launch_bounds__(kFB) void k_cath_fold(const tpe_cat_seg* __restrict__ segs,
                                                   const uint32_t* __restrict__ cnt, int nch,
                                                   int64_t n_rows,
                                                   const double* __restrict__ lists,
                                                   double* __restrict__ p,
                                                   int32_t* __restrict__ err) {
  __shared__ double s_l[kFoldN];
  __shared__ FoldX X;
  __shared__ int64_t s_meta[3];
  const int seg = blockIdx.y, k = blockIdx.x;
  const tpe_cat_seg S = segs[seg];
  if (k >= S.n_cat) return;  // (block-uniform)
  const int lane = lane_id();
  const uint32_t* C = cnt + (int64_t)seg * nch * kCathStride;
  if (threadIdx.x < kWave) {  // this category's list: after the lists of categories < k
    int64_t before = 0, n_k = 0, members = 0;
    for (int q = lane; q < nch; q += kWave) {
      const uint32_t* Cq = C + (int64_t)q * kCathStride;
      for (int j = 0; j < k; ++j) before += Cq[1 + j];
      n_k += Cq[1 + k];
      members += Cq[0];
    }
    for (int o = 32; o >= 1; o >>= 1) {
      before += __shfl_xor(before, o, kWave);
      n_k += __shfl_xor(n_k, o, kWave);
      members += __shfl_xor(members, o, kWave);
    }
    if (lane == 0) {
      s_meta[0] = before;
      s_meta[1] = n_k;
      if (k == 0 && members != (int64_t)S.n_obs && err) atomicOr(err, 4);
    }
  }
  __syncthreads();
  const int64_t n_k = s_meta[1];
  const double* L = lists + (int64_t)seg * n_rows + s_meta[0];
  double cntv = 0.0;
  int64_t done = 0;
  for (int64_t f0 = 0; f0 < n_k; f0 += kFoldN) {
    const int m = (int)min((int64_t)kFoldN, n_k - f0);
    double t[kFSE];
#pragma unroll
    for (int u = 0; u < kFSE; ++u) {  // (all loads in flight, then the stores)
      const int i = u * kFB + (int)threadIdx.x;
      t[u] = i < m ? L[f0 + i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kFSE; ++u) {
      const int i = u * kFB + (int)threadIdx.x;
      if (i < m) s_l[i] = t[u];
    }
    __syncthreads();
    int f = 0;
    if (done < kSerialHits) {  // the chain's first entries: one thread, one add each
      f = (int)min((int64_t)m, kSerialHits - done);
      if (threadIdx.x < kWave) {
        const double sv = serial_fold(cntv, s_l, f, lane);
        if (threadIdx.x == 0) X.S = sv;
      }
      __syncthreads();
      cntv = X.S;
    }
    if (f < m) cntv = block_seq_fold(cntv, s_l + f, m - f, X);
    done += m;
    __syncthreads();  // (s_l is restaged next)
  }
  if (threadIdx.x == 0) {
    double pseudo;
    if (S.mode == 0) {
      pseudo = cntv + S.prior_weight;  // tpe.py:589
    } else {
      const double pk = p[S.prior_p_off + k];
      pseudo = cntv + (double)S.n_cat * (S.prior_weight * pk);  // tpe.py:603
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

extern "C" int64_t tpe_cat_hist_scratch_bytes(int n_seg, int max_cat, int64_t n_rows) {
  if (n_seg < 0 || max_cat < 0 || n_rows < 0) return -1;
  if (n_seg == 0 || n_rows < kCathMinRows || max_cat > kCathMaxCat) return 0;
  return cath_count_bytes(n_seg, n_rows) + (int64_t)8 * n_seg * n_rows;
}

extern "C" int tpe_cat_posterior_hist(const double* vals, const uint8_t* active, int64_t ld,
                                      const int32_t* rows, int64_t n_rows,
                                      const uint8_t* is_below, const tpe_gather* gathers,
                                      const tpe_cat_seg* segs, int n_seg, int max_cat,
                                      double* p_pool, double* logp_pool, double* cdf_pool,
                                      void* work, int64_t work_bytes, int32_t* err,
                                      void* stream) {
  if (n_seg < 0 || n_rows < 0 ||
      (n_seg > 0 && (!vals || !active || !is_below || !gathers || !segs || !p_pool ||
                     !logp_pool || !cdf_pool))) {
    set_error("tpe_cat_posterior_hist: bad arguments");
    return TPE_E_ARG;
  }
  if (n_seg == 0) return TPE_OK;
  if (n_seg > 65535 || max_cat < 0) {
    set_error("tpe_cat_posterior_hist: n_seg=%d max_cat=%d", n_seg, max_cat);
    return TPE_E_ARG;
  }
  if (work_bytes < 0) {
    set_error("tpe_cat_posterior_hist: work_bytes=%lld", (long long)work_bytes);
    return TPE_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  const int64_t need = tpe_cat_hist_scratch_bytes(n_seg, max_cat, n_rows);
  if (need > 0 && work && work_bytes >= need && max_cat >= 1) {
    // a long history: chunked (k_cath_*); the same bits as k_cat_counts_hist
    const int64_t nch = cath_chunks(n_rows);
    if (nch > INT32_MAX) {
      set_error("tpe_cat_posterior_hist: n_rows=%lld", (long long)n_rows);
      return TPE_E_UNSUPPORTED;
    }
    uint32_t* cnt = static_cast<uint32_t*>(work);
    double* lists = reinterpret_cast<double*>(static_cast<char*>(work) +
                                              cath_count_bytes(n_seg, n_rows));
    const dim3 g((unsigned)nch, n_seg);
    hipLaunchKernelGGL(k_cath_count, g, dim3(kCathBS), 0, st, vals, active, ld, rows, n_rows,
                       is_below, gathers, segs, cnt);
    hipLaunchKernelGGL(k_cath_emit, g, dim3(kCathBS), 0, st, vals, active, ld, rows, n_rows,
                       is_below, gathers, segs, cnt, lists);
    hipLaunchKernelGGL(k_cath_fold, dim3(max_cat, n_seg), dim3(kFB), 0, st, segs, cnt,
                       (int)nch, n_rows, lists, p_pool, err);
  } else {
    hipLaunchKernelGGL(k_cat_counts_hist, dim3(std::max(max_cat, 1), n_seg), dim3(kCHB), 0, st,
                       vals, active, ld, rows, n_rows, is_below, gathers, segs, p_pool, err);
  }
  hipLaunchKernelGGL(k_cat_finalize, dim3(n_seg), dim3(kCatBS), 0, st, segs, p_pool, logp_pool,
                     cdf_pool);
  return check_launch("tpe_cat_posterior_hist");
}
