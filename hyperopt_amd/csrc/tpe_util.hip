// tpe_util.hip -- error reporting shared by every C-ABI entry point.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "tpe_common.hpp"

namespace tpe {
namespace {
thread_local char g_err[512] = "";
thread_local int g_defer_check = 0;  // > 0 inside tpe_run_ops (see defer_launch_checks)
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// Inside a batch of records (tpe_run_ops) the launch status is read once at
// the end of the batch instead of after every entry point: hipGetLastError
// costs a few us of host time per call.
void defer_launch_checks(bool on) { g_defer_check += on ? 1 : -1; }

int check_launch(const char* what) {
  if (g_defer_check > 0) return TPE_OK;
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return TPE_E_LAUNCH;
  }
  return TPE_OK;
}
}  // namespace tpe

extern "C" const char* tpe_last_error(void) { return tpe::g_err; }
extern "C" int tpe_abi_version(void) { return TPE_ABI_VERSION; }

// sizes of the ABI structs, so bindings can check their mirrors
extern "C" int tpe_struct_sizes(int32_t* out, int n) {
  const int32_t s[11] = {(int32_t)sizeof(tpe_seg),     (int32_t)sizeof(tpe_cat_seg),
                         (int32_t)sizeof(tpe_job),     (int32_t)sizeof(tpe_best),
                         (int32_t)sizeof(tpe_table),   (int32_t)sizeof(tpe_gather),
                         (int32_t)sizeof(tpe_history), (int32_t)sizeof(tpe_prior),
                         (int32_t)sizeof(tpe_op),      (int32_t)sizeof(tpe_band),
                         (int32_t)sizeof(tpe_colspec)};
  for (int i = 0; i < n && i < 11; ++i) out[i] = s[i];
  return 11;
}

// ---- host: the below split's rows (ap_split_trials, tpe.py:623-646) -------
// The rows of argsort(losses, kind="stable")[:k] -- the k smallest losses,
// NaN after +inf, ties to the earlier row -- in ascending row order, in one
// pass over the losses keeping the k best (value, row) pairs sorted (k is
// n_below <= 25 on the suggest path, so a loss enters the kept set ~k ln(T/k)
// times).  Returns the number written (min(k, n)), or -1 on bad arguments.
namespace {
inline bool loss_before(double a, int64_t ia, double b, int64_t ib) {
  const bool na = a != a, nb = b != b;
  if (na || nb) return na ? (nb && ia < ib) : true;  // NaN sorts last
  return a < b || (a == b && ia < ib);
}
}  // namespace

extern "C" int64_t tpe_smallest_rows(const double* losses, int64_t n, int64_t k, int64_t* out) {
  if (n < 0 || k < 0 || (n > 0 && !losses) || (k > 0 && !out)) return -1;
  if (k > n) k = n;
  if (k == 0) return 0;
  if (k > 4096) {  // not the suggest path's shape: full stable order
    std::vector<int64_t> idx((size_t)n);
    for (int64_t i = 0; i < n; ++i) idx[(size_t)i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
      return loss_before(losses[a], a, losses[b], b);
    });
    std::sort(idx.begin(), idx.begin() + k);
    std::copy(idx.begin(), idx.begin() + k, out);
    return k;
  }
  std::vector<double> kv((size_t)k);
  std::vector<int64_t> ki((size_t)k);
  int64_t m = 0;  // kept pairs, ascending
  auto insert = [&](double v, int64_t i) {  // (v, i) beats the kept worst, or the set is not full
    int64_t p = m < k ? m++ : k - 1;  // slot freed at the end, then shifted into place
    while (p > 0 && loss_before(v, i, kv[(size_t)(p - 1)], ki[(size_t)(p - 1)])) {
      kv[(size_t)p] = kv[(size_t)(p - 1)];
      ki[(size_t)p] = ki[(size_t)(p - 1)];
      --p;
    }
    kv[(size_t)p] = v;
    ki[(size_t)p] = i;
  };
  constexpr int64_t kChunk = 64;
  int64_t i = 0;
  while (i < n) {
    const double worst = m == k ? kv[(size_t)(k - 1)] : NAN;
    if (!(worst == worst)) {  // filling, or NaN kept: the general rule, one loss
      const double v = losses[i];
      if (m < k || loss_before(v, i, worst, ki[(size_t)(k - 1)])) insert(v, i);
      ++i;
      continue;
    }
    // the kept worst is a number and every kept row precedes this chunk: a
    // loss beats it iff it is smaller (equal ones come later, NaN never
    // does) -- one vectorisable test per chunk, then only its hits
    const int64_t end = std::min(n, i + kChunk);
    bool any = false;
    for (int64_t j = i; j < end; ++j) any |= losses[j] < worst;
    if (any) {
      double w = worst;
      for (int64_t j = i; j < end; ++j) {
        if (losses[j] < w) {
          insert(losses[j], j);
          w = kv[(size_t)(k - 1)];
        }
      }
    }
    i = end;
  }
  std::sort(ki.begin(), ki.end());
  std::copy(ki.begin(), ki.end(), out);
  return k;
}

// ---- host: the split and the level inputs of one history in one pass -----
// The below rows (tpe_smallest_rows), a 0/1 flag per row, and per label the
// below set's size nb[j] (active below rows) and the above set's size
// na[j] = n_active[j] - nb[j] (every row is below or above: no from_tid
// aliasing) -- what tpe.suggest's split_masks + LevelInputs compute with a
// dozen numpy calls.  active: T x L bytes, row-major.  Returns the number of
// below rows, or -1 on bad arguments.
extern "C" int64_t tpe_split_inputs(const double* losses, int64_t T, int64_t n_below,
                                    const uint8_t* active, int64_t L, const int64_t* n_active,
                                    uint8_t* isb, int64_t* below_rows, int64_t* nb, int64_t* na) {
  if (T < 0 || L < 0 || n_below < 0 || (T > 0 && (!losses || !isb)) ||
      (L > 0 && (!nb || !na || !n_active || (T > 0 && !active))) || (n_below > 0 && !below_rows))
    return -1;
  const int64_t k = tpe_smallest_rows(losses, T, n_below, below_rows);
  if (k < 0) return -1;
  memset(isb, 0, (size_t)T);
  for (int64_t j = 0; j < L; ++j) nb[j] = 0;
  for (int64_t i = 0; i < k; ++i) {
    const int64_t r = below_rows[i];
    isb[r] = 1;
    const uint8_t* a = active + r * L;
    for (int64_t j = 0; j < L; ++j) nb[j] += a[j] != 0;
  }
  for (int64_t j = 0; j < L; ++j) na[j] = n_active[j] - nb[j];
  return k;
}

// ---------------------------------------------------------------------------
// The hardware transcendentals the fp32 error bounds lean on,
// measured exhaustively: v_exp_f32 (the build's terms, mix_eps' 2^-22) over
// every fp32 x in [-126, 12] (results >= 2^-126: no subnormal outputs), as the
// relative error against exp2 in fp64; v_log_f32 (the two-polynomial
// fallback's kEtaLog2 = 2^-22) over every positive normal fp32 p, as
// |log2f(p) - log2(p)| / max(1, |log2 p|).  Device-side fp64 references (each
// within 1 fp64 ulp).  out[0], out[1]: the two maxima (device, 2 doubles).
// ---------------------------------------------------------------------------
namespace tpe {
namespace {
__global__ __launch_bounds__(256) void k_ulp_check(unsigned long long* out) {
  double ee = 0.0, el = 0.0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32);
       i += stride) {
    const float x = __uint_as_float((uint32_t)i);
    if (x >= -126.0f && x <= 12.0f) {
      const double r = exp2((double)x);
      const double g = (double)__builtin_amdgcn_exp2f(x);
      ee = fmax(ee, fabs(g - r) / r);
    }
    if (x > 0.0f && x >= 0x1.0p-126f && isfinite(x)) {
      const double r = log2((double)x);
      const double g = (double)__builtin_amdgcn_logf(x);
      el = fmax(el, fabs(g - r) / fmax(1.0, fabs(r)));
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    ee = fmax(ee, __shfl_xor(ee, o, 64));
    el = fmax(el, __shfl_xor(el, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {  // non-negative doubles order as their bits
    atomicMax(out, (unsigned long long)__double_as_longlong(ee));
    atomicMax(out + 1, (unsigned long long)__double_as_longlong(el));
  }
}
}  // namespace
}  // namespace tpe

extern "C" int tpe_check_transcendentals(double* out, void* stream) {
  if (!out) {
    tpe::set_error("tpe_check_transcendentals: null pointer");
    return TPE_E_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(out, 0, 2 * sizeof(double), st) != hipSuccess) {
    tpe::set_error("tpe_check_transcendentals: hipMemsetAsync failed");
    return TPE_E_LAUNCH;
  }
  hipLaunchKernelGGL(tpe::k_ulp_check, dim3(8192), dim3(256), 0, st,
                     reinterpret_cast<unsigned long long*>(out));
  return tpe::check_launch("tpe_check_transcendentals");
}
