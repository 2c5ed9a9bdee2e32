// tpe_util.hip -- error reporting shared by every C-ABI entry point.
#include <stdarg.h>
#include <stdio.h>

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
  constexpr int64_t kChunk = 64;
  for (int64_t i = 0; i < n; ++i) {
    const double v = losses[i];
    if (m == k) {
      const double worst = kv[(size_t)(k - 1)];
      if (worst == worst && (i % kChunk) == 0 && i + kChunk <= n) {
        // a chunk without a loss below the kept worst changes nothing (equal
        // losses come later than the kept one, NaN never beats a number):
        // one vectorisable test per chunk
        bool any = false;
        for (int64_t j = i; j < i + kChunk; ++j) any |= losses[j] < worst;
        if (!any) {
          i += kChunk - 1;
          continue;
        }
      }
      if (!loss_before(v, i, worst, ki[(size_t)(k - 1)])) continue;
    }
    int64_t p = m < k ? m++ : k - 1;  // slot freed at the end, then shifted into place
    while (p > 0 && loss_before(v, i, kv[(size_t)(p - 1)], ki[(size_t)(p - 1)])) {
      kv[(size_t)p] = kv[(size_t)(p - 1)];
      ki[(size_t)p] = ki[(size_t)(p - 1)];
      --p;
    }
    kv[(size_t)p] = v;
    ki[(size_t)p] = i;
  }
  std::sort(ki.begin(), ki.end());
  std::copy(ki.begin(), ki.end(), out);
  return k;
}
