// tpe_prior.hip -- prior draws for the startup phase of tpe.suggest.
//
// Replaces the prior samplers rand.suggest evaluates through pyll.rec_eval
// (hyperopt/rand.py:15-27, hyperopt/pyll/stochastic.py:36-158): every label
// of a space gets n draws from its prior, draw i of label l a function of
// (label key, base + i) through Philox4x32-10 -- so a batch of new trials is
// one launch, and the host keeps only the labels each trial's choices make
// live (the conditional structure is resolved on the host).  Same formulas as
// numpy's RandomState samplers: uniform low + (high - low) u (53-bit u),
// normal mu + sigma z (Box-Muller in fp64), exp for the log kinds,
// np.round(x / q) * q (half to even) for the quantized ones, randint by
// floor(u K), categorical by inverse CDF of p.  Only the streams differ
// (Philox instead of MT19937), so parity is distributional (KS / chi^2,
// tests/test_gpu_prior.py).
#include "tpe_common.hpp"

namespace tpe {
namespace {
constexpr int kPBS = 256;
constexpr uint32_t kStreamPrior = 0x5052494Fu;  // "PRIO"

__global__ __launch_bounds__(kPBS) void k_prior_sample(const tpe_prior* __restrict__ priors,
                                                       const double* __restrict__ p,
                                                       int64_t n, int64_t base,
                                                       double* __restrict__ out) {
  const tpe_prior P = priors[blockIdx.y];
  const int64_t i = (int64_t)blockIdx.x * kPBS + threadIdx.x;
  if (i >= n) return;
  const U4 r = draw_words(P.key, base + i, 0u, kStreamPrior);
  const double u = u01_f64(r.x, r.y);  // [0, 1), 53 bits
  double v;
  switch (P.kind) {
    case TPE_PRIOR_UNIFORM:
    case TPE_PRIOR_LOGUNIFORM:
      v = P.a + (P.b - P.a) * u;
      if (P.kind == TPE_PRIOR_LOGUNIFORM) v = exp(v);
      break;
    case TPE_PRIOR_NORMAL:
    case TPE_PRIOR_LOGNORMAL:
      v = P.a + P.b * normal_f64(r.x, r.y, r.z);
      if (P.kind == TPE_PRIOR_LOGNORMAL) v = exp(v);
      break;
    case TPE_PRIOR_RANDINT: {
      const double k = floor(u * (P.b - P.a));
      v = P.a + fmin(k, P.b - P.a - 1.0);
      break;
    }
    default: {  // categorical: first k with cumsum(p)[k] > u * sum(p)
      const double* pk = p + P.p_off;
      double tot = 0.0;
      for (int k = 0; k < P.n_cat; ++k) tot += pk[k];
      const double t = u * tot;
      double c = 0.0;
      int k = 0;
      for (; k < P.n_cat - 1; ++k) {
        c += pk[k];
        if (c > t) break;
      }
      v = (double)k;
    }
  }
  if (P.q > 0.0) v = rint(v / P.q) * P.q;
  out[(int64_t)blockIdx.y * n + i] = v;
}
}  // namespace
}  // namespace tpe

using namespace tpe;

extern "C" int tpe_prior_sample(const tpe_prior* priors, const tpe_prior* host_priors,
                                int n_priors, const double* p, int64_t n, int64_t base,
                                double* out, void* stream) {
  if (n_priors < 0 || n_priors > 65535 || n < 0 || base < 0 ||
      (n_priors > 0 && !host_priors)) {
    set_error("tpe_prior_sample: bad arguments (n_priors=%d n=%lld)", n_priors, (long long)n);
    return TPE_E_ARG;
  }
  if (n_priors == 0 || n == 0) return TPE_OK;
  for (int j = 0; j < n_priors; ++j) {
    const tpe_prior& P = host_priors[j];
    if (P.kind < TPE_PRIOR_UNIFORM || P.kind > TPE_PRIOR_CATEGORICAL) {
      set_error("tpe_prior_sample: prior %d has kind %d", j, P.kind);
      return TPE_E_ARG;
    }
    if (P.kind == TPE_PRIOR_CATEGORICAL && (P.n_cat < 1 || P.p_off < 0 || !p)) {
      set_error("tpe_prior_sample: categorical prior %d without probabilities", j);
      return TPE_E_ARG;
    }
    if (P.kind == TPE_PRIOR_RANDINT && !(P.b > P.a)) {
      set_error("tpe_prior_sample: randint prior %d has high <= low", j);
      return TPE_E_ARG;
    }
  }
  if (!priors || !out) {
    set_error("tpe_prior_sample: null pointer");
    return TPE_E_ARG;
  }
  const int64_t gx = (n + kPBS - 1) / kPBS;
  if (gx > INT32_MAX) {
    set_error("tpe_prior_sample: n=%lld too large", (long long)n);
    return TPE_E_UNSUPPORTED;
  }
  hipLaunchKernelGGL(k_prior_sample, dim3((unsigned)gx, (unsigned)n_priors), dim3(kPBS), 0,
                     (hipStream_t)stream, priors, p, n, base, out);
  return check_launch("tpe_prior_sample");
}
