// tpe_dist.hip -- the cross-GPU argmax of a suggest level over RCCL.
//
// SURVEY §8(b)'s max-loc all-reduce: every rank holds one tpe_best record per
// label of the level (an empty record -- index -1 -- for labels it did not
// score); the records are all-gathered over the caller's RCCL communicator
// (xGMI inside a node) and folded on the device by tpe_best_combine with
// np.argmax's rules (tpe.py:650-658: first maximum, NaN wins), so every rank
// ends with the same per-label winners.  This is what hyperopt_amd/dist.py
// does through torch.distributed; the entry point lets a host without torch
// (cgo / JNI / N-API bindings of this ABI) do the same with its own
// communicator.
//
// RCCL is bound at the first call by dlopen("librccl.so.1"): a process that
// already holds an RCCL (torch's bundled one, or the host's) gets that copy,
// so the communicator and the collective come from the same library; the
// shared object itself carries no link-time RCCL dependency.
#include <dlfcn.h>
#include <mutex>
#include <rccl/rccl.h>

#include "tpe_common.hpp"

extern "C" int tpe_best_combine(const tpe_best* sets, int n_sets, int n_labels, tpe_best* out,
                                void* stream);

namespace tpe {
namespace {
typedef ncclResult_t (*AllGatherFn)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                                    hipStream_t);
typedef ncclResult_t (*CommCountFn)(const ncclComm_t, int*);
typedef const char* (*ErrorStringFn)(ncclResult_t);
typedef ncclResult_t (*AsyncErrorFn)(ncclComm_t, ncclResult_t*);

struct Rccl {
  AllGatherFn all_gather = nullptr;
  CommCountFn comm_count = nullptr;
  ErrorStringFn error_string = nullptr;
  AsyncErrorFn async_error = nullptr;
  bool ok = false;
  char why[256] = "not loaded";  // the loader's error, kept (dlerror() is one-shot)
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
    if (!h) h = dlopen("librccl.so", RTLD_NOW);
    auto keep = [](const char* e, const char* dflt) {
      snprintf(r.why, sizeof(r.why), "%s", e ? e : dflt);
    };
    if (!h) {
      keep(dlerror(), "dlopen failed");
      return;
    }
    r.all_gather = reinterpret_cast<AllGatherFn>(dlsym(h, "ncclAllGather"));
    r.comm_count = reinterpret_cast<CommCountFn>(dlsym(h, "ncclCommCount"));
    r.error_string = reinterpret_cast<ErrorStringFn>(dlsym(h, "ncclGetErrorString"));
    r.async_error = reinterpret_cast<AsyncErrorFn>(dlsym(h, "ncclCommGetAsyncError"));
    r.ok = r.all_gather && r.comm_count;
    if (!r.ok) keep(dlerror(), "ncclAllGather / ncclCommCount not exported");
  });
  return r;
}

// A non-blocking communicator (torch creates them for eagerly initialised
// process groups) may answer ncclInProgress: poll its state until the call
// has been enqueued, as RCCL's non-blocking API asks.
ncclResult_t settle(const Rccl& r, ncclComm_t comm, ncclResult_t e) {
  while (e == ncclInProgress && r.async_error) {
    ncclResult_t st = ncclSuccess;
    const ncclResult_t q = r.async_error(comm, &st);
    if (q != ncclSuccess) return q;
    e = st;
  }
  return e;
}
}  // namespace
}  // namespace tpe

namespace tpe {
namespace {
// label slot s <- the records of the jobs mapped to it, folded in job order
// (a rank may hold several candidate ranges of one label); empty if none
__global__ void k_scatter_best(const tpe_best* __restrict__ by_job,
                               const int32_t* __restrict__ slot, int n_jobs,
                               tpe_best* __restrict__ out, int n_slots) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_slots) return;
  tpe_best b;
  b.score = 0.0;
  b.index = -1;
  b.value = 0.0;
  int64_t n = 0;
  bool inexact = false;  // a job whose band overflowed (n_scored -1): the label is owed
  for (int j = 0; j < n_jobs; ++j) {
    if (slot[j] != s) continue;
    const tpe_best o = by_job[j];
    n += o.n_scored;
    inexact = inexact || o.n_scored < 0;
    if (better(o.score, o.index, b.score, b.index)) b = o;
  }
  b.n_scored = inexact ? -1 : n;
  out[s] = b;
}
}  // namespace
}  // namespace tpe

using namespace tpe;

extern "C" int tpe_best_scatter(const tpe_best* by_job, const int32_t* slot, int n_jobs,
                                tpe_best* out, int n_slots, void* stream) {
  if (n_jobs < 0 || n_slots < 0 || (n_slots > 0 && !out) || (n_jobs > 0 && (!by_job || !slot))) {
    set_error("tpe_best_scatter: bad arguments (n_jobs=%d n_slots=%d)", n_jobs, n_slots);
    return TPE_E_ARG;
  }
  if (n_slots == 0) return TPE_OK;
  hipLaunchKernelGGL(k_scatter_best, dim3((n_slots + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, by_job, slot, n_jobs, out, n_slots);
  return check_launch("tpe_best_scatter");
}

extern "C" int tpe_maxloc_allreduce(const tpe_best* local, tpe_best* gathered, tpe_best* out,
                                    int n_labels, void* comm, void* stream) {
  if (n_labels < 0 || (n_labels > 0 && (!local || !gathered || !out || !comm))) {
    set_error("tpe_maxloc_allreduce: bad arguments (n_labels=%d)", n_labels);
    return TPE_E_ARG;
  }
  if (n_labels == 0) return TPE_OK;
  const Rccl& r = rccl();
  if (!r.ok) {
    set_error("tpe_maxloc_allreduce: librccl.so.1 not loadable (%s)", r.why);
    return TPE_E_UNSUPPORTED;
  }
  int world = 0;
  ncclResult_t e = settle(r, static_cast<ncclComm_t>(comm),
                          r.comm_count(static_cast<ncclComm_t>(comm), &world));
  if (e != ncclSuccess || world < 1) {
    set_error("tpe_maxloc_allreduce: ncclCommCount: %s",
              r.error_string ? r.error_string(e) : "error");
    return TPE_E_ARG;
  }
  e = settle(r, static_cast<ncclComm_t>(comm),
             r.all_gather(local, gathered, (size_t)n_labels * sizeof(tpe_best), ncclUint8,
                          static_cast<ncclComm_t>(comm), static_cast<hipStream_t>(stream)));
  if (e != ncclSuccess) {
    set_error("tpe_maxloc_allreduce: ncclAllGather: %s",
              r.error_string ? r.error_string(e) : "error");
    return TPE_E_LAUNCH;
  }
  return tpe_best_combine(gathered, world, n_labels, out, stream);
}
