// tpe_ops.hip -- the level launcher (tpe_run_ops, include/tpe_hip.h).
//
// A suggest level is ~20 stream operations (history gather, Parzen fit,
// categorical posteriors, table build, scoring launches, side-stream
// fork/join, upload and readback).  Issued one ctypes call at a time they
// cost ~8 us of host time each -- at a one-eighth label share on 8 GPUs that
// host time, not the GPU, sets the level's length.
// Here the binding hands over the whole level as an array of records and the
// calls are made from C++: each record names an entry point of this library
// and carries its arguments as 64-bit words, converted back to the entry
// point's parameter types by the call adapter below (the prototypes in
// tpe_hip.h drive the conversion, so a record can only call a function with
// exactly its declared arity).
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <type_traits>
#include <utility>

#include <unistd.h>

#include "tpe_common.hpp"

namespace tpe {
namespace {

// one argument word, convertible to any pointer or integer parameter type
struct Word {
  int64_t v;
  template <class T>
  operator T*() const {
    return reinterpret_cast<T*>(static_cast<intptr_t>(v));
  }
  template <class T, class = std::enable_if_t<std::is_integral<T>::value>>
  operator T() const {
    return static_cast<T>(v);
  }
};

template <class R, class... Ps, size_t... I>
R invoke(R (*f)(Ps...), const int64_t* a, std::index_sequence<I...>) {
  return f(Word{a[I]}...);
}

// calls f with the record's words; TPE_E_ARG when the record's arity differs
template <class R, class... Ps>
int call(R (*f)(Ps...), const tpe_op& op, const char* name) {
  if (op.n_args != (int)sizeof...(Ps)) {
    set_error("tpe_run_ops: %s takes %d arguments, record has %d", name, (int)sizeof...(Ps),
              op.n_args);
    return TPE_E_ARG;
  }
  return (int)invoke(f, op.a, std::index_sequence_for<Ps...>{});
}

void* ptr(int64_t v) { return reinterpret_cast<void*>(static_cast<intptr_t>(v)); }

int runtime(hipError_t e, const char* what) {
  if (e == hipSuccess) return TPE_OK;
  set_error("tpe_run_ops: %s: %s", what, hipGetErrorString(e));
  return TPE_E_LAUNCH;
}

int run_one(const tpe_op& op) {
#define TPE_CALL(CODE, FN) \
  case CODE:               \
    return call(&FN, op, #FN)
  switch (op.code) {
    TPE_CALL(TPE_OP_GATHER_OBS, tpe_gather_obs);
    TPE_CALL(TPE_OP_GATHER_OBS_MULTI, tpe_gather_obs_multi);
    TPE_CALL(TPE_OP_PARZEN_FIT, tpe_parzen_fit);
    TPE_CALL(TPE_OP_CAT_POSTERIOR, tpe_cat_posterior);
    TPE_CALL(TPE_OP_TABLE_BUILD, tpe_table_build);
    TPE_CALL(TPE_OP_SCORE_TABLE, tpe_score_table);
    TPE_CALL(TPE_OP_SCORE_TABLE_FAST, tpe_score_table_fast);
    TPE_CALL(TPE_OP_SCORE_PRUNED64, tpe_score_pruned64);
    TPE_CALL(TPE_OP_SCORE_CONTINUOUS, tpe_score_continuous);
    TPE_CALL(TPE_OP_SORT_CANDIDATES, tpe_sort_candidates);
    TPE_CALL(TPE_OP_SCORE_SORTED, tpe_score_sorted);
    TPE_CALL(TPE_OP_LATTICE_SAMPLE, tpe_lattice_sample);
    TPE_CALL(TPE_OP_LATTICE_COMPACT, tpe_lattice_compact);
    TPE_CALL(TPE_OP_SCORE_QUANTIZED, tpe_score_quantized);
    TPE_CALL(TPE_OP_SCORE_CATEGORICAL, tpe_score_categorical);
    TPE_CALL(TPE_OP_SAMPLE, tpe_sample);
    TPE_CALL(TPE_OP_BEST_SCATTER, tpe_best_scatter);
    TPE_CALL(TPE_OP_MAXLOC_ALLREDUCE, tpe_maxloc_allreduce);
    TPE_CALL(TPE_OP_LATTICE_SUGGEST, tpe_lattice_suggest);
    TPE_CALL(TPE_OP_BAND_RESCORE, tpe_band_rescore);
    TPE_CALL(TPE_OP_FIT_SORTED, tpe_fit_sorted);
    TPE_CALL(TPE_OP_HISTORY_ORDER, tpe_history_order);
    TPE_CALL(TPE_OP_CATEGORICAL_SUGGEST, tpe_categorical_suggest);
    TPE_CALL(TPE_OP_CAT_POSTERIOR_HIST, tpe_cat_posterior_hist);
#undef TPE_CALL
    case TPE_OP_EVENT_RECORD:
      return runtime(hipEventRecord((hipEvent_t)ptr(op.a[0]),
                                    (hipStream_t)ptr(op.a[1])),
                     "hipEventRecord");
    case TPE_OP_STREAM_WAIT:
      return runtime(hipStreamWaitEvent((hipStream_t)ptr(op.a[0]),
                                        (hipEvent_t)ptr(op.a[1]), 0),
                     "hipStreamWaitEvent");
    case TPE_OP_MEMCPY:
      if (op.a[3] != hipMemcpyHostToDevice && op.a[3] != hipMemcpyDeviceToHost &&
          op.a[3] != hipMemcpyDeviceToDevice) {
        set_error("tpe_run_ops: memcpy kind %lld", (long long)op.a[3]);
        return TPE_E_ARG;
      }
      return runtime(hipMemcpyAsync(ptr(op.a[0]),
                                    ptr(op.a[1]), (size_t)op.a[2],
                                    (hipMemcpyKind)op.a[3],
                                    (hipStream_t)ptr(op.a[4])),
                     "hipMemcpyAsync");
    case TPE_OP_STREAM_SYNC:
      return runtime(hipStreamSynchronize((hipStream_t)ptr(op.a[0])),
                     "hipStreamSynchronize");
    default:
      set_error("tpe_run_ops: unknown op code %d", op.code);
      return TPE_E_ARG;
  }
}

}  // namespace
}  // namespace tpe

namespace tpe {
namespace {

// ---- two issuing threads ---------------------------------------------------
// A level's records go to two streams: the main chain (fit, table, scorer,
// band) and the side stream (categorical and lattice groups), joined by event
// records.  Each launch costs the issuing thread ~4 us inside the runtime, and
// at a small label share the host's ~25 launches, not the GPU, set the
// level's length: the GPU's main stream idles while the
// host issues the side group.  With two issuing threads the caller issues the
// main stream's records and a resident worker the other streams' records,
// each in list order; event records (hipEventRecord / hipStreamWaitEvent) are
// issued in their global list order -- a thread about to issue the k-th event
// record waits until the first k-1 are issued -- so every wait sees the same
// record as in one-thread issue, and the GPU's work and dependencies are the
// ones the single thread would have queued.
bool is_event_op(int32_t c) { return c == TPE_OP_EVENT_RECORD || c == TPE_OP_STREAM_WAIT; }

// the argument word of `op` that names its stream (every entry point's last
// parameter; the runtime records' stream operand), or -1
int stream_word(const tpe_op& op) {
  switch (op.code) {
    case TPE_OP_EVENT_RECORD: return 1;
    case TPE_OP_STREAM_WAIT: return 0;
    case TPE_OP_MEMCPY: return 4;
    case TPE_OP_STREAM_SYNC: return 0;
    default: return op.n_args > 0 ? op.n_args - 1 : -1;
  }
}

inline void cpu_relax() { __builtin_ia32_pause(); }

struct Batch {
  const tpe_op* ops = nullptr;
  int n = 0;
  double* t_us = nullptr;           // TPE_OPS_TRACE: each record's issue end (us from t0)
  std::chrono::steady_clock::time_point t0;
  int64_t main = 0;                 // the caller thread's stream word
  std::atomic<int> ev_done{0};      // event records issued so far (list order)
  std::atomic<int> abort{0};        // a thread failed: the other stops at its next event record
};

// the caller's part (main = true: records on the main stream, and records
// without a stream) or the worker's (every other record), in list order
int issue_part(Batch& b, bool main, int* failed) {
  int ev = 0;
  for (int i = 0; i < b.n; ++i) {
    const tpe_op& op = b.ops[i];
    const int w = stream_word(op);
    const bool mine = (w < 0 || op.a[w] == b.main) == main;
    const bool evop = is_event_op(op.code);
    if (!mine) {
      ev += evop;
      continue;
    }
    if (evop)
      while (b.ev_done.load(std::memory_order_acquire) != ev) {
        if (b.abort.load(std::memory_order_acquire)) return TPE_OK;  // the other's failure is reported
        cpu_relax();
      }
    const int rc = run_one(op);
    if (evop) b.ev_done.store(++ev, std::memory_order_release);
    if (b.t_us)
      b.t_us[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - b.t0)
                      .count();
    if (rc != TPE_OK) {
      *failed = i;
      b.abort.store(1, std::memory_order_release);
      return rc;
    }
  }
  const hipError_t e = hipGetLastError();  // this thread's launches
  if (e != hipSuccess) {
    set_error("tpe_run_ops: a launch of the batch failed: %s", hipGetErrorString(e));
    *failed = b.n;
    b.abort.store(1, std::memory_order_release);
    return TPE_E_LAUNCH;
  }
  return TPE_OK;
}

// the resident worker: spins for kSpinUs after each batch (levels follow each
// other closely), then sleeps on a condition variable; never destroyed (a
// detached thread, so process exit does not wait for it)
class Worker {
 public:
  static Worker* get() {
    // (a forked child has no worker thread: it starts its own)
    static std::atomic<Worker*> w{nullptr};
    static std::atomic<pid_t> owner{0};
    static std::mutex make;
    const pid_t me = getpid();
    Worker* cur = w.load(std::memory_order_acquire);
    if (cur && owner.load(std::memory_order_acquire) == me) return cur;
    std::lock_guard<std::mutex> g(make);
    cur = w.load(std::memory_order_acquire);
    if (!cur || owner.load(std::memory_order_acquire) != me) {
      cur = new Worker();
      w.store(cur, std::memory_order_release);
      owner.store(me, std::memory_order_release);
    }
    return cur;
  }
  std::mutex use;  // one batch at a time (a second caller issues alone)

  void post(Batch* b, int device) {
    device_ = device;
    rc_ = TPE_OK;
    failed_ = -1;
    err_[0] = 0;
    {
      std::lock_guard<std::mutex> g(m_);
      job_.store(b, std::memory_order_release);
    }
    if (sleeping_.load(std::memory_order_acquire)) cv_.notify_one();
  }
  // waits for the posted batch; its status, failing record and message
  int wait(int* failed, char* err, size_t n) {
    while (job_.load(std::memory_order_acquire) != nullptr) cpu_relax();
    *failed = failed_;
    strncpy(err, err_, n - 1);
    err[n - 1] = 0;
    return rc_;
  }

 private:
  static constexpr double kSpinUs = 2000.0;
  Worker() { std::thread([this] { loop(); }).detach(); }
  void loop() {
    int dev = -1;
    for (;;) {
      Batch* b = job_.load(std::memory_order_acquire);
      if (!b) {
        const auto t0 = std::chrono::steady_clock::now();
        while (!(b = job_.load(std::memory_order_acquire)) &&
               std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                       .count() < kSpinUs)
          for (int k = 0; k < 64; ++k) cpu_relax();
        if (!b) {
          std::unique_lock<std::mutex> g(m_);
          sleeping_.store(true, std::memory_order_release);
          cv_.wait(g, [&] { return (b = job_.load(std::memory_order_acquire)) != nullptr; });
          sleeping_.store(false, std::memory_order_release);
        }
      }
      if (device_ != dev) {
        (void)hipSetDevice(device_);
        dev = device_;
      }
      defer_launch_checks(true);
      int failed = -1;
      const int rc = issue_part(*b, false, &failed);
      defer_launch_checks(false);
      if (rc != TPE_OK) {
        strncpy(err_, tpe_last_error(), sizeof(err_) - 1);
        err_[sizeof(err_) - 1] = 0;
      }
      rc_ = rc;
      failed_ = failed;
      job_.store(nullptr, std::memory_order_release);
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::atomic<Batch*> job_{nullptr};
  std::atomic<bool> sleeping_{false};
  int device_ = 0, rc_ = TPE_OK, failed_ = -1;
  char err_[512] = "";
};

std::atomic<int> g_issue_threads{1};

}  // namespace
}  // namespace tpe

extern "C" int tpe_set_issue_threads(int n) {
  if (n != 1 && n != 2) {
    tpe::set_error("tpe_set_issue_threads: n=%d (1 or 2)", n);
    return TPE_E_ARG;
  }
  return tpe::g_issue_threads.exchange(n);
}

extern "C" int tpe_run_ops(const tpe_op* ops, int n_ops, int* failed_op) {
  if (failed_op) *failed_op = -1;
  if (n_ops < 0 || (n_ops > 0 && !ops)) {
    tpe::set_error("tpe_run_ops: n_ops=%d", n_ops);
    return TPE_E_ARG;
  }
  // TPE_OPS_TRACE=1 (diagnostic): host time of every record on stderr
  static const bool trace = getenv("TPE_OPS_TRACE") && getenv("TPE_OPS_TRACE")[0] == '1';
  // launch status read once for the whole batch (check_launch), not per record
  struct Defer {
    Defer() { tpe::defer_launch_checks(true); }
    ~Defer() { tpe::defer_launch_checks(false); }
  } defer;
  // two issuing threads when the records use more than one stream
  int64_t main = 0;
  bool have_main = false, multi = false;
  if (tpe::g_issue_threads.load(std::memory_order_relaxed) == 2) {
    for (int i = 0; i < n_ops && !multi; ++i) {
      const int w = tpe::stream_word(ops[i]);
      if (w < 0) continue;
      if (!have_main) {
        main = ops[i].a[w];
        have_main = true;
      } else if (ops[i].a[w] != main) {
        multi = true;
      }
    }
  }
  if (multi) {
    tpe::Worker* wk = tpe::Worker::get();
    std::unique_lock<std::mutex> g(wk->use, std::try_to_lock);
    int dev = 0;
    if (g.owns_lock() && hipGetDevice(&dev) == hipSuccess) {
      tpe::Batch b;
      b.ops = ops;
      b.n = n_ops;
      b.main = main;
      double* t_us = nullptr;
      if (trace) {
        t_us = new double[n_ops];
        for (int i = 0; i < n_ops; ++i) t_us[i] = -1.0;
        b.t_us = t_us;
      }
      b.t0 = std::chrono::steady_clock::now();
      wk->post(&b, dev);
      int f_main = -1, f_side = -1;
      const int rc_main = tpe::issue_part(b, true, &f_main);
      char err[512];
      const int rc_side = wk->wait(&f_side, err, sizeof(err));
      if (t_us) {
        for (int i = 0; i < n_ops; ++i) {
          const int w = tpe::stream_word(ops[i]);
          fprintf(stderr, "op %2d code %2d %s issued at %7.2f us\n", i, ops[i].code,
                  (w < 0 || ops[i].a[w] == main) ? "caller" : "worker", t_us[i]);
        }
        delete[] t_us;
      }
      // the first failing record in list order is reported
      const bool side_first = rc_side != TPE_OK && (rc_main == TPE_OK || f_side < f_main);
      if (side_first) {
        tpe::set_error("%s", err);
        if (failed_op) *failed_op = f_side < n_ops ? f_side : -1;
        return rc_side;
      }
      if (rc_main != TPE_OK && failed_op) *failed_op = f_main < n_ops ? f_main : -1;
      return rc_main;
    }
  }
  auto t_prev = std::chrono::steady_clock::now();
  for (int i = 0; i < n_ops; ++i) {
    const int rc = tpe::run_one(ops[i]);
    if (trace) {
      const auto t = std::chrono::steady_clock::now();
      fprintf(stderr, "op %2d code %2d %7.2f us\n", i, ops[i].code,
              std::chrono::duration<double, std::micro>(t - t_prev).count());
      t_prev = t;
    }
    if (rc != TPE_OK) {
      if (failed_op) *failed_op = i;
      return rc;
    }
  }
  if (n_ops > 0) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      tpe::set_error("tpe_run_ops: a launch of the batch failed: %s", hipGetErrorString(e));
      return TPE_E_LAUNCH;
    }
  }
  return TPE_OK;
}

// ---- the level as a hipGraph ------------------------
// A level re-issued with exactly the same records (bench.py's steps, any
// suggest whose sizes repeat) is captured once -- its records issued into a
// stream capture of `stream`, the level's main stream; side-stream forks
// join back through the records' own events; work the records put on
// `from_stream` goes to `capture_stream`, since the caller's stream may be the
// null stream -- and replayed with one hipGraphLaunch on the caller's stream: the host no longer pays ~4 us per kernel launch, and the
// GPU no longer waits between kernels for the host to issue the next one.
extern "C" int tpe_ops_capture(const tpe_op* ops, int n_ops, void* from_stream,
                               void* capture_stream, void** graph_exec, int* failed_op) {
  if (failed_op) *failed_op = -1;
  if (!graph_exec || n_ops <= 0 || !ops || !capture_stream) {
    tpe::set_error("tpe_ops_capture: n_ops=%d, null argument", n_ops);
    return TPE_E_ARG;
  }
  *graph_exec = nullptr;
  hipStream_t st = (hipStream_t)capture_stream;
  hipError_t e = hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed);
  if (e != hipSuccess) return tpe::runtime(e, "hipStreamBeginCapture");
  int rc = TPE_OK;
  {
    struct Defer {
      Defer() { tpe::defer_launch_checks(true); }
      ~Defer() { tpe::defer_launch_checks(false); }
    } defer;
    for (int i = 0; i < n_ops && rc == TPE_OK; ++i) {
      const int32_t c = ops[i].code;
      if (c == TPE_OP_STREAM_SYNC || c == TPE_OP_MAXLOC_ALLREDUCE) {
        tpe::set_error("tpe_ops_capture: record %d (code %d) cannot be captured", i, c);
        rc = TPE_E_ARG;
      } else {
        // the records' main stream (possibly the null stream, which cannot
        // be captured) is issued into the capture stream instead
        tpe_op op = ops[i];
        const int w = tpe::stream_word(op);
        if (w >= 0 && op.a[w] == (int64_t)(intptr_t)from_stream)
          op.a[w] = (int64_t)(intptr_t)capture_stream;
        rc = tpe::run_one(op);
      }
      if (rc != TPE_OK && failed_op) *failed_op = i;
    }
  }
  hipGraph_t g = nullptr;
  e = hipStreamEndCapture(st, &g);  // always: the stream leaves capture mode
  (void)hipGetLastError();
  if (rc == TPE_OK && e != hipSuccess) rc = tpe::runtime(e, "hipStreamEndCapture");
  if (rc == TPE_OK) {
    hipGraphExec_t x = nullptr;
    e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    if (e != hipSuccess) {
      rc = tpe::runtime(e, "hipGraphInstantiate");
    } else {
      *graph_exec = (void*)x;
    }
  }
  if (g) (void)hipGraphDestroy(g);
  return rc;
}

extern "C" int tpe_graph_launch(void* graph_exec, void* stream) {
  if (!graph_exec) {
    tpe::set_error("tpe_graph_launch: null graph");
    return TPE_E_ARG;
  }
  return tpe::runtime(hipGraphLaunch((hipGraphExec_t)graph_exec, (hipStream_t)stream),
                      "hipGraphLaunch");
}

extern "C" int tpe_graph_destroy(void* graph_exec) {
  if (!graph_exec) return TPE_OK;
  return tpe::runtime(hipGraphExecDestroy((hipGraphExec_t)graph_exec), "hipGraphExecDestroy");
}
