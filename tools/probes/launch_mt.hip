// Host cost of kernel launches issued from one thread vs two threads on two
// streams (is hipLaunchKernel serialised across streams?).  Build and run:
//   hipcc -O2 --offload-arch=gfx950 -o /tmp/launch_mt tools/probes/launch_mt.hip -lpthread && /tmp/launch_mt
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>

__global__ void k_small(float* p, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 1.0001f + 1.0f;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void issue(hipStream_t s, float* p, int n, int k) {
  for (int i = 0; i < k; ++i) hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, s, p, n);
}

int main() {
  hipStream_t a, b;
  hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
  float *pa, *pb;
  const int n = 64 * 256;
  hipMalloc(&pa, n * 4);
  hipMalloc(&pb, n * 4);
  const int K = 25;
  for (int rep = 0; rep < 3; ++rep) {
    // warm
    issue(a, pa, n, 100); issue(b, pb, n, 100);
    hipDeviceSynchronize();
    for (int mode = 0; mode < 3; ++mode) {
      double best = 1e30;
      for (int it = 0; it < 50; ++it) {
        hipDeviceSynchronize();
        double t0 = now_us();
        if (mode == 0) {  // one thread, both streams
          issue(a, pa, n, K); issue(b, pb, n, K);
        } else if (mode == 1) {  // two threads (fresh thread per batch)
          std::thread th([&] { issue(b, pb, n, K); });
          issue(a, pa, n, K);
          th.join();
        } else {  // one thread, one stream, K launches only
          issue(a, pa, n, K);
        }
        double t1 = now_us();
        best = t1 - t0 < best ? t1 - t0 : best;
      }
      printf("rep %d mode %s: %.1f us for %d launches\n", rep,
             mode == 0 ? "1 thread 2x25" : (mode == 1 ? "2 threads 2x25" : "1 thread 1x25"), best,
             mode == 2 ? K : 2 * K);
    }
  }
  // persistent spinning worker
  std::atomic<int> go{0}, done{0};
  std::atomic<bool> stop{false};
  std::thread w([&] {
    hipSetDevice(0);
    int seen = 0;
    while (!stop.load()) {
      int g = go.load(std::memory_order_acquire);
      if (g != seen) { issue(b, pb, n, K); seen = g; done.store(g, std::memory_order_release); }
      else __builtin_ia32_pause();
    }
  });
  for (int rep = 0; rep < 3; ++rep) {
    double best = 1e30;
    for (int it = 1; it <= 50; ++it) {
      hipDeviceSynchronize();
      double t0 = now_us();
      int g = rep * 1000 + it;
      go.store(g, std::memory_order_release);
      issue(a, pa, n, K);
      while (done.load(std::memory_order_acquire) != g) __builtin_ia32_pause();
      double t1 = now_us();
      best = t1 - t0 < best ? t1 - t0 : best;
    }
    printf("rep %d mode spinning worker 2x25: %.1f us\n", rep, best);
  }
  stop.store(true);
  w.join();
  return 0;
}
