// Round-trip latency of a tiny kernel + the host's wait for it, by wait
// method: hipStreamSynchronize, hipEventSynchronize, a hipEventQuery spin,
// and a spin on a pinned host word the kernel writes; with the device's
// default schedule flag or hipDeviceScheduleSpin (argument "spin").
//   hipcc -O2 --offload-arch=gfx950 -o /tmp/sync_latency tools/probes/sync_latency.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_tiny(float* p, volatile unsigned* flag, unsigned v) {
  p[threadIdx.x] += 1.0f;
  if (threadIdx.x == 0 && flag) {
    __threadfence_system();
    *flag = v;
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "spin")) (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
  if (argc > 1 && !strcmp(argv[1], "yield")) (void)hipSetDeviceFlags(hipDeviceScheduleYield);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  float* p;
  (void)hipMalloc(&p, 4096);
  unsigned* flag;
  (void)hipHostMalloc(&flag, 64, hipHostMallocCoherent);
  *flag = 0;
  hipEvent_t e;
  (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  const int N = 400;
  for (int mode = 0; mode < 4; ++mode) {
    std::vector<double> t;
    for (int i = 0; i < N; ++i) {
      const double t0 = now_us();
      const unsigned v = mode * 100000u + i + 1;
      hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, p, mode == 3 ? flag : nullptr, v);
      if (mode == 0) {
        (void)hipStreamSynchronize(s);
      } else if (mode == 1) {
        (void)hipEventRecord(e, s);
        (void)hipEventSynchronize(e);
      } else if (mode == 2) {
        (void)hipEventRecord(e, s);
        while (hipEventQuery(e) == hipErrorNotReady) {
        }
      } else {
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) {
        }
      }
      t.push_back(now_us() - t0);
    }
    if (mode == 3) (void)hipStreamSynchronize(s);
    std::sort(t.begin(), t.end());
    const char* names[] = {"hipStreamSynchronize", "hipEventSynchronize", "hipEventQuery spin",
                           "host-word spin"};
    printf("%s %-22s p10 %6.1f  p50 %6.1f  p90 %6.1f us\n", argc > 1 ? argv[1] : "default",
           names[mode], t[N / 10], t[N / 2], t[9 * N / 10]);
  }
  return 0;
}
