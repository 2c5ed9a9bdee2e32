// Microbenchmark (diagnostic): chip-wide throughput of Philox4x32-10 on
// gfx950 in three spellings -- 64-bit products (v_mad_u64_u32), separate
// mul_hi / mul_lo, and 7 rounds for reference -- plus the fp32 Box-Muller
// pair, as Philox calls (or pairs) per ns.  Independent chains per lane.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 1024
struct U4 { uint32_t x, y, z, w; };

template <int ROUNDS>
__device__ __forceinline__ U4 philox_mad64(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1,
           (uint32_t)p0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
__device__ __forceinline__ U4 philox_hilo(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
// Threefry-4x32 (Random123 rotation constants), ROUNDS rounds, key injection
// every 4 rounds: only adds, rotates (v_alignbit) and xors
template <int ROUNDS>
__device__ __forceinline__ U4 threefry(U4 c, uint32_t k0, uint32_t k1) {
  constexpr int R0[8] = {10, 11, 13, 23, 6, 17, 25, 18};
  constexpr int R1[8] = {26, 21, 27, 5, 20, 11, 10, 20};
  const uint32_t k2 = 0, k3 = 0, k4 = 0x1BD11BDAu ^ k0 ^ k1;
  const uint32_t ks[5] = {k0, k1, k2, k3, k4};
  uint32_t x0 = c.x + k0, x1 = c.y + k1, x2 = c.z + k2, x3 = c.w + k3;
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    if ((r & 1) == 0) {
      x0 += x1; x1 = rotl(x1, R0[r & 7]); x1 ^= x0;
      x2 += x3; x3 = rotl(x3, R1[r & 7]); x3 ^= x2;
    } else {
      x0 += x3; x3 = rotl(x3, R0[r & 7]); x3 ^= x0;
      x2 += x1; x1 = rotl(x1, R1[r & 7]); x1 ^= x2;
    }
    if ((r & 3) == 3) {
      const int s = (r + 1) / 4;
      x0 += ks[s % 5]; x1 += ks[(s + 1) % 5]; x2 += ks[(s + 2) % 5];
      x3 += ks[(s + 3) % 5] + (uint32_t)s;
    }
  }
  return U4{x0, x1, x2, x3};
}

template <int V>
__global__ void k_philox(uint32_t* out, uint32_t key) {
  uint32_t acc[4] = {0, 0, 0, 0};
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      U4 ctr{t, (uint32_t)it, (uint32_t)c, 0x53414D50u};
      U4 r;
      if (V == 0) r = philox_mad64<10>(ctr, key, ~key);
      else if (V == 1) r = philox_hilo(ctr, key, ~key);
      else if (V == 2) r = philox_mad64<7>(ctr, key, ~key);
      else if (V == 3) r = threefry<13>(ctr, key, ~key);
      else r = threefry<20>(ctr, key, ~key);
      acc[c] ^= r.x ^ r.y ^ r.z ^ r.w;
    }
  }
  out[t] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
}

__global__ void k_boxmuller(float* out, uint32_t key) {
  float acc[4] = {0, 0, 0, 0};
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = t * 0x9E3779B9u ^ key, b = t * 0x85EBCA6Bu;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      a = a * 1664525u + 1013904223u;
      b = b ^ (a >> 7);
      const float u1 = 1.0f - (float)(a >> 8) * 0x1.0p-24f;
      const float u2 = (float)(b >> 8) * 0x1.0p-24f;
      const float r = __builtin_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
      acc[c] += r * __builtin_amdgcn_cosf(u2) + r * __builtin_amdgcn_sinf(u2);
    }
  }
  out[t] = acc[0] + acc[1] + acc[2] + acc[3];
}

int main() {
  const int blocks = 4096, threads = 256;
  void* out;
  hipMalloc(&out, blocks * threads * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double n = (double)blocks * threads * ITERS * 4;
  struct K { const char* name; void (*fn)(uint32_t*, uint32_t); } ks[] = {
      {"philox4x32-10 (v_mad_u64_u32)", k_philox<0>}, {"philox4x32-10 (mul_hi/mul_lo)", k_philox<1>},
      {"philox4x32-7 (v_mad_u64_u32)", k_philox<2>}, {"threefry4x32-13", k_philox<3>},
      {"threefry4x32-20", k_philox<4>}};
  for (auto& k : ks) {
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(threads), 0, 0, (uint32_t*)out, 12345u);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
    }
    printf("%-34s %8.3f ms  %8.1f G calls/s  %6.2f ps/call\n", k.name, ms, n / (ms * 1e-3) / 1e9,
           ms * 1e9 / n);
  }
  float ms = 0;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_boxmuller, dim3(blocks), dim3(threads), 0, 0, (float*)out, 12345u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
  }
  printf("%-34s %8.3f ms  %8.1f G pairs/s  %6.2f ps/pair\n", "box-muller pair (+LCG)", ms,
         n / (ms * 1e-3) / 1e9, ms * 1e9 / n);
  return 0;
}
