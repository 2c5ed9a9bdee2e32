// Microbenchmark (diagnostic): throughput of the cell gather of the table
// scorer on gfx950 -- one 64-B cell per candidate at a pseudo-random cell
// index -- in four forms:
//   A  cooperative LDS-DMA (global_load_lds_dwordx4, 4-lane groups; the
//      shipped k_score_table gather)
//   B  per-lane global_load_dwordx4 x4 into VGPRs
//   C  table copied once per block into LDS, per-lane ds_read_b128 x4
//   D  as C with 32-B cells (ds_read_b128 x2)
// for a small (710-cell, uniform-label) and a large (10000-cell, normal-label)
// table.  Candidates per thread per launch: kR; candidates/s reported.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kBS = 256, kR = 64, kWave = 64;
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_vp;
typedef const __attribute__((address_space(1))) void* glb_vp;

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
// cell of candidate i: a triangular-ish concentration (sum of two uniforms)
__device__ __forceinline__ uint32_t cell_of(uint32_t i, uint32_t nb) {
  const uint32_t h = hsh(i);
  return (uint32_t)(((h & 0xFFFF) + (h >> 16)) * (uint64_t)nb >> 17);
}

__global__ __launch_bounds__(kBS) void kA(const float* cells, int nb, float* out) {
  __shared__ f4 s_rows[(kBS / kWave) * kWave * 4];
  const int lane = threadIdx.x & 63, gi = lane & 3, gbase = lane & ~3;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  f4* rows = s_rows + wave * (kWave * 4);
  const char* cb = reinterpret_cast<const char*>(cells);
  float acc = 0.f;
  const uint32_t t = blockIdx.x * kBS + threadIdx.x;
  for (int r = 0; r < kR; ++r) {
    const uint32_t co = cell_of(t * kR + r, nb) * 64u;
#define TPE_ONE(j)                                                                              \
  {                                                                                             \
    const uint32_t cj = (uint32_t)__builtin_amdgcn_mov_dpp((int)co, j | (j << 2) | (j << 4) | (j << 6), \
                                                          0xF, 0xF, true);                     \
    __builtin_amdgcn_global_load_lds((glb_vp)(cb + cj + ((gi ^ j) * 16)), (lds_vp)(rows + j * kWave), \
                                     16, 0, 0);                                                \
  }
    TPE_ONE(0) TPE_ONE(1) TPE_ONE(2) TPE_ONE(3)
#undef TPE_ONE
    __builtin_amdgcn_s_waitcnt(0x0F70);
    const f4* slab = rows + gi * kWave;
    const f4 q0 = slab[gbase | gi], q1 = slab[gbase | (1 ^ gi)], q2 = slab[gbase | (2 ^ gi)],
             q3 = slab[gbase | (3 ^ gi)];
    __builtin_amdgcn_s_waitcnt(0xC07F);
    acc += q0.x + q1.y + q2.z + q3.w;
  }
  out[t] = acc;
}

__global__ __launch_bounds__(kBS) void kB(const float* cells, int nb, float* out) {
  const f4* c4 = reinterpret_cast<const f4*>(cells);
  float acc = 0.f;
  const uint32_t t = blockIdx.x * kBS + threadIdx.x;
  for (int r = 0; r < kR; ++r) {
    const uint32_t c = cell_of(t * kR + r, nb);
    const f4 q0 = c4[4 * c], q1 = c4[4 * c + 1], q2 = c4[4 * c + 2], q3 = c4[4 * c + 3];
    acc += q0.x + q1.y + q2.z + q3.w;
  }
  out[t] = acc;
}

template <int CELLB>
__global__ __launch_bounds__(kBS) void kC(const float* cells, int nb, float* out) {
  extern __shared__ f4 s_tab[];
  const f4* c4 = reinterpret_cast<const f4*>(cells);
  constexpr int Q = CELLB / 16;
  for (int i = threadIdx.x; i < nb * Q; i += kBS) s_tab[i] = c4[i];
  __syncthreads();
  float acc = 0.f;
  const uint32_t t = blockIdx.x * kBS + threadIdx.x;
  for (int r = 0; r < kR; ++r) {
    const uint32_t c = cell_of(t * kR + r, nb);
    f4 q = s_tab[Q * c];
#pragma unroll
    for (int k = 1; k < Q; ++k) q += s_tab[Q * c + k];
    acc += q.x + q.y + q.z + q.w;
  }
  out[t] = acc;
}

int main() {
  const int blocks = 30720 / 16;  // 30 labels x 2^22 candidates / (256 x kR)
  float *cells, *out;
  hipMalloc(&cells, 10000 * 64);
  hipMalloc(&out, blocks * kBS * 4);
  hipMemset(cells, 0, 10000 * 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double n = (double)blocks * kBS * kR;
  for (int nb : {710, 2000, 10000}) {
    for (int v = 0; v < 4; ++v) {
      if (v >= 2 && nb * (v == 2 ? 64 : 32) > 160 * 1024) continue;
      float ms = 0;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        if (v == 0) hipLaunchKernelGGL(kA, dim3(blocks), dim3(kBS), 0, 0, cells, nb, out);
        if (v == 1) hipLaunchKernelGGL(kB, dim3(blocks), dim3(kBS), 0, 0, cells, nb, out);
        if (v == 2) hipLaunchKernelGGL(kC<64>, dim3(blocks), dim3(kBS), nb * 64, 0, cells, nb, out);
        if (v == 3) hipLaunchKernelGGL(kC<32>, dim3(blocks), dim3(kBS), nb * 32, 0, cells, nb, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
      }
      printf("cells %6d  %-22s %8.3f ms  %8.1f G cand/s\n", nb,
             v == 0 ? "A lds-dma coop" : v == 1 ? "B per-lane vgpr" : v == 2 ? "C lds table 64B" : "D lds table 32B",
             ms, n / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}
