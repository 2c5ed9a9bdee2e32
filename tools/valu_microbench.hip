// Microbenchmark of the VALU instruction mix of the EI scoring loop on gfx950:
// throughput of v_fma_f32, v_pk_fma_f32, v_exp_f32 and of the actual pair
// recipe (fma, fma, exp, add), whole chip, 8 independent chains per lane.
// Output: ops per SIMD per cycle, with the in-kernel clock measured by
// s_memtime / s_memrealtime (100 MHz).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));

#define ITERS 4096
struct Stamp { unsigned long long t0, t1, r0, r1; };

__device__ __forceinline__ void stamp_begin(Stamp* s) {
  if (threadIdx.x == 0) { s[blockIdx.x].t0 = __builtin_amdgcn_s_memtime(); s[blockIdx.x].r0 = __builtin_amdgcn_s_memrealtime(); }
}
__device__ __forceinline__ void stamp_end(Stamp* s) {
  if (threadIdx.x == 0) { s[blockIdx.x].t1 = __builtin_amdgcn_s_memtime(); s[blockIdx.x].r1 = __builtin_amdgcn_s_memrealtime(); }
}

__global__ void k_fma(float* out, Stamp* st, float a, float b) {
  float x[8]; for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3f + i;
  stamp_begin(st);
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = fmaf(x[i], a, b);
  }
  stamp_end(st);
  float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_pkfma(float* out, Stamp* st, float a, float b) {
  f2 x[4]; for (int i = 0; i < 4; ++i) x[i] = f2{threadIdx.x * 1e-3f + i, (float)i};
  f2 av = f2{a, a}, bv = f2{b, b};
  stamp_begin(st);
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = __builtin_elementwise_fma(x[i], av, bv);
  }
  stamp_end(st);
  float s = 0; for (int i = 0; i < 4; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_exp(float* out, Stamp* st, float a, float b) {
  float x[8]; for (int i = 0; i < 8; ++i) x[i] = -(threadIdx.x * 1e-3f + i);
  stamp_begin(st);
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_exp2f(x[i]) - 1.0f;
  }
  stamp_end(st);
  float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// the pair recipe: t = x*a+b ; v = c - t*t ; s += exp2(v)   (8 candidates)
__global__ void k_pair(float* out, Stamp* st, float a, float b) {
  float x[8], s[8]; for (int i = 0; i < 8; ++i) { x[i] = threadIdx.x * 1e-3f + i; s[i] = 0; }
  stamp_begin(st);
  for (int it = 0; it < ITERS; ++it) {
    const float c = -1.0f - it * 1e-7f;
#pragma unroll
    for (int i = 0; i < 8; ++i) { float t = fmaf(x[i], a, b + it * 1e-6f); s[i] += __builtin_amdgcn_exp2f(fmaf(-t, t, c)); }
  }
  stamp_end(st);
  float r = 0; for (int i = 0; i < 8; ++i) r += s[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// pair recipe with packed fp32 math on candidate pairs
__global__ void k_pair_pk(float* out, Stamp* st, float a, float b) {
  f2 x[4], s[4]; for (int i = 0; i < 4; ++i) { x[i] = f2{threadIdx.x * 1e-3f + i, (float)i}; s[i] = f2{0, 0}; }
  stamp_begin(st);
  for (int it = 0; it < ITERS; ++it) {
    const f2 cv = f2{-1.0f - it * 1e-7f, -1.0f - it * 1e-7f};
    const f2 av = f2{a, a}, bv = f2{b + it * 1e-6f, b + it * 1e-6f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f2 t = __builtin_elementwise_fma(x[i], av, bv);
      f2 v = __builtin_elementwise_fma(-t, t, cv);
      s[i] += f2{__builtin_amdgcn_exp2f(v.x), __builtin_amdgcn_exp2f(v.y)};
    }
  }
  stamp_end(st);
  float r = 0; for (int i = 0; i < 4; ++i) r += s[i].x + s[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  const int blocks = 2048, threads = 256;
  float* out; Stamp* st;
  hipMalloc(&out, blocks * threads * 4);
  hipMalloc(&st, blocks * sizeof(Stamp));
  Stamp* hs = (Stamp*)malloc(blocks * sizeof(Stamp));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  struct K { const char* name; void (*fn)(float*, Stamp*, float, float); double ops_per_iter; } ks[] = {
    {"v_fma_f32 (8 chains)", k_fma, 8}, {"v_pk_fma_f32 (4x2 chains)", k_pkfma, 8},
    {"v_exp_f32 (+sub, 8 chains)", k_exp, 8}, {"pair fma,fma,exp,add (8 cand)", k_pair, 8},
    {"pair packed (4x2 cand)", k_pair_pk, 8}};
  for (auto& k : ks) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(threads), 0, 0, out, st, 1.0001f, 1e-4f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(hs, st, blocks * sizeof(Stamp), hipMemcpyDeviceToHost);
      double cyc = 0, rt = 0;
      for (int b = 0; b < blocks; ++b) { cyc += (double)(hs[b].t1 - hs[b].t0); rt += (double)(hs[b].r1 - hs[b].r0); }
      const double ghz = cyc / rt * 0.1;  // s_memrealtime ticks at 100 MHz
      const double lane_ops = (double)blocks * threads * ITERS * k.ops_per_iter;
      const double per_simd_cycle = lane_ops / (ms * 1e-3) / (1024.0 * ghz * 1e9);
      if (rep == 2) printf("%-34s %8.3f ms  clk %.2f GHz  %6.2f lane-ops/SIMD/cycle  (%.1f G lane-ops/s)\n",
                           k.name, ms, ghz, per_simd_cycle, lane_ops / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}
