// issue_bench.hip — instruction-issue ceilings of one gfx950 SIMD (VERDICT r01
// item 6: is a wave64 VALU instruction one per 4-cycle issue turn, or faster?).
//
// Each wave runs a long unrolled stream of independent instructions of one
// kind (8 accumulators, no dependency between neighbours), timed with
// s_memtime (shader clock) around the stream.  Launched with W waves per SIMD
// (1 .. 8, one 256-thread workgroup = 4 waves per CU x W/... see main), the
// result is instructions issued per SIMD per cycle for VALU only, SALU only,
// and VALU + SALU interleaved (co-issue from different waves).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/issue_bench tools/issue_bench.hip
// Run:   tools/issue_bench          (prints one JSON line per experiment)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kIters = 2048;  // x 8 instructions per iteration

__global__ void valu_kernel(unsigned long long* cyc, unsigned* sink) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
  const unsigned k = blockIdx.x | 1u;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; i++) {
    asm volatile(
        "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
        "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
        : "s"(k));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void salu_kernel(unsigned long long* cyc, unsigned* sink) {
  unsigned s0 = blockIdx.x, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3, s4 = s0 + 4, s5 = s0 + 5, s6 = s0 + 6,
           s7 = s0 + 7;
  const unsigned k = blockIdx.x | 1u;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; i++) {
    asm volatile(
        "s_add_u32 %0, %0, %8\n s_add_u32 %1, %1, %8\n s_add_u32 %2, %2, %8\n s_add_u32 %3, %3, %8\n"
        "s_add_u32 %4, %4, %8\n s_add_u32 %5, %5, %8\n s_add_u32 %6, %6, %8\n s_add_u32 %7, %7, %8\n"
        : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)
        : "s"(k)
        : "scc");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7;
}

// 4 VALU + 4 SALU per iteration, interleaved
__global__ void mixed_kernel(unsigned long long* cyc, unsigned* sink) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  unsigned s0 = blockIdx.x, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3;
  const unsigned k = blockIdx.x | 1u;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; i++) {
    asm volatile(
        "v_add_u32 %0, %0, %8\n s_add_u32 %4, %4, %8\n v_add_u32 %1, %1, %8\n s_add_u32 %5, %5, %8\n"
        "v_add_u32 %2, %2, %8\n s_add_u32 %6, %6, %8\n v_add_u32 %3, %3, %8\n s_add_u32 %7, %7, %8\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3)
        : "s"(k)
        : "scc");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ s0 ^ s1 ^ s2 ^ s3;
}

// a dependent VALU chain: the issue-to-issue latency of back-to-back dependent ops
__global__ void chain_kernel(unsigned long long* cyc, unsigned* sink) {
  unsigned a0 = threadIdx.x;
  const unsigned k = blockIdx.x | 1u;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; i++) {
    asm volatile(
        "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
        "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
        : "+v"(a0)
        : "s"(k));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = a0;
}

int main() {
  int dev = 0, n_cu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  const char* names[] = {"valu", "salu", "valu+salu", "valu_dependent_chain"};
  void (*kerns[])(unsigned long long*, unsigned*) = {valu_kernel, salu_kernel, mixed_kernel, chain_kernel};
  for (int kind = 0; kind < 4; kind++) {
    for (int wps : {1, 2, 4, 5, 8}) {  // waves per SIMD
      // one workgroup of 4 waves per CU and "wps" workgroups per CU: waves land
      // one per SIMD per workgroup (the dispatcher spreads a workgroup's waves)
      const int blocks = n_cu * wps, threads = 256;
      const int n_waves = blocks * 4;
      unsigned long long* cyc = nullptr;
      unsigned* sink = nullptr;
      hipMalloc(&cyc, sizeof(unsigned long long) * n_waves);
      hipMalloc(&sink, sizeof(unsigned) * blocks * threads);
      hipLaunchKernelGGL(kerns[kind], dim3(blocks), dim3(threads), 0, 0, cyc, sink);  // warm
      hipLaunchKernelGGL(kerns[kind], dim3(blocks), dim3(threads), 0, 0, cyc, sink);
      hipDeviceSynchronize();
      std::vector<unsigned long long> h(n_waves);
      hipMemcpy(h.data(), cyc, sizeof(unsigned long long) * n_waves, hipMemcpyDeviceToHost);
      double mean = 0;
      unsigned long long mx = 0;
      for (auto v : h) {
        mean += (double)v;
        mx = v > mx ? v : mx;
      }
      mean /= n_waves;
      const double instr = 8.0 * kIters;  // per wave
      // per SIMD: wps waves each issuing `instr` instructions over ~the max window
      printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"instr_per_wave\": %.0f, \"cycles_mean\": %.0f, "
             "\"cycles_max\": %llu, \"cycles_per_instr_per_wave\": %.3f, \"instr_per_cycle_per_simd\": %.3f}\n",
             names[kind], wps, instr, mean, mx, mean / instr, wps * instr / (double)mx);
      hipFree(cyc);
      hipFree(sink);
    }
  }
  return 0;
}
