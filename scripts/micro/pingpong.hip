// Microbenchmark: one-way latency of a device-scope flag hand-off between two
// workgroups (different XCDs: dispatch round-robins workgroups over the 8 XCDs),
// i.e. the hardware floor of one dataflow dependency hop.  Also the latency of
// a dependent chain of sc1 loads (pointer chase) from one wave.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef __attribute__((address_space(1))) unsigned int gu32;

__global__ void pingpong(unsigned* flag, int iters, unsigned long long* out) {
  const int me = blockIdx.x;  // 0 or 1 (other blocks idle)
  if (me > 1 || threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    const unsigned want = 2u * i + me;
    unsigned long long spins = 0;
    while (__hip_atomic_load((gu32*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
      if (++spins > 100000000ull) { out[2] = 1; return; }
    }
    __hip_atomic_fetch_add((gu32*)flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  out[me] = t1 - t0;
}

__global__ void chase(const unsigned* next, int iters, unsigned long long* out, unsigned* sink) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  unsigned p = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i)
    p = __hip_atomic_load((gu32*)(next + p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  out[3] = t1 - t0;
  *sink = p;
}

int main() {
  unsigned* flag; unsigned long long* out; unsigned* next; unsigned* sink;
  const int iters = 20000;
  const size_t n = 32u << 20;  // 128 MB chase table (> L2, < MALL)
  hipMalloc(&flag, 256); hipMalloc(&out, 64); hipMalloc(&next, n * 4); hipMalloc(&sink, 4);
  unsigned* h = (unsigned*)malloc(n * 4);
  unsigned long long x = 88172645463325252ull;
  for (size_t i = 0; i < n; ++i) h[i] = 0;
  // random cycle with a stride > 4 KB so every hop misses the L2
  unsigned cur = 0;
  for (int i = 0; i < iters + 10; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    unsigned nx = (unsigned)(x % n);
    h[cur] = nx; cur = nx;
  }
  hipMemcpy(next, h, n * 4, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) {
    hipMemset(flag, 0, 256); hipMemset(out, 0, 64);
    hipLaunchKernelGGL(pingpong, dim3(16), dim3(64), 0, 0, flag, iters, out);
    hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, next, iters, out, sink);
    hipDeviceSynchronize();
    unsigned long long o[4];
    hipMemcpy(o, out, 32, hipMemcpyDeviceToHost);
    // s_memrealtime: 100 MHz
    printf("pingpong one-way %.3f us   sc1 load chase %.3f us/hop   (timeout %llu)\n",
           o[0] * 10.0 / 1000.0 / (2.0 * iters), o[3] * 10.0 / 1000.0 / iters, o[2]);
  }
  return 0;
}
