// Per-window digest of the executor's output records (runtime/rerate.py).
//
// A full-history re-rate accounts for every per-participant record it wrote (the
// reference writes one per participant and match, /root/reference/rater.py:151-169,
// committed per batch at worker.py:194) without moving 2 GB of rows per window to
// the host: one streaming pass over the packed 128-B rows (csrc/common.h RateOut)
// reduces them to
//
//   [0]              matches with records (status rated / AFK / invalid rosters)
//   [1]              participant records written (non-NaN shared mu)
//   [2 + f*S + j]    fp64 sum over matches of field f (s_mu, s_sig, delta, m_mu,
//                    m_sig) of slot j, NaN skipped
//   [2 + 5*S]        fp64 sum of quality, NaN skipped
//
// Deterministic by construction -- a resumed run must reproduce the digests of the
// windows it re-rates bit for bit: a fixed grid, per-lane accumulation in row order,
// fixed-order wave butterflies, a fixed-order sum over the waves of a workgroup into
// one partial row per workgroup, and one workgroup summing the partials in order.
// No atomics.  The pass is HBM-bound (one read of each row, non-temporal: nothing of
// it is reused), replacing seven torch nansum passes and a reduction per field.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "common.h"
#include "kernels.h"

namespace ana {

namespace {

typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int kDigestThreads = 256;
constexpr int kDigestBlocks = 1024;  // 4 workgroups per CU; fixed for determinism

template <int K>
struct DigestShape {
  static constexpr int S = 2 * K;
  static constexpr int D = 3 + 5 * S;      // outputs
  static constexpr int F = 5 * S + 2;      // floats of a row that matter
  static constexpr int V = (F + 3) / 4;    // 16-B loads per row
};

__device__ inline double wave_sum(double v) {
  // fixed butterfly order: the same bits on every run
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int K>
__global__ void __launch_bounds__(kDigestThreads) records_digest_kernel(const float* __restrict__ rows,
                                                                        int64_t M, int64_t W,
                                                                        double* __restrict__ partial) {
  using Sh = DigestShape<K>;
  constexpr int S = Sh::S, D = Sh::D, V = Sh::V;
  double acc[D];
#pragma unroll
  for (int d = 0; d < D; ++d) acc[d] = 0.0;
  const int64_t stride = (int64_t)gridDim.x * kDigestThreads;
  for (int64_t i = (int64_t)blockIdx.x * kDigestThreads + threadIdx.x; i < M; i += stride) {
    const v4f* r = reinterpret_cast<const v4f*>(rows + i * W);
    float f[4 * V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const v4f x = __builtin_nontemporal_load(r + v);
      f[4 * v + 0] = x[0];
      f[4 * v + 1] = x[1];
      f[4 * v + 2] = x[2];
      f[4 * v + 3] = x[3];
    }
    const uint32_t status = __float_as_uint(f[5 * S + 1]) & 0xffu;
    acc[0] += (status == kRated || status == kAfk || status == kInvalidRosters) ? 1.0 : 0.0;
#pragma unroll
    for (int j = 0; j < S; ++j) acc[1] += (f[j] == f[j]) ? 1.0 : 0.0;
#pragma unroll
    for (int c = 0; c < 5 * S + 1; ++c) {
      const float x = f[c];
      acc[2 + c] += (x == x) ? (double)x : 0.0;
    }
  }
  __shared__ double red[kDigestThreads / 64][D];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const double s = wave_sum(acc[d]);
    if (lane == 0) red[wave][d] = s;
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += kDigestThreads) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kDigestThreads / 64; ++w) s += red[w][d];
    partial[(int64_t)blockIdx.x * D + d] = s;
  }
}

__global__ void __launch_bounds__(64) digest_finish_kernel(const double* __restrict__ partial, int D, int blocks,
                                                           double* __restrict__ out) {
  for (int d = threadIdx.x; d < D; d += 64) {
    double s = 0.0;
    for (int b = 0; b < blocks; ++b) s += partial[(int64_t)b * D + d];  // in workgroup order
    out[d] = s;
  }
}

}  // namespace

size_t records_digest_scratch_doubles(int K) { return (size_t)kDigestBlocks * (3 + 10 * K); }

int launch_records_digest(int K, const float* rows, int64_t M, int64_t W, double* scratch, double* out,
                          hipStream_t s) {
  if (K < 1 || K > 5 || W < 5 * 2 * K + 2 || (W & 3)) return (int)hipErrorInvalidValue;
  const int D = 3 + 10 * K;
  switch (K) {
#define ANA_DIGEST_CASE(k)                                                                                      \
  case k:                                                                                                       \
    hipLaunchKernelGGL(records_digest_kernel<k>, dim3(kDigestBlocks), dim3(kDigestThreads), 0, s, rows, M, W,  \
                       scratch);                                                                                \
    break;
    ANA_DIGEST_CASE(1) ANA_DIGEST_CASE(2) ANA_DIGEST_CASE(3) ANA_DIGEST_CASE(4) ANA_DIGEST_CASE(5)
#undef ANA_DIGEST_CASE
  }
  hipLaunchKernelGGL(digest_finish_kernel, dim3(1), dim3(64), 0, s, scratch, D, kDigestBlocks, out);
  return (int)hipGetLastError();
}

}  // namespace ana
