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
// windows it re-rates bit for bit: a fixed grid, per-lane accumulation in a fixed order,
// a fixed-order sum over the lanes of a workgroup into one partial row per workgroup,
// and a fixed-order tree over the partials.  No atomics.  The pass is HBM-bound (one
// read of each row, non-temporal: nothing of it is reused), replacing seven torch
// nansum passes and a reduction per field.
//
// Coalesced: the rows are read as one flat array of 16-B quads, lane i of the grid
// taking quads i, i + stride, ... -- a wave reads 1 KB of consecutive rows per load --
// and since the stride is a multiple of the Q quads of a row, every lane sees ONE quad
// position of every row it visits: four fields, four fp64 sums.  The first version
// gave each lane whole rows (8 16-B loads at a 128-B lane stride, 33 fp64 sums per
// lane) and ran at 1.18 ms per 16M-match window beside 1.04 ms for a one-wave finish
// over the 1024 partials (profiles/r6/prof_rerate_kernel_stats.txt).
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "common.h"
#include "kernels.h"

namespace ana {

namespace {

typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int kDigestThreads = 256;
constexpr int kDigestBlocks = 1024;  // 4 workgroups per CU; fixed for determinism
constexpr int kDigestUnroll = 4;     // quads in flight per lane

__device__ inline double wave_sum(double v) {
  // fixed butterfly order: the same bits on every run
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Q = W / 4 quads per row, a divisor of kDigestThreads (packed rows: 32 or 64 floats),
// so a lane's quad position is threadIdx.x % Q in every workgroup.
template <int K>
__global__ void __launch_bounds__(kDigestThreads) records_digest_kernel(const float* __restrict__ rows,
                                                                        int64_t M, int Q,
                                                                        double* __restrict__ partial,
                                                                        unsigned long long* __restrict__ hist) {
  constexpr int S = 2 * K;
  constexpr int D = 3 + 5 * S;  // outputs
  constexpr int F = 5 * S + 2;  // floats of a row that matter: 5 S fields, quality, status
  const int t = threadIdx.x;
  const int q = t % Q;
  // this lane's four fields 4q + c: summed (< 5S + 1: the slot fields and quality),
  // counted as participant records (< S: a non-NaN shared mu), the status word (5S + 1)
  bool sum_c[4], part_c[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    sum_c[c] = 4 * q + c < F - 1;
    part_c[c] = 4 * q + c < S;
  }
  const bool has_status = (F - 1) / 4 == q;
  const int status_c = (F - 1) % 4;
  const bool active = 4 * q < F;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  uint32_t npart = 0u, nmatch = 0u;
  // status histogram (hist != nullptr): the four common codes in registers, the rest
  // through LDS atomics; integer sums, so the order does not matter
  __shared__ uint32_t lhist[256];
  lhist[t] = 0u;
  uint32_t nst[4] = {0u, 0u, 0u, 0u};
  const bool want_hist = hist != nullptr && has_status;
  const v4f* src = reinterpret_cast<const v4f*>(rows);
  const int64_t nq = M * Q;
  const int64_t stride = (int64_t)gridDim.x * kDigestThreads;
  auto fold = [&](const v4f x) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float v = x[c];
      acc[c] += (sum_c[c] && v == v) ? (double)v : 0.0;
      npart += (part_c[c] && v == v) ? 1u : 0u;
    }
    const uint32_t st = __float_as_uint(x[status_c]) & 0xffu;
    nmatch += (has_status && (st == kRated || st == kAfk || st == kInvalidRosters)) ? 1u : 0u;
    if (want_hist) {
#pragma unroll
      for (int k = 0; k < 4; ++k) nst[k] += st == (uint32_t)k ? 1u : 0u;
      if (st >= 4u) atomicAdd(&lhist[st], 1u);
    }
  };
  __syncthreads();  // lhist zeroed
  int64_t i = (int64_t)blockIdx.x * kDigestThreads + t;
  if (active) {
    for (; i + (kDigestUnroll - 1) * stride < nq; i += kDigestUnroll * stride) {
      v4f x[kDigestUnroll];
#pragma unroll
      for (int u = 0; u < kDigestUnroll; ++u) x[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
      for (int u = 0; u < kDigestUnroll; ++u) fold(x[u]);
    }
    for (; i < nq; i += stride) fold(__builtin_nontemporal_load(src + i));
  }
  // one partial row per workgroup: output d sums the lanes of its quad position in lane order
  __shared__ double lacc[4][kDigestThreads];
  __shared__ uint32_t lcnt[2][kDigestThreads];
#pragma unroll
  for (int c = 0; c < 4; ++c) lacc[c][t] = acc[c];
  lcnt[0][t] = nmatch;
  lcnt[1][t] = npart;
  if (want_hist) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (nst[k]) atomicAdd(&lhist[k], nst[k]);
  }
  __syncthreads();
  if (hist != nullptr && lhist[t] != 0u) atomicAdd(&hist[t], (unsigned long long)lhist[t]);
  if (t < D) {
    double s = 0.0;
    if (t < 2) {
      uint64_t n = 0;
      for (int u = 0; u < kDigestThreads; ++u) n += lcnt[t][u];
      s = (double)n;
    } else {
      const int f = t - 2, fq = f / 4, fc = f % 4;
      for (int u = fq; u < kDigestThreads; u += Q) s += lacc[fc][u];
    }
    partial[(int64_t)blockIdx.x * D + t] = s;
  }
}

// one workgroup per output: lane l sums partials l, l + 256, ... in order, then a fixed
// butterfly per wave and the four waves in order
__global__ void __launch_bounds__(kDigestThreads) digest_finish_kernel(const double* __restrict__ partial, int D,
                                                                       int blocks, double* __restrict__ out) {
  const int d = blockIdx.x;
  double s = 0.0;
  for (int b = threadIdx.x; b < blocks; b += kDigestThreads) s += partial[(int64_t)b * D + d];
  s = wave_sum(s);
  __shared__ double w[kDigestThreads / 64];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = 0.0;
#pragma unroll
    for (int k = 0; k < kDigestThreads / 64; ++k) r += w[k];
    out[d] = r;
  }
}

}  // namespace

size_t records_digest_scratch_doubles(int K) { return (size_t)kDigestBlocks * (3 + 10 * K); }

int launch_records_digest(int K, const float* rows, int64_t M, int64_t W, double* scratch, double* out,
                          int64_t* hist, hipStream_t s) {
  if (K < 1 || K > 5 || W < 5 * 2 * K + 2 || (W & 3)) return (int)hipErrorInvalidValue;
  const int Q = (int)(W / 4);
  if (Q > kDigestThreads || kDigestThreads % Q != 0) return (int)hipErrorInvalidValue;
  const int D = 3 + 10 * K;
  switch (K) {
#define ANA_DIGEST_CASE(k)                                                                                      \
  case k:                                                                                                       \
    hipLaunchKernelGGL(records_digest_kernel<k>, dim3(kDigestBlocks), dim3(kDigestThreads), 0, s, rows, M, Q,  \
                       scratch, reinterpret_cast<unsigned long long*>(hist));                                   \
    break;
    ANA_DIGEST_CASE(1) ANA_DIGEST_CASE(2) ANA_DIGEST_CASE(3) ANA_DIGEST_CASE(4) ANA_DIGEST_CASE(5)
#undef ANA_DIGEST_CASE
  }
  hipLaunchKernelGGL(digest_finish_kernel, dim3(D), dim3(kDigestThreads), 0, s, scratch, D, kDigestBlocks, out);
  return (int)hipGetLastError();
}

}  // namespace ana
