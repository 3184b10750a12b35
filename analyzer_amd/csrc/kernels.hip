// MI355X (gfx950) kernels of the rating engine.
//
//  K7  gen_roster_kernel / gen_stream_kernel: synthetic inputs (counter RNG).
//  K5  schedule: one stable LSD radix sort of the slots (radix_sort.hip)
//      by player, fused with the record decode and the link write, gives per
//      slot the match of the player's next occurrence and a has-earlier flag
//      (link, 4 B); the executor derives each match's dependency count from
//      its links and counts the (zeroed) deps counters up to it.
//  The executor that consumes the schedule lives in dataflow.hip.
//
// Reference semantics: /root/reference/rater.py:69-169; the sequential loop the
// engine replaces is /root/reference/worker.py:176-192 (ORDER BY created_at).
#include <hip/hip_runtime.h>

#include "common.h"
#include "gen_core.h"
#include "kernels.h"
#include "rate_core.h"

namespace ana {

#define ANA_HIP_CHECK(expr)                                                            \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return (int)e_;                                              \
  } while (0)

// ------------------------------------------------------------------ generators
__global__ void gen_roster_kernel(GenRosterParams g, float* __restrict__ state,
                                  float* __restrict__ attrs) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= g.num_players) return;
  float st[kRowFloats], at[4];
  gen_player(g, p, st, at);
  float4* s4 = reinterpret_cast<float4*>(state + p * kRowFloats);
#pragma unroll
  for (int k = 0; k < kRowFloats / 4; ++k)
    s4[k] = make_float4(st[4 * k], st[4 * k + 1], st[4 * k + 2], st[4 * k + 3]);
  reinterpret_cast<float4*>(attrs)[p] = make_float4(at[0], at[1], at[2], at[3]);
}

template <int K>
__global__ void gen_stream_kernel(GenStreamParams g, int32_t* __restrict__ rec, int64_t M) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  constexpr int R = 2 * K + 2;
  int32_t r[R];
  gen_match<K>(g, m, r);
  if constexpr (R % 4 == 0) {
    int4* dst = reinterpret_cast<int4*>(rec + m * R);
#pragma unroll
    for (int k = 0; k < R / 4; ++k) dst[k] = make_int4(r[4 * k], r[4 * k + 1], r[4 * k + 2], r[4 * k + 3]);
  } else {
#pragma unroll
    for (int k = 0; k < R; ++k) rec[m * R + k] = r[k];
  }
}

int launch_gen_roster(const GenRosterParams& g, float* state, float* attrs, hipStream_t s) {
  if (g.num_players <= 0) return 0;
  const int64_t blocks = (g.num_players + 255) / 256;
  hipLaunchKernelGGL(gen_roster_kernel, dim3((unsigned)blocks), dim3(256), 0, s, g, state, attrs);
  return (int)hipGetLastError();
}

int launch_gen_stream(int K, const GenStreamParams& g, int32_t* rec, int64_t M, hipStream_t s) {
  if (M <= 0) return 0;
  const unsigned blocks = (unsigned)((M + 255) / 256);
  switch (K) {
#define ANA_GEN_CASE(k) \
  case k: hipLaunchKernelGGL(gen_stream_kernel<k>, dim3(blocks), dim3(256), 0, s, g, rec, M); break;
    ANA_GEN_CASE(1) ANA_GEN_CASE(2) ANA_GEN_CASE(3) ANA_GEN_CASE(4) ANA_GEN_CASE(5)
#undef ANA_GEN_CASE
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// Zero every tag of the roster (after an epoch wrap, or for a roster of unknown origin).
__global__ void reset_tags_kernel(float4* __restrict__ state, int64_t granules) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= granules) return;
  float4 v = state[i];
  v.y = 0.f;
  v.w = 0.f;
  state[i] = v;
}

int launch_reset_tags(float* state, int64_t P, hipStream_t s) {
  const int64_t n = P * kGranules;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(reset_tags_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<float4*>(state), n);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------- schedule
static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

size_t schedule_workspace_bytes(int64_t nslots, int64_t num_players) {
  (void)num_players;
  return 4 * align_up(nslots * 4) + align_up(radix_sort_workspace_bytes(nslots));
}

int launch_schedule(int K, const int32_t* rec, int64_t M, int64_t P, uint32_t* link,
                    int32_t* deps, void* ws, size_t ws_bytes, uint32_t* overflow, hipStream_t s) {
  const int64_t n = M * 2 * K;
  ANA_HIP_CHECK(hipMemsetAsync(overflow, 0, 4, s));
  if (n <= 0) return 0;
  if (n > kMaxSlots || P >= 0x7fffffffLL || K < 1 || K > 5) return (int)hipErrorInvalidValue;
  if (ws_bytes < schedule_workspace_bytes(n, P)) return (int)hipErrorInvalidValue;
  ANA_HIP_CHECK(hipMemsetAsync(deps, 0, (size_t)M * 4, s));
  char* p = static_cast<char*>(ws);
  uint32_t* keys_a = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* vals_a = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* keys_b = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* vals_b = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  return launch_sched_sort(K, rec, M, (uint32_t)P, keys_a, vals_a, keys_b, vals_b, p, link, s);
}

}  // namespace ana
