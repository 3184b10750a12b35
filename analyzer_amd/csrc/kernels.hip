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

#include <cstdlib>

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

// Read every roster row once, so the rating launch behind it finds them in the
// Infinity Cache instead of HBM (the prepass in front of it streams several
// hundred MB through that cache).  The loads feed an xor whose only use is a
// store under a condition the host makes false (`never`), so they stay.
__global__ void __launch_bounds__(256) warm_rows_kernel(const uint4* __restrict__ rows, int64_t n,
                                                        uint32_t never, uint32_t* __restrict__ sink) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint4 v = rows[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == never) sink[threadIdx.x] = acc;
}

int launch_warm_rows(const float* state, int64_t P, uint32_t* sink, hipStream_t s) {
  const int64_t n = P * kGranules;
  if (n <= 0) return 0;
  // 8 granules per thread at 1M players: 1024 workgroups, 4 per CU
  const int64_t want = (n + 256 * 8 - 1) / (256 * 8);
  const unsigned blocks = (unsigned)(want < 1 ? 1 : (want > 4096 ? 4096 : want));
  hipLaunchKernelGGL(warm_rows_kernel, dim3(blocks), dim3(256), 0, s,
                     reinterpret_cast<const uint4*>(state), n, 0x5a5a5a5au, sink);
  return (int)hipGetLastError();
}

// An all-reduce stand-in for pricing DP steps on ONE GPU (parallel/sweep.py
// ``emulate``): what an RCCL ring all-reduce of the merge operands does to this GPU
// -- `channels` workgroups (RCCL's channel count, one CU each) stream the operand
// buffer `passes` times (the local reads / reduce / writes of a ring: about 3x the
// size) and hold their CUs until `ticks` of the 100-MHz s_memrealtime clock have
// passed since the first wave started (the xGMI transfer time of the modelled link
// bandwidth).  The buffer is rewritten unchanged (each word xor 0 with a runtime
// zero), so the merge decodes exactly what one rank's identity all-reduce leaves.
__global__ void __launch_bounds__(256) emulate_allreduce_kernel(uint4* buf, int64_t n, int passes, uint32_t zero,
                                                               uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  constexpr int U = 8;  // loads in flight per lane (a dependent load per iteration would be latency-bound)
  for (int q = 0; q < passes; ++q)
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += U * stride) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + u * stride;
        v[u] = i < n ? buf[i] : uint4{0, 0, 0, 0};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + u * stride;
        v[u].x ^= zero;
        if (i < n) buf[i] = v[u];
      }
    }
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

int launch_emulate_allreduce(void* buf, int64_t bytes, int channels, int passes, double us, hipStream_t s) {
  const int64_t n = bytes / 16;
  if (n <= 0 || channels < 1) return 0;
  const uint64_t ticks = (uint64_t)(us > 0 ? us * 100.0 : 0.0);  // s_memrealtime: 100 MHz
  hipLaunchKernelGGL(emulate_allreduce_kernel, dim3((unsigned)channels), dim3(256), 0, s,
                     reinterpret_cast<uint4*>(buf), n, passes, 0u, ticks);
  return (int)hipGetLastError();
}

// Device-side launch epoch of a captured graph: one bump per replay, before the
// rate launch that reads it (the host resets the tags and the counter before 255).
__global__ void epoch_bump_kernel(int32_t* e) { e[0] += 1; }

int launch_epoch_bump(int32_t* e, hipStream_t s) {
  hipLaunchKernelGGL(epoch_bump_kernel, dim3(1), dim3(1), 0, s, e);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------- schedule
static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

size_t schedule_workspace_bytes(int64_t nslots, int64_t num_players) {
  (void)num_players;
  return 4 * align_up(nslots * 4) + align_up(radix_sort_workspace_bytes(nslots));
}

// Micro-batch schedule (a worker batch of <= kSmallSched slots, e.g. 500 3v3 or
// 5v5 matches): ONE workgroup keys the slots (player, or past the last player
// for matches that touch no state), sorts (key << 32 | slot) -- stable by slot,
// like the radix path --, writes every slot's link from its sorted neighbours
// and zeroes the completion counters: one dispatch instead of the radix path's
// ~12, which are launch-bound at this size.  The bitonic network keeps E
// consecutive elements per thread in registers: exchanges closer than E run in
// registers, closer than 64 E (one wave) through lane shuffles, and only the
// few wider ones through LDS with a barrier.
constexpr int kSmallSched = 8192;
constexpr int kSmallThreads = 1024;

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}

template <int K, int E>
__global__ void __launch_bounds__(kSmallThreads)
sched_small_kernel(const int32_t* __restrict__ rec, int64_t M, uint32_t kend, uint32_t* __restrict__ link,
                   int32_t* __restrict__ deps, uint32_t* __restrict__ overflow) {
  constexpr int S = 2 * K, R = S + 2;
  constexpr int NP = kSmallThreads * E;  // padded sort size
  __shared__ uint64_t kv[NP];
  const int tid = threadIdx.x;
  const int n = (int)(M * S);
  for (int m = tid; m < (int)M; m += kSmallThreads) {
    int32_t r[R];
#pragma unroll
    for (int k = 0; k < R; ++k) r[k] = rec[(int64_t)m * R + k];
    const bool rates = early_status<K>(r, (int64_t)kend) == kRated;
    const uint32_t m0 = (uint32_t)r[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const int pos = j < K ? j : j - K;
      const bool in_roster = pos < (j < K ? meta_n0(m0) : meta_n1(m0));
      const uint32_t key = rates && in_roster ? (uint32_t)r[j] : kend;
      kv[m * S + j] = ((uint64_t)key << 32) | (uint32_t)(m * S + j);
    }
    deps[m] = 0;
  }
  for (int i = n + tid; i < NP; i += kSmallThreads) kv[i] = ~0ull;
  if (tid == 0) *overflow = 0u;
  __syncthreads();
  uint64_t x[E];
#pragma unroll
  for (int q = 0; q < E; ++q) x[q] = kv[tid * E + q];
  for (int k = 2; k <= NP; k <<= 1) {
    for (int j = k >> 1; j >= E; j >>= 1) {
      const bool wave = j < 64 * E;
      if (!wave) {  // partner in another wave: exchange through LDS
        __syncthreads();
#pragma unroll
        for (int q = 0; q < E; ++q) kv[tid * E + q] = x[q];
        __syncthreads();
      }
#pragma unroll
      for (int q = 0; q < E; ++q) {  // partner: same register of lane ^ j / E, or LDS
        const int i = tid * E + q;
        const uint64_t y = wave ? shfl_xor64(x[q], j / E) : kv[i ^ j];
        const bool lower = (i & j) == 0, asc = (i & k) == 0;
        const uint64_t lo = x[q] < y ? x[q] : y, hi = x[q] < y ? y : x[q];
        x[q] = lower == asc ? lo : hi;
      }
    }
    // partners in this thread's registers (compile-time indices: no scratch)
#pragma unroll
    for (int jj = E / 2; jj > 0; jj >>= 1) {
      if (jj >= k) continue;
#pragma unroll
      for (int q = 0; q < E; ++q) {
        const int qp = q ^ jj;
        if (qp > q) {
          const int i = tid * E + q;
          const uint64_t a = x[q], b = x[qp];
          if ((a > b) == ((i & k) == 0)) {
            x[q] = b;
            x[qp] = a;
          }
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < E; ++q) kv[tid * E + q] = x[q];
  __syncthreads();
  for (int p = tid; p < n; p += kSmallThreads) {
    const uint64_t v64 = kv[p];
    const uint32_t key = (uint32_t)(v64 >> 32), v = (uint32_t)v64;
    uint32_t w = kNoMatch;
    if (key < kend) {
      if (p + 1 < n && (uint32_t)(kv[p + 1] >> 32) == key) w = (uint32_t)kv[p + 1] / (uint32_t)S;
      if (p > 0 && (uint32_t)(kv[p - 1] >> 32) == key) w |= kLinkHasPred;
    }
    link[v] = w;
  }
}

// Micro-batch schedule without a sort (default; ANA_SCHED_SMALL=bitonic selects the
// kernel above for A/B).  A link only needs, per slot, the next slot of the same
// player and whether an earlier one exists -- not a total order.  So: key every
// slot into LDS, push each keyed slot onto an LDS list per hash bucket (one
// ds atomic swap: the lists are unordered), then every slot walks its bucket's
// list and keeps the smallest later slot with its key (its successor) and
// whether any earlier slot has it (its predecessor flag) -- the same links as
// the stable sort.  4096 buckets for <= 8192 slots: lists of ~1-2 slots, three
// barriers instead of the bitonic network's ~80 dependent exchange stages.
// LDS: 16 KB heads + 16 KB u16 list links + 32 KB keys.
constexpr int kHashBuckets = 4096;

template <int K>
__global__ void __launch_bounds__(kSmallThreads)
sched_hash_kernel(const int32_t* __restrict__ rec, int64_t M, uint32_t kend, uint32_t* __restrict__ link,
                  int32_t* __restrict__ deps, uint32_t* __restrict__ overflow, int nz,
                  int32_t* __restrict__ epoch_bump) {
  constexpr int S = 2 * K, R = S + 2;
  __shared__ uint32_t head[kHashBuckets];
  __shared__ uint16_t nxt[kSmallSched];
  __shared__ uint32_t skey[kSmallSched];
  const int tid = threadIdx.x;
  const int n = (int)(M * S);
  for (int b = tid; b < kHashBuckets; b += kSmallThreads) head[b] = 0xffffffffu;
  for (int m = tid; m < (int)M; m += kSmallThreads) {
    int32_t r[R];
    const int32_t* src = rec + (int64_t)m * R;
    if constexpr (R % 4 == 0) {
#pragma unroll
      for (int k = 0; k < R / 4; ++k) {
        const int4 v = reinterpret_cast<const int4*>(src)[k];
        r[4 * k] = v.x; r[4 * k + 1] = v.y; r[4 * k + 2] = v.z; r[4 * k + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < R; ++k) r[k] = src[k];
    }
    const bool rates = early_status<K>(r, (int64_t)kend) == kRated;
    const uint32_t m0 = (uint32_t)r[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const int pos = j < K ? j : j - K;
      const bool in_roster = pos < (j < K ? meta_n0(m0) : meta_n1(m0));
      skey[m * S + j] = rates && in_roster ? (uint32_t)r[j] : kend;
    }
    deps[m] = 0;
  }
  if (tid < nz) overflow[tid] = 0u;
  if (epoch_bump && tid == 0) epoch_bump[0] += 1;  // graph replays: the launch epoch (epoch_bump_kernel)
  __syncthreads();
  for (int i = tid; i < n; i += kSmallThreads) {
    const uint32_t key = skey[i];
    if (key < kend) {
      const uint32_t h = (key * 0x9E3779B1u) >> (32 - 12);
      nxt[i] = (uint16_t)atomicExch(&head[h], (uint32_t)i);  // 0xffff: end of list
    }
  }
  __syncthreads();
  for (int i = tid; i < n; i += kSmallThreads) {
    const uint32_t key = skey[i];
    uint32_t w = kNoMatch;
    if (key < kend) {
      uint32_t succ = 0xffffffffu;
      bool pred = false;
      for (uint32_t t = head[(key * 0x9E3779B1u) >> (32 - 12)]; t < (uint32_t)kSmallSched;) {
        if (t != (uint32_t)i && skey[t] == key) {
          if (t > (uint32_t)i) succ = t < succ ? t : succ;
          else pred = true;
        }
        t = nxt[t];  // 0xffff ends the walk (>= kSmallSched)
      }
      if (succ != 0xffffffffu) w = succ / (uint32_t)S;
      if (pred) w |= kLinkHasPred;
    }
    link[i] = w;
  }
}

int launch_schedule(int K, const int32_t* rec, int64_t M, int64_t P, uint32_t* link,
                    int32_t* deps, void* ws, size_t ws_bytes, uint32_t* overflow, hipStream_t s,
                    bool zero_ctrl, int32_t* epoch_bump, int sort_nt) {
  // zero_ctrl: also zero the executor's control words (overflow = ctrl[0], ctrl[1..15]) for
  // a rate launch that follows on this stream and then skips its own zeroing dispatch
  const int nz = zero_ctrl ? 16 : 1;
  const int64_t n = M * 2 * K;
  if (n > 0 && n <= kSmallSched && P < 0x7fffffffLL && K >= 1 && K <= 5) {
    const int e = n <= 2048 ? 2 : n <= 4096 ? 4 : 8;  // elements per thread
    const char* small_e = getenv("ANA_SCHED_SMALL");  // per schedule (A/B in one process)
    const bool bitonic = small_e && small_e[0] == 'b';
    switch (K) {
#define ANA_SMALL_CASE(k)                                                                            \
  case k:                                                                                            \
    if (!bitonic)                                                                                    \
      hipLaunchKernelGGL((sched_hash_kernel<k>), dim3(1), dim3(kSmallThreads), 0, s, rec, M,         \
                         (uint32_t)P, link, deps, overflow, nz, epoch_bump);                         \
    else if (e == 2)                                                                                      \
      hipLaunchKernelGGL((sched_small_kernel<k, 2>), dim3(1), dim3(kSmallThreads), 0, s, rec, M,     \
                         (uint32_t)P, link, deps, overflow);                                         \
    else if (e == 4)                                                                                 \
      hipLaunchKernelGGL((sched_small_kernel<k, 4>), dim3(1), dim3(kSmallThreads), 0, s, rec, M,     \
                         (uint32_t)P, link, deps, overflow);                                         \
    else                                                                                             \
      hipLaunchKernelGGL((sched_small_kernel<k, 8>), dim3(1), dim3(kSmallThreads), 0, s, rec, M,     \
                         (uint32_t)P, link, deps, overflow);                                         \
    break;
      ANA_SMALL_CASE(1) ANA_SMALL_CASE(2) ANA_SMALL_CASE(3) ANA_SMALL_CASE(4) ANA_SMALL_CASE(5)
#undef ANA_SMALL_CASE
    }
    if (bitonic && zero_ctrl) ANA_HIP_CHECK(hipMemsetAsync(overflow, 0, 64, s));
    if (bitonic && epoch_bump) hipLaunchKernelGGL(epoch_bump_kernel, dim3(1), dim3(1), 0, s, epoch_bump);
    return (int)hipGetLastError();
  }
  if (n <= 0) {
    ANA_HIP_CHECK(hipMemsetAsync(overflow, 0, 4 * (size_t)nz, s));
    if (epoch_bump) hipLaunchKernelGGL(epoch_bump_kernel, dim3(1), dim3(1), 0, s, epoch_bump);
    return 0;
  }
  if (n > kMaxSlots || P >= 0x7fffffffLL || K < 1 || K > 5) return (int)hipErrorInvalidValue;
  if (ws_bytes < schedule_workspace_bytes(n, P)) return (int)hipErrorInvalidValue;
  // the counters, the control words and the epoch bump are the first sort kernel's
  // side duties (radix_sort.hip SchedInit): no fill dispatches in front of the sort
  char* p = static_cast<char*>(ws);
  uint32_t* keys_a = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* vals_a = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* keys_b = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* vals_b = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  return launch_sched_sort(K, rec, M, (uint32_t)P, keys_a, vals_a, keys_b, vals_b, p, link, s, deps,
                           overflow, nz, epoch_bump, sort_nt);
}

}  // namespace ana
