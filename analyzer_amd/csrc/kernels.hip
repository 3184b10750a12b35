// MI355X (gfx950) kernels of the rating engine.
//
//  K7  gen_roster_kernel / gen_stream_kernel: synthetic inputs (counter RNG).
//  K5  schedule: one stable hipCUB/rocPRIM onesweep radix sort of the slots
//      by player gives, per slot, its occurrence index among the window's
//      stateful matches and the slot of the player's NEXT occurrence (link),
//      and per match the number of distinct players with an earlier
//      occurrence (deps).
//  K1-K4, K3, K6  rate_dataflow_kernel: ONE launch rates the whole window in
//      exact per-player chronological order, with no rounds and no grid
//      barrier (Kahn's algorithm over the per-player chains):
//      * 8 sharded tickets (MICROARCH "dequeue") hand out chunks of 64
//        consecutive matches; a wave holds up to 4 chunks (256 matches, records
//        cached in LDS), so ~1M matches wait in flight across the GPU -- the
//        per-player dependency levels of a random stream spread over hundreds
//        of thousands of matches, and a narrower window starves the GPU;
//      * waiting costs nothing per match: a wave polls the deps counters of
//        its chunks with one coalesced 4-B sc1 load per lane;
//      * the oldest ready matches go to the wave's lane groups (G lanes = one
//        match, one roster slot per lane); a group gathers its players'
//        16-B granules {mu, tag, sigma, tag} with sc1 buffer loads, seeds,
//        rates both tracks, publishes the granules with sc1 stores, drains
//        vmcnt, then decrements the deps counter of each player's next match
//        (MICROARCH "Valid forms" row 1: sc1 stores -> vmcnt(0) -> agent
//        atomic; consumer polls sc1 and then loads sc1).  The tag of the shared
//        granule is re-checked on the consumer side as a second safety net.
//      Claims are monotone per ticket shard and every claimed match is held by
//      a running wave, so the oldest unfinished match is always ready: no
//      deadlock whatever the residency.  Spins back off and give up after 5 s.
//
// Reference semantics: /root/reference/rater.py:69-169; the sequential loop it
// replaces is /root/reference/worker.py:176-192 (ORDER BY created_at).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "common.h"
#include "gen_core.h"
#include "kernels.h"
#include "rate_core.h"

namespace ana {

typedef __attribute__((address_space(1))) unsigned int gu32;
typedef int v4i __attribute__((ext_vector_type(4)));

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
// Slots of matches that touch no state (unsupported mode, rosters != 2, AFK,
// malformed) are keyed past the last player so they neither wait nor publish.
template <int K>
__global__ void sched_keys_kernel(const int32_t* __restrict__ rec, int64_t M, uint32_t P,
                                  uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  constexpr int S = 2 * K;
  MatchWork<float, K> w;
  decode_record<float, K>(rec + m * (S + 2), (int64_t)P, w);
  const bool rates = w.status == kRated;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    keys[m * S + j] = rates && w.id[j] >= 0 ? (uint32_t)w.id[j] : P;
    vals[m * S + j] = (uint32_t)(m * S + j);
  }
}

__global__ void sched_segstart_kernel(const uint32_t* __restrict__ keys, int64_t n,
                                      uint32_t kend, uint32_t* __restrict__ segstart) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = keys[i];
  if (k < kend && (i == 0 || keys[i - 1] != k)) segstart[k] = (uint32_t)i;
}

// link[slot] = (occurrence index of the slot's player, next slot of that player or -1)
__global__ void sched_link_kernel(const uint32_t* __restrict__ keys,
                                  const uint32_t* __restrict__ vals, int64_t n, uint32_t kend,
                                  const uint32_t* __restrict__ segstart, uint2* __restrict__ link,
                                  uint32_t* __restrict__ overflow) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = keys[i];
  if (k >= kend) return;
  const uint32_t o = (uint32_t)i - segstart[k];
  if (o > kMaxOcc) atomicOr(overflow, 1u);
  const uint32_t nxt = (i + 1 < n && keys[i + 1] == k) ? vals[i + 1] : 0xffffffffu;
  link[vals[i]] = make_uint2(o, nxt);
}

// deps[m] = number of distinct players of m with an earlier occurrence in the window
template <int K>
__global__ void sched_deps_kernel(const int32_t* __restrict__ rec, const uint2* __restrict__ link,
                                  int64_t M, uint32_t P, int32_t* __restrict__ deps) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  constexpr int S = 2 * K;
  MatchWork<float, K> w;
  decode_record<float, K>(rec + m * (S + 2), (int64_t)P, w);
  int d = 0;
  if (w.status == kRated) {
#pragma unroll
    for (int j = 0; j < S; ++j)
      if (w.first[j] == j && link[m * S + j].x > 0u) ++d;
  }
  deps[m] = d;
}

static int key_bits(uint64_t kmax) {
  int b = 1;
  while (b < 32 && (1ull << b) <= kmax) ++b;
  return b;
}

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

size_t schedule_workspace_bytes(int64_t nslots, int64_t num_players) {
  size_t cub = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, cub, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (uint32_t*)nullptr, (int)nslots, 0,
                                           key_bits((uint64_t)num_players));
  return 4 * align_up(nslots * 4) + align_up(((size_t)num_players + 1) * 4) + align_up(cub);
}

int launch_schedule(int K, const int32_t* rec, int64_t M, int64_t P, uint32_t* link,
                    int32_t* deps, void* ws, size_t ws_bytes, uint32_t* overflow, hipStream_t s) {
  const int64_t n = M * 2 * K;
  ANA_HIP_CHECK(hipMemsetAsync(overflow, 0, 4, s));
  if (n <= 0) return 0;
  if (n > 0x7fffffffLL || P >= 0x7fffffffLL) return (int)hipErrorInvalidValue;
  char* p = static_cast<char*>(ws);
  uint32_t* keys_in = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* vals_in = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* keys_out = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* vals_out = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* segstart = reinterpret_cast<uint32_t*>(p); p += align_up(((size_t)P + 1) * 4);
  size_t cub_bytes = ws_bytes - (size_t)(p - static_cast<char*>(ws));
  const unsigned mb = (unsigned)((M + 255) / 256);
  const unsigned nb = (unsigned)((n + 255) / 256);
  uint2* link2 = reinterpret_cast<uint2*>(link);
  switch (K) {
#define ANA_KEY_CASE(k)                                                                     \
  case k:                                                                                   \
    hipLaunchKernelGGL(sched_keys_kernel<k>, dim3(mb), dim3(256), 0, s, rec, M, (uint32_t)P, \
                       keys_in, vals_in);                                                   \
    break;
    ANA_KEY_CASE(1) ANA_KEY_CASE(2) ANA_KEY_CASE(3) ANA_KEY_CASE(4) ANA_KEY_CASE(5)
#undef ANA_KEY_CASE
    default: return (int)hipErrorInvalidValue;
  }
  ANA_HIP_CHECK(hipGetLastError());
  ANA_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(p, cub_bytes, keys_in, keys_out, vals_in,
                                                   vals_out, (int)n, 0, key_bits((uint64_t)P), s));
  hipLaunchKernelGGL(sched_segstart_kernel, dim3(nb), dim3(256), 0, s, keys_out, n, (uint32_t)P,
                     segstart);
  hipLaunchKernelGGL(sched_link_kernel, dim3(nb), dim3(256), 0, s, keys_out, vals_out, n,
                     (uint32_t)P, segstart, link2, overflow);
  switch (K) {
#define ANA_DEPS_CASE(k)                                                                      \
  case k:                                                                                     \
    hipLaunchKernelGGL(sched_deps_kernel<k>, dim3(mb), dim3(256), 0, s, rec, link2, M,         \
                       (uint32_t)P, deps);                                                    \
    break;
    ANA_DEPS_CASE(1) ANA_DEPS_CASE(2) ANA_DEPS_CASE(3) ANA_DEPS_CASE(4) ANA_DEPS_CASE(5)
#undef ANA_DEPS_CASE
  }
  return (int)hipGetLastError();
}

// --------------------------------------------------------------- rate (dataflow)
constexpr uint64_t kTimeoutTicks = 500000000ull;  // 5 s of the 100 MHz s_memrealtime clock
constexpr int kHeads = 8;                          // ticket shards (MICROARCH "dequeue")
constexpr int kChunk = 64;                         // matches per ticket = one per lane
constexpr int kHeld = 4;                           // chunks a wave keeps in flight
constexpr int kWavesPerBlock = 4;

// Sum over the G lanes of this lane's group (groups are aligned, G | 64).
template <int G>
__device__ __forceinline__ float group_sum(float x) {
#pragma unroll
  for (int off = G / 2; off >= 1; off >>= 1) x += __shfl_xor(x, off);
  return x;
}

__device__ __forceinline__ v4i granule(float mu, uint32_t tag, float sig) {
  v4i v;
  v.x = __float_as_int(mu);
  v.y = (int)tag;
  v.z = __float_as_int(sig);
  v.w = (int)tag;
  return v;
}

// position of the k-th (0-based) set bit of x (x has more than k bits set)
__device__ __forceinline__ int nth_set_bit(uint64_t x, int k) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint64_t low = x & ((w == 64 ? 0ull : (1ull << w)) - 1ull);
    const int c = __popcll(low);
    if (k >= c) {
      k -= c;
      x >>= w;
      pos += w;
    } else {
      x = low;
    }
  }
  return pos;
}

// early outcome of a match that touches no state (decided when its chunk is claimed)
template <int K>
__device__ __forceinline__ uint8_t early_status(const int32_t* r, int64_t P) {
  constexpr int S = 2 * K;
  const uint32_t m0 = (uint32_t)r[S], m1 = (uint32_t)r[S + 1];
  const int n0 = meta_n0(m0), n1 = meta_n1(m0);
  bool bad = n0 > K || n1 > K;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int pos = j < K ? j : j - K;
    if (pos < (j < K ? n0 : n1) && (r[j] < 0 || (int64_t)r[j] >= P)) bad = true;
  }
  if (meta_mode(m0) >= kModes) return kUnsupportedMode;
  if (bad) return kErrBadRecord;
  if (meta_nrosters(m0) != 2) return kInvalidRosters;
  if (meta_afk(m1)) return kAfk;
  return kRated;
}

template <int K>
__global__ void __launch_bounds__(256)
rate_dataflow_kernel(const int32_t* __restrict__ rec, const uint2* __restrict__ link,
                     int32_t* deps, float* state, const float* __restrict__ attrs,
                     float* __restrict__ first_prior, RateOut out, uint32_t* ctrl,
                     RateParams prm) {
  constexpr int S = 2 * K;
  constexpr int R = S + 2;
  constexpr int G = S <= 2 ? 2 : (S <= 4 ? 4 : (S <= 8 ? 8 : 16));
  constexpr int NG = 64 / G;
  __shared__ int32_t lrec[kWavesPerBlock][kHeld][kChunk * R];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int j = lane % G;
  const int g = lane / G;
  const int gbase = lane - j;
  const uint64_t gmask = (((1ull << G) - 1ull) << gbase);
  const bool r0 = j < K;
  const int rpos = r0 ? j : j - K;
  const int64_t M = prm.num_matches;
  const int64_t P = prm.num_players;
  const float beta2 = prm.beta2, tau2 = prm.tau2, us = prm.unknown_sigma;
  const uint32_t ehi = (uint32_t)prm.epoch << kTagBits;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(state, 0, (int)(P * kRowFloats * 4), 0x00020000);
  const int head = blockIdx.x % kHeads;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();

  // wave-uniform ring of held chunks
  int64_t cbase[kHeld];
  uint64_t pend[kHeld];
#pragma unroll
  for (int h = 0; h < kHeld; ++h) {
    cbase[h] = -1;
    pend[h] = 0ull;
  }
  bool exhausted = false;
  uint32_t spins = 0;

  for (;;) {
    // -------------------------------------------- claim chunks into free ring slots
#pragma unroll
    for (int h = 0; h < kHeld; ++h) {
      if (cbase[h] < 0 && !exhausted) {
        unsigned t = 0;
        if (lane == 0)
          t = __hip_atomic_fetch_add((gu32*)&ctrl[4 + head], 1u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
        t = __shfl(t, 0);
        const int64_t c = (int64_t)t * kHeads + head;
        if (c * kChunk >= M) {
          exhausted = true;
        } else {
          cbase[h] = c * kChunk;
          const int64_t m = cbase[h] + lane;
          int32_t r[R];
          if (m < M) {
            const int32_t* src = rec + m * R;
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
          } else {
#pragma unroll
            for (int k = 0; k < R; ++k) r[k] = -1;
          }
#pragma unroll
          for (int k = 0; k < R; ++k) lrec[wv][h][lane * R + k] = r[k];
          const uint8_t est = m < M ? early_status<K>(r, P) : kRated;
          if (m < M && est != kRated) {  // no state, no dependencies: finish it now
#pragma unroll
            for (int q = 0; q < S; ++q) {
              out.s_mu[m * S + q] = NAN;
              out.s_sig[m * S + q] = NAN;
              out.delta[m * S + q] = NAN;
              out.m_mu[m * S + q] = NAN;
              out.m_sig[m * S + q] = NAN;
            }
            out.quality[m] = (est == kAfk || est == kInvalidRosters) ? 0.f : NAN;
            out.status[m] = est;
          }
          pend[h] = __ballot(m < M && est == kRated);
          if (pend[h] == 0ull) cbase[h] = -1;  // nothing stateful in this chunk
        }
      }
    }
    bool held = false;
#pragma unroll
    for (int h = 0; h < kHeld; ++h) held |= cbase[h] >= 0;
    if (!held) {
      if (exhausted) break;
      continue;
    }

    // -------------------------------------------- poll the dependency counters
    uint64_t ready[kHeld];
#pragma unroll
    for (int h = 0; h < kHeld; ++h) {
      int d = 1;
      if ((pend[h] >> lane) & 1ull)
        d = (int)__hip_atomic_load((gu32*)(deps + cbase[h] + lane), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
      ready[h] = __ballot(d == 0) & pend[h];
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // later loads stay below the poll

    // -------------------------------------------- oldest ready matches -> groups
    // ring slots are visited in claim order (oldest chunk = smallest base)
    int my_h = -1, my_bit = 0, nassigned = 0;
#pragma unroll
    for (int pass = 0; pass < kHeld; ++pass) {
      // pick the oldest remaining chunk with ready matches
      int best = -1;
      int64_t bb = 0;
#pragma unroll
      for (int h = 0; h < kHeld; ++h)
        if (ready[h] && (best < 0 || cbase[h] < bb)) { best = h; bb = cbase[h]; }
      if (best < 0 || nassigned >= NG) break;
      uint64_t rdy = 0;
#pragma unroll
      for (int h = 0; h < kHeld; ++h) if (h == best) rdy = ready[h];
      const int cnt = __popcll(rdy);
      const int take = cnt < NG - nassigned ? cnt : NG - nassigned;
      if (g >= nassigned && g < nassigned + take) {
        my_h = best;
        my_bit = nth_set_bit(rdy, g - nassigned);
      }
      // clear the taken bits (the lowest `take` set bits)
      uint64_t taken = rdy;
      if (take < cnt) taken &= (nth_set_bit(rdy, take) == 0 ? 0ull : ((1ull << nth_set_bit(rdy, take)) - 1ull));
#pragma unroll
      for (int h = 0; h < kHeld; ++h)
        if (h == best) { pend[h] &= ~taken; ready[h] = 0ull; }
      nassigned += take;
    }

    bool worked = nassigned > 0;
    if (my_h >= 0) {
      // ------------------------------------------ this group's match
      int64_t cb = 0;
#pragma unroll
      for (int h = 0; h < kHeld; ++h) if (h == my_h) cb = cbase[h];
      const int64_t m = cb + my_bit;
      const int32_t* lr = &lrec[wv][my_h][my_bit * R];
      const uint32_t m0 = (uint32_t)lr[S], m1 = (uint32_t)lr[S + 1];
      const int mode = meta_mode(m0), n0 = meta_n0(m0), n1 = meta_n1(m0);
      const int rank0 = meta_winner0(m1) ? 0 : 1, rank1 = meta_winner1(m1) ? 0 : 1;
      const bool inr = j < S && rpos < (r0 ? n0 : n1);
      const int32_t id = inr ? lr[j] : -1;
      int first = j, prevdup = -1;
      bool islast = true;
#pragma unroll
      for (int q = 0; q < S; ++q) {
        const int32_t oid = __shfl(id, gbase + q);
        if (id >= 0 && oid == id) {
          if (q < j) {
            if (first == j) first = q;
            prevdup = q;
          }
          if (q > j) islast = false;
        }
      }
      const bool own = inr && first == j;
      const uint2 lk = inr ? link[m * S + j] : make_uint2(0u, 0xffffffffu);
      v4i gs = {0, 0, 0, 0}, gm = {0, 0, 0, 0};
      const int off = id * (kRowFloats * 4);
      if (own) {
        gs = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
        gm = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * (1 + mode), 0, 16);
        // belt and braces: the shared granule must carry the previous occurrence's tag
        for (uint32_t tries = 0; lk.x != 0u && ((uint32_t)gs.y != (ehi | lk.x) ||
                                                 (uint32_t)gs.w != (ehi | lk.x)); ++tries) {
          if (tries > 1000000u) {
            atomicOr(&ctrl[2], 1u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          gs = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
          gm = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * (1 + mode), 0, 16);
        }
      }
      const float smu = __int_as_float(gs.x), ssg = __int_as_float(gs.z);
      const float mmu = __int_as_float(gm.x), msg = __int_as_float(gm.z);
      float pms = 0.f, pss = 1.f, pmm = 0.f, psm = 1.f;
      uint32_t pflags = 0;
      uint8_t lst = kRated;
      if (own)
        lst = player_prior<float>(smu, ssg, mmu, msg, attrs + (int64_t)id * 4, us, prm.vst, pms,
                                  pss, pmm, psm, pflags);
      const uint64_t eb = __ballot(lst != kRated) & gmask;
      uint8_t gst = kRated;
      if (eb) gst = (uint8_t)__shfl((int)lst, (int)__builtin_ctzll(eb));
      // duplicates see the pre-match values of their first occurrence
      const int src = gbase + first;
      pms = __shfl(pms, src);
      pss = __shfl(pss, src);
      pmm = __shfl(pmm, src);
      psm = __shfl(psm, src);
      pflags = (uint32_t)__shfl((int)pflags, src);
      const float rsmu = __shfl(smu, src), rssg = __shfl(ssg, src);
      const float rmmu = __shfl(mmu, src), rmsg = __shfl(msg, src);
      if (gst == kRated && (n0 == 0 || n1 == 0)) gst = kErrEmptyRoster;
      float nsm = NAN, nss = NAN, nmm = NAN, nms = NAN, dl = NAN, q = NAN;
      if (gst == kRated) {
        const float sgn = r0 ? 1.f : -1.f;
        const float s_c2 = group_sum<G>(inr ? pss * pss + tau2 : 0.f);
        const float s_d = group_sum<G>(inr ? sgn * pms : 0.f);
        const float m_c2 = group_sum<G>(inr ? psm * psm + tau2 : 0.f);
        const float m_d = group_sum<G>(inr ? sgn * pmm : 0.f);
        const float m_q = group_sum<G>(inr ? psm * psm : 0.f);
        const int n = n0 + n1;
        const float nb2 = (float)n * beta2;
        q = quality_from_sums<float>(n, m_q, m_d, beta2);
        const UpdCoef<float> ks = update_coef<float>(s_d, nb2 + s_c2, rank0, rank1);
        const UpdCoef<float> km = update_coef<float>(m_d, nb2 + m_c2, rank0, rank1);
        apply_coef<float>(ks, r0, pms, pss, tau2, nsm, nss);
        apply_coef<float>(km, r0, pmm, psm, tau2, nmm, nms);
        const bool bad_num = inr && !(isfinite(nsm) && isfinite(nss) && isfinite(nmm) &&
                                      isfinite(nms) && isfinite(q));
        if ((__ballot(bad_num) & gmask) != 0ull) gst = kErrNumeric;
        // conservative-skill delta (rater.py:150-153), in slot (= write) order
        const float cur = nsm - nss;
        const float prevw = __shfl(cur, gbase + (prevdup >= 0 ? prevdup : j));
        if (prevdup >= 0) dl = cur - prevw;
        else if (pflags & 1u) dl = cur - (pms - pss);
        else dl = 0.f;
      }
      const bool ok = gst == kRated && inr;
      if (inr && islast) {  // publish: new values, or the untouched ones on error
        const uint32_t tag = ehi | (lk.x + 1u);
        __builtin_amdgcn_raw_buffer_store_b128(ok ? granule(nmm, tag, nms) : granule(rmmu, tag, rmsg),
                                               rs, off + 16 * (1 + mode), 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(ok ? granule(nsm, tag, nss) : granule(rsmu, tag, rssg),
                                               rs, off, 0, 16);
      }
      if (ok && prm.record_first_prior && own) {
        float* fp = first_prior + (int64_t)id * kRowFloats;
        if (pflags & 2u) { fp[0] = pms; fp[2] = pss; }
        if (pflags & 4u) { fp[4 * (1 + mode)] = pmm; fp[4 * (1 + mode) + 2] = psm; }
      }
      if (j < S) {
        out.s_mu[m * S + j] = ok ? nsm : NAN;
        out.s_sig[m * S + j] = ok ? nss : NAN;
        out.delta[m * S + j] = ok ? dl : NAN;
        out.m_mu[m * S + j] = ok ? nmm : NAN;
        out.m_sig[m * S + j] = ok ? nms : NAN;
      }
      if (j == 0) {
        out.quality[m] = gst == kRated ? q : NAN;
        out.status[m] = gst;
      }
      // release: every store of this wave has landed before a successor is notified
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (inr && islast && lk.y != 0xffffffffu)
        __hip_atomic_fetch_add((gu32*)(deps + lk.y / S), 0xffffffffu, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }

    // -------------------------------------------- retire finished chunks
#pragma unroll
    for (int h = 0; h < kHeld; ++h)
      if (cbase[h] >= 0 && pend[h] == 0ull) cbase[h] = -1;

    if (worked) {
      spins = 0;
    } else {
      if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks) {
        if (lane == 0) atomicOr(&ctrl[1], 1u);
#pragma unroll
        for (int h = 0; h < kHeld; ++h)
          if (cbase[h] >= 0 && ((pend[h] >> lane) & 1ull)) out.status[cbase[h] + lane] = kNotProcessed;
        return;  // give up: the host sees ctrl[1] and raises
      }
      spins = spins < 8u ? spins + 1u : 8u;
      for (uint32_t k = 0; k < spins; ++k) __builtin_amdgcn_s_sleep(2);
    }
  }
}

int launch_rate(int K, const int32_t* rec, const uint32_t* link, int32_t* deps, float* state,
                const float* attrs, float* first_prior, const RateOut& out, uint32_t* ctrl,
                const RateParams& prm, int blocks, hipStream_t s) {
  const int64_t M = prm.num_matches;
  // ctrl[0] = schedule overflow (kept), [1] timeout, [2] protocol, [3] spare, [4..11] tickets
  ANA_HIP_CHECK(hipMemsetAsync(ctrl + 1, 0, 11 * 4, s));
  if (M <= 0) return 0;
  if ((int64_t)prm.num_players * kRowFloats * 4 >= 0x7fffffffLL) return (int)hipErrorInvalidValue;
  if (prm.epoch < 1 || prm.epoch > 255) return (int)hipErrorInvalidValue;
  if (blocks < kHeads) blocks = kHeads;
  const uint2* link2 = reinterpret_cast<const uint2*>(link);
  switch (K) {
#define ANA_RATE_CASE(k)                                                                      \
  case k:                                                                                     \
    hipLaunchKernelGGL(rate_dataflow_kernel<k>, dim3((unsigned)blocks), dim3(256), 0, s, rec,  \
                       link2, deps, state, attrs, first_prior, out, ctrl, prm);               \
    break;
    ANA_RATE_CASE(1) ANA_RATE_CASE(2) ANA_RATE_CASE(3) ANA_RATE_CASE(4) ANA_RATE_CASE(5)
#undef ANA_RATE_CASE
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace ana
