// K5 device levelizer: the conflict-free round of every match of a window, for
// the exact data-parallel mode (parallel/exact_dp.py).
//
//   level[m] = 0                                   if m touches no state
//            = 1 + max level of its players' previous matches   otherwise
//
// (host mirror: host.cpp levels_k, which walks the window in order.)  On the
// device the same recurrence runs as a dataflow over the schedule the rating
// uses (radix prepass: link[m][j] = the next match of slot j's player | has an
// earlier one; deps[m] zeroed): a match is final once every distinct player
// with an earlier occurrence has notified it.  It then pushes its level to the
// next match of each of its players (atomicMax into pushed[]), waits for those
// atomics, and bumps that match's counter.  Readers poll their counter and read pushed[]
// after it, so every push they need has landed.  Lane = match: a wave claims
// 64-match chunks (one ticket counter), holds up to four, and polls them with
// coalesced loads -- a 10M-match 3v3 window (~900 levels) takes milliseconds,
// where the host walk takes a fraction of a second.
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"

namespace ana {

namespace {

constexpr int kLvlHeld = 4;
constexpr int kLvlBlocks = 512;
constexpr int kLvlThreads = 256;
constexpr uint64_t kLvlTimeoutTicks = 500000000ull;  // 5 s of s_memrealtime (100 MHz) without progress

typedef unsigned int gu32 __attribute__((address_space(1)));

// ctrl: [0] chunk ticket, [1] retired chunks (progress), [2] depth (max level), [3] error flag
template <int K>
__global__ void __launch_bounds__(kLvlThreads)
levels_kernel(const int32_t* __restrict__ rec, const uint32_t* __restrict__ link, int32_t* deps,
              int32_t* pushed, int32_t* __restrict__ level, int64_t M, int64_t P, uint32_t* ctrl) {
  constexpr int S = 2 * K;
  constexpr int R = S + 2;
  const int lane = threadIdx.x & 63;
  int64_t cbase[kLvlHeld];
  uint64_t pend[kLvlHeld];
  uint32_t need[kLvlHeld];
  uint32_t pub[kLvlHeld][S];  // per slot: the match this match notifies (kNoMatch: none)
#pragma unroll
  for (int h = 0; h < kLvlHeld; ++h) {
    cbase[h] = -1;
    pend[h] = 0ull;
    need[h] = 0u;
#pragma unroll
    for (int a = 0; a < S; ++a) pub[h][a] = kNoMatch;
  }
  bool exhausted = false;
  int32_t depth = 0;
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t seen = 0, spins = 0;
  for (;;) {
    // ---- claim a chunk into a free slot
    int free_h = -1;
#pragma unroll
    for (int h = kLvlHeld - 1; h >= 0; --h)
      if (cbase[h] < 0) free_h = h;
    bool claimed = false;
    if (free_h >= 0 && !exhausted) {
      unsigned t = 0;
      if (lane == 0)
        t = __hip_atomic_fetch_add((gu32*)&ctrl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t = __builtin_amdgcn_readfirstlane(t);
      const int64_t c0 = (int64_t)t * 64;
      if (c0 >= M) {
        exhausted = true;
      } else {
        claimed = true;
        const int64_t m = c0 + lane;
        bool rated = false;
        uint32_t nd = 0u;
        uint32_t pb[S];
#pragma unroll
        for (int a = 0; a < S; ++a) pb[a] = kNoMatch;
        if (m < M) {
          int32_t r[R];
#pragma unroll
          for (int k = 0; k < R; ++k) r[k] = rec[m * R + k];
          if (early_status<K>(r, P) == kRated) {
            rated = true;
            uint32_t lk[S];
#pragma unroll
            for (int a = 0; a < S; ++a) lk[a] = link[m * S + a];
            const uint32_t m0 = (uint32_t)r[S];
            // in-roster slots carry players (the schedule keyed exactly these); a player
            // named twice counts once (its first slot) and notifies once (its last slot)
#pragma unroll
            for (int a = 0; a < S; ++a) {
              const bool ina = (a < K ? a : a - K) < (a < K ? meta_n0(m0) : meta_n1(m0));
              bool firsto = ina, lasto = ina;
#pragma unroll
              for (int b = 0; b < S; ++b) {
                const bool inb = (b < K ? b : b - K) < (b < K ? meta_n0(m0) : meta_n1(m0));
                if (b < a && inb && r[b] == r[a]) firsto = false;
                if (b > a && inb && r[b] == r[a]) lasto = false;
              }
              if (firsto && (lk[a] & kLinkHasPred)) ++nd;
              if (lasto) pb[a] = lk[a] & kMatchMask;
            }
          } else {
            level[m] = 0;  // no state: goes with round 1 (exact_dp.RoundPlan)
          }
        }
        const uint64_t pm = __ballot(rated);
#pragma unroll
        for (int h = 0; h < kLvlHeld; ++h)
          if (h == free_h) {
            cbase[h] = pm ? c0 : -1;
            pend[h] = pm;
            need[h] = nd;
#pragma unroll
            for (int a = 0; a < S; ++a) pub[h][a] = pb[a];
          }
        if (!pm && lane == 0)
          __hip_atomic_fetch_add((gu32*)&ctrl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }

    // ---- poll the held matches, finish the ready ones.  No cache-maintaining
    // fences: the counters and pushed[] are only touched by device-scope atomics
    // (performed past the per-XCD L2s), so ordering needs just the issue order on
    // the reader (its pushed[] loads follow the polls they depend on) and a wait
    // for the pushes' acknowledgements before the notifies on the writer.
    uint32_t d[kLvlHeld];
#pragma unroll
    for (int h = 0; h < kLvlHeld; ++h) {
      d[h] = 0xffffffffu;
      if (cbase[h] >= 0 && ((pend[h] >> lane) & 1ull))
        d[h] = __hip_atomic_load((gu32*)(deps + cbase[h] + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    bool rdy[kLvlHeld];
    uint64_t rb[kLvlHeld];
    bool worked = false;
#pragma unroll
    for (int h = 0; h < kLvlHeld; ++h) {
      rdy[h] = cbase[h] >= 0 && ((pend[h] >> lane) & 1ull) && d[h] == need[h];
      rb[h] = __ballot(rdy[h]);
      worked |= rb[h] != 0ull;
    }
    if (worked) {
      asm volatile("" ::: "memory");
      int32_t l[kLvlHeld];
#pragma unroll
      for (int h = 0; h < kLvlHeld; ++h)
        l[h] = rdy[h] ? (int32_t)__hip_atomic_load((gu32*)(pushed + cbase[h] + lane), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT) + 1
                      : 0;
#pragma unroll
      for (int h = 0; h < kLvlHeld; ++h) {
        if (!rdy[h]) continue;
        level[cbase[h] + lane] = l[h];
        depth = l[h] > depth ? l[h] : depth;
#pragma unroll
        for (int a = 0; a < S; ++a)
          if (pub[h][a] != kNoMatch)
            __hip_atomic_fetch_max(pushed + pub[h][a], l[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the pushes land before the notifies
#pragma unroll
      for (int h = 0; h < kLvlHeld; ++h) {
        if (rdy[h]) {
#pragma unroll
          for (int a = 0; a < S; ++a)
            if (pub[h][a] != kNoMatch)
              __hip_atomic_fetch_add((gu32*)(deps + pub[h][a]), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        pend[h] &= ~rb[h];
        if (cbase[h] >= 0 && pend[h] == 0ull) {
          cbase[h] = -1;
          if (lane == 0)
            __hip_atomic_fetch_add((gu32*)&ctrl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }

    bool held = false;
#pragma unroll
    for (int h = 0; h < kLvlHeld; ++h) held |= cbase[h] >= 0;
    if (exhausted && !held) break;
    if (worked || claimed) {
      spins = 0;
      continue;
    }
    // ---- nothing ready: back off; give up after kLvlTimeoutTicks without any chunk retiring
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    const uint32_t p = __hip_atomic_load((gu32*)&ctrl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (p != seen) {
      seen = p;
      t0 = now;
    } else if (now - t0 > kLvlTimeoutTicks) {
      if (lane == 0) atomicOr(&ctrl[3], 1u);
      break;
    }
    spins = spins < 8u ? spins + 1u : 8u;
    for (uint32_t k = 0; k < spins; ++k) __builtin_amdgcn_s_sleep(2);
  }
  // wave maximum -> ctrl[2]
  for (int off = 32; off >= 1; off >>= 1) {
    const int32_t o = __shfl_xor(depth, off);
    depth = o > depth ? o : depth;
  }
  if (lane == 0 && depth > 0)
    __hip_atomic_fetch_max((gu32*)&ctrl[2], (unsigned)depth, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

int launch_levels(int K, const int32_t* rec, const uint32_t* link, int32_t* deps, int32_t* pushed,
                  int32_t* level, int64_t M, int64_t P, uint32_t* ctrl, hipStream_t s) {
  if (M <= 0) return 0;
  if (M * 2 * K > kMaxSlots) return (int)hipErrorInvalidValue;
  const int64_t chunks = (M + 63) / 64;
  const int64_t waves = chunks < (int64_t)kLvlBlocks * 4 ? chunks : (int64_t)kLvlBlocks * 4;
  const dim3 grid((unsigned)((waves + 3) / 4)), block(kLvlThreads);
  switch (K) {
#define ANA_LVL_CASE(k) \
  case k: hipLaunchKernelGGL((levels_kernel<k>), grid, block, 0, s, rec, link, deps, pushed, level, M, P, ctrl); break;
    ANA_LVL_CASE(1) ANA_LVL_CASE(2) ANA_LVL_CASE(3) ANA_LVL_CASE(4) ANA_LVL_CASE(5)
#undef ANA_LVL_CASE
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace ana
