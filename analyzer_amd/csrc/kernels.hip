// MI355X (gfx950) kernels of the rating engine.
//
//  K7  gen_roster_kernel / gen_stream_kernel  synthetic inputs (counter RNG)
//  K5  schedule: per-slot occurrence index = how many earlier rated matches
//      of the stream the same player is in.  Stable radix sort of (player,
//      slot) pairs (hipCUB/rocPRIM onesweep) + two linear passes.
//  K1-K4+K3+K6  rate_dataflow_kernel: one persistent launch rates the whole
//      stream in exact chronological-per-player order without rounds or grid
//      barriers: a wave claims 64 consecutive matches (one per lane) from a
//      monotone ticket, each lane waits until every player's version counter
//      equals the slot's occurrence index, then gathers, seeds, rates both
//      tracks, scatters, and releases the versions.  Claims are monotone, so
//      the oldest unfinished match is always runnable: no deadlock whatever the
//      residency.  Hand-off protocol = MI355X_MICROARCH "Valid forms", row 1:
//      sc1 (write-through) state stores -> s_waitcnt vmcnt(0) -> sc1 version
//      store; consumer polls the version with sc1 loads and reads state with
//      sc1 loads only (no L1-resident stale copy can be observed).
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
typedef __attribute__((address_space(1))) unsigned long long gu64;

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
  float st[16], at[4];
  gen_player(g, p, st, at);
  float4* s4 = reinterpret_cast<float4*>(state + p * 16);
#pragma unroll
  for (int k = 0; k < 4; ++k) s4[k] = make_float4(st[4 * k], st[4 * k + 1], st[4 * k + 2], st[4 * k + 3]);
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

// ------------------------------------------------------------------- schedule
// Slots of matches that touch no state (unsupported mode, rosters != 2, AFK)
// are keyed past the last player so they neither wait nor release.
template <int K>
__global__ void sched_keys_kernel(const int32_t* __restrict__ rec, int64_t M, uint32_t P,
                                  uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  constexpr int S = 2 * K;
  const int32_t* r = rec + m * (S + 2);
  MatchWork<float, K> w;
  decode_record<float, K>(r, (int64_t)P, w);  // same early outcome as the rate kernel
  const bool rates = w.status == kRated;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    keys[m * S + j] = rates && w.id[j] >= 0 ? (uint32_t)w.id[j] : P;
    vals[m * S + j] = (uint32_t)(m * S + j);
  }
}

__global__ void sched_segstart_kernel(const uint32_t* __restrict__ keys, int64_t n, uint32_t P,
                                      uint32_t* __restrict__ segstart) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = keys[i];
  if (k < P && (i == 0 || keys[i - 1] != k)) segstart[k] = (uint32_t)i;
}

__global__ void sched_occ_kernel(const uint32_t* __restrict__ keys,
                                 const uint32_t* __restrict__ vals, int64_t n, uint32_t P,
                                 const uint32_t* __restrict__ segstart, uint32_t* __restrict__ occ) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = keys[i];
  if (k < P) occ[vals[i]] = (uint32_t)i - segstart[k];
}

static int key_bits(uint32_t P) {
  int b = 1;
  while (b < 32 && (1ull << b) <= (uint64_t)P) ++b;
  return b;
}

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

size_t schedule_workspace_bytes(int64_t nslots, int64_t num_players) {
  size_t cub_bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (uint32_t*)nullptr, (uint32_t*)nullptr, (int)nslots, 0,
                                     key_bits((uint32_t)num_players));
  return 4 * align_up(nslots * 4) + align_up((num_players + 1) * 4) + align_up(cub_bytes);
}

int launch_schedule(int K, const int32_t* rec, int64_t M, int64_t P, uint32_t* occ, void* ws,
                    size_t ws_bytes, hipStream_t s) {
  const int64_t n = M * 2 * K;
  if (n <= 0) return 0;
  if (n > 0x7fffffffLL || P >= 0x7fffffffLL) return (int)hipErrorInvalidValue;
  char* p = static_cast<char*>(ws);
  uint32_t* keys_in = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* keys_out = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* vals_in = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* vals_out = reinterpret_cast<uint32_t*>(p); p += align_up(n * 4);
  uint32_t* segstart = reinterpret_cast<uint32_t*>(p); p += align_up((P + 1) * 4);
  size_t cub_bytes = ws_bytes - (size_t)(p - static_cast<char*>(ws));
  const unsigned mb = (unsigned)((M + 255) / 256);
  switch (K) {
#define ANA_KEY_CASE(k)                                                                        \
  case k:                                                                                      \
    hipLaunchKernelGGL(sched_keys_kernel<k>, dim3(mb), dim3(256), 0, s, rec, M, (uint32_t)P,    \
                       keys_in, vals_in);                                                      \
    break;
    ANA_KEY_CASE(1) ANA_KEY_CASE(2) ANA_KEY_CASE(3) ANA_KEY_CASE(4) ANA_KEY_CASE(5)
#undef ANA_KEY_CASE
    default: return (int)hipErrorInvalidValue;
  }
  ANA_HIP_CHECK(hipGetLastError());
  ANA_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(p, cub_bytes, keys_in, keys_out, vals_in,
                                                   vals_out, (int)n, 0, key_bits((uint32_t)P), s));
  const unsigned nb = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(sched_segstart_kernel, dim3(nb), dim3(256), 0, s, keys_out, n, (uint32_t)P,
                     segstart);
  hipLaunchKernelGGL(sched_occ_kernel, dim3(nb), dim3(256), 0, s, keys_out, vals_out, n,
                     (uint32_t)P, segstart, occ);
  return (int)hipGetLastError();
}

// --------------------------------------------------------------- rate (dataflow)
__device__ __forceinline__ float2 ld_state(const float2* p) {
  const unsigned long long b =
      __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float2(__uint_as_float((unsigned)b), __uint_as_float((unsigned)(b >> 32)));
}
__device__ __forceinline__ void st_state(float2* p, float mu, float sig) {
  const unsigned long long b =
      (unsigned long long)__float_as_uint(mu) | ((unsigned long long)__float_as_uint(sig) << 32);
  __hip_atomic_store((gu64*)p, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ld_ver(const uint32_t* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ver(uint32_t* p, unsigned v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 5 s at the 100 MHz s_memrealtime clock: a stuck wave gives up, reports, exits
constexpr uint64_t kTimeoutTicks = 500000000ull;
// matches claimed per wave per ticket (amortises the ticket atomic, MICROARCH "dequeue")
constexpr int kChunk = 256;

// Sum over the G lanes of this lane's group (groups are aligned, G | 64).
template <int G>
__device__ __forceinline__ float group_sum(float x) {
#pragma unroll
  for (int off = G / 2; off >= 1; off >>= 1) x += __shfl_xor(x, off);
  return x;
}

// One match per group of G lanes, one roster slot per lane (lanes j >= 2K idle).
// A wave claims kChunk consecutive matches; group g walks matches
// base + g, base + g + NG, ... in order, so each group is a strictly ordered
// worker and the oldest unfinished claimed match is always runnable.
template <int K>
__global__ void __launch_bounds__(256)
rate_dataflow_kernel(const int32_t* __restrict__ rec, const uint32_t* __restrict__ occ,
                     float2* state, const float* __restrict__ attrs, uint32_t* ver,
                     float2* __restrict__ first_prior, RateOut out, uint32_t* ctrl,
                     RateParams prm) {
  constexpr int S = 2 * K;
  constexpr int R = S + 2;
  constexpr int G = S <= 2 ? 2 : (S <= 4 ? 4 : (S <= 8 ? 8 : 16));
  constexpr int NG = 64 / G;
  constexpr int PER = kChunk / NG;
  const int lane = threadIdx.x & 63;
  const int g = lane / G;
  const int j = lane % G;
  const int gbase = g * G;
  const uint64_t gmask = (G == 64) ? ~0ull : (((1ull << G) - 1ull) << gbase);
  const bool r0 = j < K;
  const int rpos = r0 ? j : j - K;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const float beta2 = prm.beta2, tau2 = prm.tau2, us = prm.unknown_sigma;
  const int64_t M = prm.num_matches;
  const int64_t P = prm.num_players;

  for (;;) {
    unsigned chunk = 0;
    if (lane == 0)
      chunk = __hip_atomic_fetch_add((gu32*)&ctrl[0], 1u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
    chunk = __shfl(chunk, 0);
    const int64_t cbase = (int64_t)chunk * kChunk;
    if (cbase >= M) break;

    int i = 0;            // position in this group's sequence
    bool loaded = false;  // current match decoded
    // per-match lane state (uniform within the group except the per-slot fields)
    int64_t m = 0;
    int32_t id = -1;
    uint32_t o = 0;
    int mode = 0, n0 = 0, n1 = 0, rank0 = 1, rank1 = 1, first = 0, prevdup = -1;
    bool inr = false, islast = false, stateful = false, ready = true;

    for (;;) {
      const bool gdone = i >= PER || cbase + (int64_t)i * NG + g >= M;
      if (__all(gdone)) break;
      bool progressed = false;
      if (!gdone && !loaded) {
        m = cbase + (int64_t)i * NG + g;
        const int32_t* rr = rec + m * R;
        const uint32_t m0 = (uint32_t)rr[S], m1 = (uint32_t)rr[S + 1];
        const int32_t raw = j < S ? rr[j] : -1;
        mode = meta_mode(m0);
        n0 = meta_n0(m0);
        n1 = meta_n1(m0);
        rank0 = meta_winner0(m1) ? 0 : 1;
        rank1 = meta_winner1(m1) ? 0 : 1;
        inr = j < S && rpos < (r0 ? n0 : n1);
        const bool bad_slot = inr && (raw < 0 || (int64_t)raw >= P);
        id = inr && !bad_slot ? raw : -1;
        const bool bad = (__ballot(bad_slot) & gmask) != 0 || n0 > K || n1 > K;
        uint8_t est = kRated;
        if (mode >= kModes) est = kUnsupportedMode;
        else if (bad) est = kErrBadRecord;
        else if (meta_nrosters(m0) != 2) est = kInvalidRosters;
        else if (meta_afk(m1)) est = kAfk;
        stateful = est == kRated;
        // duplicates of one player inside the match (rater.py writes in slot order)
        first = j;
        prevdup = -1;
        islast = true;
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
        if (stateful) {
          o = inr ? occ[m * S + j] : 0u;
          ready = !(inr && first == j);  // only first occurrences wait
        } else {
          // early outcome: no state, no versions
          if (j < S) {
            out.s_mu[m * S + j] = NAN;
            out.s_sig[m * S + j] = NAN;
            out.delta[m * S + j] = NAN;
            out.m_mu[m * S + j] = NAN;
            out.m_sig[m * S + j] = NAN;
          }
          if (j == 0) {
            out.quality[m] = (est == kAfk || est == kInvalidRosters) ? 0.f : NAN;
            out.status[m] = est;
          }
          ++i;
          progressed = true;
        }
        loaded = stateful;
      }
      if (!gdone && loaded && !ready) {
        const unsigned v = ld_ver(ver + id);
        if (v == o) ready = true;
        else if (v > o) atomicOr(&ctrl[2], 1u);  // protocol violation
      }
      const uint64_t rb = __ballot(!gdone && loaded && ready);
      if ((rb & gmask) == gmask) {
        // ---------------- whole group ready: gather, seed, rate, scatter, release
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // loads stay below the poll
        const bool own = inr && first == j;
        float2 sh = make_float2(NAN, NAN), md = make_float2(NAN, NAN);
        if (own) {
          sh = ld_state(state + (int64_t)id * kTrackStride);
          md = ld_state(state + (int64_t)id * kTrackStride + 1 + mode);
        }
        float pms = 0.f, pss = 1.f, pmm = 0.f, psm = 1.f;
        uint32_t pflags = 0;
        uint8_t lst = kRated;
        if (own)
          lst = player_prior<float>(sh.x, sh.y, md.x, md.y, attrs + (int64_t)id * 4, us, prm.vst,
                                    pms, pss, pmm, psm, pflags);
        const uint64_t eb = __ballot(lst != kRated) & gmask;
        uint8_t gst = kRated;
        if (eb) gst = (uint8_t)__shfl((int)lst, (int)(__builtin_ctzll(eb)));
        // duplicates read the pre-match prior of their first occurrence
        pms = __shfl(pms, gbase + first);
        pss = __shfl(pss, gbase + first);
        pmm = __shfl(pmm, gbase + first);
        psm = __shfl(psm, gbase + first);
        pflags = (uint32_t)__shfl((int)pflags, gbase + first);
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
          if ((__ballot(bad_num) & gmask) != 0) gst = kErrNumeric;
          // conservative-skill delta (rater.py:150-153), in slot (= write) order
          const float cur = nsm - nss;
          const float prevw = __shfl(cur, gbase + (prevdup >= 0 ? prevdup : j));
          if (prevdup >= 0) dl = cur - prevw;
          else if (pflags & 1u) dl = cur - (pms - pss);
          else dl = 0.f;
        }
        if (gst == kRated && inr) {
          if (islast) {
            float2* rowp = state + (int64_t)id * kTrackStride;
            st_state(rowp, nsm, nss);
            st_state(rowp + 1 + mode, nmm, nms);
          }
          if (prm.record_first_prior && own) {
            float2* fp = first_prior + (int64_t)id * kTrackStride;
            if (pflags & 2u) fp[0] = make_float2(pms, pss);
            if (pflags & 4u) fp[1 + mode] = make_float2(pmm, psm);
          }
        }
        // every state store of this lane has left before its version moves;
        // a lane only releases the player it stored (or an untouched one)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (inr && islast) st_ver(ver + id, o + 1u);
        const bool ok = gst == kRated && inr;
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
        ++i;
        loaded = false;
        ready = true;
        progressed = true;
      }
      if (!__any(progressed)) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks) {
          if (!gdone && j == 0) out.status[m] = kNotProcessed;
          if (lane == 0) atomicOr(&ctrl[1], 1u);
          return;  // give up: the host sees ctrl[1] and raises
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }
}

int launch_rate(int K, const int32_t* rec, const uint32_t* occ, float* state, const float* attrs,
                uint32_t* ver, float* first_prior, const RateOut& out, uint32_t* ctrl,
                const RateParams& prm, int max_blocks, hipStream_t s) {
  const int64_t M = prm.num_matches;
  ANA_HIP_CHECK(hipMemsetAsync(ver, 0, (size_t)prm.num_players * 4, s));
  ANA_HIP_CHECK(hipMemsetAsync(ctrl, 0, 16, s));
  if (M <= 0) return 0;
  const int64_t chunks = (M + 63) / 64;
  int64_t blocks = (chunks + 3) / 4;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  float2* st2 = reinterpret_cast<float2*>(state);
  float2* fp2 = reinterpret_cast<float2*>(first_prior);
  switch (K) {
#define ANA_RATE_CASE(k)                                                                      \
  case k:                                                                                     \
    hipLaunchKernelGGL(rate_dataflow_kernel<k>, dim3((unsigned)blocks), dim3(256), 0, s, rec, \
                       occ, st2, attrs, ver, fp2, out, ctrl, prm);                            \
    break;
    ANA_RATE_CASE(1) ANA_RATE_CASE(2) ANA_RATE_CASE(3) ANA_RATE_CASE(4) ANA_RATE_CASE(5)
#undef ANA_RATE_CASE
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace ana
