// Split-role dataflow executor (ANA_RATE_SPLIT=1/2) -- diagnostic library only
// (python -m analyzer_amd.build_ext --diag): the production build compiles this
// file to nothing and launch_rate refuses ANA_RATE_SPLIT.
#include <hip/hip_runtime.h>

#include "common.h"
#include "dataflow_dev.h"
#include "kernels.h"
#include "rate_core.h"

#if ANA_DIAG_BUILD
namespace ana {

// ---------------------------------------------------------------------------
// Split-role executor (ANA_RATE_SPLIT=1/2, windows only; diagnostic library).
// Bit-identical to rate_dataflow_kernel and not faster: 10M 3v3 window 6.43 ms
// (8 held chunks) vs 6.52, 7.56 ms with 16; serial hop 3.1 / 5.5 us vs 2.3 --
// the scheduler's poll round trip replaces the rater's, and a local hand-off
// now goes rater -> LDS -> scheduler -> queue -> rater
// (profiles/r2/split_executor_experiment.log).  Each workgroup has one
// SCHEDULER wave and three RATER waves.  The scheduler holds kSplitHeld chunks
// (records in LDS), polls their completion counters in a loop of its own and
// pushes every ready match into an LDS ready queue; the raters pop up to NG
// matches at a time, gather, rate, publish and notify -- the same per-match
// protocol as rate_dataflow_kernel (tagged granules, no store round trip,
// local hand-off through LDS counters for successors this workgroup holds).
// A rater's iteration carries none of the readiness / assignment / polling /
// ticket bookkeeping, and readiness is seen one scheduler loop (one poll round
// trip) after the notify instead of one rater iteration.
// Slot reuse: a chunk slot is free once every match of it was enqueued (no
// pending lane) and every enqueued entry was read by a rater (lused == lenq).
constexpr int kSplitQ = 512;  // ready-queue entries (power of two)

template <int K, int G, int H>
__global__ void __launch_bounds__(256)
rate_split_kernel(const int32_t* __restrict__ rec, const uint32_t* __restrict__ link,
                  int32_t* deps, float* state, const float* __restrict__ attrs,
                  float* __restrict__ first_prior, float* __restrict__ orows, int64_t orow,
                  uint32_t* ctrl, RateParams prm) {
  constexpr int S = 2 * K;
  constexpr int R = S + 2;
  constexpr int NG = 64 / G;
  static_assert(G >= S && G <= 64, "a group holds one match");
  __shared__ int32_t lrec[H][kChunk][R];  // records of the held chunks
  __shared__ __attribute__((aligned(16))) uint32_t lloc[kChunk][H];  // local hand-off counts, [lane][slot]
  __shared__ __attribute__((aligned(16))) int32_t lcb[H];  // chunk bases (-1: free)
  __shared__ uint32_t lused[H];           // entries of slot h read by raters
  __shared__ uint32_t q[kSplitQ];         // ready queue: h << 8 | lane
  __shared__ uint32_t qhead, qtail, sdone;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t M = prm.num_matches;
  const int64_t P = prm.num_players;
  const int epoch = prm.epoch_ptr ? __builtin_amdgcn_readfirstlane(*prm.epoch_ptr) : prm.epoch;
  const int cl = prm.chunk_len;
  if (threadIdx.x < H) {
    lcb[threadIdx.x] = -1;
    lused[threadIdx.x] = 0u;
  }
  if (threadIdx.x == 0) {
    qhead = 0u;
    qtail = 0u;
    sdone = 0u;
  }
  __syncthreads();
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t seen_progress = 0;
  auto timed_out = [&](bool busy) -> bool {  // watchdog: 5 s without any chunk retiring GPU-wide
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (busy) return false;
    if (now - t0 > kProgressTicks) {
      const uint32_t p = __hip_atomic_load((gu32*)&ctrl[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (p != seen_progress) {
        seen_progress = p;
        t0 = now;
      }
    }
    return now - t0 > kTimeoutTicks;
  };

  if (wv == 0) {
    // ================================================================ scheduler
    const int head = blockIdx.x % kHeads;
    int32_t cbase[H];
    uint32_t dval[H], need[H], lenq[H];
    uint32_t pbits = 0u;  // per lane: bit h = match cbase[h] + lane is stateful and not yet enqueued
#pragma unroll
    for (int h = 0; h < H; ++h) {
      cbase[h] = -1;
      dval[h] = kNone;
      need[h] = 0u;
      lenq[h] = 0u;
    }
    bool exhausted = false, tk_pending = false, timeout = false;
    unsigned tk = 0;
    uint32_t tail = 0u, iter = 0u;
    for (;;) {
      ++iter;
      // ---- readiness (local counts: H/4 vector LDS reads) and enqueue
      uint32_t rbits = 0u;
      {
        uint32_t loc[H];
#pragma unroll
        for (int v = 0; v < H / 4; ++v) {
          const uint4 x = reinterpret_cast<const uint4*>(&lloc[lane][0])[v];
          loc[4 * v] = x.x; loc[4 * v + 1] = x.y; loc[4 * v + 2] = x.z; loc[4 * v + 3] = x.w;
        }
#pragma unroll
        for (int h = 0; h < H; ++h)
          rbits |= (((pbits >> h) & 1u) && dval[h] != kNone && dval[h] + loc[h] == need[h]) ? 1u << h : 0u;
      }
      const uint32_t rmask = wave_or(rbits);  // wave-uniform: chunks with a ready lane
      bool worked = false;
      if (rmask != 0u) {
        const uint32_t hd = __hip_atomic_load(&qhead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        uint32_t space = (uint32_t)kSplitQ - (tail - hd);
#pragma unroll
        for (int h = 0; h < H; ++h) {
          if (!((rmask >> h) & 1u)) continue;
          const uint64_t b = __ballot((rbits >> h) & 1u);
          const uint32_t n = (uint32_t)__popcll(b);
          if (n <= space) {
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
            if ((rbits >> h) & 1u) {
              q[(tail + rank) & (kSplitQ - 1)] = ((uint32_t)h << 8) | (uint32_t)lane;
              pbits &= ~(1u << h);
            }
            tail += n;
            space -= n;
            lenq[h] += n;
            worked = true;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // entries before the tail
        if (lane == 0) __hip_atomic_store(&qtail, tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      // ---- a ticket came back: load its chunk (retired below the wait)
      int staging = -1;
      int32_t r[R];
      uint32_t lks[S];
#pragma unroll
      for (int k = 0; k < R; ++k) r[k] = -1;
#pragma unroll
      for (int k = 0; k < S; ++k) lks[k] = 0u;
      if (tk_pending) {
        const unsigned t = __builtin_amdgcn_readfirstlane(tk);
        tk_pending = false;
        const int64_t c = (int64_t)t * kHeads + head;
        const int64_t nchunks = (M + cl - 1) / cl;
        if (prm.progress && lane == 0 &&
            ((c >= prm.progress_at && c < prm.progress_at + kHeads) || (c >= nchunks && c < nchunks + kHeads)))
          __hip_atomic_store(prm.progress, prm.progress_value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (c * cl >= M) {
          exhausted = true;
        } else {
#pragma unroll
          for (int h = H - 1; h >= 0; --h)
            if (cbase[h] < 0) staging = h;
#pragma unroll
          for (int h = 0; h < H; ++h)
            if (h == staging) cbase[h] = (int32_t)(c * cl);
          const int64_t m = c * cl + lane;
          if (lane < cl && m < M) {
            const int32_t* src = rec + m * R;
#pragma unroll
            for (int k = 0; k < R; ++k) r[k] = src[k];
            const uint32_t* ls = link + m * S;
#pragma unroll
            for (int k = 0; k < S; ++k) lks[k] = ls[k];
          }
        }
      }
      // ---- next ticket if a slot is free (slots are only freed below)
      {
        bool free_slot = false;
#pragma unroll
        for (int h = 0; h < H; ++h) free_slot |= cbase[h] < 0 && h != staging;
        if (free_slot && !exhausted) {
          if (lane == 0)
            tk = __hip_atomic_fetch_add((gu32*)&ctrl[4 + head], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          tk_pending = true;
        }
      }
      // ---- polls of the pending matches
#pragma unroll
      for (int h = 0; h < H; ++h)
        if ((pbits >> h) & 1u)
          dval[h] = __hip_atomic_load((gu32*)(deps + cbase[h] + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // ---- install the staged chunk
      if (staging >= 0) {
        int64_t cb = 0;
#pragma unroll
        for (int h = 0; h < H; ++h) if (h == staging) cb = cbase[h];
        const int64_t mm = lane < cl ? cb + lane : M;
        uint32_t nd = 0u;
        {
          const uint32_t m0s = (uint32_t)r[S];
          bool dup = false;
#pragma unroll
          for (int a = 0; a < S; ++a) {
            const bool ina = (a < K ? a : a - K) < (a < K ? meta_n0(m0s) : meta_n1(m0s));
            bool firsto = ina;
#pragma unroll
            for (int b = 0; b < a; ++b) {
              const bool inb = (b < K ? b : b - K) < (b < K ? meta_n0(m0s) : meta_n1(m0s));
              dup |= r[a] >= 0 && r[a] == r[b];
              if (inb && r[b] == r[a]) firsto = false;
            }
            if (firsto && (lks[a] & kLinkHasPred)) ++nd;
          }
          r[S + 1] = dup ? (r[S + 1] | 8) : (r[S + 1] & ~8);
        }
        const uint8_t est = mm < M ? early_status<K>(r, P) : kRated;
        if (mm < M && est != kRated) {  // no state, no dependencies: finish it now
#pragma unroll
          for (int q2 = 0; q2 < 5 * S; ++q2) orows[mm * orow + q2] = NAN;
          orows[mm * orow + 5 * S] = (est == kAfk || est == kInvalidRosters) ? 0.f : NAN;
          reinterpret_cast<uint8_t*>(orows + mm * orow + 5 * S + 1)[0] = est;
        }
        const bool live = mm < M && est == kRated;
#pragma unroll
        for (int h = 0; h < H; ++h)
          if (h == staging) {
            dval[h] = kNone;  // first poll next loop
            need[h] = nd;
            lenq[h] = 0u;
          }
#pragma unroll
        for (int k = 0; k < R; ++k) lrec[staging][lane][k] = r[k];
        lloc[lane][staging] = 0u;
        if (live) pbits |= 1u << staging;
        if (lane == 0) lused[staging] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // record + counts before the base
        if (lane == 0) lcb[staging] = (int32_t)cb;
        worked = true;
      }
      // ---- retire: nothing pending and every entry read
      {
        uint32_t retired = 0;
        const uint32_t pmask = wave_or(pbits);  // chunks that still have a pending lane
#pragma unroll
        for (int h = 0; h < H; ++h) {
          if (cbase[h] >= 0 && h != staging && !((pmask >> h) & 1u) &&
              __hip_atomic_load(&lused[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == lenq[h]) {
            cbase[h] = -1;
            if (lane == 0) lcb[h] = -1;
            ++retired;
          }
        }
        if (retired && lane == 0)
          __hip_atomic_fetch_add((gu32*)&ctrl[3], retired, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (retired) worked = true;
      }
      bool held = false;
#pragma unroll
      for (int h = 0; h < H; ++h) held |= cbase[h] >= 0;
      if (exhausted && !held && !tk_pending) break;
      if (timed_out(worked)) {
        timeout = true;
        break;
      }
      if (!worked) __builtin_amdgcn_s_sleep(1);
    }
    if (timeout) {
      if (lane == 0) {
        atomicOr(&ctrl[1], 1u);
        atomicOr(&ctrl[17], 1u);
      }
#pragma unroll
      for (int h = 0; h < H; ++h)
        if (cbase[h] >= 0 && ((pbits >> h) & 1u))
          reinterpret_cast<uint8_t*>(orows + (int64_t)(cbase[h] + lane) * orow + 5 * S + 1)[0] = kNotProcessed;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) {
      __hip_atomic_store(&sdone, timeout ? 2u : 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add((gu32*)&ctrl[15], iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }

  // ==================================================================== raters
  const int j = lane % G;
  const int g = lane / G;
  const int gbase = lane - j;
  const uint64_t gmask = (((1ull << G) - 1ull) << gbase);
  const bool r0 = j < K;
  const int rpos = r0 ? j : j - K;
  const float beta2 = prm.beta2, tau2 = prm.tau2, us = prm.unknown_sigma;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(state, 0, (int)(P * kRowFloats * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(link), 0, (int)(M * S * 4), 0x00020000);
  const bool local_ok = prm.local_handoff != 0;
  uint32_t n_local = 0, n_global = 0, iter = 0, popped = 0;
  for (;;) {
    // ---- pop up to NG ready matches
    uint32_t base = 0u, n = 0u;
    if (lane == 0) {
      for (;;) {
        const uint32_t hd = __hip_atomic_load(&qhead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t tl = __hip_atomic_load(&qtail, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t avail = tl - hd;
        if (avail == 0u) break;
        const uint32_t take = avail < (uint32_t)NG ? avail : (uint32_t)NG;
        uint32_t exp = hd;
        if (__hip_atomic_compare_exchange_strong(&qhead, &exp, hd + take, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP)) {
          base = hd;
          n = take;
          break;
        }
      }
    }
    n = __builtin_amdgcn_readfirstlane(n);
    base = __builtin_amdgcn_readfirstlane(base);
    if (n == 0u) {
      const uint32_t sd = __hip_atomic_load(&sdone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (sd != 0u) {
        const uint32_t hd = __hip_atomic_load(&qhead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t tl = __hip_atomic_load(&qtail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (hd == tl || sd == 2u) break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    ++iter;
    popped += n;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // ---- this group's match, record from LDS
    const bool active = (uint32_t)g < n;
    int32_t m = 0, my_id = -1;
    uint32_t m0 = 0u, m1 = 0u;
    int hs = 0;
    if (active) {
      const uint32_t e = q[(base + (uint32_t)g) & (kSplitQ - 1)];
      hs = (int)(e >> 8);
      const int b = (int)(e & 255u);
      m = lcb[hs] + b;
      if (j < S) my_id = lrec[hs][b][j];
      m0 = (uint32_t)lrec[hs][b][S];
      m1 = (uint32_t)lrec[hs][b][S + 1];
    }
    // the record is in registers: release the entry
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (active && j == 0) atomicAdd(&lused[hs], 1u);
    const int mode = meta_mode(m0);
    const int n0 = meta_n0(m0), n1 = meta_n1(m0);
    const int rank0 = meta_winner0(m1) ? 0 : 1, rank1 = meta_winner1(m1) ? 0 : 1;
    const bool inr = active && j < S && rpos < (r0 ? n0 : n1);
    const int32_t id = inr ? my_id : -1;
    bool islast = true;
    int first = j, prevdup = -1;
    const bool any_dup = __ballot(active && ((m1 >> 3) & 1u)) != 0ull;
    if (any_dup) {
#pragma unroll
      for (int q2 = 0; q2 < S; ++q2) {
        const int32_t oid = __shfl(id, gbase + q2);
        if (id >= 0 && oid == id) {
          if (q2 < j) {
            if (first == j) first = q2;
            prevdup = q2;
          }
          if (q2 > j) islast = false;
        }
      }
    }
    const bool own = inr && first == j;
    const int goff = own ? id * (kRowFloats * 4) : kOutOfRange;
    const uint32_t lk0 = __builtin_amdgcn_raw_buffer_load_b32(rl, inr ? (m * S + j) * 4 : kOutOfRange, 0, 0);
    v4i gs, gm;
    // ---- gather; a granule whose tags do not show its last writer yet is reloaded
    uint32_t counters = 0u;
    for (int attempt = 0;; ++attempt) {
      gs = __builtin_amdgcn_raw_buffer_load_b128(rs, goff, 0, 16);
      gm = __builtin_amdgcn_raw_buffer_load_b128(rs, goff + 16 * (1 + mode), 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t sa = (uint32_t)gs.y;
      const bool s_this = (sa & 0xffu) == (uint32_t)epoch;
      counters = s_this ? sa >> 8 : 0u;
      const uint32_t cnt = (counters >> (4 * mode)) & 15u;
      const bool shared_ok = !(lk0 & kLinkHasPred) || (s_this && (uint32_t)gs.w == (uint32_t)m);
      const bool mode_ok = cnt == 0u || (gm.y == epoch && (uint32_t)gm.w == cnt);
      const bool fresh = !own || (shared_ok && mode_ok);
      const bool overtaken =
          own && (((lk0 & kLinkHasPred) && s_this && (uint32_t)gs.w != kNoMatch && (uint32_t)gs.w > (uint32_t)m) ||
                  (shared_ok && gm.y == epoch && (uint32_t)gm.w == (cnt == 15u ? 1u : cnt + 1u)));
      if (__ballot(overtaken) != 0ull && lane == 0) {
        atomicOr(&ctrl[2], 1u);
        atomicOr(&ctrl[18], 1u);
      }
      const uint64_t stale = __ballot(!fresh);
      if (stale == 0ull) break;
      if (lane == 0)
        __hip_atomic_fetch_add((gu32*)&ctrl[14], (unsigned)__popcll(stale), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (attempt > (1 << 20)) {  // never observed; a broken protocol must not hang the GPU
        if (lane == 0) {
          atomicOr(&ctrl[1], 1u);
          atomicOr(&ctrl[17], 1u);
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (active) {
      const float smu = __int_as_float(gs.x), ssg = __int_as_float(gs.z);
      const float mmu = __int_as_float(gm.x), msg = __int_as_float(gm.z);
      const bool sh_null = smu != smu, md_null = mmu != mmu;
      float pms = smu, pss = ssg;
      bool seed_ok = true;
      if (__ballot(own && sh_null) != 0ull && own && sh_null) {
        const float4 at4 = reinterpret_cast<const float4*>(attrs)[id];
        const float attr[4] = {at4.x, at4.y, at4.z, at4.w};
        seed_ok = seed_prior<float>(attr, us, prm.vst, pms, pss);
      }
      const bool sh_bad = !sh_null && !(ssg == ssg && ssg != 0.f);
      const bool md_bad = !md_null && !(msg == msg && msg != 0.f);
      float pmm = md_null ? pms : mmu, psm = md_null ? pss : msg;
      uint32_t pflags = own ? ((sh_null ? 2u : 1u) | (md_null ? 4u : 0u)) : 0u;
      const uint8_t lst = !own ? (uint8_t)kRated
                               : (sh_null && !seed_ok) ? (uint8_t)kErrSeed
                               : (sh_bad || md_bad) ? (uint8_t)kErrSigma : (uint8_t)kRated;
      const uint64_t eb = __ballot(lst != kRated) & gmask;
      uint8_t gst = kRated;
      if (eb) gst = (uint8_t)__shfl((int)lst, (int)__builtin_ctzll(eb));
      float rsmu = smu, rssg = ssg, rmmu = mmu, rmsg = msg;
      uint32_t rcnt = counters;
      if (any_dup) {
        const int src = gbase + first;
        pms = __shfl(pms, src);
        pss = __shfl(pss, src);
        pmm = __shfl(pmm, src);
        psm = __shfl(psm, src);
        pflags = (uint32_t)__shfl((int)pflags, src);
        rsmu = __shfl(smu, src);
        rssg = __shfl(ssg, src);
        rcnt = (uint32_t)__shfl((int)counters, src);
        rmmu = __shfl(mmu, src);
        rmsg = __shfl(msg, src);
      }
      if (gst == kRated && (n0 == 0 || n1 == 0)) gst = kErrEmptyRoster;
      float nsm = NAN, nss = NAN, nmm = NAN, nms = NAN, dl = NAN, qv = NAN;
      if (gst == kRated) {
        const float sgn = r0 ? 1.f : -1.f;
        const float s_c2 = group_sum<G>(inr ? pss * pss + tau2 : 0.f, j, gbase);
        const float s_d = group_sum<G>(inr ? sgn * pms : 0.f, j, gbase);
        const float m_d = group_sum<G>(inr ? sgn * pmm : 0.f, j, gbase);
        const float m_q = group_sum<G>(inr ? psm * psm : 0.f, j, gbase);
        const int nn = n0 + n1;
        const float nb2 = (float)nn * beta2;
        const float m_c2 = m_q + (float)nn * tau2;
        qv = quality_from_sums<float>(nn, m_q, m_d, beta2);
        UpdCoef<float> ks, km;
        if constexpr (G == 8 || G == 16) {
          constexpr int kMirror = G == 8 ? 0x141 : 0x140;
          const bool sh = j < G / 2;
          const UpdCoef<float> k = update_coef<float>(sh ? s_d : m_d, nb2 + (sh ? s_c2 : m_c2), rank0, rank1);
          UpdCoef<float> o;
          o.a0 = dpp_mov<kMirror>(k.a0);
          o.a1 = dpp_mov<kMirror>(k.a1);
          o.wf = dpp_mov<kMirror>(k.wf);
          o.c2 = dpp_mov<kMirror>(k.c2);
          ks = sh ? k : o;
          km = sh ? o : k;
        } else {
          ks = update_coef<float>(s_d, nb2 + s_c2, rank0, rank1);
          km = update_coef<float>(m_d, nb2 + m_c2, rank0, rank1);
        }
        apply_coef<float>(ks, r0, pms, pss, tau2, nsm, nss);
        apply_coef<float>(km, r0, pmm, psm, tau2, nmm, nms);
        const bool bad_num = inr && !(isfinite(nsm) && isfinite(nss) && isfinite(nmm) && isfinite(nms) && isfinite(qv));
        if ((__ballot(bad_num) & gmask) != 0ull) gst = kErrNumeric;
        const float cur = nsm - nss;
        const float prevw = any_dup ? __shfl(cur, gbase + (prevdup >= 0 ? prevdup : j)) : cur;
        if (prevdup >= 0) dl = cur - prevw;
        else if (pflags & 1u) dl = cur - (pms - pss);
        else dl = 0.f;
      }
      const bool ok = gst == kRated && inr;
      if (inr && islast) {  // publish, then notify the player's next match
        const int off = id * (kRowFloats * 4);
        const uint32_t succ = lk0 & kMatchMask;
        const uint32_t c4 = (rcnt >> (4 * mode)) & 15u;
        const uint32_t c = c4 == 15u ? 1u : c4 + 1u;
        const uint32_t ncnt = (rcnt & ~(15u << (4 * mode))) | (c << (4 * mode));
        const uint32_t stag = (uint32_t)epoch | (ncnt << 8);
        __builtin_amdgcn_raw_buffer_store_b128(
            ok ? granule(nmm, (uint32_t)epoch, nms, c) : granule(rmmu, (uint32_t)epoch, rmsg, c),
            rs, off + 16 * (1 + mode), 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(
            ok ? granule(nsm, stag, nss, succ) : granule(rsmu, stag, rssg, succ), rs, off, 0, 16);
        if (succ != kNoMatch) {
          int lh = -1;
          int32_t lb = 0;
          if (local_ok) {
#pragma unroll
            for (int h = 0; h < H; ++h) {
              const int32_t cb = lcb[h];
              if (cb >= 0 && (int32_t)succ >= cb && (int32_t)succ < cb + cl) {
                lh = h;
                lb = cb;
              }
            }
          }
          if (lh >= 0) {
            atomicAdd(&lloc[(int32_t)succ - lb][lh], 1u);
            ++n_local;
          } else {
            __hip_atomic_fetch_add((gu32*)(deps + succ), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ++n_global;
          }
        }
      }
      if (ok && prm.record_first_prior && own) {
        float* fp = first_prior + (int64_t)id * kRowFloats;
        if (pflags & 2u) { fp[0] = pms; fp[2] = pss; }
        if (pflags & 4u) { fp[4 * (1 + mode)] = pmm; fp[4 * (1 + mode) + 2] = psm; }
      }
      float* const orm = orows + (int64_t)m * orow;
      if (j < S) {
        __builtin_nontemporal_store(ok ? nsm : NAN, orm + j);
        __builtin_nontemporal_store(ok ? nss : NAN, orm + S + j);
        __builtin_nontemporal_store(ok ? dl : NAN, orm + 2 * S + j);
        __builtin_nontemporal_store(ok ? nmm : NAN, orm + 3 * S + j);
        __builtin_nontemporal_store(ok ? nms : NAN, orm + 4 * S + j);
      }
      if (j == 0) {
        __builtin_nontemporal_store(gst == kRated ? qv : NAN, orm + 5 * S);
        reinterpret_cast<uint8_t*>(orm + 5 * S + 1)[0] = gst;
      }
    }
  }
  // hand-off statistics (per lane counts -> wave sums)
  uint32_t nl = n_local, ngl = n_global;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    nl += __shfl_xor(nl, off);
    ngl += __shfl_xor(ngl, off);
  }
  if (lane == 0) {
    // rater iterations / matches popped in the "worked iterations" / "groups" words
    __hip_atomic_fetch_add((gu32*)&ctrl[20], iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add((gu32*)&ctrl[21], popped, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add((gu32*)&ctrl[26], nl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add((gu32*)&ctrl[27], ngl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

int launch_rate_split(int K, bool tight, const int32_t* rec, const uint32_t* link, int32_t* deps, float* state,
                      const float* attrs, float* first_prior, const RateOut& out, uint32_t* ctrl,
                      const RateParams& prm, int blocks, hipStream_t s) {
#define ANA_SPLIT_LAUNCH(k, g)                                                                           \
  do {                                                                                                   \
    if (prm.split == 2)                                                                                  \
      hipLaunchKernelGGL((rate_split_kernel<k, g, 8>), dim3((unsigned)blocks), dim3(256), 0, s, rec, link,  \
                         deps, state, attrs, first_prior, out.s_mu, out.row, ctrl, prm);                 \
    else                                                                                                 \
      hipLaunchKernelGGL((rate_split_kernel<k, g, 16>), dim3((unsigned)blocks), dim3(256), 0, s, rec, link, \
                         deps, state, attrs, first_prior, out.s_mu, out.row, ctrl, prm);                 \
  } while (0)
  switch (K) {
    case 1: ANA_SPLIT_LAUNCH(1, 2); break;
    case 2: ANA_SPLIT_LAUNCH(2, 4); break;
    case 3: if (tight) ANA_SPLIT_LAUNCH(3, 6); else ANA_SPLIT_LAUNCH(3, 8); break;
    case 4: ANA_SPLIT_LAUNCH(4, 8); break;
    case 5: if (tight) ANA_SPLIT_LAUNCH(5, 10); else ANA_SPLIT_LAUNCH(5, 16); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef ANA_SPLIT_LAUNCH
  return (int)hipGetLastError();
}

}  // namespace ana
#endif  // ANA_DIAG_BUILD
