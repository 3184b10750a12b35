// K1-K4, K3, K6: the per-lane dataflow rating executor for MI355X (gfx950).
//
// Same protocol as the group executor of dataflow.hip -- one persistent launch
// per window, exact per-player chronological order (the reference's
// ORDER BY created_at + sequential loop, /root/reference/worker.py:176-192) by
// Kahn's algorithm over per-player chains, tagged granules instead of store
// acknowledgements, LDS local hand-off -- but ONE LANE RATES ONE WHOLE MATCH:
//
//  * Lane b of a wave owns match cbase[h] + b of each of its kH held chunks.
//    The lane that sees its match ready rates it in place: no pick list, no
//    mbcnt assignment, no group sums, no shuffles of priors or stale bits --
//    the ~0.35 us assignment phase and the cross-lane chains of the group
//    executor are gone, and a wave rates every ready match of its chunks in one
//    iteration (the group executor stopped at 64 / G).
//  * The records of the held chunks live in LDS ([wave][chunk][quad][lane], so
//    a lane reads its selected record with conflict-free ds_read_b128 whatever
//    chunk it picks); a lane's 2K players' shared + mode granules and links are
//    gathered by straight-line buffer loads (out-of-range offsets on idle slots).
//  * The two tracks, the team sums and the 2 x 2K closed-form updates are
//    independent per slot: the compiler interleaves them (ILP inside one lane)
//    where the group executor paid DPP butterfly latency for every sum.
//
// Claims are monotone per ticket shard and every claimed match is held by a
// running wave, so the oldest unfinished match is always ready: no deadlock
// whatever the residency.  Idle waves back off; the watchdog gives up after
// 5 s without any chunk retiring anywhere on the GPU.
#include <hip/hip_runtime.h>

#include "common.h"
#include "dataflow_dev.h"
#include "kernels.h"
#include "rate_core.h"
#include "telemetry_dev.h"

#ifndef ANA_LANE_HELD
#define ANA_LANE_HELD 4
#endif

namespace ana {

constexpr int kLaneHeld = ANA_LANE_HELD;  // chunks a wave keeps in flight
typedef float v4f __attribute__((ext_vector_type(4)));

// Per-lane bit masks pass through an empty asm so the compiler recomputes each
// (mask >> j) & 1 test from this VGPR where it is used, instead of keeping one
// 64-bit lane mask per slot and flag alive in SGPRs (that spilled ~100 SGPRs).
__device__ __forceinline__ uint32_t opaque(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}

// rate_core.h seed_prior as selects (rater.py:42-62): rank points (the larger of
// the non-NULL, non-zero ranked / blitz) with sigma 2/3 us, else the skill tier's
// vst points with sigma us; false = the reference's KeyError (tier NULL / 30 / junk)
__device__ __forceinline__ bool seed_select(v4i at, float us, const float* vst, float& mu, float& sig) {
  const float rr = __int_as_float(at.x), rb = __int_as_float(at.y), tier = __int_as_float(at.z);
  const bool hr = rr == rr && rr != 0.f, hb = rb == rb && rb != 0.f;
  const float rp = hr && hb ? fmaxf(rr, rb) : hr ? rr : rb;
  const int ti = (int)tier;
  const bool tok = tier == tier && (float)ti == tier && ti >= -1 && ti <= 29;
  const float vp = vst[tok ? ti + 1 : 0];
  const float s_rp = us * (float)(2.0 / 3.0);
  sig = (hr || hb) ? s_rp : us;
  mu = ((hr || hb) ? rp : vp) + sig;
  return hr || hb || tok;
}

template <int K>
struct LaneShape {
  static constexpr int S = 2 * K;
  static constexpr int R = S + 2;            // record words
  static constexpr int RQ = (R + 3) / 4;     // record quads in LDS
  static constexpr int OW = 5 * S + 2;       // output row words written (fields, quality, status word)
  static constexpr int OQ = (OW + 3) / 4;    // output row quads
};

template <int K, bool TELE, bool DIAG>
__global__ void __launch_bounds__(256)
rate_lane_kernel(const int32_t* __restrict__ rec, const uint32_t* __restrict__ link,
                 int32_t* deps, float* state, const float* __restrict__ attrs,
                 float* __restrict__ first_prior, float* __restrict__ orows, int64_t orow,
                 uint32_t* ctrl, RateParams prm, TelemetryParams tp) {
  using SH = LaneShape<K>;
  constexpr int S = SH::S;
  constexpr int R = SH::R;
  constexpr int RQ = SH::RQ;
  constexpr int kH = kLaneHeld;
  static_assert(kH == 2 || kH == 4, "local counts are read as one vector");
  typedef uint32_t hvec __attribute__((ext_vector_type(kH)));
  // held records: [wave][chunk][quad][lane]
  __shared__ v4i lrec[kWavesPerBlock][kH][RQ][kChunk];
  // local hand-off counters: increments of a held match's completion count by
  // publishes of THIS wave (never also added to the global counter)
  __shared__ hvec lloc[kWavesPerBlock][kChunk];
  __shared__ uint32_t ljunk[kWavesPerBlock][kChunk];  // sink of the masked lanes' hand-off adds
  __shared__ float tele[kWavesPerBlock][TELE ? tele_scratch_floats<K>() : 1];  // K8 scratch
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t M = prm.num_matches;
  const int64_t P = prm.num_players;
  const float beta2 = prm.beta2, tau2 = prm.tau2, us = prm.unknown_sigma;
  const int epoch = prm.epoch_ptr ? __builtin_amdgcn_readfirstlane(*prm.epoch_ptr) : prm.epoch;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(state, 0, (int)(P * kRowFloats * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(link), 0, (int)(M * S * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(deps, 0, (int)(M * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(attrs), 0, (int)(P * 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(
      first_prior ? first_prior : state, 0, first_prior ? (int)(P * kRowFloats * 4) : 0, 0x00020000);
  const int head = blockIdx.x % kHeads;
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t seen_progress = 0;
  const bool local_ok = prm.local_handoff != 0;
  uint32_t n_local = 0, n_global = 0;  // wave-uniform hand-off counts
  uint64_t d_issue = 0, d_wait = 0, d_after = 0, d_it0 = 0;
  uint64_t d_t[4] = {0, 0, 0, 0}, d_p[4] = {0, 0, 0, 0};
  uint64_t d_s[4] = {0, 0, 0, 0}, d_i[3] = {0, 0, 0};
  uint32_t d_worked = 0, d_rated = 0;

  int32_t cbase[kH];  // wave-uniform: first match of each held chunk, -1 = free slot
  uint32_t dval[kH];  // per lane: completion counter of its match in chunk h, as last polled
  uint32_t need[kH];  // per lane: the count at which that match is ready
  uint32_t pbits = 0; // per lane: bit h = its match in chunk h is stateful and not yet rated
#pragma unroll
  for (int h = 0; h < kH; ++h) {
    cbase[h] = -1;
    dval[h] = kNone;
    need[h] = 0u;
  }
  bool exhausted = false, tk_pending = false;
  unsigned tk = 0;
  uint32_t spins = 0, iter = 0;
  // K8 fused mode (as in dataflow.hip): aggregation waves stream spans first
  const bool tele_role = TELE && tp.role_stride > 0 && tp.impl != 0;
  const int tele_span = tele_role ? kTeleMaxSpan : kTeleTile;
  const int64_t tele_tiles = TELE && tp.evoff ? (tp.num_matches + tele_span - 1) / tele_span : 0;
  bool tele_done = tele_tiles == 0;
  auto tele_claim = [&]() -> int64_t {
    unsigned t = 0;
    if (lane == 0)
      t = __hip_atomic_fetch_add((gu32*)&ctrl[12], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t = __builtin_amdgcn_readfirstlane(t);
    return (int64_t)t < tele_tiles ? (int64_t)t : -1;
  };
  auto tele_run = [&](int64_t t) {
    if constexpr (TELE) {
      if (tele_role) telemetry_tile_mfma<K, 0, kTeleMaxSpan>(tp, t, lane, tele[wv], &ctrl[13]);
      else if (tp.impl) telemetry_tile_mfma<K>(tp, t, lane, tele[wv], &ctrl[13]);
      else telemetry_tile<K>(tp, t, lane, tele[wv], &ctrl[13]);
    }
  };
  if constexpr (TELE) {
    if (tele_role) {
      const int b = blockIdx.x, per = tp.role_stride >= 4 ? tp.role_stride / 4 : 1;
      const bool agg = tp.role_stride >= 4   ? (wv == ((b >> 3) & 3) && ((b >> 5) % per) == 0)
                       : tp.role_stride == 2 ? ((wv & 1) == ((b >> 3) & 1))
                                             : true;
      while (agg && !tele_done) {
        const int64_t t = tele_claim();
        if (t < 0) tele_done = true;
        else tele_run(t);
      }
    }
  }
  const uint32_t max_spins = prm.idle_spins > 0 ? (uint32_t)prm.idle_spins : prm.idle_spins < 0 ? 0u : 8u;
  const int cl = prm.chunk_len;

  for (;;) {
    if constexpr (DIAG) d_it0 = __builtin_amdgcn_s_memrealtime();
    // ---------------------------------------------- readiness from the last poll
    int sel = -1;
    {
      const hvec lv = lloc[wv][lane];
#pragma unroll
      for (int h = kH - 1; h >= 0; --h)
        if (((pbits >> h) & 1u) && dval[h] + lv[h] == need[h]) sel = h;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // state loads stay below the poll
    const bool act = sel >= 0;
    const bool worked = __ballot(act) != 0ull;
    if constexpr (DIAG) d_i[0] = __builtin_amdgcn_s_memrealtime();

    // ---------------------------------------------- the selected match's record (LDS)
    int32_t r[R];
    int32_t m = 0;
    {
      const int hs = act ? sel : 0;
#pragma unroll
      for (int q = 0; q < RQ; ++q) {
        const v4i v = lrec[wv][hs][q][lane];
        if (4 * q + 0 < R) r[4 * q + 0] = v.x;
        if (4 * q + 1 < R) r[4 * q + 1] = v.y;
        if (4 * q + 2 < R) r[4 * q + 2] = v.z;
        if (4 * q + 3 < R) r[4 * q + 3] = v.w;
      }
      int32_t cb = cbase[0];
#pragma unroll
      for (int h = 1; h < kH; ++h) cb = sel == h ? cbase[h] : cb;
      m = cb + lane;
    }
    const uint32_t m0 = act ? (uint32_t)r[S] : 0u, m1 = act ? (uint32_t)r[S + 1] : 0u;
    const int mode = meta_mode(m0);
    const int n0 = meta_n0(m0), n1 = meta_n1(m0);
    const int rank0 = meta_winner0(m1) ? 0 : 1, rank1 = meta_winner1(m1) ? 0 : 1;
    const bool dup = ((m1 >> 3) & 1u) != 0u;  // flagged at staging: a player named twice
    // slot facts as bit masks (bit j): in roster; owns the gather (first occurrence
    // of its player); publishes (last occurrence).  Repeated players only (rare):
    // nibble j of fsel = first slot of the same player, of psel = latest earlier
    // one (15: none); 64 bits for the 10 slots of 5v5
    int32_t id[S];
    uint32_t inr = 0u;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const bool in = act && (j < K ? j : j - K) < (j < K ? n0 : n1);
      id[j] = r[j];
      inr |= in ? 1u << j : 0u;
    }
    inr = opaque(inr);
    uint32_t own = inr, last = inr;
    uint64_t fsel = 0u, psel = ~0ull;  // 4 bits per slot: up to 16 slots
#pragma unroll
    for (int j = 0; j < S; ++j) fsel |= (uint64_t)j << (4 * j);
    if (dup) {
#pragma unroll
      for (int j = 1; j < S; ++j) {
        uint32_t f = (uint32_t)j, pv = 15u;
#pragma unroll
        for (int i = 0; i < j; ++i) {
          if (((inr >> i) & (inr >> j) & 1u) && id[i] == id[j]) {
            if (f == (uint32_t)j) f = (uint32_t)i;
            pv = (uint32_t)i;
            last &= ~(1u << i);
          }
        }
        if (f != (uint32_t)j) own &= ~(1u << j);
        fsel = (fsel & ~(15ull << (4 * j))) | ((uint64_t)f << (4 * j));
        psel = (psel & ~(15ull << (4 * j))) | ((uint64_t)pv << (4 * j));
      }
    }
    own = opaque(own);
    last = opaque(last);
    if constexpr (DIAG) d_i[1] = __builtin_amdgcn_s_memrealtime();

    // ---------------------------------------------- this lane's loads (straight-line)
    v4i gs[S], gm[S];
    uint32_t lk[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const int goff = ((own >> j) & 1u) ? id[j] * (kRowFloats * 4) : kOutOfRange;
      gs[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, goff, 0, 16);
      gm[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, goff + 16 * (1 + mode), 0, 16);
    }
#pragma unroll
    for (int q = 0; q < S / 2; ++q) {
      const v2u v = __builtin_bit_cast(
          v2u, __builtin_amdgcn_raw_buffer_load_b64(rl, act ? (m * S + 2 * q) * 4 : kOutOfRange, 0, 0));
      lk[2 * q] = v.x;
      lk[2 * q + 1] = v.y;
    }
    if constexpr (DIAG) d_i[2] = __builtin_amdgcn_s_memrealtime();

    // ---------------------------------------------- a ticket came back: stage its chunk
    int staging = -1;
    int32_t rs_[R];
    uint32_t lks[S];
#pragma unroll
    for (int k = 0; k < R; ++k) rs_[k] = -1;
#pragma unroll
    for (int k = 0; k < S; ++k) lks[k] = 0u;
    if (tk_pending) {
      const unsigned t = __builtin_amdgcn_readfirstlane(tk);
      tk_pending = false;
      const int64_t c = (int64_t)t * kHeads + head;
      const int64_t nchunks = (M + cl - 1) / cl;
      if (prm.progress && lane == 0 &&
          ((c >= prm.progress_at && c < prm.progress_at + kHeads) ||
           (c >= nchunks && c < nchunks + kHeads)))
        __hip_atomic_store(prm.progress, prm.progress_value, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      if (c * cl >= M) {
        exhausted = true;
      } else {
#pragma unroll
        for (int h = kH - 1; h >= 0; --h)
          if (cbase[h] < 0) staging = h;
#pragma unroll
        for (int h = 0; h < kH; ++h)
          if (h == staging) cbase[h] = (int32_t)(c * cl);
        const int64_t ms = c * cl + lane;
        if (lane < cl && ms < M) {
          const int32_t* src = rec + ms * R;
          if constexpr (R % 4 == 0) {
#pragma unroll
            for (int k = 0; k < R / 4; ++k) {
              const v4i v = reinterpret_cast<const v4i*>(src)[k];
              rs_[4 * k] = v.x; rs_[4 * k + 1] = v.y; rs_[4 * k + 2] = v.z; rs_[4 * k + 3] = v.w;
            }
          } else {
#pragma unroll
            for (int k = 0; k < R; ++k) rs_[k] = src[k];
          }
          const v2u* ls = reinterpret_cast<const v2u*>(link + ms * S);
#pragma unroll
          for (int k = 0; k < S / 2; ++k) {
            const v2u v = ls[k];
            lks[2 * k] = v.x;
            lks[2 * k + 1] = v.y;
          }
        }
      }
    }

    // ---------------------------------------------- next ticket if a slot is free
    {
      bool free_slot = false;
#pragma unroll
      for (int h = 0; h < kH; ++h) free_slot |= cbase[h] < 0;
      if (free_slot && !exhausted) {
        if (lane == 0)
          tk = __hip_atomic_fetch_add((gu32*)&ctrl[4 + head], 1u, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
        tk_pending = true;
      }
    }

    // ---------------------------------------------- the one wait of the iteration
    uint64_t d_w0 = 0, d_w1 = 0;
    if constexpr (DIAG) d_w0 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (DIAG) d_w1 = __builtin_amdgcn_s_memrealtime();

    // ---------------------------------------------- install the staged chunk
    if (staging >= 0) {
      int64_t cb = 0;
#pragma unroll
      for (int h = 0; h < kH; ++h) if (h == staging) cb = cbase[h];
      const int64_t mm = lane < cl ? cb + lane : M;
      // ready once every distinct player with an earlier occurrence (kLinkHasPred
      // on its first slot) has been published; flag repeated players (bit 3 of
      // meta1) so the rating skips the duplicate scan for every other match
      uint32_t nd = 0u;
      {
        const uint32_t m0s = (uint32_t)rs_[S];
        bool dp = false;
#pragma unroll
        for (int a = 0; a < S; ++a) {
          const bool ina = (a < K ? a : a - K) < (a < K ? meta_n0(m0s) : meta_n1(m0s));
          bool firsto = ina;
#pragma unroll
          for (int b = 0; b < a; ++b) {
            const bool inb = (b < K ? b : b - K) < (b < K ? meta_n0(m0s) : meta_n1(m0s));
            dp |= rs_[a] >= 0 && rs_[a] == rs_[b];
            if (inb && rs_[b] == rs_[a]) firsto = false;
          }
          if (firsto && (lks[a] & kLinkHasPred)) ++nd;
        }
        rs_[S + 1] = dp ? (rs_[S + 1] | 8) : (rs_[S + 1] & ~8);
      }
#pragma unroll
      for (int q = 0; q < RQ; ++q) {
        v4i v;
        v.x = 4 * q + 0 < R ? rs_[4 * q + 0] : 0;
        v.y = 4 * q + 1 < R ? rs_[4 * q + 1] : 0;
        v.z = 4 * q + 2 < R ? rs_[4 * q + 2] : 0;
        v.w = 4 * q + 3 < R ? rs_[4 * q + 3] : 0;
        lrec[wv][staging][q][lane] = v;
      }
      reinterpret_cast<uint32_t*>(&lloc[wv][lane])[staging] = 0u;
      const uint8_t est = mm < M ? early_status<K>(rs_, P) : kRated;
      if (mm < M && est != kRated) {  // no state, no dependencies: finish it now
        v4f* orm = reinterpret_cast<v4f*>(orows + mm * orow);
        const float qv = (est == kAfk || est == kInvalidRosters) ? 0.f : NAN;
#pragma unroll
        for (int q = 0; q < SH::OQ; ++q) {
          v4f v = {NAN, NAN, NAN, NAN};
          if (4 * q + 3 >= 5 * S) {
            if (4 * q + 0 == 5 * S) v.x = qv;
            if (4 * q + 1 == 5 * S) v.y = qv;
            if (4 * q + 2 == 5 * S) v.z = qv;
            if (4 * q + 3 == 5 * S) v.w = qv;
            const float sw = __uint_as_float((uint32_t)est);
            if (4 * q + 0 == 5 * S + 1) v.x = sw;
            if (4 * q + 1 == 5 * S + 1) v.y = sw;
            if (4 * q + 2 == 5 * S + 1) v.z = sw;
            if (4 * q + 3 == 5 * S + 1) v.w = sw;
          }
          __builtin_nontemporal_store(v, orm + q);
        }
      }
      const bool pm = mm < M && est == kRated;
      pbits = (pbits & ~(1u << staging)) | (pm ? 1u << staging : 0u);
#pragma unroll
      for (int h = 0; h < kH; ++h)
        if (h == staging) {
          dval[h] = kNone;  // first poll next iteration
          need[h] = nd;
          if (__ballot(pm) == 0ull) cbase[h] = -1;
        }
    }

    if constexpr (DIAG) d_p[0] = d_p[1] = d_p[2] = d_p[3] = d_w1;
    // ---------------------------------------------- tag check
    // A counter can reach its count before the writes it announces have landed
    // (notifications do not wait for store acknowledgements): a match whose
    // granules do not carry the tags of their last writers waits an iteration.
    uint32_t rcnt[S];  // per-mode write counters of each slot's shared granule
    bool fresh = true, overtaken = false;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const uint32_t sa = (uint32_t)gs[j].y;
      const bool s_this = (sa & 0xffu) == (uint32_t)epoch;
      rcnt[j] = s_this ? sa >> 8 : 0u;
      const uint32_t cnt = (rcnt[j] >> (4 * mode)) & 15u;
      const bool hp = (lk[j] & kLinkHasPred) != 0u;
      const bool shared_ok = !hp || (s_this && (uint32_t)gs[j].w == (uint32_t)m);
      const bool mode_ok = cnt == 0u || ((uint32_t)gm[j].y == (uint32_t)epoch && (uint32_t)gm[j].w == cnt);
      const bool o = (own >> j) & 1u;
      fresh = fresh && (!o || (shared_ok && mode_ok));
      // race detector: a shared granule of this launch tagged for a LATER reader,
      // or a mode granule one write AHEAD of the verified count
      overtaken = overtaken ||
                  (o && ((hp && s_this && (uint32_t)gs[j].w != kNoMatch && (uint32_t)gs[j].w > (uint32_t)m) ||
                         (shared_ok && (uint32_t)gm[j].y == (uint32_t)epoch &&
                          (uint32_t)gm[j].w == (cnt == 15u ? 1u : cnt + 1u))));
    }
    {
      const uint64_t ob = __ballot(act && overtaken);
      const uint64_t sb = __ballot(act && !fresh);
      if (lane == 0) {
        if (ob) {
          atomicOr(&ctrl[2], 1u);
          atomicOr(&ctrl[18], 1u);  // sticky copy (never zeroed by a launch)
        }
        if (sb)  // diagnostics: stale reads retried (those matches stay pending)
          __hip_atomic_fetch_add((gu32*)&ctrl[14], (unsigned)__popcll(sb), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    // ---------------------------------------------- rate this lane's match
    if (act && fresh) {
      // priors (rate_core.h player_prior, as selects and bit masks).  Slots outside
      // the roster loaded zeros (out-of-range gathers), so they add nothing to sums.
      float pms[S], pss[S], pmm[S], psm[S];
      uint32_t shnull = 0u, mdnull = 0u, sbad = 0u;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const float smu = __int_as_float(gs[j].x), ssg = __int_as_float(gs[j].z);
        const float mmu = __int_as_float(gm[j].x), msg = __int_as_float(gm[j].z);
        const bool shn = smu != smu, mdn = mmu != mmu;
        shnull |= shn ? 1u << j : 0u;
        mdnull |= mdn ? 1u << j : 0u;
        const bool bad = (!shn && !(ssg == ssg && ssg != 0.f)) || (!mdn && !(msg == msg && msg != 0.f));
        sbad |= bad ? 1u << j : 0u;
        pms[j] = smu;
        pss[j] = ssg;
        pmm[j] = mmu;
        psm[j] = msg;
      }
      shnull = opaque(shnull & own);
      mdnull = opaque(mdnull & own);
      sbad = opaque(sbad & own);
      uint32_t seedfail = 0u;
      if (shnull) {  // first match of a player: seed from its attributes (rare)
        v4i at[S];
#pragma unroll
        for (int j = 0; j < S; ++j)
          at[j] = __builtin_amdgcn_raw_buffer_load_b128(ra, ((shnull >> j) & 1u) ? id[j] * 16 : kOutOfRange, 0, 0);
#pragma unroll
        for (int j = 0; j < S; ++j) {
          float mu, sg;
          const bool okj = seed_select(at[j], us, prm.vst, mu, sg);
          const bool sn = (shnull >> j) & 1u;
          pms[j] = sn ? mu : pms[j];
          pss[j] = sn ? sg : pss[j];
          seedfail |= (sn && !okj) ? 1u << j : 0u;
        }
      }
#pragma unroll
      for (int j = 0; j < S; ++j) {  // a NULL mode track starts from the (seeded) shared prior
        const bool md = (mdnull >> j) & 1u;
        pmm[j] = md ? pms[j] : pmm[j];
        psm[j] = md ? pss[j] : psm[j];
      }
      // the first failing slot decides the error class (player_prior per slot in
      // order: a failed seed, else a zero / NULL sigma on either track)
      uint8_t gst = kRated;
      {
        const uint32_t e = seedfail | sbad;
        if (e) gst = (e & (~e + 1u) & seedfail) ? kErrSeed : kErrSigma;
      }
      if (gst == kRated && (n0 == 0 || n1 == 0)) gst = kErrEmptyRoster;
      uint32_t had = own & ~shnull;  // a stored shared rating existed (delta rule)
      seedfail = opaque(seedfail);
      if (dup) {  // duplicates see the pre-match values of their first occurrence
#pragma unroll
        for (int j = 1; j < S; ++j) {
          const uint32_t f = (uint32_t)(fsel >> (4 * j)) & 15u;
#pragma unroll
          for (int i = 0; i < j; ++i)
            if (f == (uint32_t)i) {
              pms[j] = pms[i]; pss[j] = pss[i]; pmm[j] = pmm[i]; psm[j] = psm[i];
              rcnt[j] = rcnt[i];
              had |= ((had >> i) & 1u) << j;
              shnull |= ((shnull >> i) & 1u) << j;
              mdnull |= ((mdnull >> i) & 1u) << j;
            }
        }
      }
      if constexpr (DIAG) d_p[1] = __builtin_amdgcn_s_memrealtime();
      // ------------------------------------------ team sums, quality, both tracks
      const int n = n0 + n1;
      float s_c2 = 0.f, s_d0 = 0.f, s_d1 = 0.f, m_d0 = 0.f, m_d1 = 0.f, m_q = 0.f;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        s_c2 = fmaf(pss[j], pss[j], s_c2);
        m_q = fmaf(psm[j], psm[j], m_q);
        if (j < K) { s_d0 += pms[j]; m_d0 += pmm[j]; }
        else { s_d1 += pms[j]; m_d1 += pmm[j]; }
      }
      const float nb2 = (float)n * beta2, nt2 = (float)n * tau2;
      const float s_d = s_d0 - s_d1, m_d = m_d0 - m_d1;
      const float q = quality_from_sums<float>(n, m_q, m_d, beta2);
      const UpdCoef<float> ks = update_coef<float>(s_d, nb2 + (s_c2 + nt2), rank0, rank1);
      const UpdCoef<float> km = update_coef<float>(m_d, nb2 + (m_q + nt2), rank0, rank1);
      float nsm[S], nss[S], nmm[S], nms[S], dl[S];
      uint32_t fin = 0u;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        apply_coef<float>(ks, j < K, pms[j], pss[j], tau2, nsm[j], nss[j]);
        apply_coef<float>(km, j < K, pmm[j], psm[j], tau2, nmm[j], nms[j]);
        const bool f = isfinite(nsm[j]) && isfinite(nss[j]) && isfinite(nmm[j]) && isfinite(nms[j]);
        fin |= f ? 1u << j : 0u;
        // conservative-skill delta (rater.py:150-153)
        dl[j] = ((had >> j) & 1u) ? (nsm[j] - nss[j]) - (pms[j] - pss[j]) : 0.f;
      }
      fin = opaque(fin);
      if (gst == kRated && (!isfinite(q) || (inr & ~fin) != 0u)) gst = kErrNumeric;
      if (dup) {  // a repeated player's delta is against its previous slot's write
#pragma unroll
        for (int j = 1; j < S; ++j) {
          const uint32_t pv = (uint32_t)(psel >> (4 * j)) & 15u;
#pragma unroll
          for (int i = 0; i < j; ++i)
            if (pv == (uint32_t)i) dl[j] = (nsm[j] - nss[j]) - (nsm[i] - nss[i]);
        }
      }
      const bool ok = gst == kRated;
      if (!ok) {  // rare: republish the untouched granules (their tags still move on)
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const int goff = (((inr & last) >> j) & 1u) ? id[j] * (kRowFloats * 4) : kOutOfRange;
          const v4i a = __builtin_amdgcn_raw_buffer_load_b128(rs, goff, 0, 16);
          const v4i b = __builtin_amdgcn_raw_buffer_load_b128(rs, goff + 16 * (1 + mode), 0, 16);
          nsm[j] = __int_as_float(a.x); nss[j] = __int_as_float(a.z);
          nmm[j] = __int_as_float(b.x); nms[j] = __int_as_float(b.z);
        }
      }
      if constexpr (DIAG) d_p[2] = __builtin_amdgcn_s_memrealtime();
      // ------------------------------------------ publish: granules, then the successors' counters
      const uint32_t pub = opaque(inr & last);
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const bool pj = (pub >> j) & 1u;
        const int off = pj ? id[j] * (kRowFloats * 4) : kOutOfRange;
        const uint32_t succ = lk[j] & kMatchMask;
        const uint32_t c4 = (rcnt[j] >> (4 * mode)) & 15u;  // write count, wraps 15 -> 1
        const uint32_t c = c4 == 15u ? 1u : c4 + 1u;
        const uint32_t ncnt = (rcnt[j] & ~(15u << (4 * mode))) | (c << (4 * mode));
        const uint32_t stag = (uint32_t)epoch | (ncnt << 8);
        __builtin_amdgcn_raw_buffer_store_b128(granule(nmm[j], (uint32_t)epoch, nms[j], c), rs,
                                               off + 16 * (1 + mode), 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(granule(nsm[j], stag, nss[j], succ), rs, off, 0, 16);
        // the successor verifies the tags, so no store wait before the notify
        const bool has = pj && succ != kNoMatch;
        int lh = -1;
        uint32_t lrel = 0u;
#pragma unroll
        for (int h = 0; h < kH; ++h) {
          const uint32_t rel = succ - (uint32_t)cbase[h];
          if (local_ok && cbase[h] >= 0 && rel < (uint32_t)cl) {
            lh = h;
            lrel = rel;
          }
        }
        const bool loc = has && lh >= 0;
        uint32_t* la = loc ? reinterpret_cast<uint32_t*>(&lloc[wv][lrel]) + lh : &ljunk[wv][lane];
        atomicAdd(la, 1u);  // held by this wave: release it through LDS, next iteration
        __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, rd, (has && !loc) ? (int)(succ * 4u) : kOutOfRange, 0, 0);
        n_local += loc ? 1u : 0u;
        n_global += (has && !loc) ? 1u : 0u;
      }
      if constexpr (DIAG) d_p[3] = __builtin_amdgcn_s_memrealtime();
      if (prm.record_first_prior) {  // sweep mode: the priors of NULL tracks
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const bool w = ok && ((own >> j) & 1u);
          const int bo = id[j] * (kRowFloats * 4);
          const int so = (w && ((shnull >> j) & 1u)) ? bo : kOutOfRange;
          const int mo = (w && ((mdnull >> j) & 1u)) ? bo + 16 * (1 + mode) : kOutOfRange;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(pms[j]), rf, so, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(pss[j]), rf, so, 8, 0);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(pmm[j]), rf, mo, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(psm[j]), rf, mo, 8, 0);
        }
      }
      // ------------------------------------------ the match's output row: full-line
      // non-temporal stores ([s_mu | s_sig | delta | m_mu | m_sig][S], quality, status)
      {
        float w[4 * SH::OQ];
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const bool in = ok && ((inr >> j) & 1u);
          w[j] = in ? nsm[j] : NAN;
          w[S + j] = in ? nss[j] : NAN;
          w[2 * S + j] = in ? dl[j] : NAN;
          w[3 * S + j] = in ? nmm[j] : NAN;
          w[4 * S + j] = in ? nms[j] : NAN;
        }
        w[5 * S] = ok ? q : NAN;
        w[5 * S + 1] = __uint_as_float((uint32_t)gst);
#pragma unroll
        for (int k = 5 * S + 2; k < 4 * SH::OQ; ++k) w[k] = 0.f;
        v4f* orm = reinterpret_cast<v4f*>(orows + (int64_t)m * orow);
#pragma unroll
        for (int qd = 0; qd < SH::OQ; ++qd)
          __builtin_nontemporal_store(v4f{w[4 * qd], w[4 * qd + 1], w[4 * qd + 2], w[4 * qd + 3]}, orm + qd);
      }
      pbits &= ~(1u << sel);
      if constexpr (DIAG) ++d_rated;
    }
    if constexpr (DIAG) {
      if (worked) {
        const uint64_t end = __builtin_amdgcn_s_memrealtime();
        ++d_worked;
        d_issue += d_w0 - d_it0;
        d_wait += d_w1 - d_w0;
        d_after += end - d_w1;
        d_s[0] += d_i[0] - d_it0;
        d_s[1] += d_i[1] - d_i[0];
        d_s[2] += d_i[2] - d_i[1];
        d_s[3] += d_w0 - d_i[2];
        // per-lane markers: take the first active lane's
        const int fl = (int)__builtin_ctzll(__ballot(act) | (1ull << 63));
        const uint64_t p1 = (uint64_t)(uint32_t)__shfl((int)(uint32_t)d_p[1], fl) |
                            ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(d_p[1] >> 32), fl) << 32);
        const uint64_t p2 = (uint64_t)(uint32_t)__shfl((int)(uint32_t)d_p[2], fl) |
                            ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(d_p[2] >> 32), fl) << 32);
        const uint64_t p3 = (uint64_t)(uint32_t)__shfl((int)(uint32_t)d_p[3], fl) |
                            ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(d_p[3] >> 32), fl) << 32);
        if (p1 >= d_w1 && p2 >= p1 && p3 >= p2 && end >= p3) {
          d_t[0] += p1 - d_w1;
          d_t[1] += p2 - p1;
          d_t[2] += p3 - p2;
          d_t[3] += end - p3;
        }
      }
    }

    // ---------------------------------------------- next iteration's counter polls, late
    ++iter;
#pragma unroll
    for (int h = 0; h < kH; ++h)  // sc1: served past the (non-coherent) L1
      dval[h] = __builtin_amdgcn_raw_buffer_load_b32(rd, ((pbits >> h) & 1u) ? (cbase[h] + lane) * 4 : kOutOfRange,
                                                     0, 16);

    // ---------------------------------------------- retire finished chunks
    {
      uint32_t retired = 0;
#pragma unroll
      for (int h = 0; h < kH; ++h)
        if (cbase[h] >= 0 && __ballot((pbits >> h) & 1u) == 0ull) {
          cbase[h] = -1;
          ++retired;
        }
      if (retired && lane == 0)
        __hip_atomic_fetch_add((gu32*)&ctrl[3], retired, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // ---------------------------------------------- done?
    bool held = false;
#pragma unroll
    for (int h = 0; h < kH; ++h) held |= cbase[h] >= 0;
    if (exhausted && !held && !tk_pending) {
      // wave totals of the per-lane hand-off counts (lanes counted their own)
      uint32_t nl = n_local, ng = n_global;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        nl += __shfl_xor(nl, off);
        ng += __shfl_xor(ng, off);
      }
      if (lane == 0) {
        __hip_atomic_fetch_add((gu32*)&ctrl[15], iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add((gu32*)&ctrl[26], nl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add((gu32*)&ctrl[27], ng, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if constexpr (DIAG) {
        uint32_t nr = d_rated;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) nr += __shfl_xor(nr, off);
        if (lane == 0) {
          __hip_atomic_fetch_add((gu32*)&ctrl[20], d_worked, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add((gu32*)&ctrl[21], nr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          atomicAdd(reinterpret_cast<unsigned long long*>(&ctrl[22]), (unsigned long long)d_issue);
          atomicAdd(reinterpret_cast<unsigned long long*>(&ctrl[24]), (unsigned long long)d_wait);
          atomicAdd(reinterpret_cast<unsigned long long*>(&ctrl[28]), (unsigned long long)d_after);
          for (int qd = 0; qd < 4; ++qd)
            atomicAdd(reinterpret_cast<unsigned long long*>(&ctrl[32 + 2 * qd]), (unsigned long long)d_t[qd]);
          for (int qd = 0; qd < 4; ++qd)
            atomicAdd(reinterpret_cast<unsigned long long*>(&ctrl[40 + 2 * qd]), (unsigned long long)d_s[qd]);
        }
      }
      if constexpr (TELE) {
        while (!tele_done) {
          const int64_t t = tele_claim();
          if (t < 0) tele_done = true;
          else tele_run(t);
        }
      }
      break;
    }

    // ---------------------------------------------- idle: back off, bounded
    if (worked || staging >= 0) {
      spins = 0;
    } else {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (now - t0 > kProgressTicks) {
        const uint32_t p = __hip_atomic_load((gu32*)&ctrl[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p != seen_progress) {
          seen_progress = p;
          t0 = now;
        }
      }
      if (now - t0 > kTimeoutTicks) {
        if (lane == 0) {
          atomicOr(&ctrl[1], 1u);
          atomicOr(&ctrl[17], 1u);  // sticky copy
        }
#pragma unroll
        for (int h = 0; h < kH; ++h)
          if (cbase[h] >= 0 && ((pbits >> h) & 1u))
            reinterpret_cast<uint8_t*>(orows + (int64_t)(cbase[h] + lane) * orow + 5 * S + 1)[0] = kNotProcessed;
        return;  // give up: the host sees ctrl[1] and raises
      }
      if constexpr (TELE) {
        if (!tele_done && ((!tp.fused_tail && !tele_role) || !held)) {
          const int64_t t = tele_claim();
          if (t >= 0) {
            tele_run(t);
            spins = 0;
            continue;
          }
          tele_done = true;
        }
      }
      spins = spins < max_spins ? spins + 1u : max_spins;
      for (uint32_t k = 0; k < spins; ++k) __builtin_amdgcn_s_sleep(2);
    }
  }
}

int launch_rate_lane(int K, const int32_t* rec, const uint32_t* link, int32_t* deps, float* state,
                     const float* attrs, float* first_prior, const RateOut& out, uint32_t* ctrl,
                     const RateParams& prm, const TelemetryParams& tp, int blocks, hipStream_t s) {
  // the output row must hold the written quads (ops/rate.py RateResult.row_floats)
  const int S = 2 * K;
  if (out.row < ((5 * S + 2 + 3) / 4) * 4 || (out.row & 3) || (((uintptr_t)out.s_mu) & 15))
    return (int)hipErrorInvalidValue;
#define ANA_LANE_LAUNCH_D(k, tele, diag)                                                         \
  hipLaunchKernelGGL((rate_lane_kernel<k, tele, diag>), dim3((unsigned)blocks), dim3(256), 0, s, \
                     rec, link, deps, state, attrs, first_prior, out.s_mu, out.row, ctrl, prm, tp)
#define ANA_LANE_LAUNCH(k)                                   \
  do {                                                       \
    if (tp.evoff) ANA_LANE_LAUNCH_D(k, true, false);         \
    else if (prm.diag) ANA_LANE_LAUNCH_D(k, false, true);    \
    else ANA_LANE_LAUNCH_D(k, false, false);                 \
  } while (0)
  switch (K) {
    case 1: ANA_LANE_LAUNCH(1); break;
    case 2: ANA_LANE_LAUNCH(2); break;
    case 3: ANA_LANE_LAUNCH(3); break;
    case 4: ANA_LANE_LAUNCH(4); break;
    case 5: ANA_LANE_LAUNCH(5); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef ANA_LANE_LAUNCH
#undef ANA_LANE_LAUNCH_D
  return (int)hipGetLastError();
}

}  // namespace ana
