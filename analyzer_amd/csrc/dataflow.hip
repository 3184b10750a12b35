// K1-K4, K3, K6: the dataflow rating executor for MI355X (gfx950).
//
// ONE persistent launch rates a whole window of matches in exact per-player
// chronological order -- the order the reference gets from
// ORDER BY created_at + a sequential loop (/root/reference/worker.py:176-192)
// -- without rounds or grid barriers (Kahn's algorithm over per-player chains):
//
//  * The schedule prepass (kernels.hip) gives every slot the match of its
//    player's next occurrence and a has-earlier flag (link).  A match is ready
//    when its completion counter (deps, zeroed by the prepass) reaches the
//    number of its distinct players with an earlier occurrence, which the wave
//    counts from the links when it stages the chunk.
//  * 8 sharded tickets (MICROARCH "dequeue") hand out chunks of 64
//    consecutive matches (32 for 5v5, ops/rate.py chunk_len).  A wave holds one
//    chunk (ANA_HELD; four until round 6), its records in registers, so 64k
//    matches wait in flight at one wave per SIMD -- several dependency levels of a
//    random stream.  Waiting costs nothing per match: the wave polls its chunk's
//    counters with one coalesced 4-B sc1 load per lane.
//  * The oldest ready matches go to the wave's lane groups (G lanes = one
//    match, one roster slot per lane).  A group gathers its players' 16-B
//    granules (sc1 buffer loads), seeds, rates both tracks (rate_core.h),
//    publishes the granules (sc1 stores) and at once increments the
//    counter of each player's next match.  The notification does not wait for
//    the stores: the shared granule is tagged with the match that reads it
//    next and carries per-mode write counters, the mode granule its write
//    count; a reader verifies both and retries the match if a write has not
//    landed, so a dependency hop costs no store round trip.
//  * Software pipeline, one memory round trip per iteration: this iteration's
//    granule/link/attribute loads, the next iteration's counter polls and the
//    next chunk ticket retire in ONE vmcnt(0) wait.
//  * Local hand-off (1v1-4v4): when the successor of a published player lies in
//    the chunk the SAME wave holds, the producer bumps that match's counter in LDS
//    instead of the global one.  Readiness = polled global count + LDS count,
//    so the successor is assigned in the very next iteration -- no poll round
//    trip -- which is what a hot player's chain (consecutive matches of one
//    player in one chunk: skewed activity) runs on.
//
// Claims are monotone per ticket shard and every claimed match is held by a
// running wave, so the oldest unfinished match is always ready: no deadlock
// whatever the residency.  Spins back off; the watchdog gives up after 5 s
// without any chunk retiring anywhere on the GPU.
#include <hip/hip_runtime.h>

#include "common.h"
#include "dataflow_dev.h"
#include "kernels.h"
#include "rate_core.h"
#include "rate_dev.h"
#include "telemetry_dev.h"

// Chunks a wave keeps in flight: ONE since round 6.  Re-measured at one wave per SIMD with
// the global counters (in-call A/B of builds, profiles/r6/held_chunks.log): 4 -> 1 held
// chunk takes config 2 7.64 -> 7.10 ms per step, config 4 8.62 -> 7.83, config 5 11.34 ->
// 10.92, quadratic / cubic skew -13 / -8 %, the serial hop 2.14 -> 2.00 us -- a wave with
// one chunk claims the next one sooner, closer to the dependency frontier, and polls and
// stages a quarter of the counters every iteration.
#ifndef ANA_HELD
#define ANA_HELD 1
#endif

namespace ana {

// The LDS local hand-off (ANA_RATE_LOCAL, on by default): compiled into the 1v1-4v4
// executors (and every executor of the diagnostic library).  Off from round 5 with four
// held chunks per wave (profiles/r5/local_handoff_off.log); with one held chunk (round 6)
// it pays for 3v3 (in-call A/B of the libraries, profiles/r6/local_handoff_on.log): serial
// hop 1.96-1.97 -> 1.85-1.87 us, cubic skew 1180 -> 1170 ms per 10M window, config 2
// 6.88 -> 6.83 ms per step, config 4 7.43 -> 7.32, config 5 10.93 -> 10.79, config 2 between
// emulated N = 8 merges 10.86-10.89 -> 10.33-10.34; quadratic skew 128.9 -> 131.4 ms; 5v5
// gained nothing (14.48 vs 14.54 with it), so its executor keeps it compiled out
#ifndef ANA_LOCAL_HANDOFF
#define ANA_LOCAL_HANDOFF 1
#endif
constexpr bool kLocalHandoff = ANA_LOCAL_HANDOFF != 0;
#ifndef ANA_LOCAL_HANDOFF_MAXK
#define ANA_LOCAL_HANDOFF_MAXK 4  // the widest team the production hand-off is compiled for (4v4: 9.56-9.58 -> 9.50-9.54 ms)
#endif


constexpr int kHeld = ANA_HELD;  // chunks a wave keeps in flight (1v1-4v4)
// 5v5 likewise: two beat four (config 3 19.23-19.27 ms per step against 20.08-20.15) and
// one beats two (18.48-18.89 against 19.27-19.62; in-call A/Bs, profiles/r6/
// config3_held_chunks.log) -- its 3,000+ dependency levels leave most held matches
// waiting, so extra chunks only add polls and staging to every iteration (and 24
// registers each: 166 -> 138 VGPRs at two); holding the records in LDS instead of
// registers (120 VGPRs, 55.7 KB of LDS) measured no faster (20.10-20.22)
#ifndef ANA_HELD5
#define ANA_HELD5 1
#endif
// K8 inline telemetry: events per match loaded with the batch's granules (more go
// through a remainder loop after the rating); per group lane ceil(64 / G) 8-B loads
constexpr int kTeleInline = 64;

// One wave iteration's assignment: per lane, its group's match and the
// participant's slot facts and granules (section 4 of the executor loop).
struct Batch {
  int32_t m = 0;
  int my_h = -1, my_bit = 0, mode = 0, n0 = 0, n1 = 0, rank0 = 1, rank1 = 1, first = 0, prevdup = -1;
  int32_t id = -1;
  bool inr = false, islast = false, own = false, any_dup = false;
  uint32_t lk0 = kNoMatch;  // schedule link (common.h): next match | has-earlier
  v4i gs = {0, 0, 0, 0}, gm = {0, 0, 0, 0};
  // K8 inline telemetry (TelemetryParams::role_stride < 0): the match's event count, a
  // match without state to rate (tele-only: early status in est), its first kTeleInline
  // events (lane j of the group holds events j, j + G, ...)
  int64_t toff = 0;
  int32_t tcnt = 0;
  bool tonly = false;
  uint8_t est = kRated;
};

// TELE: K8 fused telemetry compiled in (the plain rating launch leaves it out,
// which frees the registers its code pins): 1 = aggregation tiles taken by idle or
// dedicated waves (one-hot MFMA), 2 = inline, each lane group folds the events of the
// match it rated (TelemetryParams::role_stride < 0).  DIAG: the timing build
// (ANA_RATE_DIAG=1) -- every wave clocks its iterations and its wait with
// s_memrealtime and adds them to ctrl[20..27] at exit (launch_rate).
// WPE: the waves per SIMD the kernel is compiled for.  Plain 1v1-3v3 launches of two
// waves per SIMD (512 workgroups: config 5's 10M-player roster) take the 4-wave build
// (<= 128 VGPRs; the 3v3 kernel 137 -> 128, no spills): a radix-sort workgroup of the
// next window's prepass (2 waves per SIMD of 108-115 VGPRs) then still fits beside
// them, so that prepass can overlap the rating (config 5 11.73 -> 11.19 ms from 0.1,
// profiles/r5/executor_vgpr_cap.log).  At one wave per SIMD (256 workgroups) it fits
// anyway and the uncapped build is 0.01-0.02 ms faster.  Telemetry, diagnostic,
// tight-group and 4v4 / 5v5 instantiations would spill under the cap.
template <int K, int G, int TELE, bool DIAG, int WPE = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
rate_dataflow_kernel(const int32_t* __restrict__ rec, const uint32_t* __restrict__ link,
                     int32_t* deps, float* state, const float* __restrict__ attrs,
                     float* __restrict__ first_prior, float* __restrict__ orows, int64_t orow,
                     uint32_t* ctrl,
                     RateParams prm, TelemetryParams tp) {
  constexpr int S = 2 * K;
  constexpr int R = S + 2;
  constexpr int kH = K >= 5 ? ANA_HELD5 : kHeld;
  constexpr bool kLH = kLocalHandoff && (K <= ANA_LOCAL_HANDOFF_MAXK || ANA_DIAG_BUILD != 0);  // LDS local hand-off compiled in
  constexpr bool TILES = TELE == 1;  // K8 tiles taken by idle / dedicated waves
  constexpr bool INL = TELE == 2;    // K8 inline: each group folds its match's events
  static_assert(G >= S && G <= 64, "a group holds one match");
  constexpr int NG = 64 / G;
  static_assert(kH >= 1 && kH <= 4, "held chunks");
  // the held chunks' local hand-off counts are read as one vector (diagnostic library): 1 or 3
  // held chunks use a 2 / 4-wide one, the upper lanes unused
  typedef uint32_t hvec __attribute__((ext_vector_type(kH <= 2 ? 2 : 4)));
  // local hand-off counters: increments of each held match's completion count
  // by publishes of THIS wave (never also added to the global counter); [lane][h]
  // so a lane reads them in one ds_read_b64/b128.  Without kLH (5v5 in the
  // production library) the executor has no LDS array, no per-iteration read of it
  // and no held-chunk scan in notify
  __shared__ hvec lloc[kWavesPerBlock][kLH ? kChunk : 1];
  // this iteration's pick per group, written by the lane holding the match:
  // {match index, slot << 8 | lane in chunk, meta0, meta1, player ids...}
  constexpr int SPT = (4 + S + 3) / 4 * 4;  // inline telemetry words: {offset lo, hi, count, 0}
  constexpr int SP = SPT + (INL ? 4 : 0);
  // inline event loads per lane: kTeleInline events per group, at most 8 loads per lane
  constexpr int TT = INL ? ((kTeleInline + G - 1) / G < 8 ? (kTeleInline + G - 1) / G : 8) : 1;
  // inline telemetry: one stat block [S][8] per group, accumulated with LDS float adds
  __shared__ __attribute__((aligned(16))) float tstat[kWavesPerBlock][INL ? NG : 1][INL ? S * kStatFeatures : 4];
  __shared__ __attribute__((aligned(16))) int32_t lpick[kWavesPerBlock][NG][SP];  // v4i slots
  __shared__ float tele[kWavesPerBlock][TILES ? tele_scratch_floats<K>() : 1];  // K8 scratch
  // each group's output row, assembled here so it leaves as whole 16-B quads
  // (one store instruction writes the rows of every group: full lines, where
  // per-field stores sent 6-7 partial-line writes per match to the fabric)
  constexpr int OQ = (5 * S + 2 + 3) / 4;
  __shared__ __attribute__((aligned(16))) float lrow[kWavesPerBlock][NG][4 * OQ];
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
  // graph replays (ops/graph.py) keep the epoch in device memory, bumped before each launch
  const int epoch = prm.epoch_ptr ? __builtin_amdgcn_readfirstlane(*prm.epoch_ptr) : prm.epoch;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(state, 0, (int)(P * kRowFloats * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(link), 0, (int)(M * S * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(deps, 0, (int)(M * 4), 0x00020000);
  const int head = blockIdx.x % kHeads;
  // watchdog: give up only after kTimeoutTicks without ANY chunk retiring GPU-wide
  // (ctrl[3] counts retired chunks), so long dependency chains never trip it
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t seen_progress = 0;
  const bool local_ok = kLH && prm.local_handoff != 0;
  // hand-off statistics (wave-uniform counts, added to ctrl[26..27] at exit); stale
  // reads retried (ctrl[14])
  uint32_t n_local = 0, n_global = 0, n_stale = 0;
  // timing build: clocks of the iterations that rated something, split at the wait
  uint64_t d_issue = 0, d_wait = 0, d_after = 0, d_it0 = 0;
  uint64_t d_t[4] = {0, 0, 0, 0}, d_p[5] = {0, 0, 0, 0, 0};  // after-phase split (timing build)
  uint64_t d_s[4] = {0, 0, 0, 0}, d_i[3] = {0, 0, 0};         // issue-phase split (timing build)
  uint32_t d_worked = 0, d_groups = 0, d_near = 0, d_pend = 0;

  // per lane: the record of match cbase[h] + lane (ids, meta0, meta1), kept in
  // registers so the lane that picks a match hands the whole record to its group
  // through one LDS slot (one round trip instead of pick -> meta -> id)
  int32_t hrec[kH][R];
  int64_t hoff[kH];    // per lane (inline telemetry): first event of match cbase + lane
  int32_t hcnt[kH];    // ... and its event count
  int32_t cbase[kH];   // wave-uniform: first match of each held chunk, -1 = free slot
                       // (a window has < 2^28 slots, so match indices fit int32)
  uint64_t pend[kH];   // wave-uniform: stateful matches not yet handed to a group
  uint32_t dval[kH];   // per lane: completion counter of match cbase+lane, as last polled
  uint32_t need[kH];   // per lane: the count at which that match is ready
#pragma unroll
  for (int h = 0; h < kH; ++h) {
    cbase[h] = -1;
    pend[h] = 0ull;
#pragma unroll
    for (int k = 0; k < R; ++k) hrec[h][k] = -1;
    dval[h] = kNone;
    need[h] = 0u;
    hoff[h] = 0;
    hcnt[h] = 0;
  }
  bool exhausted = false, tk_pending = false;
  unsigned tk = 0;                 // ticket returned to lane 0
  uint32_t spins = 0, iter = 0;
  // K8 fused mode.  Default: telemetry tiles fill the time a wave would spend
  // waiting.  Role split (tp.role_stride): aggregation waves stream 63-match
  // spans from the start -- spread one per (block group, SIMD) so no SIMD and no
  // XCD gets them all -- while the rating waves keep their dependency chains
  // moving; an aggregation wave joins the rating when the events run out.
  const bool tele_role = TILES && tp.role_stride > 0 && tp.impl != 0;
  // inline: each lane group folds its match's events into the participants' stats
  // right after rating it (no tiles, nothing co-runs with the rating)
  const bool tele_inline = INL && tp.role_stride < 0 && tp.evoff != nullptr;
  const int tele_span = tele_role ? kTeleMaxSpan : kTeleTile;
  const int64_t tele_tiles = TILES && tp.evoff ? (tp.num_matches + tele_span - 1) / tele_span : 0;
  bool tele_done = tele_tiles == 0 || tele_inline;
  auto tele_claim = [&]() -> int64_t {
    unsigned t = 0;
    if (lane == 0)
      t = __hip_atomic_fetch_add((gu32*)&ctrl[12], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t = __builtin_amdgcn_readfirstlane(t);
    return (int64_t)t < tele_tiles ? (int64_t)t : -1;
  };
  auto tele_run = [&](int64_t t) {
    if constexpr (TILES) {
      if (tele_role) telemetry_tile_mfma<K, 0, kTeleMaxSpan>(tp, t, lane, tele[wv], &ctrl[13]);
      else if (tp.impl) telemetry_tile_mfma<K>(tp, t, lane, tele[wv], &ctrl[13]);
      else telemetry_tile<K>(tp, t, lane, tele[wv], &ctrl[13]);
    }
  };
  if constexpr (TILES) {
    if (tele_role) {
      const int b = blockIdx.x, per = tp.role_stride >= 4 ? tp.role_stride / 4 : 1;
      const bool agg = tp.role_stride >= 4   ? (wv == ((b >> 3) & 3) && ((b >> 5) % per) == 0)
                       : tp.role_stride == 2 ? ((wv & 1) == ((b >> 3) & 1))
                                             : true;  // 1: every wave aggregates first
      while (agg && !tele_done) {
        const int64_t t = tele_claim();
        if (t < 0) tele_done = true;
        else tele_run(t);
      }
    }
  }
  // K8 inline (software-pipelined): the events of the last rated batch, per lane,
  // folded by tele_flush in the next iteration (and at exit)
  v2u tev_prev[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) tev_prev[t] = v2u{0u, 0u};
  int32_t tp_m = -1, tp_cnt = 0;
  int64_t tp_off = 0;
  auto tele_flush = [&]() {
    if constexpr (INL) {
      if (tp_m < 0) return;  // this lane's group rated nothing last iteration
      float* const ts = tstat[wv][g];
      typedef float v4f __attribute__((ext_vector_type(4)));
      if (j < S) {
        reinterpret_cast<v4f*>(ts)[2 * j] = v4f{0.f, 0.f, 0.f, 0.f};
        reinterpret_cast<v4f*>(ts)[2 * j + 1] = v4f{0.f, 0.f, 0.f, 0.f};
      }
      uint32_t nbad = 0;
      const uint32_t mtag = (uint32_t)tp_m & 0xffffu;
      auto fold = [&](v2u ev) {
        const int32_t meta = (int32_t)ev.x;
        const int slot = event_slot(meta);
        if (event_tag(meta) != mtag || slot >= S) {  // strict attribution (telemetry_core.h)
          ++nbad;
          return;
        }
        float add;
        const int f = event_feature(event_type(meta), __uint_as_float(ev.y), add);
        if (f >= 0) atomicAdd(&ts[slot * kStatFeatures + f], add);
        atomicAdd(&ts[slot * kStatFeatures + kStatEvents], 1.f);
      };
#pragma unroll
      for (int t = 0; t < TT; ++t)
        if (j + G * t < tp_cnt) fold(tev_prev[t]);
      // events past the loaded ones (rare: > kTeleInline in one match)
      for (int e = j + G * TT; e < tp_cnt; e += G)
        fold(__builtin_nontemporal_load(reinterpret_cast<const v2u*>(tp.events + 2 * (tp_off + e))));
      if (j < S) {  // (the group's LDS writes and reads are the same wave's, in order)
        v4f* dst = reinterpret_cast<v4f*>(tp.stats + ((int64_t)tp_m * S + j) * kStatFeatures);
        __builtin_nontemporal_store(reinterpret_cast<const v4f*>(ts)[2 * j], dst);
        __builtin_nontemporal_store(reinterpret_cast<const v4f*>(ts)[2 * j + 1], dst + 1);
      }
      if (nbad) atomicAdd(&ctrl[13], nbad);  // malformed events (none in a valid stream)
      tp_m = -1;
    }
  };
  // an idle wave polls again at once by default: with most waves idle (skewed windows,
  // where the critical path crosses waves) a sleeping holder adds its back-off to every
  // global hand-off -- quadratic skew 193.5 -> 166.4 ms per 10M window, cubic 1528 -> 1457,
  // configs 2 / 3 unchanged (profiles/r5/idle_backoff_skew.log); ANA_RATE_IDLE = n > 0
  // restores a back-off of up to n s_sleep(2) rounds
  const uint32_t max_spins = prm.idle_spins > 0 ? (uint32_t)prm.idle_spins : 0u;
  const int cl = prm.chunk_len;  // matches per ticket (<= kChunk lanes)
  // chunks in the window (hoisted: a 64-bit division is ~130 scalar instructions)
  const int64_t nchunks = (M + cl - 1) / cl;

  for (;;) {
    if constexpr (DIAG) d_it0 = __builtin_amdgcn_s_memrealtime();
    // ---------------------------------------------- (2) readiness from the last poll
    // one unconditional LDS read: a free slot's stale count is masked by pend = 0,
    // and without local hand-off the counts stay 0
    uint64_t ready[kH];
    {
      hvec lv = {};
      if constexpr (kLH) lv = lloc[wv][lane];
#pragma unroll
      for (int h = 0; h < kH; ++h)
        ready[h] = __ballot(dval[h] != kNone && dval[h] + lv[h] == need[h]) & pend[h];
      if constexpr (DIAG) {
        uint32_t nn = 0, np = 0;
#pragma unroll
        for (int h = 0; h < kH; ++h) {
          nn += (uint32_t)__popcll(__ballot(dval[h] != kNone && dval[h] + lv[h] + 1u == need[h]) & pend[h]);
          np += (uint32_t)__popcll(pend[h]);
        }
        bool any = false;
#pragma unroll
        for (int h = 0; h < kH; ++h) any |= ready[h] != 0ull;
        if (any) {
          d_near += nn;
          d_pend += np;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // state loads stay below the poll
    if constexpr (DIAG) d_i[0] = __builtin_amdgcn_s_memrealtime();

    // ---------------------------------------------- (3) ready matches -> groups
    // Within a chunk, lane b's rank among the ready bits below it (mbcnt) is the
    // group it goes to: lane b writes its match into the wave's LDS pick list at
    // nassigned + rank, and group g reads entry g.  A handful of instructions
    // per chunk, where a scalar loop per picked match (~600 static instructions,
    // oldest chunk first) sat on every hop.  Chunks go in slot order: a wave
    // rarely has more ready matches than groups (2-3.4 per iteration on the
    // bench), so age order buys nothing measurable.
    // (Speculatively assigning matches one dependency short to idle groups was
    // measured slower -- 5 % of them fresh, window +3 %, profiles/r4/executor_speculation.log
    // -- and removed in round 5.)
    int my_h = -1, my_bit = 0, nassigned = 0;
#pragma unroll
    for (int h = 0; h < kH; ++h) {
      const uint64_t rdy = ready[h];
      if (rdy != 0ull && nassigned < NG) {
        const uint32_t below = __builtin_amdgcn_mbcnt_hi(
            (uint32_t)(rdy >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rdy, 0u));
        const bool mine = ((rdy >> lane) & 1ull) && nassigned + (int)below < NG;
        if (mine) {
          int32_t w[SP];
          w[0] = cbase[h] + lane;
          w[1] = (h << 8) | lane;
          w[2] = hrec[h][S];
          w[3] = hrec[h][S + 1];
#pragma unroll
          for (int k = 0; k < SPT - 4; ++k) w[4 + k] = k < S ? hrec[h][k] : -1;
          if constexpr (INL) {
            w[SPT] = (int32_t)(uint32_t)hoff[h];
            w[SPT + 1] = (int32_t)(hoff[h] >> 32);
            w[SPT + 2] = hcnt[h];
            w[SPT + 3] = 0;
          }
          v4i* dst = reinterpret_cast<v4i*>(&lpick[wv][nassigned + (int)below][0]);
#pragma unroll
          for (int q = 0; q < SP / 4; ++q) dst[q] = v4i{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
        }
        const uint64_t taken = __ballot(mine);
        pend[h] &= ~taken;
        nassigned += __popcll(taken);
      }
    }
    int32_t my_m = 0, my_id = -1;
    uint32_t my_m0 = 0u, my_m1 = 0u;
    int64_t my_toff = 0;
    int32_t my_tcnt = 0;
    if (g < nassigned) {  // two LDS reads, one wait
      const v4i pk = *reinterpret_cast<const v4i*>(&lpick[wv][g][0]);
      if constexpr (INL) {
        const v4i tk4 = *reinterpret_cast<const v4i*>(&lpick[wv][g][SPT]);
        my_toff = (int64_t)(((uint64_t)(uint32_t)tk4.y << 32) | (uint32_t)tk4.x);
        my_tcnt = tk4.z;
      }
      if (j < S) my_id = lpick[wv][g][4 + j];
      my_m = pk.x;
      my_h = (pk.y >> 8) & 255;
      my_bit = pk.y & 255;
      my_m0 = (uint32_t)pk.z;
      my_m1 = (uint32_t)pk.w;
    }
    const bool worked = nassigned > 0;
    if constexpr (DIAG) {
      d_worked += worked ? 1u : 0u;
      d_groups += (uint32_t)nassigned;
      d_i[1] = __builtin_amdgcn_s_memrealtime();
    }

    // ---------------------------------------------- (4) this group's loads
    // Straight-line for every lane (no branch around the loads): a lane without a
    // participant loads out of range (buffer bounds check: zeros, no access), so
    // nothing forces a copy of the loaded registers -- and with it an early wait
    // on the loads -- at the join of a branch.
    Batch nb;  // any_dup is wave-uniform: a match of this batch names a player twice
    {
      const int32_t m = my_m;
      const uint32_t m0 = my_m0, m1 = my_m1;  // 0 on lanes of unassigned groups: no roster
      const int mode = meta_mode(m0);
      nb.my_h = my_h;
      nb.my_bit = my_bit;
      nb.m = m;
      nb.mode = mode;
      nb.n0 = meta_n0(m0);
      nb.n1 = meta_n1(m0);
      nb.rank0 = meta_winner0(m1) ? 0 : 1;
      nb.rank1 = meta_winner1(m1) ? 0 : 1;
      // inline telemetry: a match without state to rate (AFK, invalid, unsupported,
      // malformed) still goes through a group, for its events only
      nb.tonly = INL && ((m1 >> 4) & 1u);
      nb.est = (uint8_t)(m1 >> 28);
      nb.tcnt = my_h >= 0 ? my_tcnt : 0;
      nb.toff = my_toff;
      const bool inr = my_h >= 0 && j < S && rpos < (r0 ? nb.n0 : nb.n1) && !nb.tonly;
      nb.inr = inr;
      const int32_t id = inr ? my_id : -1;
      nb.id = id;
      bool islast = true;
      int first = j, prevdup = -1;
      nb.any_dup = __ballot((m1 >> 3) & 1u) != 0ull;
      if (nb.any_dup) {  // some match of this batch repeats a player
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
      }
      nb.islast = islast;
      nb.first = first;
      nb.prevdup = prevdup;
      const bool own = inr && first == j;
      nb.own = own;
      const int goff = own ? id * (kRowFloats * 4) : kOutOfRange;
      nb.gs = __builtin_amdgcn_raw_buffer_load_b128(rs, goff, 0, 16);
      nb.gm = __builtin_amdgcn_raw_buffer_load_b128(rs, goff + 16 * (1 + mode), 0, 16);
      nb.lk0 = __builtin_amdgcn_raw_buffer_load_b32(rl, inr ? (m * S + j) * 4 : kOutOfRange, 0, 0);
    }

    // ---------------------------------------------- (1) a ticket came back: stage its chunk
    // (after this batch's loads: the top of the loop waits only for the polls)
    if constexpr (DIAG) d_i[2] = __builtin_amdgcn_s_memrealtime();
    int staging = -1;
    int32_t r[R];
    uint32_t lks[S];  // the staged match's links: its readiness count
    int64_t stoff = 0;  // inline telemetry: the staged match's first event and count
    int32_t stcnt = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) r[k] = -1;
#pragma unroll
    for (int k = 0; k < S; ++k) lks[k] = 0u;
    if (tk_pending) {
      // readfirstlane, not a shuffle: the compiler then knows the chunk bases and
      // masks derived from it are wave-uniform and keeps the bookkeeping scalar
      const unsigned t = __builtin_amdgcn_readfirstlane(tk);
      tk_pending = false;
      const int64_t c = (int64_t)t * kHeads + head;
      // tail signal: the first ticket of each shard at or past progress_at, and its
      // first ticket past the end (so a threshold beyond the window still fires)
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
        const int64_t m = c * cl + lane;
        if (lane < cl && m < M) {
          const int32_t* src = rec + m * R;
          if constexpr (R % 4 == 0) {
#pragma unroll
            for (int k = 0; k < R / 4; ++k) {
              const v4i v = reinterpret_cast<const v4i*>(src)[k];
              r[4 * k] = v.x; r[4 * k + 1] = v.y; r[4 * k + 2] = v.z; r[4 * k + 3] = v.w;
            }
          } else {
#pragma unroll
            for (int k = 0; k < R; ++k) r[k] = src[k];
          }
          const v2u* ls = reinterpret_cast<const v2u*>(link + m * S);  // S even: 8-B aligned
#pragma unroll
          for (int k = 0; k < S / 2; ++k) {
            const v2u v = ls[k];
            lks[2 * k] = v.x;
            lks[2 * k + 1] = v.y;
          }
          if (tele_inline) {
            stoff = tp.evoff[m];
            stcnt = (int32_t)(tp.evoff[m + 1] - stoff);
          }
        }
      }
    }

    // ---------------------------------------------- (10) rate a batch
    // inline telemetry: the events this iteration's groups load for the next flush
    v2u tev_next[TT];
    int32_t tn_m = -1, tn_cnt = 0;
    int64_t tn_off = 0;
    // release the successor of a published player: an LDS count when this wave holds
    // it (assigned next iteration), else its global completion counter.  The
    // successor verifies the granule tags, so no store wait precedes the notify.
    auto notify = [&](uint32_t succ) {
      if (succ == kNoMatch) return;
      int lh = -1;
      int32_t lcb = 0;
      if (kLH && local_ok) {
#pragma unroll
        for (int h = 0; h < kH; ++h)
          if (cbase[h] >= 0 && (int32_t)succ >= cbase[h] && (int32_t)succ < cbase[h] + cl) {
            lh = h;
            lcb = cbase[h];
          }
      }
      if (kLH && lh >= 0) {  // held by this wave: release it through LDS, next iteration
        atomicAdd(reinterpret_cast<uint32_t*>(&lloc[wv][(int32_t)succ - lcb]) + lh, 1u);
      } else {
        __hip_atomic_fetch_add((gu32*)(deps + succ), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const uint64_t lb = __ballot(lh >= 0);
      n_local += (uint32_t)__popcll(lb);
      n_global += (uint32_t)__popcll(__ballot(true) & ~lb);
    };
    auto rate_batch = [&](const Batch& bt) {
    int my_h = bt.my_h;
    const int my_bit = bt.my_bit;
    const int32_t m = bt.m;
    const int mode = bt.mode, n0 = bt.n0, n1 = bt.n1, rank0 = bt.rank0, rank1 = bt.rank1;
    const int first = bt.first, prevdup = bt.prevdup;
    const int32_t id = bt.id;
    const bool inr = bt.inr, islast = bt.islast, own = bt.own, any_dup = bt.any_dup;
    const uint32_t lk0 = bt.lk0;
    const v4i gs = bt.gs, gm = bt.gm;
    // A counter can reach its count before the writes it announces have landed
    // (notifications do not wait for store acknowledgements): a group whose
    // granules do not carry the tags of their last writers retries next iteration.
    // The shared granule must name this match (if the player occurred earlier in
    // the window); its counters say how many times this launch wrote the mode
    // granule, and the mode granule must carry exactly that count.
    const uint32_t sa = (uint32_t)gs.y;
    const bool s_this = (sa & 0xffu) == (uint32_t)epoch;
    const uint32_t counters = s_this ? sa >> 8 : 0u;
    const uint32_t cnt = (counters >> (4 * mode)) & 15u;
    const bool shared_ok = !(lk0 & kLinkHasPred) || (s_this && (uint32_t)gs.w == (uint32_t)m);
    const bool mode_ok = cnt == 0u || (gm.y == epoch && (uint32_t)gm.w == cnt);
    const bool fresh = !own || (shared_ok && mode_ok);
    // race detector: a shared granule of this launch tagged for a LATER reader, or a
    // mode granule one write AHEAD of the verified count, means a successor wrote
    // before this match read -- the ordering protocol broke
    const bool overtaken =
        own && (((lk0 & kLinkHasPred) && s_this && (uint32_t)gs.w != kNoMatch &&
                 (uint32_t)gs.w > (uint32_t)m) ||
                (shared_ok && gm.y == epoch && (uint32_t)gm.w == (cnt == 15u ? 1u : cnt + 1u)));
    if (__ballot(overtaken) != 0ull && lane == 0) {
      atomicOr(&ctrl[2], 1u);
      atomicOr(&ctrl[18], 1u);  // sticky copy (never zeroed by a launch)
    }
    const uint64_t stale_lanes = __ballot(!fresh);
    if (stale_lanes) {
      const bool gstale = (stale_lanes & gmask) != 0ull;
      // diagnostics (ctrl[14] at exit): stale groups
      n_stale += (uint32_t)__popcll(__ballot(gstale && j == 0));
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        uint64_t back = 0ull;
        for (int q = 0; q < NG; ++q) {
          const int bq = __shfl(gstale && my_h == h ? my_bit : -1, q * G);
          if (bq >= 0) back |= 1ull << bq;
        }
        pend[h] |= uniform64(back);
      }
      if (gstale) my_h = -1;
    }
    if constexpr (INL) {
      // K8 inline, software-pipelined: this group's events are LOADED now (HBM, cold)
      // and folded into its stats one iteration later (tele_flush, after the next
      // wait), so no rating ever waits for event data; a stale group loads nothing
      // (it is retried, and aggregated then)
      if (tele_inline && my_h >= 0) {
        tn_m = m;
        tn_cnt = bt.tcnt;
        tn_off = bt.toff;
      }
#pragma unroll
      for (int t = 0; t < TT; ++t) {
        const bool okl = tele_inline && my_h >= 0 && j + G * t < bt.tcnt;
        const int32_t* src = okl ? tp.events + 2 * (bt.toff + j + G * t)
                                 : reinterpret_cast<const int32_t*>(tp.evoff);
        tev_next[t] = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(src));
      }
    }
    if (my_h >= 0) {
      const float smu = __int_as_float(gs.x), ssg = __int_as_float(gs.z);
      const float mmu = __int_as_float(gm.x), msg = __int_as_float(gm.z);
      // seed attributes only for players without a shared rating (their first
      // match): one extra round trip in the rare iterations that need it, instead
      // of a 16-B load per participant per match (-19% executor time on the bench)
      // player_prior (rate_core.h) as selects: only the seeding of a player's
      // first match (the attribute load, rare) stays a branch
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
      // duplicates see the pre-match values of their first occurrence (the
      // broadcasts only run when the batch has a repeated player)
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
      if (bt.tonly) gst = bt.est;  // inline telemetry: a stateless match keeps its early status
      if (gst == kRated && (n0 == 0 || n1 == 0)) gst = kErrEmptyRoster;
      float nsm = NAN, nss = NAN, nmm = NAN, nms = NAN, dl = NAN, q = NAN;
      if (gst == kRated) {
        if constexpr (DIAG) d_p[1] = __builtin_amdgcn_s_memrealtime();
        // both tracks as one packed pair (rate_dev.h): roster sign times winner side
        const float lsg = (r0 == (rank0 <= rank1)) ? 1.f : -1.f;
        f2 nm2, ns2;
        rate_pair<G>(f2{pms, pmm}, f2{pss, psm}, inr, lsg, n0 + n1, rank0 == rank1, beta2, tau2, j,
                     gbase, nm2, ns2, q);
        nsm = nm2.x;
        nmm = nm2.y;
        nss = ns2.x;
        nms = ns2.y;
        const bool bad_num = inr && !(isfinite(nsm) && isfinite(nss) && isfinite(nmm) &&
                                      isfinite(nms) && isfinite(q));
        if ((__ballot(bad_num) & gmask) != 0ull) gst = kErrNumeric;
        // conservative-skill delta (rater.py:150-153), in slot (= write) order
        const float cur = nsm - nss;
        const float prevw = any_dup ? __shfl(cur, gbase + (prevdup >= 0 ? prevdup : j)) : cur;
        if (prevdup >= 0) dl = cur - prevw;
        else if (pflags & 1u) dl = cur - (pms - pss);
        else dl = 0.f;
      }
      const bool ok = gst == kRated && inr;
      if constexpr (DIAG) d_p[2] = __builtin_amdgcn_s_memrealtime();
      if (inr && islast) {  // publish: new values, or the untouched ones on error
        const int off = id * (kRowFloats * 4);
        // shared granule: tagged with the next reader + bumped mode counter;
        // mode granule: tagged with its new write count
        const uint32_t succ = lk0 & kMatchMask;
        const uint32_t c4 = (rcnt >> (4 * mode)) & 15u;  // write count, wraps 15 -> 1
        const uint32_t c = c4 == 15u ? 1u : c4 + 1u;
        const uint32_t ncnt = (rcnt & ~(15u << (4 * mode))) | (c << (4 * mode));
        const uint32_t stag = (uint32_t)epoch | (ncnt << 8);
        __builtin_amdgcn_raw_buffer_store_b128(
            ok ? granule(nmm, (uint32_t)epoch, nms, c) : granule(rmmu, (uint32_t)epoch, rmsg, c),
            rs, off + 16 * (1 + mode), 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(
            ok ? granule(nsm, stag, nss, succ) : granule(rsmu, stag, rssg, succ),
            rs, off, 0, 16);
        notify(lk0 & kMatchMask);
      }
      if constexpr (DIAG) d_p[3] = __builtin_amdgcn_s_memrealtime();
      if (ok && prm.record_first_prior && own) {
        float* fp = first_prior + (int64_t)id * kRowFloats;
        if (pflags & 2u) { fp[0] = pms; fp[2] = pss; }
        if (pflags & 4u) { fp[4 * (1 + mode)] = pmm; fp[4 * (1 + mode) + 2] = psm; }
      }
      // output records are a write-once stream: non-temporal stores into the
      // match's packed 128-B row (ops/rate.py RateResult) keep them from competing
      // with the roster for cache (-6%) and make each match one line (-3%)
      float* const orm = orows + (int64_t)m * orow;  // [s_mu | s_sig | delta | m_mu | m_sig][S], quality, status
      float* const lr = lrow[wv][g];
      if (j < S) {
        lr[j] = ok ? nsm : NAN;
        lr[S + j] = ok ? nss : NAN;
        lr[2 * S + j] = ok ? dl : NAN;
        lr[3 * S + j] = ok ? nmm : NAN;
        lr[4 * S + j] = ok ? nms : NAN;
      }
      if (j == 0) {
        // (AFK / invalid rosters: quality 0 -- only tele-only groups carry those here)
        lr[5 * S] = gst == kRated ? q : (gst == kAfk || gst == kInvalidRosters) ? 0.f : NAN;
        lr[5 * S + 1] = __uint_as_float((uint32_t)gst);  // the status byte, upper bytes 0
      }
      if (j == (G > 1 ? 1 : 0)) {
#pragma unroll
        for (int k = 5 * S + 2; k < 4 * OQ; ++k) lr[k] = 0.f;  // row padding
      }
      // (the group's LDS writes and reads are the same wave's, in order)
#pragma unroll
      for (int t = 0; t < (OQ + G - 1) / G; ++t) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        const int qd = j + t * G;
        if (qd < OQ)
          __builtin_nontemporal_store(reinterpret_cast<const v4f*>(lr)[qd], reinterpret_cast<v4f*>(orm) + qd);
      }
    }
    };

    // ---------------------------------------------- (6) next ticket if a ring slot is free
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

    // ---------------------------------------------- (7) the one wait of the iteration
    uint64_t d_w0 = 0, d_w1 = 0;
    if constexpr (DIAG) d_w0 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (DIAG) d_w1 = __builtin_amdgcn_s_memrealtime();
    if constexpr (INL) {
      // the previous iteration's event loads retired in the wait above: re-define the
      // registers here so the compiler's own wait before tele_flush cannot also wait
      // for the event loads this iteration issues in between
#pragma unroll
      for (int t = 0; t < TT; ++t) asm volatile("" : "+v"(tev_prev[t]));
    }

    // ---------------------------------------------- (9) install the staged chunk
    int64_t early_m = -1;   // a staged match with an early status: its row, after the rating
    uint8_t early_est = kRated;
    if (staging >= 0) {
      int64_t cb = 0;
#pragma unroll
      for (int h = 0; h < kH; ++h) if (h == staging) cb = cbase[h];
      const int64_t mm = lane < cl ? cb + lane : M;  // idle lanes of a short chunk
      // flag matches that name one player twice (bit 3 of meta1, free in the
      // stream layout) so processing skips the duplicate scan for the rest; the
      // match is ready once every distinct player with an earlier occurrence
      // (kLinkHasPred on its first slot) has been published: that many
      // increments of its completion counter
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
      // inline telemetry: a stateless match is handed to a group like any ready one
      // (its counter needs 0), flagged tele-only (meta1 bit 4) with its status in bits 28..31
      const bool tonly = tele_inline && mm < M && est != kRated;
      if (tonly) r[S + 1] = (int32_t)(((uint32_t)r[S + 1] & 0x0fffffffu) | 16u | ((uint32_t)est << 28));
#pragma unroll
      for (int h = 0; h < kH; ++h)
        if (h == staging) {
#pragma unroll
          for (int k = 0; k < R; ++k) hrec[h][k] = r[k];
          hoff[h] = stoff;
          hcnt[h] = stcnt;
        }
      if constexpr (kLH) reinterpret_cast<uint32_t*>(&lloc[wv][lane])[staging] = 0u;
      // no state, no dependencies: its output row is written after this iteration's
      // rating (early_row), so the rating's waits never include these stores
      if (mm < M && est != kRated && !tonly) {
        early_m = mm;
        early_est = est;
      }
      const uint64_t pm = __ballot(mm < M && (est == kRated || tonly));
#pragma unroll
      for (int h = 0; h < kH; ++h)
        if (h == staging) {
          pend[h] = pm;
          dval[h] = kNone;  // first poll next iteration
          need[h] = tonly ? 0u : nd;  // a tele-only match's links are unwritten
          if (pm == 0ull) cbase[h] = -1;
        }
    }

    if constexpr (DIAG) d_p[0] = d_p[1] = d_p[2] = d_p[3] = d_w1;
    rate_batch(nb);
    if (early_m >= 0) {  // the staged chunk's early-status matches: one full-line row each
      typedef float v4f __attribute__((ext_vector_type(4)));
      const float qv = (early_est == kAfk || early_est == kInvalidRosters) ? 0.f : NAN;
      v4f* dst = reinterpret_cast<v4f*>(orows + early_m * orow);
#pragma unroll
      for (int q = 0; q < OQ; ++q) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int pos = 4 * q + i;
          v[i] = pos < 5 * S ? NAN : pos == 5 * S ? qv : pos == 5 * S + 1 ? __uint_as_float((uint32_t)early_est) : 0.f;
        }
        __builtin_nontemporal_store(v4f{v[0], v[1], v[2], v[3]}, dst + q);
      }
    }
    if constexpr (INL) {  // fold the previous batch's events, then hand this batch's on
      tele_flush();
#pragma unroll
      for (int t = 0; t < TT; ++t) tev_prev[t] = tev_next[t];
      tp_m = tn_m;
      tp_cnt = tn_cnt;
      tp_off = tn_off;
    }
    if constexpr (DIAG) {
      if (worked) {
        const uint64_t end = __builtin_amdgcn_s_memrealtime();
        d_issue += d_w0 - d_it0;
        d_wait += d_w1 - d_w0;
        d_after += end - d_w1;
        // the issue phase: staging + readiness, assignment, this batch's loads, polls + ticket
        d_s[0] += d_i[0] - d_it0;
        d_s[1] += d_i[1] - d_i[0];
        d_s[2] += d_i[2] - d_i[1];
        d_s[3] += d_w0 - d_i[2];
        // the markers are per lane (the rating ran in the assigned groups): take lane 0's group
        const uint64_t p1 = __builtin_amdgcn_readfirstlane((uint32_t)d_p[1]) |
                            ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(d_p[1] >> 32)) << 32);
        const uint64_t p2 = __builtin_amdgcn_readfirstlane((uint32_t)d_p[2]) |
                            ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(d_p[2] >> 32)) << 32);
        const uint64_t p3 = __builtin_amdgcn_readfirstlane((uint32_t)d_p[3]) |
                            ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(d_p[3] >> 32)) << 32);
        if (p1 >= d_w1 && p2 >= p1 && p3 >= p2 && end >= p3) {
          d_t[0] += p1 - d_w1;
          d_t[1] += p2 - p1;
          d_t[2] += p3 - p2;
          d_t[3] += end - p3;
        }
      }
    }

    // ---------------------------------------------- (5) next iteration's counter polls, as late as possible:
    // the readiness at the top waits for them, so what it sees is one rating
    // phase fresher than a poll issued before the wait
    ++iter;
    // straight-line sc1 buffer loads (served past the non-coherent L1); a lane
    // whose match is not pending loads out of range and gets 0, which readiness
    // masks with pend -- no exec branch per chunk
#pragma unroll
    for (int h = 0; h < kH; ++h)
      dval[h] = __builtin_amdgcn_raw_buffer_load_b32(rd, ((pend[h] >> lane) & 1ull) ? (cbase[h] + lane) * 4 : kOutOfRange,
                                                     0, 16);

    // ---------------------------------------------- (11) retire finished chunks
    {
      uint32_t retired = 0;
#pragma unroll
      for (int h = 0; h < kH; ++h)
        if (cbase[h] >= 0 && pend[h] == 0ull) {
          cbase[h] = -1;
          ++retired;
        }
      retired = __builtin_amdgcn_readfirstlane(retired);  // uniform: no waterfall loop
      if (retired && lane == 0)
        __hip_atomic_fetch_add((gu32*)&ctrl[3], retired, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // ---------------------------------------------- (12) done?
    bool held = false;
#pragma unroll
    for (int h = 0; h < kH; ++h) held |= cbase[h] >= 0;
    if (exhausted && !held && !tk_pending) {
      tele_flush();  // inline telemetry: the last batch's events
      if (lane == 0) {  // diagnostics: wave iterations (ctrl[15]), hand-offs (ctrl[26..27])
        __hip_atomic_fetch_add((gu32*)&ctrl[15], iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add((gu32*)&ctrl[26], n_local, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add((gu32*)&ctrl[27], n_global, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n_stale) __hip_atomic_fetch_add((gu32*)&ctrl[14], n_stale, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (DIAG) {
          // iterations that rated something: [20] count, [21] groups assigned, and
          // 100 MHz s_memrealtime ticks [22..23] issue (top of the loop -> the wait),
          // [24..25] the wait, [28..29] after it (rating, publish, bookkeeping)
          __hip_atomic_fetch_add((gu32*)&ctrl[20], d_worked, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add((gu32*)&ctrl[21], d_groups, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          // [30] matches one dependency short of ready, [31] pending, summed over worked iterations
          __hip_atomic_fetch_add((gu32*)&ctrl[30], d_near, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add((gu32*)&ctrl[31], d_pend, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          atomicAdd(reinterpret_cast<unsigned long long*>(&ctrl[22]), (unsigned long long)d_issue);
          atomicAdd(reinterpret_cast<unsigned long long*>(&ctrl[24]), (unsigned long long)d_wait);
          atomicAdd(reinterpret_cast<unsigned long long*>(&ctrl[28]), (unsigned long long)d_after);
          // [32..39] the after phase split: prior + sums, update, publish, outputs + rest
          for (int q = 0; q < 4; ++q)
            atomicAdd(reinterpret_cast<unsigned long long*>(&ctrl[32 + 2 * q]), (unsigned long long)d_t[q]);
          // [40..47] the issue phase split
          for (int q = 0; q < 4; ++q)
            atomicAdd(reinterpret_cast<unsigned long long*>(&ctrl[40 + 2 * q]), (unsigned long long)d_s[q]);
        }
      }
      if constexpr (TILES) {
        while (!tele_done) {  // leftover telemetry tiles
          const int64_t t = tele_claim();
          if (t < 0) tele_done = true;
          else tele_run(t);
        }
      }
      break;
    }

    // ---------------------------------------------- (13) idle: back off, bounded
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
          if (cbase[h] >= 0 && ((pend[h] >> lane) & 1ull))
            reinterpret_cast<uint8_t*>(orows + (int64_t)(cbase[h] + lane) * orow + 5 * S + 1)[0] = kNotProcessed;
        return;  // give up: the host sees ctrl[1] and raises
      }
      if constexpr (TILES) {
        // nothing ready for a while: aggregate a telemetry tile instead of sleeping
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


// both control ranges of a launch in one dispatch: [a, a + na) and [b, b + nb)
__global__ void __launch_bounds__(64) zero_ctrl2_kernel(uint32_t* __restrict__ a, int na,
                                                        uint32_t* __restrict__ b, int nb) {
  if ((int)threadIdx.x < na) a[threadIdx.x] = 0u;
  if ((int)threadIdx.x < nb) b[threadIdx.x] = 0u;
}

int launch_rate(int K, const int32_t* rec, const uint32_t* link, int32_t* deps, float* state,
                const float* attrs, float* first_prior, const RateOut& out, uint32_t* ctrl,
                const RateParams& prm, const TelemetryParams& tp, int blocks, hipStream_t s) {
  const int64_t M = prm.num_matches;
  // ctrl[0] = schedule flag (kept), [1] timeout, [2] protocol, [3] retired chunks, [4..11] tickets,
  // [12] telemetry tile ticket, [13] malformed telemetry events, [14] stale reads retried,
  // [15] wave iterations; [16..18] sticky OR of [0..2] over launches (host clears);
  // [20..25], [28..29] timing build (see the kernel), [26] local / [27] global hand-offs
  // one-wave kernel rather than hipMemsetAsync: a 60-B fill at a 4-B offset becomes two
  // runtime fill dispatches (~4.7 us each on a 500-match micro-batch, profiles/)
  // the diagnostic words [20..51] are zeroed by every launch (not by the schedule's zeroing)
  hipLaunchKernelGGL(zero_ctrl2_kernel, dim3(1), dim3(64), 0, s, ctrl + 1, prm.ctrl_ready ? 0 : 15,
                     ctrl + 20, 32);
  if (M <= 0) return 0;
  if (prm.chunk_len < 1 || prm.chunk_len > kChunk) return (int)hipErrorInvalidValue;
  if ((int64_t)prm.num_players * kRowFloats * 4 > kOutOfRange) return (int)hipErrorInvalidValue;
  if (M * 2 * K * 4 > kOutOfRange) return (int)hipErrorInvalidValue;  // links, read by resource
  if (!prm.epoch_ptr && (prm.epoch < 1 || prm.epoch > 255)) return (int)hipErrorInvalidValue;
  // the executor writes one packed row per match (ops/rate.py RateResult.allocate)
  const int S = 2 * K;
  if (!(out.s_sig == out.s_mu + S && out.delta == out.s_mu + 2 * S && out.m_mu == out.s_mu + 3 * S &&
        out.m_sig == out.s_mu + 4 * S && out.quality == out.s_mu + 5 * S && out.qrow == out.row &&
        (void*)out.status == (void*)(out.s_mu + 5 * S + 1) && out.srow == out.row * 4))
    return (int)hipErrorInvalidValue;
  if (blocks < kHeads) blocks = kHeads;
  // lanes per match: the next power of two (DPP butterfly sums) or exactly 2K
  // (more matches per wave iteration, bpermute-tree sums).  Measured on MI355X
  // with this executor: 3v3 6.23-6.26 ms with 8 lanes vs 6.27-6.30 with 6 (10M
  // window), 5v5 18.23-18.42 ms with 10 lanes vs 18.42-18.61 with 16 (12.5M;
  // config 3 step 21.5 vs 21.9 ms, profiles/r2/tight_groups.log) -> auto = tight
  // for 5v5 only.
  const bool tight = prm.tight_groups > 0 || (prm.tight_groups < 0 && K == 5);
#define ANA_RATE_LAUNCH_W(k, g, tele, diag, w)                                                     \
  hipLaunchKernelGGL((rate_dataflow_kernel<k, g, tele, diag, w>), dim3((unsigned)blocks), dim3(256), 0, s, \
                     rec, link, deps, state, attrs, first_prior, out.s_mu, out.row, ctrl, prm, tp)
#define ANA_RATE_LAUNCH_D(k, g, tele, diag)                                                        \
  do {                                                                                             \
    if constexpr (tele == 0 && !diag && k <= 3 && (g & (g - 1)) == 0) {                            \
      if (blocks > 256) ANA_RATE_LAUNCH_W(k, g, tele, diag, 4); /* two waves per SIMD */          \
      else ANA_RATE_LAUNCH_W(k, g, tele, diag, 1);                                                 \
    } else {                                                                                       \
      ANA_RATE_LAUNCH_W(k, g, tele, diag, 1);                                                      \
    }                                                                                              \
  } while (0)
#define ANA_RATE_LAUNCH(k, g)                                      \
  do {                                                             \
    if (tp.evoff && tp.role_stride < 0) ANA_RATE_LAUNCH_D(k, g, 2, false); \
    else if (tp.evoff) ANA_RATE_LAUNCH_D(k, g, 1, false);          \
    else if (prm.diag) ANA_RATE_LAUNCH_D(k, g, 0, true);           \
    else ANA_RATE_LAUNCH_D(k, g, 0, false);                        \
  } while (0)
  switch (K) {
    case 1: ANA_RATE_LAUNCH(1, 2); break;
    case 2: ANA_RATE_LAUNCH(2, 4); break;
    case 3:
      if (tight) ANA_RATE_LAUNCH(3, 6);
      else ANA_RATE_LAUNCH(3, 8);
      break;
    case 4: ANA_RATE_LAUNCH(4, 8); break;
    case 5:
      if (tight) ANA_RATE_LAUNCH(5, 10);
      else ANA_RATE_LAUNCH(5, 16);
      break;
    default: return (int)hipErrorInvalidValue;
  }
#undef ANA_RATE_LAUNCH
#undef ANA_RATE_LAUNCH_D
  return (int)hipGetLastError();
}

}  // namespace ana
