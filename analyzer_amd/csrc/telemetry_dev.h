// K8 device side: aggregate the telemetry of one tile of matches with ONE wave
// (no barriers, so the dataflow executor can run it in its idle time).
//
// The tile's stat block [T][2K][kStatFeatures] lives in the wave's LDS
// scratch; events of the tile (contiguous: evoff is a CSR index) are streamed
// with 8-B loads (8 per lane in flight), folded in with LDS float atomics
// (ds_add_f32: contention only among a match's participants); the block then
// leaves LDS as one contiguous, coalesced store -- the per-match stat rows of
// consecutive matches are adjacent in the [M][2K][F] output.
#pragma once

#include <hip/hip_runtime.h>

#include "telemetry_core.h"

namespace ana {

template <int K, int D = 0>
__device__ __forceinline__ void telemetry_tile(const TelemetryParams& tp, int64_t tile, int lane,
                                               float* lds, uint32_t* bad_events) {
  constexpr int S = 2 * K;
  constexpr int kRow = S * kStatFeatures;
  // participant rows padded to an odd stride in LDS: rows 8 floats apart would
  // put every row's feature f in the same 4 of the 32 banks
  constexpr int kPad = kStatFeatures + 1;
  const int64_t m0 = tile * kTeleTile;
  const int64_t m1 = m0 + kTeleTile < tp.num_matches ? m0 + kTeleTile : tp.num_matches;
  const int n = (int)(m1 - m0) * kRow;
  const int npad = (int)(m1 - m0) * S * kPad;
  for (int i = lane; i < npad; i += 64) lds[i] = 0.f;
  const int64_t e0 = tp.evoff[m0], e1 = tp.evoff[m1];
  uint32_t bad = 0;
  // 8 events per lane in flight: the loads of a batch retire in one round trip
  constexpr int kBatch = 8;
  for (int64_t base = e0; base < e1; base += 64 * kBatch) {
    int2 ev[kBatch];
#pragma unroll
    for (int q = 0; q < kBatch; ++q) {
      const int64_t e = base + q * 64 + lane;
      ev[q] = e < e1 ? reinterpret_cast<const int2*>(tp.events)[e] : make_int2(-1, 0);
    }
#pragma unroll
    for (int q = 0; q < kBatch; ++q) {
      if (base + q * 64 + lane >= e1) continue;
      // the tile-relative match its tag names (tiles are far shorter than 2^16 matches)
      const int64_t ml = (int64_t)((event_tag(ev[q].x) - (uint32_t)(m0 & 0xffff)) & 0xffffu);
      const int slot = event_slot(ev[q].x);
      const int64_t e = base + q * 64 + lane;
      if (ml < 0 || ml >= m1 - m0 || slot >= S || e < tp.evoff[m0 + ml] || e >= tp.evoff[m0 + ml + 1]) {
        ++bad;
        continue;
      }
      float add;
      const int f = event_feature(event_type(ev[q].x), __int_as_float(ev[q].y), add);
      float* row = lds + (ml * S + slot) * kPad;
      if constexpr (D == 1) {  // diagnostic: no LDS adds (timing only)
        bad += f == 99;
        continue;
      }
      if (f >= 0) atomicAdd(row + f, add);
      if constexpr (D != 2) atomicAdd(row + kStatEvents, 1.f);  // D == 2: diagnostic
    }
  }
  if (bad) atomicAdd(bad_events, bad);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the LDS adds have landed (wave-local)
  float* dst = tp.stats + m0 * kRow;
  for (int i = lane; i < n; i += 64) dst[i] = lds[(i / kStatFeatures) * kPad + i % kStatFeatures];
}

}  // namespace ana

namespace ana {

// ---------------------------------------------------------------------------
// K8 on the matrix cores: the per-participant aggregation is a one-hot GEMM.
//
//   stats_tile[row][col] = sum_e  A[row][e] * B[e][col]
//
// rows = (match, slot) of the wave's span of matches (span x 2K rows, in tiles
// of 16 rows); A[row][e] = 1 iff event e is attributed to that row; B[e][col] =
// the event's contribution to 16 columns: [0] count, [1..3] kills/deaths/
// assists (1.0), [4..15] damage/gold/farm/heal as exact 3-way bf16 splits (hi,
// mid, lo: 8+8+8 significand bits = the full fp32 value).  One
// v_mfma_f32_16x16x32_bf16 folds 32 events into a 16-row tile.  This replaces
// the LDS float atomics of telemetry_tile, whose same-address conflicts
// serialise (4.45 ms for 400M events; 1.57 ms with the adds removed).
//
// Events stream linearly through the tile, 64 per lane-parallel load with
// kTeleMfmaLoads loads in flight, rotated through registers by a rolled loop.
// Each load is decoded once and scattered (b16 stores) into two operand tile
// sets in LDS, one per 32-event chunk: B^T [16 columns][32 events] and an A^T
// window [32 rows][32 events] starting at the chunk's first row tile.  All six
// fragments are read back with one wait, then MFMAs fold each chunk into two
// live accumulators that slide over the tile's row tiles (the stream visits
// them in order; a chunk whose events reach a third row tile takes extra
// windows).  A finished row tile leaves through a [16][17] LDS stage as 512
// contiguous bytes of stats rows.
//
// Attribution is strict: an event counts for the match it names iff it sits in
// that match's CSR range and its slot is < 2K; every other event is malformed
// (counted in *bad_events).  Non-finite values stay out of the GEMM (0 x Inf
// in another row's product would be NaN) and are added afterwards by a rare
// slow path.  Tile rows are 32 bf16 + 16 B of pad (80 B).
constexpr int kTeleChunk = 32;
constexpr int kTeleRowBytes = kTeleChunk * 2 + 16;
constexpr int kTeleARows = 32;
#ifndef ANA_TELE_LOADS
#define ANA_TELE_LOADS 8  // 1.87 vs 1.95 ms (4) and 2.08 ms (2) for 400M events, profiles/r2/tele_loads_ab.log
#endif
constexpr int kTeleMfmaLoads = ANA_TELE_LOADS;  // 64-event loads per lane in flight
constexpr int kTeleBOffset = kTeleARows * kTeleRowBytes;           // within a set
// A^T window + B^T, + 64 B so set 1 starts 16 banks over (both sets take stores together)
constexpr int kTeleSetBytes = kTeleBOffset + 16 * kTeleRowBytes + 64;
constexpr int kTeleRelOffset = 2 * kTeleSetBytes;
constexpr int kTeleMaxSpan = 63;  // matches per call: span + 1 CSR offsets on the lanes
constexpr int kTeleMfmaBytes = kTeleRelOffset + (kTeleMaxSpan + 4) / 4 * 16;
// per-wave LDS scratch (floats) that fits either tile routine
template <int K>
constexpr int tele_scratch_floats() {
  constexpr int atomic_floats = kTeleTile * 2 * K * (kStatFeatures + 1);
  constexpr int mfma_floats = (kTeleMfmaBytes + 15) / 16 * 4;
  return atomic_floats > mfma_floats ? atomic_floats : mfma_floats;
}

typedef __bf16 tele_bf16x8 __attribute__((ext_vector_type(8)));
typedef float tele_f32x4 __attribute__((ext_vector_type(4)));
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int tele_i32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void tele_lds_fence() {
  // LDS ops of one wave execute in order; this only pins the program order
  __asm__ __volatile__("" ::: "memory");
}

__device__ __forceinline__ void tele_st16(uint8_t* p, uint32_t v) {
  *reinterpret_cast<uint16_t*>(p) = (uint16_t)v;
}

__device__ __forceinline__ tele_f32x4 tele_mfma(uint4 a, uint4 b, tele_f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(tele_bf16x8, a),
                                                 __builtin_bit_cast(tele_bf16x8, b), c, 0, 0, 0);
}

// Aggregates the SPAN matches [tile * SPAN, +SPAN) (the fused executor claims
// kTeleTile-match tiles; the standalone kernel takes longer spans per wave).
// DIAG (timing-only builds, ANA_TELE_DEBUG 6 / 7): 3 = no MFMA, 4 = decode only
template <int K, int DIAG = 0, int SPAN = kTeleTile>
__device__ __forceinline__ void telemetry_tile_mfma(const TelemetryParams& tp, int64_t tile, int lane,
                                                    float* lds_f, uint32_t* bad_events) {
  constexpr int S = 2 * K;
  constexpr int NB = kTeleMfmaLoads;
  constexpr uint32_t kOne = 0x3f80;  // bf16 1.0
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds_f);
  int32_t* rel = reinterpret_cast<int32_t*>(lds + kTeleRelOffset);  // tile CSR, relative
  // the tile is wave-uniform (callers derive it from threadIdx.x >> 6, which the
  // compiler cannot prove): pin it, and everything derived from it, to SGPRs
  tile = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(tile >> 32)) << 32) |
                   (uint32_t)__builtin_amdgcn_readfirstlane((int)tile));
  static_assert(SPAN >= 1 && SPAN <= kTeleMaxSpan, "span must fit the lanes");
  const int64_t m0 = tile * SPAN;
  const int nm = (int)(tp.num_matches - m0 < SPAN ? tp.num_matches - m0 : SPAN);
  const int64_t off = lane <= nm ? __builtin_nontemporal_load(tp.evoff + m0 + lane) : 0;
  const int64_t e0 = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(off >> 32), 0) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)off, 0));
  const int32_t roff = (int32_t)(off - e0);  // lane j <= nm: first event of match j
  tele_lds_fence();
  if (lane <= nm) rel[lane] = roff;
  for (int i = lane; i < kTeleRelOffset / 16; i += 64)  // both operand sets start zero
    reinterpret_cast<uint4*>(lds)[i] = make_uint4(0, 0, 0, 0);
  tele_lds_fence();
  // B^T row 0 (the count column) is 1.0 for EVERY event position, kept for the whole
  // span: an event outside the rows (malformed, past the span) has an all-zero A
  // column, so only attributed events count -- no store + undo of it per event
  if (lane < 2 * kTeleChunk)
    tele_st16(lds + (lane >> 5) * kTeleSetBytes + kTeleBOffset + 2 * (lane & 31), kOne);
  tele_lds_fence();
  auto bound = [&](int j) { return __builtin_amdgcn_readlane(roff, j); };
  const int ne = __builtin_amdgcn_readfirstlane(bound(nm));
  const int t = lane & 31, half = lane >> 5;
  const int fr = lane & 15, fg = lane >> 4;  // fragment row/column and k-group
  uint8_t* mine_set = lds + half * kTeleSetBytes;
  const int2* __restrict__ evs = reinterpret_cast<const int2*>(tp.events) + e0;
  // two live 16-row accumulators: row tiles c and c + 1
  tele_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  int c = 0;
  const int nrows = nm * S;
  float* dst = tp.stats + m0 * S * kStatFeatures;
  float* st = reinterpret_cast<float*>(lds);  // [16][17] stage over set 0's A^T window
  auto shift = [&]() {  // row tile c is final: store it, slide by one
    tele_lds_fence();
#pragma unroll
    for (int j = 0; j < 4; ++j) st[(4 * fg + j) * 17 + fr] = acc0[j];
    tele_lds_fence();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int o = lane + 64 * h;
      const float* r = st + (o >> 3) * 17;
      const int f = o & 7;
      // column of feature f: 1 + f (kills..assists), 3f - 5 (+1, +2: value splits), 0 (count)
      const bool split = f >= 3 && f < kStatEvents;
      const int c0 = f < 3 ? f + 1 : split ? 3 * f - 5 : 0;
      const float x0 = r[c0], x1 = r[split ? c0 + 1 : 16], x2 = r[split ? c0 + 2 : 16];
      const float v = split ? (x0 + x1) + x2 : x0;
      // non-temporal: the stats (2 GB per 10M 3v3 window) and the events (3.2 GB) stream
      // past the Infinity Cache instead of evicting the roster the co-running executor
      // gathers from -- config 4 step 9.66 -> 9.34 ms, the kernel alone unchanged; loads
      // or stores alone 9.62 / 9.56 (profiles/r5/config4_nontemporal.log)
      if (16 * c + (o >> 3) < nrows) __builtin_nontemporal_store(v, dst + 16 * c * kStatFeatures + o);
    }
    tele_lds_fence();
    // the operand tiles are kept zero between uses: clear the stage's 1088 B
    *reinterpret_cast<uint4*>(lds + 16 * lane) = make_uint4(0, 0, 0, 0);
    if (lane < 4) *reinterpret_cast<uint4*>(lds + 1024 + 16 * lane) = make_uint4(0, 0, 0, 0);
    tele_lds_fence();
    acc0 = acc1;
    acc1 = tele_f32x4{0.f, 0.f, 0.f, 0.f};
    ++c;
  };
  uint32_t bad = 0;
  bool nonfinite = false;
  // the match whose CSR range holds position pos: the last j < nm with start_j <= pos
  // (starts are non-decreasing; empty matches share their successor's start)
  auto match_at = [&](int pos) {
    return (int)__builtin_popcountll(__builtin_amdgcn_ballot_w64(lane < nm && roff <= pos)) - 1;
  };
  // groups of NB 64-event loads: all issued, then consumed in order (counted
  // vmcnt waits); other waves on the SIMD cover the gap between groups.  Loads
  // are unconditional (positions past the span re-read its last event; the
  // decode masks them): conditional loads make the compiler wait for all.
  // (events are 8 B since round 2: half the bytes of the round-1 16-B records)
  const int elast = ne > 0 ? ne - 1 : 0;
  for (int pr = 0; pr < ne; pr += 64 * NB) {
    int2 ev[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const tele_i32x2 x = __builtin_nontemporal_load(reinterpret_cast<const tele_i32x2*>(evs + min(pr + 64 * q + lane, elast)));
      ev[q] = make_int2(x.x, x.y);
    }
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int pb = pr + 64 * q;
    if (pb >= ne) break;
    const int2 cur = ev[q];
    // the two chunks: first/last positions and the row tiles they can touch
    const int n1 = ne - pb - kTeleChunk;  // events of chunk 1 (<= 0: none)
    const int ms0 = match_at(pb);
    const int me0 = match_at((n1 > 0 ? pb + kTeleChunk : ne) - 1);
    const int ms1 = n1 > 0 ? match_at(pb + kTeleChunk) : me0;
    const int me1 = n1 > 0 ? match_at(pb + kTeleChunk + (n1 < kTeleChunk ? n1 : kTeleChunk) - 1) : me0;
    const int ilo0 = (ms0 * S) >> 4, ihi0 = ((me0 + 1) * S - 1) >> 4;
    const int ilo1 = (ms1 * S) >> 4, ihi1 = ((me1 + 1) * S - 1) >> 4;
    // decode this lane's event (branch-free); it must sit in the CSR range of the
    // match it names, and its slot must be < 2K
    const int e = pb + lane;
    // the span-relative match the event's 16-bit tag names (spans are <= 63 matches)
    const int xw = (int)((event_tag(cur.x) - (uint32_t)(m0 & 0xffff)) & 0xffffu);
    const int seg = xw >= nm ? nm - 1 : xw;
    const int slot = event_slot(cur.x);
    const int r0 = rel[seg], r1e = rel[seg + 1];
    const bool ok = e < ne && xw == seg && slot < S && e >= r0 && e < r1e;
    bad += (e < ne && !ok) ? 1u : 0u;
    const int row = seg * S + slot;
    // type -> B columns (event_feature): 0..2 kills/deaths/assists at column 1 + type,
    // 3..6 damage/gold/farm/heal as (hi, mid, lo) at columns 3 type - 5 .. 3 type - 3
    const int type = event_type(cur.x);
    const float value = __int_as_float(cur.y);
    const bool counted = ok && type < 3;
    const bool summed = ok && type >= 3 && type <= 6;
    const bool finite = __builtin_isfinite(value);
    nonfinite |= summed && !finite;
    const int col = counted ? type + 1 : (summed && finite) ? 3 * type - 5 : -1;
    const uint32_t hb = __float_as_uint(value) & 0xffff0000u;
    const float rv = value - __uint_as_float(hb);
    const uint32_t mb = __float_as_uint(rv) & 0xffff0000u;
    const uint32_t p0 = counted ? kOne : hb >> 16;
    const uint32_t p1 = mb >> 16;
    const uint32_t p2 = __float_as_uint(rv - __uint_as_float(mb)) >> 16;
    if constexpr (DIAG == 4) {
      if (ok) acc0[0] += (float)(col + p0 + p1 + p2 + row);
      continue;
    }
    // scatter this lane's event into its chunk's operand set (the tiles are zero
    // between uses: every store is undone once the fragments are read)
    const int lr = row - 16 * (half ? ilo1 : ilo0);
    uint8_t* bcol = mine_set + kTeleBOffset + 2 * t;
    uint8_t* arow = mine_set + lr * kTeleRowBytes + 2 * t;
    const bool in_a = ok && lr < kTeleARows;
    if (ok) {  // (column 0, the count, is a constant 1.0 row: see above)
      if (col >= 0) {
        tele_st16(bcol + col * kTeleRowBytes, p0);
        if (col >= 4) {
          tele_st16(bcol + (col + 1) * kTeleRowBytes, p1);
          tele_st16(bcol + (col + 2) * kTeleRowBytes, p2);
        }
      }
    }
    if (in_a) tele_st16(arow, kOne);
    tele_lds_fence();
    uint4 a[2][2], b[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint8_t* sb = lds + h * kTeleSetBytes + fr * kTeleRowBytes + fg * 16;
      b[h] = *reinterpret_cast<const uint4*>(sb + kTeleBOffset);
      a[h][0] = *reinterpret_cast<const uint4*>(sb);
      a[h][1] = *reinterpret_cast<const uint4*>(sb + 16 * kTeleRowBytes);
    }
    tele_lds_fence();
    if (ok) {
      if (col >= 0) {
        tele_st16(bcol + col * kTeleRowBytes, 0);
        if (col >= 4) {
          tele_st16(bcol + (col + 1) * kTeleRowBytes, 0);
          tele_st16(bcol + (col + 2) * kTeleRowBytes, 0);
        }
      }
    }
    if (in_a) tele_st16(arow, 0);
    tele_lds_fence();
    if constexpr (DIAG == 3) {
      acc0[0] += __uint_as_float(a[0][0].x ^ a[0][1].y ^ b[0].z ^ a[1][0].x ^ a[1][1].y ^ b[1].z);
      continue;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && n1 <= 0) break;
      const int ilo = h ? ilo1 : ilo0, ihi = h ? ihi1 : ihi0;
      while (c < ilo) shift();
      acc0 = tele_mfma(a[h][0], b[h], acc0);
      if (ihi > c) acc1 = tele_mfma(a[h][1], b[h], acc1);
      while (ihi > c + 1) {
        // rare: the chunk reaches a third row tile.  Tile c is final; the window
        // at the new c folds only its upper half (the new tile c + 1)
        shift();
        uint8_t* sa = lds + h * kTeleSetBytes;
        const int lr2 = row - 16 * c;
        const bool in2 = ok && half == h && lr2 >= 16 && lr2 < kTeleARows;
        if (in2) tele_st16(sa + lr2 * kTeleRowBytes + 2 * t, kOne);
        tele_lds_fence();
        const uint4 a1 = *reinterpret_cast<const uint4*>(sa + (16 + fr) * kTeleRowBytes + fg * 16);
        tele_lds_fence();
        if (in2) tele_st16(sa + lr2 * kTeleRowBytes + 2 * t, 0);
        tele_lds_fence();
        acc1 = tele_mfma(a1, b[h], acc1);
      }
    }
  }
  }
  while (16 * c < nrows) shift();  // the last live tiles and any tiles without events
  if (__builtin_amdgcn_ballot_w64(nonfinite)) {
    // rare slow path: add the tile's Inf/NaN values on top of the stored sums
    __threadfence();
    for (int e = lane; e < ne; e += 64) {
      const int2 x = evs[e];
      const int xm = (int)((event_tag(x.x) - (uint32_t)(m0 & 0xffff)) & 0xffffu);
      const int slot = event_slot(x.x);
      if (xm >= nm || slot >= S || e < rel[xm] || e >= rel[xm + 1]) continue;
      float add;
      const int f = event_feature(event_type(x.x), __int_as_float(x.y), add);
      if (f >= 3 && !__builtin_isfinite(add)) atomicAdd(dst + (xm * S + slot) * kStatFeatures + f, add);
    }
  }
  if (bad) atomicAdd(bad_events, bad);
}

#if ANA_DIAG_BUILD  // measured slower (3.94 vs 1.82 ms, profiles/r4/telemetry_register_fragments.log): diagnostic library only
// impl 3: the same one-hot GEMM with the fragments built in REGISTERS.  Each lane
// decodes its event once (as above) into two words in LDS -- {row | column + 1 << 10 |
// p2 << 16, p0 | p1 << 16} -- and every lane then reads the 8 records of its MFMA
// k-group (lanes 16 fg .. 16 fg + 15 read the same 64 B: broadcast, conflict-free) and
// builds its A fragment (1.0 where the event's row is the lane's row of the tile) and
// its B fragment (the event's bf16 part for the lane's column) with compares and
// selects.  Where impl 1 scatters b16 operands into LDS tiles at event-chosen rows
// (2.55 bank-conflict cycles per LDS instruction, an undo per store, 23 LDS
// instructions per 64 events), this is one 8-B store and 4-8 broadcast 16-B reads per
// 64 events, for ~4x the VALU work of the scatter.
// LDS of one impl-3 wave: [16][17] float stage, 64 decoded events, span + 1 CSR offsets
constexpr int kTeleRegsFloats = 16 * 17 + 64 * 2 + kTeleMaxSpan + 5;
template <int K, int SPAN = kTeleMaxSpan>
__device__ __forceinline__ void telemetry_tile_regs(const TelemetryParams& tp, int64_t tile, int lane,
                                                    float* lds_f, uint32_t* bad_events) {
  constexpr int S = 2 * K;
  constexpr int NB = kTeleMfmaLoads;
  constexpr uint32_t kOne = 0x3f80;  // bf16 1.0
  constexpr int kStageBytes = 16 * 17 * 4;
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds_f);
  float* st = reinterpret_cast<float*>(lds);                              // [16][17] output stage
  uint2* recs = reinterpret_cast<uint2*>(lds + kStageBytes);              // [64] decoded events
  int32_t* rel = reinterpret_cast<int32_t*>(lds + kStageBytes + 64 * 8);  // span CSR, relative
  tile = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(tile >> 32)) << 32) |
                   (uint32_t)__builtin_amdgcn_readfirstlane((int)tile));
  static_assert(SPAN >= 1 && SPAN <= kTeleMaxSpan, "span must fit the lanes");
  static_assert(SPAN * S < 1023, "rows are 10-bit in the decoded record (1023 = none)");
  const int64_t m0 = tile * SPAN;
  const int nm = (int)(tp.num_matches - m0 < SPAN ? tp.num_matches - m0 : SPAN);
  const int64_t off = lane <= nm ? tp.evoff[m0 + lane] : 0;
  const int64_t e0 = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(off >> 32), 0) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)off, 0));
  const int32_t roff = (int32_t)(off - e0);
  tele_lds_fence();
  if (lane <= nm) rel[lane] = roff;
  tele_lds_fence();
  const int ne = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(roff, nm));
  const int fr = lane & 15, fg = lane >> 4;  // fragment row / column, k-group
  const int2* __restrict__ evs = reinterpret_cast<const int2*>(tp.events) + e0;
  tele_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  int c = 0;
  const int nrows = nm * S;
  float* dst = tp.stats + m0 * S * kStatFeatures;
  auto shift = [&]() {  // row tile c is final: store it through the stage, slide by one
    tele_lds_fence();
#pragma unroll
    for (int j = 0; j < 4; ++j) st[(4 * fg + j) * 17 + fr] = acc0[j];
    tele_lds_fence();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int o = lane + 64 * h;
      const float* r = st + (o >> 3) * 17;
      const int f = o & 7;
      const bool split = f >= 3 && f < kStatEvents;
      const int c0 = f < 3 ? f + 1 : split ? 3 * f - 5 : 0;
      const float v = split ? (r[c0] + r[c0 + 1]) + r[c0 + 2] : r[c0];
      if (16 * c + (o >> 3) < nrows) dst[16 * c * kStatFeatures + o] = v;
    }
    tele_lds_fence();
    acc0 = acc1;
    acc1 = tele_f32x4{0.f, 0.f, 0.f, 0.f};
    ++c;
  };
  // A fragment of row tile tl: bf16 1.0 at k = i where the i-th event of this lane's
  // k-group lies on row 16 tl + fr
  auto a_frag = [&](const uint32_t (&row)[8], int tl) {
    const uint32_t want = (uint32_t)(16 * tl + fr);
    uint32_t w[4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
      w[p] = (row[2 * p] == want ? kOne : 0u) | (row[2 * p + 1] == want ? kOne << 16 : 0u);
    return make_uint4(w[0], w[1], w[2], w[3]);
  };
  uint32_t bad = 0;
  bool nonfinite = false;
  auto match_at = [&](int pos) {
    return (int)__builtin_popcountll(__builtin_amdgcn_ballot_w64(lane < nm && roff <= pos)) - 1;
  };
  const int elast = ne > 0 ? ne - 1 : 0;
  for (int pr = 0; pr < ne; pr += 64 * NB) {
    int2 ev[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) ev[q] = evs[min(pr + 64 * q + lane, elast)];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int pb = pr + 64 * q;
    if (pb >= ne) break;
    const int2 cur = ev[q];
    const int n1 = ne - pb - kTeleChunk;
    const int ms0 = match_at(pb);
    const int me0 = match_at((n1 > 0 ? pb + kTeleChunk : ne) - 1);
    const int ms1 = n1 > 0 ? match_at(pb + kTeleChunk) : me0;
    const int me1 = n1 > 0 ? match_at(pb + kTeleChunk + (n1 < kTeleChunk ? n1 : kTeleChunk) - 1) : me0;
    const int ilo0 = (ms0 * S) >> 4, ihi0 = ((me0 + 1) * S - 1) >> 4;
    const int ilo1 = (ms1 * S) >> 4, ihi1 = ((me1 + 1) * S - 1) >> 4;
    // decode this lane's event (as impl 1)
    const int e = pb + lane;
    const int xw = (int)((event_tag(cur.x) - (uint32_t)(m0 & 0xffff)) & 0xffffu);
    const int seg = xw >= nm ? nm - 1 : xw;
    const int slot = event_slot(cur.x);
    const int r0 = rel[seg], r1e = rel[seg + 1];
    const bool ok = e < ne && xw == seg && slot < S && e >= r0 && e < r1e;
    bad += (e < ne && !ok) ? 1u : 0u;
    const int type = event_type(cur.x);
    const float value = __int_as_float(cur.y);
    const bool counted = ok && type < 3;
    const bool summed = ok && type >= 3 && type <= 6;
    const bool finite = __builtin_isfinite(value);
    nonfinite |= summed && !finite;
    const bool split = summed && finite;
    const int col = counted ? type + 1 : split ? 3 * type - 5 : -1;
    const uint32_t hb = __float_as_uint(value) & 0xffff0000u;
    const float rv = value - __uint_as_float(hb);
    const uint32_t mb = __float_as_uint(rv) & 0xffff0000u;
    const uint32_t p0 = counted ? kOne : split ? hb >> 16 : 0u;
    const uint32_t p1 = split ? mb >> 16 : 0u;
    const uint32_t p2 = split ? __float_as_uint(rv - __uint_as_float(mb)) >> 16 : 0u;
    // an unattributed event gets row 1023 (no tile row): its A column stays zero
    const uint32_t row = ok ? (uint32_t)(seg * S + slot) : 1023u;
    tele_lds_fence();
    recs[lane] = make_uint2(row | ((uint32_t)(col + 1) << 10) | (p2 << 16), p0 | (p1 << 16));
    tele_lds_fence();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && n1 <= 0) break;
      // the 8 records of this lane's k-group in chunk h: 64 B, four 16-B reads
      const uint4* src = reinterpret_cast<const uint4*>(recs + 32 * h + 8 * fg);
      uint32_t ra[8], rb[8];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const uint4 x = src[v];
        ra[2 * v] = x.x;
        rb[2 * v] = x.y;
        ra[2 * v + 1] = x.z;
        rb[2 * v + 1] = x.w;
      }
      uint32_t rw[8], bw[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) rw[i] = ra[i] & 1023u;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        uint32_t h2[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int i = 2 * p + u;
          // column fr takes p0 / p1 / p2 at offsets 0 / 1 / 2 from the event's column
          const int d = fr - ((int)((ra[i] >> 10) & 31u) - 1);
          const uint32_t v = d == 0 ? (rb[i] & 0xffffu) : d == 1 ? (rb[i] >> 16) : d == 2 ? (ra[i] >> 16) : 0u;
          h2[u] = fr == 0 ? kOne : v;  // column 0: the event count
        }
        bw[p] = h2[0] | (h2[1] << 16);
      }
      const uint4 b = make_uint4(bw[0], bw[1], bw[2], bw[3]);
      const int ilo = h ? ilo1 : ilo0, ihi = h ? ihi1 : ihi0;
      while (c < ilo) shift();
      acc0 = tele_mfma(a_frag(rw, c), b, acc0);
      if (ihi > c) acc1 = tele_mfma(a_frag(rw, c + 1), b, acc1);
      while (ihi > c + 1) {  // rare: the chunk reaches a third row tile
        shift();
        acc1 = tele_mfma(a_frag(rw, c + 1), b, acc1);
      }
    }
  }
  }
  while (16 * c < nrows) shift();  // the last live tiles and any tiles without events
  if (__builtin_amdgcn_ballot_w64(nonfinite)) {
    // rare slow path: add the span's Inf/NaN values on top of the stored sums
    __threadfence();
    for (int e = lane; e < ne; e += 64) {
      const int2 x = evs[e];
      const int xm = (int)((event_tag(x.x) - (uint32_t)(m0 & 0xffff)) & 0xffffu);
      const int slot = event_slot(x.x);
      if (xm >= nm || slot >= S || e < rel[xm] || e >= rel[xm + 1]) continue;
      float add;
      const int f = event_feature(event_type(x.x), __int_as_float(x.y), add);
      if (f >= 3 && !__builtin_isfinite(add)) atomicAdd(dst + (xm * S + slot) * kStatFeatures + f, add);
    }
  }
  if (bad) atomicAdd(bad_events, bad);
}
#endif  // ANA_DIAG_BUILD

}  // namespace ana
