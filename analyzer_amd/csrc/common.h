// Shared definitions for the MI355X rating engine (device kernels + host mirror).
//
// Data layout:
//  * roster state: float state[P][32] = 8 granules of 16 B, one per track:
//    {mu, tag, sigma, tag}.  Tracks 0..6 = shared, casual, ranked, blitz, br,
//    5v5_casual, 5v5_ranked; granule 7 spare.  One player = one 128-B line.
//    NaN mu is the SQL NULL ("no rating yet", rater.py:115,124,150).  The two
//    tag words make every 8-B half of a granule self-validating, so a granule
//    is its own ready flag in the dataflow executor (kernels.hip); host code
//    and the generator write tag 0, which never matches a live tag.
//  * player attributes: float4 attrs[P] = (rank_points_ranked,
//    rank_points_blitz, skill_tier, unused); NaN = NULL.  Only read to seed.
//  * match stream: int32 rec[M][2K+2]: 2K player ids (-1 = empty slot; slots
//    0..K-1 roster 0, K..2K-1 roster 1), then meta0 = mode | n0<<8 | n1<<16 |
//    nrosters<<24 and meta1 = winner0 | winner1<<1 | afk_any<<2 | afk_mask<<8.
//  * schedule: uint32 link[M][2K] (kLinkWords below) and int32 deps[M], the
//    executor's completion counters (kernels.h launch_schedule).
#pragma once

#include <stdint.h>

// 1 in the diagnostic library (python -m analyzer_amd.build_ext --diag): kernel
// variants that exist only to take a kernel apart (telemetry.hip)
#ifndef ANA_DIAG_BUILD
#define ANA_DIAG_BUILD 0
#endif

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define ANA_HD __host__ __device__ __forceinline__
#else
#define ANA_HD inline
#endif

namespace ana {

constexpr int kTracks = 7;        // shared + 6 modes
constexpr int kGranules = 8;      // 16-B granules per player row
constexpr int kRowFloats = 32;    // floats per player row (128 B)
constexpr int kBaseFloats = 16;   // DP merge base row: (mu, sigma) per granule (sweep_core.h)
// Schedule link of a slot (K5), 4 bytes: the match of the player's next
// occurrence (kNoMatch: none) | kLinkHasPred if the player occurred earlier in
// the window.  A match publishes each player's shared granule tagged with that
// next match, so its reader recognises the write it waits for by its own match
// index; mode granules are verified with per-mode write counters carried in the
// shared granule's tag (csrc/dataflow.hip).
constexpr int kLinkWords = 1;
constexpr uint32_t kNoMatch = 0x0fffffffu;
constexpr uint32_t kMatchMask = 0x0fffffffu;
constexpr uint32_t kLinkHasPred = 1u << 30;      // the player occurred earlier in the window
constexpr uint32_t kNone = 0xffffffffu;
constexpr int kSlotBits = 28;     // slots of a window < 2^28 (sort values, link match fields)
constexpr int64_t kMaxSlots = 1ll << kSlotBits;
constexpr int kModes = 6;
constexpr int kModeUnsupported = 255;
constexpr int kVstTiers = 31;     // tiers -1..29

// per-match status codes (the reference's outcomes and error classes)
enum Status : uint8_t {
  kRated = 0,           // valid matchup, both tracks updated
  kAfk = 1,             // any went_afk == 1 -> quality 0, all any_afk
  kInvalidRosters = 2,  // len(rosters) != 2 -> quality 0, all any_afk
  kUnsupportedMode = 3, // nothing written
  kErrSeed = 4,         // KeyError: no rank points and tier outside -1..29
  kErrSigma = 5,        // ValueError: sigma == 0 (or NULL sigma with a mu)
  kErrEmptyRoster = 6,  // ValueError: a roster without participants
  kErrNumeric = 7,      // FloatingPointError / non-finite result
  kErrBadRecord = 8,    // malformed stream record (player id out of range, n > K)
  kNotProcessed = 255,  // poison value before the kernel runs
};

struct RateParams {
  float beta2;          // beta^2 = 1e6
  float tau2;           // tau^2 (TAU env, default 100)
  float unknown_sigma;  // UNKNOWN_PLAYER_SIGMA
  int32_t num_players;
  int64_t num_matches;
  int32_t record_first_prior;  // sweep mode: remember priors of NULL tracks
  int32_t epoch;               // 1..255: granule tag word 1 of this launch (word 3 = match)
  const int32_t* epoch_ptr;    // device: read the epoch here instead (graph replays bump it)
  const float* vst;            // vst_points[tier + 1], kVstTiers entries (device/host memory)
  int32_t idle_spins;          // dataflow: max s_sleep(2) rounds of an idle wave (<= 0: none, the default)
  int32_t tight_groups;        // dataflow: 2K lanes per match instead of the next power of two
                               // (-1 auto, 0 off, 1 on)
  int32_t local_handoff;       // dataflow: a successor held by the producing wave is released
                               // through an LDS counter, not the global one (ANA_RATE_LOCAL, default 1)
  int32_t diag;                // dataflow: 1 = the timing build (ANA_RATE_DIAG): wait/iteration
                               // clocks in ctrl[20..27]
  // Tail signal: once chunks from progress_at on are being claimed (every
  // earlier chunk is claimed, the launch is in its tail), waves store
  // progress_value to *progress (signal memory a side stream waits on with
  // hipStreamWaitValue64 before the next window's prepass).  null = off.
  uint64_t* progress;
  uint64_t progress_value;
  int64_t progress_at;         // chunk index (chunk_len matches per chunk)
  // matches per ticket, 8..64 (lanes >= chunk_len idle): 64 for windows; micro-batches
  // use short chunks so their few matches spread over more waves (fewer iterations each)
  int32_t chunk_len;
  // 1: ctrl[1..15] were zeroed by the schedule launched just before on this stream
  // (launch_schedule zero_ctrl), so the launch skips its own zeroing dispatch
  int32_t ctrl_ready;
};

// Per-match outputs.  The participant record of the reference
// (rater.py:151-169) is (s_mu, s_sig, delta) on ``participant`` and
// (m_mu, m_sig) on ``participant_items``; any_afk follows from status.
// Slot j of match m lives at field[m * row + j]; quality at quality[m * qrow],
// status at status[m * srow].  The default layout (ops/rate.py) packs one
// match per 128-B-aligned row -- [s_mu | s_sig | delta | m_mu | m_sig][2K],
// quality, status byte -- so a match's outputs are one full-line write.
struct RateOut {
  float* quality;  // match.trueskill_quality (0 for AFK/invalid, NaN = not written)
  uint8_t* status; // Status
  float* s_mu;
  float* s_sig;
  float* delta;
  float* m_mu;
  float* m_sig;
  int64_t row;     // floats between consecutive matches in the slot fields
  int64_t qrow;    // ... in quality
  int64_t srow;    // bytes between consecutive matches in status
};

ANA_HD int meta_mode(uint32_t m0) { return (int)(m0 & 0xffu); }
ANA_HD int meta_n0(uint32_t m0) { return (int)((m0 >> 8) & 0xffu); }
ANA_HD int meta_n1(uint32_t m0) { return (int)((m0 >> 16) & 0xffu); }
ANA_HD int meta_nrosters(uint32_t m0) { return (int)((m0 >> 24) & 0xffu); }
ANA_HD bool meta_winner0(uint32_t m1) { return (m1 & 1u) != 0; }
ANA_HD bool meta_winner1(uint32_t m1) { return (m1 & 2u) != 0; }
ANA_HD bool meta_afk(uint32_t m1) { return (m1 & 4u) != 0; }
ANA_HD uint32_t pack_meta0(int mode, int n0, int n1, int nrosters) {
  return (uint32_t)(mode & 0xff) | ((uint32_t)(n0 & 0xff) << 8) |
         ((uint32_t)(n1 & 0xff) << 16) | ((uint32_t)(nrosters & 0xff) << 24);
}
ANA_HD uint32_t pack_meta1(bool w0, bool w1, uint32_t afk_mask) {
  return (w0 ? 1u : 0u) | (w1 ? 2u : 0u) | (afk_mask ? 4u : 0u) | ((afk_mask & 0xffffffu) << 8);
}

// Outcome of a stream record that is decided before any state is read: kRated
// ("to be rated"), or unsupported / malformed / invalid rosters / AFK.  The
// precedence is rate_core.h decode_record's.
template <int K>
ANA_HD uint8_t early_status(const int32_t* r, int64_t P) {
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

// early_status for a runtime team size (S = 2K slots)
ANA_HD uint8_t early_status_k(const int32_t* r, int S, int64_t P) {
  switch (S / 2) {
    case 1: return early_status<1>(r, P);
    case 2: return early_status<2>(r, P);
    case 3: return early_status<3>(r, P);
    case 4: return early_status<4>(r, P);
    case 5: return early_status<5>(r, P);
    default: return kErrBadRecord;
  }
}

// ---------------------------------------------------------------- RNG (K7)
// Counter-based: every random number is a pure function of (seed, index,
// field), so device and host generators produce bit-identical streams and any
// window/shard can be regenerated independently (checkpoint/resume needs no
// RNG state beyond the seed and the stream offset).
ANA_HD uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
ANA_HD uint64_t rng_u64(uint64_t seed, uint64_t index, uint32_t field) {
  return mix64(mix64(seed ^ (0xd1b54a32d192ed03ull * (uint64_t)(field + 1))) + index);
}
// uniform in [0, 1) with 24 random bits (exactly representable in fp32)
ANA_HD float rng_unit(uint64_t seed, uint64_t index, uint32_t field) {
  return (float)(rng_u64(seed, index, field) >> 40) * (1.0f / 16777216.0f);
}

}  // namespace ana
