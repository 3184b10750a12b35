// Synthetic roster + match-stream generator, shared host/device.
//
// Replaces the reference's inputs (MySQL rows reflected at worker.py:43-83 and
// AMQP match ids consumed at worker.py:92-101) with a counter-based stream.
// All probabilities arrive pre-quantised as uint32 thresholds and all float
// arithmetic is explicit fmaf, so the MI355X kernel and the C++ host mirror
// generate bit-identical data.
#pragma once

#include <math.h>

#include "common.h"

namespace ana {

struct GenRosterParams {
  uint64_t seed;
  int64_t num_players;
  uint32_t p_tier_null;   // skill_tier NULL
  uint32_t p_tier_bad;    // skill_tier 30 (missing from vst_points)
  uint32_t p_rp_ranked;   // rank_points_ranked present
  uint32_t p_rp_blitz;    // rank_points_blitz present
  uint32_t p_rated;       // stored shared rating present
  uint32_t p_mode_rated;  // each mode track present (given shared present)
  float mu_lo, mu_span, sig_lo, sig_span;
};

struct GenStreamParams {
  uint64_t seed;
  int64_t base;           // global index of match 0 of this window/shard
  int64_t num_players;
  int32_t team_size;      // players per roster (<= K)
  int32_t skew;           // activity skew: player = floor(u^skew * P), 1 = uniform
  uint32_t mode_cdf[7];   // cumulative thresholds: modes 0..5, then "unsupported"
  uint32_t p_uneven;      // roster 1 one player short
  uint32_t p_bad_rosters; // nrosters = 3
  uint32_t p_tie;         // both rosters winner=False
  uint32_t p_afk;         // one participant went_afk
  uint32_t p_hot;         // draw the player from the hot set
  uint32_t hot_players;   // size of the hot set (activity skew)
};

ANA_HD uint32_t rng_u32(uint64_t seed, uint64_t index, uint32_t field) {
  return (uint32_t)(rng_u64(seed, index, field) >> 32);
}
// floor(u * n) for u uniform in [0, 2^32): exact integer mapping
ANA_HD uint32_t mulhi_range(uint32_t u, uint64_t n) { return (uint32_t)(((uint64_t)u * n) >> 32); }

ANA_HD void gen_player(const GenRosterParams& g, int64_t p, float* st /*32*/, float* at /*4*/) {
  const uint64_t s = g.seed;
  const uint32_t ut = rng_u32(s, p, 0);
  float tier;
  if (ut < g.p_tier_null) {
    tier = NAN;
  } else if (ut - g.p_tier_null < g.p_tier_bad) {
    tier = 30.f;
  } else {
    tier = (float)((int)mulhi_range(rng_u32(s, p, 1), 31) - 1);
  }
  at[0] = rng_u32(s, p, 2) < g.p_rp_ranked ? fmaf(2600.f, rng_unit(s, p, 3), 400.f) : NAN;
  at[1] = rng_u32(s, p, 4) < g.p_rp_blitz ? fmaf(2600.f, rng_unit(s, p, 5), 400.f) : NAN;
  at[2] = tier;
  at[3] = 0.f;
  for (int k = 0; k < kRowFloats; ++k) st[k] = (k & 1) ? 0.f : NAN;  // tags 0, values NULL
  if (rng_u32(s, p, 6) < g.p_rated) {
    const float mu = fmaf(g.mu_span, rng_unit(s, p, 7), g.mu_lo);
    st[0] = mu;
    st[2] = fmaf(g.sig_span, rng_unit(s, p, 8), g.sig_lo);
    for (int t = 1; t < kTracks; ++t) {
      if (rng_u32(s, p, 8 + 3 * t) < g.p_mode_rated) {
        st[4 * t] = mu + fmaf(300.f, rng_unit(s, p, 9 + 3 * t), -150.f);
        st[4 * t + 2] = fmaf(g.sig_span, rng_unit(s, p, 10 + 3 * t), g.sig_lo);
      }
    }
  }
}

// Writes one record of 2K+2 int32 (layout in common.h).
template <int K>
ANA_HD void gen_match(const GenStreamParams& g, int64_t m, int32_t* rec) {
  const uint64_t s = g.seed;
  const uint64_t idx = (uint64_t)(g.base + m);
  const uint32_t um = rng_u32(s, idx, 0);
  int mode = kModeUnsupported;
  for (int k = 6; k >= 0; --k)
    if (um < g.mode_cdf[k]) mode = k < 6 ? k : kModeUnsupported;
  const int n0 = g.team_size;
  const int n1 = rng_u32(s, idx, 1) < g.p_uneven ? g.team_size - 1 : g.team_size;
  const int nrosters = rng_u32(s, idx, 2) < g.p_bad_rosters ? 3 : 2;
  bool w0, w1;
  if (rng_u32(s, idx, 3) < g.p_tie) {
    w0 = w1 = false;
  } else {
    w0 = (rng_u32(s, idx, 4) & 1u) != 0;
    w1 = !w0;
  }
  uint32_t afk = 0;
  if (rng_u32(s, idx, 5) < g.p_afk) afk = 1u << mulhi_range(rng_u32(s, idx, 6), (uint64_t)(n0 + n1));
  for (int j = 0; j < 2 * K; ++j) {
    const int pos = j < K ? j : j - K;
    const int n = j < K ? n0 : n1;
    if (pos < n) {
      const uint64_t h = rng_u64(s, idx, 16 + j);
      const bool hot = (uint32_t)h < g.p_hot;
      const uint64_t range = hot ? (uint64_t)g.hot_players : (uint64_t)g.num_players;
      // power-law activity: u^skew in 32-bit fixed point (integer products only,
      // so host and device agree bit for bit); player 0 is the most active, with
      // probability P^(-1/skew) per slot (skew 3 = SURVEY App. C.5 "cubic")
      uint32_t u = (uint32_t)(h >> 32);
      const uint32_t u1 = u;
      for (int k = 1; k < g.skew; ++k) u = (uint32_t)(((uint64_t)u * u1) >> 32);
      rec[j] = (int32_t)mulhi_range(u, range);
    } else {
      rec[j] = -1;
    }
  }
  rec[2 * K] = (int32_t)pack_meta0(mode, n0, n1, nrosters);
  rec[2 * K + 1] = (int32_t)pack_meta1(w0, w1, afk);
}

}  // namespace ana
