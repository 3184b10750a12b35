// Per-player math of the data-parallel posterior merge (see sweep.hip for the
// protocol); shared by the gfx950 kernels and the host mirror.  Rows are
// kRowFloats floats: track t at mu = 4t, sigma = 4t + 2 (NaN mu = NULL).
#pragma once

#include <math.h>

#include "common.h"
#include "rate_core.h"

namespace ana {

ANA_HD void nat_params(float mu, float sig, float& pi, float& tau) {
  pi = 1.f / (sig * sig);
  tau = mu * pi;
}

// The common base every rank measures its message against, for track t: the
// window-start value (cmu, csg); for a track NULL at window start the prior the
// reference would give it -- the seed for the shared track, the window-start
// shared rating (c0mu, c0sg; else the seed) for a mode track (rater.py:115-136).
// Returns false when the track has no base (NULL and the player cannot be seeded).
ANA_HD bool track_base(int t, float cmu, float csg, float c0mu, float c0sg, bool seeded, float seed_mu,
                       float seed_sig, float& mu, float& sig) {
  if (cmu == cmu) {
    mu = cmu;
    sig = csg;
    return true;
  }
  if (t > 0 && c0mu == c0mu) {
    mu = c0mu;
    sig = c0sg;
    return true;
  }
  mu = seed_mu;
  sig = seed_sig;
  return seeded;
}

// Message encodings (both linear in the natural parameters, so sums over ranks
// -- the all-reduce, and the exclusive prefix of the causal sweeps -- stay exact
// in algebra):
//  raw    (d_pi, d_tau)
//  scaled (d_pi / pi_B, (d_tau - mu_B d_pi) / pi_B): dimensionless precision ratio and
//         a rating-point-sized mean shift -- small, well-conditioned numbers that
//         survive an fp16 / bf16 all-reduce (COMM_DTYPE), decoded against the same base B.
//
// The merge keeps its window start and causal priors as BASE rows: float[16] per
// player, (mu, sigma) of the 8 granules of the roster row (kBaseFloats) -- half the
// bytes of a roster row, and all a message needs.  The kernels (sweep.hip) run one
// lane per track on these per-track functions; the host mirror calls the same ones.

// One track t of a player's message.  (cmu, csg): the COMMON window-start value of
// the track (identical on every rank; with the start's shared value (c0mu, c0sg)
// and the seed it defines the base B, track_base), (amu, asg): the prior this rank
// rated its shard from in this sweep (== the start in the first sweep; the start
// plus the earlier ranks' messages in a causal re-sweep, parallel/sweep.py),
// (bmu, bsg): the value after the local window.  The message is nat(b) - nat(a),
// measured against a's value where a has one and against B where the track is NULL
// in a: prefix sums then telescope, so the start + the messages of ranks 0..r-1 is
// exactly rank r-1's posterior once every earlier rank rated from its exact prior.
// touched: this rank moved the track -- NULL in a and rated now, or changed (base-16
// touch counters, exact in fp32 for <= 15 ranks): their sum m makes a NULL track
// non-NULL on every rank and tells the decode how many ranks a net loss came from.
ANA_HD void sweep_delta_track(int t, float cmu, float csg, float c0mu, float c0sg, float amu, float asg,
                              float bmu, float bsg, bool seeded, float seed_mu, float seed_sig,
                              bool scaled, float& dp, float& dt, bool& touched) {
  dp = 0.f;
  dt = 0.f;
  const bool had = amu == amu;
  const bool changed = had ? (bmu != amu || bsg != asg) : bmu == bmu;
  float bm, bs;
  const bool based = track_base(t, cmu, csg, c0mu, c0sg, seeded, seed_mu, seed_sig, bm, bs);
  if (changed && based) {
    if (scaled) {  // (pi/pi_B - pi0/pi_B, (pi/pi_B)(mu - mu_B) - (pi0/pi_B)(mu0 - mu_B))
      const float r1 = bs / bsg;
      const float r0 = had ? bs / asg : 1.f;
      dp = r1 * r1 - r0 * r0;
      dt = r1 * r1 * (bmu - bm) - (had ? r0 * r0 * (amu - bm) : 0.f);
    } else {
      float p1, t1, p0, t0;
      nat_params(bmu, bsg, p1, t1);
      if (had) nat_params(amu, asg, p0, t0);
      else nat_params(bm, bs, p0, t0);
      dp = p1 - p0;
      dt = t1 - t0;
    }
  }
  touched = had ? changed : bmu == bmu;
}

// Decoded precision ratio pi / pi_B and mean-shift divisor of summed messages whose
// precision ratios x_r = pi_r / pi_B sum to 1 + S over m contributing ranks.  Net
// gain (S >= 0) or one rank: the natural-parameter sum, 1 + S -- exact for evidence.
// Net loss over m >= 2 ranks: the tau^2 dynamics every match adds, which ADD in
// variance, not in precision -- eight ranks that each lost 20 % of a low-sigma
// player's precision sum to 1 + S = -0.6, where the sequential result keeps 0.38 of it
// (the 1M-player 8-rank bench hit this on 28 tracks).  So the loss is combined in
// variance space, as if every rank lost the mean x = 1 + S / m:
//     pi / pi_B = 1 / (1 + m (1 / x - 1)) = x / (x + m (1 - x))   in (0, 1)
// (x > 0 because every x_r > 0), which agrees with 1 + S to first order and is
// exact for equal losses; the mean shift sum_r x_r dmu_r is divided by x (each rank's
// shift counted once).  Never zero or negative, so a merge clamps only on inputs no
// set of ranks can produce (the clamp count stays the safety net).
// Returns true on the variance-space branch.
ANA_HD bool merged_ratio(float S, unsigned m, float& ratio, float& mdiv) {
  ratio = 1.f + S;
  mdiv = ratio;
  if (S < 0.f && m >= 2u) {
    const float x = 1.f + S / (float)m;
    if (x > 0.f) {
      ratio = x / (x + (float)m * (1.f - x));
      mdiv = x;
      return true;
    }
  }
  return false;
}

// One track t of the decode: (amu, asg) the common window-start value of the track,
// (a0mu, a0sg) the start's shared value, (dpi, dtau) the summed messages, touched the
// summed touch count of the track.  Returns the decoded (mu, sigma).
//
// clamped: the merged precision came out at or below zero (or not finite) and was
// held at the floor -- a sigma x1000 / a meaningless mean that must never be written
// silently.  The kernels count these into a sticky word the merger raises on
// (parallel/sweep.py SweepMerger.check).  Where it comes from (root-caused in round
// 5 on the host mirror, profiles/r5/lag_bf16_root_cause.log): the one-window-late
// merge (rounds 4-5, removed) measured a rank's message against its own start Y,
// which lacks the other ranks' evidence of the previous window -- their tau^2
// dynamics included -- so Y's precision sat above the common roster C it was added
// to.  The precision a match's dynamics removes grows with pi^2 tau^2, so eight ranks'
// dynamics losses measured at Y's precision overshoot C's: 1 + sum r_pi -> 0 (-0.99
// of C in one window for a player near sigma 100) and below.  The merge measures
// every rank against the common start and keeps a wide margin (min 0.46-0.88).
ANA_HD void sweep_apply_track(int t, float amu, float asg, float a0mu, float a0sg, float dpi, float dtau,
                              unsigned touched, bool seeded, float seed_mu, float seed_sig, bool scaled,
                              float& mu, float& sg, bool& clamped) {
  mu = amu;
  sg = asg;
  clamped = false;
  const bool live = amu == amu ? (dpi != 0.f || dtau != 0.f) : touched != 0u;
  if (!live) return;
  float bm, bs;
  const bool based = track_base(t, amu, asg, a0mu, a0sg, seeded, seed_mu, seed_sig, bm, bs);
  if (!based) return;
  if (scaled) {  // pi = pi_b (1 + sum r_pi), mu = mu_b + sum r_tau / (1 + sum r_pi) (merged_ratio)
    float ratio, mdiv;
    merged_ratio(dpi, touched, ratio, mdiv);
    clamped = !(ratio > 1e-6f);
    ratio = clamped ? 1e-6f : ratio;
    mdiv = clamped ? 1e-6f : mdiv;
    mu = bm + dtau / mdiv;
    sg = bs / sqrtf(ratio);
  } else {       // raw: S = d_pi / pi_b, sum_r x_r dmu_r = d_tau / pi_b - S mu_b
    float pb, tb;
    nat_params(bm, bs, pb, tb);
    const float S = dpi / pb;
    float ratio, mdiv;
    if (merged_ratio(S, touched, ratio, mdiv)) {
      mu = bm + (dtau / pb - S * bm) / mdiv;
      sg = bs / sqrtf(ratio);
    } else {  // the natural-parameter sum
      float pi = pb + dpi;
      const float tau = tb + dtau;
      clamped = !(pi > 1e-12f);
      pi = clamped ? 1e-12f : pi;  // merged precision never below "no information"
      mu = tau / pi;
      sg = 1.f / sqrtf(pi);
    }
  }
}

// ------------------------------------------------------- causal record correction
// Rank r rated the r-th time slice of the window from the common start, so its
// per-participant records miss the evidence of the earlier slices (ranks q < r), which
// the reference's sequential loop had already folded in (/root/reference/worker.py:
// 176,191-192).  After the merge's collective every rank also holds the EXCLUSIVE
// prefix of the messages, sum_{q<r} m_q (parallel/comm.py scan_and_sum), and a record
// (mu, sigma) of player p on track t is corrected by adding that evidence in natural
// parameters -- the same additive approximation the merged roster makes for the whole
// window:  nat(rec') = nat(rec) + delta(p, t).  At 8 ranks x 1.25M-match windows over
// 100k players (the k = 8 density of the bench) the shared records' median |d mu|
// against exact sequential rating falls from 29.7 to 8.0, p99 156 -> 40
// (profiles/r5/record_correction.log).  Rank 0's prefix is zero: its records are the
// sequential ones already.
//
// delta(p, t) in raw natural parameters (d_pi, d_tau): a raw fp32 prefix is that
// already; a scaled (bf16 / fp16) prefix (r_pi, r_tau) is relative to the track's base
// B (track_base: the window-start value, else the seed / start shared value it was
// measured against):  (pi_B r_pi, pi_B (r_tau + mu_B r_pi)).  The merge's decode pass
// computes it while it still holds the window start (sweep.hip), so the per-slot pass
// over the records gathers one 64-B row per player and does no base logic.
ANA_HD void prefix_delta_track(int t, float cmu, float csg, float c0mu, float c0sg, bool seeded, float seed_mu,
                               float seed_sig, float rpi, float rtau, float& dpi, float& dtau) {
  dpi = dtau = 0.f;
  if (rpi == 0.f && rtau == 0.f) return;
  float bm, bs;
  if (!track_base(t, cmu, csg, c0mu, c0sg, seeded, seed_mu, seed_sig, bm, bs)) return;
  const float pb = 1.f / (bs * bs);
  dpi = pb * rpi;
  dtau = pb * (rtau + bm * rpi);
}

// one record (mu, sigma) += delta in natural parameters (NULL / untouched: unchanged)
ANA_HD void correct_record_track(float dpi, float dtau, float& mu, float& sg) {
  if (!(mu == mu) || (dpi == 0.f && dtau == 0.f)) return;
  const float p0 = 1.f / (sg * sg);
  const float pi = p0 + dpi;
  if (!(pi > 0.f)) return;  // (a prefix that would void the record's precision: keep the record)
  mu = (mu * p0 + dtau) / pi;
  sg = 1.f / sqrtf(pi);
}

// host mirror of the delta table of one player: c = its window-start base row, pref =
// the scaled prefix [14] (r_pi, r_tau per track), out = [16] (d_pi, d_tau per granule)
ANA_HD void prefix_delta_player(const float* c, const float* pref, const float* attr, const float* vst,
                                float unknown_sigma, float* out) {
  float seed_mu = NAN, seed_sig = NAN;
  const bool seeded = seed_prior<float>(attr, unknown_sigma, vst, seed_mu, seed_sig);
  for (int t = 0; t < kTracks; ++t)
    prefix_delta_track(t, c[2 * t], c[2 * t + 1], c[0], c[1], seeded, seed_mu, seed_sig, pref[2 * t],
                       pref[2 * t + 1], out[2 * t], out[2 * t + 1]);
  out[14] = out[15] = 0.f;
}

// Whole-player forms over base rows (host mirror): s, a: base rows [16] (start,
// prior), b: roster row [32]; o: 16 floats = message per track + the touch fields.
ANA_HD void sweep_delta_player(const float* s, const float* a, const float* b, const float* attr,
                               const float* vst, float unknown_sigma, bool scaled, float* o) {
  float seed_mu = NAN, seed_sig = NAN;
  const bool seeded = seed_prior<float>(attr, unknown_sigma, vst, seed_mu, seed_sig);
  float touch_lo = 0.f, touch_hi = 0.f;
  for (int t = 0; t < kTracks; ++t) {
    bool touched;
    sweep_delta_track(t, s[2 * t], s[2 * t + 1], s[0], s[1], a[2 * t], a[2 * t + 1], b[4 * t],
                      b[4 * t + 2], seeded, seed_mu, seed_sig, scaled, o[2 * t], o[2 * t + 1], touched);
    if (touched) {
      if (t < 4) touch_lo += (float)(1 << (4 * t));
      else touch_hi += (float)(1 << (4 * (t - 4)));
    }
  }
  o[14] = touch_lo;
  o[15] = touch_hi;
}

// a: base row of the common window start, d: summed messages (all ranks: the
// merged window; ranks < r: rank r's prior for a causal re-sweep); o: the decoded
// roster row (tags 0; granule 7 from the base row), ob: the same as a base row.
ANA_HD void sweep_apply_player(const float* a, const float* d, const float* attr,
                               const float* vst, float unknown_sigma, bool scaled, float* o, float* ob,
                               uint32_t* clamps) {
  bool cl = false;
  float seed_mu = NAN, seed_sig = NAN;
  const bool seeded = seed_prior<float>(attr, unknown_sigma, vst, seed_mu, seed_sig);
  const unsigned lo = (unsigned)d[14], hi = (unsigned)d[15];
  for (int g = 0; g < kGranules; ++g) {
    float mu = a[2 * g], sg = a[2 * g + 1];
    if (g < kTracks) {
      const unsigned touched = g < 4 ? (lo >> (4 * g)) & 15u : (hi >> (4 * (g - 4))) & 15u;
      sweep_apply_track(g, a[2 * g], a[2 * g + 1], a[0], a[1], d[2 * g], d[2 * g + 1], touched, seeded,
                        seed_mu, seed_sig, scaled, mu, sg, cl);
      if (cl && clamps) ++*clamps;
    }
    o[4 * g] = mu;
    o[4 * g + 1] = 0.f;
    o[4 * g + 2] = sg;
    o[4 * g + 3] = 0.f;
    ob[2 * g] = mu;
    ob[2 * g + 1] = sg;
  }
}

}  // namespace ana
