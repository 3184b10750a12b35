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

// The common base every rank measures its message against, for each track:
// the window-start value; for a track NULL at window start the prior the
// reference would give it -- the seed for the shared track, the window-start
// shared rating (else the seed) for a mode track (rater.py:115-136).  Returns
// false when the track has no base (NULL and the player cannot be seeded).
ANA_HD bool track_base(const float* a, int t, bool seeded, float seed_mu, float seed_sig,
                       float& mu, float& sig) {
  if (a[4 * t] == a[4 * t]) {
    mu = a[4 * t];
    sig = a[4 * t + 2];
    return true;
  }
  if (t > 0 && a[0] == a[0]) {
    mu = a[0];
    sig = a[2];
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
// s: the COMMON window-start row (identical on every rank; it defines the base B
// of each track), a: the prior this rank rated its shard from in this sweep
// (== s in the first sweep; the start plus the earlier ranks' messages in a
// causal re-sweep, parallel/sweep.py), b: the row after the local window.  The
// message is nat(b) - nat(a), measured against a's value where a has one and
// against B where the track is NULL in a: prefix sums then telescope, so the
// start + the messages of ranks 0..r-1 is exactly rank r-1's posterior once
// every earlier rank rated from its exact prior.  attr/vst/unknown_sigma: seed
// inputs.  o: 16 floats = message per track + touch fields for tracks that are
// NULL in a and rated now (base-16 counters, exact in fp32 for <= 15 ranks).
ANA_HD void sweep_delta_player(const float* s, const float* a, const float* b, const float* attr,
                               const float* vst, float unknown_sigma, bool scaled, float* o) {
  float seed_mu = NAN, seed_sig = NAN;
  const bool seeded = seed_prior<float>(attr, unknown_sigma, vst, seed_mu, seed_sig);
  float touch_lo = 0.f, touch_hi = 0.f;
  for (int t = 0; t < kTracks; ++t) {
    const float mu0 = a[4 * t], sg0 = a[4 * t + 2], mu = b[4 * t], sg = b[4 * t + 2];
    float dp = 0.f, dt = 0.f;
    const bool had = mu0 == mu0;
    const bool changed = had ? (mu != mu0 || sg != sg0) : mu == mu;
    float bm, bs;
    if (changed && track_base(s, t, seeded, seed_mu, seed_sig, bm, bs)) {
      if (scaled) {  // (pi/pi_B - pi0/pi_B, (pi/pi_B)(mu - mu_B) - (pi0/pi_B)(mu0 - mu_B))
        const float r1 = bs / sg;
        const float r0 = had ? bs / sg0 : 1.f;
        dp = r1 * r1 - r0 * r0;
        dt = r1 * r1 * (mu - bm) - (had ? r0 * r0 * (mu0 - bm) : 0.f);
      } else {
        float p1, t1, p0, t0;
        nat_params(mu, sg, p1, t1);
        if (had) nat_params(mu0, sg0, p0, t0);
        else nat_params(bm, bs, p0, t0);
        dp = p1 - p0;
        dt = t1 - t0;
      }
    }
    if (!had && mu == mu) {
      if (t < 4) touch_lo += (float)(1 << (4 * t));
      else touch_hi += (float)(1 << (4 * (t - 4)));
    }
    o[2 * t] = dp;
    o[2 * t + 1] = dt;
  }
  o[14] = touch_lo;
  o[15] = touch_hi;
}

// a: common window-start row, d: summed messages (all ranks: the merged window;
// ranks < r: rank r's prior for a causal re-sweep), attr: player attributes,
// o: decoded row (tags reset to 0; spare floats copied).
ANA_HD void sweep_apply_player(const float* a, const float* d, const float* attr,
                               const float* vst, float unknown_sigma, bool scaled, float* o) {
  float seed_mu = NAN, seed_sig = NAN;
  const bool seeded = seed_prior<float>(attr, unknown_sigma, vst, seed_mu, seed_sig);
  const unsigned lo = (unsigned)d[14], hi = (unsigned)d[15];
  for (int t = 0; t < kTracks; ++t) {
    const float mu0 = a[4 * t], sg0 = a[4 * t + 2];
    const unsigned touched = t < 4 ? (lo >> (4 * t)) & 15u : (hi >> (4 * (t - 4))) & 15u;
    float mu = mu0, sg = sg0, bm, bs;
    const bool live = mu0 == mu0 ? (d[2 * t] != 0.f || d[2 * t + 1] != 0.f) : touched != 0u;
    if (live && track_base(a, t, seeded, seed_mu, seed_sig, bm, bs)) {
      if (scaled) {  // pi = pi_b (1 + sum r_pi), mu = mu_b + sum r_tau / (1 + sum r_pi)
        float ratio = 1.f + d[2 * t];
        ratio = ratio > 1e-6f ? ratio : 1e-6f;
        mu = bm + d[2 * t + 1] / ratio;
        sg = bs / sqrtf(ratio);
      } else {
        float pb, tb;
        nat_params(bm, bs, pb, tb);
        float pi = pb + d[2 * t];
        const float tau = tb + d[2 * t + 1];
        pi = pi > 1e-12f ? pi : 1e-12f;  // merged precision never below "no information"
        mu = tau / pi;
        sg = 1.f / sqrtf(pi);
      }
    }
    o[4 * t] = mu;
    o[4 * t + 1] = 0.f;
    o[4 * t + 2] = sg;
    o[4 * t + 3] = 0.f;
  }
  for (int k = 4 * kTracks; k < kRowFloats; ++k) o[k] = (k & 1) ? 0.f : a[k];
}

}  // namespace ana
