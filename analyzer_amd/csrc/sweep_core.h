// Per-player math of the data-parallel posterior merge (see sweep.hip for the
// protocol); shared by the gfx950 kernels and the host mirror.
#pragma once

#include <math.h>

#include "common.h"
#include "rate_core.h"

namespace ana {

ANA_HD void nat_params(float mu, float sig, float& pi, float& tau) {
  pi = 1.f / (sig * sig);
  tau = mu * pi;
}

// a: window-start row, b: row after the local window, f: priors the rate kernel
// recorded for tracks it found NULL (all kRowFloats-float rows, mu at 4t, sigma
// at 4t+2).  o: 16 floats of message = (d_pi, d_tau) per track + touch fields.
ANA_HD void sweep_delta_player(const float* a, const float* b, const float* f, float* o) {
  float touch_lo = 0.f, touch_hi = 0.f;
  for (int t = 0; t < kTracks; ++t) {
    const float mu0 = a[4 * t], sg0 = a[4 * t + 2], mu = b[4 * t], sg = b[4 * t + 2];
    float dp = 0.f, dt = 0.f;
    if (mu0 == mu0) {
      if (mu != mu0 || sg != sg0) {
        float p1, t1, p0, t0;
        nat_params(mu, sg, p1, t1);
        nat_params(mu0, sg0, p0, t0);
        dp = p1 - p0;
        dt = t1 - t0;
      }
    } else if (mu == mu) {
      float p1, t1, pf, tf;
      nat_params(mu, sg, p1, t1);
      nat_params(f[4 * t], f[4 * t + 2], pf, tf);
      dp = p1 - pf;
      dt = t1 - tf;
      if (t < 4) touch_lo += (float)(1 << (4 * t));
      else touch_hi += (float)(1 << (4 * (t - 4)));
    }
    o[2 * t] = dp;
    o[2 * t + 1] = dt;
  }
  o[14] = touch_lo;
  o[15] = touch_hi;
}

// a: window-start row, d: all-reduced messages, attr: player attributes,
// o: merged row (tags reset to 0).
ANA_HD void sweep_apply_player(const float* a, const float* d, const float* attr,
                               const float* vst, float unknown_sigma, float* o) {
  float seed_mu = NAN, seed_sig = NAN;
  const bool seeded = seed_prior<float>(attr, unknown_sigma, vst, seed_mu, seed_sig);
  float base_mu = a[0], base_sig = a[2];
  if (base_mu != base_mu) {
    base_mu = seed_mu;
    base_sig = seed_sig;
  }
  const unsigned lo = (unsigned)d[14], hi = (unsigned)d[15];
  for (int t = 0; t < kTracks; ++t) {
    const float mu0 = a[4 * t], sg0 = a[4 * t + 2];
    const unsigned touched = t < 4 ? (lo >> (4 * t)) & 15u : (hi >> (4 * (t - 4))) & 15u;
    float mu = mu0, sg = sg0, pb = 0.f, tb = 0.f;
    bool have = false;
    if (mu0 == mu0) {
      nat_params(mu0, sg0, pb, tb);
      have = d[2 * t] != 0.f || d[2 * t + 1] != 0.f;
    } else if (touched && seeded) {
      if (t == 0) nat_params(seed_mu, seed_sig, pb, tb);
      else nat_params(base_mu, base_sig, pb, tb);
      have = true;
    }
    if (have) {
      float pi = pb + d[2 * t];
      const float tau = tb + d[2 * t + 1];
      pi = pi > 1e-12f ? pi : 1e-12f;  // merged precision never below "no information"
      mu = tau / pi;
      sg = 1.f / sqrtf(pi);
    }
    o[4 * t] = mu;
    o[4 * t + 1] = 0.f;
    o[4 * t + 2] = sg;
    o[4 * t + 3] = 0.f;
  }
  for (int k = 4 * kTracks; k < kRowFloats; ++k) o[k] = (k & 1) ? 0.f : a[k];
}

}  // namespace ana
