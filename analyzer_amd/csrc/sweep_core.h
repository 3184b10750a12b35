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

// s0: window-start row (16 floats), s: row after the local window, fp: priors the
// rate kernel recorded for tracks it found NULL.  o: 16 floats of message.
ANA_HD void sweep_delta_player(const float* a, const float* b, const float* f, float* o) {
  float touch_lo = 0.f, touch_hi = 0.f;
  for (int t = 0; t < kTracks; ++t) {
    const float mu0 = a[2 * t], sg0 = a[2 * t + 1], mu = b[2 * t], sg = b[2 * t + 1];
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
      nat_params(f[2 * t], f[2 * t + 1], pf, tf);
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
// o: merged row.
ANA_HD void sweep_apply_player(const float* a, const float* d, const float* attr,
                               const float* vst, float unknown_sigma, float* o) {
  float seed_mu = NAN, seed_sig = NAN;
  const bool seeded = seed_prior<float>(attr, unknown_sigma, vst, seed_mu, seed_sig);
  float base_mu = a[0], base_sig = a[1];
  if (base_mu != base_mu) {
    base_mu = seed_mu;
    base_sig = seed_sig;
  }
  const unsigned lo = (unsigned)d[14], hi = (unsigned)d[15];
  for (int t = 0; t < kTracks; ++t) {
    const float mu0 = a[2 * t], sg0 = a[2 * t + 1];
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
    o[2 * t] = mu;
    o[2 * t + 1] = sg;
  }
  o[14] = a[14];
  o[15] = a[15];
}

}  // namespace ana
