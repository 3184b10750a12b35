// Device-only rating math of the dataflow executor (dataflow.hip): both tracks of a
// participant -- shared and mode -- as ONE packed pair, so every non-transcendental
// step is a single v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 for the two tracks.
//
// Same closed form as rate_core.h (/root/reference/rater.py:138-169
// through trueskill's 2-team factor graph), with a shorter chain:
//  * team sums: the four group sums (sigma^2 + tau^2 and the signed mu of both
//    tracks) run as one interleaved DPP butterfly, so no step waits on its own
//    hazard nops;
//  * coefficients from ONE reciprocal square root per track: t = d rsq(c2),
//    a = v rsq(c2), w / c2 = w rsq(c2)^2 -- no sqrt, no division;
//  * v/w without erfc: a branch-free rational form of the Mills ratio (below), one
//    formula for wins, losses and big upsets, evaluated for both tracks at once.
// The host mirror (host.cpp -> rate_core.h, fp64) stays the oracle; this form agrees
// with it within the device tolerances of tests/test_engine_gpu.py.
#pragma once

#include <hip/hip_runtime.h>

#include "dataflow_dev.h"

namespace ana {

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 rcp2(f2 x) {
  return f2{__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y)};
}
__device__ __forceinline__ f2 rsq2(f2 x) {
  return f2{__builtin_amdgcn_rsqf(x.x), __builtin_amdgcn_rsqf(x.y)};
}
__device__ __forceinline__ f2 sqrt2(f2 x) {
  return f2{__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
}
__device__ __forceinline__ f2 exp2_2(f2 x) {
  return f2{__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
}

// v = pdf(t) / cdf(t) and w = v (v + t) of a win with zero draw margin, for both
// tracks.  With a = |t| and h(a) = 1 / R(a) - a (R = Mills ratio):
//   t <= 0:  v = a + h,                   v + t = h         (no cancellation for upsets)
//   t >  0:  v = phi D / (D - phi), D = a + h,  v + t = v + a
// h is a rational function of s = a / (a + 4) times 1 / (a + 4): bounded on
// [0, inf), decaying as 1/a, never overflowing.  Coefficients: least-squares fit of
// relative error (scripts/fit_vw.py; tests/test_rate_dev_vw.py checks them against
// 50-digit mpmath); fp32 evaluation vs fp64: relative error of v and w <= 8.4e-7 for
// t < 4, 2.4e-6 for t in [4, 6) and 9e-6 for t in [6, 15), where v < 2e-5 / 1e-9.
// A tie (equal ranks) takes the eps -> 0 draw limit v = -t, w = 1.
__device__ __forceinline__ void vw_pair(f2 t, bool tie, f2& v, f2& w) {
  constexpr float kK = 4.f;
  const f2 a = f2{__builtin_fabsf(t.x), __builtin_fabsf(t.y)};
  const f2 r = rcp2(a + kK);
  const f2 s = a * r;
  f2 P = f2{-2.972561717e-01f, -2.972561717e-01f};
  P = P * s + 1.921151161e+00f;
  P = P * s + -4.613346577e+00f;
  P = P * s + 7.719998837e+00f;
  P = P * s + -5.827823639e+00f;
  P = P * s + 3.191538334e+00f;
  f2 Q = f2{8.244409561e-01f, 8.244409561e-01f};
  Q = Q * s + -7.769815922e-01f;
  Q = Q * s + 2.051106215e+00f;
  Q = Q * s + -1.004303694e+00f;
  Q = Q * s + 1.f;
  const f2 h = r * P * rcp2(Q);
  // phi(a) = exp(-a^2 / 2) / sqrt(2 pi); underflows to 0 for a > ~13 (v = w = 0)
  const f2 phi = exp2_2(a * a * -0.72134752044448170f) * 0.39894228040143268f;
  const f2 D = a + h;
  const f2 vp = phi * D * rcp2(D - phi);
  const f2 vq = vp + a;
  v.x = t.x <= 0.f ? D.x : vp.x;
  v.y = t.y <= 0.f ? D.y : vp.y;
  f2 vt;
  vt.x = t.x <= 0.f ? h.x : vq.x;
  vt.y = t.y <= 0.f ? h.y : vq.y;
  w = v * vt;
  if (tie) {
    v = -t;
    w = f2{1.f, 1.f};
  }
}

template <int C>
__device__ __forceinline__ void dpp_add4(float& x0, float& x1, float& x2, float& x3) {
  const float y0 = dpp_mov<C>(x0), y1 = dpp_mov<C>(x1), y2 = dpp_mov<C>(x2), y3 = dpp_mov<C>(x3);
  x0 += y0;
  x1 += y1;
  x2 += y2;
  x3 += y3;
}

// Four sums over the G lanes of a group at once (result in every lane of the
// group).  Power-of-two groups: the steps of the four DPP butterflies interleaved,
// so each step's VALU -> DPP hazard is covered by the other sums' instructions;
// tight groups (G = 2K) take group_sum's bpermute tree per sum.
template <int G>
__device__ __forceinline__ void group_sum4(float& x0, float& x1, float& x2, float& x3, int j, int gbase) {
  if constexpr ((G & (G - 1)) == 0 && G <= 16) {
    if constexpr (G >= 2) dpp_add4<0xb1>(x0, x1, x2, x3);   // quad_perm [1,0,3,2]
    if constexpr (G >= 4) dpp_add4<0x4e>(x0, x1, x2, x3);   // quad_perm [2,3,0,1]
    if constexpr (G >= 8) dpp_add4<0x141>(x0, x1, x2, x3);  // row_half_mirror
    if constexpr (G >= 16) dpp_add4<0x140>(x0, x1, x2, x3); // row_mirror
  } else {
    x0 = group_sum<G>(x0, j, gbase);
    x1 = group_sum<G>(x1, j, gbase);
    x2 = group_sum<G>(x2, j, gbase);
    x3 = group_sum<G>(x3, j, gbase);
  }
}

// One participant's two-track update (win/loss or tie) and the match quality.
//   pm, ps   prior (mu, sigma) of the (shared, mode) tracks
//   lsg      +1 / -1: this lane's roster, times the winner side (+1 on ties)
//   x        in: this lane's four sum terms, must be 0 on lanes outside the rosters
// Returns the posterior pair through nm / ns and the quality (mode track, sigma
// without tau: SURVEY A.4) through q.
template <int G>
__device__ __forceinline__ void rate_pair(f2 pm, f2 ps, bool inr, float lsg, int n, bool tie,
                                          float beta2, float tau2, int j, int gbase, f2& nm, f2& ns,
                                          float& q) {
  const f2 s2 = ps * ps + tau2;
  float x0 = inr ? s2.x : 0.f, x1 = inr ? s2.y : 0.f;
  float x2 = inr ? lsg * pm.x : 0.f, x3 = inr ? lsg * pm.y : 0.f;
  group_sum4<G>(x0, x1, x2, x3, j, gbase);
  const float nb2 = (float)n * beta2;
  const f2 c2 = f2{x0, x1} + nb2;
  const f2 rc = rsq2(c2);
  // x2, x3 = the winner side's mu sum minus the loser side's (roster 0 minus roster
  // 1 on ties): the same in every lane of the group, so t = d / c is per match
  f2 v, w;
  vw_pair(f2{x2, x3} * rc, tie, v, w);
  nm = pm + s2 * ((v * rc) * lsg);
  ns = sqrt2(s2 - s2 * s2 * (w * (rc * rc)));
  // quality: den = n beta^2 + sum sigma^2 (mode track) = c2.y - n tau^2
  const float rd = __builtin_amdgcn_rcpf(c2.y - (float)n * tau2);
  q = __builtin_amdgcn_sqrtf(nb2 * rd * __builtin_amdgcn_exp2f(x3 * x3 * rd * -1.4426950408889634f));
}

}  // namespace ana
