// Per-match TrueSkill core shared by the MI355X kernels and the C++ host mirror.
//
// Semantics: /root/reference/rater.py:69-169.  Math:
// the two-team closed form of expectation propagation,
// which equals trueskill 0.4.4's factor graph for two teams; ties take the
// exact eps->0 draw limit (v = -t, w = 1) that the reference's 50-digit mpmath
// run produces.  T is float on device, double (oracle) or float on the host.
#pragma once

#include <math.h>

#include "common.h"

namespace ana {

template <typename T>
ANA_HD bool is_nan(T x) { return x != x; }

// v = pdf(t)/cdf(t), w = v (v + t) for a win with zero draw margin, stable for
// t << 0 (big upsets): there v = u + h(u), w = (u + h) h with u = -t and h the
// Mills-ratio continued fraction, avoiding the v(v+t) cancellation.
template <typename T>
ANA_HD void vw_win(T t, T& v, T& w) {
  if (t < (T)-5) {
    const T u = -t;
    T f = u;
    constexpr int terms = sizeof(T) == 4 ? 16 : 48;
#pragma unroll
    for (int k = terms; k >= 2; --k) f = u + (T)k / f;
    const T h = (T)1 / f;
    v = u + h;
    w = v * h;
  } else {
    // cdf(t) >= 2.8e-7 here, so erfc keeps full relative precision and the
    // plain pdf/cdf ratio is as accurate as the erfcx form (which costs ~70
    // VGPRs in ocml); pdf underflow for t > 13 gives the exact v = w = 0 limit.
    const T cdf = (T)0.5 * erfc(-t * (T)0.70710678118654752);
    v = (T)0.39894228040143268 * exp((T)-0.5 * t * t) / cdf;
    w = v * (v + t);
  }
}

// Work record for one match with up to K players per roster (S = 2K slots).
template <typename T, int K>
struct MatchWork {
  static constexpr int S = 2 * K;
  int32_t id[S];
  int8_t first[S];    // first slot carrying the same player (== j when first); -1 empty
  int8_t prevdup[S];  // latest earlier slot with the same player, -1 if none
  uint32_t last;      // bit j: no later slot carries this player (bitmask, not bool[]:
                      // a divergent bool array costs an SGPR pair per element)
  int n0, n1, mode, nrosters;
  int rank0, rank1;   // int(not roster.winner)
  uint8_t status;
  // priors (after seeding / mode fallback)
  T ms[S], ss[S], mm[S], sm[S];
  uint32_t had_shared;  // bit j: stored shared rating existed (delta != 0 rule)
  // results
  T quality;
  T ns_mu[S], ns_sig[S], nm_mu[S], nm_sig[S], delta[S];
};

// Decode a stream record.  Sets status to kRated ("to be rated") or to the
// early outcome (unsupported / invalid rosters / AFK) that needs no state.
template <typename T, int K>
ANA_HD void decode_record(const int32_t* rec, int64_t num_players, MatchWork<T, K>& w) {
  constexpr int S = 2 * K;
  const uint32_t m0 = (uint32_t)rec[S], m1 = (uint32_t)rec[S + 1];
  w.mode = meta_mode(m0);
  w.n0 = meta_n0(m0);
  w.n1 = meta_n1(m0);
  w.nrosters = meta_nrosters(m0);
  w.rank0 = meta_winner0(m1) ? 0 : 1;
  w.rank1 = meta_winner1(m1) ? 0 : 1;
  bool bad = w.n0 > K || w.n1 > K;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int pos = j < K ? j : j - K;
    const int n = j < K ? w.n0 : w.n1;
    const int32_t id = rec[j];
    const bool in_roster = pos < n;
    if (in_roster && (id < 0 || (int64_t)id >= num_players)) bad = true;
    w.id[j] = in_roster && id >= 0 && (int64_t)id < num_players ? id : -1;
  }
  w.last = 0;
  w.had_shared = 0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    w.first[j] = w.id[j] < 0 ? (int8_t)-1 : (int8_t)j;
    w.prevdup[j] = -1;
    if (w.id[j] >= 0) w.last |= 1u << j;
#pragma unroll
    for (int i = 0; i < j; ++i) {
      if (w.id[j] >= 0 && w.id[i] == w.id[j]) {
        if (w.first[j] == j) w.first[j] = (int8_t)i;
        w.prevdup[j] = (int8_t)i;
        w.last &= ~(1u << i);
      }
    }
  }
  if (w.mode >= kModes) {
    w.status = kUnsupportedMode;
  } else if (bad) {
    w.status = kErrBadRecord;
  } else if (w.nrosters != 2) {
    w.status = kInvalidRosters;
  } else if (meta_afk(m1)) {
    w.status = kAfk;
  } else {
    w.status = kRated;
  }
}

// Seed a player with no shared rating (rater.py:42-62).  false = KeyError.
template <typename T>
ANA_HD bool seed_prior(const float* attr, T unknown_sigma, const float* vst, T& mu, T& sig) {
  const float rr = attr[0], rb = attr[1], tier = attr[2];
  float rp = NAN;
  if (rr == rr && rr != 0.f) rp = rr;
  if (rb == rb && rb != 0.f && (rp != rp || rb > rp)) rp = rb;
  if (rp == rp) {
    sig = unknown_sigma * (T)(2.0 / 3.0);
    mu = (T)rp + sig;
    return true;
  }
  if (tier != tier) return false;
  const int ti = (int)tier;
  if ((float)ti != tier || ti < -1 || ti > 29) return false;
  sig = unknown_sigma;
  mu = (T)vst[ti + 1] + sig;
  return true;
}

// Turn raw stored state into priors for slot j (first-of-dup slots only);
// returns a status (kRated = fine).  shared/mode are the stored (mu, sigma).
// Priors of one player from its stored (mu, sigma) on both tracks.  Returns a
// status (kRated = fine); flags: bit0 had a stored shared rating, bit1 shared
// was NULL (seeded), bit2 mode track was NULL (fell back to the shared prior).
template <typename T>
ANA_HD uint8_t player_prior(T sh_mu, T sh_sig, T md_mu, T md_sig, const float* attr,
                            T unknown_sigma, const float* vst, T& ms, T& ss, T& mm, T& sm,
                            uint32_t& flags) {
  flags = 0;
  if (is_nan(sh_mu)) {
    if (!seed_prior<T>(attr, unknown_sigma, vst, sh_mu, sh_sig)) return kErrSeed;
    flags |= 2u;
  } else if (!(sh_sig == sh_sig) || sh_sig == (T)0) {
    return kErrSigma;
  } else {
    flags |= 1u;
  }
  ms = sh_mu;
  ss = sh_sig;
  if (is_nan(md_mu)) {
    flags |= 4u;
    md_mu = sh_mu;
    md_sig = sh_sig;
  } else if (!(md_sig == md_sig) || md_sig == (T)0) {
    return kErrSigma;
  }
  mm = md_mu;
  sm = md_sig;
  return kRated;
}

// null_mask gets bit 2j (shared track was NULL) and bit 2j+1 (mode track was NULL).
template <typename T, int K>
ANA_HD uint8_t make_prior(MatchWork<T, K>& w, int j, T sh_mu, T sh_sig, T md_mu, T md_sig,
                          const float* attr, T unknown_sigma, const float* vst,
                          uint32_t& null_mask) {
  uint32_t f = 0;
  const uint8_t st = player_prior<T>(sh_mu, sh_sig, md_mu, md_sig, attr, unknown_sigma, vst,
                                     w.ms[j], w.ss[j], w.mm[j], w.sm[j], f);
  if (st != kRated) return st;
  if (f & 1u) w.had_shared |= 1u << j;
  if (f & 2u) null_mask |= 1u << (2 * j);
  if (f & 4u) null_mask |= 1u << (2 * j + 1);
  return kRated;
}

template <typename T, int K>
ANA_HD void copy_dup_priors(MatchWork<T, K>& w) {
  // compile-time indices only (a runtime-indexed register array spills to scratch)
#pragma unroll
  for (int j = 1; j < 2 * K; ++j) {
#pragma unroll
    for (int i = 0; i < j; ++i) {
      if (w.first[j] == i) {
        w.ms[j] = w.ms[i];
        w.ss[j] = w.ss[i];
        w.mm[j] = w.mm[i];
        w.sm[j] = w.sm[i];
        if ((w.had_shared >> i) & 1u) w.had_shared |= 1u << j;
      }
    }
  }
}

// Closed-form update coefficients for one track, given the team sums.
//   d  = sum(mu | roster 0) - sum(mu | roster 1),  c2 = n beta^2 + sum(sigma^2 + tau^2)
// A player with s2 = sigma^2 + tau^2 moves to
//   mu' = mu + s2 * (roster 0 ? a0 : a1),   sigma' = sqrt(s2 (1 - s2/c2 * wf)).
// Win/loss: t = +-d/c, (v, w) = vw_win(t); tie: the draw limit v = -t, w = 1.
template <typename T>
struct UpdCoef {
  T a0, a1, wf, c2;
};

template <typename T>
ANA_HD UpdCoef<T> update_coef(T d, T c2, int rank0, int rank1) {
  UpdCoef<T> k;
  k.c2 = c2;
  if (rank0 == rank1) {
    k.a0 = -d / c2;
    k.a1 = d / c2;
    k.wf = (T)1;
  } else {
    const T c = sqrt(c2);
    const T sgn = rank0 < rank1 ? (T)1 : (T)-1;
    T v, w;
    vw_win<T>(sgn * d / c, v, w);
    k.a0 = sgn * v / c;
    k.a1 = -k.a0;
    k.wf = w;
  }
  return k;
}

template <typename T>
ANA_HD void apply_coef(const UpdCoef<T>& k, bool roster0, T mu, T sig, T tau2, T& mu_out,
                       T& sig_out) {
  const T s2 = sig * sig + tau2;
  mu_out = mu + s2 * (roster0 ? k.a0 : k.a1);
  sig_out = sqrt(s2 * ((T)1 - s2 / k.c2 * k.wf));
}

template <typename T>
ANA_HD T quality_from_sums(int n, T sum_sig2, T d, T beta2) {
  const T nb2 = (T)n * beta2;
  const T den = nb2 + sum_sig2;
  return sqrt(nb2 / den) * exp(-d * d / ((T)2 * den));
}

// One track of the two-team closed-form update; returns false on non-finite.
template <typename T, int K>
ANA_HD bool update_track(const T (&mu)[2 * K], const T (&sig)[2 * K], int n0, int n1, int rank0,
                         int rank1, T beta2, T tau2, T (&mu_out)[2 * K], T (&sig_out)[2 * K]) {
  T sum_s2 = 0, d = 0;
#pragma unroll
  for (int j = 0; j < 2 * K; ++j) {
    const bool in0 = j < K && j < n0;
    const bool in1 = j >= K && j - K < n1;
    if (in0 || in1) sum_s2 += sig[j] * sig[j] + tau2;
    if (in0) d += mu[j];
    if (in1) d -= mu[j];
  }
  const UpdCoef<T> k = update_coef<T>(d, (T)(n0 + n1) * beta2 + sum_s2, rank0, rank1);
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 2 * K; ++j) {
    apply_coef<T>(k, j < K, mu[j], sig[j], tau2, mu_out[j], sig_out[j]);
    const bool used = (j < K && j < n0) || (j >= K && j - K < n1);
    if (used && !(isfinite(mu_out[j]) && isfinite(sig_out[j]))) ok = false;
  }
  return ok;
}

// Match quality on the mode track, sigma without tau.
template <typename T, int K>
ANA_HD T match_quality(const T (&mu)[2 * K], const T (&sig)[2 * K], int n0, int n1, T beta2) {
  T sum_s2 = 0, d = 0;
#pragma unroll
  for (int j = 0; j < 2 * K; ++j) {
    const bool in0 = j < K && j < n0;
    const bool in1 = j >= K && j - K < n1;
    if (in0 || in1) sum_s2 += sig[j] * sig[j];
    if (in0) d += mu[j];
    if (in1) d -= mu[j];
  }
  return quality_from_sums<T>(n0 + n1, sum_s2, d, beta2);
}

// Everything after the priors: quality, both tracks, deltas (rater.py:138-169).
template <typename T, int K>
ANA_HD void rate_priors(MatchWork<T, K>& w, T beta2, T tau2) {
  if (w.n0 == 0 || w.n1 == 0) {  // TrueSkill.validate_rating_groups -> ValueError
    w.status = kErrEmptyRoster;
    return;
  }
  w.quality = match_quality<T, K>(w.mm, w.sm, w.n0, w.n1, beta2);
  const bool ok1 = update_track<T, K>(w.ms, w.ss, w.n0, w.n1, w.rank0, w.rank1, beta2, tau2,
                                      w.ns_mu, w.ns_sig);
  const bool ok2 = update_track<T, K>(w.mm, w.sm, w.n0, w.n1, w.rank0, w.rank1, beta2, tau2,
                                      w.nm_mu, w.nm_sig);
  if (!(ok1 && ok2) || !isfinite(w.quality)) {
    w.status = kErrNumeric;
    return;
  }
#pragma unroll
  for (int j = 0; j < 2 * K; ++j) {
    const int pd = w.prevdup[j];
    T prev = 0;
    bool has_prev = false;
    if (pd >= 0) {  // same player earlier in this match: its write is visible
#pragma unroll
      for (int i = 0; i < 2 * K; ++i)
        if (i == pd) prev = w.ns_mu[i] - w.ns_sig[i];
      has_prev = true;
    } else if ((w.had_shared >> j) & 1u) {
      prev = w.ms[j] - w.ss[j];
      has_prev = true;
    }
    w.delta[j] = has_prev ? (w.ns_mu[j] - w.ns_sig[j]) - prev : (T)0;
  }
}

}  // namespace ana
