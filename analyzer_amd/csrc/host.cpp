// Host (CPU) mirror of the engine: the same per-match core as the MI355X
// kernels, run sequentially in stream order.  It is the exact-semantics oracle
// for the device dataflow executor (fp64 by default) and the CPU path for the
// plumbing configuration (BASELINE config 1).  It is not a fallback for GPU
// tensors: device tensors always go to the HIP kernels.
#include "host.h"

#include <math.h>
#include <string.h>

#include <vector>

#include "gen_core.h"
#include "rate_core.h"

namespace ana {

void host_gen_roster(const GenRosterParams& g, float* state, float* attrs) {
  for (int64_t p = 0; p < g.num_players; ++p) gen_player(g, p, state + p * kRowFloats, attrs + p * 4);
}

template <int K>
static void gen_stream_k(const GenStreamParams& g, int32_t* rec, int64_t M) {
  for (int64_t m = 0; m < M; ++m) gen_match<K>(g, m, rec + m * (2 * K + 2));
}

int host_gen_stream(int K, const GenStreamParams& g, int32_t* rec, int64_t M) {
  switch (K) {
    case 1: gen_stream_k<1>(g, rec, M); return 0;
    case 2: gen_stream_k<2>(g, rec, M); return 0;
    case 3: gen_stream_k<3>(g, rec, M); return 0;
    case 4: gen_stream_k<4>(g, rec, M); return 0;
    case 5: gen_stream_k<5>(g, rec, M); return 0;
    default: return -1;
  }
}

// Same outputs as the device schedule (common.h kLinkWords): link[slot] =
// next match of the player | has-earlier flag; deps[m].  Slots of matches that
// rate nothing are left unwritten.
template <int K>
static void schedule_k(const int32_t* rec, int64_t M, int64_t P, uint32_t* link, int32_t* deps) {
  constexpr int S = 2 * K;
  std::vector<uint32_t> last((size_t)P, kNone);
  for (int64_t m = 0; m < M; ++m) {
    MatchWork<float, K> w;
    decode_record<float, K>(rec + m * (S + 2), P, w);
    deps[m] = 0;
    if (w.status != kRated) continue;
    for (int j = 0; j < S; ++j) {
      if (w.id[j] < 0) continue;
      const uint32_t slot = (uint32_t)(m * S + j);
      const size_t p = (size_t)w.id[j];
      link[slot] = kNoMatch;
      if (last[p] != kNone) {
        link[last[p]] = (link[last[p]] & ~kMatchMask) | (uint32_t)m;
        link[slot] |= kLinkHasPred;
        if (w.first[j] == j) ++deps[m];
      }
      last[p] = slot;
    }
  }
}

void host_gen_event_counts(const GenEventParams& g, int64_t base, int64_t M, int64_t* counts) {
  for (int64_t m = 0; m < M; ++m) counts[m] = gen_event_count(g, (uint64_t)(base + m));
}

int host_gen_events(int K, const GenEventParams& g, int64_t base, const int32_t* rec,
                    const int64_t* evoff, int64_t M, int32_t* events) {
  if (K < 1 || K > 5) return -1;
  const int S = 2 * K;
  for (int64_t m = 0; m < M; ++m) {
    const uint32_t m0 = (uint32_t)rec[m * (S + 2) + S];
    const int n0 = meta_n0(m0) < K ? meta_n0(m0) : K, n1 = meta_n1(m0) < K ? meta_n1(m0) : K;
    for (int64_t e = evoff[m]; e < evoff[m + 1]; ++e) {
      int32_t* ev = events + e * 2;
      gen_event(g, (uint64_t)(base + m), e - evoff[m], (int32_t)m, n0 + n1, ev);
      const int r = event_slot(ev[0]);
      ev[0] = (ev[0] & ~0xff) | (r < n0 ? r : K + (r - n0));
    }
  }
  return 0;
}

int64_t host_telemetry(int K, const TelemetryParams& tp) {
  const int S = 2 * K;
  const int64_t M = tp.num_matches;
  int64_t bad = 0;
  for (int64_t i = 0; i < M * S * kStatFeatures; ++i) tp.stats[i] = 0.f;
  for (int64_t m = 0; m < M; ++m)
    for (int64_t e = tp.evoff[m]; e < tp.evoff[m + 1]; ++e) {
      const int32_t* ev = tp.events + e * 2;
      const int slot = event_slot(ev[0]);
      if (event_tag(ev[0]) != (uint32_t)(m & 0xffff) || slot >= S) {  // strict attribution
        ++bad;
        continue;
      }
      float value, add;
      memcpy(&value, ev + 1, 4);
      const int f = event_feature(event_type(ev[0]), value, add);
      float* row = tp.stats + ((int64_t)m * S + slot) * kStatFeatures;
      if (f >= 0) row[f] += add;
      row[kStatEvents] += 1.f;
    }
  return bad;
}

template <int K>
static int64_t levels_k(const int32_t* rec, int64_t M, int64_t P, int32_t* level) {
  constexpr int S = 2 * K;
  std::vector<int32_t> last((size_t)P, 0);
  int64_t depth = 0;
  for (int64_t m = 0; m < M; ++m) {
    MatchWork<float, K> w;
    decode_record<float, K>(rec + m * (S + 2), P, w);
    level[m] = 0;
    if (w.status != kRated) continue;
    int32_t l = 0;
    for (int j = 0; j < S; ++j)
      if (w.id[j] >= 0 && last[(size_t)w.id[j]] > l) l = last[(size_t)w.id[j]];
    ++l;
    for (int j = 0; j < S; ++j)
      if (w.id[j] >= 0) last[(size_t)w.id[j]] = l;
    level[m] = l;
    if (l > depth) depth = l;
  }
  return depth;
}

int64_t host_levels(int K, const int32_t* rec, int64_t M, int64_t P, int32_t* level) {
  switch (K) {
    case 1: return levels_k<1>(rec, M, P, level);
    case 2: return levels_k<2>(rec, M, P, level);
    case 3: return levels_k<3>(rec, M, P, level);
    case 4: return levels_k<4>(rec, M, P, level);
    case 5: return levels_k<5>(rec, M, P, level);
    default: return -1;
  }
}

int host_schedule(int K, const int32_t* rec, int64_t M, int64_t P, uint32_t* link, int32_t* deps) {
  switch (K) {
    case 1: schedule_k<1>(rec, M, P, link, deps); return 0;
    case 2: schedule_k<2>(rec, M, P, link, deps); return 0;
    case 3: schedule_k<3>(rec, M, P, link, deps); return 0;
    case 4: schedule_k<4>(rec, M, P, link, deps); return 0;
    case 5: schedule_k<5>(rec, M, P, link, deps); return 0;
    default: return -1;
  }
}

template <typename T, int K>
static void rate_k(const int32_t* rec, float* state, const float* attrs, float* first_prior,
                   const RateOut& out, const RateParams& prm) {
  constexpr int S = 2 * K;
  const T beta2 = (T)prm.beta2, tau2 = (T)prm.tau2, us = (T)prm.unknown_sigma;
  for (int64_t m = 0; m < prm.num_matches; ++m) {
    MatchWork<T, K> w;
    decode_record<T, K>(rec + m * (S + 2), prm.num_players, w);
    uint32_t nulls = 0;
    if (w.status == kRated) {
      uint8_t st = kRated;
      for (int j = 0; j < S && st == kRated; ++j) {
        if (w.first[j] != j) continue;
        const float* row = state + (int64_t)w.id[j] * kRowFloats;
        const float* gm = row + 4 * (1 + w.mode);
        st = make_prior<T, K>(w, j, (T)row[0], (T)row[2], (T)gm[0], (T)gm[2],
                              attrs + (int64_t)w.id[j] * 4, us, prm.vst, nulls);
      }
      w.status = st;
      if (st == kRated) {
        copy_dup_priors<T, K>(w);
        rate_priors<T, K>(w, beta2, tau2);
      }
    }
    const bool rated = w.status == kRated;
    if (rated) {
      for (int j = 0; j < S; ++j) {
        if (w.id[j] < 0) continue;
        float* row = state + (int64_t)w.id[j] * kRowFloats;
        float* gm = row + 4 * (1 + w.mode);
        if ((w.last >> j) & 1u) {  // host mirror writes tag 0 (never a live device tag)
          row[0] = (float)w.ns_mu[j];
          row[2] = (float)w.ns_sig[j];
          gm[0] = (float)w.nm_mu[j];
          gm[2] = (float)w.nm_sig[j];
          row[1] = row[3] = gm[1] = gm[3] = 0.f;
        }
        if (prm.record_first_prior && first_prior && w.first[j] == j) {
          float* fp = first_prior + (int64_t)w.id[j] * kRowFloats;
          if ((nulls >> (2 * j)) & 1u) { fp[0] = (float)w.ms[j]; fp[2] = (float)w.ss[j]; }
          if ((nulls >> (2 * j + 1)) & 1u) {
            fp[4 * (1 + w.mode)] = (float)w.mm[j];
            fp[4 * (1 + w.mode) + 2] = (float)w.sm[j];
          }
        }
      }
    }
    const bool afkish = w.status == kAfk || w.status == kInvalidRosters;
    out.quality[m * out.qrow] = rated ? (float)w.quality : (afkish ? 0.f : NAN);
    out.status[m * out.srow] = w.status;
    for (int j = 0; j < S; ++j) {
      const bool on = rated && w.id[j] >= 0;
      out.s_mu[m * out.row + j] = on ? (float)w.ns_mu[j] : NAN;
      out.s_sig[m * out.row + j] = on ? (float)w.ns_sig[j] : NAN;
      out.delta[m * out.row + j] = on ? (float)w.delta[j] : NAN;
      out.m_mu[m * out.row + j] = on ? (float)w.nm_mu[j] : NAN;
      out.m_sig[m * out.row + j] = on ? (float)w.nm_sig[j] : NAN;
    }
  }
}

template <typename T>
static int rate_t(int K, const int32_t* rec, float* state, const float* attrs, float* first_prior,
                  const RateOut& out, const RateParams& prm) {
  switch (K) {
    case 1: rate_k<T, 1>(rec, state, attrs, first_prior, out, prm); return 0;
    case 2: rate_k<T, 2>(rec, state, attrs, first_prior, out, prm); return 0;
    case 3: rate_k<T, 3>(rec, state, attrs, first_prior, out, prm); return 0;
    case 4: rate_k<T, 4>(rec, state, attrs, first_prior, out, prm); return 0;
    case 5: rate_k<T, 5>(rec, state, attrs, first_prior, out, prm); return 0;
    default: return -1;
  }
}

int host_rate(int K, bool fp64, const int32_t* rec, float* state, const float* attrs,
              float* first_prior, const RateOut& out, const RateParams& prm) {
  return fp64 ? rate_t<double>(K, rec, state, attrs, first_prior, out, prm)
              : rate_t<float>(K, rec, state, attrs, first_prior, out, prm);
}

}  // namespace ana

#include "sweep_core.h"

namespace ana {

// s0, a, s2: base rows [P][kBaseFloats] (sweep_core.h); s: roster rows [P][32]
void host_sweep_delta(const float* s0, const float* a, const float* s, const float* attrs,
                      const float* vst, float unknown_sigma, bool scaled, float* buf, int64_t P) {
  for (int64_t p = 0; p < P; ++p)
    sweep_delta_player(s0 + p * kBaseFloats, a + p * kBaseFloats, s + p * kRowFloats, attrs + p * 4,
                       vst, unknown_sigma, scaled, buf + p * 16);
}

void host_sweep_apply(const float* s0, const float* buf, const float* attrs, float* s, float* s2,
                      bool scaled, const float* vst, float unknown_sigma, int64_t P, uint32_t* clamps) {
  for (int64_t p = 0; p < P; ++p) {
    float ob[kBaseFloats];
    sweep_apply_player(s0 + p * kBaseFloats, buf + p * 16, attrs + p * 4, vst, unknown_sigma, scaled,
                       s + p * kRowFloats, ob, clamps);
    if (s2)
      for (int k = 0; k < kBaseFloats; ++k) s2[p * kBaseFloats + k] = ob[k];
  }
}

void host_correct_records(int K, const int32_t* rec, int64_t M, float* rows, int64_t orow, const float* delta,
                          int64_t P) {
  const int S = 2 * K;
  for (int64_t m = 0; m < M; ++m) {
    float* row = rows + m * orow;
    if (reinterpret_cast<const uint8_t*>(row + 5 * S + 1)[0] != kRated) continue;
    const int32_t* r = rec + m * (S + 2);
    const uint32_t m0 = (uint32_t)r[S];
    const int t = 1 + meta_mode(m0);
    for (int j = 0; j < S; ++j) {
      if ((j < K ? j : j - K) >= (j < K ? meta_n0(m0) : meta_n1(m0))) continue;
      const int32_t p = r[j];
      if (p < 0 || p >= P) continue;
      const float* d = delta + (int64_t)p * 16;
      correct_record_track(d[0], d[1], row[j], row[S + j]);
      correct_record_track(d[2 * t], d[2 * t + 1], row[3 * S + j], row[4 * S + j]);
    }
  }
}

void host_prefix_delta(const float* s0, const float* prefix, const float* attrs, const float* vst,
                       float unknown_sigma, float* delta, int64_t P) {
  for (int64_t p = 0; p < P; ++p)
    prefix_delta_player(s0 + p * kBaseFloats, prefix + p * 14, attrs + p * 4, vst, unknown_sigma, delta + p * 16);
}

}  // namespace ana
