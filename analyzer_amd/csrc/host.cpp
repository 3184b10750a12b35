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
  for (int64_t p = 0; p < g.num_players; ++p) gen_player(g, p, state + p * 16, attrs + p * 4);
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

template <int K>
static void schedule_k(const int32_t* rec, int64_t M, int64_t P, uint32_t* occ) {
  constexpr int S = 2 * K;
  std::vector<uint32_t> cnt((size_t)P, 0u);
  for (int64_t m = 0; m < M; ++m) {
    MatchWork<float, K> w;
    decode_record<float, K>(rec + m * (S + 2), P, w);
    for (int j = 0; j < S; ++j) {
      occ[m * S + j] = 0;
      if (w.status == kRated && w.id[j] >= 0) occ[m * S + j] = cnt[(size_t)w.id[j]]++;
    }
  }
}

int host_schedule(int K, const int32_t* rec, int64_t M, int64_t P, uint32_t* occ) {
  switch (K) {
    case 1: schedule_k<1>(rec, M, P, occ); return 0;
    case 2: schedule_k<2>(rec, M, P, occ); return 0;
    case 3: schedule_k<3>(rec, M, P, occ); return 0;
    case 4: schedule_k<4>(rec, M, P, occ); return 0;
    case 5: schedule_k<5>(rec, M, P, occ); return 0;
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
        const float* row = state + (int64_t)w.id[j] * 2 * kTrackStride;
        st = make_prior<T, K>(w, j, (T)row[0], (T)row[1], (T)row[2 + 2 * w.mode],
                              (T)row[3 + 2 * w.mode], attrs + (int64_t)w.id[j] * 4, us, prm.vst,
                              nulls);
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
        float* row = state + (int64_t)w.id[j] * 2 * kTrackStride;
        if ((w.last >> j) & 1u) {
          row[0] = (float)w.ns_mu[j];
          row[1] = (float)w.ns_sig[j];
          row[2 + 2 * w.mode] = (float)w.nm_mu[j];
          row[3 + 2 * w.mode] = (float)w.nm_sig[j];
        }
        if (prm.record_first_prior && first_prior && w.first[j] == j) {
          float* fp = first_prior + (int64_t)w.id[j] * 2 * kTrackStride;
          if ((nulls >> (2 * j)) & 1u) { fp[0] = (float)w.ms[j]; fp[1] = (float)w.ss[j]; }
          if ((nulls >> (2 * j + 1)) & 1u) {
            fp[2 + 2 * w.mode] = (float)w.mm[j];
            fp[3 + 2 * w.mode] = (float)w.sm[j];
          }
        }
      }
    }
    const bool afkish = w.status == kAfk || w.status == kInvalidRosters;
    out.quality[m] = rated ? (float)w.quality : (afkish ? 0.f : NAN);
    out.status[m] = w.status;
    for (int j = 0; j < S; ++j) {
      const bool on = rated && w.id[j] >= 0;
      out.s_mu[m * S + j] = on ? (float)w.ns_mu[j] : NAN;
      out.s_sig[m * S + j] = on ? (float)w.ns_sig[j] : NAN;
      out.delta[m * S + j] = on ? (float)w.delta[j] : NAN;
      out.m_mu[m * S + j] = on ? (float)w.nm_mu[j] : NAN;
      out.m_sig[m * S + j] = on ? (float)w.nm_sig[j] : NAN;
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

void host_sweep_delta(const float* s0, const float* s, const float* fp, float* buf, int64_t P) {
  for (int64_t p = 0; p < P; ++p) sweep_delta_player(s0 + p * 16, s + p * 16, fp + p * 16, buf + p * 16);
}

void host_sweep_apply(const float* s0, const float* buf, const float* attrs, float* s,
                      const float* vst, float unknown_sigma, int64_t P) {
  for (int64_t p = 0; p < P; ++p)
    sweep_apply_player(s0 + p * 16, buf + p * 16, attrs + p * 4, vst, unknown_sigma, s + p * 16);
}

}  // namespace ana
