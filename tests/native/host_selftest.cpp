// Native self-test of the C++ host mirror, built with -fsanitize=address,undefined
// (SURVEY §5 "race detection / sanitizers": host code only -- GPU ASan is not
// available on this pool).  Exercises every host entry point on generated data,
// including edge records (uneven/empty rosters, AFK, ties, unsupported modes, bad
// tiers, duplicated players, 5v5), and checks the schedule invariants the
// dataflow executor relies on.  Exit code 0 = pass.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "host.h"

using namespace ana;

static int fails = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                          \
    }                                                                   \
  } while (0)

static uint32_t prob(double p) { return (uint32_t)(p * 4294967295.0); }

static void run(int K, int64_t P, int64_t M, uint64_t seed) {
  const int S = 2 * K, R = S + 2;
  GenRosterParams gr{};
  gr.seed = seed; gr.num_players = P;
  gr.p_tier_null = prob(0.02); gr.p_tier_bad = prob(0.02); gr.p_rp_ranked = prob(0.3);
  gr.p_rp_blitz = prob(0.15); gr.p_rated = prob(0.5); gr.p_mode_rated = prob(0.5);
  gr.mu_lo = 1000.f; gr.mu_span = 1500.f; gr.sig_lo = 80.f; gr.sig_span = 300.f;
  std::vector<float> state((size_t)P * kRowFloats), attrs((size_t)P * 4);
  host_gen_roster(gr, state.data(), attrs.data());

  GenStreamParams gs{};
  gs.seed = seed + 1; gs.base = 0; gs.num_players = P; gs.team_size = K;
  const double cdf[7] = {0.25, 0.6, 0.7, 0.8, 0.88, 0.96, 1.0};
  for (int i = 0; i < 7; ++i) gs.mode_cdf[i] = prob(cdf[i]);
  gs.p_uneven = prob(0.1); gs.p_bad_rosters = prob(0.03); gs.p_tie = prob(0.05);
  gs.p_afk = prob(0.05); gs.p_hot = prob(0.2); gs.hot_players = 3;
  std::vector<int32_t> rec((size_t)M * R);
  CHECK(host_gen_stream(K, gs, rec.data(), M) == 0);

  // schedule invariants
  std::vector<uint32_t> link((size_t)M * S * kLinkWords, 0xdeadbeefu);
  std::vector<int32_t> deps(M);
  CHECK(host_schedule(K, rec.data(), M, P, link.data(), deps.data()) == 0);
  std::vector<int32_t> level(M);
  const int64_t depth = host_levels(K, rec.data(), M, P, level.data());
  CHECK(depth >= 1 && depth <= M);
  for (int64_t m = 0; m < M; ++m) {
    if (level[m] == 0) CHECK(deps[m] == 0);
    for (int j = 0; j < S; ++j) {
      const int32_t id = rec[m * R + j];
      if (id < 0 || level[m] == 0) continue;
      const uint32_t succ = link[m * S + j] & kMatchMask;
      if (succ != kNoMatch) {
        CHECK((int64_t)succ >= m && (int64_t)succ < M);
        bool found = false;  // the successor really contains the player
        for (int q = 0; q < S; ++q) found |= rec[(int64_t)succ * R + q] == id;
        CHECK(found);
      }
    }
  }

  // rate in both precisions, with and without first-prior recording
  std::vector<float> st64 = state, st32 = state, fp(state.size(), NAN);
  std::vector<float> q(M), smu(M * S), ssg(M * S), dl(M * S), mmu(M * S), msg(M * S);
  std::vector<uint8_t> status(M);
  RateOut out{q.data(), status.data(), smu.data(), ssg.data(), dl.data(), mmu.data(), msg.data(),
              S, 1, 1};
  std::vector<float> vst(kVstTiers);
  for (int t = 0; t < kVstTiers; ++t) vst[t] = 500.f + 70.f * t;
  RateParams prm{};
  prm.beta2 = 1e6f; prm.tau2 = 100.f; prm.unknown_sigma = 500.f;
  prm.num_players = (int32_t)P; prm.num_matches = M; prm.epoch = 1; prm.vst = vst.data();
  CHECK(host_rate(K, true, rec.data(), st64.data(), attrs.data(), nullptr, out, prm) == 0);
  int rated = 0;
  for (int64_t m = 0; m < M; ++m) {
    CHECK(status[m] <= kErrBadRecord);
    if (status[m] == kRated) {
      ++rated;
      CHECK(q[m] >= 0.f && q[m] <= 1.f);
      for (int j = 0; j < S; ++j)
        if (rec[m * R + j] >= 0) CHECK(isfinite(smu[m * S + j]) && ssg[m * S + j] > 0.f);
    }
  }
  CHECK(rated > M / 2);
  prm.record_first_prior = 1;
  CHECK(host_rate(K, false, rec.data(), st32.data(), attrs.data(), fp.data(), out, prm) == 0);
  double maxd = 0;
  for (size_t i = 0; i < state.size(); i += 2)
    if (!isnan(st64[i])) maxd = fmax(maxd, fabs((double)st64[i] - st32[i]));
  CHECK(maxd < 5.0);

  // DP merge round trip (raw and base-relative encodings): messages of "after"
  // against "before", then apply, reproduces "after"
  // (the merge keeps its window start as base rows: (mu, sigma) per granule)
  std::vector<float> base((size_t)P * kBaseFloats);
  for (int64_t p = 0; p < P; ++p)
    for (int g = 0; g < kGranules; ++g) {
      base[p * kBaseFloats + 2 * g] = state[p * kRowFloats + 4 * g];
      base[p * kBaseFloats + 2 * g + 1] = state[p * kRowFloats + 4 * g + 2];
    }
  for (int scaled = 0; scaled < 2; ++scaled) {
    std::vector<float> buf((size_t)P * 16), merged(state.size()), copy(base.size());
    host_sweep_delta(base.data(), base.data(), st64.data(), attrs.data(), vst.data(), 500.f, scaled,
                     buf.data(), P);
    host_sweep_apply(base.data(), buf.data(), attrs.data(), merged.data(), copy.data(), scaled,
                     vst.data(), 500.f, P);
    for (int64_t p = 0; p < P; ++p)  // the base-row copy is the decoded row's (mu, sigma)
      for (int g = 0; g < kGranules; ++g) {
        CHECK(memcmp(&merged[p * kRowFloats + 4 * g], &copy[p * kBaseFloats + 2 * g], 4) == 0);
        CHECK(memcmp(&merged[p * kRowFloats + 4 * g + 2], &copy[p * kBaseFloats + 2 * g + 1], 4) == 0);
      }
    for (int64_t p = 0; p < P; ++p)
      for (int t = 0; t < kTracks; ++t) {
        const float a = st64[p * kRowFloats + 4 * t], b = merged[p * kRowFloats + 4 * t];
        CHECK(isnan(a) == isnan(b));
        if (!isnan(a)) CHECK(fabs(a - b) < 0.05f + 1e-4f * fabs(a));
      }
  }

  // telemetry
  GenEventParams ge{seed + 2, 0, 12};
  std::vector<int64_t> counts(M), evoff(M + 1, 0);
  host_gen_event_counts(ge, 0, M, counts.data());
  for (int64_t m = 0; m < M; ++m) evoff[m + 1] = evoff[m] + counts[m];
  std::vector<int32_t> events((size_t)evoff[M] * 4 + 4);
  CHECK(host_gen_events(K, ge, 0, rec.data(), evoff.data(), M, events.data()) == 0);
  std::vector<float> stats((size_t)M * S * kStatFeatures);
  TelemetryParams tp{evoff.data(), events.data(), stats.data(), M};
  CHECK(host_telemetry(K, tp) == 0);
  double ev = 0;
  for (int64_t m = 0; m < M; ++m)
    for (int j = 0; j < S; ++j) ev += stats[(m * S + j) * kStatFeatures + kStatEvents];
  CHECK((int64_t)ev == evoff[M]);
}

int main() {
  for (int K = 1; K <= 5; ++K) run(K, 40 + 10 * K, 3000, 100 + K);
  run(3, 7, 2000, 9);  // tiny roster: heavy duplication within matches
  if (fails) {
    fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  printf("host selftest ok\n");
  return 0;
}
