// Host (CPU) mirror of the engine kernels; see host.cpp.
#pragma once

#include <stdint.h>

#include "common.h"
#include "gen_core.h"
#include "telemetry_core.h"

namespace ana {

void host_gen_roster(const GenRosterParams& g, float* state, float* attrs);
int host_gen_stream(int K, const GenStreamParams& g, int32_t* rec, int64_t M);
int host_schedule(int K, const int32_t* rec, int64_t M, int64_t P, uint32_t* link, int32_t* deps);
// K5 levelizer: level[m] = 1 + max level of the previous matches of m's players
// (1 for a player's first match), 0 for matches that touch no state.  Returns
// the number of levels (conflict-free rounds).
// K8 host mirror: generation (counts per match, then events given the CSR
// offsets) and aggregation into stats [M][2K][kStatFeatures].
void host_gen_event_counts(const GenEventParams& g, int64_t base, int64_t M, int64_t* counts);
int host_gen_events(int K, const GenEventParams& g, int64_t base, const int32_t* rec,
                    const int64_t* evoff, int64_t M, int32_t* events);
int64_t host_telemetry(int K, const TelemetryParams& tp);
int64_t host_levels(int K, const int32_t* rec, int64_t M, int64_t P, int32_t* level);
int host_rate(int K, bool fp64, const int32_t* rec, float* state, const float* attrs,
              float* first_prior, const RateOut& out, const RateParams& prm);

}  // namespace ana

namespace ana {
void host_sweep_delta(const float* s0, const float* a, const float* s, const float* attrs,
                      const float* vst, float unknown_sigma, bool scaled, float* buf, int64_t P);
// clamps (nullable): += decoded tracks whose merged precision hit the floor (sweep_core.h)
void host_sweep_apply(const float* s0, const float* buf, const float* attrs, float* s, float* s2,
                      bool scaled, const float* vst, float unknown_sigma, int64_t P, uint32_t* clamps = nullptr);
// causal record correction: rows [M][orow] += delta [P][16] (raw natural-parameter
// increments per track) of each slot's player; the delta table of a scaled prefix
// [P][14] (fp32) against the window start s0 [P][16]
void host_correct_records(int K, const int32_t* rec, int64_t M, float* rows, int64_t orow, const float* delta,
                          int64_t P);
void host_prefix_delta(const float* s0, const float* prefix, const float* attrs, const float* vst,
                       float unknown_sigma, float* delta, int64_t P);
}  // namespace ana
