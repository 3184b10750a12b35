// Host-callable launchers of the MI355X kernels (implemented in kernels.hip).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime_api.h>

#include "common.h"
#include "gen_core.h"
#include "telemetry_core.h"

namespace ana {

int launch_gen_roster(const GenRosterParams& g, float* state, float* attrs, hipStream_t s);
int launch_gen_stream(int K, const GenStreamParams& g, int32_t* rec, int64_t M, hipStream_t s);

int launch_reset_tags(float* state, int64_t P, hipStream_t s);
// read every roster row once (Infinity Cache warm-up in front of a rating launch);
// sink: >= 256 words, written only under a condition that is never true in practice
int launch_warm_rows(const float* state, int64_t P, uint32_t* sink, hipStream_t s);
// e[0] += 1 on the stream (the device epoch of graph replays, RateParams::epoch_ptr)
int launch_epoch_bump(int32_t* e, hipStream_t s);
// DP pricing on one GPU: an all-reduce stand-in over `bytes` of `buf` (unchanged) on
// `channels` workgroups, `passes` streams of the buffer, held at least `us` microseconds
int launch_emulate_allreduce(void* buf, int64_t bytes, int channels, int passes, double us, hipStream_t s);

size_t schedule_workspace_bytes(int64_t nslots, int64_t num_players);

// Deterministic per-window digest of the packed output rows [M, W] (digest.hip):
// out[3 + 10K] fp64 = matches with records, participant records, the NaN-skipping
// column sums of s_mu / s_sig / delta / m_mu / m_sig per slot, the quality sum.
// scratch: records_digest_scratch_doubles(K) doubles.  hist (nullable) int64[256]:
// the window's status counts are ADDED to it (the run's running status histogram).
size_t records_digest_scratch_doubles(int K);
int launch_records_digest(int K, const float* rows, int64_t M, int64_t W, double* scratch, double* out,
                          int64_t* hist, hipStream_t s);

// Stable LSD radix sort of (key, value) pairs on the low ``bits`` key bits
// (radix_sort.hip).  Ping-pongs between the two buffer pairs; *result_in_alt
// says which holds the result.  ws: radix_sort_workspace_bytes(n) bytes.
size_t radix_sort_workspace_bytes(int64_t n);
int launch_radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt,
                            int64_t n, int bits, void* ws, int* result_in_alt, hipStream_t s);
// The schedule's sort (radix_sort.hip): link[slot] for every slot of a
// stateful match (next match of its player | kLinkHasPred), from a stable sort
// of the stream's slots by player fused with the record decode and the links.
// ws: radix_sort_workspace_bytes(M * 2K) bytes; ka..vb: M * 2K words each.
// deps [M] (zeroed by the first kernel), ctrl[0..nz) (zeroed), epoch_bump (+1): the
// schedule's fill work, folded into that kernel (null / 0: skipped)
int launch_sched_sort(int K, const int32_t* rec, int64_t M, uint32_t num_players, uint32_t* ka,
                      uint32_t* va, uint32_t* kb, uint32_t* vb, void* ws, uint32_t* link,
                      hipStream_t s, int32_t* deps = nullptr, uint32_t* ctrl = nullptr, int nz = 0,
                      int32_t* epoch_bump = nullptr, int sort_nt = -1);
// Device levelizer (levels.hip): level[m] = 0 for a match without state, else
// 1 + the largest level of its players' previous matches -- the exact-DP rounds --
// as a dataflow over a fresh schedule (link, deps zeroed; deps are consumed).
// pushed: int32 [M] zeroed scratch; ctrl: uint32 [4] zeroed ([2] depth, [3] error).
int launch_levels(int K, const int32_t* rec, const uint32_t* link, int32_t* deps, int32_t* pushed,
                  int32_t* level, int64_t M, int64_t P, uint32_t* ctrl, hipStream_t s);
// link: uint32 [M][2K] = next match of the player (kNoMatch: none) | kLinkHasPred
//       if the player has an earlier occurrence in the window
// deps: int32 [M] zeroed: the completion counters the executor counts up (a
//       match is ready when its counter reaches the number of its players with
//       kLinkHasPred, which the executor reads from the links)
// overflow: zeroed (reserved for schedule error reporting)
int launch_schedule(int K, const int32_t* rec, int64_t M, int64_t P, uint32_t* link,
                    int32_t* deps, void* ws, size_t ws_bytes, uint32_t* overflow, hipStream_t s,
                    bool zero_ctrl = false, int32_t* epoch_bump = nullptr, int sort_nt = -1);

// out must be the packed layout (one row per match: [s_mu | s_sig | delta |
// m_mu | m_sig][2K], quality, status byte), else hipErrorInvalidValue.
// tp.evoff == nullptr: no telemetry; otherwise idle waves aggregate telemetry
// tiles (K8 fused streaming mode).  ctrl[12] = telemetry tile ticket,
// ctrl[13] = malformed events.
int launch_rate(int K, const int32_t* rec, const uint32_t* link, int32_t* deps, float* state,
                const float* attrs, float* first_prior, const RateOut& out, uint32_t* ctrl,
                const RateParams& prm, const TelemetryParams& tp, int blocks, hipStream_t s);


// K8 (telemetry.hip)
int launch_gen_event_counts(const GenEventParams& g, int64_t base, int64_t M, int64_t* counts,
                            hipStream_t s);
int launch_gen_events(int K, const GenEventParams& g, int64_t base, const int32_t* rec,
                      const int64_t* evoff, int64_t M, int32_t* events, hipStream_t s);
// K8 implementation: 1 = one-hot MFMA (default), 0 = LDS float atomics (ANA_TELE_IMPL)
int tele_impl();
int launch_telemetry(int K, const TelemetryParams& tp, uint32_t* bad, hipStream_t s);

}  // namespace ana

namespace ana {
// s0: common window start, a: the rank's prior of this sweep (may be s0), s: posterior
int launch_sweep_delta(const float* s0, const float* a, const float* s, const float* attrs,
                       const float* vst, float unknown_sigma, int scaled, float* buf, int64_t P,
                       hipStream_t st);
// decoded rows to s and (s2 != nullptr) s2; clamps (nullable): += decoded tracks whose
// merged precision hit the floor (sweep_core.h sweep_apply_track), here and below
int launch_sweep_apply(const float* s0, const float* buf, const float* attrs, float* s, float* s2,
                       const float* vst, float unknown_sigma, int scaled, int64_t P, uint32_t* clamps,
                       hipStream_t st);
// compressed merges: msg [P][14] bf16 (bf16 != 0) or fp16 + cnt [P] int32 (touch fields lo | hi << 16);
// mstride / cstride: row strides in 32-bit words (7 / 1 for separate tensors, 8 / 8 for the
// split collective's [P][8]-word operand rows with the touch word last)
int launch_sweep_delta_packed(const float* s0, const float* a, const float* s, const float* attrs,
                              const float* vst, float unknown_sigma, int bf16, void* msg, int32_t* cnt,
                              int64_t P, hipStream_t st, int64_t mstride = 7, int64_t cstride = 1);
// split collective (parallel/comm.py): recv [N][blk][8] words -> total [blk][8] (+ the exclusive
// prefixes pref [N][blk][7] when non-null)
int launch_sweep_block_reduce(const int32_t* recv, int N, int64_t blk, int bf16, int32_t* total, int32_t* pref,
                              hipStream_t st);
// prefix (nullable): the scaled exclusive prefix of the messages (same type as msg) ->
// delta [P][16] fp32, the record correction's increments (sweep_core.h prefix_delta_track)
int launch_sweep_apply_packed(const float* s0, const void* msg, const int32_t* cnt, int bf16,
                              const float* attrs, float* s, float* s2, const float* vst, float unknown_sigma,
                              int64_t P, uint32_t* clamps, const void* prefix, float* delta, hipStream_t st,
                              int64_t mstride = 7, int64_t cstride = 1);
int launch_prefix_delta(const float* s0, const void* prefix, int bf16, const float* attrs, const float* vst,
                        float unknown_sigma, float* delta, int64_t P, hipStream_t st);
// causal record correction: rows = RateResult's packed rows [M][orow] += delta [P][16]
// fp32 (raw natural-parameter increments per track) of each slot's player
int launch_correct_records(int K, const int32_t* rec, int64_t M, float* rows, int64_t orow, const float* delta,
                           int64_t P, hipStream_t st);
// C2 exact-DP exchange (sweep.hip): fixed-capacity [cap][33] entries of changed rows
int launch_pack_rows(const int32_t* rec, int K, int64_t m, const uint8_t* status, int64_t sstride,
                     const float* state, float* out, int64_t cap, hipStream_t st);
int launch_unpack_rows(const float* buf, int64_t n, float* state, hipStream_t st);
// exact-DP race detector: matches idx[0..m) of round ``round`` share no player
// (owner: P 64-bit claims, zeroed once; *flag |= 1 on a conflict)
int launch_check_round(const int32_t* rec, int K, const int64_t* idx, int64_t m, int64_t P, uint32_t round,
                       unsigned long long* owner, uint32_t* flag, hipStream_t st);
}  // namespace ana
