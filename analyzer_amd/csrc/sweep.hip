// Data-parallel posterior merge (SURVEY K9 + C1; BASELINE config 3 / north star).
//
// Every rank holds the full roster (128 B/player), rates its own shard of the
// window exactly (kernels.hip), then the ranks combine what they learned:
// in natural parameters (pi = 1/sigma^2, tau = mu/sigma^2) a Gaussian posterior
// is prior x likelihood messages, so the per-rank message is
//     delta_g = nat(post_g) - nat(prior_g)
// and the merged posterior is  nat(prior) + sum_g delta_g  -- one dense
// all-reduce (SUM) of a [P][8][2] fp32 buffer over RCCL/xGMI.
//
// Every rank's message is decoded against the SAME base (sweep_core.h
// track_base): the window-start value, or for a track NULL at window start the
// prior the reference would assign (seed / window-start shared).  Causal
// re-sweeps (parallel/sweep.py) re-rate rank r's shard from the start plus the
// messages of ranks < r (an exclusive prefix over ranks); the message is then
// measured from that prior, so the prefix telescopes to rank r-1's posterior.  A track only
// one rank touched therefore merges to exactly that rank's posterior; tracks
// several ranks touched combine as independent evidence (the sweep-mode
// approximation of concurrent shards).  Slot 7 of each player's buffer row
// carries touch counts for NULL-start tracks (base-16 fields, exact in fp32
// for <= 15 ranks) so a track touched on any rank becomes non-NULL everywhere.
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"
#include "rate_core.h"
#include "sweep_core.h"

namespace ana {

// Layout: EIGHT LANES PER PLAYER, lane t = granule t of the 128-B roster row
// (tracks 0..6, granule 7 the spare).  Every access is then a whole-wave run of
// contiguous bytes -- a wave reads 1 KB of roster rows, 512 B of base rows
// (float2 (mu, sigma) per granule, sweep_core.h kBaseFloats) per instruction, and
// writes its players' messages as one 224-B run -- where one thread per player
// touched 64 rows 16 B at a time (8 loads per row, none of them coalesced).  The
// per-track math is sweep_core.h's (the host mirror runs the same functions);
// the shared track's start value and the touch fields cross lanes by shuffles
// within the 8-lane group.  Base rows instead of full start rows: 64 of the 128
// B per player on every start read and write (-26 % merge traffic).
constexpr int kLanesPerPlayer = kGranules;  // 8

// The window-start base rows and the message operands are touched once per merge:
// non-temporal accesses keep them from displacing the roster, which the next rating
// reads from the Infinity Cache.  It pays together with the loads-only non-temporal
// sort of the prepass in the rating's tail (runtime/engine.py sort_nt): eight forced
// merges per step 9.08-9.13 ms with both, 9.32-9.40 with either one or neither
// (profiles/r4/merge_nt_and_sort_nt.log).  ANA_MERGE_NT=0 (build time): plain accesses.
#ifndef ANA_MERGE_NT
#define ANA_MERGE_NT 1
#endif
typedef float merge_f2 __attribute__((ext_vector_type(2)));
typedef int merge_i2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t merge_ld(const uint32_t* p) {
  if constexpr (ANA_MERGE_NT != 0) return __builtin_nontemporal_load(p);
  else return *p;
}
__device__ __forceinline__ float2 merge_ld(const float2* p) {
  if constexpr (ANA_MERGE_NT != 0) {
    const merge_f2 v = __builtin_nontemporal_load(reinterpret_cast<const merge_f2*>(p));
    return make_float2(v.x, v.y);
  } else {
    return *p;
  }
}
__device__ __forceinline__ int2 merge_ld(const int2* p) {
  if constexpr (ANA_MERGE_NT != 0) {
    const merge_i2 v = __builtin_nontemporal_load(reinterpret_cast<const merge_i2*>(p));
    return make_int2(v.x, v.y);
  } else {
    return *p;
  }
}
__device__ __forceinline__ void merge_st(uint32_t* p, uint32_t v) {
  if constexpr (ANA_MERGE_NT != 0) __builtin_nontemporal_store(v, p);
  else *p = v;
}
__device__ __forceinline__ void merge_st(float2* p, float2 v) {
  if constexpr (ANA_MERGE_NT != 0) __builtin_nontemporal_store(merge_f2{v.x, v.y}, reinterpret_cast<merge_f2*>(p));
  else *p = v;
}
__device__ __forceinline__ void merge_st(int2* p, int2 v) {
  if constexpr (ANA_MERGE_NT != 0) __builtin_nontemporal_store(merge_i2{v.x, v.y}, reinterpret_cast<merge_i2*>(p));
  else *p = v;
}
constexpr int kRowVec = kRowFloats / 4;      // 16-B vectors per roster row (C2 exchange below)

struct TrackLane {
  int64_t p;  // player
  int t;      // granule / track
  int gbase;  // first lane of the player's group
};

__device__ __forceinline__ TrackLane track_lane() {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  return TrackLane{gid / kLanesPerPlayer, (int)(gid % kLanesPerPlayer), lane & ~(kLanesPerPlayer - 1)};
}

// += the wave's clamped decodes (sweep_apply_track): one atomic from the first active
// lane, only in the (rare) waves that clamped
__device__ __forceinline__ void count_clamps(bool clamped, uint32_t* clamps) {
  const uint64_t b = __ballot(clamped);
  if (b && clamps && (int)(threadIdx.x & 63) == __builtin_ctzll(__ballot(true)))
    atomicAdd(clamps, (uint32_t)__popcll(b));
}

// sum over the 8 lanes of a player's group (every lane gets it)
__device__ __forceinline__ float group8_sum(float x) {
  x += __shfl_xor(x, 1);
  x += __shfl_xor(x, 2);
  x += __shfl_xor(x, 4);
  return x;
}

__device__ __forceinline__ void lane_seed(const float4* __restrict__ attrs, int64_t p, const float* vst,
                                          float unknown_sigma, bool& seeded, float& seed_mu,
                                          float& seed_sig) {
  const float4 at = attrs[p];  // one 16-B line per group: broadcast
  const float attr[4] = {at.x, at.y, at.z, at.w};
  seed_mu = NAN;
  seed_sig = NAN;
  seeded = seed_prior<float>(attr, unknown_sigma, vst, seed_mu, seed_sig);
}

// this lane's track message (tracks 0..6) and the player's touch fields (lo, hi)
__device__ __forceinline__ void lane_delta(const TrackLane& L, const float2* __restrict__ s0,
                                          const float2* a0, const float4* __restrict__ s,
                                          const float4* __restrict__ attrs, const float* vst,
                                          float unknown_sigma, bool scaled, float& dp, float& dt,
                                          float& lo, float& hi) {
  const float2 c = merge_ld(s0 + L.p * kLanesPerPlayer + L.t);
  const float2 a = a0 != s0 ? a0[L.p * kLanesPerPlayer + L.t] : c;
  const float4 b = s[L.p * kLanesPerPlayer + L.t];
  const float c0mu = __shfl(c.x, L.gbase), c0sg = __shfl(c.y, L.gbase);
  bool seeded;
  float seed_mu, seed_sig;
  lane_seed(attrs, L.p, vst, unknown_sigma, seeded, seed_mu, seed_sig);
  bool touched = false;
  dp = dt = 0.f;
  if (L.t < kTracks)
    sweep_delta_track(L.t, c.x, c.y, c0mu, c0sg, a.x, a.y, b.x, b.z, seeded, seed_mu, seed_sig, scaled,
                      dp, dt, touched);
  const float field = touched ? (float)(1 << (4 * (L.t & 3))) : 0.f;
  lo = group8_sum(L.t < 4 ? field : 0.f);
  hi = group8_sum(L.t >= 4 ? field : 0.f);
}

// decode this lane's track: roster granule {mu, 0, sigma, 0} and base (mu, sigma)
__device__ __forceinline__ void lane_apply(const TrackLane& L, const float2* __restrict__ s0, float dpi,
                                          float dtau, uint32_t lo, uint32_t hi,
                                          const float4* __restrict__ attrs, const float* vst,
                                          float unknown_sigma, bool scaled, float4* s, float2* s2,
                                          uint32_t* clamps) {
  const float2 c = merge_ld(s0 + L.p * kLanesPerPlayer + L.t);
  const float c0mu = __shfl(c.x, L.gbase), c0sg = __shfl(c.y, L.gbase);
  bool seeded;
  float seed_mu, seed_sig;
  lane_seed(attrs, L.p, vst, unknown_sigma, seeded, seed_mu, seed_sig);
  float mu = c.x, sg = c.y;  // granule 7: the spare floats of the base row
  bool clamped = false;
  if (L.t < kTracks) {
    const uint32_t touched = L.t < 4 ? (lo >> (4 * L.t)) & 15u : (hi >> (4 * (L.t - 4))) & 15u;
    sweep_apply_track(L.t, c.x, c.y, c0mu, c0sg, dpi, dtau, touched, seeded, seed_mu, seed_sig, scaled,
                      mu, sg, clamped);
  }
  count_clamps(clamped, clamps);
  s[L.p * kLanesPerPlayer + L.t] = make_float4(mu, 0.f, sg, 0.f);
  if (s2) merge_st(s2 + L.p * kLanesPerPlayer + L.t, make_float2(mu, sg));
}

// s0: base rows of the common window start, a0: this rank's prior of the sweep
// (base rows; may alias s0), s: roster rows after the local window; buf: [P][16]
// fp32 messages = a float2 per lane (lane 7: the touch fields)
__global__ void __launch_bounds__(256)
sweep_delta_kernel(const float2* __restrict__ s0, const float2* a0, const float4* __restrict__ s,
                   const float4* __restrict__ attrs, const float* __restrict__ vst, float unknown_sigma,
                   int scaled, float2* __restrict__ buf, int64_t P) {
  const TrackLane L = track_lane();
  if (L.p >= P) return;  // whole groups leave together (grid = 8 lanes per player)
  float dp, dt, lo, hi;
  lane_delta(L, s0, a0, s, attrs, vst, unknown_sigma, scaled != 0, dp, dt, lo, hi);
  buf[L.p * kLanesPerPlayer + L.t] = L.t < kTracks ? make_float2(dp, dt) : make_float2(lo, hi);
}

// decoded rows go to s and, when given, base rows to s2: the final merge of a
// window writes the next window's common start there (no per-window snapshot
// copy), a causal re-sweep writes the rank's prior for the next message
__global__ void __launch_bounds__(256)
sweep_apply_kernel(const float2* __restrict__ s0, const float2* __restrict__ buf,
                   const float4* __restrict__ attrs, float4* s, float2* s2, const float* __restrict__ vst,
                   float unknown_sigma, int scaled, int64_t P, uint32_t* clamps) {
  const TrackLane L = track_lane();
  if (L.p >= P) return;
  const float2 d = buf[L.p * kLanesPerPlayer + L.t];
  const uint32_t lo = (uint32_t)__shfl(d.x, L.gbase + kTracks), hi = (uint32_t)__shfl(d.y, L.gbase + kTracks);
  lane_apply(L, s0, d.x, d.y, lo, hi, attrs, vst, unknown_sigma, scaled != 0, s, s2, clamps);
}

// ------------------------------------------------- compressed (fp16 / bf16) messages
// COMM_DTYPE=bf16/fp16 merges write / read the all-reduce operands directly:
// msg [P][14] in the 16-bit type (round to nearest even, as torch's .to()) --
// lane t < 7 one 4-B word (its track's two halves) --, cnt [P] int32 (the
// base-16 touch fields, exact integers; lane 7).
// The empty asm pins x as the rounded fp32 message: without it the compiler folds
// the message's last fma into the conversion (v_fma_mixlo_f16, one rounding
// instead of two), which is not what the fp32 path + .to() produce on ties.
template <typename H>
__device__ __forceinline__ uint16_t to_half_bits(float x);
template <>
__device__ __forceinline__ uint16_t to_half_bits<__bf16>(float x) {
  asm("" : "+v"(x));
  return __builtin_bit_cast(uint16_t, (__bf16)x);
}
template <>
__device__ __forceinline__ uint16_t to_half_bits<_Float16>(float x) {
  asm("" : "+v"(x));
  return __builtin_bit_cast(uint16_t, (_Float16)x);
}
template <typename H>
__device__ __forceinline__ float from_half_bits(uint32_t b) {
  return (float)__builtin_bit_cast(H, (uint16_t)b);
}

template <typename H>
__global__ void __launch_bounds__(256)
sweep_delta_packed_kernel(const float2* __restrict__ s0, const float2* a0, const float4* __restrict__ s,
                          const float4* __restrict__ attrs, const float* __restrict__ vst,
                          float unknown_sigma, uint32_t* __restrict__ msg, uint32_t* __restrict__ cnt, int64_t P,
                          int64_t mstride, int64_t cstride) {
  const TrackLane L = track_lane();
  if (L.p >= P) return;
  float dp, dt, lo, hi;
  lane_delta(L, s0, a0, s, attrs, vst, unknown_sigma, true, dp, dt, lo, hi);
  if (L.t < kTracks)  // 14 halves = 7 words (28 B per player, contiguous over the wave)
    merge_st(msg + L.p * mstride + L.t, (uint32_t)to_half_bits<H>(dp) | ((uint32_t)to_half_bits<H>(dt) << 16));
  else
    merge_st(cnt + L.p * cstride, (uint32_t)lo | ((uint32_t)hi << 16));  // 4 + 3 nibbles: 32 B per player on the wire
}

// prefix (nullable, the scaled exclusive prefix of the messages, H [P][14]) -> delta
// [P][8] float2: the raw natural-parameter increments of the causal record correction
// (sweep_core.h prefix_delta_track), computed from the window start before the decode
// overwrites it
template <typename H>
__global__ void __launch_bounds__(256)
sweep_apply_packed_kernel(const float2* __restrict__ s0, const uint32_t* __restrict__ msg,
                          const uint32_t* __restrict__ cnt, const float4* __restrict__ attrs, float4* s,
                          float2* s2, const float* __restrict__ vst, float unknown_sigma, int64_t P,
                          uint32_t* clamps, const uint32_t* __restrict__ pref, float2* __restrict__ delta,
                          int64_t mstride, int64_t cstride) {
  const TrackLane L = track_lane();
  if (L.p >= P) return;
  const uint32_t w = L.t < kTracks ? merge_ld(msg + L.p * mstride + L.t) : 0u;
  const uint32_t c = merge_ld(cnt + L.p * cstride);  // broadcast within the group: lo | hi << 16
  if (pref) {  // (before lane_apply: it may overwrite the window start through s2)
    const float2 cs = merge_ld(s0 + L.p * kLanesPerPlayer + L.t);
    const float c0mu = __shfl(cs.x, L.gbase), c0sg = __shfl(cs.y, L.gbase);
    float dpi = 0.f, dtau = 0.f;
    const uint32_t pw = L.t < kTracks ? merge_ld(pref + L.p * kTracks + L.t) : 0u;
    const float rpi = from_half_bits<H>(pw & 0xffffu), rtau = from_half_bits<H>(pw >> 16);
    if (L.t < kTracks && (rpi != 0.f || rtau != 0.f)) {
      bool seeded = false;
      float seed_mu = NAN, seed_sig = NAN;
      if (!(cs.x == cs.x) || !(c0mu == c0mu)) lane_seed(attrs, L.p, vst, unknown_sigma, seeded, seed_mu, seed_sig);
      prefix_delta_track(L.t, cs.x, cs.y, c0mu, c0sg, seeded, seed_mu, seed_sig, rpi, rtau, dpi, dtau);
    }
    delta[L.p * kLanesPerPlayer + L.t] = make_float2(dpi, dtau);
  }
  lane_apply(L, s0, from_half_bits<H>(w & 0xffffu), from_half_bits<H>(w >> 16), c & 0xffffu, c >> 16, attrs,
             vst, unknown_sigma, true, s, s2, clamps);
}

// the same delta table on its own (simulations, tests): one lane per track
template <typename H>
__global__ void __launch_bounds__(256)
prefix_delta_kernel(const float2* __restrict__ s0, const uint32_t* __restrict__ pref, const float4* __restrict__ attrs,
                    const float* __restrict__ vst, float unknown_sigma, float2* __restrict__ delta, int64_t P) {
  const TrackLane L = track_lane();
  if (L.p >= P) return;
  const float2 cs = s0[L.p * kLanesPerPlayer + L.t];
  const float c0mu = __shfl(cs.x, L.gbase), c0sg = __shfl(cs.y, L.gbase);
  float dpi = 0.f, dtau = 0.f;
  if (L.t < kTracks) {
    const uint32_t pw = pref[L.p * kTracks + L.t];
    bool seeded;
    float seed_mu, seed_sig;
    lane_seed(attrs, L.p, vst, unknown_sigma, seeded, seed_mu, seed_sig);
    prefix_delta_track(L.t, cs.x, cs.y, c0mu, c0sg, seeded, seed_mu, seed_sig, from_half_bits<H>(pw & 0xffffu),
                       from_half_bits<H>(pw >> 16), dpi, dtau);
  }
  delta[L.p * kLanesPerPlayer + L.t] = make_float2(dpi, dtau);
}

// ------------------------------------------------- split collective: the owner's block reduce
// The merge's exchange (parallel/comm.py split_exchange) is all-to-all -> this reduce ->
// all-gather on the critical path, an all-reduce's volume, and -- deferred, beside the
// next window's rating -- an all-to-all that returns each rank its exclusive prefix.
// Rank b owns row block b of the [P][8]-word operand rows (words 0..6: a track's two
// 16-bit message halves, word 7: the touch fields lo | hi << 16) and receives block b of
// every rank: recv [N][blk][8].  One lane per word: the halves are summed in fp32 in rank
// order and rounded once to the wire type (what torch's fp32 cumsum + .to() gives), the
// touch word as an integer (nibble fields, <= 15 ranks: no carries).  pref (nullable)
// [N][blk][7]: rank q's exclusive prefix of the halves (ranks < q; zeros for q = 0), the
// record correction's input -- the touch word has no prefix.
template <typename H>
__global__ void __launch_bounds__(256)
sweep_block_reduce_kernel(const uint32_t* __restrict__ recv, int N, int64_t blk, uint32_t* __restrict__ total,
                          uint32_t* __restrict__ pref) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = gid >> 3;
  const int w = (int)(gid & 7);
  if (row >= blk) return;
  if (w == kTracks) {
    uint32_t c = 0u;
    for (int q = 0; q < N; ++q) c += merge_ld(recv + ((int64_t)q * blk + row) * 8 + w);
    merge_st(total + row * 8 + w, c);
    return;
  }
  float a = 0.f, b = 0.f;
  for (int q = 0; q < N; ++q) {
    if (pref)  // the prefix of rank q: the sum so far, rounded once
      merge_st(pref + ((int64_t)q * blk + row) * kTracks + w,
               (uint32_t)to_half_bits<H>(a) | ((uint32_t)to_half_bits<H>(b) << 16));
    const uint32_t x = merge_ld(recv + ((int64_t)q * blk + row) * 8 + w);
    a += from_half_bits<H>(x & 0xffffu);
    b += from_half_bits<H>(x >> 16);
  }
  merge_st(total + row * 8 + w, (uint32_t)to_half_bits<H>(a) | ((uint32_t)to_half_bits<H>(b) << 16));
}

int launch_sweep_block_reduce(const int32_t* recv, int N, int64_t blk, int bf16, int32_t* total, int32_t* pref,
                              hipStream_t st) {
  if (blk <= 0 || N <= 0) return 0;
  const dim3 grid((unsigned)((blk * 8 + 255) / 256));
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, reinterpret_cast<const uint32_t*>(recv), N, blk,
                       reinterpret_cast<uint32_t*>(total), reinterpret_cast<uint32_t*>(pref));
  };
  if (bf16) args(sweep_block_reduce_kernel<__bf16>);
  else args(sweep_block_reduce_kernel<_Float16>);
  return (int)hipGetLastError();
}

// ------------------------------------------------- causal record correction
// A block corrects a tile of kCorrTile consecutive matches.  Their output rows are one
// contiguous span (tile * orow floats): it is copied into LDS with fully coalesced
// 16-B loads (a wave covers 1 KB per instruction), each thread then corrects its own
// match's row in LDS -- status check, 2K independent 16-B delta-table reads of its
// players ([P][8] float2: the shared and the mode pair of a slot share one 64-B line),
// the 4K fields rewritten -- and the span goes back with coalesced 16-B stores.  LDS
// rows are padded to orow + 1 words so the per-thread field accesses (stride orow + 1)
// hit distinct banks.  One thread per match reading its own 128-B row (8 16-B loads at
// a 128-B lane stride) ran at 1.6 TB/s, 0.29 ms per 1.25M-match window
// (profiles/r5/correct_micro.log); one thread per slot 0.23 ms in the step.
constexpr int kCorrTile = 256;

template <int K>
__global__ void __launch_bounds__(kCorrTile)
correct_records_kernel(const int32_t* __restrict__ rec, int64_t M, float* rows, int64_t orow,
                       const float2* __restrict__ delta, int64_t P) {
  constexpr int S = 2 * K;
  typedef float v4f __attribute__((ext_vector_type(4)));
  extern __shared__ float tile[];  // [blockDim.x][orow + 1]
  const int T = (int)blockDim.x;    // matches per tile (kCorrTile, or half of it for wide rows)
  const int ld = (int)orow + 1;
  const int64_t m0 = (int64_t)blockIdx.x * T;
  const int n = (int)(M - m0 < T ? M - m0 : T);
  const int rq = (int)(orow >> 2);  // 16-B quads per row
  const int nq = n * rq;
  const v4f* src = reinterpret_cast<const v4f*>(rows + m0 * orow);
  for (int q = threadIdx.x; q < nq; q += T) {
    const v4f v = __builtin_nontemporal_load(src + q);
    float* d = tile + (q / rq) * ld + (q % rq) * 4;
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  }
  __syncthreads();
  const int i = threadIdx.x;
  float* f = tile + i * ld;
  if (i < n && (__float_as_uint(f[5 * S + 1]) & 0xffu) == kRated) {
    const int32_t* r = rec + (m0 + i) * (S + 2);
    int32_t ids[S];
#pragma unroll
    for (int j = 0; j < S; ++j) ids[j] = r[j];
    const uint32_t mm = (uint32_t)r[S];
    const int t = 1 + meta_mode(mm);
    const int n0 = meta_n0(mm), n1 = meta_n1(mm);
    float2 ds[S], dm[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const bool in = (j < K ? j : j - K) < (j < K ? n0 : n1) && ids[j] >= 0 && ids[j] < P;
      const int64_t base = (int64_t)(in ? ids[j] : 0) * kGranules;
      ds[j] = in ? delta[base] : make_float2(0.f, 0.f);
      dm[j] = in ? delta[base + t] : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < S; ++j) {
      correct_record_track(ds[j].x, ds[j].y, f[j], f[S + j]);
      correct_record_track(dm[j].x, dm[j].y, f[3 * S + j], f[4 * S + j]);
    }
  }
  __syncthreads();
  v4f* dst = reinterpret_cast<v4f*>(rows + m0 * orow);
  for (int q = threadIdx.x; q < nq; q += T) {
    const float* d = tile + (q / rq) * ld + (q % rq) * 4;
    __builtin_nontemporal_store(v4f{d[0], d[1], d[2], d[3]}, dst + q);
  }
}

int launch_correct_records(int K, const int32_t* rec, int64_t M, float* rows, int64_t orow, const float* delta,
                           int64_t P, hipStream_t st) {
  if (M <= 0) return 0;
  if (orow % 4 != 0 || orow < 5 * 2 * K + 2) return (int)hipErrorInvalidValue;  // RateResult.allocate rows
  int T = kCorrTile;
  while (T > 64 && (size_t)T * (size_t)(orow + 1) * sizeof(float) > 64 * 1024) T /= 2;
  const size_t lds = (size_t)T * (size_t)(orow + 1) * sizeof(float);
  if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)((M + T - 1) / T));
  const float2* d = reinterpret_cast<const float2*>(delta);
  const dim3 blk(T);
  switch (K) {
    case 1: hipLaunchKernelGGL(correct_records_kernel<1>, grid, blk, lds, st, rec, M, rows, orow, d, P); break;
    case 2: hipLaunchKernelGGL(correct_records_kernel<2>, grid, blk, lds, st, rec, M, rows, orow, d, P); break;
    case 3: hipLaunchKernelGGL(correct_records_kernel<3>, grid, blk, lds, st, rec, M, rows, orow, d, P); break;
    case 4: hipLaunchKernelGGL(correct_records_kernel<4>, grid, blk, lds, st, rec, M, rows, orow, d, P); break;
    case 5: hipLaunchKernelGGL(correct_records_kernel<5>, grid, blk, lds, st, rec, M, rows, orow, d, P); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

static dim3 track_grid(int64_t P) {
  return dim3((unsigned)((P * kLanesPerPlayer + 255) / 256));
}

int launch_sweep_delta_packed(const float* s0, const float* a, const float* s, const float* attrs,
                              const float* vst, float unknown_sigma, int bf16, void* msg, int32_t* cnt,
                              int64_t P, hipStream_t st, int64_t mstride, int64_t cstride) {
  if (P <= 0) return 0;
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, track_grid(P), dim3(256), 0, st, reinterpret_cast<const float2*>(s0),
                       reinterpret_cast<const float2*>(a), reinterpret_cast<const float4*>(s),
                       reinterpret_cast<const float4*>(attrs), vst, unknown_sigma,
                       reinterpret_cast<uint32_t*>(msg), reinterpret_cast<uint32_t*>(cnt), P, mstride, cstride);
  };
  if (bf16) args(sweep_delta_packed_kernel<__bf16>);
  else args(sweep_delta_packed_kernel<_Float16>);
  return (int)hipGetLastError();
}

int launch_sweep_apply_packed(const float* s0, const void* msg, const int32_t* cnt, int bf16,
                              const float* attrs, float* s, float* s2, const float* vst, float unknown_sigma,
                              int64_t P, uint32_t* clamps, const void* prefix, float* delta, hipStream_t st,
                              int64_t mstride, int64_t cstride) {
  if (P <= 0) return 0;
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, track_grid(P), dim3(256), 0, st, reinterpret_cast<const float2*>(s0),
                       reinterpret_cast<const uint32_t*>(msg), reinterpret_cast<const uint32_t*>(cnt),
                       reinterpret_cast<const float4*>(attrs), reinterpret_cast<float4*>(s),
                       reinterpret_cast<float2*>(s2), vst, unknown_sigma, P, clamps,
                       reinterpret_cast<const uint32_t*>(prefix), reinterpret_cast<float2*>(delta), mstride, cstride);
  };
  if (bf16) args(sweep_apply_packed_kernel<__bf16>);
  else args(sweep_apply_packed_kernel<_Float16>);
  return (int)hipGetLastError();
}

int launch_prefix_delta(const float* s0, const void* prefix, int bf16, const float* attrs, const float* vst,
                        float unknown_sigma, float* delta, int64_t P, hipStream_t st) {
  if (P <= 0) return 0;
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, track_grid(P), dim3(256), 0, st, reinterpret_cast<const float2*>(s0),
                       reinterpret_cast<const uint32_t*>(prefix), reinterpret_cast<const float4*>(attrs), vst,
                       unknown_sigma, reinterpret_cast<float2*>(delta), P);
  };
  if (bf16) args(prefix_delta_kernel<__bf16>);
  else args(prefix_delta_kernel<_Float16>);
  return (int)hipGetLastError();
}

int launch_sweep_delta(const float* s0, const float* a, const float* s, const float* attrs,
                       const float* vst, float unknown_sigma, int scaled, float* buf, int64_t P,
                       hipStream_t st) {
  if (P <= 0) return 0;
  hipLaunchKernelGGL(sweep_delta_kernel, track_grid(P), dim3(256), 0, st,
                     reinterpret_cast<const float2*>(s0), reinterpret_cast<const float2*>(a),
                     reinterpret_cast<const float4*>(s), reinterpret_cast<const float4*>(attrs), vst,
                     unknown_sigma, scaled, reinterpret_cast<float2*>(buf), P);
  return (int)hipGetLastError();
}

int launch_sweep_apply(const float* s0, const float* buf, const float* attrs, float* s, float* s2,
                       const float* vst, float unknown_sigma, int scaled, int64_t P, uint32_t* clamps,
                       hipStream_t st) {
  if (P <= 0) return 0;
  hipLaunchKernelGGL(sweep_apply_kernel, track_grid(P), dim3(256), 0, st,
                     reinterpret_cast<const float2*>(s0), reinterpret_cast<const float2*>(buf),
                     reinterpret_cast<const float4*>(attrs), reinterpret_cast<float4*>(s),
                     reinterpret_cast<float2*>(s2), vst, unknown_sigma, scaled, P, clamps);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------ C2 exact DP exchange
// One round of exact DP (parallel/exact_dp.py): every rank rated a disjoint
// slice of a conflict-free round, so each player changed on at most one rank.
// pack: one 33-float entry per slot of the slice -- the player's 128-B row,
// then its id (as float bits; -1 = no entry: unrated match or empty slot);
// entries past the slice are -1, so the buffer has the fixed capacity the
// all-gather needs and nothing is counted on the host.
__global__ void pack_rows_kernel(const int32_t* __restrict__ rec, int S, int64_t m,
                                 const uint8_t* __restrict__ status, int64_t sstride,
                                 const float4* __restrict__ state, float* __restrict__ out,
                                 int64_t cap) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= cap) return;
  const int K = S / 2;
  int32_t id = -1;
  if (e < m * S) {
    const int64_t i = e / S;
    const int j = (int)(e % S);
    const int32_t* r = rec + i * (S + 2);
    const uint32_t m0 = (uint32_t)r[S];
    const int n = j < K ? (int)meta_n0(m0) : (int)meta_n1(m0);
    if (status[i * sstride] == kRated && (j < K ? j : j - K) < n) id = r[j];
  }
  float* o = out + e * 33;
  if (id >= 0) {
#pragma unroll
    for (int k = 0; k < kRowVec; ++k) {
      const float4 v = state[(int64_t)id * kRowVec + k];
      o[4 * k] = v.x; o[4 * k + 1] = v.y; o[4 * k + 2] = v.z; o[4 * k + 3] = v.w;
    }
  }
  o[32] = __int_as_float(id);
}

// unpack: write every entry with an id into the roster; tag words are zeroed
// (they belong to another rank's launch epochs)
__global__ void unpack_rows_kernel(const float* __restrict__ buf, int64_t n, float* __restrict__ state) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const float* b = buf + e * 33;
  const int32_t id = __float_as_int(b[32]);
  if (id < 0) return;
#pragma unroll
  for (int k = 0; k < kRowFloats; ++k) state[(int64_t)id * kRowFloats + k] = (k & 1) ? 0.f : b[k];
}

// Race detector for exact DP: the matches of one round must share no
// player.  owner[p] holds (round + 1) << 32 | (match + 1) of the last claim; a
// slot whose player was claimed in the SAME round by ANOTHER match sets *flag.
// Rounds only grow, so the table never needs clearing between rounds.
__global__ void check_round_kernel(const int32_t* __restrict__ rec, int S, const int64_t* __restrict__ idx,
                                   int64_t m, int64_t P, uint32_t round,
                                   unsigned long long* __restrict__ owner, uint32_t* __restrict__ flag) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= m * S) return;
  const int K = S / 2;
  const int64_t i = e / S;
  const int j = (int)(e % S);
  const int64_t mi = idx[i];
  const int32_t* r = rec + mi * (S + 2);
  const uint32_t m0 = (uint32_t)r[S];
  const int n = j < K ? (int)meta_n0(m0) : (int)meta_n1(m0);
  const int32_t p = r[j];
  if (early_status_k(r, S, P) != kRated || (j < K ? j : j - K) >= n || p < 0 || p >= P) return;
  const unsigned long long mine = ((unsigned long long)(round + 1u) << 32) | (unsigned long long)(mi + 1);
  unsigned long long cur = owner[p];
  for (;;) {
    if ((uint32_t)(cur >> 32) == round + 1u) {  // claimed this round
      if (cur != mine) atomicOr(flag, 1u);
      return;
    }
    const unsigned long long prev = atomicCAS(owner + p, cur, mine);
    if (prev == cur) return;
    cur = prev;
  }
}

int launch_check_round(const int32_t* rec, int K, const int64_t* idx, int64_t m, int64_t P, uint32_t round,
                       unsigned long long* owner, uint32_t* flag, hipStream_t st) {
  if (m <= 0) return 0;
  const int64_t n = m * 2 * K;
  hipLaunchKernelGGL(check_round_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, rec, 2 * K, idx,
                     m, P, round, owner, flag);
  return (int)hipGetLastError();
}

int launch_pack_rows(const int32_t* rec, int K, int64_t m, const uint8_t* status, int64_t sstride,
                     const float* state, float* out, int64_t cap, hipStream_t st) {
  if (cap <= 0) return 0;
  hipLaunchKernelGGL(pack_rows_kernel, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, st, rec, 2 * K,
                     m, status, sstride, reinterpret_cast<const float4*>(state), out, cap);
  return (int)hipGetLastError();
}

int launch_unpack_rows(const float* buf, int64_t n, float* state, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(unpack_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, buf, n,
                     state);
  return (int)hipGetLastError();
}

}  // namespace ana
