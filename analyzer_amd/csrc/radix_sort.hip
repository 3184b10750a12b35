// K5 building block: stable LSD radix sort of (u32 key, u32 value) pairs for
// gfx950, written to CO-RUN with the persistent dataflow executor.
//
// hipCUB's onesweep sort chains its tiles through a decoupled look-back: tile
// t spins until tile t-1 has published its prefix.  Next to the rating
// kernel (which keeps the memory system busy with latency-bound sc1 traffic)
// every link of that chain waits microseconds and one 60M-slot pass stretches
// from 0.4 ms to 9.5 ms (rocprofv3 trace, profiles/).  This sort is
// reduce-then-scan instead: every pass is three launches whose workgroups
// never wait on each other --
//   upsweep   per-tile digit histograms (LDS atomics, one row per digit),
//   rowscan   one workgroup per digit: exclusive scan of its row over tiles,
//   downsweep per tile: stable rank in wave order (8 ballots -> peer mask),
//             wave prefixes in LDS, local scatter into an LDS-sorted tile,
//             then coalesced runs to the global digit offsets.
// 8192-element tiles (512 threads x 16: the per-(tile, digit) runs the downsweeps write
// average 32 elements, whole 128-B lines; 4096-element tiles measured 0.03-0.04 ms slower
// per 10M 3v3 prepass, profiles/r3/sort_tile_8192.log); 8-bit digits (10-bit ones for the
// schedule are an opt-in experiment, ANA_SORT_RB: fewer passes but measured slower).
//
// The schedule prepass (launch_sched_sort) fuses both ends: pass 0 computes its
// keys from the match records, and the last pass writes each slot's link from
// its LDS neighbours instead of the sorted pairs (only run-boundary pairs go out,
// for the fix-up).  For 10M 3v3 matches that drops a 480-MB key/value write, the
// re-reads of it and a separate 720-MB link pass.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace ana {

namespace {

#ifndef ANA_SORT_THREADS
#define ANA_SORT_THREADS 512  // threads per tile (x 16 items = 8192 elements; 256: 4096, A/B)
#endif
constexpr int kThreads = ANA_SORT_THREADS;
constexpr int kWaves = kThreads / 64;
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;
constexpr int kRadix = 256;      // 8-bit digits (generic sort; schedule keys > 20 bits)
constexpr int kRadixMax = 1024;  // 10-bit digits: the schedule of <= 2^20 players in 2 passes

// Tile of this workgroup.  Workgroups go round-robin over the 8 XCDs; giving
// each XCD a contiguous range of tiles puts the digit runs that consecutive
// tiles write next to each other into one L2, which merges them into full
// lines before they leave for HBM.
__device__ __forceinline__ int64_t xcd_tile(int64_t tiles) {
  const int64_t i = blockIdx.x, q = tiles >> 3, r = tiles & 7, x = i & 7;
  return x * q + (x < r ? x : r) + (i >> 3);
}

// NT: streaming (non-temporal) accesses for the sort's key/value/link traffic, so
// a prepass that co-runs with the dataflow executor does not evict the roster
// the executor keeps in the Infinity Cache.  Opt-in (ANA_SORT_NT=1): measured on
// MI355X the prepass slows 1.75 -> 4.35 ms (the digit runs lose L2 write
// combining) and the bench step 8.1 -> 9.2 ms.  ANA_SORT_NT=2: non-temporal loads
// only (each pass streams its input once; the scattered stores keep L2 combining).
template <int NT>
__device__ __forceinline__ uint32_t ld32(const uint32_t* p) {
  if constexpr (NT >= 1) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int NT>
__device__ __forceinline__ void st32(uint32_t* p, uint32_t v) {
  if constexpr (NT == 1) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// exclusive scan of one value per thread over a 256-thread block
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t x, uint32_t* wsum,
                                                         uint32_t* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t inc = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(inc, off);
    if (lane >= off) inc += y;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) {
    if (w < wv) before += wsum[w];
    all += wsum[w];
  }
  if (total) *total = all;
  __syncthreads();  // wsum may be reused by the caller
  return before + inc - x;
}

// The schedule's first pass sorts the slots of the match stream straight from
// the records: key = the slot's player (kend if the match touches no state or
// the slot is empty), value = the slot index.  A workgroup decodes each match
// of its tile once (one thread per match, one 16-B-vector record load) into an
// LDS key array, instead of every slot re-decoding its whole match.
template <int KS>
__device__ __forceinline__ void decode_tile_keys(const int32_t* __restrict__ rec, uint32_t kend,
                                                 int64_t base, int64_t n, uint32_t* lk) {
  constexpr int S = 2 * KS, R = S + 2;
  const uint32_t lo = (uint32_t)base;  // slots < kMaxSlots
  const uint32_t hi = (uint32_t)(base + kTile < n ? base + kTile : n);
  const uint32_t m_lo = lo / S, m_hi = (hi + S - 1) / S;
  for (uint32_t m = m_lo + threadIdx.x; m < m_hi; m += kThreads) {
    const int32_t* src = rec + (int64_t)m * R;
    int32_t r[R];
    if constexpr (R % 4 == 0) {
#pragma unroll
      for (int k = 0; k < R / 4; ++k) {
        const int4 v = reinterpret_cast<const int4*>(src)[k];
        r[4 * k] = v.x; r[4 * k + 1] = v.y; r[4 * k + 2] = v.z; r[4 * k + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < R; ++k) r[k] = src[k];
    }
    const bool rates = early_status<KS>(r, (int64_t)kend) == kRated;
    const uint32_t m0 = (uint32_t)r[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const uint32_t slot = m * S + j;
      const int pos = j < KS ? j : j - KS;
      const bool in_roster = pos < (j < KS ? meta_n0(m0) : meta_n1(m0));
      if (slot >= lo && slot < hi) lk[slot - lo] = rates && in_roster ? (uint32_t)r[j] : kend;
    }
  }
}

// What the schedule's first kernel also does, so the prepass needs no fill
// dispatches of its own: zero the window's completion counters (each tile its
// matches), the control words, and bump the device launch epoch (graph replays).
struct SchedInit {
  int32_t* deps = nullptr;       // [M] completion counters
  uint32_t* ctrl = nullptr;      // ctrl[0..nz) zeroed by block 0
  int nz = 0;
  int32_t* epoch_bump = nullptr; // += 1 by block 0
};

// KS > 0: keys from the match stream (decode_tile_keys), and the SchedInit duties.
template <int KS, int RB = 8, int NT = 0>
__global__ void __launch_bounds__(kThreads)
radix_upsweep(const uint32_t* __restrict__ keys, const int32_t* __restrict__ rec, uint32_t kend,
              int64_t n, int shift, uint32_t* __restrict__ counts, int64_t tiles, SchedInit init = {}) {
  constexpr int kR = 1 << RB;
  __shared__ uint32_t hist[kWaves][kR];
  __shared__ uint32_t lkeys[KS > 0 ? kTile : 1];
  const int tid = threadIdx.x, wv = tid >> 6;
  for (int i = tid; i < kWaves * kR; i += kThreads) (&hist[0][0])[i] = 0u;
  const int64_t tile = xcd_tile(tiles);
  const int64_t base = tile * kTile;
  if constexpr (KS > 0) {
    if (init.deps) {  // the matches whose slots start in this tile (every match has its first slot in one)
      constexpr int S = 2 * KS;
      const int64_t hi = base + kTile < n ? base + kTile : n;
      for (int64_t m = (base + S - 1) / S + tid; m < (hi + S - 1) / S; m += kThreads) init.deps[m] = 0;
    }
    if (blockIdx.x == 0) {
      if (tid < init.nz) init.ctrl[tid] = 0u;
      if (tid == 0 && init.epoch_bump) init.epoch_bump[0] += 1;
    }
  }
  if constexpr (KS > 0) decode_tile_keys<KS>(rec, kend, base, n, lkeys);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const int64_t idx = base + k * kThreads + tid;
    if (idx < n) {
      const uint32_t key = KS > 0 ? lkeys[k * kThreads + tid] : ld32<NT>(keys + idx);
      atomicAdd(&hist[wv][(key >> shift) & (kR - 1)], 1u);
    }
  }
  __syncthreads();
#pragma unroll
  for (int d = tid; d < kR; d += kThreads) {
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) c += hist[w][d];
    counts[(int64_t)d * tiles + tile] = c;
  }
}

// exclusive scan over kR per-digit values held as DPT = kR / kThreads consecutive
// digits per thread (v[] in, prefixes out); *total = the sum of all
template <int DPT>
__device__ __forceinline__ void digits_exclusive_scan(uint32_t (&v)[DPT], uint32_t* wsum,
                                                      uint32_t* total) {
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const uint32_t x = v[j];
    v[j] = s;
    s += x;
  }
  const uint32_t before = block_exclusive_scan(s, wsum, total);
#pragma unroll
  for (int j = 0; j < DPT; ++j) v[j] += before;
}

// One workgroup per digit: counts[d][*] <- exclusive prefix over tiles; totals[d] <- row sum.
__global__ void __launch_bounds__(kThreads)
radix_rowscan(uint32_t* __restrict__ counts, int64_t tiles, uint32_t* __restrict__ totals) {
  __shared__ uint32_t wsum[kWaves];
  constexpr int kPer = 4;
  uint32_t* row = counts + (int64_t)blockIdx.x * tiles;
  uint32_t carry = 0;
  for (int64_t start = 0; start < tiles; start += kThreads * kPer) {
    uint32_t v[kPer], s = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int64_t t = start + (int64_t)threadIdx.x * kPer + q;
      v[q] = t < tiles ? row[t] : 0u;
      s += v[q];
    }
    uint32_t all;
    uint32_t ex = carry + block_exclusive_scan(s, wsum, &all);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int64_t t = start + (int64_t)threadIdx.x * kPer + q;
      if (t < tiles) row[t] = ex;
      ex += v[q];
    }
    carry += all;
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// The two ends of one (tile, digit) run of the schedule's last pass (first and last
// key / value; kf = kRunEmpty: the tile has no element of that digit).
struct RunEnds {
  uint32_t kf, vf, kl, vl;
};
constexpr uint32_t kRunEmpty = 0xffffffffu;

// KS > 0: elements come from the match stream (decode_tile_keys).  LINK (the schedule's
// last pass): instead of writing the sorted pairs, write every slot's link from
// its neighbours in the LDS-sorted tile -- within a (tile, digit) run they are
// its global neighbours -- and only the run-boundary pairs, whose outer
// neighbour lives in another tile (sched_fixup completes those links).
// bnd (LINK, last pass with nd <= kRunsMaxDigits digits): the boundary pairs go to a
// [tile][nd] RunEnds table instead of their global sorted positions, so this pass
// needs no digit offsets -- no upsweep / rowscan in front of it -- and sched_runs_fixup
// links each run to the nearest non-empty run of its digit in an earlier tile.
template <int KS, bool LINK, int RB = 8, int NT = 0>
__global__ void __launch_bounds__(kThreads)
radix_downsweep(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                const int32_t* __restrict__ rec, uint32_t kend,
                uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, int64_t n, int shift,
                const uint32_t* __restrict__ counts, const uint32_t* __restrict__ totals,
                int64_t tiles, int slots_per_match, uint32_t* __restrict__ link,
                uint32_t vlo = 0u, uint32_t vhi = 0xffffffffu, int bounds = 1,
                RunEnds* __restrict__ bnd = nullptr, int nd = 0) {
  constexpr int kR = 1 << RB;
  constexpr int DPT = kR >= kThreads ? kR / kThreads : 1;  // digits per thread in the scans
  static_assert(kR % kThreads == 0 || kThreads % kR == 0, "radix and block must divide");
  __shared__ uint32_t skey[kTile];
  __shared__ uint32_t sval[kTile];
  __shared__ uint32_t wcnt[kWaves][kR];
  __shared__ uint32_t tstart[kR];
  __shared__ uint32_t gstart[kR];
  __shared__ uint32_t wsum[kWaves];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t tile = xcd_tile(tiles);
  const int64_t base = tile * kTile;
  for (int i = tid; i < kWaves * kR; i += kThreads) (&wcnt[0][0])[i] = 0u;
  const bool local_ends = LINK && bnd != nullptr;  // uniform: no global digit offsets needed
  if (!local_ends) {  // global start of each digit for this tile
    uint32_t v[DPT];
#pragma unroll
    for (int j = 0; j < DPT; ++j) v[j] = tid * DPT + j < kR ? totals[tid * DPT + j] : 0u;
    digits_exclusive_scan<DPT>(v, wsum, nullptr);
#pragma unroll
    for (int j = 0; j < DPT; ++j)
      if (tid * DPT + j < kR) gstart[tid * DPT + j] = v[j] + counts[(int64_t)(tid * DPT + j) * tiles + tile];
  }
  if constexpr (KS > 0) decode_tile_keys<KS>(rec, kend, base, n, sval);  // sval: scratch until the scatter
  __syncthreads();

  // wave wv owns tile elements [wv*kItems*64, (wv+1)*kItems*64) in (item, lane) order,
  // so (wave, item, lane) order is tile order and the ranks below are stable
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  uint32_t key[kItems], val[kItems], rank[kItems];
#pragma unroll
  for (int it = 0; it < kItems; ++it) {
    const int64_t idx = base + (int64_t)(wv * kItems + it) * 64 + lane;
    const bool valid = idx < n;
    // pads sort last: digit 255, after every real key
    if constexpr (KS > 0) key[it] = valid ? sval[(wv * kItems + it) * 64 + lane] : 0xffffffffu;
    else key[it] = valid ? ld32<NT>(kin + idx) : 0xffffffffu;
    if constexpr (KS == 0) val[it] = valid ? ld32<NT>(vin + idx) : 0u;
    else val[it] = (uint32_t)idx;
  }
#pragma unroll
  for (int it = 0; it < kItems; ++it) {
    const uint32_t d = (key[it] >> shift) & (kR - 1);
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const uint64_t bal = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? bal : ~bal;
    }
    const uint32_t before = (uint32_t)__popcll(peers & lt_mask);
    const uint32_t run = wcnt[wv][d];
    rank[it] = run + before;
    if (before == (uint32_t)__popcll(peers) - 1u) wcnt[wv][d] = run + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  {  // per-digit prefix over waves, then tile-local digit starts
    uint32_t v[DPT];
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      const int d = tid * DPT + j;
      uint32_t s = 0;
      if (d < kR) {  // (threads past kR own no digit: they add 0 to the scan)
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
          const uint32_t c = wcnt[w][d];
          wcnt[w][d] = s;
          s += c;
        }
      }
      v[j] = s;
    }
    digits_exclusive_scan<DPT>(v, wsum, nullptr);
#pragma unroll
    for (int j = 0; j < DPT; ++j)
      if (tid * DPT + j < kR) tstart[tid * DPT + j] = v[j];
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < kItems; ++it) {
    const uint32_t d = (key[it] >> shift) & (kR - 1);
    const uint32_t pos = tstart[d] + wcnt[wv][d] + rank[it];
    skey[pos] = key[it];
    sval[pos] = val[it];
  }
  __syncthreads();
  const int64_t nvalid = n - base < kTile ? n - base : kTile;
  if constexpr (LINK) {
    if (local_ends && bounds && tid < nd) {  // digits without an element in this tile
      const uint32_t e = tid + 1 < kR ? tstart[tid + 1] : (uint32_t)kTile;
      if (tstart[tid] == e) bnd[tile * nd + tid].kf = kRunEmpty;
    }
  }
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const int i = k * kThreads + tid;
    if (i < nvalid) {
      const uint32_t kk = skey[i];
      const uint32_t d = (kk >> shift) & (kR - 1);
      const int64_t o = local_ends ? 0 : (int64_t)gstart[d] + (i - (int64_t)tstart[d]);
      if constexpr (!LINK) {
        st32<NT>(kout + o, kk);
        st32<NT>(vout + o, sval[i]);
      } else {
        const int hi = d + 1 < (uint32_t)kR ? (int)tstart[d + 1] : kTile;
        const bool first = i == (int)tstart[d];
        const bool last = i + 1 == hi || i + 1 >= nvalid;
        const uint32_t v = sval[i];
        if (bounds && (first || last)) {  // the fix-up reads the boundary pairs of every run
          if (local_ends) {
            if ((int)d < nd) {  // (pads sort to digit kR - 1, past the schedule's digits)
              RunEnds* r = bnd + tile * nd + d;
              if (first) { r->kf = kk; r->vf = v; }
              if (last) { r->kl = kk; r->vl = v; }
            }
          } else {
            st32<NT>(kout + o, kk);
            st32<NT>(vout + o, v);
          }
        }
        if (kk < kend && v >= vlo && v < vhi) {  // this part's slot range (link_parts)
          uint32_t w = (!last && skey[i + 1] == kk) ? sval[i + 1] / (uint32_t)slots_per_match
                                                     : kNoMatch;
          if (!first && skey[i - 1] == kk) w |= kLinkHasPred;
          // (non-temporal link stores alone measured 3.6 vs 1.6 ms per prepass: L2 write
          // combining of these random 4-B stores matters, profiles/r3/ab_link_nt.log)
          st32<NT>(link + v, w);
        }
      }
    }
  }
}

// The LINK pass in parts by slot range.  Its link stores are random 4-B writes,
// each its own fabric request (PMC: one TCC_EA0_WRREQ per store), and they stay
// cheap only while the link array they land in fits the 256-MB Infinity Cache:
// 60M 3v3 slots (240 MB) take 0.85 ms, 96M (config 5, 384 MB) 2.61 ms and 125M
// 5v5 slots (500 MB) 3.35 ms.  A larger array is written in ceil(bytes / 256 MB)
// passes over the sorted pairs, each storing only the links of its slot range
// (the LDS sort is repeated; the boundary pairs go out once): config 5 in two
// parts 2 x 0.91 ms, its step 13.40 -> 12.56 ms.  Splitting config 2's 240 MB
// as well costs more than it saves (8.13 -> 8.46 ms).  ANA_LINK_PARTS overrides
// the count (1 = one pass).
// ANA_SCHED_RUNS=0: the last pass with digit offsets + sched_fixup (the round-2 path),
// for A/B; default: the run table (radix_downsweep bnd, sched_runs_fixup)
static bool local_runs() {  // per schedule: tests switch it at run time
  const char* e = getenv("ANA_SCHED_RUNS");
  return !(e && atoi(e) == 0);
}

static int link_parts(int64_t n) {
  if (const char* e = getenv("ANA_LINK_PARTS")) {  // per launch: tests switch it at run time
    const int v = atoi(e);
    if (v >= 1) return v > 16 ? 16 : v;
  }
  const int64_t bytes = n * 4, part = 256ll << 20;
  return (int)((bytes + part - 1) / part);
}

// Completes the links of the run-boundary slots of the LINK pass: one thread per
// (tile, digit) run; its first pair's predecessor and its last pair's successor
// are the last / first pairs of the neighbouring runs, which that pass wrote.
// Grid: (tile groups of 256, digits); blocks of empty digits exit at once.
template <int RB = 8>
__global__ void __launch_bounds__(kThreads)
sched_fixup(const uint32_t* __restrict__ kout, const uint32_t* __restrict__ vout, int64_t n,
            uint32_t kend, const uint32_t* __restrict__ counts, const uint32_t* __restrict__ totals,
            int64_t tiles, int slots_per_match, uint32_t* __restrict__ link) {
  constexpr int kR = 1 << RB;
  __shared__ uint32_t wsum[kWaves];
  const int d = blockIdx.y;
  const uint32_t tot = totals[d];
  if (tot == 0) return;
  uint32_t below = 0;
#pragma unroll
  for (int j = threadIdx.x; j < kR; j += kThreads) below += j < d ? totals[j] : 0u;
  uint32_t all = 0;
  const uint32_t before = block_exclusive_scan(below, wsum, &all);
  (void)before;
  const uint32_t dstart = all;  // sum of the totals of the digits below d
  const int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (t >= tiles) return;
  const uint32_t* row = counts + (int64_t)d * tiles;
  const uint32_t c0 = row[t];
  const uint32_t c1 = t + 1 < tiles ? row[t + 1] : tot;
  if (c1 == c0) return;
  const int64_t of = (int64_t)dstart + c0, ol = (int64_t)dstart + c1 - 1;
  const uint32_t kf = kout[of], kl = kout[ol];
  const bool pred = kf < kend && of > 0 && kout[of - 1] == kf;
  const bool succ = kl < kend && ol + 1 < n && kout[ol + 1] == kl;
  const uint32_t nxt = succ ? vout[ol + 1] / (uint32_t)slots_per_match : kNoMatch;
  if (of == ol) {
    if (kf < kend) link[vout[of]] = nxt | (pred ? kLinkHasPred : 0u);
    return;
  }
  if (pred) {
    const uint32_t v = vout[of];
    link[v] |= kLinkHasPred;
  }
  if (succ) {
    const uint32_t v = vout[ol];
    link[v] = (link[v] & ~kMatchMask) | nxt;
  }
}

// The last pass's run table -> links across tiles (sched_runs_fixup): the
// predecessor of the first pair of run (t, d) is the last pair of the nearest
// non-empty run (t' < t, d).  Segments of kThreads tiles: sched_runs_last finds each
// segment's last non-empty tile per digit, sched_runs_fixup takes the nearest one
// before its segment as the carry and a block max-scan of the non-empty tiles inside
// it.  Grids (segments, nd); nd <= kRunsMaxDigits keeps the table small.
constexpr int kRunsMaxDigits = 32;

__global__ void __launch_bounds__(kThreads)
sched_runs_last(const RunEnds* __restrict__ bnd, int64_t tiles, int nd, int32_t* __restrict__ seglast) {
  __shared__ int32_t wmax[kWaves];
  const int d = blockIdx.y;
  const int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  int32_t x = (t < tiles && bnd[t * nd + d].kf != kRunEmpty) ? (int32_t)t : -1;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x = max(x, __shfl_xor(x, off));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t m = wmax[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) m = max(m, wmax[w]);
    seglast[(int64_t)d * gridDim.x + blockIdx.x] = m;
  }
}

__global__ void __launch_bounds__(kThreads)
sched_runs_fixup(const RunEnds* __restrict__ bnd, int64_t tiles, int nd, const int32_t* __restrict__ seglast,
                 uint32_t kend, int slots_per_match, uint32_t* __restrict__ link) {
  __shared__ int32_t wmax[kWaves];
  __shared__ int32_t carry_s;
  const int d = blockIdx.y, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t seg = blockIdx.x;
  // carry: the last non-empty tile of digit d before this segment (seglast grows with the segment)
  if (wv == 0) {
    int32_t c = -1;
    for (int64_t q = lane; q < seg; q += 64) c = max(c, seglast[(int64_t)d * gridDim.x + q]);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) c = max(c, __shfl_xor(c, off));
    if (lane == 0) carry_s = c;
  }
  const int64_t t = seg * kThreads + threadIdx.x;
  RunEnds me = {kRunEmpty, 0u, kRunEmpty, 0u};
  if (t < tiles) me = bnd[t * nd + d];
  const bool full = me.kf != kRunEmpty;
  // inclusive max-scan of the non-empty tiles: wave, then across the block's waves
  int32_t x = full ? (int32_t)t : -1;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(x, off);
    if (lane >= off) x = max(x, y);
  }
  if (lane == 63) wmax[wv] = x;
  __syncthreads();
  int32_t before = carry_s;
  for (int w = 0; w < wv; ++w) before = max(before, wmax[w]);
  int32_t ex = __shfl_up(x, 1);  // exclusive within the wave
  ex = lane == 0 ? -1 : ex;
  const int32_t pred = max(before, ex);
  if (!full || pred < 0 || me.kf >= kend) return;
  const RunEnds pr = bnd[(int64_t)pred * nd + d];
  if (pr.kl != me.kf) return;  // the key starts here: no earlier occurrence
  // the two boundary links: each word gets its bits from one thread each (atomics on
  // disjoint fields, so a one-pair run that is both a first and a last is safe)
  atomicOr(&link[me.vf], kLinkHasPred);
  atomicAnd(&link[pr.vl], ~kMatchMask | (me.vf / (uint32_t)slots_per_match));
}

}  // namespace

size_t radix_sort_workspace_bytes(int64_t n) {
  const int64_t tiles = (n + kTile - 1) / kTile;
  return (size_t)(tiles * kRadixMax + kRadixMax) * 4;
}

int launch_radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt,
                            int64_t n, int bits, void* ws, int* result_in_alt, hipStream_t s) {
  *result_in_alt = 0;
  if (n <= 0) return 0;
  if (n > 0x7fffffffLL || bits < 1 || bits > 32) return (int)hipErrorInvalidValue;
  const int64_t tiles = (n + kTile - 1) / kTile;
  uint32_t* counts = static_cast<uint32_t*>(ws);
  uint32_t* totals = counts + tiles * kRadix;
  uint32_t *ki = keys, *vi = vals, *ko = keys_alt, *vo = vals_alt;
  for (int shift = 0; shift < bits; shift += 8) {
    hipLaunchKernelGGL(radix_upsweep<0>, dim3((unsigned)tiles), dim3(kThreads), 0, s, ki, nullptr,
                       0u, n, shift, counts, tiles);
    hipLaunchKernelGGL(radix_rowscan, dim3(kRadix), dim3(kThreads), 0, s, counts, tiles, totals);
    hipLaunchKernelGGL((radix_downsweep<0, false>), dim3((unsigned)tiles), dim3(kThreads), 0, s, ki,
                       vi, nullptr, 0u, ko, vo, n, shift, counts, totals, tiles, 1, nullptr);
    std::swap(ki, ko);
    std::swap(vi, vo);
    *result_in_alt ^= 1;
  }
  return (int)hipGetLastError();
}

// The schedule's sort (K5): the slots of the stream by player, stable, fused at
// both ends -- the first pass reads the records (no key array is written), the
// last pass writes links instead of sorted pairs, then sched_fixup.  RB-bit
// digits (8; 10 as an experiment).
template <int K, int RB, int NT>
static void sched_sort_k(const int32_t* rec, int64_t n, uint32_t kend, int bits, uint32_t* ka,
                         uint32_t* va, uint32_t* kb, uint32_t* vb, uint32_t* counts,
                         int64_t tiles, uint32_t* link, const SchedInit& init, hipStream_t s) {
  constexpr int S = 2 * K;
  constexpr int kR = 1 << RB;
  uint32_t* totals = counts + tiles * kR;
  const dim3 grid((unsigned)tiles), block(kThreads);
  const uint32_t *ki = nullptr, *vi = nullptr;
  uint32_t *ko = kb, *vo = vb;
  for (int shift = 0; shift < bits; shift += RB) {
    const bool first = shift == 0, last = shift + RB >= bits;
    // the last pass of a multi-pass sort over few digits (1M players: bits 16..19, 16
    // digits): run ends in a table, no digit offsets (radix_downsweep bnd)
    const int nd = bits - shift < RB ? 1 << (bits - shift) : kR;
    if (last && !first && nd <= kRunsMaxDigits && local_runs()) {
      RunEnds* bnd = reinterpret_cast<RunEnds*>(counts);  // pass counts are consumed by now
      const int64_t nseg = (tiles + kThreads - 1) / kThreads;
      int32_t* seglast = reinterpret_cast<int32_t*>(bnd + tiles * nd);
      const int parts = link_parts(n);
      for (int q = 0; q < parts; ++q)
        hipLaunchKernelGGL((radix_downsweep<0, true, RB, NT>), grid, block, 0, s, ki, vi, nullptr, kend, ko, vo,
                           n, shift, counts, totals, tiles, S, link, (uint32_t)(n * q / parts),
                           (uint32_t)(n * (q + 1) / parts), q == 0 ? 1 : 0, bnd, nd);
      const dim3 sgrid((unsigned)nseg, (unsigned)nd);
      hipLaunchKernelGGL(sched_runs_last, sgrid, block, 0, s, bnd, tiles, nd, seglast);
      hipLaunchKernelGGL(sched_runs_fixup, sgrid, block, 0, s, bnd, tiles, nd, seglast, kend, S, link);
      break;
    }
    if (first)
      hipLaunchKernelGGL((radix_upsweep<K, RB, NT>), grid, block, 0, s, nullptr, rec, kend, n, shift, counts, tiles,
                         init);
    else
      hipLaunchKernelGGL((radix_upsweep<0, RB, NT>), grid, block, 0, s, ki, nullptr, kend, n, shift, counts, tiles);
    hipLaunchKernelGGL(radix_rowscan, dim3(kR), block, 0, s, counts, tiles, totals);
    const int parts = last ? link_parts(n) : 1;
    if (first && last)
      for (int q = 0; q < parts; ++q)
        hipLaunchKernelGGL((radix_downsweep<K, true, RB, NT>), grid, block, 0, s, nullptr, nullptr, rec, kend, ko,
                           vo, n, shift, counts, totals, tiles, S, link, (uint32_t)(n * q / parts),
                           (uint32_t)(n * (q + 1) / parts), q == 0 ? 1 : 0);
    else if (first)
      hipLaunchKernelGGL((radix_downsweep<K, false, RB, NT>), grid, block, 0, s, nullptr, nullptr, rec, kend, ko,
                         vo, n, shift, counts, totals, tiles, S, nullptr);
    else if (last)
      for (int q = 0; q < parts; ++q)
        hipLaunchKernelGGL((radix_downsweep<0, true, RB, NT>), grid, block, 0, s, ki, vi, nullptr, kend, ko, vo,
                           n, shift, counts, totals, tiles, S, link, (uint32_t)(n * q / parts),
                           (uint32_t)(n * (q + 1) / parts), q == 0 ? 1 : 0);
    else
      hipLaunchKernelGGL((radix_downsweep<0, false, RB, NT>), grid, block, 0, s, ki, vi, nullptr, kend, ko, vo, n,
                         shift, counts, totals, tiles, S, nullptr);
    if (last)
      hipLaunchKernelGGL((sched_fixup<RB>), dim3((unsigned)((tiles + kThreads - 1) / kThreads), kR), block,
                         0, s, ko, vo, n, kend, counts, totals, tiles, S, link);
    ki = ko;
    vi = vo;
    ko = ko == kb ? ka : kb;
    vo = vo == vb ? va : vb;
  }
}

int launch_sched_sort(int K, const int32_t* rec, int64_t M, uint32_t num_players, uint32_t* ka,
                      uint32_t* va, uint32_t* kb, uint32_t* vb, void* ws, uint32_t* link,
                      hipStream_t s, int32_t* deps, uint32_t* ctrl, int nz, int32_t* epoch_bump,
                      int sort_nt) {
  const int64_t n = M * 2 * K;
  if (n <= 0) return 0;
  if (n > kMaxSlots) return (int)hipErrorInvalidValue;
  int bits = 1;  // keys run up to num_players (= "no state")
  while (bits < 32 && (1ull << bits) <= (uint64_t)num_players) ++bits;
  const int64_t tiles = (n + kTile - 1) / kTile;
  uint32_t* counts = static_cast<uint32_t*>(ws);
  SchedInit init;
  init.deps = deps;
  init.ctrl = ctrl;
  init.nz = ctrl ? nz : 0;
  init.epoch_bump = epoch_bump;
  // ANA_SORT_RB=10: 10-bit digits (2 passes for <= 2^20 players instead of 3).  Measured
  // on MI355X, 10M 3v3 / 1M players: 3.11 ms vs 1.76 ms for 8-bit digits (1024
  // per-tile runs of ~4 elements scatter the pass's writes) -> off by default.
  // read per schedule, like ANA_SCHED_RUNS / ANA_LINK_PARTS: A/B runs and tests switch
  // them inside one process
  const char* rb_e = getenv("ANA_SORT_RB");
  const char* nt_e = getenv("ANA_SORT_NT");
  const int rb_env = rb_e ? atoi(rb_e) : 8;
  // sort_nt >= 0: the caller's choice (WindowPipeline: loads-only between DP merges)
  const int nt = nt_e ? atoi(nt_e) : sort_nt >= 0 ? sort_nt : 0;
  const bool wide = bits <= 20 && rb_env == 10;
  switch (K) {
#define ANA_SORT_CASE(k)                                                                         \
  case k:                                                                                        \
    if (wide) sched_sort_k<k, 10, 0>(rec, n, num_players, bits, ka, va, kb, vb, counts, tiles, link, init, s); \
    else if (nt == 1) sched_sort_k<k, 8, 1>(rec, n, num_players, bits, ka, va, kb, vb, counts, tiles, link, init, s); \
    else if (nt == 2) sched_sort_k<k, 8, 2>(rec, n, num_players, bits, ka, va, kb, vb, counts, tiles, link, init, s); \
    else sched_sort_k<k, 8, 0>(rec, n, num_players, bits, ka, va, kb, vb, counts, tiles, link, init, s); \
    break;
    ANA_SORT_CASE(1) ANA_SORT_CASE(2) ANA_SORT_CASE(3) ANA_SORT_CASE(4) ANA_SORT_CASE(5)
#undef ANA_SORT_CASE
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace ana
