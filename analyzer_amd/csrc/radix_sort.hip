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
// 8-bit digits, 4096-element tiles (256 threads x 16), ceil(bits / 8) passes.
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"

namespace ana {

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;
constexpr int kRadix = 256;

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

__global__ void __launch_bounds__(kThreads)
radix_upsweep(const uint32_t* __restrict__ keys, int64_t n, int shift, uint32_t* __restrict__ counts,
              int64_t tiles) {
  __shared__ uint32_t hist[kWaves][kRadix];
  const int tid = threadIdx.x, wv = tid >> 6;
  for (int i = tid; i < kWaves * kRadix; i += kThreads) (&hist[0][0])[i] = 0u;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const int64_t idx = base + k * kThreads + tid;
    if (idx < n) atomicAdd(&hist[wv][(keys[idx] >> shift) & (kRadix - 1)], 1u);
  }
  __syncthreads();
  uint32_t c = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) c += hist[w][tid];
  counts[(int64_t)tid * tiles + blockIdx.x] = c;
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

__global__ void __launch_bounds__(kThreads)
radix_downsweep(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, int64_t n, int shift,
                const uint32_t* __restrict__ counts, const uint32_t* __restrict__ totals,
                int64_t tiles) {
  __shared__ uint32_t skey[kTile];
  __shared__ uint32_t sval[kTile];
  __shared__ uint32_t wcnt[kWaves][kRadix];
  __shared__ uint32_t tstart[kRadix];
  __shared__ uint32_t gstart[kRadix];
  __shared__ uint32_t wsum[kWaves];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t base = (int64_t)blockIdx.x * kTile;
  for (int i = tid; i < kWaves * kRadix; i += kThreads) (&wcnt[0][0])[i] = 0u;
  {  // global start of each digit for this tile
    const uint32_t dstart = block_exclusive_scan(totals[tid], wsum, nullptr);
    gstart[tid] = dstart + counts[(int64_t)tid * tiles + blockIdx.x];
  }
  __syncthreads();

  // wave wv owns tile elements [wv*kItems*64, (wv+1)*kItems*64) in (item, lane) order,
  // so (wave, item, lane) order is tile order and the ranks below are stable
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  uint32_t key[kItems], val[kItems], rank[kItems];
#pragma unroll
  for (int it = 0; it < kItems; ++it) {
    const int64_t idx = base + (int64_t)(wv * kItems + it) * 64 + lane;
    const bool valid = idx < n;
    key[it] = valid ? kin[idx] : 0xffffffffu;  // pads sort last: digit 255, after every real key
    val[it] = valid ? vin[idx] : 0u;
  }
#pragma unroll
  for (int it = 0; it < kItems; ++it) {
    const uint32_t d = (key[it] >> shift) & (kRadix - 1);
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
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
    uint32_t c[kWaves], s = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      c[w] = wcnt[w][tid];
      wcnt[w][tid] = s;
      s += c[w];
    }
    tstart[tid] = block_exclusive_scan(s, wsum, nullptr);
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < kItems; ++it) {
    const uint32_t d = (key[it] >> shift) & (kRadix - 1);
    const uint32_t pos = tstart[d] + wcnt[wv][d] + rank[it];
    skey[pos] = key[it];
    sval[pos] = val[it];
  }
  __syncthreads();
  const int64_t nvalid = n - base < kTile ? n - base : kTile;
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const int i = k * kThreads + tid;
    if (i < nvalid) {
      const uint32_t kk = skey[i];
      const uint32_t d = (kk >> shift) & (kRadix - 1);
      const int64_t o = (int64_t)gstart[d] + (i - (int64_t)tstart[d]);
      kout[o] = kk;
      vout[o] = sval[i];
    }
  }
}

}  // namespace

size_t radix_sort_workspace_bytes(int64_t n) {
  const int64_t tiles = (n + kTile - 1) / kTile;
  return (size_t)(tiles * kRadix + kRadix) * 4;
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
    hipLaunchKernelGGL(radix_upsweep, dim3((unsigned)tiles), dim3(kThreads), 0, s, ki, n, shift,
                       counts, tiles);
    hipLaunchKernelGGL(radix_rowscan, dim3(kRadix), dim3(kThreads), 0, s, counts, tiles, totals);
    hipLaunchKernelGGL(radix_downsweep, dim3((unsigned)tiles), dim3(kThreads), 0, s, ki, vi, ko, vo,
                       n, shift, counts, totals, tiles);
    std::swap(ki, ko);
    std::swap(vi, vo);
    *result_in_alt ^= 1;
  }
  return (int)hipGetLastError();
}

}  // namespace ana
