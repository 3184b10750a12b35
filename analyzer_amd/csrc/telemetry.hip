// K8 kernels for gfx950: synthetic telemetry generation (K7 extension) and the
// standalone per-participant aggregation.  The same wave-tile routine
// (telemetry_dev.h) also runs inside the dataflow executor's idle time
// (dataflow.hip), which is the fused streaming mode of BASELINE config 4.
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"
#include "telemetry_dev.h"

namespace ana {

// events per match (counts[m]) for the CSR offsets; the scan runs on the host side of the op
__global__ void gen_event_counts_kernel(GenEventParams g, int64_t base, int64_t M,
                                        int64_t* __restrict__ counts) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m < M) counts[m] = gen_event_count(g, (uint64_t)(base + m));
}

// one wave per match: lanes write the match's events with coalesced 16-B stores
template <int K>
__global__ void __launch_bounds__(256)
gen_events_kernel(GenEventParams g, int64_t base, const int32_t* __restrict__ rec,
                  const int64_t* __restrict__ evoff, int64_t M, int32_t* __restrict__ events) {
  constexpr int S = 2 * K;
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * 4;
  for (int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); m < M; m += waves) {
    const uint32_t m0 = (uint32_t)rec[m * (S + 2) + S];
    const int n0 = meta_n0(m0) < K ? meta_n0(m0) : K, n1 = meta_n1(m0) < K ? meta_n1(m0) : K;
    const int64_t e0 = evoff[m], e1 = evoff[m + 1];
    for (int64_t e = e0 + lane; e < e1; e += 64) {
      int32_t ev[4];
      gen_event(g, (uint64_t)(base + m), e - e0, (int32_t)m, n0 + n1, ev);
      const int r = event_slot(ev[1]);  // participant index -> record slot
      ev[1] = (ev[1] & ~0xff) | (r < n0 ? r : K + (r - n0));
      reinterpret_cast<int4*>(events)[e] = make_int4(ev[0], ev[1], ev[2], ev[3]);
    }
  }
}

template <int K>
__global__ void __launch_bounds__(256) telemetry_kernel(TelemetryParams tp, uint32_t* bad) {
  __shared__ float scratch[4][kTeleTile * 2 * K * (kStatFeatures + 1)];
  const int wv = threadIdx.x >> 6;
  const int64_t tiles = (tp.num_matches + kTeleTile - 1) / kTeleTile;
  const int64_t t = (int64_t)blockIdx.x * 4 + wv;
  if (t < tiles) telemetry_tile<K>(tp, t, threadIdx.x & 63, scratch[wv], bad);
}

int launch_gen_event_counts(const GenEventParams& g, int64_t base, int64_t M, int64_t* counts,
                            hipStream_t s) {
  if (M <= 0) return 0;
  hipLaunchKernelGGL(gen_event_counts_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, g,
                     base, M, counts);
  return (int)hipGetLastError();
}

int launch_gen_events(int K, const GenEventParams& g, int64_t base, const int32_t* rec,
                      const int64_t* evoff, int64_t M, int32_t* events, hipStream_t s) {
  if (M <= 0) return 0;
  const unsigned blocks = (unsigned)((M + 3) / 4 < 65536 ? (M + 3) / 4 : 65536);
  switch (K) {
#define ANA_GENEV_CASE(k)                                                                      \
  case k:                                                                                      \
    hipLaunchKernelGGL(gen_events_kernel<k>, dim3(blocks), dim3(256), 0, s, g, base, rec, evoff, \
                       M, events);                                                             \
    break;
    ANA_GENEV_CASE(1) ANA_GENEV_CASE(2) ANA_GENEV_CASE(3) ANA_GENEV_CASE(4) ANA_GENEV_CASE(5)
#undef ANA_GENEV_CASE
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

int launch_telemetry(int K, const TelemetryParams& tp, uint32_t* bad, hipStream_t s) {
  if (tp.num_matches <= 0) return 0;
  const int64_t tiles = (tp.num_matches + kTeleTile - 1) / kTeleTile;
  const unsigned blocks = (unsigned)((tiles + 3) / 4);
  switch (K) {
#define ANA_TELE_CASE(k)                                                                         \
  case k: hipLaunchKernelGGL(telemetry_kernel<k>, dim3(blocks), dim3(256), 0, s, tp, bad); break;
    ANA_TELE_CASE(1) ANA_TELE_CASE(2) ANA_TELE_CASE(3) ANA_TELE_CASE(4) ANA_TELE_CASE(5)
#undef ANA_TELE_CASE
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace ana
