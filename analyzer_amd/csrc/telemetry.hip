// K8 kernels for gfx950: synthetic telemetry generation (K7 extension) and the
// standalone per-participant aggregation.  The same wave-tile routine
// (telemetry_dev.h) also runs inside the dataflow executor's idle time
// (dataflow.hip), which is the fused streaming mode of BASELINE config 4.
#include <hip/hip_runtime.h>

#include <cstdlib>

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

// one wave per match: lanes write the match's events with coalesced 8-B stores
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
      int32_t ev[2];
      gen_event(g, (uint64_t)(base + m), e - e0, (int32_t)m, n0 + n1, ev);
      const int r = event_slot(ev[0]);  // participant index -> record slot
      ev[0] = (ev[0] & ~0xff) | (r < n0 ? r : K + (r - n0));
      reinterpret_cast<int2*>(events)[e] = make_int2(ev[0], ev[1]);
    }
  }
}

// D: 0 = LDS float atomics (telemetry_tile, 16-match tiles), 3 = one-hot MFMA
// (telemetry_tile_mfma over SPAN-match spans), 1 / 2 = timing-only diagnostics
// of the atomic version, 6 / 7 = of the MFMA version (ANA_TELE_DEBUG)
template <int K, int D, int SPAN>
__global__ void __launch_bounds__(256) telemetry_kernel(TelemetryParams tp, uint32_t* bad) {
#if ANA_DIAG_BUILD
  // impl 3 (D 10) needs only its stage, decoded records and CSR: 1.9 KB per wave
  __shared__ float scratch[4][D == 10 ? kTeleRegsFloats : tele_scratch_floats<K>()];
#else
  __shared__ float scratch[4][tele_scratch_floats<K>()];
#endif
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t tiles = (tp.num_matches + SPAN - 1) / SPAN;
  const int64_t t = (int64_t)blockIdx.x * 4 + wv;
  if (t >= tiles) return;
#if ANA_DIAG_BUILD
  if constexpr (D == 10) telemetry_tile_regs<K, SPAN>(tp, t, threadIdx.x & 63, scratch[wv], bad);
  else
#endif
  if constexpr (D >= 3) telemetry_tile_mfma<K, D - 3, SPAN>(tp, t, threadIdx.x & 63, scratch[wv], bad);
  else telemetry_tile<K, D>(tp, t, threadIdx.x & 63, scratch[wv], bad);
}

// impl 2: ONE LANE PER STAT ROW.  Lane (q, j) of a wave owns the stat row of slot j
// of the wave's q-th match (64 / 2K matches per wave) and walks that match's whole
// CSR range, folding the events of its slot: every event is read by the 2K lanes of
// its match (one broadcast line per instruction), and each lane adds only its own.
// The row's seven sums live in LDS at a lane-private stride of 9 floats (the
// feature is per-event data, and a register array indexed by it would be a select
// chain over all seven), added with ds_add_f32 (IEEE round to nearest, in issue
// order), the event count in a register.  Sums run in event order
// per row, the order of the host mirror, so the result is the host's bit for bit
// (Inf / NaN values included); a malformed event is counted once, by slot 0's lane.
// 4 events in flight per lane; the loop runs to the longest range of the wave.
template <int K>
__global__ void __launch_bounds__(256) telemetry_rows_kernel(TelemetryParams tp, uint32_t* bad) {
  constexpr int S = 2 * K;
  constexpr int MPW = 64 / S;   // matches per wave
  constexpr int kStride = 9;    // LDS floats per lane (8 sums + pad: conflict-free lane stride)
  constexpr int kAhead = 4;     // event loads in flight per lane
  __shared__ float rows[256 * kStride];
  const int lane = threadIdx.x & 63;
  const int64_t task = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int q = lane / S, slot = lane % S;
  const int64_t m = task * MPW + q;
  const bool act = q < MPW && m < tp.num_matches;
  const int64_t e0 = act ? tp.evoff[m] : 0;
  const int n = act ? (int)(tp.evoff[m + 1] - e0) : 0;
  int nmax = n;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) nmax = max(nmax, __shfl_xor(nmax, off));
  float* const acc = rows + threadIdx.x * kStride;
#pragma unroll
  for (int k = 0; k < kStatFeatures - 1; ++k) acc[k] = 0.f;
  const uint32_t mtag = (uint32_t)m & 0xffffu;
  float cnt = 0.f;
  uint32_t nbad = 0;
  const int32_t* const dummy = reinterpret_cast<const int32_t*>(tp.evoff);
  for (int i = 0; i < nmax; i += kAhead) {
    int2 ev[kAhead];
#pragma unroll
    for (int u = 0; u < kAhead; ++u) {
      const bool ok = i + u < n;
      ev[u] = *reinterpret_cast<const int2*>(ok ? tp.events + 2 * (e0 + i + u) : dummy);
    }
#pragma unroll
    for (int u = 0; u < kAhead; ++u) {
      if (i + u >= n) continue;
      const int32_t meta = ev[u].x;
      const int es = event_slot(meta);
      const bool good = event_tag(meta) == mtag && es < S;
      if (!good) {
        nbad += slot == 0 ? 1u : 0u;
        continue;
      }
      if (es != slot) continue;
      cnt += 1.f;
      float add;
      const int f = event_feature(event_type(meta), __int_as_float(ev[u].y), add);
      // lane-private LDS word: a ds_add without return -- fire and forget, applied in
      // issue order, so consecutive events of one feature never wait on a read-back
      if (f >= 0) atomicAdd(&acc[f], add);
    }
  }
  if (act) {
    float4* dst = reinterpret_cast<float4*>(tp.stats + (m * S + slot) * kStatFeatures);
    dst[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    dst[1] = make_float4(acc[4], acc[5], acc[6], cnt);
  }
  if (nbad) atomicAdd(bad, nbad);
}

template <int K>
static void launch_tele_rows(const TelemetryParams& tp, uint32_t* bad, hipStream_t s) {
  constexpr int MPW = 64 / (2 * K);
  const int64_t tasks = (tp.num_matches + MPW - 1) / MPW;
  hipLaunchKernelGGL(telemetry_rows_kernel<K>, dim3((unsigned)((tasks + 3) / 4)), dim3(256), 0, s, tp, bad);
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

int tele_impl() {
  const char* e = getenv("ANA_TELE_IMPL");
  return e ? atoi(e) : 1;
}

template <int K, int D, int SPAN>
static void launch_tele(const TelemetryParams& tp, uint32_t* bad, hipStream_t s) {
  const int64_t tiles = (tp.num_matches + SPAN - 1) / SPAN;
  hipLaunchKernelGGL((telemetry_kernel<K, D, SPAN>), dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, s,
                     tp, bad);
}

// The production library instantiates the two implementations only; the
// diagnostic variants (no adds / no MFMA / decode only) and the tuning spans
// are in the diagnostic build (python -m analyzer_amd.build_ext --diag).
template <int K>
static void launch_tele_k(const TelemetryParams& tp, uint32_t* bad, hipStream_t s, int impl, int dbg,
                          int span) {
#if ANA_DIAG_BUILD
  if (dbg == 1) return launch_tele<K, 1, kTeleTile>(tp, bad, s);
  if (dbg == 2) return launch_tele<K, 2, kTeleTile>(tp, bad, s);
#endif
  if (impl == 0) return launch_tele<K, 0, kTeleTile>(tp, bad, s);
  if (impl == 2) return launch_tele_rows<K>(tp, bad, s);
#if ANA_DIAG_BUILD
  if (impl == 3) return launch_tele<K, 10, kTeleMaxSpan>(tp, bad, s);
  const int d = dbg == 6 ? 6 : dbg == 7 ? 7 : 3;
#define ANA_TELE_SPAN(sp)                                                                     \
  if (span == sp) {                                                                           \
    if (d == 6) return launch_tele<K, 6, sp>(tp, bad, s);                                     \
    if (d == 7) return launch_tele<K, 7, sp>(tp, bad, s);                                     \
    return launch_tele<K, 3, sp>(tp, bad, s);                                                 \
  }
  ANA_TELE_SPAN(16) ANA_TELE_SPAN(32)
#undef ANA_TELE_SPAN
  if (d == 6) return launch_tele<K, 6, kTeleMaxSpan>(tp, bad, s);
  if (d == 7) return launch_tele<K, 7, kTeleMaxSpan>(tp, bad, s);
#else
  (void)dbg;
  (void)span;
#endif
  return launch_tele<K, 3, kTeleMaxSpan>(tp, bad, s);
}

int launch_telemetry(int K, const TelemetryParams& tp, uint32_t* bad, hipStream_t s) {
  if (tp.num_matches <= 0) return 0;
  // ANA_TELE_IMPL: 1 (default) one-hot MFMA, 0 LDS atomics, 2 one lane per stat row, 3 (diagnostic
  // library only) one-hot MFMA with register-built fragments (telemetry_tile_regs); ANA_TELE_SPAN: matches per
  // wave of the MFMA kernel (16, 32, 63); ANA_TELE_DEBUG (diagnostic, timing only):
  // atomic version 1 = no LDS adds, 2 = no count adds; MFMA version 6 = no MFMA, 7 = decode only
  const char* dbg_env = getenv("ANA_TELE_DEBUG");
  const char* span_env = getenv("ANA_TELE_SPAN");
  const int dbg = dbg_env ? atoi(dbg_env) : 0;
  const int span = span_env ? atoi(span_env) : kTeleMaxSpan;
  const int impl = tele_impl();
#if !ANA_DIAG_BUILD
  // diagnostic / tuning variants are not in this library: refuse instead of
  // silently timing the production kernel under their name
  if (dbg != 0 || span != kTeleMaxSpan || impl == 3) return (int)hipErrorNotSupported;
#endif
  switch (K) {
    case 1: launch_tele_k<1>(tp, bad, s, impl, dbg, span); break;
    case 2: launch_tele_k<2>(tp, bad, s, impl, dbg, span); break;
    case 3: launch_tele_k<3>(tp, bad, s, impl, dbg, span); break;
    case 4: launch_tele_k<4>(tp, bad, s, impl, dbg, span); break;
    case 5: launch_tele_k<5>(tp, bad, s, impl, dbg, span); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace ana
