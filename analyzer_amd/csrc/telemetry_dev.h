// K8 device side: aggregate the telemetry of one tile of matches with ONE wave
// (no barriers, so the dataflow executor can run it in its idle time).
//
// The tile's stat block [T][2K][kStatFeatures] lives in the wave's LDS
// scratch; events of the tile (contiguous: evoff is a CSR index) are streamed
// with 16-B loads (8 per lane in flight), folded in with LDS float atomics
// (ds_add_f32: contention only among a match's participants); the block then
// leaves LDS as one contiguous, coalesced store -- the per-match stat rows of
// consecutive matches are adjacent in the [M][2K][F] output.
#pragma once

#include <hip/hip_runtime.h>

#include "telemetry_core.h"

namespace ana {

template <int K>
__device__ __forceinline__ void telemetry_tile(const TelemetryParams& tp, int64_t tile, int lane,
                                               float* lds, uint32_t* bad_events) {
  constexpr int S = 2 * K;
  constexpr int kRow = S * kStatFeatures;
  // participant rows padded to an odd stride in LDS: rows 8 floats apart would
  // put every row's feature f in the same 4 of the 32 banks
  constexpr int kPad = kStatFeatures + 1;
  const int64_t m0 = tile * kTeleTile;
  const int64_t m1 = m0 + kTeleTile < tp.num_matches ? m0 + kTeleTile : tp.num_matches;
  const int n = (int)(m1 - m0) * kRow;
  const int npad = (int)(m1 - m0) * S * kPad;
  for (int i = lane; i < npad; i += 64) lds[i] = 0.f;
  const int64_t e0 = tp.evoff[m0], e1 = tp.evoff[m1];
  uint32_t bad = 0;
  // 8 events per lane in flight: the loads of a batch retire in one round trip
  constexpr int kBatch = 8;
  for (int64_t base = e0; base < e1; base += 64 * kBatch) {
    int4 ev[kBatch];
#pragma unroll
    for (int q = 0; q < kBatch; ++q) {
      const int64_t e = base + q * 64 + lane;
      ev[q] = e < e1 ? reinterpret_cast<const int4*>(tp.events)[e] : make_int4(-1, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < kBatch; ++q) {
      if (base + q * 64 + lane >= e1) continue;
      const int64_t ml = (int64_t)ev[q].x - m0;
      const int slot = event_slot(ev[q].y);
      if (ml < 0 || ml >= m1 - m0 || slot >= S) {
        ++bad;
        continue;
      }
      float add;
      const int f = event_feature(event_type(ev[q].y), __int_as_float(ev[q].z), add);
      float* row = lds + (ml * S + slot) * kPad;
      if (f >= 0) atomicAdd(row + f, add);
      atomicAdd(row + kStatEvents, 1.f);
    }
  }
  if (bad) atomicAdd(bad_events, bad);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the LDS adds have landed (wave-local)
  float* dst = tp.stats + m0 * kRow;
  for (int i = lane; i < n; i += 64) dst[i] = lds[(i / kStatFeatures) * kPad + i % kStatFeatures];
}

}  // namespace ana
