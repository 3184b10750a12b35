// K8: per-event telemetry -> per-participant stat vectors (the
// ``participant_stats`` table the reference maps but never fills,
// /root/reference/worker.py:75-78; its telemetry path only forwards asset URLs
// to the "telesuck" queue, worker.py:148-161).  Shared by the gfx950 kernels
// (standalone and fused into the dataflow executor) and the host mirror.
//
// Event (8 B, int2): x = slot | type << 8 | (window-local match index & 0xffff) << 16,
// y = value (float bits).  Events of a window are grouped by match (one
// telemetry file per match) and indexed by a CSR offset array evoff[M + 1], so
// the match is implied by the position: the 16-bit match tag only checks it.
// An event is attributed to the match whose CSR range holds it iff its tag
// names that match (mod 2^16) and its slot is < 2K; other events are counted as
// malformed.  (Round 1 used 16-B events with the full match index and the game
// time; the aggregation reads neither, and the stream is bandwidth-bound.)
#pragma once

#include <math.h>
#include <stdint.h>

#include "common.h"

namespace ana {

constexpr int kStatFeatures = 8;  // per participant, float32
constexpr int kTeleTile = 16;     // matches per aggregation tile (one wave)
enum StatFeature : int {
  kStatKills = 0,
  kStatDeaths = 1,
  kStatAssists = 2,
  kStatDamage = 3,
  kStatGold = 4,
  kStatFarm = 5,
  kStatHealing = 6,
  kStatEvents = 7,  // number of events attributed to the participant
};
enum EventType : int {
  kEvKill = 0,
  kEvDeath = 1,
  kEvAssist = 2,
  kEvDamage = 3,
  kEvGold = 4,
  kEvFarm = 5,
  kEvHeal = 6,
  kEvOther = 7,  // counted only
  kEvTypes = 8,
};

ANA_HD int event_slot(int32_t meta) { return meta & 0xff; }
ANA_HD int event_type(int32_t meta) { return (meta >> 8) & 0xff; }
ANA_HD uint32_t event_tag(int32_t meta) { return (uint32_t)meta >> 16; }  // match & 0xffff
ANA_HD int32_t event_meta(int slot, int type, int64_t match) {
  return (int32_t)((uint32_t)slot | ((uint32_t)type << 8) | ((uint32_t)(match & 0xffff) << 16));
}

// feature touched by an event type and the amount it adds (-1: none)
ANA_HD int event_feature(int type, float value, float& add) {
  switch (type) {
    case kEvKill: add = 1.f; return kStatKills;
    case kEvDeath: add = 1.f; return kStatDeaths;
    case kEvAssist: add = 1.f; return kStatAssists;
    case kEvDamage: add = value; return kStatDamage;
    case kEvGold: add = value; return kStatGold;
    case kEvFarm: add = value; return kStatFarm;
    case kEvHeal: add = value; return kStatHealing;
    default: add = 0.f; return -1;
  }
}

struct TelemetryParams {
  const int64_t* evoff;   // [M + 1] CSR offsets into events (nullptr: no telemetry)
  const int32_t* events;  // [E, 2]
  float* stats;           // [M, 2K, kStatFeatures]
  int64_t num_matches;
  int32_t impl = 1;       // device tile routine: 1 one-hot MFMA, 0 LDS float atomics
  int32_t fused_tail = 0; // fused executor: 0 = any idle wave aggregates, 1 = only waves
                          // holding no chunks (the window's tail; measured slower: 15.9 vs 14.6 ms)
  int32_t role_stride = 2; // fused executor, MFMA impl: > 0 = one wave in role_stride is an
                           // aggregation wave (63-match spans) until the events are done, then
                           // joins the rating; the rating waves never hold a tile while they
                           // hold matches.  0 = idle rating waves take 16-match tiles.
};

struct GenEventParams {
  uint64_t seed;
  int32_t min_events;     // events per match: uniform in [min, max]
  int32_t max_events;
};

// events of match m (global index g = base + m): count, then event e of it
ANA_HD int32_t gen_event_count(const GenEventParams& g, uint64_t gm) {
  const uint32_t span = (uint32_t)(g.max_events - g.min_events + 1);
  return g.min_events + (int32_t)(rng_u64(g.seed, gm, 40) % span);
}

ANA_HD void gen_event(const GenEventParams& g, uint64_t gm, int64_t e, int32_t m_local,
                      int32_t nslots, int32_t* out) {
  const uint64_t h = rng_u64(g.seed ^ mix64((uint64_t)e), gm, 41);
  const int slot = nslots > 0 ? (int)((h & 0xffff) % (uint32_t)nslots) : 0;
  // type mix: damage-heavy like real telemetry
  const uint32_t r = (uint32_t)((h >> 16) & 0xff);
  const int type = r < 12 ? kEvKill : r < 24 ? kEvDeath : r < 44 ? kEvAssist : r < 140 ? kEvDamage
                 : r < 190 ? kEvGold : r < 230 ? kEvFarm : r < 245 ? kEvHeal : kEvOther;
  const float u = (float)((h >> 24) & 0xffffff) * (1.f / 16777216.f);
  // explicit fmaf: host and device round identically (no contraction differences)
  const float value = type == kEvDamage ? fmaf(950.f, u, 50.f) : type == kEvGold ? fmaf(290.f, u, 10.f)
                    : type == kEvFarm ? fmaf(9.f, u, 1.f) : type == kEvHeal ? fmaf(480.f, u, 20.f) : 1.f;
  out[0] = event_meta(slot, type, m_local);
  union { float f; int32_t i; } v;
  v.f = value;
  out[1] = v.i;
}

}  // namespace ana
