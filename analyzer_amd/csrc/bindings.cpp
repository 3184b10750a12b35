// PyTorch bindings of the engine.  Device (ROCm) tensors run the gfx950
// kernels of kernels.hip on the current HIP stream; CPU tensors run the host
// mirror of host.cpp.  Every shape/dtype/device assumption a kernel makes is
// checked here, on the host, before anything is launched.
#include <torch/extension.h>

#include <cstdlib>
#include <ATen/hip/HIPContext.h>

#include <string>
#include <tuple>
#include <vector>

#include "common.h"
#include "gen_core.h"
#include "host.h"
#include "ingest.h"
#include "kernels.h"

namespace {

using torch::Tensor;

void check_hip(int err, const char* what) {
  TORCH_CHECK(err == 0, what, " failed: ", hipGetErrorString((hipError_t)err), " (", err, ")");
}

void check(const Tensor& t, const char* name, torch::ScalarType dt, const torch::Device& dev) {
  TORCH_CHECK(t.defined(), name, " is undefined");
  TORCH_CHECK(t.scalar_type() == dt, name, " must be ", c10::toString(dt), ", got ",
              c10::toString(t.scalar_type()));
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.device() == dev, name, " is on ", t.device(), " but expected ", dev);
}

// strided output views: rows of `inner` contiguous elements, any row stride
int64_t check_rows_view(const Tensor& t, const char* name, torch::ScalarType dt,
                        const torch::Device& dev, int64_t rows, int64_t inner) {
  TORCH_CHECK(t.defined(), name, " is undefined");
  TORCH_CHECK(t.scalar_type() == dt, name, " must be ", c10::toString(dt));
  TORCH_CHECK(t.device() == dev, name, " is on ", t.device(), " but expected ", dev);
  if (inner == 1) {
    TORCH_CHECK(t.dim() == 1 && t.size(0) == rows, name, " must have ", rows, " entries");
    return rows > 1 ? t.stride(0) : 1;
  }
  TORCH_CHECK(t.dim() == 2 && t.size(0) == rows && t.size(1) == inner, name, " must be [", rows,
              ", ", inner, "]");
  TORCH_CHECK(t.stride(1) == 1 && (rows <= 1 || t.stride(0) >= inner), name,
              " rows must be contiguous and non-overlapping");
  return rows > 1 ? t.stride(0) : inner;
}

hipStream_t stream_of(const Tensor& t) {
  return at::hip::getCurrentHIPStream(t.device().index()).stream();
}

uint32_t u32(int64_t v, const char* name) {
  TORCH_CHECK(v >= 0 && v <= 0xffffffffLL, name, " must fit in uint32");
  return (uint32_t)v;
}

// --------------------------------------------------------------------- K7
void gen_roster(Tensor state, Tensor attrs, int64_t seed, int64_t p_tier_null, int64_t p_tier_bad,
                int64_t p_rp_ranked, int64_t p_rp_blitz, int64_t p_rated, int64_t p_mode_rated,
                double mu_lo, double mu_span, double sig_lo, double sig_span) {
  const auto dev = state.device();
  check(state, "state", torch::kFloat32, dev);
  check(attrs, "attrs", torch::kFloat32, dev);
  TORCH_CHECK(state.dim() == 2 && state.size(1) == ana::kRowFloats, "state must be [P, 32]");
  TORCH_CHECK(attrs.dim() == 2 && attrs.size(1) == 4 && attrs.size(0) == state.size(0),
              "attrs must be [P, 4]");
  ana::GenRosterParams g{};
  g.seed = (uint64_t)seed;
  g.num_players = state.size(0);
  g.p_tier_null = u32(p_tier_null, "p_tier_null");
  g.p_tier_bad = u32(p_tier_bad, "p_tier_bad");
  g.p_rp_ranked = u32(p_rp_ranked, "p_rp_ranked");
  g.p_rp_blitz = u32(p_rp_blitz, "p_rp_blitz");
  g.p_rated = u32(p_rated, "p_rated");
  g.p_mode_rated = u32(p_mode_rated, "p_mode_rated");
  g.mu_lo = (float)mu_lo;
  g.mu_span = (float)mu_span;
  g.sig_lo = (float)sig_lo;
  g.sig_span = (float)sig_span;
  if (dev.is_cuda()) {
    check_hip(ana::launch_gen_roster(g, state.data_ptr<float>(), attrs.data_ptr<float>(),
                                     stream_of(state)), "gen_roster");
  } else {
    ana::host_gen_roster(g, state.data_ptr<float>(), attrs.data_ptr<float>());
  }
}

void gen_stream(Tensor rec, int64_t K, int64_t seed, int64_t base, int64_t num_players,
                int64_t team_size, std::vector<int64_t> mode_cdf, int64_t p_uneven,
                int64_t p_bad_rosters, int64_t p_tie, int64_t p_afk, int64_t p_hot,
                int64_t hot_players, int64_t skew) {
  const auto dev = rec.device();
  check(rec, "rec", torch::kInt32, dev);
  TORCH_CHECK(K >= 1 && K <= 5, "K (players per roster slot block) must be 1..5");
  TORCH_CHECK(rec.dim() == 2 && rec.size(1) == 2 * K + 2, "rec must be [M, 2K+2]");
  TORCH_CHECK(team_size >= 1 && team_size <= K, "team_size must be in 1..K");
  TORCH_CHECK(num_players >= 1 && num_players < 0x7fffffffLL, "num_players out of range");
  TORCH_CHECK(hot_players >= 1 && hot_players <= num_players, "hot_players must be 1..num_players");
  TORCH_CHECK(mode_cdf.size() == 7, "mode_cdf must have 7 thresholds");
  TORCH_CHECK(skew >= 1 && skew <= 8, "skew must be 1..8");
  ana::GenStreamParams g{};
  g.seed = (uint64_t)seed;
  g.base = base;
  g.num_players = num_players;
  g.team_size = (int32_t)team_size;
  g.skew = (int32_t)skew;
  for (int k = 0; k < 7; ++k) g.mode_cdf[k] = u32(mode_cdf[k], "mode_cdf");
  g.p_uneven = u32(p_uneven, "p_uneven");
  g.p_bad_rosters = u32(p_bad_rosters, "p_bad_rosters");
  g.p_tie = u32(p_tie, "p_tie");
  g.p_afk = u32(p_afk, "p_afk");
  g.p_hot = u32(p_hot, "p_hot");
  g.hot_players = u32(hot_players, "hot_players");
  const int64_t M = rec.size(0);
  if (dev.is_cuda()) {
    check_hip(ana::launch_gen_stream((int)K, g, rec.data_ptr<int32_t>(), M, stream_of(rec)),
              "gen_stream");
  } else {
    TORCH_CHECK(ana::host_gen_stream((int)K, g, rec.data_ptr<int32_t>(), M) == 0, "bad K");
  }
}

// --------------------------------------------------------------------- K5
int64_t schedule_workspace_bytes(int64_t nslots, int64_t num_players) {
  return (int64_t)ana::schedule_workspace_bytes(nslots, num_players);
}

// Stable sort of int32 (key, value) pairs by the low ``bits`` key bits on the
// device (the K5 radix sort, exposed for tests and tools).  Returns new tensors.
std::vector<Tensor> sort_pairs(Tensor keys, Tensor vals, int64_t bits) {
  const auto dev = keys.device();
  TORCH_CHECK(dev.is_cuda(), "sort_pairs runs on the device");
  check(keys, "keys", torch::kInt32, dev);
  check(vals, "vals", torch::kInt32, dev);
  const int64_t n = keys.numel();
  TORCH_CHECK(vals.numel() == n, "keys and vals must have the same length");
  TORCH_CHECK(bits >= 1 && bits <= 32, "bits must be 1..32");
  auto ka = keys.clone(), va = vals.clone();
  auto kb = torch::empty_like(ka), vb = torch::empty_like(va);
  auto ws = torch::empty({(int64_t)ana::radix_sort_workspace_bytes(n)},
                         keys.options().dtype(torch::kUInt8));
  int in_alt = 0;
  auto u = [](Tensor& t) { return reinterpret_cast<uint32_t*>(t.data_ptr<int32_t>()); };
  check_hip(ana::launch_radix_sort_pairs(u(ka), u(va), u(kb), u(vb), n, (int)bits,
                                         ws.data_ptr<uint8_t>(), &in_alt, stream_of(keys)),
            "sort_pairs");
  return in_alt ? std::vector<Tensor>{kb, vb} : std::vector<Tensor>{ka, va};
}

// K5 host levelizer (conflict-free rounds for the exact DP mode).
std::tuple<Tensor, int64_t> levels(Tensor rec, int64_t K, int64_t num_players) {
  TORCH_CHECK(!rec.is_cuda(), "levels runs on the host (pass a CPU stream)");
  check(rec, "rec", torch::kInt32, rec.device());
  TORCH_CHECK(K >= 1 && K <= 5, "K must be 1..5");
  TORCH_CHECK(rec.dim() == 2 && rec.size(1) == 2 * K + 2, "rec must be [M, 2K+2]");
  auto level = torch::empty({rec.size(0)}, rec.options());
  const int64_t depth = ana::host_levels((int)K, rec.data_ptr<int32_t>(), rec.size(0), num_players,
                                         level.data_ptr<int32_t>());
  return {level, depth};
}

// K5 device levelizer over a fresh schedule (its deps are consumed): (level [M], depth).
std::tuple<Tensor, int64_t> levels_device(Tensor rec, int64_t K, int64_t num_players, Tensor link,
                                          Tensor deps) {
  const auto dev = rec.device();
  TORCH_CHECK(dev.is_cuda(), "levels_device runs on the device (host: levels)");
  check(rec, "rec", torch::kInt32, dev);
  check(link, "link", torch::kInt32, dev);
  check(deps, "deps", torch::kInt32, dev);
  TORCH_CHECK(K >= 1 && K <= 5, "K must be 1..5");
  TORCH_CHECK(rec.dim() == 2 && rec.size(1) == 2 * K + 2, "rec must be [M, 2K+2]");
  const int64_t M = rec.size(0);
  TORCH_CHECK(link.dim() == 2 && link.size(0) == M && link.size(1) == 2 * K, "link must be [M, 2K]");
  TORCH_CHECK(deps.numel() == M, "deps must have M entries");
  TORCH_CHECK(M * 2 * K <= ana::kMaxSlots, "more than 2^28 slots in one window (split the stream)");
  TORCH_CHECK(num_players >= 1 && num_players < 0x7fffffffLL, "num_players out of range");
  auto level = torch::empty({M}, rec.options());
  auto pushed = torch::zeros({M}, rec.options());
  auto ctrl = torch::zeros({4}, rec.options());
  check_hip(ana::launch_levels((int)K, rec.data_ptr<int32_t>(),
                               reinterpret_cast<const uint32_t*>(link.data_ptr<int32_t>()),
                               deps.data_ptr<int32_t>(), pushed.data_ptr<int32_t>(),
                               level.data_ptr<int32_t>(), M, num_players,
                               reinterpret_cast<uint32_t*>(ctrl.data_ptr<int32_t>()), stream_of(rec)),
            "levels");
  const auto c = ctrl.cpu();
  TORCH_CHECK(c[3].item<int32_t>() == 0,
              "device levelizer made no progress for 5 s (schedule and stream disagree)");
  return {level, (int64_t)c[2].item<int32_t>()};
}

void schedule(Tensor rec, int64_t K, int64_t num_players, Tensor link, Tensor deps,
              Tensor workspace, Tensor ctrl, bool zero_ctrl, int64_t epoch_bump_ptr, int64_t sort_nt) {
  const auto dev = rec.device();
  check(rec, "rec", torch::kInt32, dev);
  check(link, "link", torch::kInt32, dev);
  check(deps, "deps", torch::kInt32, dev);
  TORCH_CHECK(K >= 1 && K <= 5, "K must be 1..5");
  TORCH_CHECK(rec.dim() == 2 && rec.size(1) == 2 * K + 2, "rec must be [M, 2K+2]");
  const int64_t M = rec.size(0);
  TORCH_CHECK(link.dim() == 2 && link.size(0) == M && link.size(1) == 2 * K, "link must be [M, 2K]");
  TORCH_CHECK(deps.numel() == M, "deps must have M entries");
  TORCH_CHECK(num_players >= 1 && num_players < 0x7fffffffLL, "num_players out of range");
  TORCH_CHECK(M * 2 * K <= ana::kMaxSlots, "more than 2^28 slots in one window (split the stream)");
  if (dev.is_cuda()) {
    check(workspace, "workspace", torch::kUInt8, dev);
    check(ctrl, "ctrl", torch::kInt32, dev);
    TORCH_CHECK(ctrl.numel() >= 52, "ctrl must have 52 entries");
    const size_t need = ana::schedule_workspace_bytes(M * 2 * K, num_players);
    TORCH_CHECK((size_t)workspace.numel() >= need, "workspace too small: need ", need, " bytes");
    check_hip(ana::launch_schedule((int)K, rec.data_ptr<int32_t>(), M, num_players,
                                   reinterpret_cast<uint32_t*>(link.data_ptr<int32_t>()),
                                   deps.data_ptr<int32_t>(), workspace.data_ptr<uint8_t>(),
                                   (size_t)workspace.numel(),
                                   reinterpret_cast<uint32_t*>(ctrl.data_ptr<int32_t>()),
                                   stream_of(rec), zero_ctrl,
                                   reinterpret_cast<int32_t*>((intptr_t)epoch_bump_ptr), (int)sort_nt),
              "schedule");
  } else {
    TORCH_CHECK(ana::host_schedule((int)K, rec.data_ptr<int32_t>(), M, num_players,
                                   reinterpret_cast<uint32_t*>(link.data_ptr<int32_t>()),
                                   deps.data_ptr<int32_t>()) == 0,
                "bad K");
  }
}

// knobs (EngineConfig, config.py): [rate_idle, rate_local, rate_diag, rate_tight,
// tele_fused_tail, tele_role] -- executor / fused-telemetry tuning, per BatchRater
constexpr size_t kKnobs = 6;

static ana::TelemetryParams telemetry_params(const Tensor& evoff, const Tensor& events,
                                             const Tensor& stats, int64_t M, int64_t K,
                                             const torch::Device& dev, const std::vector<int64_t>& knobs) {
  ana::TelemetryParams tp{nullptr, nullptr, nullptr, M};
  if (evoff.numel() == 0) return tp;
  check(evoff, "evoff", torch::kInt64, dev);
  check(events, "events", torch::kInt32, dev);
  check(stats, "stats", torch::kFloat32, dev);
  TORCH_CHECK(evoff.numel() == M + 1, "evoff must have M + 1 entries");
  TORCH_CHECK(events.dim() == 2 && events.size(1) == 2, "events must be [E, 2] (8-B events, telemetry_core.h)");
  TORCH_CHECK(stats.numel() == M * 2 * K * ana::kStatFeatures, "stats must be [M, 2K, 8]");
  tp.evoff = evoff.data_ptr<int64_t>();
  tp.events = events.data_ptr<int32_t>();
  tp.stats = stats.data_ptr<float>();
  if (dev.is_cuda()) tp.impl = ana::tele_impl();
  tp.fused_tail = (int32_t)knobs[4];
  // fused: < 0 inline in the rating groups (default, 11.4 ms per config 4 step); N > 0 one wave
  // in N aggregates tiles first (N = 2: 14.4 -> 11.4-11.7 ms, profiles/r2/tele_role_split.log)
  tp.role_stride = (int32_t)knobs[5];
  return tp;
}

// ------------------------------------------------------------ K1-K4, K6
void rate(Tensor rec, int64_t K, Tensor link, Tensor deps, Tensor state, Tensor attrs,
          Tensor first_prior, Tensor quality, Tensor status, Tensor s_mu, Tensor s_sig,
          Tensor delta, Tensor m_mu, Tensor m_sig, Tensor ctrl, Tensor vst, double beta2,
          double tau2, double unknown_sigma, bool record_first_prior, int64_t blocks,
          int64_t epoch, bool host_fp64, Tensor tele_evoff, Tensor tele_events, Tensor tele_stats,
          int64_t progress, int64_t progress_value, int64_t progress_at, int64_t epoch_ptr,
          int64_t chunk_len, bool ctrl_ready, std::vector<int64_t> knobs) {
  const auto dev = rec.device();
  TORCH_CHECK(knobs.size() == kKnobs, "knobs must be [idle, local, diag, tight, tele_fused_tail, tele_role]");
  check(rec, "rec", torch::kInt32, dev);
  check(state, "state", torch::kFloat32, dev);
  check(attrs, "attrs", torch::kFloat32, dev);

  check(vst, "vst", torch::kFloat32, dev);
  TORCH_CHECK(K >= 1 && K <= 5, "K must be 1..5");
  TORCH_CHECK(rec.dim() == 2 && rec.size(1) == 2 * K + 2, "rec must be [M, 2K+2]");
  const int64_t M = rec.size(0);
  const int64_t S = 2 * K;
  TORCH_CHECK(state.dim() == 2 && state.size(1) == ana::kRowFloats, "state must be [P, 32]");
  const int64_t P = state.size(0);
  TORCH_CHECK(P >= 1 && P * ana::kRowFloats * 4 < 0x7fffffffLL,
              "roster size out of range (<= 16.7M players per device roster)");
  TORCH_CHECK(attrs.dim() == 2 && attrs.size(0) == P && attrs.size(1) == 4, "attrs must be [P, 4]");
  const int64_t qrow = check_rows_view(quality, "quality", torch::kFloat32, dev, M, 1);
  const int64_t srow = check_rows_view(status, "status", torch::kUInt8, dev, M, 1);
  const int64_t row = check_rows_view(s_mu, "s_mu", torch::kFloat32, dev, M, S);
  for (const Tensor* t : {&s_sig, &delta, &m_mu, &m_sig})
    TORCH_CHECK(check_rows_view(*t, "per-slot output", torch::kFloat32, dev, M, S) == row,
                "per-slot outputs must share one row stride");
  TORCH_CHECK(vst.numel() == ana::kVstTiers, "vst must have 31 entries (tiers -1..29)");
  float* fp = nullptr;
  if (record_first_prior) {
    check(first_prior, "first_prior", torch::kFloat32, dev);
    TORCH_CHECK(first_prior.sizes() == state.sizes(), "first_prior must match state");
    fp = first_prior.data_ptr<float>();
  }
  ana::RateOut out{quality.data_ptr<float>(), status.data_ptr<uint8_t>(), s_mu.data_ptr<float>(),
                   s_sig.data_ptr<float>(), delta.data_ptr<float>(), m_mu.data_ptr<float>(),
                   m_sig.data_ptr<float>(), row, qrow, srow};
  ana::RateParams prm{};
  prm.beta2 = (float)beta2;
  prm.tau2 = (float)tau2;
  prm.unknown_sigma = (float)unknown_sigma;
  prm.num_players = (int32_t)P;
  prm.num_matches = M;
  prm.record_first_prior = record_first_prior ? 1 : 0;
  prm.epoch_ptr = reinterpret_cast<const int32_t*>((intptr_t)epoch_ptr);
  TORCH_CHECK(prm.epoch_ptr ? dev.is_cuda() : (epoch >= 1 && epoch <= 255), "epoch must be 1..255");
  prm.epoch = (int32_t)epoch;
  prm.vst = vst.data_ptr<float>();
  prm.idle_spins = (int32_t)knobs[0];
  prm.local_handoff = (int32_t)knobs[1];
  prm.diag = (int32_t)knobs[2];
  prm.tight_groups = (int32_t)knobs[3];
  prm.progress = reinterpret_cast<uint64_t*>((intptr_t)progress);
  prm.progress_value = (uint64_t)progress_value;
  prm.progress_at = progress_at;
  TORCH_CHECK(chunk_len >= 1 && chunk_len <= 64, "chunk_len must be 1..64");
  prm.chunk_len = (int32_t)chunk_len;
  prm.ctrl_ready = ctrl_ready ? 1 : 0;
  const ana::TelemetryParams tp = telemetry_params(tele_evoff, tele_events, tele_stats, M, K, dev, knobs);
  if (dev.is_cuda()) {
    check(link, "link", torch::kInt32, dev);
    check(deps, "deps", torch::kInt32, dev);
    check(ctrl, "ctrl", torch::kInt32, dev);
    TORCH_CHECK(link.numel() == M * S * ana::kLinkWords, "link must be [M, 2K]");
    TORCH_CHECK(deps.numel() == M, "deps must have M entries");
    TORCH_CHECK(ctrl.numel() >= 52, "ctrl must have 52 entries");
    TORCH_CHECK(blocks >= 1 && blocks <= 65535, "blocks must be 1..65535");
    // the executor writes packed rows; other layouts go through a packed buffer
    const bool packed = out.s_sig == out.s_mu + S && out.delta == out.s_mu + 2 * S &&
                        out.m_mu == out.s_mu + 3 * S && out.m_sig == out.s_mu + 4 * S &&
                        out.quality == out.s_mu + 5 * S && qrow == row &&
                        (void*)out.status == (void*)(out.s_mu + 5 * S + 1) && srow == row * 4;
    Tensor staged;
    if (!packed) {
      const int64_t W = (5 * S + 2 + 31) / 32 * 32;
      staged = torch::empty({M, W}, state.options());
      float* b = staged.data_ptr<float>();
      out = ana::RateOut{b + 5 * S, reinterpret_cast<uint8_t*>(b + 5 * S + 1), b, b + S, b + 2 * S,
                         b + 3 * S, b + 4 * S, W, W, W * 4};
    }
    const int rc = ana::launch_rate((int)K, rec.data_ptr<int32_t>(),
                                    reinterpret_cast<const uint32_t*>(link.data_ptr<int32_t>()),
                                    deps.data_ptr<int32_t>(), state.data_ptr<float>(),
                                    attrs.data_ptr<float>(), fp, out,
                                    reinterpret_cast<uint32_t*>(ctrl.data_ptr<int32_t>()), prm, tp,
                                    (int)blocks, stream_of(rec));
    check_hip(rc, "rate");
    if (!packed) {
      using torch::indexing::Slice;
      s_mu.copy_(staged.index({Slice(), Slice(0, S)}));
      s_sig.copy_(staged.index({Slice(), Slice(S, 2 * S)}));
      delta.copy_(staged.index({Slice(), Slice(2 * S, 3 * S)}));
      m_mu.copy_(staged.index({Slice(), Slice(3 * S, 4 * S)}));
      m_sig.copy_(staged.index({Slice(), Slice(4 * S, 5 * S)}));
      quality.copy_(staged.index({Slice(), 5 * S}));
      status.copy_(staged.view(torch::kUInt8).index({Slice(), 4 * (5 * S + 1)}));
    }
    if (prm.progress)  // releases the waiter even if the launch ended without firing
      check_hip((int)hipStreamWriteValue64(stream_of(rec), prm.progress, prm.progress_value, 0),
                "hipStreamWriteValue64");
  } else {
    TORCH_CHECK(ana::host_rate((int)K, host_fp64, rec.data_ptr<int32_t>(), state.data_ptr<float>(),
                               attrs.data_ptr<float>(), fp, out, prm) == 0, "bad K");
    if (tp.evoff) ana::host_telemetry((int)K, tp);
  }
}

// ------------------------------------------------------------------ K8
Tensor gen_event_counts(int64_t M, int64_t seed, int64_t min_events, int64_t max_events,
                        int64_t base, torch::Device device) {
  TORCH_CHECK(min_events >= 0 && max_events >= min_events, "need 0 <= min_events <= max_events");
  ana::GenEventParams g{(uint64_t)seed, (int32_t)min_events, (int32_t)max_events};
  auto counts = torch::empty({M}, torch::TensorOptions().dtype(torch::kInt64).device(device));
  if (device.is_cuda())
    check_hip(ana::launch_gen_event_counts(g, base, M, counts.data_ptr<int64_t>(),
                                           at::hip::getCurrentHIPStream(device.index()).stream()),
              "gen_event_counts");
  else
    ana::host_gen_event_counts(g, base, M, counts.data_ptr<int64_t>());
  return counts;
}

void gen_events(Tensor rec, int64_t K, Tensor evoff, int64_t seed, int64_t min_events,
                int64_t max_events, int64_t base, Tensor events) {
  const auto dev = rec.device();
  check(rec, "rec", torch::kInt32, dev);
  check(evoff, "evoff", torch::kInt64, dev);
  check(events, "events", torch::kInt32, dev);
  TORCH_CHECK(K >= 1 && K <= 5 && rec.dim() == 2 && rec.size(1) == 2 * K + 2, "rec must be [M, 2K+2]");
  const int64_t M = rec.size(0);
  TORCH_CHECK(evoff.numel() == M + 1, "evoff must have M + 1 entries");
  TORCH_CHECK(events.dim() == 2 && events.size(1) == 2, "events must be [E, 2] (8-B events, telemetry_core.h)");
  ana::GenEventParams g{(uint64_t)seed, (int32_t)min_events, (int32_t)max_events};
  if (dev.is_cuda())
    check_hip(ana::launch_gen_events((int)K, g, base, rec.data_ptr<int32_t>(),
                                     evoff.data_ptr<int64_t>(), M, events.data_ptr<int32_t>(),
                                     stream_of(rec)), "gen_events");
  else
    TORCH_CHECK(ana::host_gen_events((int)K, g, base, rec.data_ptr<int32_t>(),
                                     evoff.data_ptr<int64_t>(), M, events.data_ptr<int32_t>()) == 0,
                "bad K");
}

// standalone aggregation; bad (device: int32[>=1] counter, host: ignored) counts malformed events
int64_t telemetry(Tensor evoff, Tensor events, int64_t K, Tensor stats, Tensor bad) {
  const auto dev = events.device();
  TORCH_CHECK(K >= 1 && K <= 5, "K must be 1..5");
  const int64_t M = evoff.numel() - 1;
  TORCH_CHECK(M >= 0, "evoff must have M + 1 entries");
  // standalone: the fused-executor knobs do not apply
  const ana::TelemetryParams tp = telemetry_params(evoff, events, stats, M, K, dev, {0, 1, 0, -1, 0, 2});
  if (!tp.evoff) return 0;
  if (dev.is_cuda()) {
    check(bad, "bad", torch::kInt32, dev);
    TORCH_CHECK(bad.numel() >= 1, "bad must have an entry");
    const int rc = ana::launch_telemetry((int)K, tp, reinterpret_cast<uint32_t*>(bad.data_ptr<int32_t>()),
                                         stream_of(events));
    TORCH_CHECK(rc != (int)hipErrorNotSupported,
                "ANA_TELE_DEBUG / ANA_TELE_SPAN select diagnostic telemetry variants, which only the "
                "diagnostic library has: python -m analyzer_amd.build_ext --diag, then "
                "ANA_NATIVE_LIB=<path of analyzer_amd/_C_diag*.so>");
    check_hip(rc, "telemetry");
    return -1;
  }
  return ana::host_telemetry((int)K, tp);
}

// ------------------------------------------------------------- K9 / C1
void check_rows(const Tensor& t, const char* name, int64_t P, int64_t cols, const torch::Device& dev,
                torch::ScalarType ty = torch::kFloat32) {
  check(t, name, ty, dev);
  TORCH_CHECK(t.dim() == 2 && t.size(0) == P && t.size(1) == cols, name, " must be [P, ", cols, "]");
}

// s0: common window start, prior: this rank's prior of the sweep (s0 itself in
// the first sweep), s: the posterior after the local shard
// K9 merge: s0 / prior / s2 are base rows [P, 16] = (mu, sigma) of the 8 granules
// (sweep_core.h kBaseFloats); s is the roster [P, 32]
void sweep_delta(Tensor s0, Tensor prior, Tensor s, Tensor attrs, Tensor vst, double unknown_sigma,
                 bool scaled, Tensor buf) {
  const auto dev = s.device();
  const int64_t P = s.size(0);
  check_rows(s0, "s0 (base rows)", P, ana::kBaseFloats, dev);
  check_rows(prior, "prior (base rows)", P, ana::kBaseFloats, dev);
  check_rows(s, "state", P, ana::kRowFloats, dev);
  check_rows(attrs, "attrs", P, 4, dev);
  check_rows(buf, "buf", P, 16, dev);
  check(vst, "vst", torch::kFloat32, dev);
  TORCH_CHECK(vst.numel() == ana::kVstTiers, "vst must have 31 entries");
  if (dev.is_cuda()) {
    check_hip(ana::launch_sweep_delta(s0.data_ptr<float>(), prior.data_ptr<float>(),
                                      s.data_ptr<float>(), attrs.data_ptr<float>(),
                                      vst.data_ptr<float>(), (float)unknown_sigma, scaled ? 1 : 0,
                                      buf.data_ptr<float>(), P, stream_of(s)), "sweep_delta");
  } else {
    ana::host_sweep_delta(s0.data_ptr<float>(), prior.data_ptr<float>(), s.data_ptr<float>(),
                          attrs.data_ptr<float>(), vst.data_ptr<float>(), (float)unknown_sigma,
                          scaled, buf.data_ptr<float>(), P);
  }
}

// clamps: int32 [1] (empty: not counted) += the decoded tracks whose merged precision
// hit the floor (sweep_core.h sweep_apply_track); the merger raises on it
static uint32_t* clamp_ptr(const c10::optional<Tensor>& c, const torch::Device& dev) {
  if (!c.has_value() || !c->defined() || c->numel() == 0) return nullptr;
  check(*c, "clamps", torch::kInt32, dev);
  return reinterpret_cast<uint32_t*>(c->data_ptr<int32_t>());
}

// decoded rows to s and, if s2 is non-empty, base rows [P, 16] (sweep_core.h) to s2
void sweep_apply(Tensor s0, Tensor buf, Tensor attrs, Tensor s, Tensor s2, Tensor vst,
                 double unknown_sigma, bool scaled, const c10::optional<Tensor>& clamps) {
  const auto dev = s.device();
  uint32_t* cl = clamp_ptr(clamps, dev);
  const int64_t P = s.size(0);
  check_rows(s0, "s0 (base rows)", P, ana::kBaseFloats, dev);
  check_rows(buf, "buf", P, 16, dev);
  check_rows(attrs, "attrs", P, 4, dev);
  check_rows(s, "state", P, ana::kRowFloats, dev);
  float* p2 = nullptr;
  if (s2.numel()) {
    check_rows(s2, "s2 (base rows)", P, ana::kBaseFloats, dev);
    p2 = s2.data_ptr<float>();
  }
  check(vst, "vst", torch::kFloat32, dev);
  TORCH_CHECK(vst.numel() == ana::kVstTiers, "vst must have 31 entries");
  if (dev.is_cuda()) {
    check_hip(ana::launch_sweep_apply(s0.data_ptr<float>(), buf.data_ptr<float>(),
                                      attrs.data_ptr<float>(), s.data_ptr<float>(), p2,
                                      vst.data_ptr<float>(), (float)unknown_sigma, scaled ? 1 : 0, P, cl,
                                      stream_of(s)), "sweep_apply");
  } else {
    ana::host_sweep_apply(s0.data_ptr<float>(), buf.data_ptr<float>(), attrs.data_ptr<float>(),
                          s.data_ptr<float>(), p2, scaled, vst.data_ptr<float>(),
                          (float)unknown_sigma, P, cl);
  }
}

// compressed merge operands: msg [P, 14] bf16/fp16, cnt [P, 1] int32 = the two base-16 touch
// fields packed as lo | hi << 16 (4 + 3 nibbles; sweep.hip); the CPU path goes through the
// fp32 host mirror and torch's conversions
// msg: [P, 14] rows with unit column stride and an even row stride (a separate [P, 14]
// tensor, or columns 0..13 of the split collective's [P, 16] operand rows); cnt: [P, 1] int32
// with any row stride (its own tensor, or word 7 of those rows)
static void check_operands(const Tensor& msg, const Tensor& cnt, int64_t P, const torch::Device& dev) {
  TORCH_CHECK(msg.device() == dev && msg.dim() == 2 && msg.size(0) == P && msg.size(1) == 14 &&
                  msg.stride(1) == 1 && msg.stride(0) % 2 == 0 &&
                  (msg.scalar_type() == torch::kBFloat16 || msg.scalar_type() == torch::kHalf),
              "msg must be [P, 14] bf16/fp16 rows (unit column stride, even row stride) on the state's device");
  TORCH_CHECK(cnt.device() == dev && cnt.scalar_type() == torch::kInt32 && cnt.dim() == 2 && cnt.size(0) == P &&
                  cnt.size(1) == 1,
              "cnt must be [P, 1] int32 on the state's device");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(msg.data_ptr()) % 4 == 0, "msg rows must be 4-B aligned");
}

static Tensor pack_touch(const Tensor& lohi) {  // [P, 2] float fields -> [P, 1] int32
  const Tensor x = lohi.to(torch::kInt32);
  return x.slice(1, 0, 1).bitwise_or(x.slice(1, 1, 2).bitwise_left_shift(16));
}
static Tensor unpack_touch(const Tensor& cnt) {  // [P, 1] int32 -> [P, 2] (lo, hi)
  return torch::cat({cnt.bitwise_and(0xffff), cnt.bitwise_right_shift(16)}, 1);
}
void sweep_delta_packed(Tensor s0, Tensor prior, Tensor s, Tensor attrs, Tensor vst, double unknown_sigma,
                        Tensor msg, Tensor cnt) {
  const auto dev = s.device();
  const int64_t P = s.size(0);
  check_rows(s0, "s0 (base rows)", P, ana::kBaseFloats, dev);
  check_rows(prior, "prior (base rows)", P, ana::kBaseFloats, dev);
  check_rows(s, "state", P, ana::kRowFloats, dev);
  check_rows(attrs, "attrs", P, 4, dev);
  check_operands(msg, cnt, P, dev);
  check(vst, "vst", torch::kFloat32, dev);
  TORCH_CHECK(vst.numel() == ana::kVstTiers, "vst must have 31 entries");
  if (dev.is_cuda()) {
    check_hip(ana::launch_sweep_delta_packed(s0.data_ptr<float>(), prior.data_ptr<float>(), s.data_ptr<float>(),
                                             attrs.data_ptr<float>(), vst.data_ptr<float>(), (float)unknown_sigma,
                                             msg.scalar_type() == torch::kBFloat16 ? 1 : 0, msg.data_ptr(),
                                             cnt.data_ptr<int32_t>(), P, stream_of(s), msg.stride(0) / 2,
                                             cnt.stride(0)),
              "sweep_delta_packed");
    return;
  }
  Tensor buf = torch::empty({P, 16}, s.options());
  ana::host_sweep_delta(s0.data_ptr<float>(), prior.data_ptr<float>(), s.data_ptr<float>(),
                        attrs.data_ptr<float>(), vst.data_ptr<float>(), (float)unknown_sigma, true,
                        buf.data_ptr<float>(), P);
  msg.copy_(buf.slice(1, 0, 14));
  cnt.copy_(pack_touch(buf.slice(1, 14, 16)));
}

void prefix_delta(Tensor s0, Tensor prefix, Tensor attrs, Tensor vst, double unknown_sigma, Tensor delta);

void sweep_apply_packed(Tensor s0, Tensor msg, Tensor cnt, Tensor attrs, Tensor s, Tensor s2, Tensor vst,
                        double unknown_sigma, const c10::optional<Tensor>& clamps,
                        const c10::optional<Tensor>& prefix, const c10::optional<Tensor>& delta) {
  const auto dev = s.device();
  uint32_t* cl = clamp_ptr(clamps, dev);
  const int64_t P = s.size(0);
  check_rows(s0, "s0 (base rows)", P, ana::kBaseFloats, dev);
  check_operands(msg, cnt, P, dev);
  check_rows(attrs, "attrs", P, 4, dev);
  check_rows(s, "state", P, ana::kRowFloats, dev);
  float* p2 = nullptr;
  if (s2.numel()) {
    check_rows(s2, "s2 (base rows)", P, ana::kBaseFloats, dev);
    p2 = s2.data_ptr<float>();
  }
  check(vst, "vst", torch::kFloat32, dev);
  TORCH_CHECK(vst.numel() == ana::kVstTiers, "vst must have 31 entries");
  const bool with_prefix = prefix.has_value() && prefix->defined() && prefix->numel() > 0;
  if (with_prefix) {
    TORCH_CHECK(delta.has_value() && delta->defined(), "a prefix needs a delta table");
    TORCH_CHECK(prefix->scalar_type() == msg.scalar_type() && prefix->is_contiguous() && prefix->device() == dev &&
                    prefix->sizes() == msg.sizes(),
                "prefix must be a contiguous [P, 14] tensor of msg's type");
    check_rows(*delta, "delta", P, 16, dev);
  }
  if (dev.is_cuda()) {
    check_hip(ana::launch_sweep_apply_packed(s0.data_ptr<float>(), msg.data_ptr(), cnt.data_ptr<int32_t>(),
                                             msg.scalar_type() == torch::kBFloat16 ? 1 : 0,
                                             attrs.data_ptr<float>(), s.data_ptr<float>(), p2,
                                             vst.data_ptr<float>(), (float)unknown_sigma, P, cl,
                                             with_prefix ? prefix->data_ptr() : nullptr,
                                             with_prefix ? delta->data_ptr<float>() : nullptr, stream_of(s),
                                             msg.stride(0) / 2, cnt.stride(0)),
              "sweep_apply_packed");
    return;
  }
  if (with_prefix)  // (before the host decode: it overwrites the window start through s2)
    prefix_delta(s0, *prefix, attrs, vst, unknown_sigma, *delta);
  Tensor buf = torch::empty({P, 16}, s.options());
  buf.slice(1, 0, 14).copy_(msg);
  buf.slice(1, 14, 16).copy_(unpack_touch(cnt));
  ana::host_sweep_apply(s0.data_ptr<float>(), buf.data_ptr<float>(), attrs.data_ptr<float>(),
                        s.data_ptr<float>(), p2, true, vst.data_ptr<float>(), (float)unknown_sigma, P, cl);
}

// the split collective's owner reduce (sweep.hip): recv [N * blk, 8] int32 words of
// bf16 / fp16 halves + the touch word -> total [blk, 8] and, when given, the exclusive
// prefixes pref [N * blk, 7] (device tensors; the CPU path is parallel/comm.py)
void sweep_block_reduce(Tensor recv, int64_t N, bool bf16, Tensor total, const c10::optional<Tensor>& pref) {
  const auto dev = recv.device();
  TORCH_CHECK(dev.is_cuda(), "sweep_block_reduce: device tensors (the host path is parallel/comm.py)");
  check(recv, "recv", torch::kInt32, dev);
  check(total, "total", torch::kInt32, dev);
  TORCH_CHECK(N >= 1 && recv.dim() == 2 && recv.size(1) == 8 && recv.size(0) % N == 0, "recv must be [N * blk, 8]");
  const int64_t blk = recv.size(0) / N;
  TORCH_CHECK(total.dim() == 2 && total.size(0) == blk && total.size(1) == 8, "total must be [blk, 8]");
  int32_t* pp = nullptr;
  if (pref.has_value() && pref->defined() && pref->numel()) {
    check(*pref, "pref", torch::kInt32, dev);
    TORCH_CHECK(pref->dim() == 2 && pref->size(0) == N * blk && pref->size(1) == 7, "pref must be [N * blk, 7]");
    pp = pref->data_ptr<int32_t>();
  }
  check_hip(ana::launch_sweep_block_reduce(recv.data_ptr<int32_t>(), (int)N, blk, bf16 ? 1 : 0,
                                           total.data_ptr<int32_t>(), pp, stream_of(recv)),
            "sweep_block_reduce");
}

// causal record correction of a window's records (parallel/sweep.py): rows = RateResult
// packed [M, row] += delta [P, 16] fp32 (raw natural-parameter increments per track)
void correct_records(Tensor rec, int64_t K, Tensor rows, Tensor delta) {
  const auto dev = rows.device();
  check(rec, "rec", torch::kInt32, dev);
  TORCH_CHECK(K >= 1 && K <= 5 && rec.dim() == 2 && rec.size(1) == 2 * K + 2, "rec must be [M, 2K+2]");
  const int64_t M = rec.size(0);
  TORCH_CHECK(rows.dim() == 2 && rows.size(0) == M && rows.scalar_type() == torch::kFloat32 && rows.stride(1) == 1 &&
                  rows.size(1) >= 5 * 2 * K + 2,
              "rows must be RateResult.packed [M, row] fp32");
  const int64_t P = delta.size(0);
  check_rows(delta, "delta", P, 16, dev);
  if (dev.is_cuda()) {
    check_hip(ana::launch_correct_records((int)K, rec.data_ptr<int32_t>(), M, rows.data_ptr<float>(), rows.stride(0),
                                          delta.data_ptr<float>(), P, stream_of(rows)),
              "correct_records");
    return;
  }
  ana::host_correct_records((int)K, rec.data_ptr<int32_t>(), M, rows.data_ptr<float>(), rows.stride(0),
                            delta.data_ptr<float>(), P);
}

// the record correction's delta table [P, 16] of a scaled (bf16 / fp16) prefix [P, 14]
// against the window start s0 [P, 16] (the fused decode computes it in production)
void prefix_delta(Tensor s0, Tensor prefix, Tensor attrs, Tensor vst, double unknown_sigma, Tensor delta) {
  const auto dev = s0.device();
  const int64_t P = s0.size(0);
  check_rows(s0, "s0 (base rows)", P, ana::kBaseFloats, dev);
  check_rows(attrs, "attrs", P, 4, dev);
  check_rows(delta, "delta", P, 16, dev);
  check(vst, "vst", torch::kFloat32, dev);
  TORCH_CHECK(prefix.device() == dev && prefix.is_contiguous() && prefix.dim() == 2 && prefix.size(0) == P &&
                  prefix.size(1) == 14 &&
                  (prefix.scalar_type() == torch::kBFloat16 || prefix.scalar_type() == torch::kHalf),
              "prefix must be a contiguous bf16 / fp16 [P, 14]");
  if (dev.is_cuda()) {
    check_hip(ana::launch_prefix_delta(s0.data_ptr<float>(), prefix.data_ptr(),
                                       prefix.scalar_type() == torch::kBFloat16 ? 1 : 0, attrs.data_ptr<float>(),
                                       vst.data_ptr<float>(), (float)unknown_sigma, delta.data_ptr<float>(), P,
                                       stream_of(s0)),
              "prefix_delta");
    return;
  }
  Tensor pf = prefix.to(torch::kFloat32).contiguous();
  ana::host_prefix_delta(s0.data_ptr<float>(), pf.data_ptr<float>(), attrs.data_ptr<float>(), vst.data_ptr<float>(),
                         (float)unknown_sigma, delta.data_ptr<float>(), P);
}

// ------------------------------------------------------------- C2 exchange
// rec: the rank's slice of one round [m, 2K+2]; status: its per-match status
// (any row stride); out: [cap, 33] float entries, cap >= m * 2K
void pack_rows(Tensor rec, int64_t K, Tensor status, Tensor state, Tensor out) {
  const auto dev = state.device();
  check(rec, "rec", torch::kInt32, dev);
  check(state, "state", torch::kFloat32, dev);
  check(out, "out", torch::kFloat32, dev);
  TORCH_CHECK(K >= 1 && K <= 5 && rec.dim() == 2 && rec.size(1) == 2 * K + 2, "rec must be [m, 2K+2]");
  const int64_t m = rec.size(0);
  TORCH_CHECK(state.dim() == 2 && state.size(1) == ana::kRowFloats, "state must be [P, 32]");
  TORCH_CHECK(out.dim() == 2 && out.size(1) == 33 && out.size(0) >= m * 2 * K, "out must be [cap >= m*2K, 33]");
  const int64_t sstride = check_rows_view(status, "status", torch::kUInt8, dev, m, 1);
  const int64_t P = state.size(0);
  if (dev.is_cuda()) {
    check_hip(ana::launch_pack_rows(rec.data_ptr<int32_t>(), (int)K, m, status.data_ptr<uint8_t>(), sstride,
                                    state.data_ptr<float>(), out.data_ptr<float>(), out.size(0),
                                    stream_of(state)), "pack_rows");
    return;
  }
  const int S = 2 * (int)K;
  const int32_t* r = rec.data_ptr<int32_t>();
  const uint8_t* st = status.data_ptr<uint8_t>();
  const float* sp = state.data_ptr<float>();
  float* o = out.data_ptr<float>();
  for (int64_t e = 0; e < out.size(0); ++e) {
    int32_t id = -1;
    if (e < m * S) {
      const int64_t i = e / S;
      const int j = (int)(e % S);
      const uint32_t m0 = (uint32_t)r[i * (S + 2) + S];
      const int n = j < K ? (int)ana::meta_n0(m0) : (int)ana::meta_n1(m0);
      const int32_t v = r[i * (S + 2) + j];
      if (st[i * sstride] == ana::kRated && (j < K ? j : j - K) < n && v >= 0 && v < P) id = v;
    }
    if (id >= 0)
      for (int k = 0; k < ana::kRowFloats; ++k) o[e * 33 + k] = sp[(int64_t)id * ana::kRowFloats + k];
    int32_t* oi = reinterpret_cast<int32_t*>(o + e * 33 + 32);
    *oi = id;
  }
}

// C2 race detector: rec [M, 2K+2] (the window), idx int64 [m] (one round's matches),
// owner int64 [P] (zeroed once per window), flag int32 [1]
void check_round(Tensor rec, int64_t K, Tensor idx, int64_t round, Tensor owner, Tensor flag) {
  const auto dev = rec.device();
  check(rec, "rec", torch::kInt32, dev);
  check(idx, "idx", torch::kInt64, dev);
  check(owner, "owner", torch::kInt64, dev);
  check(flag, "flag", torch::kInt32, dev);
  TORCH_CHECK(K >= 1 && K <= 5 && rec.dim() == 2 && rec.size(1) == 2 * K + 2, "rec must be [M, 2K+2]");
  TORCH_CHECK(round >= 0 && round < 0xffffffffLL, "round out of range");
  const int64_t m = idx.numel(), P = owner.numel();
  if (dev.is_cuda()) {
    check_hip(ana::launch_check_round(rec.data_ptr<int32_t>(), (int)K, idx.data_ptr<int64_t>(), m, P,
                                      (uint32_t)round,
                                      reinterpret_cast<unsigned long long*>(owner.data_ptr<int64_t>()),
                                      reinterpret_cast<uint32_t*>(flag.data_ptr<int32_t>()), stream_of(rec)),
              "check_round");
    return;
  }
  const int S = 2 * (int)K;
  const int32_t* rp = rec.data_ptr<int32_t>();
  const int64_t* ip = idx.data_ptr<int64_t>();
  uint64_t* own = reinterpret_cast<uint64_t*>(owner.data_ptr<int64_t>());
  int32_t* fl = flag.data_ptr<int32_t>();
  for (int64_t i = 0; i < m; ++i) {
    const int32_t* r = rp + ip[i] * (S + 2);
    if (ana::early_status_k(r, S, P) != ana::kRated) continue;
    const uint32_t m0 = (uint32_t)r[S];
    const uint64_t mine = ((uint64_t)(round + 1) << 32) | (uint64_t)(ip[i] + 1);
    for (int j = 0; j < S; ++j) {
      const int n = j < K ? (int)ana::meta_n0(m0) : (int)ana::meta_n1(m0);
      const int32_t p = r[j];
      if ((j < K ? j : j - K) >= n || p < 0 || p >= P) continue;
      if ((uint32_t)(own[p] >> 32) == (uint32_t)(round + 1)) {
        if (own[p] != mine) fl[0] |= 1;
      } else {
        own[p] = mine;
      }
    }
  }
}

void unpack_rows(Tensor buf, Tensor state) {
  const auto dev = state.device();
  check(buf, "buf", torch::kFloat32, dev);
  check(state, "state", torch::kFloat32, dev);
  TORCH_CHECK(buf.dim() == 2 && buf.size(1) == 33, "buf must be [n, 33]");
  TORCH_CHECK(state.dim() == 2 && state.size(1) == ana::kRowFloats, "state must be [P, 32]");
  const int64_t n = buf.size(0), P = state.size(0);
  if (dev.is_cuda()) {
    check_hip(ana::launch_unpack_rows(buf.data_ptr<float>(), n, state.data_ptr<float>(), stream_of(state)),
              "unpack_rows");
    return;
  }
  const float* b = buf.data_ptr<float>();
  float* sp = state.data_ptr<float>();
  for (int64_t e = 0; e < n; ++e) {
    const int32_t id = *reinterpret_cast<const int32_t*>(b + e * 33 + 32);
    if (id < 0 || id >= P) continue;
    for (int k = 0; k < ana::kRowFloats; ++k) sp[(int64_t)id * ana::kRowFloats + k] = (k & 1) ? 0.f : b[e * 33 + k];
  }
}

// A HIP stream restricted to ``num_cus`` compute units, spread evenly over the
// device's CUs (and so over its XCDs).  Used for the schedule prepass so its
// bandwidth-bound kernels trickle alongside the latency-bound executor instead
// of bursting.  Returns the raw handle for torch.cuda.ExternalStream; the
// stream lives until process exit (one per pipeline).
int64_t cu_masked_stream(int64_t device, int64_t num_cus, bool invert) {
  hipDeviceProp_t prop;
  check_hip((int)hipGetDeviceProperties(&prop, (int)device), "hipGetDeviceProperties");
  const int total = prop.multiProcessorCount;
  TORCH_CHECK(num_cus >= 1 && num_cus <= total, "num_cus must be 1..", total);
  std::vector<uint32_t> mask((total + 31) / 32, 0u);
  for (int64_t i = 0; i < num_cus; ++i) {
    const int cu = (int)(i * total / num_cus);
    mask[cu / 32] |= 1u << (cu % 32);
  }
  if (invert) {  // every CU but those N (the complement of the same call without invert)
    for (int c = 0; c < total; ++c) mask[c / 32] ^= 1u << (c % 32);
    TORCH_CHECK(num_cus < total, "an inverted mask needs num_cus < ", total);
  }
  int prev = 0;
  check_hip((int)hipGetDevice(&prev), "hipGetDevice");
  check_hip((int)hipSetDevice((int)device), "hipSetDevice");
  hipStream_t st = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data());
  check_hip((int)hipSetDevice(prev), "hipSetDevice");
  check_hip((int)e, "hipExtStreamCreateWithCUMask");
  return (int64_t)reinterpret_cast<intptr_t>(st);
}

// Tail overlap (runtime/engine.py): an 8-B word in signal memory that the
// executor stores its launch number to when the launch reaches its tail, and a
// stream wait on it.  The handle is the device address (lives until exit).
int64_t progress_signal(int64_t device) {
  int prev = 0;
  check_hip((int)hipGetDevice(&prev), "hipGetDevice");
  check_hip((int)hipSetDevice((int)device), "hipSetDevice");
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, 8, hipMallocSignalMemory);
  if (e == hipSuccess) e = hipMemset(p, 0, 8);
  check_hip((int)hipSetDevice(prev), "hipSetDevice");
  check_hip((int)e, "hipExtMallocWithFlags(hipMallocSignalMemory)");
  return (int64_t)reinterpret_cast<intptr_t>(p);
}

void stream_wait_value64(int64_t stream, int64_t ptr, int64_t value) {
  check_hip((int)hipStreamWaitValue64(reinterpret_cast<hipStream_t>((intptr_t)stream),
                                      reinterpret_cast<void*>((intptr_t)ptr), (uint64_t)value,
                                      hipStreamWaitValueGte),
            "hipStreamWaitValue64");
}

// the host side of a tail gate: write ``value`` to the signal word in stream order (releases
// waiters whose launch will not come, runtime/engine.py)
void stream_write_value64(int64_t stream, int64_t ptr, int64_t value) {
  check_hip((int)hipStreamWriteValue64(reinterpret_cast<hipStream_t>((intptr_t)stream),
                                       reinterpret_cast<void*>((intptr_t)ptr), (uint64_t)value, 0),
            "hipStreamWriteValue64");
}

bool can_wait_value(int64_t device) {
  int v = 0;
  return hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, (int)device) ==
             hipSuccess && v != 0;
}

// ------------------------------------------------------------------ ingest (P3)
void write_record_file(const std::string& path, Tensor rec, int64_t K) {
  check(rec, "rec", torch::kInt32, torch::Device(torch::kCPU));
  TORCH_CHECK(rec.dim() == 2 && rec.size(1) == 2 * K + 2, "rec must be [M, 2K+2]");
  ana::write_record_file(path, rec.data_ptr<int32_t>(), rec.size(0), (int)K);
}

static py::object reader_acquire(ana::RecordReader& r) {
  int slot = 0;
  int64_t base = 0, n = 0;
  bool ok;
  {
    py::gil_scoped_release nogil;  // the producer thread may still be reading
    ok = r.acquire(&slot, &base, &n);
  }
  if (!ok) return py::none();
  auto t = torch::from_blob(r.slot_data(slot), {n, 2 * (int64_t)r.K() + 2},
                            torch::TensorOptions().dtype(torch::kInt32));
  return py::make_tuple(slot, base, t);
}

void epoch_bump(Tensor e) {
  TORCH_CHECK(e.is_cuda() && e.scalar_type() == torch::kInt32 && e.numel() >= 1, "epoch must be a device int32 tensor");
  check_hip(ana::launch_epoch_bump(e.data_ptr<int32_t>(), stream_of(e)), "epoch_bump");
}

// the all-reduce stand-in of one-GPU DP pricing (kernels.hip emulate_allreduce_kernel)
void emulate_allreduce(Tensor buf, int64_t channels, int64_t passes, double us) {
  TORCH_CHECK(buf.is_cuda() && buf.is_contiguous(), "emulate_allreduce: a contiguous device tensor");
  check_hip(ana::launch_emulate_allreduce(buf.data_ptr(), (int64_t)(buf.numel() * buf.element_size()), (int)channels,
                                          (int)passes, us, stream_of(buf)),
            "emulate_allreduce");
}

void warm_rows(Tensor state, Tensor sink) {
  const auto dev = state.device();
  check(state, "state", torch::kFloat32, dev);
  check(sink, "sink", torch::kInt32, dev);
  TORCH_CHECK(state.dim() == 2 && state.size(1) == ana::kRowFloats, "state must be [P, 32]");
  TORCH_CHECK(sink.numel() >= 256, "sink needs 256 words");
  if (!dev.is_cuda()) return;  // nothing to warm on the host
  check_hip(ana::launch_warm_rows(state.data_ptr<float>(), state.size(0),
                                  reinterpret_cast<uint32_t*>(sink.data_ptr<int32_t>()), stream_of(state)),
            "warm_rows");
}

// runtime/rerate.py window digest of the packed output rows (digest.hip); out [3 + 10K] fp64
void records_digest(Tensor rows, int64_t K, Tensor scratch, Tensor out, const c10::optional<Tensor>& hist) {
  const auto dev = rows.device();
  check(rows, "rows", torch::kFloat32, dev);
  check(scratch, "scratch", torch::kFloat64, dev);
  check(out, "out", torch::kFloat64, dev);
  TORCH_CHECK(K >= 1 && K <= 5, "records_digest: K in 1..5");
  TORCH_CHECK(rows.dim() == 2 && rows.size(1) >= 10 * K + 2 && rows.size(1) % 4 == 0 &&
                  256 % (rows.size(1) / 4) == 0,
              "records_digest: rows must be the packed [M, W] output rows (W / 4 a divisor of 256)");
  TORCH_CHECK(out.numel() == 3 + 10 * K, "records_digest: out needs 3 + 10K doubles");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(rows.data_ptr()) % 16 == 0, "records_digest: rows must be 16-B aligned");
  TORCH_CHECK(dev.is_cuda(), "records_digest: device rows (the host path is runtime/rerate.py window_digest)");
  TORCH_CHECK((size_t)scratch.numel() >= ana::records_digest_scratch_doubles((int)K), "records_digest: scratch too small");
  int64_t* h = nullptr;
  if (hist.has_value()) {
    check(*hist, "hist", torch::kInt64, dev);
    TORCH_CHECK(hist->numel() == 256, "records_digest: hist must be int64[256]");
    h = hist->data_ptr<int64_t>();
  }
  check_hip(ana::launch_records_digest((int)K, rows.data_ptr<float>(), rows.size(0), rows.size(1),
                                       scratch.data_ptr<double>(), out.data_ptr<double>(), h, stream_of(rows)),
            "records_digest");
}

int64_t records_digest_scratch(int64_t K) { return (int64_t)ana::records_digest_scratch_doubles((int)K); }

void reset_tags(Tensor state) {
  const auto dev = state.device();
  check(state, "state", torch::kFloat32, dev);
  TORCH_CHECK(state.dim() == 2 && state.size(1) == ana::kRowFloats, "state must be [P, 32]");
  if (dev.is_cuda()) {
    check_hip(ana::launch_reset_tags(state.data_ptr<float>(), state.size(0), stream_of(state)),
              "reset_tags");
  } else {
    float* p = state.data_ptr<float>();
    for (int64_t i = 0; i < state.numel(); i += 2) p[i + 1] = 0.f;
  }
}

}  // namespace

void register_batch_host(pybind11::module& m);      // batch_host.cpp
void register_telemetry_file(pybind11::module& m);  // telemetry_file.cpp

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  register_batch_host(m);
  register_telemetry_file(m);
  m.doc() = "analyzer_amd native engine: gfx950 HIP kernels + C++ host mirror";
  m.def("gen_roster", &gen_roster, "K7: synthetic roster (state [P,16], attrs [P,4])");
  m.def("gen_stream", &gen_stream, "K7: synthetic match stream rec [M, 2K+2]");
  m.def("schedule_workspace_bytes", &schedule_workspace_bytes);
  m.def("levels_device", &levels_device);
  m.def("sort_pairs", &sort_pairs, "stable LSD radix sort of int32 (key, value) pairs (device)");
  m.def("levels", &levels, "K5 host levelizer: per-match conflict-free round (0 = stateless)");
  m.def("schedule", &schedule, "K5: per-slot occurrence index (chronological order per player)");
  m.def("rate", &rate, "K1-K4/K6: exact dataflow rating of a stream");
  m.def("gen_event_counts", &gen_event_counts, "K8/K7: synthetic telemetry events per match");
  m.def("gen_events", &gen_events, "K8/K7: synthetic telemetry events (CSR by match)");
  m.def("telemetry", &telemetry, "K8: per-participant telemetry aggregation [M, 2K, 8]");
  m.attr("STAT_FEATURES") = ana::kStatFeatures;
  m.def("sweep_delta", &sweep_delta, "K9: per-rank natural-parameter messages for the DP merge");
  m.def("sweep_apply", &sweep_apply, "K9: decode summed messages against the common start (-> s, s2)",
        py::arg("s0"), py::arg("buf"), py::arg("attrs"), py::arg("s"), py::arg("s2"), py::arg("vst"),
        py::arg("unknown_sigma"), py::arg("scaled"), py::arg("clamps") = py::none());
  m.def("sweep_delta_packed", &sweep_delta_packed, "K9: messages straight into bf16/fp16 + int32 all-reduce operands");
  m.def("sweep_apply_packed", &sweep_apply_packed,
        "K9: decode bf16/fp16 + int32 summed messages (-> s, s2); with a prefix also the record-correction delta table",
        py::arg("s0"), py::arg("msg"), py::arg("cnt"), py::arg("attrs"), py::arg("s"), py::arg("s2"), py::arg("vst"),
        py::arg("unknown_sigma"), py::arg("clamps") = py::none(), py::arg("prefix") = py::none(),
        py::arg("delta") = py::none());
  m.def("correct_records", &correct_records,
        "K9: causal correction of a window's records: += the delta table of the earlier ranks' messages");
  m.def("sweep_block_reduce", &sweep_block_reduce, "K9: owner block sum (+ exclusive prefixes) of the split collective",
        py::arg("recv"), py::arg("N"), py::arg("bf16"), py::arg("total"), py::arg("pref") = py::none());
  m.def("prefix_delta", &prefix_delta, "K9: the record correction's delta table of a scaled message prefix");
  m.def("pack_rows", &pack_rows, "C2: changed rows of a round slice -> fixed-capacity [cap, 33] entries");
  m.def("check_round", &check_round, "C2 race detector: one round's matches share no player (flag |= 1)");
  m.def("unpack_rows", &unpack_rows, "C2: write gathered entries (id >= 0) into the roster, tags zeroed");
  m.def("write_record_file", &write_record_file, "P3: write a match-record file (ANAREC01)");
  py::class_<ana::RecordReader>(m, "RecordReader")
      .def(py::init<const std::string&, int64_t, int, bool>(), py::arg("path"), py::arg("window"),
           py::arg("slots") = 3, py::arg("pinned") = true)
      .def_property_readonly("K", &ana::RecordReader::K)
      .def_property_readonly("num_matches", &ana::RecordReader::num_matches)
      .def_property_readonly("window", &ana::RecordReader::window)
      .def_property_readonly("num_windows", &ana::RecordReader::num_windows)
      .def_property_readonly("pinned", &ana::RecordReader::pinned)
      .def("acquire", &reader_acquire,
           "next filled window as (slot, base, tensor view of pinned memory) or None at EOF")
      .def("release", &ana::RecordReader::release, "return the oldest acquired slot");
  m.def("cu_masked_stream", &cu_masked_stream, "HIP stream limited to N CUs (spread over XCDs), or to the others",
        py::arg("device"), py::arg("num_cus"), py::arg("invert") = false);
  m.def("progress_signal", &progress_signal, "8-B signal-memory word for the executor's tail signal");
  m.def("stream_wait_value64", &stream_wait_value64, "hipStreamWaitValue64(stream, ptr, >= value)");
  m.def("stream_write_value64", &stream_write_value64, "hipStreamWriteValue64(stream, ptr, value)");
  m.def("can_wait_value", &can_wait_value, "hipDeviceAttributeCanUseStreamWaitValue");
  m.def("reset_tags", &reset_tags, "zero the dataflow tags of a roster");
  m.def("records_digest", &records_digest, "deterministic fp64 digest of a window's packed output rows "
        "(+ its status counts added to hist)", py::arg("rows"), py::arg("K"), py::arg("scratch"),
        py::arg("out"), py::arg("hist") = py::none());
  m.def("records_digest_scratch", &records_digest_scratch, "scratch doubles of records_digest");
  m.def("emulate_allreduce", &emulate_allreduce,
        "DP pricing on one GPU: an all-reduce stand-in (buffer unchanged) on N CUs for >= us microseconds");
  m.def("warm_rows", &warm_rows, "read every roster row once (cache warm-up before a rating launch)");
  m.def("epoch_bump", &epoch_bump, "device launch epoch += 1 (graph replays)");
  m.attr("ROW_FLOATS") = ana::kRowFloats;
  m.attr("N_TRACKS") = ana::kTracks;
  m.attr("VST_TIERS") = ana::kVstTiers;
}
