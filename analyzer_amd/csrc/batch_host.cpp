// Native host path of the streaming worker's columnar batches (SURVEY W7/W8,
// runtime/columnar.py + runtime/resident.py).
//
// The reference rates a worker batch by walking ORM objects attribute by
// attribute (/root/reference/worker.py:169-199, rater.py:69-169).  Our worker
// moves a batch as columns, and at BATCHSIZE=500 the GPU part of a batch is
// ~50 us -- the cost is the host: a few dozen numpy calls per stage at 5-10 us
// each.  These four passes replace them with one O(batch) loop each:
//
//   batch_gather   store match rows -> batch columns (ColumnarSession.load_batch)
//   batch_encode   batch columns -> stream records [M, 2K+2] (csrc/common.h),
//                  resident-roster rows of the batch's players (new players get
//                  the next free rows; their stored ratings are fetched by the
//                  caller), and each slot's index into the batch's unique players
//   batch_finish   packed executor rows [M, W] + final player rows -> result
//                  columns (status, quality, 5 x [M, 2, K]) and the tracks the
//                  rated matches wrote per player
//   batch_commit   result columns -> the columnar store's numpy columns
//                  (ColumnarSession._write_batch)
//
// All tensors are CPU tensors (numpy arrays shared with torch.from_numpy); the
// Python side keeps the rare cases (rosters beyond the second) and the numpy
// fallback the tests compare against.
#include <torch/extension.h>

#include "key_index.h"

#include <stdint.h>

#include <cmath>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace {

using torch::Tensor;

constexpr int kRated = 0, kAfk = 1, kInvalid = 2;  // csrc/common.h status codes
constexpr int kTracks = 7;

void need(bool ok, const char* what) {
  if (!ok) throw std::invalid_argument(what);
}

template <typename T>
T* ptr(Tensor& t, torch::ScalarType ty, const char* name) {
  need(t.device().is_cpu() && t.scalar_type() == ty && t.is_contiguous(), name);
  return t.data_ptr<T>();
}

// ---------------------------------------------------------------- gather
std::vector<Tensor> batch_gather(Tensor rows, Tensor m_nr, Tensor m_r0, Tensor m_mode, Tensor r_np,
                                 Tensor r_winner, Tensor r_p0, Tensor p_player, Tensor p_afk) {
  const int64_t M = rows.numel();
  const int64_t* row = ptr<int64_t>(rows, torch::kInt64, "rows: int64");
  const int32_t* nr = ptr<int32_t>(m_nr, torch::kInt32, "m_nr: int32");
  const int64_t* r0 = ptr<int64_t>(m_r0, torch::kInt64, "m_r0: int64");
  const int16_t* md = ptr<int16_t>(m_mode, torch::kInt16, "m_mode: int16");
  const int32_t* rn = ptr<int32_t>(r_np, torch::kInt32, "r_np: int32");
  const int8_t* rw = ptr<int8_t>(r_winner, torch::kInt8, "r_winner: int8");
  const int64_t* rp = ptr<int64_t>(r_p0, torch::kInt64, "r_p0: int64");
  const int64_t* pp = ptr<int64_t>(p_player, torch::kInt64, "p_player: int64");
  const int8_t* pa = ptr<int8_t>(p_afk, torch::kInt8, "p_afk: int8");
  const int64_t nm = m_nr.numel(), nros = r_np.numel(), nparts = p_player.numel();
  int64_t K = 1;
  for (int64_t i = 0; i < M; ++i) {
    need(row[i] >= 0 && row[i] < nm, "batch_gather: match row out of range");
    for (int ri = 0; ri < 2 && ri < nr[row[i]]; ++ri) {
      const int64_t r = r0[row[i]] + ri;
      need(r >= 0 && r < nros, "batch_gather: roster row out of range");
      K = std::max<int64_t>(K, rn[r]);
    }
  }
  auto i64 = torch::TensorOptions().dtype(torch::kInt64);
  Tensor mode = torch::empty({M}, i64), nro = torch::empty({M}, i64), n = torch::zeros({M, 2}, i64);
  Tensor win = torch::zeros({M, 2}, torch::TensorOptions().dtype(torch::kBool));
  Tensor afk = torch::zeros({M}, i64);
  Tensor player = torch::full({M, 2, K}, -1, i64), part = torch::full({M, 2, K}, -1, i64);
  int64_t *o_mode = mode.data_ptr<int64_t>(), *o_nr = nro.data_ptr<int64_t>(), *o_n = n.data_ptr<int64_t>();
  bool* o_win = win.data_ptr<bool>();
  int64_t *o_afk = afk.data_ptr<int64_t>(), *o_pl = player.data_ptr<int64_t>(), *o_pt = part.data_ptr<int64_t>();
  for (int64_t i = 0; i < M; ++i) {
    const int64_t m = row[i];
    o_mode[i] = md[m];
    o_nr[i] = nr[m];
    int64_t mask = 0;
    int k = 0;  // participant ordinal over the first two rosters (AFK bit min(k, 23))
    for (int ri = 0; ri < nr[m]; ++ri) {
      const int64_t r = r0[m] + ri;
      need(r < nros, "batch_gather: roster row out of range");
      const int64_t p0 = rp[r], np_ = rn[r];
      need(p0 >= 0 && p0 + np_ <= nparts, "batch_gather: participant row out of range");
      if (ri >= 2) {  // rosters beyond the second: their AFKs set bit 23 only
        for (int64_t q = 0; q < np_; ++q)
          if (pa[p0 + q] == 1) mask |= int64_t(1) << 23;
        continue;
      }
      o_n[2 * i + ri] = np_;
      o_win[2 * i + ri] = rw[r] == 1;
      for (int64_t q = 0; q < np_; ++q, ++k) {
        const int64_t s = (i * 2 + ri) * K + q;
        o_pt[s] = p0 + q;
        o_pl[s] = pp[p0 + q];
        if (pa[p0 + q] == 1) mask |= int64_t(1) << std::min(k, 23);
      }
    }
    o_afk[i] = mask;
  }
  return {mode, nro, n, win, afk, player, part};
}

// ---------------------------------------------------------------- encode
// by_key (int64, mutable): store player key -> resident row, -1 = not resident.
// Keys not resident yet get rows next_row, next_row + 1, ... in first-seen
// order and are returned in new_keys (the caller uploads their stored ratings
// and resets by_key[new_keys] = -1 if that fails).
std::vector<Tensor> batch_encode(Tensor player, Tensor mode, Tensor n, Tensor nrosters, Tensor winner,
                                 Tensor afk, Tensor by_key, int64_t next_row) {
  need(player.dim() == 3 && player.size(1) == 2, "player: [M, 2, K]");
  const int64_t M = player.size(0), K = player.size(2), S = 2 * K, B = by_key.numel();
  const int64_t* pl = ptr<int64_t>(player, torch::kInt64, "player: int64");
  const int64_t* md = ptr<int64_t>(mode, torch::kInt64, "mode: int64");
  const int64_t* nn = ptr<int64_t>(n, torch::kInt64, "n: int64");
  const int64_t* nr = ptr<int64_t>(nrosters, torch::kInt64, "nrosters: int64");
  const bool* wn = ptr<bool>(winner, torch::kBool, "winner: bool");
  const int64_t* af = ptr<int64_t>(afk, torch::kInt64, "afk: int64");
  int64_t* bk = ptr<int64_t>(by_key, torch::kInt64, "by_key: int64");
  need(next_row + M * S < (int64_t(1) << 31), "batch_encode: roster rows exceed int32");
  Tensor rec = torch::empty({M, S + 2}, torch::TensorOptions().dtype(torch::kInt32));
  Tensor pos = torch::full({M, 2, K}, -1, torch::TensorOptions().dtype(torch::kInt32));
  int32_t* o_rec = rec.data_ptr<int32_t>();
  int32_t* o_pos = pos.data_ptr<int32_t>();
  // key -> index among this batch's unique players: a scratch map the size of
  // by_key, reset on the way out (O(batch), no hashing)
  for (int64_t j = 0; j < M * S; ++j) {  // validate, and start the (random) misses early
    need(pl[j] < B, "batch_encode: player key beyond by_key");
    if (pl[j] >= 0) __builtin_prefetch(bk + pl[j]);
  }
  static thread_local std::vector<int32_t> seen;
  if ((int64_t)seen.size() < B) seen.resize(B, -1);
  std::vector<int64_t> uk, ur, nk;
  uk.reserve(M * S);
  ur.reserve(M * S);
  for (int64_t i = 0; i < M; ++i) {
    int32_t* r = o_rec + i * (S + 2);
    for (int64_t s = 0; s < S; ++s) {
      const int64_t key = pl[i * S + s];
      if (key < 0) {
        r[s] = -1;
        continue;
      }
      int32_t u = seen[key];
      if (u < 0) {
        u = seen[key] = (int32_t)uk.size();
        int64_t row = bk[key];
        if (row < 0) {
          row = bk[key] = next_row + (int64_t)nk.size();
          nk.push_back(key);
        }
        uk.push_back(key);
        ur.push_back(row);
      }
      o_pos[i * S + s] = u;
      r[s] = (int32_t)ur[u];
    }
    const int64_t n0 = std::min<int64_t>(nn[2 * i], 255), n1 = std::min<int64_t>(nn[2 * i + 1], 255);
    const uint32_t m0 = (uint32_t)(md[i] & 0xff) | (uint32_t)(n0 << 8) | (uint32_t)(n1 << 16) |
                        (uint32_t)(std::min<int64_t>(nr[i], 255) << 24);
    const int64_t a = af[i];
    const uint32_t m1 = (wn[2 * i] ? 1u : 0u) | (wn[2 * i + 1] ? 2u : 0u) | (a != 0 ? 4u : 0u) |
                        ((uint32_t)(a & 0xffffff) << 8);
    r[S] = (int32_t)m0;
    r[S + 1] = (int32_t)m1;
  }
  for (int64_t k : uk) seen[k] = -1;
  auto i64 = torch::TensorOptions().dtype(torch::kInt64);
  auto vec = [&](const std::vector<int64_t>& v) {
    Tensor t = torch::empty({(int64_t)v.size()}, i64);
    std::copy(v.begin(), v.end(), t.data_ptr<int64_t>());
    return t;
  };
  return {rec, vec(uk), vec(ur), pos, vec(nk)};
}

// ---------------------------------------------------------------- finish
// packed: [M, W] float32 executor rows ([s_mu | s_sig | delta | m_mu | m_sig][2K],
// quality, status byte -- ops/rate.RateResult); final: [U, 32] float32 roster
// rows of the batch's unique players (uniq order) or an empty tensor.
std::vector<Tensor> batch_finish(Tensor packed, Tensor final_rows, Tensor mode, Tensor pos, Tensor uniq_keys,
                                 int64_t K) {
  const int64_t M = packed.size(0), W = packed.size(1), S = 2 * K, U = uniq_keys.numel();
  need(W >= 5 * S + 2, "packed: row too short for K");
  const float* pk = ptr<float>(packed, torch::kFloat32, "packed: float32");
  const int64_t* md = ptr<int64_t>(mode, torch::kInt64, "mode: int64");
  const int32_t* ps = ptr<int32_t>(pos, torch::kInt32, "pos: int32");
  const int64_t* uk = ptr<int64_t>(uniq_keys, torch::kInt64, "uniq_keys: int64");
  need(pos.numel() == M * S, "pos: [M, 2, K]");
  auto f64 = torch::TensorOptions().dtype(torch::kFloat64);
  Tensor status = torch::empty({M}, torch::TensorOptions().dtype(torch::kUInt8));
  Tensor quality = torch::empty({M}, f64);
  Tensor fields = torch::empty({5, M, 2, K}, f64);
  uint8_t* o_st = status.data_ptr<uint8_t>();
  double* o_q = quality.data_ptr<double>();
  double* o_f = fields.data_ptr<double>();
  std::vector<uint8_t> touched((size_t)U * kTracks, 0);
  for (int64_t i = 0; i < M; ++i) {
    const float* row = pk + i * W;
    const uint8_t st = reinterpret_cast<const uint8_t*>(row + 5 * S + 1)[0];
    o_st[i] = st;
    o_q[i] = row[5 * S];
    for (int f = 0; f < 5; ++f)
      for (int64_t s = 0; s < S; ++s) o_f[(f * M + i) * S + s] = row[f * S + s];
    if (st == kRated && md[i] >= 0 && md[i] < kTracks - 1)
      for (int64_t s = 0; s < S; ++s) {
        const int32_t u = ps[i * S + s];
        if (u < 0) continue;
        need(u < U, "pos: index beyond the unique players");
        touched[(size_t)u * kTracks] = 1;
        touched[(size_t)u * kTracks + 1 + md[i]] = 1;
      }
  }
  int64_t h = 0;
  for (int64_t u = 0; u < U; ++u) h += touched[(size_t)u * kTracks];
  Tensor fkeys = torch::empty({h}, torch::TensorOptions().dtype(torch::kInt64));
  Tensor fvals = torch::empty({h, 14}, f64);
  Tensor ftr = torch::zeros({h, kTracks}, torch::TensorOptions().dtype(torch::kBool));
  if (h) {
    need(final_rows.numel() == U * 32, "final: [U, 32]");
    const float* fr = ptr<float>(final_rows, torch::kFloat32, "final: float32");
    int64_t* ok = fkeys.data_ptr<int64_t>();
    double* ov = fvals.data_ptr<double>();
    bool* ot = ftr.data_ptr<bool>();
    int64_t j = 0;
    for (int64_t u = 0; u < U; ++u) {
      if (!touched[(size_t)u * kTracks]) continue;
      ok[j] = uk[u];
      for (int t = 0; t < kTracks; ++t) {  // granule t = {mu, tag, sigma, tag}
        ov[j * 14 + 2 * t] = fr[u * 32 + 4 * t];
        ov[j * 14 + 2 * t + 1] = fr[u * 32 + 4 * t + 2];
        ot[j * kTracks + t] = touched[(size_t)u * kTracks + t] != 0;
      }
      ++j;
    }
  }
  return {status, quality, fields, fkeys, fvals, ftr};
}

// ---------------------------------------------------------------- commit
// ColumnarSession._write_batch for the first two rosters (the caller handles
// any_afk of rosters beyond the second and the telemetry stats).
void batch_commit(Tensor rows, Tensor status, Tensor quality, Tensor part, Tensor fields, Tensor mode,
                  Tensor final_keys, Tensor final_vals, Tensor final_tracks, Tensor mt_quality, Tensor pt_i_afk,
                  Tensor pt_ts, Tensor pt_i_rating, Tensor pl_rating) {
  const int64_t M = rows.numel(), K = part.size(2), S = 2 * K;
  const int64_t* rw = ptr<int64_t>(rows, torch::kInt64, "rows: int64");
  const uint8_t* st = ptr<uint8_t>(status, torch::kUInt8, "status: uint8");
  const double* q = ptr<double>(quality, torch::kFloat64, "quality: float64");
  const int64_t* pt = ptr<int64_t>(part, torch::kInt64, "part: int64");
  const double* fd = ptr<double>(fields, torch::kFloat64, "fields: float64");
  const int64_t* md = ptr<int64_t>(mode, torch::kInt64, "mode: int64");
  double* mq = ptr<double>(mt_quality, torch::kFloat64, "match quality: float64");
  int8_t* ia = ptr<int8_t>(pt_i_afk, torch::kInt8, "any_afk: int8");
  double* ts = ptr<double>(pt_ts, torch::kFloat64, "ts: float64");
  double* ir = ptr<double>(pt_i_rating, torch::kFloat64, "item ratings: float64");
  double* pr = ptr<double>(pl_rating, torch::kFloat64, "player ratings: float64");
  const int64_t nm = mt_quality.numel(), np_ = pt_i_afk.numel(), npl = pl_rating.size(0);
  need(fields.numel() == 5 * M * S && part.size(0) == M, "fields/part shapes");
  for (int64_t i = 0; i < M; ++i) {
    const int s = st[i];
    const bool rated = s == kRated, afk = s == kAfk || s == kInvalid;
    if (!rated && !afk) continue;
    need(rw[i] >= 0 && rw[i] < nm, "batch_commit: match row out of range");
    mq[rw[i]] = rated ? q[i] : 0.0;
    if (rated) need(md[i] >= 0 && md[i] < kTracks - 1, "batch_commit: rated match of no mode");
    for (int64_t j = 0; j < S; ++j) {
      const int64_t p = pt[i * S + j];
      if (p < 0) continue;
      need(p < np_, "batch_commit: participant row out of range");
      ia[p] = afk ? 1 : 0;
      if (!rated) continue;
      ts[p * 3 + 0] = fd[(0 * M + i) * S + j];
      ts[p * 3 + 1] = fd[(1 * M + i) * S + j];
      ts[p * 3 + 2] = fd[(2 * M + i) * S + j];
      ir[p * 12 + 2 * md[i]] = fd[(3 * M + i) * S + j];
      ir[p * 12 + 2 * md[i] + 1] = fd[(4 * M + i) * S + j];
    }
  }
  const int64_t H = final_keys.numel();
  if (!H) return;
  const int64_t* fk = ptr<int64_t>(final_keys, torch::kInt64, "final_keys: int64");
  const double* fv = ptr<double>(final_vals, torch::kFloat64, "final_vals: float64");
  const bool* ft = ptr<bool>(final_tracks, torch::kBool, "final_tracks: bool");
  for (int64_t j = 0; j < H; ++j) {
    need(fk[j] >= 0 && fk[j] < npl, "batch_commit: player row out of range");
    for (int t = 0; t < kTracks; ++t)
      if (ft[j * kTracks + t]) {
        pr[fk[j] * 14 + 2 * t] = fv[j * 14 + 2 * t];
        pr[fk[j] * 14 + 2 * t + 1] = fv[j * 14 + 2 * t + 1];
      }
  }
}

// ---------------------------------------------------------------- stage
// Stored ratings [N, 14] (mu, sigma per track; NaN = NULL) and attributes [N, 3]
// of player keys -> upload rows [k, 36]: the roster state row (8 granules of
// {mu, tag, sigma, tag}; a NULL mu makes the track NULL) and the 4 attribute
// floats (ResidentRoster._upload_arrays, in one pass, into a pinned buffer).
void batch_stage_players(Tensor keys, Tensor rating, Tensor attr, Tensor out) {
  const int64_t k = keys.numel(), N = rating.size(0);
  const int64_t* kk = ptr<int64_t>(keys, torch::kInt64, "keys: int64");
  const double* rt = ptr<double>(rating, torch::kFloat64, "rating: float64 [N, 14]");
  const double* at = ptr<double>(attr, torch::kFloat64, "attr: float64 [N, 3]");
  float* o = ptr<float>(out, torch::kFloat32, "out: float32 [k, 36]");
  need(rating.size(1) == 14 && attr.size(1) == 3 && attr.size(0) >= N, "rating [N, 14] / attr [N, 3]");
  need(out.numel() >= k * 36, "out: [k, 36]");
  const float nan = std::nanf("");
  for (int64_t j = 0; j < k; ++j) {  // validate, and start the (random) row misses early
    need(kk[j] >= 0 && kk[j] < N, "batch_stage_players: key out of range");
    __builtin_prefetch(rt + kk[j] * 14);
    __builtin_prefetch(rt + kk[j] * 14 + 8);
    __builtin_prefetch(at + kk[j] * 3);
  }
  for (int64_t j = 0; j < k; ++j) {
    const double* r = rt + kk[j] * 14;
    float* row = o + j * 36;
    for (int t = 0; t < kTracks; ++t) {
      const double mu = r[2 * t];
      row[4 * t] = (float)mu;
      row[4 * t + 1] = 0.f;
      row[4 * t + 2] = std::isnan(mu) ? nan : (float)r[2 * t + 1];
      row[4 * t + 3] = 0.f;
    }
    row[28] = nan, row[29] = 0.f, row[30] = nan, row[31] = 0.f;
    const double* a = at + kk[j] * 3;
    row[32] = (float)a[0], row[33] = (float)a[1], row[34] = (float)a[2], row[35] = 0.f;
  }
}

// ---------------------------------------------------------------- key index
// Python binding of ana::KeyMap (key_index.h): keys are str or bytes objects.
std::string_view key_view(PyObject* o) {
  char* p = nullptr;
  Py_ssize_t n = 0;
  if (PyBytes_Check(o)) {
    if (PyBytes_AsStringAndSize(o, &p, &n) != 0) throw pybind11::error_already_set();
    return std::string_view(p, (size_t)n);
  }
  const char* u = PyUnicode_AsUTF8AndSize(o, &n);
  if (!u) throw pybind11::error_already_set();
  return std::string_view(u, (size_t)n);
}

std::vector<std::string_view> key_views(const pybind11::list& keys) {
  std::vector<std::string_view> kv(pybind11::len(keys));
  for (size_t i = 0; i < kv.size(); ++i) kv[i] = key_view(keys[i].ptr());
  return kv;
}

class KeyIndex {
 public:
  int64_t size() const { return map_.size(); }

  void add(pybind11::list keys, int64_t first_row) {
    const std::vector<std::string_view> kv = key_views(keys);
    map_.reserve(map_.size() + (int64_t)kv.size());
    for (size_t i = 0; i < kv.size(); ++i) map_.add(kv[i], first_row + (int64_t)i);
  }

  Tensor lookup(pybind11::list keys) const {
    const std::vector<std::string_view> kv = key_views(keys);
    Tensor out = torch::empty({(int64_t)kv.size()}, torch::TensorOptions().dtype(torch::kInt64));
    map_.lookup(kv.data(), (int64_t)kv.size(), out.data_ptr<int64_t>());
    return out;
  }

 private:
  ana::KeyMap map_;
};

}  // namespace

void register_batch_host(pybind11::module& m) {
  pybind11::class_<KeyIndex>(m, "KeyIndex", "W7: api id -> store row, batched lookups with prefetch")
      .def(pybind11::init<>())
      .def("add", &KeyIndex::add, "add(keys, first_row): keys[i] -> first_row + i")
      .def("lookup", &KeyIndex::lookup, "rows of keys (str or bytes), -1 where absent")
      .def("__len__", &KeyIndex::size);
  m.def("batch_stage_players", &batch_stage_players, "W8: stored player rows -> resident upload rows [k, 36]");
  m.def("batch_gather", &batch_gather, "W7: columnar store rows -> batch columns (worker load)");
  m.def("batch_encode", &batch_encode, "W8: batch columns -> stream records + resident rows");
  m.def("batch_finish", &batch_finish, "W8: packed executor rows -> result columns + touched tracks");
  m.def("batch_commit", &batch_commit, "W8: result columns -> columnar store (worker commit)");
}
