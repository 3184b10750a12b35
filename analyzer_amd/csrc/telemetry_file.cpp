// Telemetry event files: the event source of DOTELEMETRY=true
// for real stores.
//
// The reference forwards each match's telemetry asset URL to a "telesuck"
// queue (/root/reference/worker.py:148-161) and leaves participant_stats
// (worker.py:75-78) to a downstream service.  Here the downloaded events of
// many matches are kept in one memory-mapped file keyed by match api id, and
// the worker gathers a batch's events from it straight into the CSR layout the
// aggregation kernels read (csrc/telemetry_core.h), in pinned memory:
//
//   ANATEL01 file: 64-B header {magic, int64 n, int64 E, int64 id_bytes, 4 x
//   int64 reserved}, then evoff int64[n + 1] (CSR over the events), id_off
//   int64[n + 1] (byte offsets of the ids), the id bytes, and E events of 8 B:
//   {roster << 4 | position, type << 8} | value (float bits).
//
// ``gather(ids, K)`` maps (roster, position) to the batch's slot roster * K +
// position (slot 0xff -- malformed, counted by the kernels -- for a position
// >= K or a third roster) and stamps each event with its batch-local match tag.
#include <torch/extension.h>

#include <fcntl.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "key_index.h"

namespace {

using torch::Tensor;

constexpr char kMagic[8] = {'A', 'N', 'A', 'T', 'E', 'L', '0', '1'};

struct Header {
  char magic[8];
  int64_t n, E, id_bytes;
  int64_t reserved[4];
};
static_assert(sizeof(Header) == 64, "header layout");

std::string_view py_key(PyObject* o) {
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

// ids: n match api ids; evoff: int64 [n + 1]; events: int32 [E, 2] in the file
// encoding (roster << 4 | position, type << 8)
void write_telemetry_file(const std::string& path, pybind11::list ids, Tensor evoff, Tensor events) {
  const int64_t n = (int64_t)pybind11::len(ids);
  TORCH_CHECK(evoff.device().is_cpu() && evoff.scalar_type() == torch::kInt64 && evoff.is_contiguous() &&
                  evoff.numel() == n + 1, "evoff must be a contiguous CPU int64 [n + 1]");
  TORCH_CHECK(events.device().is_cpu() && events.scalar_type() == torch::kInt32 && events.is_contiguous() &&
                  events.dim() == 2 && events.size(1) == 2, "events must be a contiguous CPU int32 [E, 2]");
  const int64_t* off = evoff.data_ptr<int64_t>();
  const int64_t E = events.size(0);
  TORCH_CHECK(off[0] == 0 && off[n] == E, "evoff must run from 0 to E");
  for (int64_t i = 0; i < n; ++i) TORCH_CHECK(off[i] <= off[i + 1], "evoff must be non-decreasing");
  std::vector<int64_t> id_off((size_t)n + 1, 0);
  std::string bytes;
  for (int64_t i = 0; i < n; ++i) {
    const std::string_view k = py_key(ids[i].ptr());
    bytes.append(k.data(), k.size());
    id_off[i + 1] = (int64_t)bytes.size();
  }
  Header h{};
  memcpy(h.magic, kMagic, 8);
  h.n = n;
  h.E = E;
  h.id_bytes = (int64_t)bytes.size();
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot open " + path + " for writing");
  bool ok = fwrite(&h, sizeof(h), 1, f) == 1;
  ok = ok && fwrite(off, sizeof(int64_t), (size_t)n + 1, f) == (size_t)n + 1;
  ok = ok && fwrite(id_off.data(), sizeof(int64_t), (size_t)n + 1, f) == (size_t)n + 1;
  ok = ok && (bytes.empty() || fwrite(bytes.data(), 1, bytes.size(), f) == bytes.size());
  ok = ok && (E == 0 || fwrite(events.data_ptr<int32_t>(), 8, (size_t)E, f) == (size_t)E);
  ok = (fclose(f) == 0) && ok;
  if (!ok) throw std::runtime_error("short write to " + path);
}

class TelemetryFile {
 public:
  explicit TelemetryFile(const std::string& path) : path_(path) {
    fd_ = open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("cannot open " + path);
    struct stat st {};
    if (fstat(fd_, &st) != 0 || st.st_size < (off_t)sizeof(Header)) fail("too short for a header");
    size_ = (size_t)st.st_size;
    void* p = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (p == MAP_FAILED) fail("mmap failed");
    base_ = static_cast<const uint8_t*>(p);
    Header h;
    memcpy(&h, base_, sizeof(h));
    if (memcmp(h.magic, kMagic, 8) != 0) fail("not an ANATEL01 telemetry file");
    n_ = h.n;
    E_ = h.E;
    if (n_ < 0 || E_ < 0 || h.id_bytes < 0) fail("bad header");
    // every header term is bounded by the file size before it is added, so a corrupt
    // header cannot wrap the size check (the index arrays and events are mapped reads)
    const size_t avail = size_ - sizeof(Header);
    if ((uint64_t)n_ >= avail / 16) fail("truncated");  // two int64 arrays of n + 1
    const size_t idx = 16 * ((size_t)n_ + 1);
    if ((uint64_t)h.id_bytes > avail - idx) fail("truncated");
    if ((uint64_t)E_ > (avail - idx - (size_t)h.id_bytes) / 8) fail("truncated");
    evoff_ = reinterpret_cast<const int64_t*>(base_ + sizeof(Header));
    const int64_t* id_off = evoff_ + n_ + 1;
    const char* ids = reinterpret_cast<const char*>(id_off + n_ + 1);
    events_ = reinterpret_cast<const int32_t*>(ids + h.id_bytes);
    if (evoff_[0] != 0 || evoff_[n_] != E_) fail("bad event offsets");
    if (id_off[0] != 0) fail("bad index");
    map_.reserve(n_);
    for (int64_t i = 0; i < n_; ++i) {
      // evoff_ runs 0 .. E_ and is non-decreasing, so every event range lies inside the
      // file; id_off likewise inside the id bytes
      if (evoff_[i] > evoff_[i + 1] || evoff_[i + 1] > E_ || id_off[i] > id_off[i + 1] ||
          id_off[i + 1] > h.id_bytes)
        fail("bad index");
      try {
        map_.add(std::string_view(ids + id_off[i], (size_t)(id_off[i + 1] - id_off[i])), i);
      } catch (const std::invalid_argument&) {
        fail("a match id appears twice");
      }
    }
    madvise(const_cast<uint8_t*>(base_), size_, MADV_RANDOM);
  }
  ~TelemetryFile() {
    if (base_) munmap(const_cast<uint8_t*>(base_), size_);
    if (fd_ >= 0) close(fd_);
  }
  TelemetryFile(const TelemetryFile&) = delete;
  TelemetryFile& operator=(const TelemetryFile&) = delete;

  int64_t num_matches() const { return n_; }
  int64_t num_events() const { return E_; }

  // the batch's events in CSR order: (evoff int64 [B + 1], events int32 [E_b, 2]),
  // pinned when asked (the caller copies them to the device asynchronously)
  std::vector<Tensor> gather(pybind11::list ids, int64_t K, bool pinned) const {
    TORCH_CHECK(K >= 1 && K <= 5, "K must be 1..5");
    const int64_t B = (int64_t)pybind11::len(ids);
    std::vector<std::string_view> kv((size_t)B);
    for (int64_t i = 0; i < B; ++i) kv[i] = py_key(ids[i].ptr());
    std::vector<int64_t> row((size_t)B);
    map_.lookup(kv.data(), B, row.data());
    auto opt = torch::TensorOptions().pinned_memory(pinned);
    Tensor evoff = torch::empty({B + 1}, opt.dtype(torch::kInt64));
    int64_t* o = evoff.data_ptr<int64_t>();
    o[0] = 0;
    for (int64_t i = 0; i < B; ++i) o[i + 1] = o[i] + (row[i] >= 0 ? evoff_[row[i] + 1] - evoff_[row[i]] : 0);
    Tensor events = torch::empty({o[B], 2}, opt.dtype(torch::kInt32));
    int32_t* e = events.data_ptr<int32_t>();
    for (int64_t i = 0; i < B; ++i) {
      if (row[i] < 0) continue;
      const int32_t* src = events_ + 2 * evoff_[row[i]];
      const int64_t cnt = evoff_[row[i] + 1] - evoff_[row[i]];
      int32_t* dst = e + 2 * o[i];
      const uint32_t tag = (uint32_t)(i & 0xffff) << 16;
      for (int64_t j = 0; j < cnt; ++j) {
        const uint32_t meta = (uint32_t)src[2 * j];
        const uint32_t r = (meta >> 4) & 0xf, pos = meta & 0xf;
        const uint32_t slot = (r < 2 && pos < (uint32_t)K) ? r * (uint32_t)K + pos : 0xffu;
        dst[2 * j] = (int32_t)(slot | (meta & 0xff00u) | tag);
        dst[2 * j + 1] = src[2 * j + 1];
      }
    }
    return {evoff, events};
  }

 private:
  [[noreturn]] void fail(const char* what) {
    if (base_) munmap(const_cast<uint8_t*>(base_), size_);
    if (fd_ >= 0) close(fd_);
    base_ = nullptr;
    fd_ = -1;
    throw std::runtime_error(path_ + ": " + what);
  }

  std::string path_;
  int fd_ = -1;
  size_t size_ = 0;
  const uint8_t* base_ = nullptr;
  int64_t n_ = 0, E_ = 0;
  const int64_t* evoff_ = nullptr;
  const int32_t* events_ = nullptr;
  ana::KeyMap map_;
};

}  // namespace

void register_telemetry_file(pybind11::module& m) {
  m.def("write_telemetry_file", &write_telemetry_file,
        "K8: write an ANATEL01 telemetry file (ids, evoff [n+1], events [E,2] in file encoding)");
  pybind11::class_<TelemetryFile>(m, "TelemetryFile", "K8: memory-mapped ANATEL01 telemetry events by match api id")
      .def(pybind11::init<const std::string&>(), pybind11::arg("path"))
      .def_property_readonly("num_matches", &TelemetryFile::num_matches)
      .def_property_readonly("num_events", &TelemetryFile::num_events)
      .def("gather", &TelemetryFile::gather, pybind11::arg("ids"), pybind11::arg("K"),
           pybind11::arg("pinned") = false,
           "a batch's events: (evoff [B+1] int64, events [E,2] int32, batch slots and match tags)");
}
