// Native ingest (SURVEY P3 / N5 "host ingest ring buffer"): a background thread
// reads fixed-size windows of match records from a record file into a
// single-producer / single-consumer ring of pinned host buffers; the consumer
// (the Python pipeline) takes a filled slot, enqueues its H2D copy on a copy
// stream and releases the slot once the copy has completed.  The reference's
// ingest is a blocking pika consumer handing one message at a time to Python
// (/root/reference/worker.py:92-101); here the device never waits on the host
// in steady state.
//
// Record file: 32-byte header {magic "ANAREC01", int32 K, int32 pad, int64 M,
// int64 reserved} followed by M records of 2K+2 int32 (csrc/common.h layout).
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "ingest.h"

namespace ana {

static constexpr char kMagic[8] = {'A', 'N', 'A', 'R', 'E', 'C', '0', '1'};

struct RecordFileHeader {
  char magic[8];
  int32_t K;
  int32_t pad;
  int64_t M;
  int64_t reserved;
};
static_assert(sizeof(RecordFileHeader) == 32, "header layout");

void write_record_file(const std::string& path, const int32_t* rec, int64_t M, int K) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot open " + path + " for writing");
  RecordFileHeader h{};
  memcpy(h.magic, kMagic, 8);
  h.K = K;
  h.M = M;
  const size_t R = (size_t)(2 * K + 2);
  bool ok = fwrite(&h, sizeof(h), 1, f) == 1;
  ok = ok && (M == 0 || fwrite(rec, sizeof(int32_t) * R, (size_t)M, f) == (size_t)M);
  ok = (fclose(f) == 0) && ok;
  if (!ok) throw std::runtime_error("short write to " + path);
}

RecordReader::RecordReader(const std::string& path, int64_t window, int slots, bool pinned)
    : path_(path), window_(window), slots_(slots) {
  if (window <= 0 || slots < 2) throw std::invalid_argument("window > 0 and slots >= 2 required");
  file_ = fopen(path.c_str(), "rb");
  if (!file_) throw std::runtime_error("cannot open " + path);
  try {
    RecordFileHeader h{};
    if (fread(&h, sizeof(h), 1, file_) != 1 || memcmp(h.magic, kMagic, 8) != 0)
      throw std::runtime_error(path + " is not an ANAREC01 record file");
    K_ = h.K;
    M_ = h.M;
    if (K_ < 1 || K_ > 5 || M_ < 0) throw std::runtime_error(path + ": bad header");
    const size_t bytes = (size_t)window_ * (size_t)(2 * K_ + 2) * sizeof(int32_t);
    buf_.assign(slots_, nullptr);
    slot_pinned_.assign(slots_, false);
    n_.assign(slots_, 0);
    base_.assign(slots_, 0);
    for (int s = 0; s < slots_; ++s) {
      // each slot remembers its own allocator: under pinned-memory pressure some
      // slots may be pinned and later ones plain malloc
      void* p = nullptr;
      if (pinned && hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess) {
        slot_pinned_[s] = true;
      } else {
        (void)hipGetLastError();
        p = malloc(bytes);
        if (!p) throw std::bad_alloc();
      }
      buf_[s] = static_cast<int32_t*>(p);
    }
    producer_ = std::thread(&RecordReader::run, this);
  } catch (...) {
    release_buffers();
    throw;
  }
}

void RecordReader::release_buffers() {
  for (size_t s = 0; s < buf_.size(); ++s) {
    if (!buf_[s]) continue;
    if (slot_pinned_[s]) (void)hipHostFree(buf_[s]);
    else free(buf_[s]);
    buf_[s] = nullptr;
  }
  if (file_) fclose(file_);
  file_ = nullptr;
}

bool RecordReader::pinned() const {
  for (bool b : slot_pinned_)
    if (!b) return false;
  return !slot_pinned_.empty();
}

RecordReader::~RecordReader() {
  stop_.store(true, std::memory_order_release);
  if (producer_.joinable()) producer_.join();
  release_buffers();
}

int64_t RecordReader::num_windows() const { return (M_ + window_ - 1) / window_; }

// producer: fill slot (head % slots) while the ring is not full
void RecordReader::run() {
  const size_t R = (size_t)(2 * K_ + 2);
  for (int64_t w = 0; w < num_windows(); ++w) {
    for (;;) {  // wait for a free slot
      if (stop_.load(std::memory_order_acquire)) return;
      const uint64_t head = head_.load(std::memory_order_relaxed);
      if (head - tail_.load(std::memory_order_acquire) < (uint64_t)slots_) break;
      std::this_thread::yield();
    }
    const uint64_t head = head_.load(std::memory_order_relaxed);
    const int s = (int)(head % (uint64_t)slots_);
    const int64_t base = w * window_;
    const int64_t n = (M_ - base) < window_ ? (M_ - base) : window_;
    if (fseeko(file_, (off_t)(sizeof(RecordFileHeader) + (size_t)base * R * sizeof(int32_t)), SEEK_SET) != 0 ||
        fread(buf_[s], R * sizeof(int32_t), (size_t)n, file_) != (size_t)n) {
      error_.store(true, std::memory_order_release);
      head_.store(head + 1, std::memory_order_release);  // wake the consumer
      return;
    }
    n_[s] = n;
    base_[s] = base;
    head_.store(head + 1, std::memory_order_release);  // publish the slot
  }
}

// consumer side: ``next_`` = next window to hand out, ``tail_`` = oldest window
// still held (acquired, not yet released); several windows may be held at once
bool RecordReader::acquire(int* slot, int64_t* base, int64_t* n) {
  const uint64_t next = next_;
  if ((int64_t)next >= num_windows()) return false;
  while (head_.load(std::memory_order_acquire) <= next) std::this_thread::yield();
  if (error_.load(std::memory_order_acquire)) throw std::runtime_error("read error in " + path_);
  next_ = next + 1;
  const int s = (int)(next % (uint64_t)slots_);
  *slot = s;
  *base = base_[s];
  *n = n_[s];
  return true;
}

void RecordReader::release(int slot) {
  const uint64_t tail = tail_.load(std::memory_order_relaxed);
  if (tail >= next_ || slot != (int)(tail % (uint64_t)slots_))
    throw std::logic_error("slots are released in acquisition order");
  tail_.store(tail + 1, std::memory_order_release);
}

}  // namespace ana
