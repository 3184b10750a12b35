// Native record-file ingest: SPSC ring of pinned host windows filled by a
// background thread (see ingest.cpp).
#pragma once

#include <stdint.h>
#include <stdio.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

namespace ana {

void write_record_file(const std::string& path, const int32_t* rec, int64_t M, int K);

class RecordReader {
 public:
  RecordReader(const std::string& path, int64_t window, int slots, bool pinned);
  ~RecordReader();
  RecordReader(const RecordReader&) = delete;
  RecordReader& operator=(const RecordReader&) = delete;

  int K() const { return K_; }
  int64_t num_matches() const { return M_; }
  int64_t window() const { return window_; }
  int64_t num_windows() const;
  // every slot is pinned host memory (slots fall back to malloc one by one)
  bool pinned() const;
  int32_t* slot_data(int slot) const { return buf_[slot]; }

  // blocks until the next window is filled; false at end of file
  bool acquire(int* slot, int64_t* base, int64_t* n);
  // hand the oldest acquired slot back to the producer
  void release(int slot);

 private:
  void run();
  void release_buffers();

  std::string path_;
  int64_t window_;
  int slots_;
  int K_ = 0;
  int64_t M_ = 0;
  FILE* file_ = nullptr;
  std::vector<int32_t*> buf_;
  std::vector<bool> slot_pinned_;
  std::vector<int64_t> n_, base_;
  std::atomic<uint64_t> head_{0}, tail_{0};
  uint64_t next_ = 0;  // consumer-only cursor
  std::atomic<bool> stop_{false}, error_{false};
  std::thread producer_;
};

}  // namespace ana
