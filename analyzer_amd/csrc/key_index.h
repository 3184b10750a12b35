// api id -> row map for batched lookups (csrc/batch_host.cpp KeyIndex binding,
// csrc/ingest.cpp TelemetryFile).
//
// A Python dict lookup of a fresh string costs ~250 ns on a 10^5..10^6-entry
// dict: the misses on the table and on the stored key are taken one after the
// other.  Here a batch of keys is hashed first, every probe slot is prefetched,
// and then probed, so the misses of different keys overlap.  Open addressing,
// linear probing; a slot holds the 64-bit hash, the row and the key's place in
// a byte arena (the key bytes are compared on a hash match).
#pragma once

#include <stdint.h>

#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace ana {

class KeyMap {
 public:
  KeyMap() { rehash(1024); }

  int64_t size() const { return n_; }

  void reserve(int64_t n) {
    if (2 * n > (int64_t)slots_.size()) rehash(next_pow2(4 * n));
  }

  // key -> row; throws on a duplicate key
  void add(std::string_view key, int64_t row) {
    if (2 * (n_ + 1) > (int64_t)slots_.size()) rehash(next_pow2(4 * (n_ + 1)));
    const uint64_t h = hash(key);
    size_t j = h & mask_;
    while (slots_[j].len != kEmpty) {
      if (slots_[j].h == h && key_at(slots_[j]) == key)
        throw std::invalid_argument("duplicate key " + std::string(key));
      j = (j + 1) & mask_;
    }
    slots_[j] = Slot{h, row, (uint64_t)arena_.size(), (uint32_t)key.size()};
    arena_.append(key.data(), key.size());
    ++n_;
  }

  // rows of k keys (-1 where absent): hash all, prefetch all, then probe
  void lookup(const std::string_view* keys, int64_t k, int64_t* out) const {
    std::vector<uint64_t> hv((size_t)k);
    for (int64_t i = 0; i < k; ++i) {
      hv[i] = hash(keys[i]);
      __builtin_prefetch(&slots_[hv[i] & mask_]);
    }
    for (int64_t i = 0; i < k; ++i) {  // second pass: the key bytes of hash matches
      const Slot& s = slots_[hv[i] & mask_];
      if (s.h == hv[i]) __builtin_prefetch(arena_.data() + s.off);
    }
    for (int64_t i = 0; i < k; ++i) {
      size_t j = hv[i] & mask_;
      out[i] = -1;
      while (slots_[j].len != kEmpty) {
        if (slots_[j].h == hv[i] && key_at(slots_[j]) == keys[i]) {
          out[i] = slots_[j].row;
          break;
        }
        j = (j + 1) & mask_;
      }
    }
  }

 private:
  static constexpr uint32_t kEmpty = 0xffffffffu;
  struct Slot {
    uint64_t h;
    int64_t row;
    uint64_t off;
    uint32_t len;
  };
  std::vector<Slot> slots_;
  std::string arena_;
  size_t mask_ = 0;
  int64_t n_ = 0;

  static size_t next_pow2(int64_t v) {
    size_t p = 1024;
    while ((int64_t)p < v) p <<= 1;
    return p;
  }
  static uint64_t hash(std::string_view k) {  // FNV-1a 64 + a final avalanche
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : k) h = (h ^ c) * 1099511628211ull;
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    return h;
  }
  std::string_view key_at(const Slot& s) const { return std::string_view(arena_.data() + s.off, s.len); }
  void rehash(size_t cap) {
    std::vector<Slot> old;
    old.swap(slots_);
    slots_.assign(cap, Slot{0, 0, 0, kEmpty});
    mask_ = cap - 1;
    for (const Slot& s : old) {
      if (s.len == kEmpty) continue;
      size_t j = s.h & mask_;
      while (slots_[j].len != kEmpty) j = (j + 1) & mask_;
      slots_[j] = s;
    }
  }
};

}  // namespace ana
