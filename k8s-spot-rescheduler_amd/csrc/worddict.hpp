// worddict.hpp — interning of int32 word sequences for the host encoder.
// intern() returns a dense id per distinct sequence, in first-insertion
// order; the words live in one arena and the index is open addressing over
// 64-bit hashes, so interning allocates nothing once the arena has grown.
#pragma once

#include <cstdint>
#include <cstring>
#include <vector>

namespace sr {

inline uint64_t hash_words(const int32_t* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
  for (size_t i = 0; i < n; ++i) {
    h = (h ^ static_cast<uint32_t>(p[i])) * 0xff51afd7ed558ccdull;
    h ^= h >> 32;
  }
  return h;
}

class WordDict {
 public:
  void clear() {
    words_.clear();
    off_.assign(1, 0);
    slots_.clear();
  }
  size_t size() const { return off_.size() - 1; }
  const int32_t* data(int32_t id) const { return words_.data() + off_[id]; }
  size_t len(int32_t id) const { return off_[id + 1] - off_[id]; }

  int32_t intern(const int32_t* p, size_t n, bool* inserted = nullptr) {
    return intern(p, n, hash_words(p, n), inserted);
  }
  int32_t intern(const std::vector<int32_t>& v, bool* inserted = nullptr) {
    return intern(v.data(), v.size(), inserted);
  }
  // `h` must be a function of the words alone (callers may hash differently,
  // but consistently within one dictionary).
  int32_t intern(const int32_t* p, size_t n, uint64_t h, bool* inserted) {
    if ((size() + 1) * 2 > slots_.size()) grow();
    const size_t mask = slots_.size() - 1;
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      Slot& s = slots_[i];
      if (s.id < 0) {
        const int32_t id = static_cast<int32_t>(size());
        words_.insert(words_.end(), p, p + n);
        off_.push_back(words_.size());
        s = Slot{h, id};
        if (inserted) *inserted = true;
        return id;
      }
      if (s.hash == h && len(s.id) == n && (n == 0 || std::memcmp(data(s.id), p, n * sizeof(int32_t)) == 0)) {
        if (inserted) *inserted = false;
        return s.id;
      }
    }
  }

 private:
  struct Slot {
    uint64_t hash;
    int32_t id;
  };
  void grow() {
    std::vector<Slot> old;
    old.swap(slots_);
    slots_.assign(old.empty() ? 64 : old.size() * 2, Slot{0, -1});
    const size_t mask = slots_.size() - 1;
    for (const Slot& s : old)
      if (s.id >= 0) {
        size_t i = s.hash & mask;
        while (slots_[i].id >= 0) i = (i + 1) & mask;
        slots_[i] = s;
      }
  }
  std::vector<int32_t> words_;
  std::vector<size_t> off_{0};
  std::vector<Slot> slots_;
};

}  // namespace sr
