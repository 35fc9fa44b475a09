// worddict.hpp — interning of int32 word sequences for the host encoder.
// intern() returns a dense id per distinct sequence, in first-insertion
// order; the words live in one arena and the index is open addressing over
// 64-bit hashes, so interning allocates nothing once the arena has grown.
//
// Arena layout: each entry is its length followed by its words, and a slot
// holds the arena position of its entry's words, so a lookup touches one slot
// and one arena run (the offsets table is only read through data()/len()).
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
    off_.clear();
    slots_.clear();
  }
  size_t size() const { return off_.size(); }
  const int32_t* data(int32_t id) const { return words_.data() + off_[id]; }
  size_t len(int32_t id) const { return static_cast<uint32_t>(words_[off_[id] - 1]); }

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
        words_.push_back(static_cast<int32_t>(n));
        const size_t w0 = words_.size();
        words_.insert(words_.end(), p, p + n);
        off_.push_back(w0);
        s = Slot{h, id, w0};
        if (inserted) *inserted = true;
        return id;
      }
      if (s.hash == h) {
        const int32_t* e = words_.data() + s.off;
        if (static_cast<uint32_t>(e[-1]) == n && (n == 0 || std::memcmp(e, p, n * sizeof(int32_t)) == 0)) {
          if (inserted) *inserted = false;
          return s.id;
        }
      }
    }
  }
  // Lookup only (-1 if absent); safe to call from many threads while no
  // thread interns.
  int32_t find(const int32_t* p, size_t n, uint64_t h) const {
    if (slots_.empty()) return -1;
    const size_t mask = slots_.size() - 1;
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      const Slot& s = slots_[i];
      if (s.id < 0) return -1;
      if (s.hash == h) {
        const int32_t* e = words_.data() + s.off;
        if (static_cast<uint32_t>(e[-1]) == n && (n == 0 || std::memcmp(e, p, n * sizeof(int32_t)) == 0)) return s.id;
      }
    }
  }

 private:
  struct Slot {
    uint64_t hash;
    int32_t id;
    size_t off;  // arena position of the entry's words
  };
  void grow() {
    std::vector<Slot> old;
    old.swap(slots_);
    slots_.assign(old.empty() ? 64 : old.size() * 2, Slot{0, -1, 0});
    const size_t mask = slots_.size() - 1;
    for (const Slot& s : old)
      if (s.id >= 0) {
        size_t i = s.hash & mask;
        while (slots_[i].id >= 0) i = (i + 1) & mask;
        slots_[i] = s;
      }
  }
  std::vector<int32_t> words_;
  std::vector<size_t> off_;
  std::vector<Slot> slots_;
};

}  // namespace sr
