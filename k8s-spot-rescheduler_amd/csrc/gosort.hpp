// gosort.hpp — Go 1.16 sort.Slice, reproduced exactly (tie order included).
//
// The reference sorts with sort.Slice, which is NOT stable: pods with equal
// CPU requests (nodes/nodes.go:76-80) and nodes with equal RequestedCPU
// (nodes/nodes.go:95-101) come out in the order Go's pattern of comparisons
// and swaps leaves them.  That order decides first-fit placements, so it is
// part of the answer.  Go <= 1.18 implements sort.Slice as quickSort_func
// (go/src/sort/zfuncversion.go, generated from sort.go): introsort with an
// insertion-sort cutoff at 12 elements, a gap-6 shell pass, Tukey's ninther
// for spans > 40, a duplicate-protection pass, and heapsort at depth
// 2*ceil(lg(n+1)).  go.mod:3 pins Go 1.15 and Dockerfile:3 builds with 1.16.
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

namespace sr {

// Sorts data[0..n) of element ids; less(x, y) compares two element ids.
template <class T, class Less>
class GoSlice {
 public:
  GoSlice(T* data, Less less) : d_(data), less_(less) {}

  void sort(int n) { quick(0, n, max_depth(n)); }

  // A span of quickSort_func's recursion: quick(a, b, depth) sorts it exactly
  // as the serial sort would, independently of every other span.
  struct Span {
    int a, b, depth;
  };
  // One partition step of quick() on a span longer than `grain` (the same
  // pivot, the same swaps): its two sub-spans, or the span itself when the
  // serial sort would finish it here (short, or at depth 0: heapsort).
  void split(const Span& s, int grain, Span* lo, Span* hi, bool* leaf) {
    *leaf = s.b - s.a <= grain || s.depth == 0;
    if (*leaf) return;
    const int depth = s.depth - 1;
    auto [mlo, mhi] = pivot(s.a, s.b);
    *lo = Span{s.a, mlo, depth};
    *hi = Span{mhi, s.b, depth};
  }
  void finish(const Span& s) { quick(s.a, s.b, s.depth); }
  static int depth_of(int n) { return max_depth(n); }

 private:
  T* d_;
  Less less_;

  bool lt(int i, int j) const { return less_(d_[i], d_[j]); }
  void sw(int i, int j) { std::swap(d_[i], d_[j]); }

  static int max_depth(int n) {
    int depth = 0;
    for (int i = n; i > 0; i >>= 1) ++depth;
    return depth * 2;
  }

  void insertion(int a, int b) {
    for (int i = a + 1; i < b; ++i)
      for (int j = i; j > a && lt(j, j - 1); --j) sw(j, j - 1);
  }

  void sift_down(int lo, int hi, int first) {
    int root = lo;
    while (true) {
      int child = 2 * root + 1;
      if (child >= hi) return;
      if (child + 1 < hi && lt(first + child, first + child + 1)) ++child;
      if (!lt(first + root, first + child)) return;
      sw(first + root, first + child);
      root = child;
    }
  }

  void heap(int a, int b) {
    const int first = a, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; --i) sift_down(i, hi, first);
    for (int i = hi - 1; i >= 0; --i) {
      sw(first, first + i);
      sift_down(0, i, first);
    }
  }

  // Leaves the median of {m0, m1, m2} at m1 (Go's argument order: m1, m0, m2).
  void median3(int m1, int m0, int m2) {
    if (lt(m1, m0)) sw(m1, m0);
    if (lt(m2, m1)) {
      sw(m2, m1);
      if (lt(m1, m0)) sw(m1, m0);
    }
  }

  std::pair<int, int> pivot(int lo, int hi) {
    const int m = static_cast<int>((static_cast<unsigned>(lo) + static_cast<unsigned>(hi)) >> 1);
    if (hi - lo > 40) {
      const int s = (hi - lo) / 8;
      median3(lo, lo + s, lo + 2 * s);
      median3(m, m - s, m + s);
      median3(hi - 1, hi - 1 - s, hi - 1 - 2 * s);
    }
    median3(lo, m, hi - 1);

    const int p = lo;
    int a = lo + 1, c = hi - 1;
    while (a < c && lt(a, p)) ++a;
    int b = a;
    while (true) {
      while (b < c && !lt(p, b)) ++b;
      while (b < c && lt(p, c - 1)) --c;
      if (b >= c) break;
      sw(b, c - 1);
      ++b;
      --c;
    }
    bool protect = hi - c < 5;
    if (!protect && hi - c < (hi - lo) / 4) {
      int dups = 0;
      if (!lt(p, hi - 1)) {
        sw(c, hi - 1);
        ++c;
        ++dups;
      }
      if (!lt(b - 1, p)) {
        --b;
        ++dups;
      }
      if (!lt(m, p)) {
        sw(m, b - 1);
        --b;
        ++dups;
      }
      protect = dups > 1;
    }
    if (protect) {
      while (true) {
        while (a < b && !lt(b - 1, p)) --b;
        while (a < b && lt(a, p)) ++a;
        if (a >= b) break;
        sw(a, b - 1);
        ++a;
        --b;
      }
    }
    sw(p, b - 1);
    return {b - 1, c};
  }

  void quick(int a, int b, int depth) {
    while (b - a > 12) {
      if (depth == 0) {
        heap(a, b);
        return;
      }
      --depth;
      auto [mlo, mhi] = pivot(a, b);
      if (mlo - a < b - mhi) {
        quick(a, mlo, depth);
        a = mhi;
      } else {
        quick(mhi, b, depth);
        b = mlo;
      }
    }
    if (b - a > 1) {
      for (int i = a + 6; i < b; ++i)
        if (lt(i, i - 6)) sw(i, i - 6);
      insertion(a, b);
    }
  }
};

template <class T, class Less>
inline void go_sort_slice(T* data, int n, Less less) {
  GoSlice<T, Less>(data, less).sort(n);
}

// The same sort with the recursion's independent spans on a thread pool:
// partition steps level by level (each span's pivot and swaps are the serial
// sort's), then the remaining spans sorted in parallel.  Identical output:
// quickSort_func sorts the two sides of a pivot independently, and the side it
// recurses into first only changes its stack depth.
// par(n, fn): runs fn(i) for i in [0, n), in any order or concurrently.
template <class T, class Less, class Par>
inline void go_sort_slice_parallel(T* data, int n, Less less, Par par, int grain = 4096) {
  using S = GoSlice<T, Less>;
  using Span = typename S::Span;
  if (n <= 2 * grain) {
    S(data, less).sort(n);
    return;
  }
  std::vector<Span> level{Span{0, n, S::depth_of(n)}}, leaves;
  while (!level.empty() && leaves.size() < 256) {
    std::vector<Span> lo(level.size()), hi(level.size());
    std::vector<char> leaf(level.size());
    par(static_cast<int>(level.size()), [&](int i) {
      bool lf = false;
      S(data, less).split(level[static_cast<size_t>(i)], grain, &lo[static_cast<size_t>(i)], &hi[static_cast<size_t>(i)], &lf);
      leaf[static_cast<size_t>(i)] = lf;
    });
    std::vector<Span> next;
    for (size_t i = 0; i < level.size(); ++i) {
      if (leaf[i]) {
        leaves.push_back(level[i]);
      } else {
        next.push_back(lo[i]);
        next.push_back(hi[i]);
      }
    }
    level.swap(next);
  }
  leaves.insert(leaves.end(), level.begin(), level.end());
  par(static_cast<int>(leaves.size()), [&](int i) { S(data, less).finish(leaves[static_cast<size_t>(i)]); });
}

// Several independent slices, each sorted exactly as go_sort_slice would sort
// it, their spans sharing each level's pool dispatch.
template <class T, class Less, class Par>
inline void go_sort_slices_parallel(const std::vector<std::pair<T*, int>>& slices, Less less, Par par,
                                    int grain = 4096) {
  using S = GoSlice<T, Less>;
  using Span = typename S::Span;
  struct Item {
    T* data;
    Span sp;
  };
  std::vector<Item> level, leaves;
  for (const auto& sl : slices)
    if (sl.second > 1) (sl.second <= 2 * grain ? leaves : level).push_back(Item{sl.first, Span{0, sl.second, S::depth_of(sl.second)}});
  while (!level.empty() && leaves.size() < 256) {
    std::vector<Span> lo(level.size()), hi(level.size());
    std::vector<char> leaf(level.size());
    par(static_cast<int>(level.size()), [&](int i) {
      bool lf = false;
      const Item& it = level[static_cast<size_t>(i)];
      S(it.data, less).split(it.sp, grain, &lo[static_cast<size_t>(i)], &hi[static_cast<size_t>(i)], &lf);
      leaf[static_cast<size_t>(i)] = lf;
    });
    std::vector<Item> next;
    for (size_t i = 0; i < level.size(); ++i) {
      if (leaf[i]) {
        leaves.push_back(level[i]);
      } else {
        next.push_back(Item{level[i].data, lo[i]});
        next.push_back(Item{level[i].data, hi[i]});
      }
    }
    level.swap(next);
  }
  leaves.insert(leaves.end(), level.begin(), level.end());
  par(static_cast<int>(leaves.size()), [&](int i) {
    const Item& it = leaves[static_cast<size_t>(i)];
    S(it.data, less).finish(it.sp);
  });
}

}  // namespace sr
