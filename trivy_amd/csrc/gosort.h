// Go's sort.Slice (go1.23 sort/zsortfunc.go pdqsort_func) restated: the
// reference sorts findings with sort.Slice (scanner.go:452-457,
// analyzer.go:224-235), which is unstable for n > 12, so equal keys keep
// Go's order only if the algorithm is the same.
#pragma once
#include <cstdint>
#include <functional>
#include <utility>
#include <vector>

namespace tsg {

template <typename T>
class GoSort {
 public:
  using Less = std::function<bool(size_t, size_t)>;
  GoSort(std::vector<T>* v, Less less) : v_(v), less_(std::move(less)) {}
  void run() {
    size_t n = v_->size();
    int limit = 0;
    for (size_t x = n; x; x >>= 1) ++limit;
    pdq(0, static_cast<long>(n), limit);
  }

 private:
  std::vector<T>* v_;
  Less less_;
  bool lt(long i, long j) { return less_(i, j); }
  void sw(long i, long j) { std::swap((*v_)[i], (*v_)[j]); }

  void ins(long a, long b) {
    for (long i = a + 1; i < b; ++i)
      for (long j = i; j > a && lt(j, j - 1); --j) sw(j, j - 1);
  }
  void sift(long lo, long hi, long first) {
    long root = lo;
    for (;;) {
      long child = 2 * root + 1;
      if (child >= hi) return;
      if (child + 1 < hi && lt(first + child, first + child + 1)) ++child;
      if (!lt(first + root, first + child)) return;
      sw(first + root, first + child);
      root = child;
    }
  }
  void heap(long a, long b) {
    long first = a, lo = 0, hi = b - a;
    for (long i = (hi - 1) / 2; i >= 0; --i) sift(i, hi, first);
    for (long i = hi - 1; i >= 0; --i) { sw(first, first + i); sift(lo, i, first); }
  }
  enum Hint { kUnknown, kIncreasing, kDecreasing };
  void pdq(long a, long b, int limit) {
    bool was_balanced = true, was_partitioned = true;
    for (;;) {
      long length = b - a;
      if (length <= 12) { ins(a, b); return; }
      if (limit == 0) { heap(a, b); return; }
      if (!was_balanced) { break_patterns(a, b); --limit; }
      Hint hint;
      long pivot = choose_pivot(a, b, &hint);
      if (hint == kDecreasing) {
        reverse(a, b);
        pivot = (b - 1) - (pivot - a);
        hint = kIncreasing;
      }
      if (was_balanced && was_partitioned && hint == kIncreasing) {
        if (partial_ins(a, b)) return;
      }
      if (a > 0 && !lt(a - 1, pivot)) {
        a = partition_equal(a, b, pivot);
        continue;
      }
      bool already;
      long mid = partition(a, b, pivot, &already);
      was_partitioned = already;
      long left = mid - a, right = b - mid;
      long thr = length / 8;
      if (left < right) {
        was_balanced = left >= thr;
        pdq(a, mid, limit);
        a = mid + 1;
      } else {
        was_balanced = right >= thr;
        pdq(mid + 1, b, limit);
        b = mid;
      }
    }
  }
  long partition(long a, long b, long pivot, bool* already) {
    sw(a, pivot);
    long i = a + 1, j = b - 1;
    while (i <= j && lt(i, a)) ++i;
    while (i <= j && !lt(j, a)) --j;
    if (i > j) { sw(j, a); *already = true; return j; }
    sw(i, j); ++i; --j;
    for (;;) {
      while (i <= j && lt(i, a)) ++i;
      while (i <= j && !lt(j, a)) --j;
      if (i > j) break;
      sw(i, j); ++i; --j;
    }
    sw(j, a);
    *already = false;
    return j;
  }
  long partition_equal(long a, long b, long pivot) {
    sw(a, pivot);
    long i = a + 1, j = b - 1;
    for (;;) {
      while (i <= j && !lt(a, i)) ++i;
      while (i <= j && lt(a, j)) --j;
      if (i > j) break;
      sw(i, j); ++i; --j;
    }
    return i;
  }
  bool partial_ins(long a, long b) {
    long i = a + 1;
    for (int step = 0; step < 5; ++step) {
      while (i < b && !lt(i, i - 1)) ++i;
      if (i == b) return true;
      if (b - a < 50) return false;
      sw(i, i - 1);
      if (i - a >= 2) {
        for (long j = i - 1; j >= 1; --j) { if (!lt(j, j - 1)) break; sw(j, j - 1); }
      }
      if (b - i >= 2) {
        for (long j = i + 1; j < b; ++j) { if (!lt(j, j - 1)) break; sw(j, j - 1); }
      }
    }
    return false;
  }
  void break_patterns(long a, long b) {
    long length = b - a;
    if (length >= 8) {
      uint64_t r = static_cast<uint64_t>(length);
      int bits = 0;
      for (uint64_t x = static_cast<uint64_t>(length); x; x >>= 1) ++bits;
      uint64_t modulus = 1ull << bits;
      long idx = a + (length / 4) * 2 - 1;
      for (int i = 0; i < 3; ++i) {
        r ^= r << 13; r ^= r >> 7; r ^= r << 17;
        long other = static_cast<long>(r & (modulus - 1));
        if (other >= length) other -= length;
        sw(idx - 1 + i, a + other);
      }
    }
  }
  long median(long x, long y, long z, int* swaps) {
    auto order2 = [&](long& p, long& q) { if (lt(q, p)) { ++*swaps; std::swap(p, q); } };
    order2(x, y);
    order2(y, z);
    order2(x, y);
    return y;
  }
  long choose_pivot(long a, long b, Hint* hint) {
    long l = b - a;
    int swaps = 0;
    long i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
      if (l >= 50) {
        i = median(i - 1, i, i + 1, &swaps);
        j = median(j - 1, j, j + 1, &swaps);
        k = median(k - 1, k, k + 1, &swaps);
      }
      j = median(i, j, k, &swaps);
    }
    *hint = swaps == 0 ? kIncreasing : swaps == 12 ? kDecreasing : kUnknown;
    return j;
  }
  void reverse(long a, long b) {
    for (long i = a, j = b - 1; i < j; ++i, --j) sw(i, j);
  }
};

}  // namespace tsg
