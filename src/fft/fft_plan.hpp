// Radix factorisation and twiddle tables shared by host and GPU engines.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <functional>
#include <map>
#include <vector>

#include "fft/codelets.hpp"

namespace spfft {

// Factorises n into the radices executed by the Stockham passes. Prefers the
// large power-of-two codelets (fewer passes = fewer LDS / memory round trips),
// then the odd codelets, then any remaining prime (generic O(R) path).
inline std::vector<int> factorize_radices(int n) {
  std::vector<int> r;
  if (n <= 1) return r;
  while (n % 16 == 0) {
    r.push_back(16);
    n /= 16;
  }
  for (int f : {8, 4, 2}) {
    if (n % f == 0) {
      r.push_back(f);
      n /= f;
    }
  }
  for (int f : {9, 3, 5, 7, 11, 13}) {
    while (n % f == 0) {
      r.push_back(f);
      n /= f;
    }
  }
  for (int p = 17; n > 1 && static_cast<long long>(p) * p <= n; p += 2) {
    while (n % p == 0) {
      r.push_back(p);
      n /= p;
    }
  }
  if (n > 1) r.push_back(n);
  return r;
}

// Radix plan of the host Stockham engine (and of the GPU run-time engine's fp64
// in-place plans, see rt_pfa): the fewest passes over the codelets (incl. the
// prime-factor composites 6, 10, 12, 15, 20), then the
// fewest non-power-of-two passes, then larger radices first; power-of-two
// radices lead. Factors without a codelet (primes > 13) keep their own passes.
// Example: 240 = 16 * 15 (2 passes) instead of 16 * 3 * 5.
inline std::vector<int> stockham_radices(int n) {
  static const int kCand[] = {20, 16, 15, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2};
  auto codelet = [&](int r) {
    for (int c : kCand)
      if (c == r) return true;
    return false;
  };
  std::vector<int> rest;
  long long m = 1;
  for (int r : factorize_radices(n)) {
    if (codelet(r))
      m *= r;
    else
      rest.push_back(r);
  }
  struct Best {
    int passes = 1 << 20, odd = 1 << 20;
    std::vector<int> seq;  // descending
  };
  std::map<long long, Best> memo;
  std::function<Best(long long)> solve = [&](long long v) -> Best {
    Best best;
    if (v == 1) {
      best.passes = best.odd = 0;
      return best;
    }
    auto it = memo.find(v);
    if (it != memo.end()) return it->second;
    for (int c : kCand) {
      if (v % c) continue;
      const Best sub = solve(v / c);
      const int passes = sub.passes + 1, odd = sub.odd + ((c & (c - 1)) ? 1 : 0);
      std::vector<int> seq = sub.seq;
      seq.push_back(c);
      std::sort(seq.begin(), seq.end(), [](int a, int b) { return a > b; });
      if (passes < best.passes || (passes == best.passes && odd < best.odd) ||
          (passes == best.passes && odd == best.odd && seq > best.seq)) {
        best.passes = passes;
        best.odd = odd;
        best.seq = seq;
      }
    }
    memo[v] = best;
    return best;
  };
  const std::vector<int> seq = solve(m).seq;
  std::vector<int> out;
  for (int r : seq)
    if (!(r & (r - 1))) out.push_back(r);
  for (int r : seq)
    if (r & (r - 1)) out.push_back(r);
  out.insert(out.end(), rest.begin(), rest.end());
  return out;
}

// tw[m] = exp(-2 pi i m / n), m in [0, n), rounded from long double.
template <typename T>
std::vector<cx<T>> make_twiddles(int n) {
  std::vector<cx<T>> tw(static_cast<std::size_t>(n > 0 ? n : 1));
  const long double twoPi = 6.283185307179586476925286766559005768L;
  for (int m = 0; m < n; ++m) {
    // reduce to the first octant-ish range by symmetry for accuracy
    const long double a = twoPi * static_cast<long double>(m) / static_cast<long double>(n);
    tw[m].x = static_cast<T>(std::cos(a));
    tw[m].y = static_cast<T>(-std::sin(a));
  }
  if (n % 4 == 0) {  // exact values at the quarter points
    tw[n / 4].x = T(0);
    tw[n / 4].y = T(-1);
    if (n / 2 < n) {
      tw[n / 2].x = T(-1);
      tw[n / 2].y = T(0);
    }
    tw[3 * n / 4].x = T(0);
    tw[3 * n / 4].y = T(1);
  } else if (n % 2 == 0) {
    tw[n / 2].x = T(-1);
    tw[n / 2].y = T(0);
  }
  return tw;
}

}  // namespace spfft
