// Radix factorisation and twiddle tables shared by host and GPU engines.
#pragma once

#include <cmath>
#include <cstdint>
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
