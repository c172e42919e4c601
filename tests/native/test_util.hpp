// Minimal self-contained test harness + dense DFT oracle for the native C/C++
// test programs (gtest is not available offline; reference: tests/test_util/).
#pragma once

#include <cmath>
#include <complex>
#include <cstdio>
#include <functional>
#include <random>
#include <string>
#include <vector>

namespace spfft_test {

using cd = std::complex<double>;

struct Registry {
  std::vector<std::pair<std::string, std::function<void()>>> tests;
  static Registry& get() {
    static Registry r;
    return r;
  }
};

struct Failure {
  std::string what;
};

#define SPFFT_TEST(NAME)                                                             \
  static void NAME();                                                                \
  static int NAME##_reg = (spfft_test::Registry::get().tests.emplace_back(#NAME, NAME), 0); \
  static void NAME()

#define EXPECT_TRUE(c)                                                                       \
  do {                                                                                       \
    if (!(c)) throw spfft_test::Failure{std::string(__FILE__) + ":" + std::to_string(__LINE__) + ": " #c}; \
  } while (0)

#define EXPECT_EQ(a, b) EXPECT_TRUE((a) == (b))

template <class E, class F>
void expect_throw(F&& f, const char* what) {
  try {
    f();
  } catch (const E&) {
    return;
  } catch (...) {
    throw Failure{std::string("wrong exception type: ") + what};
  }
  throw Failure{std::string("no exception: ") + what};
}

inline int run_all(int rank = 0) {
  int failed = 0;
  for (auto& t : Registry::get().tests) {
    try {
      t.second();
      if (rank == 0) std::printf("[       OK ] %s\n", t.first.c_str());
    } catch (const Failure& f) {
      ++failed;
      std::printf("[  FAILED  ] %s (rank %d): %s\n", t.first.c_str(), rank, f.what.c_str());
    } catch (const std::exception& e) {
      ++failed;
      std::printf("[  FAILED  ] %s (rank %d): exception %s\n", t.first.c_str(), rank, e.what());
    }
  }
  if (rank == 0) std::printf("%zu tests, %d failed\n", Registry::get().tests.size(), failed);
  return failed;
}

// dense cube F[x][y][z] -> its 1D DFTs along every axis with exp(sign 2 pi i ...)
inline void dft_axis(std::vector<cd>& a, int nx, int ny, int nz, int axis, int sign) {
  const int n = axis == 0 ? nx : (axis == 1 ? ny : nz);
  std::vector<cd> w(n), line(n), out(n);
  for (int k = 0; k < n; ++k) {
    const double ang = sign * 2.0 * M_PI * k / n;
    w[k] = cd(std::cos(ang), std::sin(ang));
  }
  auto at = [&](int x, int y, int z) -> cd& { return a[(static_cast<size_t>(x) * ny + y) * nz + z]; };
  const int o1 = axis == 0 ? ny : nx, o2 = axis == 2 ? ny : nz;
  for (int i = 0; i < o1; ++i)
    for (int j = 0; j < o2; ++j) {
      for (int k = 0; k < n; ++k)
        line[k] = axis == 0 ? at(k, i, j) : (axis == 1 ? at(i, k, j) : at(i, j, k));
      for (int k = 0; k < n; ++k) {
        cd s = 0;
        for (int m = 0; m < n; ++m) s += line[m] * w[(static_cast<long long>(k) * m) % n];
        out[k] = s;
      }
      for (int k = 0; k < n; ++k)
        (axis == 0 ? at(k, i, j) : (axis == 1 ? at(i, k, j) : at(i, j, k))) = out[k];
    }
}

inline int storage(int n, int i) { return i < 0 ? i + n : i; }

// sparse (x,y,z) triplets + values -> dense space domain [z][y][x] (backward, unnormalised)
inline std::vector<cd> dense_backward(const std::vector<int>& idx, const std::vector<cd>& vals,
                                      int nx, int ny, int nz) {
  std::vector<cd> F(static_cast<size_t>(nx) * ny * nz);
  for (size_t i = 0; i < vals.size(); ++i)
    F[(static_cast<size_t>(storage(nx, idx[3 * i])) * ny + storage(ny, idx[3 * i + 1])) * nz +
      storage(nz, idx[3 * i + 2])] = vals[i];
  for (int ax = 0; ax < 3; ++ax) dft_axis(F, nx, ny, nz, ax, +1);
  std::vector<cd> S(F.size());
  for (int x = 0; x < nx; ++x)
    for (int y = 0; y < ny; ++y)
      for (int z = 0; z < nz; ++z) S[(static_cast<size_t>(z) * ny + y) * nx + x] = F[(static_cast<size_t>(x) * ny + y) * nz + z];
  return S;
}

// random sparse index set: each stick kept with probability pStick, each z with pFill
inline std::vector<int> random_indices(std::mt19937& rng, int nx, int ny, int nz, double pStick,
                                       double pFill, bool centered) {
  std::uniform_real_distribution<double> u(0.0, 1.0);
  std::vector<int> idx;
  for (int x = 0; x < nx; ++x)
    for (int y = 0; y < ny; ++y) {
      if (u(rng) >= pStick) continue;
      for (int z = 0; z < nz; ++z) {
        if (u(rng) >= pFill) continue;
        int t[3] = {x, y, z};
        const int d[3] = {nx, ny, nz};
        if (centered)
          for (int k = 0; k < 3; ++k)
            if (t[k] >= d[k] / 2 + 1) t[k] -= d[k];
        idx.insert(idx.end(), t, t + 3);
      }
    }
  return idx;
}

inline double max_rel(const cd* a, const cd* b, size_t n) {
  double m = 0, r = 1e-300;
  for (size_t i = 0; i < n; ++i) {
    m = std::max(m, std::abs(a[i] - b[i]));
    r = std::max(r, std::abs(b[i]));
  }
  return m / r;
}

}  // namespace spfft_test
