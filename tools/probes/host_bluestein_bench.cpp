// Host prime-length throughput: W lines at a time through the batched engine
// (HostFftBatch: Rader for primes with a smooth n - 1, else Bluestein) against
// the scalar engine line by line (HostFft, the round-3 path for lengths with a
// prime factor above kBluesteinPrime).
//   clang++ -O3 -march=x86-64-v3 -std=c++17 -I src tools/probes/host_bluestein_bench.cpp
#include <chrono>
#include <cstdio>
#include <vector>

#include "fft/host_fft_batch.hpp"

using namespace spfft;

template <typename T>
void bench(int n, int lines) {
  using B = HostFftBatch<T>;
  using VC = typename B::VC;
  constexpr int W = B::W;
  B fb(n);
  HostFft<T> fs(n);
  std::vector<VC> a(n), b(n);
  std::vector<cx<T>> line(n), work(fs.scratch_size());
  for (int i = 0; i < n; ++i)
    for (int l = 0; l < W; ++l) set_lane<T>(a[i], l, mk<T>(T(i % 7) - 3, T(l)));
  // correctness: lane 0 of the batch against the scalar engine
  for (int i = 0; i < n; ++i) line[i] = lane<T>(a[i], 0);
  std::vector<VC> c = a;
  fb.run(c.data(), b.data(), -1);
  fs.execute(line.data(), 1, line.data(), 1, -1, work.data());
  double err = 0;
  for (int i = 0; i < n; ++i) {
    const cx<T> d = lane<T>(c[i], 0) - line[i];
    err = std::max(err, double(std::abs(d.x) + std::abs(d.y)));
  }
  using clk = std::chrono::steady_clock;
  auto t0 = clk::now();
  for (int k = 0; k < lines / W; ++k) fb.run(a.data(), b.data(), k & 1 ? 1 : -1);
  auto t1 = clk::now();
  for (int k = 0; k < lines; ++k) {
    for (int i = 0; i < n; ++i) line[i] = lane<T>(a[i], k % W);
    fs.execute(line.data(), 1, line.data(), 1, k & 1 ? 1 : -1, work.data());
    for (int i = 0; i < n; ++i) set_lane<T>(a[i], k % W, line[i]);
  }
  auto t2 = clk::now();
  const double tb = std::chrono::duration<double>(t1 - t0).count(), ts = std::chrono::duration<double>(t2 - t1).count();
  std::printf("%s n=%d bluestein=%d rader=%d: batched %.1f ns/line, scalar %.1f ns/line, speed-up %.2fx, max diff %.2e\n",
              sizeof(T) == 8 ? "fp64" : "fp32", n, fb.bluestein() ? 1 : 0, fb.rader() ? 1 : 0, 1e9 * tb / lines, 1e9 * ts / lines,
              ts / tb, err);
}

int main() {
  for (int n : {101, 211, 1009, 2 * 101, 67}) {
    bench<double>(n, 40000);
    bench<float>(n, 40000);
  }
  return 0;
}
