// x-stage kernels, fp64 transforms, and the host helpers of the stage engines
// (run-time plans, Bluestein tables, engine descriptions).
#include <string>
#include <vector>
#include <tuple>
#include <mutex>
#include <map>

#include "kernels/stage_launch.hpp"

// after the HIP headers (codelets use __forceinline__ under hipcc)
#include "fft/host_fft.hpp"

namespace spfft {
namespace dev {

template void launch_x_backward<double>(const XArgs&, bool, const cx<double>*, void*, const cx<double>*,
                                     const cx<double>*, hipStream_t);
template void launch_x_forward<double>(const XArgs&, bool, const void*, cx<double>*, const cx<double>*,
                                    const cx<double>*, hipStream_t);

// ------------------------------------------------------------------ helpers
namespace {
RtPlan make_rt_plan_from(int n, std::size_t elemBytes, const std::vector<int>& r, bool pfa) {
  RtPlan p{};
  p.n = n;
  if (r.size() > 16) throw GPUFFTError();
  p.np = static_cast<int>(r.size());
  auto magic = [](long long d) -> unsigned {
    return d <= 1 ? 0u : static_cast<unsigned>(((1ull << 32) + d - 1) / d);
  };
  p.inplace = 1;
  long long ns = 1;
  for (int i = 0; i < p.np; ++i) {
    p.radix[i] = r[i];
    p.nsMagic[i] = magic(ns);
    ns *= r[i];
    if (!rt_codelet_radix(r[i], pfa)) p.inplace = 0;
  }
  p.nMagic = magic(n);
  // the register staging of the in-place passes is sized for lines * n <= kRtElems
  // and rt_iters(R) butterflies per lane in a pass of radix R
  if (n > kRtElems) p.inplace = 0;
  auto fits = [&](int log2) {
    for (int i = 0; i < p.np; ++i)
      if ((static_cast<long long>(n / p.radix[i]) << log2) >
          static_cast<long long>(rt_iters(p.radix[i])) * kRtThreads)
        return false;
    return true;
  };
  if (!fits(0)) p.inplace = 0;  // a pass too long for one workgroup: ping-pong passes
  const std::size_t budget =
      p.inplace ? static_cast<std::size_t>(kRtElems) * elemBytes : static_cast<std::size_t>(kLdsBudget);
  // in-place plans keep one LDS region; ping-pong plans (a generic prime pass) two
  const std::size_t regions = p.inplace ? 1 : 2;
  if (regions * static_cast<std::size_t>(n + 1) * elemBytes > 160 * 1024) throw GPUFFTError();
  // Lines: a power of two (line-fast engines split lane indices with shifts).
  // Line stride: the passes run lines fastest, so a 16-lane LDS access group
  // spans lines; lds_line_stride_ok puts them on distinct bank slots (the rule
  // of the compile-time line-fast engines, fft_device.hpp).
  int lines = static_cast<int>(budget / (regions * static_cast<std::size_t>(n + 1) * elemBytes));
  if (lines > kMaxThreads) lines = kMaxThreads;
  if (lines < 1) lines = 1;
  p.linesLog2 = 0;
  while ((2 << p.linesLog2) <= lines) ++p.linesLog2;
  if (p.inplace)
    while (p.linesLog2 > 0 && !fits(p.linesLog2)) --p.linesLog2;
  for (;;) {
    p.lines = 1 << p.linesLog2;
    p.ls = n;
    while (!lds_line_stride_ok(p.ls, p.lines, static_cast<int>(elemBytes))) ++p.ls;
    if (p.linesLog2 == 0 || regions * p.lines * static_cast<std::size_t>(p.ls) * elemBytes <= budget)
      break;
    --p.linesLog2;
  }
  return p;
}
}  // namespace

RtPlan make_rt_plan(int n, std::size_t elemBytes) {
  // fewest-pass plans over the composite codelets (6, 10, 12, 15, 20) where the
  // kernels instantiate them; ping-pong plans (a generic prime pass, or lines too
  // long for the in-place staging) keep the prime radices
  if (rt_pfa(elemBytes == sizeof(cx<double>))) {
    const RtPlan p = make_rt_plan_from(n, elemBytes, stockham_radices(n), true);
    if (p.inplace) return p;
  }
  return make_rt_plan_from(n, elemBytes, factorize_radices(n), false);
}

std::string describe_engine(int n, bool dbl, bool lineFast) {
  std::string out;
  auto fmt = [&](auto eng, int threads, int lines, std::size_t lds) {
    (void)eng;
    out = "n=" + std::to_string(n) + " lines=" + std::to_string(lines) + " threads=" +
          std::to_string(threads) + " lds=" + std::to_string(lds);
  };
  if (dbl) {
    if (lineFast) with_engine<double, +1, true>(n, fmt);
    else with_engine<double, +1, false>(n, fmt);
  } else {
    if (lineFast) with_engine<float, +1, true>(n, fmt);
    else with_engine<float, +1, false>(n, fmt);
  }
  return (has_ct_kernel(n) ? "ct " : "rt ") + out;
}

// ------------------------------------------------------------- Bluestein
bool use_bluestein(int n, std::size_t elemBytes) {
  if (n < 2 || has_ct_kernel(n)) return false;
  const std::vector<int> r = factorize_radices(n);
  if (r.empty() || r.back() <= kBluesteinPrime) return false;
  int m = 1;
  while (m < 2 * n - 1) m *= 2;
  return 2 * static_cast<std::size_t>(m) * elemBytes <= 160 * 1024;
}

namespace {
template <typename T>
void fill_bluestein(int n, int m, std::vector<cx<T>>& chirp, std::vector<cx<T>>& filt,
                    std::vector<cx<T>>& tw) {
  const long double pi = 3.141592653589793238462643383279502884L;
  chirp.resize(n);
  for (int j = 0; j < n; ++j) {
    const long long q = (static_cast<long long>(j) * j) % (2LL * n);
    const long double a = pi * static_cast<long double>(q) / static_cast<long double>(n);
    chirp[j] = mk<T>(static_cast<T>(std::cos(a)), static_cast<T>(-std::sin(a)));
  }
  // filters: FFT_m of b (b_j = conj(d_j), b_{m-j} = conj(d_j)), computed on the host
  // in long double precision via the host engine in double
  HostFft<double> fft(m);
  std::vector<cx<double>> work(fft.scratch_size()), b(m);
  filt.resize(2 * static_cast<std::size_t>(m));
  for (int s = 0; s < 2; ++s) {
    for (auto& v : b) v = mk<double>(0.0, 0.0);
    for (int j = 0; j < n; ++j) {
      const long long q = (static_cast<long long>(j) * j) % (2LL * n);
      const long double a = pi * static_cast<long double>(q) / static_cast<long double>(n);
      // conj(d_j) with d_j = exp(S i a): S = -1 -> exp(+i a), S = +1 -> exp(-i a)
      const cx<double> c = mk<double>(static_cast<double>(std::cos(a)),
                                      static_cast<double>(s == 0 ? std::sin(a) : -std::sin(a)));
      b[j] = c;
      if (j > 0) b[m - j] = c;
    }
    fft.execute(b.data(), 1, b.data(), 1, -1, work.data());
    for (int j = 0; j < m; ++j)
      filt[static_cast<std::size_t>(s) * m + j] = mk<T>(static_cast<T>(b[j].x), static_cast<T>(b[j].y));
  }
  tw = make_twiddles<T>(m);
}
}  // namespace

BlueTables bluestein_tables(int n, bool dbl) {
  static std::mutex mutex;
  static std::map<std::tuple<int, int, bool>, std::pair<BlueTables, DeviceBuffer*>> cache;
  int device = 0;
  gpu_check(hipGetDevice(&device), "hipGetDevice");
  std::lock_guard<std::mutex> lock(mutex);
  auto it = cache.find(std::make_tuple(device, n, dbl));
  if (it != cache.end()) return it->second.first;
  int m = 1;
  while (m < 2 * n - 1) m *= 2;
  const std::size_t eb = dbl ? sizeof(cx<double>) : sizeof(cx<float>);
  BlueTables t;
  t.pm = make_rt_plan(m, eb);
  t.pm.ls = m;
  t.pm.lines = std::max<std::size_t>(1, kLdsBudget / (2 * static_cast<std::size_t>(m) * eb));
  if (t.pm.lines > 16) t.pm.lines = 16;
  // one allocation: chirp [n] | filters [2m] | twiddles [m]; lives for the process
  auto* buf = new DeviceBuffer((static_cast<std::size_t>(n) + 3 * static_cast<std::size_t>(m)) * eb);
  auto upload = [&](auto& chirp, auto& filt, auto& tw) {
    char* base = buf->data<char>();
    gpu_check(hipMemcpy(base, chirp.data(), n * eb, hipMemcpyHostToDevice), "hipMemcpy");
    gpu_check(hipMemcpy(base + n * eb, filt.data(), 2 * m * eb, hipMemcpyHostToDevice), "hipMemcpy");
    gpu_check(hipMemcpy(base + (n + 2 * static_cast<std::size_t>(m)) * eb, tw.data(), m * eb,
                        hipMemcpyHostToDevice),
              "hipMemcpy");
    t.chirp = base;
    t.filt = base + n * eb;
    t.twm = base + (n + 2 * static_cast<std::size_t>(m)) * eb;
  };
  if (dbl) {
    std::vector<cx<double>> c, f, w;
    fill_bluestein<double>(n, m, c, f, w);
    upload(c, f, w);
  } else {
    std::vector<cx<float>> c, f, w;
    fill_bluestein<float>(n, m, c, f, w);
    upload(c, f, w);
  }
  cache.emplace(std::make_tuple(device, n, dbl), std::make_pair(t, buf));
  return t;
}

std::size_t in_lds_engine_bytes(int n, std::size_t elemBytes, int& lines) {
  if (use_bluestein(n, elemBytes)) {
    int m = 1;
    while (m < 2 * n - 1) m *= 2;
    lines = static_cast<int>(std::min<std::size_t>(
        16, std::max<std::size_t>(1, kLdsBudget / (2 * static_cast<std::size_t>(m) * elemBytes))));
    return 2 * static_cast<std::size_t>(lines) * m * elemBytes;
  }
  const RtPlan p = make_rt_plan(n, elemBytes);
  lines = p.lines;
  return static_cast<std::size_t>(p.inplace ? 1 : 2) * p.lines * p.ls * elemBytes;
}

int max_device_fft_length(bool dbl) { return (160 * 1024) / (2 * (dbl ? 16 : 8)) - 1; }

bool has_ct_kernel(int n) {
  switch (n) {
    case 16: case 32: case 64: case 128: case 256: case 512: case 1024:
#define SPFFT_MR_HAS(NN) case NN:
    SPFFT_MR_SIZES(SPFFT_MR_HAS)
#undef SPFFT_MR_HAS
      return true;
    default:
      return false;
  }
}

}  // namespace dev
}  // namespace spfft
