// x-stage launchers: [z][column][y] <-> space domain rows (C2C, C2R, R2C).
#include <string>

#include "kernels/stage_kernels.hpp"

namespace spfft {
namespace dev {

template <typename T>
void launch_x_backward(const XArgs& a, bool r2c, const cx<T>* inter, void* space,
                       const cx<T>* tw, const cx<T>* twHalf, hipStream_t stream) {
  if (a.L <= a.zBegin || a.Y <= 0) return;
  if (r2c && twHalf && a.n % 2 == 0 && a.n >= 4) {
    with_engine<T, +1, true>(a.n / 2, [&](auto eng, int threads, int lines, std::size_t lds) {
      auto k = x_backward_c2r_kernel<decltype(eng), T>;
      const std::size_t ldsTotal =
          lds + std::size_t(lines) * sizeof(cx<T>) + std::size_t(a.n / 2 + 1) * sizeof(int) + 16;
      prepare_kernel(k, ldsTotal);
      hipLaunchKernelGGL(k, dim3(ceil_div(a.Y, lines), a.L - a.zBegin), dim3(threads), ldsTotal,
                         stream, eng, a, inter, static_cast<T*>(space), twHalf, tw);
      gpu_check_launch("x_backward_c2r", stream);
    });
    return;
  }
  with_engine<T, +1, true>(a.n, [&](auto eng, int threads, int lines, std::size_t lds) {
    auto k = r2c ? x_backward_kernel<decltype(eng), T, true> : x_backward_kernel<decltype(eng), T, false>;
    const std::size_t ldsTotal = lds + std::size_t(a.n) * sizeof(int) + 16;
    prepare_kernel(k, ldsTotal);
    hipLaunchKernelGGL(k, dim3(ceil_div(a.Y, lines), a.L - a.zBegin), dim3(threads), ldsTotal, stream, eng, a,
                       inter, space, tw);
    gpu_check_launch("x_backward", stream);
  });
}

template <typename T>
void launch_x_forward(const XArgs& a, bool r2c, const void* space, cx<T>* inter,
                      const cx<T>* tw, const cx<T>* twHalf, hipStream_t stream) {
  if (a.L <= a.zBegin || a.Y <= 0) return;
  if (r2c && twHalf && a.n % 2 == 0 && a.n >= 4) {
    with_engine<T, -1, true>(a.n / 2, [&](auto eng, int threads, int lines, std::size_t lds) {
      auto k = x_forward_r2c_kernel<decltype(eng), T>;
      const std::size_t ldsTotal = lds + std::size_t(a.n / 2 + 1) * sizeof(int) + 16;
      prepare_kernel(k, ldsTotal);
      hipLaunchKernelGGL(k, dim3(ceil_div(a.Y, lines), a.L - a.zBegin), dim3(threads), ldsTotal,
                         stream, eng, a, static_cast<const T*>(space), inter, twHalf, tw);
      gpu_check_launch("x_forward_r2c", stream);
    });
    return;
  }
  with_engine<T, -1, true>(a.n, [&](auto eng, int threads, int lines, std::size_t lds) {
    auto k = r2c ? x_forward_kernel<decltype(eng), T, true> : x_forward_kernel<decltype(eng), T, false>;
    const std::size_t ldsTotal = lds + std::size_t(a.n) * sizeof(int) + 16;
    prepare_kernel(k, ldsTotal);
    hipLaunchKernelGGL(k, dim3(ceil_div(a.Y, lines), a.L - a.zBegin), dim3(threads), ldsTotal, stream, eng, a,
                       space, inter, tw);
    gpu_check_launch("x_forward", stream);
  });
}

template void launch_x_backward<double>(const XArgs&, bool, const cx<double>*, void*,
                                        const cx<double>*, const cx<double>*, hipStream_t);
template void launch_x_backward<float>(const XArgs&, bool, const cx<float>*, void*,
                                       const cx<float>*, const cx<float>*, hipStream_t);
template void launch_x_forward<double>(const XArgs&, bool, const void*, cx<double>*,
                                       const cx<double>*, const cx<double>*, hipStream_t);
template void launch_x_forward<float>(const XArgs&, bool, const void*, cx<float>*,
                                      const cx<float>*, const cx<float>*, hipStream_t);

// ------------------------------------------------------------------ helpers
RtPlan make_rt_plan(int n, std::size_t elemBytes) {
  RtPlan p{};
  p.n = n;
  const std::vector<int> r = factorize_radices(n);
  if (r.size() > 16) throw GPUFFTError();
  p.np = static_cast<int>(r.size());
  for (int i = 0; i < p.np; ++i) p.radix[i] = r[i];
  p.ls = n + 1;
  const std::size_t line = 2 * static_cast<std::size_t>(p.ls) * elemBytes;
  if (line > 160 * 1024) throw GPUFFTError();
  int lines = static_cast<int>(kLdsBudget / line);
  if (lines > kMaxThreads) lines = kMaxThreads;
  if (lines < 1) lines = 1;
  p.lines = lines;
  return p;
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

int max_device_fft_length(bool dbl) { return (160 * 1024) / (2 * (dbl ? 16 : 8)) - 1; }

bool has_ct_kernel(int n) {
  return n == 16 || n == 32 || n == 64 || n == 128 || n == 256 || n == 512 || n == 1024;
}

}  // namespace dev
}  // namespace spfft
