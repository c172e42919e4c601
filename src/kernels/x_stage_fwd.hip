// x-stage forward launcher: space domain rows -> [z][column][y] (C2C, R2C);
// its own translation unit so the x-stage kernels compile in parallel.
// The packed-real R2C x stage runs the row-mapped engine (the first FFT pass
// loads the real rows directly) rather than the line-fast one with the rows
// staged through LDS: 58.9 -> 56.8 us at 256^3 (profiles/r2_s1/shape_ab.txt).
#include "kernels/stage_kernels.hpp"

namespace spfft {
namespace dev {

template <typename T>
void launch_x_forward(const XArgs& a, bool r2c, const void* space, cx<T>* inter,
                      const cx<T>* tw, const cx<T>* twHalf, hipStream_t stream) {
  if (a.L <= a.zBegin || a.Y <= 0) return;
  if (r2c && twHalf && a.n % 2 == 0 && a.n >= 4) {
    with_engine<T, -1, false>(a.n / 2, [&](auto eng, int threads, int lines, std::size_t lds) {
      auto k = x_forward_r2c_kernel<decltype(eng), T>;
      const std::size_t ldsTotal = lds + std::size_t(a.n / 2 + 1) * sizeof(int) + 16;
      prepare_kernel(k, ldsTotal);
      hipLaunchKernelGGL(k, dim3(ceil_div(a.Y, lines), a.L - a.zBegin, batch_dim(a.batch)), dim3(threads), ldsTotal,
                         stream, eng, a, static_cast<const T*>(space), inter, twHalf, tw);
      gpu_check_launch("x_forward_r2c", stream);
    });
    return;
  }
  with_engine<T, -1, true>(a.n, [&](auto eng, int threads, int lines, std::size_t lds) {
    auto k = r2c ? x_forward_kernel<decltype(eng), T, true> : x_forward_kernel<decltype(eng), T, false>;
    const std::size_t ldsTotal = lds + std::size_t(a.n) * sizeof(int) + 16;
    prepare_kernel(k, ldsTotal);
    hipLaunchKernelGGL(k, dim3(ceil_div(a.Y, lines), a.L - a.zBegin, batch_dim(a.batch)), dim3(threads), ldsTotal, stream, eng, a,
                       space, inter, tw);
    gpu_check_launch("x_forward", stream);
  });
}

template void launch_x_forward<double>(const XArgs&, bool, const void*, cx<double>*,
                                       const cx<double>*, const cx<double>*, hipStream_t);
template void launch_x_forward<float>(const XArgs&, bool, const void*, cx<float>*,
                                      const cx<float>*, const cx<float>*, hipStream_t);

}  // namespace dev
}  // namespace spfft
