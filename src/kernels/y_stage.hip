// y-stage launchers: exchange layout <-> [z][column][y] with the y-FFT.
#include "kernels/stage_kernels.hpp"

namespace spfft {
namespace dev {

template <typename T, typename BT>
void launch_y_backward(const YArgs& a, const BT* in, cx<T>* inter, const cx<T>* tw,
                       hipStream_t stream) {
  if (a.colEnd <= a.colBegin || a.L <= a.zBegin) return;
  with_engine<T, +1, true>(a.n, [&](auto eng, int threads, int lines, std::size_t lds) {
    auto k = y_backward_kernel<decltype(eng), T, BT>;
    const std::size_t ldsTotal = lds + col_entries_lds(a, true, y_table<decltype(eng), true>());
    prepare_kernel(k, ldsTotal);
    hipLaunchKernelGGL(k, y_grid(a.colEnd - a.colBegin, ceil_div(a.L - a.zBegin, lines), batch_dim(a.batch)), dim3(threads), ldsTotal, stream, eng, a,
                       in, inter, tw);
    gpu_check_launch("y_backward", stream);
  });
}

template void launch_y_backward<double, cx<double>>(const YArgs&, const cx<double>*, cx<double>*,
                                                    const cx<double>*, hipStream_t);
template void launch_y_backward<double, cx<float>>(const YArgs&, const cx<float>*, cx<double>*,
                                                   const cx<double>*, hipStream_t);
template void launch_y_backward<float, cx<float>>(const YArgs&, const cx<float>*, cx<float>*,
                                                  const cx<float>*, hipStream_t);

}  // namespace dev
}  // namespace spfft
