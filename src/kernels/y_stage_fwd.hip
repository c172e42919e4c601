// y-stage forward launcher: [z][column][y] -> exchange layout with the y-FFT
// (its own translation unit so the y-stage kernels compile in parallel).
#include "kernels/stage_kernels.hpp"

namespace spfft {
namespace dev {

template <typename T, typename BT>
void launch_y_forward(const YArgs& a, const cx<T>* inter, BT* out, const cx<T>* tw,
                      hipStream_t stream) {
  if (a.colEnd <= a.colBegin || a.L <= a.zBegin) return;
  with_engine<T, -1, true, !std::is_same<T, float>::value>(a.n, [&](auto eng, int threads, int lines, std::size_t lds) {
    auto k = y_forward_kernel<decltype(eng), T, BT>;
    const std::size_t ldsTotal = lds + col_entries_lds(a, false, y_table<decltype(eng), has_store_pos<decltype(eng)>::value>());
    prepare_kernel(k, ldsTotal);
    hipLaunchKernelGGL(k, y_grid(a.colEnd - a.colBegin, ceil_div(a.L - a.zBegin, lines), batch_dim(a.batch)), dim3(threads), ldsTotal, stream, eng, a,
                       inter, out, tw);
    gpu_check_launch("y_forward", stream);
  });
}

template void launch_y_forward<double, cx<double>>(const YArgs&, const cx<double>*, cx<double>*,
                                                   const cx<double>*, hipStream_t);
template void launch_y_forward<double, cx<float>>(const YArgs&, const cx<double>*, cx<float>*,
                                                  const cx<double>*, hipStream_t);
template void launch_y_forward<float, cx<float>>(const YArgs&, const cx<float>*, cx<float>*,
                                                 const cx<float>*, hipStream_t);

}  // namespace dev
}  // namespace spfft
