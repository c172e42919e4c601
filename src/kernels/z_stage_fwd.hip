// z-stage forward launcher: unpack / z-FFT / compress with scaling (its own
// translation unit so the z-stage kernels compile in parallel).
#include "kernels/stage_kernels.hpp"

namespace spfft {
namespace dev {

template <typename T, typename BT>
void launch_z_forward(const ZArgs& a, const BT* in, cx<T>* values, T scale, const cx<T>* tw,
                      hipStream_t stream) {
  if (a.numSticks <= a.stickBegin) return;
  with_engine<T, -1>(a.n, [&](auto eng, int threads, int lines, std::size_t lds) {
    using E = decltype(eng);
    auto k = a.desc ? z_forward_desc_kernel<E, T, BT> : z_forward_kernel<E, T, BT>;
    std::size_t ldsTotal = 0;
    const ZArgs b = z_args_for_lds(a, lds, lines, &ldsTotal);
    prepare_kernel(k, ldsTotal);
    hipLaunchKernelGGL(k, dim3(ceil_div(a.numSticks - a.stickBegin, lines), 1, batch_dim(a.batch)), dim3(threads), ldsTotal, stream, eng, b,
                       in, values, scale, tw);
    gpu_check_launch("z_forward", stream);
  });
}

template void launch_z_forward<double, cx<double>>(const ZArgs&, const cx<double>*, cx<double>*,
                                                   double, const cx<double>*, hipStream_t);
template void launch_z_forward<double, cx<float>>(const ZArgs&, const cx<float>*, cx<double>*,
                                                  double, const cx<double>*, hipStream_t);
template void launch_z_forward<float, cx<float>>(const ZArgs&, const cx<float>*, cx<float>*, float,
                                                 const cx<float>*, hipStream_t);

}  // namespace dev
}  // namespace spfft
