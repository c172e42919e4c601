// z-stage launchers: fused decompress / hermitian fill / z-FFT / pack and the
// reverse (unpack / z-FFT / compress with scaling).
#include "kernels/stage_kernels.hpp"

namespace spfft {
namespace dev {

template <typename T, typename BT>
void launch_z_backward(const ZArgs& a, const cx<T>* values, BT* out, const cx<T>* tw,
                       hipStream_t stream) {
  if (a.numSticks <= a.stickBegin) return;
  with_engine<T, +1>(a.n, [&](auto eng, int threads, int lines, std::size_t lds) {
    using E = decltype(eng);
    auto k = a.desc ? z_backward_desc_kernel<E, T, BT> : z_backward_kernel<E, T, BT>;
    std::size_t ldsTotal = 0;
    const ZArgs b = z_args_for_lds(a, lds, lines, &ldsTotal);
    prepare_kernel(k, ldsTotal);
    hipLaunchKernelGGL(k, dim3(ceil_div(a.numSticks - a.stickBegin, lines), 1, batch_dim(a.batch)), dim3(threads), ldsTotal, stream, eng, b,
                       values, out, tw);
    gpu_check_launch("z_backward", stream);
  });
}

template void launch_z_backward<double, cx<double>>(const ZArgs&, const cx<double>*, cx<double>*,
                                                    const cx<double>*, hipStream_t);
template void launch_z_backward<double, cx<float>>(const ZArgs&, const cx<double>*, cx<float>*,
                                                   const cx<double>*, hipStream_t);
template void launch_z_backward<float, cx<float>>(const ZArgs&, const cx<float>*, cx<float>*,
                                                  const cx<float>*, hipStream_t);

}  // namespace dev
}  // namespace spfft
