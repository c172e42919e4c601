// y-stage kernels, fp64 transforms with fp32 exchange buffers (*_FLOAT exchanges).
#include "kernels/stage_launch.hpp"

namespace spfft {
namespace dev {

template void launch_y_backward<double, cx<float>>(const YArgs&, const cx<float>*, cx<double>*, const cx<double>*,
                                             hipStream_t);
template void launch_y_forward<double, cx<float>>(const YArgs&, const cx<double>*, cx<float>*, const cx<double>*,
                                            hipStream_t);

}  // namespace dev
}  // namespace spfft
