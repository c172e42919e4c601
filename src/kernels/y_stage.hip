// y-stage kernels, fp64 transforms with fp64 exchange buffers.
#include "kernels/stage_launch.hpp"

namespace spfft {
namespace dev {

template void launch_y_backward<double, cx<double>>(const YArgs&, const cx<double>*, cx<double>*, const cx<double>*,
                                             hipStream_t);
template void launch_y_forward<double, cx<double>>(const YArgs&, const cx<double>*, cx<double>*, const cx<double>*,
                                            hipStream_t);

}  // namespace dev
}  // namespace spfft
