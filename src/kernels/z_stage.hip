// z-stage kernels, fp64 transforms with fp64 exchange buffers.
#include "kernels/stage_launch.hpp"

namespace spfft {
namespace dev {

template void launch_z_backward<double, cx<double>>(const ZArgs&, const cx<double>*, cx<double>*, const cx<double>*,
                                             hipStream_t);
template void launch_z_forward<double, cx<double>>(const ZArgs&, const cx<double>*, cx<double>*, double, const cx<double>*,
                                            hipStream_t);

}  // namespace dev
}  // namespace spfft
