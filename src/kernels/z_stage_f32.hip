// z-stage kernels, fp32 transforms.
#include "kernels/stage_launch.hpp"

namespace spfft {
namespace dev {

template void launch_z_backward<float, cx<float>>(const ZArgs&, const cx<float>*, cx<float>*, const cx<float>*,
                                             hipStream_t);
template void launch_z_forward<float, cx<float>>(const ZArgs&, const cx<float>*, cx<float>*, float, const cx<float>*,
                                            hipStream_t);

}  // namespace dev
}  // namespace spfft
