// y-stage kernels, fp32 transforms.
#include "kernels/stage_launch.hpp"

namespace spfft {
namespace dev {

template void launch_y_backward<float, cx<float>>(const YArgs&, const cx<float>*, cx<float>*, const cx<float>*,
                                             hipStream_t);
template void launch_y_forward<float, cx<float>>(const YArgs&, const cx<float>*, cx<float>*, const cx<float>*,
                                            hipStream_t);

}  // namespace dev
}  // namespace spfft
