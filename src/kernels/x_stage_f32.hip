// x-stage kernels, fp32 transforms.
#include "kernels/stage_launch.hpp"

namespace spfft {
namespace dev {

template void launch_x_backward<float>(const XArgs&, bool, const cx<float>*, void*, const cx<float>*,
                                     const cx<float>*, hipStream_t);
template void launch_x_forward<float>(const XArgs&, bool, const void*, cx<float>*, const cx<float>*,
                                    const cx<float>*, hipStream_t);

}  // namespace dev
}  // namespace spfft
