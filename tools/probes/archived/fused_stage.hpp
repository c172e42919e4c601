// Fused single-GPU path (see fused_stage.hip): plane-major sticks and the
// persistent, XCD-cooperative y/x kernels with an L2-resident plane ring.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>

#include "fft/codelets.hpp"
#include "plan/index_plan.hpp"

namespace spfft {
namespace dev {

constexpr int kMaxRing = 8;

struct FusedArgs {
  int S;            // local sticks
  long long Sp;     // plane stride of the plane-major stick array [Z][Sp]
  int X, Y, Z;      // transform dims (space rows are X long)
  int ncols;        // x-columns holding sticks
  const int* colOffsets;  // ncols + 1
  const int* colY;        // per stick entry
  const int* colX;        // per column
  const int* entryCol;    // per stick entry: its column
  const StickDesc* desc;  // per stick
  long long scratchPlane;   // elements of one ring buffer (Y * scratchStride)
  long long scratchStride;  // row stride of a ring buffer [y][column]
  int ring;                 // ring buffers per XCD (<= kMaxRing)
  int lag;                  // steps between a plane's two phases (< ring)
  unsigned* ctrl;           // zeroed before each persistent launch
  unsigned* failure;        // host-mapped error word
  long long timeout;        // spin bound, wall-clock ticks
  int debug;                // timing probes only (SPFFT_FUSED_DEBUG): 1 = skip waits
};

constexpr int kFusedCtrlWords = 16 + 8 * 2 * kMaxRing;

bool fused_supported(int x, int y, int z);
template <typename T>
int fused_blocks_per_cu(int x, int y);
template <typename T>
void launch_z_backward_pm(const FusedArgs& a, const cx<T>* values, cx<T>* sticks, const cx<T>* tw,
                          hipStream_t stream);
template <typename T>
void launch_z_forward_pm(const FusedArgs& a, const cx<T>* sticks, cx<T>* values, T scale,
                         const cx<T>* tw, hipStream_t stream);
template <typename T>
void launch_yx_backward(const FusedArgs& a, int grid, const cx<T>* sticks, cx<T>* space,
                        cx<T>* scratch, const cx<T>* twy, const cx<T>* twx, hipStream_t stream);
template <typename T>
void launch_xy_forward(const FusedArgs& a, int grid, const cx<T>* space, cx<T>* sticks,
                       cx<T>* scratch, const cx<T>* twy, const cx<T>* twx, hipStream_t stream);

}  // namespace dev
}  // namespace spfft
