// Line FFTs that do not fit one workgroup's LDS (any length): a global-memory
// four-step engine, and Bluestein's chirp-z convolution on top of it for
// lengths whose large prime factor has no codelet. The fused stage kernels
// handle every length up to the LDS capacity; a longer axis runs as two passes
// whose loads and stores carry the stage's IO (LongIO in long_fft.hip: the
// columns pass gathers from the stage source, the rows pass stores into the
// stage destination). Replaces the GPUFFTError of rounds 1-2 (the reference's
// vendor plans take any n: src/fft/transform_1d_gpu.hpp:70,
// transform_2d_gpu.hpp:69).
//
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>

#include "fft/codelets.hpp"
#include "kernels/stage_args.hpp"

namespace spfft {
namespace dev {

struct LongPlan {
  int n = 0;
  bool bluestein = false;
  int m = 0;           // Bluestein convolution length (power of two), else n
  int n1 = 0, n2 = 0;  // four-step factors of m
  // device tables (one allocation per (device, n, precision), kept for the process)
  const void* tw1 = nullptr;    // exp(-2 pi i k / n1)
  const void* tw2 = nullptr;    // exp(-2 pi i k / n2)
  const void* twM = nullptr;    // exp(-2 pi i k / m)
  const void* chirp = nullptr;  // Bluestein d_j = exp(-i pi j^2 / n), [n]
  const void* filt = nullptr;   // FFT_m of conj(d) for S = -1 and S = +1, [2m]
  // elements per line of each work buffer
  long long line_elems() const { return m > n ? m : n; }
};

// Whether an axis of length n runs the four-step path instead of the one-workgroup
// stage kernels: lines that do not fit one workgroup's LDS next to the tables
// the axis's stage kernels keep there (y: the column entries, x: the column
// table and the C2R Nyquist line), and, on the line-fast y and x axes, run-time
// engine lengths whose workgroup would hold lines of less than one 64-byte column
// segment while n splits into two compile-time factors. Measured on MI355X,
// 4096 x 64 x 64 C2C fp64: x stage in one-line workgroups 690 / 495 us
// (forward / backward) against 383 / 308 us per 4096 elements on the four-step
// at 8192 (profiles/r4/long/).
enum LongAxis { kLongAxisZ = 0, kLongAxisY = 1, kLongAxisX = 2 };
bool needs_long_path(int n, bool dbl, LongAxis axis);
// plan (tables cached per device); throws GPUFFTError beyond 2^20 / 2
LongPlan long_plan(int n, bool dbl);

template <typename T>
struct LongBufs {
  cx<T>* in;   // natural-order input lines (stride n)
  cx<T>* w1;   // Bluestein work (stride m)
  cx<T>* w2;   // Bluestein work (stride m)
  cx<T>* out;  // natural-order output lines (stride n)
};

// Stage glue + long FFT, same semantics as the fused launchers (stage_args.hpp).
template <typename T, typename BT>
void launch_long_z_backward(const LongPlan& lp, const ZArgs& a, const cx<T>* values, BT* out,
                            const LongBufs<T>& w, hipStream_t stream);
template <typename T, typename BT>
void launch_long_z_forward(const LongPlan& lp, const ZArgs& a, const BT* in, cx<T>* values, T scale,
                           const LongBufs<T>& w, hipStream_t stream);
template <typename T, typename BT>
void launch_long_y_backward(const LongPlan& lp, const YArgs& a, const BT* in, cx<T>* inter,
                            const LongBufs<T>& w, hipStream_t stream);
template <typename T, typename BT>
void launch_long_y_forward(const LongPlan& lp, const YArgs& a, cx<T>* inter, BT* out,
                           const LongBufs<T>& w, hipStream_t stream);
// R2C with even n: lp is the plan of n / 2 (packed real rows), twFull the
// length-n twiddles; odd n: lp of n (hermitian-extended complex rows)
template <typename T>
void launch_long_x_backward(const LongPlan& lp, const XArgs& a, bool r2c, const cx<T>* inter,
                            void* space, const cx<T>* twFull, const LongBufs<T>& w, hipStream_t stream);
template <typename T>
void launch_long_x_forward(const LongPlan& lp, const XArgs& a, bool r2c, const void* space,
                           cx<T>* inter, const cx<T>* twFull, const LongBufs<T>& w, hipStream_t stream);

}  // namespace dev
}  // namespace spfft
