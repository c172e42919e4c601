// Kernel-argument structures and host launch entry points of the fused stage
// kernels. One kernel per stage and direction:
//   z stage: sparse values <-> z-sticks, z-FFT, (0,0)-stick hermitian fill,
//            pack into the per-rank exchange layout (replaces K4-K6, K8, K9,
//            K11, K13, K15 and the vendor z-FFT F1 of the reference).
//   y stage: exchange layout <-> [z][column][y] slab, y-FFT over x-columns that
//            hold sticks only, x=0 plane hermitian fill (replaces K2, K3, K7,
//            K10, K12, K14, K16 and half of F2/F3).
//   x stage: [z][column][y] <-> space domain [z][y][x], x-FFT C2C, C2R or R2C
//            (replaces the other half of F2/F3).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <string>

#include "fft/codelets.hpp"
#include "plan/index_plan.hpp"

namespace spfft {
namespace dev {

// Batched launches (multi_transform of transforms with identical plans on one
// GPU): blockIdx.z selects the transform; its input and output buffers come
// from these tables, every index table is shared. count <= 1: unbatched, the
// kernel's pointer arguments are used as given.
constexpr int kMaxBatch = 8;
struct BatchPtrs {
  int count;
  const void* in[kMaxBatch];
  void* out[kMaxBatch];
};

struct ZArgs {
  int numSticks;   // end of the stick range processed (exclusive)
  int stickBegin;  // first stick of the range (exchange pipelining chunks)
  int n;          // dimZ
  int zeroStick;  // line to hermitian-fill (R2C backward), -1 for none
  const StickRun* runs;
  const int* runOffsets;
  const StickDesc* desc;     // non-null when every stick is simple (fast path)
  int single;                // 1: exchange side is the plain [S][stickStride] array
                             // (2: distributed, segment table read from global memory)
  long long stickStride;     // element stride between sticks when single
  // otherwise, per plane z two entries: (base, stride) of its exchange segment,
  // element (stick s, plane z) at base + s * stride (base includes z)
  const long long* zTab;
  int plainSticks;  // backward: stick stores with the default cache policy (see GpuExecutor)
  // forward: streaming (nt) value stores, for value arrays larger than the
  // Infinity Cache can keep (GpuExecutor)
  int ntValueStores;
  BatchPtrs batch;
};


// A column's stick entries as at most kColRuns runs with consecutive y and
// consecutive bases: y in run r (y - y[r] < len[r]) has its entry at b0[r] +
// y * YArgs::colStride (b0 = the run's first base - y[r] * colStride). A sphere
// column is two runs (storage y = 0..h and n-h..n-1); entries from several
// ranks add runs. Workgroup-uniform, so it lives in scalar registers.
constexpr int kColRuns = 4;
struct ColDesc {
  long long b0[kColRuns];
  int y[kColRuns];
  int len[kColRuns];
  int nRuns;
};


struct YArgs {
  int ncols;     // columns of the [z][column][y] intermediate (its row count per plane)
  int colBegin;  // column range processed: [colBegin, colEnd) (exchange pipelining chunks)
  int colEnd;
  int L;       // end of the plane range processed (exclusive; = local planes)
  int zBegin;  // first plane of the range (plane chunking)
  int n;  // dimY
  int colOfX0;  // column needing the x=0 plane hermitian fill, -1 for none
  long long interStride;  // row stride of the [z][column][y] intermediate (>= n)
  // row (z, column c) of the intermediate starts at z * interZStride + c * interStride
  long long interZStride;
  const int* colOffsets;
  const int* colY;
  const long long* colBase;
  // optional per-column run descriptors (all columns qualify) and their stride
  const ColDesc* colDesc;
  long long colStride;
  int plainSticks;  // backward: stick loads with the default cache policy (see GpuExecutor)
  BatchPtrs batch;
};

struct XArgs {
  int L;       // end of the plane range (exclusive)
  int zBegin;  // first plane of the range
  int Y;
  int n;      // dimX
  int nFreq;  // dimX/2+1 for R2C, dimX for C2C
  int ncols;
  long long interStride;  // row stride of the [z][column][y] intermediate (>= Y)
  long long interZStride;  // as YArgs
  const int* colX;
  const int* xToCol;  // nFreq entries: x -> column or -1 (long-line x stage)
  BatchPtrs batch;
};

// Offset of column c's row inside one plane of the intermediate (a plane holds
// ncols * interStride < 2^31 elements: 32-bit arithmetic per lane).
template <class A>
__host__ __device__ inline int inter_row(const A& a, int c) {
  return c * static_cast<int>(a.interStride);
}

// grid z extent of a launch (1 when unbatched)
inline unsigned batch_dim(const BatchPtrs& b) { return b.count > 1 ? static_cast<unsigned>(b.count) : 1u; }

// Engine geometry for diagnostics (SPFFT_LOG).
std::string describe_engine(int n, bool dbl, bool lineFast);

// Host launchers. `tw` is the length-n twiddle table exp(-2 pi i m / n).
// BT is the exchange element type (cx<T> or cx<float> for *_FLOAT exchanges).
template <typename T, typename BT>
void launch_z_backward(const ZArgs& a, const cx<T>* values, BT* out, const cx<T>* tw,
                       hipStream_t stream);
template <typename T, typename BT>
void launch_z_forward(const ZArgs& a, const BT* in, cx<T>* values, T scale, const cx<T>* tw,
                      hipStream_t stream);
template <typename T, typename BT>
void launch_y_backward(const YArgs& a, const BT* in, cx<T>* inter, const cx<T>* tw,
                       hipStream_t stream);
template <typename T, typename BT>
void launch_y_forward(const YArgs& a, const cx<T>* inter, BT* out, const cx<T>* tw,
                      hipStream_t stream);
// twHalf: length-n/2 twiddles; when given (R2C, even n) the packed-real
// half-length kernels run instead of the hermitian-extended complex FFT.
template <typename T>
void launch_x_backward(const XArgs& a, bool r2c, const cx<T>* inter, void* space, const cx<T>* tw,
                       const cx<T>* twHalf, hipStream_t stream);
template <typename T>
void launch_x_forward(const XArgs& a, bool r2c, const void* space, cx<T>* inter, const cx<T>* tw,
                      const cx<T>* twHalf, hipStream_t stream);

// Largest run-time FFT length supported in one workgroup (LDS-resident).
int max_device_fft_length(bool doublePrecision);
// true if n has a compile-time (register-resident) kernel: the powers of two
// 16..1024 (FftCT) and the mixed-radix lengths of SPFFT_MR_SIZES (FftMR).
bool has_ct_kernel(int n);

// Non-power-of-two lengths with compile-time mixed-radix kernels (X-macro;
// user configuration: a build may list other lengths, or none, with
// -DSPFFT_MR_SIZES(X)=..., trading compile time for run-time engines).
#ifndef SPFFT_MR_SIZES
#define SPFFT_MR_SIZES(X)                                                                 \
  X(48) X(60) X(72) X(80) X(90) X(96) X(100) X(108) X(120) X(125) X(135) X(144) X(150) X(160) \
  X(180) X(192) X(200) X(216) \
  X(240) X(288) X(320) X(360) X(384) \
  X(400) X(480)
#endif

}  // namespace dev
}  // namespace spfft
