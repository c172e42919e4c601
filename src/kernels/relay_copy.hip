// Multi-segment copy for the relay data plane (device_comm.cpp: RelayDeviceComm).
// One launch moves every segment of an exchange phase: the sender's direct
// parts into the receivers' buffers and its relay parts into its buffers on
// otherwise idle GPUs (phase 1), or the receiver's pulls from those relay
// buffers (phase 2). The segments go to or come from different GPUs, so one
// launch keeps every xGMI link of the GPU busy at once; the chunks of all
// segments are dealt round-robin over the workgroups.
//
// Every workgroup starts with a system-scope acquire (drops its XCD's stale
// lines of memory other GPUs wrote) and ends with a system-scope release (its
// XCD's L2 written back before the host-side barrier that publishes the phase).
#include <hip/hip_runtime.h>

#include "gpu/gpu_runtime.hpp"
#include "kernels/relay_copy.hpp"
#include "spfft/exceptions.hpp"

namespace spfft {
namespace dev {

namespace {
constexpr int kCopyThreads = 256;

template <class Segs>
__device__ __forceinline__ int find_seg(const Segs& s, int n, long long chunk) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (s[mid].firstChunk <= chunk)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}
}  // namespace

template <class Segs>
__device__ __forceinline__ void multi_copy(const Segs& segs, int nseg, long long totalChunks) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (long long c = blockIdx.x; c < totalChunks; c += gridDim.x) {
    const CopySeg s = segs[find_seg(segs, nseg, c)];
    const long long off = (c - s.firstChunk) * kCopyChunk;
    const long long len = min(static_cast<long long>(kCopyChunk), static_cast<long long>(s.bytes) - off);
    const char* src = s.src + off;
    char* dst = s.dst + off;
    if (((reinterpret_cast<unsigned long long>(src) | reinterpret_cast<unsigned long long>(dst) |
          static_cast<unsigned long long>(len)) & 15) == 0) {
      const uint4* sv = reinterpret_cast<const uint4*>(src);
      uint4* dv = reinterpret_cast<uint4*>(dst);
      const long long nv = len >> 4;
      for (long long i = threadIdx.x; i < nv; i += kCopyThreads) dv[i] = sv[i];
    } else {
      // exchange blocks are whole complex elements: multiples of 8 bytes
      const uint2* sv = reinterpret_cast<const uint2*>(src);
      uint2* dv = reinterpret_cast<uint2*>(dst);
      const long long nv = len >> 3;
      for (long long i = threadIdx.x; i < nv; i += kCopyThreads) dv[i] = sv[i];
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ void __launch_bounds__(kCopyThreads)
    multi_copy_kernel(const CopySeg* __restrict__ segs, int nseg, long long totalChunks) {
  multi_copy(segs, nseg, totalChunks);
}

__global__ void __launch_bounds__(kCopyThreads)
    multi_copy_inline_kernel(const SegPack segs, int nseg, long long totalChunks) {
  multi_copy(segs.s, nseg, totalChunks);
}

void launch_multi_copy(const CopySeg* devSegs, int nseg, long long totalChunks, hipStream_t stream) {
  if (nseg <= 0 || totalChunks <= 0) return;
  const long long grid = totalChunks < 2048 ? totalChunks : 2048;
  hipLaunchKernelGGL(multi_copy_kernel, dim3(static_cast<unsigned>(grid)), dim3(kCopyThreads), 0, stream,
                     devSegs, nseg, totalChunks);
  gpu_check_launch("multi_copy", stream);
}

void launch_multi_copy_inline(const SegPack& segs, int nseg, long long totalChunks, hipStream_t stream) {
  if (nseg <= 0 || totalChunks <= 0) return;
  if (nseg > kInlineSegs) throw InternalError();
  const long long grid = totalChunks < 2048 ? totalChunks : 2048;
  hipLaunchKernelGGL(multi_copy_inline_kernel, dim3(static_cast<unsigned>(grid)), dim3(kCopyThreads), 0, stream,
                     segs, nseg, totalChunks);
  gpu_check_launch("multi_copy_inline", stream);
}

}  // namespace dev
}  // namespace spfft
