// Multi-segment copy of the relay data plane (see relay_copy.hip).
#pragma once

#include <hip/hip_runtime_api.h>

namespace spfft {
namespace dev {

// Bytes per chunk a workgroup copies at a time.
constexpr long long kCopyChunk = 64 * 1024;

// One contiguous copy; firstChunk = number of chunks of the segments before it
// (segments ordered, the chunk space is their concatenation).
struct CopySeg {
  const char* src;
  char* dst;
  unsigned long long bytes;
  long long firstChunk;
};

// Copies every segment (device-resident table of nseg entries, totalChunks
// chunks in all) in one launch on `stream`.
void launch_multi_copy(const CopySeg* devSegs, int nseg, long long totalChunks, hipStream_t stream);

// Segments passed by value in the kernel arguments (at most kInlineSegs): no
// host-to-device copy of the table ahead of the launch.
constexpr int kInlineSegs = 96;
struct SegPack {
  CopySeg s[kInlineSegs];
};
void launch_multi_copy_inline(const SegPack& segs, int nseg, long long totalChunks, hipStream_t stream);

}  // namespace dev
}  // namespace spfft
