// Thin HIP runtime layer (one backend: HIP on gfx950; no CUDA macros).
// Error -> exception mapping as in the reference (src/gpu_util/gpu_runtime_api.hpp:112-124),
// RAII stream/event/device-guard, pointer classification
// (reference: src/gpu_util/gpu_pointer_translation.hpp:38-61).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>

#include "spfft/exceptions.hpp"

namespace spfft {

[[noreturn]] void throw_gpu_error(hipError_t err, const char* what);

inline void gpu_check(hipError_t err, const char* what = "") {
  if (err != hipSuccess) throw_gpu_error(err, what);
}

// Debug mode (SPFFT_GPU_SYNC_DEBUG=1): synchronise and check after every launch
// (reference: src/gpu_util/gpu_runtime.hpp:58-72 does this in Debug builds).
bool gpu_sync_debug();
// Synchronous calls poll the stream instead of blocking (SPFFT_SYNC=spin, default)
// or block in the runtime (SPFFT_SYNC=block).
bool gpu_sync_spin();
void gpu_check_launch(const char* kernel, hipStream_t stream);

class DeviceGuard {
public:
  explicit DeviceGuard(int device);
  ~DeviceGuard();
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;

private:
  int previous_ = -1;
  bool switched_ = false;
};

class GpuStream {
public:
  // non-blocking stream on the current device; highPriority: the device's
  // greatest stream priority (communication streams, so their kernels are
  // dispatched ahead of queued compute workgroups)
  explicit GpuStream(bool highPriority = false);
  ~GpuStream();
  GpuStream(const GpuStream&) = delete;
  GpuStream& operator=(const GpuStream&) = delete;
  hipStream_t get() const { return stream_; }
  // HIP streams the library currently owns (private transform streams, RCCL
  // channel streams): with GPU_MAX_HW_QUEUES = 4, every stream beyond the
  // queue count shares a hardware queue with another one and serialises
  // behind it.
  static int live();

private:
  hipStream_t stream_ = nullptr;
};

class GpuEvent {
public:
  explicit GpuEvent(bool timing = false);  // timing disabled unless asked for
  ~GpuEvent();
  GpuEvent(const GpuEvent&) = delete;
  GpuEvent& operator=(const GpuEvent&) = delete;
  hipEvent_t get() const { return event_; }
  void record(hipStream_t s) { gpu_check(hipEventRecord(event_, s), "hipEventRecord"); }
  void wait_on(hipStream_t s) { gpu_check(hipStreamWaitEvent(s, event_, 0), "hipStreamWaitEvent"); }

private:
  hipEvent_t event_ = nullptr;
};

class DeviceBuffer {
public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(std::size_t bytes);
  ~DeviceBuffer();
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  template <typename U = void>
  U* data() const {
    return static_cast<U*>(ptr_);
  }
  std::size_t bytes() const { return bytes_; }

private:
  void* ptr_ = nullptr;
  std::size_t bytes_ = 0;
};

// True once the process is exiting (atexit): destructors then leave GPU
// resources to the driver instead of calling into a runtime that may already be
// tearing down.
bool process_exiting();

// true if ptr is device (or managed) memory accessible by the GPU kernels.
bool is_device_pointer(const void* ptr);
int current_device();

}  // namespace spfft
