#include "gpu/gpu_runtime.hpp"

#include <atomic>
#include <cstdlib>
#include <string>

#include "core/common.hpp"
#include "core/host_buffer.hpp"

namespace spfft {

namespace {
std::atomic<bool> gExiting{false};
struct ExitHook {
  ExitHook() { std::atexit([] { gExiting.store(true); }); }
} gExitHook;
}  // namespace

bool process_exiting() { return gExiting.load(); }

void throw_gpu_error(hipError_t err, const char* what) {
  set_error_detail(std::string(what ? what : "") + ": " + hipGetErrorName(err) + " (" +
                   hipGetErrorString(err) + ")");
  switch (err) {
    case hipErrorMemoryAllocation: throw GPUAllocationError();
    case hipErrorLaunchFailure:
    case hipErrorLaunchOutOfResources:
    case hipErrorInvalidDeviceFunction:
    case hipErrorNoBinaryForGpu: throw GPULaunchError();
    case hipErrorNoDevice:
    case hipErrorInsufficientDriver: throw GPUNoDeviceError();
    case hipErrorInvalidValue: throw GPUInvalidValueError();
    case hipErrorInvalidDevicePointer: throw GPUInvalidDevicePointerError();
    default: throw GPUError();
  }
}

bool gpu_sync_debug() {
  static const bool on = [] {
    const char* e = std::getenv("SPFFT_GPU_SYNC_DEBUG");
    return e && e[0] == '1';
  }();
  return on;
}

bool gpu_sync_spin() {
  static const bool spin = [] {
    const char* e = std::getenv("SPFFT_SYNC");
    return !(e && std::string(e) == "block");
  }();
  return spin;
}

void gpu_check_launch(const char* kernel, hipStream_t stream) {
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) throw_gpu_error(err == hipErrorInvalidValue ? hipErrorLaunchFailure : err, kernel);
  if (gpu_sync_debug()) {
    gpu_check(hipStreamSynchronize(stream), kernel);
    gpu_check(hipGetLastError(), kernel);
  }
}

DeviceGuard::DeviceGuard(int device) {
  gpu_check(hipGetDevice(&previous_), "hipGetDevice");
  if (device >= 0 && device != previous_) {
    gpu_check(hipSetDevice(device), "hipSetDevice");
    switched_ = true;
  }
}

DeviceGuard::~DeviceGuard() {
  if (switched_) (void)hipSetDevice(previous_);
}

namespace {
std::atomic<int> gLiveStreams{0};
}
GpuStream::GpuStream(bool highPriority) {
  int lo = 0, hi = 0;
  if (highPriority && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess) {
    gpu_check(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "hipStreamCreate");
  } else {
    (void)hipGetLastError();
    gpu_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
  }
  ++gLiveStreams;
}
GpuStream::~GpuStream() {
  if (stream_) --gLiveStreams;
  if (stream_ && !process_exiting()) (void)hipStreamDestroy(stream_);
}
int GpuStream::live() { return gLiveStreams.load(); }

GpuEvent::GpuEvent(bool timing) {
  gpu_check(hipEventCreateWithFlags(&event_, timing ? hipEventDefault : hipEventDisableTiming),
            "hipEventCreate");
}
GpuEvent::~GpuEvent() {
  if (event_ && !process_exiting()) (void)hipEventDestroy(event_);
}

DeviceBuffer::DeviceBuffer(std::size_t bytes) : bytes_(bytes) {
  if (bytes) {
    hipError_t err = hipMalloc(&ptr_, bytes);
    if (err != hipSuccess) {
      (void)hipGetLastError();
      ptr_ = nullptr;
      throw GPUAllocationError();
    }
  }
}

DeviceBuffer::~DeviceBuffer() {
  if (ptr_ && !process_exiting()) (void)hipFree(ptr_);
}

bool is_device_pointer(const void* ptr) {
  if (!ptr) return false;
  hipPointerAttribute_t attr;
  hipError_t err = hipPointerGetAttributes(&attr, ptr);
  if (err != hipSuccess) {
    (void)hipGetLastError();  // unregistered host memory
    return false;
  }
  return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

int current_device() {
  int d = 0;
  gpu_check(hipGetDevice(&d), "hipGetDevice");
  return d;
}

bool gpu_host_register(void* ptr, std::size_t bytes) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    (void)hipGetLastError();
    return false;
  }
  if (hipHostRegister(ptr, bytes, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return true;
}

void gpu_host_unregister(void* ptr) {
  if (!process_exiting()) (void)hipHostUnregister(ptr);
}

}  // namespace spfft
