// Page-aligned host allocation, optionally page-locked for fast DMA
// (reference: src/memory/host_array.hpp:102,211-233, aligned_allocation.cpp:40-52).
#pragma once

#include <cstddef>
#include <cstdlib>
#include <utility>

#include "spfft/exceptions.hpp"

namespace spfft {

// Implemented in gpu/gpu_runtime.cpp (hipHostRegister / hipHostUnregister).
bool gpu_host_register(void* ptr, std::size_t bytes);
void gpu_host_unregister(void* ptr);

class HostBuffer {
public:
  HostBuffer() = default;
  HostBuffer(std::size_t bytes, bool pinned) { allocate(bytes, pinned); }
  ~HostBuffer() { release(); }
  HostBuffer(const HostBuffer&) = delete;
  HostBuffer& operator=(const HostBuffer&) = delete;
  HostBuffer(HostBuffer&& o) noexcept { swap(o); }
  HostBuffer& operator=(HostBuffer&& o) noexcept {
    swap(o);
    return *this;
  }

  void allocate(std::size_t bytes, bool pinned) {
    release();
    if (bytes == 0) return;
    constexpr std::size_t page = 4096;
    const std::size_t rounded = (bytes + page - 1) / page * page;
    void* p = nullptr;
    if (posix_memalign(&p, page, rounded) != 0 || !p) throw HostAllocationError();
    ptr_ = p;
    bytes_ = rounded;
    pinned_ = pinned && gpu_host_register(ptr_, bytes_);
  }
  void release() {
    if (ptr_) {
      if (pinned_) gpu_host_unregister(ptr_);
      std::free(ptr_);
    }
    ptr_ = nullptr;
    bytes_ = 0;
    pinned_ = false;
  }
  void swap(HostBuffer& o) noexcept {
    std::swap(ptr_, o.ptr_);
    std::swap(bytes_, o.bytes_);
    std::swap(pinned_, o.pinned_);
  }

  template <typename U = void>
  U* data() const {
    return static_cast<U*>(ptr_);
  }
  std::size_t bytes() const { return bytes_; }
  bool pinned() const { return pinned_; }

private:
  void* ptr_ = nullptr;
  std::size_t bytes_ = 0;
  bool pinned_ = false;
};

// Returns true if [a, a+na) and [b, b+nb) do not overlap
// (reference: src/memory/array_view_utility.hpp:45-52).
inline bool disjoint(const void* a, std::size_t na, const void* b, std::size_t nb) {
  const char* pa = static_cast<const char*>(a);
  const char* pb = static_cast<const char*>(b);
  return pa + na <= pb || pb + nb <= pa;
}

}  // namespace spfft
