#include "gpu/ipc_arena.hpp"

#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <list>
#include <mutex>
#include <random>

#include "gpu/gpu_runtime.hpp"
#include "spfft/exceptions.hpp"

namespace spfft {

struct IpcLease::Block {
  void* base = nullptr;
  std::size_t bytes = 0;  // whole allocation, header included
  int device = 0;
  bool uncached = false;
  std::uint64_t serial = 0;
  IpcHeader header{};
  hipIpcMemHandle_t handle{};
  bool handleValid = false;
};

namespace {

std::mutex gArenaMutex;
// Free blocks in release order (oldest first). Blocks in use are owned by
// their lease. Never destroyed: blocks still listed at process exit are left
// to the driver (destructors of statics may run after the HIP runtime is gone).
std::list<IpcLease::Block*>& free_list() {
  static auto* l = new std::list<IpcLease::Block*>();
  return *l;
}
IpcArenaStats gStats{0, 0, 0, 0};
std::uint64_t gSerial = 0;

std::size_t pool_cap() {
  static const std::size_t cap = [] {
    const char* e = std::getenv("SPFFT_IPC_POOL_BYTES");
    return e && *e ? static_cast<std::size_t>(std::atof(e)) : (std::size_t(2) << 30);
  }();
  return cap;
}

std::uint64_t fresh_nonce(std::uint64_t serial) {
  static std::mt19937_64 rng([] {
    std::random_device rd;
    const auto t = static_cast<std::uint64_t>(std::chrono::steady_clock::now().time_since_epoch().count());
    return (static_cast<std::uint64_t>(rd()) << 32) ^ rd() ^ t ^ static_cast<std::uint64_t>(getpid());
  }());
  std::uint64_t n = 0;
  while (n == 0) n = rng() ^ (serial * 0x9E3779B97F4A7C15ull);
  return n;
}

std::size_t round_block(std::size_t payload) {
  const std::size_t need = payload + kIpcHeaderBytes;
  return ((need + kIpcBlockGranule - 1) / kIpcBlockGranule) * kIpcBlockGranule;
}

// (runs in destructors: never throws, whatever state the device is in)
void free_block(IpcLease::Block* b) {
  if (!process_exiting()) {
    int prev = -1;
    if (hipGetDevice(&prev) == hipSuccess && prev != b->device) (void)hipSetDevice(b->device);
    (void)hipFree(b->base);
    if (prev >= 0 && prev != b->device) (void)hipSetDevice(prev);
    (void)hipGetLastError();
  }
  ++gStats.freed;
  delete b;
}

// Caller holds gArenaMutex. Frees the oldest free blocks beyond the cap.
void trim_locked() {
  auto& fl = free_list();
  while (gStats.freeBytes > pool_cap() && !fl.empty()) {
    IpcLease::Block* b = fl.front();
    fl.pop_front();
    gStats.freeBytes -= b->bytes;
    free_block(b);
  }
}

}  // namespace

std::unique_ptr<IpcLease> ipc_acquire(int device, std::size_t payloadBytes, bool uncached) {
  const std::size_t bytes = round_block(payloadBytes);
  IpcLease::Block* b = nullptr;
  {
    std::lock_guard<std::mutex> lock(gArenaMutex);
    // best fit among the free blocks of this device and kind, at most twice
    // the size asked for (plus one granule)
    auto& fl = free_list();
    auto best = fl.end();
    for (auto it = fl.begin(); it != fl.end(); ++it) {
      IpcLease::Block* c = *it;
      if (c->device != device || c->uncached != uncached || c->bytes < bytes ||
          c->bytes > 2 * bytes + kIpcBlockGranule)
        continue;
      if (best == fl.end() || c->bytes < (*best)->bytes) best = it;
    }
    if (best != fl.end()) {
      b = *best;
      fl.erase(best);
      gStats.freeBytes -= b->bytes;
      ++gStats.reused;
    }
  }
  DeviceGuard guard(device);
  if (!b) {
    std::unique_ptr<IpcLease::Block> nb(new IpcLease::Block());
    nb->bytes = bytes;
    nb->device = device;
    nb->uncached = uncached;
    hipError_t err = uncached ? hipExtMallocWithFlags(&nb->base, bytes, hipDeviceMallocUncached)
                              : hipMalloc(&nb->base, bytes);
    if (err != hipSuccess && uncached) {
      (void)hipGetLastError();
      err = hipMalloc(&nb->base, bytes);
    }
    if (err != hipSuccess) {
      (void)hipGetLastError();
      throw GPUAllocationError();
    }
    gpu_check(hipIpcGetMemHandle(&nb->handle, nb->base), "hipIpcGetMemHandle");
    nb->handleValid = true;
    {
      std::lock_guard<std::mutex> lock(gArenaMutex);
      nb->serial = ++gSerial;
      ++gStats.allocated;
    }
    b = nb.release();
  }
  b->header.magic = kIpcMagic;
  b->header.pid = static_cast<std::uint64_t>(getpid());
  b->header.serial = b->serial;
  b->header.nonce = fresh_nonce(b->serial);
  // synchronous: the header is in memory before the handle is announced
  gpu_check(hipMemcpy(b->base, &b->header, sizeof(IpcHeader), hipMemcpyHostToDevice), "hipMemcpy");
  return std::unique_ptr<IpcLease>(new IpcLease(b, payloadBytes));
}

IpcLease::~IpcLease() {
  if (!block_) return;
  std::lock_guard<std::mutex> lock(gArenaMutex);
  if (discard_) {
    free_block(block_);
    return;
  }
  free_list().push_back(block_);
  gStats.freeBytes += block_->bytes;
  trim_locked();
}

void* IpcLease::data() const { return static_cast<char*>(block_->base) + kIpcHeaderBytes; }

IpcExport IpcLease::describe() const {
  IpcExport e{};
  e.handle = block_->handle;
  e.header = block_->header;
  e.payloadBytes = payload_;
  e.valid = 1;
  return e;
}

IpcArenaStats ipc_arena_stats() {
  std::lock_guard<std::mutex> lock(gArenaMutex);
  return gStats;
}

void* ipc_open_checked(const IpcExport& e, std::string* why) {
  void* base = nullptr;
  gpu_check(hipIpcOpenMemHandle(&base, e.handle, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  IpcHeader seen{};
  gpu_check(hipMemcpy(&seen, base, sizeof(IpcHeader), hipMemcpyDeviceToHost), "hipMemcpy");
  if (seen.magic != e.header.magic || seen.pid != e.header.pid || seen.serial != e.header.serial ||
      seen.nonce != e.header.nonce) {
    if (why) {
      char b[256];
      std::snprintf(b, sizeof(b),
                    "stale IPC mapping: block %llu of pid %llu announced nonce %016llx, the mapping "
                    "shows pid %llu block %llu nonce %016llx",
                    static_cast<unsigned long long>(e.header.serial),
                    static_cast<unsigned long long>(e.header.pid),
                    static_cast<unsigned long long>(e.header.nonce), static_cast<unsigned long long>(seen.pid),
                    static_cast<unsigned long long>(seen.serial), static_cast<unsigned long long>(seen.nonce));
      *why = b;
    }
    (void)hipIpcCloseMemHandle(base);
    return nullptr;
  }
  return static_cast<char*>(base) + kIpcHeaderBytes;
}

void ipc_close(void* payload) {
  if (!payload || process_exiting()) return;
  (void)hipIpcCloseMemHandle(static_cast<char*>(payload) - kIpcHeaderBytes);
}

}  // namespace spfft
