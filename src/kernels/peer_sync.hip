// Stream-ordered all-rank barrier for the peer-write (UNBUFFERED / IPC) data
// plane (device_comm.cpp: PeerDeviceComm orders the rounds of one plane).
// Lane q of workgroup 0 publishes this rank's epoch into rank q's flag array
// (system-scope store; the flag arrays are uncached device memory mapped into
// every rank), then polls its own array until every rank has reached the
// epoch.
//
// Flag array of a rank (2P + 3 words): [0, P) the epoch rank q last reached,
// [P, 2P) nonzero once rank q gave up waiting (timeout), [2P] arrivals of this
// rank's barrier workgroups, [2P + 1] the epoch workgroup 0 has released the
// others at, [2P + 2] the XCDs the round's workgroups ran on. The poll is bounded:
// after `timeoutTicks` wall-clock ticks the kernel records the failure in a
// host-mapped word, marks it in every peer's array (so the peers' barriers
// stop waiting at once instead of each running into its own timeout) and
// exits: a missing peer never leaves a wave spinning on the GPU. A nonzero
// host word (an abort written by the host) or a peer's mark also ends the
// wait, with the cause in the host word (bit 0 own timeout, bit 1 host abort,
// bit 2 a peer gave up).
#include <hip/hip_runtime.h>

#include "kernels/peer_sync.hpp"
#include "gpu/gpu_runtime.hpp"
#include "spfft/exceptions.hpp"

#include <map>
#include <mutex>

namespace spfft {
namespace dev {

// XCD (accelerator complex die) this wave runs on.
__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x & 15u;
}

// One barrier round. Every workgroup first writes back the L2 of the XCD it
// runs on (system-scope release), records that XCD and counts its arrival;
// workgroup 0 waits for all arrivals, checks that the round's workgroups
// covered every XCD of the device (xcdMask, from the setup census), publishes
// the epoch to every peer and waits for theirs, then releases the others
// through the `go` word; every workgroup ends with a system-scope acquire
// (drops its XCD's stale L1/L2 lines of memory that peers wrote). The stage
// kernels' stores into peer memory carry no fence of their own: this round's
// per-XCD write-back publishes them (a fence per storing wave was measured at
// ~10x the stage time, profiles/r6/shared_gpu). The dispatcher deals the 16
// workgroups round-robin over the 8 XCDs, but nothing is assumed: a round
// that missed an XCD fails (kPeerXcdMiss) instead of publishing.
__global__ void __launch_bounds__(64)
    peer_barrier_kernel(unsigned long long* const* __restrict__ peerFlags,
                        unsigned long long* myFlags, int me, int P, unsigned long long epoch,
                        unsigned int* failure, long long timeoutTicks, unsigned xcdMask) {
  unsigned long long* arrive = myFlags + 2 * P;
  unsigned long long* go = myFlags + 2 * P + 1;
  unsigned long long* seen = myFlags + 2 * P + 2;
  const long long t0 = wall_clock64();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_or(seen, 1ull << xcc_id(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(arrive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (blockIdx.x == 0) {
    // every workgroup's write-back is done
    if (threadIdx.x == 0) {
      const unsigned long long target = epoch * gridDim.x;
      while (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
        if (__hip_atomic_load(failure, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;
        if (wall_clock64() - t0 > timeoutTicks) {
          __hip_atomic_fetch_or(failure, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      // (the next round's workgroups start after this kernel has ended)
      const unsigned long long got = __hip_atomic_exchange(seen, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((got & xcdMask) != xcdMask) {
        __hip_atomic_fetch_or(failure, kPeerXcdMiss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int r = 0; r < P; ++r)
          __hip_atomic_store(peerFlags[r] + P + me, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __syncthreads();
    const bool failed = __hip_atomic_load(failure, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    if (!failed)
      for (int q = threadIdx.x; q < P; q += blockDim.x)
        __hip_atomic_store(peerFlags[q] + me, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (int q = threadIdx.x; q < P && !failed; q += blockDim.x) {
      while (__hip_atomic_load(myFlags + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
        // a failure recorded by another lane or an abort from the host ...
        if (__hip_atomic_load(failure, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;
        // ... or a peer that gave up ends the wait
        if (__hip_atomic_load(myFlags + P + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
          __hip_atomic_fetch_or(failure, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        if (wall_clock64() - t0 > timeoutTicks) {
          __hip_atomic_fetch_or(failure, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          for (int r = 0; r < P; ++r)
            __hip_atomic_store(peerFlags[r] + P + me, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(go, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else if (threadIdx.x == 0) {
    while (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (__hip_atomic_load(failure, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;
      __builtin_amdgcn_s_sleep(4);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ void __launch_bounds__(64) xcd_census_kernel(unsigned* mask) {
  if (threadIdx.x == 0) atomicOr(mask, 1u << xcc_id());
}

unsigned xcd_mask(int device) {
  static std::mutex m;
  static std::map<int, unsigned> cache;
  std::lock_guard<std::mutex> lock(m);
  auto it = cache.find(device);
  if (it != cache.end()) return it->second;
  DeviceGuard guard(device);
  DeviceBuffer word(sizeof(unsigned));
  gpu_check(hipMemset(word.data(), 0, sizeof(unsigned)), "hipMemset");
  hipLaunchKernelGGL(xcd_census_kernel, dim3(4096), dim3(64), 0, nullptr, word.data<unsigned>());
  gpu_check_launch("xcd_census", nullptr);
  unsigned v = 0;
  gpu_check(hipMemcpy(&v, word.data(), sizeof(unsigned), hipMemcpyDeviceToHost), "hipMemcpy");
  if (v == 0) throw InternalError();
  cache[device] = v;
  return v;
}

// ------------------------------------------------------ route self-test
// (PeerDeviceComm::self_test) Pattern word i of the message src -> dst.
__device__ __forceinline__ unsigned long long selftest_word(unsigned long long nonce, int src, int dst,
                                                            long long i) {
  return nonce ^ (static_cast<unsigned long long>(src) << 56) ^ (static_cast<unsigned long long>(dst) << 48) ^
         (static_cast<unsigned long long>(i) * 0x9E3779B97F4A7C15ull);
}

// Every workgroup reads the whole region with plain loads, so each XCD's L2
// holds its lines (the stale-line case the barrier round must clear).
__global__ void __launch_bounds__(256) selftest_warm_kernel(const ulonglong2* p, long long n,
                                                            unsigned long long* sink) {
  unsigned long long acc = 0;
  for (long long i = threadIdx.x; i < n; i += blockDim.x) {
    const ulonglong2 v = p[i];
    acc ^= v.x ^ v.y;
  }
  if (acc == 0x5eed5eed5eed5eedull) *sink = acc;  // (keeps the loads)
}

// The stage kernels' store flavour: 16-byte non-temporal stores, no fence.
__global__ void __launch_bounds__(256) selftest_store_kernel(ulonglong2* dst, long long n,
                                                             unsigned long long nonce, int src,
                                                             int to, int corrupt) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += 256ll * gridDim.x) {
    unsigned long long a = selftest_word(nonce, src, to, 2 * i), b = selftest_word(nonce, src, to, 2 * i + 1);
    if (corrupt && i == n - 1) b ^= 1;
    __builtin_nontemporal_store(a, &dst[i].x);
    __builtin_nontemporal_store(b, &dst[i].y);
  }
}

__global__ void __launch_bounds__(256) selftest_check_kernel(const ulonglong2* src, long long n,
                                                             unsigned long long nonce, int from,
                                                             int me, unsigned long long* bad) {
  unsigned long long wrong = 0;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += 256ll * gridDim.x) {
    const unsigned long long a = __builtin_nontemporal_load(&src[i].x), b = __builtin_nontemporal_load(&src[i].y);
    wrong += (a != selftest_word(nonce, from, me, 2 * i)) + (b != selftest_word(nonce, from, me, 2 * i + 1));
  }
  if (wrong) atomicAdd(bad, wrong);
}

void launch_selftest_warm(const void* region, std::size_t bytes, unsigned long long* sink, hipStream_t s) {
  hipLaunchKernelGGL(selftest_warm_kernel, dim3(64), dim3(256), 0, s, static_cast<const ulonglong2*>(region),
                     static_cast<long long>(bytes / 16), sink);
  gpu_check_launch("selftest_warm", s);
}
void launch_selftest_store(void* dst, std::size_t bytes, unsigned long long nonce, int src, int to, int corrupt,
                           hipStream_t s) {
  hipLaunchKernelGGL(selftest_store_kernel, dim3(32), dim3(256), 0, s, static_cast<ulonglong2*>(dst),
                     static_cast<long long>(bytes / 16), nonce, src, to, corrupt);
  gpu_check_launch("selftest_store", s);
}
void launch_selftest_check(const void* src, std::size_t bytes, unsigned long long nonce, int from, int me,
                           unsigned long long* bad, hipStream_t s) {
  hipLaunchKernelGGL(selftest_check_kernel, dim3(32), dim3(256), 0, s, static_cast<const ulonglong2*>(src),
                     static_cast<long long>(bytes / 16), nonce, from, me, bad);
  gpu_check_launch("selftest_check", s);
}

void launch_peer_barrier(unsigned long long* const* peerFlags, unsigned long long* myFlags, int me,
                         int P, unsigned long long epoch, unsigned int* failure,
                         long long timeoutTicks, unsigned xcdMask, hipStream_t stream) {
  hipLaunchKernelGGL(peer_barrier_kernel, dim3(kPeerBarrierGroups), dim3(64), 0, stream, peerFlags,
                     myFlags, me, P, epoch, failure, timeoutTicks, xcdMask);
  gpu_check_launch("peer_barrier", stream);
}

}  // namespace dev
}  // namespace spfft
