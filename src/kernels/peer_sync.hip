// Stream-ordered all-rank barrier for the peer-write (UNBUFFERED / IPC) data
// plane (device_comm.cpp: PeerDeviceComm orders the rounds of one plane).
// Lane q of workgroup 0 publishes this rank's epoch into rank q's flag array
// (system-scope store; the flag arrays are uncached device memory mapped into
// every rank), then polls its own array until every rank has reached the
// epoch.
//
// Flag array of a rank (2P + 2 words): [0, P) the epoch rank q last reached,
// [P, 2P) nonzero once rank q gave up waiting (timeout), [2P] arrivals of this
// rank's barrier workgroups, [2P + 1] the epoch workgroup 0 has released the
// others at. The poll is bounded:
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

namespace spfft {
namespace dev {

// One barrier round. Every workgroup first writes back the L2 of the XCD it
// runs on (system-scope release) and counts its arrival; workgroup 0 waits
// for all arrivals, publishes the epoch to every peer and waits for theirs,
// then releases the others through the `go` word; every workgroup ends with a
// system-scope acquire (drops its XCD's stale L1/L2 lines of memory that peers
// wrote). With gridDim.x >= 16, workgroups dealt round-robin over the 8 XCDs
// cover each XCD twice: the stage kernels' stores into peer memory have left
// every XCD's L2 before a peer can see the epoch, independent of the scope of
// the CP's end-of-kernel release.
__global__ void __launch_bounds__(64)
    peer_barrier_kernel(unsigned long long* const* __restrict__ peerFlags,
                        unsigned long long* myFlags, int me, int P, unsigned long long epoch,
                        unsigned int* failure, long long timeoutTicks) {
  unsigned long long* arrive = myFlags + 2 * P;
  unsigned long long* go = myFlags + 2 * P + 1;
  const long long t0 = wall_clock64();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
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

void launch_peer_barrier(unsigned long long* const* peerFlags, unsigned long long* myFlags, int me,
                         int P, unsigned long long epoch, unsigned int* failure,
                         long long timeoutTicks, hipStream_t stream) {
  hipLaunchKernelGGL(peer_barrier_kernel, dim3(kPeerBarrierGroups), dim3(64), 0, stream, peerFlags,
                     myFlags, me, P, epoch, failure, timeoutTicks);
  gpu_check_launch("peer_barrier", stream);
}

}  // namespace dev
}  // namespace spfft
