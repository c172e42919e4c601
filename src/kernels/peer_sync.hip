// Stream-ordered all-rank barrier for the peer-write (UNBUFFERED / IPC) data
// plane. One 64-lane workgroup per call, launched on the process's peer
// channel stream (device_comm.cpp: PeerChannel), so the barriers of a process
// run one after another in host call order. Lane q publishes this rank's
// epoch into rank q's flag array (system-scope release store; the flag arrays
// are uncached device memory mapped into every rank), then polls its own
// array until every rank has reached the epoch.
//
// Flag array of a rank (2P words): [0, P) the epoch rank q last reached,
// [P, 2P) nonzero once rank q gave up waiting (timeout). The poll is bounded:
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

__global__ void __launch_bounds__(64)
    peer_barrier_kernel(unsigned long long* const* __restrict__ peerFlags,
                        unsigned long long* myFlags, int me, int P, unsigned long long epoch,
                        unsigned int* failure, long long timeoutTicks) {
  // everything this rank's stream wrote before (local or remote) is visible
  // system-wide before the epoch is published (the hand-off event in front of
  // this kernel is a system-scope release of every XCD's L2, PeerChannel)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int q = threadIdx.x; q < P; q += blockDim.x)
    __hip_atomic_store(peerFlags[q] + me, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const long long t0 = wall_clock64();
  for (int q = threadIdx.x; q < P; q += blockDim.x) {
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
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

void launch_peer_barrier(unsigned long long* const* peerFlags, unsigned long long* myFlags, int me,
                         int P, unsigned long long epoch, unsigned int* failure,
                         long long timeoutTicks, hipStream_t stream) {
  hipLaunchKernelGGL(peer_barrier_kernel, dim3(1), dim3(64), 0, stream, peerFlags, myFlags, me, P,
                     epoch, failure, timeoutTicks);
  gpu_check_launch("peer_barrier", stream);
}

}  // namespace dev
}  // namespace spfft
