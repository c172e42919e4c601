// Device-side synchronisation for the peer-write exchange (see peer_sync.hip).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>

namespace spfft {
namespace dev {

// Workgroups of one barrier round (>= 2 per XCD when dealt round-robin).
constexpr int kPeerBarrierGroups = 16;
// Words of a rank's flag array: 2P + 3 (see peer_sync.hip).
inline int peer_flag_words(int P) { return 2 * P + 3; }
// Failure-word bit set by a barrier round whose workgroups did not run on
// every XCD of the device (their write-back / invalidate would have missed an
// L2; see peer_sync.hip).
constexpr unsigned kPeerXcdMiss = 8;

// Bit mask of the XCDs (HW_REG_XCC_ID) this device dispatches workgroups to,
// from a census launch of many workgroups; cached per device ordinal.
// Synchronous; call once at data-plane setup.
unsigned xcd_mask(int device);

// Enqueues one barrier round `epoch` (strictly increasing per communicator and
// identical on every rank). peerFlags[q] = rank q's flag array (P entries)
// mapped into this process; myFlags = this rank's own array.
void launch_peer_barrier(unsigned long long* const* peerFlags, unsigned long long* myFlags, int me,
                         int P, unsigned long long epoch, unsigned int* failure,
                         long long timeoutTicks, unsigned xcdMask, hipStream_t stream);

// Route self-test of the peer-write plane (PeerDeviceComm::self_test):
// warm every XCD's L2 with a region (plain loads), store the pattern of the
// message src -> to (16-byte non-temporal stores, the stage kernels' flavour;
// corrupt != 0 flips one bit: fault injection), count the words of a received
// message from -> me that differ from the pattern into *bad.
void launch_selftest_warm(const void* region, std::size_t bytes, unsigned long long* sink, hipStream_t s);
void launch_selftest_store(void* dst, std::size_t bytes, unsigned long long nonce, int src, int to, int corrupt,
                           hipStream_t s);
void launch_selftest_check(const void* src, std::size_t bytes, unsigned long long nonce, int from, int me,
                           unsigned long long* bad, hipStream_t s);

}  // namespace dev
}  // namespace spfft
