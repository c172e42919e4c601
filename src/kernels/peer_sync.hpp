// Device-side synchronisation for the peer-write exchange (see peer_sync.hip).
#pragma once

#include <hip/hip_runtime_api.h>

namespace spfft {
namespace dev {

// Workgroups of one barrier round (>= 2 per XCD when dealt round-robin).
constexpr int kPeerBarrierGroups = 16;
// Words of a rank's flag array: 2P + 2 (see peer_sync.hip).
inline int peer_flag_words(int P) { return 2 * P + 2; }

// Enqueues one barrier round `epoch` (strictly increasing per communicator and
// identical on every rank). peerFlags[q] = rank q's flag array (P entries)
// mapped into this process; myFlags = this rank's own array.
void launch_peer_barrier(unsigned long long* const* peerFlags, unsigned long long* myFlags, int me,
                         int P, unsigned long long epoch, unsigned int* failure,
                         long long timeoutTicks, hipStream_t stream);

}  // namespace dev
}  // namespace spfft
