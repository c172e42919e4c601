// Device-side synchronisation for the peer-write exchange (see peer_sync.hip).
#pragma once

#include <hip/hip_runtime_api.h>

namespace spfft {
namespace dev {

// Enqueues one barrier round `epoch` (strictly increasing per communicator and
// identical on every rank). peerFlags[q] = rank q's flag array (P entries)
// mapped into this process; myFlags = this rank's own array.
void launch_peer_barrier(unsigned long long* const* peerFlags, unsigned long long* myFlags, int me,
                         int P, unsigned long long epoch, unsigned int* failure,
                         long long timeoutTicks, hipStream_t stream);

}  // namespace dev
}  // namespace spfft
