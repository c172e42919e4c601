/* Test-only entry points of libspfft_amd_testing.so (not installed, not in the
 * release library). */
#ifndef SPFFT_AMD_TEST_HOOKS_H
#define SPFFT_AMD_TEST_HOOKS_H

#include "spfft/amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Collective. Node-local shared-memory collectives (the relay data plane's host
   synchronisation) over `comm`: `iters` rounds of a checked allgather plus a barrier
   through one shared segment, then the same through the communicator itself.
   *shmUs / *commUs: microseconds per round (shmUs < 0 if the ranks could not share a
   segment). SPFFT_MPI_ERROR if a round delivered wrong data. */
SPFFT_EXPORT SpfftError spfft_amd_test_comm_shm_check(SpfftAmdComm comm, int iters, double* shmUs,
                                                      double* commUs);
/* 1: this library reads the SPFFT_FAULT_* switches (core/fault.hpp). */
SPFFT_EXPORT int spfft_amd_test_fault_injection(void);
/* 1 if the relay plane would use the GPU at this PCI location as an idle relay. */
SPFFT_EXPORT int spfft_amd_test_relay_candidate_idle(int domain, int bus, int device);

#ifdef __cplusplus
}
#endif

#endif
