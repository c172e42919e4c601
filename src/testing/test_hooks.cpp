// Test-only entry points of libspfft_amd_testing.so (never in the release
// library libspfft_amd.so): probes the test suite and the benchmark tools use
// to check internals, declared in src/testing/test_hooks.h.
#include "testing/test_hooks.h"

#include <chrono>
#include <cstdlib>
#include <vector>

#include "api/c_guard.hpp"
#include "comm/shm_group.hpp"
#include "core/fault.hpp"
#include "gpu/device_comm.hpp"

using namespace spfft;

extern "C" {

SpfftError spfft_amd_test_comm_shm_check(SpfftAmdComm comm, int iters, double* shmUs, double* commUs) {
  if (!comm) {
    c_last_error() = "invalid handle";
    return SPFFT_INVALID_HANDLE_ERROR;
  }
  if (!shmUs || !commUs || iters < 1) return SPFFT_INVALID_PARAMETER_ERROR;
  return guarded([&] {
    Communicator& cm = **static_cast<CommHandle*>(comm);
    const int P = cm.size(), me = cm.rank();
    std::vector<long long> mine(4), all(static_cast<std::size_t>(4) * P);
    auto round = [&](int it, auto&& gather, auto&& barrier) {
      for (int k = 0; k < 4; ++k) mine[k] = (static_cast<long long>(it) << 20) + me * 4 + k;
      gather(mine.data(), all.data(), mine.size() * sizeof(long long));
      for (int q = 0; q < P; ++q)
        for (int k = 0; k < 4; ++k)
          if (all[static_cast<std::size_t>(q) * 4 + k] != (static_cast<long long>(it) << 20) + q * 4 + k) {
            set_error_detail("shared-memory allgather delivered wrong data");
            throw MPIError();
          }
      barrier();
    };
    auto timed = [&](auto&& gather, auto&& barrier) {
      round(-1, gather, barrier);
      const auto t0 = std::chrono::steady_clock::now();
      for (int it = 0; it < iters; ++it) round(it, gather, barrier);
      return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
    };
    auto shm = ShmGroup::create(cm, mine.size() * sizeof(long long), 60.0);
    // fault injection SHM_EXIT: the last rank leaves without a word; the
    // others' shared-memory waits must end with MPIError, not spin
    if (shm && SPFFT_FAULT(SHM_EXIT) == 1 && me == P - 1 && P > 1) std::_Exit(0);
    *shmUs = shm ? timed([&](const void* s, void* r, std::size_t n) { shm->allgather(s, r, n); },
                         [&] { shm->barrier(); })
                 : -1.0;
    *commUs = timed([&](const void* s, void* r, std::size_t n) { cm.allgather(s, r, n); },
                    [&] { cm.barrier(); });
  });
}

int spfft_amd_test_fault_injection(void) { return 1; }

int spfft_amd_test_relay_candidate_idle(int domain, int bus, int device) {
  return relay_candidate_idle(domain, bus, device) ? 1 : 0;
}

}  // extern "C"
