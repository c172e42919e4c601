// Node-local host collectives over one POSIX shared-memory segment: barrier and
// allgather for the ranks of a communicator that all run on one host.
//
// The host-synchronous relay data plane (device_comm.cpp: RelayDeviceComm)
// needs one allgather and two barriers per exchange. Through the
// torch.distributed control plane (a gloo group driven from Python callbacks)
// these cost 220-280 us per exchange with 2 ranks on one MI355X box
// (profiles/r5/relay/overhead.txt); through shared memory they are a few
// microseconds. The segment is unlinked as soon as every rank has mapped it,
// so nothing is left in /dev/shm whatever happens to the processes later.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <memory>

#include "spfft/communicator.hpp"

namespace spfft {

class ShmGroup {
public:
  // Collective over `comm`. nullptr on every rank if any rank could not map the
  // segment (e.g. ranks in different containers of one host), if the ranks do
  // not share one pid namespace or cannot see each other's pids (the exit
  // detection below needs them), or if SPFFT_SHM_COLLECTIVES=0. Waits give up after `timeoutSeconds` (0: never)
  // and as soon as a waited-for process has exited, with MPIError.
  static std::unique_ptr<ShmGroup> create(Communicator& comm, std::size_t maxPayload, double timeoutSeconds);
  ~ShmGroup();
  ShmGroup(const ShmGroup&) = delete;
  ShmGroup& operator=(const ShmGroup&) = delete;

  int rank() const { return me_; }
  int size() const { return P_; }
  void barrier();
  // `bytes` <= maxPayload; recv holds size() * bytes
  void allgather(const void* send, void* recv, std::size_t bytes);

private:
  struct alignas(64) Slot {
    std::atomic<std::uint64_t> epoch;
    std::atomic<long long> pid;
  };
  ShmGroup() = default;
  Slot* slot(int q) const;
  char* payload(int parity, int q) const;

  void* base_ = nullptr;
  std::size_t bytes_ = 0, stride_ = 0;
  int me_ = 0, P_ = 0;
  std::uint64_t epoch_ = 0, gathers_ = 0;
  double timeout_ = 0;
};

}  // namespace spfft
