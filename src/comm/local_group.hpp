// In-process communicator group: N ranks driven by N threads of one process.
// Used for multi-rank tests without MPI and for P-virtual-rank runs on one GPU
// ("in-process loopback exchanger").
#pragma once

#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <vector>

#include "spfft/communicator.hpp"

namespace spfft {

struct LocalGroupState {
  explicit LocalGroupState(int n) : size(n), slots(n, nullptr) {}
  void barrier();

  int size;
  std::mutex mutex;
  std::condition_variable cv;
  int arrived = 0;
  std::uint64_t generation = 0;
  std::vector<const void*> slots;  // one published pointer per rank
};

class LocalGroupCommunicator : public Communicator {
public:
  LocalGroupCommunicator(std::shared_ptr<LocalGroupState> state, int rank)
      : state_(std::move(state)), rank_(rank) {}

  int rank() const override { return rank_; }
  int size() const override { return state_->size; }
  void allgather(const void* send, void* recv, std::size_t bytes) override;
  void alltoallv(const void* send, const std::size_t* sendCounts, const std::size_t* sendDispls,
                 void* recv, const std::size_t* recvCounts,
                 const std::size_t* recvDispls) override;
  void barrier() override { state_->barrier(); }
  std::shared_ptr<Communicator> duplicate() const override;
  bool is_local_group() const override { return true; }

private:
  std::shared_ptr<LocalGroupState> state_;
  int rank_;
};

}  // namespace spfft
