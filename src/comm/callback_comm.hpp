// Communicator implemented by user callbacks (C API); the Python front end
// plugs torch.distributed in here.
#pragma once

#include <memory>

#include "spfft/amd.h"
#include "spfft/communicator.hpp"

namespace spfft {

class CallbackCommunicator : public Communicator {
public:
  explicit CallbackCommunicator(const SpfftAmdCommCallbacks& cb);
  int rank() const override { return holder_->cb.rank; }
  int size() const override { return holder_->cb.size; }
  void allgather(const void* send, void* recv, std::size_t bytes) override;
  void alltoallv(const void* send, const std::size_t* sendCounts, const std::size_t* sendDispls,
                 void* recv, const std::size_t* recvCounts,
                 const std::size_t* recvDispls) override;
  void barrier() override;
  std::shared_ptr<Communicator> duplicate() const override {
    return std::make_shared<CallbackCommunicator>(*this);
  }

private:
  struct Holder {
    explicit Holder(const SpfftAmdCommCallbacks& c) : cb(c) {}
    ~Holder();
    SpfftAmdCommCallbacks cb;
  };
  std::shared_ptr<Holder> holder_;
};

}  // namespace spfft
