#include <algorithm>
#include <cstring>
#include <vector>

#include "comm/callback_comm.hpp"
#include "comm/local_group.hpp"
#include "spfft/communicator.hpp"
#include "spfft/exceptions.hpp"

namespace spfft {

Communicator::~Communicator() = default;
ExchangeRequest::~ExchangeRequest() = default;

namespace {
struct CompletedRequest : ExchangeRequest {
  void wait() override {}
};
}  // namespace

std::unique_ptr<ExchangeRequest> Communicator::ialltoallv(const void* send, const std::size_t* sc,
                                                          const std::size_t* sd, void* recv,
                                                          const std::size_t* rc,
                                                          const std::size_t* rd) {
  alltoallv(send, sc, sd, recv, rc, rd);
  return std::unique_ptr<ExchangeRequest>(new CompletedRequest());
}

void Communicator::alltoallw(const void* send, const StridedLayout* sl, void* recv,
                             const StridedLayout* rl) {
  const int P = size();
  std::vector<std::size_t> sc(P), sd(P), rc(P), rd(P);
  std::size_t st = 0, rt = 0;
  for (int r = 0; r < P; ++r) {
    sc[r] = sl[r].count * sl[r].blockBytes;
    sd[r] = st;
    st += sc[r];
    rc[r] = rl[r].count * rl[r].blockBytes;
    rd[r] = rt;
    rt += rc[r];
  }
  std::vector<char> sbuf(std::max<std::size_t>(st, 1)), rbuf(std::max<std::size_t>(rt, 1));
  for (int r = 0; r < P; ++r)
    for (std::size_t b = 0; b < sl[r].count; ++b)
      std::memcpy(sbuf.data() + sd[r] + b * sl[r].blockBytes,
                  static_cast<const char*>(send) + sl[r].offset + b * sl[r].strideBytes, sl[r].blockBytes);
  alltoallv(sbuf.data(), sc.data(), sd.data(), rbuf.data(), rc.data(), rd.data());
  for (int r = 0; r < P; ++r)
    for (std::size_t b = 0; b < rl[r].count; ++b)
      std::memcpy(static_cast<char*>(recv) + rl[r].offset + b * rl[r].strideBytes,
                  rbuf.data() + rd[r] + b * rl[r].blockBytes, rl[r].blockBytes);
}

std::unique_ptr<ExchangeRequest> Communicator::ialltoallw(const void* send, const StridedLayout* sl,
                                                          void* recv, const StridedLayout* rl) {
  alltoallw(send, sl, recv, rl);
  return std::unique_ptr<ExchangeRequest>(new CompletedRequest());
}

void Communicator::barrier() {
  char token = 0;
  std::vector<char> all(static_cast<std::size_t>(size()));
  allgather(&token, all.data(), 1);
}

// ---------------------------------------------------------------------------
void LocalGroupState::barrier() {
  std::unique_lock<std::mutex> lock(mutex);
  const std::uint64_t gen = generation;
  if (++arrived == size) {
    arrived = 0;
    ++generation;
    cv.notify_all();
  } else {
    cv.wait(lock, [&] { return generation != gen; });
  }
}

void LocalGroupCommunicator::allgather(const void* send, void* recv, std::size_t bytes) {
  state_->slots[rank_] = send;
  state_->barrier();
  for (int r = 0; r < state_->size; ++r) {
    std::memcpy(static_cast<char*>(recv) + r * bytes, state_->slots[r], bytes);
  }
  state_->barrier();
}

namespace {
struct A2AView {
  const void* send;
  const std::size_t* counts;
  const std::size_t* displs;
};
}  // namespace

void LocalGroupCommunicator::alltoallv(const void* send, const std::size_t* sendCounts,
                                       const std::size_t* sendDispls, void* recv,
                                       const std::size_t* recvCounts,
                                       const std::size_t* recvDispls) {
  A2AView mine{send, sendCounts, sendDispls};
  state_->slots[rank_] = &mine;
  state_->barrier();
  for (int q = 0; q < state_->size; ++q) {
    const auto* v = static_cast<const A2AView*>(state_->slots[q]);
    const std::size_t n = v->counts[rank_];
    if (n != recvCounts[q]) throw MPIError();
    if (n) {
      std::memcpy(static_cast<char*>(recv) + recvDispls[q],
                  static_cast<const char*>(v->send) + v->displs[rank_], n);
    }
  }
  state_->barrier();
}

std::shared_ptr<Communicator> LocalGroupCommunicator::duplicate() const {
  std::shared_ptr<LocalGroupState> fresh;
  if (rank_ == 0) fresh = std::make_shared<LocalGroupState>(state_->size);
  state_->slots[rank_] = rank_ == 0 ? &fresh : nullptr;
  state_->barrier();
  auto shared = *static_cast<const std::shared_ptr<LocalGroupState>*>(state_->slots[0]);
  state_->barrier();
  return std::make_shared<LocalGroupCommunicator>(std::move(shared), rank_);
}

std::vector<std::shared_ptr<Communicator>> create_local_communicators(int size) {
  if (size < 1) throw InvalidParameterError();
  auto state = std::make_shared<LocalGroupState>(size);
  std::vector<std::shared_ptr<Communicator>> comms;
  for (int r = 0; r < size; ++r) comms.push_back(std::make_shared<LocalGroupCommunicator>(state, r));
  return comms;
}

// ---------------------------------------------------------------------------
CallbackCommunicator::CallbackCommunicator(const SpfftAmdCommCallbacks& cb)
    : holder_(std::make_shared<Holder>(cb)) {
  if (!cb.allgather || !cb.alltoallv || cb.size < 1 || cb.rank < 0 || cb.rank >= cb.size)
    throw InvalidParameterError();
}

CallbackCommunicator::Holder::~Holder() {
  if (cb.destroy) cb.destroy(cb.context);
}

void CallbackCommunicator::allgather(const void* send, void* recv, std::size_t bytes) {
  if (holder_->cb.allgather(holder_->cb.context, send, recv, bytes) != 0) throw MPIError();
}

void CallbackCommunicator::alltoallv(const void* send, const std::size_t* sendCounts,
                                     const std::size_t* sendDispls, void* recv,
                                     const std::size_t* recvCounts,
                                     const std::size_t* recvDispls) {
  if (holder_->cb.alltoallv(holder_->cb.context, send, sendCounts, sendDispls, recv, recvCounts,
                            recvDispls) != 0)
    throw MPIError();
}

void CallbackCommunicator::barrier() {
  if (holder_->cb.barrier) {
    if (holder_->cb.barrier(holder_->cb.context) != 0) throw MPIError();
  } else {
    Communicator::barrier();
  }
}

}  // namespace spfft
