#include "gpu/device_comm.hpp"

#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "core/timing.hpp"
#include "gpu/gpu_runtime.hpp"
#include "spfft/exceptions.hpp"

namespace spfft {

DeviceComm::~DeviceComm() = default;

namespace {

inline void nccl_check(ncclResult_t r) {
  if (r != ncclSuccess) throw MPIError();
}

class RcclDeviceComm : public DeviceComm {
public:
  RcclDeviceComm(const std::shared_ptr<Communicator>& comm, int device)
      : comm_(comm), rank_(comm->rank()), size_(comm->size()) {
    DeviceGuard guard(device);
    ncclUniqueId id;
    std::memset(&id, 0, sizeof(id));
    if (rank_ == 0) nccl_check(ncclGetUniqueId(&id));
    std::vector<ncclUniqueId> all(size_);
    comm_->allgather(&id, all.data(), sizeof(id));
    nccl_check(ncclCommInitRank(&nccl_, size_, all[0], rank_));
  }
  ~RcclDeviceComm() override {
    if (nccl_ && !process_exiting()) (void)ncclCommDestroy(nccl_);
  }

  void alltoallv(const void* send, const std::int64_t* sc, const std::int64_t* sd, void* recv,
                 const std::int64_t* rc, const std::int64_t* rd, hipStream_t stream) override {
    SPFFT_TIMED_SCOPE("rccl_alltoallv");
    const char* s = static_cast<const char*>(send);
    char* r = static_cast<char*>(recv);
    // the local block never leaves the GPU
    if (sc[rank_] > 0)
      gpu_check(hipMemcpyAsync(r + rd[rank_], s + sd[rank_], static_cast<std::size_t>(sc[rank_]),
                               hipMemcpyDeviceToDevice, stream),
                "hipMemcpyAsync");
    nccl_check(ncclGroupStart());
    for (int k = 1; k < size_; ++k) {
      // staggered peer order so every xGMI link is busy from the start
      const int to = (rank_ + k) % size_;
      const int from = (rank_ - k + size_) % size_;
      if (sc[to] > 0) nccl_check(ncclSend(s + sd[to], static_cast<std::size_t>(sc[to]), ncclChar, to, nccl_, stream));
      if (rc[from] > 0)
        nccl_check(ncclRecv(r + rd[from], static_cast<std::size_t>(rc[from]), ncclChar, from, nccl_, stream));
    }
    nccl_check(ncclGroupEnd());
  }
  bool host_synchronous() const override { return false; }

private:
  std::shared_ptr<Communicator> comm_;
  int rank_, size_;
  ncclComm_t nccl_ = nullptr;
};

class LoopbackDeviceComm : public DeviceComm {
public:
  explicit LoopbackDeviceComm(const std::shared_ptr<Communicator>& comm) : comm_(comm) {}

  void alltoallv(const void* send, const std::int64_t* sc, const std::int64_t* sd, void* recv,
                 const std::int64_t* rc, const std::int64_t* rd, hipStream_t stream) override {
    SPFFT_TIMED_SCOPE("loopback_alltoallv");
    const int P = comm_->size(), me = comm_->rank();
    gpu_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    struct View {
      const char* send;
      const std::int64_t* counts;
      const std::int64_t* displs;
    };
    View mine{static_cast<const char*>(send), sc, sd};
    std::vector<View> all(P);
    comm_->allgather(&mine, all.data(), sizeof(View));
    for (int q = 0; q < P; ++q) {
      const std::int64_t n = all[q].counts[me];
      if (n != rc[q]) throw MPIError();
      if (n > 0)
        gpu_check(hipMemcpyAsync(static_cast<char*>(recv) + rd[q], all[q].send + all[q].displs[me],
                                 static_cast<std::size_t>(n), hipMemcpyDefault, stream),
                  "hipMemcpyAsync");
    }
    gpu_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    comm_->barrier();  // senders may reuse their buffers only after every pull
  }
  bool host_synchronous() const override { return true; }

private:
  std::shared_ptr<Communicator> comm_;
};

}  // namespace

std::unique_ptr<DeviceComm> DeviceComm::create(const std::shared_ptr<Communicator>& comm,
                                               int device) {
  if (!comm) throw InternalError();
  if (comm->is_local_group()) return std::unique_ptr<DeviceComm>(new LoopbackDeviceComm(comm));
  return std::unique_ptr<DeviceComm>(new RcclDeviceComm(comm, device));
}

}  // namespace spfft
