#include "gpu/device_comm.hpp"

#include <rccl/rccl.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "core/common.hpp"
#include "core/timing.hpp"
#include "gpu/gpu_runtime.hpp"
#include "kernels/peer_sync.hpp"
#include "spfft/exceptions.hpp"

namespace spfft {

DeviceComm::~DeviceComm() = default;

namespace {

inline void nccl_check(ncclResult_t r) {
  if (r != ncclSuccess) {
    set_error_detail(std::string("RCCL: ") + ncclGetErrorString(r) + " " + ncclGetLastError(nullptr));
    throw MPIError();
  }
}

class RcclDeviceComm : public DeviceComm {
public:
  // Collective on comm. Never throws between the collectives, so every rank
  // takes part in both allgathers; ok() tells whether this rank's RCCL
  // communicator came up (DeviceComm::create agrees on the outcome).
  RcclDeviceComm(const std::shared_ptr<Communicator>& comm, int device, bool faultInit)
      : comm_(comm), rank_(comm->rank()), size_(comm->size()) {
    DeviceGuard guard(device);
    struct IdMsg {
      ncclUniqueId id;
      int ok;
    };
    IdMsg mine;
    std::memset(&mine, 0, sizeof(mine));
    mine.ok = 1;
    if (rank_ == 0 && ncclGetUniqueId(&mine.id) != ncclSuccess) mine.ok = 0;
    std::vector<IdMsg> all(size_);
    comm_->allgather(&mine, all.data(), sizeof(IdMsg));
    if (!all[0].ok) {
      detail_ = "RCCL: ncclGetUniqueId failed on rank 0";
      return;
    }
    if (faultInit) {  // fault injection (SPFFT_FAULT_RCCL_INIT=1 on every rank)
      detail_ = "RCCL: initialisation failure injected (SPFFT_FAULT_RCCL_INIT)";
      return;
    }
    const ncclResult_t r = ncclCommInitRank(&nccl_, size_, all[0].id, rank_);
    if (r != ncclSuccess) {
      detail_ = std::string("RCCL: ncclCommInitRank: ") + ncclGetErrorString(r);
      nccl_ = nullptr;
    }
  }
  bool ok() const { return nccl_ != nullptr; }
  const std::string& detail() const { return detail_; }
  ~RcclDeviceComm() override {
    if (nccl_ && !process_exiting()) (void)ncclCommDestroy(nccl_);
  }

  void alltoallv(const void* send, const std::int64_t* sc, const std::int64_t* sd, void* recv,
                 const std::int64_t* rc, const std::int64_t* rd, hipStream_t stream) override {
    SPFFT_TIMED_SCOPE("rccl_alltoallv");
    if (aborted_) {
      set_error_detail("RCCL: the communicator was aborted after an earlier failure");
      throw MPIError();
    }
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
  const char* kind() const override { return "rccl"; }
  bool healthy(std::string* detail) override {
    if (aborted_) return false;
    ncclResult_t r = ncclSuccess;
    if (ncclCommGetAsyncError(nccl_, &r) != ncclSuccess) return true;  // cannot tell
    if (r == ncclSuccess || r == ncclInProgress) return true;
    if (detail) *detail = std::string("RCCL asynchronous error: ") + ncclGetErrorString(r);
    return false;
  }
  void check() override {
    std::string d;
    if (!healthy(&d)) {
      set_error_detail(d.empty() ? "RCCL: communicator aborted" : d);
      throw MPIError();
    }
  }
  void abort() override {
    if (aborted_ || !nccl_) return;
    aborted_ = true;
    (void)ncclCommAbort(nccl_);
    nccl_ = nullptr;
  }

private:
  std::shared_ptr<Communicator> comm_;
  int rank_, size_;
  ncclComm_t nccl_ = nullptr;
  bool aborted_ = false;
  std::string detail_;
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
  const char* kind() const override { return "loopback"; }

private:
  std::shared_ptr<Communicator> comm_;
};

// ------------------------------------------------------------- peer writes
class PeerDeviceComm : public DeviceComm {
public:
  PeerDeviceComm(const std::shared_ptr<Communicator>& comm, int device, void* const buffers[2],
                 bool ipc)
      : comm_(comm), device_(device), me_(comm->rank()), P_(comm->size()), ipc_(ipc) {
    DeviceGuard guard(device);
    const std::size_t fbytes = ((static_cast<std::size_t>(std::max(P_, 1)) * 8 + 4095) / 4096) * 4096;
    // flags are polled by the barrier kernel: uncached so remote stores are seen
    if (hipExtMallocWithFlags(&flags_, fbytes, hipDeviceMallocUncached) != hipSuccess) {
      (void)hipGetLastError();
      gpu_check(hipMalloc(&flags_, fbytes), "hipMalloc");
    }
    gpu_check(hipMemset(flags_, 0, fbytes), "hipMemset");
    gpu_check(hipHostMalloc(reinterpret_cast<void**>(&failHost_), 64,
                            hipHostMallocMapped | hipHostMallocCoherent),
              "hipHostMalloc");
    *failHost_ = 0;
    gpu_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&failDev_), failHost_, 0),
              "hipHostGetDevicePointer");

    void* local[3] = {buffers[0], buffers[1], flags_};
    peers_.assign(P_, {nullptr, nullptr, nullptr});
    if (ipc_) {
      struct Exported {
        hipIpcMemHandle_t h[3];
        int valid[3];
      };
      Exported mine;
      std::memset(&mine, 0, sizeof(mine));
      for (int i = 0; i < 3; ++i) {
        if (!local[i]) continue;
        gpu_check(hipIpcGetMemHandle(&mine.h[i], local[i]), "hipIpcGetMemHandle");
        mine.valid[i] = 1;
      }
      std::vector<Exported> all(P_);
      comm_->allgather(&mine, all.data(), sizeof(Exported));
      for (int q = 0; q < P_; ++q) {
        for (int i = 0; i < 3; ++i) {
          if (q == me_) {
            peers_[q][i] = local[i];
          } else if (all[q].valid[i]) {
            void* p = nullptr;
            gpu_check(hipIpcOpenMemHandle(&p, all[q].h[i], hipIpcMemLazyEnablePeerAccess),
                      "hipIpcOpenMemHandle");
            opened_.push_back(p);
            peers_[q][i] = p;
          }
        }
      }
    } else {
      struct Raw {
        void* p[3];
        int device;
      };
      Raw mine{{local[0], local[1], local[2]}, device};
      std::vector<Raw> all(P_);
      comm_->allgather(&mine, all.data(), sizeof(Raw));
      for (int q = 0; q < P_; ++q) {
        for (int i = 0; i < 3; ++i) peers_[q][i] = all[q].p[i];
        if (all[q].device != device) {
          const hipError_t e = hipDeviceEnablePeerAccess(all[q].device, 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) gpu_check(e, "hipDeviceEnablePeerAccess");
          (void)hipGetLastError();
        }
      }
    }
    std::vector<unsigned long long*> table(P_);
    for (int q = 0; q < P_; ++q) {
      table[q] = static_cast<unsigned long long*>(peers_[q][2]);
      if (!table[q]) throw InternalError();
    }
    table_.reset(new DeviceBuffer(sizeof(void*) * P_));
    gpu_check(hipMemcpy(table_->data(), table.data(), sizeof(void*) * P_, hipMemcpyHostToDevice),
              "hipMemcpy");
    int rateKHz = 0;
    gpu_check(hipDeviceGetAttribute(&rateKHz, hipDeviceAttributeWallClockRate, device),
              "hipDeviceGetAttribute");
    const char* env = std::getenv("SPFFT_PEER_TIMEOUT");
    const double seconds = env && *env ? std::max(0.1, std::atof(env)) : 30.0;
    timeoutTicks_ = static_cast<long long>(seconds * 1e3 * std::max(rateKHz, 1));
    gpu_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    comm_->barrier();  // every flag array is zeroed before the first barrier round
  }

  ~PeerDeviceComm() override {
    if (process_exiting()) return;
    DeviceGuard guard(device_);
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    if (flags_) (void)hipFree(flags_);
    if (failHost_) (void)hipHostFree(failHost_);
  }

  void alltoallv(const void*, const std::int64_t*, const std::int64_t*, void*, const std::int64_t*,
                 const std::int64_t*, hipStream_t) override {
    throw InternalError();  // the stage kernels move the data themselves
  }
  bool host_synchronous() const override { return false; }
  bool peer_writes() const override { return true; }
  void* peer_buffer(int rank, int slot) const override { return peers_.at(rank).at(slot); }
  void prepare_write(int slot, hipStream_t stream) override {
    if (readPending_[slot & 1]) barrier(stream);
  }
  void complete_writes(hipStream_t stream) override { barrier(stream); }
  void note_read(int slot) override { readPending_[slot & 1] = true; }
  void check() override {
    std::string d;
    if (!healthy(&d)) {
      set_error_detail(d);
      throw MPIError();
    }
  }
  bool healthy(std::string* detail) override {
    const unsigned f = __atomic_load_n(failHost_, __ATOMIC_ACQUIRE);
    if (f == 0) return true;
    if (detail)
      *detail = f == kAborted ? "peer exchange: aborted (host-side timeout or an earlier failure)"
                              : "peer exchange: a rank did not reach the exchange barrier in time";
    return false;
  }
  void abort() override {
    // the barrier kernels poll this word and stop waiting
    unsigned expected = 0;
    __atomic_compare_exchange_n(failHost_, &expected, kAborted, false, __ATOMIC_ACQ_REL,
                                __ATOMIC_ACQUIRE);
  }
  const char* kind() const override { return ipc_ ? "ipc" : "peer"; }

private:
  static constexpr unsigned kAborted = 2;
  void barrier(hipStream_t stream) {
    SPFFT_TIMED_SCOPE("peer_barrier");
    if (__atomic_load_n(failHost_, __ATOMIC_ACQUIRE) == kAborted) check();
    DeviceGuard guard(device_);
    if (ipc_) {
      dev::launch_peer_barrier(table_->data<unsigned long long*>(),
                               static_cast<unsigned long long*>(flags_), me_, P_, ++epoch_,
                               failDev_, timeoutTicks_, stream);
    } else {
      // ranks of one process share its few hardware queues: a spinning barrier
      // kernel could sit in front of the very work it waits for, so in-process
      // groups meet on the host instead
      gpu_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
      comm_->barrier();
    }
    readPending_[0] = readPending_[1] = false;
  }

  std::shared_ptr<Communicator> comm_;
  int device_, me_, P_;
  bool ipc_;
  void* flags_ = nullptr;
  unsigned int* failHost_ = nullptr;
  unsigned int* failDev_ = nullptr;
  std::vector<std::array<void*, 3>> peers_;
  std::vector<void*> opened_;
  std::unique_ptr<DeviceBuffer> table_;
  unsigned long long epoch_ = 0;
  long long timeoutTicks_ = 0;
  bool readPending_[2] = {false, false};
};

struct NodeInfo {
  std::uint64_t host;
  int domain, bus, device;
  int prefer;  // SPFFT_GPU_EXCHANGE: 0 auto, 1 rccl, 2 peer (ipc)
};

std::uint64_t host_hash() {
  char name[256] = {0};
  (void)gethostname(name, sizeof(name) - 1);
  std::uint64_t h = 1469598103934665603ull;  // FNV-1a
  for (const char* c = name; *c; ++c) h = (h ^ static_cast<unsigned char>(*c)) * 1099511628211ull;
  return h;
}

}  // namespace

std::unique_ptr<DeviceComm> DeviceComm::create(const std::shared_ptr<Communicator>& comm,
                                               int device, SpfftExchangeType exchange,
                                               void* const buffers[2]) {
  if (!comm) throw InternalError();
  const bool unbuffered = exchange == SPFFT_EXCH_UNBUFFERED;
  if (comm->is_local_group()) {
    if (unbuffered) return std::unique_ptr<DeviceComm>(new PeerDeviceComm(comm, device, buffers, false));
    return std::unique_ptr<DeviceComm>(new LoopbackDeviceComm(comm));
  }
  // data-plane choice, identical on every rank (decided from allgathered facts)
  NodeInfo mine{};
  mine.host = host_hash();
  mine.device = device;
  {
    DeviceGuard guard(device);
    (void)hipDeviceGetAttribute(&mine.domain, hipDeviceAttributePciDomainID, device);
    (void)hipDeviceGetAttribute(&mine.bus, hipDeviceAttributePciBusId, device);
    (void)hipDeviceGetAttribute(&mine.device, hipDeviceAttributePciDeviceId, device);
  }
  const char* env = std::getenv("SPFFT_GPU_EXCHANGE");
  const std::string pref = env ? env : "";
  mine.prefer = pref == "rccl" ? 1 : (pref == "ipc" || pref == "peer" ? 2 : 0);
  const int P = comm->size();
  std::vector<NodeInfo> all(P);
  comm->allgather(&mine, all.data(), sizeof(NodeInfo));
  bool oneNode = true, sharedDevice = false;
  for (int q = 0; q < P; ++q) {
    oneNode = oneNode && all[q].host == all[0].host;
    for (int r = 0; r < q; ++r)
      sharedDevice = sharedDevice || (all[q].host == all[r].host && all[q].domain == all[r].domain &&
                                      all[q].bus == all[r].bus && all[q].device == all[r].device);
  }
  const int prefer = all[0].prefer;
  // fault injection for the fallback below: every rank's RCCL initialisation
  // reports failure (ranks sharing a device then try RCCL first as well)
  const char* fenv = std::getenv("SPFFT_FAULT_RCCL_INIT");
  const bool faultInit = fenv && std::atoi(fenv) != 0;
  const bool peer =
      oneNode && prefer != 1 && (unbuffered || (sharedDevice && !faultInit) || prefer == 2);
  if (peer) return std::unique_ptr<DeviceComm>(new PeerDeviceComm(comm, device, buffers, true));
  std::unique_ptr<RcclDeviceComm> rccl(new RcclDeviceComm(comm, device, faultInit));
  // every rank learns whether every RCCL communicator came up
  int ok = rccl->ok() ? 1 : 0;
  std::vector<int> oks(P);
  comm->allgather(&ok, oks.data(), sizeof(int));
  bool allOk = true;
  for (int v : oks) allOk = allOk && v != 0;
  if (allOk) return std::unique_ptr<DeviceComm>(rccl.release());
  const std::string why = rccl->ok() ? std::string("RCCL: another rank failed to initialise") : rccl->detail();
  rccl->abort();
  rccl.reset();
  // one node: the peer-write data plane (IPC handles over xGMI) moves the data
  // instead; across nodes there is no fallback
  if (!oneNode || prefer == 1) {
    set_error_detail(why);
    throw MPIError();
  }
  if (comm->rank() == 0)
    std::fprintf(stderr, "spfft: %s; using the peer-write (IPC) data plane\n", why.c_str());
  return std::unique_ptr<DeviceComm>(new PeerDeviceComm(comm, device, buffers, true));
}

}  // namespace spfft
