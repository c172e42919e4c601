#include "gpu/device_comm.hpp"

#include <rccl/rccl.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "core/common.hpp"
#include "core/timing.hpp"
#include "gpu/gpu_runtime.hpp"
#include "kernels/peer_sync.hpp"
#include "spfft/exceptions.hpp"

namespace spfft {

DeviceComm::~DeviceComm() = default;

double comm_timeout_seconds() {
  // default 120 s: a dead or missing peer becomes an MPIError instead of a hang;
  // SPFFT_COMM_TIMEOUT=0 waits forever
  static const double t = [] {
    const char* e = std::getenv("SPFFT_COMM_TIMEOUT");
    return e && *e ? std::max(0.0, std::atof(e)) : 120.0;
  }();
  return t;
}

namespace {

// ------------------------------------------------------------- RCCL channel
// One RCCL communicator plus the stream that carries every exchange issued on
// it. Grids of one process whose communicators have the same members on the
// same devices share one channel (DeviceComm::create): `bench.py --gpus 8`
// with 4 transforms builds one RCCL communicator per rank, not four, and every
// exchange of the process runs on one stream in host call order, the order
// every rank issues them in (transforms are collective). Concurrent kernels of
// several communicators, whose relative order can differ between ranks, are
// the classic multi-communicator hang; a single ordered channel cannot do it.
struct NcclChannel {
  ncclComm_t comm = nullptr;
  int device = 0, rank = 0, size = 0;
  std::unique_ptr<GpuStream> stream;
  std::unique_ptr<GpuEvent> in, out;
  std::mutex m;
  bool aborted = false;
  std::string detail;  // why initialisation failed (comm == nullptr)

  ~NcclChannel() {
    if (comm && !process_exiting()) (void)ncclCommDestroy(comm);
  }
  bool ok() const { return comm != nullptr; }

  // Non-blocking communicator calls return ncclInProgress while RCCL works in
  // the background: poll until done, abort past the deadline (a rank that
  // never arrives cannot leave the others inside RCCL).
  ncclResult_t settle(ncclResult_t r, double seconds) {
    using clock = std::chrono::steady_clock;
    const auto t0 = clock::now();
    while (r == ncclInProgress) {
      if (seconds > 0 && std::chrono::duration<double>(clock::now() - t0).count() > seconds) {
        detail = "RCCL: no progress within SPFFT_COMM_TIMEOUT = " + std::to_string(seconds) + " s";
        return ncclInProgress;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(100));
      if (ncclCommGetAsyncError(comm, &r) != ncclSuccess) r = ncclSystemError;
    }
    return r;
  }

  // Collective over `group` (rank r of the channel = rank r of group, or a
  // size-1 channel when selfOnly). Never throws between the collectives.
  void init(Communicator* group, bool selfOnly, int injectFault) {
    DeviceGuard guard(device);
    struct IdMsg {
      ncclUniqueId id;
      int ok;
    };
    IdMsg mine;
    std::memset(&mine, 0, sizeof(mine));
    mine.ok = 1;
    if ((selfOnly || rank == 0) && ncclGetUniqueId(&mine.id) != ncclSuccess) mine.ok = 0;
    IdMsg root = mine;
    if (!selfOnly) {
      std::vector<IdMsg> all(size);
      group->allgather(&mine, all.data(), sizeof(IdMsg));
      root = all[0];
    }
    if (!root.ok) {
      detail = "RCCL: ncclGetUniqueId failed on rank 0";
      return;
    }
    // fault injection: 1 = every rank fails, 2 = only the last rank fails (the
    // others then wait for it until the init deadline and abort)
    if (injectFault == 1 || (injectFault == 2 && rank == size - 1)) {
      detail = "RCCL: initialisation failure injected (SPFFT_FAULT_RCCL_INIT)";
      return;
    }
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&comm, size, root.id, rank, &cfg);
    if (r == ncclInProgress || r == ncclSuccess) r = settle(r, comm_timeout_seconds());
    if (r != ncclSuccess) {
      if (detail.empty()) detail = std::string("RCCL: ncclCommInitRankConfig: ") + ncclGetErrorString(r);
      if (comm) (void)ncclCommAbort(comm);
      comm = nullptr;
      return;
    }
    stream.reset(new GpuStream(true));
    in.reset(new GpuEvent());
    out.reset(new GpuEvent());
  }

  void check_usable() {
    if (aborted || !comm) {
      set_error_detail("RCCL: the communicator was aborted after an earlier failure");
      throw MPIError();
    }
  }
  void nccl_check(ncclResult_t r, const char* what) {
    if (r == ncclInProgress) r = settle(r, comm_timeout_seconds());
    if (r != ncclSuccess) {
      set_error_detail(std::string("RCCL ") + what + ": " + ncclGetErrorString(r) + " " +
                       (detail.empty() ? ncclGetLastError(comm) : detail));
      throw MPIError();
    }
  }

  struct Xfer {
    const char* send;  // peer-bound block (or nullptr)
    char* recv;        // arriving block (or nullptr)
    std::size_t bytes;
    int peer;
  };
  // Enqueues the transfers after the work queued so far on `caller`; `caller`
  // continues once every block has arrived.
  void run(const std::vector<Xfer>& xs, hipStream_t caller) {
    std::lock_guard<std::mutex> lock(m);
    check_usable();
    DeviceGuard guard(device);
    hipStream_t cs = stream->get();
    in->record(caller);
    in->wait_on(cs);
    nccl_check(ncclGroupStart(), "ncclGroupStart");
    for (const Xfer& x : xs) {
      if (x.send) nccl_check(ncclSend(x.send, x.bytes, ncclChar, x.peer, comm, cs), "ncclSend");
      if (x.recv) nccl_check(ncclRecv(x.recv, x.bytes, ncclChar, x.peer, comm, cs), "ncclRecv");
    }
    nccl_check(ncclGroupEnd(), "ncclGroupEnd");
    out->record(cs);
    out->wait_on(caller);
  }

  bool healthy(std::string* why) {
    if (aborted) {
      if (why) *why = "RCCL: communicator aborted";
      return false;
    }
    ncclResult_t r = ncclSuccess;
    if (!comm || ncclCommGetAsyncError(comm, &r) != ncclSuccess) return true;  // cannot tell
    if (r == ncclSuccess || r == ncclInProgress) return true;
    if (why) *why = std::string("RCCL asynchronous error: ") + ncclGetErrorString(r);
    return false;
  }
  void abort() {
    std::lock_guard<std::mutex> lock(m);
    if (aborted || !comm) return;
    aborted = true;
    (void)ncclCommAbort(comm);
    comm = nullptr;
  }
};

// Process-wide channel registry, keyed by the member list (host, pid, device of
// every rank, in rank order) and the device.
std::mutex gChannelMutex;
std::map<std::string, std::weak_ptr<NcclChannel>>& channel_registry() {
  static auto* r = new std::map<std::string, std::weak_ptr<NcclChannel>>();  // outlives atexit
  return *r;
}
std::atomic<int> gChannelsCreated{0};

// SPFFT_FAULT_EXCHANGE_ABORT=N (fault injection, failure-detection tests): the
// N-th exchange of a data plane aborts its RCCL communicator first, so that
// exchange and every later one fail with MPIError
int fault_abort_at() {
  const char* e = std::getenv("SPFFT_FAULT_EXCHANGE_ABORT");
  return e && *e ? std::atoi(e) : 0;
}

class RcclDeviceComm : public DeviceComm {
public:
  explicit RcclDeviceComm(std::shared_ptr<NcclChannel> ch) : ch_(std::move(ch)), faultAt_(fault_abort_at()) {}

  void alltoallv(const void* send, const std::int64_t* sc, const std::int64_t* sd, void* recv,
                 const std::int64_t* rc, const std::int64_t* rd, hipStream_t stream) override {
    SPFFT_TIMED_SCOPE("rccl_alltoallv");
    if (++calls_ == faultAt_) ch_->abort();
    ch_->check_usable();
    const int me = ch_->rank, P = ch_->size;
    const char* s = static_cast<const char*>(send);
    char* r = static_cast<char*>(recv);
    // the local block never leaves the GPU
    if (sc[me] > 0)
      gpu_check(hipMemcpyAsync(r + rd[me], s + sd[me], static_cast<std::size_t>(sc[me]),
                               hipMemcpyDeviceToDevice, stream),
                "hipMemcpyAsync");
    std::vector<NcclChannel::Xfer> xs;
    xs.reserve(2 * P);
    for (int k = 1; k < P; ++k) {
      // staggered peer order so every xGMI link is busy from the start
      const int to = (me + k) % P;
      const int from = (me - k + P) % P;
      if (sc[to] > 0) xs.push_back({s + sd[to], nullptr, static_cast<std::size_t>(sc[to]), to});
      if (rc[from] > 0) xs.push_back({nullptr, r + rd[from], static_cast<std::size_t>(rc[from]), from});
    }
    if (!xs.empty()) ch_->run(xs, stream);
  }
  bool host_synchronous() const override { return false; }
  const char* kind() const override { return "rccl"; }
  bool healthy(std::string* detail) override { return ch_->healthy(detail); }
  void check() override {
    std::string d;
    if (!healthy(&d)) {
      set_error_detail(d);
      throw MPIError();
    }
  }
  void abort() override { ch_->abort(); }
  std::string describe() const override {
    char b[96];
    std::snprintf(b, sizeof(b), "rccl comm %p (%d ranks, %d channels in process)",
                  static_cast<void*>(ch_->comm), ch_->size, gChannelsCreated.load());
    return b;
  }

private:
  std::shared_ptr<NcclChannel> ch_;
  int faultAt_ = 0, calls_ = 0;
};

// In-process virtual ranks (local group) with every block moved by RCCL: each
// virtual rank owns a size-1 RCCL communicator and receives the blocks of every
// rank q (itself included) by a grouped ncclSend/ncclRecv pair to itself, on
// the channel stream, with the real counts and displacements. This runs the
// RCCL data path (group semantics, stream hand-off, byte layouts, async-error
// polling, abort) on a single GPU, where RCCL refuses two ranks per device.
class RcclSelfDeviceComm : public DeviceComm {
public:
  RcclSelfDeviceComm(const std::shared_ptr<Communicator>& comm, std::shared_ptr<NcclChannel> ch)
      : comm_(comm), ch_(std::move(ch)), faultAt_(fault_abort_at()) {}

  void alltoallv(const void* send, const std::int64_t* sc, const std::int64_t* sd, void* recv,
                 const std::int64_t* rc, const std::int64_t* rd, hipStream_t stream) override {
    SPFFT_TIMED_SCOPE("rccl_self_alltoallv");
    if (++calls_ == faultAt_) ch_->abort();
    ch_->check_usable();
    const int P = comm_->size(), me = comm_->rank();
    // every virtual rank's send buffer is complete before anyone pulls from it
    gpu_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    struct View {
      const char* send;
      const std::int64_t* counts;
      const std::int64_t* displs;
    };
    View mine{static_cast<const char*>(send), sc, sd};
    std::vector<View> all(P);
    comm_->allgather(&mine, all.data(), sizeof(View));
    std::vector<NcclChannel::Xfer> xs;
    for (int k = 0; k < P; ++k) {
      const int q = (me - k + P) % P;
      const std::int64_t n = all[q].counts[me];
      if (n != rc[q]) throw MPIError();
      if (n <= 0) continue;
      xs.push_back({all[q].send + all[q].displs[me], nullptr, static_cast<std::size_t>(n), 0});
      xs.push_back({nullptr, static_cast<char*>(recv) + rd[q], static_cast<std::size_t>(n), 0});
    }
    if (!xs.empty()) ch_->run(xs, stream);
    gpu_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    comm_->barrier();  // senders may reuse their buffers only after every pull
  }
  bool host_synchronous() const override { return true; }
  const char* kind() const override { return "rccl-self"; }
  bool healthy(std::string* detail) override { return ch_->healthy(detail); }
  void check() override {
    std::string d;
    if (!healthy(&d)) {
      set_error_detail(d);
      throw MPIError();
    }
  }
  void abort() override { ch_->abort(); }

private:
  std::shared_ptr<Communicator> comm_;
  std::shared_ptr<NcclChannel> ch_;
  int faultAt_ = 0, calls_ = 0;
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
  long long pid;
  int domain, bus, device, ordinal;
  int prefer;  // SPFFT_GPU_EXCHANGE: 0 auto, 1 rccl, 2 peer (ipc)
  int fault;   // SPFFT_FAULT_RCCL_INIT (rank 0's value is used everywhere)
};

std::uint64_t host_hash() {
  char name[256] = {0};
  (void)gethostname(name, sizeof(name) - 1);
  std::uint64_t h = 1469598103934665603ull;  // FNV-1a
  for (const char* c = name; *c; ++c) h = (h ^ static_cast<unsigned char>(*c)) * 1099511628211ull;
  return h;
}

int env_choice(const char* name) {
  const char* env = std::getenv(name);
  const std::string v = env ? env : "";
  return v == "rccl" ? 1 : (v == "ipc" || v == "peer" ? 2 : 0);
}

int env_fault() {
  const char* e = std::getenv("SPFFT_FAULT_RCCL_INIT");
  return e && *e ? std::atoi(e) : 0;
}

bool share_channels() {
  const char* e = std::getenv("SPFFT_RCCL_SHARE");
  return !(e && *e == '0');
}

// The process's channel for `key`, created collectively if any rank lacks a
// live one (the reuse decision is allgathered, so every rank either reuses or
// takes part in the new communicator's initialisation).
std::shared_ptr<NcclChannel> acquire_channel(Communicator* group, const std::string& key, int device,
                                             int rank, int size, bool selfOnly, int fault) {
  std::shared_ptr<NcclChannel> ch;
  const bool share = share_channels() && fault == 0;
  if (share) {
    std::lock_guard<std::mutex> lock(gChannelMutex);
    auto it = channel_registry().find(key);
    if (it != channel_registry().end()) ch = it->second.lock();
    if (ch && (ch->aborted || !ch->ok())) ch.reset();
  }
  int have = ch ? 1 : 0;
  if (!selfOnly) {
    std::vector<int> all(size);
    group->allgather(&have, all.data(), sizeof(int));
    for (int v : all) have = have && v;
  }
  if (have) return ch;
  ch = std::make_shared<NcclChannel>();
  ch->device = device;
  ch->rank = selfOnly ? 0 : rank;
  ch->size = selfOnly ? 1 : size;
  ch->init(group, selfOnly, fault);
  if (ch->ok()) {
    ++gChannelsCreated;
    if (share) {
      std::lock_guard<std::mutex> lock(gChannelMutex);
      channel_registry()[key] = ch;
    }
  }
  return ch;
}

}  // namespace

int DeviceComm::rccl_channels_created() { return gChannelsCreated.load(); }

std::unique_ptr<DeviceComm> DeviceComm::create(const std::shared_ptr<Communicator>& comm,
                                               int device, SpfftExchangeType exchange,
                                               void* const buffers[2]) {
  if (!comm) throw InternalError();
  const bool unbuffered = exchange == SPFFT_EXCH_UNBUFFERED;
  const int prefLocal = env_choice("SPFFT_GPU_EXCHANGE");
  if (comm->is_local_group()) {
    // virtual ranks of one process: SPFFT_GPU_EXCHANGE=rccl moves every block
    // through RCCL (size-1 communicator per virtual rank); otherwise peer
    // writes (UNBUFFERED) or device-to-device copies
    if (prefLocal == 1) {
      char key[64];
      std::snprintf(key, sizeof(key), "self/%d/%d/%d", device, comm->rank(), comm->size());
      auto ch = acquire_channel(comm.get(), key, device, comm->rank(), comm->size(), true, 0);
      if (!ch->ok()) {
        set_error_detail(ch->detail);
        throw MPIError();
      }
      return std::unique_ptr<DeviceComm>(new RcclSelfDeviceComm(comm, ch));
    }
    if (unbuffered) return std::unique_ptr<DeviceComm>(new PeerDeviceComm(comm, device, buffers, false));
    return std::unique_ptr<DeviceComm>(new LoopbackDeviceComm(comm));
  }
  // data-plane choice, identical on every rank (decided from allgathered facts)
  NodeInfo mine{};
  mine.host = host_hash();
  mine.pid = static_cast<long long>(getpid());
  mine.ordinal = device;
  {
    DeviceGuard guard(device);
    (void)hipDeviceGetAttribute(&mine.domain, hipDeviceAttributePciDomainID, device);
    (void)hipDeviceGetAttribute(&mine.bus, hipDeviceAttributePciBusId, device);
    (void)hipDeviceGetAttribute(&mine.device, hipDeviceAttributePciDeviceId, device);
  }
  mine.prefer = prefLocal;
  mine.fault = env_fault();
  const int P = comm->size();
  std::vector<NodeInfo> all(P);
  comm->allgather(&mine, all.data(), sizeof(NodeInfo));
  bool oneNode = true, sharedDevice = false;
  std::string key = "rccl";
  for (int q = 0; q < P; ++q) {
    oneNode = oneNode && all[q].host == all[0].host;
    for (int r = 0; r < q; ++r)
      sharedDevice = sharedDevice || (all[q].host == all[r].host && all[q].domain == all[r].domain &&
                                      all[q].bus == all[r].bus && all[q].device == all[r].device);
    char m[96];
    std::snprintf(m, sizeof(m), "/%llx:%lld:%d.%d.%d", static_cast<unsigned long long>(all[q].host),
                  all[q].pid, all[q].domain, all[q].bus, all[q].ordinal);
    key += m;
  }
  // every rank decides from rank 0's settings (environments may differ)
  const int prefer = all[0].prefer;
  const int fault = all[0].fault;
  const bool peer =
      oneNode && prefer != 1 && (unbuffered || (sharedDevice && fault == 0) || prefer == 2);
  if (peer) return std::unique_ptr<DeviceComm>(new PeerDeviceComm(comm, device, buffers, true));
  auto ch = acquire_channel(comm.get(), key, device, comm->rank(), P, false, fault);
  // every rank learns whether every RCCL communicator came up
  int ok = ch->ok() ? 1 : 0;
  std::vector<int> oks(P);
  comm->allgather(&ok, oks.data(), sizeof(int));
  bool allOk = true;
  for (int v : oks) allOk = allOk && v != 0;
  if (allOk) return std::unique_ptr<DeviceComm>(new RcclDeviceComm(ch));
  const std::string why = ch->ok() ? std::string("RCCL: another rank failed to initialise") : ch->detail;
  ch->abort();
  ch.reset();
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
