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
#include <random>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "core/common.hpp"
#include "core/fault.hpp"
#include "core/timing.hpp"
#include "gpu/gpu_runtime.hpp"
#include "gpu/ipc_arena.hpp"
#include "kernels/peer_sync.hpp"
#include "kernels/relay_copy.hpp"
#include "spfft/exceptions.hpp"
#include "comm/shm_group.hpp"

namespace spfft {

DeviceComm::~DeviceComm() = default;

double comm_timeout_seconds() {
  // default 0 = no limit: waiting for a slower rank is not an error (MPI
  // semantics); failures are still detected through the data plane's
  // asynchronous error state while the host waits
  static const double t = [] {
    const char* e = std::getenv("SPFFT_COMM_TIMEOUT");
    return e && *e ? std::max(0.0, std::atof(e)) : 0.0;
  }();
  return t;
}

double comm_init_timeout_seconds() {
  const double t = comm_timeout_seconds();
  return t > 0 ? t : 300.0;
}

void append_alltoallv(std::vector<Transfer>& out, int me, int P, const std::int64_t* sc,
                      const std::int64_t* sd, const std::int64_t* rc, const std::int64_t* rd) {
  // the own block never leaves the GPU
  if (sc[me] != rc[me]) throw MPIError();
  if (sc[me] > 0) out.push_back({Transfer::kLocal, me, sd[me], rd[me], sc[me]});
  for (int k = 1; k < P; ++k) {
    const int to = (me + k) % P;
    const int from = (me - k + P) % P;
    if (sc[to] > 0) out.push_back({Transfer::kSend, to, sd[to], 0, sc[to]});
    if (rc[from] > 0) out.push_back({Transfer::kRecv, from, rd[from], 0, rc[from]});
  }
}

void DeviceComm::alltoallv(const void* send, const std::int64_t* sc, const std::int64_t* sd,
                           void* recv, const std::int64_t* rc, const std::int64_t* rd,
                           hipStream_t stream) {
  std::vector<Transfer> xs;
  xs.reserve(2 * 8);
  // (rank and size come from the plane: the counts have one entry per rank)
  append_alltoallv(xs, plane_rank(), plane_size(), sc, sd, rc, rd);
  exchange(send, recv, xs, stream, nullptr);
}

namespace {

// ------------------------------------------------------------- RCCL channel
// One RCCL communicator plus the stream that carries every exchange issued on
// it. Grids of one process whose communicators have the same members on the
// same devices and the same ordering domain (Communicator::channel_domain)
// share one channel (DeviceComm::create): `bench.py --gpus 8` with 4
// transforms builds one RCCL communicator per rank, not four, and every
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
  bool highPriority = true;  // channel stream priority (see channel_priority)
  std::string detail;  // why initialisation failed (comm == nullptr)

  ~NcclChannel() {
    if (comm && !process_exiting()) (void)ncclCommDestroy(comm);
  }
  bool ok() const { return comm != nullptr; }

  // Non-blocking communicator calls return ncclInProgress while RCCL works in
  // the background: poll until done, give up past the deadline (a rank that
  // never arrives cannot leave the others inside RCCL).
  ncclResult_t settle(ncclResult_t r, double seconds) {
    using clock = std::chrono::steady_clock;
    const auto t0 = clock::now();
    while (r == ncclInProgress) {
      if (seconds > 0 && std::chrono::duration<double>(clock::now() - t0).count() > seconds) {
        detail = "RCCL: no progress within " + std::to_string(seconds) + " s";
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
      detail = "RCCL: initialisation failure injected (fault injection RCCL_INIT)";
      return;
    }
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&comm, size, root.id, rank, &cfg);
    if (r == ncclInProgress || r == ncclSuccess) r = settle(r, comm_init_timeout_seconds());
    if (r != ncclSuccess) {
      if (detail.empty()) detail = std::string("RCCL: ncclCommInitRankConfig: ") + ncclGetErrorString(r);
      if (comm) (void)ncclCommAbort(comm);
      comm = nullptr;
      return;
    }
    stream.reset(new GpuStream(highPriority));
    in.reset(new GpuEvent());
    out.reset(new GpuEvent());
  }

  void check_usable() {
    if (aborted || !comm) {
      set_error_detail("RCCL: the communicator was aborted after an earlier failure");
      throw MPIError();
    }
  }
  // A failed call leaves the communicator (and an open group) in an undefined
  // state: the channel is aborted before the error propagates, so later
  // exchanges on it fail fast instead of reusing it. Caller holds `m`.
  // Per-exchange calls wait under SPFFT_COMM_TIMEOUT (default 0 = no limit, a
  // slow peer is not an error; asynchronous errors still end the wait): the
  // channel is shared by every grid of the process, and a deadline here would
  // abort all of them for one late peer.
  void nccl_check(ncclResult_t r, const char* what) {
    if (r == ncclInProgress) r = settle(r, comm_timeout_seconds());
    if (r != ncclSuccess) {
      set_error_detail(std::string("RCCL ") + what + ": " +
                       (r == ncclInProgress ? std::string("no progress") : ncclGetErrorString(r)) + " " +
                       (detail.empty() ? ncclGetLastError(comm) : detail));
      abort_locked();
      throw MPIError();
    }
  }

  struct Xfer {
    const char* send;  // peer-bound block (or nullptr)
    char* recv;        // arriving block (or nullptr)
    std::size_t bytes;
    int peer;
  };
  // Enqueues the transfers. sync == nullptr: after the work queued so far on
  // `caller`, which continues once every block has arrived (one event pair).
  // Otherwise on the channel stream after sync->ready, recording sync->done.
  // `local` copies run on the same stream, ahead of the group.
  void run(const std::vector<Xfer>& xs, const std::vector<Xfer>& local, hipStream_t caller,
           const ExchangeSync* sync) {
    std::lock_guard<std::mutex> lock(m);
    check_usable();
    DeviceGuard guard(device);
    hipStream_t cs = stream->get();
    if (sync) {
      if (sync->ready) gpu_check(hipStreamWaitEvent(cs, sync->ready, 0), "hipStreamWaitEvent");
      if (sync->begin) gpu_check(hipEventRecord(sync->begin, cs), "hipEventRecord");
    } else {
      in->record(caller);
      in->wait_on(cs);
    }
    for (const Xfer& x : local)
      gpu_check(hipMemcpyAsync(x.recv, x.send, x.bytes, hipMemcpyDeviceToDevice, cs), "hipMemcpyAsync");
    if (!xs.empty()) {
      nccl_check(ncclGroupStart(), "ncclGroupStart");
      for (const Xfer& x : xs) {
        const ncclResult_t r = x.send ? ncclSend(x.send, x.bytes, ncclChar, x.peer, comm, cs)
                                      : ncclRecv(x.recv, x.bytes, ncclChar, x.peer, comm, cs);
        if (r != ncclSuccess && r != ncclInProgress) {
          (void)ncclGroupEnd();
          nccl_check(r, x.send ? "ncclSend" : "ncclRecv");
        }
      }
      nccl_check(ncclGroupEnd(), "ncclGroupEnd");
    }
    if (sync) {
      if (sync->done) gpu_check(hipEventRecord(sync->done, cs), "hipEventRecord");
      if (sync->end) gpu_check(hipEventRecord(sync->end, cs), "hipEventRecord");
    } else {
      out->record(cs);
      out->wait_on(caller);
    }
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
  void abort_locked() {
    if (aborted || !comm) return;
    aborted = true;
    (void)ncclCommAbort(comm);
    comm = nullptr;
  }
  void abort() {
    std::lock_guard<std::mutex> lock(m);
    abort_locked();
  }
};

// Process-wide channel registry, keyed by the member list (host, pid, device of
// every rank, in rank order), the ordering domain and the device.
std::mutex gChannelMutex;
std::map<std::string, std::weak_ptr<NcclChannel>>& channel_registry() {
  static auto* r = new std::map<std::string, std::weak_ptr<NcclChannel>>();  // outlives atexit
  return *r;
}
std::atomic<int> gChannelsCreated{0};

// PCI location of a device ordinal of this process
struct PciId {
  int domain, bus, device;
  bool operator==(const PciId& o) const { return domain == o.domain && bus == o.bus && device == o.device; }
};
PciId pci_of(int ordinal) {
  PciId id{-1, -1, -1};
  (void)hipDeviceGetAttribute(&id.domain, hipDeviceAttributePciDomainID, ordinal);
  (void)hipDeviceGetAttribute(&id.bus, hipDeviceAttributePciBusId, ordinal);
  (void)hipDeviceGetAttribute(&id.device, hipDeviceAttributePciDeviceId, ordinal);
  (void)hipGetLastError();
  return id;
}

// "dddd:bb:dd" of a PCI location
std::string pci_string(const PciId& id) {
  char b[32];
  std::snprintf(b, sizeof(b), "%04x:%02x:%02x", id.domain & 0xffff, id.bus & 0xff, id.device & 0xff);
  return b;
}

// JSON list of the distinct entries of `ids`, in first-seen order
std::string json_distinct(const std::vector<std::string>& ids) {
  std::vector<std::string> seen;
  for (const std::string& i : ids)
    if (std::find(seen.begin(), seen.end(), i) == seen.end()) seen.push_back(i);
  std::string o = "[";
  for (std::size_t k = 0; k < seen.size(); ++k) o += (k ? ", \"" : "\"") + seen[k] + "\"";
  return o + "]";
}

// Every rank's device, as PCI location strings (collective)
std::vector<std::string> group_devices(Communicator& comm, int device) {
  PciId mine = pci_of(device);
  std::vector<PciId> all(comm.size());
  comm.allgather(&mine, all.data(), sizeof(PciId));
  std::vector<std::string> out;
  for (const PciId& q : all) out.push_back(pci_string(q));
  return out;
}

// Fault injection EXCHANGE_ABORT = N (testing library, core/fault.hpp): the
// N-th exchange of a data plane aborts its RCCL communicator first, so that
// exchange and every later one fail with MPIError
int fault_abort_at() { return SPFFT_FAULT(EXCHANGE_ABORT); }

class RcclDeviceComm : public DeviceComm {
public:
  explicit RcclDeviceComm(std::shared_ptr<NcclChannel> ch) : ch_(std::move(ch)), faultAt_(fault_abort_at()) {}

  void exchange(const void* send, void* recv, const std::vector<Transfer>& ts, hipStream_t stream,
                const ExchangeSync* sync) override {
    SPFFT_TIMED_SCOPE("rccl_exchange");
    if (++calls_ == faultAt_) ch_->abort();
    ch_->check_usable();
    const char* s = static_cast<const char*>(send);
    char* r = static_cast<char*>(recv);
    std::vector<NcclChannel::Xfer> xs, local;
    xs.reserve(ts.size());
    for (const Transfer& t : ts) {
      const std::size_t n = static_cast<std::size_t>(t.bytes);
      switch (t.kind) {
        case Transfer::kLocal:
          local.push_back({s + t.offset, r + t.dstOffset, n, t.peer});
          break;
        case Transfer::kSend:
          xs.push_back({s + t.offset, nullptr, n, t.peer});
          break;
        default:
          xs.push_back({nullptr, r + t.offset, n, t.peer});
      }
    }
    if (xs.empty() && local.empty() && !sync) return;
    ch_->run(xs, local, stream, sync);
  }
  int plane_rank() const override { return ch_->rank; }
  int plane_size() const override { return ch_->size; }
  bool host_synchronous() const override { return false; }
  hipStream_t channel_stream() const override { return ch_->stream->get(); }
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

// ExchangeSync on the caller's stream (host-synchronous planes)
void sync_begin(const ExchangeSync* sync, hipStream_t stream) {
  if (!sync) return;
  if (sync->ready) gpu_check(hipStreamWaitEvent(stream, sync->ready, 0), "hipStreamWaitEvent");
  if (sync->begin) gpu_check(hipEventRecord(sync->begin, stream), "hipEventRecord");
}
void sync_end(const ExchangeSync* sync, hipStream_t stream) {
  if (!sync) return;
  if (sync->done) gpu_check(hipEventRecord(sync->done, stream), "hipEventRecord");
  if (sync->end) gpu_check(hipEventRecord(sync->end, stream), "hipEventRecord");
}

// In-process planes see every virtual rank's transfer list: the blocks rank
// `me` receives are paired with the senders' lists by NCCL's matching rule (the
// m-th send q -> me with the m-th receive me <- q; the own block with itself),
// which is exactly what a multi-rank RCCL communicator does with the lists
// RcclDeviceComm passes it.
struct PlaneView {
  const char* send;
  const std::vector<Transfer>* xs;
};
struct Pairing {
  const char* src;
  char* dst;
  std::size_t bytes;
};
bool pair_transfers(int me, const std::vector<PlaneView>& all, char* recv, std::vector<Pairing>& out) {
  const int P = static_cast<int>(all.size());
  const std::vector<Transfer>& mine = *all[me].xs;
  for (int k = 0; k < P; ++k) {
    const int q = (me - k + P) % P;
    std::vector<const Transfer*> sends, recvs;
    for (const Transfer& t : *all[q].xs)
      if (q == me ? t.kind == Transfer::kLocal : (t.kind == Transfer::kSend && t.peer == me))
        sends.push_back(&t);
    for (const Transfer& t : mine)
      if (q == me ? t.kind == Transfer::kLocal : (t.kind == Transfer::kRecv && t.peer == q))
        recvs.push_back(&t);
    if (sends.size() != recvs.size()) return false;
    for (std::size_t m = 0; m < sends.size(); ++m) {
      if (sends[m]->bytes != recvs[m]->bytes) return false;
      const std::int64_t dst = q == me ? recvs[m]->dstOffset : recvs[m]->offset;
      out.push_back({all[q].send + sends[m]->offset, recv + dst, static_cast<std::size_t>(sends[m]->bytes)});
    }
  }
  return true;
}

// Collective: every virtual rank's list is visible, the receive side is
// paired. All ranks fail together (an error flag is agreed before anyone
// throws), so no virtual rank is left waiting in a later collective.
std::vector<Pairing> pair_in_group(Communicator& comm, const void* send, void* recv,
                                   const std::vector<Transfer>& xs) {
  const int P = comm.size(), me = comm.rank();
  PlaneView mine{static_cast<const char*>(send), &xs};
  std::vector<PlaneView> all(P);
  comm.allgather(&mine, all.data(), sizeof(PlaneView));
  std::vector<Pairing> pairs;
  int ok = pair_transfers(me, all, static_cast<char*>(recv), pairs) ? 1 : 0;
  std::vector<int> oks(P);
  comm.allgather(&ok, oks.data(), sizeof(int));
  for (int v : oks)
    if (!v) {
      set_error_detail("exchange: transfer lists of the ranks do not match");
      throw MPIError();
    }
  return pairs;
}

// In-process virtual ranks (local group) with every block moved by RCCL: each
// virtual rank owns a size-1 RCCL communicator and receives the blocks of every
// rank q (itself included) by a grouped ncclSend/ncclRecv pair to itself, on
// the channel stream, with the real transfer lists. This runs the RCCL data
// path (group semantics, stream hand-off, byte layouts, async-error polling,
// abort) on a single GPU inside one process.
class RcclSelfDeviceComm : public DeviceComm {
public:
  RcclSelfDeviceComm(const std::shared_ptr<Communicator>& comm, std::shared_ptr<NcclChannel> ch)
      : comm_(comm), ch_(std::move(ch)), faultAt_(fault_abort_at()) {}

  void exchange(const void* send, void* recv, const std::vector<Transfer>& xs, hipStream_t stream,
                const ExchangeSync* sync) override {
    SPFFT_TIMED_SCOPE("rccl_self_exchange");
    if (++calls_ == faultAt_) ch_->abort();
    ch_->check_usable();
    sync_begin(sync, stream);
    // every virtual rank's send buffer is complete before anyone pulls from it
    gpu_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    const std::vector<Pairing> pairs = pair_in_group(*comm_, send, recv, xs);
    std::vector<NcclChannel::Xfer> cx;
    for (const Pairing& p : pairs) {
      cx.push_back({p.src, nullptr, p.bytes, 0});
      cx.push_back({nullptr, p.dst, p.bytes, 0});
    }
    if (!cx.empty()) ch_->run(cx, {}, stream, nullptr);
    gpu_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    comm_->barrier();  // senders may reuse their buffers only after every pull
    sync_end(sync, stream);
  }
  int plane_rank() const override { return comm_->rank(); }
  int plane_size() const override { return comm_->size(); }
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

  void exchange(const void* send, void* recv, const std::vector<Transfer>& xs, hipStream_t stream,
                const ExchangeSync* sync) override {
    SPFFT_TIMED_SCOPE("loopback_exchange");
    sync_begin(sync, stream);
    gpu_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    for (const Pairing& p : pair_in_group(*comm_, send, recv, xs))
      gpu_check(hipMemcpyAsync(p.dst, p.src, p.bytes, hipMemcpyDefault, stream), "hipMemcpyAsync");
    gpu_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    comm_->barrier();  // senders may reuse their buffers only after every pull
    sync_end(sync, stream);
  }
  int plane_rank() const override { return comm_->rank(); }
  int plane_size() const override { return comm_->size(); }
  bool host_synchronous() const override { return true; }
  const char* kind() const override { return "loopback"; }

private:
  std::shared_ptr<Communicator> comm_;
};

// ------------------------------------------------------------- peer writes
// Where the barrier rounds of the cross-process peer plane run
// (SPFFT_PEER_BARRIER, documented in docs/USER_GUIDE.md):
//  - "stream" (default): the barrier kernel on the caller's stream, right
//    behind the stage kernel it frames. The rounds of one plane stay in issue
//    order when transforms of one grid run on different streams: a round
//    issued on another stream than the previous round first waits for that
//    round (an event), so epochs are never published out of order;
//  - "channel": every round of the process on one ordered stream per member
//    set (PeerChannel), handed over by events. Costs two event hops per round:
//    +52 us per round against "host" at 128^3 on 2 ranks sharing a GPU
//    (profiles/r5/ipc);
//  - "host": stream synchronise + communicator barrier, as in-process groups.
enum class PeerBarrier { kStream, kChannel, kHost };
PeerBarrier peer_barrier_mode() {
  static const PeerBarrier m = [] {
    const char* e = std::getenv("SPFFT_PEER_BARRIER");
    const std::string v = e ? e : "";
    return v == "host" ? PeerBarrier::kHost : (v == "channel" ? PeerBarrier::kChannel : PeerBarrier::kStream);
  }();
  return m;
}

// The ordered stream of a process's peer barriers in "channel" mode: one per
// member set and device (the key of the RCCL channels, so the same
// ordering-domain rules apply), shared by every grid and transform of the
// process that talks to the same ranks. Each round is handed over from the
// caller's stream with an event, runs on this stream, and hands back with a
// second event, so the rounds of one process run one at a time in host call
// order, the order every rank issues them in (transforms are collective).
struct PeerChannel {
  int device = 0;
  std::unique_ptr<GpuStream> stream;
  hipEvent_t in = nullptr, out = nullptr;
  std::mutex m;

  PeerChannel(int dev, bool highPriority) : device(dev) {
    DeviceGuard guard(device);
    stream.reset(new GpuStream(highPriority));
    gpu_check(hipEventCreateWithFlags(&in, hipEventDisableTiming), "hipEventCreateWithFlags");
    gpu_check(hipEventCreateWithFlags(&out, hipEventDisableTiming), "hipEventCreateWithFlags");
  }
  ~PeerChannel() {
    if (process_exiting()) return;
    if (in) (void)hipEventDestroy(in);
    if (out) (void)hipEventDestroy(out);
  }
};

std::mutex gPeerChannelMutex;
std::map<std::string, std::weak_ptr<PeerChannel>>& peer_channel_registry() {
  static auto* r = new std::map<std::string, std::weak_ptr<PeerChannel>>();  // outlives atexit
  return *r;
}

std::shared_ptr<PeerChannel> acquire_peer_channel(const std::string& key, int device, bool highPriority) {
  std::lock_guard<std::mutex> lock(gPeerChannelMutex);
  auto& reg = peer_channel_registry();
  auto it = reg.find(key);
  std::shared_ptr<PeerChannel> ch = it != reg.end() ? it->second.lock() : nullptr;
  if (!ch) {
    ch = std::make_shared<PeerChannel>(device, highPriority);
    reg[key] = ch;
  }
  return ch;
}

// A failed route self-test of the peer-write plane (every rank throws it).
struct PeerSelfTestFailed : MPIError {};

unsigned long long fresh_test_nonce() {
  std::random_device rd;
  const auto t = static_cast<unsigned long long>(std::chrono::steady_clock::now().time_since_epoch().count());
  return ((static_cast<unsigned long long>(rd()) << 32) ^ rd() ^ t ^ static_cast<unsigned long long>(getpid())) | 1ull;
}

// Fault injection PEER_SELFTEST (testing library): the last rank corrupts one
// word of its message to rank 0 in the peer plane's self-test.
bool fault_flag_peer_selftest() { return SPFFT_FAULT(PEER_SELFTEST) == 1; }

class PeerDeviceComm : public DeviceComm {
public:
  // In-process group (ipc == false): `buffers` are the grid's exchange sides,
  // shared by plain pointers. Across processes (ipc == true) the exchange
  // sides and the flag array are leased from the IPC arena (ipc_arena.hpp)
  // and the grid switches to them (local_buffer); `bytes` are the sides'
  // sizes.
  PeerDeviceComm(const std::shared_ptr<Communicator>& comm, int device, void* const buffers[2],
                 const std::size_t bytes[2], bool ipc, const std::string& channelKey,
                 bool highPriority = true)
      : comm_(comm), device_(device), me_(comm->rank()), P_(comm->size()), ipc_(ipc) {
    DeviceGuard guard(device);
    gpu_check(hipHostMalloc(reinterpret_cast<void**>(&failHost_), 64,
                            hipHostMallocMapped | hipHostMallocCoherent),
              "hipHostMalloc");
    *failHost_ = 0;
    gpu_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&failDev_), failHost_, 0),
              "hipHostGetDevicePointer");
    peers_.assign(P_, {nullptr, nullptr, nullptr});
    const std::size_t fbytes = static_cast<std::size_t>(dev::peer_flag_words(std::max(P_, 1))) * 8;
    if (ipc_) {
      xcdMask_ = dev::xcd_mask(device);
      open_ipc(bytes, fbytes);
      mode_ = peer_barrier_mode();
      if (mode_ == PeerBarrier::kChannel) channel_ = acquire_peer_channel(channelKey, device, highPriority);
      if (mode_ == PeerBarrier::kStream)
        gpu_check(hipEventCreateWithFlags(&orderEv_, hipEventDisableTiming), "hipEventCreateWithFlags");
      int rateKHz = 0;
      gpu_check(hipDeviceGetAttribute(&rateKHz, hipDeviceAttributeWallClockRate, device),
                "hipDeviceGetAttribute");
      timeoutTicks_ = static_cast<long long>(peer_timeout_seconds() * 1e3 * std::max(rateKHz, 1));
      comm_->barrier();  // every flag array is zeroed before the first barrier round
      devices_ = group_devices(*comm_, device);
      try {
        self_test();
      } catch (...) {
        // (every rank fails together; the destructor does not run for a
        // constructor that throws)
        for (void* p : opened_) ipc_close(p);
        opened_.clear();
        if (flags_) flags_->discard();
        if (orderEv_) (void)hipEventDestroy(orderEv_);
        if (failHost_) (void)hipHostFree(failHost_);
        throw;
      }
      return;
    } else {
      // in-process groups meet on the host: ranks of one process share its few
      // hardware queues, so a spinning barrier kernel could sit in front of
      // the very work it waits for
      struct Raw {
        void* p[2];
        int device;
      };
      Raw mine{{buffers[0], buffers[1]}, device};
      std::vector<Raw> all(P_);
      comm_->allgather(&mine, all.data(), sizeof(Raw));
      for (int q = 0; q < P_; ++q) {
        for (int i = 0; i < 2; ++i) peers_[q][i] = all[q].p[i];
        if (all[q].device != device) {
          const hipError_t e = hipDeviceEnablePeerAccess(all[q].device, 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) gpu_check(e, "hipDeviceEnablePeerAccess");
          (void)hipGetLastError();
        }
      }
    }
    gpu_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    comm_->barrier();
  }

  ~PeerDeviceComm() override {
    if (process_exiting()) return;
    try {
      DeviceGuard guard(device_);
      // the last barrier round of this plane has finished before its flag
      // array goes back to the arena (the caller's streams were synchronised
      // by the executors; the channel stream may still hold the round)
      if (channel_) (void)hipStreamSynchronize(channel_->stream->get());
      if (orderEv_) {
        (void)hipEventSynchronize(orderEv_);
        (void)hipEventDestroy(orderEv_);
      }
      for (void* p : opened_) ipc_close(p);
      // a plane that saw a failure may still receive a late peer's marks:
      // its flag array is not reused
      if (__atomic_load_n(failHost_, __ATOMIC_ACQUIRE) != 0 && flags_) flags_->discard();
      if (failHost_) (void)hipHostFree(failHost_);
    } catch (...) {
    }
  }

  void exchange(const void*, void*, const std::vector<Transfer>&, hipStream_t,
                const ExchangeSync*) override {
    throw InternalError();  // the stage kernels move the data themselves
  }
  int plane_rank() const override { return me_; }
  int plane_size() const override { return P_; }
  bool host_synchronous() const override { return false; }
  bool peer_writes() const override { return true; }
  void* peer_buffer(int rank, int slot) const override { return peers_.at(rank).at(slot); }
  void* local_buffer(int slot) const override {
    if (!ipc_ || slot < 0 || slot > 1 || !sides_[slot]) return nullptr;
    return sides_[slot]->data();
  }
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
    if (detail) {
      if (f & kAborted)
        *detail = "peer exchange: aborted (host-side timeout or an earlier failure)";
      else if (f & kTimedOut)
        *detail = "peer exchange: a rank did not reach the exchange barrier within SPFFT_PEER_TIMEOUT";
      else if (f & dev::kPeerXcdMiss)
        *detail = "peer exchange: a barrier round's workgroups did not run on every XCD (its L2 write-back "
                  "would have missed one); nothing was published";
      else if (f & kPeerGaveUp)
        *detail = "peer exchange: a peer rank gave up waiting at the exchange barrier";
      else
        *detail = "peer exchange: failure word " + std::to_string(f);
    }
    return false;
  }
  void abort() override {
    // the barrier kernels poll this word and stop waiting
    __atomic_fetch_or(failHost_, kAborted, __ATOMIC_ACQ_REL);
  }
  const char* kind() const override { return ipc_ ? "ipc" : "peer"; }
  std::string info_json() const override {
    char b[512];
    const char* where = mode_ == PeerBarrier::kStream ? "stream" : mode_ == PeerBarrier::kChannel ? "channel" : "host";
    std::snprintf(b, sizeof(b),
                  "{\"kind\": \"%s\", \"ranks\": %d, \"barrier\": \"%s\", \"xcd_mask\": %u, "
                  "\"self_test\": \"%s\", \"self_test_ms\": %.3f, \"devices\": %s}",
                  kind(), P_, where, xcdMask_, selfTest_.c_str(), selfTestMs_, json_distinct(devices_).c_str());
    return b;
  }
  std::string describe() const override {
    if (!ipc_) return kind();
    const IpcArenaStats s = ipc_arena_stats();
    char b[160];
    const char* where = mode_ == PeerBarrier::kStream ? "caller stream"
                        : mode_ == PeerBarrier::kChannel ? "peer channel" : "host";
    std::snprintf(b, sizeof(b), "ipc (%d ranks, barrier on %s; arena: %lld blocks allocated, %lld reused, %lld freed)",
                  P_, where, s.allocated, s.reused, s.freed);
    return std::string(b) + "; self-test " + selfTest_;
  }

private:
  static constexpr unsigned kTimedOut = 1, kAborted = 2, kPeerGaveUp = 4;

  // Leases the two exchange sides and the flag array, announces them
  // (handles + headers) and maps every peer's, checking each mapping's header
  // against the announcement. Every rank learns every rank's outcome before
  // anyone throws, so no rank is left in a later collective.
  void open_ipc(const std::size_t bytes[2], std::size_t fbytes) {
    struct Announce {
      IpcExport e[3];
    };
    struct Outcome {
      int ok;
      char why[200];
    };
    Announce mine{};
    Outcome res{1, {0}};
    try {
      for (int i = 0; i < 2; ++i)
        if (bytes[i] > 0) sides_[i] = ipc_acquire(device_, bytes[i], false);
      flags_ = ipc_acquire(device_, fbytes, true);
      gpu_check(hipMemset(flags_->data(), 0, fbytes), "hipMemset");
      for (int i = 0; i < 2; ++i)
        if (sides_[i]) mine.e[i] = sides_[i]->describe();
      mine.e[2] = flags_->describe();
      // fault injection IPC_NONCE (testing library): the last rank announces
      // a nonce its flag array does not carry, as a stale mapping would show
      if (SPFFT_FAULT(IPC_NONCE) == 1 && me_ == P_ - 1) mine.e[2].header.nonce ^= 1;
    } catch (const std::exception& ex) {
      res.ok = 0;
      std::snprintf(res.why, sizeof(res.why), "IPC arena: %s", ex.what());
    }
    std::vector<Announce> all(P_);
    comm_->allgather(&mine, all.data(), sizeof(Announce));
    if (res.ok) {
      try {
        for (int q = 0; q < P_ && res.ok; ++q) {
          for (int i = 0; i < 3 && res.ok; ++i) {
            if (q == me_) {
              peers_[q][i] = i < 2 ? (sides_[i] ? sides_[i]->data() : nullptr) : flags_->data();
              continue;
            }
            if (!all[q].e[i].valid) {
              if (i == 2) {
                res.ok = 0;
                std::snprintf(res.why, sizeof(res.why), "rank %d announced no flag array", q);
              }
              continue;
            }
            std::string why;
            void* p = ipc_open_checked(all[q].e[i], &why);
            if (!p) {
              res.ok = 0;
              std::snprintf(res.why, sizeof(res.why), "rank %d <- rank %d: %s", me_, q, why.c_str());
              break;
            }
            opened_.push_back(p);
            peers_[q][i] = p;
          }
        }
      } catch (const std::exception& ex) {
        res.ok = 0;
        std::snprintf(res.why, sizeof(res.why), "hipIpcOpenMemHandle: %s %s", ex.what(),
                      error_detail().c_str());
      }
    }
    std::vector<Outcome> outs(P_);
    comm_->allgather(&res, outs.data(), sizeof(Outcome));
    for (const Outcome& o : outs) {
      if (o.ok) continue;
      for (void* p : opened_) ipc_close(p);
      opened_.clear();
      set_error_detail(std::string("peer exchange setup: ") + o.why);
      throw MPIError();
    }
    std::vector<unsigned long long*> table(P_);
    for (int q = 0; q < P_; ++q) table[q] = static_cast<unsigned long long*>(peers_[q][2]);
    table_.reset(new DeviceBuffer(sizeof(void*) * P_));
    gpu_check(hipMemcpy(table_->data(), table.data(), sizeof(void*) * P_, hipMemcpyHostToDevice),
              "hipMemcpy");
  }

  static double peer_timeout_seconds() {
    const char* env = std::getenv("SPFFT_PEER_TIMEOUT");
    return env && *env ? std::max(0.1, std::atof(env)) : 30.0;
  }

  // Route self-test (the relay plane's, for the peer-write path): one exchange
  // of a known pattern through the real path. Every rank fills its receive
  // region with old contents and reads it from every XCD (stale L2 lines are
  // the hazard of remote stores), meets the others on the host, stores the
  // pattern into every peer's side with the stage kernels' store flavour, runs
  // one barrier round, and checks every word it received. Every rank learns
  // every outcome; any wrong word fails the plane on every rank
  // (PeerSelfTestFailed: DeviceComm::create falls back to RCCL where it can).
  void self_test() {
    const auto t0 = std::chrono::steady_clock::now();
    struct Side {
      unsigned long long bytes[2];
      unsigned long long nonce;
    };
    Side mine{{sides_[0] ? static_cast<unsigned long long>(sides_[0]->bytes()) : 0ull,
               sides_[1] ? static_cast<unsigned long long>(sides_[1]->bytes()) : 0ull},
              fresh_test_nonce()};
    std::vector<Side> all(P_);
    comm_->allgather(&mine, all.data(), sizeof(Side));
    unsigned long long minb[2] = {~0ull, ~0ull};
    for (const Side& q : all)
      for (int i = 0; i < 2; ++i) minb[i] = std::min(minb[i], q.bytes[i]);
    const unsigned long long nonce = all[0].nonce;
    // the slab side (the z stage's remote stores) when every rank has room
    int slot = minb[1] / P_ >= 16 ? 1 : (minb[0] / P_ >= 16 ? 0 : -1);
    if (slot < 0 || P_ < 2) {
      selfTest_ = "skipped (an exchange side too small)";
      return;
    }
    const std::size_t per = std::min<unsigned long long>(minb[slot] / P_, 256ull << 10) / 16 * 16;
    DeviceGuard guard(device_);
    GpuStream st(false);
    DeviceBuffer words(2 * sizeof(unsigned long long));
    unsigned long long* bad = words.data<unsigned long long>();
    char* region = static_cast<char*>(peers_[me_][slot]);
    gpu_check(hipMemsetAsync(bad, 0, 2 * sizeof(unsigned long long), st.get()), "hipMemsetAsync");
    gpu_check(hipMemsetAsync(region, 0xA5, per * P_, st.get()), "hipMemsetAsync");
    dev::launch_selftest_warm(region, per * P_, bad + 1, st.get());
    gpu_check(hipStreamSynchronize(st.get()), "hipStreamSynchronize");
    comm_->barrier();  // every receiver's L2 holds the old contents before any store
    const int corrupt = fault_flag_peer_selftest() && me_ == P_ - 1 ? 1 : 0;
    for (int k = 1; k < P_; ++k) {
      const int q = (me_ + k) % P_;
      dev::launch_selftest_store(static_cast<char*>(peers_[q][slot]) + me_ * per, per, nonce, me_, q,
                                 corrupt && q == 0, st.get());
    }
    barrier(st.get());
    for (int q = 0; q < P_; ++q)
      if (q != me_) dev::launch_selftest_check(region + q * per, per, nonce, q, me_, bad, st.get());
    unsigned long long wrong = 0;
    gpu_check(hipMemcpyAsync(&wrong, bad, sizeof(wrong), hipMemcpyDeviceToHost, st.get()), "hipMemcpyAsync");
    gpu_check(hipStreamSynchronize(st.get()), "hipStreamSynchronize");
    lastStream_ = nullptr;
    std::string d;
    const int ok = healthy(&d) ? 1 : 0;
    struct Res {
      unsigned long long wrong;
      int ok;
    };
    Res r{wrong, ok};
    std::vector<Res> res(P_);
    comm_->allgather(&r, res.data(), sizeof(Res));
    const double ms = 1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    char b[256];
    for (int q = 0; q < P_; ++q) {
      if (res[q].wrong == 0 && res[q].ok) continue;
      std::snprintf(b, sizeof(b),
                    "peer-write plane route self-test failed: rank %d received %llu wrong words of %zu-byte "
                    "messages%s",
                    q, res[q].wrong, per, res[q].ok ? "" : " (barrier failure)");
      set_error_detail(b);
      throw PeerSelfTestFailed();
    }
    std::snprintf(b, sizeof(b), "ok (%d ranks x %zu KiB, slot %d, %.2f ms)", P_, per >> 10, slot, ms);
    selfTest_ = b;
    selfTestMs_ = ms;
  }

  void barrier(hipStream_t stream) {
    SPFFT_TIMED_SCOPE("peer_barrier");
    if (__atomic_load_n(failHost_, __ATOMIC_ACQUIRE) != 0) check();
    DeviceGuard guard(device_);
    unsigned long long* const* table = table_ ? table_->data<unsigned long long*>() : nullptr;
    unsigned long long* mine = flags_ ? static_cast<unsigned long long*>(flags_->data()) : nullptr;
    if (mode_ == PeerBarrier::kChannel) {
      std::lock_guard<std::mutex> lock(channel_->m);
      hipStream_t cs = channel_->stream->get();
      gpu_check(hipEventRecord(channel_->in, stream), "hipEventRecord");
      gpu_check(hipStreamWaitEvent(cs, channel_->in, 0), "hipStreamWaitEvent");
      dev::launch_peer_barrier(table, mine, me_, P_, ++epoch_, failDev_, timeoutTicks_, xcdMask_, cs);
      gpu_check(hipEventRecord(channel_->out, cs), "hipEventRecord");
      gpu_check(hipStreamWaitEvent(stream, channel_->out, 0), "hipStreamWaitEvent");
    } else if (mode_ == PeerBarrier::kStream) {
      // rounds of this plane in issue order across streams
      if (lastStream_ != stream && epoch_ > 0)
        gpu_check(hipStreamWaitEvent(stream, orderEv_, 0), "hipStreamWaitEvent");
      dev::launch_peer_barrier(table, mine, me_, P_, ++epoch_, failDev_, timeoutTicks_, xcdMask_, stream);
      gpu_check(hipEventRecord(orderEv_, stream), "hipEventRecord");
      lastStream_ = stream;
    } else {
      gpu_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
      comm_->barrier();
    }
    readPending_[0] = readPending_[1] = false;
  }

  std::shared_ptr<Communicator> comm_;
  int device_, me_, P_;
  bool ipc_;
  unsigned int* failHost_ = nullptr;
  unsigned int* failDev_ = nullptr;
  std::unique_ptr<IpcLease> sides_[2];
  std::unique_ptr<IpcLease> flags_;
  std::vector<std::array<void*, 3>> peers_;
  std::vector<void*> opened_;
  std::unique_ptr<DeviceBuffer> table_;
  PeerBarrier mode_ = PeerBarrier::kHost;  // (in-process groups: always host)
  std::shared_ptr<PeerChannel> channel_;
  hipEvent_t orderEv_ = nullptr;  // "stream" mode: the last round, for the next stream
  hipStream_t lastStream_ = nullptr;
  unsigned long long epoch_ = 0;
  long long timeoutTicks_ = 0;
  unsigned xcdMask_ = 0;
  bool readPending_[2] = {false, false};
  std::string selfTest_ = "not run";
  double selfTestMs_ = 0;
  std::vector<std::string> devices_;  // every rank's GPU (PCI location)
};

// ------------------------------------------------- stream-ordered barriers
// The barrier rounds of a cross-process data plane (peer_sync.hip) with flag
// arrays of its own: leased from the IPC arena (uncached), mapped by every
// rank, one epoch per round. Used by the relay plane; setup and teardown are
// collective and agree on failure (every rank throws MPIError together).
struct BarrierRounds {
  int device = 0, me = 0, P = 1;
  unsigned* failHost = nullptr;
  unsigned* failDev = nullptr;
  std::unique_ptr<IpcLease> flags;
  std::vector<void*> opened;
  std::unique_ptr<DeviceBuffer> table;
  unsigned long long epoch = 0;
  long long timeoutTicks = 0;
  unsigned xcdMask = 0;

  void setup(Communicator& comm, int dev) {
    device = dev;
    me = comm.rank();
    P = comm.size();
    DeviceGuard guard(device);
    gpu_check(hipHostMalloc(reinterpret_cast<void**>(&failHost), 64, hipHostMallocMapped | hipHostMallocCoherent),
              "hipHostMalloc");
    *failHost = 0;
    gpu_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&failDev), failHost, 0), "hipHostGetDevicePointer");
    xcdMask = dev::xcd_mask(device);
    int rateKHz = 0;
    gpu_check(hipDeviceGetAttribute(&rateKHz, hipDeviceAttributeWallClockRate, device), "hipDeviceGetAttribute");
    const char* env = std::getenv("SPFFT_PEER_TIMEOUT");
    const double seconds = env && *env ? std::max(0.1, std::atof(env)) : 30.0;
    timeoutTicks = static_cast<long long>(seconds * 1e3 * std::max(rateKHz, 1));
    struct Outcome {
      int ok;
      char why[160];
    };
    Outcome res{1, {0}};
    IpcExport mine{};
    const std::size_t fbytes = static_cast<std::size_t>(dev::peer_flag_words(P)) * 8;
    try {
      flags = ipc_acquire(device, fbytes, true);
      gpu_check(hipMemset(flags->data(), 0, fbytes), "hipMemset");
      mine = flags->describe();
    } catch (const std::exception& ex) {
      res.ok = 0;
      std::snprintf(res.why, sizeof(res.why), "barrier flags: %s", ex.what());
    }
    std::vector<IpcExport> all(P);
    comm.allgather(&mine, all.data(), sizeof(IpcExport));
    std::vector<unsigned long long*> tab(P, nullptr);
    if (res.ok) {
      try {
        for (int q = 0; q < P && res.ok; ++q) {
          if (q == me) {
            tab[q] = static_cast<unsigned long long*>(flags->data());
            continue;
          }
          std::string why;
          void* p = all[q].valid ? ipc_open_checked(all[q], &why) : nullptr;
          if (!p) {
            res.ok = 0;
            std::snprintf(res.why, sizeof(res.why), "flags of rank %d: %s", q,
                          all[q].valid ? why.c_str() : "not announced");
            break;
          }
          opened.push_back(p);
          tab[q] = static_cast<unsigned long long*>(p);
        }
        if (res.ok) {
          table.reset(new DeviceBuffer(sizeof(void*) * P));
          gpu_check(hipMemcpy(table->data(), tab.data(), sizeof(void*) * P, hipMemcpyHostToDevice), "hipMemcpy");
        }
      } catch (const std::exception& ex) {
        res.ok = 0;
        std::snprintf(res.why, sizeof(res.why), "barrier flags: %s", ex.what());
      }
    }
    std::vector<Outcome> outs(P);
    comm.allgather(&res, outs.data(), sizeof(Outcome));
    for (const Outcome& o : outs)
      if (!o.ok) {
        release();
        set_error_detail(std::string("data plane barrier setup: ") + o.why);
        throw MPIError();
      }
    gpu_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    comm.barrier();  // every flag array is zeroed before the first round
  }
  // one round on `stream` (the caller keeps every round of the plane on one stream)
  void round(hipStream_t stream) {
    dev::launch_peer_barrier(table->data<unsigned long long*>(), static_cast<unsigned long long*>(flags->data()),
                             me, P, ++epoch, failDev, timeoutTicks, xcdMask, stream);
  }
  bool healthy(std::string* detail) const {
    const unsigned f = failHost ? __atomic_load_n(failHost, __ATOMIC_ACQUIRE) : 0u;
    if (f == 0) return true;
    if (detail) {
      if (f & 2u)
        *detail = "data plane barrier: aborted (host-side timeout or an earlier failure)";
      else if (f & 1u)
        *detail = "data plane barrier: a rank did not arrive within SPFFT_PEER_TIMEOUT";
      else if (f & dev::kPeerXcdMiss)
        *detail = "data plane barrier: a round's workgroups did not run on every XCD";
      else
        *detail = "data plane barrier: a peer rank gave up waiting";
    }
    return false;
  }
  void abort() {
    if (failHost) __atomic_fetch_or(failHost, 2u, __ATOMIC_ACQ_REL);
  }
  void release() {
    for (void* p : opened) ipc_close(p);
    opened.clear();
  }
  ~BarrierRounds() {
    if (process_exiting()) return;
    release();
    if (failHost && __atomic_load_n(failHost, __ATOMIC_ACQUIRE) != 0 && flags) flags->discard();
    if (failHost) (void)hipHostFree(failHost);
  }
};

// ------------------------------------------------------------ relay routing
// Ranks on distinct GPUs of one node that leave other GPUs of the node idle
// (the driver's N = 2 and N = 4 runs on an 8-GPU node): every peer message is
// split into a direct part and one part per idle GPU c, which goes p -> c -> q
// over two xGMI links that the direct route does not use. With K idle GPUs and
// N ranks each pair's message is cut into N - 1 + K shares, the direct link
// carrying N - 1 of them and each relay one, which balances the load of every
// link direction (p -> q carries N - 1 shares; p -> c and c -> q carry one
// share per peer, N - 1 in all): the exchange takes (N - 1) / (N - 1 + K) of
// the direct-only link time, 1/7 at N = 2 on 8 GPUs, 3/7 at N = 4.
//
// Two phases per exchange, each one multi-segment copy launch on the caller's
// device (kernels/relay_copy.hip):
//  1. push: the relay shares into this rank's relay buffers on the idle GPUs
//     (memory this process allocates there, from the IPC arena, and exports
//     to the peers);
//  2. pull, after a barrier: each receiver copies its direct part out of the
//     sender's send side and its relay shares out of the senders' relay
//     buffers; a second barrier frees the buffers.
// The executors register their exchanges at plan time (register_exchange:
// the ranks' transfer lists are gathered once, the split and both copy
// tables stay on the device); a registered exchange is stream-ordered: push,
// device barrier round (BarrierRounds, the peer plane's barrier kernel), pull,
// device barrier round, on one ordered stream per member set and device.
// Unregistered exchanges gather the lists per call and separate the phases
// with host barriers.
// No GPU writes into another rank's GPU memory: a receiver's L2 may hold lines
// of its own buffers from an earlier read, which a remote store would leave
// stale. Remote memory is only read (its lines are dropped by the copy
// kernel's system-scope acquire) or written on an idle GPU that runs no
// kernels.
// Every rank computes every rank's split from the gathered transfer lists,
// so the layouts agree without further messages. Shares are multiples of 16
// bytes; messages below SPFFT_RELAY_MIN_BYTES (default 1 MiB, rank 0's value)
// go direct only.
// SPFFT_RELAY: "auto" (default: through GPUs of the node that are idle, when
// the group is the node's whole job and the model says it pays), "0" off,
// "force" (relay through K = SPFFT_RELAY_VIRTUAL virtual relays on the rank's
// own GPU: exercises the layouts and phases on a one-GPU box).
class RelayDeviceComm : public DeviceComm {
public:
  RelayDeviceComm(const std::shared_ptr<Communicator>& comm, int device, const std::size_t bytes[2],
                  const std::vector<int>& relayDevices, const std::string& channelKey,
                  bool highPriority = true)
      : comm_(comm), device_(device), me_(comm->rank()), P_(comm->size()),
        K_(static_cast<int>(relayDevices.size())), relayDev_(relayDevices) {
    DeviceGuard guard(device);
    const char* e = std::getenv("SPFFT_RELAY_MIN_BYTES");
    // relay capacity per idle GPU: a rank's relayed bytes per relay are at
    // most its send side / (N - 1 + K)
    const std::size_t side = std::max(bytes[0], bytes[1]);
    relayCap_ = side / static_cast<std::size_t>(std::max(1, P_ - 1 + K_)) + 4096;
    // Every rank splits every sender's messages (exchange()), so each sender's
    // capacity and the size threshold must be known everywhere: the caps are
    // allgathered (side sizes differ per rank under COMPACT_BUFFERED) and the
    // threshold is rank 0's. Side sizes feed the self-test's message size.
    struct Setup {
      unsigned long long cap, sides[2];
      long long minBytes;
    };
    Setup su{relayCap_, {bytes[0], bytes[1]}, e && *e ? static_cast<long long>(std::atof(e)) : (1LL << 20)};
    std::vector<Setup> sus(P_);
    comm_->allgather(&su, sus.data(), sizeof(Setup));
    minBytes_ = sus[0].minBytes;
    capOf_.resize(P_);
    minSide_ = ~0ull;
    for (int q = 0; q < P_; ++q) {
      capOf_[q] = static_cast<long long>(sus[q].cap);
      minSide_ = std::min<unsigned long long>(minSide_, std::min(sus[q].sides[0], sus[q].sides[1]));
    }
    struct Announce {
      IpcExport e[2 + kMaxRelays];
    };
    struct Outcome {
      int ok;
      char why[200];
    };
    Announce mine{};
    Outcome res{1, {0}};
    if (K_ > kMaxRelays) throw InternalError();
    try {
      // the copy kernels read other GPUs' memory: peer access to every device
      int ndev = 0;
      if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
      for (int d = 0; d < ndev; ++d)
        if (d != device) (void)hipDeviceEnablePeerAccess(d, 0);
      (void)hipGetLastError();
      for (int i = 0; i < 2; ++i)
        if (bytes[i] > 0) {
          sides_[i] = ipc_acquire(device, bytes[i], false);
          mine.e[i] = sides_[i]->describe();
        }
      for (int c = 0; c < K_; ++c) {
        if (relayDev_[c] != device) {
          int can = 0;
          gpu_check(hipDeviceCanAccessPeer(&can, device, relayDev_[c]), "hipDeviceCanAccessPeer");
          if (!can) throw GPUError();
        }
        relay_.push_back(ipc_acquire(relayDev_[c], relayCap_, false));
        mine.e[2 + c] = relay_.back()->describe();
      }
    } catch (const std::exception& ex) {
      res.ok = 0;
      std::snprintf(res.why, sizeof(res.why), "relay setup: %s %s", ex.what(), error_detail().c_str());
    }
    std::vector<Announce> all(P_);
    comm_->allgather(&mine, all.data(), sizeof(Announce));
    peers_.assign(P_, std::vector<char*>(2 + K_, nullptr));
    if (res.ok) {
      try {
        for (int q = 0; q < P_ && res.ok; ++q)
          for (int i = 0; i < 2 + K_ && res.ok; ++i) {
            if (q == me_) {
              peers_[q][i] = static_cast<char*>(i < 2 ? (sides_[i] ? sides_[i]->data() : nullptr)
                                                      : relay_[i - 2]->data());
              continue;
            }
            if (!all[q].e[i].valid) continue;
            std::string why;
            void* p = ipc_open_checked(all[q].e[i], &why);
            if (!p) {
              res.ok = 0;
              std::snprintf(res.why, sizeof(res.why), "rank %d <- rank %d: %s", me_, q, why.c_str());
              break;
            }
            opened_.push_back(p);
            peers_[q][i] = static_cast<char*>(p);
          }
      } catch (const std::exception& ex) {
        res.ok = 0;
        std::snprintf(res.why, sizeof(res.why), "hipIpcOpenMemHandle: %s %s", ex.what(), error_detail().c_str());
      }
    }
    std::vector<Outcome> outs(P_);
    comm_->allgather(&res, outs.data(), sizeof(Outcome));
    for (const Outcome& o : outs) {
      if (o.ok) continue;
      for (void* p : opened_) ipc_close(p);
      opened_.clear();
      set_error_detail(std::string("relay data plane: ") + o.why);
      throw MPIError();
    }
    gpu_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    // device barrier rounds and the plane's stream (registered exchanges); a
    // failed setup (agreed by every rank) unmaps the peers' buffers before the
    // constructor unwinds
    try {
      bar_.setup(*comm_, device);
    } catch (...) {
      for (void* p : opened_) ipc_close(p);
      opened_.clear();
      throw;
    }
    // one ordered stream per member set and device, shared by every relay
    // plane of the process: the barrier rounds of all its grids run in host
    // issue order, the order every rank issues them in (transforms are
    // collective), whatever hardware queue the stream lands on
    channel_ = acquire_peer_channel(channelKey, device, highPriority);
    gpu_check(hipEventCreateWithFlags(&evIn_, hipEventDisableTiming), "hipEventCreateWithFlags");
    gpu_check(hipEventCreateWithFlags(&evOut_, hipEventDisableTiming), "hipEventCreateWithFlags");
    // the per-exchange host collectives (one allgather, two barriers) through
    // shared memory when every rank maps the segment, else through comm
    shmPayload_ = sizeof(Transfer) * static_cast<std::size_t>(2 * P_ + 1);
    shm_ = ShmGroup::create(*comm_, shmPayload_, comm_timeout_seconds());
    devices_ = group_devices(*comm_, device);
    for (int c : relayDev_) devices_.push_back(pci_string(pci_of(c)));
    comm_->barrier();
    const auto t0 = std::chrono::steady_clock::now();
    self_test();
    selfTestMs_ = 1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }

  // Collective. One exchange of a known pattern through every route (direct
  // parts and relay shares) before the plane carries data; a wrong byte on any
  // rank raises MPIError on every rank, and DeviceComm::create falls back to
  // the RCCL plane. (The routes cross GPUs whose caches the one-GPU test box
  // cannot exercise; a plane that does not deliver must not be used.)
  void self_test() {
    DeviceGuard guard(device_);
    // the same message size on every rank (the smallest side of the group), so
    // every rank makes the same collective calls with matching counts
    long long per = static_cast<long long>(minSide_ / static_cast<unsigned long long>(P_)) / 64 * 64;
    per = std::min<long long>(per, 2LL << 20);
    int ok = 1;
    if (per >= 64) {
      const int words = static_cast<int>(per / 8);
      std::vector<unsigned long long> pattern(static_cast<std::size_t>(words) * P_);
      auto word = [](int from, int to, int i) {
        return (static_cast<unsigned long long>(from) << 48) ^ (static_cast<unsigned long long>(to) << 32) ^
               static_cast<unsigned long long>(i) * 2654435761ull;
      };
      for (int q = 0; q < P_; ++q)
        for (int i = 0; i < words; ++i) pattern[static_cast<std::size_t>(q) * words + i] = word(me_, q, i);
      // fault injection RELAY_SELFTEST (testing library)
      if (SPFFT_FAULT(RELAY_SELFTEST) == 1 && me_ == P_ - 1 && P_ > 1) pattern[static_cast<std::size_t>((me_ + 1) % P_) * words] ^= 1;
      void* send = sides_[0]->data();
      void* recv = sides_[1]->data();
      gpu_check(hipMemcpy(send, pattern.data(), pattern.size() * 8, hipMemcpyHostToDevice), "hipMemcpy");
      gpu_check(hipMemset(recv, 0, pattern.size() * 8), "hipMemset");
      std::vector<std::int64_t> cnt(P_, per), dsp(P_);
      for (int q = 0; q < P_; ++q) dsp[q] = static_cast<std::int64_t>(q) * per;
      std::vector<Transfer> xs;
      append_alltoallv(xs, me_, P_, cnt.data(), dsp.data(), cnt.data(), dsp.data());
      const long long saved = minBytes_;
      minBytes_ = 0;  // every route, whatever the production threshold
      // the registered path the executors use: device barriers, plane stream
      const std::size_t before = reg_.size();
      const int id = register_exchange(0, xs);
      minBytes_ = saved;
      exchange_registered(id, nullptr, nullptr);
      gpu_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
      if (reg_.size() > before) reg_.pop_back();  // (its split ignored the threshold)
      std::vector<unsigned long long> got(pattern.size());
      gpu_check(hipMemcpy(got.data(), recv, got.size() * 8, hipMemcpyDeviceToHost), "hipMemcpy");
      for (int q = 0; q < P_ && ok; ++q)
        for (int i = 0; i < words; ++i)
          if (got[static_cast<std::size_t>(q) * words + i] != word(q, me_, i)) {
            ok = 0;
            break;
          }
    }
    std::vector<int> oks(P_);
    comm_->allgather(&ok, oks.data(), sizeof(int));
    for (int q = 0; q < P_; ++q)
      if (!oks[q]) {
        for (void* p : opened_) ipc_close(p);
        opened_.clear();
        set_error_detail("relay data plane: self-test exchange delivered wrong data to rank " + std::to_string(q));
        throw MPIError();
      }
  }

  ~RelayDeviceComm() override {
    if (process_exiting()) return;
    try {
      DeviceGuard guard(device_);
      // the last registered exchange has finished before its buffers go
      if (channel_) (void)hipStreamSynchronize(channel_->stream->get());
      if (evIn_) (void)hipEventDestroy(evIn_);
      if (evOut_) (void)hipEventDestroy(evOut_);
      for (void* p : opened_) ipc_close(p);
    } catch (...) {
    }
  }

  // Split of every peer message (from every rank's transfer list; `all` holds
  // W entries per rank, unused ones of kind -1) into the direct part and one
  // share per relay, and this rank's copy segments: phase 1 (own block; relay
  // shares into this rank's relay buffers) and phase 2 (direct parts out of the
  // senders' send sides, relay shares out of the senders' relay buffers). A list
  // may hold several messages per ordered pair (pipelined steps carry one
  // all-to-all per plane chunk): the m-th send p -> q pairs with the m-th
  // receive q <- p (NCCL's matching rule).
  void build_segs(const char* s, char* r, int sendSlot, const std::vector<Transfer>& xs,
                  const std::vector<Transfer>& all, int W, std::vector<dev::CopySeg>& push,
                  std::vector<dev::CopySeg>& pull) const {
    struct Msg {
      int p, q;
      long long so, ro, nb, base, roff;
    };
    std::vector<Msg> msgs;
    std::map<std::tuple<int, int, int>, std::size_t> byKey;  // (p, q, m) -> message
    std::vector<int> nSend(P_ * P_, 0), nRecv(P_ * P_, 0);
    for (int p = 0; p < P_; ++p)
      for (int i = 0; i < W; ++i) {
        const Transfer& t = all[static_cast<std::size_t>(p) * W + i];
        if (t.kind != Transfer::kSend || t.peer < 0 || t.peer >= P_) continue;
        const int m = nSend[p * P_ + t.peer]++;
        byKey[std::make_tuple(p, t.peer, m)] = msgs.size();
        msgs.push_back(Msg{p, t.peer, t.offset, -1, t.bytes, 0, 0});
      }
    for (int q = 0; q < P_; ++q)
      for (int i = 0; i < W; ++i) {
        const Transfer& t = all[static_cast<std::size_t>(q) * W + i];
        if (t.kind != Transfer::kRecv || t.peer < 0 || t.peer >= P_) continue;
        const int m = nRecv[t.peer * P_ + q]++;
        auto it = byKey.find(std::make_tuple(t.peer, q, m));
        if (it == byKey.end() || msgs[it->second].nb != t.bytes) mismatch();
        msgs[it->second].ro = t.offset;
      }
    if (nSend != nRecv) mismatch();
    // shares: base per relay (16-byte multiple), the direct part the rest; a
    // sender's relay buffer holds its shares in message order
    std::vector<long long> used(P_, 0);
    for (Msg& g : msgs) {
      long long b = 0;
      if (g.q != g.p && K_ > 0 && g.nb >= minBytes_) b = (g.nb / (P_ - 1 + K_)) / 16 * 16;
      if (used[g.p] + b > capOf_[g.p]) b = 0;  // sender p's relay buffers
      g.base = b;
      g.roff = used[g.p];
      used[g.p] += b;
    }
    auto add = [](std::vector<dev::CopySeg>& v, const char* src, char* dst, long long bytes) {
      if (bytes > 0) v.push_back(dev::CopySeg{src, dst, static_cast<unsigned long long>(bytes), 0});
    };
    push.clear();
    pull.clear();
    for (const Transfer& t : xs)
      if (t.kind == Transfer::kLocal) add(push, s + t.offset, r + t.dstOffset, t.bytes);
    for (const Msg& g : msgs) {
      if (g.p == g.q || g.nb == 0) continue;
      const long long direct = g.nb - K_ * g.base;
      if (g.p == me_)
        for (int c = 0; c < K_ && g.base > 0; ++c)
          add(push, s + g.so + direct + c * g.base, peers_[me_][2 + c] + g.roff, g.base);
      if (g.q == me_) {
        add(pull, peers_[g.p][sendSlot] + g.so, r + g.ro, direct);
        for (int c = 0; c < K_ && g.base > 0; ++c)
          add(pull, peers_[g.p][2 + c] + g.roff, r + g.ro + direct + c * g.base, g.base);
      }
    }
    auto number = [](std::vector<dev::CopySeg>& v) {
      long long chunks = 0;
      for (dev::CopySeg& g : v) {
        g.firstChunk = chunks;
        chunks += (static_cast<long long>(g.bytes) + dev::kCopyChunk - 1) / dev::kCopyChunk;
      }
    };
    number(push);
    number(pull);
  }

  // every rank's transfer list, padded to the longest (W entries per rank,
  // returned in *W)
  std::vector<Transfer> gather_lists(const std::vector<Transfer>& xs, bool host, int* W) {
    const int mine = static_cast<int>(xs.size());
    std::vector<int> sizes(P_);
    if (host)
      host_allgather(&mine, sizes.data(), sizeof(int));
    else
      comm_->allgather(&mine, sizes.data(), sizeof(int));
    *W = std::max(1, *std::max_element(sizes.begin(), sizes.end()));
    std::vector<Transfer> wire(*W, Transfer{-1, 0, 0, 0, 0});
    std::copy(xs.begin(), xs.end(), wire.begin());
    std::vector<Transfer> all(static_cast<std::size_t>(*W) * P_);
    if (host)
      host_allgather(wire.data(), all.data(), sizeof(Transfer) * *W);
    else
      comm_->allgather(wire.data(), all.data(), sizeof(Transfer) * *W);
    return all;
  }

  int slot_of(const void* p) const { return p == local_buffer(0) ? 0 : (p == local_buffer(1) ? 1 : -1); }

  // Unregistered exchange (host-synchronous): the lists are gathered per call,
  // the phases are separated by host barriers.
  void exchange(const void* send, void* recv, const std::vector<Transfer>& xs, hipStream_t stream,
                const ExchangeSync* sync) override {
    SPFFT_TIMED_SCOPE("relay_exchange");
    DeviceGuard guard(device_);
    const int recvSlot = slot_of(recv);
    const int sendSlot = 1 - recvSlot;
    // the grid's exchange sides only
    if (recvSlot < 0 || send != local_buffer(sendSlot)) throw InternalError();
    check();
    sync_begin(sync, stream);
    // (the host collective overlaps the GPU work still queued ahead of the
    // exchange; the stream is synchronised before the barrier that lets peers
    // read this rank's send side)
    int W = 0;
    const std::vector<Transfer> all = gather_lists(xs, true, &W);
    std::vector<dev::CopySeg> push, pull;
    build_segs(static_cast<const char*>(send), static_cast<char*>(recv), sendSlot, xs, all, W, push, pull);
    run_segs(push, stream);
    gpu_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    host_barrier();
    if (!pull.empty()) {
      run_segs(pull, stream);
      gpu_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    }
    host_barrier();  // send sides and relay buffers are free again
    sync_end(sync, stream);
  }

  // Registered exchanges (the executors' plans): the split and both segment
  // tables are computed once, collectively, at plan time and kept on the
  // device; an exchange is then four launches on the plane's stream and no
  // host round trip: push, barrier round, pull, barrier round (the senders'
  // send sides and relay buffers are free again).
  int register_exchange(int sendSlot, const std::vector<Transfer>& xs) override {
    DeviceGuard guard(device_);
    int W = 0;
    const std::vector<Transfer> all = gather_lists(xs, false, &W);
    // the same exchange registered again (another transform of the grid with
    // the same plan): every rank sees the same gathered lists, so every rank
    // reuses the same entry
    for (std::size_t i = 0; i < reg_.size(); ++i)
      if (reg_[i].sendSlot == sendSlot && same_lists(reg_[i].lists, all)) return static_cast<int>(i);
    std::vector<dev::CopySeg> push, pull;
    const char* s = static_cast<const char*>(local_buffer(sendSlot));
    char* r = static_cast<char*>(local_buffer(1 - sendSlot));
    if (!xs.empty() && (!s || !r)) throw InternalError();
    build_segs(s, r, sendSlot, xs, all, W, push, pull);
    Registered g;
    g.sendSlot = sendSlot;
    g.lists = all;
    auto up = [](std::unique_ptr<DeviceBuffer>& b, const std::vector<dev::CopySeg>& v) {
      if (v.empty()) return;
      b.reset(new DeviceBuffer(v.size() * sizeof(dev::CopySeg)));
      gpu_check(hipMemcpy(b->data(), v.data(), v.size() * sizeof(dev::CopySeg), hipMemcpyHostToDevice), "hipMemcpy");
    };
    up(g.push, push);
    up(g.pull, pull);
    g.nPush = static_cast<int>(push.size());
    g.nPull = static_cast<int>(pull.size());
    g.chPush = push.empty() ? 0 : push.back().firstChunk + (static_cast<long long>(push.back().bytes) + dev::kCopyChunk - 1) / dev::kCopyChunk;
    g.chPull = pull.empty() ? 0 : pull.back().firstChunk + (static_cast<long long>(pull.back().bytes) + dev::kCopyChunk - 1) / dev::kCopyChunk;
    reg_.push_back(std::move(g));
    return static_cast<int>(reg_.size()) - 1;
  }

  void exchange_registered(int id, hipStream_t stream, const ExchangeSync* sync) override {
    SPFFT_TIMED_SCOPE("relay_exchange");
    DeviceGuard guard(device_);
    check();
    const Registered& g = reg_.at(static_cast<std::size_t>(id));
    std::lock_guard<std::mutex> lock(channel_->m);
    hipStream_t cs = channel_->stream->get();
    if (!sync) {
      gpu_check(hipEventRecord(evIn_, stream), "hipEventRecord");
      gpu_check(hipStreamWaitEvent(cs, evIn_, 0), "hipStreamWaitEvent");
    }
    sync_begin(sync, cs);
    if (g.nPush) dev::launch_multi_copy(g.push->data<dev::CopySeg>(), g.nPush, g.chPush, cs);
    bar_.round(cs);
    if (g.nPull) dev::launch_multi_copy(g.pull->data<dev::CopySeg>(), g.nPull, g.chPull, cs);
    bar_.round(cs);
    sync_end(sync, cs);
    if (!sync) {
      gpu_check(hipEventRecord(evOut_, cs), "hipEventRecord");
      gpu_check(hipStreamWaitEvent(stream, evOut_, 0), "hipStreamWaitEvent");
    }
  }
  hipStream_t channel_stream() const override { return channel_ ? channel_->stream->get() : nullptr; }
  void check() override {
    std::string d;
    if (!bar_.healthy(&d)) {
      set_error_detail(d);
      throw MPIError();
    }
  }
  bool healthy(std::string* detail) override { return bar_.healthy(detail); }
  void abort() override { bar_.abort(); }

  int plane_rank() const override { return me_; }
  int plane_size() const override { return P_; }
  bool host_synchronous() const override { return false; }
  int max_pipeline_steps() const override { return 0; }
  void* local_buffer(int slot) const override {
    if (slot < 0 || slot > 1 || !sides_[slot]) return nullptr;
    return sides_[slot]->data();
  }
  const char* kind() const override { return "relay"; }
  std::string describe() const override {
    std::string d = "relay (" + std::to_string(P_) + " ranks, " + std::to_string(K_) + " relay GPU(s):";
    for (int c : relayDev_) d += " " + std::to_string(c);
    return d + (shm_ ? "; host sync: shared memory)" : "; host sync: communicator)");
  }
  int relay_count() const override { return K_; }
  std::string info_json() const override {
    char b[512];
    std::snprintf(b, sizeof(b),
                  "{\"kind\": \"relay\", \"ranks\": %d, \"relay_gpus\": %d, \"self_test\": \"ok\", "
                  "\"self_test_ms\": %.3f, \"devices\": %s}",
                  P_, K_, selfTestMs_, json_distinct(devices_).c_str());
    return b;
  }

private:
  static constexpr int kMaxRelays = 8;
  [[noreturn]] void mismatch() const {
    set_error_detail("relay exchange: transfer lists of the ranks do not match");
    throw MPIError();
  }
  void host_barrier() {
    if (shm_)
      shm_->barrier();
    else
      comm_->barrier();
  }
  void host_allgather(const void* send, void* recv, std::size_t bytes) {
    if (shm_ && bytes <= shmPayload_)
      shm_->allgather(send, recv, bytes);
    else
      comm_->allgather(send, recv, bytes);
  }
  // one host-built segment table: in the kernel arguments when it fits, else
  // through the staging buffer (host-synchronous path only)
  void run_segs(const std::vector<dev::CopySeg>& segs, hipStream_t stream) {
    if (segs.empty()) return;
    const long long chunks = segs.back().firstChunk +
                             (static_cast<long long>(segs.back().bytes) + dev::kCopyChunk - 1) / dev::kCopyChunk;
    if (segs.size() <= static_cast<std::size_t>(dev::kInlineSegs)) {
      std::copy(segs.begin(), segs.end(), inlineSegs_.s);
      dev::launch_multi_copy_inline(inlineSegs_, static_cast<int>(segs.size()), chunks, stream);
      return;
    }
    if (!segsDev_ || segsDev_->bytes() < segs.size() * sizeof(dev::CopySeg))
      segsDev_.reset(new DeviceBuffer(segs.size() * sizeof(dev::CopySeg)));
    gpu_check(hipMemcpyAsync(segsDev_->data(), segs.data(), segs.size() * sizeof(dev::CopySeg),
                             hipMemcpyHostToDevice, stream),
              "hipMemcpyAsync");
    dev::launch_multi_copy(segsDev_->data<dev::CopySeg>(), static_cast<int>(segs.size()), chunks, stream);
    gpu_check(hipStreamSynchronize(stream), "hipStreamSynchronize");  // the staging buffer is reused
  }

  struct Registered {
    std::unique_ptr<DeviceBuffer> push, pull;
    int nPush = 0, nPull = 0;
    long long chPush = 0, chPull = 0;
    int sendSlot = 0;
    std::vector<Transfer> lists;  // every rank's list as gathered (identity of the entry)
  };
  static bool same_lists(const std::vector<Transfer>& a, const std::vector<Transfer>& b) {
    if (a.size() != b.size()) return false;
    for (std::size_t i = 0; i < a.size(); ++i)
      if (a[i].kind != b[i].kind || a[i].peer != b[i].peer || a[i].offset != b[i].offset ||
          a[i].dstOffset != b[i].dstOffset || a[i].bytes != b[i].bytes)
        return false;
    return true;
  }

  std::shared_ptr<Communicator> comm_;
  int device_, me_, P_, K_;
  std::vector<int> relayDev_;
  long long minBytes_ = 0;
  std::size_t relayCap_ = 0;
  std::vector<long long> capOf_;     // every rank's relay capacity (per relay buffer)
  std::vector<std::string> devices_;  // ranks' GPUs and relay GPUs (PCI locations)
  double selfTestMs_ = 0;
  unsigned long long minSide_ = 0;   // smallest exchange side of the group
  std::unique_ptr<IpcLease> sides_[2];
  std::vector<std::unique_ptr<IpcLease>> relay_;
  std::vector<std::vector<char*>> peers_;  // [rank][0: stick side, 1: slab side, 2 + c: relay c]
  std::vector<void*> opened_;
  std::unique_ptr<DeviceBuffer> segsDev_;
  std::unique_ptr<ShmGroup> shm_;
  std::size_t shmPayload_ = 0;  // largest allgather the shared segment carries
  dev::SegPack inlineSegs_{};
  std::vector<Registered> reg_;       // registered exchanges (plan time)
  BarrierRounds bar_;                 // device barrier rounds of the registered path
  std::shared_ptr<PeerChannel> channel_;  // ordered stream of the registered exchanges
  hipEvent_t evIn_ = nullptr, evOut_ = nullptr;
};

struct NodeInfo {
  std::uint64_t host;
  long long pid;
  int domain, bus, device, ordinal;
  unsigned long long channelDomain;  // Communicator::channel_domain
  int prefer;  // SPFFT_GPU_EXCHANGE: 0 auto, 1 rccl, 2 peer (ipc)
  int fault;   // fault injection RCCL_INIT (rank 0's value is used everywhere)
  int relay;   // SPFFT_RELAY: 0 auto, 1 off, 2 force (virtual relays)
  int relayVirtual;  // SPFFT_RELAY_VIRTUAL
  unsigned long long stickBytes;  // this rank's stick side (per-peer message estimate)
  int localSize;  // the launcher's ranks on this node (0 unknown)
};

// SPFFT_RELAY=auto: whether relaying through K idle GPUs beats the direct
// links for per-peer messages of m bytes among n ranks, at the measured link
// rate (measure_link_GBps; 70 GB/s if unknown). Direct: m at one link's rate;
// relay: two stream-ordered hops (push, pull) of (n - 1) / (n - 1 + K) of m
// each plus two barrier rounds (~10 us each). Relay is chosen when it models
// at least 20% faster: N = 2 at 256^3 fp64 (52 MB per peer, K = 6: 750 vs
// 235 us at 70 GB/s) relays; small problems stay on RCCL.
bool relay_pays(double m, int n, int k, double linkGBps) {
  const double bytesPerUs = (linkGBps > 0 ? linkGBps : 70.0) * 1e3;
  constexpr double kBarrierUs = 20.0;
  const double direct = m / bytesPerUs;
  const double relay = 2.0 * m * (n - 1) / (n - 1 + k) / bytesPerUs + kBarrierUs;
  return relay < 0.8 * direct;
}

double measure_link_GBps(Communicator& comm, int device);

// The link rate of a member set's node (measured once per process and key).
double node_link_rate(Communicator& comm, int device, const std::string& key) {
  static std::mutex m;
  static std::map<std::string, double> cache;
  {
    std::lock_guard<std::mutex> lock(m);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  const double r = measure_link_GBps(comm, device);
  std::lock_guard<std::mutex> lock(m);
  cache[key] = r;
  return r;
}

int env_relay() {
  const char* e = std::getenv("SPFFT_RELAY");
  const std::string v = e ? e : "";
  return v == "0" || v == "off" ? 1 : (v == "force" ? 2 : 0);
}

// Collective (ranks of one node on distinct GPUs). The usable one-way rate of
// one xGMI link: every rank copies 8 MiB into its right neighbour's memory (an
// IPC-mapped arena block), all links of the ring at once, best of 3 timed
// copies; the median over ranks in GB/s (0 if the probe could not run). It
// replaces the link-rate assumption of the relay decision and is reported in
// the plane info (bench.py's model).
double measure_link_GBps(Communicator& comm, int device) {
  constexpr std::size_t kBytes = std::size_t(8) << 20;
  const int P = comm.size(), me = comm.rank();
  DeviceGuard guard(device);
  int ok = 1;
  std::unique_ptr<IpcLease> target;
  std::unique_ptr<DeviceBuffer> src;
  IpcExport mine{};
  try {
    target = ipc_acquire(device, kBytes, false);
    src.reset(new DeviceBuffer(kBytes));
    gpu_check(hipMemset(src->data(), 1, kBytes), "hipMemset");
    mine = target->describe();
  } catch (const std::exception&) {
    ok = 0;
  }
  std::vector<IpcExport> all(P);
  comm.allgather(&mine, all.data(), sizeof(IpcExport));
  void* dst = nullptr;
  const int right = (me + 1) % P;
  if (ok && all[right].valid) {
    try {
      std::string why;
      dst = ipc_open_checked(all[right], &why);
      const int ndev = [] {
        int n = 0;
        return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
      }();
      for (int d = 0; d < ndev; ++d)
        if (d != device) (void)hipDeviceEnablePeerAccess(d, 0);
      (void)hipGetLastError();
    } catch (const std::exception&) {
      dst = nullptr;
    }
  }
  double best = 0;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  comm.barrier();
  if (dst && hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess) {
    GpuStream st(false);
    for (int it = 0; it < 4; ++it) {
      (void)hipEventRecord(e0, st.get());
      (void)hipMemcpyAsync(dst, src->data(), kBytes, hipMemcpyDeviceToDevice, st.get());
      (void)hipEventRecord(e1, st.get());
      float ms = 0;
      if (hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&ms, e0, e1) == hipSuccess && it > 0 &&
          ms > 0)
        best = std::max(best, kBytes / (ms * 1e-3) / 1e9);
    }
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  (void)hipGetLastError();
  comm.barrier();  // every copy into a peer's block is done before the blocks go
  if (dst) ipc_close(dst);
  std::vector<double> rates(P);
  comm.allgather(&best, rates.data(), sizeof(double));
  std::sort(rates.begin(), rates.end());
  return rates[P / 2];
}

// Ranks of this job on this node according to the launcher (torchrun,
// Open MPI, MPICH/Hydra), 0 if unknown.
int launcher_local_size() {
  for (const char* v : {"LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS"}) {
    const char* e = std::getenv(v);
    if (e && *e) return std::atoi(e);
  }
  return 0;
}

// Collective. The GPUs of this node that no rank of the group runs on and
// that every rank can see, as this process's ordinals, in rank 0's order
// (at most kMaxRelay).
std::vector<int> idle_devices(Communicator& comm, const std::vector<PciId>& used) {
  constexpr int kMaxDev = 16, kMaxRelay = 8;
  struct Visible {
    int n;
    PciId id[kMaxDev];
  };
  Visible mine{};
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
  (void)hipGetLastError();
  mine.n = std::min(count, kMaxDev);
  for (int d = 0; d < mine.n; ++d) mine.id[d] = pci_of(d);
  const int P = comm.size();
  std::vector<Visible> all(P);
  comm.allgather(&mine, all.data(), sizeof(Visible));
  // candidates: rank 0's devices no rank uses and nothing else uses either
  // (rank 0 decides from the driver's counters; the list is agreed below)
  std::vector<PciId> cand;
  std::vector<int> idle(all[0].n, 0);
  if (comm.rank() == 0)
    for (int d = 0; d < all[0].n; ++d) idle[d] = relay_candidate_idle(all[0].id[d].domain, all[0].id[d].bus, all[0].id[d].device) ? 1 : 0;
  std::vector<int> idleAll(static_cast<std::size_t>(all[0].n) * P);
  if (all[0].n > 0) comm.allgather(idle.data(), idleAll.data(), sizeof(int) * all[0].n);
  for (int d = 0; d < all[0].n; ++d) {
    bool inUse = false;
    for (const PciId& u : used) inUse = inUse || u == all[0].id[d];
    if (!inUse && idleAll[d] && static_cast<int>(cand.size()) < kMaxRelay) cand.push_back(all[0].id[d]);
  }
  // keep those every rank sees; this process's ordinal of each
  std::vector<int> out;
  for (const PciId& c : cand) {
    int mineOrd = -1;
    bool everyone = true;
    for (int q = 0; q < P; ++q) {
      int ord = -1;
      for (int d = 0; d < all[q].n; ++d)
        if (all[q].id[d] == c) ord = d;
      everyone = everyone && ord >= 0;
      if (q == comm.rank()) mineOrd = ord;
    }
    if (everyone) out.push_back(mineOrd);
  }
  return out;
}

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

int env_fault() { return SPFFT_FAULT(RCCL_INIT); }

bool share_channels() {
  const char* e = std::getenv("SPFFT_RCCL_SHARE");
  return !(e && *e == '0');
}

// The process's channel for `key`, created collectively if any rank lacks a
// live one (the reuse decision is allgathered, so every rank either reuses or
// takes part in the new communicator's initialisation).
std::shared_ptr<NcclChannel> acquire_channel(Communicator* group, const std::string& key, int device,
                                             int rank, int size, bool selfOnly, int fault,
                                             bool highPriority = true) {
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
  ch->highPriority = highPriority;
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

// Bytes of device memory in use on the GPU at a PCI location, from the amdgpu
// driver's sysfs (no HIP context on that GPU); -1 if unknown. SPFFT_SYSFS_ROOT
// (tests) replaces /sys.
long long vram_used_bytes_at(int domain, int bus, int device) {
  const char* root = std::getenv("SPFFT_SYSFS_ROOT");
  char path[256];
  std::snprintf(path, sizeof(path), "%s/bus/pci/devices/%04x:%02x:%02x.0/mem_info_vram_used",
                root && *root ? root : "/sys", domain & 0xffff, bus & 0xff, device & 0xff);
  std::FILE* f = std::fopen(path, "r");
  if (!f) return -1;
  long long v = -1;
  if (std::fscanf(f, "%lld", &v) != 1) v = -1;
  std::fclose(f);
  return v;
}

// A relay candidate must be idle: nothing holds memory on it beyond the
// driver's own reservation (another job, or another communicator of this job,
// would otherwise get this job's buffers and link traffic). Unknown usage
// counts as busy. Measured on the MI355X hosts of the round-6 pool: idle GPUs
// report 284 MiB (297766912 B) in use, GPUs with a torch process 1.5 GB and
// more (profiles/r6/relay/vram_used.txt).
constexpr long long kIdleVramBytes = 512ll << 20;
bool relay_candidate_idle(int domain, int bus, int device) {
  const long long used = vram_used_bytes_at(domain, bus, device);
  return used >= 0 && used <= kIdleVramBytes;
}

int DeviceComm::rccl_channels_created() { return gChannelsCreated.load(); }

void DeviceComm::exchange_registered(int, hipStream_t, const ExchangeSync*) { throw InternalError(); }

std::string DeviceComm::info() const {
  std::string j = info_json();
  if (linkGBps_ > 0 && !j.empty() && j.back() == '}') {
    char b[96];
    std::snprintf(b, sizeof(b), ", \"link_GBps_measured\": %.1f, \"link_kind\": \"%s\"}", linkGBps_,
                  linkKind_);
    j.pop_back();
    j += b;
  }
  if (channelPriority_ && !j.empty() && j.back() == '}') {
    j.pop_back();
    j += std::string(", \"channel_priority\": \"") + channelPriority_ + "\"}";
  }
  return j;
}

std::unique_ptr<DeviceComm> DeviceComm::create(const std::shared_ptr<Communicator>& comm,
                                               int device, SpfftExchangeType exchange,
                                               void* const buffers[2], const std::size_t bytes[2]) {
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
    if (unbuffered) return std::unique_ptr<DeviceComm>(new PeerDeviceComm(comm, device, buffers, bytes, false, std::string()));
    return std::unique_ptr<DeviceComm>(new LoopbackDeviceComm(comm));
  }
  // SPFFT_RCCL_VIRTUAL_HOSTS=1 (rehearsals on a box with fewer GPUs than
  // ranks): RCCL refuses two ranks of one host on one device ("Duplicate
  // GPU"), so every rank claims a host of its own (NCCL_HOSTID) and the ranks
  // talk over RCCL's socket transport on loopback. The exchanges then run the
  // multi-rank RcclDeviceComm path that ships to 8 GPUs: peer ids, staggered
  // send/receive order, grouped calls, channel stream hand-offs.
  const char* vh = std::getenv("SPFFT_RCCL_VIRTUAL_HOSTS");
  const bool virtualHosts = vh && *vh == '1';
  // Rehearsal mode only. The host id is set once per process, before this
  // process's first RCCL initialisation, and is keyed on the process (not on
  // its rank in whichever communicator comes first), so every communicator
  // the process joins later sees the same host.
  if (virtualHosts) {
    static std::once_flag once;
    std::call_once(once, [] {
      const std::string id = "spfft-virtual-host-" + std::to_string(static_cast<long long>(getpid()));
      setenv("NCCL_HOSTID", id.c_str(), 1);
      setenv("NCCL_IB_DISABLE", "1", 0);
      setenv("NCCL_SOCKET_IFNAME", "lo", 0);
    });
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
  mine.channelDomain = comm->channel_domain();
  mine.prefer = virtualHosts ? 1 : prefLocal;
  mine.fault = env_fault();
  mine.relay = env_relay();
  mine.stickBytes = bytes[0];
  mine.localSize = launcher_local_size();
  {
    const char* rv = std::getenv("SPFFT_RELAY_VIRTUAL");
    mine.relayVirtual = rv && *rv ? std::max(1, std::min(8, std::atoi(rv))) : 2;
  }
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
    char m[128];
    std::snprintf(m, sizeof(m), "/%llx:%lld:%d.%d.%d:%llx", static_cast<unsigned long long>(all[q].host),
                  all[q].pid, all[q].domain, all[q].bus, all[q].ordinal, all[q].channelDomain);
    key += m;
  }
  // every rank decides from rank 0's settings (environments may differ)
  const int prefer = all[0].prefer;
  const int fault = all[0].fault;
  // relay routing through idle GPUs of the node (RelayDeviceComm): the buffered
  // exchanges of ranks on distinct GPUs when other GPUs are idle (SPFFT_RELAY
  // auto), or through virtual relays on the ranks' own GPUs (force, tests)
  const int relayMode = all[0].relay;
  // ranks of one node: the peer copy rate, measured (setup cost a few ms,
  // once per member set); an xGMI link between distinct GPUs, the GPU's own
  // memory when ranks share one (rehearsals; not used for plane decisions)
  const double linkGBps = oneNode && P > 1 ? node_link_rate(*comm, device, key) : 0.0;
  // Channel streams are high priority (their rounds and collectives dispatch
  // ahead of queued stage work) except when ranks share a device: with another
  // process's high-priority queue on the GPU, both processes' stage kernels ran
  // about 2x slower, for the rest of the process even after the queue's stream
  // was destroyed (2 ranks on one GPU, 256^3: 3304 vs 3930-3975 transforms/s;
  // one process alone shows no effect; profiles/r6/probe_state)
  const bool highPriority = !sharedDevice;
  auto finish = [&](std::unique_ptr<DeviceComm> dc) {
    dc->set_link_rate(linkGBps, sharedDevice ? "same-device" : "xgmi");
    dc->set_channel_priority(highPriority);
    return dc;
  };
  // auto relay only when this group is every rank of the job on the node (the
  // launcher's local size): GPUs that no rank of this group uses may belong
  // to another communicator of the job
  const int localSize = all[0].localSize;
  if (oneNode && !unbuffered && fault == 0 && prefer == 0 && relayMode != 1 &&
      (relayMode == 2 || (!sharedDevice && (localSize == 0 || localSize == P)))) {
    std::vector<int> relays;
    if (relayMode == 2) {
      relays.assign(all[0].relayVirtual, device);
    } else {
      std::vector<PciId> used;
      for (int q = 0; q < P; ++q) used.push_back(PciId{all[q].domain, all[q].bus, all[q].device});
      relays = idle_devices(*comm, used);
    }
    double perPeer = 0;
    for (int q = 0; q < P; ++q) perPeer = std::max(perPeer, static_cast<double>(all[q].stickBytes) / P);
    const bool pays = relayMode == 2 || relay_pays(perPeer, P, static_cast<int>(relays.size()),
                                                   sharedDevice ? 0.0 : linkGBps);
    if (!relays.empty() && pays) {
      try {
        return finish(std::unique_ptr<DeviceComm>(new RelayDeviceComm(comm, device, bytes, relays, "relay" + key, highPriority)));
      } catch (const MPIError&) {
        // every rank agreed on the failure (setup or self-test): the next plane
        if (comm->rank() == 0)
          std::fprintf(stderr, "spfft: %s; not relaying\n", error_detail().c_str());
      }
    }
  }
  const bool peer =
      oneNode && prefer != 1 && (unbuffered || (sharedDevice && fault == 0) || prefer == 2);
  if (peer) {
    try {
      return finish(std::unique_ptr<DeviceComm>(new PeerDeviceComm(comm, device, buffers, bytes, true, "peer" + key, highPriority)));
    } catch (const PeerSelfTestFailed&) {
      // every rank saw the failure: ranks on distinct devices move the data
      // through RCCL instead (UNBUFFERED included); ranks sharing a device
      // have no other plane (RCCL refuses them)
      if (sharedDevice || !oneNode || prefer == 2) throw;
      if (comm->rank() == 0) std::fprintf(stderr, "spfft: %s; using RCCL\n", error_detail().c_str());
    }
  }
  auto ch = acquire_channel(comm.get(), key, device, comm->rank(), P, false, fault, highPriority);
  // every rank learns whether every RCCL communicator came up
  int ok = ch->ok() ? 1 : 0;
  std::vector<int> oks(P);
  comm->allgather(&ok, oks.data(), sizeof(int));
  bool allOk = true;
  for (int v : oks) allOk = allOk && v != 0;
  if (allOk) return finish(std::unique_ptr<DeviceComm>(new RcclDeviceComm(ch)));
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
  return finish(std::unique_ptr<DeviceComm>(new PeerDeviceComm(comm, device, buffers, bytes, true, "peer" + key, highPriority)));
}

}  // namespace spfft
