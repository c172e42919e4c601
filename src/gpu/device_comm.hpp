// GPU data plane for the pencil <-> slab redistribution.
//  - RcclDeviceComm: RCCL grouped send/recv (all-to-all-v) on the process's
//    shared RCCL channel (one communicator and one ordered comm stream per
//    member set and device, handed off to and from the caller's stream by
//    events); xGMI peer links carry every peer pair concurrently. Replaces
//    MPI_Alltoall(v) on staged host buffers
//    (reference: src/transpose/transpose_mpi_compact_buffered_gpu.cpp:195-282).
//  - RcclSelfDeviceComm: in-process virtual ranks whose blocks all move through
//    RCCL (ncclSend/ncclRecv to self on a size-1 communicator per virtual rank):
//    the RCCL data path on a single GPU (SPFFT_GPU_EXCHANGE=rccl).
//  - PeerDeviceComm: zero-copy peer writes. Every rank maps the exchange
//    buffers of every other rank (IPC handles across processes, plain pointers
//    inside a local group); the producing stage kernel (z-stage backward,
//    y-stage forward) stores its output straight into the receiver's buffer
//    over xGMI, framed by stream-ordered barrier kernels. This is the
//    UNBUFFERED exchange (the reference's MPI_Alltoallw with derived datatypes,
//    src/transpose/transpose_mpi_unbuffered_gpu.cpp:174-230, without any
//    intermediate copy) and the data plane for ranks that share one GPU, where
//    RCCL refuses to run.
//  - LoopbackDeviceComm: in-process local group, device-to-device copies.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "spfft/communicator.hpp"
#include "spfft/types.h"

namespace spfft {

// Seconds a distributed call may wait for its exchange (the watched stream
// wait) before it aborts the data plane and throws MPIError.
// SPFFT_COMM_TIMEOUT, default 0 = no limit (MPI semantics: a slow peer is not
// an error).
double comm_timeout_seconds();
// Deadline of the collective RCCL initialisation: SPFFT_COMM_TIMEOUT when set
// and > 0, else 300 s (a rank that never arrives must not leave the others
// inside RCCL forever).
double comm_init_timeout_seconds();

// One point-to-point transfer of an exchange as issued to the data plane.
struct Transfer {
  enum Kind : int { kSend = 0, kRecv = 1, kLocal = 2 };
  int kind;
  int peer;                // destination (kSend), source (kRecv); the own rank for kLocal
  std::int64_t offset;     // bytes into the send buffer (kSend, kLocal source) or receive buffer (kRecv)
  std::int64_t dstOffset;  // kLocal: bytes into the receive buffer
  std::int64_t bytes;
};

// Appends the transfer list of one all-to-all-v (byte counts and
// displacements, one entry per rank) to `out`: the own block first (kLocal),
// then the peers in staggered order, k = 1..P-1: send to me+k, receive from
// me-k, so that every xGMI link carries traffic from the start. Zero-byte
// blocks are omitted. Every data plane pairs the m-th send q -> r with the m-th
// receive r <- q (NCCL's point-to-point matching rule).
void append_alltoallv(std::vector<Transfer>& out, int me, int P, const std::int64_t* sendCounts,
                      const std::int64_t* sendDispls, const std::int64_t* recvCounts,
                      const std::int64_t* recvDispls);

// Stream hand-off of an asynchronous exchange (pipelined plans): the transfers
// start after `ready` (recorded by the caller; null = no wait) and `done` is
// recorded once every block has arrived. The caller's stream does not wait.
// `begin` / `end` (optional timing events) are recorded right before the
// transfers start and after they completed, on the stream that runs them.
struct ExchangeSync {
  hipEvent_t ready;
  hipEvent_t done;
  hipEvent_t begin;
  hipEvent_t end;
};

// Whether an idle-GPU relay candidate (PCI location) is idle: the amdgpu
// driver reports at most 512 MiB of its memory in use (sysfs
// mem_info_vram_used, its own reservation is ~284 MiB on MI355X;
// SPFFT_SYSFS_ROOT replaces /sys in tests). Unknown usage counts as busy. The
// relay plane never leases memory on a busy GPU.
bool relay_candidate_idle(int domain, int bus, int device);

class DeviceComm {
public:
  // Collective. `buffers` are the grid's two exchange slots (0 = stick side,
  // 1 = slab side; base pointers of device allocations of `bytes` bytes).
  static std::unique_ptr<DeviceComm> create(const std::shared_ptr<Communicator>& comm, int device,
                                            SpfftExchangeType exchange, void* const buffers[2],
                                            const std::size_t bytes[2]);
  virtual ~DeviceComm();

  // Runs a transfer list (collective: every rank calls with its own list).
  // sync == nullptr: enqueued after the work on `stream`, and `stream` waits
  // until every block has arrived. Otherwise see ExchangeSync; data planes
  // without a stream of their own run it on `stream`.
  virtual void exchange(const void* send, void* recv, const std::vector<Transfer>& xs,
                        hipStream_t stream, const ExchangeSync* sync) = 0;
  // Collective for planes that precompute their exchanges (the relay plane):
  // every rank registers its transfer list of one exchange (sent from its side
  // `sendSlot`, received into the other side) in the same order, at plan time.
  // Returns the id for exchange_registered, or -1 (the plane does not
  // register; then the call is not collective and exchange() is used).
  virtual int register_exchange(int /*sendSlot*/, const std::vector<Transfer>& /*xs*/) { return -1; }
  // Runs a registered exchange, stream-ordered (sync as for exchange()).
  virtual void exchange_registered(int id, hipStream_t stream, const ExchangeSync* sync);
  // Byte counts / displacements, one entry per rank, as one exchange().
  void alltoallv(const void* send, const std::int64_t* sendCounts, const std::int64_t* sendDispls,
                 void* recv, const std::int64_t* recvCounts, const std::int64_t* recvDispls,
                 hipStream_t stream);
  // This rank and the number of ranks of the exchange (entries of alltoallv's arrays).
  virtual int plane_rank() const = 0;
  virtual int plane_size() const = 0;
  // true if exchange() returns only after the data moved (host-synchronous).
  virtual bool host_synchronous() const = 0;
  // The stream that carries this plane's asynchronous exchanges (the RCCL
  // channel stream shared by every grid of the process), null if none.
  virtual hipStream_t channel_stream() const { return nullptr; }

  // Peer-write data plane: stage kernels store into peer_buffer(r, slot)
  // directly. Every rank issues the same sequence of calls (transforms are
  // collective), so the host-side bookkeeping below mirrors the peers' state:
  //   prepare_write(slot): before remote stores into `slot` of the peers; a
  //     barrier round is enqueued only if some rank may still read that slot
  //     (a note_read(slot) since the last round);
  //   complete_writes(): barrier round after the remote stores, before the
  //     receivers read;
  //   note_read(slot): a local kernel reading `slot` was enqueued.
  virtual bool peer_writes() const { return false; }
  virtual void* peer_buffer(int /*rank*/, int /*slot*/) const { return nullptr; }
  virtual void prepare_write(int /*slot*/, hipStream_t /*stream*/) {}
  virtual void complete_writes(hipStream_t /*stream*/) {}
  virtual void note_read(int /*slot*/) {}
  // Exchange side `slot` (0 stick side, 1 slab side) owned by the data plane,
  // which the grid uses instead of its own allocation (the cross-process peer
  // plane leases exported memory from the IPC arena); null if the grid's own
  // buffer is used.
  virtual void* local_buffer(int /*slot*/) const { return nullptr; }
  // Most exchange steps a direction should be cut into (0: any; host-
  // synchronous planes that pay a host round trip per step want 1).
  virtual int max_pipeline_steps() const { return 0; }
  // Idle GPUs the plane relays through (RelayDeviceComm), 0 otherwise.
  virtual int relay_count() const { return 0; }
  // Throws if an asynchronous failure (e.g. a barrier timeout) was recorded.
  virtual void check() {}
  // Failure detection while the host waits on a stream that carries exchanges:
  // false (with a description) once the data plane has recorded an
  // asynchronous error (RCCL: ncclCommGetAsyncError; peer writes: a barrier
  // that timed out). Cheap enough to poll every millisecond.
  virtual bool healthy(std::string* /*detail*/) { return true; }
  // Abandons in-flight communication after a failure or a host-side timeout
  // (RCCL: ncclCommAbort; peer writes: the barrier kernels stop waiting). The
  // data plane is unusable afterwards: every later exchange throws MPIError.
  virtual void abort() {}
  virtual const char* kind() const = 0;
  // One line for SPFFT_LOG (e.g. which RCCL communicator a grid uses).
  virtual std::string describe() const { return kind(); }
  // The plane's setup facts as one JSON object: "kind", and where they apply
  // "self_test" / "self_test_ms" (route self-test at setup), "devices" (PCI
  // bus ids of every GPU the plane touches: the ranks' and any relay GPUs),
  // "link_GBps_measured" (copy probe at setup). Stable for the plane's life.
  virtual std::string info_json() const { return std::string("{\"kind\": \"") + kind() + "\"}"; }
  // info_json() plus "link_GBps_measured" when the link probe ran
  std::string info() const;
  // priority of the plane's channel streams ("high" / "normal"; DeviceComm::create)
  void set_channel_priority(bool high) { channelPriority_ = high ? "high" : "normal"; }
  void set_link_rate(double gbps, const char* kind) {
    linkGBps_ = gbps;
    linkKind_ = kind;
  }
  double link_rate() const { return linkGBps_; }
  // RCCL communicators this process has created (shared channels count once).
  static int rccl_channels_created();

private:
  double linkGBps_ = 0;  // measured peer copy rate (ranks of one node), 0 if none
  const char* linkKind_ = "xgmi";  // "xgmi" (distinct GPUs) or "same-device"
  const char* channelPriority_ = nullptr;
};

}  // namespace spfft
