// GPU data plane for the pencil <-> slab redistribution.
//  - RcclDeviceComm: RCCL grouped send/recv (all-to-all-v) enqueued on the
//    execution stream; xGMI peer links carry every peer pair concurrently.
//    Replaces MPI_Alltoall(v/w) on staged host buffers
//    (reference: src/transpose/transpose_mpi_compact_buffered_gpu.cpp:195-282).
//  - LoopbackDeviceComm: in-process local group (several virtual ranks on
//    one or more GPUs of one process) using device-to-device peer copies.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <memory>

#include "spfft/communicator.hpp"

namespace spfft {

class DeviceComm {
public:
  static std::unique_ptr<DeviceComm> create(const std::shared_ptr<Communicator>& comm, int device);
  virtual ~DeviceComm();

  // Byte counts / displacements, one entry per rank. Enqueued on `stream`;
  // the receive buffer is complete when the stream reaches this point.
  virtual void alltoallv(const void* send, const std::int64_t* sendCounts,
                         const std::int64_t* sendDispls, void* recv,
                         const std::int64_t* recvCounts, const std::int64_t* recvDispls,
                         hipStream_t stream) = 0;
  // true if alltoallv() returns only after the data moved (host-synchronous).
  virtual bool host_synchronous() const = 0;
};

}  // namespace spfft
