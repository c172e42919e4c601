/*
 * spfft::Communicator — the control-plane / host-data-plane abstraction of
 * SpFFT-AMD (SpFFT-AMD addition; the reference hard-wires MPI, see
 * src/mpi_util/mpi_communicator_handle.hpp:43-74).
 *
 * Implementations shipped:
 *  - MPI (libspfft_amd_mpi, wraps a duplicated MPI_Comm),
 *  - callbacks (C API; used by the Python front end over torch.distributed),
 *  - an in-process "local group" of N ranks driven by N threads (tests, and
 *    P-virtual-rank runs on a single GPU).
 * The GPU data plane (RCCL over xGMI) is bootstrapped through allgather().
 */
#ifndef SPFFT_COMMUNICATOR_HPP
#define SPFFT_COMMUNICATOR_HPP

#include <cstddef>
#include <memory>
#include <vector>

#include "spfft/config.h"

namespace spfft {

/* A started host exchange: wait() completes it. The send and receive buffers
 * stay in use until then. */
class SPFFT_EXPORT ExchangeRequest {
public:
  virtual ~ExchangeRequest();
  virtual void wait() = 0;
};

/* One peer's part of an alltoallw (SpFFT-AMD): `count` blocks of `blockBytes`
 * bytes, `strideBytes` apart, starting at byte `offset` of the buffer. */
struct StridedLayout {
  std::size_t offset;
  std::size_t count;
  std::size_t blockBytes;
  std::size_t strideBytes;
};

class SPFFT_EXPORT Communicator {
public:
  virtual ~Communicator();

  virtual int rank() const = 0;
  virtual int size() const = 0;

  /* Every rank contributes `bytes` bytes; recv receives size()*bytes in rank order. */
  virtual void allgather(const void* send, void* recv, std::size_t bytes) = 0;

  /* Host-memory all-to-all with per-peer byte counts and byte displacements. */
  virtual void alltoallv(const void* send, const std::size_t* sendCounts,
                         const std::size_t* sendDispls, void* recv, const std::size_t* recvCounts,
                         const std::size_t* recvDispls) = 0;

  /* Non-blocking alltoallv (the reference's MPI_Ialltoallv exchanges,
   * src/transpose/transpose_mpi_compact_buffered_host.cpp:189,274). The count
   * and displacement arrays may be released on return. The default runs
   * alltoallv() at once and returns a completed request. */
  virtual std::unique_ptr<ExchangeRequest> ialltoallv(const void* send, const std::size_t* sendCounts,
                                                      const std::size_t* sendDispls, void* recv,
                                                      const std::size_t* recvCounts,
                                                      const std::size_t* recvDispls);

  /* All-to-all between strided layouts (one per rank on each side), with no
   * intermediate copy where the transport supports it: the MPI communicator
   * runs MPI_Alltoallw with hvector datatypes, the reference's UNBUFFERED
   * exchange (src/transpose/transpose_mpi_unbuffered_host.cpp:66-181). The
   * default packs into temporary buffers around alltoallv(). */
  virtual void alltoallw(const void* send, const StridedLayout* sendLayouts, void* recv,
                         const StridedLayout* recvLayouts);
  /* Non-blocking alltoallw (MPI_Ialltoallw); the layout arrays may be released on
   * return. The default runs alltoallw() at once. */
  virtual std::unique_ptr<ExchangeRequest> ialltoallw(const void* send,
                                                      const StridedLayout* sendLayouts,
                                                      void* recv,
                                                      const StridedLayout* recvLayouts);

  virtual void barrier();

  /* A communicator with the same members but an independent message space. */
  virtual std::shared_ptr<Communicator> duplicate() const = 0;

  /* True for the in-process local group (GPU data plane uses peer copies instead of RCCL). */
  virtual bool is_local_group() const { return false; }

  /* Ordering domain of the GPU data plane. Grids whose communicators have the
   * same members and the same domain on every rank share one RCCL communicator,
   * whose exchanges run in host call order (the order every rank issues them
   * in, transforms being collective on their communicator). MPI: the user
   * communicator the grid was built from, so grids on distinct MPI
   * communicators, which MPI_THREAD_MULTIPLE lets threads drive concurrently,
   * never share one. 0 (default) = members only. */
  virtual unsigned long long channel_domain() const { return 0; }
};

/* Creates `size` communicators forming one in-process group; element r has rank r.
 * Each must be driven by its own thread (collectives block until all arrive). */
SPFFT_EXPORT std::vector<std::shared_ptr<Communicator>> create_local_communicators(int size);

}  // namespace spfft

#endif
