/*
 * spfft::GridFloat — owner of the (host and HBM) buffers and of the communicator
 * that all Transforms created from it share.
 *
 * API-compatible with SpFFT's Grid (reference: include/spfft/grid.hpp:65-198):
 *  - local and distributed constructors,
 *  - copy = deep copy (new buffers, duplicated communicator), move = cheap,
 *  - create_transform() plus the nine getters.
 * Additional (SpFFT-AMD): a distributed constructor that takes a
 * spfft::Communicator instead of an MPI_Comm (used by the torch.distributed
 * front end and by in-process multi-rank tests).
 */
#ifndef SPFFT_GRID_FLOAT_HPP
#define SPFFT_GRID_FLOAT_HPP

#include <memory>

#include "spfft/communicator.hpp"
#include "spfft/config.h"
#include "spfft/transform_float.hpp"
#include "spfft/types.h"

#ifdef SPFFT_AMD_MPI_API
#include <mpi.h>
#endif

namespace spfft {

template <typename T>
class GridImpl;

class SPFFT_EXPORT GridFloat {
public:
  /* Single-rank grid. maxNumThreads < 1 selects the hardware concurrency. */
  GridFloat(int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns,
       SpfftProcessingUnitType processingUnit, int maxNumThreads);

#ifdef SPFFT_AMD_MPI_API
  /* Distributed grid over an MPI communicator (collective; implemented in libspfft_amd_mpi). */
  GridFloat(int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns, int maxLocalZLength,
       SpfftProcessingUnitType processingUnit, int maxNumThreads, MPI_Comm comm,
       SpfftExchangeType exchangeType);
#endif

  /* Distributed grid over any spfft::Communicator (collective). */
  GridFloat(int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns, int maxLocalZLength,
       SpfftProcessingUnitType processingUnit, int maxNumThreads,
       std::shared_ptr<Communicator> comm, SpfftExchangeType exchangeType);

  GridFloat(const GridFloat& other);
  GridFloat(GridFloat&&) = default;
  GridFloat& operator=(const GridFloat& other);
  GridFloat& operator=(GridFloat&&) = default;

  TransformFloat create_transform(SpfftProcessingUnitType processingUnit,
                             SpfftTransformType transformType, int dimX, int dimY, int dimZ,
                             int localZLength, int numLocalElements,
                             SpfftIndexFormatType indexFormat, const int* indices) const;

  int max_dim_x() const;
  int max_dim_y() const;
  int max_dim_z() const;
  int max_num_local_z_columns() const;
  int max_local_z_length() const;
  SpfftProcessingUnitType processing_unit() const;
  int device_id() const;
  int num_threads() const;

#ifdef SPFFT_AMD_MPI_API
  MPI_Comm communicator() const;
#endif
  /* The communicator of a distributed grid (nullptr for a local grid). */
  std::shared_ptr<Communicator> spfft_communicator() const;

  /* Internal: implementation access for the MPI front end. */
  explicit GridFloat(std::shared_ptr<GridImpl<float>> impl);
  const std::shared_ptr<GridImpl<float>>& impl() const { return grid_; }

private:
  std::shared_ptr<GridImpl<float>> grid_;
};

}  // namespace spfft

#endif
