/*
 * C API of the Grid (reference: include/spfft/grid.h). Handles are opaque;
 * every function returns an SpfftError code and never throws.
 */
#ifndef SPFFT_GRID_H
#define SPFFT_GRID_H

#include "spfft/config.h"
#include "spfft/errors.h"
#include "spfft/types.h"

#ifdef SPFFT_AMD_MPI_API
#include <mpi.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef void* SpfftGrid;

SPFFT_EXPORT SpfftError spfft_grid_create(SpfftGrid* grid, int maxDimX, int maxDimY, int maxDimZ,
                                          int maxNumLocalZColumns,
                                          SpfftProcessingUnitType processingUnit,
                                          int maxNumThreads);

#ifdef SPFFT_AMD_MPI_API
SPFFT_EXPORT SpfftError spfft_grid_create_distributed(SpfftGrid* grid, int maxDimX, int maxDimY,
                                                      int maxDimZ, int maxNumLocalZColumns,
                                                      int maxLocalZLength,
                                                      SpfftProcessingUnitType processingUnit,
                                                      int maxNumThreads, MPI_Comm comm,
                                                      SpfftExchangeType exchangeType);
SPFFT_EXPORT SpfftError spfft_grid_communicator(SpfftGrid grid, MPI_Comm* comm);
#endif

SPFFT_EXPORT SpfftError spfft_grid_destroy(SpfftGrid grid);
SPFFT_EXPORT SpfftError spfft_grid_max_dim_x(SpfftGrid grid, int* dimX);
SPFFT_EXPORT SpfftError spfft_grid_max_dim_y(SpfftGrid grid, int* dimY);
SPFFT_EXPORT SpfftError spfft_grid_max_dim_z(SpfftGrid grid, int* dimZ);
SPFFT_EXPORT SpfftError spfft_grid_max_num_local_z_columns(SpfftGrid grid,
                                                           int* maxNumLocalZColumns);
SPFFT_EXPORT SpfftError spfft_grid_max_local_z_length(SpfftGrid grid, int* maxLocalZLength);
SPFFT_EXPORT SpfftError spfft_grid_processing_unit(SpfftGrid grid,
                                                   SpfftProcessingUnitType* processingUnit);
SPFFT_EXPORT SpfftError spfft_grid_device_id(SpfftGrid grid, int* deviceId);
SPFFT_EXPORT SpfftError spfft_grid_num_threads(SpfftGrid grid, int* numThreads);

#ifdef __cplusplus
}
#endif

#endif
