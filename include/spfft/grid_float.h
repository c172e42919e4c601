/*
 * C API of the single-precision Grid (reference: include/spfft/grid_float.h). Handles are opaque;
 * every function returns an SpfftError code and never throws.
 */
#ifndef SPFFT_GRID_FLOAT_H
#define SPFFT_GRID_FLOAT_H

#include "spfft/config.h"
#include "spfft/errors.h"
#include "spfft/types.h"

#ifdef SPFFT_AMD_MPI_API
#include <mpi.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef void* SpfftFloatGrid;

SPFFT_EXPORT SpfftError spfft_float_grid_create(SpfftFloatGrid* grid, int maxDimX, int maxDimY, int maxDimZ,
                                          int maxNumLocalZColumns,
                                          SpfftProcessingUnitType processingUnit,
                                          int maxNumThreads);

#ifdef SPFFT_AMD_MPI_API
SPFFT_EXPORT SpfftError spfft_float_grid_create_distributed(SpfftFloatGrid* grid, int maxDimX, int maxDimY,
                                                      int maxDimZ, int maxNumLocalZColumns,
                                                      int maxLocalZLength,
                                                      SpfftProcessingUnitType processingUnit,
                                                      int maxNumThreads, MPI_Comm comm,
                                                      SpfftExchangeType exchangeType);
SPFFT_EXPORT SpfftError spfft_float_grid_communicator(SpfftFloatGrid grid, MPI_Comm* comm);
#endif

SPFFT_EXPORT SpfftError spfft_float_grid_destroy(SpfftFloatGrid grid);
SPFFT_EXPORT SpfftError spfft_float_grid_max_dim_x(SpfftFloatGrid grid, int* dimX);
SPFFT_EXPORT SpfftError spfft_float_grid_max_dim_y(SpfftFloatGrid grid, int* dimY);
SPFFT_EXPORT SpfftError spfft_float_grid_max_dim_z(SpfftFloatGrid grid, int* dimZ);
SPFFT_EXPORT SpfftError spfft_float_grid_max_num_local_z_columns(SpfftFloatGrid grid,
                                                           int* maxNumLocalZColumns);
SPFFT_EXPORT SpfftError spfft_float_grid_max_local_z_length(SpfftFloatGrid grid, int* maxLocalZLength);
SPFFT_EXPORT SpfftError spfft_float_grid_processing_unit(SpfftFloatGrid grid,
                                                   SpfftProcessingUnitType* processingUnit);
SPFFT_EXPORT SpfftError spfft_float_grid_device_id(SpfftFloatGrid grid, int* deviceId);
SPFFT_EXPORT SpfftError spfft_float_grid_num_threads(SpfftFloatGrid grid, int* numThreads);

#ifdef __cplusplus
}
#endif

#endif
