/*
 * C API of the Transform (reference: include/spfft/transform.h).
 */
#ifndef SPFFT_TRANSFORM_H
#define SPFFT_TRANSFORM_H

#include "spfft/config.h"
#include "spfft/errors.h"
#include "spfft/grid.h"
#include "spfft/types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef void* SpfftTransform;

SPFFT_EXPORT SpfftError spfft_transform_create(SpfftTransform* transform, SpfftGrid grid,
                                               SpfftProcessingUnitType processingUnit,
                                               SpfftTransformType transformType, int dimX, int dimY,
                                               int dimZ, int localZLength, int numLocalElements,
                                               SpfftIndexFormatType indexFormat,
                                               const int* indices);
SPFFT_EXPORT SpfftError spfft_transform_destroy(SpfftTransform transform);
SPFFT_EXPORT SpfftError spfft_transform_clone(SpfftTransform transform,
                                              SpfftTransform* newTransform);
SPFFT_EXPORT SpfftError spfft_transform_forward(SpfftTransform transform,
                                                SpfftProcessingUnitType inputLocation,
                                                double* output, SpfftScalingType scaling);
SPFFT_EXPORT SpfftError spfft_transform_backward(SpfftTransform transform, const double* input,
                                                 SpfftProcessingUnitType outputLocation);
SPFFT_EXPORT SpfftError spfft_transform_get_space_domain(SpfftTransform transform,
                                                         SpfftProcessingUnitType dataLocation,
                                                         double** data);
SPFFT_EXPORT SpfftError spfft_transform_dim_x(SpfftTransform transform, int* dimX);
SPFFT_EXPORT SpfftError spfft_transform_dim_y(SpfftTransform transform, int* dimY);
SPFFT_EXPORT SpfftError spfft_transform_dim_z(SpfftTransform transform, int* dimZ);
SPFFT_EXPORT SpfftError spfft_transform_local_z_length(SpfftTransform transform, int* localZLength);
SPFFT_EXPORT SpfftError spfft_transform_local_slice_size(SpfftTransform transform, int* size);
SPFFT_EXPORT SpfftError spfft_transform_local_z_offset(SpfftTransform transform, int* offset);
SPFFT_EXPORT SpfftError spfft_transform_global_size(SpfftTransform transform,
                                                    long long int* globalSize);
SPFFT_EXPORT SpfftError spfft_transform_num_local_elements(SpfftTransform transform,
                                                           int* numLocalElements);
SPFFT_EXPORT SpfftError spfft_transform_num_global_elements(SpfftTransform transform,
                                                            long long int* numGlobalElements);
SPFFT_EXPORT SpfftError spfft_transform_device_id(SpfftTransform transform, int* deviceId);
SPFFT_EXPORT SpfftError spfft_transform_num_threads(SpfftTransform transform, int* numThreads);
/* SpFFT-AMD additions: the C API of the reference has no type()/processing_unit() getters. */
SPFFT_EXPORT SpfftError spfft_transform_type(SpfftTransform transform, SpfftTransformType* type);
SPFFT_EXPORT SpfftError spfft_transform_processing_unit(SpfftTransform transform,
                                                        SpfftProcessingUnitType* processingUnit);

#ifdef SPFFT_AMD_MPI_API
SPFFT_EXPORT SpfftError spfft_transform_communicator(SpfftTransform transform, MPI_Comm* comm);
#endif

#ifdef __cplusplus
}
#endif

#endif
