/*
 * C API of the single-precision Transform (reference: include/spfft/transform_float.h).
 */
#ifndef SPFFT_TRANSFORM_FLOAT_H
#define SPFFT_TRANSFORM_FLOAT_H

#include "spfft/config.h"
#include "spfft/errors.h"
#include "spfft/grid_float.h"
#include "spfft/types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef void* SpfftFloatTransform;

SPFFT_EXPORT SpfftError spfft_float_transform_create(SpfftFloatTransform* transform, SpfftFloatGrid grid,
                                               SpfftProcessingUnitType processingUnit,
                                               SpfftTransformType transformType, int dimX, int dimY,
                                               int dimZ, int localZLength, int numLocalElements,
                                               SpfftIndexFormatType indexFormat,
                                               const int* indices);
SPFFT_EXPORT SpfftError spfft_float_transform_destroy(SpfftFloatTransform transform);
SPFFT_EXPORT SpfftError spfft_float_transform_clone(SpfftFloatTransform transform,
                                              SpfftFloatTransform* newTransform);
SPFFT_EXPORT SpfftError spfft_float_transform_forward(SpfftFloatTransform transform,
                                                SpfftProcessingUnitType inputLocation,
                                                float* output, SpfftScalingType scaling);
SPFFT_EXPORT SpfftError spfft_float_transform_backward(SpfftFloatTransform transform, const float* input,
                                                 SpfftProcessingUnitType outputLocation);
SPFFT_EXPORT SpfftError spfft_float_transform_get_space_domain(SpfftFloatTransform transform,
                                                         SpfftProcessingUnitType dataLocation,
                                                         float** data);
SPFFT_EXPORT SpfftError spfft_float_transform_dim_x(SpfftFloatTransform transform, int* dimX);
SPFFT_EXPORT SpfftError spfft_float_transform_dim_y(SpfftFloatTransform transform, int* dimY);
SPFFT_EXPORT SpfftError spfft_float_transform_dim_z(SpfftFloatTransform transform, int* dimZ);
SPFFT_EXPORT SpfftError spfft_float_transform_local_z_length(SpfftFloatTransform transform, int* localZLength);
SPFFT_EXPORT SpfftError spfft_float_transform_local_slice_size(SpfftFloatTransform transform, int* size);
SPFFT_EXPORT SpfftError spfft_float_transform_local_z_offset(SpfftFloatTransform transform, int* offset);
SPFFT_EXPORT SpfftError spfft_float_transform_global_size(SpfftFloatTransform transform,
                                                    long long int* globalSize);
SPFFT_EXPORT SpfftError spfft_float_transform_num_local_elements(SpfftFloatTransform transform,
                                                           int* numLocalElements);
SPFFT_EXPORT SpfftError spfft_float_transform_num_global_elements(SpfftFloatTransform transform,
                                                            long long int* numGlobalElements);
SPFFT_EXPORT SpfftError spfft_float_transform_device_id(SpfftFloatTransform transform, int* deviceId);
SPFFT_EXPORT SpfftError spfft_float_transform_num_threads(SpfftFloatTransform transform, int* numThreads);
/* SpFFT-AMD additions: the C API of the reference has no type()/processing_unit() getters. */
SPFFT_EXPORT SpfftError spfft_float_transform_type(SpfftFloatTransform transform, SpfftTransformType* type);
SPFFT_EXPORT SpfftError spfft_float_transform_processing_unit(SpfftFloatTransform transform,
                                                        SpfftProcessingUnitType* processingUnit);

#ifdef SPFFT_AMD_MPI_API
SPFFT_EXPORT SpfftError spfft_float_transform_communicator(SpfftFloatTransform transform, MPI_Comm* comm);
#endif

#ifdef __cplusplus
}
#endif

#endif
