/*
 * C API for overlapped execution of independent transforms
 * (reference: include/spfft/multi_transform_float.h). `transforms` is an array of
 * transform handles (the reference reinterprets it with the wrong stride,
 * src/spfft/multi_transform.cpp:57,71 — fixed here).
 */
#ifndef SPFFT_MULTI_TRANSFORM_FLOAT_H
#define SPFFT_MULTI_TRANSFORM_FLOAT_H

#include "spfft/config.h"
#include "spfft/errors.h"
#include "spfft/transform_float.h"
#include "spfft/types.h"

#ifdef __cplusplus
extern "C" {
#endif

SPFFT_EXPORT SpfftError spfft_float_multi_transform_forward(int numTransforms, SpfftFloatTransform* transforms,
                                                      SpfftProcessingUnitType* inputLocations,
                                                      float** outputPointers,
                                                      SpfftScalingType* scalingTypes);

SPFFT_EXPORT SpfftError spfft_float_multi_transform_backward(int numTransforms,
                                                       SpfftFloatTransform* transforms,
                                                       float** inputPointers,
                                                       SpfftProcessingUnitType* outputLocations);

#ifdef __cplusplus
}
#endif

#endif
