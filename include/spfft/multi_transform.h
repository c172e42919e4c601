/*
 * C API for overlapped execution of independent transforms
 * (reference: include/spfft/multi_transform.h). `transforms` is an array of
 * transform handles (the reference reinterprets it with the wrong stride,
 * src/spfft/multi_transform.cpp:57,71 — fixed here).
 */
#ifndef SPFFT_MULTI_TRANSFORM_H
#define SPFFT_MULTI_TRANSFORM_H

#include "spfft/config.h"
#include "spfft/errors.h"
#include "spfft/transform.h"
#include "spfft/types.h"

#ifdef __cplusplus
extern "C" {
#endif

SPFFT_EXPORT SpfftError spfft_multi_transform_forward(int numTransforms, SpfftTransform* transforms,
                                                      SpfftProcessingUnitType* inputLocations,
                                                      double** outputPointers,
                                                      SpfftScalingType* scalingTypes);

SPFFT_EXPORT SpfftError spfft_multi_transform_backward(int numTransforms,
                                                       SpfftTransform* transforms,
                                                       double** inputPointers,
                                                       SpfftProcessingUnitType* outputLocations);

#ifdef __cplusplus
}
#endif

#endif
