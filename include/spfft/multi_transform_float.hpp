/*
 * Execute several independent transforms with overlapped stages
 * in single precision (reference: include/spfft/multi_transform.hpp:48-64). The transforms must not
 * share a Grid (their buffers would alias) — InvalidParameterError otherwise.
 */
#ifndef SPFFT_MULTI_TRANSFORM_FLOAT_HPP
#define SPFFT_MULTI_TRANSFORM_FLOAT_HPP

#include "spfft/config.h"
#include "spfft/transform_float.hpp"
#include "spfft/types.h"

namespace spfft {

SPFFT_EXPORT void multi_transform_forward(int numTransforms, TransformFloat* transforms,
                                          SpfftProcessingUnitType* inputLocations,
                                          float** outputPointers, SpfftScalingType* scalingTypes);

SPFFT_EXPORT void multi_transform_backward(int numTransforms, TransformFloat* transforms,
                                           float** inputPointers,
                                           SpfftProcessingUnitType* outputLocations);

}  // namespace spfft

#endif
