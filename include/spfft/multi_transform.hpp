/*
 * Execute several independent transforms with overlapped stages
 * (reference: include/spfft/multi_transform.hpp:48-64). The transforms must not
 * share a Grid (their buffers would alias) — InvalidParameterError otherwise.
 */
#ifndef SPFFT_MULTI_TRANSFORM_HPP
#define SPFFT_MULTI_TRANSFORM_HPP

#include "spfft/config.h"
#include "spfft/transform.hpp"
#include "spfft/types.h"

namespace spfft {

SPFFT_EXPORT void multi_transform_forward(int numTransforms, Transform* transforms,
                                          SpfftProcessingUnitType* inputLocations,
                                          double** outputPointers, SpfftScalingType* scalingTypes);

SPFFT_EXPORT void multi_transform_backward(int numTransforms, Transform* transforms,
                                           double** inputPointers,
                                           SpfftProcessingUnitType* outputLocations);

}  // namespace spfft

#endif
