/* Umbrella header of the C++ API. */
#ifndef SPFFT_SPFFT_HPP
#define SPFFT_SPFFT_HPP

#include "spfft/communicator.hpp"
#include "spfft/config.h"
#include "spfft/exceptions.hpp"
#include "spfft/grid.hpp"
#include "spfft/grid_float.hpp"
#include "spfft/multi_transform.hpp"
#include "spfft/multi_transform_float.hpp"
#include "spfft/transform.hpp"
#include "spfft/transform_float.hpp"
#include "spfft/types.h"

#endif
