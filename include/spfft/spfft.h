/* Umbrella header of the C API (also pulls in multi_transform.h, which the
 * reference's spfft.h forgets: SURVEY.md §7.8). */
#ifndef SPFFT_SPFFT_H
#define SPFFT_SPFFT_H

#include "spfft/config.h"
#include "spfft/errors.h"
#include "spfft/grid.h"
#include "spfft/grid_float.h"
#include "spfft/multi_transform.h"
#include "spfft/multi_transform_float.h"
#include "spfft/transform.h"
#include "spfft/transform_float.h"
#include "spfft/types.h"
#include "spfft/amd.h"

#endif
