/*
 * Public enumerations of SpFFT-AMD.
 *
 * The numeric values are ABI: they are mirrored by the Fortran module
 * (spfft.f90) and must match SpFFT (reference: include/spfft/types.h:33-106).
 */
#ifndef SPFFT_TYPES_H
#define SPFFT_TYPES_H

#include "spfft/config.h"

/* How the pencil (z-stick) <-> slab (xy-plane) redistribution is exchanged. */
/* C++ sees the enumerations with a fixed underlying int: any int a C caller
 * passes is then a valid value that the API validation rejects with an error
 * code (without a fixed type, loading an out-of-range value is undefined in C++,
 * flagged by UBSan, tools/sanitize.py). Same layout as the C enumerations. */
#ifdef __cplusplus
#define SPFFT_ENUM_INT : int
#else
#define SPFFT_ENUM_INT
#endif

enum SpfftExchangeType SPFFT_ENUM_INT {
  SPFFT_EXCH_DEFAULT = 0,                /* = COMPACT_BUFFERED */
  SPFFT_EXCH_BUFFERED = 1,               /* padded all-to-all (ncclAllToAll / MPI_Alltoall) */
  SPFFT_EXCH_BUFFERED_FLOAT = 2,         /* padded, exchanged in fp32 */
  SPFFT_EXCH_COMPACT_BUFFERED = 3,       /* exact-size all-to-allv */
  SPFFT_EXCH_COMPACT_BUFFERED_FLOAT = 4, /* exact-size, exchanged in fp32 */
  SPFFT_EXCH_UNBUFFERED = 5              /* zero-copy exchange (no separate pack buffer) */
};

/* Where data lives / where a transform executes. Bit flags for a Grid. */
enum SpfftProcessingUnitType SPFFT_ENUM_INT { SPFFT_PU_HOST = 1, SPFFT_PU_GPU = 2 };

/* Format of the frequency-domain index list. */
enum SpfftIndexFormatType SPFFT_ENUM_INT { SPFFT_INDEX_TRIPLETS = 0 };

/* Complex-to-complex or real(space)-to-complex(frequency). */
enum SpfftTransformType SPFFT_ENUM_INT { SPFFT_TRANS_C2C = 0, SPFFT_TRANS_R2C = 1 };

/* Optional 1/(Nx*Ny*Nz) scaling, applied in the forward direction only. */
enum SpfftScalingType SPFFT_ENUM_INT { SPFFT_NO_SCALING = 0, SPFFT_FULL_SCALING = 1 };

#ifndef __cplusplus
typedef enum SpfftExchangeType SpfftExchangeType;
typedef enum SpfftProcessingUnitType SpfftProcessingUnitType;
typedef enum SpfftTransformType SpfftTransformType;
typedef enum SpfftIndexFormatType SpfftIndexFormatType;
typedef enum SpfftScalingType SpfftScalingType;
#endif

#endif
