/*
 * Error codes returned by the C API.
 *
 * Codes 0..22 are identical to SpFFT (reference: include/spfft/errors.h:33-126).
 * SPFFT_INTERNAL_ERROR (23) is new: the reference reports an internal error as
 * SPFFT_FFTW_ERROR (reference quirk, include/spfft/exceptions.hpp:174); appending
 * a code keeps every existing value unchanged.
 */
#ifndef SPFFT_ERRORS_H
#define SPFFT_ERRORS_H

#include "spfft/config.h"

enum SpfftError {
  SPFFT_SUCCESS = 0,
  SPFFT_UNKNOWN_ERROR = 1,
  SPFFT_INVALID_HANDLE_ERROR = 2,
  SPFFT_OVERFLOW_ERROR = 3,
  SPFFT_ALLOCATION_ERROR = 4,
  SPFFT_INVALID_PARAMETER_ERROR = 5,
  SPFFT_DUPLICATE_INDICES_ERROR = 6,
  SPFFT_INVALID_INDICES_ERROR = 7,
  SPFFT_MPI_SUPPORT_ERROR = 8,
  SPFFT_MPI_ERROR = 9,
  SPFFT_MPI_PARAMETER_MISMATCH_ERROR = 10,
  SPFFT_HOST_EXECUTION_ERROR = 11,
  SPFFT_FFTW_ERROR = 12, /* host FFT engine failure (name kept for compatibility) */
  SPFFT_GPU_ERROR = 13,
  SPFFT_GPU_PRECEDING_ERROR = 14,
  SPFFT_GPU_SUPPORT_ERROR = 15,
  SPFFT_GPU_ALLOCATION_ERROR = 16,
  SPFFT_GPU_LAUNCH_ERROR = 17,
  SPFFT_GPU_NO_DEVICE_ERROR = 18,
  SPFFT_GPU_INVALID_VALUE_ERROR = 19,
  SPFFT_GPU_INVALID_DEVICE_PTR_ERROR = 20,
  SPFFT_GPU_COPY_ERROR = 21,
  SPFFT_GPU_FFT_ERROR = 22,
  SPFFT_INTERNAL_ERROR = 23
};

#ifndef __cplusplus
typedef enum SpfftError SpfftError;
#endif

#endif
