/*
 * Exception hierarchy of the C++ API. Every exception maps to exactly one
 * SpfftError code (returned unchanged by the C API); class names and the
 * GPU sub-hierarchy follow SpFFT (reference: include/spfft/exceptions.hpp:40-302).
 *
 * Difference to the reference: InternalError reports SPFFT_INTERNAL_ERROR
 * instead of SPFFT_FFTW_ERROR (reference quirk at exceptions.hpp:174).
 */
#ifndef SPFFT_EXCEPTIONS_HPP
#define SPFFT_EXCEPTIONS_HPP

#include <stdexcept>

#include "spfft/config.h"
#include "spfft/errors.h"

namespace spfft {

class SPFFT_EXPORT GenericError : public std::exception {
public:
  const char* what() const noexcept override { return "SpFFT: generic error"; }
  virtual SpfftError error_code() const noexcept { return SPFFT_UNKNOWN_ERROR; }
};

#define SPFFT_AMD_DECLARE_ERROR(NAME, BASE, CODE, TEXT)                          \
  class SPFFT_EXPORT NAME : public BASE {                                        \
  public:                                                                        \
    const char* what() const noexcept override { return "SpFFT: " TEXT; }        \
    SpfftError error_code() const noexcept override { return CODE; }             \
  };

SPFFT_AMD_DECLARE_ERROR(OverflowError, GenericError, SPFFT_OVERFLOW_ERROR, "overflow error")
SPFFT_AMD_DECLARE_ERROR(HostAllocationError, GenericError, SPFFT_ALLOCATION_ERROR,
                        "host allocation error")
SPFFT_AMD_DECLARE_ERROR(InvalidParameterError, GenericError, SPFFT_INVALID_PARAMETER_ERROR,
                        "invalid parameter")
SPFFT_AMD_DECLARE_ERROR(DuplicateIndicesError, GenericError, SPFFT_DUPLICATE_INDICES_ERROR,
                        "duplicate z-stick indices across ranks")
SPFFT_AMD_DECLARE_ERROR(InvalidIndicesError, GenericError, SPFFT_INVALID_INDICES_ERROR,
                        "frequency index out of bounds")
SPFFT_AMD_DECLARE_ERROR(MPISupportError, GenericError, SPFFT_MPI_SUPPORT_ERROR,
                        "distributed support not available")
SPFFT_AMD_DECLARE_ERROR(MPIError, GenericError, SPFFT_MPI_ERROR, "communication error")
SPFFT_AMD_DECLARE_ERROR(MPIParameterMismatchError, GenericError,
                        SPFFT_MPI_PARAMETER_MISMATCH_ERROR, "parameters differ between ranks")
SPFFT_AMD_DECLARE_ERROR(HostExecutionError, GenericError, SPFFT_HOST_EXECUTION_ERROR,
                        "host execution error")
SPFFT_AMD_DECLARE_ERROR(FFTWError, GenericError, SPFFT_FFTW_ERROR, "host FFT engine error")
SPFFT_AMD_DECLARE_ERROR(InternalError, GenericError, SPFFT_INTERNAL_ERROR, "internal error")

class SPFFT_EXPORT GPUError : public GenericError {
public:
  const char* what() const noexcept override { return "SpFFT: GPU error"; }
  SpfftError error_code() const noexcept override { return SPFFT_GPU_ERROR; }
};

SPFFT_AMD_DECLARE_ERROR(GPUSupportError, GPUError, SPFFT_GPU_SUPPORT_ERROR,
                        "GPU support not available")
SPFFT_AMD_DECLARE_ERROR(GPUPrecedingError, GPUError, SPFFT_GPU_PRECEDING_ERROR,
                        "GPU error raised before SpFFT was called")
SPFFT_AMD_DECLARE_ERROR(GPUAllocationError, GPUError, SPFFT_GPU_ALLOCATION_ERROR,
                        "GPU allocation error")
SPFFT_AMD_DECLARE_ERROR(GPULaunchError, GPUError, SPFFT_GPU_LAUNCH_ERROR, "GPU kernel launch error")
SPFFT_AMD_DECLARE_ERROR(GPUNoDeviceError, GPUError, SPFFT_GPU_NO_DEVICE_ERROR, "no GPU available")
SPFFT_AMD_DECLARE_ERROR(GPUInvalidValueError, GPUError, SPFFT_GPU_INVALID_VALUE_ERROR,
                        "invalid value passed to the GPU runtime")
SPFFT_AMD_DECLARE_ERROR(GPUInvalidDevicePointerError, GPUError,
                        SPFFT_GPU_INVALID_DEVICE_PTR_ERROR, "invalid GPU pointer")
SPFFT_AMD_DECLARE_ERROR(GPUCopyError, GPUError, SPFFT_GPU_COPY_ERROR, "GPU memory copy error")
SPFFT_AMD_DECLARE_ERROR(GPUFFTError, GPUError, SPFFT_GPU_FFT_ERROR, "GPU FFT error")

#undef SPFFT_AMD_DECLARE_ERROR

}  // namespace spfft

#endif
