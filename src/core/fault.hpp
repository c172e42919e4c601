// Fault injection for the failure-detection tests.
//
// Compiled into the testing library only: CMake builds libspfft_amd_testing.so
// (kernels shared with the release library, host code built with
// SPFFT_FAULT_INJECTION=1, plus the test probes of src/testing/). The release
// library libspfft_amd.so reads no fault switch: SPFFT_FAULT(NAME) is the
// constant 0 there and every injection site folds away.
//
// SPFFT_FAULT(NAME) = the integer value of the environment variable
// SPFFT_FAULT_<NAME> (0 when unset), read at each call.
#pragma once

#if defined(SPFFT_FAULT_INJECTION) && SPFFT_FAULT_INJECTION
#include <cstdlib>
namespace spfft {
inline int fault_value(const char* var) {
  const char* e = std::getenv(var);
  return e && *e ? std::atoi(e) : 0;
}
}  // namespace spfft
#define SPFFT_FAULT(NAME) ::spfft::fault_value("SPFFT_FAULT_" #NAME)
#else
#define SPFFT_FAULT(NAME) 0
#endif
