// Exception -> SpfftError conversion of the C entry points (c_api.cpp and the
// testing library's probes, src/testing/): the message of the last failure
// of the calling thread is kept for spfft_amd_last_error_message.
#pragma once

#include <exception>
#include <memory>
#include <string>

#include "core/common.hpp"
#include "spfft/communicator.hpp"
#include "spfft/errors.h"
#include "spfft/exceptions.hpp"

namespace spfft {

// the calling thread's last error message (c_api.cpp)
std::string& c_last_error();

// SpfftAmdComm handles point at one of these
using CommHandle = std::shared_ptr<Communicator>;

template <class F>
SpfftError guarded(F&& f) {
  error_detail().clear();
  try {
    f();
    c_last_error().clear();
    return SPFFT_SUCCESS;
  } catch (const GenericError& e) {
    c_last_error() = e.what();
    if (!error_detail().empty()) c_last_error() += " [" + error_detail() + "]";
    return e.error_code();
  } catch (const std::exception& e) {
    c_last_error() = e.what();
    return SPFFT_UNKNOWN_ERROR;
  } catch (...) {
    c_last_error() = "unknown error";
    return SPFFT_UNKNOWN_ERROR;
  }
}

}  // namespace spfft
