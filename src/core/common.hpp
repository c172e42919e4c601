// Common internal definitions of SpFFT-AMD.
#pragma once

#include <cstddef>
#include <cstdint>
#include <limits>
#include <string>

#include "spfft/exceptions.hpp"
#include "spfft/types.h"

namespace spfft {

using i64 = std::int64_t;

// Detail text for the next error reported through the C API's
// spfft_amd_last_error_message (the exception classes carry fixed texts, as in
// the reference); consumed by the API guard of the same thread.
inline std::string& error_detail() {
  static thread_local std::string detail;
  return detail;
}
inline void set_error_detail(std::string text) { error_detail() = std::move(text); }

// Throws InvalidParameterError unless cond holds.
inline void require_param(bool cond) {
  if (!cond) throw InvalidParameterError();
}

// Product of non-negative ints as 64-bit, with an OverflowError above `limit`.
inline i64 checked_mul(i64 a, i64 b, i64 limit = std::numeric_limits<i64>::max()) {
  if (a < 0 || b < 0) throw InvalidParameterError();
  if (a != 0 && b > limit / a) throw OverflowError();
  return a * b;
}

inline bool is_exchange_float(SpfftExchangeType t) {
  return t == SPFFT_EXCH_BUFFERED_FLOAT || t == SPFFT_EXCH_COMPACT_BUFFERED_FLOAT;
}
inline bool is_exchange_buffered(SpfftExchangeType t) {
  return t == SPFFT_EXCH_BUFFERED || t == SPFFT_EXCH_BUFFERED_FLOAT;
}

}  // namespace spfft
