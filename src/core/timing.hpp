// Host timing tree + roctx ranges (replaces the reference's rt_graph timer,
// src/timing/rt_graph.hpp:107-173, timing.hpp:45-60).
//
// Scopes form a tree per call path; each node keeps every sample so the report
// has count / total / mean / median / min / max / share of parent. Enabled at
// run time (SPFFT_TIMING=1 or spfft_amd_timing_enable). Independently of that,
// every scope emits a roctx range (visible with rocprofv3 --marker-trace).
#pragma once

#include <initializer_list>
#include <string>

namespace spfft {
namespace timing {

// Level 0 off, 1 host scopes (the reference's rt_graph timer), 2 host scopes
// plus GPU stage intervals (hipEvents at every stage boundary, one record per
// stage: extra host API calls on every transform).
bool enabled();
bool gpu_stages();
void set_level(int level);
void reset();
std::string report_json();
std::string report_text();
// Adds one sample (seconds) to the node root/path[0]/path[1]/... (GPU-side
// stage times measured with hipEvents, which are known only after the fact).
void add_sample(std::initializer_list<const char*> path, double seconds);

class Scope {
public:
  explicit Scope(const char* name);
  ~Scope();
  Scope(const Scope&) = delete;
  Scope& operator=(const Scope&) = delete;

private:
  void* node_ = nullptr;
  long long startNs_ = 0;
  bool marker_ = false;
};

}  // namespace timing
}  // namespace spfft

#define SPFFT_TIMING_CONCAT2(a, b) a##b
#define SPFFT_TIMING_CONCAT(a, b) SPFFT_TIMING_CONCAT2(a, b)
#define SPFFT_TIMED_SCOPE(name) \
  ::spfft::timing::Scope SPFFT_TIMING_CONCAT(spfftTimingScope_, __LINE__)(name)
