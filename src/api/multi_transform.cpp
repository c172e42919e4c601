// Overlapped execution of independent transforms
// (reference: src/spfft/multi_transform_internal.hpp:47-145).
//
// GPU transforms each own a stream, so enqueuing stage k of every transform
// before stage k+1 lets the GPU overlap transform i's exchange with transform
// j's FFT kernels; host transforms run their stages in between.
#include <algorithm>
#include <set>
#include <vector>

#include "api/transform_impl.hpp"
#include "core/timing.hpp"
#include "spfft/multi_transform.hpp"
#include "spfft/multi_transform_float.hpp"

namespace spfft {
namespace {

template <typename T>
void check_distinct_grids(const std::vector<TransformImpl<T>*>& ts) {
  std::set<const GridImpl<T>*> grids;
  for (auto* t : ts) {
    if (!t) throw InvalidParameterError();
    if (!grids.insert(t->grid().get()).second) throw InvalidParameterError();
  }
}

// Batched groups (GpuExecutor::backward_batch / forward_batch): GPU transforms
// that can share launches, grouped by plan key in call order, at most
// dev::kMaxBatch per group; small grids batch join-free members only, large
// grids run sub-batches of batch_split() on their leaders' streams. Returns,
// per transform, whether a batch ran it. `tag(i)` must match within a group
// (the forward scaling).
template <typename T, class Eligible, class Tag, class Run>
std::vector<bool> run_batches(const std::vector<TransformImpl<T>*>& ts, Eligible eligible, Tag tag,
                              Run run) {
  const int n = static_cast<int>(ts.size());
  std::vector<bool> done(n, false);
  for (auto* t : ts)
    if (t->is_gpu()) t->gpu()->ensure_stream();  // the stream comparisons below need them
  auto ok = [&](int j) {
    return !done[j] && ts[j]->is_gpu() && ts[j]->gpu()->batchable() && eligible(j);
  };
  for (int i = 0; i < n; ++i) {
    if (!ok(i)) continue;
    GpuExecutor<T>* lead = ts[i]->gpu();
    const bool large = lead->batch_large();
    std::vector<int> group{i};
    for (int j = i + 1; j < n && static_cast<int>(group.size()) < dev::kMaxBatch; ++j)
      if (ok(j) && ts[j]->gpu()->batch_key() == lead->batch_key() && tag(j) == tag(i) &&
          (large || ts[j]->gpu()->batch_join_free(*lead)))
        group.push_back(j);
    if (group.size() < 2) continue;
    // sub-batches overlap only on different streams: one shared stream keeps one batch
    bool oneStream = true;
    for (int j : group) oneStream = oneStream && ts[j]->gpu()->stream() == lead->stream();
    const std::size_t split =
        large && !oneStream ? static_cast<std::size_t>(lead->batch_split()) : group.size();
    for (std::size_t k = 0; k < group.size(); k += split)
      run(std::vector<int>(group.begin() + k, group.begin() + std::min(group.size(), k + split)));
    for (int j : group) done[j] = true;
  }
  return done;
}

template <typename T>
void multi_forward(const std::vector<TransformImpl<T>*>& ts,
                   const SpfftProcessingUnitType* inputLocations, T* const* outputs,
                   const SpfftScalingType* scalings) {
  SPFFT_TIMED_SCOPE("multi_forward");
  check_distinct_grids(ts);
  const int n = static_cast<int>(ts.size());
  for (int i = 0; i < n; ++i)
    if (scalings[i] != SPFFT_NO_SCALING && scalings[i] != SPFFT_FULL_SCALING)
      throw InvalidParameterError();
  const std::vector<bool> batched = run_batches<T>(
      ts,
      [&](int i) {
        return inputLocations[i] == SPFFT_PU_GPU &&
               (ts[i]->plan().numLocalElements == 0 || is_device_pointer(outputs[i]));
      },
      [&](int i) { return static_cast<int>(scalings[i]); },
      [&](const std::vector<int>& g) {
        std::vector<GpuExecutor<T>*> ex;
        std::vector<T*> outs;
        for (int j : g) {
          ex.push_back(ts[j]->gpu());
          outs.push_back(outputs[j]);
        }
        GpuExecutor<T>::forward_batch(ex, outs, scalings[g[0]]);
      });
  for (int i = 0; i < n; ++i)
    if (ts[i]->is_gpu() && !batched[i]) ts[i]->forward_xy(inputLocations[i]);
  for (int i = 0; i < n; ++i)
    if (!ts[i]->is_gpu()) {
      ts[i]->forward_xy(inputLocations[i]);
      ts[i]->forward_exchange(true);
    }
  for (int i = 0; i < n; ++i)
    if (ts[i]->is_gpu() && !batched[i]) {
      ts[i]->forward_exchange(true);
      ts[i]->forward_z(outputs[i], scalings[i]);
    }
  for (int i = 0; i < n; ++i)
    if (!ts[i]->is_gpu()) ts[i]->forward_z(outputs[i], scalings[i]);
  for (int i = 0; i < n; ++i)
    if (ts[i]->is_gpu() && ts[i]->gpu()->synchronous()) ts[i]->synchronize();
}

template <typename T>
void multi_backward(const std::vector<TransformImpl<T>*>& ts, const T* const* inputs,
                    const SpfftProcessingUnitType* outputLocations) {
  SPFFT_TIMED_SCOPE("multi_backward");
  check_distinct_grids(ts);
  const int n = static_cast<int>(ts.size());
  const std::vector<bool> batched = run_batches<T>(
      ts,
      [&](int i) {
        return outputLocations[i] == SPFFT_PU_GPU &&
               (ts[i]->plan().numLocalElements == 0 || is_device_pointer(inputs[i]));
      },
      [](int) { return 0; },
      [&](const std::vector<int>& g) {
        std::vector<GpuExecutor<T>*> ex;
        std::vector<const T*> ins;
        for (int j : g) {
          ex.push_back(ts[j]->gpu());
          ins.push_back(inputs[j]);
        }
        GpuExecutor<T>::backward_batch(ex, ins);
      });
  for (int i = 0; i < n; ++i)
    if (ts[i]->is_gpu() && !batched[i]) ts[i]->backward_z(inputs[i]);
  for (int i = 0; i < n; ++i)
    if (!ts[i]->is_gpu()) {
      ts[i]->backward_z(inputs[i]);
      ts[i]->backward_exchange(true);
    }
  for (int i = 0; i < n; ++i)
    if (ts[i]->is_gpu() && !batched[i]) {
      ts[i]->backward_exchange(true);
      ts[i]->backward_xy(outputLocations[i]);
    }
  for (int i = 0; i < n; ++i)
    if (!ts[i]->is_gpu()) ts[i]->backward_xy(outputLocations[i]);
  for (int i = 0; i < n; ++i)
    if (ts[i]->is_gpu() && ts[i]->gpu()->synchronous()) ts[i]->synchronize();
}

template <typename TR, typename T>
std::vector<TransformImpl<T>*> impls(int n, TR* transforms) {
  if (n < 0 || (n > 0 && !transforms)) throw InvalidParameterError();
  std::vector<TransformImpl<T>*> v;
  for (int i = 0; i < n; ++i) v.push_back(transforms[i].impl().get());
  return v;
}

}  // namespace

void multi_transform_forward(int numTransforms, Transform* transforms,
                             SpfftProcessingUnitType* inputLocations, double** outputPointers,
                             SpfftScalingType* scalingTypes) {
  multi_forward<double>(impls<Transform, double>(numTransforms, transforms), inputLocations,
                        outputPointers, scalingTypes);
}

void multi_transform_backward(int numTransforms, Transform* transforms, double** inputPointers,
                              SpfftProcessingUnitType* outputLocations) {
  multi_backward<double>(impls<Transform, double>(numTransforms, transforms), inputPointers,
                         outputLocations);
}

void multi_transform_forward(int numTransforms, TransformFloat* transforms,
                             SpfftProcessingUnitType* inputLocations, float** outputPointers,
                             SpfftScalingType* scalingTypes) {
  multi_forward<float>(impls<TransformFloat, float>(numTransforms, transforms), inputLocations,
                       outputPointers, scalingTypes);
}

void multi_transform_backward(int numTransforms, TransformFloat* transforms, float** inputPointers,
                              SpfftProcessingUnitType* outputLocations) {
  multi_backward<float>(impls<TransformFloat, float>(numTransforms, transforms), inputPointers,
                        outputLocations);
}

// used by the C API (array of handles)
void multi_forward_handles(int n, Transform** ts, SpfftProcessingUnitType* in, double** out,
                           SpfftScalingType* sc) {
  std::vector<TransformImpl<double>*> v;
  for (int i = 0; i < n; ++i) v.push_back(ts[i] ? ts[i]->impl().get() : nullptr);
  multi_forward<double>(v, in, out, sc);
}
void multi_backward_handles(int n, Transform** ts, double** in, SpfftProcessingUnitType* out) {
  std::vector<TransformImpl<double>*> v;
  for (int i = 0; i < n; ++i) v.push_back(ts[i] ? ts[i]->impl().get() : nullptr);
  multi_backward<double>(v, in, out);
}
void multi_forward_handles(int n, TransformFloat** ts, SpfftProcessingUnitType* in, float** out,
                           SpfftScalingType* sc) {
  std::vector<TransformImpl<float>*> v;
  for (int i = 0; i < n; ++i) v.push_back(ts[i] ? ts[i]->impl().get() : nullptr);
  multi_forward<float>(v, in, out, sc);
}
void multi_backward_handles(int n, TransformFloat** ts, float** in, SpfftProcessingUnitType* out) {
  std::vector<TransformImpl<float>*> v;
  for (int i = 0; i < n; ++i) v.push_back(ts[i] ? ts[i]->impl().get() : nullptr);
  multi_backward<float>(v, in, out);
}

}  // namespace spfft
