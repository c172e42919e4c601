// Public Transform / TransformFloat (reference: src/spfft/transform.cpp, transform_float.cpp).
#include "api/grid_impl.hpp"
#include "api/transform_impl.hpp"
#include "spfft/transform.hpp"
#include "spfft/transform_float.hpp"

namespace spfft {

#define SPFFT_AMD_DEFINE_TRANSFORM(TRANSFORM, T)                                                 \
  TRANSFORM::TRANSFORM(std::shared_ptr<TransformImpl<T>> impl) : transform_(std::move(impl)) {}  \
  TRANSFORM TRANSFORM::clone() const { return TRANSFORM(transform_->clone()); }                 \
  SpfftTransformType TRANSFORM::type() const { return transform_->plan().type; }                \
  int TRANSFORM::dim_x() const { return transform_->plan().dimX; }                               \
  int TRANSFORM::dim_y() const { return transform_->plan().dimY; }                               \
  int TRANSFORM::dim_z() const { return transform_->plan().dimZ; }                               \
  int TRANSFORM::local_z_length() const { return transform_->plan().local_planes(); }            \
  int TRANSFORM::local_z_offset() const { return transform_->plan().local_plane_offset(); }      \
  int TRANSFORM::local_slice_size() const {                                                      \
    const auto& p = transform_->plan();                                                          \
    return p.dimX * p.dimY * p.local_planes();                                                   \
  }                                                                                              \
  long long int TRANSFORM::global_size() const {                                                 \
    const auto& p = transform_->plan();                                                          \
    return static_cast<long long>(p.dimX) * p.dimY * p.dimZ;                                     \
  }                                                                                              \
  int TRANSFORM::num_local_elements() const { return transform_->plan().numLocalElements; }      \
  long long int TRANSFORM::num_global_elements() const {                                         \
    return transform_->plan().numGlobalElements;                                                 \
  }                                                                                              \
  SpfftProcessingUnitType TRANSFORM::processing_unit() const {                                   \
    return transform_->processing_unit();                                                        \
  }                                                                                              \
  int TRANSFORM::device_id() const { return transform_->grid()->device_id(); }                   \
  int TRANSFORM::num_threads() const { return transform_->grid()->num_threads(); }               \
  T* TRANSFORM::space_domain_data(SpfftProcessingUnitType dataLocation) {                        \
    return transform_->space_domain_data(dataLocation);                                          \
  }                                                                                              \
  void TRANSFORM::forward(SpfftProcessingUnitType inputLocation, T* output,                      \
                          SpfftScalingType scaling) {                                            \
    transform_->forward(inputLocation, output, scaling);                                         \
  }                                                                                              \
  void TRANSFORM::backward(const T* input, SpfftProcessingUnitType outputLocation) {             \
    transform_->backward(input, outputLocation);                                                 \
  }                                                                                              \
  void TRANSFORM::set_execution_stream(void* hipStream, bool synchronous) {                      \
    transform_->set_stream(hipStream, synchronous);                                              \
  }                                                                                              \
  void TRANSFORM::synchronize() { transform_->synchronize(); }                                   \
  void TRANSFORM::reset_execution_stream() { transform_->reset_stream(); }                       \
  std::shared_ptr<Communicator> TRANSFORM::spfft_communicator() const {                          \
    return transform_->grid()->communicator();                                                   \
  }                                                                                              \
  void TRANSFORM::forward_xy(SpfftProcessingUnitType inputLocation) {                            \
    transform_->forward_xy(inputLocation);                                                       \
  }                                                                                              \
  void TRANSFORM::forward_exchange(bool nonBlocking) { transform_->forward_exchange(nonBlocking); } \
  void TRANSFORM::forward_z(T* output, SpfftScalingType scaling) {                               \
    transform_->forward_z(output, scaling);                                                      \
  }                                                                                              \
  void TRANSFORM::backward_z(const T* input) { transform_->backward_z(input); }                  \
  void TRANSFORM::backward_exchange(bool nonBlocking) {                                          \
    transform_->backward_exchange(nonBlocking);                                                  \
  }                                                                                              \
  void TRANSFORM::backward_xy(SpfftProcessingUnitType outputLocation) {                          \
    transform_->backward_xy(outputLocation);                                                     \
  }

SPFFT_AMD_DEFINE_TRANSFORM(Transform, double)
SPFFT_AMD_DEFINE_TRANSFORM(TransformFloat, float)

#undef SPFFT_AMD_DEFINE_TRANSFORM

}  // namespace spfft
