#include "api/transform_impl.hpp"

#include "core/timing.hpp"
#include "spfft/exceptions.hpp"

namespace spfft {

namespace {
template <typename T>
void check_against_grid(const GridImpl<T>& g, SpfftProcessingUnitType exec, int dimX, int dimY,
                        int dimZ) {
  // reference: src/spfft/transform_internal.cpp:52-77
  if (dimX > g.max_dim_x() || dimY > g.max_dim_y() || dimZ > g.max_dim_z())
    throw InvalidParameterError();
  if (!(exec & g.processing_unit())) throw InvalidParameterError();
  if (exec != SPFFT_PU_HOST && exec != SPFFT_PU_GPU) throw InvalidParameterError();
}
}  // namespace

template <typename T>
TransformImpl<T>::TransformImpl(std::shared_ptr<GridImpl<T>> grid,
                                SpfftProcessingUnitType executionUnit, SpfftTransformType type,
                                int dimX, int dimY, int dimZ, int localZLength,
                                int numLocalElements, SpfftIndexFormatType format,
                                const int* indices)
    : grid_(std::move(grid)), exec_(executionUnit) {
  if (!grid_) throw InvalidParameterError();
  if (dimX < 0 || dimY < 0 || dimZ < 0 || localZLength < 0 || numLocalElements < 0 ||
      (!indices && numLocalElements > 0))
    throw InvalidParameterError();
  // Purely local checks may throw before any collective; the distributed plan
  // construction reports errors to every rank (plan/index_plan.cpp).
  if (grid_->local()) check_against_grid(*grid_, exec_, dimX, dimY, dimZ);
  plan_ = std::make_shared<const IndexPlan>(grid_->local() ? nullptr : grid_->communicator().get(),
                                            type, dimX, dimY, dimZ, localZLength,
                                            numLocalElements, format, indices);
  check_against_grid(*grid_, exec_, dimX, dimY, dimZ);
  if (plan_->local_planes() > grid_->max_local_z_length()) throw InvalidParameterError();
  if (plan_->local_sticks() > grid_->max_num_local_z_columns()) throw InvalidParameterError();
  create_executor();
}

template <typename T>
TransformImpl<T>::TransformImpl(std::shared_ptr<GridImpl<T>> grid,
                                SpfftProcessingUnitType executionUnit,
                                std::shared_ptr<const IndexPlan> plan)
    : grid_(std::move(grid)), exec_(executionUnit), plan_(std::move(plan)) {
  create_executor();
}

template <typename T>
void TransformImpl<T>::create_executor() {
  if (exec_ == SPFFT_PU_HOST)
    host_.reset(new HostExecutor<T>(grid_, plan_));
  else
    gpu_.reset(new GpuExecutor<T>(grid_, plan_));
}

template <typename T>
std::shared_ptr<TransformImpl<T>> TransformImpl<T>::clone() const {
  auto newGrid = std::make_shared<GridImpl<T>>(*grid_);
  return std::make_shared<TransformImpl<T>>(newGrid, exec_, plan_);
}

template <typename T>
T* TransformImpl<T>::space_domain_data(SpfftProcessingUnitType location) {
  if (exec_ == SPFFT_PU_HOST) {
    if (location != SPFFT_PU_HOST) throw InvalidParameterError();
    return host_->space_domain();
  }
  return gpu_->space_domain(location);
}

template <typename T>
void TransformImpl<T>::forward(SpfftProcessingUnitType inputLocation, T* output,
                               SpfftScalingType scaling) {
  SPFFT_TIMED_SCOPE("forward");
  if (scaling != SPFFT_NO_SCALING && scaling != SPFFT_FULL_SCALING) throw InvalidParameterError();
  if (gpu_ && gpu_->forward_graph(inputLocation, output, scaling)) {
    if (gpu_->synchronous()) gpu_->synchronize();
    return;
  }
  forward_xy(inputLocation);
  forward_exchange(false);
  forward_z(output, scaling);
  if (gpu_ && gpu_->synchronous()) gpu_->synchronize();
}

template <typename T>
void TransformImpl<T>::backward(const T* input, SpfftProcessingUnitType outputLocation) {
  SPFFT_TIMED_SCOPE("backward");
  if (gpu_ && gpu_->backward_graph(input, outputLocation)) {
    if (gpu_->synchronous()) gpu_->synchronize();
    return;
  }
  backward_z(input);
  backward_exchange(false);
  backward_xy(outputLocation);
  if (gpu_ && gpu_->synchronous()) gpu_->synchronize();
}

template <typename T>
void TransformImpl<T>::forward_xy(SpfftProcessingUnitType inputLocation) {
  if (host_) {
    if (inputLocation != SPFFT_PU_HOST) throw InvalidParameterError();
    host_->forward_xy();
  } else {
    gpu_->forward_xy(inputLocation);
  }
}

template <typename T>
void TransformImpl<T>::forward_exchange(bool nonBlocking) {
  if (host_)
    host_->forward_exchange(nonBlocking);
  else
    gpu_->forward_exchange(nonBlocking);
}

template <typename T>
void TransformImpl<T>::forward_z(T* output, SpfftScalingType scaling) {
  if (scaling != SPFFT_NO_SCALING && scaling != SPFFT_FULL_SCALING) throw InvalidParameterError();
  if (host_)
    host_->forward_z(output, scaling);
  else
    gpu_->forward_z(output, scaling);
}

template <typename T>
void TransformImpl<T>::backward_z(const T* input) {
  if (host_)
    host_->backward_z(input);
  else
    gpu_->backward_z(input);
}

template <typename T>
void TransformImpl<T>::backward_exchange(bool nonBlocking) {
  if (host_)
    host_->backward_exchange(nonBlocking);
  else
    gpu_->backward_exchange(nonBlocking);
}

template <typename T>
void TransformImpl<T>::backward_xy(SpfftProcessingUnitType outputLocation) {
  if (host_) {
    if (outputLocation != SPFFT_PU_HOST) throw InvalidParameterError();
    host_->backward_xy();
  } else {
    gpu_->backward_xy(outputLocation);
  }
}

template <typename T>
void TransformImpl<T>::synchronize() {
  if (gpu_) gpu_->synchronize();
}

template <typename T>
void TransformImpl<T>::set_stream(void* stream, bool synchronous) {
  if (!gpu_) throw InvalidParameterError();
  gpu_->set_stream(static_cast<hipStream_t>(stream), synchronous);
}

template <typename T>
void TransformImpl<T>::reset_stream() {
  if (!gpu_) throw InvalidParameterError();
  gpu_->reset_stream();
}

template class TransformImpl<double>;
template class TransformImpl<float>;

}  // namespace spfft
