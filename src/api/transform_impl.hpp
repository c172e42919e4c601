// TransformImpl<T>: validated plan + executor (reference: src/spfft/transform_internal.{hpp,cpp}).
#pragma once

#include <memory>

#include "api/grid_impl.hpp"
#include "gpu/gpu_executor.hpp"
#include "host/host_executor.hpp"
#include "plan/index_plan.hpp"

namespace spfft {

template <typename T>
class TransformImpl {
public:
  TransformImpl(std::shared_ptr<GridImpl<T>> grid, SpfftProcessingUnitType executionUnit,
                SpfftTransformType type, int dimX, int dimY, int dimZ, int localZLength,
                int numLocalElements, SpfftIndexFormatType format, const int* indices);
  TransformImpl(std::shared_ptr<GridImpl<T>> grid, SpfftProcessingUnitType executionUnit,
                std::shared_ptr<const IndexPlan> plan);

  std::shared_ptr<TransformImpl> clone() const;

  void forward(SpfftProcessingUnitType inputLocation, T* output, SpfftScalingType scaling);
  void backward(const T* input, SpfftProcessingUnitType outputLocation);

  void forward_xy(SpfftProcessingUnitType inputLocation);
  void forward_exchange(bool nonBlocking);
  void forward_z(T* output, SpfftScalingType scaling);
  void backward_z(const T* input);
  void backward_exchange(bool nonBlocking);
  void backward_xy(SpfftProcessingUnitType outputLocation);
  void synchronize();
  void set_stream(void* stream, bool synchronous);
  void reset_stream();

  T* space_domain_data(SpfftProcessingUnitType location);

  const IndexPlan& plan() const { return *plan_; }
  const std::shared_ptr<GridImpl<T>>& grid() const { return grid_; }
  SpfftProcessingUnitType processing_unit() const { return exec_; }
  bool is_gpu() const { return static_cast<bool>(gpu_); }
  GpuExecutor<T>* gpu() { return gpu_.get(); }

private:
  void create_executor();

  std::shared_ptr<GridImpl<T>> grid_;
  SpfftProcessingUnitType exec_;
  std::shared_ptr<const IndexPlan> plan_;
  std::unique_ptr<HostExecutor<T>> host_;
  std::unique_ptr<GpuExecutor<T>> gpu_;
};

}  // namespace spfft
