// Host (CPU) execution engine: the same three-stage pipeline as the GPU path
// (z-stick FFT with fused decompress/symmetry/pack; y-column FFT with fused
// unpack/plane-symmetry; x-row FFT C2C or C2R) on the hand-written host FFT,
// parallelised with the ThreadPool. Distributed exchange through the grid's
// Communicator (reference: src/execution/execution_host.{hpp,cpp}).
#pragma once

#include <memory>
#include <vector>

#include "api/grid_impl.hpp"
#include "fft/host_fft.hpp"
#include "plan/index_plan.hpp"

namespace spfft {

template <typename T>
class HostExecutor {
public:
  HostExecutor(std::shared_ptr<GridImpl<T>> grid, std::shared_ptr<const IndexPlan> plan);

  // Step-wise API (reference: execution_host.hpp:70-81).
  void backward_z(const T* input);
  void backward_exchange();
  void backward_xy();
  void forward_xy();
  void forward_exchange();
  void forward_z(T* output, SpfftScalingType scaling);

  T* space_domain() { return static_cast<T*>(grid_->host_slot(GridImpl<T>::kSpace)); }

private:
  template <typename BT>
  void z_backward(const cx<T>* values, BT* stickSide);
  template <typename BT>
  void y_backward(const BT* slabSide, cx<T>* inter);
  template <typename BT>
  void y_forward(const cx<T>* inter, BT* slabSide);
  template <typename BT>
  void z_forward(const BT* stickSide, cx<T>* values, T scale);
  void x_backward(const cx<T>* inter, T* space);
  void x_forward(const T* space, cx<T>* inter);
  void exchange(bool backward);
  void poison(bool backward);
  cx<T>* scratch(int thread, std::size_t n);

  std::shared_ptr<GridImpl<T>> grid_;
  std::shared_ptr<const IndexPlan> plan_;
  ExchangeLayout layout_;
  bool floatExchange_ = false;
  HostFft<T> fftX_, fftY_, fftZ_;
  std::vector<std::vector<cx<T>>> scratch_;
};

}  // namespace spfft
