// Host (CPU) execution engine: the same three-stage pipeline as the GPU path
// (z-stick FFT with fused decompress/symmetry/pack; y-column FFT with fused
// unpack/plane-symmetry; x-row FFT C2C or C2R) on the hand-written host FFT,
// parallelised with the ThreadPool. Distributed exchange through the grid's
// Communicator (reference: src/execution/execution_host.{hpp,cpp}).
#pragma once

#include <memory>
#include <vector>

#include "api/grid_impl.hpp"
#include "fft/host_fft_batch.hpp"
#include "plan/index_plan.hpp"
#include "spfft/communicator.hpp"

namespace spfft {

template <typename T>
class HostExecutor {
public:
  HostExecutor(std::shared_ptr<GridImpl<T>> grid, std::shared_ptr<const IndexPlan> plan);

  // Step-wise API (reference: execution_host.hpp:70-81).
  void backward_z(const T* input);
  // nonBlocking: start the exchange and return; the next stage of the same
  // direction (backward_xy / forward_z) completes it (reference:
  // src/spfft/transform_internal.cpp:195-198, 277-282)
  void backward_exchange(bool nonBlocking = false);
  void backward_xy();
  void forward_xy();
  void forward_exchange(bool nonBlocking = false);
  void forward_z(T* output, SpfftScalingType scaling);

  T* space_domain() { return static_cast<T*>(grid_->host_slot(GridImpl<T>::kSpace)); }

private:
  using Fft = HostFftBatch<T>;
  using VC = typename HostSimd<T>::VC;
  using V = typename HostSimd<T>::V;
  static constexpr int W = HostSimd<T>::W;
  void fft(const Fft& f, VC* a, VC* b, int nl, int sign);
  template <typename BT>
  void z_backward(const cx<T>* values, BT* stickSide);
  template <typename BT>
  void z_forward(const BT* stickSide, cx<T>* values, T scale);
  template <typename BT>
  void yx_backward(const BT* slabSide, cx<T>* inter, T* space);
  template <typename BT>
  void xy_forward(const T* space, cx<T>* inter, BT* slabSide);
  template <typename BT>
  void y_col_backward(const BT* slab, int c, int z0, int nl, VC* a, VC* w);
  template <typename BT>
  void y_col_forward(VC* a, int c, int z0, int nl, BT* slab, VC* w);
  template <class Col>
  void x_rows_backward(Col col, int nl, T* const* rows, VC* a, VC* w);
  template <class Put>
  void x_rows_forward(const T* const* rows, int nl, Put put, VC* a, VC* w);
  std::size_t block_scratch() const;
  // column stride of the fused plane-block buffer: dimY + 1 elements, so the
  // x-line gathers (one element per column) do not all hit one cache set
  i64 block_stride() const { return plan_->dimY + 1; }
  void exchange(bool backward, bool nonBlocking);
  void exchange_strided(bool backward, bool nonBlocking);
  void finish_exchange();
  std::unique_ptr<ExchangeRequest> pending_;
  void poison(bool backward);
  VC* scratch(int thread, std::size_t n);

  std::shared_ptr<GridImpl<T>> grid_;
  std::shared_ptr<const IndexPlan> plan_;
  ExchangeLayout layout_;
  bool floatExchange_ = false;
  bool unbuffered_ = false;  // UNBUFFERED: natural stick layout, strided alltoallw
  bool packedReal_ = false;  // R2C with even dimX: half-length x FFTs
  bool fuseXY_ = false;      // y/x stages fused per block of W planes
  Fft fftX_, fftY_, fftZ_;
  std::vector<cx<T>> twX_;   // exp(-2 pi i m / dimX)
  std::vector<std::vector<VC>> scratch_;
};

}  // namespace spfft
