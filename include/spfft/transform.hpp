/*
 * spfft::Transform — a planned sparse 3D FFT bound to a Grid.
 *
 * API-compatible with SpFFT's Transform (reference: include/spfft/transform.hpp:58-211):
 * copies are shallow (share the plan), clone() is deep (new Grid), forward()
 * writes the sparse frequency values in the order of the index triplets given
 * at creation, backward() fills the dense space-domain slab returned by
 * space_domain_data(). Both calls are synchronous by default.
 *
 * SpFFT-AMD extensions: an explicit HIP stream (asynchronous mode), and the
 * step-wise API used by the multi-transform scheduler.
 */
#ifndef SPFFT_TRANSFORM_HPP
#define SPFFT_TRANSFORM_HPP

#include <memory>

#include "spfft/config.h"
#include "spfft/types.h"

#ifdef SPFFT_AMD_MPI_API
#include <mpi.h>
#endif

namespace spfft {

template <typename T>
class GridImpl;
template <typename T>
class TransformImpl;
class Grid;

class SPFFT_EXPORT Transform {
public:
  using ValueType = double;

  Transform(const Transform&) = default;
  Transform(Transform&&) = default;
  Transform& operator=(const Transform&) = default;
  Transform& operator=(Transform&&) = default;

  /* Deep copy with an independent, newly allocated Grid. */
  Transform clone() const;

  SpfftTransformType type() const;
  int dim_x() const;
  int dim_y() const;
  int dim_z() const;
  int local_z_length() const;
  int local_z_offset() const;
  int local_slice_size() const;
  long long int global_size() const;
  int num_local_elements() const;
  long long int num_global_elements() const;
  SpfftProcessingUnitType processing_unit() const;
  int device_id() const;
  int num_threads() const;
#ifdef SPFFT_AMD_MPI_API
  MPI_Comm communicator() const;
#endif

  /* Dense slab [localZ][dimY][dimX] (interleaved complex, or real for R2C). */
  double* space_domain_data(SpfftProcessingUnitType dataLocation);

  void forward(SpfftProcessingUnitType inputLocation, double* output,
               SpfftScalingType scaling = SPFFT_NO_SCALING);
  void backward(const double* input, SpfftProcessingUnitType outputLocation);

  /* ---- SpFFT-AMD extensions ------------------------------------------------ */
  /* Run GPU work on `hipStream` (a hipStream_t; nullptr = legacy default stream).
   * With synchronous == false the calls return after enqueueing; call
   * synchronize() before touching results. */
  void set_execution_stream(void* hipStream, bool synchronous);
  /* Back to the private stream (ordered after the legacy default stream, synchronous). */
  void reset_execution_stream();
  void synchronize();

  /* Step-wise execution (forward = xy, exchange, z; backward = z, exchange, xy). */
  void forward_xy(SpfftProcessingUnitType inputLocation);
  void forward_exchange(bool nonBlockingExchange);
  void forward_z(double* output, SpfftScalingType scaling);
  void backward_z(const double* input);
  void backward_exchange(bool nonBlockingExchange);
  void backward_xy(SpfftProcessingUnitType outputLocation);

  /* The communicator of a distributed transform (nullptr if local). */
  std::shared_ptr<class Communicator> spfft_communicator() const;

  /* Internal. */
  explicit Transform(std::shared_ptr<TransformImpl<double>> impl);
  const std::shared_ptr<TransformImpl<double>>& impl() const { return transform_; }

private:
  std::shared_ptr<TransformImpl<double>> transform_;
};

}  // namespace spfft

#endif
