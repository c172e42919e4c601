// Public Grid / GridFloat (reference: src/spfft/grid.cpp, grid_float.cpp).
#include "api/grid_impl.hpp"
#include "api/transform_impl.hpp"
#include "spfft/grid.hpp"
#include "spfft/grid_float.hpp"

namespace spfft {

#define SPFFT_AMD_DEFINE_GRID(GRID, TRANSFORM, T)                                                 \
  GRID::GRID(int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns,                      \
             SpfftProcessingUnitType processingUnit, int maxNumThreads)                           \
      : grid_(std::make_shared<GridImpl<T>>(maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns,       \
                                            processingUnit, maxNumThreads)) {}                    \
  GRID::GRID(int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns, int maxLocalZLength, \
             SpfftProcessingUnitType processingUnit, int maxNumThreads,                           \
             std::shared_ptr<Communicator> comm, SpfftExchangeType exchangeType)                  \
      : grid_(std::make_shared<GridImpl<T>>(maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns,       \
                                            maxLocalZLength, processingUnit, maxNumThreads,       \
                                            std::move(comm), exchangeType)) {}                    \
  GRID::GRID(std::shared_ptr<GridImpl<T>> impl) : grid_(std::move(impl)) {}                       \
  GRID::GRID(const GRID& other) : grid_(std::make_shared<GridImpl<T>>(*other.grid_)) {}           \
  GRID& GRID::operator=(const GRID& other) {                                                      \
    if (this != &other) grid_ = std::make_shared<GridImpl<T>>(*other.grid_);                      \
    return *this;                                                                                 \
  }                                                                                               \
  TRANSFORM GRID::create_transform(SpfftProcessingUnitType processingUnit,                        \
                                   SpfftTransformType transformType, int dimX, int dimY, int dimZ, \
                                   int localZLength, int numLocalElements,                        \
                                   SpfftIndexFormatType indexFormat, const int* indices) const {  \
    return TRANSFORM(std::make_shared<TransformImpl<T>>(grid_, processingUnit, transformType,     \
                                                        dimX, dimY, dimZ, localZLength,           \
                                                        numLocalElements, indexFormat, indices)); \
  }                                                                                               \
  int GRID::max_dim_x() const { return grid_->max_dim_x(); }                                      \
  int GRID::max_dim_y() const { return grid_->max_dim_y(); }                                      \
  int GRID::max_dim_z() const { return grid_->max_dim_z(); }                                      \
  int GRID::max_num_local_z_columns() const { return grid_->max_num_local_z_columns(); }          \
  int GRID::max_local_z_length() const { return grid_->max_local_z_length(); }                    \
  SpfftProcessingUnitType GRID::processing_unit() const { return grid_->processing_unit(); }      \
  int GRID::device_id() const { return grid_->device_id(); }                                      \
  int GRID::num_threads() const { return grid_->num_threads(); }                                  \
  std::shared_ptr<Communicator> GRID::spfft_communicator() const { return grid_->communicator(); }

SPFFT_AMD_DEFINE_GRID(Grid, Transform, double)
SPFFT_AMD_DEFINE_GRID(GridFloat, TransformFloat, float)

#undef SPFFT_AMD_DEFINE_GRID

}  // namespace spfft
