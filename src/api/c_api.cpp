// C API (reference: extern "C" blocks of src/spfft/{grid,transform,multi_transform}[_float].cpp)
// plus the SpFFT-AMD extensions of spfft/amd.h. Every entry point converts
// exceptions into SpfftError codes; a null handle is SPFFT_INVALID_HANDLE_ERROR.
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "api/c_guard.hpp"
#include "api/transform_impl.hpp"
#include "comm/callback_comm.hpp"
#include "comm/shm_group.hpp"
#include "gpu/gpu_runtime.hpp"
#include "core/common.hpp"
#include "core/timing.hpp"
#include "gpu/device_comm.hpp"
#include "gpu/gpu_executor.hpp"
#include "spfft/amd.h"
#include "spfft/exceptions.hpp"
#include "spfft/grid.hpp"
#include "spfft/grid_float.hpp"
#include "spfft/multi_transform.h"
#include "spfft/multi_transform_float.h"
#include "spfft/transform.hpp"
#include "spfft/transform_float.hpp"

namespace spfft {
void multi_forward_handles(int n, Transform** ts, SpfftProcessingUnitType* in, double** out,
                           SpfftScalingType* sc);
void multi_backward_handles(int n, Transform** ts, double** in, SpfftProcessingUnitType* out);
void multi_forward_handles(int n, TransformFloat** ts, SpfftProcessingUnitType* in, float** out,
                           SpfftScalingType* sc);
void multi_backward_handles(int n, TransformFloat** ts, float** in, SpfftProcessingUnitType* out);
}  // namespace spfft

using namespace spfft;

std::string& spfft::c_last_error() {
  static thread_local std::string msg;
  return msg;
}

namespace {

template <class H>
H* handle(void* h) {
  if (!h) throw InvalidParameterError();
  return static_cast<H*>(h);
}

struct InvalidHandle {};

template <class H, class F>
SpfftError with_handle(void* h, F&& f) {
  if (!h) {
    c_last_error() = "invalid handle";
    return SPFFT_INVALID_HANDLE_ERROR;
  }
  return guarded([&] { f(*static_cast<H*>(h)); });
}


// Minimal DLPack (v0.8 ABI) structures for zero-copy export of the space domain.
struct DLDeviceX {
  int32_t device_type;  // 1 = CPU, 10 = ROCm
  int32_t device_id;
};
struct DLDataTypeX {
  uint8_t code;  // 2 = float, 5 = complex
  uint8_t bits;
  uint16_t lanes;
};
struct DLTensorX {
  void* data;
  DLDeviceX device;
  int32_t ndim;
  DLDataTypeX dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensorX {
  DLTensorX dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensorX*);
};

template <typename TR>
struct DlpackHolder {
  DLManagedTensorX managed;
  int64_t shape[3];
  TR owner;  // shares the transform (and its grid) until torch drops the view
};

template <typename TR>
void dlpack_delete(DLManagedTensorX* m) {
  delete static_cast<DlpackHolder<TR>*>(m->manager_ctx);
}

template <typename TR, typename T>
void* export_space_domain(TR& t, SpfftProcessingUnitType loc) {
  auto* h = new DlpackHolder<TR>{DLManagedTensorX{}, {0, 0, 0}, t};
  const bool real = t.type() == SPFFT_TRANS_R2C;
  h->shape[0] = t.local_z_length();
  h->shape[1] = t.dim_y();
  h->shape[2] = t.dim_x();
  DLTensorX& d = h->managed.dl_tensor;
  d.data = t.space_domain_data(loc);
  d.device.device_type = loc == SPFFT_PU_GPU ? 10 : 1;
  d.device.device_id = loc == SPFFT_PU_GPU ? t.device_id() : 0;
  d.ndim = 3;
  d.dtype.code = real ? 2 : 5;
  d.dtype.bits = static_cast<uint8_t>(sizeof(T) * 8 * (real ? 1 : 2));
  d.dtype.lanes = 1;
  d.shape = h->shape;
  d.strides = nullptr;
  d.byte_offset = 0;
  h->managed.manager_ctx = h;
  h->managed.deleter = &dlpack_delete<TR>;
  return &h->managed;
}

}  // namespace

namespace {
template <class Impl>
const char* data_plane_of(Impl& impl) {
  if (!(impl.processing_unit() & SPFFT_PU_GPU) || impl.local()) return "none";
  return impl.device_comm().kind();
}
// (a per-thread copy: valid until the thread's next call)
template <class Impl>
const char* data_plane_info_of(Impl& impl) {
  static thread_local std::string buf;
  if (!(impl.processing_unit() & SPFFT_PU_GPU) || impl.local())
    buf = "{\"kind\": \"none\"}";
  else
    buf = impl.device_comm().info();
  return buf.c_str();
}
}  // namespace

namespace {
template <typename T, class X>
void exchange_plan_of(X& x, int* chunks, int* stickBlocks, int* peerWrites, int* relays) {
  auto* g = x.impl()->gpu();
  *chunks = g ? g->exchange_chunks() : 0;
  *stickBlocks = g ? g->exchange_stick_blocks() : 0;
  *peerWrites = g && g->exchange_peer_writes() ? 1 : 0;
  *relays = g && x.impl()->plan().size > 1 ? x.impl()->grid()->device_comm().relay_count() : 0;
}
}  // namespace

extern "C" {

// ------------------------------------------------------------------ grids
#define SPFFT_AMD_C_GRID(PREFIX, GRID, GRIDH)                                                     \
  SpfftError PREFIX##grid_create(GRIDH* grid, int maxDimX, int maxDimY, int maxDimZ,              \
                                 int maxNumLocalZColumns, SpfftProcessingUnitType processingUnit, \
                                 int maxNumThreads) {                                             \
    if (!grid) return SPFFT_INVALID_PARAMETER_ERROR;                                              \
    return guarded([&] {                                                                          \
      *grid = new GRID(maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns, processingUnit,            \
                       maxNumThreads);                                                            \
    });                                                                                           \
  }                                                                                               \
  SpfftError PREFIX##grid_destroy(GRIDH grid) {                                                   \
    if (!grid) return SPFFT_INVALID_HANDLE_ERROR;                                                 \
    return guarded([&] { delete static_cast<GRID*>(grid); });                                     \
  }                                                                                               \
  SpfftError PREFIX##grid_max_dim_x(GRIDH g, int* v) {                                            \
    return with_handle<GRID>(g, [&](GRID& x) { *v = x.max_dim_x(); });                            \
  }                                                                                               \
  SpfftError PREFIX##grid_max_dim_y(GRIDH g, int* v) {                                            \
    return with_handle<GRID>(g, [&](GRID& x) { *v = x.max_dim_y(); });                            \
  }                                                                                               \
  SpfftError PREFIX##grid_max_dim_z(GRIDH g, int* v) {                                            \
    return with_handle<GRID>(g, [&](GRID& x) { *v = x.max_dim_z(); });                            \
  }                                                                                               \
  SpfftError PREFIX##grid_max_num_local_z_columns(GRIDH g, int* v) {                              \
    return with_handle<GRID>(g, [&](GRID& x) { *v = x.max_num_local_z_columns(); });              \
  }                                                                                               \
  SpfftError PREFIX##grid_max_local_z_length(GRIDH g, int* v) {                                   \
    return with_handle<GRID>(g, [&](GRID& x) { *v = x.max_local_z_length(); });                   \
  }                                                                                               \
  SpfftError PREFIX##grid_processing_unit(GRIDH g, SpfftProcessingUnitType* v) {                  \
    return with_handle<GRID>(g, [&](GRID& x) { *v = x.processing_unit(); });                      \
  }                                                                                               \
  SpfftError PREFIX##grid_device_id(GRIDH g, int* v) {                                            \
    return with_handle<GRID>(g, [&](GRID& x) { *v = x.device_id(); });                           \
  }                                                                                               \
  SpfftError PREFIX##grid_num_threads(GRIDH g, int* v) {                                          \
    return with_handle<GRID>(g, [&](GRID& x) { *v = x.num_threads(); });                          \
  }

SPFFT_AMD_C_GRID(spfft_, Grid, SpfftGrid)
SPFFT_AMD_C_GRID(spfft_float_, GridFloat, SpfftFloatGrid)

// ------------------------------------------------------------- transforms
#define SPFFT_AMD_C_TRANSFORM(PREFIX, GRID, TRANSFORM, GRIDH, TRH, T)                              \
  SpfftError PREFIX##transform_create(TRH* transform, GRIDH grid,                                  \
                                      SpfftProcessingUnitType processingUnit,                      \
                                      SpfftTransformType transformType, int dimX, int dimY,        \
                                      int dimZ, int localZLength, int numLocalElements,            \
                                      SpfftIndexFormatType indexFormat, const int* indices) {      \
    if (!grid) return SPFFT_INVALID_HANDLE_ERROR;                                                  \
    if (!transform) return SPFFT_INVALID_PARAMETER_ERROR;                                          \
    return guarded([&] {                                                                           \
      *transform = new TRANSFORM(static_cast<GRID*>(grid)->create_transform(                       \
          processingUnit, transformType, dimX, dimY, dimZ, localZLength, numLocalElements,         \
          indexFormat, indices));                                                                  \
    });                                                                                            \
  }                                                                                                \
  SpfftError PREFIX##transform_destroy(TRH transform) {                                            \
    if (!transform) return SPFFT_INVALID_HANDLE_ERROR;                                             \
    return guarded([&] { delete static_cast<TRANSFORM*>(transform); });                            \
  }                                                                                                \
  SpfftError PREFIX##transform_clone(TRH transform, TRH* newTransform) {                           \
    if (!newTransform) return SPFFT_INVALID_PARAMETER_ERROR;                                       \
    return with_handle<TRANSFORM>(transform,                                                       \
                                  [&](TRANSFORM& t) { *newTransform = new TRANSFORM(t.clone()); }); \
  }                                                                                                \
  SpfftError PREFIX##transform_forward(TRH transform, SpfftProcessingUnitType inputLocation,       \
                                       T* output, SpfftScalingType scaling) {                      \
    return with_handle<TRANSFORM>(                                                                 \
        transform, [&](TRANSFORM& t) { t.forward(inputLocation, output, scaling); });              \
  }                                                                                                \
  SpfftError PREFIX##transform_backward(TRH transform, const T* input,                             \
                                        SpfftProcessingUnitType outputLocation) {                  \
    return with_handle<TRANSFORM>(transform,                                                       \
                                  [&](TRANSFORM& t) { t.backward(input, outputLocation); });        \
  }                                                                                                \
  SpfftError PREFIX##transform_get_space_domain(TRH transform,                                     \
                                                SpfftProcessingUnitType dataLocation, T** data) {  \
    return with_handle<TRANSFORM>(                                                                 \
        transform, [&](TRANSFORM& t) { *data = t.space_domain_data(dataLocation); });              \
  }                                                                                                \
  SpfftError PREFIX##transform_dim_x(TRH t, int* v) {                                              \
    return with_handle<TRANSFORM>(t, [&](TRANSFORM& x) { *v = x.dim_x(); });                       \
  }                                                                                                \
  SpfftError PREFIX##transform_dim_y(TRH t, int* v) {                                              \
    return with_handle<TRANSFORM>(t, [&](TRANSFORM& x) { *v = x.dim_y(); });                       \
  }                                                                                                \
  SpfftError PREFIX##transform_dim_z(TRH t, int* v) {                                              \
    return with_handle<TRANSFORM>(t, [&](TRANSFORM& x) { *v = x.dim_z(); });                       \
  }                                                                                                \
  SpfftError PREFIX##transform_local_z_length(TRH t, int* v) {                                     \
    return with_handle<TRANSFORM>(t, [&](TRANSFORM& x) { *v = x.local_z_length(); });              \
  }                                                                                                \
  SpfftError PREFIX##transform_local_slice_size(TRH t, int* v) {                                   \
    return with_handle<TRANSFORM>(t, [&](TRANSFORM& x) { *v = x.local_slice_size(); });            \
  }                                                                                                \
  SpfftError PREFIX##transform_local_z_offset(TRH t, int* v) {                                     \
    return with_handle<TRANSFORM>(t, [&](TRANSFORM& x) { *v = x.local_z_offset(); });              \
  }                                                                                                \
  SpfftError PREFIX##transform_global_size(TRH t, long long int* v) {                              \
    return with_handle<TRANSFORM>(t, [&](TRANSFORM& x) { *v = x.global_size(); });                 \
  }                                                                                                \
  SpfftError PREFIX##transform_num_local_elements(TRH t, int* v) {                                 \
    return with_handle<TRANSFORM>(t, [&](TRANSFORM& x) { *v = x.num_local_elements(); });          \
  }                                                                                                \
  SpfftError PREFIX##transform_num_global_elements(TRH t, long long int* v) {                      \
    return with_handle<TRANSFORM>(t, [&](TRANSFORM& x) { *v = x.num_global_elements(); });         \
  }                                                                                                \
  SpfftError PREFIX##transform_device_id(TRH t, int* v) {                                          \
    return with_handle<TRANSFORM>(t, [&](TRANSFORM& x) { *v = x.device_id(); });                   \
  }                                                                                                \
  SpfftError PREFIX##transform_num_threads(TRH t, int* v) {                                        \
    return with_handle<TRANSFORM>(t, [&](TRANSFORM& x) { *v = x.num_threads(); });                 \
  }                                                                                                \
  SpfftError PREFIX##transform_type(TRH t, SpfftTransformType* v) {                                \
    return with_handle<TRANSFORM>(t, [&](TRANSFORM& x) { *v = x.type(); });                        \
  }                                                                                                \
  SpfftError PREFIX##transform_processing_unit(TRH t, SpfftProcessingUnitType* v) {                \
    return with_handle<TRANSFORM>(t, [&](TRANSFORM& x) { *v = x.processing_unit(); });             \
  }                                                                                                \
  SpfftError PREFIX##multi_transform_forward(int n, TRH* transforms,                               \
                                             SpfftProcessingUnitType* inputLocations,              \
                                             T** outputPointers, SpfftScalingType* scalingTypes) { \
    if (n > 0 && !transforms) return SPFFT_INVALID_PARAMETER_ERROR;                                \
    for (int i = 0; i < n; ++i)                                                                    \
      if (!transforms[i]) return SPFFT_INVALID_HANDLE_ERROR;                                       \
    return guarded([&] {                                                                           \
      multi_forward_handles(n, reinterpret_cast<TRANSFORM**>(transforms), inputLocations,          \
                            outputPointers, scalingTypes);                                         \
    });                                                                                            \
  }                                                                                                \
  SpfftError PREFIX##multi_transform_backward(int n, TRH* transforms, T** inputPointers,           \
                                              SpfftProcessingUnitType* outputLocations) {          \
    if (n > 0 && !transforms) return SPFFT_INVALID_PARAMETER_ERROR;                                \
    for (int i = 0; i < n; ++i)                                                                    \
      if (!transforms[i]) return SPFFT_INVALID_HANDLE_ERROR;                                       \
    return guarded([&] {                                                                           \
      multi_backward_handles(n, reinterpret_cast<TRANSFORM**>(transforms), inputPointers,          \
                             outputLocations);                                                     \
    });                                                                                            \
  }

SPFFT_AMD_C_TRANSFORM(spfft_, Grid, Transform, SpfftGrid, SpfftTransform, double)
SPFFT_AMD_C_TRANSFORM(spfft_float_, GridFloat, TransformFloat, SpfftFloatGrid,
                      SpfftFloatTransform, float)

// ------------------------------------------------------- SpFFT-AMD additions
SpfftError spfft_amd_comm_create_callbacks(SpfftAmdComm* comm,
                                           const SpfftAmdCommCallbacks* callbacks) {
  if (!comm || !callbacks) return SPFFT_INVALID_PARAMETER_ERROR;
  return guarded([&] {
    *comm = new CommHandle(std::make_shared<CallbackCommunicator>(*callbacks));
  });
}

SpfftError spfft_amd_comm_create_local_group(int size, SpfftAmdComm* comms) {
  if (!comms || size < 1) return SPFFT_INVALID_PARAMETER_ERROR;
  return guarded([&] {
    auto group = create_local_communicators(size);
    for (int r = 0; r < size; ++r) comms[r] = new CommHandle(group[r]);
  });
}

SpfftError spfft_amd_comm_destroy(SpfftAmdComm comm) {
  if (!comm) return SPFFT_INVALID_HANDLE_ERROR;
  return guarded([&] { delete static_cast<CommHandle*>(comm); });
}

SpfftError spfft_amd_comm_rank(SpfftAmdComm comm, int* rank) {
  return with_handle<CommHandle>(comm, [&](CommHandle& c) { *rank = c->rank(); });
}

SpfftError spfft_amd_comm_size(SpfftAmdComm comm, int* size) {
  return with_handle<CommHandle>(comm, [&](CommHandle& c) { *size = c->size(); });
}

SpfftError spfft_amd_grid_create_distributed(SpfftGrid* grid, int maxDimX, int maxDimY,
                                             int maxDimZ, int maxNumLocalZColumns,
                                             int maxLocalZLength,
                                             SpfftProcessingUnitType processingUnit,
                                             int maxNumThreads, SpfftAmdComm comm,
                                             SpfftExchangeType exchangeType) {
  if (!grid) return SPFFT_INVALID_PARAMETER_ERROR;
  return with_handle<CommHandle>(comm, [&](CommHandle& c) {
    *grid = new Grid(maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns, maxLocalZLength,
                     processingUnit, maxNumThreads, c, exchangeType);
  });
}

SpfftError spfft_amd_float_grid_create_distributed(SpfftFloatGrid* grid, int maxDimX, int maxDimY,
                                                   int maxDimZ, int maxNumLocalZColumns,
                                                   int maxLocalZLength,
                                                   SpfftProcessingUnitType processingUnit,
                                                   int maxNumThreads, SpfftAmdComm comm,
                                                   SpfftExchangeType exchangeType) {
  if (!grid) return SPFFT_INVALID_PARAMETER_ERROR;
  return with_handle<CommHandle>(comm, [&](CommHandle& c) {
    *grid = new GridFloat(maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns, maxLocalZLength,
                          processingUnit, maxNumThreads, c, exchangeType);
  });
}

SpfftError spfft_amd_grid_exchange_type(SpfftGrid grid, SpfftExchangeType* type) {
  return with_handle<Grid>(grid, [&](Grid& g) { *type = g.impl()->exchange_type(); });
}
SpfftError spfft_amd_float_grid_exchange_type(SpfftFloatGrid grid, SpfftExchangeType* type) {
  return with_handle<GridFloat>(grid, [&](GridFloat& g) { *type = g.impl()->exchange_type(); });
}

SpfftError spfft_amd_grid_data_plane(SpfftGrid grid, const char** name) {
  if (!name) return SPFFT_INVALID_PARAMETER_ERROR;
  return with_handle<Grid>(grid, [&](Grid& g) { *name = data_plane_of(*g.impl()); });
}
SpfftError spfft_amd_float_grid_data_plane(SpfftFloatGrid grid, const char** name) {
  if (!name) return SPFFT_INVALID_PARAMETER_ERROR;
  return with_handle<GridFloat>(grid, [&](GridFloat& g) { *name = data_plane_of(*g.impl()); });
}
SpfftError spfft_amd_grid_data_plane_info(SpfftGrid grid, const char** json) {
  if (!json) return SPFFT_INVALID_PARAMETER_ERROR;
  return with_handle<Grid>(grid, [&](Grid& g) { *json = data_plane_info_of(*g.impl()); });
}
SpfftError spfft_amd_float_grid_data_plane_info(SpfftFloatGrid grid, const char** json) {
  if (!json) return SPFFT_INVALID_PARAMETER_ERROR;
  return with_handle<GridFloat>(grid, [&](GridFloat& g) { *json = data_plane_info_of(*g.impl()); });
}

SpfftError spfft_amd_grid_device_bytes(SpfftGrid grid, unsigned long long* bytes) {
  if (!bytes) return SPFFT_INVALID_PARAMETER_ERROR;
  return with_handle<Grid>(grid, [&](Grid& g) { *bytes = g.impl()->device_bytes(); });
}
SpfftError spfft_amd_float_grid_device_bytes(SpfftFloatGrid grid, unsigned long long* bytes) {
  if (!bytes) return SPFFT_INVALID_PARAMETER_ERROR;
  return with_handle<GridFloat>(grid, [&](GridFloat& g) { *bytes = g.impl()->device_bytes(); });
}

SpfftError spfft_amd_rccl_communicators(int* count) {
  if (!count) return SPFFT_INVALID_PARAMETER_ERROR;
  *count = spfft::DeviceComm::rccl_channels_created();
  return SPFFT_SUCCESS;
}

SpfftError spfft_amd_library_streams(int* count) {
  if (!count) return SPFFT_INVALID_PARAMETER_ERROR;
  *count = spfft::GpuStream::live();
  return SPFFT_SUCCESS;
}

SpfftError spfft_amd_transform_exchange_plan(SpfftTransform t, int* chunks, int* stickBlocks,
                                             int* peerWrites, int* relays) {
  if (!chunks || !stickBlocks || !peerWrites || !relays) return SPFFT_INVALID_PARAMETER_ERROR;
  return with_handle<Transform>(
      t, [&](Transform& x) { exchange_plan_of<double>(x, chunks, stickBlocks, peerWrites, relays); });
}
SpfftError spfft_amd_float_transform_exchange_plan(SpfftFloatTransform t, int* chunks,
                                                   int* stickBlocks, int* peerWrites, int* relays) {
  if (!chunks || !stickBlocks || !peerWrites || !relays) return SPFFT_INVALID_PARAMETER_ERROR;
  return with_handle<TransformFloat>(
      t, [&](TransformFloat& x) { exchange_plan_of<float>(x, chunks, stickBlocks, peerWrites, relays); });
}

SpfftError spfft_amd_transform_set_stream(SpfftTransform t, void* stream, int synchronous) {
  return with_handle<Transform>(
      t, [&](Transform& x) { x.set_execution_stream(stream, synchronous != 0); });
}
SpfftError spfft_amd_float_transform_set_stream(SpfftFloatTransform t, void* stream,
                                                int synchronous) {
  return with_handle<TransformFloat>(
      t, [&](TransformFloat& x) { x.set_execution_stream(stream, synchronous != 0); });
}
SpfftError spfft_amd_transform_reset_stream(SpfftTransform t) {
  return with_handle<Transform>(t, [&](Transform& x) { x.reset_execution_stream(); });
}
SpfftError spfft_amd_float_transform_reset_stream(SpfftFloatTransform t) {
  return with_handle<TransformFloat>(t, [&](TransformFloat& x) { x.reset_execution_stream(); });
}
SpfftError spfft_amd_transform_synchronize(SpfftTransform t) {
  return with_handle<Transform>(t, [&](Transform& x) { x.synchronize(); });
}
SpfftError spfft_amd_float_transform_synchronize(SpfftFloatTransform t) {
  return with_handle<TransformFloat>(t, [&](TransformFloat& x) { x.synchronize(); });
}
SpfftError spfft_amd_transform_local_z_offset_rank(SpfftTransform t, int rank, int* offset,
                                                   int* length) {
  return with_handle<Transform>(t, [&](Transform& x) {
    const auto& p = x.impl()->plan();
    if (rank < 0 || rank >= p.size) throw InvalidParameterError();
    *offset = p.planeOffsets[rank];
    *length = p.planesPerRank[rank];
  });
}

SpfftError spfft_amd_transform_space_domain_dlpack(SpfftTransform t, SpfftProcessingUnitType loc,
                                                   void** managedTensor) {
  if (!managedTensor) return SPFFT_INVALID_PARAMETER_ERROR;
  return with_handle<Transform>(
      t, [&](Transform& x) { *managedTensor = export_space_domain<Transform, double>(x, loc); });
}
SpfftError spfft_amd_float_transform_space_domain_dlpack(SpfftFloatTransform t,
                                                         SpfftProcessingUnitType loc,
                                                         void** managedTensor) {
  if (!managedTensor) return SPFFT_INVALID_PARAMETER_ERROR;
  return with_handle<TransformFloat>(t, [&](TransformFloat& x) {
    *managedTensor = export_space_domain<TransformFloat, float>(x, loc);
  });
}

SpfftError spfft_amd_transform_forward_xy(SpfftTransform t, SpfftProcessingUnitType loc) {
  return with_handle<Transform>(t, [&](Transform& x) { x.forward_xy(loc); });
}
SpfftError spfft_amd_transform_forward_exchange(SpfftTransform t, int nonBlocking) {
  return with_handle<Transform>(t, [&](Transform& x) { x.forward_exchange(nonBlocking != 0); });
}
SpfftError spfft_amd_transform_forward_z(SpfftTransform t, double* output,
                                         SpfftScalingType scaling) {
  return with_handle<Transform>(t, [&](Transform& x) { x.forward_z(output, scaling); });
}
SpfftError spfft_amd_transform_backward_z(SpfftTransform t, const double* input) {
  return with_handle<Transform>(t, [&](Transform& x) { x.backward_z(input); });
}
SpfftError spfft_amd_transform_backward_exchange(SpfftTransform t, int nonBlocking) {
  return with_handle<Transform>(t, [&](Transform& x) { x.backward_exchange(nonBlocking != 0); });
}
SpfftError spfft_amd_transform_backward_xy(SpfftTransform t, SpfftProcessingUnitType loc) {
  return with_handle<Transform>(t, [&](Transform& x) { x.backward_xy(loc); });
}
SpfftError spfft_amd_float_transform_forward_xy(SpfftFloatTransform t, SpfftProcessingUnitType loc) {
  return with_handle<TransformFloat>(t, [&](TransformFloat& x) { x.forward_xy(loc); });
}
SpfftError spfft_amd_float_transform_forward_exchange(SpfftFloatTransform t, int nonBlocking) {
  return with_handle<TransformFloat>(t, [&](TransformFloat& x) { x.forward_exchange(nonBlocking != 0); });
}
SpfftError spfft_amd_float_transform_forward_z(SpfftFloatTransform t, float* output,
                                               SpfftScalingType scaling) {
  return with_handle<TransformFloat>(t, [&](TransformFloat& x) { x.forward_z(output, scaling); });
}
SpfftError spfft_amd_float_transform_backward_z(SpfftFloatTransform t, const float* input) {
  return with_handle<TransformFloat>(t, [&](TransformFloat& x) { x.backward_z(input); });
}
SpfftError spfft_amd_float_transform_backward_exchange(SpfftFloatTransform t, int nonBlocking) {
  return with_handle<TransformFloat>(t, [&](TransformFloat& x) { x.backward_exchange(nonBlocking != 0); });
}
SpfftError spfft_amd_float_transform_backward_xy(SpfftFloatTransform t, SpfftProcessingUnitType loc) {
  return with_handle<TransformFloat>(t, [&](TransformFloat& x) { x.backward_xy(loc); });
}

SpfftError spfft_amd_timing_enable(int enable) {
  timing::set_level(enable);
  return SPFFT_SUCCESS;
}
SpfftError spfft_amd_timing_reset(void) {
  timing::reset();
  return SPFFT_SUCCESS;
}

static SpfftError copy_report(const std::string& s, char* buffer, size_t size, size_t* required) {
  if (required) *required = s.size() + 1;
  if (buffer && size > 0) {
    const size_t n = s.size() < size - 1 ? s.size() : size - 1;
    std::memcpy(buffer, s.data(), n);
    buffer[n] = '\0';
  }
  return SPFFT_SUCCESS;
}

SpfftError spfft_amd_timing_json(char* buffer, size_t size, size_t* required) {
  return copy_report(timing::report_json(), buffer, size, required);
}
SpfftError spfft_amd_timing_print(char* buffer, size_t size, size_t* required) {
  return copy_report(timing::report_text(), buffer, size, required);
}

const char* spfft_amd_last_error_message(void) { return c_last_error().c_str(); }

int spfft_amd_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

const char* spfft_amd_build_info(void) {
  return "SpFFT-AMD 1.0.0 target=gfx950";
}

}  // extern "C"
