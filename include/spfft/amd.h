/*
 * SpFFT-AMD C extensions (not part of the SpFFT reference API):
 *  - communicators that do not need MPI (callbacks, in-process local group),
 *  - distributed grids over such communicators,
 *  - explicit HIP streams / asynchronous execution, step-wise execution,
 *  - timing report (host timer tree, JSON) and last-error text.
 */
#ifndef SPFFT_AMD_H
#define SPFFT_AMD_H

#include <stddef.h>

#include "spfft/config.h"
#include "spfft/errors.h"
#include "spfft/grid.h"
#include "spfft/grid_float.h"
#include "spfft/transform.h"
#include "spfft/transform_float.h"
#include "spfft/types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef void* SpfftAmdComm;

/* A communicator implemented by the caller. Each function returns 0 on success.
 *  allgather: every rank contributes `bytes`; recv holds size*bytes in rank order.
 *  alltoallv: host buffers, counts and displacements in bytes (size entries each).
 *  destroy:   optional, called once when the last user of the communicator is gone. */
typedef struct SpfftAmdCommCallbacks {
  void* context;
  int rank;
  int size;
  int (*allgather)(void* context, const void* send, void* recv, size_t bytes);
  int (*alltoallv)(void* context, const void* send, const size_t* sendCounts,
                   const size_t* sendDispls, void* recv, const size_t* recvCounts,
                   const size_t* recvDispls);
  int (*barrier)(void* context);
  void (*destroy)(void* context);
} SpfftAmdCommCallbacks;

SPFFT_EXPORT SpfftError spfft_amd_comm_create_callbacks(SpfftAmdComm* comm,
                                                        const SpfftAmdCommCallbacks* callbacks);
/* Creates `size` communicators of one in-process group (comms[r] has rank r). */
SPFFT_EXPORT SpfftError spfft_amd_comm_create_local_group(int size, SpfftAmdComm* comms);
SPFFT_EXPORT SpfftError spfft_amd_comm_destroy(SpfftAmdComm comm);
SPFFT_EXPORT SpfftError spfft_amd_comm_rank(SpfftAmdComm comm, int* rank);
SPFFT_EXPORT SpfftError spfft_amd_comm_size(SpfftAmdComm comm, int* size);
SPFFT_EXPORT SpfftError spfft_amd_grid_create_distributed(
    SpfftGrid* grid, int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns,
    int maxLocalZLength, SpfftProcessingUnitType processingUnit, int maxNumThreads,
    SpfftAmdComm comm, SpfftExchangeType exchangeType);
SPFFT_EXPORT SpfftError spfft_amd_float_grid_create_distributed(
    SpfftFloatGrid* grid, int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns,
    int maxLocalZLength, SpfftProcessingUnitType processingUnit, int maxNumThreads,
    SpfftAmdComm comm, SpfftExchangeType exchangeType);
SPFFT_EXPORT SpfftError spfft_amd_grid_exchange_type(SpfftGrid grid, SpfftExchangeType* type);
/* GPU data plane of a distributed grid: "rccl", "ipc" (peer writes across
 * processes), "peer" (peer writes inside a local group), "loopback",
 * "rccl-self" (local group moved by RCCL), or "none" (local or host-only
 * grid). Collective on first call (creates the data plane). */
SPFFT_EXPORT SpfftError spfft_amd_grid_data_plane(SpfftGrid grid, const char** name);
SPFFT_EXPORT SpfftError spfft_amd_float_grid_data_plane(SpfftFloatGrid grid, const char** name);
/* The data plane's setup facts as a JSON object ("kind"; "self_test",
 * "self_test_ms", "devices", "link_GBps_measured", "channel_priority" where they
 * apply). The string
 * stays valid until the calling thread's next call of this function.
 * Collective on first call. */
SPFFT_EXPORT SpfftError spfft_amd_grid_data_plane_info(SpfftGrid grid, const char** json);
SPFFT_EXPORT SpfftError spfft_amd_float_grid_data_plane_info(SpfftFloatGrid grid, const char** json);
/* Device memory a grid allocated (exchange buffers, intermediate, space domain). */
SPFFT_EXPORT SpfftError spfft_amd_grid_device_bytes(SpfftGrid grid, unsigned long long* bytes);
SPFFT_EXPORT SpfftError spfft_amd_float_grid_device_bytes(SpfftFloatGrid grid,
                                                          unsigned long long* bytes);
/* Number of RCCL communicators this process has created. Grids whose
 * communicators have the same members on the same devices share one
 * (SPFFT_RCCL_SHARE=0: one per grid). */
SPFFT_EXPORT SpfftError spfft_amd_rccl_communicators(int* count);
/* HIP streams the library currently owns: private transform streams (created
 * on a transform's first call unless it was given a stream before) and RCCL
 * channel streams (one per shared communicator). */
SPFFT_EXPORT SpfftError spfft_amd_library_streams(int* count);
/* Exchange plan of a GPU transform: plane chunks K and stick blocks I of the
 * pipelined all-to-all (1 and 1: one exchange per direction), whether the
 * stage kernels write into the peers directly (UNBUFFERED / IPC plane), and
 * the number of idle GPUs the exchange relays through (relay plane). Host
 * transforms report zeros. */
SPFFT_EXPORT SpfftError spfft_amd_transform_exchange_plan(SpfftTransform transform, int* chunks,
                                                          int* stickBlocks, int* peerWrites,
                                                          int* relays);
SPFFT_EXPORT SpfftError spfft_amd_float_transform_exchange_plan(SpfftFloatTransform transform,
                                                                int* chunks, int* stickBlocks,
                                                                int* peerWrites, int* relays);
SPFFT_EXPORT SpfftError spfft_amd_float_grid_exchange_type(SpfftFloatGrid grid,
                                                           SpfftExchangeType* type);

/* Execute on `hipStream` (hipStream_t, NULL = legacy default stream).
 * synchronous = 0: return after enqueue. reset_stream: back to the private stream. */
SPFFT_EXPORT SpfftError spfft_amd_transform_set_stream(SpfftTransform transform, void* hipStream,
                                                       int synchronous);
SPFFT_EXPORT SpfftError spfft_amd_float_transform_set_stream(SpfftFloatTransform transform,
                                                             void* hipStream, int synchronous);
SPFFT_EXPORT SpfftError spfft_amd_transform_reset_stream(SpfftTransform transform);
SPFFT_EXPORT SpfftError spfft_amd_float_transform_reset_stream(SpfftFloatTransform transform);
SPFFT_EXPORT SpfftError spfft_amd_transform_synchronize(SpfftTransform transform);
SPFFT_EXPORT SpfftError spfft_amd_float_transform_synchronize(SpfftFloatTransform transform);
SPFFT_EXPORT SpfftError spfft_amd_transform_local_z_offset_rank(SpfftTransform transform, int rank,
                                                                int* offset, int* length);

/* Zero-copy DLPack export (DLManagedTensor*) of the space domain [localZ][Y][X];
 * the tensor keeps the transform and its grid alive until its deleter runs. */
SPFFT_EXPORT SpfftError spfft_amd_transform_space_domain_dlpack(SpfftTransform transform,
                                                                SpfftProcessingUnitType location,
                                                                void** managedTensor);
SPFFT_EXPORT SpfftError spfft_amd_float_transform_space_domain_dlpack(
    SpfftFloatTransform transform, SpfftProcessingUnitType location, void** managedTensor);

/* Step-wise execution (forward: xy, exchange, z; backward: z, exchange, xy). */
SPFFT_EXPORT SpfftError spfft_amd_transform_forward_xy(SpfftTransform t,
                                                       SpfftProcessingUnitType inputLocation);
SPFFT_EXPORT SpfftError spfft_amd_transform_forward_exchange(SpfftTransform t, int nonBlocking);
SPFFT_EXPORT SpfftError spfft_amd_transform_forward_z(SpfftTransform t, double* output,
                                                      SpfftScalingType scaling);
SPFFT_EXPORT SpfftError spfft_amd_transform_backward_z(SpfftTransform t, const double* input);
SPFFT_EXPORT SpfftError spfft_amd_transform_backward_exchange(SpfftTransform t, int nonBlocking);
SPFFT_EXPORT SpfftError spfft_amd_transform_backward_xy(SpfftTransform t,
                                                        SpfftProcessingUnitType outputLocation);
/* The same steps for single precision transforms. */
SPFFT_EXPORT SpfftError spfft_amd_float_transform_forward_xy(SpfftFloatTransform t,
                                                             SpfftProcessingUnitType inputLocation);
SPFFT_EXPORT SpfftError spfft_amd_float_transform_forward_exchange(SpfftFloatTransform t, int nonBlocking);
SPFFT_EXPORT SpfftError spfft_amd_float_transform_forward_z(SpfftFloatTransform t, float* output,
                                                            SpfftScalingType scaling);
SPFFT_EXPORT SpfftError spfft_amd_float_transform_backward_z(SpfftFloatTransform t, const float* input);
SPFFT_EXPORT SpfftError spfft_amd_float_transform_backward_exchange(SpfftFloatTransform t, int nonBlocking);
SPFFT_EXPORT SpfftError spfft_amd_float_transform_backward_xy(SpfftFloatTransform t,
                                                              SpfftProcessingUnitType outputLocation);

/* Timer tree (SPFFT_TIMING=1 or spfft_amd_timing_enable). enable: 0 off, 1 host
 * scopes only (like the reference's timer), 2 host scopes and GPU stage times
 * (a hipEvent per stage boundary, nodes gpu/<direction>/<stage>). */
SPFFT_EXPORT SpfftError spfft_amd_timing_enable(int enable);
SPFFT_EXPORT SpfftError spfft_amd_timing_reset(void);
/* Writes a JSON report into buffer (truncated to size-1); *required = full length + 1. */
SPFFT_EXPORT SpfftError spfft_amd_timing_json(char* buffer, size_t size, size_t* required);
SPFFT_EXPORT SpfftError spfft_amd_timing_print(char* buffer, size_t size, size_t* required);

/* Text of the last error raised in this thread (empty if none). */
SPFFT_EXPORT const char* spfft_amd_last_error_message(void);
/* Number of HIP devices visible (0 when no GPU runtime/device). */
SPFFT_EXPORT int spfft_amd_device_count(void);
/* Library build information ("gfx950", version, ...). */
SPFFT_EXPORT const char* spfft_amd_build_info(void);

#ifdef __cplusplus
}
#endif

#endif
