// GridImpl<T>: the memory arena + communicator shared by all transforms of a
// Grid (reference: src/spfft/grid_internal.{hpp,cpp}). Buffers are sized for the
// grid maxima so any transform up to those sizes runs without allocation.
#pragma once

#include <memory>
#include <mutex>

#include "core/common.hpp"
#include "core/host_buffer.hpp"
#include "core/thread_pool.hpp"
#include "spfft/communicator.hpp"
#include "spfft/types.h"

namespace spfft {

class DeviceBuffer;   // gpu/device_buffer.hpp
class DeviceComm;     // gpu/device_comm.hpp

// Largest row/stick padding (elements) a transform may add to its buffers.
constexpr int kMaxPad = 32;

// Row padding (elements) of the GPU stick rows and intermediate rows: n + pad
// elements of elemBytes make an odd multiple of 128 bytes, so every row starts
// on a cache line (a row that starts mid-line costs a partial line at each end:
// fp32 rows of 256 + 8 elements made the y and x stages read 1.5x their bytes,
// TCC_EA0_RDREQ in profiles/r4/pmc) and consecutive rows do not share a
// 256-byte channel stride. Short rows (< 1 KB) keep a pad of 8.
inline int aligned_row_pad(int n, int elemBytes) {
  const int line = 128 / elemBytes;
  if (static_cast<long long>(n) * elemBytes < 1024 || line < 1) return 8;
  for (int p = 0; p <= kMaxPad; ++p)
    if ((n + p) % line == 0 && ((n + p) / line) % 2 == 1) return p;
  return 8;
}

template <typename T>
class GridImpl {
public:
  // Local grid.
  GridImpl(int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns,
           SpfftProcessingUnitType pu, int numThreads);
  // Distributed grid (collective over comm).
  GridImpl(int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns, int maxLocalZLength,
           SpfftProcessingUnitType pu, int numThreads, std::shared_ptr<Communicator> comm,
           SpfftExchangeType exchangeType);
  // Deep copy: new buffers, duplicated communicator (collective if distributed).
  GridImpl(const GridImpl& other);
  ~GridImpl();

  int max_dim_x() const { return maxX_; }
  int max_dim_y() const { return maxY_; }
  int max_dim_z() const { return maxZ_; }
  int max_num_local_z_columns() const { return maxSticks_; }
  int max_local_z_length() const { return maxLocalZ_; }
  SpfftProcessingUnitType processing_unit() const { return pu_; }
  int device_id() const { return deviceId_; }
  int num_threads() const { return numThreads_; }
  SpfftExchangeType exchange_type() const { return exchange_; }
  bool local() const { return !comm_ || comm_->size() == 1; }
  const std::shared_ptr<Communicator>& communicator() const { return comm_; }

  ThreadPool& pool();

  // Buffer slots (complex<T> element counts fixed at construction).
  enum Slot { kStickSide = 0, kSlabSide = 1, kInter = 2, kSpace = 3, kNumSlots = 4 };
  i64 slot_elements(Slot s) const {
    if (s == kStickSide) return exchElems_;
    if (s == kSlabSide) return local() ? exchElems_ : slabElems_;
    return planeElems_;
  }
  // Device allocation of a slot. The [z][column][y] intermediate of the GPU
  // y/x stages is capped (SPFFT_INTER_BYTES, default 2 GiB, at least one
  // plane): larger slabs run the y/x stages in plane ranges that reuse it, so
  // a GPU grid holds the exchange sides (sized by sticks, tools/memory_model.py),
  // the space domain and a bounded intermediate (reference: 2 slab-sized
  // arrays, src/spfft/grid_internal.cpp:185-221).
  i64 device_slot_elements(Slot s) const { return s == kInter ? interDevElems_ : slot_elements(s); }

  // Host memory (allocated on first use; pinned if the grid has the GPU bit).
  void* host_slot(Slot s);
  // Device memory (GPU grids only).
  void* device_slot(Slot s);

  // Bytes of device memory the grid allocated (exchange sides, intermediate, space).
  std::size_t device_bytes() const;

  // RCCL / peer-copy data plane (GPU distributed grids), created on first use.
  DeviceComm& device_comm();

  // Transforms of one grid share buffers; execution is serialised by this lock.
  std::mutex& exec_mutex() { return execMutex_; }

private:
  void init(int maxDimX, int maxDimY, int maxDimZ, int maxSticks, int maxLocalZ,
            SpfftProcessingUnitType pu, int numThreads);
  void allocate_device();

  int maxX_ = 0, maxY_ = 0, maxZ_ = 0, maxSticks_ = 0, maxLocalZ_ = 0;
  SpfftProcessingUnitType pu_ = SPFFT_PU_HOST;
  int numThreads_ = 1;
  int deviceId_ = 0;
  SpfftExchangeType exchange_ = SPFFT_EXCH_COMPACT_BUFFERED;
  std::shared_ptr<Communicator> comm_;
  i64 exchElems_ = 0, slabElems_ = 0, planeElems_ = 0, interDevElems_ = 0;

  std::unique_ptr<ThreadPool> pool_;
  HostBuffer host_[kNumSlots];
  std::unique_ptr<DeviceBuffer> dev_[kNumSlots];
  std::unique_ptr<DeviceComm> devComm_;
  // exchange sides owned by the data plane (DeviceComm::local_buffer)
  void* sideOverride_[2] = {nullptr, nullptr};
  std::size_t sideOverrideBytes_[2] = {0, 0};
  std::mutex allocMutex_;
  std::mutex execMutex_;
};

}  // namespace spfft
