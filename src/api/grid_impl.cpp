#include "api/grid_impl.hpp"

#include <algorithm>
#include <cstdlib>
#include <climits>
#include <thread>
#include <vector>

#include "gpu/device_comm.hpp"
#include "gpu/gpu_runtime.hpp"
#include "spfft/exceptions.hpp"

namespace spfft {

namespace {
int resolve_threads(int n) {
  if (n >= 1) return n;
  const unsigned hw = std::thread::hardware_concurrency();
  return hw ? static_cast<int>(hw) : 1;
}
bool valid_pu(SpfftProcessingUnitType pu) { return (pu & (SPFFT_PU_HOST | SPFFT_PU_GPU)) != 0; }
}  // namespace

template <typename T>
void GridImpl<T>::init(int maxDimX, int maxDimY, int maxDimZ, int maxSticks, int maxLocalZ,
                       SpfftProcessingUnitType pu, int numThreads) {
  // argument checks (reference: grid_internal.cpp:60-66, 131-145)
  if (maxDimX <= 0 || maxDimY <= 0 || maxDimZ <= 0 || maxSticks < 0 || maxLocalZ < 0)
    throw InvalidParameterError();
  if (!valid_pu(pu)) throw InvalidParameterError();
  maxX_ = maxDimX;
  maxY_ = maxDimY;
  maxZ_ = maxDimZ;
  maxSticks_ = maxSticks;
  maxLocalZ_ = maxLocalZ;
  pu_ = pu;
  numThreads_ = resolve_threads(numThreads);
  // 64-bit sizes; the public API keeps int (reference quirk: int views, gpu_array_view.hpp:71)
  // room for row / stick padding (kMaxPad elements per row or stick)
  planeElems_ = checked_mul(checked_mul(maxX_, maxY_ + kMaxPad), std::max(1, maxLocalZ_));
  // exchange sides sized for what they hold, not for a slab (the reference
  // sizes both arrays max(Nx Ny Lmax, Nz Smax), grid_internal.cpp:198-202):
  // stick side = local sticks x (dimZ + pad); slab side (distributed) = all
  // ranks' sticks x local planes (set by the distributed constructor)
  exchElems_ = std::max<i64>(1, checked_mul(maxZ_ + kMaxPad, maxSticks_));
  slabElems_ = exchElems_;
  {
    const char* e = std::getenv("SPFFT_INTER_BYTES");
    const double capBytes = e && *e ? std::atof(e) : 2.0 * (1 << 30);
    const i64 onePlane = checked_mul(maxX_, maxY_ + kMaxPad);
    const i64 cap = static_cast<i64>(capBytes / (2.0 * sizeof(T)));
    interDevElems_ = std::min(planeElems_, std::max(onePlane, cap));
  }
  if (pu_ & SPFFT_PU_GPU) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
      (void)hipGetLastError();
      throw GPUNoDeviceError();
    }
    deviceId_ = current_device();
  }
}

template <typename T>
GridImpl<T>::GridImpl(int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns,
                      SpfftProcessingUnitType pu, int numThreads) {
  init(maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns, maxDimZ, pu, numThreads);
  if (pu_ & SPFFT_PU_GPU) allocate_device();
}

template <typename T>
GridImpl<T>::GridImpl(int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns,
                      int maxLocalZLength, SpfftProcessingUnitType pu, int numThreads,
                      std::shared_ptr<Communicator> comm, SpfftExchangeType exchangeType) {
  if (!comm) throw InvalidParameterError();
  comm_ = comm->duplicate();
  // local validation first, then a collective agreement on PU / exchange / errors
  // (reference: grid_internal.cpp:147-167) so no rank is left inside a collective.
  int status = 0;
  if (maxDimX <= 0 || maxDimY <= 0 || maxDimZ <= 0 || maxNumLocalZColumns < 0 ||
      maxLocalZLength < 0 || !valid_pu(pu))
    status = 1;
  if (exchangeType < SPFFT_EXCH_DEFAULT || exchangeType > SPFFT_EXCH_UNBUFFERED) status = 1;
  struct Info {
    int status, pu, exch, maxSticks, maxLocalZ;
  };
  Info mine{status, static_cast<int>(pu), static_cast<int>(exchangeType), maxNumLocalZColumns,
            maxLocalZLength};
  std::vector<Info> all(comm_->size());
  comm_->allgather(&mine, all.data(), sizeof(Info));
  int gMaxSticks = 0, gMaxLocalZ = 0;
  i64 sumSticks = 0;
  for (const auto& i : all) {
    if (i.status) {
      if (status) throw InvalidParameterError();
      throw MPIParameterMismatchError();
    }
    if (i.pu != mine.pu || i.exch != mine.exch) throw MPIParameterMismatchError();
    gMaxSticks = std::max(gMaxSticks, i.maxSticks);
    gMaxLocalZ = std::max(gMaxLocalZ, i.maxLocalZ);
    sumSticks += i.maxSticks;
  }
  exchange_ = exchangeType == SPFFT_EXCH_DEFAULT ? SPFFT_EXCH_COMPACT_BUFFERED : exchangeType;
  init(maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns, maxLocalZLength, pu, numThreads);
  if (comm_->size() > 1) {
    slabElems_ = std::max<i64>(1, checked_mul(sumSticks, std::max(1, maxLocalZ_)));
    if (is_exchange_buffered(exchange_)) {
      const i64 padded = checked_mul(checked_mul(gMaxSticks, gMaxLocalZ), comm_->size());
      exchElems_ = std::max(exchElems_, padded);
      slabElems_ = std::max(slabElems_, padded);
    }
  }
  if (pu_ & SPFFT_PU_GPU) allocate_device();
}

template <typename T>
GridImpl<T>::GridImpl(const GridImpl& o)
    : maxX_(o.maxX_),
      maxY_(o.maxY_),
      maxZ_(o.maxZ_),
      maxSticks_(o.maxSticks_),
      maxLocalZ_(o.maxLocalZ_),
      pu_(o.pu_),
      numThreads_(o.numThreads_),
      deviceId_(o.deviceId_),
      exchange_(o.exchange_),
      comm_(o.comm_ ? o.comm_->duplicate() : nullptr),
      exchElems_(o.exchElems_),
      slabElems_(o.slabElems_),
      planeElems_(o.planeElems_),
      interDevElems_(o.interDevElems_) {
  if (pu_ & SPFFT_PU_GPU) {
    DeviceGuard guard(deviceId_);
    allocate_device();
  }
}

template <typename T>
GridImpl<T>::~GridImpl() {
  if ((pu_ & SPFFT_PU_GPU) && !process_exiting()) {
    // release device resources on the grid's device
    try {
      DeviceGuard guard(deviceId_);
      devComm_.reset();  // (returns leased exchange sides to the IPC arena)
      for (auto& d : dev_) d.reset();
    } catch (...) {
    }
  }
}

template <typename T>
ThreadPool& GridImpl<T>::pool() {
  std::lock_guard<std::mutex> lock(allocMutex_);
  if (!pool_) pool_.reset(new ThreadPool(numThreads_));
  return *pool_;
}

template <typename T>
void GridImpl<T>::allocate_device() {
  const std::size_t cb = sizeof(T) * 2;
  dev_[kStickSide].reset(new DeviceBuffer(static_cast<std::size_t>(exchElems_) * cb));
  if (!local()) dev_[kSlabSide].reset(new DeviceBuffer(static_cast<std::size_t>(slabElems_) * cb));
  dev_[kInter].reset(new DeviceBuffer(static_cast<std::size_t>(interDevElems_) * cb));
  dev_[kSpace].reset(new DeviceBuffer(static_cast<std::size_t>(planeElems_) * cb));
}

template <typename T>
std::size_t GridImpl<T>::device_bytes() const {
  std::size_t b = 0;
  for (const auto& d : dev_)
    if (d) b += d->bytes();
  return b + sideOverrideBytes_[0] + sideOverrideBytes_[1];
}

template <typename T>
void* GridImpl<T>::host_slot(Slot s) {
  std::lock_guard<std::mutex> lock(allocMutex_);
  if (s == kSlabSide && local()) s = kStickSide;
  if (!host_[s].data()) {
    const std::size_t elems = static_cast<std::size_t>(slot_elements(s));
    host_[s].allocate(std::max<std::size_t>(1, elems) * sizeof(T) * 2, (pu_ & SPFFT_PU_GPU) != 0);
  }
  return host_[s].data();
}

template <typename T>
void* GridImpl<T>::device_slot(Slot s) {
  if (!(pu_ & SPFFT_PU_GPU)) throw InvalidParameterError();
  if (s == kSlabSide && local()) s = kStickSide;
  if (s <= kSlabSide && sideOverride_[s]) return sideOverride_[s];
  return dev_[s]->data();
}

template <typename T>
DeviceComm& GridImpl<T>::device_comm() {
  std::lock_guard<std::mutex> lock(allocMutex_);
  if (!devComm_) {
    void* const buffers[2] = {dev_[kStickSide] ? dev_[kStickSide]->data() : nullptr,
                              dev_[kSlabSide] ? dev_[kSlabSide]->data() : nullptr};
    const std::size_t bytes[2] = {dev_[kStickSide] ? dev_[kStickSide]->bytes() : 0,
                                  dev_[kSlabSide] ? dev_[kSlabSide]->bytes() : 0};
    devComm_ = DeviceComm::create(comm_, deviceId_, exchange_, buffers, bytes);
    // a data plane that owns the exchange sides (cross-process peer writes:
    // memory leased from the IPC arena) replaces the grid's own allocations
    for (int s = 0; s < 2; ++s) {
      if (void* p = devComm_->local_buffer(s)) {
        sideOverride_[s] = p;
        sideOverrideBytes_[s] = dev_[s] ? dev_[s]->bytes() : 0;
        dev_[s].reset();
      }
    }
  }
  return *devComm_;
}

template class GridImpl<double>;
template class GridImpl<float>;

}  // namespace spfft
