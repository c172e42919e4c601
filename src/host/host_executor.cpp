#include "host/host_executor.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "core/timing.hpp"
#include "spfft/exceptions.hpp"

namespace spfft {
namespace {

template <typename T>
inline bool nonzero(const cx<T>& v) {
  return v.x != T(0) || v.y != T(0);
}

// Hermitian completion of one line, only where the mirrored source is non-zero,
// in the two half passes of the reference (src/symmetry/symmetry_host.hpp:43-94).
template <typename T>
void hermitian_fill(cx<T>* v, int n) {
  for (int k = 1; k <= n / 2; ++k)
    if (nonzero(v[k])) v[n - k] = conj(v[k]);
  for (int k = n / 2 + 1; k < n; ++k)
    if (nonzero(v[k])) v[n - k] = conj(v[k]);
}

template <typename To, typename From>
inline cx<To> cvt(const cx<From>& v) {
  return mk<To>(static_cast<To>(v.x), static_cast<To>(v.y));
}

}  // namespace

template <typename T>
HostExecutor<T>::HostExecutor(std::shared_ptr<GridImpl<T>> grid,
                              std::shared_ptr<const IndexPlan> plan)
    : grid_(std::move(grid)), plan_(std::move(plan)) {
  const bool distributed = plan_->size > 1;
  layout_ = make_exchange_layout(*plan_, distributed && is_exchange_buffered(grid_->exchange_type()));
  floatExchange_ = distributed && is_exchange_float(grid_->exchange_type());
  if (layout_.stickTotal > grid_->slot_elements(GridImpl<T>::kStickSide) ||
      layout_.slabTotal > grid_->slot_elements(GridImpl<T>::kSlabSide))
    throw InvalidParameterError();
  fftX_ = HostFft<T>(plan_->dimX);
  fftY_ = HostFft<T>(plan_->dimY);
  fftZ_ = HostFft<T>(plan_->dimZ);
  scratch_.resize(grid_->pool().num_threads());
}

template <typename T>
cx<T>* HostExecutor<T>::scratch(int thread, std::size_t n) {
  auto& s = scratch_[thread];
  if (s.size() < n) s.resize(n);
  return s.data();
}

// ---------------------------------------------------------------- backward
template <typename T>
template <typename BT>
void HostExecutor<T>::z_backward(const cx<T>* values, BT* stick) {
  const IndexPlan& p = *plan_;
  const int Z = p.dimZ;
  const bool r2c = p.type == SPFFT_TRANS_R2C;
  grid_->pool().parallel_for(p.local_sticks(), 16, [&](i64 b, i64 e, int t) {
    cx<T>* buf = scratch(t, static_cast<std::size_t>(Z) + fftZ_.scratch_size());
    cx<T>* fs = buf + Z;
    for (i64 s = b; s < e; ++s) {
      std::fill(buf, buf + Z, mk<T>(T(0), T(0)));
      for (int q = p.stickRunOffsets[s]; q < p.stickRunOffsets[s + 1]; ++q) {
        const StickRun& r = p.runs[q];
        std::copy(values + r.valueStart, values + r.valueStart + r.length, buf + r.zStart);
      }
      if (r2c && s == p.zeroStick) hermitian_fill(buf, Z);
      fftZ_.execute(buf, 1, buf, 1, +1, fs);
      for (int r = 0; r < p.size; ++r) {
        BT* dst = stick + layout_.stickDispl[r] + s * layout_.stickStride[r];
        const cx<T>* src = buf + p.planeOffsets[r];
        for (int z = 0; z < p.planesPerRank[r]; ++z) dst[z] = cvt<typename BT::value_type>(src[z]);
      }
    }
  });
}

template <typename T>
template <typename BT>
void HostExecutor<T>::y_backward(const BT* slab, cx<T>* inter) {
  const IndexPlan& p = *plan_;
  const int Y = p.dimY, L = p.local_planes(), C = p.num_columns();
  const bool r2c = p.type == SPFFT_TRANS_R2C;
  grid_->pool().parallel_for(static_cast<i64>(C) * L, std::max(1, L / 4), [&](i64 b, i64 e, int t) {
    cx<T>* col = scratch(t, static_cast<std::size_t>(Y) + fftY_.scratch_size());
    cx<T>* fs = col + Y;
    for (i64 task = b; task < e; ++task) {
      const int c = static_cast<int>(task / L), zl = static_cast<int>(task % L);
      std::fill(col, col + Y, mk<T>(T(0), T(0)));
      for (int k = p.colOffsets[c]; k < p.colOffsets[c + 1]; ++k)
        col[p.colY[k]] = cvt<T>(slab[layout_.colEntryBase[k] + zl]);
      if (r2c && c == p.colOfX0) hermitian_fill(col, Y);
      fftY_.execute(col, 1, inter + (static_cast<i64>(zl) * C + c) * Y, 1, +1, fs);
    }
  });
}

template <typename T>
void HostExecutor<T>::x_backward(const cx<T>* inter, T* space) {
  const IndexPlan& p = *plan_;
  const int X = p.dimX, Y = p.dimY, L = p.local_planes(), C = p.num_columns();
  const bool r2c = p.type == SPFFT_TRANS_R2C;
  grid_->pool().parallel_for(static_cast<i64>(L) * Y, 16, [&](i64 b, i64 e, int t) {
    cx<T>* row = scratch(t, static_cast<std::size_t>(X) + fftX_.scratch_size());
    cx<T>* fs = row + X;
    for (i64 rIdx = b; rIdx < e; ++rIdx) {
      const i64 zl = rIdx / Y, y = rIdx % Y;
      std::fill(row, row + X, mk<T>(T(0), T(0)));
      for (int c = 0; c < C; ++c) row[p.colX[c]] = inter[(zl * C + c) * Y + y];
      if (!r2c) {
        fftX_.execute(row, 1, reinterpret_cast<cx<T>*>(space) + rIdx * X, 1, +1, fs);
      } else {
        for (int x = p.dimXFreq; x < X; ++x) row[x] = conj(row[X - x]);
        fftX_.execute(row, 1, row, 1, +1, fs);
        T* out = space + rIdx * X;
        for (int x = 0; x < X; ++x) out[x] = row[x].x;
      }
    }
  });
}

// ----------------------------------------------------------------- forward
template <typename T>
void HostExecutor<T>::x_forward(const T* space, cx<T>* inter) {
  const IndexPlan& p = *plan_;
  const int X = p.dimX, Y = p.dimY, L = p.local_planes(), C = p.num_columns();
  const bool r2c = p.type == SPFFT_TRANS_R2C;
  grid_->pool().parallel_for(static_cast<i64>(L) * Y, 16, [&](i64 b, i64 e, int t) {
    cx<T>* row = scratch(t, static_cast<std::size_t>(X) + fftX_.scratch_size());
    cx<T>* fs = row + X;
    for (i64 rIdx = b; rIdx < e; ++rIdx) {
      const i64 zl = rIdx / Y, y = rIdx % Y;
      if (!r2c) {
        fftX_.execute(reinterpret_cast<const cx<T>*>(space) + rIdx * X, 1, row, 1, -1, fs);
      } else {
        const T* in = space + rIdx * X;
        for (int x = 0; x < X; ++x) row[x] = mk<T>(in[x], T(0));
        fftX_.execute(row, 1, row, 1, -1, fs);
      }
      for (int c = 0; c < C; ++c) inter[(zl * C + c) * Y + y] = row[p.colX[c]];
    }
  });
}

template <typename T>
template <typename BT>
void HostExecutor<T>::y_forward(const cx<T>* inter, BT* slab) {
  const IndexPlan& p = *plan_;
  const int Y = p.dimY, L = p.local_planes(), C = p.num_columns();
  grid_->pool().parallel_for(static_cast<i64>(C) * L, std::max(1, L / 4), [&](i64 b, i64 e, int t) {
    cx<T>* col = scratch(t, static_cast<std::size_t>(Y) + fftY_.scratch_size());
    cx<T>* fs = col + Y;
    for (i64 task = b; task < e; ++task) {
      const int c = static_cast<int>(task / L), zl = static_cast<int>(task % L);
      fftY_.execute(inter + (static_cast<i64>(zl) * C + c) * Y, 1, col, 1, -1, fs);
      for (int k = p.colOffsets[c]; k < p.colOffsets[c + 1]; ++k)
        slab[layout_.colEntryBase[k] + zl] = cvt<typename BT::value_type>(col[p.colY[k]]);
    }
  });
}

template <typename T>
template <typename BT>
void HostExecutor<T>::z_forward(const BT* stick, cx<T>* values, T factor) {
  const IndexPlan& p = *plan_;
  const int Z = p.dimZ;
  grid_->pool().parallel_for(p.local_sticks(), 16, [&](i64 b, i64 e, int t) {
    cx<T>* buf = scratch(t, static_cast<std::size_t>(Z) + fftZ_.scratch_size());
    cx<T>* fs = buf + Z;
    for (i64 s = b; s < e; ++s) {
      for (int r = 0; r < p.size; ++r) {
        const BT* src = stick + layout_.stickDispl[r] + s * layout_.stickStride[r];
        cx<T>* dst = buf + p.planeOffsets[r];
        for (int z = 0; z < p.planesPerRank[r]; ++z) dst[z] = cvt<T>(src[z]);
      }
      fftZ_.execute(buf, 1, buf, 1, -1, fs);
      for (int q = p.stickRunOffsets[s]; q < p.stickRunOffsets[s + 1]; ++q) {
        const StickRun& r = p.runs[q];
        for (int j = 0; j < r.length; ++j) values[r.valueStart + j] = scale(buf[r.zStart + j], factor);
      }
    }
  });
}

// ------------------------------------------------------------------ stages
// SPFFT_POISON=1: NaN-fill the work buffers a direction writes before reading
// them (debug aid; see GpuExecutor::poison).
template <typename T>
void HostExecutor<T>::poison(bool backward) {
  const char* env = std::getenv("SPFFT_POISON");
  if (!env || env[0] != '1') return;
  auto fill = [&](typename GridImpl<T>::Slot slot) {
    std::memset(grid_->host_slot(slot), 0xFF,
                static_cast<std::size_t>(grid_->slot_elements(slot)) * sizeof(cx<T>));
  };
  fill(GridImpl<T>::kStickSide);
  fill(GridImpl<T>::kInter);
  if (plan_->size > 1) fill(GridImpl<T>::kSlabSide);
  if (backward) fill(GridImpl<T>::kSpace);
}

template <typename T>
void HostExecutor<T>::backward_z(const T* input) {
  SPFFT_TIMED_SCOPE("backward_z");
  poison(true);
  void* stick = grid_->host_slot(GridImpl<T>::kStickSide);
  const auto* values = reinterpret_cast<const cx<T>*>(input);
  if (plan_->numLocalElements > 0 && !input) throw InvalidParameterError();
  if (floatExchange_)
    z_backward(values, static_cast<cx<float>*>(stick));
  else
    z_backward(values, static_cast<cx<T>*>(stick));
}

template <typename T>
void HostExecutor<T>::exchange(bool backward) {
  if (plan_->size <= 1) return;
  const std::size_t elemBytes = floatExchange_ ? sizeof(cx<float>) : sizeof(cx<T>);
  const int P = plan_->size;
  std::vector<std::size_t> sc(P), sd(P), rc(P), rd(P);
  for (int r = 0; r < P; ++r) {
    const std::size_t stickC = layout_.stickCount[r] * elemBytes, stickD = layout_.stickDispl[r] * elemBytes;
    const std::size_t slabC = layout_.slabCount[r] * elemBytes, slabD = layout_.slabDispl[r] * elemBytes;
    if (backward) {
      sc[r] = stickC, sd[r] = stickD, rc[r] = slabC, rd[r] = slabD;
    } else {
      sc[r] = slabC, sd[r] = slabD, rc[r] = stickC, rd[r] = stickD;
    }
  }
  void* stick = grid_->host_slot(GridImpl<T>::kStickSide);
  void* slab = grid_->host_slot(GridImpl<T>::kSlabSide);
  if (backward)
    grid_->communicator()->alltoallv(stick, sc.data(), sd.data(), slab, rc.data(), rd.data());
  else
    grid_->communicator()->alltoallv(slab, sc.data(), sd.data(), stick, rc.data(), rd.data());
}

template <typename T>
void HostExecutor<T>::backward_exchange() {
  SPFFT_TIMED_SCOPE("backward_exchange");
  exchange(true);
}

template <typename T>
void HostExecutor<T>::backward_xy() {
  SPFFT_TIMED_SCOPE("backward_xy");
  const bool dist = plan_->size > 1;
  void* slab = grid_->host_slot(dist ? GridImpl<T>::kSlabSide : GridImpl<T>::kStickSide);
  auto* inter = static_cast<cx<T>*>(grid_->host_slot(GridImpl<T>::kInter));
  if (floatExchange_)
    y_backward(static_cast<const cx<float>*>(slab), inter);
  else
    y_backward(static_cast<const cx<T>*>(slab), inter);
  x_backward(inter, space_domain());
}

template <typename T>
void HostExecutor<T>::forward_xy() {
  SPFFT_TIMED_SCOPE("forward_xy");
  poison(false);
  const bool dist = plan_->size > 1;
  auto* inter = static_cast<cx<T>*>(grid_->host_slot(GridImpl<T>::kInter));
  x_forward(space_domain(), inter);
  void* slab = grid_->host_slot(dist ? GridImpl<T>::kSlabSide : GridImpl<T>::kStickSide);
  if (floatExchange_)
    y_forward(inter, static_cast<cx<float>*>(slab));
  else
    y_forward(inter, static_cast<cx<T>*>(slab));
}

template <typename T>
void HostExecutor<T>::forward_exchange() {
  SPFFT_TIMED_SCOPE("forward_exchange");
  exchange(false);
}

template <typename T>
void HostExecutor<T>::forward_z(T* output, SpfftScalingType scaling) {
  SPFFT_TIMED_SCOPE("forward_z");
  if (plan_->numLocalElements > 0 && !output) throw InvalidParameterError();
  const T factor =
      scaling == SPFFT_FULL_SCALING
          ? static_cast<T>(1.0 / (static_cast<double>(plan_->dimX) * plan_->dimY * plan_->dimZ))
          : T(1);
  void* stick = grid_->host_slot(GridImpl<T>::kStickSide);
  auto* values = reinterpret_cast<cx<T>*>(output);
  if (floatExchange_)
    z_forward(static_cast<const cx<float>*>(stick), values, factor);
  else
    z_forward(static_cast<const cx<T>*>(stick), values, factor);
}

template class HostExecutor<double>;
template class HostExecutor<float>;

}  // namespace spfft
