#include "host/host_executor.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "core/timing.hpp"
#include "spfft/exceptions.hpp"

namespace spfft {
namespace {

template <typename T>
inline bool nonzero(const cx<T>& v) {
  return v.x != T(0) || v.y != T(0);
}

template <typename To, typename From>
inline cx<To> cvt(const cx<From>& v) {
  return mk<To>(static_cast<To>(v.x), static_cast<To>(v.y));
}

// Hermitian completion of lane l of a batch line, only where the mirrored
// source is non-zero, in the two half passes of the reference
// (src/symmetry/symmetry_host.hpp:43-94).
template <typename T>
void hermitian_lane(typename HostSimd<T>::VC* a, int n, int l) {
  for (int k = 1; k <= n / 2; ++k) {
    const cx<T> v = lane<T>(a[k], l);
    if (nonzero(v)) set_lane<T>(a[n - k], l, conj(v));
  }
  for (int k = n / 2 + 1; k < n; ++k) {
    const cx<T> v = lane<T>(a[k], l);
    if (nonzero(v)) set_lane<T>(a[n - k], l, conj(v));
  }
}

}  // namespace

template <typename T>
HostExecutor<T>::HostExecutor(std::shared_ptr<GridImpl<T>> grid,
                              std::shared_ptr<const IndexPlan> plan)
    : grid_(std::move(grid)), plan_(std::move(plan)) {
  const IndexPlan& p = *plan_;
  const bool distributed = p.size > 1;
  layout_ = make_exchange_layout(p, distributed && is_exchange_buffered(grid_->exchange_type()));
  floatExchange_ = distributed && is_exchange_float(grid_->exchange_type());
  unbuffered_ = distributed && grid_->exchange_type() == SPFFT_EXCH_UNBUFFERED;
  if (unbuffered_) {
    // UNBUFFERED: the stick side keeps the natural [stick][z] layout (the z
    // stage writes whole sticks) and the exchange gathers each rank's planes
    // out of it with strided datatypes (Communicator::alltoallw)
    const i64 S = p.local_sticks();
    for (int r = 0; r < p.size; ++r) {
      layout_.stickDispl[r] = p.planeOffsets[r];
      layout_.stickStride[r] = p.dimZ;
      layout_.stickCount[r] = S * p.planesPerRank[r];
    }
    layout_.stickTotal = S * p.dimZ;
  }
  if (layout_.stickTotal > grid_->slot_elements(GridImpl<T>::kStickSide) ||
      layout_.slabTotal > grid_->slot_elements(GridImpl<T>::kSlabSide))
    throw InvalidParameterError();
  // packed-real x stage (R2C, even dimX): one half-length complex FFT per row
  packedReal_ = p.type == SPFFT_TRANS_R2C && p.dimX % 2 == 0 && p.dimX >= 2;
  fftX_ = Fft(packedReal_ ? p.dimX / 2 : p.dimX);
  fftY_ = Fft(p.dimY);
  fftZ_ = Fft(p.dimZ);
  twX_ = make_twiddles<T>(p.dimX);
  // fused y/x per plane block when the blocks keep every thread busy and the
  // block buffer stays cache-sized (SPFFT_HOST_FUSE=0/1 forces)
  {
    const int threads = grid_->pool().num_threads();
    const i64 blocks = (p.local_planes() + W - 1) / W;
    const std::size_t blockBytes = static_cast<std::size_t>(p.num_columns()) * p.dimY * sizeof(VC);
    fuseXY_ = blocks >= 2 * threads && blockBytes <= (std::size_t(8) << 20);
    const char* e = std::getenv("SPFFT_HOST_FUSE");
    if (e && *e) fuseXY_ = e[0] == '1';
  }
  scratch_.resize(grid_->pool().num_threads());
}

template <typename T>
typename HostExecutor<T>::VC* HostExecutor<T>::scratch(int thread, std::size_t n) {
  auto& s = scratch_[thread];
  if (s.size() < n) s.resize(n);
  return s.data();
}

// W lines of a batch through `f` (a: n batch elements, b: n scratch elements;
// every length runs batched, Bluestein lengths included).
template <typename T>
void HostExecutor<T>::fft(const Fft& f, VC* a, VC* b, int /*nl*/, int sign) {
  f.run(a, b, sign);
}

// ---------------------------------------------------------------- backward
template <typename T>
template <typename BT>
void HostExecutor<T>::z_backward(const cx<T>* values, BT* stick) {
  SPFFT_TIMED_SCOPE("z_fft");
  const IndexPlan& p = *plan_;
  const int Z = p.dimZ;
  const bool r2c = p.type == SPFFT_TRANS_R2C;
  const i64 S = p.local_sticks();
  grid_->pool().parallel_for((S + W - 1) / W, 4, [&](i64 b, i64 e, int t) {
    VC* a = scratch(t, block_scratch());
    VC* w = a + Z;
    for (i64 blk = b; blk < e; ++blk) {
      const i64 s0 = blk * W;
      const int nl = static_cast<int>(std::min<i64>(W, S - s0));
      std::fill(a, a + Z, vzero<T>());
      for (int l = 0; l < nl; ++l) {
        const i64 s = s0 + l;
        for (int q = p.stickRunOffsets[s]; q < p.stickRunOffsets[s + 1]; ++q) {
          const StickRun& r = p.runs[q];
          for (int j = 0; j < r.length; ++j) set_lane<T>(a[r.zStart + j], l, values[r.valueStart + j]);
        }
        if (r2c && s == p.zeroStick) hermitian_lane<T>(a, Z, l);
      }
      fft(fftZ_, a, w, nl, +1);
      for (int l = 0; l < nl; ++l) {
        const i64 s = s0 + l;
        for (int r = 0; r < p.size; ++r) {
          BT* dst = stick + layout_.stickDispl[r] + s * layout_.stickStride[r];
          const VC* src = a + p.planeOffsets[r];
          for (int z = 0; z < p.planesPerRank[r]; ++z)
            dst[z] = cvt<typename BT::value_type>(lane<T>(src[z], l));
        }
      }
    }
  });
}

// ------------------------------------------------------- y and x line sets
// Column c's y-lines of planes z0 .. z0+nl-1 (one batch) from the slab side:
// a stick entry's W plane values are contiguous there. Result in a[0..Y).
template <typename T>
template <typename BT>
void HostExecutor<T>::y_col_backward(const BT* slab, int c, int z0, int nl, VC* a, VC* w) {
  const IndexPlan& p = *plan_;
  const int Y = p.dimY;
  std::fill(a, a + Y, vzero<T>());
  for (int k = p.colOffsets[c]; k < p.colOffsets[c + 1]; ++k) {
    const BT* src = slab + layout_.colEntryBase[k] + z0;
    VC& d = a[p.colY[k]];
    if (std::is_same<BT, cx<T>>::value && nl == W)
      d = load_aos<T>(reinterpret_cast<const cx<T>*>(src));
    else
      for (int l = 0; l < nl; ++l) set_lane<T>(d, l, cvt<T>(src[l]));
  }
  if (p.type == SPFFT_TRANS_R2C && c == p.colOfX0)
    for (int l = 0; l < nl; ++l) hermitian_lane<T>(a, Y, l);
  fft(fftY_, a, w, nl, +1);
}

// Column c's y-lines (a[0..Y), forward-transformed in place) -> slab side.
template <typename T>
template <typename BT>
void HostExecutor<T>::y_col_forward(VC* a, int c, int z0, int nl, BT* slab, VC* w) {
  const IndexPlan& p = *plan_;
  fft(fftY_, a, w, nl, -1);
  for (int k = p.colOffsets[c]; k < p.colOffsets[c + 1]; ++k) {
    BT* dst = slab + layout_.colEntryBase[k] + z0;
    const VC& v = a[p.colY[k]];
    if (std::is_same<BT, cx<T>>::value && nl == W)
      store_aos<T>(reinterpret_cast<cx<T>*>(dst), v);
    else
      for (int l = 0; l < nl; ++l) dst[l] = cvt<typename BT::value_type>(lane<T>(v, l));
  }
}

// nl space rows (row l starts at rows[l]) from their column values col(c)
// (batch elements, lanes = rows): x-FFT C2C, packed-real C2R, or complex C2R.
// a: X+1 elements, w: 2X+1 elements of scratch.
template <typename T>
template <class Col>
void HostExecutor<T>::x_rows_backward(Col col, int nl, T* const* rows, VC* a, VC* w) {
  const IndexPlan& p = *plan_;
  const int X = p.dimX, C = p.num_columns();
  const int n = fftX_.size();
  VC* xv = packedReal_ ? w + X : a;  // X[x] for x in [0, dimXFreq)
  std::fill(xv, xv + (packedReal_ ? n + 1 : X), vzero<T>());
  for (int c = 0; c < C; ++c) xv[p.colX[c]] = col(c);
  if (p.type != SPFFT_TRANS_R2C) {
    fft(fftX_, a, w, nl, +1);
    for (int l = 0; l < nl; ++l) {
      cx<T>* out = reinterpret_cast<cx<T>*>(rows[l]);
      for (int x = 0; x < X; ++x) out[x] = lane<T>(a[x], l);
    }
  } else if (packedReal_) {
    // C2R as a half-length complex FFT: Z[k] = (X[k] + conj X[h-k]) +
    // i (X[k] - conj X[h-k]) w^k, w = exp(+2 pi i / X); imaginary parts of
    // X[0] and X[h] ignored; row = interleave(Re, Im) of IDFT_h(Z)
    const int h = n;
    for (int k = 0; k < h; ++k) {
      VC xk = xv[k], xm = xv[h - k];
      if (k == 0) {
        xk.y = V(T(0));
        xm.y = V(T(0));
      }
      VC xmc = xm;
      xmc.y = -xm.y;
      const VC sm = xk + xmc, d = xk - xmc;
      const VC dw = twv<+1>(d, twX_[k]);  // d * exp(+2 pi i k / X)
      VC z;
      z.x = sm.x - dw.y;
      z.y = sm.y + dw.x;
      a[k] = z;
    }
    fft(fftX_, a, w, nl, +1);
    for (int l = 0; l < nl; ++l) {
      cx<T>* out = reinterpret_cast<cx<T>*>(rows[l]);  // (x[2m], x[2m+1]) pairs
      for (int m = 0; m < h; ++m) out[m] = lane<T>(a[m], l);
    }
  } else {
    for (int x = p.dimXFreq; x < X; ++x) {
      a[x] = a[X - x];
      a[x].y = -a[x].y;
    }
    fft(fftX_, a, w, nl, +1);
    for (int l = 0; l < nl; ++l)
      for (int x = 0; x < X; ++x) rows[l][x] = lane<T>(a[x], l).x;
  }
}

// nl space rows -> column values put(c, batch element) (lanes = rows).
template <typename T>
template <class Put>
void HostExecutor<T>::x_rows_forward(const T* const* rows, int nl, Put put, VC* a, VC* w) {
  const IndexPlan& p = *plan_;
  const int X = p.dimX, C = p.num_columns();
  const int n = fftX_.size();
  if (nl < W) std::fill(a, a + n + 1, vzero<T>());
  if (p.type != SPFFT_TRANS_R2C) {
    for (int l = 0; l < nl; ++l) {
      const cx<T>* in = reinterpret_cast<const cx<T>*>(rows[l]);
      for (int x = 0; x < X; ++x) set_lane<T>(a[x], l, in[x]);
    }
    fft(fftX_, a, w, nl, -1);
    for (int c = 0; c < C; ++c) put(c, a[p.colX[c]]);
  } else if (packedReal_) {
    // R2C as a half-length complex FFT of y[m] = x[2m] + i x[2m+1]:
    // X[k] = (Y[k] + conj Y[h-k]) / 2 + w^k (Y[k] - conj Y[h-k]) / (2i),
    // w = exp(-2 pi i / X), Y[h] = Y[0]
    const int h = n;
    for (int l = 0; l < nl; ++l) {
      const cx<T>* in = reinterpret_cast<const cx<T>*>(rows[l]);
      for (int m = 0; m < h; ++m) set_lane<T>(a[m], l, in[m]);
    }
    fft(fftX_, a, w, nl, -1);
    for (int c = 0; c < C; ++c) {
      const int k = p.colX[c];
      const VC yk = a[k == h ? 0 : k];
      VC ym = a[k == 0 ? 0 : h - k];
      ym.y = -ym.y;
      VC ev = yk + ym;
      ev.x *= T(0.5);
      ev.y *= T(0.5);
      const VC dd = yk - ym;
      VC o;  // (yk - ym) / (2i)
      o.x = dd.y * T(0.5);
      o.y = -dd.x * T(0.5);
      put(c, ev + twv<-1>(o, twX_[k]));
    }
  } else {
    for (int l = 0; l < nl; ++l)
      for (int x = 0; x < X; ++x) set_lane<T>(a[x], l, mk<T>(rows[l][x], T(0)));
    fft(fftX_, a, w, nl, -1);
    for (int c = 0; c < C; ++c) put(c, a[p.colX[c]]);
  }
}

// Fused y/x stages (fuseXY_): a task is a block of W planes; its y-lines of
// every column are transformed into a cache-resident plane-block buffer
// (columns x y, lanes = planes) and the x-lines of every row read it from
// there, so the intermediate never goes to memory (the host's DRAM bandwidth
// per core, not the FFT arithmetic, bounds the separate stages).
template <typename T>
std::size_t HostExecutor<T>::block_scratch() const {
  const IndexPlan& p = *plan_;
  const std::size_t X = p.dimX, Y = p.dimY, Z = p.dimZ;
  const std::size_t line = std::max({X, Y, Z});
  return (fuseXY_ ? static_cast<std::size_t>(p.num_columns()) * block_stride() : 0) + 4 * line + 8;
}

// ---------------------------------------------------------------- backward
template <typename T>
template <typename BT>
void HostExecutor<T>::yx_backward(const BT* slab, cx<T>* inter, T* space) {
  const IndexPlan& p = *plan_;
  const int X = p.dimX, Y = p.dimY, L = p.local_planes(), C = p.num_columns();
  const bool r2c = p.type == SPFFT_TRANS_R2C;
  const i64 nb = (L + W - 1) / W;
  auto row = [&](i64 z, i64 y) -> T* {
    return r2c ? space + (z * Y + y) * X : reinterpret_cast<T*>(reinterpret_cast<cx<T>*>(space) + (z * Y + y) * X);
  };
  if (fuseXY_) {
    SPFFT_TIMED_SCOPE("yx_fft");
    grid_->pool().parallel_for(nb, 1, [&](i64 b, i64 e, int t) {
      VC* P = scratch(t, block_scratch());
      const i64 ps = block_stride();
      VC* a = P + static_cast<std::size_t>(C) * ps;
      VC* w = a + X + 1;
      for (i64 zb = b; zb < e; ++zb) {
        const int z0 = static_cast<int>(zb) * W;
        const int nl = std::min(W, L - z0);
        for (int c = 0; c < C; ++c) y_col_backward(slab, c, z0, nl, P + c * ps, w);
        T* rows[W];
        for (int y = 0; y < Y; ++y) {
          for (int l = 0; l < nl; ++l) rows[l] = row(z0 + l, y);
          x_rows_backward([&](int c) { return P[c * ps + y]; }, nl, rows, a, w);
        }
      }
    });
    return;
  }
  {
    SPFFT_TIMED_SCOPE("y_fft");
    grid_->pool().parallel_for(C * nb, 4, [&](i64 b, i64 e, int t) {
      VC* a = scratch(t, block_scratch());
      VC* w = a + Y;
      for (i64 task = b; task < e; ++task) {
        const int c = static_cast<int>(task / nb);
        const int z0 = static_cast<int>(task % nb) * W;
        const int nl = std::min(W, L - z0);
        y_col_backward(slab, c, z0, nl, a, w);
        for (int l = 0; l < nl; ++l) {
          cx<T>* out = inter + (static_cast<i64>(z0 + l) * C + c) * Y;
          for (int y = 0; y < Y; ++y) out[y] = lane<T>(a[y], l);
        }
      }
    });
  }
  SPFFT_TIMED_SCOPE("x_fft");
  // task = (plane, block of W consecutive rows): a column's W values are
  // contiguous in the [z][column][y] intermediate
  const i64 yb = (Y + W - 1) / W;
  grid_->pool().parallel_for(static_cast<i64>(L) * yb, 4, [&](i64 b, i64 e, int t) {
    VC* a = scratch(t, block_scratch());
    VC* w = a + X + 1;
    for (i64 task = b; task < e; ++task) {
      const i64 zl = task / yb;
      const int y0 = static_cast<int>(task % yb) * W;
      const int nl = std::min(W, Y - y0);
      T* rows[W];
      for (int l = 0; l < nl; ++l) rows[l] = row(zl, y0 + l);
      x_rows_backward([&](int c) {
        const cx<T>* src = inter + (zl * C + c) * Y + y0;
        if (nl == W) return load_aos<T>(src);
        VC v = vzero<T>();
        for (int l = 0; l < nl; ++l) set_lane<T>(v, l, src[l]);
        return v;
      }, nl, rows, a, w);
    }
  });
}

// ----------------------------------------------------------------- forward
template <typename T>
template <typename BT>
void HostExecutor<T>::xy_forward(const T* space, cx<T>* inter, BT* slab) {
  const IndexPlan& p = *plan_;
  const int X = p.dimX, Y = p.dimY, L = p.local_planes(), C = p.num_columns();
  const bool r2c = p.type == SPFFT_TRANS_R2C;
  const i64 nb = (L + W - 1) / W;
  auto row = [&](i64 z, i64 y) -> const T* {
    return r2c ? space + (z * Y + y) * X
               : reinterpret_cast<const T*>(reinterpret_cast<const cx<T>*>(space) + (z * Y + y) * X);
  };
  if (fuseXY_) {
    SPFFT_TIMED_SCOPE("xy_fft");
    grid_->pool().parallel_for(nb, 1, [&](i64 b, i64 e, int t) {
      VC* P = scratch(t, block_scratch());
      const i64 ps = block_stride();
      VC* a = P + static_cast<std::size_t>(C) * ps;
      VC* w = a + X + 1;
      for (i64 zb = b; zb < e; ++zb) {
        const int z0 = static_cast<int>(zb) * W;
        const int nl = std::min(W, L - z0);
        const T* rows[W];
        for (int y = 0; y < Y; ++y) {
          for (int l = 0; l < nl; ++l) rows[l] = row(z0 + l, y);
          x_rows_forward(rows, nl, [&](int c, const VC& v) { P[c * ps + y] = v; }, a, w);
        }
        for (int c = 0; c < C; ++c) y_col_forward(P + c * ps, c, z0, nl, slab, w);
      }
    });
    return;
  }
  {
    SPFFT_TIMED_SCOPE("x_fft");
    const i64 yb = (Y + W - 1) / W;
    grid_->pool().parallel_for(static_cast<i64>(L) * yb, 4, [&](i64 b, i64 e, int t) {
      VC* a = scratch(t, block_scratch());
      VC* w = a + X + 1;
      for (i64 task = b; task < e; ++task) {
        const i64 zl = task / yb;
        const int y0 = static_cast<int>(task % yb) * W;
        const int nl = std::min(W, Y - y0);
        const T* rows[W];
        for (int l = 0; l < nl; ++l) rows[l] = row(zl, y0 + l);
        x_rows_forward(rows, nl, [&](int c, const VC& v) {
          cx<T>* dst = inter + (zl * C + c) * Y + y0;
          if (nl == W)
            store_aos<T>(dst, v);
          else
            for (int l = 0; l < nl; ++l) dst[l] = lane<T>(v, l);
        }, a, w);
      }
    });
  }
  SPFFT_TIMED_SCOPE("y_fft");
  grid_->pool().parallel_for(C * nb, 4, [&](i64 b, i64 e, int t) {
    VC* a = scratch(t, block_scratch());
    VC* w = a + Y;
    for (i64 task = b; task < e; ++task) {
      const int c = static_cast<int>(task / nb);
      const int z0 = static_cast<int>(task % nb) * W;
      const int nl = std::min(W, L - z0);
      if (nl < W) std::fill(a, a + Y, vzero<T>());
      for (int l = 0; l < nl; ++l) {
        const cx<T>* in = inter + (static_cast<i64>(z0 + l) * C + c) * Y;
        for (int y = 0; y < Y; ++y) set_lane<T>(a[y], l, in[y]);
      }
      y_col_forward(a, c, z0, nl, slab, w);
    }
  });
}

template <typename T>
template <typename BT>
void HostExecutor<T>::z_forward(const BT* stick, cx<T>* values, T factor) {
  SPFFT_TIMED_SCOPE("z_fft");
  const IndexPlan& p = *plan_;
  const int Z = p.dimZ;
  const i64 S = p.local_sticks();
  grid_->pool().parallel_for((S + W - 1) / W, 4, [&](i64 b, i64 e, int t) {
    VC* a = scratch(t, block_scratch());
    VC* w = a + Z;
    for (i64 blk = b; blk < e; ++blk) {
      const i64 s0 = blk * W;
      const int nl = static_cast<int>(std::min<i64>(W, S - s0));
      if (nl < W) std::fill(a, a + Z, vzero<T>());
      for (int l = 0; l < nl; ++l) {
        const i64 s = s0 + l;
        for (int r = 0; r < p.size; ++r) {
          const BT* src = stick + layout_.stickDispl[r] + s * layout_.stickStride[r];
          VC* dst = a + p.planeOffsets[r];
          for (int z = 0; z < p.planesPerRank[r]; ++z) set_lane<T>(dst[z], l, cvt<T>(src[z]));
        }
      }
      fft(fftZ_, a, w, nl, -1);
      for (int l = 0; l < nl; ++l) {
        const i64 s = s0 + l;
        for (int q = p.stickRunOffsets[s]; q < p.stickRunOffsets[s + 1]; ++q) {
          const StickRun& r = p.runs[q];
          for (int j = 0; j < r.length; ++j)
            values[r.valueStart + j] = scale(lane<T>(a[r.zStart + j], l), factor);
        }
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
  finish_exchange();
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
void HostExecutor<T>::finish_exchange() {
  if (!pending_) return;
  SPFFT_TIMED_SCOPE("exchange_wait");
  std::unique_ptr<ExchangeRequest> r = std::move(pending_);
  r->wait();
}

template <typename T>
void HostExecutor<T>::exchange(bool backward, bool nonBlocking) {
  finish_exchange();
  if (plan_->size <= 1) return;
  if (unbuffered_) {
    exchange_strided(backward, nonBlocking);
    return;
  }
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
  const void* src = backward ? stick : slab;
  void* dst = backward ? slab : stick;
  if (nonBlocking)
    pending_ = grid_->communicator()->ialltoallv(src, sc.data(), sd.data(), dst, rc.data(), rd.data());
  else
    grid_->communicator()->alltoallv(src, sc.data(), sd.data(), dst, rc.data(), rd.data());
}

// UNBUFFERED: rank r's planes of every local stick move straight out of (into)
// the [stick][z] array as one strided layout (S blocks of planes(r) elements,
// dimZ apart); the slab side holds each rank's block contiguously.
template <typename T>
void HostExecutor<T>::exchange_strided(bool backward, bool nonBlocking) {
  SPFFT_TIMED_SCOPE("alltoallw");
  const IndexPlan& p = *plan_;
  const std::size_t eb = sizeof(cx<T>);
  const int P = p.size;
  const std::size_t S = static_cast<std::size_t>(p.local_sticks());
  std::vector<StridedLayout> stickL(P), slabL(P);
  for (int r = 0; r < P; ++r) {
    const std::size_t planes = static_cast<std::size_t>(p.planesPerRank[r]);
    stickL[r] = StridedLayout{static_cast<std::size_t>(p.planeOffsets[r]) * eb, planes ? S : 0, planes * eb,
                              static_cast<std::size_t>(p.dimZ) * eb};
    const std::size_t bytes = static_cast<std::size_t>(layout_.slabCount[r]) * eb;
    slabL[r] = StridedLayout{static_cast<std::size_t>(layout_.slabDispl[r]) * eb, bytes ? 1u : 0u, bytes, bytes};
  }
  void* stick = grid_->host_slot(GridImpl<T>::kStickSide);
  void* slab = grid_->host_slot(GridImpl<T>::kSlabSide);
  Communicator& c = *grid_->communicator();
  if (backward) {
    if (nonBlocking)
      pending_ = c.ialltoallw(stick, stickL.data(), slab, slabL.data());
    else
      c.alltoallw(stick, stickL.data(), slab, slabL.data());
  } else {
    if (nonBlocking)
      pending_ = c.ialltoallw(slab, slabL.data(), stick, stickL.data());
    else
      c.alltoallw(slab, slabL.data(), stick, stickL.data());
  }
}

template <typename T>
void HostExecutor<T>::backward_exchange(bool nonBlocking) {
  SPFFT_TIMED_SCOPE(nonBlocking ? "backward_exchange_start" : "backward_exchange");
  exchange(true, nonBlocking);
}

template <typename T>
void HostExecutor<T>::backward_xy() {
  SPFFT_TIMED_SCOPE("backward_xy");
  finish_exchange();
  const bool dist = plan_->size > 1;
  void* slab = grid_->host_slot(dist ? GridImpl<T>::kSlabSide : GridImpl<T>::kStickSide);
  auto* inter = static_cast<cx<T>*>(grid_->host_slot(GridImpl<T>::kInter));
  if (floatExchange_)
    yx_backward(static_cast<const cx<float>*>(slab), inter, space_domain());
  else
    yx_backward(static_cast<const cx<T>*>(slab), inter, space_domain());
}

template <typename T>
void HostExecutor<T>::forward_xy() {
  SPFFT_TIMED_SCOPE("forward_xy");
  finish_exchange();
  poison(false);
  const bool dist = plan_->size > 1;
  auto* inter = static_cast<cx<T>*>(grid_->host_slot(GridImpl<T>::kInter));
  void* slab = grid_->host_slot(dist ? GridImpl<T>::kSlabSide : GridImpl<T>::kStickSide);
  if (floatExchange_)
    xy_forward(space_domain(), inter, static_cast<cx<float>*>(slab));
  else
    xy_forward(space_domain(), inter, static_cast<cx<T>*>(slab));
}

template <typename T>
void HostExecutor<T>::forward_exchange(bool nonBlocking) {
  SPFFT_TIMED_SCOPE(nonBlocking ? "forward_exchange_start" : "forward_exchange");
  exchange(false, nonBlocking);
}

template <typename T>
void HostExecutor<T>::forward_z(T* output, SpfftScalingType scaling) {
  SPFFT_TIMED_SCOPE("forward_z");
  finish_exchange();
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
