// Batched host FFT: W lines at once in structure-of-arrays form.
//
// A batch element cx<V> holds element j of W lines (V = W-wide clang vector
// of T), so every Stockham butterfly runs on W lines with full-width SIMD
// instructions (AVX2 / AVX-512) and twiddles are broadcast scalars. The stage
// kernels of the host executor gather W lines into a batch buffer (and scatter
// the results) with contiguous W-element runs wherever the layout allows, so
// the gathers are cache-line sized. Replaces FFTW's plan-many batches of the
// reference host path (reference: src/fft/transform_1d_host.hpp:49-130,
// fftw_plan_1d.hpp:46-166); lengths with a prime factor above kBluesteinPrime
// keep the scalar Bluestein engine (HostFft) line by line.
#pragma once

#include <utility>
#include <vector>

#include "fft/codelets.hpp"
#include "fft/fft_plan.hpp"
#include "fft/host_fft.hpp"

namespace spfft {

#ifndef SPFFT_HOST_SIMD_BYTES
#define SPFFT_HOST_SIMD_BYTES 32
#endif

template <typename T>
struct HostSimd {
  static constexpr int W = SPFFT_HOST_SIMD_BYTES / static_cast<int>(sizeof(T));
  typedef T V __attribute__((ext_vector_type(W)));
  using VC = cx<V>;
};

// a * w (S = -1) or a * conj(w) (S = +1), w a scalar twiddle broadcast to all lanes
template <int S, typename V, typename T>
inline cx<V> twv(const cx<V>& a, const cx<T>& w) {
  cx<V> r;
  if (S > 0) {
    r.x = a.x * w.x + a.y * w.y;
    r.y = a.y * w.x - a.x * w.y;
  } else {
    r.x = a.x * w.x - a.y * w.y;
    r.y = a.x * w.y + a.y * w.x;
  }
  return r;
}

template <typename T>
class HostFftBatch {
public:
  using Simd = HostSimd<T>;
  using V = typename Simd::V;
  using VC = typename Simd::VC;
  static constexpr int W = Simd::W;

  HostFftBatch() = default;
  explicit HostFftBatch(int n) : n_(n), radices_(stockham_radices(n)), tw_(make_twiddles<T>(n)) {
    batched_ = n <= 1 || radices_.empty() || radices_.back() <= kBluesteinPrime;
    if (!batched_) scalar_ = HostFft<T>(n);
  }

  int size() const { return n_; }
  // false: the length needs Bluestein; run scalar() line by line instead
  bool batched() const { return batched_; }
  const HostFft<T>& scalar() const { return scalar_; }

  // In-place transform of the W lines held in a[0..n); b is scratch of n
  // elements. sign +1: exp(+2 pi i jk/n) (backward), -1: forward.
  void run(VC* a, VC* b, int sign) const {
    if (n_ <= 1) return;
    const VC* res = sign > 0 ? passes<+1>(a, b) : passes<-1>(a, b);
    if (res != a)
      for (int i = 0; i < n_; ++i) a[i] = res[i];
  }

private:
  template <int S>
  const VC* passes(VC* a, VC* b) const {
    int ns = 1;
    VC* src = a;
    VC* dst = b;
    for (int r : radices_) {
      switch (r) {
        case 2: pass<2, S>(src, dst, ns); break;
        case 3: pass<3, S>(src, dst, ns); break;
        case 4: pass<4, S>(src, dst, ns); break;
        case 5: pass<5, S>(src, dst, ns); break;
        case 6: pass<6, S>(src, dst, ns); break;
        case 7: pass<7, S>(src, dst, ns); break;
        case 8: pass<8, S>(src, dst, ns); break;
        case 9: pass<9, S>(src, dst, ns); break;
        case 10: pass<10, S>(src, dst, ns); break;
        case 11: pass<11, S>(src, dst, ns); break;
        case 12: pass<12, S>(src, dst, ns); break;
        case 13: pass<13, S>(src, dst, ns); break;
        case 15: pass<15, S>(src, dst, ns); break;
        case 16: pass<16, S>(src, dst, ns); break;
        case 20: pass<20, S>(src, dst, ns); break;
        default: pass_generic<S>(src, dst, ns, r); break;
      }
      ns *= r;
      std::swap(src, dst);
    }
    return src;
  }

  // Stockham pass: butterfly j reads src[j + r n/R], twiddles w_{ns R}^{(j mod
  // ns) r}, writes dst[(j - j mod ns) R + j mod ns + r ns]. The first pass
  // (ns = 1) has no twiddles and is unrolled over consecutive j.
  template <int R, int S>
  void pass(const VC* __restrict__ src, VC* __restrict__ dst, int ns) const {
    const int nb = n_ / R;
    const int twStride = n_ / (ns * R);
    for (int j0 = 0; j0 < nb; j0 += ns) {
      // j0 .. j0+ns-1 share the output block (j0 R)
      for (int k = 0; k < ns; ++k) {
        const int j = j0 + k;
        VC v[R];
        for (int r = 0; r < R; ++r) v[r] = src[j + r * nb];
        if (k != 0)
          for (int r = 1; r < R; ++r) v[r] = twv<S>(v[r], tw_[k * r * twStride]);
        Dft<R, S, V>::run(v);
        VC* d = dst + j0 * R + k;
        for (int r = 0; r < R; ++r) d[r * ns] = v[r];
      }
    }
  }

  template <int S>
  void pass_generic(const VC* src, VC* dst, int ns, int R) const {
    const int nb = n_ / R;
    const int twStride = n_ / (ns * R);
    const int dftStride = n_ / R;
    std::vector<VC> v(R);
    for (int j = 0; j < nb; ++j) {
      const int k = j % ns;
      for (int r = 0; r < R; ++r) {
        v[r] = src[j + r * nb];
        if (k != 0 && r != 0) v[r] = twv<S>(v[r], tw_[static_cast<long long>(k) * r * twStride]);
      }
      const int base = (j - k) * R + k;
      for (int q = 0; q < R; ++q) {
        VC acc = v[0];
        for (int r = 1; r < R; ++r) {
          const int e = static_cast<int>((static_cast<long long>(r) * q) % R);
          acc = acc + twv<S>(v[r], tw_[e * dftStride]);
        }
        dst[base + q * ns] = acc;
      }
    }
  }

  int n_ = 0;
  bool batched_ = true;
  std::vector<int> radices_;
  std::vector<cx<T>> tw_;
  HostFft<T> scalar_;
};

// Lane access of a batch element through its memory (re lanes then im lanes):
// scalar loads and stores, no vector insert / extract with a run-time index.
template <typename T>
inline cx<T> lane(const typename HostSimd<T>::VC& v, int l) {
  typedef const T __attribute__((may_alias)) A;
  A* p = reinterpret_cast<A*>(&v);
  return mk<T>(p[l], p[HostSimd<T>::W + l]);
}
template <typename T>
inline void set_lane(typename HostSimd<T>::VC& v, int l, cx<T> x) {
  typedef T __attribute__((may_alias)) A;
  A* p = reinterpret_cast<A*>(&v);
  p[l] = x.x;
  p[HostSimd<T>::W + l] = x.y;
}
template <typename T>
inline typename HostSimd<T>::VC vzero() {
  typename HostSimd<T>::VC z;
  z.x = typename HostSimd<T>::V(T(0));
  z.y = typename HostSimd<T>::V(T(0));
  return z;
}
// W consecutive interleaved complex values <-> one batch element.
template <typename T>
inline typename HostSimd<T>::VC load_aos(const cx<T>* src) {
  constexpr int W = HostSimd<T>::W;
  typename HostSimd<T>::VC v;
  T re[W], im[W];
  for (int l = 0; l < W; ++l) {
    re[l] = src[l].x;
    im[l] = src[l].y;
  }
  __builtin_memcpy(&v.x, re, sizeof(re));
  __builtin_memcpy(&v.y, im, sizeof(im));
  return v;
}
template <typename T>
inline void store_aos(cx<T>* dst, const typename HostSimd<T>::VC& v) {
  constexpr int W = HostSimd<T>::W;
  T re[W], im[W];
  __builtin_memcpy(re, &v.x, sizeof(re));
  __builtin_memcpy(im, &v.y, sizeof(im));
  for (int l = 0; l < W; ++l) dst[l] = mk<T>(re[l], im[l]);
}

}  // namespace spfft
