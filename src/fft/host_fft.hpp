// Host (CPU) 1D FFT engine: mixed-radix Stockham autosort with the shared
// codelets, any length (primes without a codelet use an O(R)-per-output pass).
// Replaces the FFTW plans of the reference host path
// (reference: src/fft/transform_1d_host.hpp, fftw_plan_1d.hpp).
#pragma once

#include <algorithm>
#include <cstring>
#include <vector>

#include "fft/codelets.hpp"
#include "fft/fft_plan.hpp"

namespace spfft {

template <typename T>
class HostFft {
public:
  HostFft() = default;
  explicit HostFft(int n) : n_(n), radices_(factorize_radices(n)), tw_(make_twiddles<T>(n)) {}

  int size() const { return n_; }
  // Scratch elements execute() needs.
  std::size_t scratch_size() const { return 2 * static_cast<std::size_t>(n_); }

  // out[k] = sum_j in[j*inStride] exp(sign 2 pi i j k / n), written to out[k*outStride].
  // `scratch` must hold scratch_size() elements; in/out may alias.
  void execute(const cx<T>* in, std::ptrdiff_t inStride, cx<T>* out, std::ptrdiff_t outStride,
               int sign, cx<T>* scratch) const {
    if (n_ <= 0) return;
    cx<T>* a = scratch;
    cx<T>* b = scratch + n_;
    for (int i = 0; i < n_; ++i) a[i] = in[i * inStride];
    if (sign > 0)
      run<+1>(a, b);
    else
      run<-1>(a, b);
    cx<T>* res = (radices_.size() % 2 == 0) ? a : b;
    for (int i = 0; i < n_; ++i) out[i * outStride] = res[i];
  }

private:
  template <int S>
  void run(cx<T>* a, cx<T>* b) const {
    int ns = 1;
    cx<T>* src = a;
    cx<T>* dst = b;
    for (int r : radices_) {
      switch (r) {
        case 2: pass<2, S>(src, dst, ns); break;
        case 3: pass<3, S>(src, dst, ns); break;
        case 4: pass<4, S>(src, dst, ns); break;
        case 5: pass<5, S>(src, dst, ns); break;
        case 7: pass<7, S>(src, dst, ns); break;
        case 8: pass<8, S>(src, dst, ns); break;
        case 9: pass<9, S>(src, dst, ns); break;
        case 11: pass<11, S>(src, dst, ns); break;
        case 13: pass<13, S>(src, dst, ns); break;
        case 16: pass<16, S>(src, dst, ns); break;
        default: pass_generic<S>(src, dst, ns, r); break;
      }
      ns *= r;
      std::swap(src, dst);
    }
  }

  // One Stockham pass: butterfly j reads src[j + r*n/R], applies twiddles
  // w_{ns*R}^{(j mod ns) r}, and writes dst[(j - j mod ns) R + j mod ns + r ns].
  template <int R, int S>
  void pass(const cx<T>* src, cx<T>* dst, int ns) const {
    const int nb = n_ / R;
    const int twStride = n_ / (ns * R);
    for (int j = 0; j < nb; ++j) {
      const int k = j % ns;
      cx<T> v[R];
      for (int r = 0; r < R; ++r) v[r] = src[j + r * nb];
      if (k != 0) {
        for (int r = 1; r < R; ++r) v[r] = twm<S>(v[r], tw_[k * r * twStride]);
      }
      Dft<R, S, T>::run(v);
      const int base = (j - k) * R + k;
      for (int r = 0; r < R; ++r) dst[base + r * ns] = v[r];
    }
  }

  template <int S>
  void pass_generic(const cx<T>* src, cx<T>* dst, int ns, int R) const {
    const int nb = n_ / R;
    const int twStride = n_ / (ns * R);
    const int dftStride = n_ / R;
    std::vector<cx<T>> v(R);
    for (int j = 0; j < nb; ++j) {
      const int k = j % ns;
      for (int r = 0; r < R; ++r) {
        v[r] = src[j + r * nb];
        if (k != 0 && r != 0) v[r] = twm<S>(v[r], tw_[static_cast<long long>(k) * r * twStride]);
      }
      const int base = (j - k) * R + k;
      for (int q = 0; q < R; ++q) {
        cx<T> acc = v[0];
        for (int r = 1; r < R; ++r) {
          const int e = static_cast<int>((static_cast<long long>(r) * q) % R);
          acc = acc + twm<S>(v[r], tw_[e * dftStride]);
        }
        dst[base + q * ns] = acc;
      }
    }
  }

  int n_ = 0;
  std::vector<int> radices_;
  std::vector<cx<T>> tw_;
};

}  // namespace spfft
