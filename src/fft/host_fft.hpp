// Host (CPU) 1D FFT engine: mixed-radix Stockham autosort with the shared
// codelets, any length (primes without a codelet use an O(R)-per-output pass).
// Replaces the FFTW plans of the reference host path
// (reference: src/fft/transform_1d_host.hpp, fftw_plan_1d.hpp).
#pragma once

#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "fft/codelets.hpp"
#include "fft/fft_plan.hpp"

namespace spfft {

// Lengths whose factorisation keeps a prime above this bound run through
// Bluestein's chirp-z algorithm (O(n log n)) instead of the O(R)-per-output
// generic prime pass.
constexpr int kBluesteinPrime = 61;

template <typename T>
class HostFft {
public:
  HostFft() = default;
  explicit HostFft(int n) : n_(n), radices_(stockham_radices(n)), tw_(make_twiddles<T>(n)) {
    if (!radices_.empty() && radices_.back() > kBluesteinPrime) init_bluestein();
  }

  int size() const { return n_; }
  bool bluestein() const { return static_cast<bool>(inner_); }
  // Scratch elements execute() needs.
  std::size_t scratch_size() const {
    return inner_ ? static_cast<std::size_t>(m_) + inner_->scratch_size()
                  : 2 * static_cast<std::size_t>(n_);
  }

  // out[k] = sum_j in[j*inStride] exp(sign 2 pi i j k / n), written to out[k*outStride].
  // `scratch` must hold scratch_size() elements; in/out may alias.
  void execute(const cx<T>* in, std::ptrdiff_t inStride, cx<T>* out, std::ptrdiff_t outStride,
               int sign, cx<T>* scratch) const {
    if (n_ <= 0) return;
    if (inner_) {
      bluestein_execute(in, inStride, out, outStride, sign, scratch);
      return;
    }
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
  // Bluestein: jk = (j^2 + k^2 - (k-j)^2) / 2, so with d_j = exp(S i pi j^2 / n)
  // X_k = d_k sum_j (x_j d_j) conj(d_{k-j}): a circular convolution of length
  // m >= 2n-1 (power of two) done with the mixed-radix engine.
  void init_bluestein() {
    m_ = 1;
    while (m_ < 2 * n_ - 1) m_ *= 2;
    inner_ = std::make_shared<HostFft<T>>(m_);
    chirp_.resize(n_);
    const long double pi = 3.141592653589793238462643383279502884L;
    for (int j = 0; j < n_; ++j) {
      const long long q = (static_cast<long long>(j) * j) % (2LL * n_);  // exact phase reduction
      const long double a = pi * static_cast<long double>(q) / static_cast<long double>(n_);
      chirp_[j].x = static_cast<T>(std::cos(a));
      chirp_[j].y = static_cast<T>(-std::sin(a));  // d_j for S = -1
    }
    std::vector<cx<T>> work(inner_->scratch_size());
    for (int s = 0; s < 2; ++s) {
      const int sign = s == 0 ? -1 : +1;
      std::vector<cx<T>> b(m_, mk<T>(T(0), T(0)));
      for (int j = 0; j < n_; ++j) {
        const cx<T> dj = sign < 0 ? chirp_[j] : conj(chirp_[j]);
        b[j] = conj(dj);
        if (j > 0) b[m_ - j] = conj(dj);
      }
      inner_->execute(b.data(), 1, b.data(), 1, -1, work.data());
      (s == 0 ? filterMinus_ : filterPlus_) = std::move(b);
    }
  }

  void bluestein_execute(const cx<T>* in, std::ptrdiff_t inStride, cx<T>* out,
                         std::ptrdiff_t outStride, int sign, cx<T>* scratch) const {
    cx<T>* a = scratch;
    cx<T>* work = scratch + m_;
    for (int j = 0; j < n_; ++j) {
      const cx<T> dj = sign < 0 ? chirp_[j] : conj(chirp_[j]);
      a[j] = cmul(in[j * inStride], dj);
    }
    for (int j = n_; j < m_; ++j) a[j] = mk<T>(T(0), T(0));
    inner_->execute(a, 1, a, 1, -1, work);
    const std::vector<cx<T>>& f = sign < 0 ? filterMinus_ : filterPlus_;
    for (int j = 0; j < m_; ++j) a[j] = cmul(a[j], f[j]);
    inner_->execute(a, 1, a, 1, +1, work);
    const T inv = T(1) / static_cast<T>(m_);
    for (int k = 0; k < n_; ++k) {
      const cx<T> dk = sign < 0 ? chirp_[k] : conj(chirp_[k]);
      out[k * outStride] = scale(cmul(a[k], dk), inv);
    }
  }

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
  // Bluestein state (shared by copies: immutable after construction)
  int m_ = 0;
  std::shared_ptr<HostFft<T>> inner_;
  std::vector<cx<T>> chirp_, filterMinus_, filterPlus_;
};

}  // namespace spfft
