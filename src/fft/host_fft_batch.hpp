// Batched host FFT: W lines at once in structure-of-arrays form.
//
// A batch element cx<V> holds element j of W lines (V = W-wide clang vector
// of T), so every Stockham butterfly runs on W lines with full-width SIMD
// instructions (AVX2 / AVX-512) and twiddles are broadcast scalars. The stage
// kernels of the host executor gather W lines into a batch buffer (and scatter
// the results) with contiguous W-element runs wherever the layout allows, so
// the gathers are cache-line sized. Replaces FFTW's plan-many batches of the
// reference host path (reference: src/fft/transform_1d_host.hpp:49-130,
// fftw_plan_1d.hpp:46-166). Lengths with a prime factor above kBluesteinPrime
// run Bluestein's chirp-z convolution on W lines at once: two batched
// power-of-two FFTs of length m >= 2n-1 with the chirp and filter products in
// between, in a per-thread scratch buffer that is reused across calls.
#pragma once

#include <cmath>
#include <memory>
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
    if (n > 1 && !radices_.empty() && radices_.back() > kBluesteinPrime) {
      if (!init_rader()) init_bluestein();
    }
  }

  int size() const { return n_; }
  // every length runs batched (Bluestein lengths through the chirp-z path)
  bool batched() const { return true; }
  bool bluestein() const { return static_cast<bool>(blue_); }
  bool rader() const { return static_cast<bool>(rader_); }

  // In-place transform of the W lines held in a[0..n); b is scratch of n
  // elements. sign +1: exp(+2 pi i jk/n) (backward), -1: forward.
  void run(VC* a, VC* b, int sign) const {
    if (n_ <= 1) return;
    if (rader_) {
      rader_run(a, sign);
      return;
    }
    if (blue_) {
      bluestein_run(a, sign);
      return;
    }
    const VC* res = sign > 0 ? passes<+1>(a, b) : passes<-1>(a, b);
    if (res != a)
      for (int i = 0; i < n_; ++i) a[i] = res[i];
  }

private:
  // Bluestein: jk = (j^2 + k^2 - (k-j)^2) / 2, so with c_j = exp(S i pi j^2 / n)
  // X_k = c_k sum_j (x_j c_j) conj(c_{k-j}): a circular convolution of length
  // m >= 2n-1 (power of two) through the batched engine; the filter spectra
  // (one per sign) are computed once.
  struct Blue {
    int m = 0;
    std::shared_ptr<const HostFftBatch> inner;
    std::vector<cx<T>> chirp;       // c_j for S = -1
    std::vector<cx<T>> filter[2];   // [0]: S = -1, [1]: S = +1
  };
  void init_bluestein() {
    auto b = std::make_shared<Blue>();
    int m = 1;
    while (m < 2 * n_ - 1) m *= 2;
    b->m = m;
    b->inner = std::make_shared<const HostFftBatch>(m);
    b->chirp.resize(n_);
    const long double pi = 3.141592653589793238462643383279502884L;
    for (int j = 0; j < n_; ++j) {
      const long long q = (static_cast<long long>(j) * j) % (2LL * n_);  // exact phase reduction
      const long double ang = pi * static_cast<long double>(q) / static_cast<long double>(n_);
      b->chirp[j] = mk<T>(static_cast<T>(std::cos(ang)), static_cast<T>(-std::sin(ang)));
    }
    std::vector<VC> work(2 * static_cast<std::size_t>(m));
    for (int s = 0; s < 2; ++s) {
      VC* f = work.data();
      for (int j = 0; j < m; ++j) f[j] = zero();
      for (int j = 0; j < n_; ++j) {
        const cx<T> cj = s == 0 ? b->chirp[j] : conj(b->chirp[j]);
        f[j] = broadcast(conj(cj));
        if (j > 0) f[m - j] = f[j];
      }
      b->inner->run(f, f + m, -1);
      b->filter[s].resize(m);
      for (int j = 0; j < m; ++j) b->filter[s][j] = lane0(f[j]);
    }
    blue_ = std::move(b);
  }
  static VC zero() {
    VC z;
    z.x = V(T(0));
    z.y = V(T(0));
    return z;
  }
  static VC broadcast(cx<T> v) {
    VC r;
    r.x = V(v.x);
    r.y = V(v.y);
    return r;
  }
  static cx<T> lane0(const VC& v) { return mk<T>(v.x[0], v.y[0]); }
  void bluestein_run(VC* a, int sign) const {
    const Blue& b = *blue_;
    const int m = b.m;
    // per-thread scratch, grown once and reused by every later call
    thread_local std::vector<VC> tls;
    if (tls.size() < 2 * static_cast<std::size_t>(m)) tls.resize(2 * static_cast<std::size_t>(m));
    VC* u = tls.data();
    const bool plus = sign > 0;
    for (int j = 0; j < n_; ++j)
      u[j] = plus ? twv<+1>(a[j], b.chirp[j]) : twv<-1>(a[j], b.chirp[j]);  // x_j c_j
    for (int j = n_; j < m; ++j) u[j] = zero();
    b.inner->run(u, u + m, -1);
    const std::vector<cx<T>>& f = b.filter[plus ? 1 : 0];
    for (int j = 0; j < m; ++j) u[j] = twv<-1>(u[j], f[j]);
    b.inner->run(u, u + m, +1);
    const T inv = T(1) / static_cast<T>(m);
    for (int k = 0; k < n_; ++k) {
      VC v = plus ? twv<+1>(u[k], b.chirp[k]) : twv<-1>(u[k], b.chirp[k]);
      v.x *= inv;
      v.y *= inv;
      a[k] = v;
    }
  }

  // Rader (prime n whose n - 1 has a direct Stockham plan, e.g. 101 = 4 * 25 + 1):
  // with a generator g of the multiplicative group mod n, a_q = x_{g^q} and
  // b_q = w^{g^-q} (w = exp(S 2 pi i / n)), X_{g^-q} = x_0 + (a (*) b)_q, a cyclic
  // convolution of length n - 1: two batched FFTs of length n - 1 instead of
  // Bluestein's two of length >= 2n - 1 (a power of two: 256 for 101).
  struct Rader {
    std::shared_ptr<const HostFftBatch> inner;
    std::vector<int> in, out;       // g^q, g^-q mod n (q = 0 .. n-2)
    std::vector<cx<T>> filter[2];   // FFT_{n-1}(b) / (n - 1): [0] S = -1, [1] S = +1
  };
  static bool is_prime(int n) {
    if (n < 2) return false;
    for (int d = 2; static_cast<long long>(d) * d <= n; ++d)
      if (n % d == 0) return false;
    return true;
  }
  bool init_rader() {
    if (!is_prime(n_) || n_ < 5) return false;
    const std::vector<int> inner = stockham_radices(n_ - 1);
    if (inner.empty() || inner.back() > kBluesteinPrime) return false;
    // smallest generator: g^((n-1)/f) != 1 for every prime factor f of n - 1
    std::vector<int> fac;
    for (int q = n_ - 1, d = 2; q > 1; ++d) {
      if (static_cast<long long>(d) * d > q) d = q;
      if (q % d == 0) {
        fac.push_back(d);
        while (q % d == 0) q /= d;
      }
    }
    auto pw = [&](long long b, long long e) {
      long long r = 1;
      b %= n_;
      for (; e; e >>= 1, b = b * b % n_)
        if (e & 1) r = r * b % n_;
      return r;
    };
    int g = 2;
    for (;; ++g) {
      bool ok = true;
      for (int f : fac) ok = ok && pw(g, (n_ - 1) / f) != 1;
      if (ok) break;
    }
    auto r = std::make_shared<Rader>();
    const int m = n_ - 1;
    r->inner = std::make_shared<const HostFftBatch>(m);
    r->in.resize(m);
    r->out.resize(m);
    const long long ginv = pw(g, n_ - 2);
    long long x = 1, y = 1;
    for (int q = 0; q < m; ++q) {
      r->in[q] = static_cast<int>(x);
      r->out[q] = static_cast<int>(y);
      x = x * g % n_;
      y = y * ginv % n_;
    }
    std::vector<VC> work(2 * static_cast<std::size_t>(m));
    const long double pi = 3.141592653589793238462643383279502884L;
    for (int s = 0; s < 2; ++s) {
      VC* f = work.data();
      for (int q = 0; q < m; ++q) {
        const long double ang = 2 * pi * static_cast<long double>(r->out[q]) / static_cast<long double>(n_);
        const T c = static_cast<T>(std::cos(ang)), sn = static_cast<T>(std::sin(ang));
        f[q] = broadcast(mk<T>(c, s == 0 ? -sn : sn));
      }
      r->inner->run(f, f + m, -1);
      r->filter[s].resize(m);
      const T inv = T(1) / static_cast<T>(m);
      for (int q = 0; q < m; ++q) r->filter[s][q] = mk<T>(f[q].x[0] * inv, f[q].y[0] * inv);
    }
    rader_ = std::move(r);
    return true;
  }
  void rader_run(VC* a, int sign) const {
    const Rader& r = *rader_;
    const int m = n_ - 1;
    thread_local std::vector<VC> tls;
    if (tls.size() < 2 * static_cast<std::size_t>(m)) tls.resize(2 * static_cast<std::size_t>(m));
    VC* u = tls.data();
    VC x0 = a[0], sum = a[0];
    for (int q = 0; q < m; ++q) {
      u[q] = a[r.in[q]];
      sum = sum + u[q];
    }
    r.inner->run(u, u + m, -1);
    const std::vector<cx<T>>& f = r.filter[sign > 0 ? 1 : 0];
    for (int q = 0; q < m; ++q) u[q] = twv<-1>(u[q], f[q]);
    r.inner->run(u, u + m, +1);
    a[0] = sum;
    for (int q = 0; q < m; ++q) a[r.out[q]] = x0 + u[q];
  }

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
  std::vector<int> radices_;
  std::vector<cx<T>> tw_;
  std::shared_ptr<const Blue> blue_;  // immutable after construction (shared by copies)
  std::shared_ptr<const Rader> rader_;
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
