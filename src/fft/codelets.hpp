// Small-DFT codelets shared by the host FFT engine and the CDNA4 kernels.
//
// Sign convention (SpFFT, docs/source/details.rst:6-13): the forward
// (space -> frequency) transform uses exp(-2*pi*i*n*k/N) and the backward
// transform exp(+2*pi*i*n*k/N). Codelets take the sign S in {-1, +1} as a
// template argument so that every +-i rotation folds into add/sub at compile time.
#pragma once

#include "fft/dft_constants.hpp"

#if defined(__HIPCC__)
#define SPFFT_HD __host__ __device__ __forceinline__
#else
#define SPFFT_HD inline
#endif

namespace spfft {

template <typename T>
struct alignas(2 * sizeof(T)) cx {
  using value_type = T;
  T x, y;
};

template <typename T>
SPFFT_HD cx<T> mk(T a, T b) {
  cx<T> r;
  r.x = a;
  r.y = b;
  return r;
}
template <typename T>
SPFFT_HD cx<T> operator+(cx<T> a, cx<T> b) {
  return mk<T>(a.x + b.x, a.y + b.y);
}
template <typename T>
SPFFT_HD cx<T> operator-(cx<T> a, cx<T> b) {
  return mk<T>(a.x - b.x, a.y - b.y);
}
template <typename T>
SPFFT_HD cx<T> scale(cx<T> a, T s) {
  return mk<T>(a.x * s, a.y * s);
}
template <typename T>
SPFFT_HD cx<T> cmul(cx<T> a, cx<T> b) {
  return mk<T>(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// a * conj(b)
template <typename T>
SPFFT_HD cx<T> cmulc(cx<T> a, cx<T> b) {
  return mk<T>(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}
template <typename T>
SPFFT_HD cx<T> conj(cx<T> a) {
  return mk<T>(a.x, -a.y);
}
// (S * i) * a
template <int S, typename T>
SPFFT_HD cx<T> rot(cx<T> a) {
  return S > 0 ? mk<T>(-a.y, a.x) : mk<T>(a.y, -a.x);
}
// a * exp(S * i * theta) with (c, s) = (cos theta, sin theta)
template <int S, typename T>
SPFFT_HD cx<T> twc(cx<T> a, T c, T s) {
  return S > 0 ? mk<T>(a.x * c - a.y * s, a.x * s + a.y * c)
               : mk<T>(a.x * c + a.y * s, a.y * c - a.x * s);
}
// Multiply by a stored twiddle w (= exp(-i theta)); S = +1 uses conj(w).
template <int S, typename T>
SPFFT_HD cx<T> twm(cx<T> a, cx<T> w) {
  return S > 0 ? cmulc(a, w) : cmul(a, w);
}

// In-place DFT of length R on v[0..R-1] (natural order in and out).
template <int R, int S, typename T>
struct Dft;

template <int S, typename T>
struct Dft<1, S, T> {
  static SPFFT_HD void run(cx<T>*) {}
};

template <int S, typename T>
struct Dft<2, S, T> {
  static SPFFT_HD void run(cx<T>* v) {
    const cx<T> a = v[0], b = v[1];
    v[0] = a + b;
    v[1] = a - b;
  }
};

template <int S, typename T>
struct Dft<4, S, T> {
  static SPFFT_HD void run(cx<T>* v) {
    const cx<T> t0 = v[0] + v[2], t1 = v[0] - v[2];
    const cx<T> t2 = v[1] + v[3], t3 = rot<S>(v[1] - v[3]);
    v[0] = t0 + t2;
    v[2] = t0 - t2;
    v[1] = t1 + t3;
    v[3] = t1 - t3;
  }
};

template <int S, typename T>
struct Dft<8, S, T> {
  static SPFFT_HD void run(cx<T>* v) {
    cx<T> e[4] = {v[0], v[2], v[4], v[6]};
    cx<T> o[4] = {v[1], v[3], v[5], v[7]};
    Dft<4, S, T>::run(e);
    Dft<4, S, T>::run(o);
    const T c = T(fftc::SQRT1_2);
    // w8^1 = c(1 + S i), w8^2 = S i, w8^3 = c(-1 + S i)
    const cx<T> o1 = scale(mk<T>(o[1].x - T(S) * o[1].y, o[1].y + T(S) * o[1].x), c);
    const cx<T> o2 = rot<S>(o[2]);
    const cx<T> o3 = scale(mk<T>(-o[3].x - T(S) * o[3].y, -o[3].y + T(S) * o[3].x), c);
    v[0] = e[0] + o[0];
    v[4] = e[0] - o[0];
    v[1] = e[1] + o1;
    v[5] = e[1] - o1;
    v[2] = e[2] + o2;
    v[6] = e[2] - o2;
    v[3] = e[3] + o3;
    v[7] = e[3] - o3;
  }
};

// 16 = 4 x 4: column DFTs, internal twiddles w16^(n2*k1), row DFTs, transposed output.
template <int S, typename T>
struct Dft<16, S, T> {
  static SPFFT_HD void run(cx<T>* v) {
    cx<T> y[4][4];
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
      y[n2][0] = v[n2];
      y[n2][1] = v[4 + n2];
      y[n2][2] = v[8 + n2];
      y[n2][3] = v[12 + n2];
      Dft<4, S, T>::run(y[n2]);
    }
#pragma unroll
    for (int n2 = 1; n2 < 4; ++n2) {
#pragma unroll
      for (int k1 = 1; k1 < 4; ++k1) {
        const int m = n2 * k1;
        if (m == 4) {
          y[n2][k1] = rot<S>(y[n2][k1]);
        } else {
          y[n2][k1] = twc<S>(y[n2][k1], T(fftc::C16[m]), T(fftc::S16[m]));
        }
      }
    }
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
      cx<T> r[4] = {y[0][k1], y[1][k1], y[2][k1], y[3][k1]};
      Dft<4, S, T>::run(r);
      v[k1] = r[0];
      v[k1 + 4] = r[1];
      v[k1 + 8] = r[2];
      v[k1 + 12] = r[3];
    }
  }
};

// 32 = 2 x 16: DFT-16 of the even and the odd elements, then one radix-2 layer
// with the twiddles w32^k (the fp32 line-fast N = 512 shape runs 32 x 16, one
// LDS exchange per line instead of two).
template <int S, typename T>
struct Dft<32, S, T> {
  static SPFFT_HD void run(cx<T>* v) {
    cx<T> e[16], o[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      e[i] = v[2 * i];
      o[i] = v[2 * i + 1];
    }
    Dft<16, S, T>::run(e);
    Dft<16, S, T>::run(o);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      cx<T> w;
      if (k == 0)
        w = o[k];
      else if (k == 8)
        w = rot<S>(o[k]);
      else
        w = twc<S>(o[k], T(fftc::C32[k]), T(fftc::S32[k]));
      v[k] = e[k] + w;
      v[k + 16] = e[k] - w;
    }
  }
};

// Odd lengths via symmetric pairs: X_k = A_k + S i B_k, X_{R-k} = A_k - S i B_k.
template <int R, int S, typename T, const double (*CT)[(R - 1) / 2], const double (*ST)[(R - 1) / 2]>
struct DftOdd {
  static SPFFT_HD void run(cx<T>* v) {
    constexpr int H = (R - 1) / 2;
    cx<T> a[H], b[H];
    cx<T> sum = v[0];
#pragma unroll
    for (int n = 1; n <= H; ++n) {
      a[n - 1] = v[n] + v[R - n];
      b[n - 1] = v[n] - v[R - n];
      sum = sum + a[n - 1];
    }
    const cx<T> x0 = v[0];
    v[0] = sum;
#pragma unroll
    for (int k = 1; k <= H; ++k) {
      cx<T> A = x0, B = mk<T>(T(0), T(0));
#pragma unroll
      for (int n = 1; n <= H; ++n) {
        const T c = T(CT[n - 1][k - 1]);
        const T s = T(ST[n - 1][k - 1]);
        A = mk<T>(A.x + c * a[n - 1].x, A.y + c * a[n - 1].y);
        B = mk<T>(B.x + s * b[n - 1].x, B.y + s * b[n - 1].y);
      }
      const cx<T> iB = rot<S>(B);
      v[k] = A + iB;
      v[R - k] = A - iB;
    }
  }
};

template <int S, typename T>
struct Dft<3, S, T> : DftOdd<3, S, T, fftc::C3, fftc::S3> {};
template <int S, typename T>
struct Dft<5, S, T> : DftOdd<5, S, T, fftc::C5, fftc::S5> {};
template <int S, typename T>
struct Dft<7, S, T> : DftOdd<7, S, T, fftc::C7, fftc::S7> {};
template <int S, typename T>
struct Dft<9, S, T> : DftOdd<9, S, T, fftc::C9, fftc::S9> {};
template <int S, typename T>
struct Dft<11, S, T> : DftOdd<11, S, T, fftc::C11, fftc::S11> {};
template <int S, typename T>
struct Dft<13, S, T> : DftOdd<13, S, T, fftc::C13, fftc::S13> {};

// Coprime composites N = N1 N2 by the prime-factor (Good-Thomas) algorithm:
// input n = (N2 n1 + N1 n2) mod N, output k with k = k1 (mod N1), k = k2 (mod N2).
// No twiddles; after unrolling both index maps are register permutations.
SPFFT_HD constexpr int pfa_inverse(int a, int m) {
  int r = 1;
  while ((a * r) % m != 1) ++r;
  return r;
}
template <int N1, int N2, int S, typename T>
struct DftPfa {
  static SPFFT_HD void run(cx<T>* v) {
    constexpr int N = N1 * N2;
    constexpr int E1 = N2 * pfa_inverse(N2 % N1, N1);  // = 1 (mod N1), 0 (mod N2)
    constexpr int E2 = N1 * pfa_inverse(N1 % N2, N2);  // = 0 (mod N1), 1 (mod N2)
    cx<T> a[N2][N1];
#pragma unroll
    for (int n2 = 0; n2 < N2; ++n2) {
#pragma unroll
      for (int n1 = 0; n1 < N1; ++n1) a[n2][n1] = v[(N2 * n1 + N1 * n2) % N];
      Dft<N1, S, T>::run(a[n2]);
    }
#pragma unroll
    for (int k1 = 0; k1 < N1; ++k1) {
      cx<T> b[N2];
#pragma unroll
      for (int n2 = 0; n2 < N2; ++n2) b[n2] = a[n2][k1];
      Dft<N2, S, T>::run(b);
#pragma unroll
      for (int k2 = 0; k2 < N2; ++k2) v[(k1 * E1 + k2 * E2) % N] = b[k2];
    }
  }
};
template <int S, typename T>
struct Dft<6, S, T> : DftPfa<2, 3, S, T> {};
template <int S, typename T>
struct Dft<10, S, T> : DftPfa<2, 5, S, T> {};
template <int S, typename T>
struct Dft<12, S, T> : DftPfa<4, 3, S, T> {};
template <int S, typename T>
struct Dft<15, S, T> : DftPfa<3, 5, S, T> {};
template <int S, typename T>
struct Dft<20, S, T> : DftPfa<4, 5, S, T> {};

// Radices with a dedicated codelet; anything else runs through the generic
// O(R) per-output path (any prime).
SPFFT_HD constexpr bool has_codelet(int r) {
  return r == 2 || r == 3 || r == 4 || r == 5 || r == 7 || r == 8 || r == 9 || r == 11 ||
         r == 13 || r == 16;
}

}  // namespace spfft
