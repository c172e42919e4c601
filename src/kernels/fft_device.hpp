// Block-level FFT engines for CDNA4 (gfx950): a workgroup transforms B lines
// of length N that sit in (or stream through) LDS.
//
//  FftCT<T, N, S>: compile-time length. Each lane keeps E = N/TP elements in
//    VGPRs, executes E/R radix-R butterflies per Stockham pass and exchanges
//    through LDS between passes (2 barriers per pass). LDS rows are padded by
//    one element per 256-byte bank row, and consecutive lines start 16 bytes
//    apart in the bank space, so both the strided pass writes and the
//    column-wise gathers of the stage kernels are bank-conflict free.
//  FftRT<T, S>: run-time length (any N, mixed radix incl. generic primes).
//    Lengths whose radices all have codelets run in place: each pass stages
//    the lane's butterflies in VGPRs between two barriers, work items lines
//    fastest, divisions by precomputed reciprocals. Lengths with a generic
//    prime pass ping-pong between two LDS regions. Used for lengths without
//    a CT shape.
//
// Sign S = +1 is the backward (frequency -> space) direction.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "fft/codelets.hpp"

namespace spfft {
namespace dev {

constexpr int kMaxThreads = 256;

// LDS per workgroup for the FFT lines of the default shapes
constexpr int kLdsBudget = 64 * 1024;
// Lines of the line-fast mapping (at most; a power of two)
constexpr int kLfMaxLines = 16;
// Elements per workgroup of the in-place run-time engine (lines * n): it bounds
// the lanes' register staging (lines * n / (R * threads) butterflies per pass).
// 4096 = 64 KB of complex<double>, 32 KB of complex<float>: the best of the
// 32/64 KB budgets measured for each precision (profiles/README.md, session 5).
constexpr int kRtElems = 4096;
// Workgroup size of the run-time engine kernels.
constexpr int kRtThreads = 256;

template <typename T>
struct LdsGeom;
template <>
struct LdsGeom<double> {
  static constexpr int kShift = 4;  // 16 x 16 B elements per 256 B bank row
  static constexpr int kMod = 16;
};
template <>
struct LdsGeom<float> {
  // one pad element per 16 x 8 B elements: LDS writes and ds_read2 bank on 32
  // banks (128 B) per 16-lane group, so a pad per 256 B bank row left the
  // row-mapped stride-R Stockham writes 2-way conflicted (tools/lds_bank_model.py)
  static constexpr int kShift = 4;
  static constexpr int kMod = 32;
};

// Pad shift of an engine with E elements per lane: fp32 shapes of 32 elements
// per lane (N = 1024) keep one pad per 256 B, whose simpler index arithmetic
// keeps them within their registers (a pad per 128 B made them spill).
template <typename T>
__host__ __device__ constexpr int pad_shift(int e) {
  return (sizeof(T) == 4 && e > 16) ? 5 : LdsGeom<T>::kShift;
}
__host__ __device__ constexpr int pad_index(int i, int shift) { return i + (i >> shift); }
// Line stride: holds pad_index(N-1) and is == 1 (mod kMod) so that line b+1
// starts one element further in the bank space than line b.
template <typename T>
__host__ __device__ constexpr int padded_stride(int n, int shift) {
  return ((n + (n >> shift) + LdsGeom<T>::kMod - 1) / LdsGeom<T>::kMod) * LdsGeom<T>::kMod + 1;
}

// Lines per workgroup: as many as fit the LDS budget and the thread cap, with
// the workgroup a whole number of waves.
__host__ __device__ constexpr int lines_per_block(int tp, int lineBytes, int budget = kLdsBudget,
                                                  int maxThreads = kMaxThreads) {
  int b = maxThreads / tp;
  if (b * lineBytes > budget) b = budget / lineBytes;
  if (b < 1) b = 1;
  if (tp < 64) {
    const int q = 64 / tp;
    b = (b / q) * q;
    if (b < q) b = q;
  }
  return b;
}

// --------------------------------------------------------------- CT shapes
// E = elements per lane, R0..R2 = radices (1 = pass absent); every radix divides E.
template <int N>
struct CtShape;
template <>
struct CtShape<16> {
  static constexpr int E = 16, R0 = 16, R1 = 1, R2 = 1;
};
template <>
struct CtShape<32> {
  static constexpr int E = 8, R0 = 8, R1 = 4, R2 = 1;
};
template <>
struct CtShape<64> {
  static constexpr int E = 8, R0 = 8, R1 = 8, R2 = 1;
};
template <>
struct CtShape<128> {
  static constexpr int E = 16, R0 = 16, R1 = 8, R2 = 1;
};
template <>
struct CtShape<256> {
  static constexpr int E = 16, R0 = 16, R1 = 16, R2 = 1;
};
template <>
struct CtShape<512> {
  static constexpr int E = 8, R0 = 8, R1 = 8, R2 = 8;
};
template <>
struct CtShape<1024> {
  static constexpr int E = 16, R0 = 16, R1 = 16, R2 = 4;
};

// Shape per precision: E is raised where the default would leave the line-fast
// mapping fewer lines than one 128-byte column segment needs (8 lines of
// complex<double>, 16 of complex<float>); those shapes get an 80 KB LDS budget
// (two workgroups per CU).
template <typename T, int N>
struct CtShapeT : CtShape<N> {
  static constexpr int kBudget = kLdsBudget;
};
template <int N>
struct CtShapeT<void, N> : CtShape<N> {
  static constexpr int kBudget = kLdsBudget;
};
template <>
struct CtShapeT<double, 512> {
  static constexpr int E = 16, R0 = 16, R1 = 16, R2 = 2, kBudget = 80 * 1024;
};
template <>
struct CtShapeT<float, 512> {
  static constexpr int E = 32, R0 = 16, R1 = 16, R2 = 2, kBudget = 80 * 1024;
};
template <>
struct CtShapeT<float, 1024> {
  static constexpr int E = 32, R0 = 16, R1 = 16, R2 = 4, kBudget = 80 * 1024;
};

// Shape per stage kind: S = +1 backward / -1 forward, LF = line-fast (y and x
// stages) vs row-mapped (z stage). For complex<double> N = 256 the radix-8
// shape (E = 8, 256 threads per 8 lines) doubles the waves per SIMD that the
// LDS budget allows, which the memory-bound stages turn into bandwidth:
// measured on MI355X at 256^3 (profiles/r2_s1/shape_ab.txt) x backward 97.6 ->
// 93.1 us, x/y forward -1 us. The row-mapped z backward also takes it: with
// the twiddle powers (FftCT::kTwPow) 68.8-71.4 -> 62.0-62.3 us against E = 16
// (profiles/r5/ab/f64b); the forward z stage keeps E = 16 (65.7 vs 71.7 us with
// E = 8 in round 2).
struct CtShape256E8 {
  static constexpr int E = 8, R0 = 8, R1 = 8, R2 = 4, kBudget = kLdsBudget;
};
template <typename T, int N, int S, bool LF>
struct CtShapeSel : std::conditional<LF, CtShapeT<T, N>, CtShapeT<void, N>>::type {};
// N = 128 likewise (radices 8, 8, 2; 16 lanes per line): 256^3 R2C 6467 ->
// 6820 transforms/s (packed-real x stage on N/2 = 128), 128^3 C2C 23770 ->
// 25550 (profiles/r2_s1/shape_ab.txt)
// ... and for the row-mapped forward engines of N = 128 (z forward at 128^3:
// 14.8 -> 11.9 us, 128^3 C2C +3.6%; the row-mapped packed-real R2C x stage)
struct CtShape128E8 {
  static constexpr int E = 8, R0 = 8, R1 = 8, R2 = 2, kBudget = kLdsBudget;
};
template <>
struct CtShapeSel<double, 128, 1, false> : CtShape128E8 {};
template <>
struct CtShapeSel<double, 128, 1, true> : CtShape128E8 {};
template <>
struct CtShapeSel<double, 128, -1, true> : CtShape128E8 {};
template <>
struct CtShapeSel<double, 128, -1, false> : CtShape128E8 {};
// Wide (512-thread) line-fast shapes for the long fp32 / fp64 lines, where the
// default shapes leave 2 waves per SIMD under the LDS budget. Measured on
// MI355X (profiles/r2_s1/wide_ab.txt): 512^3 R2C fp32 1400 -> 1438, 512^3 C2C
// fp64 498 -> 511 transforms/s; for fp32 N = 256 the wide shape was slower
// (6064 -> 5703 at 256^3 C2C fp32) and is not used.
// N = 1024 (measured at 1024^3 C2C fp64, profiles/r2_s1/wide_ab.txt: 24.2 ->
// 47.0 transforms/s) line-fast: with the 64 KB budget only 2 (fp64) / 8 (fp32) lines fit,
// i.e. 32 / 64-byte column segments; these shapes take 8 / 16 lines (128-byte
// segments) in one 139 KB workgroup of 512 threads per CU.
struct CtShapeD1024W {
  static constexpr int E = 16, R0 = 16, R1 = 16, R2 = 4, kBudget = 150 * 1024, kMaxThr = 512;
};
struct CtShapeF1024W {
  static constexpr int E = 32, R0 = 16, R1 = 16, R2 = 4, kBudget = 150 * 1024, kMaxThr = 512;
};
template <>
struct CtShapeSel<double, 1024, 1, true> : CtShapeD1024W {};
template <>
struct CtShapeSel<double, 1024, -1, true> : CtShapeD1024W {};
template <>
struct CtShapeSel<float, 1024, 1, true> : CtShapeF1024W {};
template <>
struct CtShapeSel<float, 1024, -1, true> : CtShapeF1024W {};
struct CtShapeF512W {
  static constexpr int E = 16, R0 = 16, R1 = 16, R2 = 2, kBudget = 80 * 1024, kMaxThr = 512;
  static constexpr bool kTwTable = true;
};
// fp32 N = 512 line-fast forward engines: 32 elements per lane, radices 32 x 16
// (one LDS exchange per line instead of two; 256 threads, 16 lines). Measured on
// MI355X, same box (profiles/r5/ab/f512e32): y forward 218.4 -> 202.5 us (512^3
// R2C fp32), x forward 575.7 -> 410.0 and y forward 411.2 -> 386.0 us (512^3 C2C
// fp32). The backward kernels keep the 512-thread radix-16 shape: at 174 VGPRs
// and half the waves per SIMD the 32-element shape gained nothing there
// (y backward 219.2 -> 219.7, x backward 377.6 -> 384.1 us).
struct CtShapeF512E32 {
  static constexpr int E = 32, R0 = 32, R1 = 16, R2 = 1, kBudget = 80 * 1024, kMaxThr = 256;
};
template <>
struct CtShapeSel<float, 512, -1, true> : CtShapeF512E32 {};
// (1024-thread radix-8 backward shape: y backward 229 -> 293 us, x backward
// 391 -> 363 us at 512^3; a 512-thread radix-8 fp32 N = 256 shape: kernel sum
// 264 -> 293 us; profiles/r5/ab/f32w)
template <>
struct CtShapeSel<float, 512, 1, true> : CtShapeF512W {};
struct CtShapeD512W {
  static constexpr int E = 8, R0 = 8, R1 = 8, R2 = 8, kBudget = 80 * 1024, kMaxThr = 512;
};
template <>
struct CtShapeSel<double, 512, 1, true> : CtShapeD512W {};
template <>
struct CtShapeSel<double, 512, -1, true> : CtShapeD512W {};
// (re-measured in round 5 with twiddle powers: the 16-element line-fast shape,
// 128 threads per 8 lines, is still slower, x backward 92.0 -> 99.0 us,
// profiles/r5/ab/lf16)
template <>
struct CtShapeSel<double, 256, 1, true> : CtShape256E8 {};
template <>
struct CtShapeSel<double, 256, -1, true> : CtShape256E8 {};
template <>
struct CtShapeSel<double, 256, 1, false> : CtShape256E8 {};
// fp32 N = 512 z backward (row-mapped): 16 elements per lane, radices 16 x 16 x 2
// (32 lanes per line). Measured on MI355X, same box (profiles/r5/ab/z512): 512^3
// R2C z backward 145.9 -> 139.3 us; for the z forward it is slower (112 -> 133
// us) and the 32-element shape slower in both (169 / 153 us).
struct CtShapeZ512B {
  static constexpr int E = 16, R0 = 16, R1 = 16, R2 = 2, kBudget = kLdsBudget;
};
template <>
struct CtShapeSel<float, 512, 1, false> : CtShapeZ512B {};
// (fp32 z backward likewise: 31.1 -> 28.9-29.3 us at 256^3; the z forward
// stages are no faster with E = 8 in either precision, profiles/r5/ab/zf)
template <>
struct CtShapeSel<float, 256, 1, false> : CtShape256E8 {};

// Twiddles of a pass: one table entry per butterfly group and its powers
// formed in registers (twiddle_powers), unless the shape declares
// kTwTable = true (every power read from the table). Powers measured on MI355X
// (profiles/r5/ab/twpow): 256^3 C2C fp32 kernel sum 282.7 -> 262.6 us, fp64
// 494.6 -> 486.0 us, 512^3 R2C fp32 z forward 150.5 -> 111.1 us. The wide fp32
// N = 512 backward shape keeps the table: powers took its y stage from 125 to
// 130 VGPRs, past the occupancy step of its 512-thread workgroups (221 -> 295 us).
template <class Sh, class = void>
struct ShapeTwTable : std::false_type {};
template <class Sh>
struct ShapeTwTable<Sh, std::void_t<decltype(Sh::kTwTable)>> : std::integral_constant<bool, Sh::kTwTable> {};

// Workgroup size cap of a shape: Sh::kMaxThr where a shape declares it (wide
// 512-thread shapes), else kMaxThreads.
template <class Sh, class = void>
struct ShapeMaxThreads {
  static constexpr int value = kMaxThreads;
};
template <class Sh>
struct ShapeMaxThreads<Sh, std::void_t<decltype(Sh::kMaxThr)>> {
  static constexpr int value = Sh::kMaxThr;
};

struct NoLoad {};  // input already placed in LDS at Engine::in_at(b, pos)

// Element loads of the first pass. A load functor may also take the element's
// offset from the lane's first position t (pos = t + off, off a compile-time
// constant of the unrolled load): a kernel that addresses the lane's elements
// from one base pointer then does no arithmetic on pos, which the compiler
// cannot recover once it has turned t + off into t | off.
template <class Load>
__device__ __forceinline__ auto load_at(Load& load, int b, int t, int off) {
  if constexpr (std::is_invocable<Load&, int, int, int>::value)
    return load(b, t + off, off);
  else
    return load(b, t + off);
}

// largest power of two <= b, at most 16 (line-fast lane mapping)
__host__ __device__ constexpr int lf_lines(int b) {
  int p = 1;
  while (p * 2 <= b && p * 2 <= kLfMaxLines) p *= 2;
  return p;
}

// Line stride of the line-fast mapping (lane = line b fastest, then position t).
// gfx950 LDS banking (MI355X_MICROARCH.md §LDS): every ds_write and ds_read2 is
// serviced in 16-lane groups on 32 banks (128 B), ds_read_b128 in four
// non-contiguous 16-lane groups on 64 banks. A 16-lane group of 8-byte elements
// (fp32) holds 16/B positions of B lines, so the lines must fall on distinct
// 8-byte slots of 128 B: stride == 16/B (mod 32/B), odd for B = 16. For 16-byte
// elements (fp64) B = 8 lines are best at stride == 7 or 9 (mod 16) (4/3 of the
// conflict-free cycles, the b128 read groups mix lines and positions), B = 16
// at odd strides. The round-3 stride (== kMod/B, made for 64 banks) left every
// exchange 2-way conflicted: tools/lds_bank_model.py models each access, and
// SQ_LDS_BANK_CONFLICT measured 43-47% of the LDS cycles of the y stages
// (profiles/r4/pmc).
__host__ __device__ constexpr bool lds_line_stride_ok(int ls, int lines, int elemBytes) {
  if (elemBytes == 16 && lines == 8) return ls % 16 == 7 || ls % 16 == 9;
  const int m = lines >= 16 ? 1 : (elemBytes == 8 ? 16 : 8) / lines;
  return ls % (2 * m) == m;
}
template <typename T>
__host__ __device__ constexpr int lf_padded_stride(int n, int b, int shift) {
  int ls = n + ((n - 1) >> shift) + 1;
  while (!lds_line_stride_ok(ls, b, 2 * static_cast<int>(sizeof(T)))) ++ls;
  return ls;
}

// Twiddles w^1 .. w^(R-1) of one radix-R butterfly group from w = w^1 (one
// table load instead of R - 1): products of at most log2(R) + 1 factors, so
// the error stays within a few ulp.
template <int R, typename T>
__device__ __forceinline__ void twiddle_powers(cx<T> w, cx<T> (&p)[R - 1]) {
  p[0] = w;
#pragma unroll
  for (int r = 2; r < R; ++r) {
    // r = a + b with a the largest power of two below r (or r / 2 for powers of two)
    int a = 1;
    while (a * 2 < r) a *= 2;
    p[r - 1] = cmul(p[a - 1], p[r - a - 1]);
  }
}

// LF (line-fast) selects the lane -> (line b, lane t) mapping:
//  false: t fastest (a line's TP lanes adjacent; row-contiguous global access),
//  true:  b fastest (B lines adjacent; column-contiguous global access, e.g. a
//         stick's z-run or an intermediate column's y-run).
template <typename T, int N, int S, bool LF = false, bool TwPre = true>
struct FftCT {
  // line-fast engines (column access) take the precision-specific shape; the
  // row-mapped engine of the z stage keeps the default (fewer VGPRs per lane);
  // CtShapeSel overrides per stage kind where measured faster
  using Sh = CtShapeSel<T, N, S, LF>;
  static constexpr int E = Sh::E;
  static constexpr int TP = N / E;  // lanes per line
  static constexpr int PS = pad_shift<T>(E);
  static constexpr int LS0 = padded_stride<T>(N, PS);
  static constexpr int kMaxThr = ShapeMaxThreads<Sh>::value;
  static constexpr int B0 =
      lines_per_block(TP, LS0 * static_cast<int>(sizeof(cx<T>)), Sh::kBudget, kMaxThr);
  static constexpr int B = LF ? lf_lines(B0) : B0;
  static constexpr int LS = LF ? lf_padded_stride<T>(N, B, PS) : LS0;
  static constexpr int NT = B * TP;
  static constexpr int RL = Sh::R2 > 1 ? Sh::R2 : (Sh::R1 > 1 ? Sh::R1 : Sh::R0);
  static constexpr bool kTwPow = !ShapeTwTable<Sh>::value;

  static constexpr int lines() { return B; }
  static constexpr int threads() { return NT; }
  static constexpr std::size_t lds_bytes() { return std::size_t(B) * LS * sizeof(cx<T>); }
  __device__ static int in_at(int b, int pos) { return b * LS + pad_index(pos, PS); }
  __device__ static int out_at(int b, int pos) { return b * LS + pad_index(pos, PS); }

  // butterflies of one pass on the lane's registers (input order: v[k*R + r]
  // holds element j + r*N/R with j = t + k*TP)
  using TwT = T;  // twiddle table precision

  template <int R, int NS>
  __device__ static void compute(cx<T> (&v)[E], int t, const cx<TwT>* __restrict__ tw) {
#pragma unroll
    for (int k = 0; k < E / R; ++k) {
      if (NS > 1) {
        const int j = t + k * TP;
        const int kk = j % NS;
        if constexpr (kTwPow) {
          cx<T> p[R - 1];
          twiddle_powers<R>(tw[kk * (N / (NS * R))], p);
#pragma unroll
          for (int r = 1; r < R; ++r) v[k * R + r] = twm<S>(v[k * R + r], p[r - 1]);
        } else {
#pragma unroll
          for (int r = 1; r < R; ++r)
            v[k * R + r] = twm<S>(v[k * R + r], tw[kk * r * (N / (NS * R))]);
        }
      }
      Dft<R, S, T>::run(&v[k * R]);
    }
  }

  // write pass outputs (Stockham positions) to LDS and read the next pass inputs
  template <int R, int NS, int RN>
  __device__ static void exchange(cx<T> (&v)[E], cx<T>* line, int t) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < E / R; ++k) {
      const int j = t + k * TP;
      const int kk = j % NS;
      const int base = (j - kk) * R + kk;
#pragma unroll
      for (int r = 0; r < R; ++r) line[pad_index(base + r * NS, PS)] = v[k * R + r];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < E / RN; ++k) {
      const int j = t + k * TP;
#pragma unroll
      for (int r = 0; r < RN; ++r) v[k * RN + r] = line[pad_index(j + r * (N / RN), PS)];
    }
  }

  // Twiddles of a pass, fetched into registers ahead of the pass: their loads
  // are issued before the LDS exchange that precedes the pass, so the table
  // read (an L1/L2 hit) overlaps the exchange instead of following it.
  // (not for the 32-element shapes of N = 1024: their registers are full)
  static constexpr bool kTwPrefetch = TwPre && E <= 16;
  // (kTwPow: one table entry per butterfly group, its powers formed in compute_tw)
  template <int R, int NS>
  struct PassTw {
    cx<TwT> w[kTwPow ? E / R : (E / R) * (R - 1)];
  };
  template <int R, int NS>
  __device__ static void fetch_tw(PassTw<R, NS>& p, int t, const cx<TwT>* __restrict__ tw) {
#pragma unroll
    for (int k = 0; k < E / R; ++k) {
      const int kk = (t + k * TP) % NS;
      if constexpr (kTwPow) {
        p.w[k] = tw[kk * (N / (NS * R))];
      } else {
#pragma unroll
        for (int r = 1; r < R; ++r) p.w[k * (R - 1) + r - 1] = tw[kk * r * (N / (NS * R))];
      }
    }
  }
  template <int R, int NS>
  __device__ static void compute_tw(cx<T> (&v)[E], const PassTw<R, NS>& p) {
#pragma unroll
    for (int k = 0; k < E / R; ++k) {
      if constexpr (kTwPow) {
        cx<T> w[R - 1];
        twiddle_powers<R>(p.w[k], w);
#pragma unroll
        for (int r = 1; r < R; ++r) v[k * R + r] = twm<S>(v[k * R + r], w[r - 1]);
      } else {
#pragma unroll
        for (int r = 1; r < R; ++r) v[k * R + r] = twm<S>(v[k * R + r], p.w[k * (R - 1) + r - 1]);
      }
      Dft<R, S, T>::run(&v[k * R]);
    }
  }

  template <class Load>
  __device__ __forceinline__ static void transform(cx<T> (&v)[E], cx<T>* lds, const cx<TwT>* __restrict__ tw,
                                   Load load, int b, int t) {
    cx<T>* line = lds + b * LS;
#pragma unroll
    for (int k = 0; k < E / Sh::R0; ++k) {
      const int j = t + k * TP;
#pragma unroll
      for (int r = 0; r < Sh::R0; ++r) {
        if constexpr (std::is_same<Load, NoLoad>::value)
          v[k * Sh::R0 + r] = line[pad_index(j + r * (N / Sh::R0), PS)];
        else
          v[k * Sh::R0 + r] = load_at(load, b, t, k * TP + r * (N / Sh::R0));
      }
    }
    compute<Sh::R0, 1>(v, t, tw);
    if constexpr (kTwPrefetch) {
      if constexpr (Sh::R1 > 1) {
        PassTw<Sh::R1, Sh::R0> p1;
        fetch_tw(p1, t, tw);
        exchange<Sh::R0, 1, Sh::R1>(v, line, t);
        compute_tw(v, p1);
      }
      if constexpr (Sh::R2 > 1) {
        PassTw<Sh::R2, Sh::R0 * Sh::R1> p2;
        fetch_tw(p2, t, tw);
        exchange<Sh::R1, Sh::R0, Sh::R2>(v, line, t);
        compute_tw(v, p2);
      }
    } else {
      if constexpr (Sh::R1 > 1) {
        exchange<Sh::R0, 1, Sh::R1>(v, line, t);
        compute<Sh::R1, Sh::R0>(v, t, tw);
      }
      if constexpr (Sh::R2 > 1) {
        exchange<Sh::R1, Sh::R0, Sh::R2>(v, line, t);
        compute<Sh::R2, Sh::R0 * Sh::R1>(v, t, tw);
      }
    }
  }

  // Result delivered to store(b, pos, value); stores of a lane are at
  // pos = t + k*TP + r*N/RL (consecutive lanes -> consecutive positions).
  // Contract: run() stores only the lane's own line (b == lane_line()); the z
  // forward kernel keeps that line's stick descriptor in registers and relies
  // on it (asserted there in debug builds).
  __device__ static int lane_line() { return LF ? threadIdx.x % B : threadIdx.x / TP; }
  __device__ static int lane_pos() { return LF ? threadIdx.x / B : threadIdx.x % TP; }

  // The positions run() hands to store(), in call order: call i of store()
  // receives position pos of fn(i, pos) (kStoreSlots calls, all unrolled).
  static constexpr int kStoreSlots = E;
  template <class Fn>
  __device__ static void for_each_store_pos(Fn fn) {
    const int t = lane_pos();
#pragma unroll
    for (int k = 0; k < E / RL; ++k) {
#pragma unroll
      for (int r = 0; r < RL; ++r) fn(k * RL + r, t + k * TP + r * (N / RL));
    }
  }

  template <class Load, class Store>
  __device__ __forceinline__ static void run(cx<T>* lds, const cx<TwT>* __restrict__ tw, Load load, Store store) {
    const int b = lane_line(), t = lane_pos();
    cx<T> v[E];
    transform(v, lds, tw, load, b, t);
#pragma unroll
    for (int k = 0; k < E / RL; ++k) {
      const int j = t + k * TP;
#pragma unroll
      for (int r = 0; r < RL; ++r) store(b, j + r * (N / RL), v[k * RL + r]);
    }
  }

  // Result left in LDS at out_at(b, pos); ends with a barrier.
  template <class Load>
  __device__ __forceinline__ static void run_to_lds(cx<T>* lds, const cx<TwT>* __restrict__ tw, Load load) {
    const int b = lane_line(), t = lane_pos();
    cx<T> v[E];
    transform(v, lds, tw, load, b, t);
    __syncthreads();
    cx<T>* line = lds + b * LS;
#pragma unroll
    for (int k = 0; k < E / RL; ++k) {
      const int j = t + k * TP;
#pragma unroll
      for (int r = 0; r < RL; ++r) line[pad_index(j + r * (N / RL), PS)] = v[k * RL + r];
    }
    __syncthreads();
  }
};

// ------------------------------------------------ compile-time mixed radix
// Lengths built from the codelet radices that are not powers of two (240 =
// 16 * 15, 200 = 20 * 10, 192 = 16 * 12, ...) get the FftCT treatment instead
// of the run-time engine: the first pass is loaded straight from global memory,
// the last pass stored straight from registers, the passes in between
// exchanged through LDS, and every index is a compile-time constant. A pass of
// radix R has N / R butterflies, spread over the line's TP lanes (lanes past
// the count idle in that pass). mr_plan picks the radices (at most 4 passes,
// non-increasing) and TP that minimise the padded lane work sum_i TP * ceil(N /
// R_i / TP) * R_i under a register cap per lane (mr_sel).
// Plan limits per stage kind, measured on MI355X at 192^3, 200^3 and 240^3
// (profiles/r2_s1/mr_ab.txt): the forward stages run fastest with the
// fewest passes (up to 20 elements per lane, 200 = 20 * 10); the backward
// stages with at most 16 (200 = 10 * 10 * 2); the fp64 backward line-fast
// stages (the y stage's sparse stick loads) with at least 32 lanes per line;
// the row-mapped z stages with 256-thread workgroups.
struct MrSel {
  int emax, minTp, maxThr;
};
template <typename T, int S, bool LF>
__host__ __device__ constexpr MrSel mr_sel() {
  if (S < 0) return MrSel{20, 2, 256};
  if (!LF) return MrSel{16, 2, 256};
  return MrSel{16, sizeof(T) == 8 ? 32 : 2, 512};
}

struct MrPlan {
  int np, r[4], tp, e, cost;
};

__host__ __device__ constexpr bool mr_codelet(int r) {
  return (r >= 2 && r <= 13) || r == 15 || r == 16 || r == 20;
}
__host__ __device__ constexpr int mr_cdiv(int a, int b) { return (a + b - 1) / b; }

__host__ __device__ constexpr MrPlan mr_score(int n, MrPlan p, int emax, int minTp) {
  p.tp = 0;
  p.cost = 1 << 30;
  for (int tp = minTp; tp <= 64; ++tp) {
    int cost = 0, e = 0;
    for (int i = 0; i < p.np; ++i) {
      const int k = mr_cdiv(n / p.r[i], tp);
      cost += tp * k * p.r[i];
      if (k * p.r[i] > e) e = k * p.r[i];
    }
    if (e > emax) continue;
    if (cost < p.cost || (cost == p.cost && e < p.e)) {
      p.tp = tp;
      p.e = e;
      p.cost = cost;
    }
  }
  return p;
}

__host__ __device__ constexpr void mr_search(int n, int m, MrPlan cur, int maxr, int emax,
                                             int minTp, MrPlan& best) {
  if (m == 1) {
    const MrPlan s = mr_score(n, cur, emax, minTp);
    if (s.tp && s.cost < best.cost) best = s;
    return;
  }
  if (cur.np == 4) return;
  for (int a = maxr; a >= 2; --a) {
    if (!mr_codelet(a) || m % a) continue;
    MrPlan next = cur;
    next.r[next.np++] = a;
    mr_search(n, m / a, next, a, emax, minTp, best);
  }
}

__host__ __device__ constexpr MrPlan mr_plan(int n, int emax, int minTp) {
  MrPlan best{0, {1, 1, 1, 1}, 0, 0, 1 << 30};
  mr_search(n, n, MrPlan{0, {1, 1, 1, 1}, 0, 0, 0}, 20, emax, minTp, best);
  return best;
}

// Same interface and lane mapping as FftCT (LF: lines fastest).
template <typename T, int N, int S, bool LF = false>
struct FftMR {
  static constexpr MrSel Sel = mr_sel<T, S, LF>();
  static constexpr MrPlan P = mr_plan(N, Sel.emax, Sel.minTp);
  static_assert(P.np > 0, "length has no mixed-radix plan");
  static constexpr int NP = P.np;
  static constexpr int TP = P.tp;
  static constexpr int E = P.e;
  static constexpr int PS = pad_shift<T>(E);
  static constexpr int LS0 = padded_stride<T>(N, PS);
  static constexpr int kMaxThr = Sel.maxThr;
  static constexpr int B0 =
      lines_per_block(TP, LS0 * static_cast<int>(sizeof(cx<T>)), kLdsBudget, kMaxThr);
  static constexpr int B = LF ? lf_lines(B0) : B0;
  static constexpr int LS = LF ? lf_padded_stride<T>(N, B, PS) : LS0;
  static constexpr int NT = B * TP;

  static constexpr int lines() { return B; }
  static constexpr int threads() { return NT; }
  static constexpr std::size_t lds_bytes() { return std::size_t(B) * LS * sizeof(cx<T>); }
  __device__ static int in_at(int b, int pos) { return b * LS + pad_index(pos, PS); }
  __device__ static int out_at(int b, int pos) { return b * LS + pad_index(pos, PS); }
  __device__ static int lane_line() { return LF ? threadIdx.x % B : threadIdx.x / TP; }
  __device__ static int lane_pos() { return LF ? threadIdx.x / B : threadIdx.x % TP; }

  template <int I>
  static constexpr int radix() { return P.r[I]; }
  template <int I>
  static constexpr int stride_ns() {  // product of the radices before pass I
    int ns = 1;
    for (int i = 0; i < I; ++i) ns *= P.r[i];
    return ns;
  }
  template <int I>
  static constexpr int iters() { return mr_cdiv(N / radix<I>(), TP); }
  template <int I>
  __device__ static bool active(int j) { return (N / radix<I>()) % TP == 0 || j < N / radix<I>(); }

  // pass I inputs: v[k*R + r] = element j + r*N/R of the line, j = t + k*TP
  template <int I, class Load>
  __device__ static void gather(cx<T> (&v)[E], const cx<T>* line, Load load, int b, int t) {
    constexpr int R = radix<I>(), NB = N / R;
#pragma unroll
    for (int k = 0; k < iters<I>(); ++k) {
      const int j = t + k * TP;
      if (!active<I>(j)) continue;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (std::is_same<Load, NoLoad>::value)
          v[k * R + r] = line[pad_index(j + r * NB, PS)];
        else
          v[k * R + r] = load_at(load, b, t, k * TP + r * NB);
      }
    }
  }

  template <int I>
  __device__ static void butterflies(cx<T> (&v)[E], int t, const cx<T>* __restrict__ tw) {
    constexpr int R = radix<I>(), NS = stride_ns<I>();
#pragma unroll
    for (int k = 0; k < iters<I>(); ++k) {
      const int j = t + k * TP;
      if (!active<I>(j)) continue;
      if (NS > 1) {
        const int kk = j % NS;
#pragma unroll
        for (int r = 1; r < R; ++r)
          v[k * R + r] = twm<S>(v[k * R + r], tw[kk * r * (N / (NS * R))]);
      }
      Dft<R, S, T>::run(&v[k * R]);
    }
  }

  // pass I outputs to their Stockham positions in LDS
  template <int I>
  __device__ static void scatter(cx<T> (&v)[E], cx<T>* line, int t) {
    constexpr int R = radix<I>(), NS = stride_ns<I>();
#pragma unroll
    for (int k = 0; k < iters<I>(); ++k) {
      const int j = t + k * TP;
      if (!active<I>(j)) continue;
      const int kk = j % NS;
      const int base = (j - kk) * R + kk;
#pragma unroll
      for (int r = 0; r < R; ++r) line[pad_index(base + r * NS, PS)] = v[k * R + r];
    }
  }

  template <int I>
  __device__ static void later_passes(cx<T> (&v)[E], cx<T>* line, int t, const cx<T>* __restrict__ tw) {
    __syncthreads();
    scatter<I - 1>(v, line, t);
    __syncthreads();
    gather<I>(v, line, NoLoad{}, 0, t);
    butterflies<I>(v, t, tw);
    if constexpr (I + 1 < NP) later_passes<I + 1>(v, line, t, tw);
  }

  template <class Load>
  __device__ __forceinline__ static void transform(cx<T> (&v)[E], cx<T>* lds, const cx<T>* __restrict__ tw,
                                   Load load, int b, int t) {
    cx<T>* line = lds + b * LS;
    gather<0>(v, line, load, b, t);
    butterflies<0>(v, t, tw);
    if constexpr (NP > 1) later_passes<1>(v, line, t, tw);
  }

  // Result delivered to store(b, pos, value), only for the lane's own line
  // (the FftCT contract); consecutive lanes -> consecutive positions.
  template <class Load, class Store>
  __device__ __forceinline__ static void run(cx<T>* lds, const cx<T>* __restrict__ tw, Load load, Store store) {
    const int b = lane_line(), t = lane_pos();
    cx<T> v[E];
    transform(v, lds, tw, load, b, t);
    constexpr int RL = radix<NP - 1>(), NB = N / RL;
#pragma unroll
    for (int k = 0; k < iters<NP - 1>(); ++k) {
      const int j = t + k * TP;
      if (!active<NP - 1>(j)) continue;
#pragma unroll
      for (int r = 0; r < RL; ++r) store(b, j + r * NB, v[k * RL + r]);
    }
  }

  // Result left in LDS at out_at(b, pos); ends with a barrier.
  template <class Load>
  __device__ __forceinline__ static void run_to_lds(cx<T>* lds, const cx<T>* __restrict__ tw, Load load) {
    const int b = lane_line(), t = lane_pos();
    cx<T> v[E];
    transform(v, lds, tw, load, b, t);
    __syncthreads();
    cx<T>* line = lds + b * LS;
    constexpr int RL = radix<NP - 1>(), NB = N / RL;
#pragma unroll
    for (int k = 0; k < iters<NP - 1>(); ++k) {
      const int j = t + k * TP;
      if (!active<NP - 1>(j)) continue;
#pragma unroll
      for (int r = 0; r < RL; ++r) line[pad_index(j + r * NB, PS)] = v[k * RL + r];
    }
    __syncthreads();
  }
};

// Compile-time engine core of a length: FftCT for powers of two, else FftMR.
template <typename T, int N, int S, bool LF, bool TwPre = true>
struct CtCore {
  using type = typename std::conditional<(N & (N - 1)) == 0, FftCT<T, N, S, LF, TwPre>,
                                         FftMR<T, N, S, LF>>::type;
};

// ---------------------------------------------------------------- RT engine
struct RtPlan {
  int n;       // length
  int np;      // number of passes
  int ls;      // line stride (elements)
  int lines;   // lines per block (a power of two)
  int linesLog2;
  int inplace;          // 1: every radix has a codelet -> one LDS region, register-staged passes
  unsigned nMagic;      // ceil(2^32 / n): idx / n == umulhi(idx, nMagic) for idx * n < 2^32
  int radix[16];
  unsigned nsMagic[16];  // ceil(2^32 / ns) of each pass (ns = product of the earlier radices)
};

// Prime-factor composite radices (6, 10, 12, 15, 20) in the run-time engine:
// fewer passes per transform (240 = 16 * 15 instead of 16 * 5 * 3). Measured on
// MI355X (profiles/README.md, session 12): +10-13% for fp64 at 100^3-240^3, but
// -7% for fp32 at 240^3, where the larger pass switch costs more than the saved
// pass: fp64 only.
__host__ __device__ constexpr bool rt_pfa(bool dbl) { return dbl; }
__host__ __device__ constexpr bool rt_composite_radix(int r) {
  return r == 6 || r == 10 || r == 12 || r == 15 || r == 20;
}

// Butterflies per lane in an in-place pass of radix R: at most kRtElems /
// kRtThreads (16) elements per lane for every radix, so the register staging is
// the same for all radices (make_rt_plan sizes the lines so that each pass
// fits; a plan that cannot falls back to the ping-pong passes).
__host__ __device__ constexpr int rt_iters(int r) {
  return (kRtElems / kRtThreads) / r > 0 ? (kRtElems / kRtThreads) / r : 1;
}

// Radices with a codelet (the in-place run-time passes are instantiated for these).
__host__ __device__ constexpr bool rt_codelet_radix(int r, bool pfa) {
  return r == 2 || r == 3 || r == 4 || r == 5 || r == 7 || r == 8 || r == 9 || r == 11 ||
         r == 13 || r == 16 || (pfa && rt_composite_radix(r));
}

// A kernel-uniform value the compiler must treat as produced here: without it,
// the per-radix products of p.n (n / R, r * n / R for every radix of the pass
// switches) are hoisted into the kernel prologue, where they exceed the SGPR
// file and spill (measured: 276-596 spilled SGPRs per run-time kernel).
__device__ __forceinline__ int opaque_uniform(int v) {
  v = __builtin_amdgcn_readfirstlane(v);
  asm volatile("" : "+s"(v));
  return v;
}

template <typename T, int S>
struct FftRT {
  __device__ static int in_at(const RtPlan& p, int b, int pos) { return b * p.ls + pos; }

  // In-place Stockham pass of radix R over all lines of the block (blockDim.x ==
  // kRtThreads). Work item idx -> (line b = idx mod lines, butterfly j = idx /
  // lines): lines fastest, so a wave's LDS accesses spread over the lines' bank
  // offsets (plan stride, make_rt_plan). Every lane loads all its butterflies
  // into registers before the barrier and stores after it.
  template <int R>
  __device__ static void pass_inplace(const RtPlan& p, cx<T>* buf, int ns, unsigned nsMagic,
                                      const cx<T>* __restrict__ tw) {
    constexpr int kIt = rt_iters(R);
    const int n = opaque_uniform(p.n);
    const int nb = n / R;
    const int total = nb << p.linesLog2;
    const int twStride = n / (ns * R);
    cx<T> v[kIt][R];
    int dst[kIt];
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int idx = threadIdx.x + it * kRtThreads;
      if (idx < total) {
        const int b = idx & (p.lines - 1);
        const int j = idx >> p.linesLog2;
        const int kk =
            ns == 1 ? 0 : j - ns * static_cast<int>(__umulhi(static_cast<unsigned>(j), nsMagic));
        const cx<T>* s = buf + b * p.ls + j;
#pragma unroll
        for (int r = 0; r < R; ++r) v[it][r] = s[r * nb];
        if (kk) {
#pragma unroll
          for (int r = 1; r < R; ++r) v[it][r] = twm<S>(v[it][r], tw[kk * r * twStride]);
        }
        Dft<R, S, T>::run(v[it]);
        dst[it] = b * p.ls + (j - kk) * R + kk;
      }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int idx = threadIdx.x + it * kRtThreads;
      if (idx < total) {
#pragma unroll
        for (int r = 0; r < R; ++r) buf[dst[it] + r * ns] = v[it][r];
      }
    }
    __syncthreads();
  }

  __device__ static void run_inplace(const RtPlan& p, cx<T>* buf, const cx<T>* __restrict__ tw) {
    int ns = 1;
    for (int i = 0; i < p.np; ++i) {
      const unsigned m = p.nsMagic[i];
      const int r = p.radix[i];
      if (rt_pfa(sizeof(T) == 8) && rt_composite_radix(r)) {
        if constexpr (rt_pfa(sizeof(T) == 8)) {
          switch (r) {
            case 6: pass_inplace<6>(p, buf, ns, m, tw); break;
            case 10: pass_inplace<10>(p, buf, ns, m, tw); break;
            case 12: pass_inplace<12>(p, buf, ns, m, tw); break;
            case 15: pass_inplace<15>(p, buf, ns, m, tw); break;
            default: pass_inplace<20>(p, buf, ns, m, tw); break;
          }
        }
      } else {
        switch (r) {
          case 2: pass_inplace<2>(p, buf, ns, m, tw); break;
          case 3: pass_inplace<3>(p, buf, ns, m, tw); break;
          case 4: pass_inplace<4>(p, buf, ns, m, tw); break;
          case 5: pass_inplace<5>(p, buf, ns, m, tw); break;
          case 7: pass_inplace<7>(p, buf, ns, m, tw); break;
          case 8: pass_inplace<8>(p, buf, ns, m, tw); break;
          case 9: pass_inplace<9>(p, buf, ns, m, tw); break;
          case 11: pass_inplace<11>(p, buf, ns, m, tw); break;
          case 13: pass_inplace<13>(p, buf, ns, m, tw); break;
          default: pass_inplace<16>(p, buf, ns, m, tw); break;
        }
      }
      ns *= p.radix[i];
    }
  }

  template <int R>
  __device__ static void pass(const RtPlan& p, const cx<T>* src, cx<T>* dst, int ns,
                              const cx<T>* __restrict__ tw) {
    const int n = opaque_uniform(p.n);
    const int nb = n / R;
    const int twStride = n / (ns * R);
    const int total = p.lines * nb;
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
      const int b = idx / nb, j = idx - b * nb;
      const int kk = j % ns;
      const cx<T>* s = src + b * p.ls;
      cx<T> v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = s[j + r * nb];
      if (kk) {
#pragma unroll
        for (int r = 1; r < R; ++r) v[r] = twm<S>(v[r], tw[kk * r * twStride]);
      }
      Dft<R, S, T>::run(v);
      cx<T>* d = dst + b * p.ls + (j - kk) * R + kk;
#pragma unroll
      for (int r = 0; r < R; ++r) d[r * ns] = v[r];
    }
  }

  __device__ static void pass_generic(const RtPlan& p, const cx<T>* src, cx<T>* dst, int ns,
                                      int R, const cx<T>* __restrict__ tw) {
    const int nb = p.n / R;
    const int twStride = p.n / (ns * R);
    const int dftStride = p.n / R;
    const int total = p.lines * nb * R;
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
      const int q = idx % R;
      const int rest = idx / R;
      const int b = rest / nb, j = rest - b * nb;
      const int kk = j % ns;
      const cx<T>* s = src + b * p.ls;
      cx<T> acc = s[j];
      for (int r = 1; r < R; ++r) {
        cx<T> x = s[j + r * nb];
        if (kk) x = twm<S>(x, tw[static_cast<long long>(kk) * r * twStride]);
        const int e = static_cast<int>((static_cast<long long>(r) * q) % R);
        acc = acc + twm<S>(x, tw[e * dftStride]);
      }
      dst[b * p.ls + (j - kk) * R + kk + q * ns] = acc;
    }
  }

  // Input in region 0 at in_at(b, pos); returns the region holding the result
  // (index b*ls + pos). Ends with a barrier.
  __device__ __forceinline__ static cx<T>* run_in_lds(const RtPlan& p, cx<T>* lds, const cx<T>* __restrict__ tw) {
    if (p.inplace) {
      run_inplace(p, lds, tw);
      return lds;
    }
    return run_between(p, lds, lds + p.lines * p.ls, tw);
  }

  // Ping-pong between two LDS regions (input in src); returns the result region.
  __device__ __forceinline__ static cx<T>* run_between(const RtPlan& p, cx<T>* src, cx<T>* dst,
                                       const cx<T>* __restrict__ tw) {
    int ns = 1;
    for (int i = 0; i < p.np; ++i) {
      const int R = p.radix[i];
      switch (R) {
        case 2: pass<2>(p, src, dst, ns, tw); break;
        case 3: pass<3>(p, src, dst, ns, tw); break;
        case 4: pass<4>(p, src, dst, ns, tw); break;
        case 5: pass<5>(p, src, dst, ns, tw); break;
        case 7: pass<7>(p, src, dst, ns, tw); break;
        case 8: pass<8>(p, src, dst, ns, tw); break;
        case 9: pass<9>(p, src, dst, ns, tw); break;
        case 11: pass<11>(p, src, dst, ns, tw); break;
        case 13: pass<13>(p, src, dst, ns, tw); break;
        case 16: pass<16>(p, src, dst, ns, tw); break;
        default: pass_generic(p, src, dst, ns, R, tw); break;
      }
      __syncthreads();
      ns *= R;
      cx<T>* tmp = src;
      src = dst;
      dst = tmp;
    }
    return src;
  }
};

}  // namespace dev
}  // namespace spfft
