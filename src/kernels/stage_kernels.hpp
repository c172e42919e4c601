// Device code of the fused stage kernels (included by stage_launch.hpp and long_fft.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cassert>
#include <type_traits>

#include "gpu/gpu_runtime.hpp"
#include "kernels/fft_device.hpp"
#include "kernels/stage_args.hpp"
#include "fft/fft_plan.hpp"

namespace spfft {
namespace dev {

// Streaming global accesses: every stage reads and writes each element once, so
// loads and stores carry the non-temporal hint (measured on MI355X: 268 MB copy
// 6.15-6.28 TB/s with nt vs 5.65-5.88 TB/s without, tools/probes/hbm_copy.hip).
template <typename T>
__device__ __forceinline__ cx<T> ld_stream(const cx<T>* p) {
  using V = T __attribute__((ext_vector_type(2)));
  const V v = __builtin_nontemporal_load(reinterpret_cast<const V*>(p));
  return mk<T>(v.x, v.y);
}
template <typename T>
__device__ __forceinline__ void st_stream(cx<T>* p, cx<T> v) {
  using V = T __attribute__((ext_vector_type(2)));
  V w;
  w.x = v.x;
  w.y = v.y;
  __builtin_nontemporal_store(w, reinterpret_cast<V*>(p));
}
// Stick-side accesses of the backward z -> y hand-off: streaming (nt), or with
// the default cache policy (Plain: the lines stay in the 256 MB Infinity
// Cache, where the y stage finds them; GpuExecutor::plainHandoff_). Plain is a
// template parameter of the kernels, not a run-time flag: with a run-time
// branch the compiler merged the two stores (loads) of the branch into one and
// dropped the non-temporal hint, so every stick access ran plain (512^3 R2C
// fp32 z backward 146 -> 206 us, z forward 112 -> 129 us; profiles/r6/ntmerge).
template <bool Plain, typename T>
__device__ __forceinline__ cx<T> ld_stick(const cx<T>* p) {
  if constexpr (Plain) return *p;
  else return ld_stream(p);
}
template <bool Plain, typename T>
__device__ __forceinline__ void st_stick(cx<T>* p, cx<T> v) {
  if constexpr (Plain) *p = v;
  else st_stream(p, v);
}
// The [z][column][y] intermediate is streamed like the rest.
template <typename T>
__device__ __forceinline__ cx<T> ld_inter(const cx<T>* p) {
  return ld_stream(p);
}
template <typename T>
__device__ __forceinline__ void st_inter(cx<T>* p, cx<T> v) {
  st_stream(p, v);
}
// Sparse frequency values: a stick's values rarely start on a cache-line
// boundary, so neighbouring workgroups share lines; plain accesses keep them.
template <typename T>
__device__ __forceinline__ cx<T> ld_values(const cx<T>* p) {
  return *p;
}
template <typename T>
__device__ __forceinline__ void st_values(cx<T>* p, cx<T> v) {
  *p = v;
}
template <typename T>
__device__ __forceinline__ T ld_stream_real(const T* p) {
  return __builtin_nontemporal_load(p);
}
template <typename T>
__device__ __forceinline__ void st_stream_real(T* p, T v) {
  __builtin_nontemporal_store(v, p);
}

// Loads issued per lane before the first dependent LDS store: keeps U global
// loads in flight per lane (memory-level parallelism for the gathers).
constexpr int kGatherUnroll = 16;

// for idx in [0, total): lds[dst(idx)] = load(idx) (dst < 0: skip), U loads in flight.
template <typename T, class Load, class Dst>
__device__ __forceinline__ void gather_to_lds(cx<T>* lds, int total, Load load, Dst dst) {
  for (int base = threadIdx.x; base < total; base += blockDim.x * kGatherUnroll) {
    cx<T> v[kGatherUnroll];
#pragma unroll
    for (int u = 0; u < kGatherUnroll; ++u) {
      const int idx = base + u * static_cast<int>(blockDim.x);
      if (idx < total) v[u] = load(idx);
    }
#pragma unroll
    for (int u = 0; u < kGatherUnroll; ++u) {
      const int idx = base + u * static_cast<int>(blockDim.x);
      if (idx < total) {
        const int d = dst(idx);
        if (d >= 0) lds[d] = v[u];
      }
    }
  }
}

// for idx in [0, total): st(idx, lds[src(idx)]), U LDS reads in flight per lane
// before the dependent global stores (a plain loop waits out the LDS latency of
// every element).
template <typename T, class Src, class St>
__device__ __forceinline__ void scatter_from_lds(const cx<T>* lds, int total, Src src, St st) {
  for (int base = threadIdx.x; base < total; base += blockDim.x * kGatherUnroll) {
    cx<T> v[kGatherUnroll];
#pragma unroll
    for (int u = 0; u < kGatherUnroll; ++u) {
      const int idx = base + u * static_cast<int>(blockDim.x);
      if (idx < total) v[u] = lds[src(idx)];
    }
#pragma unroll
    for (int u = 0; u < kGatherUnroll; ++u) {
      const int idx = base + u * static_cast<int>(blockDim.x);
      if (idx < total) st(idx, v[u]);
    }
  }
}


// LDS -> global copy-out of a stage kernel: the run-time engines batch their LDS
// reads (scatter_from_lds, measured +5-7% at 100^3-240^3); the compile-time
// engines keep the plain loop (batching measured 1-2% slower at 128^3-256^3).
// A full tile of a compile-time engine (every line present) copies with a
// fully unrolled loop of compile-time trip count E: its LDS reads issue back to
// back instead of one read, wait and store per iteration.
template <class Eng, typename T, class Src, class St>
__device__ __forceinline__ void copy_out(const cx<T>* lds, int total, Src src, St st) {
  if constexpr (Eng::kBatchedCopy) {
    scatter_from_lds(lds, total, src, st);
  } else {
    using F = typename Eng::F;
    // (mixed-radix shapes can leave lanes idle: their tiles need not split evenly)
    constexpr bool kEven = (F::B * Eng::kN) % F::NT == 0;
    if (kEven && total == F::B * Eng::kN) {
      constexpr int kIters = kEven ? F::B * Eng::kN / F::NT : 1;
      cx<T> v[kIters];
#pragma unroll
      for (int i = 0; i < kIters; ++i) v[i] = lds[src(static_cast<int>(threadIdx.x) + i * F::NT)];
#pragma unroll
      for (int i = 0; i < kIters; ++i) st(static_cast<int>(threadIdx.x) + i * F::NT, v[i]);
      return;
    }
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) st(idx, lds[src(idx)]);
  }
}

// ------------------------------------------------------------ engine adapters
// TwPre: the FftCT twiddle prefetch (off for the kernels where its registers
// cost occupancy: the fp32 y forward kernels measured 61 -> 65 us at 256^3 and
// 260 -> 384 us at 512^3 with it, 129+ VGPRs, one 512-thread workgroup per CU)
template <typename T, int N, int S, bool LF = false, bool TwPre = true>
struct CtEng {
  using F = typename CtCore<T, N, S, LF, TwPre>::type;
  static constexpr int kN = N;
  static constexpr bool kBatchedCopy = false;
  static constexpr bool kLineFast = LF;
  static constexpr int kBlock = F::NT > kMaxThreads ? F::NT : kMaxThreads;
  __device__ __forceinline__ int lines() const { return F::B; }
  __device__ __forceinline__ int n() const { return N; }
  __device__ __forceinline__ int in_at(int b, int pos) const { return F::in_at(b, pos); }
  __device__ __forceinline__ int out_at(int b, int pos) const { return F::out_at(b, pos); }
  __device__ __forceinline__ int input_elems() const { return F::B * F::LS; }
  __device__ __forceinline__ int lds_bytes() const { return static_cast<int>(F::lds_bytes()); }
  template <class St>
  __device__ __forceinline__ void lds_to_global(cx<T>* lds, const cx<T>* __restrict__ tw, St st) const {
    F::run(lds, tw, NoLoad{}, st);
  }
  template <class Ld>
  __device__ __forceinline__ void global_to_lds(cx<T>* lds, const cx<T>* __restrict__ tw, Ld ld) const {
    F::run_to_lds(lds, tw, ld);
  }
  __device__ __forceinline__ void lds_to_lds(cx<T>* lds, const cx<T>* __restrict__ tw) const {
    F::run_to_lds(lds, tw, NoLoad{});
  }
  template <class Ld, class St>
  __device__ __forceinline__ void global_to_global(cx<T>* lds, const cx<T>* __restrict__ tw, Ld ld, St st) const {
    F::run(lds, tw, ld, st);
  }
  // host side
  static int h_lines() { return F::B; }
  static int h_threads() { return F::NT; }
  static std::size_t h_lds() { return F::lds_bytes(); }
};

// Run-time length engine. LF (line-fast) engines walk the global side with the
// line index fastest — consecutive lanes touch consecutive lines, i.e. the
// contiguous z-run of a stick or y-run of an intermediate column — like the
// compile-time line-fast mapping; row engines walk positions fastest.
template <typename T, int S, bool LF = false>
struct RtEng {
  static constexpr bool kBatchedCopy = true;
  static constexpr bool kLineFast = LF;
  static constexpr int kBlock = kRtThreads;
  RtPlan p;
  __device__ __forceinline__ int lines() const { return p.lines; }
  __device__ __forceinline__ int n() const { return p.n; }
  __device__ __forceinline__ int in_at(int b, int pos) const { return b * p.ls + pos; }
  __device__ __forceinline__ int out_at(int b, int pos) const {
    return ((!p.inplace && (p.np & 1)) ? p.lines * p.ls : 0) + b * p.ls + pos;
  }
  __device__ __forceinline__ int input_elems() const { return p.lines * p.ls; }
  __device__ __forceinline__ int lds_bytes() const {
    return (p.inplace ? 1 : 2) * p.lines * p.ls * static_cast<int>(sizeof(cx<T>));
  }
  // global-side element idx -> (line b, position pos); plan lines are a power
  // of two (make_rt_plan), so the line-fast split is a mask and a shift, and
  // the row split divides by a precomputed reciprocal
  __device__ __forceinline__ void split(int idx, int& b, int& pos) const {
    if (LF) {
      b = idx & (p.lines - 1);
      pos = idx >> p.linesLog2;
    } else {
      b = p.n == 1 ? idx : static_cast<int>(__umulhi(static_cast<unsigned>(idx), p.nMagic));
      pos = idx - b * p.n;
    }
  }
  template <class St>
  __device__ __forceinline__ void lds_to_global(cx<T>* lds, const cx<T>* __restrict__ tw, St st) const {
    const cx<T>* res = FftRT<T, S>::run_in_lds(p, lds, tw);
    store_from(res, st);
  }
  // input -> LDS at in_at(b, pos), no barrier (kernels with several input
  // paths stage each and then run the FFT once: one inlined copy of the passes)
  template <class Ld>
  __device__ __forceinline__ void stage(cx<T>* lds, Ld ld) const {
    gather_to_lds(lds, p.lines * p.n, [&](int idx) {
      int b, pos;
      split(idx, b, pos);
      return ld(b, pos);
    }, [&](int idx) {
      int b, pos;
      split(idx, b, pos);
      return b * p.ls + pos;
    });
  }
  template <class Ld>
  __device__ __forceinline__ void global_to_lds(cx<T>* lds, const cx<T>* __restrict__ tw, Ld ld) const {
    stage(lds, ld);
    __syncthreads();
    FftRT<T, S>::run_in_lds(p, lds, tw);
  }
  __device__ __forceinline__ void lds_to_lds(cx<T>* lds, const cx<T>* __restrict__ tw) const {
    FftRT<T, S>::run_in_lds(p, lds, tw);
  }
  template <class Ld, class St>
  __device__ __forceinline__ void global_to_global(cx<T>* lds, const cx<T>* __restrict__ tw, Ld ld, St st) const {
    global_to_lds(lds, tw, ld);
    store_from(lds + out_at(0, 0), st);
  }
  // result region res (index b * ls + pos) -> st(b, pos, v)
  template <class St>
  __device__ __forceinline__ void store_from(const cx<T>* res, St st) const {
    scatter_from_lds(res, p.lines * p.n, [&](int idx) {
      int b, pos;
      split(idx, b, pos);
      return b * p.ls + pos;
    }, [&](int idx, cx<T> v) {
      int b, pos;
      split(idx, b, pos);
      st(b, pos, v);
    });
  }
};

// Bluestein engine for lengths with a large prime factor (chirp-z: one
// convolution of power-of-two length m >= 2n-1 done with two run-time FFTs in
// LDS). X_k = d_k sum_j (x_j d_j) conj(d_{k-j}), d_j = exp(S i pi j^2 / n).
// Tables (device, per length): chirp d (S = -1) [n], FFT_m of the conj(d)
// filter for S = -1 and S = +1 [2m], twiddles of length m [m].
template <typename T, int S>
struct BlueEng {
  static constexpr bool kBatchedCopy = true;
  static constexpr bool kLineFast = false;
  static constexpr int kBlock = kMaxThreads;
  RtPlan pm;  // length m, ls = m
  int nn;
  const cx<T>* chirp;
  const cx<T>* filt;
  const cx<T>* twm;
  __device__ __forceinline__ int lines() const { return pm.lines; }
  __device__ __forceinline__ int n() const { return nn; }
  __device__ __forceinline__ int in_at(int b, int pos) const { return b * pm.ls + pos; }
  __device__ __forceinline__ int out_at(int b, int pos) const { return b * pm.ls + pos; }
  __device__ __forceinline__ int input_elems() const { return pm.lines * pm.ls; }
  __device__ __forceinline__ int lds_bytes() const { return 2 * pm.lines * pm.ls * static_cast<int>(sizeof(cx<T>)); }
  __device__ __forceinline__ cx<T> d(int j) const { return S < 0 ? chirp[j] : conj(chirp[j]); }
  __device__ __forceinline__ void run(cx<T>* lds) const {
    const int m = pm.n, total = pm.lines * m;
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
      const int b = idx / m, j = idx - b * m;
      cx<T>& v = lds[b * pm.ls + j];
      v = j < nn ? cmul(v, d(j)) : mk<T>(T(0), T(0));
    }
    __syncthreads();
    cx<T>* A = lds;
    cx<T>* B = lds + pm.lines * pm.ls;
    cx<T>* r = FftRT<T, -1>::run_between(pm, A, B, twm);
    const cx<T>* f = filt + (S < 0 ? 0 : m);
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
      const int b = idx / m, j = idx - b * m;
      r[b * pm.ls + j] = cmul(r[b * pm.ls + j], f[j]);
    }
    __syncthreads();
    cx<T>* r2 = FftRT<T, +1>::run_between(pm, r, r == A ? B : A, twm);
    const T inv = T(1) / static_cast<T>(m);
    for (int idx = threadIdx.x; idx < pm.lines * nn; idx += blockDim.x) {
      const int b = idx / nn, k = idx - b * nn;
      A[b * pm.ls + k] = scale(cmul(r2[b * pm.ls + k], d(k)), inv);
    }
    __syncthreads();
  }
  template <class St>
  __device__ __forceinline__ void lds_to_global(cx<T>* lds, const cx<T>* __restrict__, St st) const {
    run(lds);
    store_from(lds, st);
  }
  template <class Ld>
  __device__ __forceinline__ void stage(cx<T>* lds, Ld ld) const {
    gather_to_lds(lds, pm.lines * nn, [&](int idx) {
      const int b = idx / nn;
      return ld(b, idx - b * nn);
    }, [&](int idx) {
      const int b = idx / nn;
      return in_at(b, idx - b * nn);
    });
  }
  template <class Ld>
  __device__ __forceinline__ void global_to_lds(cx<T>* lds, const cx<T>* __restrict__, Ld ld) const {
    stage(lds, ld);
    __syncthreads();
    run(lds);
  }
  __device__ __forceinline__ void lds_to_lds(cx<T>* lds, const cx<T>* __restrict__) const { run(lds); }
  template <class Ld, class St>
  __device__ __forceinline__ void global_to_global(cx<T>* lds, const cx<T>* __restrict__ tw, Ld ld, St st) const {
    global_to_lds(lds, tw, ld);
    store_from(lds, st);
  }
  template <class St>
  __device__ __forceinline__ void store_from(const cx<T>* lds, St st) const {
    scatter_from_lds(lds, pm.lines * nn, [&](int idx) {
      const int b = idx / nn;
      return out_at(b, idx - b * nn);
    }, [&](int idx, cx<T> v) {
      const int b = idx / nn;
      st(b, idx - b * nn, v);
    });
  }
};

template <typename To, typename From>
__device__ __forceinline__ cx<To> cvt(const cx<From>& v) {
  return mk<To>(static_cast<To>(v.x), static_cast<To>(v.y));
}
template <typename T>
__device__ __forceinline__ bool nonzero(const cx<T>& v) {
  return v.x != T(0) || v.y != T(0);
}
template <typename T>
__device__ __forceinline__ cx<T> czero() {
  return mk<T>(T(0), T(0));
}

// Hermitian completion (only where the source is non-zero) of `count` LDS lines
// starting at line b0, with the two half passes of the reference
// (src/symmetry/gpu_kernels/symmetry_kernels.cu:56-78, 119-141) as two
// barrier-separated phases of one workgroup.
template <class Eng, typename T>
__device__ void hermitian_lines(const Eng& eng, cx<T>* lds, int b0, int count, int n) {
  const int h1 = n / 2;          // k in [1, n/2]
  const int h2 = n - 1 - h1;     // k in [n/2+1, n-1]
  for (int idx = threadIdx.x; idx < count * h1; idx += blockDim.x) {
    const int b = b0 + idx / h1, k = 1 + idx % h1;
    const cx<T> v = lds[eng.in_at(b, k)];
    if (nonzero(v)) lds[eng.in_at(b, n - k)] = conj(v);
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < count * h2; idx += blockDim.x) {
    const int b = b0 + idx / h2, k = h1 + 1 + idx % h2;
    const cx<T> v = lds[eng.in_at(b, k)];
    if (nonzero(v)) lds[eng.in_at(b, n - k)] = conj(v);
  }
  __syncthreads();
}

template <typename T>
__device__ __forceinline__ void zero_lds(cx<T>* lds, int count) {
  for (int i = threadIdx.x; i < count; i += blockDim.x) lds[i] = czero<T>();
}

// A workgroup-uniform value materialised in a scalar register at this point:
// the compiler may not sink its (scalar) load into later branches.
__device__ __forceinline__ int pin_uniform(int v) {
  v = __builtin_amdgcn_readfirstlane(v);
  asm volatile("" : "+s"(v));
  return v;
}

__device__ __forceinline__ long long pin_uniform64(long long v) {
  int lo = pin_uniform(static_cast<int>(v)), hi = pin_uniform(static_cast<int>(v >> 32));
  return (static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo);
}

// Exchange-side element of (stick s, plane pos): the plain stick array of a
// single rank, else the plane's segment (one 16-byte table entry per plane:
// no dependent loads). The arguments are pinned in scalar registers once per
// kernel (read through ZArgs per element, their scalar loads were sunk into
// every element's branch and waited out there).
struct SegMap {
  int single;
  long long stride;
  const long long* tab;
  __device__ explicit SegMap(const ZArgs& a)
      : single(pin_uniform(a.single)), stride(pin_uniform64(a.stickStride)), tab(a.zTab) {}
  __device__ long long at(int s, int pos) const {
    if (single == 1) return static_cast<long long>(s) * stride + pos;
    using V = long long __attribute__((ext_vector_type(2)));
    const V t = *reinterpret_cast<const V*>(tab + 2 * pos);
    return t.x + static_cast<long long>(s) * t.y;
  }
};

__device__ __forceinline__ long long seg_index(const ZArgs& a, int s, int pos) {
  return SegMap(a).at(s, pos);
}

#define SPFFT_LDS_DECL(T)                                         \
  extern __shared__ __attribute__((aligned(16))) char spfftSmem[]; \
  cx<T>* lds = reinterpret_cast<cx<T>*>(spfftSmem)

// Row side of a line-fast kernel: lanes walk along rows (row-contiguous global
// loads) into the FFT lines in LDS; line-fast lanes would touch B rows with
// (64/B)-element segments per wave instruction (32 B segments for fp32 B=16).
// Row b of the tile starts at base + b * stride: complex elements, or real ones
// (E == T) loaded with a zero imaginary part.
template <typename E>
struct RowSrc {
  const E* base;
  long long stride;
};
template <typename T, typename E>
__device__ __forceinline__ cx<T> row_elem(const E* p) {
  if constexpr (std::is_same<E, T>::value)
    return mk<T>(ld_stream_real(p), T(0));
  else
    return ld_stream(p);
}
template <class Eng, typename T, typename E>
__device__ __forceinline__ void stage_rows(const Eng& eng, cx<T>* lds, int rows, int len, RowSrc<E> src) {
  if constexpr (!Eng::kBatchedCopy) {
    // full tile of a compile-time engine: the trip count, and each unrolled
    // load's row and position offsets, are compile-time (the row products are
    // scalar), so the generic loop's per-element guards, divisions and 64-bit
    // row multiplies go (fp32 y forward: 3 quarter-rate multiplies per load)
    using F = typename Eng::F;
    constexpr int N = Eng::kN, NT = F::NT, B = F::B;
    constexpr int kIters = B * N / NT;
    // (not the wide 512-thread engines: their kernels sit at the 128-VGPR
    // occupancy step, fp32 512 y forward 127 -> 131 VGPRs and 241 -> 316 us with it)
    if constexpr ((B * N) % NT == 0 && (NT % N == 0 || N % NT == 0) && kIters <= 32 &&
                  NT <= kMaxThreads) {
      if (rows == B) {
        const int tid = static_cast<int>(threadIdx.x);
        cx<T> v[kIters];
        if constexpr (NT % N == 0) {
          constexpr int RP = NT / N;  // rows per pass of the workgroup
          const int b0 = tid / N, p = tid % N;
          const E* p0 = src.base + static_cast<long long>(b0) * src.stride + p;
#pragma unroll
          for (int i = 0; i < kIters; ++i) v[i] = row_elem<T>(p0 + (i * RP) * src.stride);
#pragma unroll
          for (int i = 0; i < kIters; ++i) lds[eng.in_at(b0 + i * RP, p)] = v[i];
        } else {
          constexpr int C = N / NT;  // passes per row
          const E* p0 = src.base + tid;
#pragma unroll
          for (int i = 0; i < kIters; ++i) v[i] = row_elem<T>(p0 + (i / C) * src.stride + (i % C) * NT);
#pragma unroll
          for (int i = 0; i < kIters; ++i) lds[eng.in_at(i / C, tid + (i % C) * NT)] = v[i];
        }
        __syncthreads();
        return;
      }
    }
  }
  gather_to_lds(lds, rows * len, [&](int idx) {
    const int b = idx / len;
    if (b >= rows) return czero<T>();
    return row_elem<T>(src.base + static_cast<long long>(b) * src.stride + (idx - b * len));
  }, [&](int idx) {
    const int b = idx / len;
    return eng.in_at(b, idx - b * len);
  });
  __syncthreads();
}

// Exclusive prefix sum of n ints in LDS (one wave, 64-wide shuffle scans); writes
// out[0..n] (out[n] = total). Ends with a barrier.
__device__ __forceinline__ void wave_exclusive_scan(const int* in, int* out, int n) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int carry = 0;
    for (int c = 0; c < n; c += 64) {
      const int i = c + lane;
      const int v = i < n ? in[i] : 0;
      int x = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
      }
      if (i < n) out[i] = carry + x - v;
      carry += __shfl(x, 63, 64);
    }
    if (lane == 0) out[n] = carry;
  }
  __syncthreads();
}

// Run table of a block of sticks staged in LDS (after the FFT lines):
// the gather/scatter between sparse values and sticks is then one flat loop
// with all loads independent (value index = first + idx when the block's runs
// are consecutive in value order, the common stick-major input).
struct RunTable {
  StickRun* runs;
  int* start;  // exclusive prefix of run lengths, count+1 entries
  int count;
  int total;
  bool contiguous;
};

constexpr int kRunsPerLine = 4;  // table capacity per stick line

__host__ __device__ constexpr std::size_t run_table_bytes(int lines) {
  return std::size_t(kRunsPerLine) * lines * (sizeof(StickRun) + sizeof(int)) + 16 >
                 std::size_t(lines) * sizeof(StickDesc)
             ? std::size_t(kRunsPerLine) * lines * (sizeof(StickRun) + sizeof(int)) + 16
             : std::size_t(lines) * sizeof(StickDesc);
}

// Returns false if the block's runs do not fit the table (caller falls back).
__device__ __forceinline__ bool load_run_table(const ZArgs& a, int s0, int lines, char* base,
                                               RunTable& t) {
  const int s1 = min(s0 + lines, a.numSticks);
  const int q0 = a.runOffsets[s0];
  const int q1 = a.runOffsets[s1];
  const int R = q1 - q0;
  if (R > kRunsPerLine * lines) return false;  // block-uniform
  t.runs = reinterpret_cast<StickRun*>(base);
  int* lens = reinterpret_cast<int*>(base + sizeof(StickRun) * kRunsPerLine * lines);
  t.start = lens;  // scanned in place into a shifted copy below
  int ok = 1;
  for (int i = threadIdx.x; i < R; i += blockDim.x) {
    const StickRun r = a.runs[q0 + i];
    t.runs[i] = r;
    if (i > 0) {
      const StickRun p = a.runs[q0 + i - 1];
      if (p.valueStart + p.length != r.valueStart) ok = 0;
    }
  }
  t.contiguous = __syncthreads_and(ok) != 0;
  // prefix of lengths (wave 0), lengths read from the staged runs
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int carry = 0;
    for (int c = 0; c < R; c += 64) {
      const int i = c + lane;
      const int v = i < R ? t.runs[i].length : 0;
      int x = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
      }
      if (i < R) lens[i] = carry + x - v;
      carry += __shfl(x, 63, 64);
    }
    if (lane == 0) lens[R] = carry;
  }
  __syncthreads();
  t.count = R;
  t.total = lens[R];
  return true;
}

// index of the run containing flat element idx (binary search over start[])
__device__ __forceinline__ int find_run(const RunTable& t, int idx) {
  int lo = 0, hi = t.count - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t.start[mid] <= idx)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

// Exchange-side addressing of the z stage kernels. A single rank's stick array
// is pure arithmetic (stride pinned in scalar registers). Distributed plans
// stage their per-plane segment table, (base, stride) per plane z (ZArgs::zTab),
// in LDS once per workgroup: read from global memory per element, a table
// entry's wait (s_waitcnt vmcnt) also waited out every data load the lane had
// issued before it, while LDS reads count separately (lgkmcnt). Only
// distributed launches reserve the table's LDS: at 256^3 fp64 its 4 KB cost
// the z forward kernel a third of its workgroups per CU (66 -> 73 us), as did
// computing a single rank's table in LDS. (A kernel template per plan kind
// doubled the z kernels and tripled their compile time.)
// Distributed launches whose engine leaves no room for the table (long z lines
// near the LDS limit) read it from global memory instead (ZArgs::single = 2,
// set by the launcher: z_args_for_lds).
struct ZSeg {
  int single;
  long long stride;
  const long long* tab;   // LDS (distributed plans)
  const long long* gtab;  // global memory (single == 2)
  __device__ ZSeg(const ZArgs& a, char* ldsTab, int n)
      : single(pin_uniform(a.single)), stride(pin_uniform64(a.stickStride)),
        tab(reinterpret_cast<const long long*>(ldsTab)), gtab(a.zTab) {
    if (single == 0) {
      long long* t = reinterpret_cast<long long*>(ldsTab);
      for (int i = threadIdx.x; i < 2 * n; i += blockDim.x) t[i] = a.zTab[i];
      __syncthreads();
    }
  }
  __device__ long long at(int s, int pos) const {
    using V = long long __attribute__((ext_vector_type(2)));
    if (single == 1) return static_cast<long long>(s) * stride + pos;
    if (single == 2) {
      const V t = *reinterpret_cast<const V*>(gtab + 2 * pos);
      return t.x + static_cast<long long>(s) * t.y;
    }
    const V t = *reinterpret_cast<const V*>(tab + 2 * pos);
    return t.x + static_cast<long long>(s) * t.y;
  }
};
// LDS offset of ZSeg's table behind the FFT lines and the desc / run table
__host__ __device__ constexpr std::size_t zseg_lds_offset(std::size_t fftBytes, int lines) {
  return (fftBytes + run_table_bytes(lines) + 15) / 16 * 16;
}
inline std::size_t zseg_lds_bytes(const ZArgs& a) {
  return a.single ? 0 : std::size_t(2) * a.n * sizeof(long long) + 16;
}
// The launch's arguments and LDS bytes: a distributed plan's segment table
// moves to global memory when it would push the workgroup past the LDS limit.
inline ZArgs z_args_for_lds(const ZArgs& a, std::size_t fftBytes, int lines, std::size_t* ldsTotal) {
  ZArgs b = a;
  constexpr std::size_t kLimit = 160 * 1024;
  if (!b.single && zseg_lds_offset(fftBytes, lines) + zseg_lds_bytes(b) > kLimit) b.single = 2;
  *ldsTotal = zseg_lds_offset(fftBytes, lines) + zseg_lds_bytes(b);
  return b;
}

// Workgroup -> tile mapping: the dispatcher deals consecutive workgroups
// round-robin to the 8 XCDs. An XCD-contiguous remap was measured slower on
// MI355X at 256^3 (x/y stages 3-6 us, bench -4.5%, profiles/r2_s1/shape_ab.txt):
// the stages have no cross-workgroup reuse for an XCD's L2, and round-robin
// spreads the addresses in flight over all eight XCDs' paths to HBM.
__device__ __forceinline__ void block_tile(int& bx, int& by) {
  bx = blockIdx.x;
  by = blockIdx.y;
}
__device__ __forceinline__ int block_tile_x() { return blockIdx.x; }

// Batched launch (ZArgs/YArgs/XArgs::batch): the workgroup's transform
// (blockIdx.z) supplies the input and output buffers; the index tables are
// shared by every transform of the batch.
#define SPFFT_BATCH_SELECT(a, IN, OUT)                                   \
  if ((a).batch.count > 1) {                                           \
    IN = static_cast<decltype(IN)>((a).batch.in[blockIdx.z]);          \
    OUT = static_cast<decltype(OUT)>((a).batch.out[blockIdx.z]);       \
  }

// ---------------------------------------------------------------- z stage
template <class Eng, typename T, typename BT>
__global__ void __launch_bounds__(Eng::kBlock)
    z_backward_kernel(Eng eng, ZArgs a, const cx<T>* __restrict__ values, BT* __restrict__ out,
                      const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  SPFFT_BATCH_SELECT(a, values, out);
  const int B = eng.lines();
  const int s0 = a.stickBegin + block_tile_x() * B;
  const ZSeg seg(a, reinterpret_cast<char*>(lds) + zseg_lds_offset(eng.lds_bytes(), B), eng.n());
  zero_lds(lds, eng.input_elems());
  RunTable tab;
  char* tableBase = reinterpret_cast<char*>(lds) + eng.lds_bytes();
  if (load_run_table(a, s0, B, tableBase, tab)) {
    // decompress: flat over the block's values, kGatherUnroll loads in flight per lane
    if (tab.contiguous) {
      const cx<T>* src = values + tab.runs[0].valueStart;
      gather_to_lds(lds, tab.total, [&](int idx) { return src[idx]; }, [&](int idx) {
        const int q = find_run(tab, idx);
        return eng.in_at(tab.runs[q].stick - s0, tab.runs[q].zStart + idx - tab.start[q]);
      });
    } else {
      gather_to_lds(lds, tab.total, [&](int idx) {
        const int q = find_run(tab, idx);
        return ld_values(&values[tab.runs[q].valueStart + idx - tab.start[q]]);
      }, [&](int idx) {
        const int q = find_run(tab, idx);
        return eng.in_at(tab.runs[q].stick - s0, tab.runs[q].zStart + idx - tab.start[q]);
      });
    }
  } else {
    // many short runs (unsorted input): one wave per stick
    __syncthreads();  // zero-fill complete
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    for (int b = wave; b < B; b += nw) {
      const int s = s0 + b;
      if (s >= a.numSticks) break;
      const int q1 = a.runOffsets[s + 1];
      for (int q = a.runOffsets[s]; q < q1; ++q) {
        const StickRun r = a.runs[q];
        for (int j = lane; j < r.length; j += 64)
          lds[eng.in_at(b, r.zStart + j)] = ld_values(&values[r.valueStart + j]);
      }
    }
  }
  __syncthreads();
  if (a.zeroStick >= s0 && a.zeroStick < s0 + B) hermitian_lines(eng, lds, a.zeroStick - s0, 1, a.n);
  eng.lds_to_global(lds, tw, [&](int b, int pos, cx<T> v) {
    const int s = s0 + b;
    if (s < a.numSticks) st_stream(&out[seg.at(s, pos)], cvt<typename BT::value_type>(v));
  });
}

template <class Eng, typename T, typename BT>
__global__ void __launch_bounds__(Eng::kBlock)
    z_forward_kernel(Eng eng, ZArgs a, const BT* __restrict__ in, cx<T>* __restrict__ values,
                     T scale, const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  SPFFT_BATCH_SELECT(a, in, values);
  const int B = eng.lines();
  const int s0 = a.stickBegin + block_tile_x() * B;
  const ZSeg seg(a, reinterpret_cast<char*>(lds) + zseg_lds_offset(eng.lds_bytes(), B), eng.n());
  eng.global_to_lds(lds, tw, [&](int b, int pos) -> cx<T> {
    const int s = s0 + b;
    if (s >= a.numSticks) return czero<T>();
    return cvt<T>(ld_stream(&in[seg.at(s, pos)]));
  });
  // compress (+ scaling)
  RunTable tab;
  char* tableBase = reinterpret_cast<char*>(lds) + eng.lds_bytes();
  if (load_run_table(a, s0, B, tableBase, tab)) {
    for (int idx = threadIdx.x; idx < tab.total; idx += blockDim.x) {
      const int q = find_run(tab, idx);
      const StickRun& r = tab.runs[q];
      const int off = idx - tab.start[q];
      st_values(&values[r.valueStart + off], spfft::scale(lds[eng.out_at(r.stick - s0, r.zStart + off)], scale));
    }
  } else {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    for (int b = wave; b < B; b += nw) {
      const int s = s0 + b;
      if (s >= a.numSticks) break;
      const int q1 = a.runOffsets[s + 1];
      for (int q = a.runOffsets[s]; q < q1; ++q) {
        const StickRun r = a.runs[q];
        for (int j = lane; j < r.length; j += 64)
          st_values(&values[r.valueStart + j], spfft::scale(lds[eng.out_at(b, r.zStart + j)], scale));
      }
    }
  }
}

// z stage for "simple" sticks (values of a stick contiguous, <= 2 z-runs; the
// common stick-major input): every lane maps its FFT positions z straight to
// value offsets, so values are loaded into registers and written back with
// coalesced accesses and no LDS staging or zero-fill.
__device__ __forceinline__ int desc_offset(const StickDesc& q, int z) {
  int j = z - q.z0;
  if (j >= 0 && j < q.len0) return j;
  j = z - q.z1;
  if (j >= 0 && j < q.count - q.len0) return q.len0 + j;
  return -1;
}

template <class Eng, typename T, typename BT, bool Plain>
__global__ void __launch_bounds__(Eng::kBlock)
    z_backward_desc_kernel(Eng eng, ZArgs a, const cx<T>* __restrict__ values,
                           BT* __restrict__ out, const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  SPFFT_BATCH_SELECT(a, values, out);
  const int B = eng.lines();
  const int n = eng.n();
  const int s0 = a.stickBegin + block_tile_x() * B;
  const int nl = min(B, a.numSticks - s0);
  const ZSeg seg(a, reinterpret_cast<char*>(lds) + zseg_lds_offset(eng.lds_bytes(), B), eng.n());
  auto store = [&](int b, int pos, cx<T> v) {
    if (b < nl) st_stick<Plain>(&out[seg.at(s0 + b, pos)], cvt<typename BT::value_type>(v));
  };
  StickDesc* d = reinterpret_cast<StickDesc*>(reinterpret_cast<char*>(lds) + eng.lds_bytes());
  for (int b = threadIdx.x; b < nl; b += blockDim.x) d[b] = a.desc[s0 + b];
  __syncthreads();
  auto load = [&](int b, int z) -> cx<T> {
    if (b >= nl) return czero<T>();
    const StickDesc& q = d[b];
    const int j = desc_offset(q, z);
    return j < 0 ? czero<T>() : ld_values(&values[q.valueStart + j]);
  };
  if constexpr (Eng::kBatchedCopy) {
    // run-time engines: one staged path for every block (a single inlined copy
    // of the pass switch keeps the kernel's register demand down)
    eng.stage(lds, load);
    __syncthreads();
    if (a.zeroStick >= s0 && a.zeroStick < s0 + nl) hermitian_lines(eng, lds, a.zeroStick - s0, 1, n);
    eng.lds_to_global(lds, tw, store);
  } else if (a.zeroStick >= s0 && a.zeroStick < s0 + nl) {
    // block holding the (0,0) stick of an R2C transform: stage for the hermitian fill
    for (int idx = threadIdx.x; idx < B * n; idx += blockDim.x) {
      const int b = idx / n, z = idx - b * n;
      lds[eng.in_at(b, z)] = load(b, z);
    }
    __syncthreads();
    hermitian_lines(eng, lds, a.zeroStick - s0, 1, n);
    eng.lds_to_global(lds, tw, store);
  } else {
    // compile-time engines load only the lane's own line (b == lane_line(),
    // the FftCT/FftMR contract): its descriptor is read from LDS once into
    // registers and the value offset is a branch-free select. Reading d[b] in
    // the load lambda re-read the descriptor from LDS for every element, each
    // read waited out before the dependent value load could issue.
    const int lb = Eng::F::lane_line();
    StickDesc q = d[lb < nl ? lb : 0];
    int z0 = q.z0, len0 = q.len0, z1 = q.z1, len1 = q.count - q.len0, vs = q.valueStart;
    if (lb >= nl) len0 = len1 = 0;
    asm volatile("" : "+v"(z0), "+v"(len0), "+v"(z1), "+v"(len1), "+v"(vs));
    const cx<T>* vals = values + vs;
    eng.global_to_global(lds, tw, [&](int, int z) -> cx<T> {
      const unsigned j0 = static_cast<unsigned>(z - z0), j1 = static_cast<unsigned>(z - z1);
      const bool in0 = j0 < static_cast<unsigned>(len0);
      const bool in1 = j1 < static_cast<unsigned>(len1);
      const int j = in0 ? static_cast<int>(j0) : len0 + static_cast<int>(j1);
      // streamed value loads: 256^3 fp64 79.2 -> 63.4 us, 512^3 R2C fp32 219 ->
      // 133 us, fp32 256^3 neutral (T = 1, same box; profiles/r6/ntmerge)
      return (in0 || in1) ? ld_stream(&vals[j]) : czero<T>();
    }, store);
  }
}

template <class Eng, typename T, typename BT, bool NtValues>
__global__ void __launch_bounds__(Eng::kBlock)
    z_forward_desc_kernel(Eng eng, ZArgs a, const BT* __restrict__ in, cx<T>* __restrict__ values,
                          T scale, const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  SPFFT_BATCH_SELECT(a, in, values);
  const int B = eng.lines();
  const int s0 = a.stickBegin + block_tile_x() * B;
  const int nl = min(B, a.numSticks - s0);
  const ZSeg seg(a, reinterpret_cast<char*>(lds) + zseg_lds_offset(eng.lds_bytes(), B), eng.n());
  if constexpr (!Eng::kBatchedCopy) {
    // compile-time engines: the lane's own stick descriptor in registers, no
    // LDS round trip (69.6 -> 65.0 us at 256^3, profiles/r1_s14/zdesc_ab/
    // summary.txt; the same change in the backward kernel, whose value loads
    // are on the critical path, measured 81 -> 104 us). This relies on the
    // compile-time engines' run() storing only the lane's own line
    // (b == lane_line()); the assert guards that contract in debug builds.
    const int lb = Eng::F::lane_line();
    StickDesc q{};
    if (lb < nl) q = a.desc[s0 + lb];
    const int z0 = q.z0, len0 = lb < nl ? q.len0 : 0, z1 = q.z1, len1 = lb < nl ? q.count - q.len0 : 0;
    cx<T>* vals = values + q.valueStart;
    auto store = [&](int b, int pos, cx<T> v) {
      assert(b == lb);
      // branch-free value offset (as in the backward kernel); one predicated store
      const unsigned j0 = static_cast<unsigned>(pos - z0), j1 = static_cast<unsigned>(pos - z1);
      const bool in0 = j0 < static_cast<unsigned>(len0);
      const bool in1 = j1 < static_cast<unsigned>(len1);
      const int j = in0 ? static_cast<int>(j0) : len0 + static_cast<int>(j1);
      if (in0 || in1) {
        if constexpr (NtValues) st_stream(&vals[j], spfft::scale(v, scale));
        else st_values(&vals[j], spfft::scale(v, scale));
      }
    };
    // Lanes past the last stick load a valid stick (min(lb, nl - 1)) and store
    // nothing (len0 = len1 = 0): no guard per element. Loads only the lane's own
    // line (b == lb, the FftCT/FftMR contract).
    const int ls = s0 + min(lb, nl - 1);
    if (seg.single == 1) {
      // plain stick rows (one rank): the row is the lane's base pointer, each
      // element a constant offset from it; no segment-mode branch and no 64-bit
      // multiply per element (the other modes below read a table per position)
      const BT* row = in + static_cast<long long>(ls) * seg.stride + Eng::F::lane_pos();
      eng.global_to_global(lds, tw, [&](int, int, int off) -> cx<T> { return cvt<T>(ld_stream(&row[off])); },
                           store);
    } else {
      eng.global_to_global(lds, tw, [&](int, int pos) -> cx<T> {
        return cvt<T>(ld_stream(&in[seg.at(ls, pos)]));
      }, store);
    }
  } else {
    StickDesc* d = reinterpret_cast<StickDesc*>(reinterpret_cast<char*>(lds) + eng.lds_bytes());
    for (int b = threadIdx.x; b < nl; b += blockDim.x) d[b] = a.desc[s0 + b];
    __syncthreads();
    eng.global_to_global(lds, tw, [&](int b, int pos) -> cx<T> {
      if (b >= nl) return czero<T>();
      return cvt<T>(ld_stream(&in[seg.at(s0 + b, pos)]));
    }, [&](int b, int pos, cx<T> v) {
      if (b >= nl) return;
      const StickDesc& q = d[b];
      const int j = desc_offset(q, pos);
      if (j >= 0) {
        if constexpr (NtValues) st_stream(&values[q.valueStart + j], spfft::scale(v, scale));
        else st_values(&values[q.valueStart + j], spfft::scale(v, scale));
      }
    });
  }
}

// y-stage tile order: plane blocks fastest in the grid, so the workgroups in
// flight cover a few whole columns: each stick is read (or written) entirely
// while it is open in the DRAM row buffers, and the [z][column][y] rows of a
// plane are written as one contiguous run.
__device__ __forceinline__ int y_tile_col() {
  int bx, by;
  block_tile(bx, by);
  return by;
}
__device__ __forceinline__ int y_tile_zblock() {
  int bx, by;
  block_tile(bx, by);
  return bx;
}
inline dim3 y_grid(int cols, int zblocks, unsigned batch = 1) { return dim3(zblocks, cols, batch); }

// ---------------------------------------------------------------- y stage
// Whether the column with run descriptor d has a stick entry at y, and its base
// (uniform loop bound nRuns: a sphere column tests its 2 runs only).
__device__ __forceinline__ bool col_desc_find(const ColDesc& d, long long stride, int y,
                                              long long& base) {
  long long b0 = 0;
  bool hit = false;
#pragma unroll
  for (int r = 0; r < kColRuns; ++r) {
    if (r < d.nRuns) {
      const bool in = static_cast<unsigned>(y - d.y[r]) < static_cast<unsigned>(d.len[r]);
      b0 = in ? d.b0[r] : b0;
      hit = hit || in;
    }
  }
  base = b0 + static_cast<long long>(static_cast<unsigned>(y) * static_cast<unsigned>(stride));
  return hit;
}

// Stick entries of the workgroup's column: through the column's run descriptor
// (workgroup-uniform, scalar registers, no prologue) when the plan has one, else
// through the entry list staged in LDS (colBase per entry, y -> entry table).
// Every kernel keeps a single FFT call site whichever source is used: the
// run-time engines inline their whole pass switch per call site, and a second
// copy doubled their register demand (profiles/r2_s1/rt_regression.txt).
// engines whose store positions can be enumerated ahead of run() (FftCT)
template <class Eng, class = void>
struct has_store_pos : std::false_type {};
template <class Eng>
struct has_store_pos<Eng, std::void_t<decltype(Eng::F::kStoreSlots)>> : std::true_type {};
// "No stick entry" in the y -> base tables. Bases are element offsets from the
// stage's buffer, and the peer-write plane's are offsets to the peers' buffers,
// which lie below the local one as often as above: -1 would be a valid base.
constexpr long long kNoBase = -(1LL << 62);

template <class Eng>
struct ColEntries {
  bool useDesc;
  ColDesc d;
  long long stride;
  long long* yBase;  // LDS: y -> stick-side base or kNoBase (table mode)
  long long* cBase;  // LDS: colBase per entry (list mode)
  int* yEnt;         // LDS: y -> entry or -1 (list mode)
  int* cY;           // LDS: entry -> y (list mode)
  int ne;
  // table: build only yBase, the y -> base table (the backward y stage's loads
  // then cost one LDS read per element instead of a descriptor search per
  // element and lane); it shares its LDS with the list-mode arrays, which the
  // table mode does not use
  __device__ ColEntries(const Eng& eng, const YArgs& a, void* ldsBase, int c, bool allowDesc,
                        bool table = false) {
    const int n = eng.n();
    useDesc = allowDesc && a.colDesc != nullptr;
    stride = a.colStride;
    char* base = reinterpret_cast<char*>(ldsBase) + eng.lds_bytes();
    yBase = reinterpret_cast<long long*>(base);
    cBase = yBase;
    yEnt = reinterpret_cast<int*>(cBase + n);
    cY = yEnt + n;
    ne = 0;
    if (useDesc) {
      d = a.colDesc[c];
      if (table) {
        for (int y = threadIdx.x; y < n; y += blockDim.x) {
          long long b;
          yBase[y] = col_desc_find(d, stride, y, b) ? b : kNoBase;
        }
        __syncthreads();
      }
      return;
    }
    const int k0 = a.colOffsets[c];
    ne = a.colOffsets[c + 1] - k0;
    if (table) {
      for (int y = threadIdx.x; y < n; y += blockDim.x) yBase[y] = kNoBase;
      __syncthreads();
      for (int e = threadIdx.x; e < ne; e += blockDim.x) yBase[a.colY[k0 + e]] = a.colBase[k0 + e];
      __syncthreads();
      return;
    }
    for (int y = threadIdx.x; y < n; y += blockDim.x) yEnt[y] = -1;
    __syncthreads();
    for (int e = threadIdx.x; e < ne; e += blockDim.x) {
      const int y = a.colY[k0 + e];
      cBase[e] = a.colBase[k0 + e];
      yEnt[y] = e;
      cY[e] = y;
    }
    __syncthreads();
  }
  // whether the column has an entry at y; its base (add the plane) in base
  __device__ bool find(int y, long long& base) const {
    if (useDesc) return col_desc_find(d, stride, y, base);
    const int e = yEnt[y];
    base = e < 0 ? 0 : cBase[e];
    return e >= 0;
  }
};

// LDS the y-stage kernels reserve behind the FFT lines for ColEntries: the list
// mode (colBase, y -> entry, entry -> y) where it can run, and the y -> base
// table (table: the kernel runs table mode; both share one region). With column
// run descriptors only the backward R2C x = 0 column (hermitian fill) runs list
// mode; C2C forward plans reserve nothing, which keeps fp32 N = 256 at 4
// workgroups per CU.
inline std::size_t col_entries_lds(const YArgs& a, bool backward, bool table = false) {
  const bool list = !a.colDesc || (backward && a.colOfX0 >= 0);
  std::size_t bytes = list ? std::size_t(a.n) * (sizeof(long long) + 2 * sizeof(int)) : 0;
  if (table) bytes = std::max(bytes, std::size_t(a.n) * sizeof(long long));
  return bytes ? bytes + 16 : 0;
}

constexpr std::size_t kLdsPerWorkgroup = 160 * 1024;

// Whether a y-stage kernel with engine Eng runs table mode: compile-time
// engines (one LDS read per element replaces their per-element search) whose
// FFT lines leave room for the table next to the list-mode arrays.
template <class Eng, bool Enabled>
constexpr bool y_table() {
  if constexpr (Eng::kBatchedCopy || !Enabled) {
    return false;
  } else {
    constexpr int n = Eng::kN;
    return Eng::F::lds_bytes() + std::size_t(n) * (sizeof(long long) + 2 * sizeof(int)) + 16 <=
           kLdsPerWorkgroup;
  }
}

// Backward y stage with the line-fast engine: lane (line = plane zz, pos = y)
// loads straight from the stick side — consecutive lanes read consecutive z
// of one stick (coalesced) — with no LDS staging of the input. The x = 0
// column of an R2C transform is gathered into LDS for the hermitian fill.
template <class Eng, typename T, typename BT, bool Plain>
__global__ void __launch_bounds__(Eng::kBlock)
    y_backward_kernel(Eng eng, YArgs a, const BT* __restrict__ in, cx<T>* __restrict__ inter,
                      const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  SPFFT_BATCH_SELECT(a, in, inter);
  const int B = eng.lines();
  const int n = eng.n();
  const int c = a.colBegin + y_tile_col();
  const int z0 = a.zBegin + y_tile_zblock() * B;
  const int zl = min(B, a.L - z0);
  const bool x0 = c == a.colOfX0;
  constexpr bool kTable = y_table<Eng, true>();
  const ColEntries<Eng> ce(eng, a, lds, c, !x0, kTable && !x0);
  auto load = [&](int b, int pos) -> cx<T> {
    if constexpr (kTable) {
      const long long base = ce.yBase[pos];
      // masked load: the lanes of a missing stick issue no request at all (a shared
      // zero source instead: fp32 512^3 R2C y backward 228 -> 212 us, 256^3 neutral;
      // profiles/r5/ab/ymask)
      cx<T> v = czero<T>();
      if (base != kNoBase && b < zl) v = cvt<T>(ld_stick<Plain>(in + (base + z0 + b)));
      return v;
    } else {
      long long base;
      if (!ce.find(pos, base) || b >= zl) return czero<T>();
      return cvt<T>(ld_stream(&in[base + z0 + b]));
    }
  };
  // the x = 0 column of an R2C transform: gathered into LDS, hermitian fill
  auto stage_x0 = [&]() {
    zero_lds(lds, eng.input_elems());
    __syncthreads();
    gather_to_lds(lds, ce.ne * zl, [&](int idx) {
      const int e = idx / zl, zz = idx - e * zl;
      return cvt<T>(ld_stream(&in[ce.cBase[e] + z0 + zz]));
    }, [&](int idx) {
      const int e = idx / zl, zz = idx - e * zl;
      return eng.in_at(zz, ce.cY[e]);
    });
    __syncthreads();
    hermitian_lines(eng, lds, 0, B, n);
  };
  if constexpr (Eng::kBatchedCopy) {
    // run-time engines: stage either input path, then one FFT
    if (!x0) {
      eng.stage(lds, load);
      __syncthreads();
    } else {
      stage_x0();
    }
    eng.lds_to_lds(lds, tw);
  } else if (!x0) {
    eng.global_to_lds(lds, tw, load);
  } else {
    stage_x0();
    eng.lds_to_lds(lds, tw);
  }
  // rows of [z][column][y] are contiguous: coalesced copy-out
  copy_out<Eng>(lds, zl * n, [&](int idx) {
    const int b = idx / n;
    return eng.out_at(b, idx - b * n);
  }, [&](int idx, cx<T> v) {
    const int b = idx / n;
    st_inter(&inter[static_cast<long long>(z0 + b) * a.interZStride + inter_row(a, c) + idx - b * n], v);
  });
}

// Forward y stage, line-fast engine: lanes read rows of the intermediate and
// write each stick's z-run of this plane block directly (consecutive lanes ->
// consecutive z of one stick); no LDS staging on either side.
template <class Eng, typename T, typename BT>
__global__ void __launch_bounds__(Eng::kBlock)
    y_forward_kernel(Eng eng, YArgs a, const cx<T>* __restrict__ inter, BT* __restrict__ out,
                     const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  SPFFT_BATCH_SELECT(a, inter, out);
  const int B = eng.lines();
  const int n = eng.n();
  const int c = a.colBegin + y_tile_col();
  const int z0 = a.zBegin + y_tile_zblock() * B;
  const int zl = min(B, a.L - z0);
  constexpr bool kTable = y_table<Eng, has_store_pos<Eng>::value>();
  const ColEntries<Eng> ce(eng, a, lds, c, true, kTable);
  const RowSrc<cx<T>> rows{inter + static_cast<long long>(z0) * a.interZStride + inter_row(a, c),
                           a.interZStride};
  if constexpr (kTable) {
    // compile-time engines: the stick bases of the lane's output positions are
    // read from the y -> base table before the FFT (their LDS latency overlaps
    // the row loads); the stores then need no descriptor search per element
    using F = typename Eng::F;
    long long bases[F::kStoreSlots];
    F::for_each_store_pos([&](int i, int pos) { bases[i] = ce.yBase[pos]; });
    int slot = 0;
    stage_rows(eng, lds, zl, n, rows);
    eng.lds_to_global(lds, tw, [&](int b, int, cx<T> v) {
      const long long base = bases[slot++];
      if (base != kNoBase && b < zl) st_stream(&out[base + z0 + b], cvt<typename BT::value_type>(v));
    });
    return;
  }
  auto store = [&](int b, int pos, cx<T> v) {
    long long base;
    if (ce.find(pos, base) && b < zl) st_stream(&out[base + z0 + b], cvt<typename BT::value_type>(v));
  };
  stage_rows(eng, lds, zl, n, rows);
  eng.lds_to_global(lds, tw, store);
}

// x stage column lookup: every x of [0, nFreq) holds a column (e.g. a sphere
// of radius N/2) -> colX is the identity and no table is built; otherwise the
// workgroup stages the x -> column table in LDS. The table build is a
// dependent global load plus two barriers in front of every workgroup's main
// loads, so the dense case skips it.
__device__ __forceinline__ bool x_dense(const XArgs& a) { return a.ncols == a.nFreq; }
__device__ __forceinline__ void build_xcol(const XArgs& a, int* xCol, int count) {
  if (x_dense(a)) return;
  for (int x = threadIdx.x; x < count; x += blockDim.x) xCol[x] = -1;
  __syncthreads();
  for (int c = threadIdx.x; c < a.ncols; c += blockDim.x) xCol[a.colX[c]] = c;
  __syncthreads();
}
__device__ __forceinline__ int xcol_of(const XArgs& a, const int* xCol, int x) {
  return x_dense(a) ? (x < a.nFreq ? x : -1) : xCol[x];
}

// Packed-real C2R with the pre-pass folded into the first FFT pass's loads
// (compile-time engines): 66.9 -> 54.8 us at 256^3 fp64, R2C bench +2% fp64,
// +3% fp32 (profiles/r2_s1/shape_ab.txt); the run-time engines stage the
// pre-pass in LDS.

// ---------------------------------------------------------------- x stage
// Backward x stage with the line-fast engine: lane (line = row y, pos = x)
// reads column x of the intermediate (consecutive lanes -> consecutive y),
// zero for x without sticks; C2R completes the row by hermitian symmetry on
// the fly. The result is written row-contiguous from LDS.
template <class Eng, typename T, bool R2C>
__global__ void __launch_bounds__(Eng::kBlock)
    x_backward_kernel(Eng eng, XArgs a, const cx<T>* __restrict__ inter, void* __restrict__ space,
                      const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  SPFFT_BATCH_SELECT(a, inter, space);
  const int B = eng.lines();
  const int n = eng.n();
  int tx, ty;
  block_tile(tx, ty);
  const int zl = a.zBegin + ty;
  const int y0 = tx * B;
  int* xCol = reinterpret_cast<int*>(reinterpret_cast<char*>(lds) + eng.lds_bytes());
  build_xcol(a, xCol, n);
  const cx<T>* src = inter + static_cast<long long>(zl) * a.interZStride + y0;
  const int yl = min(B, a.Y - y0);
  // kernel arguments the per-element loads use, pinned in scalar registers up
  // front (left to the compiler, their scalar loads were sunk into every
  // element's branch, each waited out before that element's load could issue)
  const int rowStride = pin_uniform(static_cast<int>(a.interStride)), nFreq = pin_uniform(a.nFreq);
  const int dense = pin_uniform(x_dense(a) ? 1 : 0);
  auto col_of = [&](int x) { return dense ? (x < nFreq ? x : -1) : xCol[x]; };
  auto load = [&](int b, int pos) -> cx<T> {
    if (b >= yl) return czero<T>();
    if (R2C && pos >= nFreq) {
      const int c = col_of(n - pos);
      return c < 0 ? czero<T>() : conj(ld_inter(&src[c * rowStride + b]));
    }
    const int c = col_of(pos);
    return c < 0 ? czero<T>() : ld_inter(&src[c * rowStride + b]);
  };
  const long long row0 = (static_cast<long long>(zl) * a.Y + y0) * n;
  eng.global_to_lds(lds, tw, load);
  copy_out<Eng>(lds, yl * n, [&](int idx) {
    const int b = idx / n;
    return eng.out_at(b, idx - b * n);
  }, [&](int idx, cx<T> v) {
    if (R2C)
      st_stream_real(&static_cast<T*>(space)[row0 + idx], v.x);
    else
      st_stream(&static_cast<cx<T>*>(space)[row0 + idx], v);
  });
}

// Forward x stage, line-fast engine: lanes read row segments of the space
// domain and write the columns that hold sticks straight into [z][column][y]
// (consecutive lanes -> consecutive y); R2C reads real rows.
template <class Eng, typename T, bool R2C>
__global__ void __launch_bounds__(Eng::kBlock)
    x_forward_kernel(Eng eng, XArgs a, const void* __restrict__ space, cx<T>* __restrict__ inter,
                     const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  SPFFT_BATCH_SELECT(a, space, inter);
  const int B = eng.lines();
  const int n = eng.n();
  int tx, ty;
  block_tile(tx, ty);
  const int zl = a.zBegin + ty;
  const int y0 = tx * B;
  int* xCol = reinterpret_cast<int*>(reinterpret_cast<char*>(lds) + eng.lds_bytes());
  build_xcol(a, xCol, n);
  const int yl = min(B, a.Y - y0);
  cx<T>* dst = inter + static_cast<long long>(zl) * a.interZStride + y0;
  const long long row0 = (static_cast<long long>(zl) * a.Y + y0) * n;
  // arguments of the per-element stores pinned in scalar registers (see x_backward_kernel)
  const int rowStride = pin_uniform(static_cast<int>(a.interStride)), nFreq = pin_uniform(a.nFreq);
  const int dense = pin_uniform(x_dense(a) ? 1 : 0);
  auto store = [&](int b, int pos, cx<T> v) {
    const int c = dense ? (pos < nFreq ? pos : -1) : xCol[pos];
    if (c >= 0 && b < yl) st_inter(&dst[c * rowStride + b], v);
  };
  if constexpr (R2C)
    stage_rows(eng, lds, yl, n, RowSrc<T>{static_cast<const T*>(space) + row0, n});
  else
    stage_rows(eng, lds, yl, n, RowSrc<cx<T>>{static_cast<const cx<T>*>(space) + row0, n});
  eng.lds_to_global(lds, tw, store);
}

// Packed-real x stage (R2C transforms with even dimX): a real row of length n
// is the complex sequence y[m] = x[2m] + i x[2m+1] of length h = n/2, so one
// half-length FFT plus a twiddle pre-pass (C2R) or post-pass (R2C) replaces the
// hermitian-extended length-n complex FFT: half the butterflies, half the LDS
// traffic, and the real row is read/written as h contiguous complex values.
//   C2R: Z[k] = (X[k] + conj X[h-k]) + i (X[k] - conj X[h-k]) w^k,  y = IDFT_h(Z)
//   R2C: Y = DFT_h(y),  X[k] = (Y[k] + conj Y[h-k])/2 + w^k (Y[k] - conj Y[h-k])/(2i)
// with w = exp(S 2 pi i / n); the imaginary parts of X[0] and X[h] are ignored
// (they cannot contribute to a real signal), as in the complex C2R path.
// first-pass radix of a compile-time engine (0: mixed-radix engines)
template <class F, class = void>
struct FirstRadix {
  static constexpr int value = 0;
};
template <class F>
struct FirstRadix<F, std::void_t<typename F::Sh>> {
  static constexpr int value = F::Sh::R0;
};

template <class Eng, typename T>
__global__ void __launch_bounds__(Eng::kBlock)
    x_backward_c2r_kernel(Eng eng, XArgs a, const cx<T>* __restrict__ inter, T* __restrict__ space,
                          const cx<T>* __restrict__ twh, const cx<T>* __restrict__ twn) {
  SPFFT_LDS_DECL(T);
  SPFFT_BATCH_SELECT(a, inter, space);
  const int B = eng.lines();
  const int h = eng.n();
  const long long n = 2 * static_cast<long long>(h);
  int tx, ty;
  block_tile(tx, ty);
  const int zl = a.zBegin + ty;
  const int y0 = tx * B;
  // LDS: FFT lines | X[h] (Nyquist) per line | xCol table
  cx<T>* nyq = reinterpret_cast<cx<T>*>(reinterpret_cast<char*>(lds) + eng.lds_bytes());
  int* xCol = reinterpret_cast<int*>(nyq + B);
  build_xcol(a, xCol, h + 1);
  const cx<T>* src = inter + static_cast<long long>(zl) * a.interZStride + y0;
  const int yl = min(B, a.Y - y0);
  if constexpr (!Eng::kBatchedCopy) {
    // pre-pass folded into the FFT's first-pass loads: the lane that needs Z[k]
    // loads X[k] and X[h-k] itself (the mirror column is the same workgroup's
    // data, so its second read is served by the caches; plain loads keep it there:
    // streamed loads measured 197.7 -> 239.1 us at 512^3 R2C fp32, profiles/r6/ntmerge/c2r_ab.txt)
    // arguments of the per-element loads pinned in scalar registers (see x_backward_kernel)
    const int rowStride = pin_uniform(static_cast<int>(a.interStride)), nFreq = pin_uniform(a.nFreq);
    const int dense = pin_uniform(x_dense(a) ? 1 : 0);
    auto col = [&](int k, int b) -> cx<T> {
      const int c = dense ? (k < nFreq ? k : -1) : xCol[k];
      return (c < 0 || b >= yl) ? czero<T>() : src[c * rowStride + b];
    };
    // twiddle w^k of position k = t + off, off = kk*TP + r*(h/R0): the table
    // entry of t + kk*TP times the compile-time root exp(-i pi r / R0), so a
    // lane loads one entry per kk instead of one per element: 131 -> 115 VGPRs
    // (fp32 h = 256), x backward at 512^3 R2C fp32 259.2 -> 217.9 us, 256^3 R2C
    // fp64 55.5 -> 54.5 us (profiles/r5/ab/c2r_twiddles)
    constexpr int R0 = FirstRadix<typename Eng::F>::value, Q = R0 ? Eng::kN / R0 : 1;
    eng.global_to_lds(lds, twh, [&](int b, int k, int off) -> cx<T> {
      cx<T> xk = col(k, b);
      cx<T> xm = col(h - k, b);
      if (k == 0) {
        xk.y = T(0);
        xm.y = T(0);
      }
      const cx<T> xmc = conj(xm);
      const int r = off / Q;
      cx<T> w = twn[k - r * Q];
      if constexpr (R0 == 16) {
        if (r) w = cmul(w, mk<T>(T(fftc::C32[r & 15]), T(-fftc::S32[r & 15])));
      } else if constexpr (R0 == 8) {
        if (r) w = cmul(w, mk<T>(T(fftc::C16[r & 15]), T(-fftc::S16[r & 15])));
      } else {
        w = twn[k];
      }
      return (xk + xmc) + rot<+1>(twm<+1>(xk - xmc, w));
    });
    cx<T>* out = reinterpret_cast<cx<T>*>(space + (static_cast<long long>(zl) * a.Y + y0) * n);
    copy_out<Eng>(lds, yl * h, [&](int idx) {
      const int b = idx / h;
      return eng.out_at(b, idx - b * h);
    }, [&](int idx, cx<T> v) { st_stream(&out[idx], v); });
    return;
  }
  // columns X[0..h] of the block's rows, each element loaded once (lanes run
  // over rows: contiguous column segments)
  gather_to_lds(lds, h * B, [&](int idx) -> cx<T> {
    const int k = idx / B, b = idx - k * B;
    const int c = xcol_of(a, xCol, k);
    return (c < 0 || b >= yl) ? czero<T>() : ld_inter(&src[inter_row(a, c) + b]);
  }, [&](int idx) {
    const int k = idx / B;
    return eng.in_at(idx - k * B, k);
  });
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const int c = xcol_of(a, xCol, h);
    nyq[b] = (c < 0 || b >= yl) ? czero<T>() : ld_inter(&src[inter_row(a, c) + b]);
  }
  __syncthreads();
  // pre-pass in place, pairs (k, h-k): Z[k] = (X[k] + conj X[h-k]) + i (X[k] - conj X[h-k]) w^k
  for (int idx = threadIdx.x; idx < B * (h / 2 + 1); idx += blockDim.x) {
    const int k = idx / B, b = idx - k * B;
    const int m = h - k;
    cx<T> xk = lds[eng.in_at(b, k)];
    cx<T> xm = m == h ? nyq[b] : lds[eng.in_at(b, m)];
    if (k == 0) {
      xk.y = T(0);
      xm.y = T(0);
    }
    const cx<T> xmc = conj(xm), xkc = conj(xk);
    lds[eng.in_at(b, k)] = (xk + xmc) + rot<+1>(twm<+1>(xk - xmc, twn[k]));
    if (m != k && m < h) lds[eng.in_at(b, m)] = (xm + xkc) + rot<+1>(twm<+1>(xm - xkc, twn[m]));
  }
  __syncthreads();
  eng.lds_to_lds(lds, twh);
  // the yl rows are contiguous in the space domain: one coalesced copy-out
  cx<T>* out = reinterpret_cast<cx<T>*>(space + (static_cast<long long>(zl) * a.Y + y0) * n);
  copy_out<Eng>(lds, yl * h, [&](int idx) {
    const int b = idx / h;
    return eng.out_at(b, idx - b * h);
  }, [&](int idx, cx<T> v) { st_stream(&out[idx], v); });
}

template <class Eng, typename T>
__global__ void __launch_bounds__(Eng::kBlock)
    x_forward_r2c_kernel(Eng eng, XArgs a, const T* __restrict__ space, cx<T>* __restrict__ inter,
                         const cx<T>* __restrict__ twh, const cx<T>* __restrict__ twn) {
  SPFFT_LDS_DECL(T);
  SPFFT_BATCH_SELECT(a, space, inter);
  const int B = eng.lines();
  const int h = eng.n();
  const long long n = 2 * static_cast<long long>(h);
  int tx, ty;
  block_tile(tx, ty);
  const int zl = a.zBegin + ty;
  const int y0 = tx * B;
  int* xCol = reinterpret_cast<int*>(reinterpret_cast<char*>(lds) + eng.lds_bytes());
  build_xcol(a, xCol, h + 1);
  const int yl = min(B, a.Y - y0);
  const cx<T>* row0 = reinterpret_cast<const cx<T>*>(space + (static_cast<long long>(zl) * a.Y + y0) * n);
  auto rowLoad = [&](int b, int m) -> cx<T> {
    return b >= yl ? czero<T>() : ld_stream(row0 + static_cast<long long>(b) * h + m);
  };
  if constexpr (!Eng::kBatchedCopy && !Eng::kLineFast) {
    // row-mapped engine (launch_x_forward): a line's lanes are adjacent, so the
    // first pass loads the real rows straight from global memory
    eng.global_to_lds(lds, twh, rowLoad);
  } else {
    stage_rows(eng, lds, yl, h, RowSrc<cx<T>>{row0, h});
    eng.lds_to_lds(lds, twh);
  }
  cx<T>* dst = inter + static_cast<long long>(zl) * a.interZStride + y0;
  // post pass over the pairs (k, h - k), k <= h/2: both outputs need the same
  // two LDS values, and w^(h-k) = -conj(w^k) (w = exp(-2 pi i / n), n = 2h), so
  // a pair costs two LDS reads and one twiddle load instead of four and two
  // (512^3 R2C fp32 x forward 224-226 -> 214-216 us, 256^3 R2C fp64 55 -> 53 us,
  // profiles/r5/ab/r2cpair). Lanes run over rows first, so the column stores are
  // contiguous.
  for (int idx = threadIdx.x; idx < B * (h / 2 + 1); idx += blockDim.x) {
    const int b = idx % B, k = idx / B, m = h - k;
    if (b >= yl) continue;
    const int ck = xcol_of(a, xCol, k), cm = xcol_of(a, xCol, m);
    if (ck < 0 && cm < 0) continue;
    const cx<T> A = lds[eng.out_at(b, k == h ? 0 : k)];
    const cx<T> Bv = lds[eng.out_at(b, m == h ? 0 : m)];
    const cx<T> wk = twn[k];
    if (ck >= 0) {
      const cx<T> ym = conj(Bv);
      const cx<T> e = scale(A + ym, T(0.5));
      const cx<T> o = scale(rot<-1>(A - ym), T(0.5));
      st_inter(&dst[inter_row(a, ck) + b], e + twm<-1>(o, wk));
    }
    if (cm >= 0 && m != k) {
      const cx<T> ym = conj(A);
      const cx<T> e = scale(Bv + ym, T(0.5));
      const cx<T> o = scale(rot<-1>(Bv - ym), T(0.5));
      st_inter(&dst[inter_row(a, cm) + b], e + twm<-1>(o, mk<T>(-wk.x, wk.y)));
    }
  }
}

// ------------------------------------------------------------ host helpers
RtPlan make_rt_plan(int n, std::size_t elemBytes);

// Bluestein plan and device tables of length n (cached per device), or
// nullptr-tables when n does not use Bluestein.
struct BlueTables {
  RtPlan pm;
  const void* chirp = nullptr;
  const void* filt = nullptr;
  const void* twm = nullptr;
};
bool use_bluestein(int n, std::size_t elemBytes);
// LDS bytes and lines per workgroup of the one-workgroup engine (run-time or
// Bluestein) of a length without a compile-time kernel; throws GPUFFTError when
// a line does not fit
std::size_t in_lds_engine_bytes(int n, std::size_t elemBytes, int& lines);
BlueTables bluestein_tables(int n, bool dbl);

template <class K>
inline void prepare_kernel(K kernel, std::size_t ldsBytes) {
  if (ldsBytes > 64 * 1024) {
    gpu_check(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(ldsBytes)),
              "hipFuncSetAttribute");
  }
}

// Calls f(engine, threads, lines, ldsBytes) with the CT engine of length n if
// there is one, else with the RT engine.
template <typename T, int S, bool LF = false, bool TwPre = true, class F>
inline void with_engine(int n, F&& f) {
  switch (n) {
#define SPFFT_CT_CASE(NN)                                                         \
  case NN: {                                                                      \
    using E = CtEng<T, NN, S, LF, TwPre>;                                                \
    f(E{}, E::h_threads(), E::h_lines(), E::h_lds());                             \
    return;                                                                       \
  }
    SPFFT_CT_CASE(16)
    SPFFT_CT_CASE(32)
    SPFFT_CT_CASE(64)
    SPFFT_CT_CASE(128)
    SPFFT_CT_CASE(256)
    SPFFT_CT_CASE(512)
    SPFFT_CT_CASE(1024)
#define SPFFT_MR_CASE(NN) SPFFT_CT_CASE(NN)
    SPFFT_MR_SIZES(SPFFT_MR_CASE)
#undef SPFFT_MR_CASE
#undef SPFFT_CT_CASE
    default: {
      if (use_bluestein(n, sizeof(cx<T>))) {
        const BlueTables bt = bluestein_tables(n, sizeof(T) == 8);
        BlueEng<T, S> e{bt.pm, n, static_cast<const cx<T>*>(bt.chirp),
                        static_cast<const cx<T>*>(bt.filt), static_cast<const cx<T>*>(bt.twm)};
        f(e, kMaxThreads, e.pm.lines, std::size_t(2) * e.pm.lines * e.pm.ls * sizeof(cx<T>));
        return;
      }
      RtEng<T, S, LF> e{make_rt_plan(n, sizeof(cx<T>))};
      f(e, kRtThreads, e.p.lines,
        std::size_t(e.p.inplace ? 1 : 2) * e.p.lines * e.p.ls * sizeof(cx<T>));
      return;
    }
  }
}

inline unsigned ceil_div(long long a, long long b) { return static_cast<unsigned>((a + b - 1) / b); }

}  // namespace dev
}  // namespace spfft
