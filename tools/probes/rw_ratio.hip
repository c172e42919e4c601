// HBM read/write asymmetry probe: stream R bytes in and W bytes out with the
// stage kernels' access style (non-temporal 16-byte loads and stores, 256
// threads, 4 elements per lane), for the z-stage byte mix of 256^3 C2C fp64
// (backward: 140 MB of values in, 210 MB of sticks out; forward: the reverse)
// and a 1:1 copy of the same total. If the write-heavy mix is slower at equal
// total bytes, the backward/forward kernel-time gap is the memory system's.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/rw_ratio.hip -o /tmp/rw_ratio
#include <hip/hip_runtime.h>

#include <cstdio>

struct alignas(16) d2 {
  double x, y;
};

// out[j] = in[j * nr / nw]: every input element read once from HBM (repeated
// reads of an element hit the caches), every output element written once
__global__ void __launch_bounds__(256) mix(const d2* __restrict__ in, d2* __restrict__ out,
                                           long long nr, long long nw) {
  const long long base = (static_cast<long long>(blockIdx.x) * 256) * 4;
  d2 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long long j = base + k * 256 + threadIdx.x;
    const long long i = j < nw ? (j * nr) / nw : 0;
    v[k].x = __builtin_nontemporal_load(&in[i].x);
    v[k].y = __builtin_nontemporal_load(&in[i].y);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long long j = base + k * 256 + threadIdx.x;
    if (j < nw) {
      __builtin_nontemporal_store(v[k].x, &out[j].x);
      __builtin_nontemporal_store(v[k].y, &out[j].y);
    }
  }
}

// every output element written from the next input element, nr > nw: extra
// input read by a second load per lane
__global__ void __launch_bounds__(256) shrink(const d2* __restrict__ in, d2* __restrict__ out,
                                              long long nr, long long nw) {
  const long long base = (static_cast<long long>(blockIdx.x) * 256) * 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long long j = base + k * 256 + threadIdx.x;
    if (j >= nw) continue;
    const long long i0 = (j * nr) / nw, i1 = ((j + 1) * nr) / nw;
    d2 acc{0, 0};
    for (long long i = i0; i < i1; ++i) {
      acc.x += __builtin_nontemporal_load(&in[i].x);
      acc.y += __builtin_nontemporal_load(&in[i].y);
    }
    __builtin_nontemporal_store(acc.x, &out[j].x);
    __builtin_nontemporal_store(acc.y, &out[j].y);
  }
}

int main() {
  const long long MB = 1000000;
  const long long maxElems = 420 * MB / 16;
  d2 *a, *b;
  if (hipMalloc(&a, maxElems * 16) != hipSuccess || hipMalloc(&b, maxElems * 16) != hipSuccess) return 1;
  (void)hipMemset(a, 0, maxElems * 16);
  (void)hipMemset(b, 0, maxElems * 16);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  struct Case {
    const char* name;
    long long rb, wb;
  } cases[] = {{"write-heavy 140 MB in / 210 MB out (z backward mix)", 140 * MB, 210 * MB},
               {"read-heavy  210 MB in / 140 MB out (z forward mix)", 210 * MB, 140 * MB},
               {"balanced    175 MB in / 175 MB out", 175 * MB, 175 * MB},
               {"write-heavy 210 MB in / 268 MB out (y backward mix)", 210 * MB, 268 * MB},
               {"read-heavy  268 MB in / 210 MB out (y forward mix)", 268 * MB, 210 * MB}};
  for (const Case& c : cases) {
    const long long nr = c.rb / 16, nw = c.wb / 16;
    const bool grow = nw >= nr;
    const unsigned blocks = static_cast<unsigned>((nw + 1023) / 1024);
    float best = 1e30f;
    for (int it = 0; it < 12; ++it) {
      (void)hipEventRecord(e0, 0);
      if (grow)
        hipLaunchKernelGGL(mix, dim3(blocks), dim3(256), 0, 0, a, b, nr, nw);
      else
        hipLaunchKernelGGL(shrink, dim3(blocks), dim3(256), 0, 0, a, b, nr, nw);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (it > 1 && ms < best) best = ms;
    }
    std::printf("%-55s %8.1f us %7.0f GB/s\n", c.name, best * 1e3,
                (c.rb + c.wb) / (best * 1e-3) / 1e9);
  }
  return 0;
}
