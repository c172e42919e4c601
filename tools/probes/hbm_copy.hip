// HBM calibration: streaming copy patterns at the stage-kernel working-set size
// (256^3 complex double = 268 MB). Prints time and read+write GB/s per pattern.
#include <hip/hip_runtime.h>
#include <cstdio>

struct alignas(16) d2 { double x, y; };
#define CK(x) (void)(x)

__global__ void copy_gs(const d2* __restrict__ a, d2* __restrict__ b, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) b[i] = a[i];
}
// E elements per lane, block-strided (lane t holds t, t+T, ...); all loads, then all stores
template <int E, bool NT>
__global__ void copy_block(const d2* __restrict__ a, d2* __restrict__ b, long long n) {
  const long long base = (long long)blockIdx.x * blockDim.x * E;
  d2 v[E];
#pragma unroll
  for (int k = 0; k < E; ++k) {
    long long i = base + k * blockDim.x + threadIdx.x;
    if (NT) { v[k].x = __builtin_nontemporal_load(&a[i].x); v[k].y = __builtin_nontemporal_load(&a[i].y); }
    else v[k] = a[i];
  }
#pragma unroll
  for (int k = 0; k < E; ++k) {
    long long i = base + k * blockDim.x + threadIdx.x;
    if (NT) { __builtin_nontemporal_store(v[k].x, &b[i].x); __builtin_nontemporal_store(v[k].y, &b[i].y); }
    else b[i] = v[k];
  }
}
// E elements per lane, wave-private chunk (wave w owns 64*E contiguous elements)
template <int E>
__global__ void copy_wave(const d2* __restrict__ a, d2* __restrict__ b, long long n) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long base = ((long long)blockIdx.x * (blockDim.x >> 6) + w) * 64 * E;
  d2 v[E];
#pragma unroll
  for (int k = 0; k < E; ++k) v[k] = a[base + k * 64 + lane];
#pragma unroll
  for (int k = 0; k < E; ++k) b[base + k * 64 + lane] = v[k];
}
// persistent: each block loops over tiles of T*E, software-pipelined (load tile i+1 before storing tile i)
template <int E>
__global__ void copy_pipe(const d2* __restrict__ a, d2* __restrict__ b, long long n) {
  const long long tile = (long long)blockDim.x * E;
  const long long ntiles = n / tile;
  d2 v[E], w[E];
  long long t = blockIdx.x;
  if (t >= ntiles) return;
#pragma unroll
  for (int k = 0; k < E; ++k) v[k] = a[t * tile + k * blockDim.x + threadIdx.x];
  for (; t < ntiles; t += gridDim.x) {
    const long long tn = t + gridDim.x;
    if (tn < ntiles) {
#pragma unroll
      for (int k = 0; k < E; ++k) w[k] = a[tn * tile + k * blockDim.x + threadIdx.x];
    }
#pragma unroll
    for (int k = 0; k < E; ++k) b[t * tile + k * blockDim.x + threadIdx.x] = v[k];
#pragma unroll
    for (int k = 0; k < E; ++k) v[k] = w[k];
  }
}

int main() {
  const long long n = 256LL * 256 * 256;
  d2 *a, *b;
  CK(hipMalloc(&a, n * 16)); CK(hipMalloc(&b, n * 16));
  CK(hipMemset(a, 0, n * 16)); CK(hipMemset(b, 0, n * 16));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipEventRecord(e0));
    const int R = 20;
    for (int i = 0; i < R; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / R;
    printf("%-34s %8.1f us  %7.0f GB/s\n", name, us, 2.0 * n * 16 / (us * 1e3));
  };
  char nm[80];
  for (int blocks : {2048, 16384, 65536}) {
    snprintf(nm, 80, "grid-stride, %d blocks", blocks);
    timeit(nm, [&] { copy_gs<<<blocks, 256>>>(a, b, n); });
  }
  timeit("block E=1 t256", [&] { copy_block<1, false><<<n / 256, 256>>>(a, b, n); });
  timeit("block E=4 t256", [&] { copy_block<4, false><<<n / 1024, 256>>>(a, b, n); });
  timeit("block E=8 t256", [&] { copy_block<8, false><<<n / 2048, 256>>>(a, b, n); });
  timeit("block E=16 t128", [&] { copy_block<16, false><<<n / 2048, 128>>>(a, b, n); });
  timeit("block E=16 t128 nt", [&] { copy_block<16, true><<<n / 2048, 128>>>(a, b, n); });
  timeit("block E=4 t256 nt", [&] { copy_block<4, true><<<n / 1024, 256>>>(a, b, n); });
  timeit("wave E=4", [&] { copy_wave<4><<<n / 1024, 256>>>(a, b, n); });
  timeit("wave E=16", [&] { copy_wave<16><<<n / 4096, 256>>>(a, b, n); });
  for (int g : {1024, 2048, 4096}) {
    snprintf(nm, 80, "pipelined E=8 t256, %d blocks", g);
    timeit(nm, [&] { copy_pipe<8><<<g, 256>>>(a, b, n); });
    snprintf(nm, 80, "pipelined E=16 t128, %d blocks", g);
    timeit(nm, [&] { copy_pipe<16><<<g, 128>>>(a, b, n); });
  }
  timeit("hipMemcpy D2D", [&] { CK(hipMemcpyAsync(b, a, n * 16, hipMemcpyDeviceToDevice, 0)); });
  return 0;
}
