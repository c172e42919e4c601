// Persistent-kernel copy rates (268 MB): static tile stride, atomic work queue,
// with and without register prefetch. Decides whether a cooperative persistent
// stage kernel can stream at HBM rate on MI355X.
#include <hip/hip_runtime.h>
#include <cstdio>

struct alignas(16) d2 { double x, y; };
#define CK(x) (void)(x)

template <int E>
__device__ __forceinline__ void tile_copy(const d2* __restrict__ a, d2* __restrict__ b, long long base) {
  d2 v[E];
#pragma unroll
  for (int k = 0; k < E; ++k) {
    const long long i = base + k * blockDim.x + threadIdx.x;
    v[k].x = __builtin_nontemporal_load(&a[i].x);
    v[k].y = __builtin_nontemporal_load(&a[i].y);
  }
#pragma unroll
  for (int k = 0; k < E; ++k) {
    const long long i = base + k * blockDim.x + threadIdx.x;
    __builtin_nontemporal_store(v[k].x, &b[i].x);
    __builtin_nontemporal_store(v[k].y, &b[i].y);
  }
}

template <int E>
__global__ void copy_static(const d2* __restrict__ a, d2* __restrict__ b, long long ntiles) {
  const long long tile = (long long)blockDim.x * E;
  for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) tile_copy<E>(a, b, t * tile);
}
template <int E>
__global__ void copy_static_contig(const d2* __restrict__ a, d2* __restrict__ b, long long ntiles) {
  // each block owns a contiguous range of tiles
  const long long tile = (long long)blockDim.x * E;
  const long long per = (ntiles + gridDim.x - 1) / gridDim.x;
  const long long t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
  for (long long t = t0; t < t1; ++t) tile_copy<E>(a, b, t * tile);
}
template <int E>
__global__ void copy_queue(const d2* __restrict__ a, d2* __restrict__ b, long long ntiles, unsigned* q) {
  const long long tile = (long long)blockDim.x * E;
  __shared__ long long t;
  for (;;) {
    if (threadIdx.x == 0) t = atomicAdd(q, 1u);
    __syncthreads();
    const long long tt = t;
    __syncthreads();
    if (tt >= ntiles) break;
    tile_copy<E>(a, b, tt * tile);
  }
}
template <int E>
__global__ void copy_block(const d2* __restrict__ a, d2* __restrict__ b, long long n) {
  tile_copy<E>(a, b, (long long)blockIdx.x * blockDim.x * E);
}

int main() {
  const long long n = 256LL * 256 * 256;
  d2 *a, *b;
  unsigned* q;
  CK(hipMalloc(&a, n * 16)); CK(hipMalloc(&b, n * 16)); CK(hipMalloc(&q, 64));
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
    printf("%-40s %8.1f us  %7.0f GB/s\n", name, us, 2.0 * n * 16 / (us * 1e3));
  };
  char nm[96];
  timeit("block E=4 t256 (reference)", [&] { copy_block<4><<<n / 1024, 256>>>(a, b, n); });
  timeit("block E=8 t256", [&] { copy_block<8><<<n / 2048, 256>>>(a, b, n); });
  for (int g : {256, 512, 1024, 2048}) {
    const long long nt4 = n / 1024;
    snprintf(nm, 96, "static stride E=4, %d blocks", g);
    timeit(nm, [&] { copy_static<4><<<g, 256>>>(a, b, nt4); });
    snprintf(nm, 96, "static contiguous E=4, %d blocks", g);
    timeit(nm, [&] { copy_static_contig<4><<<g, 256>>>(a, b, nt4); });
    snprintf(nm, 96, "atomic queue E=4, %d blocks", g);
    timeit(nm, [&] { CK(hipMemsetAsync(q, 0, 4, 0)); copy_queue<4><<<g, 256>>>(a, b, nt4, q); });
    snprintf(nm, 96, "atomic queue E=8, %d blocks", g);
    timeit(nm, [&] { CK(hipMemsetAsync(q, 0, 4, 0)); copy_queue<8><<<g, 256>>>(a, b, n / 2048, q); });
  }
  return 0;
}
