// Achievable HBM write bandwidth on this device (diagnostic): a store-only kernel over a 1 GiB buffer in the shapes
// the K* build uses (16-byte stores, plain / non-temporal), a read+write copy and hipMemsetAsync, so the K* build's
// roofline fraction (its 8 n C bytes written per chunk against the 8 TB/s peak) can be read against what a pure
// write stream reaches.  Prints GB/s per variant (median of 9).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 write_peak.hip -o write_peak
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

template <int NT>
__global__ void __launch_bounds__(256) store_kernel(d2* __restrict__ p, size_t n2, double v) {
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += stride) {
    d2 x = {v + (double)i, v};
    if constexpr (NT) __builtin_nontemporal_store(x, p + i);
    else p[i] = x;
  }
}

// the K* build's store shape: a workgroup owns 64 rows x 256 columns of a row-major matrix (row length ld), wave w
// columns 64w .. 64w+63; one store instruction writes 512 B of each of two rows (16 B per lane)
__global__ void __launch_bounds__(256) rows_kernel(double* __restrict__ p, size_t ld, double v) {
  const size_t r0 = (size_t)blockIdx.y * 64, c0 = (size_t)blockIdx.x * 256;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, half = lane >> 5, l = lane & 31;
#pragma unroll 8
  for (int r = 0; r < 64; r += 2) {
    d2 x = {v + r, v};
    *reinterpret_cast<d2*>(p + (r0 + r + half) * ld + c0 + 64 * w + 2 * l) = x;
  }
}

// U 16-byte stores in flight per lane per iteration, each instruction wave-contiguous (1 KB), consecutive instructions
// 1 KB apart (a workgroup covers 4U KB per iteration)
template <int U>
__global__ void __launch_bounds__(256) store_unrolled(d2* __restrict__ p, size_t n2, double v) {
  const size_t per = (size_t)256 * U;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (size_t base = (size_t)blockIdx.x * per; base < n2; base += (size_t)gridDim.x * per) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      d2 x = {v + u, v};
      __builtin_nontemporal_store(x, p + base + (size_t)(w * U + u) * 64 + lane);
    }
  }
}

// the K* shape with R rows per store round: a workgroup owns 64 rows x 256 columns, every wave issues R row stores
// back to back (16 B per lane, 2 rows per instruction) before the next group
template <int R>
__global__ void __launch_bounds__(256) rows_nt_kernel(double* __restrict__ p, size_t ld, double v) {
  const size_t r0 = (size_t)blockIdx.y * 64, c0 = (size_t)blockIdx.x * 256;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, half = lane >> 5, l = lane & 31;
  for (int r = 0; r < 64; r += 2 * R) {
#pragma unroll
    for (int q = 0; q < R; ++q) {
      d2 x = {v + r + q, v};
      __builtin_nontemporal_store(x, reinterpret_cast<d2*>(p + (r0 + r + 2 * q + half) * ld + c0 + 64 * w + 2 * l));
    }
  }
}

__global__ void __launch_bounds__(256) copy_kernel(const d2* __restrict__ a, d2* __restrict__ b, size_t n2) {
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += stride) b[i] = a[i];
}

int main() {
  const size_t bytes = (size_t)1 << 30, n2 = bytes / 16;
  d2 *p, *q;
  CK(hipMalloc(&p, bytes));
  CK(hipMalloc(&q, bytes));
  CK(hipMemset(p, 0, bytes));
  CK(hipMemset(q, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double moved, auto&& launch) {
    std::vector<float> t;
    launch();
    CK(hipDeviceSynchronize());
    for (int r = 0; r < 9; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    CK(hipGetLastError());
    std::sort(t.begin(), t.end());
    printf("%-44s %8.3f ms  %7.1f GB/s\n", name, t[4], moved / (t[4] * 1e-3) / 1e9);
  };
  for (int g : {1024, 2048, 4096, 8192, 16384}) {
    char nm[64];
    snprintf(nm, sizeof nm, "store 16B plain, grid %d", g);
    timeit(nm, bytes, [&] { store_kernel<0><<<g, 256>>>(p, n2, 1.0); });
    snprintf(nm, sizeof nm, "store 16B nontemporal, grid %d", g);
    timeit(nm, bytes, [&] { store_kernel<1><<<g, 256>>>(p, n2, 1.0); });
  }
  const size_t ld = 32768, rows = bytes / 8 / ld;  // the K* chunk shape: 4096 x 32768
  timeit("K* shape: 64 x 256 blocks, 512 B row segments", bytes,
         [&] { rows_kernel<<<dim3((unsigned)(ld / 256), (unsigned)(rows / 64)), 256>>>((double*)p, ld, 1.0); });
  timeit("K* shape, nontemporal, 4 rows per round", bytes,
         [&] { rows_nt_kernel<4><<<dim3((unsigned)(ld / 256), (unsigned)(rows / 64)), 256>>>((double*)p, ld, 1.0); });
  timeit("K* shape, nontemporal, 16 rows per round", bytes,
         [&] { rows_nt_kernel<16><<<dim3((unsigned)(ld / 256), (unsigned)(rows / 64)), 256>>>((double*)p, ld, 1.0); });
  for (int g : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "store 4 x 16B unrolled nt, grid %d", g);
    timeit(nm, bytes, [&] { store_unrolled<4><<<g, 256>>>(p, n2, 1.0); });
    snprintf(nm, sizeof nm, "store 8 x 16B unrolled nt, grid %d", g);
    timeit(nm, bytes, [&] { store_unrolled<8><<<g, 256>>>(p, n2, 1.0); });
  }
  timeit("copy 16B (read + write bytes)", 2.0 * bytes, [&] { copy_kernel<<<8192, 256>>>(p, q, n2); });
  timeit("hipMemsetAsync", bytes, [&] { CK(hipMemsetAsync(p, 0, bytes)); });
  printf("WRITE PEAK DONE\n");
  return 0;
}
