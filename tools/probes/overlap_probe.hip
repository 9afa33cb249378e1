// Does a dependent-free next launch start before the previous one ends on gfx950?  (diagnostic, not product)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 overlap_probe.hip -o overlap_probe
// Kernel A (one workgroup) spins ~20 us; kernel B (one workgroup) stamps its start.  Plain stores only (no
// synchronisation between the kernels).  Modes: 0 plain back-to-back launches on one stream, 1 the second launch with
// hipExtAnyOrderLaunch, 2 the second launch on another stream.  Printed (100 MHz ticks -> us, median of 30):
// B start - A end (negative = the launches overlapped).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

__global__ void kernel_a(unsigned long long* st, unsigned ticks) {
  const unsigned long long t0 = now();
  while (now() - t0 < ticks) {}
  const unsigned long long t1 = now();
  if (threadIdx.x == 0) {
    st[0] = t0;
    st[1] = t1;
  }
}

__global__ void kernel_b(unsigned long long* st) {
  const unsigned long long t0 = now();
  if (threadIdx.x == 0) st[2] = t0;
}

int main() {
  unsigned long long* st;
  CK(hipMalloc(&st, 64 * sizeof(unsigned long long)));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  for (int mode = 0; mode < 3; ++mode) {
    std::vector<double> gap;
    for (int it = 0; it < 31; ++it) {
      hipLaunchKernelGGL(kernel_a, dim3(1), dim3(64), 0, s0, st, 2000u);
      if (mode == 0) hipLaunchKernelGGL(kernel_b, dim3(1), dim3(64), 0, s0, st);
      else if (mode == 1)
        hipExtLaunchKernelGGL(kernel_b, dim3(1), dim3(64), 0, s0, nullptr, nullptr, hipExtAnyOrderLaunch, st);
      else hipLaunchKernelGGL(kernel_b, dim3(1), dim3(64), 0, s1, st);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      unsigned long long h[3];
      CK(hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost));
      if (it == 0) continue;
      gap.push_back(((double)(long long)(h[2] - h[1])) / 100.0);
    }
    std::sort(gap.begin(), gap.end());
    printf("mode %d (%s): B start - A end median %.2f us (min %.2f max %.2f)\n", mode,
           mode == 0 ? "same stream" : mode == 1 ? "any-order flag" : "second stream", gap[gap.size() / 2], gap.front(),
           gap.back());
  }
  return 0;
}
