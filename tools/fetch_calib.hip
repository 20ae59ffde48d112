// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE (gfx950) against known byte counts
// for the access widths the chain's kernels use (MI355X_MICROARCH.md "HBM": only 16 B/lane streaming
// reads and stores are calibrated there).
//
// Each kernel streams exactly BYTES bytes (1 GiB: four times the 256 MiB Infinity Cache, so the
// counters see HBM traffic) with W bytes per lane, fully coalesced:
//   rd<W>: loads, folds them into one value per workgroup (8 bytes written per workgroup, noise)
//   wr<W>: stores
// Usage: rocprofv3 --pmc FETCH_SIZE -T -d DIR -o calib -- ./fetch_calib
//        rocprofv3 --pmc WRITE_SIZE -T -d DIR -o calib -- ./fetch_calib
// then tools/fetch_calib.py DIR prints counter bytes / true bytes per kernel.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr size_t BYTES = size_t(1) << 30;

struct W16 { uint4 v; };
__device__ __forceinline__ uint64_t fold(uint16_t v) { return v; }
__device__ __forceinline__ uint64_t fold(uint32_t v) { return v; }
__device__ __forceinline__ uint64_t fold(uint2 v) { return (uint64_t)v.x + v.y; }
__device__ __forceinline__ uint64_t fold(W16 v) { return (uint64_t)v.v.x + v.v.y + v.v.z + v.v.w; }
__device__ __forceinline__ void fill(uint16_t &v, size_t i) { v = (uint16_t)i; }
__device__ __forceinline__ void fill(uint32_t &v, size_t i) { v = (uint32_t)i; }
__device__ __forceinline__ void fill(uint2 &v, size_t i) { v = make_uint2((uint32_t)i, (uint32_t)i + 1); }
__device__ __forceinline__ void fill(W16 &v, size_t i) { v.v = make_uint4((uint32_t)i, (uint32_t)i + 1, (uint32_t)i + 2, (uint32_t)i + 3); }

template <class T>
__global__ __launch_bounds__(256) void rd_kernel(const T *__restrict__ in, size_t n, uint64_t *__restrict__ out) {
  uint64_t acc = 0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    acc += fold(in[i]);
  }
  __shared__ uint64_t red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t s = 0;
    for (int t = 0; t < 256; t++) s += red[t];
    out[blockIdx.x] = s;
  }
}

template <class T>
__global__ __launch_bounds__(256) void wr_kernel(T *__restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    T v;
    fill(v, i);
    out[i] = v;
  }
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main() {
  void *buf = nullptr;
  uint64_t *red = nullptr;
  const int grid = 256 * 16;
  CK(hipMalloc(&buf, BYTES));
  CK(hipMalloc(&red, grid * sizeof(uint64_t)));
  CK(hipMemset(buf, 1, BYTES));
  CK(hipDeviceSynchronize());
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(rd_kernel<uint16_t>, dim3(grid), dim3(256), 0, 0, (const uint16_t *)buf, BYTES / 2, red);
    hipLaunchKernelGGL(rd_kernel<uint32_t>, dim3(grid), dim3(256), 0, 0, (const uint32_t *)buf, BYTES / 4, red);
    hipLaunchKernelGGL(rd_kernel<uint2>, dim3(grid), dim3(256), 0, 0, (const uint2 *)buf, BYTES / 8, red);
    hipLaunchKernelGGL(rd_kernel<W16>, dim3(grid), dim3(256), 0, 0, (const W16 *)buf, BYTES / 16, red);
    hipLaunchKernelGGL(wr_kernel<uint16_t>, dim3(grid), dim3(256), 0, 0, (uint16_t *)buf, BYTES / 2);
    hipLaunchKernelGGL(wr_kernel<uint32_t>, dim3(grid), dim3(256), 0, 0, (uint32_t *)buf, BYTES / 4);
    hipLaunchKernelGGL(wr_kernel<uint2>, dim3(grid), dim3(256), 0, 0, (uint2 *)buf, BYTES / 8);
    hipLaunchKernelGGL(wr_kernel<W16>, dim3(grid), dim3(256), 0, 0, (W16 *)buf, BYTES / 16);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
  }
  std::printf("fetch_calib: %zu bytes per kernel, widths 2 4 8 16\n", BYTES);
  CK(hipFree(buf));
  CK(hipFree(red));
  return 0;
}
