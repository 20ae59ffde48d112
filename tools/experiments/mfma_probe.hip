// Operand-layout probe for the two MFMA forms a GF(2) matrix product can use on gfx950:
//   v_mfma_scale_f32_32x32x64_f8f6f4 with fp4 (e2m1) A and B, unit E8M0 scales, and
//   v_mfma_i32_32x32x32_i8.
// One wave; every lane's A and B registers come from random 0/1 elements (fp4 nibble 0x0 / 0x2 = 1.0,
// i8 byte 0 / 1); the accumulators go to a file that tools/experiments/mfma_probe.py matches against
// candidate lane maps.  Also times back-to-back fp4 MFMAs on one wave per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void fp4_k(const v8i *a, const v8i *b, v16f *c) {
  v16f C = {};
  C = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[threadIdx.x], b[threadIdx.x], C, 4, 4, 0, 127, 0, 127);
  c[threadIdx.x] = C;
}
__global__ void i8_k(const v4i *a, const v4i *b, v16i *c) {
  v16i C = {};
  C = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[threadIdx.x], b[threadIdx.x], C, 0, 0, 0);
  c[threadIdx.x] = C;
}
// throughput: N dependent-free MFMAs on 4 accumulators per wave
__global__ void fp4_rate(const v8i *a, const v8i *b, v16f *c, int n) {
  v8i A = a[threadIdx.x & 63], B = b[threadIdx.x & 63];
  v16f C0 = {}, C1 = {}, C2 = {}, C3 = {};
  for (int i = 0; i < n; i++) {
    C0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, C0, 4, 4, 0, 127, 0, 127);
    C1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(B, A, C1, 4, 4, 0, 127, 0, 127);
    C2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, A, C2, 4, 4, 0, 127, 0, 127);
    C3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(B, B, C3, 4, 4, 0, 127, 0, 127);
  }
  c[blockIdx.x * blockDim.x + threadIdx.x] = C0 + C1 + C2 + C3;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char **argv) {
  const char *out = argc > 1 ? argv[1] : "mfma_probe.bin";
  srand(12345);
  std::vector<uint32_t> a4(64 * 8), b4(64 * 8), a8(64 * 4), b8(64 * 4);
  for (auto &w : a4) { uint32_t v = 0; for (int j = 0; j < 8; j++) v |= (uint32_t)((rand() >> 7) & 1) << (4 * j + 1); w = v; }
  for (auto &w : b4) { uint32_t v = 0; for (int j = 0; j < 8; j++) v |= (uint32_t)((rand() >> 7) & 1) << (4 * j + 1); w = v; }
  for (auto &w : a8) { uint32_t v = 0; for (int j = 0; j < 4; j++) v |= (uint32_t)((rand() >> 7) & 1) << (8 * j); w = v; }
  for (auto &w : b8) { uint32_t v = 0; for (int j = 0; j < 4; j++) v |= (uint32_t)((rand() >> 7) & 1) << (8 * j); w = v; }
  void *da4, *db4, *dc4, *da8, *db8, *dc8, *dcr;
  CK(hipMalloc(&da4, 64 * 32)); CK(hipMalloc(&db4, 64 * 32)); CK(hipMalloc(&dc4, 64 * 64));
  CK(hipMalloc(&da8, 64 * 16)); CK(hipMalloc(&db8, 64 * 16)); CK(hipMalloc(&dc8, 64 * 64));
  CK(hipMemcpy(da4, a4.data(), 64 * 32, hipMemcpyHostToDevice));
  CK(hipMemcpy(db4, b4.data(), 64 * 32, hipMemcpyHostToDevice));
  CK(hipMemcpy(da8, a8.data(), 64 * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(db8, b8.data(), 64 * 16, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(fp4_k, dim3(1), dim3(64), 0, 0, (const v8i *)da4, (const v8i *)db4, (v16f *)dc4);
  hipLaunchKernelGGL(i8_k, dim3(1), dim3(64), 0, 0, (const v4i *)da8, (const v4i *)db8, (v16i *)dc8);
  CK(hipDeviceSynchronize());
  std::vector<float> c4(64 * 16);
  std::vector<int32_t> c8(64 * 16);
  CK(hipMemcpy(c4.data(), dc4, 64 * 64, hipMemcpyDeviceToHost));
  CK(hipMemcpy(c8.data(), dc8, 64 * 64, hipMemcpyDeviceToHost));
  FILE *f = fopen(out, "wb");
  fwrite(a4.data(), 4, a4.size(), f); fwrite(b4.data(), 4, b4.size(), f); fwrite(c4.data(), 4, c4.size(), f);
  fwrite(a8.data(), 4, a8.size(), f); fwrite(b8.data(), 4, b8.size(), f); fwrite(c8.data(), 4, c8.size(), f);
  fclose(f);
  // rate: 1024 workgroups of 256 threads (one wave per SIMD), n iterations of 4 MFMAs
  const int n = 4096, nwg = 1024;
  CK(hipMalloc(&dcr, (size_t)nwg * 256 * 64));
  hipLaunchKernelGGL(fp4_rate, dim3(nwg), dim3(256), 0, 0, (const v8i *)da4, (const v8i *)db4, (v16f *)dcr, n);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(fp4_rate, dim3(nwg), dim3(256), 0, 0, (const v8i *)da4, (const v8i *)db4, (v16f *)dcr, n);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double macs = (double)nwg * 4 * n * 4 * 32.0 * 32 * 64;
  printf("fp4 32x32x64 rate: %.3f ms, %.1f TMAC/s (%.1f dense TFLOP/s)\n", ms, macs / ms / 1e9, 2 * macs / ms / 1e9);
  printf("wrote %s\n", out);
  return 0;
}
