// store_rate.hip -- measured IQ store rate of a 32K symbol per CU (verdict r3 item 2a).
//
// The 32K OFDM kernel (ofdm32_kernel) ends each (symbol, frame) workgroup with the IQ store of one
// symbol: GI + N = 2048 + 32768 complex64 samples = 278,528 bytes, written by 1024 threads as 16-byte
// non-temporal stores in the o32_store_pairs pattern (thread (a, b) holds samples b + 32 a + 1024 r;
// lane pairs b, b ^ 1 swap so each lane stores two consecutive samples; the last G samples also go
// to the guard interval).  This program issues exactly that store stream with nothing else in the
// workgroup, so its time per symbol is the store phase's cost in isolation:
//   lone   : G workgroups of 1024 threads (one per CU: 96 KB of LDS is reserved so no second one fits),
//            each storing K symbols back to back, G = 1, 8, 32, 64, 128, 256  -> per-CU rate vs the
//            number of CUs storing at the same time
//   grid   : one workgroup per symbol, 11520 symbols (the bench's 192 cfg3 frames x 60), as the OFDM
//            kernel's grid issues them -> the all-CU aggregate
// Usage: ./store_rate  (prints one JSON line per case; tools/store_rate.sh builds and runs it)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int NT = 1024, N = 32768, G = 2048, SYM = N + G;   // samples per symbol incl. GI
constexpr size_t SYM_BYTES = (size_t)SYM * 8;

__device__ __forceinline__ float swap_adjacent_lane(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
}

// one symbol's store, o32_store_pairs' address pattern and instruction mix (NT: non-temporal stores,
// as the OFDM kernel; else plain write-back stores)
template <bool NT_ST = true>
__device__ __forceinline__ void store_symbol(char *base, uint32_t tid, float seed) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  const uint32_t ta = ((tid >> 4) & 15u) | (((tid >> 8) & 1u) << 4), tb = (tid & 15u) | (((tid >> 9) & 1u) << 4);
  const uint32_t nout = tb + 32u * ta;
  const bool odd = nout & 1u;
  const uint32_t n0 = nout & ~1u;
#pragma unroll
  for (uint32_t k = 0; k < 16; k++) {
    const float2 e = make_float2(seed + (float)k, seed - (float)k), d = make_float2(seed * (float)k, (float)tid);
    const float2 re = make_float2(swap_adjacent_lane(e.x), swap_adjacent_lane(e.y));
    const float2 rd = make_float2(swap_adjacent_lane(d.x), swap_adjacent_lane(d.y));
    const float2 lo = odd ? rd : e, hi = odd ? d : re;
    const uint32_t n = n0 + 1024u * (2u * k + (odd ? 1u : 0u));
    if (NT_ST) {
      __builtin_nontemporal_store(f4v{lo.x, lo.y, hi.x, hi.y}, (f4v *)(base + ((uint32_t)G + n) * 8u));
      if (n >= (uint32_t)(N - G)) __builtin_nontemporal_store(f4v{lo.x, lo.y, hi.x, hi.y}, (f4v *)(base + (n - (uint32_t)(N - G)) * 8u));
    } else {
      *(f4v *)(base + ((uint32_t)G + n) * 8u) = f4v{lo.x, lo.y, hi.x, hi.y};
      if (n >= (uint32_t)(N - G)) *(f4v *)(base + (n - (uint32_t)(N - G)) * 8u) = f4v{lo.x, lo.y, hi.x, hi.y};
    }
  }
}

template <bool NT_ST>
__global__ __launch_bounds__(NT) void lone_kernel(char *out, int K) {
  extern __shared__ char pad[];   // occupancy: one workgroup per CU
  if (threadIdx.x == 0xFFFFFFFFu) pad[0] = 0;
  for (int s = 0; s < K; s++) store_symbol<NT_ST>(out + ((size_t)blockIdx.x * K + s) * SYM_BYTES, threadIdx.x, (float)s);
}

template <bool NT_ST>
__global__ __launch_bounds__(NT) void grid_kernel(char *out) {
  extern __shared__ char pad[];
  if (threadIdx.x == 0xFFFFFFFFu) pad[0] = 0;
  store_symbol<NT_ST>(out + (size_t)blockIdx.x * SYM_BYTES, threadIdx.x, (float)blockIdx.x);
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
  const int NSYM = 11520;
  char *buf = nullptr;
  CK(hipMalloc(&buf, (size_t)NSYM * SYM_BYTES));
  CK(hipMemset(buf, 0, (size_t)NSYM * SYM_BYTES));
  for (const void *fn : {(const void *)lone_kernel<true>, (const void *)lone_kernel<false>, (const void *)grid_kernel<true>,
                         (const void *)grid_kernel<false>})
    CK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const double clk = prop.clockRate * 1e3;   // Hz (peak engine clock)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grids[] = {1, 8, 32, 64, 128, 256};
  for (int nt = 1; nt >= 0; nt--)
  for (int g : grids) {
    const int K = 45;   // the bench's symbols per CU (11520 / 256)
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
      CK(hipEventRecord(e0));
      if (nt) hipLaunchKernelGGL(lone_kernel<true>, dim3(g), dim3(NT), 96 * 1024, 0, buf, K);
      else hipLaunchKernelGGL(lone_kernel<false>, dim3(g), dim3(NT), 96 * 1024, 0, buf, K);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep && ms < best) best = ms;
    }
    const double us = best * 1e3 / K;
    std::printf("{\"case\": \"lone\", \"nontemporal\": %d, \"workgroups\": %d, \"symbols_per_wg\": %d, \"us_per_symbol_per_cu\": %.3f, "
                "\"GBs_per_cu\": %.1f, \"GBs_total\": %.1f, \"cycles_per_symbol_at_peak_clock\": %.0f}\n",
                nt, g, K, us, SYM_BYTES / us * 1e-3, SYM_BYTES * g / us * 1e-3, us * 1e-6 * clk);
  }
  for (int nt = 1; nt >= 0; nt--) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
      CK(hipEventRecord(e0));
      if (nt) hipLaunchKernelGGL(grid_kernel<true>, dim3(NSYM), dim3(NT), 96 * 1024, 0, buf);
      else hipLaunchKernelGGL(grid_kernel<false>, dim3(NSYM), dim3(NT), 96 * 1024, 0, buf);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep && ms < best) best = ms;
    }
    const double us_cu = best * 1e3 / (NSYM / 256.0);
    std::printf("{\"case\": \"grid\", \"nontemporal\": %d, \"symbols\": %d, \"ms\": %.4f, \"GBs_total\": %.1f, \"us_per_symbol_per_cu\": %.3f, "
                "\"cycles_per_symbol_at_peak_clock\": %.0f}\n",
                nt, NSYM, best, SYM_BYTES * NSYM / (best * 1e-3) * 1e-9, us_cu, us_cu * 1e-6 * clk);
  }
  CK(hipFree(buf));
  return 0;
}
