// store_rate.hip -- measured IQ store rate of a 32K symbol per CU (verdict r3 item 2a).
//
// The 32K OFDM kernel (ofdm32_kernel) ends each (symbol, frame) workgroup with the IQ store of one
// symbol: GI + N = 2048 + 32768 complex64 samples = 278,528 bytes, written by 1024 threads as 16-byte
// non-temporal stores in the o32_store_pairs pattern (thread (a, b) holds samples b + 32 a + 1024 r;
// lane pairs b, b ^ 1 swap so each lane stores two consecutive samples; the last G samples also go
// to the guard interval).  This program issues store streams of one symbol per workgroup with nothing
// else in the workgroup, so its time per symbol is the store phase's cost in isolation:
//   pattern  o32     : the kernel's own address pattern (8 runs of 128 B per wave-instruction)
//            contig16: 16-byte stores, each wave-instruction one contiguous 1 KB
//            contig8 : 8-byte stores, each wave-instruction one contiguous 512 B
//   lone     : G workgroups of 1024 threads (one per CU: 96 KB of LDS is reserved so no second one fits),
//              each storing K symbols back to back, G = 1, 8, 32, 64, 128, 256  -> per-CU rate vs the
//              number of CUs storing at the same time; drain = 1 adds an s_waitcnt vmcnt(0) + barrier
//              after every symbol (the kernel's situation: a workgroup's symbol must complete before
//              the CU takes the next), so drain - no drain = the completion latency per symbol
//   grid     : one workgroup per symbol, 11520 symbols (the bench's 192 cfg3 frames x 60), as the OFDM
//              kernel's grid issues them -> the all-CU aggregate
// Usage: hipcc -O3 --offload-arch=gfx950 -o tools/store_rate tools/store_rate.hip && tools/store_rate
// (one JSON line per case)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int NT = 1024, N = 32768, G = 2048, SYM = N + G;   // samples per symbol incl. GI
constexpr size_t SYM_BYTES = (size_t)SYM * 8;
constexpr int O32 = 0, CONTIG16 = 1, CONTIG8 = 2;
static const char *PAT_NAME[3] = {"o32", "contig16", "contig8"};

__device__ __forceinline__ float swap_adjacent_lane(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
}

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

template <bool NT_ST, class V>
__device__ __forceinline__ void st(char *p, V v) {
  if (NT_ST) __builtin_nontemporal_store(v, (V *)p);
  else *(V *)p = v;
}

// one symbol's store in pattern PAT
template <int PAT, bool NT_ST>
__device__ __forceinline__ void store_symbol(char *base, uint32_t tid, float seed) {
  if (PAT == CONTIG16) {
#pragma unroll
    for (uint32_t i = 0; i < SYM_BYTES / (16 * NT); i++)
      st<NT_ST>(base + (size_t)i * 16 * NT + 16u * tid, f4v{seed + (float)i, seed, (float)tid, seed - (float)i});
    return;
  }
  if (PAT == CONTIG8) {
#pragma unroll
    for (uint32_t i = 0; i < SYM_BYTES / (8 * NT); i++)
      st<NT_ST>(base + (size_t)i * 8 * NT + 8u * tid, f2v{seed + (float)i, (float)tid});
    return;
  }
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
    st<NT_ST>(base + ((uint32_t)G + n) * 8u, f4v{lo.x, lo.y, hi.x, hi.y});
    if (n >= (uint32_t)(N - G)) st<NT_ST>(base + (n - (uint32_t)(N - G)) * 8u, f4v{lo.x, lo.y, hi.x, hi.y});
  }
}

template <int PAT, bool NT_ST, bool DRAIN>
__global__ __launch_bounds__(NT) void lone_kernel(char *out, int K) {
  extern __shared__ char pad[];   // occupancy: one workgroup per CU
  if (threadIdx.x == 0xFFFFFFFFu) pad[0] = 0;
  for (int s = 0; s < K; s++) {
    store_symbol<PAT, NT_ST>(out + ((size_t)blockIdx.x * K + s) * SYM_BYTES, threadIdx.x, (float)s);
    if (DRAIN) {
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this symbol's stores complete
      __syncthreads();
    }
  }
}

// the kernel's duty cycle: every CU alternates SLEEP x 64 x 127 idle cycles (the OFDM kernel's
// compute phases) with one symbol's store and its drain, K symbols, the CUs' phases staggered by
// blockIdx; (time - K x idle) / K = a symbol's store phase among the other CUs' stores
template <int PAT>
__global__ __launch_bounds__(NT) void duty_kernel(char *out, int K, int sleeps, int do_store) {
  extern __shared__ char pad[];
  if (threadIdx.x == 0xFFFFFFFFu) pad[0] = 0;
  for (int i = 0; i < (int)(blockIdx.x & 7u) * sleeps / 8; i++) __builtin_amdgcn_s_sleep(127);
  for (int s = 0; s < K; s++) {
    for (int i = 0; i < sleeps; i++) __builtin_amdgcn_s_sleep(127);
    if (do_store) store_symbol<PAT, true>(out + ((size_t)blockIdx.x * K + s) * SYM_BYTES, threadIdx.x, (float)s);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
  }
}

template <int PAT, bool NT_ST>
__global__ __launch_bounds__(NT) void grid_kernel(char *out) {
  extern __shared__ char pad[];
  if (threadIdx.x == 0xFFFFFFFFu) pad[0] = 0;
  store_symbol<PAT, NT_ST>(out + (size_t)blockIdx.x * SYM_BYTES, threadIdx.x, (float)blockIdx.x);
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
      return 1;                                                                \
    }                                                                          \
  } while (0)

template <class F>
static float best_ms(hipEvent_t e0, hipEvent_t e1, F launch) {
  float best = 1e30f;
  for (int rep = 0; rep < 5; rep++) {
    (void)hipEventRecord(e0);
    launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep && ms < best) best = ms;
  }
  return best;
}

template <int PAT, bool NT_ST, bool DRAIN>
static int run_lone(char *buf, double clk, hipEvent_t e0, hipEvent_t e1) {
  CK(hipFuncSetAttribute((const void *)lone_kernel<PAT, NT_ST, DRAIN>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
  const int grids[] = {1, 8, 32, 64, 128, 256};
  for (int g : grids) {
    const int K = 45;   // the bench's symbols per CU (11520 / 256)
    const float ms = best_ms(e0, e1, [&] { hipLaunchKernelGGL((lone_kernel<PAT, NT_ST, DRAIN>), dim3(g), dim3(NT), 96 * 1024, 0, buf, K); });
    CK(hipGetLastError());
    const double us = ms * 1e3 / K;
    std::printf("{\"case\": \"lone\", \"pattern\": \"%s\", \"nontemporal\": %d, \"drain\": %d, \"workgroups\": %d, \"symbols_per_wg\": %d, "
                "\"us_per_symbol_per_cu\": %.3f, \"GBs_per_cu\": %.1f, \"GBs_total\": %.1f, \"cycles_per_symbol_at_peak_clock\": %.0f}\n",
                PAT_NAME[PAT], (int)NT_ST, (int)DRAIN, g, K, us, SYM_BYTES / us * 1e-3, SYM_BYTES * g / us * 1e-3, us * 1e-6 * clk);
  }
  return 0;
}

template <int PAT, bool NT_ST>
static int run_grid(char *buf, int nsym, double clk, hipEvent_t e0, hipEvent_t e1) {
  CK(hipFuncSetAttribute((const void *)grid_kernel<PAT, NT_ST>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
  const float ms = best_ms(e0, e1, [&] { hipLaunchKernelGGL((grid_kernel<PAT, NT_ST>), dim3(nsym), dim3(NT), 96 * 1024, 0, buf); });
  CK(hipGetLastError());
  const double us_cu = ms * 1e3 / (nsym / 256.0);
  std::printf("{\"case\": \"grid\", \"pattern\": \"%s\", \"nontemporal\": %d, \"symbols\": %d, \"ms\": %.4f, \"GBs_total\": %.1f, "
              "\"us_per_symbol_per_cu\": %.3f, \"cycles_per_symbol_at_peak_clock\": %.0f}\n",
              PAT_NAME[PAT], (int)NT_ST, nsym, ms, SYM_BYTES * nsym / (ms * 1e-3) * 1e-9, us_cu, us_cu * 1e-6 * clk);
  return 0;
}

template <int PAT>
static int run_duty(char *buf, hipEvent_t e0, hipEvent_t e1) {
  CK(hipFuncSetAttribute((const void *)duty_kernel<PAT>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
  const int K = 45;
  for (int sleeps : {0, 3, 6, 9}) {
    const float ms = best_ms(e0, e1, [&] { hipLaunchKernelGGL((duty_kernel<PAT>), dim3(256), dim3(NT), 96 * 1024, 0, buf, K, sleeps, 1); });
    const float sl = best_ms(e0, e1, [&] { hipLaunchKernelGGL((duty_kernel<PAT>), dim3(256), dim3(NT), 96 * 1024, 0, buf, K, sleeps, 0); });
    CK(hipGetLastError());
    std::printf("{\"case\": \"duty\", \"pattern\": \"%s\", \"cus\": 256, \"symbols_per_cu\": %d, \"idle_us_per_symbol\": %.3f, "
                "\"ms\": %.4f, \"store_us_per_symbol\": %.3f}\n",
                PAT_NAME[PAT], K, sl * 1e3 / K, ms, (ms - sl) * 1e3 / K);
  }
  return 0;
}

int main() {
  const int NSYM = 11520;
  char *buf = nullptr;
  CK(hipMalloc(&buf, (size_t)NSYM * SYM_BYTES));
  CK(hipMemset(buf, 0, (size_t)NSYM * SYM_BYTES));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const double clk = prop.clockRate * 1e3;   // Hz (peak engine clock)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  if (run_lone<O32, true, false>(buf, clk, e0, e1) || run_lone<O32, true, true>(buf, clk, e0, e1) ||
      run_lone<O32, false, false>(buf, clk, e0, e1) || run_lone<CONTIG16, true, false>(buf, clk, e0, e1) ||
      run_lone<CONTIG16, true, true>(buf, clk, e0, e1) || run_lone<CONTIG8, true, false>(buf, clk, e0, e1) ||
      run_grid<O32, true>(buf, NSYM, clk, e0, e1) || run_grid<O32, false>(buf, NSYM, clk, e0, e1) ||
      run_grid<CONTIG16, true>(buf, NSYM, clk, e0, e1) || run_grid<CONTIG8, true>(buf, NSYM, clk, e0, e1) ||
      run_duty<O32>(buf, e0, e1) || run_duty<CONTIG16>(buf, e0, e1))
    return 1;
  CK(hipFree(buf));
  return 0;
}
