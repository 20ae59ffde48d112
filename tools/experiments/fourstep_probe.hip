// fourstep_probe.hip -- verdict r4 item 3 ("one structural attempt at the 32K OFDM's latency bound"):
// prototype of the 32K IFFT as two kernels with small workgroups, so loads, exchanges and IQ store
// drains of different symbols overlap on a CU, the intermediate (256 KB per symbol) passed through
// memory in chunks small enough to stay in the 256 MB Infinity Cache (MALL).
//
// With m = m0 + 32 m1 + 1024 m2 (input bin) and n = n2 + 32 n1 + 1024 n0 (output sample), the same
// 32 x 32 x 32 decomposition as ofdm32_kernel:
//   K1, workgroup (symbol, m0 group g of 8): thread (m0, m1) holds m2 = 0..31: DFT over m2, twiddle
//       w^((m0 + 32 m1) n2); LDS exchange to thread (m0, n2) holding m1 = 0..31: DFT over m1, twiddle
//       w_1024^(m0 n1); store Y[s][n1][g][n2][m0 & 7] (2 KB runs)
//   K2, workgroup (symbol, n1 group h of 8): thread (n1, n2) loads Y[s][n1][*][n2][*] (m0 = 0..31):
//       DFT over m0 -> x[n2 + 32 n1 + 1024 n0], normalisation, GI, IQ store (512 B per wave store)
// K1's input is emulated as the chain's scatter: 8192 data slots per workgroup, each a 2-byte
// constellation index pair and a 2-byte bin, constellation lookup from LDS, random bin scatter into LDS.
// Synthetic data; timing only (the arithmetic is the production kernel's, the result is not checked).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o fourstep_probe fourstep_probe.hip
//   ./fourstep_probe [symbols=76800] [chunk_symbols=480]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

constexpr int N = 32768, G = 2048, NT = 256, NSLOT = 8192;

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmulf(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ constexpr float kC[32] = {
    1.0f, 0.98078528f, 0.92387953f, 0.83146961f, 0.70710678f, 0.55557023f, 0.38268343f, 0.19509032f,
    0.0f, -0.19509032f, -0.38268343f, -0.55557023f, -0.70710678f, -0.83146961f, -0.92387953f, -0.98078528f,
    -1.0f, -0.98078528f, -0.92387953f, -0.83146961f, -0.70710678f, -0.55557023f, -0.38268343f, -0.19509032f,
    0.0f, 0.19509032f, 0.38268343f, 0.55557023f, 0.70710678f, 0.83146961f, 0.92387953f, 0.98078528f};
__device__ constexpr float kS[32] = {
    0.0f, 0.19509032f, 0.38268343f, 0.55557023f, 0.70710678f, 0.83146961f, 0.92387953f, 0.98078528f,
    1.0f, 0.98078528f, 0.92387953f, 0.83146961f, 0.70710678f, 0.55557023f, 0.38268343f, 0.19509032f,
    0.0f, -0.19509032f, -0.38268343f, -0.55557023f, -0.70710678f, -0.83146961f, -0.92387953f, -0.98078528f,
    -1.0f, -0.98078528f, -0.92387953f, -0.83146961f, -0.70710678f, -0.55557023f, -0.38268343f, -0.19509032f};
__host__ __device__ constexpr int brev5(int i) {
  return ((i & 1) << 4) | ((i & 2) << 2) | (i & 4) | ((i & 8) >> 2) | ((i & 16) >> 4);
}
__device__ __forceinline__ void dft32(float2 *x) {
#pragma unroll
  for (int i = 0; i < 32; i++) {
    const int j = brev5(i);
    if (i < j) { float2 t = x[i]; x[i] = x[j]; x[j] = t; }
  }
#pragma unroll
  for (int len = 2; len <= 32; len <<= 1) {
#pragma unroll
    for (int i = 0; i < 32; i += len)
#pragma unroll
      for (int k = 0; k < len / 2; k++) {
        const float2 a = x[i + k], b = x[i + k + len / 2];
        const float2 t = k == 0 ? b : cmulf(b, make_float2(kC[k * (32 / len)], kS[k * (32 / len)]));
        x[i + k] = cadd(a, t);
        x[i + k + len / 2] = csub(a, t);
      }
    __builtin_amdgcn_sched_barrier(0);
  }
}
// v[r] *= w^(e r) for r = 1..31 from table lookups (tw: w^i, i < 32768 in the two-level LDS form)
__device__ __forceinline__ float2 tw_at(const float2 *tw, uint32_t i) {
  i &= 32767u;
  return cmulf(tw[128 + (i >> 7)], tw[i & 127u]);
}
__device__ __forceinline__ void twiddle(float2 *v, const float2 *tw, uint32_t e) {
  const float2 w1 = tw_at(tw, e), w2 = tw_at(tw, 2 * e), w4 = tw_at(tw, 4 * e), w8 = tw_at(tw, 8 * e),
               w16 = tw_at(tw, 16 * e);
#pragma unroll
  for (int r = 1; r < 32; r++) {
    float2 w = make_float2(1.f, 0.f);
    if (r & 1) w = w1;
    if (r & 2) w = (r & 1) ? cmulf(w, w2) : w2;
    if (r & 4) w = (r & 3) ? cmulf(w, w4) : w4;
    if (r & 8) w = (r & 7) ? cmulf(w, w8) : w8;
    if (r & 16) w = (r & 15) ? cmulf(w, w16) : w16;
    v[r] = cmulf(v[r], w);
  }
}

struct K1Args {
  const uint16_t *pairs;   // per (symbol, group): NSLOT constellation index pairs
  const uint16_t *bins;    // per group: NSLOT bins (0..8191 within the group's 8192 bins), shared by symbols
  const float2 *qam;       // 256
  const float2 *tw;        // 128 + 256
  float2 *y;               // intermediate: per chunk symbol 32768 values
  int sym0;                // first symbol of the chunk (pairs index)
};
// K1: 256 threads, LDS: 8192 bins, one pad slot per 32 (66 KB) + constellation (2 KB) + twiddles (3 KB)
__global__ __launch_bounds__(NT) void k1(K1Args a) {
  extern __shared__ float2 lds[];
  float2 *q = lds + 8448, *tw = q + 256;
  const int t = threadIdx.x, wg = blockIdx.x, s = wg >> 2, g = wg & 3;
  q[t] = a.qam[t];
  for (int i = t; i < 384; i += NT) tw[i] = a.tw[i];
  __syncthreads();
  // scatter: 8192 slots, 32 per thread, 16-byte loads of 8 pairs / 8 bins
  const uint4 *pp = (const uint4 *)(a.pairs + ((size_t)(a.sym0 + s) * 4 + g) * NSLOT);
  const uint4 *bb = (const uint4 *)(a.bins + (size_t)g * NSLOT);
  uint4 pv[4], bv[4];
#pragma unroll
  for (int u = 0; u < 4; u++) {
    pv[u] = pp[t + NT * u];
    bv[u] = bb[t + NT * u];
  }
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const uint32_t pw[4] = {pv[u].x, pv[u].y, pv[u].z, pv[u].w}, bw[4] = {bv[u].x, bv[u].y, bv[u].z, bv[u].w};
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t p = (pw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu, b = (bw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
      const uint32_t bin = b + (b >> 5);
      lds[bin] = make_float2(q[p & 0xFF].x, q[p >> 8].y);
    }
  }
  __syncthreads();
  // thread (m0l = t & 7, m1 = t >> 3): bins m0l + 8 m1 + 256 m2 within the group (group-local index)
  const int m0l = t & 7, m1 = t >> 3, m0 = 8 * g + m0l;
  float2 v[32];
#pragma unroll
  for (int r = 0; r < 32; r++) {
    const uint32_t k = (uint32_t)(m0l + 8 * m1 + 256 * r);
    v[r] = lds[k + (k >> 5)];
  }
  dft32(v);
  twiddle(v, tw, (uint32_t)(m0 + 32 * m1));
  __syncthreads();
  // exchange: write (m0l, m1, n2 = r), read as thread (m0l, n2 = t >> 3) the values m1 = r
#pragma unroll
  for (int r = 0; r < 32; r++) {
    const uint32_t e = (uint32_t)(m0l + 8 * r + 256 * m1);
    lds[e + (e >> 5)] = v[r];
  }
  __syncthreads();
  const int n2 = t >> 3;
#pragma unroll
  for (int r = 0; r < 32; r++) {
    const uint32_t e = (uint32_t)(m0l + 8 * n2 + 256 * r);
    v[r] = lds[e + (e >> 5)];
  }
  dft32(v);
  twiddle(v, tw, (uint32_t)(32 * m0));   // w_1024^(m0 n1) = w^(32 m0 n1)
  // Y[s][n1][g][n2][m0l]: per n1 a 2 KB run of the workgroup
  float2 *y = a.y + (size_t)s * N + (size_t)g * 256 + n2 * 8 + m0l;
#pragma unroll
  for (int r = 0; r < 32; r++) y[(size_t)r * 1024] = v[r];
}

struct K2Args {
  const float2 *y;
  float2 *out;   // per chunk symbol N + G samples
  float nrm;
};
__global__ __launch_bounds__(NT) void k2(K2Args a) {
  const int t = threadIdx.x, wg = blockIdx.x, s = wg >> 2, h = wg & 3;
  const int n2 = t & 31, n1 = 8 * h + (t >> 5);
  const float2 *y = a.y + (size_t)s * N + (size_t)n1 * 1024 + n2 * 8;
  float2 v[32];
#pragma unroll
  for (int g = 0; g < 4; g++) {
    const float4 *p = (const float4 *)(y + g * 256);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const float4 w = p[k];
      v[8 * g + 2 * k] = make_float2(w.x, w.y);
      v[8 * g + 2 * k + 1] = make_float2(w.z, w.w);
    }
  }
  dft32(v);
  float2 *o = a.out + (size_t)s * (N + G);
  const uint32_t nb = (uint32_t)(n2 + 32 * n1);
#pragma unroll
  for (int r = 0; r < 32; r++) {
    const uint32_t n = nb + 1024u * r;
    const float2 x = make_float2(v[r].x * a.nrm, v[r].y * a.nrm);
    __builtin_nontemporal_store(__builtin_bit_cast(uint64_t, x), (uint64_t *)(o + G + n));
    if (n >= (uint32_t)(N - G)) __builtin_nontemporal_store(__builtin_bit_cast(uint64_t, x), (uint64_t *)(o + n - (N - G)));
  }
}

int main(int argc, char **argv) {
  const int NS = argc > 1 ? std::atoi(argv[1]) : 76800;
  const int C = argc > 2 ? std::atoi(argv[2]) : 480;
  const int NBUF = argc > 3 ? std::atoi(argv[3]) : 2;   // intermediate buffers (chunks in flight)
  std::vector<uint16_t> pairs((size_t)NS * 4 * NSLOT), bins(4 * NSLOT);
  uint32_t x = 12345;
  auto rnd = [&]() { x = x * 1664525u + 1013904223u; return x >> 8; };
  for (auto &p : pairs) p = (uint16_t)(rnd() & 0xFFFF);
  for (int g = 0; g < 4; g++) {   // a random permutation of the group's 8192 bins
    std::vector<uint16_t> perm(NSLOT);
    for (int i = 0; i < NSLOT; i++) perm[i] = (uint16_t)i;
    for (int i = NSLOT - 1; i > 0; i--) std::swap(perm[i], perm[rnd() % (i + 1)]);
    for (int i = 0; i < NSLOT; i++) bins[g * NSLOT + i] = perm[i];
  }
  std::vector<float2> qam(256), tw(384);
  for (int i = 0; i < 256; i++) qam[i] = make_float2((i & 15) * 0.1f, (i >> 4) * 0.1f);
  for (int i = 0; i < 384; i++) {
    const double ph = 2 * 3.141592653589793 * (i < 128 ? i : 128 * (i - 128)) / 32768.0;
    tw[i] = make_float2((float)std::cos(ph), (float)std::sin(ph));
  }
  uint16_t *dp, *db;
  float2 *dq, *dtw, *dy, *dout;
  CK(hipMalloc(&dp, pairs.size() * 2));
  CK(hipMalloc(&db, bins.size() * 2));
  CK(hipMalloc(&dq, 256 * 8));
  CK(hipMalloc(&dtw, 384 * 8));
  CK(hipMalloc(&dy, (size_t)NBUF * C * N * 8));
  CK(hipMalloc(&dout, (size_t)NS * (N + G) * 8));
  CK(hipMemcpy(dp, pairs.data(), pairs.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, bins.data(), bins.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dq, qam.data(), 256 * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dtw, tw.data(), 384 * 8, hipMemcpyHostToDevice));
  const int lds1 = (8448 + 256 + 384) * 8;
  CK(hipFuncSetAttribute((const void *)k1, hipFuncAttributeMaxDynamicSharedMemorySize, lds1));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](int mode) {   // 0: K1 only, 1: K2 only, 2: both alternating per chunk
    for (int c0 = 0, ci = 0; c0 < NS; c0 += C, ci++) {
      const int n = NS - c0 < C ? NS - c0 : C;
      float2 *y = dy + (size_t)(ci % NBUF) * C * N;
      if (mode != 1) {
        K1Args a{dp, db, dq, dtw, y, c0};
        hipLaunchKernelGGL(k1, dim3(4 * n), dim3(NT), lds1, 0, a);
      }
      if (mode != 0) {
        K2Args b{y, dout + (size_t)c0 * (N + G), 1.0f / 181.0f};
        hipLaunchKernelGGL(k2, dim3(4 * n), dim3(NT), 0, 0, b);
      }
    }
    CK(hipGetLastError());
  };
  const char *names[3] = {"K1 only", "K2 only", "K1+K2 chunked"};
  for (int mode = 0; mode < 3; mode++) {
    run(mode);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
      CK(hipEventRecord(e0, 0));
      run(mode);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    const double iq = (double)NS * (N + G) * 8, pr = (double)NS * N * 2;
    std::printf("{\"mode\": \"%s\", \"symbols\": %d, \"chunk\": %d, \"nbuf\": %d, \"ms\": %.4f, "
                "\"ms_per_1280_frames\": %.4f, \"minimal_GBs\": %.1f}\n",
                names[mode], NS, C, NBUF, best, best * 76800.0 / NS, (iq + pr) / (best * 1e-3) / 1e9);
  }
  return 0;
}
