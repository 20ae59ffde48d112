// t2_kernels.hip -- gfx950 (MI355X / CDNA4) kernels of the DVB-T2 transmit chain.
//
//   fec_kernel   one workgroup per FEC block: BBFRAME build (header, CRC-8 sync
//                replacement, scrambling) + BCH (256-lane chunked byte-table division,
//                Horner-combined with GF(2) shift matrices via wave ballots) + LDPC as a
//                quasi-cyclic array of 360-bit rotations with a bit-packed accumulate scan.
//                Reference: lib/bbheaderbch_bb_impl.cc:648-742 (+ ldpc_calculate :625-646).
//   map_kernel   one workgroup per FEC block: column-twist bit interleave + demux + QAM LUT
//                + rotated-constellation Q delay, optionally cell-interleaved through LDS.
//                Reference: lib/interleavermod_bc_impl.cc:270-704, framemapper :1973-1998.
//   ofdm_kernel  one workgroup per OFDM symbol: gather (frame map + time/frequency
//                interleave + pilots, all pre-composed into one int32 map) fused into the
//                first pass of a 3-pass register/LDS IFFT, normalisation, guard interval, P1.
//                Reference: lib/framemapperfint_cc_impl.cc:1999-2142,
//                           lib/pilotgenp1insert_cc_impl.cc:2784-2907.
// No MFMA: these are bitwise / permutation / complex-FFT paths.
#include "t2_kernels.h"

namespace t2 {

// ============================================================================ helpers
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmulf(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

__device__ __forceinline__ uint32_t rd_lane_u32(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t rd_lane_u64(uint64_t v, int l) {
  uint32_t lo = rd_lane_u32((uint32_t)v, l), hi = rd_lane_u32((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// ============================================================================ FEC kernel
constexpr int FEC_THREADS = 256;
constexpr int FEC_FRAME_BYTES = 6752;   // >= max nbch/8 (6750)
constexpr int FEC_MAX_GROUPS = 150;     // nbch / 360 (5/6 normal)
constexpr int FEC_MAX_Q = 90;
constexpr int FEC_MAX_ENT = 656;
// dynamic LDS carve (bytes)
constexpr int SM_FRAME = 0;
constexpr int SM_CRC8 = SM_FRAME + FEC_FRAME_BYTES;          // 256
constexpr int SM_CRCSH = SM_CRC8 + 256;                      // 2048
constexpr int SM_SYNC = SM_CRCSH + 2048;                     // 64
constexpr int SM_BTAB = SM_SYNC + 64;                        // 256*3*8 = 6144
constexpr int SM_WACC = SM_BTAB + 6144;                      // 4*3*8 = 96
constexpr int SM_D = SM_WACC + 96;                           // 150*24*4 = 14400
constexpr int SM_ROWA = SM_D + FEC_MAX_GROUPS * 24 * 4;      // 90*12*4 = 4320
constexpr int SM_ROWB = SM_ROWA + FEC_MAX_Q * 12 * 4;
constexpr int SM_W = SM_ROWB + FEC_MAX_Q * 12 * 4;           // 16*4
constexpr int SM_ENT = SM_W + 64;                            // 656*4
constexpr int SM_RP = SM_ENT + FEC_MAX_ENT * 4;              // 96*2
constexpr int FEC_SMEM = SM_RP + 96 * 2;
static_assert(SM_BTAB % 16 == 0 && SM_D % 16 == 0 && SM_ENT % 16 == 0, "LDS carve alignment");

// stream position of payload byte J (counted over the payload bytes of the whole stream)
__device__ __forceinline__ int64_t payload_pos(int64_t J, int hem) {
  return hem ? 188 * (J / 187) + 1 + (J % 187) : J;
}

__device__ __forceinline__ uint8_t get_byte192(const uint64_t w[3], int lowbit) {
  // 8 bits [lowbit, lowbit+8) of a 192-bit value; lowbit multiple of 8
  return (uint8_t)(w[lowbit >> 6] >> (lowbit & 63));
}

template <int MODE>
__global__ __launch_bounds__(FEC_THREADS) void fec_kernel(FecDev d, FecIO io) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t B = io.first_block + blockIdx.x;
  const int L = d.kbch >> 3;           // BBFRAME bytes
  const int NB = d.nbch >> 3;          // info bytes (BBFRAME + BCH parity)
  const int P = d.P;
  uint8_t *frame = smem + SM_FRAME;
  uint8_t *crc8 = smem + SM_CRC8;
  uint8_t *crcsh = smem + SM_CRCSH;
  uint8_t *syncv = smem + SM_SYNC;
  uint64_t *btab = (uint64_t *)(smem + SM_BTAB);
  uint64_t *wacc = (uint64_t *)(smem + SM_WACC);
  uint32_t *D = (uint32_t *)(smem + SM_D);
  uint32_t *rowA = (uint32_t *)(smem + SM_ROWA);
  uint32_t *rowB = (uint32_t *)(smem + SM_ROWB);
  uint32_t *Wv = (uint32_t *)(smem + SM_W);
  uint32_t *ents = (uint32_t *)(smem + SM_ENT);
  uint16_t *rp = (uint16_t *)(smem + SM_RP);

  // ---- stage constant tables into LDS
  for (int i = tid; i < 768; i += FEC_THREADS) btab[i] = d.bch_tab[i];
  for (int i = tid; i < d.nent; i += FEC_THREADS) ents[i] = d.ldpc_ent[i];
  for (int i = tid; i <= d.q; i += FEC_THREADS) rp[i] = d.ldpc_rowptr[i];

  if (MODE == FEC_BITS_TO_BITS) {
    // pack nbch unpacked info bits
    const uint8_t *src = io.in + (int64_t)blockIdx.x * d.nbch;
    for (int k = tid; k < NB; k += FEC_THREADS) {
      uint32_t v = 0;
      for (int e = 0; e < 8; e++) v |= (uint32_t)(src[8 * k + e] & 1) << (7 - e);
      frame[k] = (uint8_t)v;
    }
    __syncthreads();
  } else {
    for (int i = tid; i < 256; i += FEC_THREADS) crc8[i] = d.crc8_tab[i];
    for (int i = tid; i < 2048; i += FEC_THREADS) crcsh[i] = d.crc8_shift[i];
    // ---- block geometry (closed form in the absolute block index B; reference keeps
    //      count / crc / fec_block as running state, bbheader:661-734)
    const int pay_full = (d.kbch - 80) >> 3;
    int64_t npad_before = 0;
    int padding = 0;
    if (d.inband) {
      npad_before = (B + d.fec_blocks - 1) / d.fec_blocks;
      padding = (B % d.fec_blocks) == 0 ? 104 : 0;
    }
    const int npay = (d.kbch - 80 - padding) >> 3;
    const int64_t J0 = B * pay_full - 13 * npad_before;
    const int64_t pos0 = payload_pos(J0, d.hem);
    int count0;   // TS packet position of the next input byte at block start
    if (d.hem) count0 = J0 == 0 ? 0 : (int)((payload_pos(J0 - 1, 1) + 1) % 188);
    else count0 = (int)(pos0 % 188);
    __syncthreads();
    // ---- CRC-8 of each packet whose sync slot falls in this block (NM only):
    //      8 lanes per packet, 24-byte chunks combined with zero-extension tables
    if (!d.hem) {
      const int first_slot = (188 - count0) % 188;
      const int nslots = first_slot < npay ? (npay - 1 - first_slot) / 188 + 1 : 0;
      const int m = tid >> 3, k = tid & 7;
      uint8_t part = 0;
      int64_t p = pos0 + first_slot + 188 * (int64_t)m;   // sync position
      bool active = m < nslots && p > 0;
      if (active) {
        int64_t b0 = p - 187 + 24 * k - io.ts_base;
        int n = min(24, 187 - 24 * k);
        uint8_t c = 0;
        for (int i = 0; i < n; i++) c = crc8[io.in[b0 + i] ^ c];
        part = crcsh[k * 256 + c];
      }
      uint32_t v = part;
      v ^= __shfl_xor(v, 1);
      v ^= __shfl_xor(v, 2);
      v ^= __shfl_xor(v, 4);
      if (k == 0 && m < nslots) syncv[m] = active ? (uint8_t)v : 0;
      __syncthreads();
      for (int j = tid; j < npay; j += FEC_THREADS) {
        int64_t pos = pos0 + j;
        int r = (int)((count0 + j) % 188);
        frame[10 + j] = r == 0 ? syncv[(j - first_slot) / 188] : io.in[pos - io.ts_base];
      }
    } else {
      for (int j = tid; j < npay; j += FEC_THREADS) frame[10 + j] = io.in[payload_pos(J0 + j, 1) - io.ts_base];
    }
    if (tid == 0) {
      // BBHEADER (bbheader:272-325): MATYPE-1 = TS, SIS, CCM, ISSYI 0, NPD 0, RO 0; ISI 0
      uint8_t h[10];
      h[0] = 0xF0;
      h[1] = 0x00;
      int upl = d.hem ? 0 : 188 * 8, dfl = d.kbch - 80 - padding, sync = d.hem ? 0 : 0x47;
      int syncd = count0 == 0 ? 0 : (188 - count0) * 8;
      h[2] = (uint8_t)(upl >> 8); h[3] = (uint8_t)upl;
      h[4] = (uint8_t)(dfl >> 8); h[5] = (uint8_t)dfl;
      h[6] = (uint8_t)sync;
      h[7] = (uint8_t)(syncd >> 8); h[8] = (uint8_t)syncd;
      // CRC-8 over the 72 header bits, LSB-first register with 0xAB (add_crc8_bits :247-270)
      uint32_t crc = 0;
      for (int n = 0; n < 72; n++) {
        uint32_t b = ((h[n >> 3] >> (7 - (n & 7))) & 1) ^ (crc & 1);
        crc >>= 1;
        if (b) crc ^= 0xAB;
      }
      if (d.hem) crc ^= 0x80;
      uint32_t rev = 0;   // bits written LSB of the register first
      for (int n = 0; n < 8; n++) rev |= ((crc >> n) & 1) << (7 - n);
      h[9] = (uint8_t)rev;
      for (int i = 0; i < 10; i++) frame[i] = h[i];
      if (padding) {
        // in-band type B (bbheader:327-355): 01, 65 zero bits, TS rate (27 bits), 10 zeros
        uint8_t ib[13] = {0x40, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int n = 0; n < 27; n++)
          if ((d.ts_rate >> (26 - n)) & 1) {
            int bit = 67 + n;
            ib[bit >> 3] |= 1 << (7 - (bit & 7));
          }
        for (int i = 0; i < 13; i++) frame[10 + npay + i] = ib[i];
      }
    }
    __syncthreads();
    for (int i = tid; i < L; i += FEC_THREADS) frame[i] ^= d.prbs[i];   // BB scrambling
    __syncthreads();

    // ---- BCH: lane t divides its chunk; Horner across lanes then waves
    {
      const int C = d.chunk;
      const int lo = L - (FEC_THREADS - tid) * C, hi = L - (FEC_THREADS - 1 - tid) * C;
      const int tw = (P - 8) >> 6, tsft = (P - 8) & 63;
      uint64_t r0 = 0, r1 = 0, r2 = 0;
      for (int i = max(lo, 0); i < hi; i++) {
        uint32_t top = (uint32_t)(((tw == 0 ? r0 : tw == 1 ? r1 : r2) >> tsft) & 0xFF);
        uint32_t idx = top ^ frame[i];
        r2 = (r2 << 8) | (r1 >> 56);
        r1 = (r1 << 8) | (r0 >> 56);
        r0 <<= 8;
        if (P < 192) {
          if (P <= 128) { r2 = 0; if (P < 128) r1 &= (1ull << (P - 64)) - 1; }
          else r2 &= (1ull << (P - 128)) - 1;
        }
        r0 ^= btab[idx * 3 + 0];
        r1 ^= btab[idx * 3 + 1];
        r2 ^= btab[idx * 3 + 2];
      }
      // per-lane rows of M1 (v -> v x^(8C)) and M2 (v -> v x^(8*64*C))
      uint64_t m1[3][3], m2[3][3];
      for (int s = 0; s < 3; s++)
        for (int k = 0; k < 3; k++) {
          m1[s][k] = d.bch_m1[(lane + 64 * s) * 3 + k];
          m2[s][k] = d.bch_m2[(lane + 64 * s) * 3 + k];
        }
      uint64_t a0 = rd_lane_u64(r0, 0), a1 = rd_lane_u64(r1, 0), a2 = rd_lane_u64(r2, 0);
      for (int l = 1; l < 64; l++) {
        uint64_t n0 = __ballot(__popcll((m1[0][0] & a0) ^ (m1[0][1] & a1) ^ (m1[0][2] & a2)) & 1);
        uint64_t n1 = __ballot(__popcll((m1[1][0] & a0) ^ (m1[1][1] & a1) ^ (m1[1][2] & a2)) & 1);
        uint64_t n2 = __ballot(__popcll((m1[2][0] & a0) ^ (m1[2][1] & a1) ^ (m1[2][2] & a2)) & 1);
        a0 = n0 ^ rd_lane_u64(r0, l);
        a1 = n1 ^ rd_lane_u64(r1, l);
        a2 = n2 ^ rd_lane_u64(r2, l);
      }
      if (lane == 0) { wacc[wave * 3 + 0] = a0; wacc[wave * 3 + 1] = a1; wacc[wave * 3 + 2] = a2; }
      __syncthreads();
      if (wave == 0) {
        a0 = wacc[0]; a1 = wacc[1]; a2 = wacc[2];
        for (int w = 1; w < 4; w++) {
          uint64_t n0 = __ballot(__popcll((m2[0][0] & a0) ^ (m2[0][1] & a1) ^ (m2[0][2] & a2)) & 1);
          uint64_t n1 = __ballot(__popcll((m2[1][0] & a0) ^ (m2[1][1] & a1) ^ (m2[1][2] & a2)) & 1);
          uint64_t n2 = __ballot(__popcll((m2[2][0] & a0) ^ (m2[2][1] & a1) ^ (m2[2][2] & a2)) & 1);
          a0 = n0 ^ wacc[w * 3 + 0];
          a1 = n1 ^ wacc[w * 3 + 1];
          a2 = n2 ^ wacc[w * 3 + 2];
        }
        // parity bits MSB (x^(P-1)) first, appended after the BBFRAME
        uint64_t acc[3] = {a0, a1, a2};
        for (int k = lane; k < P / 8; k += 64) frame[L + k] = get_byte192(acc, P - 8 - 8 * k);
      }
      __syncthreads();
    }
    if (MODE == FEC_TS_TO_BITS) {
      uint8_t *dst = io.out + (int64_t)blockIdx.x * d.nbch;
      for (int i = tid; i < d.nbch; i += FEC_THREADS) dst[i] = (frame[i >> 3] >> (7 - (i & 7))) & 1;
      return;
    }
  }

  // ---- LDPC.  Doubled info groups: D[g][k] = big-endian word k of d_g || d_g || d_g[0..47]
  const int ngroups = d.nbch / 360;
  for (int it = tid; it < ngroups * 24; it += FEC_THREADS) {
    int g = it / 24, k = it - g * 24;
    const uint8_t *gb = frame + 45 * g;
    int b = 4 * k;
    uint32_t w = ((uint32_t)gb[b % 45] << 24) | ((uint32_t)gb[(b + 1) % 45] << 16) |
                 ((uint32_t)gb[(b + 2) % 45] << 8) | (uint32_t)gb[(b + 3) % 45];
    D[it] = w;
  }
  __syncthreads();
  // row a, word w of p[a][c] = XOR over entries (g, b) of d_g[(c - b) mod 360]
  const int q = d.q;
  for (int it = tid; it < q * 12; it += FEC_THREADS) {
    int a = it / 12, w = it - a * 12;
    uint32_t acc = 0;
    for (int e = rp[a]; e < rp[a + 1]; e++) {
      uint32_t ent = ents[e];
      int g = ent >> 16, b = ent & 0xFFFF;
      int o = 32 * w + 360 - b;
      const uint32_t *dg = D + g * 24 + (o >> 5);
      uint64_t win = ((uint64_t)dg[0] << 32) | dg[1];
      acc ^= (uint32_t)(win >> (32 - (o & 31)));
    }
    if (w == 11) acc &= 0xFF000000u;
    rowA[it] = acc;
  }
  __syncthreads();
  // inclusive prefix XOR over rows a (Hillis-Steele)
  uint32_t *cur = rowA, *nxt = rowB;
  for (int dd = 1; dd < q; dd <<= 1) {
    for (int it = tid; it < q * 12; it += FEC_THREADS) {
      int a = it / 12;
      uint32_t v = cur[it];
      if (a >= dd) v ^= cur[it - 12 * dd];
      nxt[it] = v;
    }
    __syncthreads();
    uint32_t *t = cur; cur = nxt; nxt = t;
  }
  // exclusive bit-prefix XOR of the last row (the column parities) along c
  if (tid == 0) {
    uint32_t carry = 0;
    for (int w = 0; w < 12; w++) {
      uint32_t x = cur[(q - 1) * 12 + w];
      uint32_t y = x;
      y ^= y >> 1; y ^= y >> 2; y ^= y >> 4; y ^= y >> 8; y ^= y >> 16;
      uint32_t ex = y ^ x;
      if (carry) ex = ~ex;
      Wv[w] = ex;
      carry ^= y & 1;
    }
    Wv[11] &= 0xFF000000u;
  }
  __syncthreads();
  for (int it = tid; it < q * 12; it += FEC_THREADS) cur[it] ^= Wv[it % 12];
  __syncthreads();
  // parity bit of row a (interleaved position 360 a + c) / natural index a + q c
  auto pbit = [&](int a, int c) -> uint32_t { return (cur[a * 12 + (c >> 5)] >> (31 - (c & 31))) & 1; };

  if (MODE == FEC_BITS_TO_BITS) {
    uint8_t *dst = io.out + (int64_t)blockIdx.x * d.nldpc;
    for (int i = tid; i < d.nbch; i += FEC_THREADS) dst[i] = (frame[i >> 3] >> (7 - (i & 7))) & 1;
    const int pbits = d.nldpc - d.nbch;
    for (int j = tid; j < pbits; j += FEC_THREADS) dst[d.nbch + j] = (uint8_t)pbit(j % q, j / q);
    return;
  }
  // FEC_TS_TO_TEMPU: assemble the interleaver input bytes in LDS (over D), store as words
  uint8_t *stage = (uint8_t *)D;
  const int cwb = d.nldpc >> 3, pb = cwb - NB;
  for (int i = tid; i < NB; i += FEC_THREADS) stage[i] = frame[i];
  if (d.parity_il) {
    for (int i = tid; i < pb; i += FEC_THREADS) {
      int a = i / 45, k = i - 45 * a;
      stage[NB + i] = (uint8_t)(cur[a * 12 + (k >> 2)] >> (24 - 8 * (k & 3)));
    }
  } else {
    for (int i = tid; i < pb; i += FEC_THREADS) {
      uint32_t v = 0;
      for (int e = 0; e < 8; e++) {
        int j = 8 * i + e;
        v |= pbit(j % q, j / q) << (7 - e);
      }
      stage[NB + i] = (uint8_t)v;
    }
  }
  __syncthreads();
  uint32_t *dstw = (uint32_t *)(io.out + (int64_t)blockIdx.x * io.cw_stride);
  const uint32_t *srcw = (const uint32_t *)stage;
  for (int i = tid; i < cwb / 4 + (cwb & 3 ? 1 : 0); i += FEC_THREADS) dstw[i] = srcw[i];
}

hipError_t launch_fec(int mode, const FecDev &d, const FecIO &io, hipStream_t s) {
  if (io.nblocks <= 0) return hipSuccess;
  dim3 grid(io.nblocks), block(FEC_THREADS);
  switch (mode) {
    case FEC_TS_TO_TEMPU: hipLaunchKernelGGL(fec_kernel<FEC_TS_TO_TEMPU>, grid, block, FEC_SMEM, s, d, io); break;
    case FEC_TS_TO_BITS: hipLaunchKernelGGL(fec_kernel<FEC_TS_TO_BITS>, grid, block, FEC_SMEM, s, d, io); break;
    default: hipLaunchKernelGGL(fec_kernel<FEC_BITS_TO_BITS>, grid, block, FEC_SMEM, s, d, io); break;
  }
  return hipGetLastError();
}

// ============================================================================ map kernel
constexpr int MAP_THREADS = 512;
constexpr int MAP_LDS_MAX = 160 * 1024;
// LDS: [LUT 2 KB][cell indices, cs bytes][codeword bytes | cell-interleave staging (8 cs)]
__host__ __device__ inline int map_idx_bytes(int cs) { return (cs + 15) & ~15; }
__host__ __device__ inline bool map_stage_in_lds(int cs) { return 2048 + map_idx_bytes(cs) + 8 * cs <= MAP_LDS_MAX; }
__host__ __device__ inline int map_smem(int cs, int cw_bytes, int apply_ci) {
  int region = cw_bytes;
  if (apply_ci && map_stage_in_lds(cs) && 8 * cs > region) region = 8 * cs;
  return 2048 + map_idx_bytes(cs) + ((region + 15) & ~15);
}

__global__ __launch_bounds__(MAP_THREADS) void map_kernel(MapDev d, MapIO io) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int blk = blockIdx.x;
  float2 *lut = (float2 *)smem;
  uint8_t *idx = smem + 2048;
  uint8_t *cw = smem + 2048 + map_idx_bytes(d.cs);
  float2 *stage = (float2 *)cw;
  const bool lds_stage = map_stage_in_lds(d.cs);
  const int cs = d.cs, nl = d.nldpc;
  for (int i = tid; i < 256; i += MAP_THREADS) lut[i] = d.lut[i];
  // ---- interleaver input bits (tempu) into LDS
  if (io.packed_in) {
    const uint32_t *src = (const uint32_t *)(io.in + (int64_t)blk * io.cw_stride);
    uint32_t *dst = (uint32_t *)cw;
    for (int i = tid; i < nl / 32; i += MAP_THREADS) dst[i] = src[i];
    if ((nl & 31) && tid == 0) dst[nl / 32] = src[nl / 32];
  } else {
    const uint8_t *src = io.in + (int64_t)blk * nl;
    const int nbch = d.nbch, q = d.q;
    for (int k = tid; k < nl / 8; k += MAP_THREADS) {
      uint32_t v = 0;
      for (int e = 0; e < 8; e++) {
        int i = 8 * k + e, sidx = i;
        if (d.parity_il && i >= nbch) {        // tempu[nbch + 360 t + s] = in[nbch + q s + t]
          int r = i - nbch, t = r / 360, s = r - 360 * t;
          sidx = nbch + q * s + t;
        }
        v |= (uint32_t)(src[sidx] & 1) << (7 - e);
      }
      cw[k] = (uint8_t)v;
    }
  }
  __syncthreads();
  auto bit = [&](int i) -> uint32_t { return (cw[i >> 3] >> (7 - (i & 7))) & 1; };
  // ---- cell indices: column-twist write / row read / demux (interleavermod:351-403 ...)
  if (d.mode == 0) {
    for (int j = tid; j < cs; j += MAP_THREADS) idx[j] = (uint8_t)((bit(2 * j) << 1) | bit(2 * j + 1));
  } else {
    const int W = d.W, R = d.R, mod = d.mod;
    for (int j = tid; j < R; j += MAP_THREADS) {
      uint32_t pack = 0;
      for (int e = 0; e < W; e++) {
        int r = j - d.twist[e];
        r += r < 0 ? R : 0;
        pack |= bit(e * R + r) << (W - 1 - d.mux[e]);
      }
      if (d.mode == 1) {
        idx[2 * j] = (uint8_t)(pack >> mod);
        idx[2 * j + 1] = (uint8_t)(pack & ((1u << mod) - 1));
      } else {
        idx[j] = (uint8_t)(pack & 0xFF);
      }
    }
  }
  __syncthreads();
  // ---- constellation + cyclic Q delay; optional cell interleaver via LDS
  const int r_in_frame = blk % d.F;
  const int shift = io.apply_ci ? d.ci_shift[r_in_frame] : 0;
  float2 *dst = io.out + (int64_t)blk * cs;
  for (int j = tid; j < cs; j += MAP_THREADS) {
    float2 v = lut[idx[j]];
    if (d.rotation) v.y = lut[idx[j == 0 ? cs - 1 : j - 1]].y;
    if (io.apply_ci) {
      int t = d.ci_perm[j] + shift;
      t -= t >= cs ? cs : 0;
      if (lds_stage) stage[t] = v;
      else dst[t] = v;   // QPSK normal: 259 KB of cells do not fit LDS, scatter directly
    } else {
      dst[j] = v;
    }
  }
  if (io.apply_ci && lds_stage) {
    __syncthreads();
    for (int j = tid; j < cs; j += MAP_THREADS) dst[j] = stage[j];
  }
}

hipError_t launch_map(const MapDev &d, const MapIO &io, hipStream_t s) {
  if (io.nblocks <= 0) return hipSuccess;
  int smem = map_smem(d.cs, d.nldpc / 8 + 4, io.apply_ci);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void *)map_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, MAP_LDS_MAX);
    attr_set = true;
  }
  hipLaunchKernelGGL(map_kernel, dim3(io.nblocks), dim3(MAP_THREADS), smem, s, d, io);
  return hipGetLastError();
}

// ============================================================================ OFDM kernel
// exp(+2 pi i k / 32): exact at multiples of pi/2
__device__ constexpr float kCos32[32] = {
    1.0f, 0.98078528040323043f, 0.92387953251128674f, 0.83146961230254524f, 0.70710678118654757f,
    0.55557023301960218f, 0.38268343236508978f, 0.19509032201612828f, 0.0f, -0.19509032201612828f,
    -0.38268343236508978f, -0.55557023301960218f, -0.70710678118654757f, -0.83146961230254524f,
    -0.92387953251128674f, -0.98078528040323043f, -1.0f, -0.98078528040323043f, -0.92387953251128674f,
    -0.83146961230254524f, -0.70710678118654757f, -0.55557023301960218f, -0.38268343236508978f,
    -0.19509032201612828f, 0.0f, 0.19509032201612828f, 0.38268343236508978f, 0.55557023301960218f,
    0.70710678118654757f, 0.83146961230254524f, 0.92387953251128674f, 0.98078528040323043f};
__device__ constexpr float kSin32[32] = {
    0.0f, 0.19509032201612828f, 0.38268343236508978f, 0.55557023301960218f, 0.70710678118654757f,
    0.83146961230254524f, 0.92387953251128674f, 0.98078528040323043f, 1.0f, 0.98078528040323043f,
    0.92387953251128674f, 0.83146961230254524f, 0.70710678118654757f, 0.55557023301960218f,
    0.38268343236508978f, 0.19509032201612828f, 0.0f, -0.19509032201612828f, -0.38268343236508978f,
    -0.55557023301960218f, -0.70710678118654757f, -0.83146961230254524f, -0.92387953251128674f,
    -0.98078528040323043f, -1.0f, -0.98078528040323043f, -0.92387953251128674f, -0.83146961230254524f,
    -0.70710678118654757f, -0.55557023301960218f, -0.38268343236508978f, -0.19509032201612828f};

// in-register inverse DFT of size R (natural order in and out), radix-2 recursion
template <int R, int STRIDE = 1>
struct Dft {
  __device__ __forceinline__ static void run(float2 *x) {
    float2 e[R / 2], o[R / 2];
#pragma unroll
    for (int i = 0; i < R / 2; i++) { e[i] = x[2 * i]; o[i] = x[2 * i + 1]; }
    Dft<R / 2>::run(e);
    Dft<R / 2>::run(o);
#pragma unroll
    for (int k = 0; k < R / 2; k++) {
      float2 t;
      constexpr int sc = 32 / R;
      if (k == 0) t = o[k];
      else if (4 * k == R) t = make_float2(-o[k].y, o[k].x);          // * i
      else t = cmulf(o[k], make_float2(kCos32[k * sc], kSin32[k * sc]));
      x[k] = cadd(e[k], t);
      x[k + R / 2] = csub(e[k], t);
    }
  }
};
template <int STRIDE>
struct Dft<1, STRIDE> {
  __device__ __forceinline__ static void run(float2 *) {}
};

// N = R1 * R2 * R3; LDS exchange through padded float arrays (re, then im)
template <int R1, int R2, int R3>
struct FftGeom {
  static constexpr int N = R1 * R2 * R3, N2 = R2 * R3;
  static constexpr int U1 = N2, U2 = R1 * R3, U3 = R1 * R2;
  static constexpr int NT = U1 > U2 ? (U1 > U3 ? U1 : U3) : (U2 > U3 ? U2 : U3);
  static constexpr int LDS_FLOATS = N2 * (R1 + 1);
};

template <int R1, int R2, int R3, int NTH>
__global__ __launch_bounds__(NTH) void ofdm_kernel(OfdmDev d, OfdmIO io) {
  using Gm = FftGeom<R1, R2, R3>;
  constexpr int N = Gm::N, N2 = Gm::N2, S1 = R1 + 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float *lds = (float *)smem;
  const int tid = threadIdx.x;
  const int j = blockIdx.x;                       // symbol
  const int f = blockIdx.y;                       // frame within launch
  const int64_t frame = io.first_frame + f;
  const float2 *cells = io.cells + (int64_t)f * io.cell_stride;
  const float2 *aux = d.aux + (int64_t)(frame % d.t2frames) * d.aux_len;
  const int32_t *map = d.bin_map + (int64_t)j * N;

  if (j == 0 && !io.carriers_only) {            // P1 symbol (precomputed), pilotgen:2802-2810
    float2 *p = io.out + (int64_t)f * io.out_stride;
    for (int i = tid; i < 2048; i += Gm::NT) p[i] = d.p1[i];
  }
  // ---- pass 1: gather R1 inputs at stride N2, R1-point DFT, twiddle, -> LDS (k2, n1)
  float2 x[R1 > R2 ? (R1 > R3 ? R1 : R3) : (R2 > R3 ? R2 : R3)];
  const bool act1 = tid < Gm::U1;
  if (act1) {
    const int k2 = tid;
#pragma unroll
    for (int k1 = 0; k1 < R1; k1++) {
      int k = k2 + N2 * k1;
      int code = map[k];
      float2 v = code >= 0 ? cells[code] : aux[-code - 1];
      if (d.isinc) {
        float s = d.isinc[(k + N / 2) & (N - 1)];
        v.x *= s;
        v.y *= s;
      }
      x[k1] = v;
    }
    if (io.carriers_only) {
      float2 *o = io.out + (int64_t)f * io.out_stride + (int64_t)j * N;
#pragma unroll
      for (int k1 = 0; k1 < R1; k1++) {
        int k = k2 + N2 * k1;
        o[(k + N / 2) & (N - 1)] = x[k1];
      }
    }
  }
  if (io.carriers_only) return;
  if (act1) {
    Dft<R1>::run(x);
#pragma unroll
    for (int n1 = 1; n1 < R1; n1++) x[n1] = cmulf(x[n1], d.twiddle[n1 * tid]);
  }
  // exchange helpers: write component c of x[0..R) at base + i*stride, read back likewise
#define T2_XCHG(ACT_W, WADDR, CNT_W, ACT_R, RADDR, CNT_R)                        \
  {                                                                              \
    float2 y[CNT_R];                                                             \
    _Pragma("unroll") for (int comp = 0; comp < 2; comp++) {                     \
      if (ACT_W) {                                                               \
        _Pragma("unroll") for (int i = 0; i < CNT_W; i++) lds[WADDR] = comp ? x[i].y : x[i].x; \
      }                                                                          \
      __syncthreads();                                                           \
      if (ACT_R) {                                                               \
        _Pragma("unroll") for (int i = 0; i < CNT_R; i++) {                      \
          float v = lds[RADDR];                                                  \
          if (comp) y[i].y = v; else y[i].x = v;                                 \
        }                                                                        \
      }                                                                          \
      __syncthreads();                                                           \
    }                                                                            \
    if (ACT_R) {                                                                 \
      _Pragma("unroll") for (int i = 0; i < CNT_R; i++) x[i] = y[i];             \
    }                                                                            \
  }
  // pass 1 -> 2: A[k2][n1] at k2*S1 + n1; unit (n1 = u % R1, a = u / R1) reads k2 = a + R3*b
  const bool act2 = tid < Gm::U2;
  const int n1b = tid % R1, ab = tid / R1;
  T2_XCHG(act1, tid * S1 + i, R1, act2, (ab + R3 * i) * S1 + n1b, R2)
  if (act2) {
    Dft<R2>::run(x);
#pragma unroll
    for (int c = 1; c < R2; c++) x[c] = cmulf(x[c], d.twiddle[R1 * c * ab]);
  }
  // pass 2 -> 3: B[c][a] (n1 innermost) at (c*R3 + a)*S1 + n1; unit (n1, c = u / R1) reads a
  const bool act3 = tid < Gm::U3;
  const int cc = tid / R1;
  T2_XCHG(act2, (i * R3 + ab) * S1 + n1b, R2, act3, (cc * R3 + i) * S1 + n1b, R3)
#undef T2_XCHG
  if (!act3) return;
  Dft<R3>::run(x);
  // ---- output: x[n1 + R1*(c + R2*d)] = x[tid + U3*d]; GI = last G samples first
  const int G = d.G;
  float2 *o = io.out + (int64_t)f * io.out_stride + 2048 + (int64_t)j * (N + G);
  const float nrm = d.norm;
#pragma unroll
  for (int dd = 0; dd < R3; dd++) {
    int n = tid + Gm::U3 * dd;
    float2 v = make_float2(x[dd].x * nrm, x[dd].y * nrm);
    o[G + n] = v;
    if (n >= N - G) o[n - (N - G)] = v;
  }
}

template <int R1, int R2, int R3>
static hipError_t launch_ofdm_t(const OfdmDev &d, const OfdmIO &io, hipStream_t s) {
  using Gm = FftGeom<R1, R2, R3>;
  size_t smem = sizeof(float) * Gm::LDS_FLOATS;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void *)ofdm_kernel<R1, R2, R3, Gm::NT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr_set = true;
  }
  hipLaunchKernelGGL((ofdm_kernel<R1, R2, R3, Gm::NT>), dim3(d.Nsym, io.nframes), dim3(Gm::NT), smem, s, d, io);
  return hipGetLastError();
}

hipError_t launch_ofdm(const OfdmDev &d, const OfdmIO &io, hipStream_t s) {
  if (io.nframes <= 0) return hipSuccess;
  switch (d.N) {
    case 1024: return launch_ofdm_t<8, 8, 16>(d, io, s);
    case 2048: return launch_ofdm_t<8, 16, 16>(d, io, s);
    case 4096: return launch_ofdm_t<16, 16, 16>(d, io, s);
    case 8192: return launch_ofdm_t<16, 16, 32>(d, io, s);
    case 16384: return launch_ofdm_t<16, 32, 32>(d, io, s);
    case 32768: return launch_ofdm_t<32, 32, 32>(d, io, s);
    default: return hipErrorInvalidValue;
  }
}

// ============================================================================ gather
__global__ __launch_bounds__(256) void gather_kernel(GatherIO io) {
  int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= io.M) return;
  int code = io.map[i];
  io.out[i] = code >= 0 ? io.in[code] : io.aux[-code - 1];
}

hipError_t launch_gather(const GatherIO &io, hipStream_t s) {
  if (io.M <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_kernel, dim3((io.M + 255) / 256), dim3(256), 0, s, io);
  return hipGetLastError();
}

}  // namespace t2
