// t2_kernels.hip -- gfx950 (MI355X / CDNA4) kernels of the DVB-T2 transmit chain.
//
//   fec_kernel   persistent 256-thread workgroups looping over FEC blocks: BBFRAME build
//                (header, CRC-8 sync replacement, scrambling) + BCH (64-lane chunked byte-table
//                division, chunk remainders moved by per-lane nibble tables) + LDPC as a
//                quasi-cyclic array of 360-bit rotations with a bit-packed accumulate scan.
//                Reference: lib/bbheaderbch_bb_impl.cc:648-742 (+ ldpc_calculate :625-646).
//   chain FEC     bbch_kernel (BBFRAME from the TS + the BCH as a GF(2) product on the matrix cores),
//                 ldpc_map_kernel (LDPC, then the bit interleaver, cell and time interleaver of the
//                 block's constellation index pairs; extra workgroups generate the L1-post cells).
//                 Reference: bbheaderbch :625-742, lib/interleavermod_bc_impl.cc:270-704,
//                 framemapper :1973-2028.
//   map_kernel   block API: one workgroup per FEC block, column-twist bit interleave + demux + QAM.
//   ofdm*_kernel one workgroup per (OFDM symbol, frame): bins scattered (chain) or gathered
//                (pilotgen block) into a register/LDS IFFT, normalisation, output gain, guard
//                interval, P1.  Reference: lib/framemapperfint_cc_impl.cc:1999-2142,
//                lib/pilotgenp1insert_cc_impl.cc:2784-2907.
// MFMA only for the BCH product: the rest are bitwise / permutation / complex-FFT paths.
#include "t2_kernels.h"

#include <atomic>
#include <mutex>
#include <set>
#include <utility>

namespace t2 {

// ============================================================================ helpers
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
typedef float f2v __attribute__((ext_vector_type(2)));
// complex product as two packed-FP32 ops: t = (ax bx, ax by); (ay (-by) + t.x, ay bx + t.y)
// (operand swizzles and the negation ride on op_sel / neg_lo instead of extra moves)
__device__ __forceinline__ float2 cmulf(float2 a, float2 b) {
  const f2v av = {a.x, a.y}, bv = {b.x, b.y};
  f2v t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(av), "v"(bv));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(av), "v"(bv), "v"(t));
  return make_float2(r.x, r.y);
}
// a + i b and a - i b as one packed add each (b's halves swapped and one negated by op_sel /
// neg_lo / neg_hi); a * s for a real s as one packed multiply
__device__ __forceinline__ float2 cadd_i(float2 a, float2 b) {
  const f2v av = {a.x, a.y}, bv = {b.x, b.y};
  f2v r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(av), "v"(bv));
  return make_float2(r.x, r.y);
}
__device__ __forceinline__ float2 csub_i(float2 a, float2 b) {
  const f2v av = {a.x, a.y}, bv = {b.x, b.y};
  f2v r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(av), "v"(bv));
  return make_float2(r.x, r.y);
}
__device__ __forceinline__ float2 cscale(float2 a, float sc) {
  const f2v r = f2v{a.x, a.y} * f2v{sc, sc};
  return make_float2(r.x, r.y);
}

// a read-only table entry at a wave-uniform index through the constant address space: a scalar (SMEM)
// load, counted by lgkmcnt, so its wait never waits for the wave's outstanding vector stores (vmcnt
// retires loads and stores in order).  Only for tables the host writes before the launch.
template <class T>
__device__ __forceinline__ T kc(const T *p, int64_t i) {
  static_assert(sizeof(T) % 4 == 0, "whole dwords");
  const __attribute__((address_space(4))) uint32_t *q = (const __attribute__((address_space(4))) uint32_t *)(p + i);
  uint32_t w[sizeof(T) / 4];
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); k++) w[k] = q[k];
  T r;
  __builtin_memcpy(&r, w, sizeof(T));
  return r;
}

// uniform (SGPR) base + 32-bit unsigned byte offset: lets the compiler use the global
// saddr form (one VGPR per address instead of a 64-bit VGPR pair per element)
template <class T>
__device__ __forceinline__ T ld_off(const T *base, uint32_t byte_off) {
  return *(const T *)((const char *)base + byte_off);
}
template <class T>
__device__ __forceinline__ void st_off(T *base, uint32_t byte_off, T v) {
  *(T *)((char *)base + byte_off) = v;
}

// streaming store (nontemporal): final IQ samples are never re-read by the chain
__device__ __forceinline__ void st_nt(float2 *base, uint32_t byte_off, float2 v) {
  float2 *p = (float2 *)((char *)base + byte_off);
  __builtin_nontemporal_store(__builtin_bit_cast(uint64_t, v), (uint64_t *)p);
}

// workgroup barrier that orders LDS accesses only (the OFDM kernels): the fence of __syncthreads also
// covers global memory, and in the OFDM kernels (whose units end in IQ stores) it measured slower
// (session r5s: cfg4 OFDM 1.833 -> 1.775 ms, cfg3 7.655 -> 7.59 ms with this barrier and the scalar
// table loads, kc).  Never for global memory communicated between threads.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ uint32_t rd_lane_u32(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t rd_lane_u64(uint64_t v, int l) {
  uint32_t lo = rd_lane_u32((uint32_t)v, l), hi = rd_lane_u32((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// Raise a kernel's dynamic-LDS limit once per (kernel, device): thread-safe, and repeated for
// every device a process launches on (the attribute belongs to the current device's function).
static hipError_t lds_limit(const void *fn, int bytes) {
  static std::mutex mu;
  static std::set<std::pair<const void *, int>> done;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lock(mu);
  if (done.count({fn, dev})) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done.insert({fn, dev});
  return e;
}

// ============================================================================ FEC kernels
// Block API (bbheaderbch / ldpc blocks): fec_kernel<MODE>, one fused pass per FEC block (BBFRAME,
// BCH on one wave, LDPC).  The chain runs two launches per PLP instead (launch_fec FEC_TS_TO_BBFRAME, then
// launch_ldpc_map):
//   bbch_kernel      TS -> BBFRAME bytes (header, CRC-8 sync replacement, in-band field, BB scrambling)
//                    built in registers and stored into the codeword row, and the BCH parity of every
//                    block as a GF(2) matrix product on the matrix cores on the same pieces (blocks x
//                    message bits x parity bits, fp4 0/1 operands, exact f32 sums, parity = sum & 1),
//                    K split into slices (each XCD's L2 holds its slices' share of the generator
//                    table) whose partial parities are XORed by the LDPC stage
//   ldpc_map_kernel  info bytes + XOR of the partials -> LDPC parity -> interleaver-input codeword in
//                    LDS -> the map (column twist, demux, cell + time interleaver), see below
constexpr int FEC_THREADS = 256;
constexpr int FEC_FRAME_BYTES = 6752;   // >= max nbch/8 (6750)
constexpr int FEC_MAX_ENT = 648;        // max LDPC table entries (3/5 normal: 233280 / 360)
constexpr int FEC_DW = 13;              // LDS words per LDPC info group (fused kernel): d_g || d_g[0..56)
constexpr int FEC_DW_PASS = 16;         // chain LDPC stage: d_g || d_g[0..152), four windows without wrap
constexpr int FEC_WG_PER_CU = 7;        // fused kernel: resident workgroups per CU (72-VGPR budget)
constexpr int FEC_PASS_WG_PER_CU = 8;   // chain BB pass, LDPC + map kernel (64-VGPR budget, 32 waves per CU)
constexpr int FEC_BCH_JB = 2;           // nibble-table lookups in flight per lane in the BCH combine
constexpr int FEC_LDPC_BYTES = 4 * (FEC_DW_PASS * 150 + 12 * 30); // max over codes of 64 ngroups + 48 q

// dynamic LDS carve (bytes) of each FEC kernel kind: persistent tables (staged once; the
// workgroups loop over FEC blocks), then the per-block area, reused by phase:
//   BB phase:   [frame | raw TS bytes | CRC-8 table | CRC-8 zero-extension tables]
//   LDPC phase: [frame | D: ngroups x 13 words | rows: q x 12 words], ngroups + q = nldpc / 360 (<= 180)
// sized for the plan's code, so a launch fits as many workgroups per CU as it allows
enum FecCarveKind { CARVE_FUSED = 0, CARVE_BB = 1, CARVE_LDPC = 2 };
struct FecCarve {
  int btab, ents, hcrc, sync, w, rowp, frame, phase, crc8, crcsh, crcsl, prbs, total;
};
__host__ __device__ inline FecCarve fec_carve(int kind, int kbch, int nbch, int q) {
  FecCarve c{};
  const bool bch = kind == CARVE_FUSED, ldpc = kind != CARVE_BB, bb = kind != CARVE_LDPC;
  int o = 0;
  c.btab = o; o += bch ? 256 * 3 * 8 : 0;
  c.ents = o; o += ldpc ? FEC_MAX_ENT * 4 : 0;
  c.hcrc = o; o += bb ? 80 : 0;            // 72 header-bit CRC contributions
  c.sync = o; o += bb ? 48 : 0;            // <= 36 sync-slot CRC-8s
  c.w = o; o += ldpc ? 48 : 0;             // 12 column-parity words
  c.rowp = o; o += ldpc ? 192 : 0;         // q + 1 <= 91 LDPC row pointers
  // BB pass: T^1 .. T^24 of the CRC-8 byte table T at a compile-time offset (the lookups' addresses are
  // the byte itself plus an immediate), before the code-dependent areas
  c.crcsl = o; o += kind == CARVE_BB ? 24 * 256 : 0;
  c.frame = (o + 15) & ~15;
  c.phase = c.frame + (kind == CARVE_BB ? 0 : ((nbch / 8 + 15) & ~15));   // the BB pass stores its frame to HBM
  c.crc8 = c.phase + ((188 + (kbch - 80) / 8 + 32 + 15) & ~15);   // + slack: 16-byte staging start
  c.crcsh = c.crc8 + 256;
  c.prbs = c.crcsh + 2048;                 // BB pass: the BB-scrambler PRBS words
  const int bb_end = c.prbs + (kind == CARVE_BB ? ((kbch / 8 + 15) & ~15) : 0), ldpc_end = c.phase + 4 * ((kind == CARVE_LDPC ? FEC_DW_PASS : FEC_DW) * (nbch / 360) + 12 * q);
  c.total = kind == CARVE_BB ? bb_end : kind == CARVE_LDPC ? ldpc_end : (bb_end > ldpc_end ? bb_end : ldpc_end);
  return c;
}

// stream position of payload byte J (counted over the payload bytes of the whole stream)
__device__ __forceinline__ int64_t payload_pos(int64_t J, int hem) {
  return hem ? 188 * (J / 187) + 1 + (J % 187) : J;
}

// inclusive prefix XOR over the 64 lanes of a wave with DPP moves (VALU latency, no LDS
// crossbar): row_shr 1, 2, 4, 8 within each 16-lane row, then row_bcast:15 into rows 1 and 3 and
// row_bcast:31 into rows 2 and 3 (GFX9-family DPP)
__device__ __forceinline__ uint32_t wave_prefix_xor(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);   // row_shr:1
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);   // row_shr:2
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);   // row_shr:4
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);   // row_shr:8
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return v;
}

__device__ __forceinline__ uint8_t get_byte192(const uint64_t w[3], int lowbit) {
  // 8 bits [lowbit, lowbit+8) of a 192-bit value; lowbit multiple of 8
  return (uint8_t)(w[lowbit >> 6] >> (lowbit & 63));
}

// word k < DW of LDPC info group g laid out for 32-bit rotation windows: big-endian bytes
// (4k .. 4k+3) mod 45 of the group's 45 frame bytes (d_g || d_g[0..32 DW - 360))
// (words other than 11 are four consecutive frame bytes: two aligned word reads and a byte align;
// word 11 wraps from byte 44 to bytes 0..2)
__device__ __forceinline__ uint32_t ldpc_group_val(const uint8_t *frame, int g, int k) {
  const uint8_t *gb = frame + 45 * g;
  if (k == 11) return ((uint32_t)gb[44] << 24) | ((uint32_t)gb[0] << 16) | ((uint32_t)gb[1] << 8) | (uint32_t)gb[2];
  const int o = 45 * g + (k >= 12 ? 4 * k - 45 : 4 * k);   // frame is 4-byte aligned
  const uint32_t *fw = (const uint32_t *)frame;
  return __builtin_bswap32(__builtin_amdgcn_alignbyte(fw[(o >> 2) + 1], fw[o >> 2], (uint32_t)(o & 3)));
}
template <int DW>
__device__ __forceinline__ void ldpc_group_word(uint32_t *D, const uint8_t *frame, int g, int k) {
  D[g * DW + k] = ldpc_group_val(frame, g, k);
}

// byte-table division of frame[lo, hi) (lo clamped at 0) into the P-bit remainder r; the next message
// byte is read before the table lookup's wait (LDS returns in order, so it costs no extra round trip).
// P is a template parameter so the register geometry (top byte, masks) is compile-time.
template <int P>
__device__ __forceinline__ void bch_divide(const uint8_t *frame, const uint64_t *btab, int lo, int hi, uint64_t &r0,
                                           uint64_t &r1, uint64_t &r2) {
  constexpr int tw = (P - 8) >> 6, tsft = (P - 8) & 63;
  constexpr uint64_t k1 = P >= 128 ? ~0ull : (1ull << ((P - 64) & 63)) - 1;
  constexpr uint64_t k2 = P >= 192 ? ~0ull : P <= 128 ? 0ull : (1ull << ((P - 128) & 63)) - 1;
  int i = max(lo, 0);
  uint32_t nxt = i < hi ? frame[i] : 0u;
#pragma unroll 2
  for (; i < hi; i++) {
    const uint32_t cur = nxt;
    if (i + 1 < hi) nxt = frame[i + 1];
    const uint32_t top = (uint32_t)(((tw == 0 ? r0 : tw == 1 ? r1 : r2) >> tsft) & 0xFF);
    const uint32_t idx = top ^ cur;
    r2 = ((r2 << 8) | (r1 >> 56)) & k2;
    r1 = ((r1 << 8) | (r0 >> 56)) & k1;
    r0 <<= 8;
    r0 ^= btab[idx * 3 + 0];
    r1 ^= btab[idx * 3 + 1];
    r2 ^= btab[idx * 3 + 2];
  }
}

__device__ __forceinline__ uint64_t wave_xor64(uint64_t x) {
  const uint32_t lo = rd_lane_u32(wave_prefix_xor((uint32_t)x), 63);
  const uint32_t hi = rd_lane_u32(wave_prefix_xor((uint32_t)(x >> 32)), 63);
  return ((uint64_t)hi << 32) | lo;
}

// BCH parity of the BBFRAME frame[0..L) by one wave (bbheader:504-531): lane l divides chunk l of the
// 64 chunks of C bytes (t2_plan: bch_chunk; the chunks end at L, leading ones may be empty) by the
// byte table, then moves its remainder to the end of the message, r_l x^(8C (63 - l)) mod g, by
// per-lane nibble-table lookups (no dependency between lanes), and the wave XOR-reduces them.
// Returns the P-bit parity (uniform).
template <int P>
__device__ __forceinline__ void bch_wave(const uint8_t *frame, const uint64_t *btab, const uint64_t *ctab, int L,
                                         int C, int lane, uint64_t a[3]) {
  const int lo = L - (64 - lane) * C, hi = L - (63 - lane) * C;
  uint64_t r0 = 0, r1 = 0, r2 = 0;
  bch_divide<P>(frame, btab, lo, hi, r0, r1, r2);
  constexpr int NJ = P / 4, JB = FEC_BCH_JB;
  uint64_t s0 = 0, s1 = 0, s2 = 0;
#pragma unroll 1
  for (int j0 = 0; j0 < NJ; j0 += JB) {
    uint4 e01[JB];
    uint2 e2[JB];
#pragma unroll
    for (int u = 0; u < JB; u++) {
      const int j = j0 + u;
      if (j < NJ) {
        const uint64_t rw = j < 16 ? r0 : j < 32 ? r1 : r2;
        const uint32_t v = (uint32_t)(rw >> (4 * (j & 15))) & 15u;
        const uint32_t off = (((uint32_t)j * 16u + v) * 64u + (uint32_t)lane) * 32u;
        e01[u] = ld_off((const uint4 *)ctab, off);
        e2[u] = ld_off((const uint2 *)ctab, off + 16u);
      }
    }
#pragma unroll
    for (int u = 0; u < JB; u++) {
      if (j0 + u < NJ) {
        s0 ^= ((uint64_t)e01[u].y << 32) | e01[u].x;
        s1 ^= ((uint64_t)e01[u].w << 32) | e01[u].z;
        s2 ^= ((uint64_t)e2[u].y << 32) | e2[u].x;
      }
    }
  }
  a[0] = wave_xor64(s0);
  a[1] = wave_xor64(s1);
  a[2] = P > 128 ? wave_xor64(s2) : 0ull;
}

// LDPC parity rows: row a, word w of p[a][c] = XOR over the row's entries (g, b) of the window
// d_g[(c - b) mod 360], c = 32 w; 12 words per row at rowA.  One item = (row, 4 words): each entry is
// read once for its four windows (3 q items, one round of the workgroup for q <= 85)
__device__ __forceinline__ uint32_t ldpc_window(const uint32_t *dg, int o) {   // d_g bits [o, o + 32)
  const uint64_t win = ((uint64_t)dg[o >> 5] << 32) | dg[(o >> 5) + 1];
  return (uint32_t)(win >> (32 - (o & 31)));
}
template <int DW>
__device__ __forceinline__ void ldpc_rows(const uint32_t *D, uint32_t *rowA, const uint32_t *ents, const uint16_t *rp,
                                          int q, int t0, int nt) {
  for (int it = t0; it < q * 3; it += nt) {
    const int a = it / 3, w0 = 4 * (it - 3 * a);
    uint32_t acc[4] = {0u, 0u, 0u, 0u};
    const int e1 = rp[a + 1];
#pragma unroll 2
    for (int e = rp[a]; e < e1; e++) {
      const uint32_t ent = ents[e];
      const uint32_t *dg = D + (ent >> 16) * DW;
      int o = 32 * w0 - (int)(ent & 0xFFFF);   // window start (c - b) mod 360 for c = 32 w0
      o += o < 0 ? 360 : 0;
      if (DW >= 16) {
        // d_g || d_g[0..152): the four windows o + 32 k end by bit o + 128 < 512, so they are five
        // consecutive words with no wrap
        const int wi = o >> 5;
        const uint32_t sh = 32u - (uint32_t)(o & 31);
        uint32_t x[5];
#pragma unroll
        for (int k = 0; k < 5; k++) x[k] = dg[wi + k];
#pragma unroll
        for (int k = 0; k < 4; k++) acc[k] ^= (uint32_t)((((uint64_t)x[k] << 32) | x[k + 1]) >> sh);
      } else {
#pragma unroll
        for (int k = 0; k < 4; k++) {
          acc[k] ^= ldpc_window(dg, o);
          o += 32;
          o -= o >= 360 ? 360 : 0;
        }
      }
    }
    if (w0 == 8) acc[3] &= 0xFF000000u;
#pragma unroll
    for (int k = 0; k < 4; k++) rowA[12 * a + w0 + k] = acc[k];
  }
}

// LDPC (ldpc_calculate, bbheader:625-646) of the info groups laid out in D: parity rows, the
// accumulate as an inclusive prefix XOR over rows a (wave w scans word columns 3w..3w+2, 64 rows
// per DPP wave scan plus the carry of the previous 64), then the exclusive bit-prefix of the column
// parities along c.  Leaves p[a][c] at D + ngroups * DW (row a, 12 big-endian words); !APPLY_W leaves the
// rows without the column-parity correction, word w of every row to be XORed with Wv[w] by the reader.
template <int DW, bool APPLY_W = true>
__device__ __forceinline__ uint32_t *fec_ldpc(const FecDev &d, uint32_t *D, int ngroups, const uint32_t *ents,
                                              const uint16_t *rowp, uint32_t *Wv, int tid) {
  const int lane = tid & 63, wave = tid >> 6, q = d.q;
  uint32_t *cur = D + ngroups * DW;
  ldpc_rows<DW>(D, cur, ents, rowp, q, tid, FEC_THREADS);
  __syncthreads();
  {
    // q <= 128 (two 64-row chunks): the wave's six column chunks are read before any is written (an LDS
    // read cannot move past an LDS write it may alias: one round trip instead of six)
    uint32_t v[3][2];
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int a = 64 * h + lane;
        v[c][h] = a < q ? cur[a * 12 + 3 * wave + c] : 0u;
      }
#pragma unroll
    for (int c = 0; c < 3; c++) {
      v[c][0] = wave_prefix_xor(v[c][0]);
      v[c][1] = wave_prefix_xor(v[c][1]) ^ rd_lane_u32(v[c][0], 63);
    }
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int a = 64 * h + lane;
        if (a < q) cur[a * 12 + 3 * wave + c] = v[c][h];
      }
  }
  __syncthreads();
  if (tid < 64) {   // word w of the last row by lane w < 12: in-word prefix, carry = parity of words < w
    const uint32_t x = tid < 12 ? cur[(q - 1) * 12 + tid] : 0u;
    uint32_t y = x;
    y ^= y >> 1; y ^= y >> 2; y ^= y >> 4; y ^= y >> 8; y ^= y >> 16;
    const uint32_t p = y & 1u, carry = wave_prefix_xor(p) ^ p;
    uint32_t ex = y ^ x;
    if (carry) ex = ~ex;
    if (tid < 12) Wv[tid] = tid == 11 ? ex & 0xFF000000u : ex;
  }
  __syncthreads();
  if (APPLY_W) {
    // read-modify-write of the rows in batches of four per thread (reads first, then writes)
    for (int it0 = 0; it0 < q * 12; it0 += 4 * FEC_THREADS) {
      uint32_t x[4];
#pragma unroll
      for (int h = 0; h < 4; h++) {
        const int it = it0 + tid + h * FEC_THREADS;
        x[h] = it < q * 12 ? cur[it] ^ Wv[it % 12] : 0u;
      }
#pragma unroll
      for (int h = 0; h < 4; h++) {
        const int it = it0 + tid + h * FEC_THREADS;
        if (it < q * 12) cur[it] = x[h];
      }
    }
    __syncthreads();
  }
  return cur;
}

// BBFRAME of FEC block B (absolute index; the reference keeps count / crc / fec_block as running
// state, bbheader:661-734, here they are closed-form in B) into frame[0, L): raw TS staging, the
// sync-slot CRC-8s, BBHEADER + its CRC-8, payload words, the in-band field, BB scrambling.  Ends
// with a barrier.  crc_resident: the CRC-8 tables already sit at cv.crc8 / cv.crcsh (the BB pass
// stages them once; the fused kernel's LDPC area overlays them, so it reloads them per block).
// BBFRAME geometry of absolute FEC block B, closed form (the reference keeps count / crc / fec_block
// as running state, bbheader:661-734).  NM: the raw stream bytes [pos0 - 188, pos0 + npay) are staged
// as nq 16-byte units from the aligned stream offset 16 w0 (raw byte i = stream byte rs + i at LDS
// byte phase + delta + i)
struct BbGeom {
  int64_t J0, pos0, w0;
  int npay, padding, count0, delta, nq;
};
// x mod 188 for x >= 0 from 32-bit remainders (2^32 = 136 mod 188): a 64-bit remainder by a constant is
// a long 64-bit multiply chain on the scalar unit, and the BB pass evaluates the geometry per block
__device__ __forceinline__ int mod188(int64_t x) {
  const uint32_t hi = (uint32_t)((uint64_t)x >> 32), lo = (uint32_t)x;
  return (int)(((hi % 188u) * 136u + lo % 188u) % 188u);
}
__device__ __forceinline__ BbGeom bb_geom(const FecDev &d, const FecIO &io, int64_t B) {
  BbGeom g;
  const int pay_full = (d.kbch - 80) >> 3;
  int64_t npad_before = 0;
  g.padding = 0;
  if (d.inband) {
    npad_before = (B + d.fec_blocks - 1) / d.fec_blocks;
    g.padding = (B % d.fec_blocks) == 0 ? 104 : 0;
  }
  g.npay = (d.kbch - 80 - g.padding) >> 3;
  g.J0 = B * pay_full - 13 * npad_before;
  g.pos0 = payload_pos(g.J0, d.hem);
  // TS packet position of the next input byte at block start
  if (d.hem) g.count0 = g.J0 == 0 ? 0 : mod188(payload_pos(g.J0 - 1, 1) + 1);
  else g.count0 = mod188(g.pos0);
  const int64_t rel = g.pos0 - 188 - io.ts_base;        // >= -188
  g.w0 = (rel >= 0 ? rel : rel - 15) / 16;              // floor
  g.delta = (int)(rel - 16 * g.w0);
  g.nq = (g.delta + g.npay + 188 + 15) >> 4;
  return g;
}
// raw unit i (16 stream bytes at offset 16 (w0 + i) of the TS buffer): one 16-byte load, or byte
// loads for a misaligned buffer or at the stream edges (zeros outside)
__device__ __forceinline__ uint4 bb_raw_unit(const FecIO &io, const uint8_t *tin, int64_t w0, int i) {
  const int64_t b = 16 * (w0 + i);
  if ((((uintptr_t)tin) & 15) == 0 && b >= 0 && b + 16 <= io.ts_len) return *(const uint4 *)(tin + b);
  uint32_t w[4] = {0u, 0u, 0u, 0u};
  for (int e = 0; e < 16; e++)
    if (b + e >= 0 && b + e < io.ts_len) w[e >> 2] |= (uint32_t)tin[b + e] << (8 * (e & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}
constexpr int FEC_PRE = 2;   // raw units per thread a BB pass workgroup prefetches for its next block (nq <= 512)

// GOUT (the chain's BB pass): the BBFRAME words go straight to the block's codeword row outw, not through
// the LDS frame and a copy (fec 1.553 -> 1.539 ms per 1280 cfg3 frames)
template <bool CRC_RESIDENT, bool PRE, bool GOUT = false>
__device__ void fec_bbframe(const FecDev &d, const FecIO &io, const FecCarve &cv, unsigned char *smem, int64_t B,
                            const uint8_t *tin, int tid, const uint4 *pre = nullptr, const BbGeom *gp = nullptr,
                            uint32_t *outw = nullptr) {
  const int lane = tid & 63, wave = tid >> 6;
  const int L = d.kbch >> 3;
  uint8_t *frame = smem + cv.frame, *phase = smem + cv.phase;
  uint8_t *crc8 = smem + cv.crc8, *crcsh = smem + cv.crcsh;
  const uint8_t *crcsl = smem + cv.crcsl;   // BB pass (CRC_RESIDENT): T^1 | T^2 | .. | T^24
  const uint8_t *hcrc8 = smem + cv.hcrc;
  uint8_t *syncv = smem + cv.sync;
  const BbGeom g = gp ? *gp : bb_geom(d, io, B);
  const int npay = g.npay, padding = g.padding, count0 = g.count0;
  const int64_t J0 = g.J0, pos0 = g.pos0;
  // NM: stage the raw stream bytes once (PRE: the units this thread prefetched, unit tid + 256 k in
  // pre[k]); the CRC-8 chains and the payload words then read LDS
  const int64_t rs = pos0 - 188;
  int delta = 0, first_slot = 0;
  const uint32_t *raww = (const uint32_t *)phase;
  if (!d.hem) {
    if (!CRC_RESIDENT) {
      for (int i = tid; i < 64; i += FEC_THREADS) ((uint32_t *)crc8)[i] = ((const uint32_t *)d.crc8_tab)[i];
      for (int i = tid; i < 512; i += FEC_THREADS) ((uint32_t *)crcsh)[i] = ((const uint32_t *)d.crc8_shift)[i];
    }
    delta = g.delta;
    uint4 *rawq = (uint4 *)phase;
    if (PRE) {
#pragma unroll
      for (int k = 0; k < FEC_PRE; k++)
        if (tid + FEC_THREADS * k < g.nq) rawq[tid + FEC_THREADS * k] = pre[k];
    } else {
      for (int i = tid; i < g.nq; i += FEC_THREADS) rawq[i] = bb_raw_unit(io, tin, g.w0, i);
    }
    const uint8_t *raw = phase + delta;
    __syncthreads();
    first_slot = (188 - count0) % 188;
    const int nslots = first_slot < npay ? (npay - 1 - first_slot) / 188 + 1 : 0;
    // CRC-8 of each packet whose sync slot falls in this block: 8 lanes per packet, 24-byte
    // chunks combined with zero-extension tables; up to 36 slots per block (5/6 normal), 32 per pass
    for (int m0 = 0; m0 < nslots; m0 += FEC_THREADS / 8) {
      const int m = m0 + (tid >> 3), k = tid & 7;
      uint8_t part = 0;
      int64_t p = pos0 + first_slot + 188 * (int64_t)m;   // sync position
      bool active = m < nslots && p > 0;
      if (active) {
        const int n = k == 7 ? 19 : 24;            // 187 = 7 x 24 + 19
        uint32_t c = 0;
        if (CRC_RESIDENT) {
          // T is linear, so the register after bytes b_0 .. b_23 from c = 0 is the XOR of T^(24 - i)[b_i]:
          // 24 independent lookups (the BB pass keeps T^1 .. T^24 in LDS) instead of a chain of dependent
          // ones (slicing by 4 had six LDS round trips in a row: the CRC phase was ~0.18 ms of the pass);
          // the 19-byte last chunk is front-padded with zero bytes, T^k[0] = 0
          // the chunk's bytes as six aligned dwords (seven dword reads and a byte align each) instead of
          // 24 byte reads
          const int pad = 24 - n;
          const uint8_t *bp = raw + (p - 187 + 24 * k - rs) - pad;
          const uint32_t sh = (uint32_t)((uintptr_t)bp & 3u);
          const uint32_t *bw = (const uint32_t *)(bp - sh);
          uint32_t w7[7], t[24];
#pragma unroll
          for (int j = 0; j < 7; j++) w7[j] = bw[j];
#pragma unroll
          for (int j = 0; j < 6; j++) {
            const uint32_t a = __builtin_amdgcn_alignbyte(w7[j + 1], w7[j], sh);
#pragma unroll
            for (int e = 0; e < 4; e++) {
              const int i = 4 * j + e;
              uint32_t by = (a >> (8 * e)) & 0xFFu;
              if (i < 5) by = i >= pad ? by : 0u;   // pad is 0 or 5
              t[i] = crcsl[(23 - i) * 256 + by];
            }
          }
          // all 24 lookups in flight, then an XOR tree (a running XOR had the compiler wait per pair)
#pragma unroll
          for (int h = 12; h >= 3; h >>= 1)
#pragma unroll
            for (int i = 0; i < h; i++) t[i] ^= t[i + h];
          c = t[0] ^ t[1] ^ t[2];
        } else {
          const uint8_t *b0 = raw + (p - 187 + 24 * k - rs);
          uint8_t by[24];
#pragma unroll
          for (int i = 0; i < 24; i++) by[i] = i < n ? b0[i] : 0;
#pragma unroll
          for (int i = 0; i < 24; i++)
            if (i < n) c = crc8[by[i] ^ c];
        }
        part = crcsh[k * 256 + c];
      }
      // XOR of the 8 lanes' parts into lane k == 0: DPP quad_perm [1,0,3,2], [2,3,0,1], row_shl:4
      uint32_t v = part;
      v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, true);
      v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, true);
      v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xF, 0xF, true);
      if (k == 0 && m < nslots) {
        syncv[m] = active ? (uint8_t)v : 0;
        // the reference warns on every consumed sync byte that is not 0x47 (bbheader:703-705)
        if (io.sync_err && raw[p - rs] != 0x47) atomicAdd(io.sync_err, 1u);
      }
    }
    __syncthreads();
  }
  if (d.hem && io.sync_err) {
    // HEM drops each packet's sync byte; the one of packet p is consumed just before payload
    // byte 187 p (bbheader:673-680, warning at :675-677)
    const int64_t p0 = (J0 + 186) / 187;
    for (int64_t pk = p0 + tid; 187 * pk < J0 + npay; pk += FEC_THREADS)
      if (tin[188 * pk - io.ts_base] != 0x47) atomicAdd(io.sync_err, 1u);
  }
  // BBHEADER (bbheader:272-325), uniform across the workgroup: MATYPE (FecDev::matype: TS, SIS or MIS
  // with ISI, CCM, ISSYI 0, NPD 0, RO 0); bytes 0..7 big-endian in hw, byte 8 = SYNCD low, byte 9 = CRC-8
  const uint32_t upl = d.hem ? 0u : 188u * 8u, dfl = (uint32_t)(d.kbch - 80 - padding);
  const uint32_t syncb = d.hem ? 0u : 0x47u, syncd = count0 == 0 ? 0u : (uint32_t)(188 - count0) * 8u;
  const uint64_t hw = ((uint64_t)(uint32_t)d.matype << 48) | ((uint64_t)upl << 32) | ((uint64_t)dfl << 16) | ((uint64_t)syncb << 8) |
                      (uint64_t)(syncd >> 8);
  // CRC-8 over the 72 header bits, LSB-first register with 0xAB (add_crc8_bits :247-270): XOR
  // of the per-bit contributions (t2_plan hcrc_bits), lane n taking header bit n (and 64 + n),
  // then an XOR reduction over the wave; only wave 0 writes the header word (bytes 8..11)
  uint32_t hcrc = 0;
  if (__builtin_amdgcn_readfirstlane(wave) == 0) {
    uint32_t v = ((hw >> (63 - lane)) & 1u) ? (uint32_t)hcrc8[lane] : 0u;
    if (lane < 8 && (((syncd & 0xFFu) >> (7 - lane)) & 1u)) v ^= hcrc8[64 + lane];
    hcrc = rd_lane_u32(wave_prefix_xor(v), 63);   // XOR over the wave
    if (d.hem) hcrc ^= 0x80u;
  }
  const uint32_t hcrc_rev = __builtin_bitreverse32(hcrc) >> 24;   // register LSB written first
  auto slow_byte = [&](int pidx) -> uint32_t {   // BBFRAME byte pidx outside the bulk payload path
    if (pidx < 8) return (uint32_t)(hw >> (56 - 8 * pidx)) & 0xFFu;
    if (pidx == 8) return syncd & 0xFFu;
    if (pidx == 9) return hcrc_rev;
    const int j = pidx - 10;
    if (j < npay) {
      if (d.hem) return tin[payload_pos(J0 + j, 1) - io.ts_base];
      const int r = (count0 + j) % 188;
      return r == 0 ? (uint32_t)syncv[(j - first_slot) / 188] : (uint32_t)phase[delta + 188 + j];
    }
    const int k = j - npay;   // in-band type B (bbheader:327-355): 01, 65 zero bits, TS rate (27 bits), 10 zeros
    if (!padding || k >= 13) return 0u;
    uint32_t v = k == 0 ? 0x40u : 0u;
    for (int e = 0; e < 8; e++) {
      const int bit = 8 * k + e;
      if (bit >= 67 && bit < 94 && ((d.ts_rate >> (26 - (bit - 67))) & 1)) v |= 1u << (7 - e);
    }
    return v;
  };
  // BBFRAME words = header | payload (each sync slot carries the CRC-8 of the previous packet,
  // bbheader:701-719) | in-band field, BB-scrambled (:694-696, :724-726)
  uint32_t *framew = GOUT ? outw : (uint32_t *)frame;
  // (the BB pass keeps the PRBS in LDS: a global load per word here was waited for with vmcnt(0),
  // which also waited for the next block's prefetched TS units)
  const uint32_t *prbsw = CRC_RESIDENT ? (const uint32_t *)(smem + cv.prbs) : (const uint32_t *)d.prbs;
  // bulk payload words (NM: bytes 10 + j, j in [0, npay), whole words w in [3, wf1)) from the staged
  // stream; the few others (header, the edges, in-band field; every word in HEM) in a separate loop,
  // so the bulk loop carries no global loads or their waits
  const int nw = (L + 3) >> 2, wf1 = d.hem ? 3 : (npay + 10) >> 2;
  for (int w = 3 + tid; w < wf1; w += FEC_THREADS) {
    const int j0 = 4 * w - 10;
    const int q = delta + 188 + j0;
    uint32_t v = __builtin_amdgcn_alignbyte(raww[(q >> 2) + 1], raww[q >> 2], (uint32_t)(q & 3));
    const int r0 = (count0 + j0) % 188, e = r0 == 0 ? 0 : 188 - r0;
    if (e < 4) {
      const uint32_t sb = syncv[(j0 + e - first_slot) / 188];
      v = (v & ~(0xFFu << (8 * e))) | (sb << (8 * e));
    }
    framew[w] = v ^ prbsw[w];
  }
  for (int i = tid; i < 3 + nw - wf1; i += FEC_THREADS) {
    const int w = i < 3 ? i : wf1 + (i - 3);
    uint32_t v = 0;
    for (int e = 0; e < 4; e++) v |= slow_byte(4 * w + e) << (8 * e);
    framew[w] = v ^ prbsw[w];
  }
  __syncthreads();
}

// launch block bi of a (multi-stream) batch: its absolute FEC block index and TS base.  Stream-major
// batch: launch block bi is block bi % bps of stream bi / bps, whose TS slice (same ts_base / ts_len
// layout for every stream) starts at in + stream * ts_stride
__device__ __forceinline__ int64_t fec_block_of(const FecIO &io, int bi, const uint8_t *&tin) {
  const int sidx = io.blocks_per_stream ? bi / io.blocks_per_stream : 0;
  tin = io.in + (int64_t)sidx * io.ts_stride;
  return io.first_block + (bi - sidx * io.blocks_per_stream);
}

// fused FEC for the block API: TS -> BBFRAME + BCH (unpacked nbch bits, the bbheaderbch block) or
// unpacked nbch bits -> LDPC codeword (unpacked nldpc bits in natural order, the ldpc block)
template <int MODE>
__global__ __launch_bounds__(FEC_THREADS, FEC_WG_PER_CU) void fec_kernel(FecDev d, FecIO io) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = d.kbch >> 3;           // BBFRAME bytes
  const int NB = d.nbch >> 3;          // info bytes (BBFRAME + BCH parity)
  const int P = d.P;
  const FecCarve cv = fec_carve(CARVE_FUSED, d.kbch, d.nbch, d.q);
  uint8_t *frame = smem + cv.frame;
  uint64_t *btab = (uint64_t *)(smem + cv.btab);
  uint32_t *ents = (uint32_t *)(smem + cv.ents);
  uint32_t *D = (uint32_t *)(smem + cv.phase);
  // ---- constant tables into LDS, once: the workgroup then loops over FEC blocks
  if (MODE == FEC_TS_TO_BITS) {
    for (int i = tid; i < 768; i += FEC_THREADS) btab[i] = d.bch_tab[i];
    for (int i = tid; i < 72; i += FEC_THREADS) smem[cv.hcrc + i] = d.hcrc_bits[i];
  } else {
    for (int i = tid; i < d.nent; i += FEC_THREADS) ents[i] = d.ldpc_ent[i];
    for (int i = tid; i <= d.q; i += FEC_THREADS) ((uint16_t *)(smem + cv.rowp))[i] = d.ldpc_rowptr[i];
  }
  __syncthreads();
  for (int bi = blockIdx.x; bi < io.nblocks; bi += gridDim.x) {
    if (MODE == FEC_TS_TO_BITS) {
      const uint8_t *tin;
      const int64_t B = fec_block_of(io, bi, tin);
      fec_bbframe<false, false>(d, io, cv, smem, B, tin, tid);
      // BCH on wave 0 (raised issue priority: the block's critical path)
      if (wave == 0) {
        __builtin_amdgcn_s_setprio(1);
        uint64_t a[3];
        switch (P) {   // compile-time register geometry per BCH parity length (t = 12, 10, 8; short 12)
          case 192: bch_wave<192>(frame, btab, d.bch_ctab, L, d.chunk, lane, a); break;
          case 168: bch_wave<168>(frame, btab, d.bch_ctab, L, d.chunk, lane, a); break;
          case 160: bch_wave<160>(frame, btab, d.bch_ctab, L, d.chunk, lane, a); break;
          default: bch_wave<128>(frame, btab, d.bch_ctab, L, d.chunk, lane, a); break;
        }
        // parity MSB (x^(P-1)) first as frame[L..L + P/8) (bbheader:504-531)
        if (lane < P / 8) frame[L + lane] = get_byte192(a, P - 8 - 8 * lane);
        __builtin_amdgcn_s_setprio(0);
      }
      __syncthreads();
      uint8_t *dst = io.out + (int64_t)bi * d.nbch;
      for (int i = tid; i < d.nbch; i += FEC_THREADS) dst[i] = (frame[i >> 3] >> (7 - (i & 7))) & 1;
    } else {
      // pack nbch unpacked info bits, lay out the info groups, LDPC, unpacked natural-order output
      const uint8_t *src = io.in + (int64_t)bi * d.nbch;
      for (int k = tid; k < NB; k += FEC_THREADS) {
        uint32_t v = 0;
        for (int e = 0; e < 8; e++) v |= (uint32_t)(src[8 * k + e] & 1) << (7 - e);
        frame[k] = (uint8_t)v;
      }
      __syncthreads();
      const int ngroups = d.nbch / 360;
      for (int it = tid; it < ngroups * FEC_DW; it += FEC_THREADS) {
        const int g = it / FEC_DW;
        ldpc_group_word<FEC_DW>(D, frame, g, it - g * FEC_DW);
      }
      __syncthreads();
      const uint32_t *cur = fec_ldpc<FEC_DW>(d, D, ngroups, ents, (const uint16_t *)(smem + cv.rowp), (uint32_t *)(smem + cv.w), tid);
      const int q = d.q;
      uint8_t *dst = io.out + (int64_t)bi * d.nldpc;
      for (int i = tid; i < d.nbch; i += FEC_THREADS) dst[i] = (frame[i >> 3] >> (7 - (i & 7))) & 1;
      const int pbits = d.nldpc - d.nbch;
      for (int j = tid; j < pbits; j += FEC_THREADS) {   // parity bit of row a = j mod q, column c = j / q
        const int a = j % q, c = j / q;
        dst[d.nbch + j] = (uint8_t)((cur[a * 12 + (c >> 5)] >> (31 - (c & 31))) & 1);
      }
    }
    __syncthreads();   // frame / phase regions are reused by the next block
  }
}

// ---- chain pass 2: BCH as a GF(2) matrix product on the matrix cores
typedef int bch_v8i __attribute__((ext_vector_type(8)));
typedef float bch_v16f __attribute__((ext_vector_type(16)));

// ---- chain FEC, fused (round 6): the BB pass and the matrix-core BCH as one kernel, bbch_kernel
// The BB pass wrote each BBFRAME to HBM and the BCH pass read it back (1.7 x the FEC stage's minimal bytes).
// Here each lane builds its own A-fragment piece -- BBFRAME bytes [P0, P0 + 16), P0 = 32 q + 16 h, of its block
// (h = lane >> 5) -- straight from the TS in registers: the payload bytes of the stream with each sync slot
// replaced by the CRC-8 of the packet before it (bbheader:701-719; HEM: the sync bytes dropped, :673-680), the
// BBHEADER in chunk 0 (:272-325), the in-band type B field after the payload (:327-355), BB scrambling
// (:694-696, 724-726).  The piece is stored to the block's codeword row (the LDPC + map kernel reads the BBFRAME
// there) and multiplied on the matrix cores.
// Sync-slot CRC-8s are streamed.  The CRC register is linear, so a 16-byte piece b_0..b_15 moves it as
// s' = T^16[s] ^ G, G = XOR_i T^(16-i)[b_i]: 16 independent lookups in the power tables T^1..T^16 (LDS).  A piece
// with a sync position at offset e restarts the register after it (s' = the same lookups over bytes e+1..15) and
// its slot is recovered from s' through the inverse power tables (crc_chunk).  The two lanes of a row hand the
// register to each other once per piece.  A tile segment starting at chunk q0 first streams the CRC through the
// BBCH_PRO chunks (192 stream bytes) before it, so a sync position (one every 188 bytes) has restarted the
// register before the first slot it fills.
constexpr int BBCH_THREADS = 256;   // 4 waves: a tile of 128 FEC blocks per workgroup, two workgroups per CU (up
constexpr int BBCH_ROWS = 128;      // to 256 VGPRs: two waves per SIMD)
constexpr int BBCH_WG_PER_CU = 2;
constexpr int BBCH_PRO = 6;         // CRC prologue chunks (6 x 32 >= 188 + 4)
// T^k, T^-k, BBHEADER CRC per byte, in-band bytes, the CRC prefix masks (17 x 16 bytes)
constexpr int BBCH_TAB = 16 * 256 * 2 + 9 * 256 + 16 + 17 * 16;
// the BBFRAME pieces of 4 chunks per row are staged in LDS (row stride 144 B: conflict-free 16-byte writes) and
// stored as whole 128-byte lines: a wave's store instruction then writes 8 full lines instead of 32 rows x 32 B
constexpr int BBCH_STG_STRIDE = 144;
constexpr int BBCH_STG = BBCH_ROWS * BBCH_STG_STRIDE;
static_assert(BBCH_TAB % 16 == 0, "the staging area after the tables is read as 16-byte units");
__host__ __device__ constexpr int bbch_lds(int nt) { return 2 * 4 * nt * 64 * 16 + BBCH_TAB + BBCH_STG; }

// The stream bytes of a piece: a = bytes [rel, rel + 16) of the TS buffer, and for HEM also b = [rel + 1, rel + 17),
// each one unaligned 16-byte load (gfx9 global loads need no alignment; the compiler emits one dwordx4 for an
// align-1 pointer).  ts_fetch always issues the loads (from the buffer start when the bytes are not all inside
// [tin, tin + len): edge) and returns without waiting for them; ts_slow redoes an edge piece bytewise with zeros
// outside the buffer.  (A fast / slow branch merged inside the fetch made the compiler wait for the loads right
// there, vmcnt(0).)
struct TsWin {
  uint32_t a[4], b[4];
  uint32_t p[4];   // the chunk's BB-scrambling bytes for this lane's half (loaded with the window)
  bool edge;
};
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct __attribute__((packed, aligned(1))) U32x4Unaligned {
  u32x4 v;
};
typedef const __attribute__((address_space(1))) U32x4Unaligned *g4uptr;   // global, not flat: a flat load may read
typedef const __attribute__((address_space(1))) uint8_t *g1ptr;          // LDS, so the compiler would wait for LDS
template <bool HEM>
__device__ __forceinline__ TsWin ts_fetch(const uint8_t *tin, int64_t len, int64_t rel) {
  TsWin r;
  const uintptr_t t0 = (uintptr_t)tin, a = t0 + (uintptr_t)rel;
  r.edge = !(rel >= 0 && rel + 17 <= len);
  const uintptr_t src = r.edge ? t0 : a;   // len >= 64 (fec_chain_args_ok)
  const u32x4 x = ((g4uptr)src)->v;
#pragma unroll
  for (int k = 0; k < 4; k++) r.a[k] = x[k];
  if (HEM) {
    const u32x4 y = ((g4uptr)(src + 1))->v;
#pragma unroll
    for (int k = 0; k < 4; k++) r.b[k] = y[k];
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++) r.b[k] = 0u;
  }
  return r;
}
// bytes [rel, rel + 17) bytewise, zeros outside the buffer, into a (first 16) and b (from rel + 1)
__device__ __forceinline__ void ts_slow(const uint8_t *tin, int64_t len, int64_t rel, TsWin &w) {
  uint64_t q0 = 0, q1 = 0, q2 = 0;   // named halves, not an indexed array (that would live in scratch)
#pragma unroll 1
  for (int b = 0; b < 17; b++) {
    const int64_t p = rel + b;
    const uint64_t v = p >= 0 && p < len ? (uint64_t)*(g1ptr)(tin + p) << (8 * (b & 7)) : 0ull;
    q0 |= b < 8 ? v : 0ull;
    q1 |= b >= 8 && b < 16 ? v : 0ull;
    q2 |= b >= 16 ? v : 0ull;
  }
  w.a[0] = (uint32_t)q0; w.a[1] = (uint32_t)(q0 >> 32); w.a[2] = (uint32_t)q1; w.a[3] = (uint32_t)(q1 >> 32);
  const uint64_t r0 = (q0 >> 8) | (q1 << 56), r1 = (q1 >> 8) | (q2 << 56);
  w.b[0] = (uint32_t)r0; w.b[1] = (uint32_t)(r0 >> 32); w.b[2] = (uint32_t)r1; w.b[3] = (uint32_t)(r1 >> 32);
}
// byte i (dynamic) of four little-endian dwords, and its replacement; selects between named 64-bit values, never
// an indexed array (a select chain over an array's elements is folded into a dynamically indexed load, which
// lives in scratch memory)
__device__ __forceinline__ uint32_t byte_of(const uint32_t *d, int i) {   // i dynamic, 0 .. 15
  const uint64_t lo = ((uint64_t)d[1] << 32) | d[0], hi = ((uint64_t)d[3] << 32) | d[2];
  return (uint32_t)(((i & 8) ? hi : lo) >> (8 * (i & 7))) & 0xFFu;
}
__device__ __forceinline__ void set_byte(uint32_t *d, int i, uint32_t b) {   // i dynamic, 0 .. 15; b < 256
  // one byte permute per dword: the identity selector (bytes 4 .. 7 pick d's bytes) with byte i's selector 0
  // (b's byte 0); the four selectors as two 64-bit halves
  const uint64_t id = 0x0706050407060504ull, m = 0xFFull << (8 * (i & 7));
  const uint64_t slo = (i & 8) ? id : id & ~m, shi = (i & 8) ? id & ~m : id;
  d[0] = __builtin_amdgcn_perm(d[0], b, (uint32_t)slo);
  d[1] = __builtin_amdgcn_perm(d[1], b, (uint32_t)(slo >> 32));
  d[2] = __builtin_amdgcn_perm(d[2], b, (uint32_t)shi);
  d[3] = __builtin_amdgcn_perm(d[3], b, (uint32_t)(shi >> 32));
}

// one row's BB state over the chunks: the block's geometry and, per lane, its stream cursor
struct BbchRow {
  const uint8_t *tin;
  uint8_t *row;
  BbGeom g;
  int64_t rel;   // NM: TS offset of this lane's piece in the current chunk (BBFRAME byte P0 -> stream pos0 + P0 - 10)
  int m;         // NM: that stream position mod 188
  int64_t sh;    // HEM: stream position of payload byte J0 + P0 - 10 (the tracked chunk's piece)
  int r;         // HEM: (J0 + P0 - 10) mod 187
  bool live;
};

// NM CRC of a row's chunk (two 16-byte pieces, lane h = 0 then h = 1).  The register is linear: from s, a piece
// b_0..b_15 leads to s_full = T^16[s] ^ G, G = XOR_i t_i, t_i = T^(16-i)[b_i] (16 independent lookups, T^k at
// tp + (k-1) 256).  A piece with a sync position e < 16 restarts the register after it: A = XOR_{i>e} t_i = G ^ P,
// P = XOR_{i<=e} t_i, and its slot value is the register before byte e: s_full = T^(16-e)[slot ^ b_e] ^ A, so
// slot = T^-(16-e)[s_full ^ A] ^ b_e (T^-k at tq + (k-1) 256).  The terms are packed four to a dword, so G and
// the prefix P under a per-lane bound e are two 128-bit XOR folds, one of them masked (a per-term masked prefix
// cost ~4 VALU per term).
__device__ __forceinline__ uint32_t fold8(uint64_t x) {
  const uint32_t y = (uint32_t)x ^ (uint32_t)(x >> 32);
  return (y ^ (y >> 8) ^ (y >> 16) ^ (y >> 24)) & 0xFFu;
}
// the register at the next chunk (both lanes) from s; slot: this lane's sync slot value, be: the piece's byte
// at the sync position (e < 16)
__device__ __forceinline__ uint32_t crc_chunk(const uint8_t *tp, const uint8_t *tq, const uint4 *pmask, const uint32_t *d,
                                              int e, int h, uint32_t s, uint32_t &slot, uint32_t &be) {
  const bool sync = e < 16;
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    w[k] = 0u;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int i = 4 * k + j;
      w[k] |= (uint32_t)tp[(15 - i) * 256 + ((d[k] >> (8 * j)) & 0xFFu)] << (8 * j);
    }
  }
  const uint64_t lo = ((uint64_t)w[1] << 32) | w[0], hi = ((uint64_t)w[3] << 32) | w[2];
  const uint4 m = pmask[min(e, 16)];   // terms 0 .. e
  const uint32_t g = fold8(lo ^ hi);
  const uint32_t A = g ^ fold8((((uint64_t)(w[1] & m.y) << 32) | (w[0] & m.x)) ^ (((uint64_t)(w[3] & m.w) << 32) | (w[2] & m.z)));
  const uint32_t o0 = sync ? A : (uint32_t)tp[15 * 256 + s] ^ g;   // lane 0's register after its piece
  // every lane runs both exchanges (a lane exchange under a condition would read inactive lanes)
  const uint32_t y = (uint32_t)__shfl_xor((int)o0, 32);
  const uint32_t s_in = h ? y : s;
  const uint32_t sf = (uint32_t)tp[15 * 256 + s_in] ^ g;
  const uint64_t dlo = ((uint64_t)d[1] << 32) | d[0], dhi = ((uint64_t)d[3] << 32) | d[2];
  be = (uint32_t)(((e & 8) ? dhi : dlo) >> (8 * (e & 7))) & 0xFFu;
  slot = (uint32_t)tq[(15 - min(e, 15)) * 256 + (sf ^ A)] ^ be;
  const uint32_t o1 = sync ? A : sf;
  const uint32_t z = (uint32_t)__shfl_xor((int)o1, 32);
  return h ? o1 : z;
}

template <int NT, bool HEM>
__global__ __launch_bounds__(BBCH_THREADS, BBCH_WG_PER_CU) void bbch_kernel(FecDev d, FecIO io) {
  extern __shared__ __attribute__((aligned(16))) uint4 bsm[];
  constexpr int PER = 4 * NT * 64;                   // uint4 per chunk buffer
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int L = d.kbch >> 3;
  const uint4 *prbs16 = (const uint4 *)d.prbs;   // zero-padded to whole chunks (t2_plan FecPlan::prbs_bytes)
  uint8_t *tp = (uint8_t *)(bsm + 2 * PER), *tq = tp + 4096, *hd = tq + 4096, *ibb = hd + 9 * 256;
  uint4 *pmask = (uint4 *)(ibb + 16);   // pmask[e]: bytes 0 .. e of a piece (e = 16: all)
  uint8_t *stg = tp + BBCH_TAB;   // 16-byte aligned: BBCH_TAB is a multiple of 16
  // ---- tables, once per workgroup: T^1..T^16 and their inverses (NM), the BBHEADER CRC-8 per header byte
  // (add_crc8_bits :247-270: XOR of the per-bit contributions hcrc_bits, bit 8 b + j = bit 7 - j of byte b), the
  // in-band type B bytes (:327-355: 01, 65 zero bits, the TS rate in 27 bits, 10 zero bits)
  if (!HEM && tid < 256) {   // (BBCH_THREADS >= 256)
    uint32_t v = (uint32_t)tid;
    for (int k = 0; k < 16; k++) {
      v = d.crc8_tab[v];
      tp[k * 256 + tid] = (uint8_t)v;
    }
  }
  for (int i = tid; i < 9 * 256; i += BBCH_THREADS) {
    const int b = i >> 8, x = i & 255;
    uint32_t v = 0;
    for (int j = 0; j < 8; j++)
      if ((x >> (7 - j)) & 1) v ^= d.hcrc_bits[8 * b + j];
    hd[i] = (uint8_t)v;
  }
  if (tid < 17 * 4) {   // prefix masks
    const int e = tid >> 2, k = tid & 3, n = min(max(e + 1 - 4 * k, 0), 4);
    ((uint32_t *)pmask)[tid] = n >= 4 ? 0xFFFFFFFFu : (1u << (8 * n)) - 1u;
  }
  if (tid < 13) {
    uint32_t v = tid == 0 ? 0x40u : 0u;
    for (int e = 0; e < 8; e++) {
      const int bit = 8 * tid + e;
      if (bit >= 67 && bit < 94 && ((d.ts_rate >> (26 - (bit - 67))) & 1)) v |= 1u << (7 - e);
    }
    ibb[tid] = (uint8_t)v;
  }
  __syncthreads();
  if (!HEM && tid < 256)
    for (int k = 0; k < 16; k++) tq[k * 256 + tp[k * 256 + tid]] = (uint8_t)tid;
  __syncthreads();

  const int slice = (int)blockIdx.x % BCH_KS, per_slice = (int)gridDim.x / BCH_KS, kq = (int)blockIdx.x / BCH_KS;
  const int qs0 = slice * d.bch_nq / BCH_KS, nc = (slice + 1) * d.bch_nq / BCH_KS - qs0;   // chunks per tile
  const int64_t units = (int64_t)((io.nblocks + BBCH_ROWS - 1) / BBCH_ROWS) * nc;
  const int64_t u1 = units * (kq + 1) / per_slice;
  // chunk q's B fragments (t2_plan build_bch_mfma, lane-linear): loaded into registers a chunk ahead, written to
  // LDS buffer buf after the chunk's MFMAs.  Not LDS-DMA: the compiler cannot tell which LDS bytes a DMA writes,
  // so it waits for every outstanding DMA with vmcnt(0) before any LDS read.  (In round 5's bch_gemm_kernel that
  // wait sat right after the next chunk's DMA, so its double buffer never overlapped a DMA with the MFMAs; here
  // vmcnt(0) would also drain the BBFRAME stores.)
  // (a vector value, not a uint4 array: the array was kept in scratch memory, a store and a reload per chunk)
  constexpr int BJ = (PER + BBCH_THREADS - 1) / BBCH_THREADS;   // uint4 per thread (the last one partial for odd NT)
  typedef uint32_t bfr_t __attribute__((ext_vector_type(4 * BJ)));
  auto bload = [&](int q) -> bfr_t {
    bfr_t v;
#pragma unroll
    for (int j = 0; j < BJ; j++) {
      const int i = BBCH_THREADS * j + tid;
      // (j + 1) THREADS <= PER: the compiler does not know tid < THREADS, and a condition it cannot fold makes a branch
      const uint4 x = (BBCH_THREADS * (j + 1) <= PER || i < PER) ? d.bch_mfma[(size_t)q * PER + i] : make_uint4(0u, 0u, 0u, 0u);
      v[4 * j] = x.x;
      v[4 * j + 1] = x.y;
      v[4 * j + 2] = x.z;
      v[4 * j + 3] = x.w;
    }
    return v;
  };
  auto bstore = [&](int buf, const bfr_t &v) {
#pragma unroll
    for (int j = 0; j < BJ; j++) {
      const int i = BBCH_THREADS * j + tid;
      if (BBCH_THREADS * (j + 1) <= PER || i < PER) bsm[buf * PER + i] = make_uint4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
    }
  };

  for (int64_t u = units * kq / per_slice; u < u1;) {
    const int tile = (int)(u / nc), q0 = qs0 + (int)(u % nc);
    const int q1 = q0 + (int)min((int64_t)(qs0 + nc - q0), u1 - u);
    u += q1 - q0;
    const int row0 = tile * BBCH_ROWS + wave * 32, blk = row0 + (lane & 31);
    BbchRow R{};
    R.live = blk < io.nblocks;
    R.tin = io.in;
    if (R.live) {
      const int64_t B = fec_block_of(io, blk, R.tin);
      R.g = bb_geom(d, io, B);
    }
    R.row = io.out + (int64_t)(R.live ? blk : 0) * io.cw_stride;
    const int npay = R.g.npay;
    uint32_t crc = 0;   // NM: the CRC register at the start of this lane's row's current chunk (both lanes)
    // ---- per-lane cursors at the first chunk this segment streams
    if (!HEM) {
      const int qa = q0 - BBCH_PRO;
      const int64_t S = R.g.pos0 + 32 * qa + 16 * h - 10;   // >= pos0 - 208
      R.rel = S - io.ts_base;
      R.m = mod188(S + 376);
      // the CRC prologue: the register through the BBCH_PRO chunks before q0 (no slots, no stores)
      for (int q = qa; q < q0; q++) {
        TsWin w = ts_fetch<false>(R.tin, io.ts_len, R.rel);
        if (R.live && w.edge) ts_slow(R.tin, io.ts_len, R.rel, w);
        uint32_t pd[4];
#pragma unroll
        for (int k = 0; k < 4; k++) pd[k] = R.live ? w.a[k] : 0u;
        const int e = R.m == 0 ? 0 : 188 - R.m;
        uint32_t slot, be;
        crc = crc_chunk(tp, tq, pmask, pd, e, h, crc, slot, be);
        R.rel += 32;
        R.m += 32;
        R.m -= R.m >= 188 ? 188 : 0;
      }
    } else {
      // HEM: the tracked piece is chunk q0's, or chunk 1's where chunk 0's lane-0 piece holds the header
      const int qa = (q0 == 0 && h == 0) ? 1 : q0;
      const int64_t J = R.g.J0 + 32 * qa + 16 * h - 10;
      R.r = (int)(J % 187);
      R.sh = 188 * (J / 187) + 1 + R.r;
    }
    // ---- the piece of chunk q in four dwords; stores nothing
    auto build = [&](int q, TsWin w, uint32_t *pd) {
      const int P0 = 32 * q + 16 * h;
      if (w.edge && R.live && P0 < L && P0 - 10 < npay && (P0 >= 10 || !HEM))
        ts_slow(R.tin, io.ts_len, HEM ? R.sh - io.ts_base : R.rel, w);
      uint32_t raw[4];
#pragma unroll
      for (int k = 0; k < 4; k++) raw[k] = w.a[k];
      if (!HEM) {
        const int e = R.m == 0 ? 0 : 188 - R.m;
        uint32_t slot, be;
        crc = crc_chunk(tp, tq, pmask, raw, e, h, crc, slot, be);
#pragma unroll
        for (int k = 0; k < 4; k++) pd[k] = raw[k];
        const int j = P0 + e - 10;   // payload byte at the sync position
        if (e < 16 && j >= 0 && j < npay && R.live) {
          if (io.sync_err && be != 0x47u) atomicAdd(io.sync_err, 1u);   // bbheader:703-705
          set_byte(pd, e, slot);
        }
        R.rel += 32;
        R.m += 32;
        R.m -= R.m >= 188 ? 188 : 0;
      } else if (P0 >= 10) {
        // payload bytes with the sync byte before payload byte J' (J' mod 187 = 0) dropped: bytes e.. shift by one
        const uint32_t *b1 = w.b;
        const int es = 187 - R.r;   // the next packet's first payload byte is J + es (its sync byte before it)
        const int e = es < 16 ? es : 16;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int t = min(max(e - 4 * k, 0), 4);
          const uint32_t m = t >= 4 ? 0u : 0xFFFFFFFFu << (8 * t);   // bytes i >= e
          pd[k] = (raw[k] & ~m) | (b1[k] & m);
        }
        // the sync byte consumed before payload byte J' = J + es (bbheader:675-677), counted here for es in
        // [1, 16] (the window holds it: window byte o + es); J' = J itself was the previous piece's es = 16 (or
        // the header piece's)
        if (io.sync_err && R.live && es <= 16 && P0 - 10 + es < npay &&
            (es < 16 ? byte_of(raw, es) : byte_of(b1, 15)) != 0x47u)
          atomicAdd(io.sync_err, 1u);
        R.sh += 32;
        R.r += 32;
        if (R.r >= 187) {
          R.r -= 187;
          R.sh += 1;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; k++) pd[k] = 0u;
      }
      // the BBHEADER (bbheader:272-325): bytes 0 .. 7 = MATYPE, UPL, DFL, SYNC, SYNCD high (big-endian), byte 8 =
      // SYNCD low, byte 9 = its CRC-8 (the register's LSB first)
      if (P0 == 0) {
        const uint32_t upl = HEM ? 0u : 188u * 8u, dfl = (uint32_t)(d.kbch - 80 - R.g.padding);
        const uint32_t syncb = HEM ? 0u : 0x47u, syncd = R.g.count0 == 0 ? 0u : (uint32_t)(188 - R.g.count0) * 8u;
        const uint64_t hw = ((uint64_t)(uint32_t)d.matype << 48) | ((uint64_t)upl << 32) | ((uint64_t)dfl << 16) |
                            ((uint64_t)syncb << 8) | (uint64_t)(syncd >> 8);
        uint32_t c = HEM ? 0x80u : 0u;
#pragma unroll
        for (int b = 0; b < 8; b++) c ^= hd[b * 256 + ((hw >> (56 - 8 * b)) & 0xFF)];
        c ^= hd[8 * 256 + (syncd & 0xFF)];
        pd[0] = __builtin_bswap32((uint32_t)(hw >> 32));
        pd[1] = __builtin_bswap32((uint32_t)hw);
        pd[2] = (pd[2] & 0xFFFF0000u) | (syncd & 0xFFu) | ((__builtin_bitreverse32(c) >> 24) << 8);
        if (HEM) {   // payload bytes 0 .. 5 from the stream; the sync bytes before payload bytes J0 .. J0 + 6 (the
                     // tracked pieces count from J0 + 7 on)
#pragma unroll 1
          for (int i = 10; i < 17; i++) {
            const int64_t J = R.g.J0 + (i - 10);
            if (i < 16) set_byte(pd, i, R.live && i - 10 < npay ? (uint32_t)R.tin[payload_pos(J, 1) - io.ts_base] : 0u);
            if (io.sync_err && R.live && i - 10 < npay && J % 187 == 0 && R.tin[188 * (J / 187) - io.ts_base] != 0x47)
              atomicAdd(io.sync_err, 1u);
          }
        }
      }
      // past the payload: the in-band type B field (first BBFRAME of an interleaving frame), then zeros
      if (P0 + 16 > 10 + npay) {
#pragma unroll 1
        for (int i = max(0, 10 + npay - P0); i < 16; i++) {
          const int k = P0 + i - 10 - npay;
          set_byte(pd, i, R.g.padding && k < 13 ? (uint32_t)ibb[k] : 0u);
        }
      }
      // BB scrambling: this half's 16 PRBS bytes, loaded with the window (unconditional: past the BBFRAME the PRBS
      // padding is zero, t2_plan FecPlan::prbs_bytes)
#pragma unroll
      for (int k = 0; k < 4; k++) pd[k] ^= w.p[k];
      // (a dead row's piece is garbage: it goes to the spare row, and its own accumulator rows are never written out)
    };
    // the window the piece of chunk q needs (requested a chunk ahead)
    // (the PRBS half as a vector load with the window: two uniform scalar loads and a per-lane select cost 12
    // VALU per chunk; the chunk index is clamped to the segment, the windows past it are never built)
    auto prbs = [&](int c, TsWin &w) {
      const u32x4 v = ((const __attribute__((address_space(1))) u32x4 *)(uintptr_t)prbs16)[2 * min(c, q1 - 1) + h];
#pragma unroll
      for (int k = 0; k < 4; k++) w.p[k] = v[k];
    };
    auto fetch = [&](int q) -> TsWin {   // every lane loads (dead rows from a safe address): no branch to merge
      TsWin w = ts_fetch<HEM>(R.tin, io.ts_len, HEM ? R.sh - io.ts_base : R.rel);
      prbs(q, w);
      return w;
    };
    // the piece one chunk after the cursor's (the cursor is at the next chunk to build)
    auto fetch2 = [&](int c) -> TsWin {   // c = the chunk after the cursor's
      const int64_t rel = HEM ? R.sh + 32 + (R.r + 32 >= 187 ? 1 : 0) - io.ts_base : R.rel + 32;
      TsWin w = ts_fetch<HEM>(R.tin, io.ts_len, rel);
      prbs(c, w);
      return w;
    };

    bch_v16f acc[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] = bch_v16f{};
    uint32_t a[4];
    // the TS windows two chunks deep in two named slots, the chunk loop unrolled by two so that they trade roles
    // (one slot and a copy at the loop's end: the copy waited for the window's load with vmcnt(0), draining the
    // BBFRAME stores issued after it)
    TsWin w0, w1;
    {
      const bfr_t bs = bload(q0);
      w0 = fetch(q0);
      build(q0, w0, a);
      w1 = fetch(q0 + 1);
      __syncthreads();   // the previous segment's epilogue has read its parity words out of buffer 0
      bstore(0, bs);
    }
    __syncthreads();
    // chunk q: wn holds the window of chunk q + 1 (loaded a chunk ago), wl receives chunk q + 2's
    auto chunk = [&](int q, const TsWin &wn, TsWin &wl) {
      const int cur = (q - q0) & 1, qn = min(q + 1, q1 - 1);
      // the next chunk's B fragments and TS window, unconditionally (the last chunk's repeated, unused): an array
      // assigned under a condition and kept across it is not promoted to registers
      const bfr_t bs = bload(qn);
      wl = fetch2(q + 2);
      // this chunk's piece into the staging lines; after every 4th chunk (and the segment's last) each wave stores
      // its 32 rows' staged bytes as whole 128-byte lines, after the next chunk's loads: vmcnt retires in order,
      // so waiting for those loads (the build of q + 1, the B writes) does not drain these stores.  Every lane
      // stores (dead rows into the spare row nblocks of the buffer, masked parts to their own bytes again): a store
      // the wave may branch around would make the compiler's wait for the B loads a vmcnt(0) that drains it.
      *(uint4 *)(stg + (wave * 32 + (lane & 31)) * BBCH_STG_STRIDE + (q & 3) * 32 + h * 16) =
          make_uint4(a[0], a[1], a[2], a[3]);
      if ((q & 3) == 3 || q == q1 - 1) {
        const int qa = max(q0, q & ~3);   // the group's first chunk this segment wrote
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int r = 8 * k + (lane >> 3), part = lane & 7;   // 8 lanes per row, 16 bytes each
          const uint4 v = *(const uint4 *)(stg + (wave * 32 + r) * BBCH_STG_STRIDE + part * 16);
          const int c = (q & ~3) + (part >> 1);                  // the chunk of this part
          const int rb = row0 + r;
          const bool ok = rb < io.nblocks && c >= qa && c <= q && 32 * c + 16 * (part & 1) < L;
          // (row x stride as one 32 x 32 -> 64-bit multiply)
          uint8_t *dst = io.out + (uint64_t)(uint32_t)(ok ? rb : io.nblocks) * (uint32_t)io.cw_stride +
                         (int64_t)32 * (q & ~3) + 16 * part;
          // nontemporal: 1.2 GB of BBFRAME lines per 1280 cfg3 frames written through L2 evicted the generator-table
          // slices (FETCH_SIZE 1.145e6 -> 0.897e6 KiB per launch with these stores; FEC 1.283 -> 1.254 ms)
          __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, (u32x4 *)dst);
        }
      }
      const uint4 *bq = bsm + cur * PER;
      uint4 bc[NT], bx[NT];
#pragma unroll
      for (int t = 0; t < NT; t++) bc[t] = bq[t * 64 + lane];
#pragma unroll
      for (int s = 0; s < 4; s++) {
        if (s < 3) {
#pragma unroll
          for (int t = 0; t < NT; t++) bx[t] = bq[((s + 1) * NT + t) * 64 + lane];
        }
        // the message bits in place where fp4 allows (dword d = bits d of each nibble: 0.5, 1.0, 2.0; bit 3 is
        // the sign, so d = 3 moves down one), B's set entries 2.0, 1.0, 0.5, 0.5 (t2_plan build_bch_mfma): five
        // VALU per K-step instead of seven
        const uint32_t w = a[s];
        const bch_v8i A = {(int)(w & 0x11111111u), (int)(w & 0x22222222u), (int)(w & 0x44444444u),
                           (int)((w >> 1) & 0x44444444u), 0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < NT; t++) {
          const bch_v8i Bv = {(int)bc[t].x, (int)bc[t].y, (int)bc[t].z, (int)bc[t].w, 0, 0, 0, 0};
          acc[t] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, Bv, acc[t], 4, 4, 0, 127, 0, 127);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < NT; t++) bc[t] = bx[t];
      }
      // the MFMAs stay here, before the next piece's build: left alone, the compiler sinks them below it and
      // hoists every B-fragment read above it (all 4 K-steps' fragments live across the build: ~80 VGPRs)
#pragma unroll
      for (int t = 0; t < NT; t++) asm volatile("" : "+v"(acc[t]));
      if (q + 1 < q1) build(q + 1, wn, a);
      bstore(cur ^ 1, bs);   // the other buffer was last read before the previous barrier
      __syncthreads();
    };
    int q = q0;
    for (; q + 1 < q1; q += 2) {
      chunk(q, w1, w0);
      chunk(q + 1, w0, w1);
    }
    if (q < q1) chunk(q, w1, w0);
    // partial parities
    uint32_t *pw = (uint32_t *)bsm + wave * 32 * BCH_PART_WORDS;   // after the loop's last barrier
#pragma unroll
    for (int t = 0; t < NT; t++)
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const uint64_t m = __builtin_amdgcn_ballot_w64(((int)acc[t][r] & 1) != 0);
        const int row = (r & 3) + 8 * (r >> 2);
        if (lane == 0) pw[row * BCH_PART_WORDS + t] = __builtin_bswap32(__builtin_bitreverse32((uint32_t)m));
        if (lane == 1) pw[(row + 4) * BCH_PART_WORDS + t] = __builtin_bswap32(__builtin_bitreverse32((uint32_t)(m >> 32)));
      }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int i = lane; i < 32 * BCH_PART_WORDS; i += 64) {
      const int row = i / BCH_PART_WORDS, t = i % BCH_PART_WORDS;
      if (t < NT && row0 + row < io.nblocks) atomicXor(&io.bch_part[(int64_t)(row0 + row) * BCH_PART_WORDS + t], pw[i]);
    }
  }
}

// chain pass 3: info bytes [0, L) from the codeword row + the BCH parity (the XOR of the K slices),
// the info groups laid out, LDPC, then the interleaver-input words from word L / 4 on (the BB pass
// wrote the words before): BCH parity | LDPC parity (parity interleaved: byte m = byte m % 45 of row
// m / 45, or natural order a + q c for QPSK without parity interleaving)
// word i (bytes 4 i .. 4 i + 3, little-endian as stored) of block's interleaver-input codeword: the
// BBFRAME and BCH parity bytes from frame, then the LDPC parity rows cur (fec_ldpc), parity-interleaved
// (byte m = byte m mod 45 of row m / 45) by byte-aligning two row words where the code has the parity
// interleaver, bit by bit otherwise; zero past the codeword
// The rows come without the column-parity correction (fec_ldpc<.., false>): word w of every row is XORed with
// Wv[w] here, where it is read, instead of by a read-modify-write pass over all q x 12 row words.
__device__ __forceinline__ uint32_t ldpc_out_word(const FecDev &d, const uint8_t *frame, const uint32_t *cur,
                                                  const uint32_t *Wv, int i) {
  const int NB = d.nbch >> 3, cwb = d.nldpc >> 3, q = d.q;
  auto parity_byte = [&](int m) -> uint32_t {
    if (d.parity_il) {
      const int a = m / 45, k = m - 45 * a;
      return ((cur[a * 12 + (k >> 2)] ^ Wv[k >> 2]) >> (24 - 8 * (k & 3))) & 0xFFu;
    }
    uint32_t v = 0;
    for (int e = 0; e < 8; e++) {
      const int j = 8 * m + e, a = j % q, c = j / q;
      v |= (((cur[a * 12 + (c >> 5)] ^ Wv[c >> 5]) >> (31 - (c & 31))) & 1u) << (7 - e);
    }
    return v;
  };
  if (4 * i + 4 <= NB) return ((const uint32_t *)frame)[i];
  uint32_t v = 0;
  if (d.parity_il && 4 * i >= NB && 4 * i + 4 <= cwb) {
    // four parity bytes m .. m + 3 = bytes k .. k + 3 of row a (m = 45 a + k; rows of 12 big-endian words,
    // bytes 45 .. 47 zero): one byte align of two row words, plus, for k >= 42, the first 45 - k .. 3 bytes
    // of row a + 1 shifted in (no per-byte loop: 3 of the 45 offsets cross a row, so nearly every wave has a
    // lane there)
    const int a = (4 * i - NB) / 45, k = 4 * i - NB - 45 * a, c = k >> 2;
    const uint32_t w0 = cur[a * 12 + c] ^ Wv[c], w1 = c < 11 ? cur[a * 12 + c + 1] ^ Wv[c + 1] : 0u;
    uint32_t x = (k & 3) ? __builtin_amdgcn_alignbyte(w0, w1, (uint32_t)(4 - (k & 3))) : w0;
    if (k >= 42 && a + 1 < q) x |= (cur[(a + 1) * 12] ^ Wv[0]) >> (8 * (45 - k));
    return __builtin_bswap32(x);
  }
  for (int e = 0; e < 4; e++) {
    const int bidx = 4 * i + e;
    const uint32_t by = bidx < NB ? (uint32_t)frame[bidx] : bidx < cwb ? parity_byte(bidx - NB) : 0u;
    v |= by << (8 * e);
  }
  return v;
}

// resident FEC workgroups for a persistent launch: per_cu per CU of the current device
static int fec_grid(int nblocks, int per_cu) {
  static std::atomic<int> ncu[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  int n = ncu[dev].load(std::memory_order_relaxed);
  if (!n) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    ncu[dev].store(n, std::memory_order_relaxed);
  }
  return nblocks < n * per_cu ? nblocks : n * per_cu;
}

static bool fec_plan_fits(const FecDev &d) {
  // the LDS carve is sized for the standard codes, the BCH wave for 64 chunks: refuse anything else
  return !(d.nent > FEC_MAX_ENT || d.q > 128 || d.nbch > 8 * FEC_FRAME_BYTES || 4 * FEC_DW_PASS * (d.nbch / 360) + 48 * d.q > FEC_LDPC_BYTES ||
           (d.kbch - 80) / 8 + 218 > 16 * FEC_PRE * FEC_THREADS || ((d.kbch >> 3) + 15) / 16 > FEC_PRE * FEC_THREADS ||
           (d.P != 192 && d.P != 168 && d.P != 160 && d.P != 128) || d.chunk * 64 < d.kbch / 8);
}

// persistent launch of one FEC kernel kind: as many workgroups per CU as its LDS carve allows, up
// to cap
static hipError_t fec_launch_persistent(const void *fn, int kind, int cap, const FecDev &d, const FecIO &io,
                                        hipStream_t s) {
  const int lds = fec_carve(kind, d.kbch, d.nbch, d.q).total;
  int per_cu = (160 * 1024) / lds;
  per_cu = per_cu < 1 ? 1 : per_cu > cap ? cap : per_cu;
  void *args[2] = {(void *)&d, (void *)&io};
  return hipLaunchKernel(fn, dim3(fec_grid(io.nblocks, per_cu)), dim3(FEC_THREADS), args, lds, s);
}

template <int NT>
static hipError_t bbch_launch(const FecDev &d, const FecIO &io, hipStream_t s) {
  const int lds = bbch_lds(NT);
  const void *fn = d.hem ? (const void *)bbch_kernel<NT, true> : (const void *)bbch_kernel<NT, false>;
  hipError_t e = lds_limit(fn, lds);
  if (e != hipSuccess) return e;
  // persistent: BBCH_WG_PER_CU workgroups per CU, a multiple of BCH_KS (slices by XCD)
  const int per_slice = (fec_grid(1 << 30, BBCH_WG_PER_CU) + BCH_KS - 1) / BCH_KS;
  void *args[2] = {(void *)&d, (void *)&io};
  return hipLaunchKernel(fn, dim3(per_slice * BCH_KS), dim3(BBCH_THREADS), args, lds, s);
}

static bool fec_chain_args_ok(const FecDev &d, const FecIO &io) {
  return d.bch_mfma && io.bch_part && io.bch_part_blocks >= io.nblocks && d.bch_nt >= 4 && d.bch_nt <= 6 && io.ts_len >= 64 &&
         d.bch_nq >= 1 && d.bch_nq * 32 <= io.cw_stride;
}

hipError_t launch_fec(int mode, const FecDev &d, const FecIO &io, hipStream_t s) {
  if (io.nblocks <= 0) return hipSuccess;
  if (!fec_plan_fits(d)) return hipErrorInvalidValue;
  switch (mode) {
    case FEC_TS_TO_BBFRAME:   // the chain: BB + BCH on the matrix cores in one pass (the LDPC follows in launch_ldpc_map)
      if (!fec_chain_args_ok(d, io)) return hipErrorInvalidValue;
      return d.bch_nt == 6 ? bbch_launch<6>(d, io, s) : d.bch_nt == 5 ? bbch_launch<5>(d, io, s) : bbch_launch<4>(d, io, s);
    case FEC_TS_TO_BITS:
      return fec_launch_persistent((const void *)fec_kernel<FEC_TS_TO_BITS>, CARVE_FUSED, FEC_WG_PER_CU, d, io, s);
    default:
      return fec_launch_persistent((const void *)fec_kernel<FEC_BITS_TO_BITS>, CARVE_FUSED, FEC_WG_PER_CU, d, io, s);
  }
}

// ============================================================================ map kernel
constexpr int MAP_THREADS = 256;
constexpr int MAP_LDS_MAX = 160 * 1024 - 256;
// block API LDS: [LUT 2 KB][cell indices, cs bytes][codeword as big-endian words + a slack word]
// (<= 43 KB for QPSK normal); the chain's ldpc_map_kernel carves its own
__host__ __device__ inline int map_idx_bytes(int cs) { return (cs + 15) & ~15; }
__host__ __device__ inline int map_smem(int cs, int nldpc) { return 2048 + map_idx_bytes(cs) + ((nldpc / 8 + 4 + 15) & ~15); }

// XCD-aware block order: the hardware deals consecutive workgroups round-robin over the 8 XCDs;
// give each XCD a contiguous run of logical blocks so neighbours share its L2.
__device__ __forceinline__ int xcd_major(int i, int n) {
  const int q = n >> 3;
  return i < (q << 3) ? (i & 7) * q + (i >> 3) : i;
}

// column twist + demux of one FEC block: interleaver-input bits (big-endian words cww, one word of
// slack past the end) -> cell indices idx (one byte per cell)
template <int NT>
__device__ void map_cells(const MapDev &d, const uint32_t *cww, uint8_t *idx, int tid) {
  const int cs = d.cs;
  // ---- cell indices: column-twist write / row read / demux (interleavermod:351-403, 440-500,
  //      529-598, 626-677).  One thread per 8 rows: each column's 8 bits are one (twisted,
  //      wrapping) window of the codeword, the W windows are ordered by demuxed bit position and
  //      transposed as a bit matrix, giving each row's demuxed word directly.
  if (d.mode == 0) {
    // QPSK: cell j = codeword bits 2j, 2j+1 (no bit interleaving, interleavermod:309-314)
    uint32_t *idxw = (uint32_t *)idx;
    for (int w = tid; w < (cs + 3) >> 2; w += NT) {
      const uint32_t word = cww[w >> 2], sh = 24u - 8u * (uint32_t)(w & 3);
      const uint32_t byte = (word >> sh) & 0xFFu;   // cells 4w..4w+3
      idxw[w] = ((byte >> 6) & 3u) | (((byte >> 4) & 3u) << 8) | (((byte >> 2) & 3u) << 16) | ((byte & 3u) << 24);
    }
  } else {
    const int R = d.R, mod = d.mod;
    auto window = [&](int s) -> uint32_t {    // codeword bits [s, s + 32), MSB first
      const uint64_t v = ((uint64_t)cww[s >> 5] << 32) | cww[(s >> 5) + 1];
      return (uint32_t)((v << (s & 31)) >> 32);
    };
    // 8-bit transpose (Hacker's Delight transpose8): bit 8 i + j <-> bit 8 j + i
    auto tr8 = [](uint64_t x) -> uint64_t {
      uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
      x ^= t ^ (t << 7);
      t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
      x ^= t ^ (t << 14);
      t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
      x ^= t ^ (t << 28);
      return x;
    };
    // one thread per 16 rows (two 8-row groups g = 2 g2, 2 g2 + 1): byte b of xa / xb = the 8 bits of
    // the column feeding bit b in rows 16 g2 .. + 7 / + 8 .. + 15 (row k at bit 7 - k), both cut from
    // one 32-bit window; after the transpose byte 7 - k holds row k's demuxed bits b
    uint32_t *idxw = (uint32_t *)idx;
    auto emit = [&](int g, uint64_t lo, uint64_t hi) {
      const int j0 = 8 * g;
      if (d.mode == 1) {                         // two cells per row: pack >> mod, pack & (2^mod - 1)
        const uint32_t lo_mask = (1u << mod) - 1u;
        uint32_t wq[4];
        if (mod == 8) {
          // 256-QAM: the row's two cells are byte k of hi and byte k of lo, so each word of four cells
          // is one byte permute of a half of hi and a half of lo (v_perm: selector bytes 4..7 pick
          // the first operand's bytes, 0..3 the second's)
          const uint32_t lh = (uint32_t)(lo >> 32), hh = (uint32_t)(hi >> 32), ll = (uint32_t)lo, hl = (uint32_t)hi;
          wq[0] = __builtin_amdgcn_perm(hh, lh, 0x02060307u);
          wq[1] = __builtin_amdgcn_perm(hh, lh, 0x00040105u);
          wq[2] = __builtin_amdgcn_perm(hl, ll, 0x02060307u);
          wq[3] = __builtin_amdgcn_perm(hl, ll, 0x00040105u);
        } else {
#pragma unroll
          for (int qd = 0; qd < 4; qd++) {
            const int k0 = 2 * qd;
            const uint32_t p0 = (uint32_t)((lo >> (8 * (7 - k0))) & 0xFFu) | (uint32_t)(((hi >> (8 * (7 - k0))) & 0xFFu) << 8);
            const uint32_t p1 = (uint32_t)((lo >> (8 * (6 - k0))) & 0xFFu) | (uint32_t)(((hi >> (8 * (6 - k0))) & 0xFFu) << 8);
            wq[qd] = (p0 >> mod) | ((p0 & lo_mask) << 8) | ((p1 >> mod) << 16) | ((p1 & lo_mask) << 24);
          }
        }
        // one 16-byte LDS write of the group's four words (four b32 writes at a lane stride of 8 words
        // were 8-way bank conflicts); the last group's rows past R bytewise-guarded
        if (j0 + 6 < R) {
          *(uint4 *)(idxw + 4 * g) = make_uint4(wq[0], wq[1], wq[2], wq[3]);
        } else {
#pragma unroll
          for (int qd = 0; qd < 4; qd++)
            if (j0 + 2 * qd < R) idxw[4 * g + qd] = wq[qd];
        }
      } else {                                   // 256-QAM short: one cell per row (byte-reversed lo)
        const uint64_t rv = __builtin_bswap64(lo);
        if (j0 + 4 < R) {
          *(uint2 *)(idxw + 2 * g) = make_uint2((uint32_t)rv, (uint32_t)(rv >> 32));
        } else if (j0 < R) {
          idxw[2 * g] = (uint32_t)rv;
        }
      }
    };
    for (int g2 = tid; g2 < (R + 15) >> 4; g2 += NT) {
      const int j0 = 16 * g2;
      // xa / xb dword q: byte i = bits 31..24 / 23..16 of column 4 q + i's window, assembled with byte
      // permutes (four per four columns) instead of a shift and an OR per byte
      uint32_t xa[4], xb[4];
#pragma unroll
      for (int qd = 0; qd < 4; qd++) {
        uint32_t win[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int b = 4 * qd + i;
          const int2 cw = kc(d.col, b);   // scalar (SMEM) loads at the point of use
          const int c0 = cw.x;
          win[i] = 0u;
          if (c0 < 0) continue;
          int off = j0 - cw.y;
          off += off < 0 ? R : 0;
          win[i] = window(c0 + off);
          if (off + 16 > R) {                    // the column wraps inside these 16 rows
            const int n1 = R - off;
            win[i] = (win[i] & ~(0xFFFFFFFFu >> n1)) | (window(c0) >> n1);
          }
        }
        const uint32_t t = __builtin_amdgcn_perm(win[1], win[0], 0x06020703u);   // w0.b3 w1.b3 w0.b2 w1.b2
        const uint32_t u = __builtin_amdgcn_perm(win[3], win[2], 0x06020703u);   // w2.b3 w3.b3 w2.b2 w3.b2
        xa[qd] = __builtin_amdgcn_perm(u, t, 0x05040100u);
        xb[qd] = __builtin_amdgcn_perm(u, t, 0x07060302u);
      }
      const uint64_t xa0 = xa[0] | ((uint64_t)xa[1] << 32), xa1 = xa[2] | ((uint64_t)xa[3] << 32);
      const uint64_t xb0 = xb[0] | ((uint64_t)xb[1] << 32), xb1 = xb[2] | ((uint64_t)xb[3] << 32);
      emit(2 * g2, tr8(xa0), d.W > 8 ? tr8(xa1) : 0ull);
      emit(2 * g2 + 1, tr8(xb0), d.W > 8 ? tr8(xb1) : 0ull);
    }
  }
}

// Chain: the cell interleaver (framemapper:1973-1998) and the time-interleaver store (:1999-2028) in one
// pass, in stored-slot order, in aligned quads of four frame slots (MapDev::slot_quad): wave w takes
// 64-quad chunks c = c0 + u NT / 64 + w and lane l quad 64 c + l, whose four slots list the
// cell-interleaver INPUT index j of the cell landing there (the chain composes j = CI^-1(t) for the
// block's shift); the slot gets (idx[j], idx[j - 1]) under rotation (the rotated constellation's Q
// delay; the QAM lookup is fused into the OFDM kernel's bin scatter), else (idx[j], idx[j]).  One
// 8-byte store per full quad (2-byte stores for a quad at a run's edge, whose other slots belong to
// neighbouring blocks), so a store instruction writes 512 B of one or two contiguous runs.
// idx[-1] holds a copy of idx[cs - 1] under rotation (the caller's), so idx[j - 1] needs no wrap: both
// bytes are one address and two offsets, and a slot of another block is a flag bit of its entry rather
// than a sentinel index (three VALU per slot instead of ~11).
// rounds of MQ chunks per wave (chunk c0 + u NW + wv): one round for a normal block (<= 36 chunks; the
// wave-uniform clamp repeats a chunk without storing it), its table loads all in flight together
constexpr int MQ = 9;
struct QuadRound {
  uint2 e[MQ];
  uint32_t qa[MQ];
};
template <int NT>
__device__ __forceinline__ void map_quads_load(const MapDev &d, int blk, int tid, int c0, QuadRound &R) {
  const int r = blk % d.F;
  const uint2 *qs = d.slot_quad + (int64_t)r * d.slot_stride;
  const uint16_t *qo = d.slot_qoff + (int64_t)r * d.slot_stride;
  const int32_t *qb = d.slot_qbase + (int64_t)r * (d.slot_stride >> 6);
  const int nqd = kc(d.slot_nq, r);
  constexpr int NW = NT / 64;
  // the wave index as a scalar (readfirstlane): the chunk c derived from it is then wave-uniform for the compiler,
  // so kc(qb, c) is a scalar load (with tid >> 6 in a VGPR it was a vector load and its address math, per quad)
  const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6), nch = (nqd + 63) >> 6;
#pragma unroll
  for (int u = 0; u < MQ; u++) {
    const int c = min(c0 + u * NW + wv, nch - 1);   // wave-uniform
    R.e[u] = ld_off(qs, (uint32_t)(64 * c + lane) * 8u);
    R.qa[u] = (uint32_t)kc(qb, c) + (uint32_t)ld_off(qo, (uint32_t)(64 * c + lane) * 2u);
  }
}
// pre: the first round's table entries, loaded by the caller earlier (map_quads_load with c0 = 0), or null
template <int NT, bool ROT>
__device__ void map_store_quads(const MapDev &d, uint16_t *out_pairs, int64_t frame_stride, const uint8_t *idx,
                                int blk, int tid, const QuadRound *pre = nullptr) {
  const int r = blk % d.F;
  uint16_t *dst = out_pairs + (int64_t)(blk / d.F) * frame_stride;   // frame data region
  const int nqd = kc(d.slot_nq, r);
  constexpr int NW = NT / 64;
  // the wave index as a scalar (readfirstlane): the chunk c derived from it is then wave-uniform for the compiler,
  // so kc(qb, c) is a scalar load (with tid >> 6 in a VGPR it was a vector load and its address math, per quad)
  const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6), nch = (nqd + 63) >> 6;
  const uint8_t *ib = idx - 1;   // ib[j + 1] = idx[j], ib[j] = idx[j - 1]
  // entry bits 0..14: j; bit 15: another block's slot (j = 0 then, read and dropped)
  auto pair_of = [&](uint32_t j) -> uint32_t {
    const uint8_t *p = ib + j;
    return ROT ? (uint32_t)p[1] | ((uint32_t)p[0] << 8) : (uint32_t)p[1] * 0x101u;
  };
  for (int c0 = 0; c0 < nch; c0 += MQ * NW) {
    QuadRound R;
    if (c0 == 0 && pre)
      R = *pre;
    else
      map_quads_load<NT>(d, blk, tid, c0, R);
    // every table load lands here, before the first store: a load the compiler sinks into a store
    // branch is waited for with vmcnt(0), which also drains every store issued before it
#pragma unroll
    for (int u = 0; u < MQ; u++) asm volatile("" : "+v"(R.e[u].x), "+v"(R.e[u].y), "+v"(R.qa[u]));
#pragma unroll
    for (int u = 0; u < MQ; u++) {
      const int c = c0 + u * NW + wv;
      const uint2 e = R.e[u];
      const uint32_t j0 = e.x & 0x7FFFu, j1 = (e.x >> 16) & 0x7FFFu, j2 = e.y & 0x7FFFu, j3 = (e.y >> 16) & 0x7FFFu;
      const uint2 v = make_uint2(pair_of(j0) | (pair_of(j1) << 16), pair_of(j2) | (pair_of(j3) << 16));
      if (c < nch && 64 * c + lane < nqd) {
        if (!((e.x | e.y) & 0x80008000u)) {
          st_off((uint2 *)dst, R.qa[u] * 8u, v);
        } else {
          if (!(e.x & 0x8000u)) st_off(dst, (4u * R.qa[u] + 0u) * 2u, (uint16_t)v.x);
          if (!(e.x & 0x80000000u)) st_off(dst, (4u * R.qa[u] + 1u) * 2u, (uint16_t)(v.x >> 16));
          if (!(e.y & 0x8000u)) st_off(dst, (4u * R.qa[u] + 2u) * 2u, (uint16_t)v.y);
          if (!(e.y & 0x80000000u)) st_off(dst, (4u * R.qa[u] + 3u) * 2u, (uint16_t)(v.y >> 16));
        }
      }
    }
  }
}

// ============================================================================ L1-post
// One 256-thread workgroup per T2 frame of the launch: that frame's L1-post cells
// (framemapper:1536-1910) from the t2_plan L1PostPlan.  The codeword lives in LDS as 16200 bits
// packed MSB first: information bits 0..7031 (shortened positions zero), BCH parity 7032..7199,
// LDPC parity 7200..16199 (word-aligned at word 225).
constexpr int L1_NT = 256, L1_CW_WORDS = (16200 + 31) / 32, L1_SIG_WORDS = 64;   // <= 2048 signal bits

__device__ __forceinline__ uint32_t l1_bit(const uint32_t *w, int i) { return (w[i >> 5] >> (31 - (i & 31))) & 1u; }

// XOR of v over the workgroup (every thread gets the result); red: L1_NT / 64 words of LDS
__device__ __forceinline__ uint32_t l1_xor_all(uint32_t v, uint32_t *red, int tid) {
  v = rd_lane_u32(wave_prefix_xor(v), 63);
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
#pragma unroll
  for (int k = 0; k < L1_NT / 64; k++) t ^= red[k];
  return t;
}

// LDS words the L1-post of one frame needs (codeword, signal bits, reduction scratch)
constexpr int L1_LDS_WORDS = L1_CW_WORDS + L1_SIG_WORDS + L1_NT / 64 * 6;

// frame f's L1-post cells by one 256-thread workgroup; lds: L1_LDS_WORDS words
__device__ void l1post_frame(const L1Dev &d, const L1IO &io, int f, uint32_t *lds) {
  uint32_t *cw = lds, *sig = lds + L1_CW_WORDS, *red = sig + L1_SIG_WORDS;
  const int tid = threadIdx.x;
  const int64_t frame = io.first_frame + (io.frames_per_stream ? f % io.frames_per_stream : f);
  const uint32_t fidx = (uint32_t)(frame % d.t2frames);   // FRAME_IDX = t2_frame_num (:1648-1651)
  const int nsw = (d.nsig + 31) >> 5, L = d.nsig - 32;
  const uint32_t *tmpl = d.tmpl + (d.ncls > 1 ? (int)(fidx % (uint32_t)d.ncls) * nsw : 0);   // the frame's class
  for (int w = tid; w < L1_CW_WORDS; w += L1_NT) cw[w] = 0;
  // signal bits: the template with this frame's FRAME_IDX (8 bits, MSB first, at fidx_pos)
  if (tid < nsw) {
    uint32_t v = tmpl[tid];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int p = d.fidx_pos + k;
      if ((p >> 5) == tid && ((fidx >> (7 - k)) & 1u)) v |= 1u << (31 - (p & 31));
    }
    sig[tid] = v;
  }
  __syncthreads();
  // CRC-32 (:1203-1224) over the first L bits: crc_k ^ XOR of the set bits' contributions
  uint32_t c = 0;
  for (int i = tid; i < L; i += L1_NT)
    if (l1_bit(sig, i)) c ^= d.crc_c[i];
  const uint32_t crc = d.crc_k ^ l1_xor_all(c, red, tid);
  if (tid < 32 && ((crc >> (31 - tid)) & 1u)) atomicOr(&sig[(L + tid) >> 5], 1u << (31 - ((L + tid) & 31)));
  __syncthreads();
  if (d.scr && tid < nsw) sig[tid] ^= d.scr[tid];   // L1 scrambler (:1928-1940), v1.3.1
  __syncthreads();
  // shortening: signal bit i -> information position sig_pos[i]; BCH(168) parity = XOR of the
  // per-position remainders of the set bits (6 words, parity bit n at word n / 32, MSB first)
  uint32_t b[6] = {0, 0, 0, 0, 0, 0};
  for (int i = tid; i < d.nsig; i += L1_NT) {
    if (!l1_bit(sig, i)) continue;
    const int pos = d.sig_pos[i];
    atomicOr(&cw[pos >> 5], 1u << (31 - (pos & 31)));
#pragma unroll
    for (int k = 0; k < 6; k++) b[k] ^= d.bch_r[i * 6 + k];
  }
#pragma unroll
  for (int k = 0; k < 6; k++) b[k] = rd_lane_u32(wave_prefix_xor(b[k]), 63);
  if ((tid & 63) == 0)
#pragma unroll
    for (int k = 0; k < 6; k++) red[(tid >> 6) * 6 + k] = b[k];
  __syncthreads();
  if (tid < 168) {
    uint32_t w = 0;
#pragma unroll
    for (int r = 0; r < L1_NT / 64; r++) w ^= red[r * 6 + (tid >> 5)];
    if ((w >> (31 - (tid & 31))) & 1u) {
      const int pos = 7032 + tid;
      atomicOr(&cw[pos >> 5], 1u << (31 - (pos & 31)));
    }
  }
  __syncthreads();
  // LDPC (:1314-1364): information bit 360 g + n feeds parity (x + n q) mod pbits for each address x
  // of group g; only the signal positions and the BCH parity can be set
  uint32_t *par = cw + 225;
  for (int i = tid; i < d.nsig + 168; i += L1_NT) {
    const int pos = i < d.nsig ? (int)d.sig_pos[i] : 7032 + (i - d.nsig);
    if (!l1_bit(cw, pos)) continue;
    const int g = pos / 360, n = pos - 360 * g;
    for (int e = d.ldpc_ptr[g]; e < d.ldpc_ptr[g + 1]; e++) {
      const int j = (d.ldpc_addr[e] + n * d.q) % d.pbits;
      atomicXor(&par[j >> 5], 1u << (31 - (j & 31)));
    }
  }
  __syncthreads();
  // accumulate p[j] ^= p[j - 1]: inclusive prefix XOR within each word (from the MSB), then the
  // exclusive prefix of the word parities over the wave, five words per lane
  if (tid < 64) {
    const int nwp = (d.pbits + 31) >> 5, per = (nwp + 63) / 64;
    uint32_t x[5], par_l = 0;
#pragma unroll
    for (int k = 0; k < 5; k++) {
      const int w = tid * per + k;
      uint32_t v = (k < per && w < nwp) ? par[w] : 0u;
      v ^= v >> 1; v ^= v >> 2; v ^= v >> 4; v ^= v >> 8; v ^= v >> 16;
      x[k] = v;
      par_l ^= v & 1u;   // the word's total parity sits in its last bit
    }
    const uint32_t before = wave_prefix_xor(par_l) ^ par_l;
    uint32_t carry = before;
#pragma unroll
    for (int k = 0; k < 5; k++) {
      const int w = tid * per + k;
      if (k < per && w < nwp) par[w] = carry ? ~x[k] : x[k];
      carry ^= x[k] & 1u;
    }
  }
  __syncthreads();
  // puncture / select the N_post transmitted bits and map them (BPSK, QPSK, or the 16/64QAM column
  // interleaver + demux, :1832-1908)
  float2 *out = io.out + (int64_t)f * io.out_stride;
  for (int cidx = tid; cidx < d.lp; cidx += L1_NT) {
    float2 v;
    if (d.mode == 0) {
      v = make_float2(l1_bit(cw, d.sel[cidx]) ? -1.0f : 1.0f, 0.0f);
    } else if (d.mode == 1) {
      v = d.lut[(l1_bit(cw, d.sel[2 * cidx]) << 1) | l1_bit(cw, d.sel[2 * cidx + 1])];
    } else {
      const int k = cidx >> 1, half = d.ncols >> 1, e0 = (cidx & 1) ? half : 0;
      uint32_t pack = 0;
      for (int e = e0; e < e0 + half; e++) pack = (pack << 1) | l1_bit(cw, d.sel[d.rows * d.mux[e] + k]);
      v = d.lut[pack];
    }
    out[cidx] = v;
  }
}

__global__ __launch_bounds__(L1_NT) void l1post_kernel(L1Dev d, L1IO io) {
  __shared__ uint32_t lds[L1_LDS_WORDS];
  l1post_frame(d, io, blockIdx.x, lds);
}

static bool l1_args_ok(const L1Dev &d) {
  return d.nsig <= 32 * L1_SIG_WORDS && d.nsig >= 33 && d.pbits == 9000 && d.q > 0 && d.t2frames > 0 && d.ncls > 0 &&
         d.t2frames % d.ncls == 0;
}

hipError_t launch_l1post(const L1Dev &d, const L1IO &io, hipStream_t s) {
  if (io.nframes <= 0) return hipSuccess;
  if (!l1_args_ok(d)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(l1post_kernel, dim3(io.nframes), dim3(L1_NT), 0, s, d, io);
  return hipGetLastError();
}

// Block API (interleavermod): one 256-thread workgroup per FEC block: the natural-order codeword bits
// (one byte per bit; the parity interleaver applied on the read) packed into LDS as big-endian words,
// column twist + demux (map_cells), QAM lookup and the rotated constellation's cyclic Q delay
// (interleavermod:529-598, 626-677) into complex64 cells
__global__ __launch_bounds__(MAP_THREADS) void map_kernel(MapDev d, MapIO io) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, blk = blockIdx.x;
  float2 *lut = (float2 *)smem;
  uint8_t *idx = smem + 2048;
  uint32_t *cww = (uint32_t *)(smem + 2048 + map_idx_bytes(d.cs));
  const int cs = d.cs, nl = d.nldpc, nlw = (nl + 31) >> 5, nbch = d.nbch, q = d.q;
  for (int i = tid; i < 256; i += MAP_THREADS) lut[i] = d.lut[i];
  // bit i of the interleaver input is bit 31 - (i & 31) of word i >> 5
  const uint8_t *src = io.in + (int64_t)blk * nl;
  for (int k = tid; k <= nlw; k += MAP_THREADS) {
    uint32_t v = 0;
    for (int e = 0; e < 32; e++) {
      int i = 32 * k + e, sidx = i;
      if (i >= nl) break;
      if (d.parity_il && i >= nbch) {        // tempu[nbch + 360 t + s] = in[nbch + q s + t]
        int r = i - nbch, t = r / 360, s = r - 360 * t;
        sidx = nbch + q * s + t;
      }
      v |= (uint32_t)(src[sidx] & 1) << (31 - e);
    }
    cww[k] = v;
  }
  __syncthreads();
  map_cells<MAP_THREADS>(d, cww, idx, tid);
  __syncthreads();
  float2 *dst = io.out + (int64_t)blk * cs;
  for (int j = tid; j < cs; j += MAP_THREADS) {
    float2 v = lut[idx[j]];
    if (d.rotation) v.y = lut[idx[j == 0 ? cs - 1 : j - 1]].y;
    dst[j] = v;
  }
}

hipError_t launch_map(const MapDev &d, const MapIO &io, hipStream_t s) {
  if (io.nblocks <= 0) return hipSuccess;
  const int smem = map_smem(d.cs, d.nldpc);
  if (smem > MAP_LDS_MAX) return hipErrorInvalidValue;
  hipError_t e = lds_limit((const void *)map_kernel, MAP_LDS_MAX);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(map_kernel, dim3(io.nblocks), dim3(MAP_THREADS), smem, s, d, io);
  return hipGetLastError();
}

// ============================================================================ chain: LDPC + map
// One 256-thread workgroup per FEC block of the launch (after ceil8(L1 frames) workgroups that generate
// the frames' L1-post cells): the block's BBFRAME and the XOR of its BCH partial
// parities (the BB and matrix-core passes' output) -> LDPC parity (fec_ldpc) -> the interleaver-input
// codeword, built in LDS -> column twist + demux (map_cells) -> cell interleaver + time-interleaver
// store of the index pairs (map_store_quads).  The codeword never goes through HBM (the LDPC stage's
// 8 KB store and the map stage's 8 KB load per normal block); fio.keep_cw (test hook) stores it anyway.
// LDS: the LDPC carve (CARVE_LDPC), then, once the codeword words sit in registers, [codeword as
// big-endian words + a slack word | cell indices] overlaying it.
constexpr int LM_WORDS = 8;   // codeword words per thread: (nldpc / 8 + 3) / 4 <= LM_WORDS FEC_THREADS
__host__ __device__ inline int lm_cww_words(int nldpc) { return ((nldpc + 31) / 32 + 1 + 3) & ~3; }
__host__ __device__ inline int lm_smem(const FecDev &fd, int cs) {
  const int a = fec_carve(CARVE_LDPC, fd.kbch, fd.nbch, fd.q).total, b = 4 * lm_cww_words(fd.nldpc) + map_idx_bytes(cs);
  return a > b ? a : b;
}
static_assert(FEC_THREADS == MAP_THREADS, "ldpc_map_kernel runs the map phases at FEC_THREADS");

__global__ __launch_bounds__(FEC_THREADS, FEC_PASS_WG_PER_CU) void ldpc_map_kernel(FecDev fd, FecIO fio, MapDev md,
                                                                                   MapIO mio, L1Dev l1d, L1IO l1io) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int nl1 = (l1io.nframes + 7) & ~7;
  if ((int)blockIdx.x < nl1) {
    if ((int)blockIdx.x < l1io.nframes) l1post_frame(l1d, l1io, blockIdx.x, (uint32_t *)smem);
    return;
  }
  const int blk = xcd_major((int)blockIdx.x - nl1, (int)gridDim.x - nl1);
  const int L = fd.kbch >> 3, PB = fd.P >> 3;
  const FecCarve cv = fec_carve(CARVE_LDPC, fd.kbch, fd.nbch, fd.q);
  uint8_t *frame = smem + cv.frame;
  uint32_t *ents = (uint32_t *)(smem + cv.ents);
  uint32_t *D = (uint32_t *)(smem + cv.phase);
  uint32_t *Wv = (uint32_t *)(smem + cv.w);
  uint16_t *rowp = (uint16_t *)(smem + cv.rowp);
  const int ngroups = fd.nbch / 360, q = fd.q, nw = ((fd.nldpc >> 3) + 3) >> 2, nqi = (L + 15) >> 4;
  uint8_t *row = fio.out + (int64_t)blk * fio.cw_stride;
  {
    // the BBFRAME's 16-byte units and the BCH partial parity requested before the tables are staged
    const uint4 *rowq = (const uint4 *)row;
    uint4 u[FEC_PRE];
#pragma unroll
    for (int k = 0; k < FEC_PRE; k++)
      u[k] = tid + FEC_THREADS * k < nqi ? rowq[tid + FEC_THREADS * k] : make_uint4(0u, 0u, 0u, 0u);
    const uint32_t par = tid < (PB + 3) >> 2 ? fio.bch_part[(int64_t)blk * BCH_PART_WORDS + tid] : 0u;
    // consumed: zero the words for the next run on this buffer slot (bbch_kernel XOR-accumulates into them)
    if (tid < BCH_PART_WORDS) fio.bch_part[(int64_t)blk * BCH_PART_WORDS + tid] = 0u;
    for (int i = tid; i < fd.nent; i += FEC_THREADS) ents[i] = fd.ldpc_ent[i];
    for (int i = tid; i <= q; i += FEC_THREADS) rowp[i] = fd.ldpc_rowptr[i];
#pragma unroll
    for (int k = 0; k < FEC_PRE; k++)
      if (tid + FEC_THREADS * k < nqi) ((uint4 *)frame)[tid + FEC_THREADS * k] = u[k];
    __syncthreads();   // the 16-byte units past L land before the parity bytes overwrite them
    if (tid < (PB + 3) >> 2)
      for (int k = 0; k < 4 && 4 * tid + k < PB; k++) frame[L + 4 * tid + k] = (uint8_t)(par >> (8 * k));
    __syncthreads();
  }
  // four words of a group per item, one 16-byte LDS write
  for (int it = tid; it < ngroups * (FEC_DW_PASS / 4); it += FEC_THREADS) {
    const int g = it >> 2, k0 = 4 * (it & 3);
    *(uint4 *)(D + g * FEC_DW_PASS + k0) = make_uint4(ldpc_group_val(frame, g, k0), ldpc_group_val(frame, g, k0 + 1),
                                                      ldpc_group_val(frame, g, k0 + 2), ldpc_group_val(frame, g, k0 + 3));
  }
  __syncthreads();
  // rows without the column-parity correction: ldpc_out_word applies Wv as it reads them
  const uint32_t *cur = fec_ldpc<FEC_DW_PASS, false>(fd, D, ngroups, ents, rowp, Wv, tid);
  uint32_t w[LM_WORDS];
#pragma unroll
  for (int k = 0; k < LM_WORDS; k++) {
    const int i = tid + FEC_THREADS * k;
    w[k] = i < nw ? ldpc_out_word(fd, frame, cur, Wv, i) : 0u;
  }
  if (fio.keep_cw) {   // test hook: the row as the three-pass FEC stored it (words below L / 4 hold the BBFRAME)
    uint32_t *dstw = (uint32_t *)row;
#pragma unroll
    for (int k = 0; k < LM_WORDS; k++) {
      const int i = tid + FEC_THREADS * k;
      if (i >= (L >> 2) && i < nw) dstw[i] = w[k];
    }
  }
  __syncthreads();   // the LDPC areas are dead: the codeword and the cell indices overlay them
  uint32_t *cww = (uint32_t *)smem;
  const int ncw = lm_cww_words(fd.nldpc);
#pragma unroll
  for (int k = 0; k < LM_WORDS; k++) {
    const int i = tid + FEC_THREADS * k;
    if (i < ncw) cww[i] = __builtin_bswap32(w[k]);
  }
  uint8_t *idx = smem + 4 * ncw;
  __syncthreads();
  map_cells<FEC_THREADS>(md, cww, idx, tid);
  __syncthreads();
  if (md.rotation) {   // idx[-1] (the codeword's dead slack word) = idx[cs - 1] for map_store_quads
    if (tid == 0) idx[-1] = idx[md.cs - 1];
    __syncthreads();
    map_store_quads<FEC_THREADS, true>(md, mio.out_pairs, mio.frame_stride, idx, blk, tid);
  } else {
    map_store_quads<FEC_THREADS, false>(md, mio.out_pairs, mio.frame_stride, idx, blk, tid);
  }
}

hipError_t launch_ldpc_map(const FecDev &fd, const FecIO &fio, const MapDev &md, const MapIO &mio, hipStream_t s,
                           const L1Dev *l1d, const L1IO *l1io) {
  if (fio.nblocks <= 0) return hipSuccess;
  // the chain's layout only: packed BBFRAME rows from FEC_TS_TO_BBFRAME, the quad-table TI store
  if (!fec_plan_fits(fd) || !fec_chain_args_ok(fd, fio) || mio.nblocks != fio.nblocks || !md.slot_quad ||
      !mio.out_pairs || md.nldpc != fd.nldpc || md.cs * md.F <= 0 ||
      lm_cww_words(fd.nldpc) > LM_WORDS * FEC_THREADS || (fd.nldpc / 8 + 3) / 4 > LM_WORDS * FEC_THREADS)
    return hipErrorInvalidValue;
  int smem = lm_smem(fd, md.cs);
  L1Dev ld{};
  L1IO li{};
  if (l1d && l1io && l1io->nframes > 0) {
    if (!l1_args_ok(*l1d)) return hipErrorInvalidValue;
    ld = *l1d;
    li = *l1io;
    smem = smem > L1_LDS_WORDS * 4 ? smem : L1_LDS_WORDS * 4;
  }
  if (smem > MAP_LDS_MAX) return hipErrorInvalidValue;
  hipError_t e = lds_limit((const void *)ldpc_map_kernel, MAP_LDS_MAX);
  if (e != hipSuccess) return e;
  const int nl1 = (li.nframes + 7) & ~7;
  hipLaunchKernelGGL(ldpc_map_kernel, dim3(fio.nblocks + nl1), dim3(FEC_THREADS), smem, s, fd, fio, md, mio, ld, li);
  return hipGetLastError();
}

// ============================================================================ OFDM kernels
constexpr int OFDM_SQ16 = 4;   // data-slot quads per thread per scatter round (N <= 16K: one round)
// the first scatter round of a unit's data slots, loaded while the previous unit's transform runs
struct SlotPre {
  uint2 b[OFDM_SQ16], c[OFDM_SQ16];
  int aux;            // the first round of direct aux quads below is loaded (quad tid)
  int4 gr;            // the unit's aux group
  uint2 ab;           // quad tid's bins and values
  float4 av0, av1;
};
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

__host__ __device__ constexpr int brev_c(int i, int bits) {
  int r = 0;
  for (int b = 0; b < bits; b++) r |= ((i >> b) & 1) << (bits - 1 - b);
  return r;
}
__host__ __device__ constexpr int log2_c(int n) { return n <= 1 ? 0 : 1 + log2_c(n / 2); }

// In-register inverse DFT of size R (natural order in and out): bit-reversal by register
// renaming, then in-place radix-2 stages fenced so each stage retires before the next
// (keeps a 32-point transform inside the 128-VGPR budget of a 1024-thread workgroup).
template <int R>
struct Dft {
  __device__ __forceinline__ static void run(float2 *x) {
    constexpr int L = log2_c(R);
#pragma unroll
    for (int i = 0; i < R; i++) {
      const int j = brev_c(i, L);
      if (i < j) { float2 t = x[i]; x[i] = x[j]; x[j] = t; }
    }
#pragma unroll
    for (int len = 2; len <= R; len <<= 1) {
#pragma unroll
      for (int i = 0; i < R; i += len) {
#pragma unroll
        for (int k = 0; k < len / 2; k++) {
          float2 a = x[i + k], b = x[i + k + len / 2], t;
          if (4 * k == len && k != 0) {                                             // * i
            x[i + k] = cadd_i(a, b);
            x[i + k + len / 2] = csub_i(a, b);
            continue;
          }
          if (k == 0) t = b;
          else t = cmulf(b, make_float2(kCos32[k * (32 / len)], kSin32[k * (32 / len)]));
          x[i + k] = cadd(a, t);
          x[i + k + len / 2] = csub(a, t);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
};

// ---------------------------------------------------------------- Stockham IFFT
// Sub-transform of NSUB <= 16384 points by NT = NSUB/16 threads, 16 complex values per thread.
// Pass with radix R over units j (Ns = product of earlier radices, Stockham autosort):
//   in  : A[j + r*NSUB/R]                         (r < R)
//   out : B[(j/Ns)*Ns*R + j%Ns + r*Ns] after twiddles w^((j%Ns)*r*NSUB/(Ns*R)) and DFT_R
// Data live in LDS between passes as float2 with one pad slot per 2^PS (PS = 4 for the radix-16
// plans, 5 for the radix-32 32K halves: then the stride-33 first-pass writes, 16 lanes per
// ds_write_b64 group, and the unit-stride reads, 32 lanes per ds_read_b64 group, are
// bank-conflict free).  The first pass reads the gathered inputs from registers, the last writes
// its outputs to registers: thread t ends with n = t + NT*m, m = u + (16/R_last)*r.
template <int PS>
__device__ __forceinline__ uint32_t lds_pad(uint32_t a) { return a + (a >> PS); }

// w^i (w = exp(2 pi i / N)) from the two-level LDS table tw = [lo: w^l, l < 128][hi: w^(128 h)]
__device__ __forceinline__ float2 tw_at(const float2 *tw, uint32_t i) {
  return cmulf(tw[128 + (i >> 7)], tw[i & 127]);
}

// v[r] *= w^(r * e) for r = 1..R-1 (R <= 16): w^e, w^(4e) and (R = 16) w^(8e) from the table (tw_at), the
// other lo = w^(l e) and hi = w^(4 h e) (l, h < 4) as products of those, w^(r e) = hi * lo.  (Round 5 built every
// power from w^e alone by products of depth <= 5: a relative phase error d of w^e becomes k d in w^(k e), and
// that IFFT was 2.3-4.2 x pocketfft's float32 error at 1K-16K; with these bases it is 1.3-1.6 x on random
// symbols.  Six bases (w^(k e), k = 1, 2, 3, 4, 8, 12, as the 32K kernel) measured 1.1-1.3 x but 2-4 % slower
// OFDM, from the extra table reads.)
template <int R>
__device__ __forceinline__ void twiddle_unit(float2 *v, const float2 *tw, uint32_t e) {
  static_assert(R <= 16, "bases for r < 16");
  if (R == 1) return;
  float2 lo[4], hi[4];
  lo[1] = tw_at(tw, e);
  if (R > 2) {
    lo[2] = cmulf(lo[1], lo[1]);
    lo[3] = cmulf(lo[2], lo[1]);
  }
  if (R > 4) hi[1] = tw_at(tw, 4 * e);
  if (R > 8) {
    hi[2] = tw_at(tw, 8 * e);
    hi[3] = cmulf(hi[2], hi[1]);
  }
#pragma unroll
  for (int r = 1; r < R; r++) {
    const int h = (r >> 2) & 3, l = r & 3;
    const float2 w = h == 0 ? lo[l] : (l == 0 ? hi[h] : cmulf(hi[h], lo[l]));
    v[r] = cmulf(v[r], w);
  }
}

template <int NSUB, int NT, int R, int NS, int PS>
struct StockhamPass {
  static constexpr int V = NSUB / NT;       // values per thread
  static constexpr int U = V / R;           // units per thread
  static constexpr int PAD = 1 << PS;
  // every LDS address below is lds_pad(thread base) + a compile-time offset (immediate field)
  static_assert((NS == 1 && R % PAD == 0) || NS % PAD == 0, "pad offsets need NS == 1 (PAD | R) or PAD | NS");
  static_assert((NSUB / R) % PAD == 0, "pad offsets need PAD | NSUB / R");
  // twiddles + DFT on the thread's U units (v laid out [u][r])
  __device__ __forceinline__ static void compute(float2 *v, const float2 *tw, uint32_t tws, int tid) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (NS > 1) {
        const uint32_t j = (uint32_t)(tid + NT * u);
        twiddle_unit<R>(v + u * R, tw, (j % NS) * (uint32_t)(NSUB / (NS * R)) * tws);
      }
      __builtin_amdgcn_sched_barrier(0);
      Dft<R>::run(v + u * R);
    }
  }
  __device__ __forceinline__ static void store_lds(const float2 *v, float2 *lds, int tid) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t j = (uint32_t)(tid + NT * u);
      float2 *b = lds + lds_pad<PS>((j / NS) * (NS * R) + (j % NS));
#pragma unroll
      for (int r = 0; r < R; r++) b[r * NS + ((r * NS) >> PS)] = v[u * R + r];
    }
  }
  __device__ __forceinline__ static void load_lds(float2 *v, const float2 *lds, int tid) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const float2 *b = lds + lds_pad<PS>((uint32_t)(tid + NT * u));
#pragma unroll
      for (int r = 0; r < R; r++) v[u * R + r] = b[r * (NSUB / R) + ((r * (NSUB / R)) >> PS)];
    }
  }
};

// remaining passes after the first, radices R2.. ; NS = product of radices already applied
template <int NSUB, int NT, int PS, int NS, int... Rs>
struct StockhamTail;
template <int NSUB, int NT, int PS, int NS>
struct StockhamTail<NSUB, NT, PS, NS> {
  __device__ __forceinline__ static void run(float2 *, float2 *, const float2 *, uint32_t, int) {}
};
template <int NSUB, int NT, int PS, int NS, int R, int... Rs>
struct StockhamTail<NSUB, NT, PS, NS, R, Rs...> {
  __device__ __forceinline__ static void run(float2 *v, float2 *lds, const float2 *tw, uint32_t tws, int tid) {
    using P = StockhamPass<NSUB, NT, R, NS, PS>;
    P::load_lds(v, lds, tid);
    lds_barrier();
    P::compute(v, tw, tws, tid);
    if (sizeof...(Rs) > 0) {
      P::store_lds(v, lds, tid);
      lds_barrier();
      StockhamTail<NSUB, NT, PS, NS * R, Rs...>::run(v, lds, tw, tws, tid);
    }
  }
};

// FFT plans (N <= 16K): first pass radix V = 16 from LDS or registers, then the tail.
// RL = radix of the last pass; thread t ends with n = t + NT*(u + (V/RL)*r); PS = LDS pad shift.
template <int NSUB, int V> struct FftPlan;
template <> struct FftPlan<1024, 16> { static constexpr int RL = 4, PS = 4; using Tail = StockhamTail<1024, 64, 4, 16, 16, 4>; };
template <> struct FftPlan<2048, 16> { static constexpr int RL = 8, PS = 4; using Tail = StockhamTail<2048, 128, 4, 16, 16, 8>; };
template <> struct FftPlan<4096, 16> { static constexpr int RL = 16, PS = 4; using Tail = StockhamTail<4096, 256, 4, 16, 16, 16>; };
template <> struct FftPlan<8192, 16> { static constexpr int RL = 2, PS = 4; using Tail = StockhamTail<8192, 512, 4, 16, 16, 16, 2>; };
template <> struct FftPlan<16384, 16> { static constexpr int RL = 4, PS = 4; using Tail = StockhamTail<16384, 1024, 4, 16, 16, 16, 4>; };

// Where a transform's inputs come from.  Gather (pilotgen block: cells in carrier order, so per-bin
// loads are near unit-stride): bin k reads map[k].  Scatter (fused chain: cells in TI output order,
// randomly placed by the frequency interleaver): aux bins (map < 0) are filled from the aux
// table, then the symbol's contiguous run of data slots is streamed with unit-stride loads and
// each cell is written to LDS at its bin inv[slot].
struct BinSource {
  const int32_t *map;          // this symbol's row (natural FFT-input order)
  const float2 *data;          // uniform base; cells at cbase + code (gather), aux at abase - code
  uint32_t cbase, abase;
  const uint16_t *inv;         // scatter mode: stored bin of each data slot (null: gather mode)
  const uint16_t *pairs;       // scatter mode: constellation index pair of each slot at cbase + slot
  const float *qre, *qim;      // scatter mode: constellation real / imaginary parts in LDS
  uint32_t d0, dn, dn0;        // scatter mode: this symbol's data slots; the first dn0 feed half 0
  const uint16_t *abin;        // scatter mode: aux lists (OfdmDev)
  const float2 *aval;
  const uint32_t *aind;
  const int4 *agrp;            // this symbol's groups (halves)
  const int2 *azr;             // this symbol's zero runs (padded LDS slot ranges)
  // multi-PLP frames: this symbol's PLP boundaries (OfdmDev::plp_bnd + 2 j (nplp + 1)) and the PLPs'
  // constellation table bases in qre / qim
  int nplp;
  const int32_t *bnd;
  const int32_t *qbase;
};

// Scatter-mode fill of one group (a whole symbol, or one half of a split 32K symbol) into LDS,
// every bin written exactly once (t2_plan build_aux_lists / build_chain_layout):
//   the direct aux quads (pilots, L1-pre, dummy cells: bin + value), the indirect entries (the
//   frame's L1-post cells through its aux variant) and the data slots, streamed as aligned quads
//   of (uint16 bin, uint16 index pair) and looked up in the constellation (QAM + rotated-Q
//   delay).  Slots outside the run (quad edges) and padding bins go to a per-lane dummy slot.
// The zero run is written separately by the caller.
struct NoWork {
  __device__ __forceinline__ void operator()() const {}
};
// mid (32K): register work independent of the LDS, run once by every thread while its first round
// of data-slot loads is in flight (after the loop when the run has no slots)
template <int NT, int SQ, class Mid>
__device__ __forceinline__ void scatter_slots(float2 *lds, const BinSource &src, uint32_t r0, uint32_t rn,
                                              uint32_t dummy, int tid, const Mid &mid, uint32_t lb,
                                              const SlotPre *pre = nullptr);
// MULTI (a kernel instantiation of its own, so the one-PLP kernels keep their register allocation):
// the data slots of a multi-PLP frame, streamed PLP by PLP (a group's slots are PLP-major), each
// PLP's run looked up in its own constellation table
template <int NT, int SQ, bool MULTI = false, class Mid = NoWork>
__device__ __forceinline__ void scatter_group(float2 *lds, const BinSource &src, int g, uint32_t r0, uint32_t rn,
                                              uint32_t dummy, int tid, const Mid &mid = Mid(),
                                              const SlotPre *pre = nullptr) {
  // the prefetched values copied out first: a select between a load of them and a global load
  // would become a load through a select of the two pointers, and put SlotPre in scratch
  bool pa = false;
  int4 gr;
  uint2 pab = make_uint2(0u, 0u);
  float4 pv0 = make_float4(0.f, 0.f, 0.f, 0.f), pv1 = pv0;
  if (pre) {
    pa = pre->aux != 0;
    gr = pre->gr;
    pab = pre->ab;
    pv0 = pre->av0;
    pv1 = pre->av1;
  }
  if (!pa) gr = kc(src.agrp, g);
  for (uint32_t q = (uint32_t)tid; q < ((uint32_t)gr.y >> 2); q += NT) {
    const uint32_t e0 = (uint32_t)gr.x + 4u * q;
    uint2 b;
    float4 v01, v23;
    if (pa && q == (uint32_t)tid) {
      b = pab;
      v01 = pv0;
      v23 = pv1;
    } else {
      b = ld_off((const uint2 *)src.abin, e0 * 2u);
      v01 = ld_off((const float4 *)src.aval, e0 * 8u);
      v23 = ld_off((const float4 *)src.aval, e0 * 8u + 16u);
    }
    const uint32_t k0 = b.x & 0xFFFFu, k1 = b.x >> 16, k2 = b.y & 0xFFFFu, k3 = b.y >> 16;
    lds[k0 != 0xFFFFu ? k0 : dummy] = make_float2(v01.x, v01.y);   // bins stored padded
    lds[k1 != 0xFFFFu ? k1 : dummy] = make_float2(v01.z, v01.w);
    lds[k2 != 0xFFFFu ? k2 : dummy] = make_float2(v23.x, v23.y);
    lds[k3 != 0xFFFFu ? k3 : dummy] = make_float2(v23.z, v23.w);
  }
  for (uint32_t i = (uint32_t)tid; i < (uint32_t)gr.w; i += NT) {
    const uint32_t e = src.aind[(uint32_t)gr.z + i];
    lds[e & 0x7FFFu] = ld_off(src.data, (src.abase + (e >> 15)) * 8u);
  }
  if (MULTI) {
    mid();
    const int P = src.nplp;
    for (int p = 0; p < P; p++) {   // (uniform)
      const uint32_t a = (uint32_t)kc(src.bnd, g * (P + 1) + p), b = (uint32_t)kc(src.bnd, g * (P + 1) + p + 1);
      if (b > a) scatter_slots<NT, SQ>(lds, src, a, b - a, dummy, tid, NoWork(), (uint32_t)kc(src.qbase, p));
    }
  } else {
    scatter_slots<NT, SQ>(lds, src, r0, rn, dummy, tid, mid, 0u, pre);
  }
}

// the data slots [r0, r0 + rn): streamed as aligned octets (32K) or quads, looked up in the constellation
// table at lb of qre / qim (QAM + rotated-Q delay) and written to their bins
template <int NT, int SQ, class Mid>
__device__ __forceinline__ void scatter_slots(float2 *lds, const BinSource &src, uint32_t r0, uint32_t rn,
                                              uint32_t dummy, int tid, const Mid &mid, uint32_t lb,
                                              const SlotPre *pre) {
  if (SQ == 4) {
    // 32K kernel: slots in aligned octets, one 16-byte load of bins and one of index pairs per
    // octet (half the load instructions of quads; the pair rows are padded to a multiple of 8)
    const uint32_t o0 = r0 & ~7u, no = (r0 + rn - o0 + 7u) >> 3;
    const uint32_t lasto = no - 1u;
    bool pending = true;
    for (uint32_t g0 = 0; g0 < no; g0 += 2u * NT) {   // (no is uniform: every thread runs the same rounds)
      uint4 b[2], c[2];
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const uint32_t s = o0 + 8u * min(g0 + (uint32_t)(tid + NT * u), lasto);
        b[u] = ld_off((const uint4 *)src.inv, s * 2u);
        c[u] = ld_off((const uint4 *)src.pairs, (src.cbase + s) * 2u);
      }
      if (pending) {
        mid();
        pending = false;
      }
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const uint32_t s = o0 + 8u * min(g0 + (uint32_t)(tid + NT * u), lasto);
        // the octet's eight constellation lookups first, then its eight bin writes: in program order
        // the compiler cannot move an LDS read past an LDS write it may alias, so lookup / write pairs
        // would serialise into eight LDS round trips
        float2 v[8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
          const uint32_t cw = e < 2 ? c[u].x : e < 4 ? c[u].y : e < 6 ? c[u].z : c[u].w;
          const uint32_t pr = cw >> (16 * (e & 1));
          v[e] = make_float2(src.qre[lb + (pr & 0xFFu)], src.qim[lb + ((pr >> 8) & 0xFFu)]);
        }
#pragma unroll
        for (int e = 0; e < 8; e++) {
          const uint32_t bw = e < 2 ? b[u].x : e < 4 ? b[u].y : e < 6 ? b[u].z : b[u].w;
          const uint32_t bin = (bw >> (16 * (e & 1))) & 0xFFFFu;   // padded, within the group
          const bool in_run = s + (uint32_t)e - r0 < rn;
          lds[in_run ? bin : dummy] = v[e];
        }
      }
    }
    if (pending) mid();
    return;
  }
  const uint32_t q0 = r0 & ~3u, nq = (r0 + rn - q0 + 3u) >> 2;
  const uint32_t lastq = nq - 1u;
  for (uint32_t g0 = 0; g0 < nq; g0 += (uint32_t)SQ * NT) {
    uint2 b[SQ], c[SQ];
    if (SQ == OFDM_SQ16 && pre && g0 == 0) {   // loaded by slot_prefetch
#pragma unroll
      for (int u = 0; u < SQ; u++) {
        b[u] = pre->b[u];
        c[u] = pre->c[u];
      }
    } else {
#pragma unroll
      for (int u = 0; u < SQ; u++) {
        const uint32_t s = q0 + 4u * min(g0 + (uint32_t)(tid + NT * u), lastq);
        b[u] = ld_off((const uint2 *)src.inv, s * 2u);
        c[u] = ld_off((const uint2 *)src.pairs, (src.cbase + s) * 2u);
      }
    }
#pragma unroll
    for (int u = 0; u < SQ; u += 2) {
      // two quads' lookups, then their writes (see the 32K path)
      float2 v[8];
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const uint32_t cw = (e & 2) ? c[u + (e >> 2)].y : c[u + (e >> 2)].x;
        const uint32_t pr = cw >> (16 * (e & 1));
        v[e] = make_float2(src.qre[lb + (pr & 0xFFu)], src.qim[lb + ((pr >> 8) & 0xFFu)]);
      }
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const int uu = u + (e >> 2), ee = e & 3;
        const uint32_t s = q0 + 4u * min(g0 + (uint32_t)(tid + NT * uu), lastq);
        const uint32_t bw = (ee & 2) ? b[uu].y : b[uu].x;
        const uint32_t bin = (bw >> (16 * (ee & 1))) & 0xFFFFu;   // padded, within the group
        const bool in_run = s + (uint32_t)ee - r0 < rn;
        lds[in_run ? bin : dummy] = v[e];
      }
    }
  }
}

// the loads of scatter_slots' first round for the slots [r0, r0 + rn) of bins inv, pairs at cbase
template <int NT>
__device__ __forceinline__ void slot_prefetch(SlotPre &p, const uint16_t *inv, const uint16_t *pairs, uint32_t cbase,
                                              uint32_t r0, uint32_t rn, int tid, bool aux = false,
                                              const int4 *agrp = nullptr, const uint16_t *abin = nullptr,
                                              const float2 *aval = nullptr) {
  p.aux = aux;
  if (aux) {
    p.gr = kc(agrp, 0);
    const uint32_t q = (uint32_t)tid;
    if (q < ((uint32_t)p.gr.y >> 2)) {
      const uint32_t e0 = (uint32_t)p.gr.x + 4u * q;
      p.ab = ld_off((const uint2 *)abin, e0 * 2u);
      p.av0 = ld_off((const float4 *)aval, e0 * 8u);
      p.av1 = ld_off((const float4 *)aval, e0 * 8u + 16u);
    }
  }
  if (rn == 0) return;   // (uniform) scatter_slots runs no round
  const uint32_t q0 = r0 & ~3u, lastq = ((r0 + rn - q0 + 3u) >> 2) - 1u;
#pragma unroll
  for (int u = 0; u < OFDM_SQ16; u++) {
    const uint32_t s = q0 + 4u * min((uint32_t)(tid + NT * u), lastq);
    p.b[u] = ld_off((const uint2 *)inv, s * 2u);
    p.c[u] = ld_off((const uint2 *)pairs, (cbase + s) * 2u);
  }
}

// One NSUB-point transform (N <= 16K) by NT = NSUB/V threads, ending with
// v[u*RL + r] = y[t + NT*(u + (V/RL)*r)].  Also stores the kernel's constant tables (`stage`) to LDS.
// pre: the scatter's first round, loaded before (null: loaded here); after_scatter: run once the
// scatter is in LDS (the next unit's slot_prefetch)
template <int NSUB, int V, bool MULTI, class Stage, class After = NoWork>
__device__ __forceinline__ void sub_ifft(float2 *v, float2 *lds, const BinSource &src, const float *isinc,
                                         const float2 *tw, int tid, const Stage &stage, const SlotPre *pre = nullptr,
                                         const After &after_scatter = After(), bool nobar = false) {
  constexpr int NT = NSUB / V, N = NSUB;
  constexpr int PS = FftPlan<NSUB, V>::PS;
  if (src.inv) {
    {
      const int2 zr = kc(src.azr, 0);
      for (int i = zr.x + tid; i < zr.y; i += NT) lds[i] = make_float2(0.f, 0.f);
    }
    // nobar: the tables are in LDS already (stored once by the kernel), and the zero run, the
    // scatter's bins and its dummy slots are disjoint, so the scatter needs no barrier after the fill
    if (!nobar) {
      stage.store((unsigned char *)lds, true, tid);
      lds_barrier();
    }
    const uint32_t dummy = (uint32_t)(NSUB + (NSUB >> PS)) + (uint32_t)(tid & 63);
    scatter_group<NT, OFDM_SQ16, MULTI>(lds, src, 0, src.d0, src.dn, dummy, tid, NoWork(), pre);
    lds_barrier();
    after_scatter();
    StockhamPass<NSUB, NT, V, 1, PS>::load_lds(v, lds, tid);
    lds_barrier();
  } else {
    stage.store((unsigned char *)lds, false, tid);
#pragma unroll
    for (int c0 = 0; c0 < V; c0 += 8) {
      uint32_t off[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        int code = ld_off(src.map, (uint32_t)(tid + NT * (c0 + u)) * 4u);
        off[u] = (code >= 0 ? src.cbase + (uint32_t)code : src.abase - (uint32_t)code) * 8u;
      }
#pragma unroll
      for (int u = 0; u < 8; u++) v[c0 + u] = ld_off(src.data, off[u]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (isinc) {
#pragma unroll
    for (int r = 0; r < V; r++) {
      const uint32_t k = (uint32_t)(tid + NT * r);
      const float sc = isinc[(k + N / 2) & (N - 1)];
      v[r].x *= sc;
      v[r].y *= sc;
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  Dft<V>::run(v);
  StockhamPass<NSUB, NT, V, 1, PS>::store_lds(v, lds, tid);
  lds_barrier();
  FftPlan<NSUB, V>::Tail::run(v, lds, tw, 1u, tid);
}

template <int N>
struct OfdmShape {
  static constexpr int V = 16;                                        // values per thread
  static constexpr int NT = N / V;
  static constexpr int PS = FftPlan<N, V>::PS;
  static constexpr int FFT_LDS = (N + (N >> PS) + 64) * 8;           // padded buffer + 64 dummy slots
  // the next unit's first direct aux quad is prefetched with its data slots where the registers allow
  // it (4K, 8K: 1K, 2K and 16K would spill at the 128-VGPR cap)
  static constexpr bool AUX_PRE = N == 4096;
  static constexpr int TW_ENTRIES = 128 + N / 128;                   // two-level twiddle table
  static constexpr int QAM_OFF = FFT_LDS + TW_ENTRIES * 8;
  // with the constellation tables of nq entries (multi-PLP frames: every PLP's table, re[nq] then im[nq])
  static constexpr int lds_bytes(int nq) { return QAM_OFF + nq * 8; }
};

// value of lane l ^ 1 (DPP quad_perm [1,0,3,2])
__device__ __forceinline__ float swap_adjacent_lane(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
}

// IQ sample writer: the normalised sample times the output gain (the flowgraph's
// blocks_multiply_const_xx after pilotgen, apps/vv009-4kshort.grc:335-385; 1 = the block's own
// output), stored as complex64 (FMT 0) or as saturated round-to-nearest-even int16 I/Q at
// full scale 32767 (FMT 1, the SDR sink's sc16 wire format)
template <int FMT>
struct IqOut {
  char *base;   // sample 0 of this symbol (or of the P1 symbol)
  float gain;
  __device__ __forceinline__ void put(uint32_t n, float2 a) const {
    a = cscale(a, gain);
    if (FMT == 0) {
      st_nt((float2 *)base, n * 8u, a);
    } else {
      const float i = fminf(fmaxf(rintf(a.x * 32767.f), -32768.f), 32767.f);
      const float q = fminf(fmaxf(rintf(a.y * 32767.f), -32768.f), 32767.f);
      const uint32_t w = ((uint32_t)(int)i & 0xFFFFu) | ((uint32_t)(int)q << 16);
      __builtin_nontemporal_store(w, (uint32_t *)(base + n * 4u));
    }
  }
  // samples n, n + 1 (n even, already multiplied by the gain) as one store
  __device__ __forceinline__ void put2(uint32_t n, float2 a, float2 b) const {
    if (FMT == 0) {
      typedef float f4v __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(f4v{a.x, a.y, b.x, b.y}, (f4v *)(base + n * 8u));
    } else {
      typedef uint32_t u2v __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store(u2v{sc16(a), sc16(b)}, (u2v *)(base + n * 4u));
    }
  }
  static __device__ __forceinline__ uint32_t sc16(float2 a) {
    const float i = fminf(fmaxf(rintf(a.x * 32767.f), -32768.f), 32767.f);
    const float q = fminf(fmaxf(rintf(a.y * 32767.f), -32768.f), 32767.f);
    return ((uint32_t)(int)i & 0xFFFFu) | ((uint32_t)(int)q << 16);
  }
};

// the OFDM kernel's constant LDS tables (twiddles, constellation), held in registers between
// load() and store()
template <int N>
struct TableStage {
  using Sh = OfdmShape<N>;
  static constexpr int NT = Sh::NT, TWK = (Sh::TW_ENTRIES + NT - 1) / NT, QK = (256 + NT - 1) / NT;
  float2 tw[TWK], q[QK];
  int nq = 256;
  const float2 *qam = nullptr;
  __device__ __forceinline__ void load(const OfdmDev &d, int tid) {
    nq = d.nq;
    qam = d.qam;
#pragma unroll
    for (int k = 0; k < TWK; k++) {
      const int i = tid + k * NT;
      if (i < Sh::TW_ENTRIES) tw[k] = d.twiddle[i];
    }
    if (d.inv) {
#pragma unroll
      for (int k = 0; k < QK; k++) {
        const int i = tid + k * NT;
        if (i < 256 && i < d.nq) q[k] = d.qam[i];   // a multi-PLP table may hold fewer than 256 entries
      }
    }
  }
  __device__ __forceinline__ void store(unsigned char *smem, bool chain, int tid) const {
    float2 *twl = (float2 *)(smem + Sh::FFT_LDS);
#pragma unroll
    for (int k = 0; k < TWK; k++) {
      const int i = tid + k * NT;
      if (i < Sh::TW_ENTRIES) twl[i] = tw[k];
    }
    if (chain) {
      float *qre = (float *)(smem + Sh::QAM_OFF), *qim = qre + nq;
#pragma unroll
      for (int k = 0; k < QK; k++) {
        const int i = tid + k * NT;
        if (i < 256 && i < nq) {
          qre[i] = q[k].x;
          qim[i] = q[k].y;
        }
      }
      for (int i = 256 + tid; i < nq; i += NT) {   // the further PLPs' tables (multi-PLP frames)
        const float2 t = qam[i];
        qre[i] = t.x;
        qim[i] = t.y;
      }
    }
  }
};

// OFDM symbols of N <= 16K points: one workgroup of N / 16 threads per (symbol, frame), the
// symbol's bins in LDS, radix-16 Stockham passes, normalisation, GI copy, IQ store
// the slot run of unit u (symbol u / nframes of frame u % nframes) in the chain's scatter mode
struct UnitSlots {
  const uint16_t *inv;
  uint32_t cbase, r0, rn;
  const int4 *agrp;
};
__device__ __forceinline__ UnitSlots unit_slots(const OfdmDev &d, const OfdmIO &io, int u) {
  const int j = u / io.nframes, f = u - j * io.nframes;
  const int64_t frame = io.first_frame + (io.frames_per_stream ? f % io.frames_per_stream : f);
  const int c = d.ncls > 1 ? (int)(frame % d.ncls) : 0, jc = c * d.Nsym + j;
  return UnitSlots{d.inv + kc(d.cls_inv, c), io.cell_off + (uint32_t)f * io.cell_stride, (uint32_t)kc(d.sym_d0, jc),
                   (uint32_t)kc(d.sym_n, jc), d.agrp + 2 * jc};
}

// pf (one-PLP chain frames): in, this unit's first scatter round (loaded by the previous unit or
// the kernel); out, unit un's (un < 0: none)
template <int N, int FMT, bool MULTI>
__device__ __forceinline__ void ofdm_unit(const OfdmDev &d, const OfdmIO &io, int u, unsigned char *smem,
                                          const TableStage<N> &tabs, int tid, SlotPre *pf = nullptr, int un = -1) {
  using Sh = OfdmShape<N>;
  constexpr int NT = Sh::NT, V = Sh::V, RL = FftPlan<N, V>::RL, UL = V / RL;
  float2 *lds = (float2 *)smem;
  float2 *twl = (float2 *)(smem + Sh::FFT_LDS);
  float *qre = (float *)(smem + Sh::QAM_OFF), *qim = qre + d.nq;
  const int j = u / io.nframes;                   // symbol
  const int f = u - j * io.nframes;               // frame within launch
  const int64_t frame = io.first_frame + (io.frames_per_stream ? f % io.frames_per_stream : f);   // stream-major batch
  const float2 *data = io.data;                   // uniform base: all gathers are base + u32 offset
  const uint32_t cbase = io.cell_off + (uint32_t)f * io.cell_stride;
  const uint32_t abase = io.aux_off + (uint32_t)(frame % d.t2frames) * (uint32_t)d.aux_len - 1u;
  const int32_t *map = d.bin_map + (int64_t)j * N;
  BinSource src{map, data, cbase, abase, d.inv, io.pairs, qre, qim, 0u, 0u, 0u, d.abin, d.aval, d.aind, nullptr,
                nullptr, 1, nullptr, nullptr};
  if (d.inv) {
    // the frame's class (FRAME_INTERVAL > 1): its rows of the per-symbol tables, its slots' bins
    const int c = d.ncls > 1 ? (int)(frame % d.ncls) : 0, jc = c * d.Nsym + j;
    src.inv = d.inv + kc(d.cls_inv, c);
    src.data = io.l1;                              // indirect entries: this frame's L1-post cells
    src.abase = (uint32_t)f * io.l1_stride - 1u;
    src.d0 = (uint32_t)kc(d.sym_d0, jc);
    src.dn = (uint32_t)kc(d.sym_n, jc);
    src.dn0 = (uint32_t)kc(d.sym_n0, jc);
    src.agrp = d.agrp + 2 * jc;
    src.azr = d.azr + 2 * jc;
    src.nplp = d.nplp;
    src.bnd = d.plp_bnd ? d.plp_bnd + 2 * jc * (d.nplp + 1) : nullptr;
    src.qbase = d.plp_qbase;
  }
  if (io.carriers_only) {                          // test hook (gather mode): bins in natural order
    if (d.inv) return;
    float2 *o = io.out + (int64_t)f * io.out_stride + (int64_t)j * N;
    for (int k = tid; k < N; k += NT) {
      const int code = map[k];
      float2 v = data[code >= 0 ? cbase + (uint32_t)code : abase - (uint32_t)code];
      if (d.isinc) {
        const float sc = d.isinc[(k + N / 2) & (N - 1)];
        v.x *= sc;
        v.y *= sc;
      }
      o[(k + N / 2) & (N - 1)] = v;
    }
    return;
  }
  constexpr int SB = FMT == 0 ? 8 : 4;             // bytes per IQ sample
  if (j == 0) {                                   // P1 symbol (precomputed), pilotgen:2802-2810
    const IqOut<FMT> p{(char *)io.out + (int64_t)f * io.out_stride * SB, d.gain};
    for (int i = tid; i < 2048; i += NT) p.put((uint32_t)i, d.p1[i]);
  }
  const int G = d.G;
  const IqOut<FMT> o{(char *)io.out + ((int64_t)f * io.out_stride + 2048 + (int64_t)j * (N + G)) * SB, d.gain};
  const float nrm = d.norm;
  float2 v[V];
  if (pf) {
    auto next = [&]() {
      if (un >= 0) {
        const UnitSlots ns = unit_slots(d, io, un);
        slot_prefetch<NT>(*pf, ns.inv, io.pairs, ns.cbase, ns.r0, ns.rn, tid, OfdmShape<N>::AUX_PRE, ns.agrp, d.abin,
                          d.aval);
      }
    };
    sub_ifft<N, V, MULTI>(v, lds, src, d.isinc, twl, tid, tabs, pf, next, true);
  } else {
    sub_ifft<N, V, MULTI>(v, lds, src, d.isinc, twl, tid, tabs);
  }
  if ((((uintptr_t)o.base + (uint32_t)G * SB) & (2u * SB - 1u)) == 0) {
    // two consecutive samples per lane and store: lanes t, t ^ 1 swap half of their values
    // (as o32_store_pairs), so the even lane stores (t, t + 1) of every even m and the odd lane
    // those of every odd m, m = uu + UL r
    const bool odd = tid & 1;
    const uint32_t n0 = (uint32_t)tid & ~1u;
#pragma unroll
    for (int p = 0; p < V / 2; p++) {
      const int m0 = 2 * p, m1 = 2 * p + 1;
      const float2 e = cscale(cscale(v[(m0 % UL) * RL + m0 / UL], nrm), o.gain);
      const float2 dd = cscale(cscale(v[(m1 % UL) * RL + m1 / UL], nrm), o.gain);
      const float2 re = make_float2(swap_adjacent_lane(e.x), swap_adjacent_lane(e.y));
      const float2 rd = make_float2(swap_adjacent_lane(dd.x), swap_adjacent_lane(dd.y));
      const float2 lo = odd ? rd : e, hi = odd ? dd : re;
      const uint32_t n = n0 + (uint32_t)NT * (uint32_t)(m0 + (odd ? 1 : 0));
      o.put2((uint32_t)G + n, lo, hi);
      if (n >= (uint32_t)(N - G)) o.put2(n - (uint32_t)(N - G), lo, hi);
    }
  } else {
#pragma unroll
    for (int uu = 0; uu < UL; uu++)
#pragma unroll
      for (int r = 0; r < RL; r++) {
        const uint32_t n = (uint32_t)(tid + NT * (uu + UL * r));
        float2 a = v[uu * RL + r];
        a = cscale(a, nrm);
        o.put((uint32_t)G + n, a);
        if (n >= (uint32_t)(N - G)) o.put(n - (uint32_t)(N - G), a);
      }
  }
}

// OFDM symbols of N <= 16K points: N / 16 threads per workgroup, each workgroup a run of consecutive
// (symbol, frame) units u = symbol * nframes + frame (the same symbol of consecutive frames: the same
// slot bins and aux lists), so the constant tables are loaded once per run and one unit's IQ stores
// drain while the next unit's bins are loaded.  Runs are XCD-major, so each XCD walks a contiguous
// range of symbols for all frames of the launch and reads each symbol's tables from its own L2.
template <int N, int FMT, bool MULTI>
__global__ __launch_bounds__(OfdmShape<N>::NT, 4) void ofdm_kernel(OfdmDev d, OfdmIO io) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  // constant tables: loaded into registers here, stored to LDS once (one-PLP chain frames) or after
  // every unit's zero fill
  TableStage<N> tabs;
  tabs.load(d, tid);
  const int units = d.Nsym * io.nframes, per = (units + (int)gridDim.x - 1) / (int)gridDim.x;
  const int u0 = xcd_major(blockIdx.x, gridDim.x) * per, u1 = min(u0 + per, units);
  // one-PLP chain frames: each unit's first scatter round is loaded during the previous unit
  const bool pre = !MULTI && d.inv && !io.carriers_only;
  SlotPre pf;
  if (pre && u0 < u1) {
    const UnitSlots ns = unit_slots(d, io, u0);
    slot_prefetch<OfdmShape<N>::NT>(pf, ns.inv, io.pairs, ns.cbase, ns.r0, ns.rn, tid, OfdmShape<N>::AUX_PRE,
                                    ns.agrp, d.abin, d.aval);
    tabs.store(smem, true, tid);
    lds_barrier();
  }
#pragma nounroll
  for (int u = u0; u < u1; u++) {
    // the previous unit's last reads of the transform buffer came before its final barrier; in the
    // chain's scatter mode the next unit writes nothing else (the tables stay), elsewhere the table
    // store rewrites them, so wait for every wave there
    if (u > u0 && !pre) lds_barrier();
    // opaque per unit: otherwise every per-thread address of the unit's passes is hoisted out of the
    // loop and held in registers across it
    int t = tid;
    asm volatile("" : "+v"(t));
    if (pre)
      ofdm_unit<N, FMT, MULTI>(d, io, u, smem, tabs, t, &pf, u + 1 < u1 ? u + 1 : -1);
    else
      ofdm_unit<N, FMT, MULTI>(d, io, u, smem, tabs, t);
  }
}

// ---------------------------------------------------------------- 32K symbols
// One workgroup of 1024 threads per (symbol, frame); the whole 32768-point symbol stays in VGPRs
// (32 complex values per thread) through three radix-32 stages of a 32 x 32 x 32 decomposition.
// With m = m0 + 32 m1 + 1024 m2 (input bin) and n = n2 + 32 n1 + 1024 n0 (output sample),
//   stage A: DFT over m2, then * w^((m0 + 32 m1) n2)      thread (a, b) = (m0, m1)
//   stage B: DFT over m1, then * w_1024^(m0 n1)           thread (a, b) = (m0, n2)
//   stage C: DFT over m0 -> x[n2 + 32 n1 + 1024 n0]       thread (a, b) = (n1, n2)
// (w = exp(2 pi i / 32768); thread t <-> a = t[4..7] | t[8] << 4, b = t[0..3] | t[9] << 4).
// Each exchange keeps one coordinate of the thread (a across the first, b across the second), so
// it splits into two closed halves -- the threads with t[8] (resp. t[9]) = 0, then 1 -- and each
// half round trips through LDS alone: 16384 points, 128 KB, in an LDS of 160 KB.  The chain's bins
// arrive the same way: its data slots and aux lists are partitioned per symbol into bins < 16384
// and >= 16384 (t2_plan build_chain_layout / build_aux_lists, natural FFT-input order), which are
// m2 < 16 and m2 >= 16; the pilotgen block's gather mode loads each thread's 32 bins straight
// from global memory.  Thread (a, b) ends with samples b + 32 a + 1024 r: each IQ store is four
// runs of 16 consecutive samples per wave.
// Twiddles: a thread's 31 factors w^(e r) are products of at most three table values w^(e k),
// k in {1, 2, 3, 4, 8, 12, 16} (w_1024^m exact for stage B; the two-level w^i = hi[i >> 7] lo[i & 127]
// for stage A), so each is within a few ulp.
constexpr int O32_NT = 1024, O32_H = 16384, O32_PS = OFDM_PAD_SHIFT_32K;
constexpr int O32_DATA = (O32_H + (O32_H >> O32_PS) + 64) * 8;   // padded half + 64 dummy slots
constexpr int O32_TW1K = O32_DATA;                                // w_1024^m, m < 1024
constexpr int O32_TW2 = O32_TW1K + 1024 * 8;                      // two-level table, 128 + 256
constexpr int O32_QAM = O32_TW2 + 384 * 8;                        // constellation re[nq], im[nq]
constexpr int o32_lds_bytes(int nq) { return O32_QAM + nq * 8; }
static_assert(o32_lds_bytes(OFDM_MAX_QAM) <= 160 * 1024, "32K OFDM LDS");
static_assert((16384 + 2 * 32) * 8 <= O32_DATA, "exchange slots fit the data area");

// bins within a half as the scatter stores them (one pad slot per 32, t2_kernels.h)
__device__ __forceinline__ uint32_t o32_bin(uint32_t k) { return k + (k >> O32_PS); }
// exchange slots: two pad slots per 512 (stride-512 lane patterns spread over the banks, and even
// slots stay 16-byte aligned so exchange 1 reads its value pairs as ds_read_b128)
__device__ __forceinline__ uint32_t o32_x(uint32_t e) { return e + 2u * (e >> 9); }

// v[r] *= w^(e r) for r = 1..31 from the seven table values w^(e k) (k = 1, 2, 3, 4, 8, 12, 16):
// r = 16 t + 4 h + l -> top^t hi[h] lo[l]
template <class Lookup>
__device__ __forceinline__ void o32_twiddle(float2 *v, const Lookup &tw) {
  float2 lo[4], hi[4];
  lo[1] = tw(1); lo[2] = tw(2); lo[3] = tw(3);
  hi[1] = tw(4); hi[2] = tw(8); hi[3] = tw(12);
  const float2 top = tw(16);
#pragma unroll
  for (int r = 1; r < 32; r++) {
    const int t = r >> 4, h = (r >> 2) & 3, l = r & 3;
    float2 w = h == 0 ? lo[l] : (l == 0 ? hi[h] : cmulf(hi[h], lo[l]));
    if (t) w = (h == 0 && l == 0) ? top : cmulf(top, w);
    v[r] = cmulf(v[r], w);
  }
}

// one exchange, as two closed halves: the threads whose bit SPLIT is h write their 32 values and
// read their 32 new ones, h = 0 then 1.  Slots: exchange 1 (SPLIT 8) writes (m0 = a, m1 = b,
// n2 = r) and reads (m0 = a, m1 = r, n2 = b) at (m1 & 15) + 16 (m0 & 15) + 256 (m1 >> 4) + 512 n2;
// exchange 2 (SPLIT 9) writes (n2 = b, m0 = a, n1 = r) and reads (n2 = b, m0 = r, n1 = a) at
// (n2 & 15) + 16 (n1 & 15) + 256 (n1 >> 4) + 512 m0
template <int SPLIT>
__device__ __forceinline__ void o32_exchange(float2 *v, float2 *lds, uint32_t tid, uint32_t a, uint32_t b) {
#pragma unroll
  for (uint32_t h = 0; h < 2; h++) {
    lds_barrier();
    const bool mine = ((tid >> SPLIT) & 1u) == h;
    if (mine) {
#pragma unroll
      for (uint32_t r = 0; r < 32; r++) {
        const uint32_t e = SPLIT == 8 ? (b & 15u) + 16u * (a & 15u) + 256u * (b >> 4) + 512u * r
                                      : (b & 15u) + 16u * (r & 15u) + 256u * (r >> 4) + 512u * a;
        lds[o32_x(e)] = v[r];
      }
    }
    lds_barrier();
    if (mine) {
      if (SPLIT == 8) {
        // values r, r + 1 are adjacent, 16-byte aligned slots: one ds_read_b128 per pair (lanes
        // b = 0..15 at a stride of 514 slots cover the 64 banks; the compiler would otherwise pair
        // the 8-byte reads into ds_read2_b64, at half the LDS rate)
#pragma unroll
        for (uint32_t r = 0; r < 32; r += 2) {
          const uint32_t e = (r & 15u) + 16u * (a & 15u) + 256u * (r >> 4) + 512u * b;
          const float4 q = *(const float4 *)(lds + o32_x(e));
          v[r] = make_float2(q.x, q.y);
          v[r + 1] = make_float2(q.z, q.w);
        }
      } else {
#pragma unroll
        for (uint32_t r = 0; r < 32; r++) {
          const uint32_t e = (b & 15u) + 16u * (a & 15u) + 256u * (a >> 4) + 512u * r;
          v[r] = lds[o32_x(e)];
        }
      }
    }
  }
}

// thread t <-> a = t[4..7] | t8 << 4, b = t[0..3] | t9 << 4
__device__ __forceinline__ uint32_t o32_ta(uint32_t t) { return ((t >> 4) & 15u) | (((t >> 8) & 1u) << 4); }
__device__ __forceinline__ uint32_t o32_tb(uint32_t t) { return (t & 15u) | (((t >> 9) & 1u) << 4); }

// the last radix-2 stage of Dft<32> (len 32) from the DFT-16s of the even (e) and odd (o) inputs: the
// same operations, in the same order per output, as Dft<32>::run, whose first four stages are the two
// DFT-16s (after the 5-bit reversal, positions 0..15 hold the even inputs in 4-bit reversed order)
__device__ __forceinline__ void dft32_combine(float2 *v, const float2 *e, const float2 *o) {
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const float2 a = e[k], b = o[k];
    if (k == 8) {                                   // * i
      v[8] = cadd_i(a, b);
      v[24] = csub_i(a, b);
      continue;
    }
    const float2 t = k == 0 ? b : cmulf(b, make_float2(kCos32[k], kSin32[k]));
    v[k] = cadd(a, t);
    v[k + 16] = csub(a, t);
  }
}

// stages A (twiddle onwards), B, C with the two exchanges: v[r] = the stage-A DFT over m2 of bins
// kin + 1024 r on entry (kin = a + 32 b), sample b + 32 a + 1024 r on exit.  Every thread is past its
// last LDS access of the symbol on return.
__device__ __forceinline__ void o32_fft(float2 *v, float2 *lds, const float2 *tw1k, const float2 *tw2, uint32_t tid,
                                        uint32_t ta, uint32_t tb) {
  const uint32_t kin = ta + 32u * tb;
  // stage A: (DFT over m2, by the caller) twiddle w^((m0 + 32 m1) n2) = w^(kin r)
  o32_twiddle(v, [&](int k) {
    const uint32_t i = kin * (uint32_t)k;   // < 16384
    return cmulf(tw2[128 + (i >> 7)], tw2[i & 127u]);
  });
  o32_exchange<8>(v, lds, tid, ta, tb);
  // stage B: DFT over m1, twiddle w_1024^(m0 n1) = w_1024^(a r)
  __builtin_amdgcn_sched_barrier(0);
  Dft<32>::run(v);
  o32_twiddle(v, [&](int k) { return tw1k[(ta * (uint32_t)k) & 1023u]; });
  o32_exchange<9>(v, lds, tid, ta, tb);
  // stage C: DFT over m0 -> x[b + 32 a + 1024 r]
  __builtin_amdgcn_sched_barrier(0);
  Dft<32>::run(v);
}

// normalisation, guard interval and IQ store of samples b + 32 a + 1024 r, r in [R0, R1)
template <int FMT, int R0, int R1>
__device__ __forceinline__ void o32_store(const float2 *v, const IqOut<FMT> &o, uint32_t nout, float nrm, int G) {
  constexpr uint32_t N = 32768;
#pragma unroll
  for (uint32_t r = R0; r < R1; r++) {
    const uint32_t n = nout + 1024u * r;
    const float2 a = cscale(v[r], nrm);
    o.put((uint32_t)G + n, a);
    if (n >= N - (uint32_t)G) o.put(n - (N - (uint32_t)G), a);
  }
}

// The same store with two consecutive samples per lane (one 16-byte, or 8-byte sc16, store
// instead of two): lanes b and b ^ 1 swap half of their values (DPP quad_perm [1,0,3,2]) so the
// even-b lane holds samples (b, b + 1) of every even r and the odd-b lane those of every odd r.
// Each store instruction then writes eight runs of 16 samples per wave, half the instructions of
// o32_store (the per-CU store issue rate, not HBM, bounds the store phase).  Needs the symbol's
// sample 0 aligned to two samples (always true for the chain's frame layout; checked by the caller).
template <int FMT>
__device__ __forceinline__ void o32_store_pairs(const float2 *v, const IqOut<FMT> &o, uint32_t nout, float nrm, int G) {
  constexpr uint32_t N = 32768;
  const bool odd = nout & 1u;
  const uint32_t n0 = nout & ~1u;
#pragma unroll
  for (uint32_t k = 0; k < 16; k++) {
    const float2 e = cscale(cscale(v[2 * k], nrm), o.gain), d = cscale(cscale(v[2 * k + 1], nrm), o.gain);
    const float2 re = make_float2(swap_adjacent_lane(e.x), swap_adjacent_lane(e.y));
    const float2 rd = make_float2(swap_adjacent_lane(d.x), swap_adjacent_lane(d.y));
    const float2 lo = odd ? rd : e, hi = odd ? d : re;
    const uint32_t n = n0 + 1024u * (2u * k + (odd ? 1u : 0u));
    o.put2((uint32_t)G + n, lo, hi);
    if (n >= N - (uint32_t)G) o.put2(n - (N - (uint32_t)G), lo, hi);
  }
}

// 32K symbols, one workgroup per (symbol, frame): scatter mode (the fused chain), gather mode (the
// pilotgen block: cells already in carrier order) and the carriers-only test hook
template <int FMT, bool MULTI>
__global__ __launch_bounds__(O32_NT) void ofdm32_kernel(OfdmDev d, OfdmIO io) {
  constexpr int N = 32768, NT = O32_NT;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2 *lds = (float2 *)smem;
  float2 *tw1k = (float2 *)(smem + O32_TW1K), *tw2 = (float2 *)(smem + O32_TW2);
  const int tid = threadIdx.x;
  const uint32_t ta = o32_ta((uint32_t)tid), tb = o32_tb((uint32_t)tid);
  const uint32_t kin = ta + 32u * tb;             // stage-A input bins kin + 1024 r
  const int u = xcd_major(blockIdx.x, gridDim.x);
  const int j = u / io.nframes;                   // symbol
  const int f = u - j * io.nframes;               // frame within launch
  const int64_t frame = io.first_frame + (io.frames_per_stream ? f % io.frames_per_stream : f);   // stream-major batch
  const float2 *data = io.data;
  const uint32_t cbase = io.cell_off + (uint32_t)f * io.cell_stride;
  const uint32_t abase = io.aux_off + (uint32_t)(frame % d.t2frames) * (uint32_t)d.aux_len - 1u;
  const int32_t *map = d.bin_map + (int64_t)j * N;
  if (io.carriers_only) {                          // test hook: bins in natural order
    float2 *o = io.out + (int64_t)f * io.out_stride + (int64_t)j * N;
    for (int k = tid; k < N; k += NT) {
      const int code = map[k];
      float2 v = data[code >= 0 ? cbase + (uint32_t)code : abase - (uint32_t)code];
      if (d.isinc) {
        const float sc = d.isinc[(k + N / 2) & (N - 1)];
        v.x *= sc;
        v.y *= sc;
      }
      o[(k + N / 2) & (N - 1)] = v;
    }
    return;
  }
  constexpr int SB = FMT == 0 ? 8 : 4;
  if (j == 0) {                                   // P1 symbol (precomputed), pilotgen:2802-2810
    const IqOut<FMT> p{(char *)io.out + (int64_t)f * io.out_stride * SB, d.gain};
    for (int i = tid; i < 2048; i += NT) p.put((uint32_t)i, d.p1[i]);
  }
  // twiddle tables: loaded here, stored to LDS once the scatter inputs are in flight
  const float2 t1k = d.twiddle1k[tid];
  const float2 t2 = tid < 384 ? d.twiddle[tid] : make_float2(0.f, 0.f);
  float2 v[32];
  // EQ (inverse sinc) of the bins kin + 1024 (S r + h), r < R (before the stage-A DFT)
  auto eq = [&](float2 *x, int R, uint32_t S, uint32_t h) {
    if (d.isinc) {
#pragma unroll
      for (int r = 0; r < R; r++) {
        const float sc = d.isinc[(kin + 1024u * (S * (uint32_t)r + h) + N / 2) & (N - 1)];
        x[r].x *= sc;
        x[r].y *= sc;
      }
    }
  };
  if (d.inv) {
    // scatter mode, one stored half at a time: the bins of even m2, then of odd m2 (t2_plan.h
    // ofdm_stored_index); the even half's DFT-16 runs while the odd half's first loads are in flight
    float *qre = (float *)(smem + O32_QAM), *qim = qre + d.nq;
    const float2 tq = tid < d.nq ? d.qam[tid] : make_float2(0.f, 0.f);   // nq <= OFDM_MAX_QAM = O32_NT
    // the frame's class (FRAME_INTERVAL > 1): its rows of the per-symbol tables, its slots' bins
    const int c = d.ncls > 1 ? (int)(frame % d.ncls) : 0, jc = c * d.Nsym + j;
    BinSource src{map, io.l1, cbase, (uint32_t)f * io.l1_stride - 1u, d.inv + kc(d.cls_inv, c), io.pairs, qre, qim,
                  (uint32_t)kc(d.sym_d0, jc), (uint32_t)kc(d.sym_n, jc), (uint32_t)kc(d.sym_n0, jc), d.abin, d.aval, d.aind,
                  d.agrp + 2 * jc, d.azr + 2 * jc, d.nplp,
                  d.plp_bnd ? d.plp_bnd + 2 * jc * (d.nplp + 1) : nullptr, d.plp_qbase};
    const uint32_t dummy = (uint32_t)(O32_H + (O32_H >> O32_PS)) + (uint32_t)(tid & 63);
    // (measured and dropped: both halves' scatter inputs prefetched into registers before the
    // first half is written, in one batch or half 1 behind half 0's arrival: +11 % kernel time)
    float2 ev[16], od[16];                        // stage-A inputs m2 = 2 r, 2 r + 1
    {
      const int2 zr = kc(src.azr, 0);
      for (int i = zr.x + tid; i < zr.y; i += NT) lds[i] = make_float2(0.f, 0.f);
      if (tid < d.nq) {
        qre[tid] = tq.x;
        qim[tid] = tq.y;
      }
      tw1k[tid] = t1k;
      if (tid < 384) tw2[tid] = t2;
      lds_barrier();                            // constellation visible to the scatter
      scatter_group<NT, 4, MULTI>(lds, src, 0, src.d0, src.dn0, dummy, tid);
      lds_barrier();
#pragma unroll
      for (uint32_t r = 0; r < 16; r++) ev[r] = lds[o32_bin(kin + 1024u * r)];
    }
    lds_barrier();                              // half 0 read back before half 1 overwrites it
    {
      const int2 zr = kc(src.azr, 1);
      for (int i = zr.x + tid; i < zr.y; i += NT) lds[i] = make_float2(0.f, 0.f);
      auto dft_even = [&]() {
        eq(ev, 16, 2u, 0u);
        __builtin_amdgcn_sched_barrier(0);
        Dft<16>::run(ev);
      };
      scatter_group<NT, 4, MULTI>(lds, src, 1, src.d0 + src.dn0, src.dn - src.dn0, dummy, tid, dft_even);
      lds_barrier();
#pragma unroll
      for (uint32_t r = 0; r < 16; r++) od[r] = lds[o32_bin(kin + 1024u * r)];
    }
    eq(od, 16, 2u, 1u);
    __builtin_amdgcn_sched_barrier(0);
    Dft<16>::run(od);
    dft32_combine(v, ev, od);
  } else {
  tw1k[tid] = t1k;
  if (tid < 384) tw2[tid] = t2;
#pragma unroll
  for (int c0 = 0; c0 < 32; c0 += 8) {
    uint32_t off[8];
#pragma unroll
    for (int uu = 0; uu < 8; uu++) {
      const int code = ld_off(map, (kin + 1024u * (uint32_t)(c0 + uu)) * 4u);
      off[uu] = (code >= 0 ? cbase + (uint32_t)code : abase - (uint32_t)code) * 8u;
    }
#pragma unroll
    for (int uu = 0; uu < 8; uu++) v[c0 + uu] = ld_off(data, off[uu]);
    __builtin_amdgcn_sched_barrier(0);
  }
  eq(v, 32, 1u, 0u);
  __builtin_amdgcn_sched_barrier(0);
  Dft<32>::run(v);
  }
  o32_fft(v, lds, tw1k, tw2, (uint32_t)tid, ta, tb);   // its first barrier publishes the tables
  const IqOut<FMT> o{(char *)io.out + ((int64_t)f * io.out_stride + 2048 + (int64_t)j * (N + d.G)) * SB, d.gain};
  if ((((uintptr_t)o.base + (uint32_t)d.G * SB) & (2u * SB - 1u)) == 0)
    o32_store_pairs<FMT>(v, o, tb + 32u * ta, d.norm, d.G);
  else
    o32_store<FMT, 0, 32>(v, o, tb + 32u * ta, d.norm, d.G);
}

template <int N, int FMT, bool MULTI>
static hipError_t launch_ofdm_f(const OfdmDev &d, const OfdmIO &io, hipStream_t s) {
  if (N == 32768) {
    const void *fn = (const void *)ofdm32_kernel<FMT, MULTI>;
    const int lds = o32_lds_bytes(d.inv ? d.nq : 256);
    hipError_t e = lds_limit(fn, o32_lds_bytes(OFDM_MAX_QAM));   // the largest launch
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((ofdm32_kernel<FMT, MULTI>), dim3(d.Nsym * io.nframes), dim3(O32_NT), lds, s, d, io);
    return hipGetLastError();
  }
  constexpr int NN = N > 16384 ? 16384 : N;
  using Sh = OfdmShape<NN>;
  const int lds = Sh::lds_bytes(d.inv ? d.nq : 256);
  hipError_t e = lds_limit((const void *)ofdm_kernel<NN, FMT, MULTI>, Sh::lds_bytes(OFDM_MAX_QAM));   // the largest launch
  if (e != hipSuccess) return e;
  const int units = d.Nsym * io.nframes;
  // units per workgroup: up to 4 for 8K / 16K, 2 below (cfg4 8K: 2.09 -> 1.81 ms with the slot
  // prefetch; runs of 8 or more leave a grid tail at cfg1's 4K launch sizes, profiles/r5_ofdm_runs.txt),
  // and one per workgroup for small launches (a one-frame call keeps its latency)
  const int run = std::max(1, std::min(NN >= 8192 ? 4 : 2, units / 8192));
  hipLaunchKernelGGL((ofdm_kernel<NN, FMT, MULTI>), dim3((units + run - 1) / run), dim3(Sh::NT), lds, s, d, io);
  return hipGetLastError();
}
template <int N, int FMT>
static hipError_t launch_ofdm_m(const OfdmDev &d, const OfdmIO &io, hipStream_t s) {
  return d.inv && d.nplp > 1 ? launch_ofdm_f<N, FMT, true>(d, io, s) : launch_ofdm_f<N, FMT, false>(d, io, s);
}
template <int N>
static hipError_t launch_ofdm_t(const OfdmDev &d, const OfdmIO &io, hipStream_t s) {
  if (d.fmt == 1 && !io.carriers_only) return launch_ofdm_m<N, 1>(d, io, s);
  return d.fmt == 0 || io.carriers_only ? launch_ofdm_m<N, 0>(d, io, s) : hipErrorInvalidValue;
}

hipError_t launch_ofdm(const OfdmDev &d, const OfdmIO &io, hipStream_t s) {
  if (io.nframes <= 0) return hipSuccess;
  if (d.inv && (d.nq < 1 || d.nq > OFDM_MAX_QAM || d.nplp < 1 || d.nplp > 8 || (d.nplp > 1 && (!d.plp_bnd || !d.plp_qbase)) ||
                d.ncls < 1 || !d.cls_inv))
    return hipErrorInvalidValue;
  switch (d.N) {
    case 1024: return launch_ofdm_t<1024>(d, io, s);
    case 2048: return launch_ofdm_t<2048>(d, io, s);
    case 4096: return launch_ofdm_t<4096>(d, io, s);
    case 8192: return launch_ofdm_t<8192>(d, io, s);
    case 16384: return launch_ofdm_t<16384>(d, io, s);
    case 32768: return launch_ofdm_t<32768>(d, io, s);
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
