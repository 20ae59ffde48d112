// t2_plan.h -- configuration-time planning for the MI355X DVB-T2 chain.
//
// Everything the reference blocks compute in their constructors (FEC parameters, BCH
// generator, LDPC address tables, QAM tables, cell/frequency interleaver permutations,
// L1 signalling cells, pilot carrier maps, P1) is computed once here on the host and
// turned into the compact device-side tables the kernels consume:
//   * FecPlan   -> bit-packed BCH (byte table + Horner matrices) and a quasi-cyclic LDPC
//                  schedule (row a of the q x 360 parity array <- rotated info groups)
//   * MapPlan   -> bit-interleaver geometry + constellation LUT
//   * FramePlan -> cell interleaver shifts/permutation and a gather map from every mapped
//                  (frequency-interleaved) cell to its source cell / L1 / dummy entry
//   * PilotPlan -> per-symbol gather map from every IFFT input bin to a source cell,
//                  pilot value or zero; P1 samples; twiddles
// Reference constructors: lib/bbheaderbch_bb_impl.cc:42-196, lib/interleavermod_bc_impl.cc:42-255,
// lib/framemapperfint_cc_impl.cc:41-1190, lib/pilotgenp1insert_cc_impl.cc:43-1229.
#pragma once
#include <cstdint>
#include <vector>

namespace t2 {

struct cf32 {
  float re, im;
};

// ----------------------------------------------------------------------------- FEC
struct FecPlan {
  int normal = 0, rate = 0;
  int kbch = 0, nbch = 0, nparity = 0, nldpc = 0, q = 0, pbits = 0;
  bool parity_interleave = true;      // tempu carries parity in [a][c] (interleaved) order
  int bch_chunk = 0;                  // message bytes per lane chunk (64 lanes of one wave)
  std::vector<uint64_t> bch_tab;      // 256 x 3 words: d(x) * x^P mod g(x)
  // per-lane chunk shift as nibble tables: entry [j][v][lane] (4 words, the 4th zero) =
  // v x^(4 j) x^(8 chunk (63 - lane)) mod g for nibble j < P/4, value v < 16, lane < 64
  std::vector<uint64_t> bch_ctab;
  // the chain's BCH as a GF(2) matrix product on the matrix cores (bch_gemm_kernel): fp4 B
  // fragments [32-byte message chunk q < bch_nq][K-step u < 4][parity tile t < bch_nt][lane][4
  // dwords] of the parity-generator matrix (layout: build_bch_mfma)
  int bch_nq = 0, bch_nt = 0;
  std::vector<uint32_t> bch_mfma;
  std::vector<uint16_t> ldpc_rowptr;  // q + 1
  std::vector<uint32_t> ldpc_ent;     // (group << 16) | rotation, grouped by parity row
  std::vector<uint8_t> prbs_bytes;    // BB scrambler, kbch/8 bytes
  std::vector<uint8_t> crc8_tab;      // CRC-8 (0xD5) table, 256
  std::vector<uint8_t> crc8_shift;    // 8 x 256: crc after appending k zero bytes (packet CRC combine)
  std::vector<uint8_t> hcrc_bits;     // 72: BBHEADER CRC-8 contribution of each header bit
};
int build_fec(int framesize, int rate, int constellation, FecPlan &fp);
// fp.bch_nq / bch_nt / bch_mfma for a plan built by build_fec (the fused chain only)
int build_bch_mfma(FecPlan &fp);

// ----------------------------------------------------------------------------- bit interleave + map
enum MapMode { MAP_PAIRS = 0, MAP_TWIST2 = 1, MAP_TWIST1 = 2 };
struct MapPlan {
  int mode = 0, mod = 0, W = 0, R = 0, cs = 0, nldpc = 0, rotation = 0;
  uint8_t twist[16] = {0}, mux[16] = {0};
  cf32 lut[256] = {};
};
int build_map(int framesize, int rate, int constellation, int rotation, MapPlan &mp);
// reference QAM tables (used for data cells and L1-post cells)
void qam_table(int constellation, int rotation, cf32 *lut, int *mod);

// ----------------------------------------------------------------------------- frame mapper
struct FmParams {
  int framesize, rate, constellation, rotation, fecblocks, tiblocks, carriermode, fftsize,
      guardinterval, l1constellation, pilotpattern, t2frames, numdatasyms, paprmode, version,
      preamble, inputmode, reservedbiasbits, l1scrambled, inband;
};
// One data PLP of a multi-PLP frame (EN 302 755 6.5, 8.3.6.3).  The reference carries exactly one PLP
// (framemapper:152-250: num_plp 1, plp_type 1, time_il_type 0, frame_interval 1); a frame here carries
// nplp of them, PLP_ID = index, each with its own FEC, constellation, cell and time interleaver.
//  - TIME_IL_TYPE 0 (the reference's): one interleaving frame (fecblocks FEC blocks, tiblocks TI blocks)
//    per T2 frame.  TIME_IL_TYPE 1: one TI block (tiblocks = 1) of fecblocks FEC blocks per interleaving
//    frame, spread over P_I = ti_frames T2 frames: T2 frame i of interleaving frame m (global frame
//    m P_I + i) carries its TI output cells [i S, (i + 1) S), S = fecblocks cs / P_I.  FRAME_INTERVAL 1.
//  - Type-1 PLPs occupy one run of S data cells each, back to back in PLP_ID order after the L1
//    signalling (PLP_START = start); then the Type-2 PLPs, sub-sliced: sub-slice j (S / nss cells) of
//    every Type-2 PLP in PLP_ID order, then sub-slice j + 1 (SUB_SLICE_INTERVAL ssi, TYPE_2_START t2start).
//  - FRAME_INTERVAL I_JUMP (7.2.3.1): the PLP occurs only in the T2 frames f with f mod I_JUMP = FIRST_FRAME_IDX;
//    its interleaving frame spans P_I of those.  The frames then differ in which PLPs they carry: frame
//    class c = f mod ncls (ncls = lcm of the I_JUMPs) has its own placement (FrameClass).
struct PlpParams {
  int framesize, rate, constellation, rotation, fecblocks, tiblocks, inputmode, inband;
  int plp_type = 1, ti_type = 0, ti_frames = 1, frame_interval = 1, first_frame = 0;
};
struct PlpPlan {
  int cs = 0, F = 0, S = 0, start = 0;   // F: FEC blocks per interleaving frame; S: cells per T2 frame
  int S_if = 0, P = 1;                   // cells per interleaving frame (F cs), its T2 frames (P_I)
  int I = 1, FF = 0;                     // FRAME_INTERVAL, FIRST_FRAME_IDX
  int cycle() const { return P * I; }    // T2 frames from one interleaving frame's first frame to the next's
  int type2 = 0, ss = 0, ss_off = 0;     // Type 2: sub-slice cells, offset within a sub-slice group
  int in_off = 0;                        // framemapper block: the PLP's interleaving frame in its input buffer
  int ti_on = 0, ti_small = 1, ti_big = 1, ti_nsmall = 0;
  std::vector<int16_t> ci_perm;          // cs
  std::vector<int32_t> ci_shift;         // F
};
constexpr int MAX_PLP = 8;

// aux table (per t2_frame_num variant): [0] zero, [1..12] pilot values, then L1-pre,
// L1-post, dummy cells.  Gather codes: >= 0 cell index, < 0 -> aux index (-code - 1).
constexpr int AUX_ZERO = 0;
constexpr int AUX_PILOT0 = 1;
constexpr int AUX_L1PRE = 13;
// L1-post signalling (framemapper:1536-1910), generated per T2 frame on the GPU (l1post_kernel):
// the configurable + dynamic fields as a bit template whose only per-frame field is FRAME_IDX
// (= t2_frame_num, :1648-1651), CRC-32 (:1203-1224) as the XOR of per-bit contributions, the
// optional L1 scrambler (:1928-1940), shortening into the 7032-bit BCH information word (padding
// groups :2190-2233), BCH(168) as the XOR of per-position remainders x^(168 + 7031 - p) mod g(x)
// (:1269-1312), the LDPC 1/2 (16K) accumulate over its address table (:1314-1364), puncturing,
// and the L1 constellation with the 16/64QAM bit interleaver + demux (:1832-1908).
constexpr int L1_MAX_SIG = 2048;   // signalling bits the GPU L1-post generator holds (t2_kernels L1_SIG_WORDS)
struct L1PostPlan {
  int nsig = 0;                    // signalling bits including the CRC-32
  int fidx_pos = 0;                // bit position of FRAME_IDX (8 bits, MSB first)
  int npost = 0, lp = 0;           // transmitted bits N_post, cells Lp
  int mode = 0;                    // L1 constellation: 0 BPSK, 1 QPSK, 2 16QAM, 3 64QAM
  int ncols = 0, rows = 0;         // 16/64QAM bit interleaver geometry
  int q = 0, pbits = 0;            // LDPC: 25, 9000
  uint32_t crc_k = 0;              // CRC-32 of the all-zero message (the 0xFFFFFFFF init's share)
  std::vector<uint32_t> tmpl;      // per frame class ceil(nsig / 32) words, MSB first; FRAME_IDX and CRC fields 0
  int ncls = 1;
  std::vector<uint32_t> crc_c;     // nsig - 32: CRC-32 contribution of message bit i
  std::vector<uint32_t> scr;       // ceil(nsig / 32) words of L1 scrambler PRBS, empty when off
  std::vector<uint16_t> sig_pos;   // nsig: position of signal bit i in the 7032-bit BCH info word
  std::vector<uint32_t> bch_r;     // nsig x 6 words: BCH parity of a 1 at sig_pos[i] (parity bit n
                                   //   at word n / 32, bit 31 - n % 32)
  std::vector<uint16_t> ldpc_ptr;  // 21: address list of information group g at [ptr[g], ptr[g + 1])
  std::vector<uint16_t> ldpc_addr; // parity addresses x: info bit 360 g + n feeds (x + n q) mod pbits
  std::vector<uint16_t> sel;       // npost: codeword index (info | BCH parity | LDPC parity) per bit
  uint8_t mux[12] = {};
  cf32 lut[64] = {};
};

// The T2 frames f with f mod ncls = c: which PLPs they carry and where (8.3.6.3 over the present PLPs).
struct FrameClass {
  int S = 0, D = 0, ssi = 0, t2start = 0;   // data cells, dummy cells, SUB_SLICE_INTERVAL, TYPE_2_START
  std::vector<uint8_t> present;             // per PLP
  std::vector<int32_t> start, ss_off;       // per PLP: PLP_START (0 when absent), Type 2: offset in a sub-slice group
  std::vector<int32_t> gather_d;            // M: mapped cell -> frame data index (< S) | aux
};
// The single-PLP fields (cs, F, ci_perm, ci_shift, ti_*) are PLP 0's; S is the total over the PLPs (the
// largest of the frame classes'), D the most dummy cells of any class.
struct FramePlan {
  int nplp = 1;
  int nss = 1, ssi = 0, t2start = 0;     // SUB_SLICES_PER_FRAME, SUB_SLICE_INTERVAL, TYPE_2_START
  int unit = 1;                          // T2 frames per launch unit: lcm of the PLPs' P_I x I_JUMP (frame phases)
  int ncls = 1;                          // frame classes: lcm of the PLPs' I_JUMP (frame f has class f mod ncls)
  std::vector<FrameClass> cls;
  int S_in = 0;                          // framemapper block input: every PLP's interleaving frame (sum S_if)
  std::vector<PlpParams> plp_in;         // the PLPs' parameters
  std::vector<PlpPlan> plp;
  int cs = 0, F = 0, S = 0, M = 0, N_P2 = 0, C_P2 = 0, C_DATA = 0, N_FC = 0, C_FC = 0;
  int eta = 0, N_post = 0, N_punc = 0, Lp = 0, D = 0, num_data_symbols = 0, t2frames = 0;
  int aux_len = 0;                       // entries per variant
  std::vector<int16_t> ci_perm;          // cs
  std::vector<int32_t> ci_shift;         // F (per FEC block of a frame)
  std::vector<int32_t> gather_d;         // M: mapped cell -> frame data-region index (TI output order) | aux
  int ti_on = 0, ti_small = 1, ti_big = 1, ti_nsmall = 0;   // TI blocks: ti_nsmall of ti_small FEC blocks, then ti_big
  std::vector<int32_t> gather_in;        // unit x M: per frame phase (global frame mod unit), mapped cell ->
                                         //   framemapper input index | aux (input: the current interleaving
                                         //   frame of every PLP, PLP k's S_if cells at plp[k].in_off)
  // host_l1post: t2frames x aux_len with every variant's L1-post cells (the CPU tests' cross-check);
  // else one variant whose L1-post cells [AUX_L1PRE + 1840, + Lp) are left zero for the GPU
  std::vector<cf32> aux;
  int aux_variants = 0;
  L1PostPlan l1;
};
// host_l1post: also encode every t2_frame_num variant's L1-post on the host (tests only; the
// product generates L1-post per frame on the GPU from fp.l1)
int build_frame(const FmParams &p, FramePlan &fp, bool host_l1post = false);
// nplp PLPs; the per-PLP fields of p (framesize .. fecblocks, tiblocks, inputmode, inband) are ignored;
// nss: SUB_SLICES_PER_FRAME (1 without Type-2 PLPs)
int build_frame_mplp(const FmParams &p, const std::vector<PlpParams> &plps, FramePlan &fp, bool host_l1post = false,
                     int nss = 1);
// fp.l1 from the parameters and fp's L1 geometry (called by build_frame)
int build_l1post_plan(const FmParams &p, FramePlan &fp);
// the L1-post signalling bits before the CRC-32 (one per byte) of FRAME_IDX frame_idx (a frame of class
// frame_idx mod ncls); *fidx_pos: FRAME_IDX's first bit (framemapper:1553-1691 with the frame's PLP loops)
std::vector<uint8_t> l1post_signal(const FmParams &p, const FramePlan &fp, int frame_idx, int *fidx_pos);
// one FRAME_IDX variant's Lp L1-post cells, encoded bit by bit on the host (tests only)
int l1post_host(const FmParams &p, const FramePlan &fp, int frame_idx, cf32 *dst);

// ----------------------------------------------------------------------------- pilots + OFDM
struct PgParams {
  int carriermode, fftsize, pilotpattern, guardinterval, numdatasyms, paprmode, version, preamble,
      misogroup, equalization, bandwidth, vlength;
};
struct PilotPlan {
  int N = 0, fft = 0, C_PS = 0, K_EXT = 0, K_OFFSET = 0, G = 0, Nsym = 0, N_P2 = 0, active = 0;
  int left_nulls = 0, eq = 0;
  float normalization = 0.f;
  cf32 pilot_values[12] = {};            // aux[1..12]
  std::vector<int32_t> bin_map;          // Nsym x N, indexed by IFFT input position k (fftshifted)
  std::vector<float> isinc;              // N (pre-shift bin order), only if eq
  std::vector<cf32> p1;                  // 2048
  std::vector<cf32> twiddle;             // 128 + N/128: [lo: w^l, l < 128][hi: w^(128 h)], w = exp(2 pi i / N)
  std::vector<cf32> twiddle1k;           // 1024: exp(2 pi i m / 1024) (the 32K kernel's second pass)
};
int build_pilot(const PgParams &p, PilotPlan &pp);

int fft_points(int fftsize);

// ----------------------------------------------------------------------------- fused chain layout
// The OFDM kernels read the per-symbol map rows in IFFT-input order k; for N > 16384 the 32K
// kernel fills its bins one half (k < N/2, then k >= N/2) at a time.
inline bool ofdm_split(int N) { return N > 16384; }
// The fused chain's stored bin order.  32K: the two halves the kernel fills one at a time are the
// bins of even and of odd m2 = k >> 10 (k: natural FFT-input index), so the half read back first
// holds the even inputs of every stage-A DFT-32, whose DFT-16 then runs beside the second half's
// scatter.  Stored index s = h N/2 + kr with h = (k >> 10) & 1, kr = (k & 1023) | (k >> 11) << 10;
// N <= 16K: s = k.  (The pilotgen block's gather rows stay in natural order.)
inline int ofdm_stored_index(int N, int k) {
  return ofdm_split(N) ? ((k >> 10) & 1) * (N / 2) + ((k & 1023) | ((k >> 11) << 10)) : k;
}
std::vector<int32_t> ofdm_stored_rows(int N, int Nsym, const std::vector<int32_t> &bin_map);

// Fused chain layout.  The LDPC + map kernel writes each FEC block's cells through the cell and time
// interleavers into the frame data region, which is then in transmission (TI output) order:
// symbol j's data cells are the contiguous slots [sym_d0[j], sym_d0[j] + sym_n[j]).  The OFDM
// kernel streams that range with unit-stride loads and scatters each cell into its IFFT bin in
// LDS (inv), after filling pilot / null / L1 / dummy bins from the aux table (cmap < 0).
// For N = 32K each symbol's run is further partitioned [cells of bins < N/2 | cells of bins >= N/2]
// (each part in TI output order), so a half streams only its own cells; `part` maps the TI output
// index to that slot (empty: identity).
struct ChainLayout {
  std::vector<int32_t> cmap;     // Nsym x N, stored row order: >= 0 data slot, < 0 aux (-code - 1)
  std::vector<uint16_t> inv;     // S: data slot -> stored bin index within its symbol's row
  std::vector<int32_t> sym_d0, sym_n, sym_n0;   // Nsym: run start, length, cells of the first half
  std::vector<int32_t> part;     // S: TI output index -> data slot (split only)
  // per (symbol, half) group g = 2 j + h (h = 0 when N is not split): the first data slot of each PLP in
  // the group's slot range, plp_bnd[g * (nplp + 1) + p], p = 0..nplp (the last = the range's end); a
  // group's slots are PLP-major, so slot s of the group belongs to the PLP p with bnd[p] <= s < bnd[p + 1]
  std::vector<int32_t> plp_bnd;
};
// the layout of the T2 frames of class cls
int build_chain_layout(const FramePlan &fp, const PilotPlan &pp, ChainLayout &cl, int cls = 0);

// Non-data bins of the fused chain as compact per-(symbol, half) lists, group g = 2 j + h
// (h = 0 when N is not split), bins relative to the half.  The OFDM kernel zero-fills its
// LDS buffer, then writes:
//   direct entries (bin, value): aux cells equal in every t2_frame_num variant (pilots,
//     L1-pre, dummy cells), each group padded to a multiple of 4 with bin 0xFFFF;
//   indirect entries bin | code << 15: the per-frame L1-post cells, read from the frame's row of
//     the L1 buffer at abase + code (see build_aux_lists).
// Null bins and +0 aux values are left out (the zero fill covers them).
struct AuxLists {
  std::vector<uint16_t> dbin;
  std::vector<cf32> dval;
  std::vector<uint32_t> ind;
  std::vector<int32_t> grp;   // 4 per group: direct offset, direct count, indirect offset, count
  // 2 per group: the longest run [z0, z1) of zero bins (band-edge nulls), zeroed by the kernel
  // as a range; every other zero bin is a direct entry with value 0
  std::vector<int32_t> zrun;
};
// aux indices [l1_lo, l1_lo + l1_len) are the per-frame L1-post cells: always indirect, code = index
// within the L1-post cells + 1 (the chain reads them from the frame's row of the L1 buffer the
// l1post kernel writes); l1_len = 0: indirect codes are aux index + 1 into the frame's variant
int build_aux_lists(const ChainLayout &cl, int N, int Nsym, const std::vector<cf32> &auxv, int aux_len,
                    int t2frames, AuxLists &al, int l1_lo = 0, int l1_len = 0);
// time-interleaver output index (within the interleaving frame, [0, S_if)) of cell-interleaved cell t of FEC
// block r of PLP plp (framemapper:1999-2028)
int64_t ti_index(const FramePlan &fp, int plp, int r, int t);
// frame data-region index of cell c (< S) of PLP plp in a T2 frame of class cls (8.3.6.3: Type-1 run or Type-2
// sub-slices)
int32_t plp_cell_pos(const FramePlan &fp, int plp, int c, int cls = 0);
// where cell t of FEC block r of PLP plp lands when its interleaving frame starts at T2 frame f0 (a multiple of
// the PLP's cycle): T2 frame f0 + off (off = FIRST_FRAME_IDX + I_JUMP i for the interleaving frame's i-th frame),
// frame data index pos
struct CellDest {
  int off;
  int32_t pos;
};
inline CellDest cell_dest(const FramePlan &fp, int plp, int r, int t, int64_t f0 = 0) {
  const PlpPlan &pl = fp.plp[plp];
  const int64_t u = ti_index(fp, plp, r, t);
  const int off = pl.FF + pl.I * (int)(u / pl.S);
  return CellDest{off, plp_cell_pos(fp, plp, (int)(u % pl.S), (int)((f0 + off) % fp.ncls))};
}

// framemapper cell counts {N_P2, C_P2, C_DATA, N_FC, C_FC} (framemapper:290-356, 425-915); -1 if invalid
int frame_cell_counts(int fftsize, int carriermode, int pp, int papr, int gi, int preamble, int out[5]);

}  // namespace t2
