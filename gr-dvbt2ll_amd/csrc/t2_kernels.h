// t2_kernels.h -- device-side argument blocks and host launchers for the DVB-T2 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace t2 {

// ---------------------------------------------------------------- FEC (BB + BCH + LDPC)
enum FecMode {
  FEC_TS_TO_BBFRAME = 0, // chain: TS bytes -> BBFRAME rows + BCH partial parities (one fused pass: the BBFRAME
                         // built in registers, BCH on the matrix cores); launch_ldpc_map continues from them
  FEC_TS_TO_BITS = 1,    // bbheaderbch block: TS bytes -> unpacked nbch bits
  FEC_BITS_TO_BITS = 2,  // ldpc block: unpacked nbch bits -> unpacked nldpc bits (natural)
};

// the chain's BCH (bbch_kernel): K slices (slice = blockIdx % 2: the even XCDs take slice 0, the odd ones
// slice 1, so each XCD's L2 holds half the generator table; 2 slices measured 2 % faster than 8 and 1 %
// faster than 4 or 1 in round 4: fewer tile-segment prologues, epilogues and atomics); parity words per
// block (the slices XOR their partial parities into them)
constexpr int BCH_KS = 2;
constexpr int BCH_PART_WORDS = 8;

struct FecDev {
  const uint64_t *bch_tab;      // 256 x 3
  const uint64_t *bch_ctab;     // [P/4][16][64] x 4: lane shift nibble tables (FecPlan::bch_ctab)
  const uint16_t *ldpc_rowptr;  // q + 1
  const uint32_t *ldpc_ent;     // nent
  const uint8_t *prbs;          // kbch / 8
  const uint8_t *crc8_tab;      // 256
  const uint8_t *crc8_shift;    // 8 x 256
  const uint8_t *hcrc_bits;     // 72: BBHEADER CRC-8 contribution of each header bit
  const uint4 *bch_mfma;        // chain: fp4 B fragments of the BCH generator matrix (FecPlan::bch_mfma)
  int bch_nq, bch_nt;           // chain: 32-byte message chunks, 32-parity tiles of bch_mfma
  int kbch, nbch, P, nldpc, q, nent, chunk, parity_il;   // chunk: BCH message bytes per lane (64 lanes)
  int hem, inband, fec_blocks, ts_rate;
  // BBHEADER MATYPE-1 << 8 | MATYPE-2: 0xF000 = TS, SIS, CCM, ISSYI 0, NPD 0, RO 0, ISI 0 (the reference's
  // ctor, bbheader:168-182); 0xD000 | ISI = multiple input streams (one PLP of a multi-PLP frame, :288-298)
  int matype;
};
constexpr int MATYPE_SIS = 0xF000, MATYPE_MIS = 0xD000;

struct FecIO {
  const uint8_t *in;       // TS bytes (ts modes) or unpacked bits
  int64_t ts_base;         // absolute stream offset of in[0] (ts modes)
  int64_t ts_len;
  int64_t first_block;     // absolute FEC block index of launch block 0
  uint8_t *out;            // packed codewords (stride cw_stride) or unpacked bits
  int64_t cw_stride;
  int nblocks;
  uint32_t *sync_err;      // ts modes, optional: += TS sync bytes != 0x47 consumed (bbheader:675, 703)
  // multi-stream batch (chain, ts modes): 0 = one stream; else launch block b belongs to stream
  // b / blocks_per_stream, whose TS bytes start at in + stream * ts_stride (same ts_base, ts_len)
  int blocks_per_stream;
  int64_t ts_stride;
  // chain (FEC_TS_TO_BBFRAME): BCH parity of launch block b at bch_part + b * BCH_PART_WORDS (zero before the
  // launch, XOR-accumulated by the K slices of the fused BB + BCH pass, read and zeroed again by
  // launch_ldpc_map; room for bch_part_blocks >= nblocks).  out has a spare row at nblocks (dead lanes' stores).
  uint32_t *bch_part;
  int64_t bch_part_blocks;
  // launch_ldpc_map (test hook): 1 = also store each block's interleaver-input codeword into its row
  // (the BBFRAME already there), 0 = the codeword stays in LDS
  int keep_cw;
};

// ---------------------------------------------------------------- L1-post signalling (t2_plan.h L1PostPlan)
struct L1Dev {
  const uint32_t *tmpl;      // per frame class (frame mod ncls): signal bits, FRAME_IDX and CRC zero
  const uint32_t *crc_c;     // nsig - 32
  const uint32_t *scr;       // L1 scrambler bits or null
  const uint16_t *sig_pos;   // nsig
  const uint32_t *bch_r;     // nsig x 6
  const uint16_t *ldpc_ptr;  // 21
  const uint16_t *ldpc_addr;
  const uint16_t *sel;       // npost
  const float2 *lut;         // 64 (QPSK / 16QAM / 64QAM)
  uint32_t crc_k;
  int nsig, fidx_pos, npost, lp, mode, ncols, rows, q, pbits, t2frames, ncls;
  uint8_t mux[12];
};
struct L1IO {
  float2 *out;               // frame f's Lp cells at out + f * out_stride
  int64_t out_stride;
  int64_t first_frame;       // frame f has t2_frame_num (first_frame + f % frames_per_stream) % t2frames
  int nframes;
  int frames_per_stream;     // 0: one stream
};

// ---------------------------------------------------------------- bit interleave + QAM + CI
struct MapDev {
  const float2 *lut;       // 256 (block API)
  int mode, mod, W, R, cs, nldpc, nbch, q, rotation, parity_il;
  int F;                   // chain: FEC blocks per frame (launch block b is FEC block b mod F of frame b / F)
  // chain: block r's cell interleaver + time-interleaver store in aligned quads of four frame slots,
  // sorted by slot (map_store_quads): quad n at r * slot_stride + n holds the cell-interleaver input
  // index j < 0x8000 of each of its slots (0x8000: another block's slot) and its quad index minus
  // slot_qbase[r * slot_stride / 64 + n / 64]; slot_nq[r] quads
  const uint2 *slot_quad;
  const uint16_t *slot_qoff;
  const int32_t *slot_qbase, *slot_nq;
  int slot_stride;
  // per demuxed bit b of the row word: the column e feeding it (W-1-mux[e] = b) as (its first codeword
  // bit e*R (-1: none), its twist); int32 in device memory: uniform scalar loads where map_cells uses
  // them, no byte loads in the column loop
  const int2 *col;         // 16
};
struct MapIO {
  const uint8_t *in;   // block API: unpacked natural-order codeword bits, nldpc per block
  float2 *out;         // block API: cs cells per block
  // chain (launch_ldpc_map): per cell the constellation index pair lo = idx[j], hi = idx[j-1]
  // (rotation) or idx[j], frame k's data region at out_pairs + k * frame_stride
  uint16_t *out_pairs;
  int64_t frame_stride;
  int nblocks;
};

// ---------------------------------------------------------------- OFDM symbols
// LDS layout of a sub-transform: bin k of the half lives at float2 slot k + (k >> pad shift)
// (one pad slot per 2^shift; the chain's bin tables are stored already padded)
constexpr int OFDM_PAD_SHIFT_32K = 5;
__host__ __device__ inline int ofdm_pad_shift(int N) { return N > 16384 ? OFDM_PAD_SHIFT_32K : 4; }
__host__ __device__ inline uint32_t ofdm_padded_bin(int N, uint32_t k) {   // k: bin within its half
  return k + (k >> ofdm_pad_shift(N));
}
constexpr int OFDM_MAX_QAM = 1024;   // constellation entries the OFDM kernels hold in LDS (all PLPs' tables)
struct OfdmDev {
  const int32_t *bin_map;   // Nsym x N (natural FFT-input order): >= 0 cell index, < 0 aux entry
  // chain (scatter) mode: symbol j's cells are the slots [sym_d0[j], +sym_n[j]), slot s goes to
  // stored bin inv[s]; null -> gather mode (bin_map >= 0 codes are read per bin)
  const uint16_t *inv;       // padded bin within the symbol's half (ofdm_padded_bin)
  const int32_t *sym_d0, *sym_n, *sym_n0;   // sym_n0: slots of the bins < N/2 (32K: two halves)
  const float2 *twiddle;    // 128 + N/128: two-level table (PilotPlan::twiddle)
  const float2 *twiddle1k;  // 1024: w_1024^m (PilotPlan::twiddle1k; 32K kernel)
  const float *isinc;       // N or null
  const float2 *p1;         // 2048
  const float2 *qam;        // scatter mode: nq-entry constellation table(s); cell = (qam[b + lo].x, qam[b + hi].y),
                            // b = the cell's PLP's table base plp_qbase[p] (0 with one PLP)
  int nq;                   // entries of qam: 256 for one PLP, <= OFDM_MAX_QAM (the PLPs' tables back to back)
  // multi-PLP frames (nplp > 1): the PLP of data slot s in group g (2 j + h) is the p with
  // plp_bnd[g (nplp + 1) + p] <= s < plp_bnd[g (nplp + 1) + p + 1] (t2_plan ChainLayout::plp_bnd)
  int nplp;
  const int32_t *plp_bnd;
  const int32_t *plp_qbase;   // nplp: PLP p's table starts at entry plp_qbase[p] of qam
  // frame classes (FRAME_INTERVAL > 1: t2_plan.h FrameClass): frame f uses class c = f mod ncls, whose
  // per-symbol tables (sym_*, agrp, azr, plp_bnd) are the rows of symbol c Nsym + j and whose data slots'
  // bins start at inv + cls_inv[c]
  int ncls;
  const int32_t *cls_inv;
  // scatter mode: non-data bins as compact lists per (symbol, half) group 2 j + h (t2_plan.h
  // AuxLists): agrp[g] = {direct offset, direct count, indirect offset, indirect count}
  const uint16_t *abin;     // direct padded bins, quads (0xFFFF = padding)
  const float2 *aval;       // direct values
  const uint32_t *aind;     // indirect: padded bin | code << 15, value at aux abase + code
  const int4 *agrp;
  const int2 *azr;          // per group: padded LDS slot range [x, y) zeroed as a run (AuxLists::zrun)
  int N, G, Nsym, aux_len, t2frames;
  float norm;
  float gain;               // output gain after the normalisation (1 = pilotgen's own output)
  int fmt;                  // IQ format: 0 complex64, 1 int16 I/Q (sc16, full scale 32767)
};
struct OfdmIO {
  const float2 *data;       // gather mode: aux variants at aux_off, frame f cells at cell_off + f*cell_stride
                            // scatter mode: aux variants only
  uint32_t aux_off;         // element offset of aux variant 0 (variant v at aux_off + v*aux_len)
  uint32_t cell_off;
  uint32_t cell_stride;     // elements; scatter mode: a multiple of 4
  const uint16_t *pairs;    // scatter mode: frame f's constellation index pairs at f*cell_stride
  float2 *out;              // per frame: out_stride samples
  int64_t out_stride;
  int64_t first_frame;
  int nframes;
  int frames_per_stream;    // multi-stream batch: launch frame f is frame first_frame + f % frames_per_stream
                            // of stream f / frames_per_stream (0: one stream)
  int carriers_only;        // test hook: write pre-IFFT bins (natural bin order) instead
  // scatter mode: the indirect aux entries (per-frame L1-post cells) of frame f read l1 +
  // f * l1_stride + code - 1 (written by the l1post kernel of the same run)
  const float2 *l1;
  uint32_t l1_stride;
};

// ---------------------------------------------------------------- frame-mapper gather
struct GatherIO {
  const float2 *in;
  float2 *out;
  const int32_t *map;       // M
  const float2 *aux;        // aux_len (one variant)
  int M;
};

hipError_t launch_fec(int mode, const FecDev &d, const FecIO &io, hipStream_t s);
hipError_t launch_map(const MapDev &d, const MapIO &io, hipStream_t s);
// the chain after FEC_TS_TO_BBFRAME: LDPC of fio's BBFRAME rows + BCH partials, then the map (column twist,
// demux, cell interleaver, TI store into mio.out_pairs) of the same blocks, one kernel; l1d / l1io
// (optional): the frames' L1-post cells by extra workgroups of the same launch
hipError_t launch_ldpc_map(const FecDev &fd, const FecIO &fio, const MapDev &md, const MapIO &mio, hipStream_t s,
                           const L1Dev *l1d = nullptr, const L1IO *l1io = nullptr);
hipError_t launch_ofdm(const OfdmDev &d, const OfdmIO &io, hipStream_t s);
hipError_t launch_gather(const GatherIO &io, hipStream_t s);
hipError_t launch_l1post(const L1Dev &d, const L1IO &io, hipStream_t s);

}  // namespace t2
