/*
 * dvbt2_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the gr-dvbt2ll reference blocks, used exclusively as the
 * parity checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg.  The product (gr-dvbt2ll_amd/) never links, loads or calls this code.
 *
 * PARITY UNPINNED: the reference lib/<block>_impl.cc needs GNU Radio, gr-fft/FFTW and VOLK
 * headers and libraries that this image lacks, so it is unbuildable here, and the
 * reference ships no golden vectors or assertions (its qa_* tests are empty).
 * This restatement is pinned only by published known-answer values (CRC-8/DVB-S2,
 * CRC-32/MPEG-2, the DVB energy-dispersal PRBS), by code-structure invariants
 * (BCH divisibility, LDPC parity checks) and by cross-checks between independent
 * reference tables (C_P2/C_DATA/N_FC vs. the pilot maps).  See DESIGN.md.
 *
 * Every function cites the reference file:line it follows.  Semantics are those
 * of one general_work call per FEC block (interleavermod) and per T2 frame
 * (framemapperfint, pilotgenp1insert); see SURVEY.md section 5 for why.
 */
#ifndef DVBT2_ORACLE_H
#define DVBT2_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_bb orc_bb;
typedef struct orc_ldpc orc_ldpc;
typedef struct orc_im orc_im;
typedef struct orc_fm orc_fm;
typedef struct orc_pg orc_pg;

/* bbheaderbch_bb (include/dvbt2ll/bbheaderbch_bb.h:49) */
orc_bb *orc_bb_create(int framesize, int rate, int mode, int inband, int fecblocks, int tsrate);
int orc_bb_nbch(const orc_bb *h);
int orc_bb_kbch(const orc_bb *h);
int orc_bb_forecast(const orc_bb *h, int noutput_items);
/* returns noutput_items; *consumed = input bytes consumed */
int orc_bb_work(orc_bb *h, int noutput_items, const uint8_t *in, uint8_t *out, int *consumed);
/* one PLP of a multi-PLP frame: MATYPE SIS/MIS = multiple, MATYPE-2 ISI = isi (the PLP_ID;
 * bbheader:288-298).  Parity unpinned (the reference's ctor fixes SIS, :168). */
void orc_bb_set_isi(orc_bb *h, int isi);
void orc_bb_destroy(orc_bb *h);

/* LDPC encoder, reference-owned restatement of ldpc_calculate (lib/bbheaderbch_bb_impl.cc:533-646),
 * standing in for gr-dtv dvb_ldpc_bb (apps/vv009-4kshort.grc:386-460).  nblocks FEC blocks of
 * nbch unpacked bits -> nldpc unpacked bits (natural parity order). */
orc_ldpc *orc_ldpc_create(int framesize, int rate);
int orc_ldpc_work(orc_ldpc *h, int nblocks, const uint8_t *in, uint8_t *out);
void orc_ldpc_destroy(orc_ldpc *h);

/* interleavermod_bc (include/dvbt2ll/interleavermod_bc.h:49); out is interleaved re,im float32 */
orc_im *orc_im_create(int framesize, int rate, int constellation, int rotation);
int orc_im_cell_size(const orc_im *h);
int orc_im_work(orc_im *h, int noutput_items, const uint8_t *in, float *out, int *consumed);
void orc_im_destroy(orc_im *h);

/* framemapperfint_cc (include/dvbt2ll/framemapperfint_cc.h:49) */
orc_fm *orc_fm_create(int framesize, int rate, int constellation, int rotation, int fecblocks,
                      int tiblocks, int carriermode, int fftsize, int guardinterval,
                      int l1constellation, int pilotpattern, int t2frames, int numdatasyms,
                      int paprmode, int version, int preamble, int inputmode,
                      int reservedbiasbits, int l1scrambled, int inband);
/* nplp data PLPs in one T2 frame (EN 302 755 6.5, 7.2.3.1, 8.3.6.3; the reference carries one Type-1 PLP
 * with TIME_IL_TYPE 0 in every frame, framemapper:152-250; PARITY UNPINNED beyond that frame): plp = nplp x
 * {framesize, rate, constellation, rotation, fecblocks, tiblocks, inputmode, inband, plp_type (1 | 2),
 * ti_type (TIME_IL_TYPE 0 | 1), ti_frames (P_I: 1 for type 0; type 1: one TI block, tiblocks = 1, of
 * fecblocks FEC blocks spread over P_I T2 frames), frame_interval (I_JUMP), first_frame_idx (< I_JUMP)};
 * num_subslices = SUB_SLICES_PER_FRAME of the Type-2 PLPs (1 without any); the other arguments are the
 * common fields. */
orc_fm *orc_fm_create_mplp(int nplp, const int *plp, int num_subslices, int carriermode, int fftsize,
                           int guardinterval, int l1constellation, int pilotpattern, int t2frames, int numdatasyms,
                           int paprmode, int version, int preamble, int reservedbiasbits, int l1scrambled);
int orc_fm_l1post_cells(const orc_fm *h);
/* data cells per T2 frame (every PLP) */
int orc_fm_stream_items(const orc_fm *h);
int orc_fm_mapped_items(const orc_fm *h);
/* cells PLP plp consumes at the next orc_fm_work: its whole interleaving frame (fecblocks x cell size) on
 * the first T2 frame of the interleaving frame, else 0 */
int orc_fm_consume(const orc_fm *h, int plp);
/* the state at absolute T2 frame `frame` (t2_frame_num = frame mod t2frames; every PLP at frame mod P_I of
 * its interleaving frame -- the next work call must start interleaving frames of the PLPs it consumes) */
void orc_fm_seek(orc_fm *h, long frame);
/* test hook: T2 frame `frame`'s L1-post signalling bits before the CRC-32, one per byte; returns the count */
int orc_fm_l1post_bits(orc_fm *h, long frame, uint8_t *out, int cap);
/* one T2 frame: the consumed cells of every PLP (PLP 0 first) in -> mapped_items cells out; returns
 * mapped_items */
int orc_fm_work(orc_fm *h, const float *in, float *out);
void orc_fm_destroy(orc_fm *h);

/* pilotgenp1insert_cc (include/dvbt2ll/pilotgenp1insert_cc.h:49) */
orc_pg *orc_pg_create(int carriermode, int fftsize, int pilotpattern, int guardinterval,
                      int numdatasyms, int paprmode, int version, int preamble, int misogroup,
                      int equalization, int bandwidth, int vlength);
int orc_pg_active_items(const orc_pg *h);
int orc_pg_output_items(const orc_pg *h);
int orc_pg_num_symbols(const orc_pg *h);
/* pre-IFFT carrier vectors (after the optional EQ multiply, before fftshift):
 * num_symbols * vlength complex (re,im) floats.  Bit-exact stage. */
int orc_pg_carriers(orc_pg *h, const float *in, float *carriers);
/* full output: P1 + symbols with GI.  The IFFT is the oracle's own float radix-2 FFT
 * (FFTW is not available); use it for timing, check IQ against a float64 IFFT. */
int orc_pg_work(orc_pg *h, const float *in, float *out);
/* the 2048 P1 samples (computed with a float64 DFT then rounded) */
void orc_pg_p1(const orc_pg *h, float *p1);
float orc_pg_normalization(const orc_pg *h);
int orc_pg_guard(const orc_pg *h);
void orc_pg_destroy(orc_pg *h);

/* Known-answer helpers exposed for the CPU tests */
uint8_t orc_crc8_dvbs2(const uint8_t *buf, int len);          /* table crc_tab (bbheader:222-240) */
uint32_t orc_crc32_bits(const uint8_t *bits, int nbits);      /* add_crc32_bits (framemapper:1205-1224) */
void orc_bb_prbs(uint8_t *bits, int n);                       /* init_bb_randomiser (bbheader:357-369) */

#ifdef __cplusplus
}
#endif
#endif
