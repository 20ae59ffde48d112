/*
 * dvbt2ll_hip.h -- C ABI of the MI355X-native DVB-T2 transmit chain.
 *
 * Drop-in boundary for the four gr-dvbt2ll blocks (plus the gr-dtv LDPC block the
 * shipped flowgraph places between bbheaderbch and interleavermod).  Each block is an
 * opaque handle that reproduces the reference gr::block contract:
 *
 *   make()            -> dvbt2ll_<blk>_create()      (reference include/dvbt2ll/<blk>.h:49)
 *   set_output_multiple -> dvbt2ll_<blk>_output_multiple()
 *   forecast()        -> dvbt2ll_<blk>_forecast()
 *   general_work()    -> dvbt2ll_<blk>_general_work() (+ consume_each via *consumed)
 *
 * Buffers passed to general_work are HOST buffers owned by the caller (GNU Radio
 * circular buffers); the call is synchronous and retains no pointer.  Handles own
 * their device memory and one HIP stream.  Instances are independent; one instance
 * must not be called from two threads at once (GNU Radio never does).
 *
 * The fused chain (dvbt2ll_chain_*) runs TS bytes -> IQ for whole T2 frames with
 * device-resident buffers; it is what bench.py measures.
 *
 * Enum arguments use the reference's numeric values (include/dvbt2ll/dvbt2ll_config.h:60-202).
 * Errors: the reference throws std::bad_alloc from constructors and silently accepts
 * invalid parameter combinations; this ABI returns negative status codes instead.
 */
#ifndef DVBT2LL_HIP_H
#define DVBT2LL_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DVBT2LL_OK 0
#define DVBT2LL_EINVAL (-1)   /* invalid parameter combination                       */
#define DVBT2LL_ENOMEM (-2)   /* device/host allocation failed (reference: bad_alloc) */
#define DVBT2LL_EDEVICE (-3)  /* HIP runtime / kernel launch error                     */
#define DVBT2LL_ESHORT (-4)   /* fewer input items than forecast() requires            */

const char *dvbt2ll_strerror(int status);
const char *dvbt2ll_version(void);
/* number of visible HIP devices (0 when no GPU) -- never initialises a context */
int dvbt2ll_device_count(void);

/* ---------------------------------------------------------------------------
 * bbheaderbch_bb: TS bytes -> BBFRAME + BCH, one unpacked bit per output byte.
 * Replaces gr::dvbt2ll::bbheaderbch_bb::make(framesize, rate, mode, inband, fecblocks,
 * tsrate) (include/dvbt2ll/bbheaderbch_bb.h:49; lib/bbheaderbch_bb_impl.cc:32-37).
 * ------------------------------------------------------------------------- */
typedef struct dvbt2ll_bbheaderbch dvbt2ll_bbheaderbch;
typedef struct {
  int framesize, rate, mode, inband, fecblocks, tsrate;
} dvbt2ll_bbheaderbch_params;
int dvbt2ll_bbheaderbch_create(const dvbt2ll_bbheaderbch_params *p, int device, dvbt2ll_bbheaderbch **out);
int dvbt2ll_bbheaderbch_output_multiple(const dvbt2ll_bbheaderbch *h);             /* nbch (impl.cc:195) */
int dvbt2ll_bbheaderbch_forecast(const dvbt2ll_bbheaderbch *h, int noutput_items, int *ninput_items_required);
int dvbt2ll_bbheaderbch_general_work(dvbt2ll_bbheaderbch *h, int noutput_items, int ninput_items,
                                     const void *in, void *out, int *consumed);
/* TS sync bytes != 0x47 consumed so far (the reference logs "Transport Stream sync error!" for each,
 * lib/bbheaderbch_bb_impl.cc:675-677, 703-705; the output is unaffected in both input modes) */
int64_t dvbt2ll_bbheaderbch_sync_errors(const dvbt2ll_bbheaderbch *h);
void dvbt2ll_bbheaderbch_destroy(dvbt2ll_bbheaderbch *h);

/* ---------------------------------------------------------------------------
 * ldpc_bb: nbch unpacked bits -> nldpc unpacked bits (natural parity order).
 * Replaces gr-dtv dvb_ldpc_bb(standard=DVBT2, framesize, rate, MOD_OTHER) as wired in
 * apps/vv009-4kshort.grc:386-460; arithmetic = lib/bbheaderbch_bb_impl.cc:533-646.
 * ------------------------------------------------------------------------- */
typedef struct dvbt2ll_ldpc dvbt2ll_ldpc;
typedef struct {
  int framesize, rate;
} dvbt2ll_ldpc_params;
int dvbt2ll_ldpc_create(const dvbt2ll_ldpc_params *p, int device, dvbt2ll_ldpc **out);
int dvbt2ll_ldpc_output_multiple(const dvbt2ll_ldpc *h);                           /* nldpc */
int dvbt2ll_ldpc_forecast(const dvbt2ll_ldpc *h, int noutput_items, int *ninput_items_required);
int dvbt2ll_ldpc_general_work(dvbt2ll_ldpc *h, int noutput_items, int ninput_items, const void *in,
                              void *out, int *consumed);
void dvbt2ll_ldpc_destroy(dvbt2ll_ldpc *h);

/* ---------------------------------------------------------------------------
 * interleavermod_bc: nldpc unpacked bits -> cell_size complex64 cells per FEC block.
 * Replaces gr::dvbt2ll::interleavermod_bc::make(framesize, rate, constellation, rotation)
 * (include/dvbt2ll/interleavermod_bc.h:49; lib/interleavermod_bc_impl.cc:32-37).
 * ------------------------------------------------------------------------- */
typedef struct dvbt2ll_interleavermod dvbt2ll_interleavermod;
typedef struct {
  int framesize, rate, constellation, rotation;
} dvbt2ll_interleavermod_params;
int dvbt2ll_interleavermod_create(const dvbt2ll_interleavermod_params *p, int device,
                                  dvbt2ll_interleavermod **out);
int dvbt2ll_interleavermod_output_multiple(const dvbt2ll_interleavermod *h);       /* cell_size (:254) */
int dvbt2ll_interleavermod_forecast(const dvbt2ll_interleavermod *h, int noutput_items, int *ninput_items_required);
int dvbt2ll_interleavermod_general_work(dvbt2ll_interleavermod *h, int noutput_items, int ninput_items,
                                        const void *in, void *out, int *consumed);
void dvbt2ll_interleavermod_destroy(dvbt2ll_interleavermod *h);

/* ---------------------------------------------------------------------------
 * framemapperfint_cc: one T2 frame of stream cells -> mapped (frequency-interleaved)
 * cells.  Replaces gr::dvbt2ll::framemapperfint_cc::make(...20 parameters...)
 * (include/dvbt2ll/framemapperfint_cc.h:49; lib/framemapperfint_cc_impl.cc:31-36).
 * ------------------------------------------------------------------------- */
typedef struct dvbt2ll_framemapperfint dvbt2ll_framemapperfint;
typedef struct {
  int framesize, rate, constellation, rotation, fecblocks, tiblocks, carriermode, fftsize,
      guardinterval, l1constellation, pilotpattern, t2frames, numdatasyms, paprmode, version,
      preamble, inputmode, reservedbiasbits, l1scrambled, inband;
} dvbt2ll_framemapperfint_params;
int dvbt2ll_framemapperfint_create(const dvbt2ll_framemapperfint_params *p, int device,
                                   dvbt2ll_framemapperfint **out);
int dvbt2ll_framemapperfint_output_multiple(const dvbt2ll_framemapperfint *h);     /* mapped_items */
int dvbt2ll_framemapperfint_stream_items(const dvbt2ll_framemapperfint *h);
int dvbt2ll_framemapperfint_forecast(const dvbt2ll_framemapperfint *h, int noutput_items, int *ninput_items_required);
int dvbt2ll_framemapperfint_general_work(dvbt2ll_framemapperfint *h, int noutput_items, int ninput_items,
                                         const void *in, void *out, int *consumed);
void dvbt2ll_framemapperfint_destroy(dvbt2ll_framemapperfint *h);

/* ---------------------------------------------------------------------------
 * pilotgenp1insert_cc: one T2 frame of mapped cells -> P1 + OFDM symbols with GI.
 * Replaces gr::dvbt2ll::pilotgenp1insert_cc::make(carriermode, fftsize, pilotpattern,
 * guardinterval, numdatasyms, paprmode, version, preamble, misogroup, equalization,
 * bandwidth, vlength) (include/dvbt2ll/pilotgenp1insert_cc.h:49; impl.cc:33-38).
 * ------------------------------------------------------------------------- */
typedef struct dvbt2ll_pilotgenp1insert dvbt2ll_pilotgenp1insert;
typedef struct {
  int carriermode, fftsize, pilotpattern, guardinterval, numdatasyms, paprmode, version, preamble,
      misogroup, equalization, bandwidth, vlength;
} dvbt2ll_pilotgenp1insert_params;
int dvbt2ll_pilotgenp1insert_create(const dvbt2ll_pilotgenp1insert_params *p, int device,
                                    dvbt2ll_pilotgenp1insert **out);
int dvbt2ll_pilotgenp1insert_output_multiple(const dvbt2ll_pilotgenp1insert *h);   /* Nsym*(N+GI)+2048 */
int dvbt2ll_pilotgenp1insert_active_items(const dvbt2ll_pilotgenp1insert *h);
int dvbt2ll_pilotgenp1insert_forecast(const dvbt2ll_pilotgenp1insert *h, int noutput_items, int *ninput_items_required);
int dvbt2ll_pilotgenp1insert_general_work(dvbt2ll_pilotgenp1insert *h, int noutput_items, int ninput_items,
                                          const void *in, void *out, int *consumed);
/* test hook: the frequency-domain symbols (after EQ, before fftshift/IFFT) of one frame,
 * num_symbols * vlength complex64 written to carriers (host). */
int dvbt2ll_pilotgenp1insert_debug_carriers(dvbt2ll_pilotgenp1insert *h, const void *in, void *carriers);
void dvbt2ll_pilotgenp1insert_destroy(dvbt2ll_pilotgenp1insert *h);

/* ---------------------------------------------------------------------------
 * Fused chain: TS bytes -> IQ for whole T2 frames (BB+BCH+LDPC -> bit interleave +
 * QAM + cell interleave -> frame/time/frequency interleave + pilots + IFFT + GI + P1).
 * Equivalent to the five blocks above connected in the shipped flowgraph, each frame
 * k encoded with the state the reference would hold at that point of the stream
 * (TS offset, SYNCD count, CRC-8 of the previous packet, t2_frame_num = k % t2frames).
 * ------------------------------------------------------------------------- */
typedef struct dvbt2ll_chain dvbt2ll_chain;
typedef struct {
  dvbt2ll_framemapperfint_params fm;   /* framesize ... inband */
  int misogroup, equalization, bandwidth;
  int max_frames;                      /* largest nframes per run call */
  int tsrate;                          /* bbheaderbch tsrate: the in-band type B TS rate field */
} dvbt2ll_chain_params;
typedef struct {
  int fec_blocks_per_frame;   /* F */
  int payload_bytes_per_block; /* TS bytes consumed per FEC block (NM) */
  int64_t ts_bytes_per_frame;
  int64_t iq_samples_per_frame;
  int cell_size, stream_items, mapped_items, num_symbols, fft_size, guard_interval;
  int64_t cw_stride_bytes;     /* packed codeword stride in the internal buffer */
  /* T2 frames from one interleaving frame of the PLP to the next: 1 for the reference's PLP, P_I x
   * FRAME_INTERVAL in general (dvbt2ll_plp_params); fec_blocks_per_frame and ts_bytes_per_frame then count
   * one interleaving frame; stream_items stays the cells per T2 frame carrying the PLP */
  int frames_per_if;
} dvbt2ll_chain_info;
int dvbt2ll_chain_create(const dvbt2ll_chain_params *p, int device, dvbt2ll_chain **out);
int dvbt2ll_chain_get_info(const dvbt2ll_chain *h, dvbt2ll_chain_info *info);
/* ts_dev: device pointer to TS bytes whose first byte is absolute stream offset ts_base
 * (a multiple of 188, else DVBT2LL_EINVAL; at least one packet before the first byte the frames consume so
 * the CRC-8 of the preceding packet can be formed); ts_len bytes valid.  iq_dev receives
 * nframes * iq_samples_per_frame samples (complex64, or int16 I/Q pairs after
 * dvbt2ll_chain_set_output(.., DVBT2LL_IQ_SC16)).  stream: hipStream_t (NULL = the handle's
 * own stream).  Asynchronous on that stream. */
int dvbt2ll_chain_run_device(dvbt2ll_chain *h, const void *ts_dev, int64_t ts_base, int64_t ts_len,
                             int64_t first_frame, int nframes, void *iq_dev, void *stream);
/* multi-stream batch (BASELINE cfg4 "4 independent PLP streams", cfg5 "8-stream batch"): nstreams
 * independent single-PLP T2 signals (the reference carries one PLP per instance,
 * lib/framemapperfint_cc_impl.cc:153, so each stream is its own five-block chain) encoded in one launch of
 * the three kernels.  Stream s's TS bytes are at ts_dev + s * ts_stride, every stream laid out as
 * run_device's ts_dev (the same ts_base and ts_len; ts_stride >= ts_len); all streams encode frames
 * [first_frame, first_frame + nframes).  IQ: stream s, frame first_frame + j at sample
 * (s * nframes + j) * iq_samples_per_frame of iq_dev.  nstreams * nframes <= max_frames.
 * run_device(...) == run_streams(h, ts, 0, 1, ...).  Asynchronous on stream. */
int dvbt2ll_chain_run_streams(dvbt2ll_chain *h, const void *ts_dev, int64_t ts_stride, int nstreams,
                              int64_t ts_base, int64_t ts_len, int64_t first_frame, int nframes,
                              void *iq_dev, void *stream);
/* intermediate buffer slots (packed codewords + cell index pairs, ~310 MB per slot for 64 cfg3
 * frames): run calls take the slots round-robin, so calls issued on different streams run
 * concurrently on the GPU (one call's kernels fill the CUs the other call's kernel tails leave
 * idle).  A slot reused on a different stream than its previous run first waits for that run
 * (hipStreamWaitEvent), so any call order is safe.  1 <= nslots <= DVBT2LL_CHAIN_MAX_SLOTS;
 * synchronises the device.  Default 1.  Not part of the reference (GNU Radio runs one
 * general_work per block at a time): the pipelined form of the same calls. */
#define DVBT2LL_CHAIN_MAX_SLOTS 4
int dvbt2ll_chain_set_slots(dvbt2ll_chain *h, int nslots);
/* hipGraph launch mode: run calls issue the chain's kernels as one instantiated hipGraph, captured
 * on first use for each (nframes, IQ format, buffer slot) into a ring of DVBT2LL_CHAIN_GRAPH_RING
 * instantiations; a call re-arms the next idle instantiation of the ring (its kernel nodes'
 * arguments, hipGraphExecKernelNodeSetParams) and launches it, so back-to-back calls on one slot do
 * not wait for each other on the host (the host only waits when every instantiation of the ring is
 * still in flight).  For small per-call batches (one T2 frame per call, as GNU Radio's scheduler
 * calls a block); output identical to the direct launches.  Per-stage timing events are skipped in
 * this mode.  Default off. */
#define DVBT2LL_CHAIN_GRAPH_RING 4
int dvbt2ll_chain_set_graph(dvbt2ll_chain *h, int enable);
/* host buffers, synchronous */
int dvbt2ll_chain_run_host(dvbt2ll_chain *h, const void *ts, int64_t ts_base, int64_t ts_len,
                           int64_t first_frame, int nframes, void *iq);
/* Streaming host path (the reference's output is host memory feeding a sink,
 * lib/pilotgenp1insert_cc_impl.cc:2785-2906 -> apps/vv009-4kshort.grc:801-1623).  A submission copies the
 * TS bytes its frames need from host ts (laid out as run_device's: absolute stream offset ts_base, ts_len
 * bytes) to the device, encodes the frames and copies their IQ (the current dvbt2ll_chain_set_output format)
 * to host iq, on three HIP streams of the handle ordered by events, into the next entry of a ring of
 * DVBT2LL_HOST_RING device buffer sets: submission k + 1's copy-in and k - 1's copy-out run beside k's
 * kernels.  Returns at once with a ticket (the host blocks only when the ring entry's previous submission
 * is still in flight); ts and iq must stay valid, and iq unread, until dvbt2ll_chain_host_wait(ticket)
 * returns.  Page-locked host buffers (dvbt2ll_host_alloc, or hipHostRegister) move at the PCIe rate;
 * pageable ones work, but the runtime stages their copies and the submit call waits for them.
 * Single-PLP chains; nframes <= max_frames; submissions complete in order. */
#define DVBT2LL_HOST_RING 3
int dvbt2ll_chain_host_submit(dvbt2ll_chain *h, const void *ts, int64_t ts_base, int64_t ts_len,
                              int64_t first_frame, int nframes, void *iq, int64_t *ticket);
int dvbt2ll_chain_host_wait(dvbt2ll_chain *h, int64_t ticket);
/* frames [first_frame, first_frame + nframes) through the ring in chunks of chunk_frames (0: max_frames),
 * frame f's IQ at iq + (f - first_frame) * iq_samples_per_frame samples; synchronous */
int dvbt2ll_chain_run_host_pipelined(dvbt2ll_chain *h, const void *ts, int64_t ts_base, int64_t ts_len,
                                     int64_t first_frame, int nframes, void *iq, int chunk_frames);
/* page-locked host memory for the streaming path (page-aligned heap memory, hipHostRegister'ed); NULL on
 * failure.  Free with dvbt2ll_host_free. */
void *dvbt2ll_host_alloc(size_t bytes);
void dvbt2ll_host_free(void *p);
/* IQ output of the chain (default: gain 1, DVBT2LL_IQ_CF32 = pilotgenp1insert_cc's own complex64
 * output).  gain multiplies every normalised sample, as the blocks_multiply_const_xx that follows
 * pilotgen in apps/vv009-4kshort.grc:335-385 (const 0.2) does.  DVBT2LL_IQ_SC16 stores each sample
 * as interleaved int16 I, Q = saturate(round-half-even(x * 32767)), the sc16 wire format of the
 * flowgraph's SDR sink (apps/vv009-4kshort.grc:802-1623): 4 bytes per sample instead of 8.
 * Applies to later run calls. */
#define DVBT2LL_IQ_CF32 0
#define DVBT2LL_IQ_SC16 1
int dvbt2ll_chain_set_output(dvbt2ll_chain *h, float gain, int format);
/* per-stage kernel timing with HIP events on the launch stream: enable, then read the
 * accumulated milliseconds and launch counts of stages {0: fec, 1: map, 2: ofdm, 3: reserved (0)};
 * nstages <= 4.  The frames' L1-post signalling is generated on the GPU every run by extra
 * workgroups of the map launch (counted in stage 1). */
int dvbt2ll_chain_set_timing(dvbt2ll_chain *h, int enable);
int dvbt2ll_chain_get_timing(dvbt2ll_chain *h, double *ms, int64_t *launches, int nstages);
/* test hooks (host outputs, synchronous), last run's frame 0: packed codewords (tempu
 * order; only when that run stored them, see dvbt2ll_chain_debug_keep_codewords, else
 * DVBT2LL_EINVAL); the frame data region in the slot order the OFDM kernel reads, as stored
 * (uint16 constellation index pairs: lo = the cell's index, hi = the index whose Q part
 * it carries, i.e. the previous cell's under rotation) and as complex64 cells */
int dvbt2ll_chain_debug_codewords(dvbt2ll_chain *h, void *out, int64_t bytes);
/* test hook: enable != 0 -> the following runs also store every FEC block's packed codeword in the
 * chain's codeword buffer (the LDPC + map kernel otherwise keeps it on chip) */
int dvbt2ll_chain_debug_keep_codewords(dvbt2ll_chain *h, int enable);
int dvbt2ll_chain_debug_cell_pairs(dvbt2ll_chain *h, void *out, int64_t cells);
int dvbt2ll_chain_debug_cells(dvbt2ll_chain *h, void *out, int64_t cells);
/* TS sync bytes != 0x47 consumed by all run calls so far (bbheaderbch_bb_impl.cc:675, 703);
 * synchronises the device */
int dvbt2ll_chain_sync_errors(dvbt2ll_chain *h, int64_t *count);
int dvbt2ll_chain_synchronize(dvbt2ll_chain *h);
void dvbt2ll_chain_destroy(dvbt2ll_chain *h);

/* ---------------------------------------------------------------------------
 * Multi-PLP frames (EN 302 755 8.3.6.3): nplp Type-1 data PLPs in one T2
 * frame, PLP_ID = index, each with its own TS stream, FEC, constellation, cell interleaver and time
 * interleaver (TIME_IL_TYPE 0, FRAME_INTERVAL 1, so T2 frames stay independent), its cells placed
 * back to back after the L1 signalling in PLP_ID order (PLP_START = the cells before it); the
 * L1-post carries the PLP loops.  The reference carries exactly one PLP
 * (lib/framemapperfint_cc_impl.cc:152-250: num_plp = 1; L1-post serialised at :1553-1691): nplp = 1
 * is its frame bit for bit, nplp > 1 is not pinned by it (PARITY UNPINNED).
 * The OFDM kernels hold one constellation table per distinct (constellation, rotation) pair of the
 * frame's PLPs (PLPs that agree share it): at most 2 x (4 + 16 + 64 + 256) = 680 entries, so every
 * combination of up to DVBT2LL_MAX_PLP PLPs fits the kernels' 1024-entry table area.
 * ------------------------------------------------------------------------- */
#define DVBT2LL_MAX_PLP 8
typedef struct {
  int framesize, rate, constellation, rotation, fecblocks, tiblocks, inputmode, inband, tsrate;
  /* EN 302 755 beyond the reference's PLP (which is plp_type 1, ti_type 0, ti_frames 1,
   * lib/framemapperfint_cc_impl.cc:159, 198-200; PARITY UNPINNED otherwise):
   *   plp_type  1: Type-1 data PLP, one run of cells at its PLP_START (0 is read as 1);
   *             2: Type-2 data PLP, cut into num_subslices sub-slices (8.3.6.3);
   *   ti_type   TIME_IL_TYPE (6.5): 0 = one interleaving frame of fecblocks FEC blocks in tiblocks TI
   *             blocks per T2 frame (the reference's); 1 = one TI block (tiblocks must be 1) of fecblocks
   *             FEC blocks per interleaving frame, spread over ti_frames = P_I consecutive T2 frames
   *             (TIME_IL_LENGTH = P_I, FRAME_INTERVAL 1): T2 frame i of interleaving frame m (frames
   *             m P_I + i) carries TI output cells [i D, (i + 1) D), D = fecblocks x cell size / P_I;
   *   ti_frames P_I (0 is read as 1; must be 1 for ti_type 0; fecblocks x cell size divisible by it);
   *   frame_interval  FRAME_INTERVAL = I_JUMP (7.2.3.1; 0 is read as 1): the PLP occurs only in the T2 frames f
   *             with f mod I_JUMP = first_frame_idx (FIRST_FRAME_IDX < I_JUMP), its interleaving frame spanning
   *             P_I of them; t2frames must be a multiple of P_I x I_JUMP.  A T2 frame carries only its PLPs
   *             (the others' L1-post PLP_START and PLP_NUM_BLOCKS are 0), dummy cells fill the rest.
   * fecblocks is then PLP_NUM_BLOCKS: the FEC blocks of one interleaving frame. */
  int plp_type, ti_type, ti_frames, frame_interval, first_frame_idx;
} dvbt2ll_plp_params;
typedef struct {
  /* the common (frame, L1, OFDM) fields of framemapperfint_cc::make */
  int carriermode, fftsize, guardinterval, l1constellation, pilotpattern, t2frames, numdatasyms, paprmode,
      version, preamble, reservedbiasbits, l1scrambled;
  int nplp;                                  /* 1 .. DVBT2LL_MAX_PLP */
  dvbt2ll_plp_params plp[DVBT2LL_MAX_PLP];   /* plp[k]: PLP_ID k */
  /* SUB_SLICES_PER_FRAME of the Type-2 PLPs (0 is read as 1; must be 1 without Type-2 PLPs): the frame's
   * data cells are the Type-1 PLPs back to back in PLP_ID order, then sub-slice 0 of every Type-2 PLP
   * (PLP_ID order), sub-slice 1 of every Type-2 PLP, ...; each Type-2 PLP's cells per T2 frame divisible
   * by it.  A chain whose PLPs have interleaving frames of several T2 frames or FRAME_INTERVAL > 1 runs whole
   * launch units: first_frame and nframes multiples of the least common multiple of the PLPs' P_I x I_JUMP
   * (dvbt2ll_chain_unit_frames). */
  int num_subslices;
} dvbt2ll_mplp_params;

/* one PLP of a multi-PLP frame: the BBHEADER of every later BBFRAME says MATYPE SIS/MIS = multiple
 * input streams and MATYPE-2 (ISI) = isi (the PLP_ID), the MIS branch of the reference's add_bbheader
 * (lib/bbheaderbch_bb_impl.cc:288-298) that its ctor never selects (:168) */
int dvbt2ll_bbheaderbch_set_isi(dvbt2ll_bbheaderbch *h, int isi);

/* framemapperfint_cc with one input port per PLP (the per-PLP bbheaderbch -> ldpc -> interleavermod
 * chains feed port k with PLP k's cells): one T2 frame per general_work call, consuming
 * stream_items(k) cells from every port (framemapper:1942-1946, 2147 per port); a TIME_IL_TYPE 1 PLP's port
 * instead delivers its whole interleaving frame (fecblocks x cell size cells) on the interleaving frame's
 * first T2 frame and nothing on the other P_I - 1 (forecast and consumed say so per port) */
typedef struct dvbt2ll_framemapper_mplp dvbt2ll_framemapper_mplp;
int dvbt2ll_framemapper_mplp_create(const dvbt2ll_mplp_params *p, int device, dvbt2ll_framemapper_mplp **out);
int dvbt2ll_framemapper_mplp_output_multiple(const dvbt2ll_framemapper_mplp *h);     /* mapped_items */
int dvbt2ll_framemapper_mplp_stream_items(const dvbt2ll_framemapper_mplp *h, int plp);
/* nin_required[k] for each of the nplp ports */
int dvbt2ll_framemapper_mplp_forecast(const dvbt2ll_framemapper_mplp *h, int noutput_items, int *ninput_items_required);
/* in[k], ninput_items[k]: port k's cells (host complex64); consumed[k] per port */
int dvbt2ll_framemapper_mplp_general_work(dvbt2ll_framemapper_mplp *h, int noutput_items, const int *ninput_items,
                                          const void *const *in, void *out, int *consumed);
void dvbt2ll_framemapper_mplp_destroy(dvbt2ll_framemapper_mplp *h);

/* fused chain of a multi-PLP frame: every PLP's TS -> BBFRAME/BCH/LDPC -> map, one frame's OFDM */
typedef struct {
  dvbt2ll_mplp_params fm;
  int misogroup, equalization, bandwidth;
  int max_frames;
} dvbt2ll_mplp_chain_params;
int dvbt2ll_chain_create_mplp(const dvbt2ll_mplp_chain_params *p, int device, dvbt2ll_chain **out);
int dvbt2ll_chain_num_plps(const dvbt2ll_chain *h);
/* T2 frames of the chain's launch unit: the least common multiple of its PLPs' P_I x FRAME_INTERVAL
 * (1 for the reference's PLPs).  Every run's first_frame and nframes are multiples of it (else
 * DVBT2LL_EINVAL); create fails when max_frames is smaller. */
int dvbt2ll_chain_unit_frames(const dvbt2ll_chain *h);
/* PLP plp's FEC blocks, payload and TS bytes per frame, cell size, cells per frame (stream_items) and
 * codeword stride; the frame-wide fields as dvbt2ll_chain_get_info (which reports PLP 0's) */
int dvbt2ll_chain_get_plp_info(const dvbt2ll_chain *h, int plp, dvbt2ll_chain_info *info);
/* ts_dev[k], ts_base[k], ts_len[k]: PLP k's TS, laid out as run_device's (host arrays of nplp entries);
 * frames [first_frame, first_frame + nframes) into iq_dev.  Asynchronous on stream.  run_device on a
 * one-PLP chain == run_plps with one entry. */
int dvbt2ll_chain_run_plps(dvbt2ll_chain *h, const void *const *ts_dev, const int64_t *ts_base,
                           const int64_t *ts_len, int64_t first_frame, int nframes, void *iq_dev, void *stream);
/* run_plps with host buffers (each PLP's TS copied to the device, IQ copied back), synchronous */
int dvbt2ll_chain_run_plps_host(dvbt2ll_chain *h, const void *const *ts, const int64_t *ts_base, const int64_t *ts_len,
                                int64_t first_frame, int nframes, void *iq);
/* test hook: PLP plp's packed codewords of the last run's frame 0 (as dvbt2ll_chain_debug_codewords) */
int dvbt2ll_chain_debug_plp_codewords(dvbt2ll_chain *h, int plp, void *out, int64_t bytes);

/* ---------------------------------------------------------------------------
 * ABI version.  The parameter and info structs are passed by pointer with no size field, so a caller
 * compiled against another layout would be read or written past its struct.  Version history:
 *   1  rounds 1-4: dvbt2ll_plp_params = the first nine ints, no num_subslices, no frames_per_if;
 *   2  round 5: dvbt2ll_plp_params + plp_type .. first_frame_idx (which moves every field of
 *      dvbt2ll_mplp_params / dvbt2ll_mplp_chain_params after plp[0]), dvbt2ll_mplp_params.num_subslices,
 *      dvbt2ll_chain_info.frames_per_if.
 * dvbt2ll_abi_check(DVBT2LL_ABI_VERSION, sizeof ...) (or the DVBT2LL_ABI_CHECK() macro) returns DVBT2LL_OK when the
 * caller's header is this library's, DVBT2LL_EINVAL otherwise; the adapters and the Python mirror call it
 * before their first create.
 * ------------------------------------------------------------------------- */
#define DVBT2LL_ABI_VERSION 2
int dvbt2ll_abi_version(void);
int dvbt2ll_abi_check(int abi_version, size_t sizeof_chain_params, size_t sizeof_chain_info,
                      size_t sizeof_plp_params, size_t sizeof_mplp_params, size_t sizeof_mplp_chain_params);
#define DVBT2LL_ABI_CHECK()                                                                                      \
  dvbt2ll_abi_check(DVBT2LL_ABI_VERSION, sizeof(dvbt2ll_chain_params), sizeof(dvbt2ll_chain_info),               \
                    sizeof(dvbt2ll_plp_params), sizeof(dvbt2ll_mplp_params), sizeof(dvbt2ll_mplp_chain_params))

#ifdef __cplusplus
}
#endif
#endif /* DVBT2LL_HIP_H */
