/*
 * dvbt2_oracle.c -- TEST INFRASTRUCTURE ONLY (see dvbt2_oracle.h).
 *
 * A plain-C, bit-serial restatement of the gr-dvbt2ll reference transmit blocks.
 * It deliberately keeps the reference's one-bit-per-byte data flow and loop order
 * so a reader can check it line by line against /root/reference/lib/<block>_impl.cc; the
 * product (gr-dvbt2ll_amd/csrc) uses entirely different (bit-packed, gather-map,
 * batched) formulations.  Standard constant tables come from the generated
 * data header (tools/extract_tables.py).  Parity status: UNPINNED (see header).
 */
#include "dvbt2_oracle.h"
#include "../gr-dvbt2ll_amd/csrc/gen/dvbt2_std_tables.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* enum values, include/dvbt2ll/dvbt2ll_config.h:60-202 */
enum { C1_2 = 0, C3_5, C2_3, C3_4, C4_5, C5_6, C1_3, C2_5 };
enum { MOD_QPSK = 0, MOD_16QAM, MOD_64QAM, MOD_256QAM };
enum { FECFRAME_SHORT = 0, FECFRAME_NORMAL };
enum { INPUTMODE_NORMAL = 0, INPUTMODE_HIEFF };
enum { CARRIERS_NORMAL = 0, CARRIERS_EXTENDED };
enum { PREAMBLE_T2_SISO = 0, PREAMBLE_T2_MISO, PREAMBLE_NON_T2, PREAMBLE_T2_LITE_SISO, PREAMBLE_T2_LITE_MISO };
enum { FFTSIZE_2K = 0, FFTSIZE_8K, FFTSIZE_4K, FFTSIZE_1K, FFTSIZE_16K, FFTSIZE_32K, FFTSIZE_8K_T2GI,
       FFTSIZE_32K_T2GI, FFTSIZE_16K_T2GI = 11 };
enum { GI_1_32 = 0, GI_1_16, GI_1_8, GI_1_4, GI_1_128, GI_19_128, GI_19_256 };
enum { PAPR_OFF = 0, PAPR_ACE, PAPR_TR, PAPR_BOTH };
enum { L1_MOD_BPSK = 0, L1_MOD_QPSK, L1_MOD_16QAM, L1_MOD_64QAM };
enum { PILOT_PP1 = 0, PILOT_PP2, PILOT_PP3, PILOT_PP4, PILOT_PP5, PILOT_PP6, PILOT_PP7, PILOT_PP8 };
enum { VERSION_111 = 0, VERSION_121, VERSION_131 };
enum { MISO_TX1 = 0, MISO_TX2 };

#define FRAME_SIZE_NORMAL 64800
#define FRAME_SIZE_SHORT 16200

typedef struct { float re, im; } cf;

static int fft_points(int fftsize) {
  switch (fftsize) {
    case FFTSIZE_1K: return 1024;
    case FFTSIZE_2K: return 2048;
    case FFTSIZE_4K: return 4096;
    case FFTSIZE_8K: case FFTSIZE_8K_T2GI: return 8192;
    case FFTSIZE_16K: case FFTSIZE_16K_T2GI: return 16384;
    case FFTSIZE_32K: case FFTSIZE_32K_T2GI: return 32768;
  }
  return 0;
}

/* ------------------------------------------------------------------------- */
/* Shared FEC parameter table: bbheaderbch ctor lib/bbheaderbch_bb_impl.cc:51-165 */
typedef struct { int kbch, nbch, q, nparity; } fec_par;

static int fec_params(int framesize, int rate, fec_par *p) {
  static const int nk[6][4] = { /* kbch, nbch, q, parity */
    {32208, 32400, 90, 192}, {38688, 38880, 72, 192}, {43040, 43200, 60, 160},
    {48408, 48600, 45, 192}, {51648, 51840, 36, 192}, {53840, 54000, 30, 160}};
  static const int sk[8][3] = {
    {7032, 7200, 25}, {9552, 9720, 18}, {10632, 10800, 15}, {11712, 11880, 12},
    {12432, 12600, 10}, {13152, 13320, 8}, {5232, 5400, 30}, {6312, 6480, 27}};
  if (framesize == FECFRAME_NORMAL) {
    if (rate < 0 || rate > C5_6) return -1;
    p->kbch = nk[rate][0]; p->nbch = nk[rate][1]; p->q = nk[rate][2]; p->nparity = nk[rate][3];
  } else {
    if (rate < 0 || rate > C2_5) return -1;
    p->kbch = sk[rate][0]; p->nbch = sk[rate][1]; p->q = sk[rate][2]; p->nparity = 168;
  }
  return 0;
}

/* ------------------------------------------------------------------------- */
/* GF(2) polynomial product, poly_mult (bbheader:375-396) */
static int poly_mult(const int *a, int la, const int *b, int lb, int *out) {
  memset(out, 0, sizeof(int) * (la + lb));
  for (int i = 0; i < la; i++)
    for (int j = 0; j < lb; j++)
      if (a[i] * b[j] > 0) out[i + j]++;
  int max = 0;
  for (int i = 0; i < la + lb; i++) { out[i] &= 1; if (out[i]) max = i; }
  return max + 1;
}

/* 192-bit register as 3 x uint64, bit i = coefficient of x^i */
typedef struct { uint64_t w[3]; } r192;
static int r_bit(const r192 *r, int i) { return (int)((r->w[i >> 6] >> (i & 63)) & 1); }
static void r_set(r192 *r, int i) { r->w[i >> 6] |= 1ull << (i & 63); }
static void r_shl(r192 *r, int s) { /* s in 1..63 */
  r->w[2] = (r->w[2] << s) | (r->w[1] >> (64 - s));
  r->w[1] = (r->w[1] << s) | (r->w[0] >> (64 - s));
  r->w[0] <<= s;
}
static void r_mask(r192 *r, int nbits) {
  for (int k = 0; k < 3; k++) {
    int lo = 64 * k;
    if (nbits <= lo) r->w[k] = 0;
    else if (nbits < lo + 64) r->w[k] &= (1ull << (nbits - lo)) - 1;
  }
}

/* Generator g(x) (low P coefficients) of the BCH code: bch_poly_build_tables (bbheader:424-502) */
static void bch_generator(int normal, int nparity, r192 *g) {
  int po[2][200], len;
  int a[17];
  memset(g, 0, sizeof(*g));
  if (normal) {
    int np = nparity / 16;  /* 8, 10 or 12 minimal polynomials */
    for (int i = 0; i < 17; i++) a[i] = T2_BCH_MINPOLY_NORMAL[0][i];
    int b[17];
    for (int i = 0; i < 17; i++) b[i] = T2_BCH_MINPOLY_NORMAL[1][i];
    len = poly_mult(a, 17, b, 17, po[0]);
    int cur = 0;
    for (int k = 2; k < np; k++) {
      for (int i = 0; i < 17; i++) a[i] = T2_BCH_MINPOLY_NORMAL[k][i];
      len = poly_mult(a, 17, po[cur], len, po[cur ^ 1]);
      cur ^= 1;
    }
    for (int i = 0; i < nparity; i++) if (po[cur][i]) r_set(g, i);
  } else {
    int b[15];
    for (int i = 0; i < 15; i++) { a[i] = T2_BCH_MINPOLY_SHORT[0][i]; b[i] = T2_BCH_MINPOLY_SHORT[1][i]; }
    len = poly_mult(a, 15, b, 15, po[0]);
    int cur = 0;
    for (int k = 2; k < 12; k++) {
      for (int i = 0; i < 15; i++) a[i] = T2_BCH_MINPOLY_SHORT[k][i];
      len = poly_mult(a, 15, po[cur], len, po[cur ^ 1]);
      cur ^= 1;
    }
    for (int i = 0; i < 168; i++) if (po[cur][i]) r_set(g, i);
  }
  (void)len;
}

/* calculate_crc_table (bbheader:399-417): remainder of (byte << (P-8)) after 8 shifts */
static void bch_table(const r192 *g, int P, r192 *tab) {
  for (int d = 0; d < 256; d++) {
    r192 v = {{0, 0, 0}};
    for (int b = 0; b < 8; b++) if (d & (1 << b)) r_set(&v, P - 8 + b);
    for (int s = 0; s < 8; s++) {
      int top = r_bit(&v, P - 1);
      r_shl(&v, 1);
      if (top) { v.w[0] ^= g->w[0]; v.w[1] ^= g->w[1]; v.w[2] ^= g->w[2]; }
      r_mask(&v, P);
    }
    tab[d] = v;
  }
}

/* bch_calculate (bbheader:504-531): parity of k message bits (unpacked), appended MSB first */
static void bch_encode(const r192 *tab, int P, uint8_t *bits, int k) {
  r192 reg = {{0, 0, 0}};
  for (int j = 0; j < k / 8; j++) {
    int b = 0;
    for (int e = 0; e < 8; e++) b |= (bits[8 * j + e] & 1) << (7 - e);
    int top = 0;
    for (int e = 0; e < 8; e++) top |= r_bit(&reg, P - 8 + e) << e;
    int pos = (top ^ b) & 0xff;
    r_shl(&reg, 8);
    r_mask(&reg, P);
    reg.w[0] ^= tab[pos].w[0]; reg.w[1] ^= tab[pos].w[1]; reg.w[2] ^= tab[pos].w[2];
  }
  for (int n = 0; n < P; n++) bits[k + n] = (uint8_t)r_bit(&reg, P - 1 - n);
}

/* ------------------------------------------------------------------------- */
/* LDPC (IRA) encoder: ldpc_lookup_generate + ldpc_calculate (bbheader:533-646); the same
 * accumulate is used for the L1 codes (framemapper:1314-1364, 1498-1507, 1777-1786). */
static const t2_ldpc_code_t *ldpc_code(int normal, int rate) {
  for (int i = 0; i < T2_LDPC_NCODES; i++)
    if (T2_LDPC_CODES[i].framesize_normal == normal && T2_LDPC_CODES[i].rate == rate) return &T2_LDPC_CODES[i];
  return NULL;
}

static void ldpc_encode(const t2_ldpc_code_t *c, int nbch, int nldpc, uint8_t *cw) {
  int pbits = nldpc - nbch;
  uint8_t *p = cw + nbch;
  memset(p, 0, (size_t)pbits);
  int im = 0;
  int off = c->addr_off;
  for (int row = 0; row < c->nrows; row++) {
    int cnt = T2_LDPC_ROWLEN[c->row_off + row];
    for (int n = 0; n < 360; n++) {
      uint8_t d = cw[im];
      for (int col = 0; col < cnt; col++) {
        int x = T2_LDPC_ADDR[off + col];
        p[(x + n * c->q) % pbits] ^= d;
      }
      im++;
    }
    off += cnt;
  }
  for (int j = 1; j < pbits; j++) p[j] ^= p[j - 1];
}

/* ========================================================================= */
/* bbheaderbch_bb                                                            */
/* ========================================================================= */
struct orc_bb {
  int kbch, nbch, P, mode, inband, fec_blocks, fec_block, ts_rate;
  int sis_mis, isi;                  /* MATYPE-1 SIS/MIS bit, MATYPE-2 (bbheader:168, 281, 288-298) */
  unsigned count;
  uint8_t crc;
  int extra;
  uint8_t crc_tab[256];
  uint8_t bb_randomise[FRAME_SIZE_NORMAL];
  r192 tab[256];
};

/* build_crc8_table (bbheader:222-240), CRC_POLYR 0xD5 MSB first */
static void crc8_table(uint8_t *t) {
  for (int i = 0; i < 256; i++) {
    int r = i, crc = 0;
    for (int j = 7; j >= 0; j--) {
      if (((r >> j) & 1) ^ ((crc & 0x80) ? 1 : 0)) crc = (crc << 1) ^ 0xD5;
      else crc <<= 1;
    }
    t[i] = (uint8_t)crc;
  }
}

uint8_t orc_crc8_dvbs2(const uint8_t *buf, int len) {
  uint8_t t[256];
  crc8_table(t);
  uint8_t crc = 0;
  for (int i = 0; i < len; i++) crc = t[buf[i] ^ crc];
  return crc;
}

/* init_bb_randomiser (bbheader:357-369): PRBS 1+x^14+x^15, init 0x4A80 */
void orc_bb_prbs(uint8_t *bits, int n) {
  int sr = 0x4A80;
  for (int i = 0; i < n; i++) {
    int b = ((sr) ^ (sr >> 1)) & 1;
    bits[i] = (uint8_t)b;
    sr >>= 1;
    if (b) sr |= 0x4000;
  }
}

orc_bb *orc_bb_create(int framesize, int rate, int mode, int inband, int fecblocks, int tsrate) {
  fec_par fp;
  if (fec_params(framesize, rate, &fp)) return NULL;
  orc_bb *h = (orc_bb *)calloc(1, sizeof(orc_bb));
  h->kbch = fp.kbch; h->nbch = fp.nbch; h->P = fp.nparity;
  h->mode = mode; h->inband = inband; h->fec_blocks = fecblocks > 0 ? fecblocks : 1;
  h->ts_rate = tsrate;
  h->count = 0; h->crc = 0; h->fec_block = 0;
  h->sis_mis = 1; h->isi = 0;                      /* SIS_MIS_SINGLE (bbheader:168) */
  h->extra = (((h->kbch - 80) / 8) / 187) + 1;    /* bbheader:194 */
  crc8_table(h->crc_tab);
  orc_bb_prbs(h->bb_randomise, FRAME_SIZE_NORMAL);
  r192 g;
  bch_generator(framesize == FECFRAME_NORMAL, h->P, &g);
  bch_table(&g, h->P, h->tab);
  return h;
}
/* multiple input streams (one PLP of a multi-PLP frame): SIS/MIS = SIS_MIS_MULTIPLE, ISI = the PLP_ID.
 * The reference's ctor always sets SIS (bbheader:168); its add_bbheader already carries the MIS
 * branch (:288-298), which this enables.  Parity unpinned (the reference never takes the branch). */
void orc_bb_set_isi(orc_bb *h, int isi) { h->sis_mis = 0; h->isi = isi & 0xFF; }
int orc_bb_nbch(const orc_bb *h) { return h->nbch; }
int orc_bb_kbch(const orc_bb *h) { return h->kbch; }
void orc_bb_destroy(orc_bb *h) { free(h); }

/* forecast (bbheader:207-216) */
int orc_bb_forecast(const orc_bb *h, int nout) {
  int n = (nout - 80 - (h->nbch - h->kbch)) / 8;
  return h->mode == INPUTMODE_NORMAL ? n : n + h->extra;
}

/* add_crc8_bits (bbheader:247-270): CRC_POLY 0xAB, LSB-first register, 72 bits */
static void add_crc8_bits(uint8_t *in, int length, int hieff) {
  int crc = 0, i = 0;
  for (int n = 0; n < length; n++) {
    int b = in[i++] ^ (crc & 1);
    crc >>= 1;
    if (b) crc ^= 0xAB;
  }
  if (hieff) crc ^= 0x80;
  for (int n = 0; n < 8; n++) in[i++] = (crc & (1 << n)) ? 1 : 0;
}

static void put_bits(uint8_t *dst, int *off, unsigned v, int nbits) {
  for (int n = nbits - 1; n >= 0; n--) dst[(*off)++] = (v >> n) & 1;
}

/* add_bbheader (bbheader:272-325): TS, SIS (or MIS with ISI, :288-298), CCM, ISSYI=0, NPD=0, RO=0 */
static void add_bbheader(const orc_bb *h, uint8_t *f, unsigned count, int padding) {
  int o = 0;
  f[o++] = 1; f[o++] = 1;          /* TS_GS = 3 */
  f[o++] = (uint8_t)h->sis_mis;    /* SIS_MIS_SINGLE 1 / SIS_MIS_MULTIPLE 0 */
  f[o++] = 1;                      /* CCM */
  f[o++] = 0; f[o++] = 0;          /* ISSYI, NPD */
  f[o++] = 0; f[o++] = 0;          /* RO */
  put_bits(f, &o, h->sis_mis ? 0u : (unsigned)h->isi, 8);   /* MATYPE-2 (ISI) */
  put_bits(f, &o, h->mode == INPUTMODE_NORMAL ? 188 * 8 : 0, 16);    /* UPL */
  put_bits(f, &o, (unsigned)(h->kbch - 80 - padding), 16);           /* DFL */
  put_bits(f, &o, h->mode == INPUTMODE_NORMAL ? 0x47 : 0, 8);        /* SYNC */
  put_bits(f, &o, count == 0 ? 0 : (188 - count) * 8, 16);           /* SYNCD */
  add_crc8_bits(f, 72, h->mode == INPUTMODE_HIEFF);
}

/* add_inband_type_b (bbheader:327-355) */
static void add_inband_type_b(uint8_t *f, int ts_rate) {
  int o = 0;
  f[o++] = 0; f[o++] = 1;
  put_bits(f, &o, 0, 31); put_bits(f, &o, 0, 22); put_bits(f, &o, 0, 2); put_bits(f, &o, 0, 10);
  put_bits(f, &o, (unsigned)ts_rate, 27);
  put_bits(f, &o, 0, 10);
}

/* general_work (bbheader:648-742) */
int orc_bb_work(orc_bb *h, int nout, const uint8_t *in, uint8_t *out, int *consumed_out) {
  int consumed = 0;
  for (int i = 0; i < nout; i += h->nbch) {
    int padding = (h->fec_block == 0 && h->inband) ? 104 : 0;
    add_bbheader(h, out, h->count, padding);
    int off = 80;
    int npay = (h->kbch - 80 - padding) / 8;
    if (h->mode == INPUTMODE_HIEFF) {
      for (int j = 0; j < npay; j++) {
        if (h->count == 0) { j--; in++; }   /* sync byte dropped (warning if != 0x47) */
        else { uint8_t b = *in++; for (int n = 7; n >= 0; n--) out[off++] = (b >> n) & 1; }
        h->count = (h->count + 1) % 188;
        consumed++;
      }
    } else {
      for (int j = 0; j < npay; j++) {
        uint8_t b;
        if (h->count == 0) { in++; b = h->crc; h->crc = 0; }
        else { b = *in++; h->crc = h->crc_tab[b ^ h->crc]; }
        h->count = (h->count + 1) % 188;
        consumed++;
        for (int n = 7; n >= 0; n--) out[off++] = (b >> n) & 1;
      }
    }
    if (padding) { add_inband_type_b(out + off, h->ts_rate); off += 104; }
    for (int j = 0; j < h->kbch; j++) out[j] ^= h->bb_randomise[j];
    bch_encode(h->tab, h->P, out, h->kbch);
    if (h->inband) h->fec_block = (h->fec_block + 1) % h->fec_blocks;
    out += h->nbch;
  }
  if (consumed_out) *consumed_out = consumed;
  return nout;
}

/* ========================================================================= */
/* LDPC                                                                      */
/* ========================================================================= */
/* The block restates ldpc_calculate in its gather form (bbheader:625-646): per parity bit the XOR of the info
 * bits listed for it (the reference's ldpc_lut, built by ldpc_lookup_generate :533-598 from the same address
 * tables), then the accumulate.  The lists are built once per handle from the scatter form of ldpc_encode, so
 * both forms give the same bits (the L1 codes keep ldpc_encode).  The gather form also prices the CPU baseline
 * like the reference: one pass over the edge lists per block, no modulo per edge. */
struct orc_ldpc { const t2_ldpc_code_t *c; int nbch, nldpc; int *lut_off, *lut; };

orc_ldpc *orc_ldpc_create(int framesize, int rate) {
  fec_par fp;
  if (fec_params(framesize, rate, &fp)) return NULL;
  orc_ldpc *h = (orc_ldpc *)calloc(1, sizeof(orc_ldpc));
  if (!h) return NULL;
  h->c = ldpc_code(framesize == FECFRAME_NORMAL, rate);
  h->nbch = fp.nbch;
  h->nldpc = framesize == FECFRAME_NORMAL ? FRAME_SIZE_NORMAL : FRAME_SIZE_SHORT;
  const t2_ldpc_code_t *c = h->c;
  const int pbits = h->nldpc - h->nbch;
  h->lut_off = (int *)calloc((size_t)pbits + 1, sizeof(int));
  if (!h->lut_off) { free(h); return NULL; }
  /* two passes over the scatter form: count each parity bit's edges, then fill them in info-bit order */
  for (int pass = 0; pass < 2; pass++) {
    int *fill = NULL;
    if (pass == 1) {
      for (int i = 0; i < pbits; i++) h->lut_off[i + 1] += h->lut_off[i];
      h->lut = (int *)malloc(sizeof(int) * (size_t)(h->lut_off[pbits] ? h->lut_off[pbits] : 1));
      fill = (int *)malloc(sizeof(int) * (size_t)pbits);
      if (!h->lut || !fill) { free(fill); orc_ldpc_destroy(h); return NULL; }
      memcpy(fill, h->lut_off, sizeof(int) * (size_t)pbits);
    }
    int im = 0, off = c->addr_off;
    for (int row = 0; row < c->nrows; row++) {
      const int cnt = T2_LDPC_ROWLEN[c->row_off + row];
      for (int n = 0; n < 360; n++, im++)
        for (int col = 0; col < cnt; col++) {
          const int x = (T2_LDPC_ADDR[off + col] + n * c->q) % pbits;
          if (pass == 0) h->lut_off[x + 1]++;
          else h->lut[fill[x]++] = im;
        }
      off += cnt;
    }
    free(fill);
  }
  return h;
}
int orc_ldpc_work(orc_ldpc *h, int nblocks, const uint8_t *in, uint8_t *out) {
  const int pbits = h->nldpc - h->nbch;
  for (int b = 0; b < nblocks; b++) {
    uint8_t *cw = out + (size_t)b * h->nldpc;
    memcpy(cw, in + (size_t)b * h->nbch, (size_t)h->nbch);
    uint8_t *p = cw + h->nbch;
    for (int i = 0; i < pbits; i++) {
      uint8_t v = 0;
      for (int e = h->lut_off[i]; e < h->lut_off[i + 1]; e++) v ^= cw[h->lut[e]];
      p[i] = v;
    }
    for (int j = 1; j < pbits; j++) p[j] ^= p[j - 1];
  }
  return nblocks * h->nldpc;
}
void orc_ldpc_destroy(orc_ldpc *h) {
  if (!h) return;
  free(h->lut_off);
  free(h->lut);
  free(h);
}

/* ========================================================================= */
/* interleavermod_bc                                                          */
/* ========================================================================= */
struct orc_im {
  int frame_size, nbch, q, cell_size, mod, rate, constellation, rotation;
  cf lut[256];
  const uint8_t *twist, *mux;
  uint8_t tempu[FRAME_SIZE_NORMAL], tempv[FRAME_SIZE_NORMAL];
};

/* complex<float> *= complex<float> (libstdc++, no FMA contraction), interleavermod:180-183 */
static cf cmul_f(cf a, cf b) {
  volatile float ac = a.re * b.re, bd = a.im * b.im, ad = a.re * b.im, bc = a.im * b.re;
  cf r; r.re = ac - bd; r.im = ad + bc; return r;
}

/* Gray QAM tables + rotation, interleavermod ctor :169-253 */
static void build_qam(int constellation, int rotation, cf *lut, int *mod_out) {
  static const double l16[4] = {3.0, 1.0, -3.0, -1.0};
  static const double l64[8] = {7.0, 5.0, 1.0, 3.0, -7.0, -5.0, -1.0, -3.0};
  static const double l256[16] = {15.0, 13.0, 9.0, 11.0, 1.0, 3.0, 7.0, 5.0,
                                  -15.0, -13.0, -9.0, -11.0, -1.0, -3.0, -7.0, -5.0};
  double angle = 0.0, norm;
  int n = 0, mod = 2;
  switch (constellation) {
    case MOD_16QAM:
      mod = 4; n = 16; norm = sqrt(10.0); angle = 16.8;
      for (int i = 0; i < 16; i++) {
        int ri = ((i & 0x8) >> 2) | ((i & 0x2) >> 1), ii = ((i & 0x4) >> 1) | (i & 0x1);
        lut[i].re = (float)(l16[ri] / norm); lut[i].im = (float)(l16[ii] / norm);
      }
      break;
    case MOD_64QAM:
      mod = 6; n = 64; norm = sqrt(42.0); angle = 8.6;
      for (int i = 0; i < 64; i++) {
        int ri = ((i & 0x20) >> 3) | ((i & 0x8) >> 2) | ((i & 0x2) >> 1);
        int ii = ((i & 0x10) >> 2) | ((i & 0x4) >> 1) | (i & 0x1);
        lut[i].re = (float)(l64[ri] / norm); lut[i].im = (float)(l64[ii] / norm);
      }
      break;
    case MOD_256QAM:
      mod = 8; n = 256; norm = sqrt(170.0); angle = 3.576334375;
      for (int i = 0; i < 256; i++) {
        int ri = ((i & 0x80) >> 4) | ((i & 0x20) >> 3) | ((i & 0x8) >> 2) | ((i & 0x2) >> 1);
        int ii = ((i & 0x40) >> 3) | ((i & 0x10) >> 2) | ((i & 0x4) >> 1) | (i & 0x1);
        lut[i].re = (float)(l256[ri] / norm); lut[i].im = (float)(l256[ii] / norm);
      }
      break;
    default:
      mod = 2; n = 4; norm = sqrt(2.0); angle = 29.0;
      lut[0].re = (float)(1.0 / norm); lut[0].im = (float)(1.0 / norm);
      lut[1].re = (float)(1.0 / norm); lut[1].im = (float)(-1.0 / norm);
      lut[2].re = (float)(-1.0 / norm); lut[2].im = (float)(1.0 / norm);
      lut[3].re = (float)(-1.0 / norm); lut[3].im = (float)(-1.0 / norm);
      break;
  }
  if (rotation) {
    double a = (2.0 * M_PI * angle) / 360.0;
    cf t; t.re = (float)cos(a); t.im = (float)sin(a);
    for (int i = 0; i < n; i++) lut[i] = cmul_f(lut[i], t);
  }
  *mod_out = mod;
}

orc_im *orc_im_create(int framesize, int rate, int constellation, int rotation) {
  fec_par fp;
  if (fec_params(framesize, rate, &fp)) return NULL;
  orc_im *h = (orc_im *)calloc(1, sizeof(orc_im));
  int normal = framesize == FECFRAME_NORMAL;
  h->frame_size = normal ? FRAME_SIZE_NORMAL : FRAME_SIZE_SHORT;
  h->nbch = fp.nbch; h->q = fp.q; h->rate = rate;
  h->constellation = constellation; h->rotation = rotation;
  static const int cs_n[4] = {32400, 16200, 10800, 8100}, cs_s[4] = {8100, 4050, 2700, 2025};
  h->cell_size = normal ? cs_n[constellation] : cs_s[constellation];
  build_qam(constellation, rotation, h->lut, &h->mod);
  /* twist / mux selection, interleavermod:333-350, 422-439, 519-528, 617-625 */
  switch (constellation) {
    case MOD_16QAM:
      h->twist = normal ? T2_BI_TWIST16N : T2_BI_TWIST16S;
      if (rate == C3_5 && normal) h->mux = T2_BI_MUX16_35;
      else if (rate == C1_3 && !normal) h->mux = T2_BI_MUX16_13;
      else if (rate == C2_5 && !normal) h->mux = T2_BI_MUX16_25;
      else h->mux = T2_BI_MUX16;
      break;
    case MOD_64QAM:
      h->twist = normal ? T2_BI_TWIST64N : T2_BI_TWIST64S;
      if (rate == C3_5 && normal) h->mux = T2_BI_MUX64_35;
      else if (rate == C1_3 && !normal) h->mux = T2_BI_MUX64_13;
      else if (rate == C2_5 && !normal) h->mux = T2_BI_MUX64_25;
      else h->mux = T2_BI_MUX64;
      break;
    case MOD_256QAM:
      if (normal) {
        h->twist = T2_BI_TWIST256N;
        h->mux = rate == C3_5 ? T2_BI_MUX256_35 : rate == C2_3 ? T2_BI_MUX256_23 : T2_BI_MUX256;
      } else {
        h->twist = T2_BI_TWIST256S;
        h->mux = rate == C1_3 ? T2_BI_MUX256S_13 : rate == C2_5 ? T2_BI_MUX256S_25 : T2_BI_MUX256S;
      }
      break;
    default: break;
  }
  return h;
}
int orc_im_cell_size(const orc_im *h) { return h->cell_size; }
void orc_im_destroy(orc_im *h) { free(h); }

/* parity interleave, e.g. interleavermod:549-557 */
static void parity_interleave(orc_im *h, const uint8_t *in) {
  memcpy(h->tempu, in, (size_t)h->nbch);
  for (int t = 0; t < h->q; t++)
    for (int s = 0; s < 360; s++)
      h->tempu[h->nbch + 360 * t + s] = in[h->nbch + h->q * s + t];
}

/* one FEC block of general_work (interleavermod:270-704), one block per call semantics */
static void im_block(orc_im *h, const uint8_t *in, cf *out) {
  int cs = h->cell_size, fs = h->frame_size, mod = h->mod;
  uint8_t *tv = h->tempv;
  if (h->constellation == MOD_QPSK) {                    /* :288-331 */
    const uint8_t *src = in;
    if (h->rate == C1_3 || h->rate == C2_5) { parity_interleave(h, in); src = h->tempu; }
    for (int j = 0; j < fs / 2; j++) tv[j] = (uint8_t)((src[2 * j] << 1) | src[2 * j + 1]);
  } else {
    int w = (h->constellation == MOD_256QAM && fs == FRAME_SIZE_SHORT) ? mod : 2 * mod;
    int rows = fs / w;
    parity_interleave(h, in);
    int idx = 0;                                           /* column-twist write :558-568 */
    for (int col = 0; col < w; col++) {
      int off = h->twist[col];
      for (int r = 0; r < rows; r++) {
        tv[off + rows * col] = h->tempu[idx++];
        if (++off == rows) off = 0;
      }
    }
    idx = 0;                                               /* row read :569-587 */
    for (int j = 0; j < rows; j++)
      for (int col = 0; col < w; col++) h->tempu[idx++] = tv[rows * col + j];
    idx = 0;                                               /* demux + pack :588-598 */
    int produced = 0;
    for (int d = 0; d < rows; d++) {
      unsigned pack = 0;
      for (int e = 0; e < w; e++) pack |= (unsigned)h->tempu[idx++] << ((w - 1) - h->mux[e]);
      if (w == 2 * mod) { tv[produced++] = (uint8_t)(pack >> mod); tv[produced++] = (uint8_t)(pack & ((1u << mod) - 1)); }
      else tv[produced++] = (uint8_t)(pack & 0xff);
    }
  }
  unsigned mask = (1u << mod) - 1;
  for (int j = 0; j < cs; j++) {                           /* map + Q delay :599-613 */
    if (!h->rotation) out[j] = h->lut[tv[j] & mask];
    else {
      out[j].re = h->lut[tv[j] & mask].re;
      out[j].im = h->lut[tv[(j + cs - 1) % cs] & mask].im;
    }
  }
}

int orc_im_work(orc_im *h, int nout, const uint8_t *in, float *out, int *consumed) {
  int nb = nout / h->cell_size;
  for (int b = 0; b < nb; b++)
    im_block(h, in + (size_t)b * h->frame_size, (cf *)out + (size_t)b * h->cell_size);
  if (consumed) *consumed = nb * h->frame_size;
  return nb * h->cell_size;
}

/* ========================================================================= */
/* framemapperfint_cc                                                         */
/* ========================================================================= */
#define KBCH_1_4 3072
#define NBCH_1_4 3240
#define KBCH_1_2 7032
#define NBCH_1_2 7200
#define KSIG_PRE 200
#define KSIG_POST 350
#define NBCH_PARITY 168

/* One data PLP of the frame.  The reference carries exactly one (framemapper:152-250:
 * num_plp = 1, plp_type = 1, time_il_type = 0, frame_interval = 1); this restatement generalises its
 * per-PLP state to nplp PLPs of EN 302 755 (PARITY UNPINNED beyond the reference's frame):
 *  - PLP p has PLP_ID p, its own FEC / constellation / cell interleaver / time interleaver;
 *  - 6.5 time interleaving, TIME_IL_TYPE 0 (the reference's): one interleaving frame (fec_blocks FEC
 *    blocks in ti_blocks TI blocks) per T2 frame; TIME_IL_TYPE 1: one TI block of fec_blocks FEC blocks
 *    per interleaving frame, spread over P_I = ti_frames consecutive T2 frames, T2 frame i of the
 *    interleaving frame carrying the TI output cells [i D, (i + 1) D), D = fec_blocks cell_size / P_I
 *    FRAME_INTERVAL I_JUMP (7.2.3.1): the PLP occurs in the T2 frames f with f mod I_JUMP = FIRST_FRAME_IDX
 *    only (the superframe holds whole I_JUMP P_I cycles), an interleaving frame spanning P_I of those;
 *  - 8.3.6.3 mapping: Type-1 PLPs first, back to back in PLP_ID order, each one run of D cells at its
 *    PLP_START; then the Type-2 PLPs, each cut into N_subslices sub-slices of D / N_subslices cells,
 *    sub-slice j of every Type-2 PLP (PLP_ID order) before sub-slice j + 1 of any
 *    (SUB_SLICE_INTERVAL = the Type-2 cells per T2 frame / N_subslices, TYPE_2_START = the Type-1 cells), over
 *    the PLPs present in the T2 frame; an absent PLP signals PLP_START = PLP_NUM_BLOCKS = 0. */
#define ORC_MAX_PLP 16
#define ORC_PLP_INTS 13
typedef struct {
  int cell_size, stream_items, start, pn_degree;   /* stream_items: cells per T2 frame (D) */
  int ti_blocks, fec_blocks, small_fec, big_fec, n_big, n_small;
  int plp_cod, plp_mod, rotation, fec_type, inband_b, plp_mode;
  int plp_type, ti_type, ti_frames, if_items, phase;   /* if_items = fec_blocks cell_size */
  int frame_interval, first_frame, present;            /* I_JUMP, FIRST_FRAME_IDX; in the current T2 frame */
  int ss, ss_off;                                      /* Type 2: sub-slice cells, offset in a sub-slice group */
  int *permutations;
  cf *time_interleave, *ti_out;                        /* CI output, TI output of the interleaving frame */
} orc_plp;

struct orc_fm {
  int nplp, ksig_post;               /* ksig_post: L1-post signalling bits incl. CRC (KSIG_POST = 350 for one PLP) */
  orc_plp plp[ORC_MAX_PLP];
  int nss, ssi, t2start, ntype2;     /* SUB_SLICES_PER_FRAME, SUB_SLICE_INTERVAL, TYPE_2_START, Type-2 PLPs */
  long frame;                        /* absolute T2 frame of the next work call */
  int stream_items, mapped_items, l1_constellation, eta_mod, t2_frames, t2_frame_num;
  int l1_scrambled, N_P2, C_P2, N_FC, C_FC, C_DATA, N_post, N_punc, num_data_symbols;
  /* L1 fields that are not constant (framemapper ctor :114-250) */
  int pre_fields[32];
  int post_reserved1, post_reserved2, post_reserved3, post_reserved4, post_reserved5;
  r192 bch_short_tab[256];
  cf l1pre_cache[1840];
  cf m_bpsk[2], m_qpsk[4], m_16qam[16], m_64qam[64];
  uint8_t l1_randomize[KBCH_1_2];
  int *Heven, *Hodd, *HevenP2, *HoddP2, *HevenFC, *HoddFC;
  cf *cell_out, *frame_out, *zigzag, *dummy;
};

/* add_crc32_bits (framemapper:1205-1224) */
uint32_t orc_crc32_bits(const uint8_t *bits, int nbits) {
  uint32_t crc = 0xffffffffu;
  for (int n = 0; n < nbits; n++) {
    int b = bits[n] ^ ((crc >> 31) & 1);
    crc <<= 1;
    if (b) crc ^= 0x04C11DB7u;
  }
  return crc;
}

/* shortened/punctured L1 code pieces (framemapper:1366-1910) */
static void l1_bch_ldpc(orc_fm *h, uint8_t *buf, int k, int nbch, const t2_ldpc_code_t *code) {
  bch_encode(h->bch_short_tab, 168, buf, k);
  ldpc_encode(code, nbch, FRAME_SIZE_SHORT, buf);
}

/* add_l1pre (framemapper:1366-1534) */
static void add_l1pre(orc_fm *h, cf *out) {
  uint8_t b[FRAME_SIZE_SHORT];
  int o = 0;
  const int *f = h->pre_fields;
  put_bits(b, &o, (unsigned)f[0], 8);   /* TYPE */
  b[o++] = (uint8_t)f[1];               /* BWT_EXT */
  put_bits(b, &o, (unsigned)f[2], 3);   /* S1 */
  put_bits(b, &o, (unsigned)f[3], 3);   /* S2 */
  b[o++] = 0;
  b[o++] = 0;                           /* L1_REPETITION_FLAG */
  put_bits(b, &o, (unsigned)f[4], 3);   /* GUARD_INTERVAL */
  put_bits(b, &o, (unsigned)f[5], 4);   /* PAPR */
  put_bits(b, &o, (unsigned)f[6], 4);   /* L1_MOD */
  put_bits(b, &o, 0, 2);                /* L1_COD */
  put_bits(b, &o, 0, 2);                /* L1_FEC_TYPE */
  put_bits(b, &o, (unsigned)f[7], 18);  /* L1_POST_SIZE */
  put_bits(b, &o, (unsigned)(h->ksig_post - 32), 18);  /* L1_POST_INFO_SIZE (KSIG_POST - 32, :125) */
  put_bits(b, &o, (unsigned)f[8], 4);   /* PILOT_PATTERN */
  put_bits(b, &o, 0, 8);                /* TX_ID_AVAILABILITY */
  put_bits(b, &o, 0, 16);               /* CELL_ID */
  put_bits(b, &o, 0x3085, 16);          /* NETWORK_ID */
  put_bits(b, &o, 0x8001, 16);          /* T2_SYSTEM_ID */
  put_bits(b, &o, (unsigned)f[9], 8);   /* NUM_T2_FRAMES */
  put_bits(b, &o, (unsigned)f[10], 12); /* NUM_DATA_SYMBOLS */
  put_bits(b, &o, 0, 3);                /* REGEN_FLAG */
  b[o++] = 0;                           /* L1_POST_EXTENSION */
  put_bits(b, &o, 1, 3);                /* NUM_RF */
  put_bits(b, &o, 0, 3);                /* CURRENT_RF_IDX */
  put_bits(b, &o, (unsigned)f[11], 4);  /* T2_VERSION */
  b[o++] = (uint8_t)f[12];              /* L1_POST_SCRAMBLED */
  b[o++] = 0;                           /* T2_BASE_LITE */
  put_bits(b, &o, (unsigned)f[13], 4);  /* RESERVED */
  uint32_t crc = orc_crc32_bits(b, o);
  put_bits(b, &o, crc, 32);
  while (o < KBCH_1_4) b[o++] = 0;
  l1_bch_ldpc(h, b, KBCH_1_4, NBCH_1_4, ldpc_code(0, 100));
  for (int c = 0; c < 31; c++) {
    int g = T2_L1_PRE_PUNCTURE[c];
    for (int c2 = 0; c2 < 360; c2++) b[c2 * 36 + g + NBCH_1_4] = 0x55;
  }
  int g = T2_L1_PRE_PUNCTURE[31];
  for (int c2 = 0; c2 < 328; c2++) b[c2 * 36 + g + NBCH_1_4] = 0x55;
  int idx = 0;
  for (int w = 0; w < KSIG_PRE; w++) out[idx++] = h->m_bpsk[b[w]];
  for (int w = 0; w < NBCH_PARITY; w++) out[idx++] = h->m_bpsk[b[w + KBCH_1_4]];
  for (int w = 0; w < FRAME_SIZE_SHORT - NBCH_1_4; w++)
    if (b[w + NBCH_1_4] != 0x55) out[idx++] = h->m_bpsk[b[w + NBCH_1_4]];
}

/* add_l1post (framemapper:1536-1910); the PLP loops of the configurable (:1577-1639) and dynamic
 * (:1672-1687) parts run over the frame's PLPs */
/* the L1-post signalling bits before the CRC-32 (:1546-1691) into info; returns their count */
static int l1post_info(const orc_fm *h, uint8_t *info, int t2_frame_num) {
  int o = 0;
  put_bits(info, &o, (unsigned)h->nss, 15);  /* SUB_SLICES_PER_FRAME (1 without Type-2 PLPs) */
  put_bits(info, &o, (unsigned)h->nplp, 8);  /* NUM_PLP */
  put_bits(info, &o, 0, 4);                  /* NUM_AUX */
  put_bits(info, &o, 0, 8);                  /* AUX_CONFIG_RFU */
  put_bits(info, &o, 0, 3);                  /* RF_IDX */
  put_bits(info, &o, 729833333u, 32);        /* FREQUENCY */
  for (int p = 0; p < h->nplp; p++) {
    const orc_plp *q = &h->plp[p];
    put_bits(info, &o, (unsigned)p, 8);      /* PLP_ID */
    put_bits(info, &o, (unsigned)q->plp_type, 3);   /* PLP_TYPE: data type 1 (001) or 2 (010) */
    put_bits(info, &o, 3, 5);                /* PLP_PAYLOAD_TYPE: TS */
    info[o++] = 0;                           /* FF_FLAG */
    put_bits(info, &o, 0, 3);                /* FIRST_RF_IDX */
    put_bits(info, &o, (unsigned)q->first_frame, 8);   /* FIRST_FRAME_IDX */
    put_bits(info, &o, 1, 8);                /* PLP_GROUP_ID */
    put_bits(info, &o, (unsigned)q->plp_cod, 3);
    put_bits(info, &o, (unsigned)q->plp_mod, 3);
    info[o++] = (uint8_t)q->rotation;
    put_bits(info, &o, (unsigned)q->fec_type, 2);
    put_bits(info, &o, (unsigned)q->fec_blocks, 10);   /* PLP_NUM_BLOCKS_MAX */
    put_bits(info, &o, (unsigned)q->frame_interval, 8);   /* FRAME_INTERVAL (I_JUMP) */
    /* TIME_IL_LENGTH: N_TI (type 0) or P_I (type 1), EN 302 755 7.2.3.1 */
    put_bits(info, &o, (unsigned)(q->ti_type ? q->ti_frames : q->ti_blocks), 8);
    info[o++] = (uint8_t)q->ti_type;         /* TIME_IL_TYPE */
    info[o++] = 0;                           /* IN_BAND_A_FLAG */
    info[o++] = (uint8_t)q->inband_b;
    put_bits(info, &o, (unsigned)h->post_reserved1, 11);
    put_bits(info, &o, (unsigned)q->plp_mode, 2);
    info[o++] = 0;                           /* STATIC_FLAG */
    info[o++] = 0;                           /* STATIC_PADDING_FLAG */
  }
  put_bits(info, &o, 0, 2);                  /* FEF_LENGTH_MSB */
  put_bits(info, &o, (unsigned)h->post_reserved2, 30);
  put_bits(info, &o, (unsigned)t2_frame_num, 8);         /* FRAME_IDX */
  put_bits(info, &o, (unsigned)h->ssi, 22);      /* SUB_SLICE_INTERVAL (0 without Type-2 PLPs) */
  put_bits(info, &o, (unsigned)h->t2start, 22);  /* TYPE_2_START (0 without Type-2 PLPs) */
  put_bits(info, &o, 0, 8);                  /* L1_CHANGE_COUNTER */
  put_bits(info, &o, 0, 3);                  /* START_RF_IDX */
  put_bits(info, &o, (unsigned)h->post_reserved3, 8);
  for (int p = 0; p < h->nplp; p++) {
    /* PLP_ID (dynamic): the reference's plp_id_dynamic is never set, i.e. 0 for its one PLP */
    put_bits(info, &o, (unsigned)p, 8);
    const int in = h->plp[p].present;
    put_bits(info, &o, in ? (unsigned)h->plp[p].start : 0u, 22);        /* PLP_START (cell address after L1) */
    put_bits(info, &o, in ? (unsigned)h->plp[p].fec_blocks : 0u, 10);   /* PLP_NUM_BLOCKS (of the interleaving frame) */
    put_bits(info, &o, (unsigned)h->post_reserved4, 8);
  }
  put_bits(info, &o, (unsigned)h->post_reserved5, 8);
  return o;
}

static void add_l1post(orc_fm *h, cf *out, int t2_frame_num) {
  uint8_t info[FRAME_SIZE_SHORT], t[FRAME_SIZE_SHORT], map[KBCH_1_2];
  int o = l1post_info(h, info, t2_frame_num);
  uint32_t crc = orc_crc32_bits(info, o);
  put_bits(info, &o, crc, 32);
  if (h->l1_scrambled) for (int n = 0; n < o; n++) info[n] ^= h->l1_randomize[n];
  const uint8_t *pad = h->l1_constellation == L1_MOD_16QAM ? T2_L1_POST_PADDING_16QAM
                     : h->l1_constellation == L1_MOD_64QAM ? T2_L1_POST_PADDING_64QAM
                     : T2_L1_POST_PADDING_BQPSK;
  memset(map, 0, sizeof(map));
  int m, last;
  if (o <= 360) { m = 20 - 1; last = 360 - o; }
  else { m = (KBCH_1_2 - o) / 360; last = KBCH_1_2 - o - 360 * m; }
  for (int n = 0; n < m; n++) {
    int idx = pad[n] * 360, len = pad[n] == 19 ? 192 : 360;
    for (int w = 0; w < len; w++) map[idx++] = 7;
  }
  int idx = pad[m] * 360 + (pad[m] == 19 ? 192 : 360) - last;
  for (int w = 0; w < last; w++) map[idx++] = 7;
  idx = 0;
  for (int n = 0; n < KBCH_1_2; n++) t[n] = map[n] != 7 ? info[idx++] : 0;
  l1_bch_ldpc(h, t, KBCH_1_2, NBCH_1_2, ldpc_code(0, 101));
  const uint8_t *punc = h->l1_constellation == L1_MOD_16QAM ? T2_L1_POST_PUNCTURE_16QAM
                      : h->l1_constellation == L1_MOD_64QAM ? T2_L1_POST_PUNCTURE_64QAM
                      : T2_L1_POST_PUNCTURE_BQPSK;
  for (int c = 0; c < h->N_punc / 360; c++) {
    int g = punc[c];
    for (int c2 = 0; c2 < 360; c2++) t[c2 * 25 + g + NBCH_1_2] = 0x55;
  }
  {
    int g = punc[h->N_punc / 360];
    for (int c2 = 0; c2 < h->N_punc - (h->N_punc / 360) * 360; c2++) t[c2 * 25 + g + NBCH_1_2] = 0x55;
  }
  uint8_t il[FRAME_SIZE_SHORT];
  idx = 0;
  for (int w = 0; w < KBCH_1_2; w++) if (map[w] != 7) il[idx++] = t[w];
  for (int w = 0; w < NBCH_PARITY; w++) il[idx++] = t[w + KBCH_1_2];
  for (int w = 0; w < FRAME_SIZE_SHORT - NBCH_1_2; w++) if (t[w + NBCH_1_2] != 0x55) il[idx++] = t[w + NBCH_1_2];
  if (h->l1_constellation == L1_MOD_16QAM || h->l1_constellation == L1_MOD_64QAM) {
    int ncols = h->l1_constellation == L1_MOD_16QAM ? 8 : 12, rows = h->N_post / ncols;
    for (int k = 0; k < rows; k++)
      for (int w = 0; w < ncols; w++) t[k * ncols + w] = il[rows * w + k];
  }
  int produced = 0;
  switch (h->l1_constellation) {
    case L1_MOD_BPSK:
      for (int d = 0; d < h->N_post; d++) out[produced++] = h->m_bpsk[il[d]];
      break;
    case L1_MOD_QPSK:
      for (int d = 0; d < h->N_post / 2; d++) out[produced++] = h->m_qpsk[(il[2 * d] << 1) | il[2 * d + 1]];
      break;
    case L1_MOD_16QAM:
      for (int d = 0, index = 0; d < h->N_post / 8; d++, index += 8) {
        int pack = 0;
        for (int e = 0; e < 8; e++) pack = (pack << 1) | t[index + T2_L1_MUX16[e]];
        out[produced++] = h->m_16qam[pack >> 4];
        out[produced++] = h->m_16qam[pack & 0xf];
      }
      break;
    case L1_MOD_64QAM:
      for (int d = 0, index = 0; d < h->N_post / 12; d++, index += 12) {
        int pack = 0;
        for (int e = 0; e < 12; e++) pack = (pack << 1) | t[index + T2_L1_MUX64[e]];
        out[produced++] = h->m_64qam[pack >> 6];
        out[produced++] = h->m_64qam[pack & 0x3f];
      }
      break;
  }
}

static int cell_counts(int fft, int ext, int pp, int *c_data, int *n_fc, int *c_fc) {
  for (int i = 0; i < T2_NCELL_COUNTS; i++) {
    const t2_cell_counts_t *c = &T2_CELL_COUNTS[i];
    if (c->fft == fft && c->ext == ext && c->pp == pp + 1) {
      *c_data = c->c_data; *n_fc = c->n_fc; *c_fc = c->c_fc; return 0;
    }
  }
  *c_data = *n_fc = *c_fc = 0;
  return -1;
}

/* N_P2 / C_P2 (framemapper:290-356, pilotgen:56-119) */
static void p2_counts(int fft, int siso, int *n_p2, int *c_p2) {
  switch (fft) {
    case 1024: *n_p2 = 16; *c_p2 = siso ? 558 : 546; break;
    case 2048: *n_p2 = 8; *c_p2 = siso ? 1118 : 1098; break;
    case 4096: *n_p2 = 4; *c_p2 = siso ? 2236 : 2198; break;
    case 8192: *n_p2 = 2; *c_p2 = siso ? 4472 : 4398; break;
    case 16384: *n_p2 = 1; *c_p2 = siso ? 8944 : 8814; break;
    case 32768: *n_p2 = 1; *c_p2 = siso ? 22432 : 17612; break;
    default: *n_p2 = 1; *c_p2 = 0;
  }
}

/* C_DATA/N_FC/C_FC with PAPR-TR reduction and SISO exceptions (framemapper:425-915) */
static void active_counts(int fft, int carriermode, int pp, int papr, int gi, int siso,
                          int *c_data, int *n_fc, int *c_fc) {
  cell_counts(fft, fft >= 8192 ? carriermode : 0, pp, c_data, n_fc, c_fc);
  if (papr == PAPR_TR || papr == PAPR_BOTH) {
    int red = fft / 1024 * 9;   /* 10, 18, 36, 72, 144, 288 */
    if (fft == 1024) red = 10;
    if (*c_data) *c_data -= red;
    if (*n_fc) *n_fc -= red;
    if (*c_fc) *c_fc -= red;
  }
  if (siso) {
    if ((gi == GI_1_128 && pp == PILOT_PP7) || (gi == GI_1_32 && pp == PILOT_PP4) ||
        (gi == GI_1_16 && pp == PILOT_PP2) || (gi == GI_19_256 && pp == PILOT_PP2)) {
      *n_fc = 0; *c_fc = 0;
    }
  }
}

/* 8.3.6.3 placement over the PLPs present in T2 frame `frame`: Type-1 runs back to back in PLP_ID order, then
 * the Type-2 sub-slices; returns the frame's data cells */
static int frame_layout(orc_fm *h, long frame) {
  int cells = 0;
  for (int p = 0; p < h->nplp; p++) {
    orc_plp *d = &h->plp[p];
    d->present = frame % d->frame_interval == d->first_frame;
    d->start = 0;
  }
  for (int p = 0; p < h->nplp; p++)
    if (h->plp[p].present && h->plp[p].plp_type == 1) {
      h->plp[p].start = cells;                   /* PLP_START: the cells before it */
      cells += h->plp[p].stream_items;
    }
  int any2 = 0, off = 0;
  for (int p = 0; p < h->nplp; p++) any2 |= h->plp[p].present && h->plp[p].plp_type == 2;
  h->t2start = any2 ? cells : 0;
  for (int p = 0; p < h->nplp; p++) {
    orc_plp *d = &h->plp[p];
    if (!d->present || d->plp_type != 2) continue;
    d->ss_off = off;
    d->start = cells + off;                      /* PLP_START: its first sub-slice */
    off += d->ss;
  }
  h->ssi = off;                                  /* SUB_SLICE_INTERVAL (0 without Type-2 PLPs) */
  return cells + off * h->nss;
}

/* framemapperfint ctor (framemapper:41-1190) for nplp data PLPs; plp: nplp x ORC_PLP_INTS ints per PLP
 * {framesize, rate, constellation, rotation, fecblocks, tiblocks, inputmode, inband, plp_type (1, 2),
 * ti_type (0, 1), ti_frames (P_I), frame_interval (I_JUMP), first_frame_idx}; num_subslices:
 * SUB_SLICES_PER_FRAME (1 without Type-2 PLPs) */
orc_fm *orc_fm_create_mplp(int nplp, const int *plp, int num_subslices, int carriermode, int fftsize,
                           int guardinterval, int l1constellation, int pilotpattern, int t2frames, int numdatasyms,
                           int paprmode, int version, int preamble, int reservedbiasbits, int l1scrambled) {
  int fft = fft_points(fftsize);
  if (!fft || t2frames < 1 || nplp < 1 || nplp > ORC_MAX_PLP || num_subslices < 1) return NULL;
  orc_fm *h = (orc_fm *)calloc(1, sizeof(orc_fm));
  int siso = preamble == PREAMBLE_T2_SISO || preamble == PREAMBLE_T2_LITE_SISO;
  int v131 = version == VERSION_131, resv = reservedbiasbits && v131;
  static const int cs_n[4] = {32400, 16200, 10800, 8100}, cs_s[4] = {8100, 4050, 2700, 2025};
  h->nplp = nplp;
  /* KSIG_POST = 350 bits for one PLP (framemapperfint_cc_impl.h:32); each further PLP adds its 89
   * configurable (:1577-1639) and 48 dynamic (:1672-1687) bits */
  h->ksig_post = KSIG_POST + (nplp - 1) * (89 + 48);
  h->nss = num_subslices;
  for (int p = 0; p < nplp; p++) {
    const int *q = plp + ORC_PLP_INTS * p;
    orc_plp *d = &h->plp[p];
    if (q[4] < 1 || q[2] < 0 || q[2] > 3) { orc_fm_destroy(h); return NULL; }
    d->cell_size = q[0] == FECFRAME_NORMAL ? cs_n[q[2]] : cs_s[q[2]];
    d->fec_blocks = q[4];
    d->ti_blocks = q[5];
    d->plp_type = q[8];
    d->ti_type = q[9];
    d->ti_frames = q[10];
    d->frame_interval = q[11];
    d->first_frame = q[12];
    if (d->frame_interval < 1 || d->first_frame < 0 || d->first_frame >= d->frame_interval ||
        t2frames % (d->frame_interval * d->ti_frames)) { orc_fm_destroy(h); return NULL; }
    /* type 1 interleaving: one TI block spread over P_I >= 1 frames; type 0: P_I = 1 */
    if ((d->plp_type != 1 && d->plp_type != 2) || (d->ti_type != 0 && d->ti_type != 1) || d->ti_frames < 1 ||
        (d->ti_type == 0 && d->ti_frames != 1) || (d->ti_type == 1 && d->ti_blocks != 1) ||
        ((long)d->fec_blocks * d->cell_size) % d->ti_frames) { orc_fm_destroy(h); return NULL; }
    if (d->plp_type == 2) h->ntype2++;
    /* L1-post fields of the PLP (framemapper:165-221) */
    d->plp_cod = q[1];                         /* C1_2..C5_6 -> 0..5, C1_3 -> 6, C2_5 -> 7 (:165-193) */
    d->plp_mod = q[2];
    d->rotation = q[3];
    d->fec_type = q[0];
    d->inband_b = (q[7] && v131) ? 1 : 0;
    d->plp_mode = version == VERSION_111 ? 0 : q[6] + 1;
  }
  /* L1-pre fields (framemapper:114-150) */
  h->pre_fields[0] = 0;                        /* STREAMTYPE_TS */
  h->pre_fields[1] = carriermode;
  h->pre_fields[2] = preamble;
  h->pre_fields[3] = fftsize & 0x7;
  h->pre_fields[4] = guardinterval;
  h->pre_fields[5] = paprmode;
  h->pre_fields[6] = l1constellation;
  h->pre_fields[8] = pilotpattern;
  h->pre_fields[9] = t2frames;
  h->pre_fields[10] = numdatasyms;
  h->pre_fields[11] = version;
  h->pre_fields[12] = v131 ? l1scrambled : 0;
  h->pre_fields[13] = resv ? 0xf : 0;
  /* L1-post reserved fields (framemapper:208-250) */
  h->post_reserved1 = resv ? 0x7ff : 0;
  h->post_reserved2 = resv ? 0x3fffffff : 0;
  h->post_reserved3 = resv ? 0xff : 0;
  h->post_reserved4 = resv ? 0xff : 0;
  h->post_reserved5 = resv ? 0xff : 0;
  r192 g;
  bch_generator(0, 168, &g);
  bch_table(&g, 168, h->bch_short_tab);
  h->m_bpsk[0].re = 1.0f; h->m_bpsk[1].re = -1.0f;
  int mod_unused;
  h->l1_constellation = l1constellation;
  switch (l1constellation) {                     /* framemapper:259-289 */
    case L1_MOD_BPSK: h->eta_mod = 1; break;
    case L1_MOD_QPSK: build_qam(MOD_QPSK, 0, h->m_qpsk, &mod_unused); h->eta_mod = 2; break;
    case L1_MOD_16QAM: build_qam(MOD_16QAM, 0, h->m_16qam, &mod_unused); h->eta_mod = 4; break;
    default: build_qam(MOD_64QAM, 0, h->m_64qam, &mod_unused); h->eta_mod = 6; break;
  }
  p2_counts(fft, siso, &h->N_P2, &h->C_P2);
  active_counts(fft, carriermode, pilotpattern, paprmode, guardinterval, siso, &h->C_DATA, &h->N_FC, &h->C_FC);

  /* frequency interleaver address tables (framemapper:357-424, 916-977) */
  int max_states, pn_degree, pn_mask, xor_size;
  const int *logic;
  const uint8_t *bpe, *bpo;
  static const int l1k[2] = {0, 4}, l2k[2] = {0, 3}, l4k[2] = {0, 2}, l8k[4] = {0, 1, 4, 6},
                   l16k[6] = {0, 1, 4, 5, 9, 11}, l32k[4] = {0, 1, 2, 12};
  switch (fft) {
    case 1024: pn_degree = 9; logic = l1k; xor_size = 2; bpe = T2_FI_BITPERM1KEVEN; bpo = T2_FI_BITPERM1KODD; break;
    case 2048: pn_degree = 10; logic = l2k; xor_size = 2; bpe = T2_FI_BITPERM2KEVEN; bpo = T2_FI_BITPERM2KODD; break;
    case 4096: pn_degree = 11; logic = l4k; xor_size = 2; bpe = T2_FI_BITPERM4KEVEN; bpo = T2_FI_BITPERM4KODD; break;
    case 8192: pn_degree = 12; logic = l8k; xor_size = 4; bpe = T2_FI_BITPERM8KEVEN; bpo = T2_FI_BITPERM8KODD; break;
    case 16384: pn_degree = 13; logic = l16k; xor_size = 6; bpe = T2_FI_BITPERM16KEVEN; bpo = T2_FI_BITPERM16KODD; break;
    default: pn_degree = 14; logic = l32k; xor_size = 4; bpe = T2_FI_BITPERM32K; bpo = T2_FI_BITPERM32K; break;
  }
  pn_mask = (1 << pn_degree) - 1;
  max_states = 1 << (pn_degree + 1);
  h->Heven = (int *)calloc(32768, sizeof(int)); h->Hodd = (int *)calloc(32768, sizeof(int));
  h->HevenP2 = (int *)calloc(32768, sizeof(int)); h->HoddP2 = (int *)calloc(32768, sizeof(int));
  h->HevenFC = (int *)calloc(32768, sizeof(int)); h->HoddFC = (int *)calloc(32768, sizeof(int));
  int qe = 0, qo = 0, qeP = 0, qoP = 0, qeF = 0, qoF = 0, lfsr = 0;
  for (int i = 0; i < max_states; i++) {
    if (i == 0 || i == 1) lfsr = 0;
    else if (i == 2) lfsr = 1;
    else {
      int r = 0;
      for (int k = 0; k < xor_size; k++) r ^= (lfsr >> logic[k]) & 1;
      lfsr &= pn_mask;
      lfsr >>= 1;
      lfsr |= r << (pn_degree - 1);
    }
    int even = 0, odd = 0;
    for (int n = 0; n < pn_degree; n++) even |= ((lfsr >> n) & 1) << bpe[n];
    for (int n = 0; n < pn_degree; n++) odd |= ((lfsr >> n) & 1) << bpo[n];
    even += (i % 2) * (max_states / 2);
    odd += (i % 2) * (max_states / 2);
    if (even < h->C_DATA) h->Heven[qe++] = even;
    if (odd < h->C_DATA) h->Hodd[qo++] = odd;
    if (even < h->C_P2) h->HevenP2[qeP++] = even;
    if (odd < h->C_P2) h->HoddP2[qoP++] = odd;
    if (even < h->N_FC) h->HevenFC[qeF++] = even;
    if (odd < h->N_FC) h->HoddFC[qoF++] = odd;
  }
  if (fft == 32768) {
    for (int j = 0; j < qo; j++) h->Heven[h->Hodd[j]] = j;
    for (int j = 0; j < qoP; j++) h->HevenP2[h->HoddP2[j]] = j;
    for (int j = 0; j < qoF; j++) h->HevenFC[h->HoddFC[j]] = j;
  }
  /* L1-post size (framemapper:978-987), K_sig = ksig_post */
  int n_punc_t = (6 * (KBCH_1_2 - h->ksig_post)) / 5;
  int n_post_t = h->ksig_post + NBCH_PARITY + 9000 - n_punc_t;
  if (h->ksig_post > KBCH_1_2) { orc_fm_destroy(h); return NULL; }   /* one L1-post FEC block only */
  if (h->N_P2 == 1) h->N_post = (int)ceil((float)n_post_t / (2 * (float)h->eta_mod)) * 2 * h->eta_mod;
  else h->N_post = (int)ceil((float)n_post_t / ((float)h->eta_mod * (float)h->N_P2)) * h->eta_mod * h->N_P2;
  h->N_punc = n_punc_t - (h->N_post - n_post_t);
  h->pre_fields[7] = h->N_post / h->eta_mod;
  add_l1pre(h, h->l1pre_cache);
  h->t2_frames = t2frames;
  h->t2_frame_num = 0;
  h->l1_scrambled = v131 ? l1scrambled : 0;

  /* per PLP: cell interleaver permutation (framemapper:998-1107) and time interleaver split (:1108-1119) */
  static const int lg11[2] = {0, 3}, lg12[2] = {0, 2}, lg13[4] = {0, 1, 4, 6}, lg14[6] = {0, 1, 4, 5, 9, 11},
                   lg15[4] = {0, 1, 2, 12};
  h->stream_items = 0;
  for (int p = 0; p < nplp; p++) {
    orc_plp *d = &h->plp[p];
    int cs = d->cell_size, pn_degree, xor_size;
    const int *logic;
    if (cs == 32400) { pn_degree = 15; logic = lg15; xor_size = 4; }
    else if (cs == 16200 || cs == 10800) { pn_degree = 14; logic = lg14; xor_size = 6; }
    else if (cs == 8100) { pn_degree = 13; logic = lg13; xor_size = 4; }
    else if (cs == 4050 || cs == 2700) { pn_degree = 12; logic = lg12; xor_size = 2; }
    else { pn_degree = 11; logic = lg11; xor_size = 2; }
    int pn_mask = (1 << (pn_degree - 1)) - 1, max_states = 1 << pn_degree;
    d->pn_degree = pn_degree;
    d->permutations = (int *)calloc(32768, sizeof(int));
    int q = 0, lfsr = 0;
    for (int i = 0; i < max_states; i++) {
      if (i == 0 || i == 1) lfsr = 0;
      else if (i == 2) lfsr = 1;
      else {
        int r = 0;
        for (int k = 0; k < xor_size; k++) r ^= (lfsr >> logic[k]) & 1;
        lfsr &= pn_mask;
        lfsr >>= 1;
        lfsr |= r << (pn_degree - 2);
      }
      lfsr |= (i % 2) << (pn_degree - 1);
      if (lfsr < cs) d->permutations[q++] = lfsr;
    }
    if (d->ti_blocks == 0) { d->small_fec = 1; d->big_fec = 1; d->n_big = 0; d->n_small = d->fec_blocks; }
    else {
      d->small_fec = (int)floor(((float)d->fec_blocks) / ((float)d->ti_blocks));
      d->big_fec = (int)ceil(((float)d->fec_blocks) / ((float)d->ti_blocks));
      d->n_big = d->fec_blocks % d->ti_blocks;
      d->n_small = d->ti_blocks - d->n_big;
    }
    d->if_items = cs * d->fec_blocks;
    d->stream_items = d->if_items / d->ti_frames;
    d->time_interleave = (cf *)calloc((size_t)d->if_items, sizeof(cf));
    d->ti_out = (cf *)calloc((size_t)d->if_items, sizeof(cf));
  }
  /* 8.3.6.3: Type-1 PLPs back to back in PLP_ID order, then the sub-sliced Type-2 PLPs (frame_layout); the
   * most data cells any T2 frame of the superframe carries must fit */
  if (!h->ntype2 && num_subslices != 1) { orc_fm_destroy(h); return NULL; }
  for (int p = 0; p < nplp; p++) {
    orc_plp *d = &h->plp[p];
    if (d->plp_type != 2) continue;
    if (d->stream_items % num_subslices) { orc_fm_destroy(h); return NULL; }
    d->ss = d->stream_items / num_subslices;
  }
  for (long f = 0; f < t2frames; f++) {
    const int c = frame_layout(h, f);
    if (c > h->stream_items) h->stream_items = c;
  }
  frame_layout(h, 0);
  if (h->N_FC == 0) { h->mapped_items = h->N_P2 * h->C_P2 + numdatasyms * h->C_DATA; h->num_data_symbols = numdatasyms; }
  else { h->mapped_items = h->N_P2 * h->C_P2 + (numdatasyms - 1) * h->C_DATA + h->N_FC; h->num_data_symbols = numdatasyms - 1; }
  int fixed = h->stream_items + 1840 + h->N_post / h->eta_mod + (h->N_FC - h->C_FC);
  if (h->mapped_items < fixed) { orc_fm_destroy(h); return NULL; }   /* reference warns + overflows */
  h->cell_out = (cf *)calloc((size_t)h->mapped_items, sizeof(cf));
  h->frame_out = (cf *)calloc((size_t)h->mapped_items, sizeof(cf));
  h->zigzag = (cf *)calloc((size_t)h->mapped_items, sizeof(cf));
  /* dummy cells of a T2 frame with no data cells at all (a frame without its PLPs, FRAME_INTERVAL > 1) */
  int ndummy = h->mapped_items - (fixed - h->stream_items);
  h->dummy = (cf *)calloc((size_t)ndummy + 1, sizeof(cf));
  /* init_dummy_randomizer (framemapper:1912-1926) */
  int sr = 0x4A80;
  for (int i = 0; i < ndummy; i++) {
    int b = ((sr) ^ (sr >> 1)) & 1;
    h->dummy[i].re = b ? -1.0f : 1.0f;
    sr >>= 1;
    if (b) sr |= 0x4000;
  }
  orc_bb_prbs(h->l1_randomize, KBCH_1_2);   /* init_l1_randomizer (framemapper:1928-1940) */
  return h;
}

/* the reference's single-PLP framemapperfint_cc (include/dvbt2ll/framemapperfint_cc.h:49) */
orc_fm *orc_fm_create(int framesize, int rate, int constellation, int rotation, int fecblocks,
                      int tiblocks, int carriermode, int fftsize, int guardinterval,
                      int l1constellation, int pilotpattern, int t2frames, int numdatasyms,
                      int paprmode, int version, int preamble, int inputmode,
                      int reservedbiasbits, int l1scrambled, int inband) {
  const int plp[ORC_PLP_INTS] = {framesize, rate, constellation, rotation, fecblocks, tiblocks, inputmode, inband,
                                 1, 0, 1, 1, 0};
  return orc_fm_create_mplp(1, plp, 1, carriermode, fftsize, guardinterval, l1constellation, pilotpattern, t2frames,
                            numdatasyms, paprmode, version, preamble, reservedbiasbits, l1scrambled);
}
int orc_fm_stream_items(const orc_fm *h) { return h->stream_items; }
int orc_fm_mapped_items(const orc_fm *h) { return h->mapped_items; }
int orc_fm_l1post_cells(const orc_fm *h) { return h->N_post / h->eta_mod; }
void orc_fm_destroy(orc_fm *h) {
  if (!h) return;
  for (int p = 0; p < ORC_MAX_PLP; p++) {
    free(h->plp[p].permutations); free(h->plp[p].time_interleave); free(h->plp[p].ti_out);
  }
  free(h->Heven); free(h->Hodd); free(h->HevenP2); free(h->HoddP2); free(h->HevenFC); free(h->HoddFC);
  free(h->cell_out); free(h->frame_out); free(h->zigzag); free(h->dummy); free(h);
}

/* test hook: the L1-post signalling bits (one per byte, before the CRC-32) of absolute T2 frame `frame` as
 * orc_fm_work would build them there; returns the bit count (0 when cap is too small) */
int orc_fm_l1post_bits(orc_fm *h, long frame, uint8_t *out, int cap) {
  uint8_t info[FRAME_SIZE_SHORT];
  (void)frame_layout(h, frame);   /* orc_fm_work recomputes the placement of its own frame */
  const int o = l1post_info(h, info, (int)(frame % h->t2_frames));
  if (o > cap) return 0;
  memcpy(out, info, (size_t)o);
  return o;
}

void orc_fm_seek(orc_fm *h, long frame) {
  h->t2_frame_num = (int)(frame % h->t2_frames);
  h->frame = frame;
  for (int p = 0; p < h->nplp; p++) {   /* the PLP's T2 frames before `frame`, mod P_I */
    const orc_plp *d = &h->plp[p];
    const long before = frame > d->first_frame ? (frame - d->first_frame + d->frame_interval - 1) / d->frame_interval : 0;
    h->plp[p].phase = (int)(before % d->ti_frames);
  }
}

int orc_fm_consume(const orc_fm *h, int plp) {
  if (plp < 0 || plp >= h->nplp) return 0;
  const orc_plp *d = &h->plp[plp];
  return h->frame % d->frame_interval == d->first_frame && d->phase == 0 ? d->if_items : 0;
}

/* general_work (framemapper:1948-2151), exactly one T2 frame: in = the cells each PLP consumes this
 * frame (orc_fm_consume: a whole interleaving frame on its first T2 frame, else none), PLPs in order */
int orc_fm_work(orc_fm *h, const float *inf, float *outf) {
  const cf *in = (const cf *)inf;
  cf *out = (cf *)outf;
  const int S = frame_layout(h, h->frame);   /* this T2 frame's PLPs and their placement */
  int M = h->mapped_items;
  int Lp = h->N_post / h->eta_mod;
  for (int p = 0; p < h->nplp; p++) {
    orc_plp *d = &h->plp[p];
    int cs = d->cell_size;
    if (!d->present) continue;
    if (d->phase == 0) {   /* a new interleaving frame: cell + time interleave it (framemapper:1973-2028) */
      /* cell interleaver :1973-1998 */
      int cell_index = 0;
      for (int s = 0; s < d->n_small + d->n_big; s++) {
        int n = 0;
        int fpt = s < d->n_small ? d->small_fec : d->big_fec;
        for (int r = 0; r < fpt; r++) {
          int shift = cs;
          while (shift >= cs) {
            int temp = n;
            shift = 0;
            for (int b = 0; b < d->pn_degree; b++) { shift |= temp & 1; shift <<= 1; temp >>= 1; }
            n++;
          }
          for (int w = 0; w < cs; w++) d->time_interleave[((d->permutations[w] + shift) % cs) + cell_index] = *in++;
          cell_index += cs;
        }
      }
      /* time interleaver :1999-2028, into the interleaving frame's TI output */
      cf *cellout = d->ti_out;
      if (d->ti_blocks != 0) {
        int ti_index = 0;
        for (int s = 0; s < d->n_small + d->n_big; s++) {
          int fpt = s < d->n_small ? d->small_fec : d->big_fec;
          int ncols = 5 * fpt, rows = cs / 5;
          for (int k = 0; k < rows; k++)
            for (int w = 0; w < ncols; w++) *cellout++ = d->time_interleave[rows * w + ti_index + k];
          ti_index += rows * ncols;
        }
      } else {
        for (int w = 0; w < d->if_items; w++) *cellout++ = d->time_interleave[w];
      }
    }
    /* this T2 frame's share of the TI output into the PLP's cells of the frame (8.3.6.3) */
    const cf *src = d->ti_out + (size_t)d->phase * d->stream_items;
    if (d->plp_type == 1) {
      for (int c = 0; c < d->stream_items; c++) h->cell_out[d->start + c] = src[c];
    } else {
      for (int c = 0; c < d->stream_items; c++)
        h->cell_out[h->t2start + (c / d->ss) * h->ssi + d->ss_off + c % d->ss] = src[c];
    }
    d->phase = (d->phase + 1) % d->ti_frames;
  }
  /* frame assembly :2029-2103 */
  cf *dst = h->N_P2 == 1 ? h->frame_out : h->zigzag;
  int o = 0;
  for (int j = 0; j < 1840; j++) dst[o++] = h->l1pre_cache[j];
  add_l1post(h, dst + o, h->t2_frame_num);
  h->t2_frame_num = (h->t2_frame_num + 1) % h->t2_frames;
  h->frame++;
  o += Lp;
  for (int j = 0; j < S; j++) dst[o++] = h->cell_out[j];
  int ndummy = M - S - 1840 - Lp - (h->N_FC - h->C_FC);
  for (int j = 0; j < ndummy; j++) dst[o++] = h->dummy[j];
  for (int j = 0; j < h->N_FC - h->C_FC; j++) { dst[o].re = 0.0f; dst[o].im = 0.0f; o++; }
  if (h->N_P2 != 1) {
    cf *fo = h->frame_out, *iv = h->zigzag;
    int N_P2 = h->N_P2, C_P2 = h->C_P2, count = 0, read = 0, index = 0, save;
    for (int n = 0; n < N_P2; n++) {
      save = read;
      for (int j = 0; j < 1840 / N_P2; j++) { fo[index++] = iv[read]; count++; read += N_P2; }
      read = save + 1;
      index += C_P2 - (1840 / N_P2);
    }
    read = 1840;
    index = 1840 / N_P2;
    for (int n = 0; n < N_P2; n++) {
      save = read;
      for (int j = 0; j < Lp / N_P2; j++) { fo[index++] = iv[read]; count++; read += N_P2; }
      read = save + 1;
      index += C_P2 - (Lp / N_P2);
    }
    read = 1840 + Lp;
    index = (1840 / N_P2) + (Lp / N_P2);
    int dpart = C_P2 - (1840 / N_P2) - (Lp / N_P2);
    for (int n = 0; n < N_P2; n++) {
      for (int j = 0; j < dpart; j++) { fo[index++] = iv[read++]; count++; }
      index += C_P2 - dpart;
    }
    index -= C_P2 - dpart;
    for (int j = 0; j < M - count; j++) fo[index++] = iv[read++];
  }
  /* frequency interleaver :2104-2142, symbol parity restarts every frame */
  const cf *fin = h->frame_out;
  int symbol = 0;
  for (int j = 0; j < h->N_P2; j++) {
    const int *H = (symbol % 2) == 0 ? h->HevenP2 : h->HoddP2;
    for (int k = 0; k < h->C_P2; k++) *out++ = fin[H[k]];
    symbol++;
    fin += h->C_P2;
  }
  for (int j = 0; j < h->num_data_symbols; j++) {
    const int *H = (symbol % 2) == 0 ? h->Heven : h->Hodd;
    for (int k = 0; k < h->C_DATA; k++) *out++ = fin[H[k]];
    symbol++;
    fin += h->C_DATA;
  }
  if (h->N_FC != 0) {
    const int *H = (symbol % 2) == 0 ? h->HevenFC : h->HoddFC;
    for (int k = 0; k < h->N_FC; k++) *out++ = fin[H[k]];
  }
  return M;
}

/* ========================================================================= */
/* pilotgenp1insert_cc                                                        */
/* ========================================================================= */
enum { DATA_CARRIER = 1, P2PILOT_CARRIER, P2PAPR_CARRIER, TRPAPR_CARRIER, SCATTERED_CARRIER,
       CONTINUAL_CARRIER, P2PILOT_CARRIER_INVERTED, SCATTERED_CARRIER_INVERTED, CONTINUAL_CARRIER_INVERTED };
#define MAX_CARRIERS 27841
#define CHIPS 2624

struct orc_pg {
  int N, fft, active_items, num_symbols, left_nulls, right_nulls, pp, carrier_mode, papr_mode, eq;
  int guard, N_P2, C_P2, N_FC, C_FC, C_DATA, K_EXT, C_PS, K_OFFSET, dx, dy, miso, miso_group;
  float normalization;
  cf p2_bpsk[2], sp_bpsk[2], cp_bpsk[2], p2_bpsk_inv[2], sp_bpsk_inv[2], cp_bpsk_inv[2];
  float *inverse_sinc;
  int prbs[MAX_CARRIERS], pn_sequence[CHIPS];
  int p2_map[MAX_CARRIERS], data_map[MAX_CARRIERS], fc_map[MAX_CARRIERS];
  cf p1_time[1024], p1_timeshft[1024];
  cf *buf, *fftbuf;
  cf *tw;   /* float twiddles for the oracle FFT */
};

static const uint16_t *papr_map(int fft, int tr, int *n) {
  switch (fft) {
    case 1024: *n = 10; return tr ? T2_TR_PAPR_MAP_1K : T2_P2_PAPR_MAP_1K;
    case 2048: *n = 18; return tr ? T2_TR_PAPR_MAP_2K : T2_P2_PAPR_MAP_2K;
    case 4096: *n = 36; return tr ? T2_TR_PAPR_MAP_4K : T2_P2_PAPR_MAP_4K;
    case 8192: *n = 72; return tr ? T2_TR_PAPR_MAP_8K : T2_P2_PAPR_MAP_8K;
    case 16384: *n = 144; return tr ? T2_TR_PAPR_MAP_16K : T2_P2_PAPR_MAP_16K;
    default: *n = 288; return tr ? T2_TR_PAPR_MAP_32K : T2_P2_PAPR_MAP_32K;
  }
}

static void cdft_double(const cf *x, cf *y, int n, int sign) {
  /* the n angles' cosines / sines once (each the same double expression as a term-by-term evaluation) */
  double *ct = (double *)malloc(sizeof(double) * 2 * (size_t)n), *st = ct + n;
  for (int m = 0; m < n; m++) {
    double a = sign * 2.0 * M_PI * (double)m / n;
    ct[m] = cos(a);
    st[m] = sin(a);
  }
  for (int k = 0; k < n; k++) {
    double sr = 0, si = 0;
    for (int j = 0; j < n; j++) {
      const int m = (int)((long)j * k % n);
      double c = ct[m], s = st[m];
      sr += x[j].re * c - x[j].im * s;
      si += x[j].re * s + x[j].im * c;
    }
    y[k].re = (float)sr; y[k].im = (float)si;
  }
  free(ct);
}

orc_pg *orc_pg_create(int carriermode, int fftsize, int pilotpattern, int guardinterval,
                      int numdatasyms, int paprmode, int version, int preamble, int misogroup,
                      int equalization, int bandwidth, int vlength) {
  (void)version;
  int fft = fft_points(fftsize);
  if (!fft || vlength < fft) return NULL;
  orc_pg *h = (orc_pg *)calloc(1, sizeof(orc_pg));
  h->N = vlength; h->fft = fft; h->pp = pilotpattern; h->carrier_mode = carriermode;
  h->papr_mode = paprmode; h->eq = equalization; h->miso_group = misogroup;
  int siso = preamble == PREAMBLE_T2_SISO || preamble == PREAMBLE_T2_LITE_SISO;
  h->miso = !siso;
  p2_counts(fft, siso, &h->N_P2, &h->C_P2);
  /* C_PS / K_EXT / K_OFFSET (pilotgen:120-175) */
  switch (fft) {
    case 1024: h->C_PS = 853; break;
    case 2048: h->C_PS = 1705; break;
    case 4096: h->C_PS = 3409; break;
    case 8192: h->C_PS = carriermode ? 6913 : 6817; h->K_EXT = carriermode ? 48 : 0; h->K_OFFSET = carriermode ? 0 : 48; break;
    case 16384: h->C_PS = carriermode ? 13921 : 13633; h->K_EXT = carriermode ? 144 : 0; h->K_OFFSET = carriermode ? 0 : 144; break;
    default: h->C_PS = carriermode ? 27841 : 27265; h->K_EXT = carriermode ? 288 : 0; h->K_OFFSET = carriermode ? 0 : 288; break;
  }
  active_counts(fft, carriermode, pilotpattern, paprmode, guardinterval, siso, &h->C_DATA, &h->N_FC, &h->C_FC);
  /* init_prbs (pilotgen:1245-1266) */
  int sr = 0x7ff;
  for (int i = 0; i < MAX_CARRIERS; i++) {
    int b = ((sr) ^ (sr >> 2)) & 1;
    h->prbs[i] = sr & 1;
    sr >>= 1;
    if (b) sr |= 0x400;
  }
  for (int i = 0, j = 0; i < CHIPS / 8; i++)
    for (int k = 7; k >= 0; k--) h->pn_sequence[j++] = (T2_PN_SEQ_BYTES[i] >> k) & 1;
  /* P2 carrier map (pilotgen:668-747) */
  int C_PS = h->C_PS, K_EXT = h->K_EXT, tx2 = h->miso && misogroup == MISO_TX2;
  for (int i = 0; i < C_PS; i++) h->p2_map[i] = DATA_CARRIER;
  int step = (fft == 32768 && !h->miso) ? 6 : 3;
  for (int i = 0; i < C_PS; i += step)
    h->p2_map[i] = (tx2 && ((i / 3) % 2) && (i % 3 == 0)) ? P2PILOT_CARRIER_INVERTED : P2PILOT_CARRIER;
  if (carriermode == CARRIERS_EXTENDED) {
    for (int i = 0; i < K_EXT; i++) {
      if (tx2) {
        h->p2_map[i] = (((i / 3) % 2) && (i % 3 == 0)) ? P2PILOT_CARRIER_INVERTED : P2PILOT_CARRIER;
        int k = i + (C_PS - K_EXT);
        h->p2_map[k] = (((k / 3) % 2) && (k % 3 == 0)) ? P2PILOT_CARRIER_INVERTED : P2PILOT_CARRIER;
      } else {
        h->p2_map[i] = P2PILOT_CARRIER;
        h->p2_map[i + (C_PS - K_EXT)] = P2PILOT_CARRIER;
      }
    }
  }
  if (h->miso) {
    h->p2_map[K_EXT + 1] = P2PILOT_CARRIER; h->p2_map[K_EXT + 2] = P2PILOT_CARRIER;
    h->p2_map[C_PS - K_EXT - 2] = P2PILOT_CARRIER; h->p2_map[C_PS - K_EXT - 3] = P2PILOT_CARRIER;
  }
  {
    int np;
    const uint16_t *pm = papr_map(fft, 0, &np);
    int koff = fft >= 8192 ? K_EXT : 0;    /* 1K/2K/4K maps are not shifted (pilotgen:720,755,789) */
    for (int i = 0; i < np; i++) h->p2_map[pm[i] + koff] = P2PAPR_CARRIER;
    if (h->miso) {
      for (int i = 0; i < np; i++) {
        int ki = pm[i] + K_EXT;
        if (i < np - 1) { if ((ki % 3) == 1 && (ki + 1) != (pm[i + 1] + K_EXT)) h->p2_map[ki + 1] = P2PILOT_CARRIER; }
        else if ((ki % 3) == 1) h->p2_map[ki + 1] = P2PILOT_CARRIER;
        if (i > 0) { if ((ki % 3) == 2 && (ki - 1) != (pm[i - 1] + K_EXT)) h->p2_map[ki - 1] = P2PILOT_CARRIER; }
        else if ((ki % 3) == 2) h->p2_map[ki - 1] = P2PILOT_CARRIER;
      }
    }
  }
  /* continual pilot amplitude (pilotgen:748-924) */
  double cpa = fft <= 2048 ? 4.0 / 3.0 : fft == 4096 ? (4.0 * sqrt(2.0)) / 3.0 : 8.0 / 3.0;
  h->cp_bpsk[0].re = (float)cpa; h->cp_bpsk[1].re = (float)-cpa;
  h->cp_bpsk_inv[0].re = (float)-cpa; h->cp_bpsk_inv[1].re = (float)cpa;
  /* scattered pilot amplitude and pattern (pilotgen:927-992) */
  static const int dxs[8] = {3, 6, 6, 12, 12, 24, 24, 6}, dys[8] = {4, 2, 4, 2, 4, 2, 4, 16};
  static const double spa[8] = {4.0 / 3.0, 4.0 / 3.0, 7.0 / 4.0, 7.0 / 4.0, 7.0 / 3.0, 7.0 / 3.0, 7.0 / 3.0, 7.0 / 3.0};
  h->dx = dxs[pilotpattern]; h->dy = dys[pilotpattern];
  h->sp_bpsk[0].re = (float)spa[pilotpattern]; h->sp_bpsk[1].re = (float)-spa[pilotpattern];
  h->sp_bpsk_inv[0].re = (float)-spa[pilotpattern]; h->sp_bpsk_inv[1].re = (float)spa[pilotpattern];
  /* frame-closing symbol map (pilotgen:993-1070) */
  for (int i = 0; i < C_PS; i++) h->fc_map[i] = DATA_CARRIER;
  for (int i = 0; i < C_PS; i++)
    if (i % h->dx == 0) h->fc_map[i] = (tx2 && ((i / h->dx) % 2)) ? SCATTERED_CARRIER_INVERTED : SCATTERED_CARRIER;
  if ((fft == 1024 && (pilotpattern == PILOT_PP4 || pilotpattern == PILOT_PP5)) ||
      (fft == 2048 && pilotpattern == PILOT_PP7))
    h->fc_map[C_PS - 2] = SCATTERED_CARRIER;
  if (tx2 && ((numdatasyms + h->N_P2 - 1) % 2)) { h->fc_map[0] = SCATTERED_CARRIER_INVERTED; h->fc_map[C_PS - 1] = SCATTERED_CARRIER_INVERTED; }
  else { h->fc_map[0] = SCATTERED_CARRIER; h->fc_map[C_PS - 1] = SCATTERED_CARRIER; }
  if (paprmode == PAPR_TR || paprmode == PAPR_BOTH) {
    int np;
    const uint16_t *pm = papr_map(fft, 0, &np);    /* FC symbol uses the P2 reserved set */
    int koff = fft >= 8192 ? K_EXT : 0;
    for (int i = 0; i < np; i++) h->fc_map[pm[i] + koff] = TRPAPR_CARRIER;
  }
  h->active_items = h->N_FC == 0 ? h->N_P2 * h->C_P2 + numdatasyms * h->C_DATA
                                 : h->N_P2 * h->C_P2 + (numdatasyms - 1) * h->C_DATA + h->N_FC;
  h->left_nulls = ((vlength - C_PS) / 2) + 1;
  h->right_nulls = (vlength - C_PS) / 2;
  double p2a = (fft == 32768 && !h->miso) ? sqrt(37.0) / 5.0 : sqrt(31.0) / 5.0;
  h->p2_bpsk[0].re = (float)p2a; h->p2_bpsk[1].re = (float)-p2a;
  h->p2_bpsk_inv[0].re = (float)-p2a; h->p2_bpsk_inv[1].re = (float)p2a;
  h->normalization = (float)(5.0 / sqrt(27.0 * C_PS));
  switch (guardinterval) {
    case GI_1_32: h->guard = vlength / 32; break;
    case GI_1_16: h->guard = vlength / 16; break;
    case GI_1_8: h->guard = vlength / 8; break;
    case GI_1_4: h->guard = vlength / 4; break;
    case GI_1_128: h->guard = vlength / 128; break;
    case GI_19_128: h->guard = (vlength * 19) / 128; break;
    default: h->guard = (vlength * 19) / 256; break;
  }
  /* P1 (pilotgen:1119-1178) */
  {
    int p1r[384], ms[384], dbpsk[385];
    int s = 0x4e46;
    for (int i = 0; i < 384; i++) {
      int b = ((s) ^ (s >> 1)) & 1;
      p1r[i] = b == 0 ? 1 : -1;
      s >>= 1;
      if (b) s |= 0x4000;
    }
    int idx = 0, s1 = preamble, s2 = (fftsize & 0x7) << 1;
    for (int i = 0; i < 8; i++) for (int j = 7; j >= 0; j--) ms[idx++] = (T2_P1_S1[s1][i] >> j) & 1;
    for (int i = 0; i < 32; i++) for (int j = 7; j >= 0; j--) ms[idx++] = (T2_P1_S2[s2][i] >> j) & 1;
    for (int i = 0; i < 8; i++) for (int j = 7; j >= 0; j--) ms[idx++] = (T2_P1_S1[s1][i] >> j) & 1;
    dbpsk[0] = 1;
    for (int i = 1; i < 385; i++) dbpsk[i] = ms[i - 1] == 1 ? -dbpsk[i - 1] : dbpsk[i - 1];
    for (int i = 0; i < 384; i++) dbpsk[i] = dbpsk[i + 1] * p1r[i];
    cf fr[1024], sh[1024], x[1024];
    memset(fr, 0, sizeof(fr));
    for (int i = 0; i < 384; i++) fr[T2_P1_CARRIERS[i] + 86].re = (float)dbpsk[i];
    float inv = (float)sqrt(384.0);
    for (int pass = 0; pass < 2; pass++) {
      const cf *src = fr;
      if (pass == 1) { for (int i = 0; i < 1023; i++) sh[i + 1] = fr[i]; sh[0] = fr[1023]; src = sh; }
      for (int i = 0; i < 512; i++) { x[512 + i] = src[i]; x[i] = src[512 + i]; }
      cf *dst = pass == 0 ? h->p1_time : h->p1_timeshft;
      cdft_double(x, dst, 1024, +1);
      for (int i = 0; i < 1024; i++) { dst[i].re /= inv; dst[i].im /= inv; }
    }
  }
  /* inverse-sinc EQ (pilotgen:1179-1219) */
  {
    double fs;
    switch (bandwidth) {
      case 0: fs = 131.0 * 1000000.0 / 71.0; break;
      case 1: fs = 5.0 * 8000000.0 / 7.0; break;
      case 2: fs = 6.0 * 8000000.0 / 7.0; break;
      case 3: fs = 7.0 * 8000000.0 / 7.0; break;
      case 4: fs = 8.0 * 8000000.0 / 7.0; break;
      case 5: fs = 10.0 * 8000000.0 / 7.0; break;
      default: fs = 1.0; break;
    }
    double fstep = fs / vlength, f = 0.0, sincrms = 0.0;
    h->inverse_sinc = (float *)calloc((size_t)vlength, sizeof(float));
    for (int i = 0; i < vlength / 2; i++) {
      double x = M_PI * f / fs;
      double sinc = i == 0 ? 1.0 : sin(x) / x;
      sincrms += sinc * sinc;
      h->inverse_sinc[i + vlength / 2] = (float)(1.0 / sinc);
      h->inverse_sinc[vlength / 2 - i - 1] = (float)(1.0 / sinc);
      f = f + fstep;
    }
    sincrms = sqrt(sincrms / (vlength / 2));
    float fr = (float)sincrms;
    for (int i = 0; i < vlength; i++) h->inverse_sinc[i] *= fr;
  }
  h->num_symbols = numdatasyms + h->N_P2;
  h->buf = (cf *)calloc((size_t)vlength, sizeof(cf));
  h->fftbuf = (cf *)calloc((size_t)vlength, sizeof(cf));
  h->tw = (cf *)calloc((size_t)vlength, sizeof(cf));
  for (int i = 0; i < vlength; i++) {
    h->tw[i].re = (float)cos(2.0 * M_PI * i / vlength);
    h->tw[i].im = (float)sin(2.0 * M_PI * i / vlength);
  }
  return h;
}
int orc_pg_active_items(const orc_pg *h) { return h->active_items; }
int orc_pg_output_items(const orc_pg *h) { return h->num_symbols * (h->N + h->guard) + 2048; }
int orc_pg_num_symbols(const orc_pg *h) { return h->num_symbols; }
float orc_pg_normalization(const orc_pg *h) { return h->normalization; }
int orc_pg_guard(const orc_pg *h) { return h->guard; }
void orc_pg_destroy(orc_pg *h) {
  if (!h) return;
  free(h->inverse_sinc); free(h->buf); free(h->fftbuf); free(h->tw); free(h);
}
void orc_pg_p1(const orc_pg *h, float *p1) {
  cf *o = (cf *)p1;
  int k = 0;
  for (int j = 0; j < 542; j++) o[k++] = h->p1_timeshft[j];
  for (int j = 0; j < 1024; j++) o[k++] = h->p1_time[j];
  for (int j = 542; j < 1024; j++) o[k++] = h->p1_timeshft[j];
}

/* init_pilots (pilotgen:1285-2782) */
static void init_pilots(orc_pg *h, int symbol) {
  int C_PS = h->C_PS, tx2 = h->miso && h->miso_group == MISO_TX2;
  for (int i = 0; i < C_PS; i++) h->data_map[i] = DATA_CARRIER;
  for (int s = 0; s < T2_NCP_STEPS; s++) {
    const t2_cp_step_t *st = &T2_CP_STEPS[s];
    if (st->fft != h->fft || st->pp != h->pp + 1) continue;
    if (st->ext_only && h->carrier_mode != CARRIERS_EXTENDED) continue;
    const uint16_t *list = T2_CP_LIST + T2_CP_LIST_SPAN[st->list][0];
    for (int i = 0; i < st->count; i++) {
      int k = st->modulus ? list[i] % st->modulus : list[i];
      if (st->miso_inv && tx2 && ((k / h->dx) % 2) && ((k % h->dx) == 0)) h->data_map[k] = CONTINUAL_CARRIER_INVERTED;
      else h->data_map[k] = CONTINUAL_CARRIER;
    }
  }
  for (int i = 0; i < C_PS; i++) {
    int rem = (i - h->K_EXT) % (h->dx * h->dy);
    if (rem < 0) rem += h->dx * h->dy;
    if (rem == h->dx * (symbol % h->dy))
      h->data_map[i] = (tx2 && ((i / h->dx) % 2)) ? SCATTERED_CARRIER_INVERTED : SCATTERED_CARRIER;
  }
  if (tx2 && (symbol % 2)) { h->data_map[0] = SCATTERED_CARRIER_INVERTED; h->data_map[C_PS - 1] = SCATTERED_CARRIER_INVERTED; }
  else { h->data_map[0] = SCATTERED_CARRIER; h->data_map[C_PS - 1] = SCATTERED_CARRIER; }
  if (h->papr_mode == PAPR_TR || h->papr_mode == PAPR_BOTH) {
    int shift = h->carrier_mode == CARRIERS_NORMAL ? h->dx * (symbol % h->dy)
                                                   : h->dx * ((symbol + (h->K_EXT / h->dx)) % h->dy);
    int np;
    const uint16_t *pm = papr_map(h->fft, 1, &np);
    for (int i = 0; i < np; i++) h->data_map[pm[i] + shift] = TRPAPR_CARRIER;
  }
}

/* carrier fill (pilotgen:2811-2889) for symbol j; returns inputs consumed */
static int fill_symbol(orc_pg *h, int j, const cf *in, cf *bins) {
  int L_FC = h->N_FC != 0 ? 1 : 0, used = 0, o = 0;
  cf zero = {0.0f, 0.0f};
  for (int n = 0; n < h->left_nulls; n++) bins[o++] = zero;
  int pn = h->pn_sequence[j];
  for (int n = 0; n < h->C_PS; n++) {
    int b = h->prbs[n + h->K_OFFSET] ^ pn;
    if (j < h->N_P2) {
      int t = h->p2_map[n];
      if (t == P2PILOT_CARRIER) bins[o++] = h->p2_bpsk[b];
      else if (t == P2PILOT_CARRIER_INVERTED) bins[o++] = h->p2_bpsk_inv[b];
      else if (t == P2PAPR_CARRIER) bins[o++] = zero;
      else bins[o++] = in[used++];
    } else if (j == h->num_symbols - L_FC) {
      int t = h->fc_map[n];
      if (t == SCATTERED_CARRIER) bins[o++] = h->sp_bpsk[b];
      else if (t == SCATTERED_CARRIER_INVERTED) bins[o++] = h->sp_bpsk_inv[b];
      else if (t == TRPAPR_CARRIER) bins[o++] = zero;
      else bins[o++] = in[used++];
    } else {
      int t = h->data_map[n];
      if (t == SCATTERED_CARRIER) bins[o++] = h->sp_bpsk[b];
      else if (t == SCATTERED_CARRIER_INVERTED) bins[o++] = h->sp_bpsk_inv[b];
      else if (t == CONTINUAL_CARRIER) bins[o++] = h->cp_bpsk[b];
      else if (t == CONTINUAL_CARRIER_INVERTED) bins[o++] = h->cp_bpsk_inv[b];
      else if (t == TRPAPR_CARRIER) bins[o++] = zero;
      else bins[o++] = in[used++];
    }
  }
  for (int n = 0; n < h->right_nulls; n++) bins[o++] = zero;
  if (h->eq) for (int n = 0; n < h->N; n++) { bins[n].re *= h->inverse_sinc[n]; bins[n].im *= h->inverse_sinc[n]; }
  return used;
}

int orc_pg_carriers(orc_pg *h, const float *inf, float *carriers) {
  const cf *in = (const cf *)inf;
  cf *c = (cf *)carriers;
  for (int j = 0; j < h->num_symbols; j++) {
    if (j >= h->N_P2 && !(h->N_FC != 0 && j == h->num_symbols - 1)) init_pilots(h, j);
    in += fill_symbol(h, j, in, c + (size_t)j * h->N);
  }
  return h->num_symbols * h->N;
}

/* oracle inverse FFT: iterative radix-2, e^{+j}, unnormalized (stand-in for FFTW backward) */
static void ifft_radix2(const cf *tw, cf *x, int n) {
  for (int i = 1, j = 0; i < n; i++) {
    int bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) { cf t = x[i]; x[i] = x[j]; x[j] = t; }
  }
  for (int len = 2; len <= n; len <<= 1) {
    int st = n / len;
    for (int i = 0; i < n; i += len)
      for (int k = 0; k < len / 2; k++) {
        cf w = tw[k * st], a = x[i + k], b = x[i + k + len / 2], t;
        t.re = b.re * w.re - b.im * w.im; t.im = b.re * w.im + b.im * w.re;
        x[i + k].re = a.re + t.re; x[i + k].im = a.im + t.im;
        x[i + k + len / 2].re = a.re - t.re; x[i + k + len / 2].im = a.im - t.im;
      }
  }
}

int orc_pg_work(orc_pg *h, const float *inf, float *outf) {
  const cf *in = (const cf *)inf;
  cf *out = (cf *)outf;
  int N = h->N, G = h->guard;
  orc_pg_p1(h, (float *)out);
  out += 2048;
  for (int j = 0; j < h->num_symbols; j++) {
    if (j >= h->N_P2 && !(h->N_FC != 0 && j == h->num_symbols - 1)) init_pilots(h, j);
    in += fill_symbol(h, j, in, h->buf);
    for (int i = 0; i < N / 2; i++) { h->fftbuf[N / 2 + i] = h->buf[i]; h->fftbuf[i] = h->buf[N / 2 + i]; }
    ifft_radix2(h->tw, h->fftbuf, N);
    for (int i = 0; i < N; i++) { h->fftbuf[i].re *= h->normalization; h->fftbuf[i].im *= h->normalization; }
    memcpy(out + G, h->fftbuf, sizeof(cf) * (size_t)N);
    memcpy(out, h->fftbuf + N - G, sizeof(cf) * (size_t)G);
    out += N + G;
  }
  return h->num_symbols * (N + G) + 2048;
}
