// t2_plan.cpp -- host-side configuration planning (see t2_plan.h).
//
// Compiled with -ffp-contract=off: the float constellation, pilot and L1 cell values
// must round exactly as the reference's (which is built -O3 without -march, i.e. no FMA).
#include "t2_plan.h"

#include <cmath>
#include <cstring>
#include <algorithm>
#include <numeric>

#include "gen/dvbt2_std_tables.h"

namespace t2 {

namespace {

// enum values of include/dvbt2ll/dvbt2ll_config.h:60-202
enum { R12 = 0, R35, R23, R34, R45, R56, R13, R25 };
enum { QPSK = 0, QAM16, QAM64, QAM256 };
enum { FFT2K = 0, FFT8K, FFT4K, FFT1K, FFT16K, FFT32K, FFT8KT2GI, FFT32KT2GI, FFT16KT2GI = 11 };
enum { GI132 = 0, GI116, GI18, GI14, GI1128, GI19128, GI19256 };
enum { PAPROFF = 0, PAPRACE, PAPRTR, PAPRBOTH };
enum { PP1 = 0, PP2, PP3, PP4, PP5, PP6, PP7, PP8 };

constexpr int kNormal = 64800, kShort = 16200;

// ---------------------------------------------------------------- GF(2) polynomials < x^192
struct Poly192 {
  uint64_t w[3] = {0, 0, 0};
  bool bit(int i) const { return (w[i >> 6] >> (i & 63)) & 1; }
  void set(int i) { w[i >> 6] |= 1ull << (i & 63); }
  void flip(int i) { w[i >> 6] ^= 1ull << (i & 63); }
};

// v * x mod g for deg g = P (g holds the low P coefficients)
Poly192 times_x(Poly192 v, const Poly192 &g, int P) {
  bool top = v.bit(P - 1);
  v.w[2] = (v.w[2] << 1) | (v.w[1] >> 63);
  v.w[1] = (v.w[1] << 1) | (v.w[0] >> 63);
  v.w[0] <<= 1;
  for (int k = 0; k < 3; k++) {
    int lo = 64 * k;
    if (P <= lo) v.w[k] = 0;
    else if (P < lo + 64) v.w[k] &= (1ull << (P - lo)) - 1;
  }
  if (top)
    for (int k = 0; k < 3; k++) v.w[k] ^= g.w[k];
  return v;
}

// BCH generator: product of the first P/16 (normal) or all 12 (short) minimal polynomials
// (reference bch_poly_build_tables, bbheader:424-502)
Poly192 bch_generator(bool normal, int P) {
  std::vector<uint8_t> acc{1};
  int n = normal ? P / 16 : 12;
  for (int k = 0; k < n; k++) {
    const uint8_t *m = normal ? T2_BCH_MINPOLY_NORMAL[k] : T2_BCH_MINPOLY_SHORT[k];
    int lm = normal ? 17 : 15;
    std::vector<uint8_t> r(acc.size() + lm - 1, 0);
    for (size_t i = 0; i < acc.size(); i++)
      if (acc[i])
        for (int j = 0; j < lm; j++) r[i + j] ^= m[j];
    acc.swap(r);
  }
  Poly192 g;
  for (int i = 0; i < P; i++)
    if (acc[i]) g.set(i);
  return g;
}

const t2_ldpc_code_t *find_code(int normal, int rate) {
  for (int i = 0; i < T2_LDPC_NCODES; i++)
    if (T2_LDPC_CODES[i].framesize_normal == normal && T2_LDPC_CODES[i].rate == rate) return &T2_LDPC_CODES[i];
  return nullptr;
}

// PRBS 1 + x^14 + x^15, init 100101010000000 (BB scrambler, dummy cells, L1 scrambler)
void prbs15(uint8_t *bits, int n) {
  unsigned s = 0x4A80;
  for (int i = 0; i < n; i++) {
    unsigned b = (s ^ (s >> 1)) & 1;
    bits[i] = (uint8_t)b;
    s = (s >> 1) | (b << 14);
  }
}

int cell_size_of(int normal, int constellation) {
  static const int n[4] = {32400, 16200, 10800, 8100}, s[4] = {8100, 4050, 2700, 2025};
  if (constellation < 0 || constellation > 3) return 0;
  return normal ? n[constellation] : s[constellation];
}

}  // namespace

int fft_points(int fftsize) {
  switch (fftsize) {
    case FFT1K: return 1024;
    case FFT2K: return 2048;
    case FFT4K: return 4096;
    case FFT8K: case FFT8KT2GI: return 8192;
    case FFT16K: case FFT16KT2GI: return 16384;
    case FFT32K: case FFT32KT2GI: return 32768;
    default: return 0;
  }
}

// ============================================================================ FEC
// FEC parameters: reference bbheaderbch ctor lib/bbheaderbch_bb_impl.cc:51-165
static bool fec_numbers(int normal, int rate, int *kbch, int *nbch, int *q, int *P) {
  struct E { int k, n, q, p; };
  static const E N[6] = {{32208, 32400, 90, 192}, {38688, 38880, 72, 192}, {43040, 43200, 60, 160},
                         {48408, 48600, 45, 192}, {51648, 51840, 36, 192}, {53840, 54000, 30, 160}};
  static const E S[8] = {{7032, 7200, 25, 168}, {9552, 9720, 18, 168}, {10632, 10800, 15, 168},
                         {11712, 11880, 12, 168}, {12432, 12600, 10, 168}, {13152, 13320, 8, 168},
                         {5232, 5400, 30, 168}, {6312, 6480, 27, 168}};
  const E *e = nullptr;
  if (normal && rate >= 0 && rate <= R56) e = &N[rate];
  if (!normal && rate >= 0 && rate <= R25) e = &S[rate];
  if (!e) return false;
  *kbch = e->k; *nbch = e->n; *q = e->q; *P = e->p;
  return true;
}

int build_fec(int framesize, int rate, int constellation, FecPlan &fp) {
  int normal = framesize == 1;
  if (framesize != 0 && framesize != 1) return -1;
  if (!fec_numbers(normal, rate, &fp.kbch, &fp.nbch, &fp.q, &fp.nparity)) return -1;
  fp.normal = normal;
  fp.rate = rate;
  fp.nldpc = normal ? kNormal : kShort;
  fp.pbits = fp.nldpc - fp.nbch;
  // QPSK carries parity interleaving only for rates 1/3 and 2/5 (interleavermod:291-314)
  fp.parity_interleave = !(constellation == QPSK && rate != R13 && rate != R25);
  const int P = fp.nparity;
  Poly192 g = bch_generator(normal, P);
  // byte table: d(x) * x^P mod g
  fp.bch_tab.assign(256 * 3, 0);
  for (int d = 0; d < 256; d++) {
    Poly192 v;
    v.w[0] = (uint64_t)d;
    for (int i = 0; i < P; i++) v = times_x(v, g, P);
    for (int k = 0; k < 3; k++) fp.bch_tab[d * 3 + k] = v.w[k];
  }
  const int L = fp.kbch / 8;
  // the BBFRAME in 64 chunks, one per lane of the BCH wave (the chunks end at L)
  fp.bch_chunk = (L + 63) / 64;
  // the chunk remainder of lane l moves to the end of the message: r_l x^(8 chunk (63 - l))
  // mod g, as the XOR of P/4 nibble-table entries (one lookup per 4-bit digit of r_l)
  {
    const int NJ = P / 4;
    fp.bch_ctab.assign((size_t)NJ * 16 * 64 * 4, 0);
    Poly192 base;
    base.set(0);   // lane 63: x^0
    for (int l = 63; l >= 0; l--) {
      Poly192 pj = base;   // base x^(4 j)
      for (int j = 0; j < NJ; j++) {
        Poly192 q[4];
        q[0] = pj;
        for (int k = 1; k < 4; k++) q[k] = times_x(q[k - 1], g, P);
        for (int v = 0; v < 16; v++) {
          uint64_t *e = &fp.bch_ctab[(((size_t)j * 16 + v) * 64 + l) * 4];
          for (int k = 0; k < 4; k++)
            if ((v >> k) & 1)
              for (int w = 0; w < 3; w++) e[w] ^= q[k].w[w];
        }
        pj = times_x(q[3], g, P);
      }
      for (long i = 0; i < 8L * fp.bch_chunk; i++) base = times_x(base, g, P);
    }
  }
  // LDPC: info group gidx (360 bits) with address x lands in parity row a = x mod q with
  // cyclic offset b = x div q (columns c = (b + n) mod 360, since pbits = 360 q)
  const t2_ldpc_code_t *c = find_code(normal, rate);
  if (!c || c->q != fp.q || c->nrows * 360 != fp.nbch) return -1;
  std::vector<std::vector<uint32_t>> rows(fp.q);
  int off = c->addr_off;
  for (int gidx = 0; gidx < c->nrows; gidx++) {
    int cnt = T2_LDPC_ROWLEN[c->row_off + gidx];
    for (int e = 0; e < cnt; e++) {
      int x = T2_LDPC_ADDR[off + e];
      rows[x % fp.q].push_back(((uint32_t)gidx << 16) | (uint32_t)(x / fp.q));
    }
    off += cnt;
  }
  fp.ldpc_rowptr.assign(fp.q + 1, 0);
  fp.ldpc_ent.clear();
  for (int a = 0; a < fp.q; a++) {
    fp.ldpc_rowptr[a] = (uint16_t)fp.ldpc_ent.size();
    fp.ldpc_ent.insert(fp.ldpc_ent.end(), rows[a].begin(), rows[a].end());
  }
  fp.ldpc_rowptr[fp.q] = (uint16_t)fp.ldpc_ent.size();
  // BB scrambler bytes (init_bb_randomiser, bbheader:357-369)
  std::vector<uint8_t> bits(fp.kbch);
  prbs15(bits.data(), fp.kbch);
  fp.prbs_bytes.assign(((L + 31) & ~31) + 32, 0);   // zero-padded: the FEC kernels read whole words / chunks
  for (int i = 0; i < fp.kbch; i++) fp.prbs_bytes[i >> 3] |= bits[i] << (7 - (i & 7));
  // CRC-8 (x^8+x^7+x^6+x^4+x^2+1, MSB first) table and zero-byte extension tables
  fp.crc8_tab.assign(256, 0);
  for (int i = 0; i < 256; i++) {
    unsigned r = (unsigned)i;
    for (int k = 0; k < 8; k++) r = ((r & 0x80) ? (r << 1) ^ 0xD5u : r << 1) & 0xFFu;
    fp.crc8_tab[i] = (uint8_t)r;
  }
  // BBHEADER CRC-8 (add_crc8_bits, bbheader:247-270): LSB-first register, polynomial 0xAB, the
  // 72 header bits MSB first.  Linear with a zero start, so the CRC is the XOR of the
  // contributions of the set bits (the kernel forms it with one lane per bit)
  fp.hcrc_bits.assign(72, 0);
  for (int n = 0; n < 72; n++) {
    unsigned crc = 0;
    for (int m = 0; m < 72; m++) {
      const unsigned b = (m == n ? 1u : 0u) ^ (crc & 1u);
      crc >>= 1;
      if (b) crc ^= 0xABu;
    }
    fp.hcrc_bits[n] = (uint8_t)crc;
  }
  fp.crc8_shift.assign(8 * 256, 0);
  for (int k = 0; k < 8; k++) {
    int after = 187 - std::min(24 * k + 24, 187);
    for (int s = 0; s < 256; s++) {
      uint8_t v = (uint8_t)s;
      for (int i = 0; i < after; i++) v = fp.crc8_tab[v];
      fp.crc8_shift[k * 256 + s] = v;
    }
  }
  return 0;
}

int build_bch_mfma(FecPlan &fp) {
  if (!fp.kbch) return -1;
  const int P = fp.nparity, L = fp.kbch / 8;
  Poly192 g = bch_generator(fp.normal, P);
  // BCH as a GF(2) matrix product for the chain's MFMA pass (bbch_kernel): parity bit p (p = 0
  // the x^(P-1) coefficient, sent first) of message bit i is coefficient P-1-p of x^(kbch-1-i) x^P
  // mod g.  fp4 (e2m1) B fragments of v_mfma_scale_f32_32x32x64_f8f6f4: 32-byte message chunk q,
  // K-step u (the little-endian message word w of bytes 32 q + 16 (l >> 5) + 4 u .. + 3), parity tile
  // t, lane l, dword d, nibble e <-> bit 4 e + d of w, i.e. message byte b = 32 q + 16 (l >> 5) + 4 u +
  // (4 e + d) / 8, bit (4 e + d) % 8 (LSB first: i = 8 b + 7 - (4 e + d) % 8), parity p = 32 t + (l & 31).
  // The A fragment's dword d is the message bits left in place where it can be: w & 0x11111111 << d for
  // d = 0, 1, 2 (nibbles 0001 = 0.5, 0010 = 1.0, 0100 = 2.0) and (w >> 1) & 0x44444444 for d = 3 (bit 3 of
  // a nibble is the sign), scale 1; so B's set entries are 2.0, 1.0, 0.5, 0.5 (nibbles 0x4, 0x2, 0x1, 0x1)
  // for d = 0 .. 3 and every product of set bits is exactly 1.  Bits past kbch and parities past P are zero.
  fp.bch_nq = (L + 31) / 32;
  fp.bch_nt = (P + 31) / 32;
  std::vector<Poly192> col(fp.kbch);
  Poly192 r;
  r.set(0);
  for (int i = 0; i < P; i++) r = times_x(r, g, P);   // x^P mod g: message bit kbch - 1
  for (int i = fp.kbch - 1; i >= 0; i--) {
    col[i] = r;
    r = times_x(r, g, P);
  }
  fp.bch_mfma.assign((size_t)fp.bch_nq * 4 * fp.bch_nt * 64 * 4, 0);
  for (int q = 0; q < fp.bch_nq; q++)
    for (int u = 0; u < 4; u++)
      for (int t = 0; t < fp.bch_nt; t++)
        for (int l = 0; l < 64; l++) {
          const int p = 32 * t + (l & 31);
          uint32_t *e4 = &fp.bch_mfma[((((size_t)q * 4 + u) * fp.bch_nt + t) * 64 + l) * 4];
          for (int d = 0; d < 4; d++)
            for (int e = 0; e < 8; e++) {
              const int wb = 4 * e + d, b = 32 * q + 16 * (l >> 5) + 4 * u + wb / 8, i = 8 * b + 7 - wb % 8;
              if (i < fp.kbch && p < P && col[i].bit(P - 1 - p)) e4[d] |= (d == 0 ? 4u : d == 1 ? 2u : 1u) << (4 * e);
            }
        }
  return 0;
}

// ============================================================================ QAM / bit interleaver
// complex<float> *= complex<float> as libstdc++ performs it (no contraction)
static cf32 cmul(cf32 a, cf32 b) {
  volatile float ac = a.re * b.re, bd = a.im * b.im, ad = a.re * b.im, bc = a.im * b.re;
  return cf32{ac - bd, ad + bc};
}

// Gray-mapped QAM, optionally rotated: interleavermod ctor lib/interleavermod_bc_impl.cc:169-253
void qam_table(int constellation, int rotation, cf32 *lut, int *mod) {
  static const double a16[4] = {3, 1, -3, -1};
  static const double a64[8] = {7, 5, 1, 3, -7, -5, -1, -3};
  static const double a256[16] = {15, 13, 9, 11, 1, 3, 7, 5, -15, -13, -9, -11, -1, -3, -7, -5};
  int bits = constellation == QAM16 ? 4 : constellation == QAM64 ? 6 : constellation == QAM256 ? 8 : 2;
  int n = 1 << bits;
  static const double norm2[4] = {2.0, 10.0, 42.0, 170.0};
  static const double deg[4] = {29.0, 16.8, 8.6, 3.576334375};
  int ci = bits == 2 ? 0 : bits == 4 ? 1 : bits == 6 ? 2 : 3;
  double norm = std::sqrt(norm2[ci]);
  const double *amp = ci == 1 ? a16 : ci == 2 ? a64 : a256;
  for (int i = 0; i < n; i++) {
    if (ci == 0) {
      lut[i].re = (float)((i & 2 ? -1.0 : 1.0) / norm);
      lut[i].im = (float)((i & 1 ? -1.0 : 1.0) / norm);
      continue;
    }
    // even bit positions (from the MSB) select the real amplitude, odd ones the imaginary
    int ri = 0, ii = 0;
    for (int b = 0; b < bits / 2; b++) {
      ri |= ((i >> (bits - 1 - 2 * b)) & 1) << (bits / 2 - 1 - b);
      ii |= ((i >> (bits - 2 - 2 * b)) & 1) << (bits / 2 - 1 - b);
    }
    lut[i].re = (float)(amp[ri] / norm);
    lut[i].im = (float)(amp[ii] / norm);
  }
  if (rotation) {
    double phi = (2.0 * M_PI * deg[ci]) / 360.0;
    cf32 r{(float)std::cos(phi), (float)std::sin(phi)};
    for (int i = 0; i < n; i++) lut[i] = cmul(lut[i], r);
  }
  *mod = bits;
}

int build_map(int framesize, int rate, int constellation, int rotation, MapPlan &mp) {
  int normal = framesize == 1;
  mp.cs = cell_size_of(normal, constellation);
  if (!mp.cs) return -1;
  mp.nldpc = normal ? kNormal : kShort;
  mp.rotation = rotation ? 1 : 0;
  qam_table(constellation, rotation, mp.lut, &mp.mod);
  const uint8_t *tw = nullptr, *mx = nullptr;
  switch (constellation) {      // interleavermod:333-350, 422-439, 519-528, 617-625
    case QPSK: mp.mode = MAP_PAIRS; mp.W = 2; break;
    case QAM16:
      mp.mode = MAP_TWIST2; mp.W = 8;
      tw = normal ? T2_BI_TWIST16N : T2_BI_TWIST16S;
      mx = (rate == R35 && normal) ? T2_BI_MUX16_35 : (rate == R13 && !normal) ? T2_BI_MUX16_13
         : (rate == R25 && !normal) ? T2_BI_MUX16_25 : T2_BI_MUX16;
      break;
    case QAM64:
      mp.mode = MAP_TWIST2; mp.W = 12;
      tw = normal ? T2_BI_TWIST64N : T2_BI_TWIST64S;
      mx = (rate == R35 && normal) ? T2_BI_MUX64_35 : (rate == R13 && !normal) ? T2_BI_MUX64_13
         : (rate == R25 && !normal) ? T2_BI_MUX64_25 : T2_BI_MUX64;
      break;
    default:
      if (normal) {
        mp.mode = MAP_TWIST2; mp.W = 16; tw = T2_BI_TWIST256N;
        mx = rate == R35 ? T2_BI_MUX256_35 : rate == R23 ? T2_BI_MUX256_23 : T2_BI_MUX256;
      } else {
        mp.mode = MAP_TWIST1; mp.W = 8; tw = T2_BI_TWIST256S;
        mx = rate == R13 ? T2_BI_MUX256S_13 : rate == R25 ? T2_BI_MUX256S_25 : T2_BI_MUX256S;
      }
      break;
  }
  mp.R = mp.nldpc / mp.W;
  for (int e = 0; e < mp.W && tw; e++) {
    mp.twist[e] = tw[e];
    mp.mux[e] = mx[e];
  }
  return 0;
}

// ============================================================================ frame mapper
namespace {

struct Counts { int n_p2, c_p2, c_data, n_fc, c_fc; };

// N_P2/C_P2 (framemapper:290-356) and C_DATA/N_FC/C_FC (framemapper:425-915)
bool active_counts(int fftsize, int carriermode, int pp, int papr, int gi, int preamble, Counts &c) {
  int N = fft_points(fftsize);
  if (!N || pp < PP1 || pp > PP8) return false;
  bool siso = preamble == 0 || preamble == 3;
  int lg = 0;
  for (int t = N; t > 1024; t >>= 1) lg++;           // 0..5 for 1K..32K
  static const int np2[6] = {16, 8, 4, 2, 1, 1};
  static const int cp2s[6] = {558, 1118, 2236, 4472, 8944, 22432};
  static const int cp2m[6] = {546, 1098, 2198, 4398, 8814, 17612};
  c.n_p2 = np2[lg];
  c.c_p2 = siso ? cp2s[lg] : cp2m[lg];
  c.c_data = c.n_fc = c.c_fc = 0;
  int ext = N >= 8192 ? carriermode : 0;
  bool found = false;
  for (int i = 0; i < T2_NCELL_COUNTS; i++) {
    const t2_cell_counts_t &e = T2_CELL_COUNTS[i];
    if (e.fft == N && e.ext == ext && e.pp == pp + 1) {
      c.c_data = e.c_data; c.n_fc = e.n_fc; c.c_fc = e.c_fc; found = true;
    }
  }
  if (!found) return false;
  if (papr == PAPRTR || papr == PAPRBOTH) {
    static const int tr[6] = {10, 18, 36, 72, 144, 288};
    if (c.c_data) c.c_data -= tr[lg];
    if (c.n_fc) c.n_fc -= tr[lg];
    if (c.c_fc) c.c_fc -= tr[lg];
  }
  if (siso && ((gi == GI1128 && pp == PP7) || (gi == GI132 && pp == PP4) || (gi == GI116 && pp == PP2) ||
               (gi == GI19256 && pp == PP2)))
    c.n_fc = c.c_fc = 0;
  return true;
}

// Frequency-interleaver address generator (EN 302 755 9.4.1; framemapper:357-424, 916-960):
// yields the permuted addresses H(q) in generation order; callers keep those below a limit.
void fi_addresses(int N, bool odd, std::vector<int> &out) {
  int nr = 0;
  for (int t = N; t > 1; t >>= 1) nr++;               // log2 N
  int deg = nr - 1;
  static const uint8_t *perm_even[6] = {T2_FI_BITPERM1KEVEN, T2_FI_BITPERM2KEVEN, T2_FI_BITPERM4KEVEN,
                                        T2_FI_BITPERM8KEVEN, T2_FI_BITPERM16KEVEN, T2_FI_BITPERM32K};
  static const uint8_t *perm_odd[6] = {T2_FI_BITPERM1KODD, T2_FI_BITPERM2KODD, T2_FI_BITPERM4KODD,
                                       T2_FI_BITPERM8KODD, T2_FI_BITPERM16KODD, T2_FI_BITPERM32K};
  static const uint32_t taps[6] = {(1u << 0) | (1u << 4), (1u << 0) | (1u << 3), (1u << 0) | (1u << 2),
                                   (1u << 0) | (1u << 1) | (1u << 4) | (1u << 6),
                                   (1u << 0) | (1u << 1) | (1u << 4) | (1u << 5) | (1u << 9) | (1u << 11),
                                   (1u << 0) | (1u << 1) | (1u << 2) | (1u << 12)};
  int lg = nr - 10;
  const uint8_t *bp = odd ? perm_odd[lg] : perm_even[lg];
  out.clear();
  out.reserve(N);
  uint32_t r = 0;
  for (int i = 0; i < N; i++) {
    if (i < 2) r = 0;
    else if (i == 2) r = 1;
    else {
      uint32_t fb = __builtin_popcount(r & taps[lg]) & 1;
      r = ((r & ((1u << deg) - 1)) >> 1) | (fb << (deg - 1));
    }
    int h = 0;
    for (int n = 0; n < deg; n++) h |= ((r >> n) & 1) << bp[n];
    out.push_back(h + (i & 1) * (N / 2));
  }
}

// H tables for one cell count (P2 / data / FC); 32K uses Heven = Hodd^-1 (framemapper:961-977)
void fi_tables(int N, int ncells, std::vector<int> &Heven, std::vector<int> &Hodd) {
  std::vector<int> ae, ao;
  fi_addresses(N, false, ae);
  fi_addresses(N, true, ao);
  Heven.clear();
  Hodd.clear();
  for (int v : ae) if (v < ncells) Heven.push_back(v);
  for (int v : ao) if (v < ncells) Hodd.push_back(v);
  if (N == 32768) {
    Heven.assign(Hodd.size(), 0);
    for (size_t j = 0; j < Hodd.size(); j++) Heven[Hodd[j]] = (int)j;
  }
}

// Cell-interleaver permutation (framemapper:998-1107)
void ci_permutation(int cs, std::vector<int16_t> &perm, int *degree) {
  int deg;
  uint32_t taps;
  if (cs == 32400) { deg = 15; taps = (1u << 0) | (1u << 1) | (1u << 2) | (1u << 12); }
  else if (cs == 16200 || cs == 10800) { deg = 14; taps = (1u << 0) | (1u << 1) | (1u << 4) | (1u << 5) | (1u << 9) | (1u << 11); }
  else if (cs == 8100) { deg = 13; taps = (1u << 0) | (1u << 1) | (1u << 4) | (1u << 6); }
  else if (cs == 4050 || cs == 2700) { deg = 12; taps = (1u << 0) | (1u << 2); }
  else { deg = 11; taps = (1u << 0) | (1u << 3); }
  *degree = deg;
  perm.clear();
  uint32_t r = 0;
  for (int i = 0; i < (1 << deg); i++) {
    if (i < 2) r = 0;
    else if (i == 2) r = 1;
    else {
      uint32_t fb = __builtin_popcount(r & taps) & 1;
      r = ((r & ((1u << (deg - 1)) - 1)) >> 1) | (fb << (deg - 2));
    }
    uint32_t v = r | ((uint32_t)(i & 1) << (deg - 1));
    r = v;
    if ((int)v < cs) perm.push_back((int16_t)v);
  }
}

// ---- L1 signalling (framemapper:1366-1910)
struct Bits {
  std::vector<uint8_t> b;
  void put(uint64_t v, int n) { for (int i = n - 1; i >= 0; i--) b.push_back((v >> i) & 1); }
};

uint32_t crc32_mpeg2(const std::vector<uint8_t> &bits) {
  uint32_t crc = 0xffffffffu;
  for (uint8_t x : bits) {
    uint32_t fb = ((crc >> 31) ^ x) & 1;
    crc <<= 1;
    if (fb) crc ^= 0x04C11DB7u;
  }
  return crc;
}

// BCH(168) + LDPC of a k-bit (already shortened) block into cw (16200 bits)
void l1_encode(std::vector<uint8_t> &cw, int k, int nbch, int rate_id) {
  static const Poly192 g = bch_generator(false, 168);
  // straightforward long division (clarity over speed: config time only)
  std::vector<uint8_t> rem(168, 0);
  for (int i = 0; i < k; i++) {
    uint8_t fb = rem[167] ^ cw[i];
    for (int j = 167; j > 0; j--) rem[j] = rem[j - 1] ^ (fb & g.bit(j));
    rem[0] = fb & g.bit(0);
  }
  for (int n = 0; n < 168; n++) cw[k + n] = rem[167 - n];
  const t2_ldpc_code_t *c = find_code(0, rate_id);
  int pbits = kShort - nbch;
  std::vector<uint8_t> p(pbits, 0);
  int off = c->addr_off, im = 0;
  for (int gi = 0; gi < c->nrows; gi++) {
    int cnt = T2_LDPC_ROWLEN[c->row_off + gi];
    for (int n = 0; n < 360; n++, im++)
      if (cw[im])
        for (int e = 0; e < cnt; e++) p[(T2_LDPC_ADDR[off + e] + n * c->q) % pbits] ^= 1;
    off += cnt;
  }
  for (int j = 1; j < pbits; j++) p[j] ^= p[j - 1];
  for (int j = 0; j < pbits; j++) cw[nbch + j] = p[j];
}

}  // namespace

int build_frame(const FmParams &p, FramePlan &fp, bool host_l1post) {
  const PlpParams one{p.framesize, p.rate, p.constellation, p.rotation, p.fecblocks, p.tiblocks, p.inputmode, p.inband};
  return build_frame_mplp(p, std::vector<PlpParams>{one}, fp, host_l1post);
}

// L1-post signalling bits incl. CRC-32 for nplp PLPs: KSIG_POST = 350 for one (framemapperfint_cc_impl.h:32),
// plus 89 configurable (:1577-1639) and 48 dynamic (:1672-1687) bits per further PLP
static int ksig_post(int nplp) { return 350 + (nplp - 1) * (89 + 48); }

int build_frame_mplp(const FmParams &p, const std::vector<PlpParams> &plps_in, FramePlan &fp, bool host_l1post,
                     int nss) {
  const int nplp = (int)plps_in.size();
  if (nplp < 1 || nplp > MAX_PLP) return -1;
  if (p.t2frames < 1 || p.t2frames > 255 || p.numdatasyms < 1) return -1;
  if (nss == 0) nss = 1;
  if (nss < 1 || nss > 32767) return -1;   // SUB_SLICES_PER_FRAME: 15 bits
  std::vector<PlpParams> plps = plps_in;
  for (auto &q : plps) {                   // 0 = the reference's values
    if (q.plp_type == 0) q.plp_type = 1;
    if (q.ti_frames == 0) q.ti_frames = 1;
    if (q.frame_interval == 0) q.frame_interval = 1;
  }
  fp.nplp = nplp;
  fp.nss = nss;
  fp.plp_in = plps;
  fp.plp.assign(nplp, PlpPlan());
  int N = fft_points(p.fftsize);
  Counts c;
  if (!active_counts(p.fftsize, p.carriermode, p.pilotpattern, p.paprmode, p.guardinterval, p.preamble, c))
    return -1;
  if (!c.c_data || (c.n_fc && p.numdatasyms < 2)) return -1;
  fp.N_P2 = c.n_p2; fp.C_P2 = c.c_p2; fp.C_DATA = c.c_data; fp.N_FC = c.n_fc; fp.C_FC = c.c_fc;
  fp.t2frames = p.t2frames;
  static const int eta_of[4] = {1, 2, 4, 6};
  if (p.l1constellation < 0 || p.l1constellation > 3) return -1;
  fp.eta = eta_of[p.l1constellation];
  // L1-post size (framemapper:978-987) with K_sig = the L1-post signalling bits
  const int KSIG_POST = ksig_post(nplp), KBCH12 = 7032, KBCH14 = 3072, NBCH14 = 3240;
  if (KSIG_POST > KBCH12) return -1;
  int npunc_t = (6 * (KBCH12 - KSIG_POST)) / 5;
  int npost_t = KSIG_POST + 168 + 9000 - npunc_t;
  if (fp.N_P2 == 1) fp.N_post = (int)std::ceil((float)npost_t / (2 * (float)fp.eta)) * 2 * fp.eta;
  else fp.N_post = (int)std::ceil((float)npost_t / ((float)fp.eta * (float)fp.N_P2)) * fp.eta * fp.N_P2;
  fp.N_punc = npunc_t - (fp.N_post - npost_t);
  fp.Lp = fp.N_post / fp.eta;

  // ---- per PLP: cell interleaver (framemapper:1973-1998: per-TI-block running n, skip shifts >= cs) and
  //      time interleaver geometry (:1108-1119); PLP p's cells are data cells [start, start + S)
  // the accumulated fields start afresh, so a plan built twice is the plan built once
  fp.S = 0;
  fp.S_in = 0;
  fp.ncls = 1;
  fp.unit = 1;
  for (int k = 0; k < nplp; k++) {
    const PlpParams &q = plps[k];
    PlpPlan &pl = fp.plp[k];
    pl.ci_shift.clear();
    pl.cs = cell_size_of(q.framesize == 1, q.constellation);
    if (!pl.cs || q.fecblocks < 1 || (q.framesize != 0 && q.framesize != 1)) return -1;
    // tiblocks > fecblocks is accepted like the reference (framemapper:1114-1119): the surplus TI
    // blocks are "small" ones of floor(fecblocks / tiblocks) = 0 FEC blocks, which carry no cells
    if (q.tiblocks < 0 || q.tiblocks > 255) return -1;
    // TIME_IL_TYPE 1 (EN 302 755 6.5): one TI block per interleaving frame over P_I T2 frames; FRAME_INTERVAL
    // I_JUMP with FIRST_FRAME_IDX < I_JUMP (7.2.3.1); the superframe holds whole I_JUMP P_I cycles
    if ((q.plp_type != 1 && q.plp_type != 2) || (q.ti_type != 0 && q.ti_type != 1) || q.ti_frames < 1 ||
        q.ti_frames > 255 || (q.ti_type == 0 && q.ti_frames != 1) || (q.ti_type == 1 && q.tiblocks != 1) ||
        ((int64_t)q.fecblocks * pl.cs) % q.ti_frames || q.frame_interval < 1 || q.frame_interval > 255 ||
        q.first_frame < 0 || q.first_frame >= q.frame_interval || p.t2frames % (q.ti_frames * q.frame_interval))
      return -1;
    pl.F = q.fecblocks;
    pl.P = q.ti_frames;
    pl.I = q.frame_interval;
    pl.FF = q.first_frame;
    fp.ncls = std::lcm(fp.ncls, pl.I);
    pl.S_if = pl.cs * pl.F;
    // TIME_IL_TYPE 1: the TI block's output cells, in order, split into P_I equal runs [i S, (i + 1) S), run i in
    // the i-th T2 frame the PLP appears in (EN 302 755 6.5: "one TI-block ... mapped to P_I T2-frames"; the
    // reference has TIME_IL_TYPE 0 only, so this reading is shared by the planner and the oracle: PARITY UNPINNED)
    pl.S = pl.S_if / pl.P;
    pl.type2 = q.plp_type == 2;
    pl.in_off = fp.S_in;
    fp.S_in += pl.S_if;
    fp.unit = std::lcm(fp.unit, pl.cycle());
    int deg;
    ci_permutation(pl.cs, pl.ci_perm, &deg);
    int small_fec, big_fec, n_big, n_small;
    if (q.tiblocks == 0) { small_fec = big_fec = 1; n_big = 0; n_small = q.fecblocks; }
    else {
      small_fec = (int)std::floor((float)q.fecblocks / (float)q.tiblocks);
      big_fec = (int)std::ceil((float)q.fecblocks / (float)q.tiblocks);
      n_big = q.fecblocks % q.tiblocks;
      n_small = q.tiblocks - n_big;
    }
    pl.ti_on = q.tiblocks != 0;
    pl.ti_small = small_fec;
    pl.ti_big = big_fec;
    pl.ti_nsmall = n_small;
    for (int sb = 0; sb < n_small + n_big; sb++) {
      const int nb = sb < n_small ? small_fec : big_fec;
      unsigned n = 0;
      for (int r = 0; r < nb; r++) {
        int shift;
        do {
          unsigned rev = 0;
          for (int b = 0; b < deg; b++) rev |= ((n >> b) & 1u) << (deg - 1 - b);
          shift = (int)(rev << 1);
          n++;
        } while (shift >= pl.cs);
        pl.ci_shift.push_back(shift);
      }
    }
  }
  // 8.3.6.3 per frame class: the present Type-1 PLPs back to back in PLP_ID order, then the present Type-2
  // PLPs' sub-slices
  int ntype2 = 0;
  for (int k = 0; k < nplp; k++) {
    PlpPlan &pl = fp.plp[k];
    if (!pl.type2) continue;
    ntype2++;
    if (pl.S % nss) return -1;
    pl.ss = pl.S / nss;
  }
  if (!ntype2 && nss != 1) return -1;
  fp.cls.assign(fp.ncls, FrameClass());
  fp.S = 0;
  for (int c = 0; c < fp.ncls; c++) {
    FrameClass &fc = fp.cls[c];
    fc.present.assign(nplp, 0);
    fc.start.assign(nplp, 0);
    fc.ss_off.assign(nplp, 0);
    for (int k = 0; k < nplp; k++) fc.present[k] = c % fp.plp[k].I == fp.plp[k].FF;
    for (int k = 0; k < nplp; k++)
      if (fc.present[k] && !fp.plp[k].type2) {
        fc.start[k] = fc.S;
        fc.S += fp.plp[k].S;
      }
    bool any2 = false;
    for (int k = 0; k < nplp; k++) any2 = any2 || (fc.present[k] && fp.plp[k].type2);
    fc.t2start = any2 ? fc.S : 0;
    for (int k = 0; k < nplp; k++) {
      if (!fc.present[k] || !fp.plp[k].type2) continue;
      fc.ss_off[k] = fc.ssi;
      fc.start[k] = fc.S + fc.ssi;   // PLP_START: its first sub-slice
      fc.ssi += fp.plp[k].ss;
    }
    fc.S += fc.ssi * nss;
    fp.S = std::max(fp.S, fc.S);
  }
  {
    const FrameClass &c0 = fp.cls[0];
    fp.ssi = c0.ssi;
    fp.t2start = c0.t2start;
    for (int k = 0; k < nplp; k++) {
      fp.plp[k].start = c0.start[k];
      fp.plp[k].ss_off = c0.ss_off[k];
    }
  }
  {
    const PlpPlan &p0 = fp.plp[0];
    fp.cs = p0.cs; fp.F = p0.F; fp.ci_perm = p0.ci_perm; fp.ci_shift = p0.ci_shift;
    fp.ti_on = p0.ti_on; fp.ti_small = p0.ti_small; fp.ti_big = p0.ti_big; fp.ti_nsmall = p0.ti_nsmall;
  }
  fp.num_data_symbols = fp.N_FC ? p.numdatasyms - 1 : p.numdatasyms;
  fp.M = fp.N_P2 * fp.C_P2 + fp.num_data_symbols * fp.C_DATA + fp.N_FC;
  const int fixed0 = 1840 + fp.Lp + (fp.N_FC - fp.C_FC);
  if (fp.M < fp.S + fixed0) return -1;   // reference: "too many FEC blocks in T2 frame"
  fp.D = 0;
  for (auto &fc : fp.cls) {
    fc.D = fp.M - fixed0 - fc.S;
    fp.D = std::max(fp.D, fc.D);
  }
  // data cell of a T2 frame of phase ph (global frame mod unit) -> framemapper input index: the inverse time
  // interleave (framemapper:1999-2028) and cell interleave of its PLP, whose current interleaving frame (S_if
  // cells) is at in_off of the input
  std::vector<std::vector<int>> data_in(fp.unit);
  for (int ph = 0; ph < fp.unit; ph++) data_in[ph].assign(fp.cls[ph % fp.ncls].S, 0);
  for (int k = 0; k < nplp; k++) {
    const PlpPlan &pl = fp.plp[k];
    std::vector<int> perm_inv(pl.cs);
    for (int w = 0; w < pl.cs; w++) perm_inv[pl.ci_perm[w]] = w;
    for (int r = 0; r < pl.F; r++)
      for (int t = 0; t < pl.cs; t++) {
        const int w = perm_inv[((t - pl.ci_shift[r]) % pl.cs + pl.cs) % pl.cs];
        for (int f0 = 0; f0 < fp.unit; f0 += pl.cycle()) {   // the unit's interleaving frames of the PLP
          const CellDest cd = cell_dest(fp, k, r, t, f0);
          data_in[f0 + cd.off][cd.pos] = pl.in_off + r * pl.cs + w;
        }
      }
  }

  // ---- frame vector [L1pre | L1post | data | dummy | zeros] and the P2 zig-zag
  //      (framemapper:2029-2103): frame_out index -> frame-vector index
  const int Lp = fp.Lp, M = fp.M;
  std::vector<int> zz(M);
  if (fp.N_P2 == 1) {
    for (int f = 0; f < M; f++) zz[f] = f;
  } else {
    int NP = fp.N_P2, CP = fp.C_P2, pre = 1840 / NP, post = Lp / NP, dpart = CP - pre - post;
    int idx = 0;
    for (int n = 0; n < NP; n++) {
      for (int j = 0; j < pre; j++) zz[n * CP + j] = n + j * NP;
      for (int j = 0; j < post; j++) zz[n * CP + pre + j] = 1840 + n + j * NP;
      for (int j = 0; j < dpart; j++) zz[n * CP + pre + post + j] = 1840 + Lp + n * dpart + j;
      idx = (n + 1) * CP;
    }
    for (int f = idx, v = 1840 + Lp + NP * dpart; f < M; f++, v++) zz[f] = v;
  }
  // ---- frequency interleaver (framemapper:2104-2142), symbol parity restarts per frame
  std::vector<int> He, Ho, HeP, HoP, HeF, HoF;
  fi_tables(N, fp.C_DATA, He, Ho);
  fi_tables(N, fp.C_P2, HeP, HoP);
  if (fp.N_FC) fi_tables(N, fp.N_FC, HeF, HoF);
  if ((int)He.size() != fp.C_DATA || (int)HeP.size() != fp.C_P2) return -1;
  fp.gather_in.assign((size_t)fp.unit * M, 0);
  for (auto &fc : fp.cls) fc.gather_d.assign(M, 0);
  const int aux_dummy = AUX_L1PRE + 1840 + Lp;
  auto resolve = [&](int o, int f) {
    const int v = zz[f];
    for (int c = 0; c < fp.ncls; c++) {
      const FrameClass &fc = fp.cls[c];
      int code_d;
      if (v < 1840) code_d = -(AUX_L1PRE + v) - 1;
      else if (v < 1840 + Lp) code_d = -(AUX_L1PRE + v) - 1;
      else if (v < 1840 + Lp + fc.S) code_d = v - 1840 - Lp;
      else if (v < 1840 + Lp + fc.S + fc.D) code_d = -(aux_dummy + (v - 1840 - Lp - fc.S)) - 1;
      else code_d = -AUX_ZERO - 1;
      fp.cls[c].gather_d[o] = code_d;
      for (int ph = c; ph < fp.unit; ph += fp.ncls)
        fp.gather_in[(size_t)ph * M + o] = code_d >= 0 ? data_in[ph][code_d] : code_d;
    }
  };
  int o = 0, base = 0, symbol = 0;
  for (int j = 0; j < fp.N_P2; j++, symbol++, base += fp.C_P2) {
    const std::vector<int> &H = symbol % 2 ? HoP : HeP;
    for (int k = 0; k < fp.C_P2; k++) resolve(o++, base + H[k]);
  }
  for (int j = 0; j < fp.num_data_symbols; j++, symbol++, base += fp.C_DATA) {
    const std::vector<int> &H = symbol % 2 ? Ho : He;
    for (int k = 0; k < fp.C_DATA; k++) resolve(o++, base + H[k]);
  }
  if (fp.N_FC) {
    const std::vector<int> &H = symbol % 2 ? HoF : HeF;
    for (int k = 0; k < fp.N_FC; k++) resolve(o++, base + H[k]);
  }
  fp.gather_d = fp.cls[0].gather_d;

  // ---- L1 signalling cells
  bool v131 = p.version == 2, resv = p.reservedbiasbits && v131;
  fp.aux_len = AUX_L1PRE + 1840 + Lp + fp.D;
  fp.aux_variants = host_l1post ? fp.t2frames : 1;
  fp.aux.assign((size_t)fp.aux_variants * fp.aux_len, cf32{0.f, 0.f});
  // L1-pre (framemapper:1366-1534): BPSK, shortened/punctured LDPC(16200) 1/4
  std::vector<cf32> pre(1840);
  {
    Bits b;
    b.put(0, 8); b.put(p.carriermode, 1); b.put(p.preamble, 3); b.put(p.fftsize & 7, 3); b.put(0, 1);
    b.put(0, 1); b.put(p.guardinterval, 3); b.put(p.paprmode, 4); b.put(p.l1constellation, 4);
    b.put(0, 2); b.put(0, 2); b.put(fp.N_post / fp.eta, 18); b.put(KSIG_POST - 32, 18);
    b.put(p.pilotpattern, 4); b.put(0, 8); b.put(0, 16); b.put(0x3085, 16); b.put(0x8001, 16);
    b.put(p.t2frames, 8); b.put(p.numdatasyms, 12); b.put(0, 3); b.put(0, 1); b.put(1, 3); b.put(0, 3);
    b.put(p.version, 4); b.put(v131 ? p.l1scrambled : 0, 1); b.put(0, 1); b.put(resv ? 0xf : 0, 4);
    b.put(crc32_mpeg2(b.b), 32);
    std::vector<uint8_t> cw(kShort, 0);
    std::copy(b.b.begin(), b.b.end(), cw.begin());
    l1_encode(cw, KBCH14, NBCH14, 100);
    std::vector<uint8_t> punct(kShort - NBCH14, 0);
    for (int cgrp = 0; cgrp < 32; cgrp++) {
      int cnt = cgrp < 31 ? 360 : 328;
      for (int c2 = 0; c2 < cnt; c2++) punct[c2 * 36 + T2_L1_PRE_PUNCTURE[cgrp]] = 1;
    }
    int k = 0;
    auto bpsk = [](uint8_t x) { return cf32{x ? -1.0f : 1.0f, 0.0f}; };
    for (int w = 0; w < 200; w++) pre[k++] = bpsk(cw[w]);
    for (int w = 0; w < 168; w++) pre[k++] = bpsk(cw[KBCH14 + w]);
    for (int w = 0; w < kShort - NBCH14; w++)
      if (!punct[w]) pre[k++] = bpsk(cw[NBCH14 + w]);
    if (k != 1840) return -1;
  }
  // L1-post (framemapper:1536-1910): the per-frame GPU plan; with host_l1post also every FRAME_IDX
  // variant encoded here (the CPU tests' cross-check of the plan and of the oracle)
  std::vector<uint8_t> dummybits(fp.D > 0 ? fp.D : 1);
  prbs15(dummybits.data(), (int)dummybits.size());
  for (int v = 0; v < fp.aux_variants; v++) {
    cf32 *row = &fp.aux[(size_t)v * fp.aux_len];
    std::copy(pre.begin(), pre.end(), row + AUX_L1PRE);
    for (int i = 0; i < fp.D; i++) row[aux_dummy + i] = cf32{dummybits[i] ? -1.0f : 1.0f, 0.0f};
  }
  if (build_l1post_plan(p, fp)) return -1;
  if (host_l1post)
    for (int v = 0; v < fp.t2frames; v++)
      if (l1post_host(p, fp, v, &fp.aux[(size_t)v * fp.aux_len + AUX_L1PRE + 1840])) return -1;
  return 0;
}

// L1-post signalling bits before the CRC-32 (framemapper:1553-1691, no auxiliary streams), the
// configurable (:1577-1639) and dynamic (:1672-1687) PLP loops over the frame's PLPs (the reference's
// one PLP: PLP_ID 0, PLP_START 0): FRAME_IDX (8 bits at *fidx_pos) = frame_idx
std::vector<uint8_t> l1post_signal(const FmParams &p, const FramePlan &fp, int frame_idx, int *fidx_pos) {
  const bool v131 = p.version == 2, resv = p.reservedbiasbits && v131;
  const FrameClass &fc = fp.cls[frame_idx % fp.ncls];
  Bits b;
  b.put((uint64_t)fp.nss, 15); b.put((uint64_t)fp.nplp, 8); b.put(0, 4); b.put(0, 8); b.put(0, 3); b.put(729833333u, 32);
  for (int k = 0; k < fp.nplp; k++) {
    const PlpParams &q = fp.plp_in[k];
    // PLP_ID, PLP_TYPE (001 Type 1, 010 Type 2), PLP_PAYLOAD_TYPE TS, FF_FLAG, FIRST_RF_IDX,
    // FIRST_FRAME_IDX 0, PLP_GROUP_ID 1
    b.put((uint64_t)k, 8); b.put((uint64_t)q.plp_type, 3); b.put(3, 5); b.put(0, 1); b.put(0, 3);
    b.put((uint64_t)q.first_frame, 8); b.put(1, 8);
    // PLP_COD, PLP_MOD, PLP_ROTATION, PLP_FEC_TYPE, PLP_NUM_BLOCKS_MAX, FRAME_INTERVAL, TIME_IL_LENGTH
    // (N_TI for TIME_IL_TYPE 0, P_I for 1), TIME_IL_TYPE, IN_BAND_A_FLAG
    b.put(q.rate, 3); b.put(q.constellation, 3); b.put(q.rotation, 1); b.put(q.framesize, 2);
    b.put(q.fecblocks, 10); b.put((uint64_t)q.frame_interval, 8);
    b.put((uint64_t)(q.ti_type ? q.ti_frames : q.tiblocks), 8);
    b.put((uint64_t)q.ti_type, 1); b.put(0, 1);
    b.put((q.inband && v131) ? 1 : 0, 1); b.put(resv ? 0x7ff : 0, 11);
    b.put(p.version == 0 ? 0 : q.inputmode + 1, 2); b.put(0, 1); b.put(0, 1);
  }
  b.put(0, 2); b.put(resv ? 0x3fffffff : 0, 30);
  if (fidx_pos) *fidx_pos = (int)b.b.size();
  // FRAME_IDX, SUB_SLICE_INTERVAL, TYPE_2_START (both 0 without Type-2 PLPs), L1_CHANGE_COUNTER
  b.put((uint64_t)frame_idx, 8); b.put((uint64_t)fc.ssi, 22); b.put((uint64_t)fc.t2start, 22); b.put(0, 8);
  b.put(0, 3); b.put(resv ? 0xff : 0, 8);
  for (int k = 0; k < fp.nplp; k++) {
    // PLP_ID, PLP_START, PLP_NUM_BLOCKS (EN 302 755 7.2.3.2, L1-post dynamic); both 0 for a PLP absent from this
    // T2 frame (FRAME_INTERVAL > 1: it carries no cells here).  The reference signals one PLP in every frame, so
    // this value is the planner's and the oracle's shared reading: PARITY UNPINNED
    // (tests/test_cpu_ti_kat.py KAT_B holds the hand-derived bit strings)
    b.put((uint64_t)k, 8); b.put(fc.present[k] ? (uint64_t)fc.start[k] : 0, 22);
    b.put(fc.present[k] ? (uint64_t)fp.plp[k].F : 0, 10);
    b.put(resv ? 0xff : 0, 8);
  }
  b.put(resv ? 0xff : 0, 8);
  return b.b;
}

namespace {
const int KBCH12 = 7032, NBCH12 = 7200;

// shortening (framemapper:2190-2214): which of the 7032 information positions stay zero
std::vector<uint8_t> l1post_shortened(const FmParams &p, int nsig) {
  const uint8_t *pad = p.l1constellation == 2 ? T2_L1_POST_PADDING_16QAM
                     : p.l1constellation == 3 ? T2_L1_POST_PADDING_64QAM : T2_L1_POST_PADDING_BQPSK;
  std::vector<uint8_t> shortened(KBCH12, 0);
  int m, last;
  if (nsig <= 360) { m = 19; last = 360 - nsig; }
  else { m = (KBCH12 - nsig) / 360; last = KBCH12 - nsig - 360 * m; }
  for (int n = 0; n < m; n++) {
    int len = pad[n] == 19 ? 192 : 360;
    for (int w = 0; w < len; w++) shortened[pad[n] * 360 + w] = 1;
  }
  int gl = pad[m] == 19 ? 192 : 360;
  for (int w = 0; w < last; w++) shortened[pad[m] * 360 + gl - last + w] = 1;
  return shortened;
}

// puncturing (framemapper:2215-2233): which LDPC parity bits are not transmitted
std::vector<uint8_t> l1post_punctured(const FmParams &p, const FramePlan &fp) {
  const uint8_t *pun = p.l1constellation == 2 ? T2_L1_POST_PUNCTURE_16QAM
                     : p.l1constellation == 3 ? T2_L1_POST_PUNCTURE_64QAM : T2_L1_POST_PUNCTURE_BQPSK;
  std::vector<uint8_t> punct(kShort - NBCH12, 0);
  for (int cg = 0; cg <= fp.N_punc / 360; cg++) {
    int cnt = cg < fp.N_punc / 360 ? 360 : fp.N_punc % 360;
    for (int c2 = 0; c2 < cnt; c2++) punct[c2 * 25 + pun[cg]] = 1;
  }
  return punct;
}
}  // namespace

int build_l1post_plan(const FmParams &p, FramePlan &fp) {
  L1PostPlan &l = fp.l1;
  l = L1PostPlan();
  const bool v131 = p.version == 2;
  std::vector<uint8_t> sig = l1post_signal(p, fp, 0, &l.fidx_pos);
  const int L = (int)sig.size();           // CRC-covered bits
  l.nsig = L + 32;
  if (l.nsig > L1_MAX_SIG || l.nsig != ksig_post(fp.nplp) || l.fidx_pos + 8 > L) return -1;
  const int nw = (l.nsig + 31) / 32;
  // one template per frame class (FRAME_IDX c is a frame of class c; its FRAME_IDX bits are cleared)
  l.ncls = fp.ncls;
  l.tmpl.assign((size_t)nw * fp.ncls, 0);
  for (int c = 0; c < fp.ncls; c++) {
    int fpos = 0;
    std::vector<uint8_t> sc = l1post_signal(p, fp, c, &fpos);
    if ((int)sc.size() != L || fpos != l.fidx_pos) return -1;
    for (int k = 0; k < 8; k++) sc[fpos + k] = 0;
    for (int i = 0; i < L; i++)
      if (sc[i]) l.tmpl[(size_t)c * nw + (i >> 5)] |= 1u << (31 - (i & 31));
  }
  // CRC-32/MPEG-2 (register init all ones, no final XOR) is affine in the message: crc(m) = crc(0^L)
  // ^ XOR of c_i over the set bits, c_i = the register after a lone 1 at position i
  l.crc_k = crc32_mpeg2(std::vector<uint8_t>((size_t)L, 0));
  l.crc_c.assign(L, 0);
  uint32_t c = 0x04C11DB7u;                 // a 1 in the last message bit
  for (int i = L - 1; i >= 0; i--) {
    l.crc_c[i] = c;
    c = (c << 1) ^ ((c >> 31) ? 0x04C11DB7u : 0u);
  }
  if (v131 && p.l1scrambled) {
    std::vector<uint8_t> r(KBCH12);
    prbs15(r.data(), KBCH12);
    l.scr.assign(nw, 0);
    for (int i = 0; i < l.nsig; i++)
      if (r[i]) l.scr[i >> 5] |= 1u << (31 - (i & 31));
  }
  const std::vector<uint8_t> shortened = l1post_shortened(p, l.nsig);
  for (int n = 0; n < KBCH12; n++)
    if (!shortened[n]) l.sig_pos.push_back((uint16_t)n);
  if ((int)l.sig_pos.size() != l.nsig) return -1;
  // BCH(168): the parity of a lone 1 at information position q is x^(168 + 7031 - q) mod g(x)
  static const Poly192 g = bch_generator(false, 168);
  Poly192 v;
  v.w[0] = 1;
  for (int i = 0; i < 168; i++) v = times_x(v, g, 168);
  std::vector<Poly192> rem(KBCH12);
  for (int q = KBCH12 - 1; q >= 0; q--) {
    rem[q] = v;
    v = times_x(v, g, 168);
  }
  l.bch_r.assign((size_t)l.nsig * 6, 0);
  for (int i = 0; i < l.nsig; i++) {
    const Poly192 &r = rem[l.sig_pos[i]];
    for (int n = 0; n < 168; n++)
      if (r.bit(167 - n)) l.bch_r[(size_t)i * 6 + (n >> 5)] |= 1u << (31 - (n & 31));
  }
  // LDPC 1/2 short (the L1-post code, framemapper:1314-1364)
  const t2_ldpc_code_t *code = find_code(0, 101);
  if (!code || code->nrows * 360 != NBCH12) return -1;
  l.q = code->q;
  l.pbits = kShort - NBCH12;
  int off = code->addr_off;
  l.ldpc_ptr.assign(code->nrows + 1, 0);
  for (int gi = 0; gi < code->nrows; gi++) {
    l.ldpc_ptr[gi] = (uint16_t)l.ldpc_addr.size();
    const int cnt = T2_LDPC_ROWLEN[code->row_off + gi];
    for (int e = 0; e < cnt; e++) l.ldpc_addr.push_back((uint16_t)T2_LDPC_ADDR[off + e]);
    off += cnt;
  }
  l.ldpc_ptr[code->nrows] = (uint16_t)l.ldpc_addr.size();
  // transmitted bits: unshortened information, BCH parity, unpunctured LDPC parity
  const std::vector<uint8_t> punct = l1post_punctured(p, fp);
  for (int i = 0; i < l.nsig; i++) l.sel.push_back(l.sig_pos[i]);
  for (int n = 0; n < 168; n++) l.sel.push_back((uint16_t)(KBCH12 + n));
  for (int w = 0; w < l.pbits; w++)
    if (!punct[w]) l.sel.push_back((uint16_t)(NBCH12 + w));
  l.npost = (int)l.sel.size();
  if (l.npost != fp.N_post) return -1;
  l.lp = fp.Lp;
  l.mode = p.l1constellation;
  static const int l1c[4] = {0, QPSK, QAM16, QAM64};
  int qmod = 0;
  if (l.mode > 0) qam_table(l1c[l.mode], 0, l.lut, &qmod);
  if (l.mode >= 2) {
    l.ncols = l.mode == 2 ? 8 : 12;
    l.rows = fp.N_post / l.ncols;
    const uint8_t *mux = l.mode == 2 ? T2_L1_MUX16 : T2_L1_MUX64;
    for (int e = 0; e < l.ncols; e++) l.mux[e] = mux[e];
  }
  return 0;
}

// Host encoder of one FRAME_IDX variant's L1-post cells (tests only): the reference's order of
// operations, one bit at a time (framemapper:1536-1910)
int l1post_host(const FmParams &p, const FramePlan &fp, int frame_idx, cf32 *dst) {
  const bool v131 = p.version == 2;
  std::vector<uint8_t> bits = l1post_signal(p, fp, frame_idx, nullptr);
  const uint32_t crc = crc32_mpeg2(bits);
  for (int i = 31; i >= 0; i--) bits.push_back((crc >> i) & 1);
  const int nsig = (int)bits.size();
  if (v131 && p.l1scrambled) {
    std::vector<uint8_t> l1rand(KBCH12);
    prbs15(l1rand.data(), KBCH12);
    for (int i = 0; i < nsig; i++) bits[i] ^= l1rand[i];
  }
  const std::vector<uint8_t> shortened = l1post_shortened(p, nsig);
  std::vector<uint8_t> cw(kShort, 0);
  for (int n = 0, i = 0; n < KBCH12; n++) cw[n] = shortened[n] ? 0 : bits[i++];
  l1_encode(cw, KBCH12, NBCH12, 101);
  const std::vector<uint8_t> punct = l1post_punctured(p, fp);
  std::vector<uint8_t> post;
  for (int w = 0; w < KBCH12; w++) if (!shortened[w]) post.push_back(cw[w]);
  for (int w = 0; w < 168; w++) post.push_back(cw[KBCH12 + w]);
  for (int w = 0; w < kShort - NBCH12; w++) if (!punct[w]) post.push_back(cw[NBCH12 + w]);
  if ((int)post.size() != fp.N_post) return -1;
  cf32 l1lut[64];
  int qmod;
  static const int l1c[4] = {0, QPSK, QAM16, QAM64};
  if (p.l1constellation > 0) qam_table(l1c[p.l1constellation], 0, l1lut, &qmod);
  int produced = 0;
  if (p.l1constellation == 0) {
    for (int d = 0; d < fp.N_post; d++) dst[produced++] = cf32{post[d] ? -1.0f : 1.0f, 0.0f};
  } else if (p.l1constellation == 1) {
    for (int d = 0; d < fp.N_post / 2; d++) dst[produced++] = l1lut[(post[2 * d] << 1) | post[2 * d + 1]];
  } else {
    // column-row bit interleaver then demux by source index (framemapper:1832-1908)
    int ncols = p.l1constellation == 2 ? 8 : 12, rows = fp.N_post / ncols, half = ncols / 2;
    const uint8_t *mux = p.l1constellation == 2 ? T2_L1_MUX16 : T2_L1_MUX64;
    for (int k = 0; k < rows; k++) {
      int pack = 0;
      for (int e = 0; e < ncols; e++) pack = (pack << 1) | post[rows * mux[e] + k];
      dst[produced++] = l1lut[pack >> half];
      dst[produced++] = l1lut[pack & ((1 << half) - 1)];
    }
  }
  return produced == fp.Lp ? 0 : -1;
}

// ============================================================================ pilots + OFDM
namespace {
enum CarrierKind : uint8_t { K_DATA = 0, K_ZERO, K_P2, K_P2INV, K_SP, K_SPINV, K_CP, K_CPINV };

const uint16_t *reserved_tones(int N, bool tr, int *n) {
  switch (N) {
    case 1024: *n = 10; return tr ? T2_TR_PAPR_MAP_1K : T2_P2_PAPR_MAP_1K;
    case 2048: *n = 18; return tr ? T2_TR_PAPR_MAP_2K : T2_P2_PAPR_MAP_2K;
    case 4096: *n = 36; return tr ? T2_TR_PAPR_MAP_4K : T2_P2_PAPR_MAP_4K;
    case 8192: *n = 72; return tr ? T2_TR_PAPR_MAP_8K : T2_P2_PAPR_MAP_8K;
    case 16384: *n = 144; return tr ? T2_TR_PAPR_MAP_16K : T2_P2_PAPR_MAP_16K;
    default: *n = 288; return tr ? T2_TR_PAPR_MAP_32K : T2_P2_PAPR_MAP_32K;
  }
}

// complex IDFT in double (radix-2, unnormalised, e^{+j})
// the P1 symbol's 1024-point inverse DFT in double, term by term in the order of the oracle's
// restatement (oracle/dvbt2_oracle.c cdft_double: angle 2 pi ((j k) mod n) / n, sums over j), so the
// planner's P1 samples equal the oracle's bit for bit; the cosine / sine of each of the n angles are
// computed once, as the same double expression
void p1_idft(const std::vector<double> &x, cf32 *y) {
  const int n = (int)x.size();
  std::vector<double> c(n), sn(n);
  for (int m = 0; m < n; m++) {
    const double a = 1 * 2.0 * M_PI * (double)m / n;
    c[m] = std::cos(a);
    sn[m] = std::sin(a);
  }
  for (int k = 0; k < n; k++) {
    double sr = 0, si = 0;
    for (int j = 0; j < n; j++) {
      const int m = (int)((long)j * k % n);
      const double xr = x[j], xi = 0.0;
      sr += xr * c[m] - xi * sn[m];
      si += xr * sn[m] + xi * c[m];
    }
    y[k] = cf32{(float)sr, (float)si};
  }
}
}  // namespace

int build_pilot(const PgParams &p, PilotPlan &pp) {
  pp.fft = fft_points(p.fftsize);
  if (!pp.fft || p.vlength != pp.fft || p.numdatasyms < 1) return -1;
  const int N = pp.N = p.vlength;
  Counts c;
  if (!active_counts(p.fftsize, p.carriermode, p.pilotpattern, p.paprmode, p.guardinterval, p.preamble, c))
    return -1;
  if (!c.c_data) return -1;
  bool miso = !(p.preamble == 0 || p.preamble == 3);
  bool tx2 = miso && p.misogroup == 1;
  bool ext = p.carriermode == 1 && N >= 8192;
  pp.N_P2 = c.n_p2;
  // carriers (pilotgen:120-175)
  switch (N) {
    case 1024: pp.C_PS = 853; break;
    case 2048: pp.C_PS = 1705; break;
    case 4096: pp.C_PS = 3409; break;
    case 8192: pp.C_PS = ext ? 6913 : 6817; break;
    case 16384: pp.C_PS = ext ? 13921 : 13633; break;
    default: pp.C_PS = ext ? 27841 : 27265; break;
  }
  int kx = N == 8192 ? 48 : N == 16384 ? 144 : N == 32768 ? 288 : 0;   // extended-carrier count
  pp.K_EXT = ext ? kx : 0;
  pp.K_OFFSET = ext ? 0 : kx;
  const int C_PS = pp.C_PS, K_EXT = pp.K_EXT;
  static const int dxs[8] = {3, 6, 6, 12, 12, 24, 24, 6}, dys[8] = {4, 2, 4, 2, 4, 2, 4, 16};
  const int dx = dxs[p.pilotpattern], dy = dys[p.pilotpattern];
  // pilot amplitudes (pilotgen:748-992, 1083-1094): values built in double, stored float
  double a_p2 = (N == 32768 && !miso) ? std::sqrt(37.0) / 5.0 : std::sqrt(31.0) / 5.0;
  double a_cp = N <= 2048 ? 4.0 / 3.0 : N == 4096 ? (4.0 * std::sqrt(2.0)) / 3.0 : 8.0 / 3.0;
  static const double a_sp_t[8] = {4.0 / 3.0, 4.0 / 3.0, 7.0 / 4.0, 7.0 / 4.0, 7.0 / 3.0, 7.0 / 3.0, 7.0 / 3.0, 7.0 / 3.0};
  double amps[3] = {a_p2, a_sp_t[p.pilotpattern], a_cp};
  for (int t = 0; t < 3; t++) {
    float pos = (float)amps[t], neg = (float)-amps[t];
    pp.pilot_values[4 * t + 0] = cf32{pos, 0.f};   // normal, prbs^pn = 0
    pp.pilot_values[4 * t + 1] = cf32{neg, 0.f};   // normal, 1
    pp.pilot_values[4 * t + 2] = cf32{neg, 0.f};   // inverted, 0
    pp.pilot_values[4 * t + 3] = cf32{pos, 0.f};   // inverted, 1
  }
  // reference PRBS w_k (pilotgen:1245-1258) and PN sequence
  std::vector<uint8_t> prbs(27841);
  {
    unsigned s = 0x7ff;
    for (int i = 0; i < 27841; i++) {
      prbs[i] = s & 1;
      unsigned b = (s ^ (s >> 2)) & 1;
      s = (s >> 1) | (b << 10);
    }
  }
  auto pn = [](int j) { return (T2_PN_SEQ_BYTES[j >> 3] >> (7 - (j & 7))) & 1; };

  // --- carrier maps
  std::vector<uint8_t> p2(C_PS, K_DATA), fc(C_PS, K_DATA);
  auto p2kind = [&](int i) { return (tx2 && ((i / 3) % 2) && (i % 3 == 0)) ? K_P2INV : K_P2; };
  int step = (N == 32768 && !miso) ? 6 : 3;
  for (int i = 0; i < C_PS; i += step) p2[i] = tx2 ? p2kind(i) : K_P2;
  if (ext)
    for (int i = 0; i < K_EXT; i++) {
      p2[i] = tx2 ? p2kind(i) : K_P2;
      int k = i + C_PS - K_EXT;
      p2[k] = tx2 ? p2kind(k) : K_P2;
    }
  if (miso) p2[K_EXT + 1] = p2[K_EXT + 2] = p2[C_PS - K_EXT - 2] = p2[C_PS - K_EXT - 3] = K_P2;
  {
    int nres;
    const uint16_t *res = reserved_tones(N, false, &nres);
    int koff = N >= 8192 ? K_EXT : 0;
    for (int i = 0; i < nres; i++) p2[res[i] + koff] = K_ZERO;
    if (miso)
      for (int i = 0; i < nres; i++) {
        int ki = res[i] + K_EXT;
        bool up = (ki % 3) == 1 && (i == nres - 1 || ki + 1 != res[i + 1] + K_EXT);
        bool dn = (ki % 3) == 2 && (i == 0 || ki - 1 != res[i - 1] + K_EXT);
        if (up) p2[ki + 1] = K_P2;
        if (dn) p2[ki - 1] = K_P2;
      }
  }
  for (int i = 0; i < C_PS; i += dx) fc[i] = (tx2 && ((i / dx) % 2)) ? K_SPINV : K_SP;
  if ((N == 1024 && (p.pilotpattern == PP4 || p.pilotpattern == PP5)) || (N == 2048 && p.pilotpattern == PP7))
    fc[C_PS - 2] = K_SP;
  fc[0] = fc[C_PS - 1] = (tx2 && ((p.numdatasyms + pp.N_P2 - 1) % 2)) ? K_SPINV : K_SP;
  if (p.paprmode == PAPRTR || p.paprmode == PAPRBOTH) {
    int nres;
    const uint16_t *res = reserved_tones(N, false, &nres);
    int koff = N >= 8192 ? K_EXT : 0;
    for (int i = 0; i < nres; i++) fc[res[i] + koff] = K_ZERO;
  }
  // data-symbol maps, one per symbol phase (symbol mod dy) (init_pilots, pilotgen:1285-2782)
  std::vector<std::vector<uint8_t>> dmap(dy, std::vector<uint8_t>(C_PS, K_DATA));
  for (int ph = 0; ph < dy; ph++) {
    std::vector<uint8_t> &m = dmap[ph];
    for (int s = 0; s < T2_NCP_STEPS; s++) {
      const t2_cp_step_t &st = T2_CP_STEPS[s];
      if (st.fft != N || st.pp != p.pilotpattern + 1 || (st.ext_only && p.carriermode != 1)) continue;
      const uint16_t *list = T2_CP_LIST + T2_CP_LIST_SPAN[st.list][0];
      for (int i = 0; i < st.count; i++) {
        int k = st.modulus ? list[i] % st.modulus : list[i];
        m[k] = (st.miso_inv && tx2 && ((k / dx) % 2) && (k % dx) == 0) ? K_CPINV : K_CP;
      }
    }
    for (int i = 0; i < C_PS; i++) {
      int rem = ((i - K_EXT) % (dx * dy) + dx * dy) % (dx * dy);
      if (rem == dx * (ph % dy)) m[i] = (tx2 && ((i / dx) % 2)) ? K_SPINV : K_SP;
    }
    m[0] = m[C_PS - 1] = (tx2 && (ph % 2)) ? K_SPINV : K_SP;
    if (p.paprmode == PAPRTR || p.paprmode == PAPRBOTH) {
      int shift = p.carriermode == 0 ? dx * (ph % dy) : dx * ((ph + K_EXT / dx) % dy);
      int nres;
      const uint16_t *res = reserved_tones(N, true, &nres);
      for (int i = 0; i < nres; i++) m[res[i] + shift] = K_ZERO;
    }
  }
  pp.Nsym = p.numdatasyms + pp.N_P2;
  pp.active = c.n_fc ? pp.N_P2 * c.c_p2 + (p.numdatasyms - 1) * c.c_data + c.n_fc
                     : pp.N_P2 * c.c_p2 + p.numdatasyms * c.c_data;
  pp.left_nulls = (N - C_PS) / 2 + 1;
  // --- per-symbol gather maps, indexed by IFFT input position k (bin n = (k + N/2) mod N)
  pp.bin_map.assign((size_t)pp.Nsym * N, -AUX_ZERO - 1);
  int consumed = 0;
  for (int j = 0; j < pp.Nsym; j++) {
    const uint8_t *m = j < pp.N_P2 ? p2.data()
                     : (c.n_fc && j == pp.Nsym - 1) ? fc.data() : dmap[j % dy].data();
    int32_t *row = &pp.bin_map[(size_t)j * N];
    int pnj = pn(j);
    for (int cc = 0; cc < C_PS; cc++) {
      int n = pp.left_nulls + cc;
      int k = (n + N / 2) % N;
      int b = prbs[cc + pp.K_OFFSET] ^ pnj;
      int code;
      switch (m[cc]) {
        case K_DATA: code = consumed++; break;
        case K_ZERO: code = -AUX_ZERO - 1; break;
        case K_P2: code = -(AUX_PILOT0 + 0 + b) - 1; break;
        case K_P2INV: code = -(AUX_PILOT0 + 2 + b) - 1; break;
        case K_SP: code = -(AUX_PILOT0 + 4 + b) - 1; break;
        case K_SPINV: code = -(AUX_PILOT0 + 6 + b) - 1; break;
        case K_CP: code = -(AUX_PILOT0 + 8 + b) - 1; break;
        default: code = -(AUX_PILOT0 + 10 + b) - 1; break;
      }
      row[k] = code;
    }
  }
  if (consumed != pp.active) return -1;   // carrier maps must agree with C_P2/C_DATA/N_FC
  switch (p.guardinterval) {
    case GI132: pp.G = N / 32; break;
    case GI116: pp.G = N / 16; break;
    case GI18: pp.G = N / 8; break;
    case GI14: pp.G = N / 4; break;
    case GI1128: pp.G = N / 128; break;
    case GI19128: pp.G = (N * 19) / 128; break;
    case GI19256: pp.G = (N * 19) / 256; break;
    default: return -1;
  }
  pp.normalization = (float)(5.0 / std::sqrt(27.0 * C_PS));
  // --- P1 (pilotgen:1119-1178): DBPSK over 384 carriers, MSS from S1/S2, scrambled
  {
    int s1 = p.preamble, s2 = (p.fftsize & 7) << 1;
    std::vector<int> seq;
    for (int i = 0; i < 8; i++) for (int j = 7; j >= 0; j--) seq.push_back((T2_P1_S1[s1][i] >> j) & 1);
    for (int i = 0; i < 32; i++) for (int j = 7; j >= 0; j--) seq.push_back((T2_P1_S2[s2][i] >> j) & 1);
    for (int i = 0; i < 8; i++) for (int j = 7; j >= 0; j--) seq.push_back((T2_P1_S1[s1][i] >> j) & 1);
    std::vector<double> fr(1024, 0.0);
    int prev = 1;
    unsigned sr = 0x4e46;
    for (int i = 0; i < 384; i++) {
      int cur = seq[i] ? -prev : prev;
      prev = cur;
      unsigned b = (sr ^ (sr >> 1)) & 1;
      sr = (sr >> 1) | (b << 14);
      fr[T2_P1_CARRIERS[i] + 86] = cur * (b ? -1.0 : 1.0);
    }
    pp.p1.assign(2048, cf32{0.f, 0.f});
    float inv = (float)std::sqrt(384.0);
    std::vector<cf32> t0(1024), t1(1024);
    for (int pass = 0; pass < 2; pass++) {
      std::vector<double> re(1024);
      for (int i = 0; i < 1024; i++) {
        int src = (i + 512) % 1024;                    // fftshift
        re[i] = pass == 0 ? fr[src] : fr[(src + 1023) % 1024];   // 1-bin shifted copy
      }
      std::vector<cf32> &t = pass == 0 ? t0 : t1;
      p1_idft(re, t.data());
      for (int i = 0; i < 1024; i++) t[i] = cf32{t[i].re / inv, t[i].im / inv};
    }
    int k = 0;
    for (int j = 0; j < 542; j++) pp.p1[k++] = t1[j];
    for (int j = 0; j < 1024; j++) pp.p1[k++] = t0[j];
    for (int j = 542; j < 1024; j++) pp.p1[k++] = t1[j];
  }
  // --- inverse-sinc equaliser (pilotgen:1179-1219)
  pp.eq = p.equalization ? 1 : 0;
  if (pp.eq) {
    static const double fss[6] = {131.0 * 1000000.0 / 71.0, 5.0 * 8000000.0 / 7.0, 6.0 * 8000000.0 / 7.0,
                                  7.0 * 8000000.0 / 7.0, 8.0 * 8000000.0 / 7.0, 10.0 * 8000000.0 / 7.0};
    double fs = (p.bandwidth >= 0 && p.bandwidth < 6) ? fss[p.bandwidth] : 1.0;
    double fstep = fs / N, f = 0.0, rms = 0.0;
    pp.isinc.assign(N, 0.f);
    for (int i = 0; i < N / 2; i++) {
      double x = M_PI * f / fs, sinc = i == 0 ? 1.0 : std::sin(x) / x;
      rms += sinc * sinc;
      pp.isinc[i + N / 2] = pp.isinc[N / 2 - i - 1] = (float)(1.0 / sinc);
      f = f + fstep;
    }
    float r = (float)std::sqrt(rms / (N / 2));
    for (int i = 0; i < N; i++) pp.isinc[i] *= r;
  }
  // two-level twiddle table (kept in LDS by the OFDM kernel): w^i = hi[i >> 7] * lo[i & 127]
  pp.twiddle.resize(128 + N / 128);
  for (int e = 0; e < 128; e++) {
    double a = 2.0 * M_PI * (double)e / (double)N;
    pp.twiddle[e] = cf32{(float)std::cos(a), (float)std::sin(a)};
  }
  for (int h = 0; h < N / 128; h++) {
    double a = 2.0 * M_PI * (double)(128 * h) / (double)N;
    pp.twiddle[128 + h] = cf32{(float)std::cos(a), (float)std::sin(a)};
  }
  pp.twiddle1k.resize(1024);
  for (int m = 0; m < 1024; m++) {
    double a = 2.0 * M_PI * (double)m / 1024.0;
    pp.twiddle1k[m] = cf32{(float)std::cos(a), (float)std::sin(a)};
  }
  return 0;
}

// every symbol row of the fused chain in stored order (ofdm_stored_index)
std::vector<int32_t> ofdm_stored_rows(int N, int Nsym, const std::vector<int32_t> &bin_map) {
  if (!ofdm_split(N)) return bin_map;
  std::vector<int32_t> out(bin_map.size());
  for (int j = 0; j < Nsym; j++)
    for (int k = 0; k < N; k++) out[(size_t)j * N + ofdm_stored_index(N, k)] = bin_map[(size_t)j * N + k];
  return out;
}

int64_t ti_index(const FramePlan &fp, int plp, int r, int t) {
  const PlpPlan &pl = fp.plp[plp];
  const int cs = pl.cs;
  if (!pl.ti_on) return (int64_t)r * cs + t;
  const int ns = pl.ti_nsmall * pl.ti_small;
  int r0, nb;
  if (r < ns) { r0 = r - r % pl.ti_small; nb = pl.ti_small; }
  else { r0 = r - (r - ns) % pl.ti_big; nb = pl.ti_big; }
  const int rows = cs / 5, e = t / rows, row = t - e * rows;
  return (int64_t)r0 * cs + (int64_t)row * (5 * nb) + 5 * (r - r0) + e;
}

int32_t plp_cell_pos(const FramePlan &fp, int plp, int c, int cls) {
  const PlpPlan &pl = fp.plp[plp];
  const FrameClass &fc = fp.cls[cls];
  if (!pl.type2) return fc.start[plp] + c;
  return fc.t2start + (c / pl.ss) * fc.ssi + fc.ss_off[plp] + c % pl.ss;
}

// LDS bank pair of a stored bin as the OFDM kernels' scatter writes it (8-byte slot within its half,
// one pad slot per 2^ps: t2_kernels.h ofdm_padded_bin)
static int scatter_bank(int N, int stored) {
  const int nsub = ofdm_split(N) ? N / 2 : N, ps = ofdm_split(N) ? 5 : 4, k = stored % nsub;
  return (k + (k >> ps)) & 15;
}

// Conflict-free scatter groups.  The OFDM kernels stream a run of scatter entries in units of U (8
// data slots per lane per round for 32K, 4 for N <= 16K and for the aux quads); unit x (counted from
// the run start rounded down to U, o0) goes to lane x mod 64, and element e of every lane's unit is
// written by one ds_write_b64, whose 16-lane groups {16 g .. 16 g + 15} are bank-conflict-free when
// their bank pairs differ.  So the entries of each window of 16 units (16 U positions, from o0) at the
// same e should have distinct bank pairs.  seq holds the entries of positions [pos0, pos0 + n) in
// position order; entries may move only within their segment (seg(k) equal for consecutive k): a
// greedy first fit per position.
template <class Bank, class Seg>
static void bank_balance(std::vector<int32_t> &seq, int pos0, int U, const Bank &bank, const Seg &seg) {
  const int n = (int)seq.size(), o0 = pos0 & ~(U - 1);
  std::vector<uint16_t> used((size_t)((pos0 + n - o0) / (16 * U) + 1) * U, 0);
  // a segment's candidates bucketed by bank pair, in segment order (pos = index in the segment): each
  // pick looks at the 16 bucket heads only, O(16) instead of a scan of the remaining candidates
  std::vector<std::pair<int32_t, int32_t>> bucket[16];
  for (int k0 = 0; k0 < n;) {
    int k1 = k0 + 1;
    while (k1 < n && seg(seq[k1]) == seg(seq[k0])) k1++;
    size_t head[16] = {0};
    int left[16] = {0};   // remaining candidates per bank pair
    for (auto &bk : bucket) bk.clear();
    for (int i = k0; i < k1; i++) bucket[bank(seq[i])].push_back({i - k0, seq[i]});
    for (int b = 0; b < 16; b++) left[b] = (int)bucket[b].size();
    for (int k = k0; k < k1; k++) {
      const int p = pos0 + k, cls = ((p - o0) / (16 * U)) * U + (p - o0) % U;
      // a candidate whose bank pair is still free in this class, the most plentiful such pair first
      // (keeps the scarce ones for later positions; ties: the earliest candidate); else the earliest
      int pick = -1, best = -1, pick_pos = 1 << 30, first = -1, first_pos = 1 << 30;
      for (int b = 0; b < 16; b++) {
        if (head[b] == bucket[b].size()) continue;
        const int pos = bucket[b][head[b]].first;
        if (pos < first_pos) { first_pos = pos; first = b; }
        if (!((used[cls] >> b) & 1) && (left[b] > best || (left[b] == best && pos < pick_pos))) {
          best = left[b];
          pick = b;
          pick_pos = pos;
        }
      }
      if (pick < 0) pick = first;
      seq[k] = bucket[pick][head[pick]++].second;
      used[cls] |= (uint16_t)(1u << pick);
      left[pick]--;
    }
    k0 = k1;
  }
}

int build_chain_layout(const FramePlan &fp, const PilotPlan &pp, ChainLayout &cl, int cls) {
  if (pp.active != fp.M || pp.N > 32768 || cls < 0 || cls >= fp.ncls) return -1;
  const FrameClass &fc = fp.cls[cls];
  const int S = fc.S;
  // bins -> frame data order (TI output) via the framemapper's composed map
  std::vector<int32_t> nat(pp.bin_map.size());
  for (size_t i = 0; i < nat.size(); i++) {
    int32_t c = pp.bin_map[i];
    nat[i] = c >= 0 ? fc.gather_d[c] : c;
  }
  cl.cmap = ofdm_stored_rows(pp.N, pp.Nsym, nat);
  cl.inv.assign(S, 0);
  cl.sym_d0.assign(pp.Nsym, 0);
  cl.sym_n.assign(pp.Nsym, 0);
  std::vector<char> seen(S, 0);
  for (int j = 0; j < pp.Nsym; j++) {
    int lo = S, hi = -1, n = 0;
    for (int k = 0; k < pp.N; k++) {
      int32_t c = cl.cmap[(size_t)j * pp.N + k];
      if (c < 0) continue;
      if (c >= S || seen[c]) return -1;
      seen[c] = 1;
      cl.inv[c] = (uint16_t)k;
      lo = std::min(lo, c);
      hi = std::max(hi, c);
      n++;
    }
    if (n && hi - lo + 1 != n) return -1;   // a symbol's data slots must be one contiguous run
    cl.sym_d0[j] = n ? lo : 0;
    cl.sym_n[j] = n;
  }
  for (int s = 0; s < S; s++)
    if (!seen[s]) return -1;
  cl.sym_n0 = cl.sym_n;
  // Slot order within each symbol (32K: within each stored half): FEC-block-major, and within a
  // block's run the order bank_balance picks for the OFDM scatter's write groups.  The OFDM kernels
  // stream any order (inv follows it); block-major runs give the LDPC + map kernel, which stores one FEC
  // block per workgroup, one contiguous run per symbol (half) instead of 10-byte TI-row runs
  // scattered over the symbol (its per-cell deltas take any order inside a run).
  // (blocks numbered PLP-major: PLP k's block r is g0_k + r, so each symbol half's slots are PLP-major too)
  // (a TIME_IL_TYPE 1 PLP's blocks by the first T2 frame of the launch unit in this class that carries it: its
  // other frames' cells come from the same blocks, at the same positions when the frame boundary falls between
  // TI rows)
  std::vector<int32_t> blk_of(S), plp_of_blk;
  for (int k = 0, g0 = 0; k < fp.nplp; g0 += fp.plp[k].F, k++) {
    const PlpPlan &pl = fp.plp[k];
    int ph = cls;   // the first frame of class cls in the unit (k present there iff present in the class)
    const int off = ph % pl.cycle();
    for (int r = 0; r < pl.F; r++) {
      plp_of_blk.push_back(k);
      if (!fc.present[k]) continue;
      for (int t = 0; t < pl.cs; t++) {
        const CellDest cd = cell_dest(fp, k, r, t, ph - off);
        if (cd.off == off) blk_of[cd.pos] = g0 + r;
      }
    }
  }
  const int P = fp.nplp;
  cl.plp_bnd.assign((size_t)2 * pp.Nsym * (P + 1), 0);
  const bool split = ofdm_split(pp.N);
  const int half = pp.N / 2;
  cl.part.assign(S, 0);
  std::vector<int32_t> order;
  for (int j = 0; j < pp.Nsym; j++) {
    const int d0 = cl.sym_d0[j], n = cl.sym_n[j];
    int n0 = 0;
    if (split)
      for (int s = d0; s < d0 + n; s++) n0 += cl.inv[s] < half;
    order.resize(n);
    for (int k = 0; k < n; k++) order[k] = d0 + k;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
      const int hx = split && cl.inv[x] >= half, hy = split && cl.inv[y] >= half;
      return hx != hy ? hx < hy : blk_of[x] < blk_of[y];
    });
    // within each FEC block's run, the order the OFDM scatter's write groups want (bank_balance)
    const int nh = split ? n0 : n;
    for (int h = 0; h < (split ? 2 : 1); h++) {
      const int k0 = h ? nh : 0, k1 = h ? n : nh;
      std::vector<int32_t> seq(order.begin() + k0, order.begin() + k1);
      bank_balance(seq, d0 + k0, split ? 8 : 4, [&](int s) { return scatter_bank(pp.N, cl.inv[s]); },
                   [&](int s) { return blk_of[s]; });
      std::copy(seq.begin(), seq.end(), order.begin() + k0);
    }
    for (int k = 0; k < n; k++) cl.part[order[k]] = d0 + k;
    cl.sym_n0[j] = split ? n0 : n;
    // PLP boundaries of each group's (PLP-major) slot range
    for (int h = 0; h < 2; h++) {
      const int k0 = h ? (split ? nh : n) : 0, k1 = h ? n : nh;
      int32_t *bnd = &cl.plp_bnd[(size_t)(2 * j + h) * (P + 1)];
      for (int q = 0, k = k0; q <= P; q++) {
        while (k < k1 && plp_of_blk[blk_of[order[k]]] < q) k++;
        bnd[q] = d0 + k;
      }
      bnd[P] = d0 + k1;
      for (int k = k0; k + 1 < k1; k++)
        if (plp_of_blk[blk_of[order[k]]] > plp_of_blk[blk_of[order[k + 1]]]) return -1;
    }
  }
  std::vector<uint16_t> inv2(S);
  for (int s = 0; s < S; s++) inv2[cl.part[s]] = cl.inv[s];
  cl.inv.swap(inv2);
  for (auto &c : cl.cmap)
    if (c >= 0) c = cl.part[c];
  return 0;
}

int build_aux_lists(const ChainLayout &cl, int N, int Nsym, const std::vector<cf32> &auxv, int aux_len,
                    int t2frames, AuxLists &al, int l1_lo, int l1_len) {
  const bool split = ofdm_split(N);
  const int nsub = split ? N / 2 : N, ngrp = 2 * Nsym;
  if ((int64_t)aux_len * t2frames > (int64_t)auxv.size() || nsub > 32768) return -1;
  al.dbin.clear(); al.dval.clear(); al.ind.clear();
  al.grp.assign((size_t)4 * ngrp, 0);
  al.zrun.assign((size_t)2 * ngrp, 0);
  auto is_l1 = [&](int a) { return a >= l1_lo && a < l1_lo + l1_len; };
  auto same_in_all = [&](int a) {
    if (is_l1(a)) return false;
    for (int v = 1; v < t2frames; v++) {
      const cf32 x = auxv[a], y = auxv[(size_t)v * aux_len + a];
      if (std::memcmp(&x, &y, sizeof(cf32))) return false;
    }
    return true;
  };
  for (int g = 0; g < ngrp; g++) {
    const int j = g >> 1, h = g & 1;
    al.grp[4 * g + 0] = (int32_t)al.dbin.size();
    al.grp[4 * g + 2] = (int32_t)al.ind.size();
    if (h && !split) continue;
    const int32_t *row = &cl.cmap[(size_t)j * N + (size_t)h * nsub];
    // zero bins: AUX_ZERO, or an aux cell that is +0 in every variant
    auto is_zero = [&](int k) {
      const int32_t c = row[k];
      if (c >= 0) return false;
      if (c == -AUX_ZERO - 1) return true;
      const int a = -c - 1;
      if (a >= aux_len || !same_in_all(a)) return false;
      uint64_t bits;
      std::memcpy(&bits, &auxv[a], sizeof(bits));
      return bits == 0;
    };
    int z0 = 0, z1 = 0;
    for (int k = 0; k < nsub;) {   // longest run of zero bins
      if (!is_zero(k)) { k++; continue; }
      int e = k;
      while (e < nsub && is_zero(e)) e++;
      if (e - k > z1 - z0) { z0 = k; z1 = e; }
      k = e;
    }
    al.zrun[2 * g + 0] = z0;
    al.zrun[2 * g + 1] = z1;
    for (int k = 0; k < nsub; k++) {
      const int32_t c = row[k];
      if (c >= 0) continue;
      if (k >= z0 && k < z1) continue;   // zeroed as a range by the kernel
      if (is_zero(k)) {                  // an isolated zero bin: direct entry of value 0
        al.dbin.push_back((uint16_t)k);
        al.dval.push_back(cf32{0.f, 0.f});
        continue;
      }
      const int a = -c - 1;
      if (a >= aux_len) return -1;
      if (same_in_all(a)) {
        const cf32 v = auxv[a];
        al.dbin.push_back((uint16_t)k);
        al.dval.push_back(v);
      } else {
        // per-frame cells: L1-post cell a - l1_lo of the frame (code a - l1_lo + 1), or (no L1
        // range) aux index a of the frame's t2_frame_num variant (code a + 1)
        const int code = is_l1(a) ? a - l1_lo + 1 : a + 1;
        if (code >= (1 << 17)) return -1;
        al.ind.push_back((uint32_t)k | ((uint32_t)code << 15));
      }
    }
    {   // the group's direct entries in the order the kernel's quad write groups want (bank_balance)
      const int e0 = al.grp[4 * g + 0], ne = (int)al.dbin.size() - e0;
      std::vector<int32_t> seq(ne);
      for (int i = 0; i < ne; i++) seq[i] = e0 + i;
      const int ps = split ? 5 : 4;
      bank_balance(seq, 0, 4, [&](int i) { const int k = al.dbin[i]; return (k + (k >> ps)) & 15; },
                   [](int) { return 0; });
      std::vector<uint16_t> b2(ne);
      std::vector<cf32> v2(ne);
      for (int i = 0; i < ne; i++) {
        b2[i] = al.dbin[seq[i]];
        v2[i] = al.dval[seq[i]];
      }
      std::copy(b2.begin(), b2.end(), al.dbin.begin() + e0);
      std::copy(v2.begin(), v2.end(), al.dval.begin() + e0);
    }
    while (al.dbin.size() & 3) {   // pad to a quad: bin 0xFFFF goes to the kernel's dummy slot
      al.dbin.push_back(0xFFFF);
      al.dval.push_back(cf32{0.f, 0.f});
    }
    al.grp[4 * g + 1] = (int32_t)al.dbin.size() - al.grp[4 * g + 0];
    al.grp[4 * g + 3] = (int32_t)al.ind.size() - al.grp[4 * g + 2];
  }
  return 0;
}

}  // namespace t2

namespace t2 {
// N_P2, C_P2, C_DATA, N_FC, C_FC of a configuration (the framemapper's cell-count tables), for the
// CPU tests that cross-check them against the pilot maps symbol by symbol
int frame_cell_counts(int fftsize, int carriermode, int pp, int papr, int gi, int preamble, int out[5]) {
  Counts c;
  if (!active_counts(fftsize, carriermode, pp, papr, gi, preamble, c)) return -1;
  out[0] = c.n_p2; out[1] = c.c_p2; out[2] = c.c_data; out[3] = c.n_fc; out[4] = c.c_fc;
  return 0;
}
}  // namespace t2
