// t2_plan_probe.cpp -- host-only export of the configuration planner (t2_plan.cpp) for the
// CPU test suite: lets tests apply the product's composed gather maps with numpy and compare
// them with the oracle for every parameter combination without a GPU.  Not part of the
// GPU product library (libdvbt2ll_hip.so); built as gr-dvbt2ll_amd/csrc/_obj/libt2plan_probe.so.
#include <cstring>

#include "t2_plan.h"

using namespace t2;

// multi-PLP parameters as laid out by include/dvbt2ll_hip.h dvbt2ll_mplp_params (ints): 12 common fields
// {carriermode, fftsize, guardinterval, l1constellation, pilotpattern, t2frames, numdatasyms, paprmode,
// version, preamble, reservedbiasbits, l1scrambled}, nplp, then MAX_PLP x 12 per-PLP fields {framesize,
// rate, constellation, rotation, fecblocks, tiblocks, inputmode, inband, tsrate, plp_type, ti_type,
// ti_frames, frame_interval, first_frame_idx}, then num_subslices
constexpr int PLP_INTS = 14;
static bool parse_mplp(const int *a, FmParams &f, std::vector<PlpParams> &plps, int *nss) {
  const int n = a[12];
  if (n < 1 || n > MAX_PLP) return false;
  const int *q0 = a + 13;
  f = FmParams{q0[0], q0[1], q0[2], q0[3], q0[4], q0[5], a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8],
               a[9], q0[6], a[10], a[11], q0[7]};
  plps.clear();
  for (int k = 0; k < n; k++) {
    const int *q = a + 13 + PLP_INTS * k;
    plps.push_back(PlpParams{q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7], q[9], q[10], q[11], q[12], q[13]});
  }
  *nss = a[13 + PLP_INTS * MAX_PLP];
  return true;
}

extern "C" {

// multi-PLP frame plan: info [M, S, aux_len, t2frames, Lp, D, nplp, starts[8], cs[8], F[8], unit, nss, ssi,
// t2start, S_in, S[8], P[8], in_off[8], type2[8]] (68 ints); gather_in unit x M
int t2probe_frame_mplp(const int *mp, int *info, int32_t *gather_in, int32_t *gather_d, float *aux) {
  FmParams p;
  std::vector<PlpParams> plps;
  FramePlan fp;
  int nss = 1;
  if (!parse_mplp(mp, p, plps, &nss) || build_frame_mplp(p, plps, fp, true, nss)) return -1;
  int v[7] = {fp.M, fp.S, fp.aux_len, fp.t2frames, fp.Lp, fp.D, fp.nplp};
  memcpy(info, v, sizeof(v));
  for (int k = 0; k < 8; k++) {
    const bool in = k < fp.nplp;
    info[7 + k] = in ? fp.plp[k].start : 0;
    info[15 + k] = in ? fp.plp[k].cs : 0;
    info[23 + k] = in ? fp.plp[k].F : 0;
    info[36 + k] = in ? fp.plp[k].S : 0;
    info[44 + k] = in ? fp.plp[k].P : 0;
    info[52 + k] = in ? fp.plp[k].in_off : 0;
    info[60 + k] = in ? fp.plp[k].type2 : 0;
  }
  info[31] = fp.unit; info[32] = fp.nss; info[33] = fp.ssi; info[34] = fp.t2start; info[35] = fp.S_in;
  if (gather_in) memcpy(gather_in, fp.gather_in.data(), fp.gather_in.size() * 4);
  if (gather_d) memcpy(gather_d, fp.gather_d.data(), fp.gather_d.size() * 4);
  if (aux) memcpy(aux, fp.aux.data(), fp.aux.size() * 8);
  return 0;
}

// multi-PLP chain layout: as t2probe_chain, plus plp_bnd (2 Nsym x (nplp + 1)); info [Nsym, N, S, split, nplp]
int t2probe_chain_mplp(const int *mp, const int *pg3, int *info, int32_t *cmap, uint16_t *inv, int32_t *d0,
                       int32_t *dn, int32_t *dn0, int32_t *part, int32_t *bnd) {
  FmParams f;
  std::vector<PlpParams> plps;
  int nss = 1;
  if (!parse_mplp(mp, f, plps, &nss)) return -1;
  PgParams g{f.carriermode, f.fftsize, f.pilotpattern, f.guardinterval, f.numdatasyms, f.paprmode, f.version,
             f.preamble, pg3[0], pg3[1], pg3[2], fft_points(f.fftsize)};
  FramePlan fp;
  PilotPlan pp;
  ChainLayout cl;
  if (build_frame_mplp(f, plps, fp, false, nss) || build_pilot(g, pp) || build_chain_layout(fp, pp, cl)) return -1;
  info[0] = pp.Nsym; info[1] = pp.N; info[2] = fp.cls[0].S; info[3] = ofdm_split(pp.N) ? 1 : 0; info[4] = fp.nplp;
  if (cmap) memcpy(cmap, cl.cmap.data(), cl.cmap.size() * 4);
  if (inv) memcpy(inv, cl.inv.data(), cl.inv.size() * 2);
  if (d0) memcpy(d0, cl.sym_d0.data(), cl.sym_d0.size() * 4);
  if (dn) memcpy(dn, cl.sym_n.data(), cl.sym_n.size() * 4);
  if (dn0) memcpy(dn0, cl.sym_n0.data(), cl.sym_n0.size() * 4);
  if (part) memcpy(part, cl.part.data(), cl.part.size() * 4);
  if (bnd) memcpy(bnd, cl.plp_bnd.data(), cl.plp_bnd.size() * 4);
  return 0;
}

// multi-PLP L1-post signalling bits before the CRC-32 (one byte per bit) of FRAME_IDX frame_idx; returns the count
int t2probe_l1post_bits_mplp(const int *mp, int frame_idx, uint8_t *out, int cap) {
  FmParams p;
  std::vector<PlpParams> plps;
  FramePlan fp;
  int nss = 1;
  if (!parse_mplp(mp, p, plps, &nss) || build_frame_mplp(p, plps, fp, false, nss)) return -1;
  const std::vector<uint8_t> b = l1post_signal(p, fp, frame_idx, nullptr);
  if ((int)b.size() > cap) return -1;
  if (out) memcpy(out, b.data(), b.size());
  return (int)b.size();
}

// multi-PLP L1-post of one FRAME_IDX from the bit-by-bit host encoder; out Lp complex; info [nsig, npost, Lp]
int t2probe_l1post_mplp(const int *mp, int frame_idx, float *out, int *info) {
  FmParams p;
  std::vector<PlpParams> plps;
  FramePlan fp;
  int nss = 1;
  if (!parse_mplp(mp, p, plps, &nss) || build_frame_mplp(p, plps, fp, false, nss)) return -1;
  if (info) { info[0] = fp.l1.nsig; info[1] = fp.l1.npost; info[2] = fp.l1.lp; }
  return out ? l1post_host(p, fp, frame_idx, (cf32 *)out) : 0;
}

// info: [M, S, aux_len, t2frames, cs, F, N_P2, C_P2, C_DATA, N_FC, C_FC, Lp, D,
//        ti_on, ti_small, ti_big, ti_nsmall]
int t2probe_frame(const int *p20, int *info, int32_t *gather_in, int32_t *gather_d, float *aux, int16_t *ci_perm,
                  int32_t *ci_shift) {
  FmParams p{p20[0], p20[1], p20[2], p20[3], p20[4], p20[5], p20[6], p20[7], p20[8], p20[9],
             p20[10], p20[11], p20[12], p20[13], p20[14], p20[15], p20[16], p20[17], p20[18], p20[19]};
  FramePlan fp;
  if (build_frame(p, fp, true)) return -1;   // with every variant's L1-post encoded on the host
  int v[17] = {fp.M, fp.S, fp.aux_len, fp.t2frames, fp.cs, fp.F, fp.N_P2, fp.C_P2, fp.C_DATA, fp.N_FC, fp.C_FC,
               fp.Lp, fp.D, fp.ti_on, fp.ti_small, fp.ti_big, fp.ti_nsmall};
  memcpy(info, v, sizeof(v));
  if (gather_in) memcpy(gather_in, fp.gather_in.data(), fp.gather_in.size() * 4);
  if (gather_d) memcpy(gather_d, fp.gather_d.data(), fp.gather_d.size() * 4);
  if (ci_perm) memcpy(ci_perm, fp.ci_perm.data(), fp.ci_perm.size() * 2);
  if (ci_shift) memcpy(ci_shift, fp.ci_shift.data(), fp.ci_shift.size() * 4);
  if (aux) memcpy(aux, fp.aux.data(), fp.aux.size() * 8);
  return 0;
}

// info: [Nsym, N, active, G, C_PS, eq]; pilot_values 12 complex; p1 2048 complex; isinc N
int t2probe_pilot(const int *p12, int *info, int32_t *bin_map, float *pilot_values, float *p1, float *isinc,
                  float *norm) {
  PgParams p{p12[0], p12[1], p12[2], p12[3], p12[4], p12[5], p12[6], p12[7], p12[8], p12[9], p12[10], p12[11]};
  PilotPlan pp;
  if (build_pilot(p, pp)) return -1;
  int v[6] = {pp.Nsym, pp.N, pp.active, pp.G, pp.C_PS, pp.eq};
  memcpy(info, v, sizeof(v));
  if (bin_map) memcpy(bin_map, pp.bin_map.data(), pp.bin_map.size() * 4);
  if (pilot_values) memcpy(pilot_values, pp.pilot_values, sizeof(pp.pilot_values));
  if (p1) memcpy(p1, pp.p1.data(), pp.p1.size() * 8);
  if (isinc && pp.eq) memcpy(isinc, pp.isinc.data(), pp.isinc.size() * 4);
  if (norm) *norm = pp.normalization;
  return 0;
}

// the OFDM kernels' twiddle tables: tw 128 + N/128 complex, tw1k 1024 complex
int t2probe_twiddle(const int *p12, float *tw, float *tw1k) {
  PgParams p{p12[0], p12[1], p12[2], p12[3], p12[4], p12[5], p12[6], p12[7], p12[8], p12[9], p12[10], p12[11]};
  PilotPlan pp;
  if (build_pilot(p, pp)) return -1;
  if (tw) memcpy(tw, pp.twiddle.data(), pp.twiddle.size() * 8);
  if (tw1k) memcpy(tw1k, pp.twiddle1k.data(), pp.twiddle1k.size() * 8);
  return 0;
}

int t2probe_counts(int fftsize, int carriermode, int pp, int papr, int gi, int preamble, int *out5) {
  return frame_cell_counts(fftsize, carriermode, pp, papr, gi, preamble, out5);
}

// info: [mode, mod, W, R, cs]; lut 256 complex
int t2probe_map(int framesize, int rate, int constellation, int rotation, int *info, float *lut) {
  MapPlan mp;
  if (build_map(framesize, rate, constellation, rotation, mp)) return -1;
  int v[5] = {mp.mode, mp.mod, mp.W, mp.R, mp.cs};
  memcpy(info, v, sizeof(v));
  if (lut) memcpy(lut, mp.lut, sizeof(mp.lut));
  return 0;
}

// info: [kbch, nbch, P, q, nent, chunk, parity_il]; ldpc entries (group << 16 | rotation)
int t2probe_fec(int framesize, int rate, int constellation, int *info, uint32_t *ent, uint16_t *rowptr) {
  FecPlan fp;
  if (build_fec(framesize, rate, constellation, fp)) return -1;
  int v[7] = {fp.kbch, fp.nbch, fp.nparity, fp.q, (int)fp.ldpc_ent.size(), fp.bch_chunk, fp.parity_interleave};
  memcpy(info, v, sizeof(v));
  if (ent) memcpy(ent, fp.ldpc_ent.data(), fp.ldpc_ent.size() * 4);
  if (rowptr) memcpy(rowptr, fp.ldpc_rowptr.data(), fp.ldpc_rowptr.size() * 2);
  return 0;
}

// BCH tables of the FEC kernel: info [P, chunk, L]; tab 256 x 3 words; ctab (P/4) x 16 x 64 x 4 words
int t2probe_bch(int framesize, int rate, int *info, uint64_t *tab, uint64_t *ctab) {
  FecPlan fp;
  if (build_fec(framesize, rate, 3, fp)) return -1;
  info[0] = fp.nparity; info[1] = fp.bch_chunk; info[2] = fp.kbch / 8;
  if (tab) memcpy(tab, fp.bch_tab.data(), fp.bch_tab.size() * 8);
  if (ctab) memcpy(ctab, fp.bch_ctab.data(), fp.bch_ctab.size() * 8);
  return 0;
}

// the chain's BCH matrix-core table: info [nq, nt]; tab nq x 4 x nt x 64 x 4 words
int t2probe_bch_mfma(int framesize, int rate, int *info, uint32_t *tab) {
  FecPlan fp;
  if (build_fec(framesize, rate, 3, fp) || build_bch_mfma(fp)) return -1;
  info[0] = fp.bch_nq; info[1] = fp.bch_nt;
  if (tab) memcpy(tab, fp.bch_mfma.data(), fp.bch_mfma.size() * 4);
  return 0;
}

// fused-chain layout: cmap Nsym x N (stored row order), inv S, sym_d0/sym_n Nsym;
// info [Nsym, N, S, split]
int t2probe_chain(const int *p20, const int *pg3, int *info, int32_t *cmap, uint16_t *inv, int32_t *d0,
                  int32_t *dn, int32_t *dn0, int32_t *part) {
  FmParams f{p20[0], p20[1], p20[2], p20[3], p20[4], p20[5], p20[6], p20[7], p20[8], p20[9],
             p20[10], p20[11], p20[12], p20[13], p20[14], p20[15], p20[16], p20[17], p20[18], p20[19]};
  PgParams g{f.carriermode, f.fftsize, f.pilotpattern, f.guardinterval, f.numdatasyms, f.paprmode, f.version,
             f.preamble, pg3[0], pg3[1], pg3[2], fft_points(f.fftsize)};
  FramePlan fp;
  PilotPlan pp;
  ChainLayout cl;
  if (build_frame(f, fp) || build_pilot(g, pp) || build_chain_layout(fp, pp, cl)) return -1;
  info[0] = pp.Nsym; info[1] = pp.N; info[2] = fp.S; info[3] = ofdm_split(pp.N) ? 1 : 0;
  if (cmap) memcpy(cmap, cl.cmap.data(), cl.cmap.size() * 4);
  if (inv) memcpy(inv, cl.inv.data(), cl.inv.size() * 2);
  if (d0) memcpy(d0, cl.sym_d0.data(), cl.sym_d0.size() * 4);
  if (dn) memcpy(dn, cl.sym_n.data(), cl.sym_n.size() * 4);
  if (dn0) memcpy(dn0, cl.sym_n0.data(), cl.sym_n0.size() * 4);
  if (part) {
    if (cl.part.empty())
      for (int s = 0; s < fp.S; s++) part[s] = s;
    else
      memcpy(part, cl.part.data(), cl.part.size() * 4);
  }
  return 0;
}

// the fused chain's compact aux lists (build_aux_lists) over the per-variant aux table the chain
// uploads (frame aux cells with the 12 pilot values in every variant, as t2_capi.cpp composes
// it).  Call with null outputs first: sizes = [dbin entries, ind entries, groups, aux_len,
// t2frames]; auxv (aux_len * t2frames complex) is returned for the checker.
int t2probe_aux_lists(const int *p20, const int *pg3, int *sizes, uint16_t *dbin, float *dval, uint32_t *ind,
                      int32_t *grp, float *auxv_out, int32_t *zrun) {
  FmParams f{p20[0], p20[1], p20[2], p20[3], p20[4], p20[5], p20[6], p20[7], p20[8], p20[9],
             p20[10], p20[11], p20[12], p20[13], p20[14], p20[15], p20[16], p20[17], p20[18], p20[19]};
  PgParams g{f.carriermode, f.fftsize, f.pilotpattern, f.guardinterval, f.numdatasyms, f.paprmode, f.version,
             f.preamble, pg3[0], pg3[1], pg3[2], fft_points(f.fftsize)};
  FramePlan fp, fh;
  PilotPlan pp;
  ChainLayout cl;
  if (build_frame(f, fp) || build_frame(f, fh, true) || build_pilot(g, pp) || build_chain_layout(fp, pp, cl))
    return -1;
  // as t2_capi.cpp builds them: one aux row, the L1-post range per frame from the GPU
  std::vector<cf32> row = fp.aux;
  for (int i = 0; i < 12; i++) row[AUX_PILOT0 + i] = pp.pilot_values[i];
  AuxLists al;
  if (build_aux_lists(cl, pp.N, pp.Nsym, row, fp.aux_len, 1, al, AUX_L1PRE + 1840, fp.Lp)) return -2;
  // the checker's table: every t2_frame_num variant with its host-encoded L1-post
  std::vector<cf32> auxv = fh.aux;
  for (int v = 0; v < fp.t2frames; v++)
    for (int i = 0; i < 12; i++) auxv[(size_t)v * fp.aux_len + AUX_PILOT0 + i] = pp.pilot_values[i];
  sizes[0] = (int)al.dbin.size(); sizes[1] = (int)al.ind.size(); sizes[2] = (int)al.grp.size() / 4;
  sizes[3] = fp.aux_len; sizes[4] = fp.t2frames; sizes[5] = AUX_L1PRE + 1840;
  if (dbin) memcpy(dbin, al.dbin.data(), al.dbin.size() * 2);
  if (dval) memcpy(dval, al.dval.data(), al.dval.size() * 8);
  if (ind) memcpy(ind, al.ind.data(), al.ind.size() * 4);
  if (grp) memcpy(grp, al.grp.data(), al.grp.size() * 4);
  if (auxv_out) memcpy(auxv_out, auxv.data(), (size_t)fp.aux_len * fp.t2frames * 8);
  if (zrun) memcpy(zrun, al.zrun.data(), al.zrun.size() * 4);
  return 0;
}

// L1-post of one FRAME_IDX: cells from the GPU plan applied on the host in the l1post kernel's
// order of operations (plan = 1) or from the bit-by-bit host encoder (plan = 0); out: Lp complex.
// info (optional): [nsig, npost, Lp, mode]
int t2probe_l1post(const int *p20, int frame_idx, int plan, float *out, int *info) {
  FmParams p{p20[0], p20[1], p20[2], p20[3], p20[4], p20[5], p20[6], p20[7], p20[8], p20[9],
             p20[10], p20[11], p20[12], p20[13], p20[14], p20[15], p20[16], p20[17], p20[18], p20[19]};
  FramePlan fp;
  if (build_frame(p, fp)) return -1;
  const L1PostPlan &l = fp.l1;
  if (info) { info[0] = l.nsig; info[1] = l.npost; info[2] = l.lp; info[3] = l.mode; }
  if (!out) return 0;
  cf32 *o = (cf32 *)out;
  if (!plan) return l1post_host(p, fp, frame_idx, o);
  auto bit = [](const std::vector<uint32_t> &w, int i) { return (w[i >> 5] >> (31 - (i & 31))) & 1u; };
  auto set = [](std::vector<uint32_t> &w, int i) { w[i >> 5] |= 1u << (31 - (i & 31)); };
  std::vector<uint32_t> sig = l.tmpl;
  const uint32_t fidx = (uint32_t)(frame_idx % fp.t2frames);
  for (int k = 0; k < 8; k++)
    if ((fidx >> (7 - k)) & 1u) set(sig, l.fidx_pos + k);
  const int L = l.nsig - 32;
  uint32_t crc = l.crc_k;
  for (int i = 0; i < L; i++)
    if (bit(sig, i)) crc ^= l.crc_c[i];
  for (int k = 0; k < 32; k++)
    if ((crc >> (31 - k)) & 1u) set(sig, L + k);
  if (!l.scr.empty())
    for (size_t w = 0; w < sig.size(); w++) sig[w] ^= l.scr[w];
  std::vector<uint32_t> cw((16200 + 31) / 32, 0);
  uint32_t b[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < l.nsig; i++)
    if (bit(sig, i)) {
      set(cw, l.sig_pos[i]);
      for (int k = 0; k < 6; k++) b[k] ^= l.bch_r[(size_t)i * 6 + k];
    }
  for (int n = 0; n < 168; n++)
    if ((b[n >> 5] >> (31 - (n & 31))) & 1u) set(cw, 7032 + n);
  std::vector<uint8_t> par(l.pbits, 0);
  for (int i = 0; i < l.nsig + 168; i++) {
    const int pos = i < l.nsig ? (int)l.sig_pos[i] : 7032 + (i - l.nsig);
    if (!bit(cw, pos)) continue;
    const int g = pos / 360, n = pos % 360;
    for (int e = l.ldpc_ptr[g]; e < l.ldpc_ptr[g + 1]; e++) par[(l.ldpc_addr[e] + n * l.q) % l.pbits] ^= 1;
  }
  for (int j = 1; j < l.pbits; j++) par[j] ^= par[j - 1];
  for (int j = 0; j < l.pbits; j++)
    if (par[j]) set(cw, 7200 + j);
  for (int c = 0; c < l.lp; c++) {
    if (l.mode == 0) {
      o[c] = cf32{bit(cw, l.sel[c]) ? -1.0f : 1.0f, 0.0f};
    } else if (l.mode == 1) {
      o[c] = l.lut[(bit(cw, l.sel[2 * c]) << 1) | bit(cw, l.sel[2 * c + 1])];
    } else {
      const int k = c >> 1, half = l.ncols >> 1, e0 = (c & 1) ? half : 0;
      uint32_t pack = 0;
      for (int e = e0; e < e0 + half; e++) pack = (pack << 1) | bit(cw, l.sel[l.rows * l.mux[e] + k]);
      o[c] = l.lut[pack];
    }
  }
  return 0;
}
}
