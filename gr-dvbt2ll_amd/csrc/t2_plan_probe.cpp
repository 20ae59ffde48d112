// t2_plan_probe.cpp -- host-only export of the configuration planner (t2_plan.cpp) for the
// CPU test suite: lets tests apply the product's composed gather maps with numpy and compare
// them with the oracle for every parameter combination without a GPU.  Not part of the
// GPU product library (libdvbt2ll_hip.so); built as gr-dvbt2ll_amd/csrc/_obj/libt2plan_probe.so.
#include <cstring>

#include "t2_plan.h"

using namespace t2;

extern "C" {

// info: [M, S, aux_len, t2frames, cs, F, N_P2, C_P2, C_DATA, N_FC, C_FC, Lp, D,
//        ti_on, ti_small, ti_big, ti_nsmall]
int t2probe_frame(const int *p20, int *info, int32_t *gather_in, int32_t *gather_d, float *aux, int16_t *ci_perm,
                  int32_t *ci_shift) {
  FmParams p{p20[0], p20[1], p20[2], p20[3], p20[4], p20[5], p20[6], p20[7], p20[8], p20[9],
             p20[10], p20[11], p20[12], p20[13], p20[14], p20[15], p20[16], p20[17], p20[18], p20[19]};
  FramePlan fp;
  if (build_frame(p, fp)) return -1;
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
  FramePlan fp;
  PilotPlan pp;
  ChainLayout cl;
  if (build_frame(f, fp) || build_pilot(g, pp) || build_chain_layout(fp, pp, cl)) return -1;
  std::vector<cf32> auxv = fp.aux;
  for (int v = 0; v < fp.t2frames; v++)
    for (int i = 0; i < 12; i++) auxv[(size_t)v * fp.aux_len + AUX_PILOT0 + i] = pp.pilot_values[i];
  AuxLists al;
  if (build_aux_lists(cl, pp.N, pp.Nsym, auxv, fp.aux_len, fp.t2frames, al)) return -2;
  sizes[0] = (int)al.dbin.size(); sizes[1] = (int)al.ind.size(); sizes[2] = (int)al.grp.size() / 4;
  sizes[3] = fp.aux_len; sizes[4] = fp.t2frames;
  if (dbin) memcpy(dbin, al.dbin.data(), al.dbin.size() * 2);
  if (dval) memcpy(dval, al.dval.data(), al.dval.size() * 8);
  if (ind) memcpy(ind, al.ind.data(), al.ind.size() * 4);
  if (grp) memcpy(grp, al.grp.data(), al.grp.size() * 4);
  if (auxv_out) memcpy(auxv_out, auxv.data(), (size_t)fp.aux_len * fp.t2frames * 8);
  if (zrun) memcpy(zrun, al.zrun.data(), al.zrun.size() * 4);
  return 0;
}
}
