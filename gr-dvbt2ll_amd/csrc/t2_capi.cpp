// t2_capi.cpp -- C ABI (include/dvbt2ll_hip.h): handles, device tables, launches.
//
// Each handle mirrors one reference gr::block: the constructor work happens in
// *_create (host planning in t2_plan.cpp + one upload of the device tables), and
// *_general_work runs the block's kernels synchronously on the handle's HIP stream
// with the caller's host buffers (GNU Radio's circular buffers).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <vector>

#include "../../include/dvbt2ll_hip.h"
#include "t2_kernels.h"
#include "t2_plan.h"

using namespace t2;

namespace {

#define HIP_TRY(expr)                                   \
  do {                                                  \
    hipError_t e_ = (expr);                             \
    if (e_ != hipSuccess) {                             \
      last_hip_error() = e_;                            \
      return e_ == hipErrorOutOfMemory ? DVBT2LL_ENOMEM : DVBT2LL_EDEVICE; \
    }                                                   \
  } while (0)

hipError_t &last_hip_error() {
  static thread_local hipError_t e = hipSuccess;
  return e;
}

// device buffer with grow-on-demand
struct DevBuf {
  void *p = nullptr;
  size_t n = 0;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  int ensure(size_t bytes) {
    if (bytes <= n) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (hipMalloc(&p, bytes) != hipSuccess) return DVBT2LL_ENOMEM;
    n = bytes;
    return 0;
  }
  template <class T> T *as() const { return (T *)p; }
};

template <class T>
int upload(DevBuf &b, const std::vector<T> &v) {
  if (v.empty()) return 0;
  if (b.ensure(v.size() * sizeof(T))) return DVBT2LL_ENOMEM;
  HIP_TRY(hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}
int upload_raw(DevBuf &b, const void *src, size_t bytes) {
  if (b.ensure(bytes)) return DVBT2LL_ENOMEM;
  HIP_TRY(hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice));
  return 0;
}

struct DeviceCtx {
  int device = 0;
  hipStream_t stream = nullptr;
  int init(int dev) {
    device = dev;
    HIP_TRY(hipSetDevice(dev));
    HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    return 0;
  }
  ~DeviceCtx() {
    if (stream) { (void)hipSetDevice(device); (void)hipStreamDestroy(stream); }
  }
};

// ---------------------------------------------------------------- FEC tables on device
struct FecTables {
  FecPlan plan;
  DevBuf hcrc, tab, ctab, rowptr, ent, prbs, crc8, crcsh, bmf;
  FecDev dev{};
  // the fused chain's BCH pass on the matrix cores: the generator matrix as fp4 B fragments
  int init_chain() {
    if (build_bch_mfma(plan)) return DVBT2LL_EINVAL;
    int r = upload(bmf, plan.bch_mfma);
    if (r) return r;
    dev.bch_mfma = bmf.as<uint4>();
    dev.bch_nq = plan.bch_nq;
    dev.bch_nt = plan.bch_nt;
    return 0;
  }
  int init(int framesize, int rate, int constellation, int mode, int inband, int fecblocks, int tsrate) {
    if (build_fec(framesize, rate, constellation, plan)) return DVBT2LL_EINVAL;
    int r;
    if ((r = upload(tab, plan.bch_tab)) || (r = upload(ctab, plan.bch_ctab)) ||
        (r = upload(rowptr, plan.ldpc_rowptr)) || (r = upload(ent, plan.ldpc_ent)) ||
        (r = upload(prbs, plan.prbs_bytes)) || (r = upload(crc8, plan.crc8_tab)) || (r = upload(crcsh, plan.crc8_shift)) ||
        (r = upload(hcrc, plan.hcrc_bits)))
      return r;
    dev.bch_tab = tab.as<uint64_t>();
    dev.bch_ctab = ctab.as<uint64_t>();
    dev.ldpc_rowptr = rowptr.as<uint16_t>();
    dev.ldpc_ent = ent.as<uint32_t>();
    dev.prbs = prbs.as<uint8_t>();
    dev.crc8_tab = crc8.as<uint8_t>();
    dev.crc8_shift = crcsh.as<uint8_t>();
    dev.hcrc_bits = hcrc.as<uint8_t>();
    dev.kbch = plan.kbch; dev.nbch = plan.nbch; dev.P = plan.nparity; dev.nldpc = plan.nldpc;
    dev.q = plan.q; dev.nent = (int)plan.ldpc_ent.size(); dev.chunk = plan.bch_chunk;
    dev.parity_il = plan.parity_interleave ? 1 : 0;
    dev.hem = mode ? 1 : 0;
    dev.inband = inband ? 1 : 0;
    dev.fec_blocks = fecblocks > 0 ? fecblocks : 1;
    dev.ts_rate = tsrate;
    dev.matype = MATYPE_SIS;
    return 0;
  }
};

struct MapTables {
  MapPlan plan;
  DevBuf lut, colbuf;
  MapDev dev{};
  int init(int framesize, int rate, int constellation, int rotation, const FecPlan &fec) {
    if (build_map(framesize, rate, constellation, rotation, plan)) return DVBT2LL_EINVAL;
    int r = upload_raw(lut, plan.lut, sizeof(plan.lut));
    if (r) return r;
    dev.lut = lut.as<float2>();
    dev.mode = plan.mode; dev.mod = plan.mod; dev.W = plan.W; dev.R = plan.R; dev.cs = plan.cs;
    dev.nldpc = plan.nldpc; dev.nbch = fec.nbch; dev.q = fec.q; dev.rotation = plan.rotation;
    dev.parity_il = fec.parity_interleave ? 1 : 0;
    dev.F = 1;
    // column feeding bit b of the demuxed row word (b = W - 1 - mux[e]): its start bit and twist
    std::vector<int2> col(16, int2{-1, 0});
    for (int e = 0; e < plan.W && plan.mode != 0; e++) col[plan.W - 1 - plan.mux[e]] = int2{e * plan.R, plan.twist[e]};
    if ((r = upload(colbuf, col))) return r;
    dev.col = colbuf.as<int2>();
    return 0;
  }
};

// ---------------------------------------------------------------- L1-post tables on device
struct L1Tables {
  DevBuf tmpl, crc_c, scr, sig_pos, bch_r, ldpc_ptr, ldpc_addr, sel, lut;
  L1Dev dev{};
  int init(const FramePlan &fp) {
    const L1PostPlan &l = fp.l1;
    int r;
    if ((r = upload(tmpl, l.tmpl)) || (r = upload(crc_c, l.crc_c)) || (r = upload(scr, l.scr)) ||
        (r = upload(sig_pos, l.sig_pos)) || (r = upload(bch_r, l.bch_r)) || (r = upload(ldpc_ptr, l.ldpc_ptr)) ||
        (r = upload(ldpc_addr, l.ldpc_addr)) || (r = upload(sel, l.sel)) || (r = upload_raw(lut, l.lut, sizeof(l.lut))))
      return r;
    dev.tmpl = tmpl.as<uint32_t>();
    dev.crc_c = crc_c.as<uint32_t>();
    dev.scr = l.scr.empty() ? nullptr : scr.as<uint32_t>();
    dev.sig_pos = sig_pos.as<uint16_t>();
    dev.bch_r = bch_r.as<uint32_t>();
    dev.ldpc_ptr = ldpc_ptr.as<uint16_t>();
    dev.ldpc_addr = ldpc_addr.as<uint16_t>();
    dev.sel = sel.as<uint16_t>();
    dev.lut = lut.as<float2>();
    dev.crc_k = l.crc_k;
    dev.nsig = l.nsig; dev.fidx_pos = l.fidx_pos; dev.npost = l.npost; dev.lp = l.lp; dev.mode = l.mode;
    dev.ncols = l.ncols; dev.rows = l.rows; dev.q = l.q; dev.pbits = l.pbits; dev.t2frames = fp.t2frames;
    dev.ncls = l.ncls;
    memcpy(dev.mux, l.mux, sizeof(dev.mux));
    return 0;
  }
};

}  // namespace

// ============================================================================ common
extern "C" const char *dvbt2ll_strerror(int status) {
  switch (status) {
    case DVBT2LL_OK: return "ok";
    case DVBT2LL_EINVAL: return "invalid parameter combination";
    case DVBT2LL_ENOMEM: return "out of memory";
    case DVBT2LL_EDEVICE: return hipGetErrorString(last_hip_error());
    case DVBT2LL_ESHORT: return "not enough input items";
    default: return "unknown status";
  }
}
extern "C" const char *dvbt2ll_version(void) { return "dvbt2ll-mi355x 0.1 (gfx950)"; }
extern "C" int dvbt2ll_abi_version(void) { return DVBT2LL_ABI_VERSION; }
extern "C" int dvbt2ll_abi_check(int abi_version, size_t sizeof_chain_params, size_t sizeof_chain_info,
                                 size_t sizeof_plp_params, size_t sizeof_mplp_params, size_t sizeof_mplp_chain_params) {
  return abi_version == DVBT2LL_ABI_VERSION && sizeof_chain_params == sizeof(dvbt2ll_chain_params) &&
                 sizeof_chain_info == sizeof(dvbt2ll_chain_info) && sizeof_plp_params == sizeof(dvbt2ll_plp_params) &&
                 sizeof_mplp_params == sizeof(dvbt2ll_mplp_params) &&
                 sizeof_mplp_chain_params == sizeof(dvbt2ll_mplp_chain_params)
             ? DVBT2LL_OK
             : DVBT2LL_EINVAL;
}
extern "C" int dvbt2ll_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// ============================================================================ bbheaderbch
struct dvbt2ll_bbheaderbch {
  DeviceCtx ctx;
  FecTables fec;
  dvbt2ll_bbheaderbch_params p{};
  int64_t blocks_done = 0;       // fec_block state = blocks_done % fecblocks
  int64_t consumed_total = 0;    // absolute TS offset of the next input byte
  std::vector<uint8_t> history;  // last <= 376 consumed TS bytes (previous packet for CRC-8)
  DevBuf din, dout;
  std::vector<uint8_t> hbuf;
  DevBuf sync_err;               // device counter: TS sync bytes != 0x47 consumed so far
  uint32_t sync_err_host = 0;
};

extern "C" int dvbt2ll_bbheaderbch_create(const dvbt2ll_bbheaderbch_params *p, int device, dvbt2ll_bbheaderbch **out) {
  if (!p || !out) return DVBT2LL_EINVAL;
  *out = nullptr;
  std::unique_ptr<dvbt2ll_bbheaderbch> h(new (std::nothrow) dvbt2ll_bbheaderbch());
  if (!h) return DVBT2LL_ENOMEM;
  h->p = *p;
  if (p->inband && p->fecblocks < 1) return DVBT2LL_EINVAL;
  int r = h->ctx.init(device);
  if (r) return r;
  if ((r = h->fec.init(p->framesize, p->rate, 3, p->mode, p->inband, p->fecblocks, p->tsrate))) return r;
  if (h->sync_err.ensure(4)) return DVBT2LL_ENOMEM;
  HIP_TRY(hipMemset(h->sync_err.p, 0, 4));
  *out = h.release();
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_bbheaderbch_output_multiple(const dvbt2ll_bbheaderbch *h) { return h ? h->fec.plan.nbch : 0; }
extern "C" int dvbt2ll_bbheaderbch_forecast(const dvbt2ll_bbheaderbch *h, int nout, int *nin) {
  if (!h || !nin) return DVBT2LL_EINVAL;
  const FecPlan &f = h->fec.plan;
  int n = (nout - 80 - (f.nbch - f.kbch)) / 8;       // bbheader:207-216
  if (h->p.mode) n += (((f.kbch - 80) / 8) / 187) + 1;
  *nin = n;
  return DVBT2LL_OK;
}

// input bytes consumed by nblocks FEC blocks starting at absolute block b0 / stream offset
static int64_t bb_consumed(const FecDev &d, int64_t b0, int64_t nblocks) {
  auto J = [&](int64_t B) {
    int64_t pay = (d.kbch - 80) / 8;
    int64_t npad = d.inband ? (B + d.fec_blocks - 1) / d.fec_blocks : 0;
    return B * pay - 13 * npad;
  };
  auto pos_after = [&](int64_t B) -> int64_t {   // stream offset after block B-1
    int64_t j = J(B);
    if (!d.hem || j == 0) return j;
    int64_t last = j - 1;
    return 188 * (last / 187) + 1 + (last % 187) + 1;
  };
  return pos_after(b0 + nblocks) - pos_after(b0);
}

extern "C" int dvbt2ll_bbheaderbch_general_work(dvbt2ll_bbheaderbch *h, int nout, int nin, const void *in, void *out,
                                                int *consumed) {
  if (!h || nout < 0 || (nout && (!in || !out))) return DVBT2LL_EINVAL;
  const FecDev &d = h->fec.dev;
  int nb = nout / d.nbch;
  if (consumed) *consumed = 0;
  if (nb == 0) return 0;
  int64_t need = bb_consumed(d, h->blocks_done, nb);
  if (need > nin) return DVBT2LL_ESHORT;
  // device buffer: [history | new input]; ts_base = absolute offset of history start
  int64_t hist = (int64_t)h->history.size();
  h->hbuf.resize(hist + need);
  if (hist) memcpy(h->hbuf.data(), h->history.data(), hist);
  memcpy(h->hbuf.data() + hist, in, need);
  HIP_TRY(hipSetDevice(h->ctx.device));
  if (h->din.ensure(h->hbuf.size() + 16) || h->dout.ensure((size_t)nb * d.nbch)) return DVBT2LL_ENOMEM;
  HIP_TRY(hipMemcpyAsync(h->din.p, h->hbuf.data(), h->hbuf.size(), hipMemcpyHostToDevice, h->ctx.stream));
  FecIO io{};
  io.in = h->din.as<uint8_t>();
  io.ts_base = h->consumed_total - hist;
  io.ts_len = (int64_t)h->hbuf.size();
  io.first_block = h->blocks_done;
  io.out = h->dout.as<uint8_t>();
  io.nblocks = nb;
  io.sync_err = h->sync_err.as<uint32_t>();
  HIP_TRY(launch_fec(FEC_TS_TO_BITS, d, io, h->ctx.stream));
  HIP_TRY(hipMemcpyAsync(out, h->dout.p, (size_t)nb * d.nbch, hipMemcpyDeviceToHost, h->ctx.stream));
  HIP_TRY(hipMemcpyAsync(&h->sync_err_host, h->sync_err.p, 4, hipMemcpyDeviceToHost, h->ctx.stream));
  HIP_TRY(hipStreamSynchronize(h->ctx.stream));
  h->blocks_done += nb;
  h->consumed_total += need;
  size_t keep = std::min<size_t>(376, h->hbuf.size());
  h->history.assign(h->hbuf.end() - keep, h->hbuf.end());
  if (consumed) *consumed = (int)need;
  return nb * d.nbch;
}
extern "C" int64_t dvbt2ll_bbheaderbch_sync_errors(const dvbt2ll_bbheaderbch *h) {
  return h ? (int64_t)h->sync_err_host : 0;
}
extern "C" int dvbt2ll_bbheaderbch_set_isi(dvbt2ll_bbheaderbch *h, int isi) {
  if (!h || isi < 0 || isi > 255) return DVBT2LL_EINVAL;
  h->fec.dev.matype = MATYPE_MIS | isi;   // bbheader:288-298
  return DVBT2LL_OK;
}
extern "C" void dvbt2ll_bbheaderbch_destroy(dvbt2ll_bbheaderbch *h) { delete h; }

// ============================================================================ ldpc
struct dvbt2ll_ldpc {
  DeviceCtx ctx;
  FecTables fec;
  DevBuf din, dout;
};
extern "C" int dvbt2ll_ldpc_create(const dvbt2ll_ldpc_params *p, int device, dvbt2ll_ldpc **out) {
  if (!p || !out) return DVBT2LL_EINVAL;
  *out = nullptr;
  std::unique_ptr<dvbt2ll_ldpc> h(new (std::nothrow) dvbt2ll_ldpc());
  if (!h) return DVBT2LL_ENOMEM;
  int r = h->ctx.init(device);
  if (r) return r;
  if ((r = h->fec.init(p->framesize, p->rate, 3, 0, 0, 1, 0))) return r;
  *out = h.release();
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_ldpc_output_multiple(const dvbt2ll_ldpc *h) { return h ? h->fec.plan.nldpc : 0; }
extern "C" int dvbt2ll_ldpc_forecast(const dvbt2ll_ldpc *h, int nout, int *nin) {
  if (!h || !nin) return DVBT2LL_EINVAL;
  *nin = (nout / h->fec.plan.nldpc) * h->fec.plan.nbch;
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_ldpc_general_work(dvbt2ll_ldpc *h, int nout, int nin, const void *in, void *out, int *consumed) {
  if (!h || nout < 0 || (nout && (!in || !out))) return DVBT2LL_EINVAL;
  const FecDev &d = h->fec.dev;
  int nb = nout / d.nldpc;
  if (consumed) *consumed = 0;
  if (nb == 0) return 0;
  if ((int64_t)nb * d.nbch > nin) return DVBT2LL_ESHORT;
  HIP_TRY(hipSetDevice(h->ctx.device));
  if (h->din.ensure((size_t)nb * d.nbch) || h->dout.ensure((size_t)nb * d.nldpc)) return DVBT2LL_ENOMEM;
  HIP_TRY(hipMemcpyAsync(h->din.p, in, (size_t)nb * d.nbch, hipMemcpyHostToDevice, h->ctx.stream));
  FecIO io{};
  io.in = h->din.as<uint8_t>();
  io.out = h->dout.as<uint8_t>();
  io.nblocks = nb;
  HIP_TRY(launch_fec(FEC_BITS_TO_BITS, d, io, h->ctx.stream));
  HIP_TRY(hipMemcpyAsync(out, h->dout.p, (size_t)nb * d.nldpc, hipMemcpyDeviceToHost, h->ctx.stream));
  HIP_TRY(hipStreamSynchronize(h->ctx.stream));
  if (consumed) *consumed = nb * d.nbch;
  return nb * d.nldpc;
}
extern "C" void dvbt2ll_ldpc_destroy(dvbt2ll_ldpc *h) { delete h; }

// ============================================================================ interleavermod
struct dvbt2ll_interleavermod {
  DeviceCtx ctx;
  FecPlan fec;
  MapTables map;
  DevBuf din, dout;
};
extern "C" int dvbt2ll_interleavermod_create(const dvbt2ll_interleavermod_params *p, int device,
                                             dvbt2ll_interleavermod **out) {
  if (!p || !out) return DVBT2LL_EINVAL;
  *out = nullptr;
  std::unique_ptr<dvbt2ll_interleavermod> h(new (std::nothrow) dvbt2ll_interleavermod());
  if (!h) return DVBT2LL_ENOMEM;
  if (build_fec(p->framesize, p->rate, p->constellation, h->fec)) return DVBT2LL_EINVAL;
  int r = h->ctx.init(device);
  if (r) return r;
  if ((r = h->map.init(p->framesize, p->rate, p->constellation, p->rotation, h->fec))) return r;
  *out = h.release();
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_interleavermod_output_multiple(const dvbt2ll_interleavermod *h) { return h ? h->map.plan.cs : 0; }
extern "C" int dvbt2ll_interleavermod_forecast(const dvbt2ll_interleavermod *h, int nout, int *nin) {
  if (!h || !nin) return DVBT2LL_EINVAL;
  *nin = (nout / h->map.plan.cs) * h->map.plan.nldpc;   // interleavermod:264-268
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_interleavermod_general_work(dvbt2ll_interleavermod *h, int nout, int nin, const void *in,
                                                   void *out, int *consumed) {
  if (!h || nout < 0 || (nout && (!in || !out))) return DVBT2LL_EINVAL;
  const MapDev &d = h->map.dev;
  int nb = nout / d.cs;
  if (consumed) *consumed = 0;
  if (nb == 0) return 0;
  if ((int64_t)nb * d.nldpc > nin) return DVBT2LL_ESHORT;
  HIP_TRY(hipSetDevice(h->ctx.device));
  if (h->din.ensure((size_t)nb * d.nldpc) || h->dout.ensure((size_t)nb * d.cs * 8)) return DVBT2LL_ENOMEM;
  HIP_TRY(hipMemcpyAsync(h->din.p, in, (size_t)nb * d.nldpc, hipMemcpyHostToDevice, h->ctx.stream));
  MapIO io{};
  io.in = h->din.as<uint8_t>();
  io.out = h->dout.as<float2>();
  io.nblocks = nb;
  HIP_TRY(launch_map(d, io, h->ctx.stream));
  HIP_TRY(hipMemcpyAsync(out, h->dout.p, (size_t)nb * d.cs * 8, hipMemcpyDeviceToHost, h->ctx.stream));
  HIP_TRY(hipStreamSynchronize(h->ctx.stream));
  if (consumed) *consumed = nb * d.nldpc;
  return nb * d.cs;
}
extern "C" void dvbt2ll_interleavermod_destroy(dvbt2ll_interleavermod *h) { delete h; }

// ============================================================================ framemapperfint
static FmParams to_fm(const dvbt2ll_framemapperfint_params &p) {
  return FmParams{p.framesize, p.rate, p.constellation, p.rotation, p.fecblocks, p.tiblocks, p.carriermode,
                  p.fftsize, p.guardinterval, p.l1constellation, p.pilotpattern, p.t2frames, p.numdatasyms,
                  p.paprmode, p.version, p.preamble, p.inputmode, p.reservedbiasbits, p.l1scrambled, p.inband};
}

struct dvbt2ll_framemapperfint {
  DeviceCtx ctx;
  FramePlan plan;
  L1Tables l1;
  DevBuf map, aux, din, dout;   // aux: one row; its L1-post cells are rewritten per call on the GPU
  int t2_frame_num = 0;
};
extern "C" int dvbt2ll_framemapperfint_create(const dvbt2ll_framemapperfint_params *p, int device,
                                              dvbt2ll_framemapperfint **out) {
  if (!p || !out) return DVBT2LL_EINVAL;
  *out = nullptr;
  std::unique_ptr<dvbt2ll_framemapperfint> h(new (std::nothrow) dvbt2ll_framemapperfint());
  if (!h) return DVBT2LL_ENOMEM;
  if (build_frame(to_fm(*p), h->plan)) return DVBT2LL_EINVAL;
  int r = h->ctx.init(device);
  if (r) return r;
  if ((r = upload(h->map, h->plan.gather_in)) || (r = upload(h->aux, h->plan.aux)) || (r = h->l1.init(h->plan)))
    return r;
  *out = h.release();
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_framemapperfint_output_multiple(const dvbt2ll_framemapperfint *h) { return h ? h->plan.M : 0; }
extern "C" int dvbt2ll_framemapperfint_stream_items(const dvbt2ll_framemapperfint *h) { return h ? h->plan.S : 0; }
extern "C" int dvbt2ll_framemapperfint_forecast(const dvbt2ll_framemapperfint *h, int nout, int *nin) {
  if (!h || !nin) return DVBT2LL_EINVAL;
  *nin = h->plan.S * (nout / h->plan.M);   // framemapper:1942-1946
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_framemapperfint_general_work(dvbt2ll_framemapperfint *h, int nout, int nin, const void *in,
                                                    void *out, int *consumed) {
  if (!h || nout < 0 || (nout && (!in || !out))) return DVBT2LL_EINVAL;
  const FramePlan &f = h->plan;
  if (consumed) *consumed = 0;
  if (nout < f.M) return 0;
  if (nin < f.S) return DVBT2LL_ESHORT;
  // one T2 frame per call (the reference consumes exactly one frame, framemapper:2147)
  HIP_TRY(hipSetDevice(h->ctx.device));
  if (h->din.ensure((size_t)f.S * 8) || h->dout.ensure((size_t)f.M * 8)) return DVBT2LL_ENOMEM;
  HIP_TRY(hipMemcpyAsync(h->din.p, in, (size_t)f.S * 8, hipMemcpyHostToDevice, h->ctx.stream));
  // this frame's L1-post cells (FRAME_IDX = t2_frame_num) into the aux row, then the gather
  L1IO lio{};
  lio.out = h->aux.as<float2>() + AUX_L1PRE + 1840;
  lio.first_frame = h->t2_frame_num;
  lio.nframes = 1;
  HIP_TRY(launch_l1post(h->l1.dev, lio, h->ctx.stream));
  GatherIO io{};
  io.in = h->din.as<float2>();
  io.out = h->dout.as<float2>();
  io.map = h->map.as<int32_t>();
  io.aux = h->aux.as<float2>();
  io.M = f.M;
  HIP_TRY(launch_gather(io, h->ctx.stream));
  HIP_TRY(hipMemcpyAsync(out, h->dout.p, (size_t)f.M * 8, hipMemcpyDeviceToHost, h->ctx.stream));
  HIP_TRY(hipStreamSynchronize(h->ctx.stream));
  h->t2_frame_num = (h->t2_frame_num + 1) % f.t2frames;
  if (consumed) *consumed = f.S;
  return f.M;
}
extern "C" void dvbt2ll_framemapperfint_destroy(dvbt2ll_framemapperfint *h) { delete h; }

// ============================================================================ framemapper, multi-PLP
static bool mplp_to_plan(const dvbt2ll_mplp_params &m, FmParams &fm, std::vector<PlpParams> &plps,
                         std::vector<int> &tsrate, int *nss);

struct dvbt2ll_framemapper_mplp {
  DeviceCtx ctx;
  FramePlan plan;
  L1Tables l1;
  // din: the current interleaving frame of every PLP (PLP k's S_if cells at in_off); map: one gather row per
  // frame phase (frame mod unit)
  DevBuf map, aux, din, dout;
  int t2_frame_num = 0;
  int64_t frame = 0;            // T2 frames produced (the phase of the next one is frame mod unit)
  // cells port k consumes at the T2 frame frame + i: a whole interleaving frame on its first T2 frame
  int need(int k, int64_t i) const {
    const PlpPlan &pl = plan.plp[k];
    return (frame + i) % pl.cycle() == pl.FF ? pl.S_if : 0;
  }
};
extern "C" int dvbt2ll_framemapper_mplp_create(const dvbt2ll_mplp_params *p, int device, dvbt2ll_framemapper_mplp **out) {
  if (!p || !out) return DVBT2LL_EINVAL;
  *out = nullptr;
  FmParams fm;
  std::vector<PlpParams> plps;
  std::vector<int> tsrate;
  int nss = 1;
  if (!mplp_to_plan(*p, fm, plps, tsrate, &nss)) return DVBT2LL_EINVAL;
  std::unique_ptr<dvbt2ll_framemapper_mplp> h(new (std::nothrow) dvbt2ll_framemapper_mplp());
  if (!h) return DVBT2LL_ENOMEM;
  if (build_frame_mplp(fm, plps, h->plan, false, nss)) return DVBT2LL_EINVAL;
  int r = h->ctx.init(device);
  if (r) return r;
  if ((r = upload(h->map, h->plan.gather_in)) || (r = upload(h->aux, h->plan.aux)) || (r = h->l1.init(h->plan)))
    return r;
  *out = h.release();
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_framemapper_mplp_output_multiple(const dvbt2ll_framemapper_mplp *h) { return h ? h->plan.M : 0; }
extern "C" int dvbt2ll_framemapper_mplp_stream_items(const dvbt2ll_framemapper_mplp *h, int plp) {
  return h && plp >= 0 && plp < h->plan.nplp ? h->plan.plp[plp].S : 0;
}
extern "C" int dvbt2ll_framemapper_mplp_forecast(const dvbt2ll_framemapper_mplp *h, int nout, int *nin) {
  if (!h || !nin) return DVBT2LL_EINVAL;
  // framemapper:1942-1946: the cells of nout / M frames; a TIME_IL_TYPE 1 PLP's interleaving frame is
  // consumed whole on its first T2 frame
  for (int k = 0; k < h->plan.nplp; k++) {
    int64_t n = 0;
    for (int i = 0; i < nout / h->plan.M; i++) n += h->need(k, i);
    nin[k] = (int)std::min<int64_t>(n, INT32_MAX);
  }
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_framemapper_mplp_general_work(dvbt2ll_framemapper_mplp *h, int nout, const int *nin,
                                                     const void *const *in, void *out, int *consumed) {
  if (!h || nout < 0 || (nout && (!in || !out || !nin))) return DVBT2LL_EINVAL;
  const FramePlan &f = h->plan;
  if (consumed)
    for (int k = 0; k < f.nplp; k++) consumed[k] = 0;
  if (nout < f.M) return 0;
  for (int k = 0; k < f.nplp; k++)
    if (h->need(k, 0) && (!in[k] || nin[k] < h->need(k, 0))) return DVBT2LL_ESHORT;
  // one T2 frame per call, one frame of every port (framemapper:2147); a port whose PLP starts an interleaving
  // frame here delivers all of it
  HIP_TRY(hipSetDevice(h->ctx.device));
  if (h->din.ensure((size_t)f.S_in * 8) || h->dout.ensure((size_t)f.M * 8)) return DVBT2LL_ENOMEM;
  for (int k = 0; k < f.nplp; k++)
    if (h->need(k, 0))
      HIP_TRY(hipMemcpyAsync(h->din.as<float2>() + f.plp[k].in_off, in[k], (size_t)f.plp[k].S_if * 8,
                             hipMemcpyHostToDevice, h->ctx.stream));
  L1IO lio{};
  lio.out = h->aux.as<float2>() + AUX_L1PRE + 1840;
  lio.first_frame = h->t2_frame_num;
  lio.nframes = 1;
  HIP_TRY(launch_l1post(h->l1.dev, lio, h->ctx.stream));
  GatherIO io{};
  io.in = h->din.as<float2>();
  io.out = h->dout.as<float2>();
  io.map = h->map.as<int32_t>() + (size_t)(h->frame % f.unit) * f.M;
  io.aux = h->aux.as<float2>();
  io.M = f.M;
  HIP_TRY(launch_gather(io, h->ctx.stream));
  HIP_TRY(hipMemcpyAsync(out, h->dout.p, (size_t)f.M * 8, hipMemcpyDeviceToHost, h->ctx.stream));
  HIP_TRY(hipStreamSynchronize(h->ctx.stream));
  if (consumed)
    for (int k = 0; k < f.nplp; k++) consumed[k] = h->need(k, 0);
  h->t2_frame_num = (h->t2_frame_num + 1) % f.t2frames;
  h->frame++;
  return f.M;
}
extern "C" void dvbt2ll_framemapper_mplp_destroy(dvbt2ll_framemapper_mplp *h) { delete h; }

// ============================================================================ pilotgenp1insert
static PgParams to_pg(const dvbt2ll_pilotgenp1insert_params &p) {
  return PgParams{p.carriermode, p.fftsize, p.pilotpattern, p.guardinterval, p.numdatasyms, p.paprmode, p.version,
                  p.preamble, p.misogroup, p.equalization, p.bandwidth, p.vlength};
}

struct OfdmTables {
  DevBuf map, tw, tw1k, isinc, p1;
  OfdmDev dev{};
  // stored_map: per-symbol rows in the kernel's read order (the chain: ofdm_stored_rows; the pilotgen
  // block's gather mode: natural order)
  int init(const PilotPlan &pp, const std::vector<int32_t> &stored_map, int aux_len, int t2frames) {
    int r;
    if ((r = upload(map, stored_map))) return r;
    if ((r = upload(tw, pp.twiddle)) || (r = upload(tw1k, pp.twiddle1k)) || (r = upload(p1, pp.p1))) return r;
    if (pp.eq && (r = upload(isinc, pp.isinc))) return r;
    dev.bin_map = map.as<int32_t>();
    dev.twiddle = tw.as<float2>();
    dev.twiddle1k = tw1k.as<float2>();
    dev.isinc = pp.eq ? isinc.as<float>() : nullptr;
    dev.p1 = p1.as<float2>();
    dev.N = pp.N; dev.G = pp.G; dev.Nsym = pp.Nsym; dev.aux_len = aux_len; dev.t2frames = t2frames;
    dev.norm = pp.normalization;
    dev.gain = 1.f;
    dev.fmt = DVBT2LL_IQ_CF32;
    return 0;
  }
};

struct dvbt2ll_pilotgenp1insert {
  DeviceCtx ctx;
  PilotPlan plan;
  OfdmTables ofdm;
  DevBuf din, dout;    // din = [aux (pilot values) | one frame of mapped cells]
  int out_items = 0;
};
constexpr int PG_AUX_PAD = 16;
extern "C" int dvbt2ll_pilotgenp1insert_create(const dvbt2ll_pilotgenp1insert_params *p, int device,
                                               dvbt2ll_pilotgenp1insert **out) {
  if (!p || !out) return DVBT2LL_EINVAL;
  *out = nullptr;
  std::unique_ptr<dvbt2ll_pilotgenp1insert> h(new (std::nothrow) dvbt2ll_pilotgenp1insert());
  if (!h) return DVBT2LL_ENOMEM;
  if (build_pilot(to_pg(*p), h->plan)) return DVBT2LL_EINVAL;
  int r = h->ctx.init(device);
  if (r) return r;
  std::vector<cf32> aux(PG_AUX_PAD, cf32{0.f, 0.f});
  for (int i = 0; i < 12; i++) aux[AUX_PILOT0 + i] = h->plan.pilot_values[i];
  if ((r = h->ofdm.init(h->plan, h->plan.bin_map, PG_AUX_PAD, 1))) return r;   // gather rows: natural order
  if (h->din.ensure((size_t)(PG_AUX_PAD + h->plan.active) * 8)) return DVBT2LL_ENOMEM;
  HIP_TRY(hipMemcpy(h->din.p, aux.data(), PG_AUX_PAD * 8, hipMemcpyHostToDevice));
  h->out_items = h->plan.Nsym * (h->plan.N + h->plan.G) + 2048;
  *out = h.release();
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_pilotgenp1insert_output_multiple(const dvbt2ll_pilotgenp1insert *h) { return h ? h->out_items : 0; }
extern "C" int dvbt2ll_pilotgenp1insert_active_items(const dvbt2ll_pilotgenp1insert *h) { return h ? h->plan.active : 0; }
extern "C" int dvbt2ll_pilotgenp1insert_forecast(const dvbt2ll_pilotgenp1insert *h, int nout, int *nin) {
  if (!h || !nin) return DVBT2LL_EINVAL;
  *nin = h->plan.active * (nout / h->out_items);   // pilotgen:1240-1243
  return DVBT2LL_OK;
}
static int pg_run(dvbt2ll_pilotgenp1insert *h, const void *in, void *out, int carriers_only) {
  const PilotPlan &pp = h->plan;
  size_t out_n = carriers_only ? (size_t)pp.Nsym * pp.N : (size_t)h->out_items;
  HIP_TRY(hipSetDevice(h->ctx.device));
  if (h->dout.ensure(out_n * 8)) return DVBT2LL_ENOMEM;
  HIP_TRY(hipMemcpyAsync(h->din.as<float2>() + PG_AUX_PAD, in, (size_t)pp.active * 8, hipMemcpyHostToDevice,
                         h->ctx.stream));
  OfdmIO io{};
  io.data = h->din.as<float2>();
  io.aux_off = 0;
  io.cell_off = PG_AUX_PAD;
  io.cell_stride = (uint32_t)pp.active;
  io.out = h->dout.as<float2>();
  io.out_stride = (int64_t)out_n;
  io.first_frame = 0;
  io.nframes = 1;
  io.carriers_only = carriers_only;
  HIP_TRY(launch_ofdm(h->ofdm.dev, io, h->ctx.stream));
  HIP_TRY(hipMemcpyAsync(out, h->dout.p, out_n * 8, hipMemcpyDeviceToHost, h->ctx.stream));
  HIP_TRY(hipStreamSynchronize(h->ctx.stream));
  return 0;
}
extern "C" int dvbt2ll_pilotgenp1insert_general_work(dvbt2ll_pilotgenp1insert *h, int nout, int nin, const void *in,
                                                     void *out, int *consumed) {
  if (!h || nout < 0 || (nout && (!in || !out))) return DVBT2LL_EINVAL;
  if (consumed) *consumed = 0;
  if (nout < h->out_items) return 0;
  if (nin < h->plan.active) return DVBT2LL_ESHORT;
  int r = pg_run(h, in, out, 0);   // one T2 frame per call (pilotgen:2903)
  if (r) return r;
  if (consumed) *consumed = h->plan.active;
  return h->out_items;
}
extern "C" int dvbt2ll_pilotgenp1insert_debug_carriers(dvbt2ll_pilotgenp1insert *h, const void *in, void *carriers) {
  if (!h || !in || !carriers) return DVBT2LL_EINVAL;
  return pg_run(h, in, carriers, 1);
}
extern "C" void dvbt2ll_pilotgenp1insert_destroy(dvbt2ll_pilotgenp1insert *h) { delete h; }

// ============================================================================ chain
// One PLP of the fused chain: its FEC and map tables, the cell-interleaver / time-interleaver store
// tables, and per buffer slot its packed codewords and BCH parities.  A single-PLP chain (the
// reference's frame) has one.
struct ChainPlp {
  FecTables fec;
  MapTables map;
  DevBuf part, pbase, poff, pnq;
  DevBuf cw[DVBT2LL_CHAIN_MAX_SLOTS], bpart[DVBT2LL_CHAIN_MAX_SLOTS];
  int64_t cw_stride = 0;
  int64_t ts_per_frame = 0;   // payload bytes per interleaving frame (NM positions; HEM: before sync-byte removal)
  int pay = 0, F = 0, inputmode = 0, inband = 0;
  int P = 1;                  // T2 frames per interleaving frame (TIME_IL_TYPE 1: P_I); F, ts_per_frame are per
                              // interleaving frame
  int cyc = 1;                // T2 frames from one interleaving frame to the next (P_I x FRAME_INTERVAL)
  int64_t blocks(int64_t frames) const { return (frames + cyc - 1) / cyc * F; }   // FEC blocks of `frames` T2 frames
};

// instantiated hipGraphs of the chain's kernels (per PLP: FEC BB pass, BCH matrix-core pass; per PLP: LDPC +
// map (PLP 0's launch also generates the L1-post); OFDM) for one (nframes, IQ format, slot),
// captured once from the ordinary launch path into a ring of instantiations.  A call takes the next
// ring entry, waits for it only if it is still in flight, rewrites its kernel nodes' arguments
// (hipGraphExecKernelNodeSetParams) and launches it.
struct ChainGraph {
  int nframes = 0, fmt = -1, slot = -1;
  hipGraph_t graph = nullptr;
  std::vector<hipGraphNode_t> node;            // kernel nodes in launch order
  std::vector<hipKernelNodeParams> base;
  hipGraphExec_t exec[DVBT2LL_CHAIN_GRAPH_RING] = {};
  hipEvent_t done[DVBT2LL_CHAIN_GRAPH_RING] = {};
  bool used[DVBT2LL_CHAIN_GRAPH_RING] = {};
  // the argument bytes each instantiation's kernel nodes hold: a call whose arguments match skips
  // hipGraphExecKernelNodeSetParams (one per node, the bulk of a graph call's host time)
  std::vector<std::vector<uint8_t>> held[DVBT2LL_CHAIN_GRAPH_RING];
  int next = 0;
  ~ChainGraph() {
    for (auto &e : exec)
      if (e) (void)hipGraphExecDestroy(e);
    for (auto &e : done)
      if (e) (void)hipEventDestroy(e);
    if (graph) (void)hipGraphDestroy(graph);
  }
};

// the asynchronous host path (dvbt2ll_chain_host_submit): a ring of submissions, each with its own device TS
// and IQ buffers and three events; the TS copy-in, the kernels and the IQ copy-out of a submission run on
// three streams ordered by those events, so consecutive submissions overlap (copy-in of k + 1 and copy-out
// of k - 1 beside the kernels of k)
struct HostRing {
  hipStream_t in = nullptr, comp = nullptr, out = nullptr;
  struct Entry {
    DevBuf ts, iq;
    hipEvent_t h2d = nullptr, kern = nullptr, d2h = nullptr;
    int64_t ticket = -1;   // the submission holding the entry (-1: never used)
  } e[DVBT2LL_HOST_RING];
  int64_t next_ticket = 0;
  int init(int device) {
    if (in) return 0;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipStreamCreateWithFlags(&in, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&comp, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&out, hipStreamNonBlocking));
    for (auto &x : e) {
      HIP_TRY(hipEventCreateWithFlags(&x.h2d, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&x.kern, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&x.d2h, hipEventDisableTiming));
    }
    return 0;
  }
  hipError_t synchronize() const {
    for (hipStream_t st : {in, comp, out})
      if (st) {
        hipError_t r = hipStreamSynchronize(st);
        if (r != hipSuccess) return r;
      }
    return hipSuccess;
  }
  ~HostRing() {
    (void)synchronize();   // no copy or kernel of a submission may outlive the entries' buffers
    for (auto &x : e)
      for (hipEvent_t ev : {x.h2d, x.kern, x.d2h})
        if (ev) (void)hipEventDestroy(ev);
    for (hipStream_t st : {in, comp, out})
      if (st) (void)hipStreamDestroy(st);
  }
};

struct dvbt2ll_chain {
  DeviceCtx ctx;
  HostRing host;
  dvbt2ll_chain_params p{};   // single-PLP create parameters (PLP 0's for a multi-PLP chain)
  int nplp = 1;
  std::vector<std::unique_ptr<ChainPlp>> plps;
  FramePlan frame;
  PilotPlan pilot;
  OfdmTables ofdm;
  DevBuf aux, inv, sym_d0, sym_n, sym_n0, ts_tmp, iq_tmp;
  DevBuf ts_plp_tmp[DVBT2LL_MAX_PLP];   // run_plps_host: each PLP's TS on the device
  DevBuf abin, aval, aind, agrp, azr;   // non-data bins as compact lists (t2_plan.h AuxLists)
  DevBuf plp_bnd, plp_qbase, qam_all;   // multi-PLP frames: slot ranges per PLP, the PLPs' constellations
  DevBuf cls_inv;                       // per frame class: its data slots' bins at inv + cls_inv[c]
  std::vector<int32_t> plp_bnd_host;
  std::vector<int> qbase_host;
  DevBuf sync_err;                      // TS sync bytes != 0x47 consumed by run calls (bbheader:675, 703)
  // intermediate buffer slots (index pairs, L1-post cells; the PLPs' codewords): run calls take them
  // round-robin, so calls issued on different streams overlap; a slot reused on another stream first
  // waits for its previous run (slot_done) -- see dvbt2ll_chain_set_slots
  DevBuf pairs[DVBT2LL_CHAIN_MAX_SLOTS];
  // per-frame L1-post cells of a run (l1post_kernel -> the OFDM kernel's indirect aux entries)
  L1Tables l1;
  DevBuf l1buf[DVBT2LL_CHAIN_MAX_SLOTS];
  uint32_t l1_stride = 0;
  hipEvent_t slot_done[DVBT2LL_CHAIN_MAX_SLOTS] = {};
  hipStream_t slot_stream[DVBT2LL_CHAIN_MAX_SLOTS] = {};
  // test hook (dvbt2ll_chain_debug_keep_codewords): runs also store the codewords; per slot, whether its
  // last run did
  bool keep_cw = false;
  bool cw_kept[DVBT2LL_CHAIN_MAX_SLOTS] = {};
  bool slot_used[DVBT2LL_CHAIN_MAX_SLOTS] = {};
  // a run on the slot failed after its FEC pass may have run: its BCH partial parities are not known to be zero
  bool bpart_dirty[DVBT2LL_CHAIN_MAX_SLOTS] = {};
  int nslots = 1, next_slot = 0, last_slot = 0;
  // hipGraph mode (dvbt2ll_chain_set_graph)
  bool use_graph = false;
  hipStream_t cap_stream = nullptr;
  std::vector<std::unique_ptr<ChainGraph>> graphs;
  int max_frames = 0;
  int64_t pair_stride = 0;   // pairs buffer: frame k's slots at k * pair_stride (multiple of 8)
  int64_t iq_per_frame = 0;
  // stage timing: 4 events per run (start, after fec, after map + L1-post, after ofdm) recorded
  // on the launch stream without host synchronisation; folded into ms[] by get_timing()
  // (stages 0 fec, 1 map, 2 ofdm; stage 3 is reserved and stays 0)
  static constexpr int NEV = 4;
  bool timing = false;
  std::vector<hipEvent_t> evpool;
  size_t evused = 0;
  double ms[4] = {0, 0, 0, 0};
  int64_t launches[4] = {0, 0, 0, 0};
  hipEvent_t next_event() {
    if (evused == evpool.size()) {
      hipEvent_t e = nullptr;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      evpool.push_back(e);
    }
    return evpool[evused++];
  }
  // every run's end event is waited on (runs may sit on several streams, so the last recorded
  // event does not imply the earlier ones); the pool is emptied even when a query fails
  int fold_timing() {
    if (!evused) return 0;
    int st = 0;
    static const int stage_of[NEV - 1] = {0, 1, 2};   // event interval k -> stage
    for (size_t b = 0; b + NEV - 1 < evused && !st; b += NEV) {
      hipError_t e = hipEventSynchronize(evpool[b + NEV - 1]);
      for (int k = 0; k < NEV - 1 && e == hipSuccess; k++) {
        float t = 0;
        e = hipEventElapsedTime(&t, evpool[b + k], evpool[b + k + 1]);
        if (e == hipSuccess) {
          ms[stage_of[k]] += t;
          launches[stage_of[k]] += 1;
        }
      }
      if (e != hipSuccess) {
        last_hip_error() = e;
        st = DVBT2LL_EDEVICE;
      }
    }
    evused = 0;
    return st;
  }
  // the chain's kernels on stream s: every PLP's BB + matrix-core BCH passes, every PLP's LDPC + map
  // (PLP 0's launch has the extra workgroups that generate the frames' L1-post cells), OFDM.  ev1, ev2
  // (timing): recorded after the BB + BCH passes and after the LDPC + map kernels
  hipError_t launch_chain(const L1IO &lio, const FecIO *fio, const MapIO *mio, const OfdmIO &oio, hipStream_t s,
                          hipEvent_t ev1, hipEvent_t ev2) {
    hipError_t e = hipSuccess;
    for (int k = 0; k < nplp && e == hipSuccess; k++) e = launch_fec(FEC_TS_TO_BBFRAME, plps[k]->fec.dev, fio[k], s);
    if (e == hipSuccess && ev1) e = hipEventRecord(ev1, s);
    for (int k = 0; k < nplp && e == hipSuccess; k++)
      e = k == 0 ? launch_ldpc_map(plps[k]->fec.dev, fio[k], plps[k]->map.dev, mio[k], s, &l1.dev, &lio)
                 : launch_ldpc_map(plps[k]->fec.dev, fio[k], plps[k]->map.dev, mio[k], s);
    if (e == hipSuccess && ev2) e = hipEventRecord(ev2, s);
    if (e == hipSuccess) e = launch_ofdm(ofdm.dev, oio, s);
    return e;
  }
  // kernel nodes per run: the fused BB + BCH pass and the LDPC + map kernel per PLP, one OFDM
  int graph_nodes() const { return 2 * nplp + 1; }
  int graph_launch(const L1IO &lio, const FecIO *fio, const MapIO *mio, const OfdmIO &oio, int nframes, int slot,
                   hipStream_t s) {
    const int nk = graph_nodes();
    ChainGraph *g = nullptr;
    for (auto &c : graphs)
      if (c->nframes == nframes && c->fmt == ofdm.dev.fmt && c->slot == slot) g = c.get();
    if (!g) {
      if (!cap_stream) HIP_TRY(hipStreamCreateWithFlags(&cap_stream, hipStreamNonBlocking));
      std::unique_ptr<ChainGraph> c(new (std::nothrow) ChainGraph());
      if (!c) return DVBT2LL_ENOMEM;
      c->nframes = nframes;
      c->fmt = ofdm.dev.fmt;
      c->slot = slot;
      HIP_TRY(hipStreamBeginCapture(cap_stream, hipStreamCaptureModeThreadLocal));
      hipError_t e1 = launch_chain(lio, fio, mio, oio, cap_stream, nullptr, nullptr);
      hipError_t ec = hipStreamEndCapture(cap_stream, &c->graph);
      HIP_TRY(e1);
      HIP_TRY(ec);
      // the kernel nodes in dependency order: a linear chain of nk
      size_t n = 0;
      HIP_TRY(hipGraphGetNodes(c->graph, nullptr, &n));
      std::vector<hipGraphNode_t> nodes(n);
      HIP_TRY(hipGraphGetNodes(c->graph, nodes.data(), &n));
      std::vector<hipGraphNode_t> kn;
      for (auto nd : nodes) {
        hipGraphNodeType t;
        HIP_TRY(hipGraphNodeGetType(nd, &t));
        if (t == hipGraphNodeTypeKernel) kn.push_back(nd);
      }
      if ((int)kn.size() != nk) return DVBT2LL_EDEVICE;
      c->node.assign(nk, nullptr);
      c->base.assign(nk, hipKernelNodeParams{});
      // order: the root (no dependencies), then the node depending on it, and so on
      hipGraphNode_t prev = nullptr;
      for (int k = 0; k < nk; k++) {
        for (auto nd : kn) {
          size_t nd_n = 0;
          HIP_TRY(hipGraphNodeGetDependencies(nd, nullptr, &nd_n));
          bool ok = false;
          if (k == 0) {
            ok = nd_n == 0;
          } else if (nd_n == 1) {
            hipGraphNode_t dep = nullptr;
            size_t one = 1;
            HIP_TRY(hipGraphNodeGetDependencies(nd, &dep, &one));
            ok = dep == prev;
          }
          if (ok) { c->node[k] = nd; break; }
        }
        if (!c->node[k]) return DVBT2LL_EDEVICE;
        prev = c->node[k];
        HIP_TRY(hipGraphKernelNodeGetParams(c->node[k], &c->base[k]));
      }
      for (int r = 0; r < DVBT2LL_CHAIN_GRAPH_RING; r++) {
        HIP_TRY(hipGraphInstantiate(&c->exec[r], c->graph, nullptr, nullptr, 0));
        HIP_TRY(hipEventCreateWithFlags(&c->done[r], hipEventDisableTiming));
      }
      g = c.get();
      graphs.push_back(std::move(c));
    }
    // the ring's next instantiation; the host waits only if it is still in flight (every entry of
    // the ring is), so consecutive calls never wait for each other below that depth
    const int r = g->next;
    g->next = (r + 1) % DVBT2LL_CHAIN_GRAPH_RING;
    if (g->used[r]) HIP_TRY(hipEventSynchronize(g->done[r]));
    L1Dev ld = l1.dev, ld0{};   // PLP 0's map launch generates the L1-post, the others carry none
    L1IO li = lio, li0{};
    OfdmDev od = ofdm.dev;
    OfdmIO oi = oio;
    std::vector<FecDev> fd(nplp);
    std::vector<FecIO> fi(fio, fio + nplp);
    std::vector<MapDev> md(nplp);
    std::vector<MapIO> mi(mio, mio + nplp);
    std::vector<std::vector<void *>> args;
    for (int k = 0; k < nplp; k++) {
      fd[k] = plps[k]->fec.dev;
      md[k] = plps[k]->map.dev;
    }
    for (int k = 0; k < nplp; k++) args.push_back({&fd[k], &fi[k]});
    for (int k = 0; k < nplp; k++) args.push_back({&fd[k], &fi[k], &md[k], &mi[k], k ? &ld0 : &ld, k ? &li0 : &li});
    args.push_back({&od, &oi});
    std::vector<std::vector<size_t>> sizes;
    for (int k = 0; k < nplp; k++) sizes.push_back({sizeof(FecDev), sizeof(FecIO)});
    for (int k = 0; k < nplp; k++)
      sizes.push_back({sizeof(FecDev), sizeof(FecIO), sizeof(MapDev), sizeof(MapIO), sizeof(L1Dev), sizeof(L1IO)});
    sizes.push_back({sizeof(OfdmDev), sizeof(OfdmIO)});
    if (g->held[r].size() != (size_t)nk) g->held[r].assign(nk, {});
    for (int k = 0; k < nk; k++) {
      std::vector<uint8_t> bytes;
      for (size_t a = 0; a < args[k].size(); a++) {
        const uint8_t *b = (const uint8_t *)args[k][a];
        bytes.insert(bytes.end(), b, b + sizes[k][a]);
      }
      if (bytes == g->held[r][k]) continue;
      hipKernelNodeParams p = g->base[k];
      p.kernelParams = args[k].data();
      p.extra = nullptr;
      g->held[r][k].clear();   // unknown until the update succeeds
      HIP_TRY(hipGraphExecKernelNodeSetParams(g->exec[r], g->node[k], &p));
      g->held[r][k] = std::move(bytes);
    }
    HIP_TRY(hipGraphLaunch(g->exec[r], s));
    HIP_TRY(hipEventRecord(g->done[r], s));
    g->used[r] = true;
    return 0;
  }
  int alloc_slot(int k) {
    for (auto &pl : plps) {
      // one spare row past the largest launch: the fused FEC pass stores its dead lanes' pieces there
      if (pl->cw[k].ensure((size_t)(pl->blocks(max_frames) + 1) * pl->cw_stride) ||
          pl->bpart[k].ensure((size_t)pl->blocks(max_frames) * BCH_PART_WORDS * sizeof(uint32_t)))
        return DVBT2LL_ENOMEM;
      // the BCH partial parities start at zero (bbch_kernel XORs into them, ldpc_map_kernel zeroes what it reads)
      HIP_TRY(hipMemset(pl->bpart[k].p, 0, pl->bpart[k].n));
    }
    bpart_dirty[k] = false;
    if (pairs[k].ensure((size_t)pair_stride * max_frames * 2) || l1buf[k].ensure((size_t)l1_stride * max_frames * 8))
      return DVBT2LL_ENOMEM;
    if (!slot_done[k]) HIP_TRY(hipEventCreateWithFlags(&slot_done[k], hipEventDisableTiming));
    return 0;
  }
  ~dvbt2ll_chain() {
    // every run still in flight (the ring's streams, the slots' last runs on caller streams) ends before
    // the slot buffers and ring entries are freed
    (void)host.synchronize();
    for (int k = 0; k < DVBT2LL_CHAIN_MAX_SLOTS; k++)
      if (slot_used[k] && slot_done[k]) (void)hipEventSynchronize(slot_done[k]);
    graphs.clear();
    if (cap_stream) (void)hipStreamDestroy(cap_stream);
    for (auto &e : evpool)
      if (e) (void)hipEventDestroy(e);
    for (auto &e : slot_done)
      if (e) (void)hipEventDestroy(e);
  }
};

// the common construction of single- and multi-PLP chains: fm's common fields with plps' PLPs
static int chain_build(dvbt2ll_chain *h, const FmParams &fm, const std::vector<PlpParams> &plps,
                       const std::vector<int> &tsrate, int misogroup, int equalization, int bandwidth, int device,
                       int nss = 1) {
  PgParams pg{fm.carriermode, fm.fftsize, fm.pilotpattern, fm.guardinterval, fm.numdatasyms, fm.paprmode, fm.version,
              fm.preamble, misogroup, equalization, bandwidth, fft_points(fm.fftsize)};
  if (build_frame_mplp(fm, plps, h->frame, false, nss) || build_pilot(pg, h->pilot)) return DVBT2LL_EINVAL;
  if (h->pilot.active != h->frame.M) return DVBT2LL_EINVAL;
  const FramePlan &fp = h->frame;
  if (h->max_frames < fp.unit) return DVBT2LL_EINVAL;   // runs cover whole interleaving frames
  h->nplp = fp.nplp;
  h->pair_stride = ((int64_t)fp.S + 7) / 8 * 8;
  int r = h->ctx.init(device);
  if (r) return r;
  // OFDM side: aux bins from cmap, data cells streamed per symbol and scattered through inv
  // one layout per frame class (FRAME_INTERVAL > 1: the T2 frames carry different PLPs); class 0's is `layout`
  std::vector<ChainLayout> layouts(fp.ncls);
  for (int c = 0; c < fp.ncls; c++)
    if (build_chain_layout(fp, h->pilot, layouts[c], c)) return DVBT2LL_EINVAL;
  const ChainLayout &layout = layouts[0];
  int nq = 0;   // the PLPs' constellation tables back to back (multi-PLP); 256 entries for one PLP
  std::vector<cf32> qall;
  for (int k = 0; k < h->nplp; k++) {
    const PlpParams &q = plps[k];
    std::unique_ptr<ChainPlp> pl(new (std::nothrow) ChainPlp());
    if (!pl) return DVBT2LL_ENOMEM;
    const PlpPlan &pp = fp.plp[k];
    if ((r = pl->fec.init(q.framesize, q.rate, q.constellation, q.inputmode, q.inband, q.fecblocks, tsrate[k])))
      return r;
    // one PLP of several: multiple input streams, ISI = the PLP_ID (bbheader:288-298)
    if (h->nplp > 1) pl->fec.dev.matype = MATYPE_MIS | k;
    if ((r = pl->fec.init_chain())) return r;
    if ((r = pl->map.init(q.framesize, q.rate, q.constellation, q.rotation, pl->fec.plan))) return r;
    MapDev &md = pl->map.dev;
    // the quad table covers one launch unit (fp.unit T2 frames): rows r' = m' F + r for the unit's
    // interleaving frames m' < fp.unit / cycle and their FEC blocks r
    const int nif = fp.unit / pp.cycle(), Fu = pp.F * nif;
    md.F = Fu;
    if (pp.cs > 0x7FFF) return DVBT2LL_EINVAL;   // 15-bit cell indices in the quad table (<= 32400)
    // the LDPC + map kernel's cell interleaver + TI store in stored-slot order (layout.part: frame data slot
    // of each frame data index; a TIME_IL_TYPE 1 PLP's block r writes the P_I T2 frames of its interleaving
    // frame, frame i's slots at i * pair_stride), in aligned quads of four slots: block r's quads sorted by
    // slot, each with the cell-interleaver input index of the cell landing in each of its four slots (j with
    // (ci_perm[j] + ci_shift[r]) mod cs = t, framemapper:1973-1998; 0x8000: a slot of another block, at a
    // run's edge), its offset from its 64-quad chunk's first quad, each chunk's first quad and the block's
    // quad count.  A full quad is one 8-byte store, so a store instruction writes 512 B of one or two
    // contiguous runs (the block's cells in a symbol (half) are one run, bank-balanced inside, t2_plan
    // build_chain_layout).  A chunk whose quads would span more than 0xFFFF quads (a block's cells in two
    // T2 frames) ends early: the rest of its 64 entries are empty quads (no store).
    std::vector<std::vector<std::pair<int64_t, int>>> blk(Fu);
    std::vector<std::vector<int>> qpos(Fu);   // per block: its quads' entry index (with the chunk padding)
    int qmax = 0;
    std::vector<std::pair<int64_t, int>> cells(pp.cs);
    std::vector<int> jin(pp.cs);   // cell-interleaver input index of each output position t
    for (int rr = 0; rr < Fu; rr++) {
      const int r = rr % pp.F, f0 = rr / pp.F * pp.cycle();
      for (int j = 0; j < pp.cs; j++) jin[(pp.ci_perm[j] + pp.ci_shift[r]) % pp.cs] = j;
      for (int t = 0; t < pp.cs; t++) {
        const CellDest cd = cell_dest(fp, k, r, t, f0);
        const int fu = f0 + cd.off;   // T2 frame of the unit, of class fu mod ncls
        cells[t] = {(int64_t)fu * h->pair_stride + layouts[fu % fp.ncls].part[cd.pos], jin[t]};
      }
      std::sort(cells.begin(), cells.end());
      auto &qv = blk[rr];   // (quad index, slot-in-quad | t << 2) per cell
      for (auto &c : cells) qv.push_back({c.first >> 2, (int)(c.first & 3) | (c.second << 2)});
      int n = -1;
      int64_t qprev = -1, cbase = 0;
      for (auto &c : qv) {
        if (c.first == qprev) continue;
        qprev = c.first;
        ++n;
        if (n % 64 && c.first - cbase > 0xFFFF) n = (n + 63) & ~63;   // start a new chunk here
        if (n % 64 == 0) cbase = c.first;
        qpos[rr].push_back(n);
      }
      qmax = std::max(qmax, n + 1);
    }
    const int qst = (qmax + 63) & ~63, nchk = qst / 64;
    std::vector<uint32_t> qsrc((size_t)Fu * qst * 2 + 2, 0x80008000u);
    std::vector<uint16_t> qoff((size_t)Fu * qst + 4, 0);
    std::vector<int32_t> qb((size_t)Fu * nchk + 1, 0), qn(Fu, 0);
    for (int rr = 0; rr < Fu; rr++) {
      int n = -1, qi = -1;
      int64_t qprev = -1, cbase = 0;
      for (auto &c : blk[rr]) {
        if (c.first != qprev) {
          qprev = c.first;
          n = qpos[rr][++qi];
          if (n % 64 == 0) {
            cbase = c.first;
            if (cbase > INT32_MAX) return DVBT2LL_EINVAL;
            qb[(size_t)rr * nchk + n / 64] = (int32_t)cbase;
          }
          if (c.first - cbase > 0xFFFF) return DVBT2LL_EINVAL;
          qoff[(size_t)rr * qst + n] = (uint16_t)(c.first - cbase);
        }
        const int sl = c.second & 3, t = c.second >> 2;
        uint32_t &w = qsrc[((size_t)rr * qst + n) * 2 + (sl >> 1)];
        w = (w & ~(0xFFFFu << (16 * (sl & 1)))) | ((uint32_t)t << (16 * (sl & 1)));
      }
      qn[rr] = n + 1;
    }
    if ((r = upload(pl->part, qsrc)) || (r = upload(pl->pbase, qb)) || (r = upload(pl->poff, qoff)) ||
        (r = upload(pl->pnq, qn)))
      return r;
    md.slot_quad = pl->part.as<uint2>();
    md.slot_qoff = pl->poff.as<uint16_t>();
    md.slot_qbase = pl->pbase.as<int32_t>();
    md.slot_nq = pl->pnq.as<int32_t>();
    md.slot_stride = qst;
    pl->F = pp.F;
    pl->P = pp.P;
    pl->cyc = pp.cycle();
    pl->inputmode = q.inputmode;
    pl->inband = q.inband;
    pl->cw_stride = ((pl->fec.plan.nldpc / 8) + 255) / 256 * 256;
    pl->pay = (pl->fec.plan.kbch - 80) / 8;
    // payload bytes per interleaving frame: in-band type B takes 13 bytes of its first BBFRAME
    // (bbheader:327-355, fec_block == 0)
    pl->ts_per_frame = (int64_t)pp.F * pl->pay - (q.inband ? 13 : 0);
    // PLPs with the same constellation and rotation share one table (their LUTs are equal)
    int qb0 = -1;
    for (int k2 = 0; k2 < k && qb0 < 0; k2++)
      if (plps[k2].constellation == q.constellation && plps[k2].rotation == q.rotation) qb0 = h->qbase_host[k2];
    if (qb0 < 0) {
      qb0 = nq;
      const int entries = 1 << pl->map.plan.mod;
      for (int i = 0; i < entries; i++) qall.push_back(pl->map.plan.lut[i]);
      nq += entries;
    }
    h->qbase_host.push_back(qb0);
    h->plps.push_back(std::move(pl));
  }
  // stored bins -> padded LDS slots within their half (the kernel writes them as they are), the frame classes'
  // tables back to back (each class's bins from an 8-slot boundary: the kernel reads aligned quads / octets)
  const int nsub_h = ofdm_split(h->pilot.N) ? h->pilot.N / 2 : h->pilot.N;
  std::vector<uint16_t> inv_pad;
  std::vector<int32_t> cls_inv, sd0, sdn, sdn0, bnd_all;
  for (const ChainLayout &lc : layouts) {
    cls_inv.push_back((int32_t)inv_pad.size());
    for (size_t si = 0; si < lc.inv.size(); si++)
      inv_pad.push_back((uint16_t)ofdm_padded_bin(h->pilot.N, lc.inv[si] % nsub_h));
    inv_pad.resize(((inv_pad.size() + 7) & ~(size_t)7) + 8, 0);
    sd0.insert(sd0.end(), lc.sym_d0.begin(), lc.sym_d0.end());
    sdn.insert(sdn.end(), lc.sym_n.begin(), lc.sym_n.end());
    sdn0.insert(sdn0.end(), lc.sym_n0.begin(), lc.sym_n0.end());
    bnd_all.insert(bnd_all.end(), lc.plp_bnd.begin(), lc.plp_bnd.end());
  }
  if ((r = upload(h->inv, inv_pad)) || (r = upload(h->sym_d0, sd0)) || (r = upload(h->sym_n, sdn)) ||
      (r = upload(h->sym_n0, sdn0)) || (r = upload(h->cls_inv, cls_inv)))
    return r;
  const PilotPlan &pp = h->pilot;
  // one aux row (pilot values, L1-pre, dummy cells): the L1-post cells come per frame from the GPU
  std::vector<cf32> auxv = fp.aux;
  for (int i = 0; i < 12; i++) auxv[AUX_PILOT0 + i] = pp.pilot_values[i];
  if ((r = h->ofdm.init(pp, layout.cmap, fp.aux_len, 1))) return r;
  // the classes' aux lists back to back (a class's dummy cells differ), group offsets rebased
  AuxLists al;
  for (const ChainLayout &lc : layouts) {
    AuxLists ac;
    if (build_aux_lists(lc, pp.N, pp.Nsym, auxv, fp.aux_len, 1, ac, AUX_L1PRE + 1840, fp.Lp)) return DVBT2LL_EINVAL;
    if (ac.dbin.size() % 4) return DVBT2LL_EINVAL;   // groups of direct quads stay aligned
    for (size_t g = 0; g + 3 < ac.grp.size(); g += 4) {
      ac.grp[g] += (int32_t)al.dbin.size();
      ac.grp[g + 2] += (int32_t)al.ind.size();
    }
    al.dbin.insert(al.dbin.end(), ac.dbin.begin(), ac.dbin.end());
    al.dval.insert(al.dval.end(), ac.dval.begin(), ac.dval.end());
    al.ind.insert(al.ind.end(), ac.ind.begin(), ac.ind.end());
    al.grp.insert(al.grp.end(), ac.grp.begin(), ac.grp.end());
    al.zrun.insert(al.zrun.end(), ac.zrun.begin(), ac.zrun.end());
  }
  if ((r = h->l1.init(fp))) return r;
  h->l1_stride = (uint32_t)((fp.Lp + 3) & ~3);
  for (auto &b : al.dbin)
    if (b != 0xFFFF) b = (uint16_t)ofdm_padded_bin(pp.N, b);
  for (auto &e : al.ind) e = ofdm_padded_bin(pp.N, e & 0x7FFFu) | (e & ~0x7FFFu);
  std::vector<int32_t> zr(al.zrun.size());   // zero runs as padded slot ranges
  for (size_t g = 0; g + 1 < al.zrun.size(); g += 2) {
    const int z0 = al.zrun[g], z1 = al.zrun[g + 1];
    zr[g] = z1 > z0 ? (int32_t)ofdm_padded_bin(pp.N, (uint32_t)z0) : 0;
    zr[g + 1] = z1 > z0 ? (int32_t)ofdm_padded_bin(pp.N, (uint32_t)(z1 - 1)) + 1 : 0;
  }
  al.ind.push_back(0);   // never empty (device pointer)
  al.dbin.resize(al.dbin.size() + 4, 0xFFFF);
  al.dval.resize(al.dval.size() + 4, cf32{0.f, 0.f});
  if ((r = upload(h->abin, al.dbin)) || (r = upload(h->aval, al.dval)) || (r = upload(h->aind, al.ind)) ||
      (r = upload(h->agrp, al.grp)) || (r = upload(h->azr, zr)))
    return r;
  OfdmDev &od = h->ofdm.dev;
  od.abin = h->abin.as<uint16_t>();
  od.aval = h->aval.as<float2>();
  od.aind = h->aind.as<uint32_t>();
  od.agrp = h->agrp.as<int4>();
  od.azr = h->azr.as<int2>();
  od.inv = h->inv.as<uint16_t>();
  od.sym_d0 = h->sym_d0.as<int32_t>();
  od.sym_n = h->sym_n.as<int32_t>();
  od.sym_n0 = h->sym_n0.as<int32_t>();
  od.ncls = fp.ncls;
  od.cls_inv = h->cls_inv.as<int32_t>();
  od.nplp = h->nplp;
  if (h->nplp == 1) {
    od.qam = h->plps[0]->map.dev.lut;   // the 256-entry table (entries past the constellation are zero)
    od.nq = 256;
  } else {
    if (nq > OFDM_MAX_QAM) return DVBT2LL_EINVAL;
    h->plp_bnd_host = layout.plp_bnd;   // class 0's (the debug hook's frame 0)
    std::vector<int32_t> qb(h->qbase_host.begin(), h->qbase_host.end());
    if ((r = upload(h->qam_all, qall)) || (r = upload(h->plp_bnd, bnd_all)) || (r = upload(h->plp_qbase, qb)))
      return r;
    od.qam = h->qam_all.as<float2>();
    od.nq = nq;
    od.plp_bnd = h->plp_bnd.as<int32_t>();
    od.plp_qbase = h->plp_qbase.as<int32_t>();
  }
  h->iq_per_frame = (int64_t)pp.Nsym * (pp.N + pp.G) + 2048;
  // the OFDM kernel addresses index pairs and aux cells with 32-bit byte offsets
  if ((uint64_t)h->pair_stride * h->max_frames * 2 >= (1ull << 32) || auxv.size() * 8 >= (1ull << 32) ||
      (uint64_t)h->l1_stride * h->max_frames * 8 >= (1ull << 32))
    return DVBT2LL_EINVAL;
  if ((r = h->alloc_slot(0))) return r;
  if ((r = upload(h->aux, auxv))) return r;
  if (h->sync_err.ensure(4)) return DVBT2LL_ENOMEM;
  HIP_TRY(hipMemset(h->sync_err.p, 0, 4));
  return 0;
}

extern "C" int dvbt2ll_chain_create(const dvbt2ll_chain_params *p, int device, dvbt2ll_chain **out) {
  if (!p || !out || p->max_frames < 1) return DVBT2LL_EINVAL;
  *out = nullptr;
  const dvbt2ll_framemapperfint_params &f = p->fm;
  std::unique_ptr<dvbt2ll_chain> h(new (std::nothrow) dvbt2ll_chain());
  if (!h) return DVBT2LL_ENOMEM;
  h->p = *p;
  h->max_frames = p->max_frames;
  const PlpParams one{f.framesize, f.rate, f.constellation, f.rotation, f.fecblocks, f.tiblocks, f.inputmode, f.inband};
  int r = chain_build(h.get(), to_fm(f), {one}, {p->tsrate}, p->misogroup, p->equalization, p->bandwidth, device);
  if (r) return r;
  *out = h.release();
  return DVBT2LL_OK;
}

static bool mplp_to_plan(const dvbt2ll_mplp_params &m, FmParams &fm, std::vector<PlpParams> &plps,
                         std::vector<int> &tsrate, int *nss) {
  if (m.nplp < 1 || m.nplp > DVBT2LL_MAX_PLP) return false;
  const dvbt2ll_plp_params &q0 = m.plp[0];
  fm = FmParams{q0.framesize, q0.rate, q0.constellation, q0.rotation, q0.fecblocks, q0.tiblocks, m.carriermode,
                m.fftsize, m.guardinterval, m.l1constellation, m.pilotpattern, m.t2frames, m.numdatasyms, m.paprmode,
                m.version, m.preamble, q0.inputmode, m.reservedbiasbits, m.l1scrambled, q0.inband};
  plps.clear();
  tsrate.clear();
  for (int k = 0; k < m.nplp; k++) {
    const dvbt2ll_plp_params &q = m.plp[k];
    plps.push_back(PlpParams{q.framesize, q.rate, q.constellation, q.rotation, q.fecblocks, q.tiblocks, q.inputmode,
                             q.inband, q.plp_type, q.ti_type, q.ti_frames, q.frame_interval, q.first_frame_idx});
    tsrate.push_back(q.tsrate);
  }
  *nss = m.num_subslices;
  return true;
}

extern "C" int dvbt2ll_chain_create_mplp(const dvbt2ll_mplp_chain_params *p, int device, dvbt2ll_chain **out) {
  if (!p || !out || p->max_frames < 1) return DVBT2LL_EINVAL;
  *out = nullptr;
  FmParams fm;
  std::vector<PlpParams> plps;
  std::vector<int> tsrate;
  int nss = 1;
  if (!mplp_to_plan(p->fm, fm, plps, tsrate, &nss)) return DVBT2LL_EINVAL;
  std::unique_ptr<dvbt2ll_chain> h(new (std::nothrow) dvbt2ll_chain());
  if (!h) return DVBT2LL_ENOMEM;
  h->max_frames = p->max_frames;
  const dvbt2ll_plp_params &q0 = p->fm.plp[0];
  h->p.fm = dvbt2ll_framemapperfint_params{q0.framesize, q0.rate, q0.constellation, q0.rotation, q0.fecblocks,
                                           q0.tiblocks, fm.carriermode, fm.fftsize, fm.guardinterval,
                                           fm.l1constellation, fm.pilotpattern, fm.t2frames, fm.numdatasyms,
                                           fm.paprmode, fm.version, fm.preamble, q0.inputmode, fm.reservedbiasbits,
                                           fm.l1scrambled, q0.inband};
  h->p.misogroup = p->misogroup;
  h->p.equalization = p->equalization;
  h->p.bandwidth = p->bandwidth;
  h->p.max_frames = p->max_frames;
  h->p.tsrate = q0.tsrate;
  int r = chain_build(h.get(), fm, plps, tsrate, p->misogroup, p->equalization, p->bandwidth, device, nss);
  if (r) return r;
  *out = h.release();
  return DVBT2LL_OK;
}

extern "C" int dvbt2ll_chain_unit_frames(const dvbt2ll_chain *h) { return h ? h->frame.unit : 0; }

extern "C" int dvbt2ll_chain_num_plps(const dvbt2ll_chain *h) { return h ? h->nplp : 0; }

extern "C" int dvbt2ll_chain_get_plp_info(const dvbt2ll_chain *h, int plp, dvbt2ll_chain_info *info) {
  if (!h || !info || plp < 0 || plp >= h->nplp) return DVBT2LL_EINVAL;
  const ChainPlp &pl = *h->plps[plp];
  info->fec_blocks_per_frame = pl.F;
  info->payload_bytes_per_block = pl.pay;
  info->ts_bytes_per_frame = pl.inputmode ? (pl.ts_per_frame * 188 + 186) / 187 : pl.ts_per_frame;
  info->iq_samples_per_frame = h->iq_per_frame;
  info->cell_size = h->frame.plp[plp].cs;
  info->stream_items = h->frame.plp[plp].S;
  info->mapped_items = h->frame.M;
  info->num_symbols = h->pilot.Nsym;
  info->fft_size = h->pilot.N;
  info->guard_interval = h->pilot.G;
  info->cw_stride_bytes = pl.cw_stride;
  info->frames_per_if = pl.cyc;
  return DVBT2LL_OK;
}

extern "C" int dvbt2ll_chain_get_info(const dvbt2ll_chain *h, dvbt2ll_chain_info *info) {
  int r = dvbt2ll_chain_get_plp_info(h, 0, info);
  if (r) return r;
  info->stream_items = h->frame.S;   // the frame's data cells (every PLP)
  return DVBT2LL_OK;
}

extern "C" int dvbt2ll_chain_run_device(dvbt2ll_chain *h, const void *ts_dev, int64_t ts_base, int64_t ts_len,
                                        int64_t first_frame, int nframes, void *iq_dev, void *stream) {
  return dvbt2ll_chain_run_streams(h, ts_dev, 0, 1, ts_base, ts_len, first_frame, nframes, iq_dev, stream);
}

// stream bytes [lo, end) that frames [first, first + n) of PLP pl consume: their payload plus the packet before
// the first one touched (its CRC-8 replaces the next sync byte, bbheader:701-713)
static void ts_span(const ChainPlp &pl, int64_t first, int64_t n, int64_t *lo, int64_t *end) {
  int64_t start = first / pl.cyc * pl.ts_per_frame, e = (first + n) / pl.cyc * pl.ts_per_frame;
  if (pl.inputmode) {
    start = 188 * (start / 187) + (start % 187);
    e = 188 * (e / 187) + (e % 187) + 1;
  }
  *lo = start >= 188 ? (start / 188) * 188 - 188 : 0;
  *end = e;
}

// one run over nstreams independent single-PLP streams (nplp == 1) or over one frame sequence of
// every PLP (nstreams == 1): ts[k], base[k], len[k] per PLP (stream s of a batch at ts[0] + s * ts_stride)
static int chain_run(dvbt2ll_chain *h, const void *const *ts, const int64_t *base, const int64_t *len,
                     int64_t ts_stride, int nstreams, int64_t first_frame, int nframes, void *iq_dev, void *stream) {
  if (!h || !ts || !iq_dev || nframes < 1 || nstreams < 1 || (int64_t)nframes * nstreams > h->max_frames ||
      first_frame < 0 || (nstreams > 1 && (h->nplp > 1 || ts_stride < len[0])))
    return DVBT2LL_EINVAL;
  // whole interleaving frames of every PLP (TIME_IL_TYPE 1: P_I T2 frames each)
  if (first_frame % h->frame.unit || nframes % h->frame.unit) return DVBT2LL_EINVAL;
  const int nf = nframes * nstreams;   // frames of the launch, stream-major
  hipStream_t s = stream ? (hipStream_t)stream : h->ctx.stream;
  for (int k = 0; k < h->nplp; k++) {
    const ChainPlp &pl = *h->plps[k];
    if (!ts[k] || base[k] < 0 || base[k] % 188 != 0) return DVBT2LL_EINVAL;
    // the TS slice must cover every byte the frames consume plus the packet before the first one touched
    int64_t lo, end;
    ts_span(pl, first_frame, nframes, &lo, &end);
    if (base[k] > lo || base[k] + len[k] < end) return DVBT2LL_EINVAL;
  }
  HIP_TRY(hipSetDevice(h->ctx.device));
  const int slot = h->next_slot;
  if (h->slot_used[slot] && h->slot_stream[slot] != s) HIP_TRY(hipStreamWaitEvent(s, h->slot_done[slot], 0));
  DevBuf &pairs = h->pairs[slot];
  if (h->bpart_dirty[slot]) {
    for (auto &pl : h->plps) HIP_TRY(hipMemsetAsync(pl->bpart[slot].p, 0, pl->bpart[slot].n, s));
    h->bpart_dirty[slot] = false;
  }
  hipEvent_t ev[dvbt2ll_chain::NEV] = {};
  if (h->timing && !h->use_graph) {   // per-stage events only on the direct launch path
    if (h->evused + dvbt2ll_chain::NEV > 4096 && h->fold_timing()) return DVBT2LL_EDEVICE;
    for (auto &e : ev)
      if (!(e = h->next_event())) return DVBT2LL_EDEVICE;
    HIP_TRY(hipEventRecord(ev[0], s));
  }
  L1IO lio{};
  FecIO fio[DVBT2LL_MAX_PLP] = {};
  MapIO mio[DVBT2LL_MAX_PLP] = {};
  OfdmIO oio{};
  lio.out = h->l1buf[slot].as<float2>();
  lio.out_stride = h->l1_stride;
  lio.first_frame = first_frame;
  lio.nframes = nf;
  lio.frames_per_stream = nstreams > 1 ? nframes : 0;
  for (int k = 0; k < h->nplp; k++) {
    ChainPlp &pl = *h->plps[k];
    DevBuf &cw = pl.cw[slot];
    fio[k].in = (const uint8_t *)ts[k];
    fio[k].ts_base = base[k];
    fio[k].ts_len = len[k];
    // launch block b: FEC block b mod F of interleaving frame b / F, which fills T2 frames P (b / F) ..
    // P (b / F) + P - 1 of the launch (pairs at P pair_stride per interleaving frame)
    fio[k].first_block = first_frame / pl.cyc * pl.F;
    fio[k].out = cw.as<uint8_t>();
    fio[k].cw_stride = pl.cw_stride;
    fio[k].nblocks = (int)pl.blocks(nf);
    fio[k].sync_err = h->sync_err.as<uint32_t>();
    fio[k].blocks_per_stream = nstreams > 1 ? (int)pl.blocks(nframes) : 0;
    fio[k].ts_stride = nstreams > 1 ? ts_stride : 0;
    fio[k].bch_part = pl.bpart[slot].as<uint32_t>();
    fio[k].bch_part_blocks = pl.blocks(h->max_frames);
    fio[k].keep_cw = h->keep_cw;
    mio[k].out_pairs = pairs.as<uint16_t>();
    mio[k].frame_stride = h->pair_stride * h->frame.unit;
    mio[k].nblocks = (int)pl.blocks(nf);
  }
  oio.data = h->aux.as<float2>();
  oio.aux_off = 0;
  oio.cell_off = 0;
  oio.cell_stride = (uint32_t)h->pair_stride;
  oio.pairs = pairs.as<uint16_t>();
  oio.out = (float2 *)iq_dev;
  oio.out_stride = h->iq_per_frame;
  oio.first_frame = first_frame;
  oio.nframes = nf;
  oio.frames_per_stream = nstreams > 1 ? nframes : 0;
  oio.l1 = h->l1buf[slot].as<float2>();
  oio.l1_stride = h->l1_stride;
  if (h->use_graph) {
    int r = h->graph_launch(lio, fio, mio, oio, nf, slot, s);
    if (r) {
      h->bpart_dirty[slot] = true;
      return r;
    }
  } else {
    const hipError_t e = h->launch_chain(lio, fio, mio, oio, s, ev[1], ev[2]);
    if (e != hipSuccess) {
      h->bpart_dirty[slot] = true;
      HIP_TRY(e);
    }
    if (h->timing) HIP_TRY(hipEventRecord(ev[3], s));
  }
  HIP_TRY(hipEventRecord(h->slot_done[slot], s));
  h->slot_used[slot] = true;
  h->slot_stream[slot] = s;
  h->cw_kept[slot] = h->keep_cw;
  h->last_slot = slot;
  h->next_slot = (slot + 1) % h->nslots;
  return DVBT2LL_OK;
}

extern "C" int dvbt2ll_chain_run_streams(dvbt2ll_chain *h, const void *ts_dev, int64_t ts_stride, int nstreams,
                                         int64_t ts_base, int64_t ts_len, int64_t first_frame, int nframes,
                                         void *iq_dev, void *stream) {
  if (!h || h->nplp != 1) return DVBT2LL_EINVAL;
  const void *ts[1] = {ts_dev};
  return chain_run(h, ts, &ts_base, &ts_len, ts_stride, nstreams, first_frame, nframes, iq_dev, stream);
}

extern "C" int dvbt2ll_chain_run_plps(dvbt2ll_chain *h, const void *const *ts_dev, const int64_t *ts_base,
                                      const int64_t *ts_len, int64_t first_frame, int nframes, void *iq_dev,
                                      void *stream) {
  if (!h || !ts_dev || !ts_base || !ts_len) return DVBT2LL_EINVAL;
  return chain_run(h, ts_dev, ts_base, ts_len, 0, 1, first_frame, nframes, iq_dev, stream);
}

extern "C" int dvbt2ll_chain_set_graph(dvbt2ll_chain *h, int enable) {
  if (!h) return DVBT2LL_EINVAL;
  h->use_graph = enable != 0;
  return DVBT2LL_OK;
}

extern "C" int dvbt2ll_chain_set_slots(dvbt2ll_chain *h, int nslots) {
  if (!h || nslots < 1 || nslots > DVBT2LL_CHAIN_MAX_SLOTS) return DVBT2LL_EINVAL;
  HIP_TRY(hipSetDevice(h->ctx.device));
  HIP_TRY(hipDeviceSynchronize());   // no run in flight while slots change
  for (int k = 0; k < nslots; k++) {
    int r = h->alloc_slot(k);
    if (r) return r;
  }
  for (int k = nslots; k < DVBT2LL_CHAIN_MAX_SLOTS; k++) {
    for (auto &pl : h->plps) {
      pl->cw[k].release();
      pl->bpart[k].release();
    }
    h->pairs[k].release();
    h->l1buf[k].release();
    h->slot_used[k] = false;
  }
  h->nslots = nslots;
  h->next_slot = 0;
  if (h->last_slot >= nslots) h->last_slot = 0;
  return DVBT2LL_OK;
}

extern "C" int dvbt2ll_chain_run_host(dvbt2ll_chain *h, const void *ts, int64_t ts_base, int64_t ts_len,
                                      int64_t first_frame, int nframes, void *iq) {
  if (!h || !ts || !iq || nframes < 1 || nframes > h->max_frames || h->nplp != 1) return DVBT2LL_EINVAL;
  HIP_TRY(hipSetDevice(h->ctx.device));
  size_t iq_bytes = (size_t)nframes * h->iq_per_frame * (h->ofdm.dev.fmt == DVBT2LL_IQ_SC16 ? 4 : 8);
  if (h->ts_tmp.ensure((size_t)ts_len + 16) || h->iq_tmp.ensure(iq_bytes)) return DVBT2LL_ENOMEM;
  HIP_TRY(hipMemcpyAsync(h->ts_tmp.p, ts, (size_t)ts_len, hipMemcpyHostToDevice, h->ctx.stream));
  int r = dvbt2ll_chain_run_device(h, h->ts_tmp.p, ts_base, ts_len, first_frame, nframes, h->iq_tmp.p, nullptr);
  if (r) return r;
  HIP_TRY(hipMemcpyAsync(iq, h->iq_tmp.p, iq_bytes, hipMemcpyDeviceToHost, h->ctx.stream));
  HIP_TRY(hipStreamSynchronize(h->ctx.stream));
  return DVBT2LL_OK;
}

extern "C" int dvbt2ll_chain_run_plps_host(dvbt2ll_chain *h, const void *const *ts, const int64_t *ts_base,
                                           const int64_t *ts_len, int64_t first_frame, int nframes, void *iq) {
  if (!h || !ts || !ts_base || !ts_len || !iq || nframes < 1 || nframes > h->max_frames) return DVBT2LL_EINVAL;
  HIP_TRY(hipSetDevice(h->ctx.device));
  const void *dev[DVBT2LL_MAX_PLP];
  for (int k = 0; k < h->nplp; k++) {
    if (!ts[k] || ts_len[k] < 0) return DVBT2LL_EINVAL;
    if (h->ts_plp_tmp[k].ensure((size_t)ts_len[k] + 16)) return DVBT2LL_ENOMEM;
    HIP_TRY(hipMemcpyAsync(h->ts_plp_tmp[k].p, ts[k], (size_t)ts_len[k], hipMemcpyHostToDevice, h->ctx.stream));
    dev[k] = h->ts_plp_tmp[k].p;
  }
  const size_t iq_bytes = (size_t)nframes * h->iq_per_frame * (h->ofdm.dev.fmt == DVBT2LL_IQ_SC16 ? 4 : 8);
  if (h->iq_tmp.ensure(iq_bytes)) return DVBT2LL_ENOMEM;
  int r = dvbt2ll_chain_run_plps(h, dev, ts_base, ts_len, first_frame, nframes, h->iq_tmp.p, nullptr);
  if (r) return r;
  HIP_TRY(hipMemcpyAsync(iq, h->iq_tmp.p, iq_bytes, hipMemcpyDeviceToHost, h->ctx.stream));
  HIP_TRY(hipStreamSynchronize(h->ctx.stream));
  return DVBT2LL_OK;
}

extern "C" int dvbt2ll_chain_host_submit(dvbt2ll_chain *h, const void *ts, int64_t ts_base, int64_t ts_len,
                                         int64_t first_frame, int nframes, void *iq, int64_t *ticket) {
  // every argument check precedes the first asynchronous operation, so a refused submission leaves no copy
  // of the caller's buffers in flight (the unit check is repeated by chain_run, after the copy-in is queued)
  if (!h || !ts || !iq || !ticket || h->nplp != 1 || nframes < 1 || nframes > h->max_frames || first_frame < 0 ||
      ts_base < 0 || ts_base % 188 || first_frame % h->frame.unit || nframes % h->frame.unit)
    return DVBT2LL_EINVAL;
  const ChainPlp &pl = *h->plps[0];
  int64_t lo, end;
  ts_span(pl, first_frame, nframes, &lo, &end);
  if (ts_base > lo || ts_base + ts_len < end) return DVBT2LL_EINVAL;
  int r = h->host.init(h->ctx.device);
  if (r) return r;
  HIP_TRY(hipSetDevice(h->ctx.device));
  HostRing &R = h->host;
  const int64_t t = R.next_ticket;
  HostRing::Entry &x = R.e[t % DVBT2LL_HOST_RING];
  // the entry's previous submission must have left its buffers: its copy-out is the last thing it does
  if (x.ticket >= 0) HIP_TRY(hipEventSynchronize(x.d2h));
  const size_t iq_bytes = (size_t)nframes * h->iq_per_frame * (h->ofdm.dev.fmt == DVBT2LL_IQ_SC16 ? 4 : 8);
  if (x.ts.ensure((size_t)(end - lo) + 16) || x.iq.ensure(iq_bytes)) return DVBT2LL_ENOMEM;
  HIP_TRY(hipMemcpyAsync(x.ts.p, (const uint8_t *)ts + (lo - ts_base), (size_t)(end - lo), hipMemcpyHostToDevice,
                         R.in));
  HIP_TRY(hipEventRecord(x.h2d, R.in));
  HIP_TRY(hipStreamWaitEvent(R.comp, x.h2d, 0));
  if ((r = dvbt2ll_chain_run_device(h, x.ts.p, lo, end - lo, first_frame, nframes, x.iq.p, R.comp))) {
    // unreachable after the checks above unless the device fails; the copy-in must still end before the
    // caller may reuse ts
    (void)hipStreamSynchronize(R.in);
    return r;
  }
  HIP_TRY(hipEventRecord(x.kern, R.comp));
  HIP_TRY(hipStreamWaitEvent(R.out, x.kern, 0));
  HIP_TRY(hipMemcpyAsync(iq, x.iq.p, iq_bytes, hipMemcpyDeviceToHost, R.out));
  HIP_TRY(hipEventRecord(x.d2h, R.out));
  x.ticket = t;
  R.next_ticket = t + 1;
  *ticket = t;
  return DVBT2LL_OK;
}

extern "C" int dvbt2ll_chain_host_wait(dvbt2ll_chain *h, int64_t ticket) {
  if (!h || ticket < 0 || ticket >= h->host.next_ticket) return DVBT2LL_EINVAL;
  HIP_TRY(hipSetDevice(h->ctx.device));
  const HostRing::Entry &x = h->host.e[ticket % DVBT2LL_HOST_RING];
  // an entry reused by a later submission was waited for at that submission
  if (x.ticket == ticket) HIP_TRY(hipEventSynchronize(x.d2h));
  return DVBT2LL_OK;
}

extern "C" int dvbt2ll_chain_run_host_pipelined(dvbt2ll_chain *h, const void *ts, int64_t ts_base, int64_t ts_len,
                                                int64_t first_frame, int nframes, void *iq, int chunk_frames) {
  if (!h || !ts || !iq || nframes < 1 || chunk_frames < 0 || h->nplp != 1) return DVBT2LL_EINVAL;
  const int U = h->frame.unit;
  // chunks of whole launch units; every chunk is checked before the first one is submitted
  int c = chunk_frames ? std::min(chunk_frames, h->max_frames) : h->max_frames;
  c -= c % U;
  if (c < U || first_frame < 0 || first_frame % U || nframes % U || ts_base < 0 || ts_base % 188)
    return DVBT2LL_EINVAL;
  {
    int64_t lo, end;
    ts_span(*h->plps[0], first_frame, nframes, &lo, &end);   // the union of the chunks' spans
    if (ts_base > lo || ts_base + ts_len < end) return DVBT2LL_EINVAL;
  }
  const size_t per = (size_t)h->iq_per_frame * (h->ofdm.dev.fmt == DVBT2LL_IQ_SC16 ? 4 : 8);
  int64_t t = -1;
  for (int f = 0; f < nframes; f += c) {
    const int n = std::min(c, nframes - f);
    int r = dvbt2ll_chain_host_submit(h, ts, ts_base, ts_len, first_frame + f, n, (char *)iq + (size_t)f * per, &t);
    if (r) {
      // the chunks already submitted still copy into iq: drain them before the caller sees the error
      if (t >= 0) (void)dvbt2ll_chain_host_wait(h, t);
      return r;
    }
  }
  return dvbt2ll_chain_host_wait(h, t);
}

// page-aligned heap memory, page-locked by hipHostRegister (the copies then run at the PCIe rate, as from
// hipHostMalloc memory; the buffer stays ordinary heap memory, which the host sanitizer build tracks)
extern "C" void *dvbt2ll_host_alloc(size_t bytes) {
  const size_t n = ((bytes ? bytes : 1) + 4095) & ~(size_t)4095;
  void *p = nullptr;
  if (posix_memalign(&p, 4096, n)) return nullptr;
  if (hipHostRegister(p, n, hipHostRegisterDefault) != hipSuccess) {
    std::free(p);
    return nullptr;
  }
  return p;
}
extern "C" void dvbt2ll_host_free(void *p) {
  if (!p) return;
  (void)hipHostUnregister(p);
  std::free(p);
}

extern "C" int dvbt2ll_chain_set_output(dvbt2ll_chain *h, float gain, int format) {
  if (!h || !(gain == gain) || (format != DVBT2LL_IQ_CF32 && format != DVBT2LL_IQ_SC16)) return DVBT2LL_EINVAL;
  h->ofdm.dev.gain = gain;
  h->ofdm.dev.fmt = format;
  return DVBT2LL_OK;
}

extern "C" int dvbt2ll_chain_set_timing(dvbt2ll_chain *h, int enable) {
  if (!h) return DVBT2LL_EINVAL;
  if (h->fold_timing()) return DVBT2LL_EDEVICE;
  h->timing = enable != 0;
  for (int k = 0; k < 4; k++) { h->ms[k] = 0; h->launches[k] = 0; }
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_chain_get_timing(dvbt2ll_chain *h, double *ms, int64_t *launches, int nstages) {
  if (!h || !ms || nstages < 1) return DVBT2LL_EINVAL;
  if (h->fold_timing()) return DVBT2LL_EDEVICE;
  for (int k = 0; k < nstages && k < 4; k++) {
    ms[k] = h->ms[k];
    if (launches) launches[k] = h->launches[k];
  }
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_chain_debug_plp_codewords(dvbt2ll_chain *h, int plp, void *out, int64_t bytes) {
  if (!h || !out || bytes < 0 || plp < 0 || plp >= h->nplp) return DVBT2LL_EINVAL;
  const DevBuf &cw = h->plps[plp]->cw[h->last_slot];
  if ((size_t)bytes > cw.n || !h->cw_kept[h->last_slot]) return DVBT2LL_EINVAL;
  HIP_TRY(hipSetDevice(h->ctx.device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, cw.p, (size_t)bytes, hipMemcpyDeviceToHost));
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_chain_debug_keep_codewords(dvbt2ll_chain *h, int enable) {
  if (!h) return DVBT2LL_EINVAL;
  h->keep_cw = enable != 0;
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_chain_debug_codewords(dvbt2ll_chain *h, void *out, int64_t bytes) {
  return dvbt2ll_chain_debug_plp_codewords(h, 0, out, bytes);
}
extern "C" int dvbt2ll_chain_debug_cell_pairs(dvbt2ll_chain *h, void *out, int64_t cells) {
  if (!h || !out || cells < 0 || (size_t)cells * 2 > h->pairs[h->last_slot].n) return DVBT2LL_EINVAL;
  HIP_TRY(hipSetDevice(h->ctx.device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, h->pairs[h->last_slot].p, (size_t)cells * 2, hipMemcpyDeviceToHost));
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_chain_debug_cells(dvbt2ll_chain *h, void *out, int64_t cells) {
  // frame 0's data cells: index pairs expanded through the constellation exactly as the OFDM
  // kernel does, (lut[lo].re, lut[hi].im) with the table of the slot's PLP
  if (!h || !out || cells < 0 || (size_t)cells * 2 > h->pairs[h->last_slot].n) return DVBT2LL_EINVAL;
  std::vector<uint16_t> pr((size_t)cells);
  int r = dvbt2ll_chain_debug_cell_pairs(h, pr.data(), cells);
  if (r) return r;
  cf32 *o = (cf32 *)out;
  std::vector<int> plp_of((size_t)cells, 0);
  if (h->nplp > 1) {
    const int P = h->nplp;
    for (size_t g = 0; g + 1 <= h->plp_bnd_host.size() / (P + 1); g++)
      for (int k = 0; k < P; k++)
        for (int32_t s = h->plp_bnd_host[g * (P + 1) + k]; s < h->plp_bnd_host[g * (P + 1) + k + 1]; s++)
          if (s < cells) plp_of[s] = k;
  }
  for (int64_t i = 0; i < cells; i++) {
    const cf32 *lut = h->plps[plp_of[i]]->map.plan.lut;
    o[i] = cf32{lut[pr[i] & 0xFF].re, lut[pr[i] >> 8].im};
  }
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_chain_sync_errors(dvbt2ll_chain *h, int64_t *count) {
  if (!h || !count) return DVBT2LL_EINVAL;
  uint32_t v = 0;
  HIP_TRY(hipSetDevice(h->ctx.device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(&v, h->sync_err.p, 4, hipMemcpyDeviceToHost));
  *count = (int64_t)v;
  return DVBT2LL_OK;
}
extern "C" int dvbt2ll_chain_synchronize(dvbt2ll_chain *h) {
  if (!h) return DVBT2LL_EINVAL;
  HIP_TRY(hipSetDevice(h->ctx.device));
  HIP_TRY(hipStreamSynchronize(h->ctx.stream));
  // the streaming host path's three streams (dvbt2ll_chain_host_submit) and the slots' last runs on
  // caller streams
  HIP_TRY(h->host.synchronize());
  for (int k = 0; k < DVBT2LL_CHAIN_MAX_SLOTS; k++)
    if (h->slot_used[k] && h->slot_done[k]) HIP_TRY(hipEventSynchronize(h->slot_done[k]));
  return DVBT2LL_OK;
}
extern "C" void dvbt2ll_chain_destroy(dvbt2ll_chain *h) { delete h; }
