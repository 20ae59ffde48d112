"""Fused chain (TS -> IQ) parity vs the oracle chain; frame independence (sharding basis)."""
import numpy as np
import pytest

import dvbt2ll
from dvbt2ll.configs import CONFIGS, ts_for_frames
import oracle_lib as O
import iq_check

pytestmark = pytest.mark.gpu


def oracle_chain(cfg, nframes):
    ts, base = ts_for_frames(cfg, 0, nframes)
    F = cfg.fecblocks
    bb = O.BB(*cfg.bb_args()); ld = O.LDPC(cfg.framesize, cfg.rate); im = O.IM(*cfg.im_args())
    fm = O.FM(*cfg.fm_args()); pg = O.PG(*cfg.pg_args())
    off = 0
    out = []
    for k in range(nframes):
        bits, cons = bb.work(ts[off:], F)
        off += cons
        cells = im.work(ld.work(bits, F), F)
        mapped = fm.work(cells)
        out.append((pg.carriers(mapped), mapped))
    return out, pg


@pytest.mark.parametrize("name", ["cfg1", "cfg1q", "cfg2", "cfg3", "cfg4", "cfg5"])
def test_chain_cells_match_oracle(gpu, name):
    """stage check inside the fused chain: the cells buffer (FEC + bit interleave + QAM + cell
    and time interleaving = the frame data region in transmission order) equals the oracle's"""
    import plan_probe as PP
    cfg = CONFIGS[name]
    ts, base = ts_for_frames(cfg, 0, 1)
    F = cfg.fecblocks
    bits, _ = O.BB(*cfg.bb_args()).work(ts, F)
    cells = O.IM(*cfg.im_args()).work(O.LDPC(cfg.framesize, cfg.rate).work(bits, F), F)
    plan = PP.frame_plan(cfg.fm_args())
    cs = plan["cs"]
    r = np.repeat(np.arange(F), cs)
    jj = np.tile(np.arange(cs), F)
    t = (plan["ci_perm"][jj] + plan["ci_shift"][r]) % cs
    lay = PP.chain_layout(cfg)
    want = np.zeros(plan["S"], np.complex64)
    want[lay["part"][PP.ti_dest(plan, r, t)]] = cells
    ch = dvbt2ll.Chain(cfg, max_frames=1)
    ch.run(0, 1)
    got = ch.debug_cells(plan["S"])
    bad = np.nonzero(got.view(np.uint64) != want.view(np.uint64))[0]
    assert bad.size == 0, (bad.size, bad[:10], bad[:10] // cs)


def _check_chain(cfg, nframes):
    ref, pg = oracle_chain(cfg, nframes)
    ch = dvbt2ll.Chain(cfg, max_frames=nframes)
    iq = ch.run(0, nframes)
    per = ch.iq_per_frame
    p1 = pg.p1()
    for k in range(nframes):
        iq_check.check_frame(iq[k * per:(k + 1) * per], ref[k][0], pg.vlength, pg.guard, pg.normalization, p1,
                             "%s frame %d" % (cfg.name, k))
        iq_check.check_frame_exact(iq[k * per:(k + 1) * per], ref[k][0], cfg.pg_args(), pg.guard, pg.normalization,
                                   "%s frame %d" % (cfg.name, k))


@pytest.mark.parametrize("name", ["cfg1", "cfg1q", "cfg2", "cfg3", "cfg4", "cfg5"])
def test_chain_iq_matches_oracle(gpu, name):
    _check_chain(CONFIGS[name], 3 if name == "cfg1" else (2 if name == "cfg3" else 1))


from test_cpu_plan import GRID, grid_cfg  # noqa: E402


@pytest.mark.parametrize("name,over", GRID, ids=[g[0] for g in GRID])
def test_chain_feature_grid(gpu, name, over):
    """every FFT size, N_P2 > 1, MISO TX2, PAPR TR, extended carriers, EQ, v1.3.1 L1, L1 BPSK..16QAM"""
    cfg = grid_cfg(over)
    _check_chain(cfg, min(2, cfg.t2frames + 1))


@pytest.mark.parametrize("name", ["cfg1", "cfg3"])
def test_chain_frames_independent(gpu, name):
    """frame k computed alone (first_frame=k) equals frame k of a batched run"""
    cfg = CONFIGS[name]
    ch = dvbt2ll.Chain(cfg, max_frames=3)
    batch = ch.run(0, 3)
    per = ch.iq_per_frame
    for k in (1, 2):
        one = ch.run(k, 1)
        np.testing.assert_array_equal(one.view(np.uint32), batch[k * per:(k + 1) * per].view(np.uint32))


@pytest.mark.parametrize("name", ["cfg1", "cfg3"])
def test_chain_output_gain_and_sc16(gpu, name):
    """SURVEY 8(f) rank 1, the step after the path in apps/vv009-4kshort.grc: multiply_const (0.2)
    and the SDR sink's sc16 wire format, fused into the IQ store.  gain: bit-exactly the float
    product of pilotgen's output and the constant (two float multiplies, as the two blocks do);
    sc16: saturate(round-half-even(x * 32767)) of that product, bit-exact.  (The sink's
    conversion lives in the SDR driver, absent from the reference: parity unpinned there, the
    rounding rule is this library's documented contract.)"""
    cfg = CONFIGS[name]
    ch = dvbt2ll.Chain(cfg, max_frames=2)
    base = ch.run(0, 2)
    ch.set_output(0.2, dvbt2ll.IQ_CF32)
    scaled = ch.run(0, 2)
    want = (base.view(np.float32) * np.float32(0.2)).astype(np.float32)
    np.testing.assert_array_equal(scaled.view(np.float32), want)
    ch.set_output(0.2, dvbt2ll.IQ_SC16)
    sc = ch.run(0, 2)
    assert sc.dtype == np.int16 and sc.shape == (2 * ch.iq_per_frame, 2)
    ref = np.clip(np.rint(want.astype(np.float32) * np.float32(32767)), -32768, 32767).astype(np.int16)
    np.testing.assert_array_equal(sc.reshape(-1), ref)
    # and both against the CPU model of the GPU IFFT with the output step (bit-exact)
    ref, pg = oracle_chain(cfg, 2)
    per = ch.iq_per_frame
    for k in range(2):
        iq_check.check_frame_exact(scaled[k * per:(k + 1) * per], ref[k][0], cfg.pg_args(), pg.guard,
                                   pg.normalization, "%s x0.2 frame %d" % (name, k), gain=0.2)
        iq_check.check_frame_exact(sc[k * per:(k + 1) * per], ref[k][0], cfg.pg_args(), pg.guard,
                                   pg.normalization, "%s sc16 frame %d" % (name, k), gain=0.2, fmt=1)
    # saturation: a gain large enough to clip
    ch.set_output(40.0, dvbt2ll.IQ_SC16)
    big = ch.run(0, 1).reshape(-1)
    refb = np.clip(np.rint((base[:ch.iq_per_frame].view(np.float32) * np.float32(40.0)) * np.float32(32767)),
                   -32768, 32767).astype(np.int16)
    np.testing.assert_array_equal(big, refb)
    assert (np.abs(big.astype(np.int32)) == 32767).any() or (big == -32768).any()


def test_chain_set_output_rejects_bad_format(gpu):
    ch = dvbt2ll.Chain(CONFIGS["cfg1"], max_frames=1)
    with pytest.raises(dvbt2ll.DVBT2Error):
        ch.set_output(1.0, 7)


@pytest.mark.parametrize("name,sets,fmt,gain,nfr,batch", [
    ("cfg1", [], "cf32", 1.0, 3, 2), ("cfg1", [], "sc16", 0.2, 3, 2), ("cfg1", ["inputmode=1"], "sc16", 0.2, 3, 2),
    ("cfg1", [], "cf32", 1.0, 8, 1), ("cfg4", ["inband=1"], "sc16", 0.2, 7, 2)])
def test_tx_tool_matches_chain(gpu, tmp_path, name, sets, fmt, gain, nfr, batch):
    """dvbt2ll_tx (TS file -> IQ file, rolling TS buffer, batches in flight on the streaming ring: 8 and 4
    batches wrap its DVBT2LL_HOST_RING entries) writes exactly the chain's output for the same stream"""
    import subprocess
    from pathlib import Path
    cfg = CONFIGS[name]
    for s in sets:
        k, v = s.split("=")
        cfg = cfg.with_(**{k: int(v)})
    ts, base = ts_for_frames(cfg, 0, nfr)
    assert base == 0
    (tmp_path / "in.ts").write_bytes(ts.tobytes())
    tool = Path(__file__).resolve().parents[1] / "gr-dvbt2ll_amd" / "dvbt2ll" / "dvbt2ll_tx"
    args = [str(tool), "--preset", name, "--in", str(tmp_path / "in.ts"), "--out", str(tmp_path / "iq.bin"),
            "--format", fmt, "--gain", str(gain), "--batch", str(batch), "--frames", str(nfr)]
    for s in sets:
        args += ["--set", s]
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    ch = dvbt2ll.Chain(cfg, max_frames=nfr)
    ch.set_output(gain, dvbt2ll.IQ_SC16 if fmt == "sc16" else dvbt2ll.IQ_CF32)
    want = ch.run(0, nfr)
    got = np.frombuffer((tmp_path / "iq.bin").read_bytes(), dtype=want.dtype).reshape(want.shape)
    np.testing.assert_array_equal(got.view(np.uint8), want.view(np.uint8))


@pytest.mark.parametrize("name,nslots,nstreams", [("cfg1", 2, 2), ("cfg1", 2, 3), ("cfg3", 2, 2), ("cfg1", 4, 3)])
def test_chain_slots_on_streams(gpu, name, nslots, nstreams):
    """dvbt2ll_chain_set_slots: run calls issued round-robin on several HIP streams (calls overlap
    on the GPU; a slot reused on another stream waits for its previous run) give bit-exactly the
    IQ of sequential single-slot runs"""
    import torch
    cfg = CONFIGS[name]
    B, ncalls = 2, 6
    ref = dvbt2ll.Chain(cfg, max_frames=B)
    ch = dvbt2ll.Chain(cfg, max_frames=B)
    ch.set_slots(nslots)
    per = ch.iq_per_frame
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    ts_all, base_all = ts_for_frames(cfg, 0, B * ncalls)
    ts_dev = torch.from_numpy(ts_all).cuda()
    torch.cuda.synchronize()
    outs = [torch.empty((B * per, 2), dtype=torch.float32, device="cuda") for _ in range(ncalls)]
    for c in range(ncalls):
        ch.run_device(ts_dev.data_ptr(), base_all, len(ts_all), c * B, B, outs[c].data_ptr(),
                      streams[c % nstreams].cuda_stream)
    torch.cuda.synchronize()
    for c in range(ncalls):
        want = ref.run(c * B, B)
        got = outs[c].cpu().numpy().view(np.complex64).reshape(-1)
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32), err_msg="call %d" % c)


def test_chain_set_slots_rejects_bad_count(gpu):
    ch = dvbt2ll.Chain(CONFIGS["cfg1"], max_frames=1)
    for n in (0, 5):
        with pytest.raises(dvbt2ll.DVBT2Error):
            ch.set_slots(n)


@pytest.mark.parametrize("name", ["cfg1", "cfg3"])
def test_chain_graph_mode(gpu, name):
    """dvbt2ll_chain_set_graph: the kernels launched as one captured hipGraph per (nframes, IQ
    format), re-armed per call, give bit-exactly the direct launches' IQ -- across frame indices,
    batch sizes, output formats and slots"""
    cfg = CONFIGS[name]
    ref = dvbt2ll.Chain(cfg, max_frames=2)
    ch = dvbt2ll.Chain(cfg, max_frames=2)
    ch.set_graph(True)
    ch.set_slots(2)
    for first, n in ((0, 1), (1, 1), (3, 1), (0, 2), (5, 2), (2, 1)):
        np.testing.assert_array_equal(ch.run(first, n).view(np.uint32), ref.run(first, n).view(np.uint32),
                                      err_msg="frames %d+%d" % (first, n))
    for c in (ch, ref):
        c.set_output(0.2, dvbt2ll.IQ_SC16)
    for first, n in ((4, 1), (1, 2)):
        np.testing.assert_array_equal(ch.run(first, n), ref.run(first, n))
    ch.set_graph(False)
    np.testing.assert_array_equal(ch.run(6, 1), ref.run(6, 1))


@pytest.mark.parametrize("name", ["cfg1", "cfg3"])
def test_chain_graph_reused_buffers(gpu, name):
    """graph mode with the caller's device buffers reused: a ring instantiation whose held kernel arguments
    equal a call's skips the node re-arms (t2_capi.cpp graph_launch); calls that repeat a frame and calls
    that change it, cycling the ring (4 instantiations) on one slot, each give the direct launch's IQ"""
    import torch
    cfg = CONFIGS[name]
    ts, base = ts_for_frames(cfg, 0, 4)
    ts_d = torch.from_numpy(ts).cuda()
    ch = dvbt2ll.Chain(cfg, max_frames=1)
    iq_d = torch.empty((ch.iq_per_frame, 2), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def run(frame):
        ch.run_device(ts_d.data_ptr(), base, len(ts), frame, 1, iq_d.data_ptr(), st)
        torch.cuda.synchronize()
        return iq_d.cpu().numpy().copy()

    want = {f: run(f) for f in range(4)}      # direct launches
    ch.set_graph(True)
    for k, f in enumerate((0, 0, 1, 0, 1, 1, 2, 0, 0, 0, 0, 0, 3, 3, 0)):
        np.testing.assert_array_equal(run(f).view(np.uint32), want[f].view(np.uint32), err_msg="call %d frame %d" % (k, f))
    ch.set_graph(False)


def _stream_batch(cfg, S, first, B, graph=False, sc16=False):
    """S independent TS streams (seeds 1..S) in one dvbt2ll_chain_run_streams launch; returns the
    per-stream IQ and a single-stream reference handle's IQ of each stream's own TS"""
    import torch
    ch = dvbt2ll.Chain(cfg, max_frames=S * B)
    ref = dvbt2ll.Chain(cfg, max_frames=B)
    if graph:
        ch.set_graph(True)
    if sc16:
        for c in (ch, ref):
            c.set_output(0.2, dvbt2ll.IQ_SC16)
    per = ch.iq_per_frame
    tss = [ts_for_frames(cfg, first, B, seed=s + 1) for s in range(S)]
    base, n = tss[0][1], len(tss[0][0])
    stride = (n + 1000 + 255) // 256 * 256          # deliberately not the tight length
    buf = np.zeros((S, stride), np.uint8)
    for s, (ts, b) in enumerate(tss):
        assert b == base and len(ts) == n
        buf[s, :n] = ts
    ts_dev = torch.from_numpy(buf.reshape(-1)).cuda()
    dt = torch.int16 if sc16 else torch.float32
    iq = torch.empty((S * B * per, 2), dtype=dt, device="cuda")
    torch.cuda.synchronize()
    ch.run_streams(ts_dev.data_ptr(), stride, S, base, n, first, B, iq.data_ptr(),
                   torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = iq.cpu().numpy()
    got = got.reshape(S, B * per, 2) if sc16 else got.view(np.complex64).reshape(S, B * per)
    want = [ref.run(first, B, ts=ts, ts_base=b) for ts, b in tss]
    return got, want, tss


@pytest.mark.parametrize("name,S,first,B", [("cfg1", 3, 0, 2), ("cfg1q", 4, 5, 1), ("cfg4", 4, 0, 1),
                                            ("cfg2", 2, 1, 1)])
def test_chain_streams_batch(gpu, name, S, first, B):
    """BASELINE cfg4 / cfg5 multi-stream batching: S independent streams in one launch give, per
    stream, bit-exactly what a single-stream handle gives on that stream's TS; streams differ"""
    got, want, _ = _stream_batch(CONFIGS[name], S, first, B)
    for s in range(S):
        np.testing.assert_array_equal(got[s].view(np.uint32), want[s].view(np.uint32), err_msg="stream %d" % s)
    assert not np.array_equal(got[0], got[1])


def test_chain_streams_batch_vs_oracle(gpu):
    """stream 3 of a 4-stream cfg4-shaped (here cfg1) batch against the oracle chain on its own seed"""
    cfg = CONFIGS["cfg1"]
    got, _, tss = _stream_batch(cfg, 4, 0, 1)
    ts, base = tss[3]
    F = cfg.fecblocks
    bits, _ = O.BB(*cfg.bb_args()).work(ts, F)
    cells = O.IM(*cfg.im_args()).work(O.LDPC(cfg.framesize, cfg.rate).work(bits, F), F)
    pg = O.PG(*cfg.pg_args())
    car = pg.carriers(O.FM(*cfg.fm_args()).work(cells))
    iq_check.check_frame(got[3], car, pg.vlength, pg.guard, pg.normalization, pg.p1(), "cfg1 stream 3")
    iq_check.check_frame_exact(got[3], car, cfg.pg_args(), pg.guard, pg.normalization, "cfg1 stream 3")


@pytest.mark.parametrize("mode", ["hem", "hem_inband", "nm_inband"])
def test_chain_streams_batch_input_modes(gpu, mode):
    """the per-stream TS pointer in the HEM and in-band payload paths"""
    from test_cpu_plan import grid_cfg
    from dvbt2ll import enums as E
    over = dict(version=E.VERSION_131, tsrate=12345678)
    if mode.startswith("hem"):
        over["inputmode"] = E.INPUTMODE_HIEFF
    if mode.endswith("inband"):
        over["inband"] = E.INBAND_ON
    cfg = grid_cfg(over)
    got, want, _ = _stream_batch(cfg, 3, 2, 1)
    for s in range(3):
        np.testing.assert_array_equal(got[s].view(np.uint32), want[s].view(np.uint32), err_msg="stream %d" % s)


def test_chain_streams_batch_graph_sc16(gpu):
    """multi-stream batch through the hipGraph launch mode with the sc16 output step"""
    got, want, _ = _stream_batch(CONFIGS["cfg1"], 3, 1, 2, graph=True, sc16=True)
    for s in range(3):
        np.testing.assert_array_equal(got[s], want[s], err_msg="stream %d" % s)


def test_chain_streams_rejects_bad_args(gpu):
    import torch
    cfg = CONFIGS["cfg1"]
    ch = dvbt2ll.Chain(cfg, max_frames=4)
    ts, base = ts_for_frames(cfg, 0, 1)
    d = torch.from_numpy(np.tile(ts, 5)).cuda()
    iq = torch.empty((5 * ch.iq_per_frame, 2), dtype=torch.float32, device="cuda")
    for stride, S, B in ((len(ts), 5, 1), (len(ts), 2, 3), (len(ts) - 1, 2, 1), (len(ts), 0, 1)):
        with pytest.raises(dvbt2ll.DVBT2Error):
            ch.run_streams(d.data_ptr(), stride, S, base, len(ts), 0, B, iq.data_ptr())


from dvbt2ll import enums as E  # noqa: E402
from test_gpu_blocks import ALL_CODES, MODES  # noqa: E402


CW_CASES = [(m, i, E.MOD_16QAM) for m, i in MODES] + [(E.INPUTMODE_NORMAL, E.INBAND_OFF, E.MOD_QPSK)]


@pytest.mark.parametrize("framesize,rate", ALL_CODES)
@pytest.mark.parametrize("mode,inband,const", CW_CASES, ids=["nm", "hem", "nm-inband", "nm-qpsk"])
def test_chain_codewords_all_codes(gpu, framesize, rate, mode, inband, const):
    """the chain's FEC passes (BB pass, BCH on the matrix cores, LDPC pass) for every code x input
    mode: the packed interleaver-input codewords of two frames equal the oracle's bbheaderbch + ldpc
    output (info bits, then the parity interleaved [row a][column c] where the constellation has it)"""
    import plan_probe as PP
    cfg = CONFIGS["cfg4"].with_(framesize=framesize, rate=rate, inputmode=mode, inband=inband, constellation=const,
                                fecblocks=3)
    nb = 2 * cfg.fecblocks
    ch = dvbt2ll.Chain(cfg, max_frames=2)
    ch.debug_keep_codewords()
    ch.run(0, 2)
    got = ch.debug_codewords(nb)
    ts, base = ts_for_frames(cfg, 0, 2)
    assert base == 0
    bits, _ = O.BB(*cfg.bb_args()).work(ts, nb)
    fp = PP.fec_plan(framesize, rate, cfg.constellation)
    nbch, q = fp["nbch"], fp["q"]
    nldpc = 64800 if framesize else 16200
    cw = O.LDPC(framesize, rate).work(bits, nb).reshape(nb, nldpc)
    if fp["parity_il"]:
        t, s = np.divmod(np.arange(nldpc - nbch), 360)
        cw = cw.copy()
        cw[:, nbch:] = cw[:, nbch + q * s + t]
    want = np.packbits(cw, axis=1)
    bad = np.nonzero((got[:, :nldpc // 8] != want).any(axis=1))[0]
    assert bad.size == 0, ("blocks", bad.tolist())
