"""Multi-PLP T2 frames on the GPU (EN 302 755 8.3.6.3): several Type-1 data PLPs
per frame, each with its own TS stream, BBHEADER ISI (MIS), FEC, constellation, cell and time
interleaver, the L1-post carrying the PLP loops; through the fused chain and through the blocks,
bit-exact against the oracle generalised to several PLPs.

PARITY UNPINNED for nplp > 1: the reference carries one PLP (lib/framemapperfint_cc_impl.cc:152-250,
:1553-1691, :2029-2103).  A one-PLP frame through the same code paths is the reference's frame
(test_cpu_mplp.py, and every single-PLP test of this suite)."""
import dataclasses

import numpy as np
import pytest

import dvbt2ll
from dvbt2ll.configs import MPLP_CONFIGS, ts_for_frames
import oracle_lib as O
import iq_check

pytestmark = pytest.mark.gpu

NAMES = list(MPLP_CONFIGS)


def _device_ts(m, first, nframes):
    import torch
    bufs, bases, lens = [], [], []
    for k, p in enumerate(m.plps):
        ts, base = ts_for_frames(p, first, nframes, seed=k + 1)
        bufs.append(torch.from_numpy(ts).cuda())
        bases.append(base)
        lens.append(len(ts))
    return bufs, bases, lens


def _run(ch, m, first, nframes, fmt=dvbt2ll.IQ_CF32):
    import torch
    bufs, bases, lens = _device_ts(m, first, nframes)
    dt = torch.float32 if fmt == dvbt2ll.IQ_CF32 else torch.int16
    iq = torch.empty((nframes * ch.iq_per_frame, 2), dtype=dt, device="cuda")
    ch.run_plps([b.data_ptr() for b in bufs], bases, lens, first, nframes, iq.data_ptr(),
                torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = iq.cpu().numpy()
    return out.view(np.complex64).reshape(-1) if fmt == dvbt2ll.IQ_CF32 else out


def oracle_frames(m, nframes):
    """the oracle's per-PLP chains, the multi-PLP framemapper and pilotgen: per frame (carriers, mapped)"""
    cells, bits, cws = O.mplp_cells(m, 0, nframes)
    fm, pg = O.FMM(m), O.PG(*m.pg_args())
    out = []
    for c in cells:
        mapped = fm.work(c)
        out.append((pg.carriers(mapped), mapped))
    return out, pg, bits, cws


@pytest.mark.parametrize("name", NAMES)
def test_mplp_chain_iq(gpu, name):
    """TS of every PLP -> IQ, two T2 frames (two FRAME_IDX values), bit-exact against the CPU model of
    the GPU IFFT on the oracle's carriers and within SURVEY 8(c)'s bounds of a float64 IFFT"""
    m = MPLP_CONFIGS[name]
    ref, pg, _, _ = oracle_frames(m, 2)
    ch = dvbt2ll.Chain(m, max_frames=2)
    assert ch.nplp == m.nplp
    iq = _run(ch, m, 0, 2)
    per = ch.iq_per_frame
    for k in range(2):
        f = iq[k * per:(k + 1) * per]
        iq_check.check_frame(f, ref[k][0], pg.vlength, pg.guard, pg.normalization, pg.p1(), "%s frame %d" % (name, k))
        iq_check.check_frame_exact(f, ref[k][0], m.pg_args(), pg.guard, pg.normalization, "%s frame %d" % (name, k))


@pytest.mark.parametrize("name", NAMES)
def test_mplp_chain_codewords(gpu, name):
    """each PLP's packed codewords (BBHEADER with MIS / ISI = PLP_ID, BCH, LDPC, parity interleave) equal
    the oracle's bbheaderbch (orc_bb_set_isi) + ldpc output"""
    import plan_probe as PP
    m = MPLP_CONFIGS[name]
    _, _, bits, cws = oracle_frames(m, 1)
    ch = dvbt2ll.Chain(m, max_frames=1)
    ch.debug_keep_codewords()
    _run(ch, m, 0, 1)
    for k, p in enumerate(m.plps):
        got = ch.debug_plp_codewords(k, p.fecblocks)
        fp = PP.fec_plan(p.framesize, p.rate, p.constellation)
        nbch, q = fp["nbch"], fp["q"]
        nldpc = 64800 if p.framesize else 16200
        cw = cws[k][0].reshape(p.fecblocks, nldpc).copy()
        if fp["parity_il"]:
            t, s = np.divmod(np.arange(nldpc - nbch), 360)
            cw[:, nbch:] = cw[:, nbch + q * s + t]
        want = np.packbits(cw, axis=1)
        bad = np.nonzero((got[:, :nldpc // 8] != want).any(axis=1))[0]
        assert bad.size == 0, (name, "plp", k, bad.tolist())


def test_mplp_chain_frames_independent_and_graph(gpu):
    """frame 1 of a 2-PLP run computed alone equals frame 1 of the batch (the sharding basis holds with
    several PLPs); hipGraph mode and the sc16 output step give the direct launches' output"""
    m = MPLP_CONFIGS["mplp3_4k"]
    ch = dvbt2ll.Chain(m, max_frames=3)
    batch = _run(ch, m, 0, 3)
    per = ch.iq_per_frame
    one = _run(ch, m, 1, 1)
    np.testing.assert_array_equal(one.view(np.uint32), batch[per:2 * per].view(np.uint32))
    ch.set_graph(True)
    for _ in range(2):
        g = _run(ch, m, 0, 3)
        np.testing.assert_array_equal(g.view(np.uint32), batch.view(np.uint32))
    ch.set_output(0.2, dvbt2ll.IQ_SC16)
    sc = _run(ch, m, 0, 3, fmt=dvbt2ll.IQ_SC16)
    ref = np.clip(np.rint((batch.view(np.float32) * np.float32(0.2)) * np.float32(32767)), -32768,
                  32767).astype(np.int16)
    np.testing.assert_array_equal(sc.reshape(-1), ref)


def test_mplp_chain_rejects_bad_args(gpu):
    import torch
    m = MPLP_CONFIGS["mplp2_8k"]
    ch = dvbt2ll.Chain(m, max_frames=1)
    bufs, bases, lens = _device_ts(m, 0, 1)
    iq = torch.empty((ch.iq_per_frame, 2), dtype=torch.float32, device="cuda")
    ptrs = [b.data_ptr() for b in bufs]
    with pytest.raises(dvbt2ll.DVBT2Error):   # PLP 1's TS too short
        ch.run_plps(ptrs, bases, [lens[0], lens[1] - 200], 0, 1, iq.data_ptr())
    with pytest.raises(dvbt2ll.DVBT2Error):   # single-stream batch API on a multi-PLP chain
        ch.run_streams(ptrs[0], lens[0], 1, bases[0], lens[0], 0, 1, iq.data_ptr())
    with pytest.raises(dvbt2ll.DVBT2Error):   # a frame that cannot carry the PLPs
        dvbt2ll.Chain(m.with_(plps=m.plps + (dataclasses.replace(m.plps[0], fecblocks=30),)))


@pytest.mark.parametrize("name", ["mplp3_4k", "mplp2_8k"])
def test_mplp_blocks(gpu, name):
    """the drop-in path: per PLP bbheaderbch (set_isi) -> ldpc -> interleavermod, the multi-PLP
    framemapper (one port per PLP), pilotgen; each stage bit-exact against the oracle, two frames"""
    m = MPLP_CONFIGS[name]
    ref, pg, bits, cws = oracle_frames(m, 2)
    cells_o, _, _ = O.mplp_cells(m, 0, 2)
    fmb = dvbt2ll.framemapper_mplp_cc(m)
    pgb = dvbt2ll.pilotgenp1insert_cc(*m.pg_args())
    assert fmb.output_multiple() == O.FMM(m).mapped_items
    assert fmb.forecast(fmb.output_multiple()) == [fmb.stream_items(k) for k in range(m.nplp)]
    chains = []
    for k, p in enumerate(m.plps):
        bb = dvbt2ll.bbheaderbch_bb(*p.bb_args())
        bb.set_isi(k)
        chains.append((bb, dvbt2ll.ldpc_bb(p.framesize, p.rate), dvbt2ll.interleavermod_bc(*p.im_args()),
                       ts_for_frames(p, 0, 2, seed=k + 1)[0]))
    offs = [0] * m.nplp
    for f in range(2):
        ports = []
        for k, (p, (bb, ld, im, ts)) in enumerate(zip(m.plps, chains)):
            F = p.fecblocks
            b = np.zeros(F * bb.output_multiple(), np.uint8)
            bb.general_work([ts[offs[k]:]], [b])
            offs[k] += bb.last_consumed
            np.testing.assert_array_equal(b, bits[k][f], err_msg="bb plp %d frame %d" % (k, f))
            c = np.zeros(F * ld.output_multiple(), np.uint8)
            ld.general_work([b], [c])
            np.testing.assert_array_equal(c, cws[k][f], err_msg="ldpc plp %d frame %d" % (k, f))
            x = np.zeros(F * im.output_multiple(), np.complex64)
            im.general_work([c], [x])
            assert len(x) == fmb.stream_items(k)
            ports.append(x)
        np.testing.assert_array_equal(np.concatenate(ports).view(np.uint32), cells_o[f].view(np.uint32))
        mapped = np.zeros(fmb.output_multiple(), np.complex64)
        assert fmb.general_work(ports, [mapped]) == len(mapped)
        assert fmb.last_consumed == [len(x) for x in ports]
        np.testing.assert_array_equal(mapped.view(np.uint32), ref[f][1].view(np.uint32), err_msg="frame %d" % f)
        iq = np.zeros(pgb.output_multiple(), np.complex64)
        pgb.general_work([mapped], [iq])
        iq_check.check_frame_exact(iq, ref[f][0], m.pg_args(), pg.guard, pg.normalization, "%s blocks %d" % (name, f))
