"""TIME_IL_TYPE 1 interleaving frames (one TI block over P_I T2 frames), FRAME_INTERVAL > 1 (PLPs in every
I_JUMP-th T2 frame only: frame classes) and sub-sliced Type-2 PLPs on the GPU (EN 302 755
6.5, 7.2.3.1, 8.3.6.3): the fused chain and the drop-in blocks, bit-exact against the
oracle's framemapper generalised to both (test_cpu_ti.py pins the planner to it on the CPU).

PARITY UNPINNED: the reference implements TIME_IL_TYPE 0 Type-1 PLPs only (lib/framemapperfint_cc_impl.cc:159,
198-200, 1999-2028)."""
import dataclasses

import numpy as np
import pytest

import dvbt2ll
from dvbt2ll.configs import IF_CONFIGS, ts_for_frames
import oracle_lib as O
import iq_check
from test_gpu_mplp import _device_ts, _run, oracle_frames

pytestmark = pytest.mark.gpu

NAMES = list(IF_CONFIGS)


@pytest.mark.parametrize("name", NAMES)
def test_if_chain_iq(gpu, name):
    """TS of every PLP -> IQ over two launch units (two interleaving frames of the longest PLP), every T2
    frame bit-exact against the CPU model of the GPU IFFT on the oracle's carriers and within SURVEY 8(c)'s
    bounds of a float64 IFFT"""
    m = IF_CONFIGS[name]
    n = 2 * m.unit_frames
    ref, pg, _, _ = oracle_frames(m, n)
    ch = dvbt2ll.Chain(m, max_frames=n)
    assert ch.unit_frames == m.unit_frames
    assert [i["frames_per_if"] for i in ch.plp_info] == [p.if_frames for p in m.plps]
    iq = _run(ch, m, 0, n)
    per = ch.iq_per_frame
    for k in range(n):
        f = iq[k * per:(k + 1) * per]
        iq_check.check_frame(f, ref[k][0], pg.vlength, pg.guard, pg.normalization, pg.p1(), "%s frame %d" % (name, k))
        iq_check.check_frame_exact(f, ref[k][0], m.pg_args(), pg.guard, pg.normalization, "%s frame %d" % (name, k))


@pytest.mark.parametrize("name", NAMES)
def test_if_chain_codewords(gpu, name):
    """each PLP's packed codewords of its first interleaving frame (fecblocks FEC blocks, whatever P_I)"""
    import plan_probe as PP
    m = IF_CONFIGS[name]
    u = m.unit_frames
    _, _, bits, cws = oracle_frames(m, u)
    ch = dvbt2ll.Chain(m, max_frames=u)
    ch.debug_keep_codewords()
    _run(ch, m, 0, u)
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


@pytest.mark.parametrize("name", ["ti1_8k_p4", "mix_4k", "ti1_32k_p2p4", "ij_mix_8k", "ij2_4k_single"])
def test_if_chain_units_independent(gpu, name):
    """the sharding unit: launch unit 1 (frames u .. 2u - 1) encoded alone equals the same frames of a
    two-unit batch; runs that do not start or end on a unit boundary are refused"""
    m = IF_CONFIGS[name]
    u = m.unit_frames
    ch = dvbt2ll.Chain(m, max_frames=2 * u)
    batch = _run(ch, m, 0, 2 * u)
    per = ch.iq_per_frame
    one = _run(ch, m, u, u)
    np.testing.assert_array_equal(one.view(np.uint32), batch[u * per:].view(np.uint32))
    import torch
    bufs, bases, lens = _device_ts(m, 0, 2 * u)
    iq = torch.empty((2 * u * per, 2), dtype=torch.float32, device="cuda")
    ptrs = [b.data_ptr() for b in bufs]
    for first, nframes in ((1, u), (0, u + 1), (0, u - 1) if u > 1 else (1, 1)):
        with pytest.raises(dvbt2ll.DVBT2Error):
            ch.run_plps(ptrs, bases, lens, first, nframes, iq.data_ptr())


def test_if_chain_graph_sc16(gpu):
    """hipGraph mode and the sc16 output step on a chain with interleaving frames over several T2 frames"""
    m = IF_CONFIGS["mix_4k"]
    ch = dvbt2ll.Chain(m, max_frames=4)
    batch = _run(ch, m, 0, 4)
    ch.set_graph(True)
    for _ in range(2):
        np.testing.assert_array_equal(_run(ch, m, 0, 4).view(np.uint32), batch.view(np.uint32))
    ch.set_output(0.2, dvbt2ll.IQ_SC16)
    sc = _run(ch, m, 0, 4, fmt=dvbt2ll.IQ_SC16)
    ref = np.clip(np.rint((batch.view(np.float32) * np.float32(0.2)) * np.float32(32767)), -32768,
                  32767).astype(np.int16)
    np.testing.assert_array_equal(sc.reshape(-1), ref)


def test_if_chain_rejects_bad_config(gpu):
    m = IF_CONFIGS["ti1_8k_p4"]
    with pytest.raises(dvbt2ll.DVBT2Error):          # max_frames below the launch unit
        dvbt2ll.Chain(m, max_frames=2)
    with pytest.raises(dvbt2ll.DVBT2Error):          # TIME_IL_TYPE 1 with two TI blocks
        dvbt2ll.Chain(m.with_(plps=(dataclasses.replace(m.plps[0], tiblocks=2),)), max_frames=4)
    with pytest.raises(dvbt2ll.DVBT2Error):          # sub-slices without a Type-2 PLP
        dvbt2ll.Chain(m.with_(num_subslices=3), max_frames=4)


@pytest.mark.parametrize("name", ["mix_4k", "ti1_8k_p4", "ij_mix_8k"])
def test_if_blocks(gpu, name):
    """the drop-in path: per PLP bbheaderbch (set_isi) -> ldpc -> interleavermod once per interleaving
    frame, the multi-PLP framemapper (a TIME_IL_TYPE 1 port delivers its interleaving frame on the first of
    its T2 frames, nothing on the others), pilotgen; each stage bit-exact against the oracle over two units"""
    m = IF_CONFIGS[name]
    n = 2 * m.unit_frames
    ref, pg, bits, cws = oracle_frames(m, n)
    fmb = dvbt2ll.framemapper_mplp_cc(m)
    pgb = dvbt2ll.pilotgenp1insert_cc(*m.pg_args())
    chains = []
    for k, p in enumerate(m.plps):
        bb = dvbt2ll.bbheaderbch_bb(*p.bb_args())
        if m.nplp > 1:
            bb.set_isi(k)
        chains.append((bb, dvbt2ll.ldpc_bb(p.framesize, p.rate), dvbt2ll.interleavermod_bc(*p.im_args()),
                       ts_for_frames(p, 0, n, seed=k + 1)[0]))
    offs = [0] * m.nplp
    ifs = [0] * m.nplp
    for f in range(n):
        want_in = fmb.forecast(fmb.output_multiple())
        ports = []
        for k, (p, (bb, ld, im, ts)) in enumerate(zip(m.plps, chains)):
            if not p.starts_if(f):
                assert want_in[k] == 0
                ports.append(np.zeros(0, np.complex64))
                continue
            F = p.fecblocks
            b = np.zeros(F * bb.output_multiple(), np.uint8)
            bb.general_work([ts[offs[k]:]], [b])
            offs[k] += bb.last_consumed
            np.testing.assert_array_equal(b, bits[k][ifs[k]], err_msg="bb plp %d frame %d" % (k, f))
            c = np.zeros(F * ld.output_multiple(), np.uint8)
            ld.general_work([b], [c])
            np.testing.assert_array_equal(c, cws[k][ifs[k]], err_msg="ldpc plp %d frame %d" % (k, f))
            x = np.zeros(F * im.output_multiple(), np.complex64)
            im.general_work([c], [x])
            assert want_in[k] == len(x)
            ports.append(x)
            ifs[k] += 1
        mapped = np.zeros(fmb.output_multiple(), np.complex64)
        assert fmb.general_work(ports, [mapped]) == len(mapped)
        assert fmb.last_consumed == [len(x) for x in ports]
        np.testing.assert_array_equal(mapped.view(np.uint32), ref[f][1].view(np.uint32), err_msg="frame %d" % f)
        iq = np.zeros(pgb.output_multiple(), np.complex64)
        pgb.general_work([mapped], [iq])
        iq_check.check_frame_exact(iq, ref[f][0], m.pg_args(), pg.guard, pg.normalization, "%s blocks %d" % (name, f))


def test_if_chain_large_batch(gpu):
    """the benched shape of ti1_32k_p2: 256 T2 frames (128 interleaving frames of 390 FEC blocks) in one
    launch; the last unit and a middle unit equal the same frames encoded alone (size-independent check at
    scale)"""
    import torch
    m = IF_CONFIGS["ti1_32k_p2"]
    B = 256
    ch = dvbt2ll.Chain(m, max_frames=B)
    per = ch.iq_per_frame
    bufs, bases, lens = _device_ts(m, 0, B)
    iq = torch.empty((B * per, 2), dtype=torch.float32, device="cuda")
    ch.run_plps([b.data_ptr() for b in bufs], bases, lens, 0, B, iq.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for first in (B // 2, B - 2):
        one = _run(ch, m, first, 2)
        got = iq[first * per:(first + 2) * per].cpu().numpy().view(np.complex64).reshape(-1)
        np.testing.assert_array_equal(one.view(np.uint32), got.view(np.uint32))


@pytest.mark.parametrize("name", ["mix_4k", "mplp3_4k"])
def test_tx_tool_mplp(gpu, tmp_path, name):
    """dvbt2ll_tx --mplp (one TS file per PLP, batches of whole launch units, dvbt2ll_chain_run_plps_host)
    writes exactly the chain's IQ"""
    import subprocess
    from pathlib import Path
    from dvbt2ll.configs import MPLP_CONFIGS
    m = {**MPLP_CONFIGS, **IF_CONFIGS}[name]
    n = 4 * m.unit_frames
    args = []
    for k, p in enumerate(m.plps):
        ts, base = ts_for_frames(p, 0, n, seed=k + 1)
        assert base == 0
        (tmp_path / ("p%d.ts" % k)).write_bytes(ts.tobytes())
        args += ["--in", str(tmp_path / ("p%d.ts" % k))]
    tool = Path(__file__).resolve().parents[1] / "gr-dvbt2ll_amd" / "dvbt2ll" / "dvbt2ll_tx"
    r = subprocess.run([str(tool), "--mplp", name, *args, "--out", str(tmp_path / "iq.bin"), "--batch",
                        str(2 * m.unit_frames), "--frames", str(n)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    ch = dvbt2ll.Chain(m, max_frames=n)
    want = _run(ch, m, 0, n)
    got = np.frombuffer((tmp_path / "iq.bin").read_bytes(), dtype=np.complex64)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
