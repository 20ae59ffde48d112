"""L1-post signalling generated per T2 frame on the GPU (l1post_kernel,
framemapper:1536-1910) instead of host-encoded t2_frame_num variants.  Checked bit-exactly against
the oracle framemapper (which re-encodes L1-post every frame) through the framemapper block, for
t2frames = 255 over a whole FRAME_IDX cycle and its wrap, every L1 constellation, v1.1.1 and v1.3.1
(L1 scrambler, bias bits); and through the fused chain at frame indices around the wrap."""
import numpy as np
import pytest

import dvbt2ll
from dvbt2ll.configs import CONFIGS, ts_for_frames
import oracle_lib as O
import iq_check
from test_cpu_plan import grid_cfg

pytestmark = pytest.mark.gpu

V131 = dict(version=2, l1scrambled=1, reservedbiasbits=1)


def _cells(cfg, seed=3):
    rng = np.random.default_rng(seed)
    fm = O.FM(*cfg.fm_args())
    S = fm.stream_items
    return (rng.standard_normal(S) + 1j * rng.standard_normal(S)).astype(np.complex64)


@pytest.mark.parametrize("l1c", [0, 1, 2, 3])
@pytest.mark.parametrize("extra", [dict(), V131], ids=["v111", "v131"])
def test_framemapper_l1post_every_frame_idx(gpu, l1c, extra):
    cfg = grid_cfg(dict(l1constellation=l1c, t2frames=255, **extra))
    cells = _cells(cfg)
    fm = O.FM(*cfg.fm_args())
    blk = dvbt2ll.framemapperfint_cc(*cfg.fm_args())
    got = np.zeros(fm.mapped_items, np.complex64)
    for frame in range(258):     # FRAME_IDX 0..254, then the wrap to 0..2
        want = fm.work(cells)
        assert blk.general_work([cells], [got]) == fm.mapped_items
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), "frame %d" % frame


@pytest.mark.parametrize("name,over", [("cfg1_t2f255", dict(t2frames=255)),
                                       ("v131_16qam", dict(t2frames=7, l1constellation=2, **V131)),
                                       ("np2_4_64qam", dict(t2frames=5, l1constellation=3))])
def test_chain_l1post_across_frame_idx_wrap(gpu, name, over):
    """chain IQ bit-exact (CPU model of the GPU IFFT over the oracle carriers) at frames whose
    FRAME_IDX wraps, in one launch and as a two-stream batch"""
    import torch
    cfg = grid_cfg(over)
    T = cfg.t2frames
    first, n = T - 2, 4
    F = cfg.fecblocks
    ts, base = ts_for_frames(cfg, 0, first + n)
    bb = O.BB(*cfg.bb_args()); ld = O.LDPC(cfg.framesize, cfg.rate); im = O.IM(*cfg.im_args())
    fm = O.FM(*cfg.fm_args()); pg = O.PG(*cfg.pg_args())
    off, cars = 0, []
    for k in range(first + n):
        bits, cons = bb.work(ts[off:], F)
        off += cons
        mapped = fm.work(im.work(ld.work(bits, F), F))
        if k >= first:
            cars.append(pg.carriers(mapped))
    ch = dvbt2ll.Chain(cfg, max_frames=2 * n)
    per = ch.iq_per_frame
    iq = ch.run(first, n, ts=ts, ts_base=base)
    for k in range(n):
        iq_check.check_frame_exact(iq[k * per:(k + 1) * per], cars[k], cfg.pg_args(), pg.guard, pg.normalization,
                                   "%s frame %d" % (name, first + k))
    # the same frames as stream 1 of a 2-stream batch (stream 0: another seed)
    ts0, b0 = ts_for_frames(cfg, first, n, seed=9)
    ts1, b1 = ts_for_frames(cfg, first, n, seed=1)
    assert b0 == b1 and len(ts0) == len(ts1)
    stride = (len(ts0) + 255) // 256 * 256
    buf = np.zeros((2, stride), np.uint8)
    buf[0, :len(ts0)] = ts0
    buf[1, :len(ts1)] = ts1
    d = torch.from_numpy(buf.reshape(-1)).cuda()
    out = torch.empty((2 * n * per, 2), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ch.run_streams(d.data_ptr(), stride, 2, b0, len(ts0), first, n, out.data_ptr())
    ch.synchronize()
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.complex64).reshape(2, n * per)
    np.testing.assert_array_equal(got[1].view(np.uint32), iq.view(np.uint32))
