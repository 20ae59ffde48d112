"""The CPU restatement of the GPU IFFT (oracle/ifft_model.c): its twiddle tables are
the planner's, bit for bit, and its output is within the 8(c) IQ bounds of a float64 IFFT of the
oracle's carriers for every FFT size.  The GPU tests then require the kernels' IQ to equal this
model bit for bit (iq_check.check_frame_exact)."""
import numpy as np
import pytest

from dvbt2ll.configs import CONFIGS, ts_for_frames
import oracle_lib as O
import plan_probe as PP
import iq_check
from test_cpu_plan import GRID, grid_cfg


def _carriers(cfg):
    ts, _ = ts_for_frames(cfg, 0, 1)
    F = cfg.fecblocks
    bits, _ = O.BB(*cfg.bb_args()).work(ts, F)
    cells = O.IM(*cfg.im_args()).work(O.LDPC(cfg.framesize, cfg.rate).work(bits, F), F)
    pg = O.PG(*cfg.pg_args())
    return pg.carriers(O.FM(*cfg.fm_args()).work(cells)), pg


CASES = [(n, CONFIGS[n]) for n in ("cfg1", "cfg1q", "cfg2", "cfg3", "cfg4", "cfg5")] + \
        [(g[0], grid_cfg(g[1])) for g in GRID]


@pytest.mark.parametrize("name,cfg", CASES, ids=[c[0] for c in CASES])
def test_model_tables_equal_planner(name, cfg):
    tw, tw1k = PP.twiddle_tables(cfg.pg_args())
    mt, m1 = O.model_tables(int(cfg.pg_args()[11]))
    np.testing.assert_array_equal(tw.view(np.uint32), mt.view(np.uint32))
    np.testing.assert_array_equal(tw1k.view(np.uint32), m1.view(np.uint32))


@pytest.mark.parametrize("name,cfg", CASES, ids=[c[0] for c in CASES])
def test_model_within_iq_bounds(name, cfg):
    car, pg = _carriers(cfg)
    p1 = PP.pilot_plan(cfg.pg_args())["p1"]
    iq = O.model_frame(car, pg.guard, pg.normalization, p1)
    assert len(iq) == pg.output_items
    iq_check.check_frame(iq, car, pg.vlength, pg.guard, pg.normalization, pg.p1(), "model " + name)


def test_model_output_step():
    """gain and sc16 in the model: the float product per component, then saturate(rint(x 32767))"""
    cfg = CONFIGS["cfg1"]
    car, pg = _carriers(cfg)
    p1 = PP.pilot_plan(cfg.pg_args())["p1"]
    base = O.model_frame(car, pg.guard, pg.normalization, p1)
    g = O.model_frame(car, pg.guard, pg.normalization, p1, gain=0.2)
    np.testing.assert_array_equal(g.view(np.float32), base.view(np.float32) * np.float32(0.2))
    s = O.model_frame(car, pg.guard, pg.normalization, p1, gain=0.2, fmt=1)
    want = np.clip(np.rint(g.view(np.float32) * np.float32(32767)), -32768, 32767).astype(np.int16)
    np.testing.assert_array_equal(s.reshape(-1), want)


@pytest.mark.parametrize("N", [1024, 2048, 4096, 8192, 16384, 32768])
def test_model_random_symbols(N):
    """unit-variance random carriers (every bin active) for each transform size: the 8(c) bounds"""
    rng = np.random.default_rng(N)
    car = (rng.standard_normal((2, N)) + 1j * rng.standard_normal((2, N))).astype(np.complex64)
    G = N // 8
    y = O.model_symbols(car, G, 0.01)
    for j in range(2):
        iq_check.check_symbol(y[j * (N + G):(j + 1) * (N + G)], car[j], N, G, 0.01, "random N=%d" % N)
