"""IQ parity bounds after the IFFT, shared by the GPU tests and smoke().

The reference's IFFT backend (FFTW3f through gr-fft) is absent, so IQ cannot be compared bit for bit
with it.  Everything up to the pre-IFFT carrier vector is checked bit-exactly elsewhere; after the
IFFT the GPU output is compared with a float64 IFFT of the oracle's carriers:

    relative RMS error  ||y - x|| / ||x||          <= 1e-6
    maximum error       max |y - x| / rms(x)       <= 1e-5

and, for the record, with the error of numpy's single-precision pocketfft (an FFTW-class float
FFT) on the same carriers.  Set IQ_STATS=<file> to append every measured pair as JSON lines.
"""
import json
import os

import numpy as np

REL_RMS_MAX = 1e-6
MAX_REL_MAX = 1e-5


def symbol_reference(carriers, N, G, norm):
    """float64 IFFT (pilotgen:2890-2896: fftshift, backward FFT, scale, cyclic prefix)"""
    x = np.fft.ifft(np.fft.fftshift(carriers.astype(np.complex128))) * N * norm
    return np.concatenate([x[N - G:], x])


def errors(y, want):
    d = np.asarray(y, np.complex128) - want
    rms = np.sqrt(np.mean(np.abs(want) ** 2))
    return float(np.linalg.norm(d) / np.linalg.norm(want)), float(np.abs(d).max() / rms)


def f32_reference_errors(carriers, N, G, norm, want):
    """error of an FFTW-class single-precision IFFT (numpy pocketfft on complex64)"""
    x = np.fft.ifft(np.fft.fftshift(carriers.astype(np.complex64))) * np.float32(N) * np.float32(norm)
    return errors(np.concatenate([x[N - G:], x]).astype(np.complex64), want)


def check_symbol(y, carriers, N, G, norm, ctx=""):
    want = symbol_reference(carriers, N, G, norm)
    rel, mx = errors(y, want)
    path = os.environ.get("IQ_STATS")
    if path:
        f_rel, f_mx = f32_reference_errors(carriers, N, G, norm, want)
        with open(path, "a") as fh:
            fh.write(json.dumps({"ctx": ctx, "N": N, "rel_rms": rel, "max_rel": mx,
                                 "f32_rel_rms": f_rel, "f32_max_rel": f_mx}) + "\n")
    assert rel <= REL_RMS_MAX and mx <= MAX_REL_MAX, "%s: IQ rel rms %.3g (<= %g), max %.3g of rms (<= %g)" % (
        ctx, rel, REL_RMS_MAX, mx, MAX_REL_MAX)
    return rel, mx


def check_p1(y, want, ctx=""):
    """P1 symbol (pilotgen:1119-1178, 2802-2810): the same two bounds, relative to the P1 rms"""
    rel, mx = errors(y, np.asarray(want, np.complex128))
    assert rel <= REL_RMS_MAX and mx <= MAX_REL_MAX, "%s: P1 rel rms %.3g, max %.3g of rms" % (ctx, rel, mx)
    return rel, mx


def check_frame(iq, carriers, N, G, norm, p1, ctx=""):
    """one T2 frame of IQ: P1 then carriers.shape[0] symbols of G + N samples; returns worst errors"""
    worst = list(check_p1(iq[:2048], p1, ctx))
    for j in range(carriers.shape[0]):
        y = iq[2048 + j * (N + G): 2048 + (j + 1) * (N + G)]
        rel, mx = check_symbol(y, carriers[j], N, G, norm, "%s sym %d" % (ctx, j))
        worst = [max(worst[0], rel), max(worst[1], mx)]
    return worst


_P1 = {}


def _oracle_p1(pg_args):
    """the oracle's P1 samples for these pilotgen arguments (cached: the oracle evaluates its DFT term by term)"""
    key = tuple(pg_args)
    if key not in _P1:
        import oracle_lib as O
        _P1[key] = O.PG(*pg_args).p1()
    return _P1[key]


def check_frame_exact(iq, carriers, pg_args, G, norm, ctx="", gain=1.0, fmt=0):
    """SURVEY 8(c)'s bit-exact bar between the CPU restatement and the GPU: the frame equals, bit for
    bit, the oracle's carriers put through oracle/ifft_model.c (the OFDM kernels' operation order)
    with the oracle's P1 samples (the planner's, which the GPU copies, are bit-equal to them:
    test_cpu_plan).  Returns the number of samples compared."""
    import oracle_lib as O
    want = O.model_frame(carriers, G, norm, _oracle_p1(pg_args), gain, fmt)
    got = np.asarray(iq)
    assert got.shape == want.shape, (ctx, got.shape, want.shape)
    a, b = got.view(np.uint32).reshape(-1), want.view(np.uint32).reshape(-1)
    bad = np.nonzero(a != b)[0]
    assert bad.size == 0, "%s: %d of %d IQ words differ from the CPU model of the GPU IFFT, first at %s" % (
        ctx, bad.size, a.size, bad[:5])
    return a.size
