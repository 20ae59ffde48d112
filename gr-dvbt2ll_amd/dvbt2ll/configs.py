"""Benchmark / parity configurations and the synthetic TS source.

cfg1 is the shipped GRC flowgraph (apps/vv009-4kshort.grc:524-709); cfg2-cfg5 are the
32K/8K configurations BASELINE.json names.  Every config uses INPUTMODE_NORMAL,
INBAND_OFF, VERSION_111, T2_SISO, PAPR_OFF, MISO_TX1, EQ_OFF, 8 MHz unless overridden.
"""
from dataclasses import dataclass, field, replace

import numpy as np

from .enums import *  # noqa: F401,F403
from . import enums as E

FFT_POINTS = {E.FFTSIZE_1K: 1024, E.FFTSIZE_2K: 2048, E.FFTSIZE_4K: 4096, E.FFTSIZE_8K: 8192,
              E.FFTSIZE_8K_T2GI: 8192, E.FFTSIZE_16K: 16384, E.FFTSIZE_16K_T2GI: 16384,
              E.FFTSIZE_32K: 32768, E.FFTSIZE_32K_T2GI: 32768}


@dataclass(frozen=True)
class T2Config:
    name: str
    framesize: int
    rate: int
    constellation: int
    rotation: int
    fecblocks: int
    tiblocks: int
    carriermode: int
    fftsize: int
    guardinterval: int
    l1constellation: int
    pilotpattern: int
    t2frames: int
    numdatasyms: int
    paprmode: int = E.PAPR_OFF
    version: int = E.VERSION_111
    preamble: int = E.PREAMBLE_T2_SISO
    inputmode: int = E.INPUTMODE_NORMAL
    reservedbiasbits: int = E.RESERVED_OFF
    l1scrambled: int = E.L1_SCRAMBLED_OFF
    inband: int = E.INBAND_OFF
    misogroup: int = E.MISO_TX1
    equalization: int = E.EQUALIZATION_OFF
    bandwidth: int = E.BANDWIDTH_8_0_MHZ
    tsrate: int = 4000000

    @property
    def vlength(self):
        return FFT_POINTS[self.fftsize]

    def bb_args(self):
        return (self.framesize, self.rate, self.inputmode, self.inband, self.fecblocks, self.tsrate)

    def im_args(self):
        return (self.framesize, self.rate, self.constellation, self.rotation)

    def fm_args(self):
        return (self.framesize, self.rate, self.constellation, self.rotation, self.fecblocks,
                self.tiblocks, self.carriermode, self.fftsize, self.guardinterval,
                self.l1constellation, self.pilotpattern, self.t2frames, self.numdatasyms,
                self.paprmode, self.version, self.preamble, self.inputmode,
                self.reservedbiasbits, self.l1scrambled, self.inband)

    def pg_args(self):
        return (self.carriermode, self.fftsize, self.pilotpattern, self.guardinterval,
                self.numdatasyms, self.paprmode, self.version, self.preamble, self.misogroup,
                self.equalization, self.bandwidth, self.vlength)

    def with_(self, **kw):
        return replace(self, **kw)


CONFIGS = {
    "cfg1": T2Config("cfg1-grc-4k-short-256qam-4/5", E.FECFRAME_SHORT, E.C4_5, E.MOD_256QAM, E.ROTATION_ON,
                     8, 3, E.CARRIERS_NORMAL, E.FFTSIZE_4K, E.GI_1_32, E.L1_MOD_64QAM, E.PILOT_PP7, 2, 3),
    "cfg2": T2Config("cfg2-32k-64qam-2/3-pp7", E.FECFRAME_NORMAL, E.C2_3, E.MOD_64QAM, E.ROTATION_OFF,
                     148, 3, E.CARRIERS_NORMAL, E.FFTSIZE_32K, E.GI_1_128, E.L1_MOD_64QAM, E.PILOT_PP7, 2, 59),
    "cfg3": T2Config("cfg3-32kext-256qam-3/5-pp4-rot", E.FECFRAME_NORMAL, E.C3_5, E.MOD_256QAM, E.ROTATION_ON,
                     195, 3, E.CARRIERS_EXTENDED, E.FFTSIZE_32K, E.GI_1_16, E.L1_MOD_64QAM, E.PILOT_PP4, 2, 59),
    "cfg4": T2Config("cfg4-8k-16qam-1/2-pp7", E.FECFRAME_NORMAL, E.C1_2, E.MOD_16QAM, E.ROTATION_OFF,
                     24, 3, E.CARRIERS_NORMAL, E.FFTSIZE_8K, E.GI_1_32, E.L1_MOD_64QAM, E.PILOT_PP7, 2, 59),
    "cfg5": T2Config("cfg5-32k-256qam-5/6-pp7", E.FECFRAME_NORMAL, E.C5_6, E.MOD_256QAM, E.ROTATION_OFF,
                     197, 3, E.CARRIERS_NORMAL, E.FFTSIZE_32K, E.GI_1_128, E.L1_MOD_64QAM, E.PILOT_PP7, 2, 59),
    # BASELINE.json config 1 as worded ("4K FFT, short FECFRAME, QPSK 1/2"): the GRC flowgraph's
    # other parameters, 2 FEC blocks (the frame's capacity, SURVEY 6: fecblocks <= 2); tiblocks 3
    # as in the GRC, i.e. one empty small TI block (framemapper:1114-1119)
    "cfg1q": T2Config("cfg1q-4k-short-qpsk-1/2", E.FECFRAME_SHORT, E.C1_2, E.MOD_QPSK, E.ROTATION_ON,
                      2, 3, E.CARRIERS_NORMAL, E.FFTSIZE_4K, E.GI_1_32, E.L1_MOD_64QAM, E.PILOT_PP7, 2, 3),
}

MAX_PLP = 8   # DVBT2LL_MAX_PLP
PLP_INTS = 14   # ints of dvbt2ll_plp_params


@dataclass(frozen=True)
class PlpConfig:
    """one data PLP of a multi-PLP T2 frame (EN 302 755 8.3.6.3; the reference carries one Type-1 PLP with
    TIME_IL_TYPE 0, lib/framemapperfint_cc_impl.cc:152-250): its FEC, constellation, time interleaver and
    input stream.  plp_type 2: sub-sliced (MplpConfig.num_subslices).  ti_type 1: one TI block
    (tiblocks = 1) of `fecblocks` FEC blocks per interleaving frame, spread over ti_frames (P_I) T2 frames
    (EN 302 755 6.5).  Quacks like T2Config for ts_for_frames / the per-PLP blocks."""
    framesize: int
    rate: int
    constellation: int
    rotation: int
    fecblocks: int
    tiblocks: int
    inputmode: int = E.INPUTMODE_NORMAL
    inband: int = E.INBAND_OFF
    tsrate: int = 4000000
    plp_type: int = 1
    ti_type: int = 0
    ti_frames: int = 1
    frame_interval: int = 1
    first_frame_idx: int = 0

    @property
    def if_frames(self):
        """T2 frames from one interleaving frame's first T2 frame to the next's (P_I x FRAME_INTERVAL)"""
        return (self.ti_frames if self.ti_type else 1) * self.frame_interval

    def starts_if(self, frame):
        """whether an interleaving frame of this PLP starts at T2 frame `frame`"""
        return frame % self.if_frames == self.first_frame_idx

    def bb_args(self):
        return (self.framesize, self.rate, self.inputmode, self.inband, self.fecblocks, self.tsrate)

    def im_args(self):
        return (self.framesize, self.rate, self.constellation, self.rotation)

    def plp_args(self):
        """the dvbt2ll_plp_params layout (include/dvbt2ll_hip.h)"""
        return (self.framesize, self.rate, self.constellation, self.rotation, self.fecblocks, self.tiblocks,
                self.inputmode, self.inband, self.tsrate, self.plp_type, self.ti_type, self.ti_frames,
                self.frame_interval, self.first_frame_idx)


@dataclass(frozen=True)
class MplpConfig:
    """a T2 frame carrying len(plps) data PLPs (PLP_ID = index, PLP 0's TS seed 1, PLP k's k + 1) with the
    common (frame / L1 / OFDM) parameters; num_subslices = SUB_SLICES_PER_FRAME of its Type-2 PLPs"""
    name: str
    plps: tuple
    carriermode: int
    fftsize: int
    guardinterval: int
    l1constellation: int
    pilotpattern: int
    t2frames: int
    numdatasyms: int
    paprmode: int = E.PAPR_OFF
    version: int = E.VERSION_111
    preamble: int = E.PREAMBLE_T2_SISO
    reservedbiasbits: int = E.RESERVED_OFF
    l1scrambled: int = E.L1_SCRAMBLED_OFF
    misogroup: int = E.MISO_TX1
    equalization: int = E.EQUALIZATION_OFF
    bandwidth: int = E.BANDWIDTH_8_0_MHZ
    num_subslices: int = 1

    @property
    def nplp(self):
        return len(self.plps)

    @property
    def unit_frames(self):
        """T2 frames of the chain's launch unit: the least common multiple of the PLPs' interleaving-frame
        lengths (every run covers whole interleaving frames of every PLP)"""
        import math
        u = 1
        for p in self.plps:
            u = u * p.if_frames // math.gcd(u, p.if_frames)
        return u

    @property
    def vlength(self):
        return FFT_POINTS[self.fftsize]

    def common_args(self):
        return (self.carriermode, self.fftsize, self.guardinterval, self.l1constellation, self.pilotpattern,
                self.t2frames, self.numdatasyms, self.paprmode, self.version, self.preamble, self.reservedbiasbits,
                self.l1scrambled)

    def mplp_array(self):
        """the dvbt2ll_mplp_params layout (include/dvbt2ll_hip.h) as ints"""
        assert 1 <= self.nplp <= MAX_PLP
        a = list(self.common_args()) + [self.nplp]
        for k in range(MAX_PLP):
            a += list(self.plps[k].plp_args()) if k < self.nplp else [0] * PLP_INTS
        return a + [self.num_subslices]

    def pg_args(self):
        return (self.carriermode, self.fftsize, self.pilotpattern, self.guardinterval, self.numdatasyms,
                self.paprmode, self.version, self.preamble, self.misogroup, self.equalization, self.bandwidth,
                self.vlength)

    def with_(self, **kw):
        return replace(self, **kw)


def _plp(cfg, **kw):
    d = dict(framesize=cfg.framesize, rate=cfg.rate, constellation=cfg.constellation, rotation=cfg.rotation,
             fecblocks=cfg.fecblocks, tiblocks=cfg.tiblocks, inputmode=cfg.inputmode, inband=cfg.inband,
             tsrate=cfg.tsrate)
    d.update(kw)
    return PlpConfig(**d)


def mplp_from(cfg, name, plps):
    """a multi-PLP frame with cfg's common parameters"""
    return MplpConfig(name, tuple(plps), cfg.carriermode, cfg.fftsize, cfg.guardinterval, cfg.l1constellation,
                      cfg.pilotpattern, cfg.t2frames, cfg.numdatasyms, cfg.paprmode, cfg.version, cfg.preamble,
                      cfg.reservedbiasbits, cfg.l1scrambled, cfg.misogroup, cfg.equalization, cfg.bandwidth)


KBCH = {(1, 0): 32208, (1, 1): 38688, (1, 2): 43040, (1, 3): 48408, (1, 4): 51648, (1, 5): 53840,
        (0, 6): 5232, (0, 7): 6312, (0, 0): 7032, (0, 1): 9552, (0, 2): 10632, (0, 3): 11712,
        (0, 4): 12432, (0, 5): 13152}

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def _mix(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def ts_packets(first_packet, npackets, seed=1):
    """Deterministic synthetic MPEG-TS: 188-byte packets, sync 0x47 then 187 bytes of
    splitmix64(seed) output.  Packet p's payload depends only on (seed, p), so any slice of
    the stream can be generated independently (frame- and rank-sharded runs)."""
    p = np.arange(first_packet, first_packet + npackets, dtype=np.uint64)
    n = p[:, None] * np.uint64(24) + np.arange(24, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        words = _mix(np.uint64(seed) + (n + np.uint64(1)) * _GOLDEN)
    body = words.view(np.uint8).reshape(npackets, 192)[:, :187]
    out = np.empty((npackets, 188), np.uint8)
    out[:, 0] = 0x47
    out[:, 1:] = body
    return out.reshape(-1)


def payload_bytes_per_block(cfg):
    return (KBCH[(cfg.framesize, cfg.rate)] - 80) // 8


def payload_pos(J, hem):
    """stream position of payload byte J (HEM drops every packet's sync byte)"""
    return 188 * (J // 187) + 1 + J % 187 if hem else J


def ts_for_frames(cfg, first_frame, nframes, seed=1):
    """TS bytes needed to encode T2 frames [first_frame, first_frame+nframes).  Returns
    (buffer, base_offset) where base_offset is the absolute stream offset of buffer[0]; the
    buffer starts one packet before the first packet touched so the CRC-8 of the preceding
    packet is available (NM).  Payload per interleaving frame (one T2 frame, or P_I of them for a
    TIME_IL_TYPE 1 PLP): F BBFRAME payloads, less the 13 in-band type B bytes of its first BBFRAME
    when in-band signalling is on (bbheader:327-355)."""
    hem = cfg.inputmode != E.INPUTMODE_NORMAL
    P = getattr(cfg, "if_frames", 1)
    assert first_frame % P == 0, "a run starts at an interleaving frame"
    u0, u1 = first_frame // P, -(-(first_frame + nframes) // P)
    per_frame = cfg.fecblocks * payload_bytes_per_block(cfg) - (13 if cfg.inband != E.INBAND_OFF else 0)
    start = payload_pos(u0 * per_frame, hem)
    end = payload_pos(u1 * per_frame, hem) + 1
    p0 = max(0, start // 188 - 1)
    p1 = (end + 187) // 188
    return ts_packets(p0, p1 - p0, seed), p0 * 188


def _mplp_configs():
    c3, c1, c4 = CONFIGS["cfg3"], CONFIGS["cfg1"], CONFIGS["cfg4"]
    return {
        # cfg3's frame split between a 256-QAM 3/5 rotated PLP and a 64-QAM 2/3 PLP (the bench's 2-PLP line)
        "mplp2_32k": mplp_from(c3, "mplp2-32kext-256qam3/5rot+64qam2/3", [
            _plp(c3, fecblocks=100), _plp(c3, rate=E.C2_3, constellation=E.MOD_64QAM, rotation=E.ROTATION_OFF,
                                          fecblocks=70, tiblocks=2)]),
        # three PLPs filling the GRC's 4K short frame exactly (no dummy cells): 256-QAM 4/5 rotated, QPSK 1/2,
        # 16-QAM 3/5 HEM in two TI blocks (one of them empty)
        "mplp3_4k": mplp_from(c1, "mplp3-4k-short", [
            _plp(c1, fecblocks=2, tiblocks=1),
            _plp(c1, rate=E.C1_2, constellation=E.MOD_QPSK, rotation=E.ROTATION_OFF, fecblocks=1, tiblocks=0),
            _plp(c1, rate=E.C3_5, constellation=E.MOD_16QAM, fecblocks=1, tiblocks=2,
                 inputmode=E.INPUTMODE_HIEFF)]),
        # two 8K PLPs, normal + short FECFRAME
        "mplp2_8k": mplp_from(c4, "mplp2-8k-16qam1/2+short-256qam", [
            _plp(c4, fecblocks=12),
            _plp(c4, framesize=E.FECFRAME_SHORT, rate=E.C2_3, constellation=E.MOD_256QAM, rotation=E.ROTATION_ON,
                 fecblocks=10, tiblocks=1)]),
        # two 8K PLPs without a 256-QAM one: the OFDM kernel's constellation tables hold 4 + 16 = 20 entries
        # (fewer than the 256 a single-PLP table holds)
        "mplp2_8k_lowq": mplp_from(c4, "mplp2-8k-16qam1/2+qpsk3/4", [
            _plp(c4, fecblocks=12, tiblocks=2),
            _plp(c4, rate=E.C3_4, constellation=E.MOD_QPSK, fecblocks=5, tiblocks=1)]),
        # three 32K PLPs (one in-band type B, v1.3.1 L1 scrambling)
        "mplp3_32k": mplp_from(CONFIGS["cfg5"], "mplp3-32k-v131", [
            _plp(CONFIGS["cfg5"], fecblocks=60, tiblocks=1),
            _plp(CONFIGS["cfg5"], rate=E.C1_2, constellation=E.MOD_16QAM, rotation=E.ROTATION_ON, fecblocks=30,
                 tiblocks=2, inband=E.INBAND_ON, tsrate=7654321),
            _plp(CONFIGS["cfg5"], rate=E.C3_4, constellation=E.MOD_QPSK, fecblocks=15, tiblocks=0)]).with_(
                version=E.VERSION_131, l1scrambled=E.L1_SCRAMBLED_ON, l1constellation=E.L1_MOD_16QAM),
    }


MPLP_CONFIGS = _mplp_configs()


def _if_configs():
    """frames whose PLPs use EN 302 755 beyond the reference's one Type-1 TIME_IL_TYPE 0 PLP (SURVEY 8(f)
    rank 4): TIME_IL_TYPE 1 (one TI block spread over P_I T2 frames) and sub-sliced Type-2 PLPs"""
    c3, c1, c4, c5 = CONFIGS["cfg3"], CONFIGS["cfg1"], CONFIGS["cfg4"], CONFIGS["cfg5"]
    return {
        # cfg3's frame as one TIME_IL_TYPE 1 PLP: 390 FEC blocks in one TI block over P_I = 2 T2 frames (each
        # T2 frame carries cfg3's 195 blocks' worth of cells; the frame boundary falls between TI rows)
        "ti1_32k_p2": mplp_from(c3, "ti1-32kext-256qam3/5rot-PI2", [
            _plp(c3, fecblocks=390, tiblocks=1, ti_type=1, ti_frames=2)]),
        # cfg4's 8K frame as one TIME_IL_TYPE 1 PLP over P_I = 4 T2 frames (96 FEC blocks, HEM input), four T2
        # frames per superframe
        "ti1_8k_p4": mplp_from(c4, "ti1-8k-16qam1/2-PI4-hem", [
            _plp(c4, fecblocks=96, tiblocks=1, ti_type=1, ti_frames=4, inputmode=E.INPUTMODE_HIEFF)]).with_(
                t2frames=4),
        # cfg3's frame as a Type-1 PLP (256-QAM 3/5 rotated) and a Type-2 PLP (64-QAM 2/3, in-band type B,
        # v1.3.1) in 50 sub-slices
        "t2sub_32k": mplp_from(c3, "t2sub-32kext-type1+type2x50", [
            _plp(c3, fecblocks=100),
            _plp(c3, rate=E.C2_3, constellation=E.MOD_64QAM, rotation=E.ROTATION_OFF, fecblocks=70, tiblocks=2,
                 plp_type=2, inband=E.INBAND_ON, tsrate=5555555)]).with_(num_subslices=50, version=E.VERSION_131),
        # the GRC's 4K short frame with both extensions at once: a Type-2 TIME_IL_TYPE 1 PLP (256-QAM 4/5 short,
        # 4 FEC blocks over P_I = 2 frames: 405 TI rows, so the frame boundary cuts a row), a Type-1 QPSK PLP and
        # a Type-2 16-QAM HEM PLP, 6 sub-slices
        "mix_4k": mplp_from(c1, "mix-4k-short-type2PI2+type1+type2", [
            _plp(c1, fecblocks=4, tiblocks=1, ti_type=1, ti_frames=2, plp_type=2),
            _plp(c1, rate=E.C1_2, constellation=E.MOD_QPSK, rotation=E.ROTATION_OFF, fecblocks=1, tiblocks=1),
            _plp(c1, rate=E.C3_5, constellation=E.MOD_16QAM, fecblocks=1, tiblocks=1, plp_type=2,
                 inputmode=E.INPUTMODE_HIEFF)]).with_(num_subslices=6),
        # FRAME_INTERVAL: cfg3's frame with a 256-QAM PLP in every T2 frame and a 64-QAM PLP in the odd ones only
        # (I_JUMP 2, FIRST_FRAME_IDX 1): the even frames carry dummy cells in its place
        "ij2_32k": mplp_from(c3, "ij2-32kext-every+odd", [
            _plp(c3, fecblocks=100),
            _plp(c3, rate=E.C2_3, constellation=E.MOD_64QAM, rotation=E.ROTATION_OFF, fecblocks=70, tiblocks=2,
                 frame_interval=2, first_frame_idx=1)]),
        # one 4K short PLP every other T2 frame (I_JUMP 2): frames 1, 3, .. carry no data cells at all
        "ij2_4k_single": mplp_from(c1, "ij2-4k-short-single", [_plp(c1, frame_interval=2)]),
        # 8K, four frame classes: a Type-2 16-QAM PLP every 2nd frame, a Type-1 QPSK TIME_IL_TYPE 1 PLP (P_I = 2)
        # every 4th frame from frame 3 (interleaving frames of frames 3 + 8 m, 7 + 8 m), a Type-2 64-QAM PLP in
        # every frame; 10 sub-slices, superframe of 8 T2 frames
        "ij_mix_8k": mplp_from(c4, "ij-mix-8k", [
            _plp(c4, fecblocks=12, tiblocks=2, plp_type=2, frame_interval=2),
            _plp(c4, rate=E.C3_4, constellation=E.MOD_QPSK, rotation=E.ROTATION_ON, fecblocks=4, tiblocks=1,
                 ti_type=1, ti_frames=2, frame_interval=4, first_frame_idx=3),
            _plp(c4, rate=E.C2_3, constellation=E.MOD_64QAM, fecblocks=6, tiblocks=1, plp_type=2)]).with_(
                t2frames=8, num_subslices=10),
        # 32K, two PLPs with different interleaving-frame lengths (P_I = 2 and 4: launch unit 4 frames)
        "ti1_32k_p2p4": mplp_from(c5, "ti1-32k-PI2+PI4", [
            _plp(c5, fecblocks=120, tiblocks=1, ti_type=1, ti_frames=2),
            _plp(c5, rate=E.C1_2, constellation=E.MOD_16QAM, rotation=E.ROTATION_ON, fecblocks=200, tiblocks=1,
                 ti_type=1, ti_frames=4)]).with_(t2frames=4),
    }


IF_CONFIGS = _if_configs()
