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
    packet is available (NM).  Payload per frame: F BBFRAME payloads, less the 13 in-band type
    B bytes of the frame's first BBFRAME when in-band signalling is on (bbheader:327-355)."""
    hem = cfg.inputmode != E.INPUTMODE_NORMAL
    per_frame = cfg.fecblocks * payload_bytes_per_block(cfg) - (13 if cfg.inband != E.INBAND_OFF else 0)
    start = payload_pos(first_frame * per_frame, hem)
    end = payload_pos((first_frame + nframes) * per_frame, hem) + 1
    p0 = max(0, start // 188 - 1)
    p1 = (end + 187) // 188
    return ts_packets(p0, p1 - p0, seed), p0 * 188
