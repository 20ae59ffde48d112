#!/usr/bin/env python3
"""Phase-serial bound of the 32K OFDM kernel from one session's counters:

    python tools/ofdm_phase_model.py profiles/r3_r3f1_pmc_sq.txt profiles/r3_r3f1_bench.json

With one 16-wave workgroup per CU (the symbol fills the register file) and barriers between the
kernel's phases, each phase is bound by one resource and the phases of one symbol do not overlap:
the LDS scatter / read-back / exchanges by the LDS array, the DFT-32 stages and twiddles by VALU
issue, the IQ store by the CU's share of HBM.  A lower bound on a symbol's time on its CU is then
the sum of the three resource times:

    T_valu = SQ_INSTS_VALU / symbols x 2 cycles (a wave64 VALU instruction issues over 2 cycles,
             MI355X_MICROARCH.md) / 4 SIMDs
    T_lds  = SQ_LDS_IDX_ACTIVE / symbols (LDS-array cycles, bank conflicts included)
    T_hbm  = the symbol's minimal bytes / (8 TB/s / CUs), in cycles at the launch's measured clock
             (GRBM_GUI_ACTIVE per XCD / the rocprof launch time)

and the measured time per symbol is the launch's cycles / (symbols per CU)."""
import json
import sys

CUS, XCDS, HBM = 256, 8, 8.0e12


def counters(path, kernel="ofdm32_kernel"):
    out = {}
    for line in open(path):
        f = line.split()
        if len(f) == 3 and f[0] == kernel:
            out[f[1]] = float(f[2])
    return out


def main():
    pmc, bench = counters(sys.argv[1]), json.load(open(sys.argv[2]))
    st = bench["stages"]["ofdm"]
    # cfg3: 2091008 IQ samples per frame = P1 (2048) + 60 symbols x (32768 + 2048 GI); 60 = 59 data + 1 P2
    nsym = 60 * bench["config"]["frames_per_step_per_gpu"]
    launch_s = st["avg_launch_ms"] * 1e-3
    cycles = pmc["GRBM_GUI_ACTIVE"] / XCDS           # GPU cycles of the (profiled) launch
    clock = cycles / launch_s
    per_cu = nsym / CUS
    t_meas = cycles / per_cu
    t_valu = pmc["SQ_INSTS_VALU"] / nsym * 2 / 4
    t_lds = pmc["SQ_LDS_IDX_ACTIVE"] / nsym
    t_hbm = bench["roofline"]["min_bytes_per_launch"] / nsym / (HBM / CUS) * clock
    bound = t_valu + t_lds + t_hbm
    print(json.dumps({"symbols": nsym, "clock_GHz": round(clock / 1e9, 3), "cycles_per_symbol": round(t_meas),
                      "valu": round(t_valu), "lds": round(t_lds), "hbm_share": round(t_hbm),
                      "phase_serial_bound": round(bound), "measured_over_bound": round(t_meas / bound, 3),
                      "frac_at_bound": round(t_hbm / bound, 3)}))


if __name__ == "__main__":
    main()
