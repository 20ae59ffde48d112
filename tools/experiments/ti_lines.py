"""Cache lines per map TI-store instruction from the planner's slot map, cfg3: the round-3
mapping (four consecutive TI cells per lane), the round-4 mapping (64 consecutive cells per instruction)
and slot order (what a per-cell source table would allow).  Experiment tooling, not product."""
import numpy as np, sys
sys.path.insert(0, 'tests'); sys.path.insert(0, 'gr-dvbt2ll_amd')
import plan_probe as PP
from dvbt2ll.configs import CONFIGS
cfg = CONFIGS['cfg3']
fp = PP.frame_plan(cfg.fm_args())
cl = PP.chain_layout(cfg)
cs = fp['cs']; part = cl['part']
rows = cs // 5
def lines(addrs, seg=128):
    return len(set((a * 2) // seg for a in addrs))
tot_cur = tot_old = tot_sorted = 0; n = 0
for r in [0, 1, 64, 100, 194]:
    jj = np.arange(cs)
    t = (jj % 5) * rows + jj // 5
    slot = part[PP.ti_dest(fp, r, t)]
    # current: per instruction 64 consecutive jj
    for c0 in range(0, cs, 64):
        tot_cur += lines(slot[c0:c0 + 64]); n += 1
    # old: lane l has jj = 4 (base + l) + k -> instruction k covers jj = 4 l + k over 256
    for b in range(0, cs, 256):
        for k in range(4):
            idx = np.arange(b + k, min(b + 256, cs), 4)
            tot_old += lines(slot[idx])
    s = np.sort(slot)
    for c0 in range(0, cs, 64):
        tot_sorted += lines(s[c0:c0 + 64])
print('lines per store instruction: current %.2f old %.2f stored-order %.2f' % (tot_cur / n, tot_old / n, tot_sorted / n))

