"""Expected LDS bank-conflict cycles of the engine's walk gathers: every lane of a wave reads the
permits of its own walk step, `home + s * step mod n` -- addresses that are random to the banks.  Under the gfx950 bank
rules (MI355X_MICROARCH.md, LDS section: `ds_read_b32` is served in two groups of 32 lanes over 32 banks, `ds_read_b128`
in four groups of 16 lanes over 64 banks, four banks per lane; each extra distinct address on a busy bank costs one
cycle), a Monte Carlo over random distinct word addresses gives the extra cycles such a gather pays, as
SQ_LDS_BANK_CONFLICT counts them.  Printed per instruction and lane count.
  python tools/sim/lds_conflict_mc.py"""
import numpy as np

rng = np.random.default_rng(1)
T = 20000


def extra(lanes_per_group, groups, banks, words, active):
    tot = 0
    for _ in range(T):
        for g in range(groups):
            k = min(active - g * lanes_per_group, lanes_per_group)
            if k <= 1:
                continue
            a = rng.choice(10000, size=k, replace=False) * words
            cnt = np.zeros(banks, int)
            for x in a:
                for w in range(words):
                    cnt[(x + w) % banks] += 1
            tot += cnt.max() - 1
    return tot / T


for active in (64, 32, 16):
    print(f"active lanes {active:2d}: ds_read_b32 random gather {extra(32, 2, 32, 1, active):.2f} extra cycles per "
          f"instruction (2 base); ds_read_b128 {extra(16, 4, 64, 4, active):.2f} (4 base)")
