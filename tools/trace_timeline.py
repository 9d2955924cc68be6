"""Diagnostic: analyse a barrier timeline written by a -DOWGS_TRACE engine (env OWGS_TRACE_FILE).

For every pass-loop barrier (1 chunk start, 8 after the hot-action and per-lane walks, 2 after the queued long walks,
3 after tentative consumption, 4 before commit, 5 end of pass) and every wave: cycles from the previous barrier's departure to this arrival (the wave's own work),
which wave arrived last (the critical path), and the barrier's own cost (last arrival -> departure)."""
import sys

import numpy as np

CAP = 16384
raw = np.fromfile(sys.argv[1], dtype=np.uint64)
nw = raw.size // (2 * CAP)
ev = raw.reshape(nw, CAP, 2)
ids = (ev[:, :, 0] >> np.uint64(56)).astype(np.int64)
ta = (ev[:, :, 0] & np.uint64((1 << 56) - 1)).astype(np.int64)
td = ev[:, :, 1].astype(np.int64)
n = int((ids[0] > 0).sum())
ids, ta, td = ids[:, :n], ta[:, :n], td[:, :n]
assert (ids == ids[0]).all(), "waves disagree on the barrier sequence"
# a phase is named after what runs before the barrier that ends it: barrier 8 ends the hot-action and per-lane walks
# (and the long-walk queue's push), barrier 2 the queued long walks (round 3's files used the two names swapped)
names = {1: "chunk_start", 2: "long walks", 3: "tentative", 4: "validate", 5: "commit", 8: "speculate",
         6: "(mark) chunk loop", 7: "(mark) lane decode", 9: "re-decisions"}
work = ta[:, 1:] - td[:, :-1]  # per wave: departure of barrier k-1 -> arrival at barrier k
crit = work.max(axis=0)
last = work.argmax(axis=0)
bar = td[:, 1:].max(axis=0) - ta[:, 1:].max(axis=0)
kind = ids[0, 1:]
print(f"{n} barrier events, {nw} waves (wave {nw - 1} = I/O)")
print(f"{'phase':17s} {'count':>6s} {'crit cyc':>9s} {'barrier':>8s}   mean work per wave (cycles)   last-arriving wave histogram")
# first pass of a chunk = the pass-loop barriers between a chunk-start barrier and the next end-of-pass barrier
first = np.zeros(kind.size, dtype=bool)
state = False
for x in range(kind.size):
    if kind[x] == 1:
        state = True
    first[x] = state and kind[x] != 1
    if kind[x] == 5:
        state = False
rows = [(names[k], kind == k) for k in sorted(names)]
rows += [(names[k] + "/first", (kind == k) & first) for k in (8, 2, 3, 4, 5)]
rows += [(names[k] + "/later", (kind == k) & ~first) for k in (8, 2, 3, 4, 5)]
for label, m in rows:
    if not m.any():
        continue
    per_wave = work[:, m].mean(axis=1)
    hist = np.bincount(last[m], minlength=nw)
    print(f"{label:17s} {m.sum():6d} {crit[m].mean():9.0f} {bar[m].mean():8.0f}   "
          + " ".join(f"{x:6.0f}" for x in per_wave) + "   " + " ".join(str(x) for x in hist))
