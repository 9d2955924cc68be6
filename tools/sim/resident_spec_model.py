"""Model check of the resident engine's speculation (owgs_resident.hip) against plain sequential
decisions: per chunk, speculative walks against the chunk's start (rank-packed repeats of an action, concurrent keys
with free slots and maxConcurrent per container, shared keys decided alone), in-order validation of the longest prefix
whose targets still have room, the first one that does not decided alone (and the later decisions of its key with it).
Random small pools with heavy conflicts, every walk budget; releases between runs.  Run: python3 resident_spec_model.py
(pure Python, no GPU; ~1 minute)."""
# Model check of the resident engine's speculation + in-order validation against plain sequential decisions.
import random

def seq_decide(st, d):
    P, M, usable, n, base = st['P'], st['M'], st['usable'], st['n'], st['base']
    home, step, mem, maxc, slot, seqn = d
    for k in range(n):
        x = base + (home + k * step) % n
        if not usable[x]: continue
        if maxc <= 1:
            if P[x] >= mem: P[x] -= mem; return (x, 0)
        else:
            c, o = M.get((x, slot), (0, 0))
            if c >= 1: M[(x, slot)] = (c - 1, o + 1); return (x, 0)
            if P[x] >= mem: P[x] -= mem; M[(x, slot)] = (maxc - 1, o + 1); return (x, 0)
    H = [x for x in range(base, base + n) if usable[x]]
    if not H: return (-1, 0)
    x = H[seqn % len(H)]
    if maxc <= 1: P[x] -= mem
    else:
        c, o = M.get((x, slot), (0, 0))
        if c >= 1: M[(x, slot)] = (c - 1, o + 1)
        else: P[x] -= mem; M[(x, slot)] = (maxc - 1, o + 1)
    return (x, 1)

def spec_chunk(st, ds, budget, cursors, act_of):
    P, M, usable, n, base = st['P'], st['M'], st['usable'], st['n'], st['base']
    N = len(ds)
    sp = ['STOP'] * N; t = [-1] * N; ts = [0] * N; cv = [None] * N; out = [None] * N
    # ranks of plain decisions of the same action; first occurrence of concurrent keys
    seen_a, seen_s = {}, set()
    rank = [0] * N
    for i, d in enumerate(ds):
        home, step, mem, maxc, slot, seqn = d
        a = act_of[i]
        if maxc <= 1:
            rank[i] = seen_a.get(a, 0); seen_a[a] = rank[i] + 1
            s0 = cursors.get(a, 0)
            if s0 >= n: sp[i] = 'FAIL'; continue
            need = rank[i]; s = s0
            while True:
                x = base + (home + s * step) % n
                v = P[x]
                if usable[x] and v >= mem:
                    if v >= (need + 1) * mem: sp[i] = 'FOUND'; t[i] = x; ts[i] = s; break
                    need -= v // mem
                s += 1
                if s >= n: sp[i] = 'FAIL'; break
                if s - s0 >= budget: sp[i] = 'STOP'; ts[i] = s; break
        else:
            rank[i] = seen_a.get(a, 0); seen_a[a] = rank[i] + 1
            other = any(ds[j][3] > 1 and ds[j][4] == slot and act_of[j] != a for j in range(i))
            if other: continue
            need = rank[i]
            for s in range(min(n, budget)):
                x = base + (home + s * step) % n
                if not usable[x]: continue
                c, o = M.get((x, slot), (0, 0))
                if need < c:
                    sp[i] = 'FOUND'; t[i] = x; cv[i] = (c - need, o + need, False); break
                kp = need - c
                cn = kp // maxc + 1
                if P[x] >= cn * mem:
                    j = kp % maxc
                    cb = 0 if j == 0 else maxc - j
                    sp[i] = 'FOUND'; t[i] = x; cv[i] = (cb, o + need, j == 0); break
                need -= c + (maxc * (P[x] // mem) if P[x] >= mem else 0)
            else:
                if n <= budget and rank[i] == 0: sp[i] = 'FAIL'
    H = [x for x in range(base, base + n) if usable[x]]
    for i, d in enumerate(ds):
        home, step, mem, maxc, slot, seqn = d
        if sp[i] == 'FAIL':
            if not H: sp[i] = 'TRIV'; out[i] = (-1, 0)
            else:
                sp[i] = 'FORCED'; t[i] = H[seqn % len(H)]
                if maxc > 1:
                    c, o = M.get((t[i], slot), (0, 0)); cv[i] = (c, o, c == 0)
        if maxc <= 1 and rank[i] == 0:
            a = act_of[i]
            if sp[i] == 'FOUND' or sp[i] == 'STOP': cursors[a] = max(cursors.get(a, 0), ts[i])
            elif sp[i] in ('FORCED', 'TRIV'): cursors[a] = n
    q = 0
    while q < N:
        f = N
        S = {}
        for i in range(q, N):
            home, step, mem, maxc, slot, seqn = ds[i]
            if sp[i] in ('TRIV',): continue
            if sp[i] == 'STOP': f = i; break
            cslot = maxc > 1 and not cv[i][2]
            if sp[i] == 'FOUND' and not cslot:
                if P[t[i]] - S.get(t[i], 0) < mem: f = i; break
            if not cslot: S[t[i]] = S.get(t[i], 0) + mem
        for i in range(q, f):
            home, step, mem, maxc, slot, seqn = ds[i]
            if sp[i] == 'TRIV': continue
            cslot = maxc > 1 and not cv[i][2]
            if not cslot: P[t[i]] -= mem
            if maxc > 1:
                c, o, _ = cv[i]
                assert M.get((t[i], slot), (0, 0)) == (c, o), (M.get((t[i], slot)), c, o)
                M[(t[i], slot)] = ((c - 1) if cslot else maxc - 1, o + 1)
            out[i] = (t[i], 1 if sp[i] == 'FORCED' else 0)
        if f >= N: break
        # decide alone (from ts for plain lanes, steps before it full)
        home, step, mem, maxc, slot, seqn = ds[f]
        a = act_of[f]
        smin = max(cursors.get(a, 0), ts[f]) if maxc <= 1 else 0
        r = None
        if maxc <= 1:
            for s in range(smin, n):
                x = base + (home + s * step) % n
                if usable[x] and P[x] >= mem: P[x] -= mem; r = (x, 0); cursors[a] = max(cursors.get(a, 0), s); break
            if r is None:
                cursors[a] = n
                if not H: r = (-1, 0)
                else: x = H[seqn % len(H)]; P[x] -= mem; r = (x, 1)
        else:
            r = seq_decide(st, ds[f])
            for j in range(f + 1, N):  # later decisions of the key: their predictions assumed this one's
                if ds[j][3] > 1 and ds[j][4] == slot and sp[j] != 'TRIV': sp[j] = 'STOP'
        out[f] = r
        q = f + 1
    return out

def run(seed):
    rnd = random.Random(seed)
    n = rnd.randint(1, 40)
    usable = [rnd.random() < 0.85 for _ in range(n)]
    P0 = [rnd.randint(0, 8) * 128 for _ in range(n)]
    acts = []
    for a in range(rnd.randint(1, 12)):
        step = rnd.randint(1, max(1, n - 1))
        import math
        while math.gcd(step, n) != 1: step = rnd.randint(1, max(1, n - 1))
        acts.append((rnd.randrange(n), step, rnd.choice([128, 256, 384]), rnd.choice([1, 1, 1, 2, 3]), a % 4))
    budget = rnd.choice([1, 2, 4, 8, 16])
    stA = dict(P=list(P0), M={}, usable=usable, n=n, base=0)
    stB = dict(P=list(P0), M={}, usable=usable, n=n, base=0)
    cursors = {}
    seqn = 0
    live = []
    for run_ in range(30):
        # releases (both models identically), reset cursors (generation)
        rel = [live.pop(rnd.randrange(len(live))) for _ in range(min(len(live), rnd.randint(0, 10)))]
        for st in (stA, stB):
            for (x, a) in rel:
                h, s_, mem, maxc, slot = acts[a]
                if maxc <= 1: st['P'][x] += mem
                else:
                    c, o = st['M'][(x, slot)]
                    c += 1; o -= 1
                    if c % maxc == 0: c -= maxc; st['P'][x] += mem
                    if o == 0: del st['M'][(x, slot)]
                    else: st['M'][(x, slot)] = (c, o)
        if rel: cursors = {}
        k = rnd.randint(1, 64)
        ai = [rnd.choice(range(len(acts))) if rnd.random() < 0.5 else 0 for _ in range(k)]
        ds = [(acts[a][0], acts[a][1], acts[a][2], acts[a][3], acts[a][4], seqn + j) for j, a in enumerate(ai)]
        seqn += k
        ra = [seq_decide(stA, d) for d in ds]
        rb = spec_chunk(stB, ds, budget, cursors, ai)
        assert ra == rb, (seed, run_, ra, rb)
        assert stA['P'] == stB['P'] and stA['M'] == stB['M'], seed
        live += [(x, a) for (x, f), a in zip(ra, ai) if x >= 0]
for s in range(20000): run(s)
print("ok")
