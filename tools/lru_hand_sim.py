"""Host simulation of the LRU hand on a scaled CT4 table (2^20 slots,
4-slot home lines, flows of 4 steps, 1/32 of max_entries new flows per step): the
fraction of slots holding dead (tombstone / FREE) entries and the probe lengths of
hits and misses over 220 steps, for the hand with tombstones that inserts never
claim ("hand"), the hand with slots inserts claim ("reuse": the FREE state), and the
old exact rule with compaction ("exact").   python tools/lru_hand_sim.py MODE"""
import numpy as np, sys
rng = np.random.default_rng(1)
NS = 1 << 20; SPL = 4; NL = NS // SPL; MASK = NS - 1
MAX = NS // 4; TARGET = MAX - MAX // 8
F = MAX // 32          # new flows per step
LIFE = 4               # steps a flow is used
EMPTY, FULL, TOMB = 0, 1, 2
st = np.zeros(NS, np.int8); home = np.zeros(NS, np.int64); last = np.zeros(NS, np.int64); fid = np.full(NS, -1, np.int64)
where = {}             # flow id -> slot
H = 0
mode = sys.argv[1] if len(sys.argv) > 1 else "hand"
REUSE = mode == "reuse"
def insert(f, h, now):
    p = h
    while st[p] != EMPTY and not (REUSE and st[p] == TOMB):
        p = (p + 1) & MASK
    st[p] = FULL; home[p] = h; last[p] = now; fid[p] = f; where[f] = p
def probe_len(h, f=None):
    p = h; n = 0
    while True:
        n += 1
        if st[p] == EMPTY: return n
        if st[p] == FULL and fid[p] == f: return n
        p = (p + 1) & MASK
count = 0; nid = 0; active = []
stats = []
for step in range(220):
    now = step
    new = list(range(nid, nid + F)); nid += F
    for f in new:
        h = (int(rng.integers(0, NL)) * SPL)
        insert(f, h, now); count += 1
    active.append(new)
    if len(active) > LIFE: active.pop(0)
    # hits: every active flow (except the new) refreshes last use
    for grp in active[:-1]:
        for f in grp:
            p = where.get(f)
            if p is not None and st[p] == FULL and fid[p] == f: last[p] = now
    if count > MAX:
        full = np.nonzero(st == FULL)[0]
        Q = count - TARGET
        if mode == "exact":
            # oldest-first, with backward-shift compaction (ideal, no tombstones)
            order = full[np.argsort(last[full], kind="stable")]
            kill = order[:Q]
            for p in kill: del where[fid[p]]
            st[kill] = TOMB; fid[kill] = -1
            # compaction: rebuild positions of all FULL entries (equivalent to clean table)
            fl = np.nonzero(st == FULL)[0]
            hs, ls, fs = home[fl].copy(), last[fl].copy(), fid[fl].copy()
            st[:] = EMPTY; fid[:] = -1; where.clear()
            o = np.argsort(hs, kind="stable")
            for i in o: insert(int(fs[i]), int(hs[i]), int(ls[i]))
            count -= len(kill)
        else:
            SL = NL // 64
            samp = full[(home[full] // SPL) < SL]
            ages = last[samp]
            K = np.sort(ages)[(len(ages) + 1) // 2 - 1]
            eS = int((ages <= K).sum())
            L = min(NL, -(-Q * SL // eS))
            hl = home // SPL
            inr = ((hl - H) % NL) < L
            kill = np.nonzero((st == FULL) & (last <= K) & inr)[0]
            for p in kill: del where[fid[p]]
            st[kill] = TOMB; fid[kill] = -1
            count -= len(kill)
            # trailing cleanup within the range (+ successors): a removable slot becomes EMPTY when every slot after it up to the cluster end is removable
            lo = (H * SPL); hi = lo + L * SPL
            idx = np.arange(lo, hi + 64) & MASK
            # process from the end backward
            for p in idx[::-1]:
                if st[p] == TOMB and (((home[p]//SPL - H) % NL) < L or True):
                    q = (p + 1) & MASK
                    if st[q] == EMPTY and ((p - lo) & MASK) < L * SPL: st[p] = EMPTY
            H = (H + L) % NL
    if step % 10 == 9 or step == 219:
        nt = int((st == TOMB).sum()); nf = int((st == FULL).sum())
        sm = rng.integers(0, NL, 4000) * SPL
        miss = np.mean([probe_len(int(h)) for h in sm])
        hitf = [f for g in active for f in g[:500]]
        hit = np.mean([probe_len(int(home[where[f]]), f) for f in hitf if f in where])
        stats.append((step, nf, nt, miss, hit))
        print(f"{mode} step {step}: full {nf/NS:.3f} tomb {nt/NS:.3f} miss-probe {miss:.2f} hit-probe {hit:.2f}", flush=True)
