"""The LRU stand-in's eviction rule (the hand): the oracle's C
restatement (oracle.c o_ct_lru_evict) against a second, independent numpy
restatement written here from the rule's statement in include/gpuflow.h — age
keys, libgpuflow's CT hash and home lines, the line sample and its median, the
high-water trigger, the lines the hand passes per round, wrap-around of the hand,
the age-blind fallback of an empty sample — on random CT4 and CT6 tables over
several consecutive evictions.  The GPU's side of the same rule
is pinned against the oracle by tests/test_gpu_maps.py (eviction logs equal)."""
import numpy as np
import pytest

from oracle import oracle as O

M32 = np.uint64(0xFFFFFFFF)
BINS = 65536


def _rotl(x, r):
    x = x.astype(np.uint64)
    return ((x << np.uint64(r)) | (x >> np.uint64(32 - r))) & M32


def _mix(words, nbytes):
    """gf_hash_words (gf_common.h) over columns of u32 words, vectorized."""
    h = np.full(words.shape[0], 0x9747B28C ^ nbytes, np.uint64)
    for i in range(words.shape[1]):
        k = (words[:, i].astype(np.uint64) * np.uint64(0xCC9E2D51)) & M32
        k = (_rotl(k, 15) * np.uint64(0x1B873593)) & M32
        h ^= k
        h = (_rotl(h, 13) * np.uint64(5) + np.uint64(0xE6546B64)) & M32
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & M32
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & M32
    h ^= h >> np.uint64(16)
    return h


def ct_hash(keys):
    """gf_key_hash, mode CT: the canonical tuple (unordered addresses and ports,
    flags without TUPLE_F_IN)."""
    n, ksz = keys.shape
    pad = np.zeros((n, 40), np.uint8)
    pad[:, :ksz] = keys
    w = pad.view("<u4").astype(np.uint64)
    if ksz == 14:
        a, b, p0, p1 = w[:, 0], w[:, 1], w[:, 2] & np.uint64(0xFFFF), w[:, 2] >> np.uint64(16)
        c = np.stack([np.minimum(a, b), np.maximum(a, b), np.minimum(p0, p1) | (np.maximum(p0, p1) << np.uint64(16)),
                      (w[:, 3] & np.uint64(0xFF)) | (((w[:, 3] >> np.uint64(8)) & np.uint64(0xFE)) << np.uint64(8))], 1)
        return _mix(c, 14)
    less = np.zeros(n, bool)
    undecided = np.ones(n, bool)
    for i in range(4):
        d = undecided & (w[:, i] != w[:, 4 + i])
        less[d] = w[d, i] < w[d, 4 + i]
        undecided &= ~d
    lo = np.where(less[:, None], w[:, 0:4], w[:, 4:8])
    hi = np.where(less[:, None], w[:, 4:8], w[:, 0:4])
    p0, p1 = w[:, 8] & np.uint64(0xFFFF), w[:, 8] >> np.uint64(16)
    c = np.concatenate([lo, hi, (np.minimum(p0, p1) | (np.maximum(p0, p1) << np.uint64(16)))[:, None],
                        ((w[:, 9] & np.uint64(0xFF)) | (((w[:, 9] >> np.uint64(8)) & np.uint64(0xFE)) << np.uint64(8)))[:, None]], 1)
    return _mix(c, 40)


def age_keys(vals, now):
    lt = vals[:, 32:36].copy().view("<u4").ravel().astype(np.int64)
    fl = vals[:, 36:38].copy().view("<u2").ravel().astype(np.int64)
    to = np.where((fl & 1) & ((fl >> 1) & 1), 10, np.where(fl & 16, 43200, 300))
    lu = lt - to
    b = np.clip(lu - (now - (BINS - 1)), 0, BINS - 1)
    k = np.where(fl & 3, 0, BINS) + b
    return np.where(lu < 0, 0, k)


class Hand:
    """The rule, restated with numpy over a dict-free table (arrays of keys and values)."""

    def __init__(self, ksz, max_entries):
        self.ksz, self.max = ksz, max_entries
        self.ns = 64
        while self.ns < (8 if ksz == 14 else 4) * max_entries:    # gf_ct_slot_factor
            self.ns *= 2
        self.spl = 4 if ksz == 14 else 2
        self.nl = self.ns // self.spl
        self.sl = self.nl if self.nl <= 65536 else max(65536, self.nl >> 10)
        self.hw = max_entries - max_entries // 8          # the high-water mark
        self.hand = 0

    def home_lines(self, keys):
        return (ct_hash(keys) & np.uint64(self.ns - 1)).astype(np.int64) // self.spl

    def evict(self, keys, vals, now):
        """(kept mask, log record or None)."""
        n = len(keys)
        keep = np.ones(n, bool)
        if n <= self.hw:
            return keep, None
        hl = self.home_lines(keys)
        ak = age_keys(vals, now)
        sl = self.sl
        h0 = 0 if sl >= self.nl else self.hand          # the window ahead of the hand
        samp = np.sort(ak[((hl - h0) % self.nl) < sl])
        if not len(samp):                               # an empty window: the whole table
            sl = self.nl
            samp = np.sort(ak)
        K = int(samp[(len(samp) + 1) // 2 - 1])
        es = int((samp <= K).sum())
        h0, lines, ev, count = self.hand, 0, 0, n
        for rnd in range(3):
            if (count <= self.hw if rnd == 0 else count <= self.max) or lines >= self.nl:
                continue
            if rnd < 2:
                q = count - self.hw
                ln = -(-q * sl // es)
                ln = min(ln, self.nl - lines)
            else:
                ln = self.nl - lines
            kill = keep & (ak <= K) & (((hl - self.hand) % self.nl) < ln)
            keep &= ~kill
            count -= int(kill.sum())
            ev += int(kill.sum())
            self.hand = (self.hand + ln) % self.nl
            lines += ln
        return keep, (K, h0, lines, ev)


def _table(rng, ksz, n, now):
    keys = rng.integers(0, 256, (n, ksz), dtype=np.uint8)
    keys[:, 12 if ksz == 14 else 36] = rng.choice([6, 17, 1], n)     # nexthdr
    keys = np.unique(keys, axis=0)
    vals = np.zeros((len(keys), 48), np.uint8)
    fl = rng.choice([0, 16, 16 | 1, 16 | 3, 3], len(keys), p=[0.2, 0.6, 0.1, 0.05, 0.05]).astype(np.uint16)
    to = np.where((fl & 1) & ((fl >> 1) & 1), 10, np.where(fl & 16, 43200, 300))
    last = now - rng.integers(0, 400, len(keys))
    last[rng.random(len(keys)) < 0.02] = -5                       # last use before time 0
    vals[:, 32:36] = (np.maximum(last + to, 0)).astype("<u4").view(np.uint8).reshape(-1, 4)
    vals[:, 36:38] = fl.astype("<u2").view(np.uint8).reshape(-1, 2)
    return keys, vals


@pytest.mark.parametrize("ksz,max_entries,n0", [(14, 5000, 5400), (40, 3000, 3300), (14, 40000, 45000)])
def test_hand_matches_independent_restatement(ksz, max_entries, n0):
    rng = np.random.default_rng(ksz + max_entries)
    now = 100_000
    m = O.OMap(9, ksz, 48, max_entries)                # BPF_MAP_TYPE_LRU_HASH
    ref = Hand(ksz, max_entries)
    keys, vals = _table(rng, ksz, n0, now)
    m.update_many(keys, vals)
    events = 0
    for step in range(8):
        keep, rec = ref.evict(keys, vals, now)
        got = m.lru_evict(now)
        assert got == rec, (step, got, rec)
        keys, vals = keys[keep], vals[keep]
        kd, vd = m.dump_arrays()
        assert m.count() == len(keys) and len(kd) == len(keys)
        o = np.lexsort(kd.T[::-1])
        e = np.lexsort(keys.T[::-1])
        assert np.array_equal(kd[o], keys[e]) and np.array_equal(vd[o], vals[e])
        if rec:
            events += 1
            K, h0, lines, ev = rec
            assert m.count() <= max_entries and ev > 0
        else:
            assert m.count() <= ref.hw
        # more traffic: new entries at `now`, a later batch boundary
        now += 7
        nk, nv = _table(rng, ksz, max_entries // 6, now)
        fresh = ~(nk[:, None, :] == keys[None, :, :]).all(-1).any(1) if len(keys) < 6000 else np.ones(len(nk), bool)
        nk, nv = nk[fresh], nv[fresh]
        m.update_many(nk, nv)
        keys, vals = np.concatenate([keys, nk]), np.concatenate([vals, nv])
    assert events >= 4


def test_hand_evicts_the_older_half_only():
    """Every entry a round deletes lies in the sample's older half (age key <= the
    median key) and is homed in the lines the hand passed; younger entries of those
    lines survive."""
    rng = np.random.default_rng(3)
    now, mx = 50_000, 20000
    keys, vals = _table(rng, 14, 24000, now)
    m = O.OMap(9, 14, 48, mx)
    m.update_many(keys, vals)
    K, h0, lines, ev = m.lru_evict(now)
    kd, _ = m.dump_arrays()
    h = Hand(14, mx)
    hl = (ct_hash(keys) & np.uint64(h.ns - 1)).astype(np.int64) // h.spl
    ak = age_keys(vals, now)
    inr = ((hl - h0) % h.nl) < lines
    want_gone = inr & (ak <= K)
    assert ev == int(want_gone.sum()) and m.count() == len(keys) - ev
    samp = np.sort(ak[hl < h.sl])
    assert (samp <= K).sum() * 2 >= len(samp) and (samp < K).sum() * 2 < len(samp)
    assert (inr & (ak > K)).sum() > 0          # the younger entries of the passed lines stay


def test_hand_sampled_table_and_steady_state():
    """A table large enough to be sampled (NL > 65536 lines: SL = max(65536, NL >> 10)):
    once the count has crossed the high-water mark, each batch boundary deletes about
    what the batch inserted — the lines passed follow the inserts, not the table —
    and the count stays at or below max_entries after every call."""
    rng = np.random.default_rng(11)
    now, mx = 60_000, 40_000
    h = Hand(14, mx)
    assert h.nl > 65536 and h.sl == max(65536, h.nl >> 10) and h.sl < h.nl
    m = O.OMap(9, 14, 48, mx)
    keys, vals = _table(rng, 14, h.hw - 500, now)
    m.update_many(keys, vals)
    assert m.lru_evict(now) is None                     # below the high-water mark: nothing
    per_call = []
    for step in range(6):
        now += 5
        nk, nv = _table(rng, 14, 3000, now)
        fresh = ~np.isin(nk.view("V14").ravel(), keys.view("V14").ravel())
        nk, nv = nk[fresh], nv[fresh]
        m.update_many(nk, nv)
        keys, vals = np.concatenate([keys, nk]), np.concatenate([vals, nv])
        keep, rec = h.evict(keys, vals, now)
        got = m.lru_evict(now)
        assert got == rec, (step, got, rec)
        keys, vals = keys[keep], vals[keep]
        assert m.count() == len(keys) <= mx
        if rec:
            per_call.append((len(nk), rec[2], rec[3]))
    # steady state: every call evicts, each about what it inserted (the sample's
    # density estimate), passing far fewer lines than the table holds
    assert len(per_call) >= 5
    for ins, lines, ev in per_call[1:]:
        assert 0.8 * ins <= ev <= 1.25 * ins + 200 and lines < h.nl // 4, (ins, lines, ev)


def test_hand_empty_sample_is_not_a_flush():
    """Keys chosen so that none is homed in the sampled window (the CT hash is fixed
    and public): the sample falls back to the whole table, K is its median age, and
    at most its older half can go — never a flush (advisor r5: the old rule passed
    every line with every age eligible)."""
    rng = np.random.default_rng(5)
    now, mx = 70_000, 40_000
    h = Hand(14, mx)
    keys, vals = _table(rng, 14, 3 * mx, now)
    out = h.home_lines(keys) >= h.sl                  # the hand stands at line 0: the window is [0, SL)
    keys, vals = keys[out][: mx + 2000], vals[out][: mx + 2000]
    assert len(keys) == mx + 2000
    m = O.OMap(9, 14, 48, mx)
    m.update_many(keys, vals)
    keep, rec = h.evict(keys, vals, now)
    got = m.lru_evict(now)
    assert got == rec
    K, h0, lines, ev = got
    ak = age_keys(vals, now)
    srt = np.sort(ak)
    assert K == int(srt[(len(srt) + 1) // 2 - 1]) < 2 * BINS - 1      # the whole table's median age
    assert ev <= (ak <= K).sum() and m.count() == len(keys) - ev <= mx
    assert m.count() >= len(keys) - (ak <= K).sum() >= len(keys) // 3
