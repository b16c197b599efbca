"""Full-scale parity helpers — TEST INFRASTRUCTURE ONLY (bench.py's CPU leg and
tests/; the product never imports this).

The bench runs the CPU restatement on a *flow-group sample* of each workload:
the packets whose unordered address pair satisfies `pair_sampled` (a hash of
the pair, so a sample holds whole flow groups — every packet, CT entry and
ICMP-related entry of a pair is in or out together, which is what makes a
sampled run of the stateful path exact: conntrack state never crosses flow
groups).  The GPU classifies the full batch; its records for the
sampled packets and its CT entries of the sampled pairs must equal the
oracle's bit for bit.
"""
import numpy as np

SALT = np.uint64(0x5A3C_9E37_79B9_7F4A)
_M1, _M2 = np.uint64(0xff51afd7ed558ccd), np.uint64(0xc4ceb9fe1a85ec53)


def _fmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    x = x ^ (x >> np.uint64(33))
    x = x * _M1
    x = x ^ (x >> np.uint64(33))
    x = x * _M2
    return x ^ (x >> np.uint64(33))


def pair_sampled(a, b, div):
    """IPv4: a, b = the two addresses as raw u32 words (network-order bytes loaded
    little-endian, the column / CT-key form).  True where the unordered pair is in
    the sample (1 in `div` pairs)."""
    a = np.asarray(a).astype(np.uint32).astype(np.uint64)
    b = np.asarray(b).astype(np.uint32).astype(np.uint64)
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    return (_fmix64(((hi << np.uint64(32)) | lo) ^ SALT) >> np.uint64(40)) % np.uint64(div) == 0


def pair_sampled6(a16, b16, div):
    """IPv6: a16, b16 = uint8[n, 16] addresses."""
    a16 = np.ascontiguousarray(a16, np.uint8)
    b16 = np.ascontiguousarray(b16, np.uint8)
    ah, al = a16[:, :8].copy().view(">u8").ravel().astype(np.uint64), a16[:, 8:].copy().view(">u8").ravel().astype(np.uint64)
    bh, bl = b16[:, :8].copy().view(">u8").ravel().astype(np.uint64), b16[:, 8:].copy().view(">u8").ravel().astype(np.uint64)
    a_lt = (ah < bh) | ((ah == bh) & (al < bl))
    lh, ll = np.where(a_lt, ah, bh), np.where(a_lt, al, bl)
    hh, hl = np.where(a_lt, bh, ah), np.where(a_lt, bl, al)
    x = _fmix64(lh ^ SALT)
    x = _fmix64(x ^ ll)
    x = _fmix64(x ^ hh)
    x = _fmix64(x ^ hl)
    return (x >> np.uint64(40)) % np.uint64(div) == 0


def ct_sampled(keys, div):
    """Rows of a CT dump (ipv4_ct_tuple 14 B / ipv6_ct_tuple 40 B keys) whose
    address pair is in the sample."""
    keys = np.ascontiguousarray(keys, np.uint8)
    if keys.shape[1] == 14:
        w = keys[:, :8].copy().view("<u4")
        return pair_sampled(w[:, 0], w[:, 1], div)
    return pair_sampled6(keys[:, 0:16], keys[:, 16:32], div)


def compare_records(gpu, ref):
    """Number of differing records and the first differing position (or -1)."""
    g = np.ascontiguousarray(gpu).view(np.uint8).reshape(len(gpu), -1)
    r = np.ascontiguousarray(ref).view(np.uint8).reshape(len(ref), -1)
    if g.shape != r.shape:
        return max(len(g), len(r)), 0
    bad = np.nonzero((g != r).any(axis=1))[0]
    return int(len(bad)), int(bad[0]) if len(bad) else -1


# Frame fingerprints: one 64-bit value per rewritten frame row (snap_out), so that
# whole-stream runs compare the LB / rev-NAT / netdev rewrites without keeping
# every frame.  h = sum over the row's little-endian u64 words w_j of
# w_j * FP_MUL^(m-1-j) (mod 2^64), Horner form; FP_MUL is odd, so a change of any
# single word always changes h.  The numpy form runs on the oracle's frames, the
# torch form on the device's snap buffer (wrapping int64 arithmetic, same bits).
FP_MUL = 0x9E3779B97F4A7C15


def frame_fingerprints(rows):
    """uint64[n] fingerprints of uint8[n, stride] rows (stride a multiple of 8)."""
    rows = np.ascontiguousarray(rows, np.uint8)
    w = rows.view("<u8")
    h = np.zeros(len(rows), np.uint64)
    m = np.uint64(FP_MUL)
    with np.errstate(over="ignore"):
        for j in range(w.shape[1]):
            h = h * m + w[:, j]
    return h


def frame_fingerprints_torch(rows):
    """The same fingerprints of a uint8 [n, stride] torch tensor, on its device;
    returned as int64 (view the numpy copy as uint64)."""
    import torch
    w = rows.contiguous().view(torch.int64)
    m = FP_MUL - (1 << 64) if FP_MUL >= 1 << 63 else FP_MUL
    h = torch.zeros(rows.shape[0], dtype=torch.int64, device=rows.device)
    for j in range(w.shape[1]):
        h = h * m + w[:, j]
    return h


def _sort_rows(k, v):
    """Rows sorted by key bytes (lexicographic)."""
    if len(k) == 0:
        return k, v
    w = (k.shape[1] + 7) // 8
    pad = np.zeros((len(k), 8 * w), np.uint8)
    pad[:, :k.shape[1]] = k
    words = pad.view(">u8")                       # big-endian words: numeric order == byte order
    o = np.lexsort([words[:, j] for j in range(w - 1, -1, -1)])
    return k[o], v[o]


def compare_tables(gk, gv, rk, rv, exact_below=2_000_000):
    """Entries of two dumps (keys/values arrays): (entries compared, entries that
    differ or exist on one side only).  Dumps of up to `exact_below` rows are
    sorted row by row and compared byte for byte; larger ones (the bench's 10^8-
    entry CTs) compare as sorted 64-bit fingerprints of their (key, value) rows
    (oracle.rows_fp): an entry counts as equal when its fingerprint occurs on the
    other side, so a differing entry is missed only if its fingerprint collides
    with another entry's (~n / 2^64)."""
    if max(len(gk), len(rk)) > exact_below:
        from oracle.oracle import rows_fp
        g = np.sort(rows_fp(gk, gv))
        r = np.sort(rows_fp(rk, rv))
        if len(r) == 0 or len(g) == 0:
            return max(len(g), len(r)), max(len(g), len(r))
        if len(g) == len(r) and np.array_equal(g, r):
            return len(g), 0
        hit = r[np.minimum(np.searchsorted(r, g), len(r) - 1)] == g
        only_g = int((~hit).sum())
        hit_r = g[np.minimum(np.searchsorted(g, r), len(g) - 1)] == r
        only_r = int((~hit_r).sum())
        return max(len(g), len(r)), max(only_g, only_r)
    gk, gv = _sort_rows(np.ascontiguousarray(gk), np.ascontiguousarray(gv))
    rk, rv = _sort_rows(np.ascontiguousarray(rk), np.ascontiguousarray(rv))
    if len(gk) != len(rk):
        gs = {bytes(x) for x in gk} if len(gk) < 2_000_000 else None
        rs = {bytes(x) for x in rk} if len(rk) < 2_000_000 else None
        only = len(gs ^ rs) if gs is not None and rs is not None else abs(len(gk) - len(rk))
        return max(len(gk), len(rk)), max(only, abs(len(gk) - len(rk)))
    kd = (gk != rk).any(axis=1)
    vd = (gv != rv).any(axis=1)
    return int(len(gk)), int((kd | vd).sum())


def gpu_table_sampled(fd, ksz, vsz, div, chunk=1 << 20, pred=ct_sampled):
    """The GPU map's entries of the sampled pairs, streamed through the chunked
    dump (gf_map_lookup_batch) and filtered chunk by chunk."""
    from cilium_amd import bpf
    ks, vs = [], []
    cursor, done, total = None, False, 0
    while not done:
        k, v, cursor, done = bpf.LookupBatch(fd, cursor, chunk, ksz, vsz)
        total += len(k)
        if len(k):
            m = pred(k, div)
            ks.append(k[m]); vs.append(v[m])
    if not ks:
        return np.zeros((0, ksz), np.uint8), np.zeros((0, vsz), np.uint8), total
    return np.concatenate(ks), np.concatenate(vs), total


def oracle_table_sampled(omap, div, pred=ct_sampled):
    k, v = omap.dump_arrays()
    m = pred(k, div) if len(k) else np.zeros(0, bool)
    return k[m], v[m]


def owners_host(lb_out, nd6, pk, rank, world):
    """The owner rule of gf_pipeline_partition restated on the host (checker):
    the rank of the post-LB unordered address pair; frames that cannot reach
    conntrack stay on `rank`."""
    from cilium_amd import shard, stream
    f = pk.frames
    et = (f[:, 12].astype(np.uint32) << 8) | f[:, 13]
    v4 = (et == 0x0800) & (pk.lens >= 34)
    v6 = (et == 0x86DD) & (pk.lens >= 54)
    sa = f[:, 26:30].copy().view(">u4").ravel().astype(np.uint32)
    da = f[:, 30:34].copy().view(">u4").ravel().astype(np.uint32)
    nd = lb_out["new_daddr4"].astype(">u4").view("<u4").astype(np.uint32)      # raw be32 -> host order
    da = np.where(lb_out["slave"] > 0, nd, da)
    r = np.full(pk.n, rank, np.int64)
    r[v4] = stream.pair_rank(sa[v4], da[v4], world)
    d6 = np.where((lb_out["slave"] > 0)[:, None], nd6, f[:, 38:54])
    if v6.any():
        r[v6] = shard.pair_rank6(f[v6, 22:38], d6[v6], world)
    return r
