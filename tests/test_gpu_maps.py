"""The map API on device-authoritative maps (pkg/bpf/map.go:322-498 semantics on
the HBM replica, no whole-table pull), per-map locking under concurrent callers,
and the LRU stand-in of the CT maps — all against the oracle."""
import errno
import threading
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from cilium_amd import bpf, synth
from cilium_amd._lib import lib, gf_ct_evict_rec
from cilium_amd.datapath import Datapath, DeviceBatch, ING_OUT, to_numpy
from oracle.scenario import OracleDP


@pytest.fixture(scope="module", autouse=True)
def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def _cmp(a, b, what):
    if not np.array_equal(a, b):
        bad = np.nonzero(a != b)[0]
        raise AssertionError(f"{what}: {len(bad)} mismatches, first at {bad[0]}: gpu={a[bad[0]]} ref={b[bad[0]]}")


def test_device_map_element_ops():
    """After classify calls the CT and policy maps live in HBM.  Lookup / update /
    delete / get_next_key / the chunked dump reach their elements there (a few
    hundred bytes over PCIe per element operation, never the table), and traffic
    after host-side edits sees exactly what the oracle sees after the same edits."""
    sc = synth.fuzz(seed=21, n_packets=20000, n_batches=3)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi in range(2):
        pk = sc.batches[bi]
        io = dp.ingress(DeviceBatch(pk), sc.now + bi)
        torch.cuda.synchronize()
        _cmp(to_numpy(io, ING_OUT), ref.ingress(pk, sc.now + bi), f"ingress b{bi}")
    fd = dp.fd["ct4"]
    info0 = bpf.GetMapInfo(fd)
    want = ref.dump("ct4")
    assert info0.Entries == len(want)
    keys = sorted(want)
    rnd = np.random.default_rng(1)
    pick = [keys[i] for i in rnd.choice(len(keys), 64, replace=False)]
    for k in pick:
        assert bpf.LookupElement(fd, k, 48) == want[k]
    with pytest.raises(bpf.BPFError) as e:
        bpf.LookupElement(fd, b"\x01" * 14, 48)
    assert e.value.errno == errno.ENOENT
    info1 = bpf.GetMapInfo(fd)
    assert info1.XferD2H - info0.XferD2H < 64 * 4096, "element lookups must not pull the table"
    # edits on both sides: deletes, overwrites, NOEXIST / EXIST errors, new entries
    om = ref.m["ct4"]
    for k in pick[:16]:
        bpf.DeleteElement(fd, k)
        assert om.delete(k) == 0
    for k in pick[16:32]:
        v = bytearray(want[k]); v[32:36] = (sc.now + 7).to_bytes(4, "little")
        bpf.UpdateElement(fd, k, bytes(v), bpf.BPF_EXIST)
        assert om.update(k, bytes(v), 2) == 0
    for k in pick[32:40]:
        with pytest.raises(bpf.BPFError) as e:
            bpf.UpdateElement(fd, k, want[k], bpf.BPF_NOEXIST)
        assert e.value.errno == errno.EEXIST
    for j in range(8):
        k = bytes([10, 9, 8, j]) + bytes([100, 64, 1, j]) + bytes([0, 80, 0x9c, 0x40, 6, 0])
        v = synth.ct_vals(1, sc.now + 300, 0, 0, 300)[0].tobytes()
        bpf.UpdateElement(fd, k, v, bpf.BPF_NOEXIST)
        assert om.update(k, v, 1) == 0
    info2 = bpf.GetMapInfo(fd)
    assert info2.Entries == om.count()
    assert info2.XferD2H < info0.DeviceBytes / 4
    # the reference's dump loop on the device replica, and the chunked dump
    m = bpf.Map("ct4", 9, 14, 48, 100000)
    m.fd = fd
    kbk = {}
    m.DumpKeyByKey(lambda k, v: kbk.__setitem__(k, v))
    assert kbk == ref.dump("ct4") == dp.dump_map("ct4")
    # traffic after the edits
    pk = sc.batches[2]
    io = dp.ingress(DeviceBatch(pk), sc.now + 2)
    torch.cuda.synchronize()
    _cmp(to_numpy(io, ING_OUT), ref.ingress(pk, sc.now + 2), "ingress after edits")
    assert dp.dump_map("ct4") == ref.dump("ct4")
    for e in range(16):
        assert dp.dump_map(f"pol{e}") == ref.dump(f"pol{e}"), f"policy counters pol{e}"


def test_concurrent_map_ops_and_classify():
    """Map updates, lookups and dumps from several threads while another thread
    classifies: per-map locks serialise each map, classify calls hold the maps
    they bind; verdicts and final state equal the oracle's (the concurrent edits
    touch maps the traffic does not read, so their order does not matter)."""
    sc = synth.fuzz(seed=23, n_packets=20000, n_batches=4)
    sc.add_map(synth.MapSpec("side_hash", synth.HASH, 8, 24, 100000, 0))
    sc.add_map(synth.MapSpec("side_lpm", synth.LPM, 8, 1, 10000, synth.NO_PREALLOC))
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    errs, outs = [], []
    stop = threading.Event()

    def classify():
        try:
            for bi, pk in enumerate(sc.batches):
                io = dp.ingress(DeviceBatch(pk), sc.now + bi)
                torch.cuda.synchronize()
                outs.append(to_numpy(io, ING_OUT))
        except Exception as e:        # reported by the main thread
            errs.append(e)
        finally:
            stop.set()

    def writer(tid):
        try:
            rnd = np.random.default_rng(tid)
            fd = dp.fd["side_hash"] if tid % 2 else dp.fd["side_lpm"]
            i = 0
            while not stop.is_set() or i < 200:
                if tid % 2:
                    k = int(tid * 1_000_000 + i).to_bytes(8, "little")
                    bpf.UpdateElement(fd, k, bytes(24))
                    assert bpf.LookupElement(fd, k, 24) == bytes(24)
                else:
                    k = (24).to_bytes(4, "little") + bytes([10, tid, i % 256, 0])
                    bpf.UpdateElement(fd, k, b"\x01")
                i += 1
        except Exception as e:
            errs.append(e)

    def reader():
        try:
            while not stop.is_set():
                bpf.GetMapInfo(dp.fd["ct4"])
                bpf.GetMapInfo(dp.fd["pol0"])
        except Exception as e:
            errs.append(e)

    th = [threading.Thread(target=classify)] + [threading.Thread(target=writer, args=(t,)) for t in range(1, 5)] + \
        [threading.Thread(target=reader)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    assert len(outs) == len(sc.batches)
    for bi, pk in enumerate(sc.batches):
        _cmp(outs[bi], ref.ingress(pk, sc.now + bi), f"ingress b{bi}")
    assert dp.dump_map("ct4") == ref.dump("ct4")
    assert bpf.GetMapInfo(dp.fd["side_hash"]).Entries >= 400


def _evict_log(fd):
    recs = (gf_ct_evict_rec * 4096)()
    n = lib.gf_ct_evict_log(fd, recs, 4096)
    assert n >= 0
    return [(r.seq, r.now_sec, r.age_cut, r.hand_line, r.lines, r.evicted) for r in recs[:n]]


@pytest.mark.parametrize("seed,dt", [(4, 40), (6, 40), (5, 6000)])
def test_lru_eviction_matches_oracle(seed, dt):
    """LRU CT maps overflowing max_entries: after every batch the device evicts by
    the deterministic age rule (closing entries, then by lifetime) down to the
    7/8 watermark, exactly as the oracle's restatement of the rule; verdicts of
    the following batches, the CT contents and the eviction logs are identical,
    and the count is back under max_entries at every batch boundary.  dt = 6000 s
    between batches puts the older entries' age bins outside k_lru_hist's direct
    LDS window (the last 4096 s), through its hashed bin cache."""
    sc = synth.fuzz(seed=seed, n_packets=20000, n_batches=5, ct_max=2500, ct6_max=300)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        now = sc.now + dt * bi
        io = dp.ingress(DeviceBatch(pk), now)
        torch.cuda.synchronize()
        _cmp(to_numpy(io, ING_OUT), ref.ingress(pk, now), f"ingress b{bi}")
        for name, mx in (("ct4", 2500), ("ct6", 300)):
            assert bpf.GetMapInfo(dp.fd[name]).Entries == ref.m[name].count() <= mx, name
    for name in ("ct4", "ct6"):
        assert dp.dump_map(name) == ref.dump(name), name
        assert _evict_log(dp.fd[name]) == ref.lru_log[name], name
    assert len(ref.lru_log["ct4"]) >= 2 and len(ref.lru_log["ct6"]) >= 1


@pytest.mark.parametrize("seed", [7, 8])
def test_lru_many_sweeps_match_oracle(seed):
    """Ten batches over small LRU CT maps, a sweep after most of them: every
    eviction log entry, verdict and CT entry equals the oracle's rule."""
    sc = synth.fuzz(seed=seed, n_packets=16000, n_batches=10, ct_max=2000, ct6_max=400)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        now = sc.now + 30 * bi
        io = dp.ingress(DeviceBatch(pk), now)
        torch.cuda.synchronize()
        _cmp(to_numpy(io, ING_OUT), ref.ingress(pk, now), f"ingress b{bi}")
    for name in ("ct4", "ct6"):
        assert dp.dump_map(name) == ref.dump(name), name
        assert _evict_log(dp.fd[name]) == ref.lru_log[name], name
    assert len(ref.lru_log["ct4"]) >= 4


def test_lru_hand_wraps_and_reuses_free_slots():
    """Many evicting batches over small LRU CT maps: the hand passes the whole ring of
    home lines several times, the slots it frees are claimed again by later inserts
    (FREE), and tombstones of ct_delete are cleared on its way.  After every batch the
    verdicts and the count, and at the end both tables and both eviction logs, equal
    the oracle's restatement of the rule."""
    # (batches small enough that no batch can fill the slot array: an insert that fails
    # inside a batch depends on the lanes' order, which nothing pins)
    sc = synth.fuzz(seed=33, n_packets=2500, n_batches=16, ct_max=600, ct6_max=400)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        now = sc.now + 20 * bi
        io = dp.ingress(DeviceBatch(pk), now)
        torch.cuda.synchronize()
        _cmp(to_numpy(io, ING_OUT), ref.ingress(pk, now), f"ingress b{bi}")
        for name in ("ct4", "ct6"):
            assert bpf.GetMapInfo(dp.fd[name]).Entries == ref.m[name].count(), (bi, name)
    for name, ksz in (("ct4", 14), ("ct6", 40)):
        assert dp.dump_map(name) == ref.dump(name), name
        log = _evict_log(dp.fd[name])
        assert log == ref.lru_log[name], name
        ns = 64
        while ns < (8 * 600 if name == "ct4" else 4 * 400):      # gf_ct_slot_factor
            ns *= 2
        nl = ns // (4 if ksz == 14 else 2)
        assert len(log) >= 6 and sum(e[4] for e in log) > 2 * nl, (name, len(log), sum(e[4] for e in log), nl)


def test_concurrent_classify_two_streams():
    """Two host threads, each running its own programs (a cilium_policy array with
    its own CT, policy, CIDR and LB maps, its own prefilter) on its own HIP stream,
    enter their classify calls together: no process-wide lock (the calls overlap
    on the host), per-stream call contexts and per-object device order; every
    record and both CT maps stay bit-exact vs the oracle
    (pkg/bpf/map.go:121: per-map locks, programs concurrent on every CPU)."""
    from cilium_amd.datapath import LB_OUT
    scs = [synth.fuzz(seed=s, n_packets=12000, n_batches=3) for s in (31, 32)]
    dps = [Datapath(sc, pin_prefix=None) for sc in scs]
    refs = [OracleDP(sc) for sc in scs]
    want = []
    for sc, ref in zip(scs, refs):
        want.append([(ref.xdp(pk), ref.lb(pk)[0], ref.ingress(pk, sc.now + bi)) for bi, pk in enumerate(sc.batches)])
    bar = threading.Barrier(2)
    spans = [[], []]
    got = [[], []]
    errs = []

    def run(t):
        try:
            sc, dp = scs[t], dps[t]
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                bs = [DeviceBatch(pk) for pk in sc.batches]
                st.synchronize()
                for bi, b in enumerate(bs):
                    bar.wait()
                    a = time.perf_counter()
                    v = dp.xdp(b)
                    lo, _ = dp.lb(b)
                    io = dp.ingress(b, sc.now + bi)
                    spans[t].append((a, time.perf_counter()))
                    got[t].append((v, lo, io))
                st.synchronize()
        except Exception as e:          # reported by the main thread
            errs.append(e)
            bar.abort()

    th = [threading.Thread(target=run, args=(t,)) for t in (0, 1)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not errs, errs
    torch.cuda.synchronize()
    for t in (0, 1):
        for bi, (v, lo, io) in enumerate(got[t]):
            wx, wl, wi = want[t][bi]
            _cmp(v.cpu().numpy(), wx, f"t{t} xdp b{bi}")
            _cmp(to_numpy(lo, LB_OUT), wl, f"t{t} lb b{bi}")
            _cmp(to_numpy(io, ING_OUT), wi, f"t{t} ingress b{bi}")
        assert dps[t].dump_map("ct4") == refs[t].dump("ct4") and dps[t].dump_map("ct6") == refs[t].dump("ct6")
    overlap = sum(1 for (a0, b0), (a1, b1) in zip(spans[0], spans[1]) if a0 < b1 and a1 < b0)
    assert overlap >= 1, (spans, "classify calls never overlapped on the host")


def test_prefilter_and_endpoint_edits_between_calls_on_two_streams():
    """cilium_lxc and the /32 prefilter map edited (update and delete) between XDP
    and pipeline calls issued alternately on two torch streams: the compact address
    sets the kernels read are rebuilt on the issuing stream, ordered after the
    previous call on the other stream, and every verdict equals the oracle's after
    the same edits (the maps classify binds, not side maps)."""
    from cilium_amd.datapath import PIPE_OUT
    sc = synth.pipeline_fuzz(seed=41, n_packets=8000, n_batches=4)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    x = sc.xdp
    fix, lxc = x["cidr4_hmap"], x["lxc_map"]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    rng = np.random.default_rng(5)
    for bi, pk in enumerate(sc.batches):
        f = np.asarray(pk.frames)
        src = f[rng.integers(0, pk.n, 40), 26:30]
        dst = f[rng.integers(0, pk.n, 40), 30:34]
        # /32 entries for sources the traffic uses (then drop half of them again)
        for k, a in enumerate(src):
            key = (32).to_bytes(4, "little") + bytes(a)
            bpf.UpdateElement(dp.fd[fix], key, b"\x01")
            ref.m[fix].update(key, b"\x01")
            if k % 2:
                bpf.DeleteElement(dp.fd[fix], key)
                ref.m[fix].delete(key)
        # endpoints: delete some destinations the traffic uses, add others
        for k, a in enumerate(dst):
            key = bytes(a) + bytes(12) + b"\x01" + bytes(3)
            if k % 3 == 0:
                if ref.m[lxc].lookup(key) is not None:
                    bpf.DeleteElement(dp.fd[lxc], key)
                    ref.m[lxc].delete(key)
            else:
                val = bytes(4) + (300 + k).to_bytes(2, "little") + (1000 + k).to_bytes(2, "little") + bytes(104)
                bpf.UpdateElement(dp.fd[lxc], key, val)
                ref.m[lxc].update(key, val)
        s = streams[bi % 2]
        with torch.cuda.stream(s):
            b = DeviceBatch(pk, parse=False)
            b.parse()
            v = dp.xdp(b)
            out, _, snap = dp.pipeline(b, sc.now + bi)
        s.synchronize()
        _cmp(v.cpu().numpy(), ref.xdp(pk), f"xdp b{bi}")
        ro, _, rs = ref.pipeline(pk, sc.now + bi)
        _cmp(to_numpy(out, PIPE_OUT), ro, f"pipeline b{bi}")
        assert np.array_equal(snap.cpu().numpy(), rs), f"rewritten frames b{bi}"


def _rss_gb():
    for line in open("/proc/self/status"):
        if line.startswith("VmRSS:"):
            return int(line.split()[1]) * 1024 / 1e9
    return 0.0


def test_binding_a_large_ct_map_keeps_it_off_the_host():
    """A CT map is sized once at creation (gf_ct_slot_factor x max_entries slots).
    Binding programs to it and classifying must not build the host shadow of the
    table (Map::make_fixed_capacity returns early when the capacity is in place): at
    2^22 entries the CT4 array is 2^25 slots, 2 GB with its side array, which a pull
    would copy into this process.  The GPU's answers still equal the oracle's."""
    sc = synth.fuzz(seed=5, n_packets=4000, n_batches=2, ct_max=1 << 22, ct6_max=1 << 16)
    before = _rss_gb()
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        now = sc.now + bi
        io = dp.ingress(DeviceBatch(pk), now)
        torch.cuda.synchronize()
        _cmp(to_numpy(io, ING_OUT), ref.ingress(pk, now), f"ingress b{bi}")
    grown = _rss_gb() - before
    assert grown < 1.0, f"host memory grew by {grown:.2f} GB"
    assert bpf.GetMapInfo(dp.fd["ct4"]).Entries == ref.m["ct4"].count()


def test_lru_empty_sample_window_falls_back_to_whole_table():
    """keys chosen so that none is homed in the sample window (the SL lines
    ahead of the hand, the CT hash being public) on a table large enough to be sampled
    (NL > 65,536 lines).  The device finds the window empty, samples the whole table
    instead (k_lru_sample / k_lru_plan, wide) and evicts from its older half — never a
    flush — exactly as the oracle's restatement: the same eviction log, the same table."""
    import test_lru_hand as TH
    mx = 40_000
    rng = np.random.default_rng(21)
    sc = synth.fuzz(seed=12, n_packets=2000, n_batches=1, ct_max=mx, ct6_max=400)
    h = TH.Hand(14, mx)
    assert h.nl > 65536 and h.sl < h.nl
    now = sc.now
    keys, vals = TH._table(rng, 14, 3 * mx, now)
    out = h.home_lines(keys) >= h.sl                 # the hand stands at line 0: nothing homed in [0, SL)
    keys, vals = keys[out][: mx + 3000], vals[out][: mx + 3000]
    assert len(keys) == mx + 3000
    ct = sc.maps["ct4"]
    ct.keys, ct.vals = keys, vals
    pk = sc.batches[0]
    pk.frames[:, 12], pk.frames[:, 13] = 0x88, 0xB5  # an unknown ethertype: no packet reaches conntrack
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    io = dp.ingress(DeviceBatch(pk), now)
    torch.cuda.synchronize()
    _cmp(to_numpy(io, ING_OUT), ref.ingress(pk, now), "ingress")
    log = _evict_log(dp.fd["ct4"])
    assert log == ref.lru_log["ct4"] and len(log) == 1, (log, ref.lru_log["ct4"])
    K, evicted = log[0][2], log[0][5]
    ak = TH.age_keys(vals, now)
    srt = np.sort(ak)
    assert K == int(srt[(len(srt) + 1) // 2 - 1])     # the whole table's median age
    n_after = bpf.GetMapInfo(dp.fd["ct4"]).Entries
    assert n_after == ref.m["ct4"].count() == len(keys) - evicted <= mx
    assert evicted <= (ak <= K).sum() and n_after >= len(keys) // 3
    assert dp.dump_map("ct4") == ref.dump("ct4")
