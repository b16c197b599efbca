"""Map API (pkg/bpf replacement) semantics on the host shadow — no GPU needed.
Checked against the oracle's independent map restatement (kernel htab /
lpm_trie semantics) on random operation sequences."""
import errno
import random
import struct

import numpy as np
import pytest

from cilium_amd import bpf
from cilium_amd.maps import cidrmap, policymap, lbmap, lxcmap, ctmap
from oracle import oracle as O


def _ops(typ, ksz, vsz, maxe, seed, nops=3000, keyspace=300):
    rnd = random.Random(seed)
    fd = bpf.CreateMap(typ, ksz, vsz, maxe, bpf.BPF_F_NO_PREALLOC if typ == 11 else 0)
    om = O.OMap(typ, ksz, vsz, maxe)
    keys = []
    for _ in range(keyspace):
        if typ == 11:
            plen = rnd.randint(0, (ksz - 4) * 8 + 2)   # includes invalid prefix lengths
            keys.append(struct.pack("<I", plen) + bytes(rnd.getrandbits(8) for _ in range(ksz - 4)))
        else:
            keys.append(bytes(rnd.getrandbits(8) for _ in range(ksz)))
    from cilium_amd._lib import lib
    import ctypes as C
    for _ in range(nops):
        k = rnd.choice(keys)
        op = rnd.random()
        if op < 0.5:
            v = bytes(rnd.getrandbits(8) for _ in range(vsz))
            fl = rnd.choice([0, 0, 1, 2, 5])
            a = lib.gf_map_update_elem(fd, k, v, fl)
            b = om.update(k, v, fl)
            assert a == b, (a, b, fl)
        elif op < 0.8:
            vb = C.create_string_buffer(vsz)
            a = lib.gf_map_lookup_elem(fd, k, vb)
            ov = om.lookup(k)
            assert (a == 0) == (ov is not None)
            if a == 0:
                assert vb.raw == ov
        else:
            a = lib.gf_map_delete_elem(fd, k)
            b = om.delete(k)
            assert a == b
    return fd, om


@pytest.mark.parametrize("ksz,vsz", [(8, 24), (14, 48), (40, 48), (20, 112), (2, 6), (8, 1)])
def test_hash_semantics_vs_oracle(ksz, vsz):
    fd, om = _ops(bpf.BPF_MAP_TYPE_HASH, ksz, vsz, 200, seed=ksz * 131 + vsz)
    # full iteration via get_next_key visits every element exactly once
    got = {}
    m = bpf.Map("x", 1, ksz, vsz, 200)
    m.fd = fd
    m.DumpWithCallback(lambda k, v: got.__setitem__(k, v))
    assert got == om.dump()
    assert bpf.GetMapInfo(fd).Entries == om.count()
    # the reference's own loop (GetNextKey + LookupElement) and small dump chunks agree
    kbk, small = [], []
    m.DumpKeyByKey(lambda k, v: kbk.append((k, v)))
    m.DumpWithCallback(lambda k, v: small.append((k, v)), chunk=7)
    assert kbk == small and dict(kbk) == got


def test_lookup_batch_cursor_contract():
    """gf_map_lookup_batch: every entry exactly once across chunks, -ENOENT with the
    last chunk, an exhausted cursor keeps returning -ENOENT with count 0; LPM tries
    dump in get_next_key's post-order."""
    fd, om = _ops(bpf.BPF_MAP_TYPE_HASH, 14, 48, 500, seed=9, nops=2000, keyspace=400)
    seen, cur, done, calls = [], None, False, 0
    while not done:
        k, v, cur, done = bpf.LookupBatch(fd, cur, 13, 14, 48)
        assert len(k) <= 13
        seen += [(a.tobytes(), b.tobytes()) for a, b in zip(k, v)]
        calls += 1
    assert dict(seen) == om.dump() and len(seen) == len(om.dump())
    k, v, cur2, done = bpf.LookupBatch(fd, cur, 13, 14, 48)
    assert len(k) == 0 and done
    lfd, lom = _ops(bpf.BPF_MAP_TYPE_LPM_TRIE, 8, 1, 120, seed=3)
    lm = bpf.Map("l", 11, 8, 1, 120)
    lm.fd = lfd
    a, b = [], []
    lm.DumpKeyByKey(lambda k, v: a.append(k))
    lm.DumpWithCallback(lambda k, v: b.append(k), chunk=5)
    assert a == b


def test_gc_on_fresh_lru_ct_map():
    """ctmap.GC / Flush on a CT map that holds no entry yet — freshly opened (an
    LRU map's slot array is not materialised until its first insert) and after a
    program bound it but before any classify — deletes nothing and succeeds."""
    import ctypes as C
    from cilium_amd._lib import lib, gf_lxc_cfg
    for ksz in (14, 40):
        fd = bpf.CreateMap(bpf.BPF_MAP_TYPE_LRU_HASH, ksz, 48, 1 << 16)
        assert lib.gf_ct_gc(fd, 5000, None) == 0
        assert lib.gf_ct_gc(fd, 0xFFFFFFFF, None) == 0           # Flush
    ct4 = bpf.CreateMap(bpf.BPF_MAP_TYPE_LRU_HASH, 14, 48, 1 << 16)
    pol = bpf.CreateMap(bpf.BPF_MAP_TYPE_HASH, 8, 24, 16384)
    cfg = gf_lxc_cfg()
    cfg.lxc_id, cfg.seclabel, cfg.policy_map, cfg.ct_map4, cfg.flags = 7, 300, pol, ct4, 0x1e
    assert lib.gf_lxc_prog_load(C.byref(cfg)) > 0
    assert lib.gf_ct_gc(ct4, 5000, None) == 0
    assert lib.gf_ct_gc(ct4, 0xFFFFFFFF, None) == 0
    assert bpf.GetMapInfo(ct4).Entries == 0


@pytest.mark.parametrize("ksz", [8, 20])
def test_lpm_semantics_vs_oracle(ksz):
    fd, om = _ops(bpf.BPF_MAP_TYPE_LPM_TRIE, ksz, 1, 120, seed=ksz)
    assert bpf.GetMapInfo(fd).Entries == om.count()


def test_lpm_get_next_key_is_postorder():
    fd = bpf.CreateMap(11, 8, 1, 64, bpf.BPF_F_NO_PREALLOC)
    cm = cidrmap.CIDRMap("t", fd, 4, 0, True)
    for c in ["192.168.0.0/16", "192.168.0.0/24", "192.168.1.0/24", "192.168.128.0/24", "10.0.0.0/8"]:
        cm.InsertCIDR(c)
    # kernel lpm_trie.c example order: more specific first, left (0) before right (1)
    assert cm.CIDRDump() == ["10.0.0.0/8", "192.168.0.0/24", "192.168.1.0/24", "192.168.128.0/24",
                             "192.168.0.0/16"]
    assert cm.CIDRExists("192.168.1.0/24")
    assert cm.CIDRExists("192.168.77.0/24")       # longest-prefix lookup semantics (/16 covers it)
    assert not cm.CIDRExists("11.0.0.0/8")


def test_errors_and_limits():
    fd = bpf.CreateMap(1, 8, 24, 2)
    bpf.UpdateElement(fd, b"a" * 8, b"\x00" * 24)
    bpf.UpdateElement(fd, b"b" * 8, b"\x00" * 24)
    with pytest.raises(bpf.BPFError) as e:
        bpf.UpdateElement(fd, b"c" * 8, b"\x00" * 24)
    assert e.value.errno == errno.E2BIG
    bpf.UpdateElement(fd, b"a" * 8, b"\x01" * 24)      # replacing while full is allowed
    with pytest.raises(bpf.BPFError) as e:
        bpf.UpdateElement(fd, b"a" * 8, b"\x01" * 24, bpf.BPF_NOEXIST)
    assert e.value.errno == errno.EEXIST
    with pytest.raises(bpf.BPFError) as e:
        bpf.UpdateElement(fd, b"z" * 8, b"\x01" * 24, bpf.BPF_EXIST)
    assert e.value.errno == errno.ENOENT
    with pytest.raises(bpf.BPFError) as e:
        bpf.LookupElement(fd, b"z" * 8, 24)
    assert e.value.errno == errno.ENOENT
    with pytest.raises(bpf.BPFError):
        bpf.CreateMap(11, 8, 1, 10, 0)                 # LPM requires BPF_F_NO_PREALLOC
    with pytest.raises(bpf.BPFError):
        bpf.CreateMap(1, 0, 4, 10)
    lpm = bpf.CreateMap(11, 8, 1, 1, bpf.BPF_F_NO_PREALLOC)
    bpf.UpdateElement(lpm, struct.pack("<I4s", 8, b"\x0a\x00\x00\x00"), b"\x01")
    with pytest.raises(bpf.BPFError) as e:
        bpf.UpdateElement(lpm, struct.pack("<I4s", 16, b"\x0a\x01\x00\x00"), b"\x01")
    assert e.value.errno == errno.ENOSPC
    with pytest.raises(bpf.BPFError) as e:
        bpf.UpdateElement(lpm, struct.pack("<I4s", 33, b"\x0a\x01\x00\x00"), b"\x01")
    assert e.value.errno == errno.EINVAL


@pytest.mark.parametrize("ksz,vsz", [(14, 48), (40, 48), (8, 24)])
def test_lru_insert_never_fails_below_slot_limit(ksz, vsz):
    """BPF_MAP_TYPE_LRU_HASH never fails an insert in the kernel (it evicts).  For
    the conntrack shapes (ipv4/ipv6_ct_tuple -> ct_entry) the stand-in accepts
    inserts past max_entries up to 7/8 of its slot array (8 x max_entries for
    ipv4_ct_tuple, 4 x for ipv6_ct_tuple, rounded up to a power of 2) and evicts
    at the next classify call that binds the map as ct4 / ct6, so
    GetMapInfo may exceed max_entries in between.  Any other LRU map has no
    eviction path and stops at max_entries with E2BIG, like a HASH map.  The
    oracle's OMap has the same ceilings."""
    maxe = 100
    ct_shape = ksz in (14, 40) and vsz == 48
    lim = (1024 if ksz == 14 else 512) // 8 * 7 if ct_shape else maxe   # pow2ceil(8 / 4 * 100) slots
    fd = bpf.CreateMap(bpf.BPF_MAP_TYPE_LRU_HASH, ksz, vsz, maxe)
    om = O.OMap(bpf.BPF_MAP_TYPE_LRU_HASH, ksz, vsz, maxe)
    rnd = random.Random(ksz)
    keys = [bytes(rnd.getrandbits(8) for _ in range(ksz)) for _ in range(lim + 5)]
    from cilium_amd._lib import lib
    for i, k in enumerate(keys):
        a, b = lib.gf_map_update_elem(fd, k, bytes(vsz), 0), om.update(k, bytes(vsz), 0)
        assert a == b == (0 if i < lim else -errno.E2BIG), (i, a, b)
    assert bpf.GetMapInfo(fd).Entries == om.count() == lim
    assert (lim > maxe) == ct_shape
    # replacing an existing key at the ceiling still succeeds
    assert lib.gf_map_update_elem(fd, keys[0], bytes([1]) * vsz, 0) == 0 == om.update(keys[0], bytes([1]) * vsz, 0)
    h = bpf.CreateMap(bpf.BPF_MAP_TYPE_HASH, ksz, vsz, maxe)
    rc = [lib.gf_map_update_elem(h, k, bytes(vsz), 0) for k in keys[:maxe + 1]]
    assert rc[:maxe] == [0] * maxe and rc[maxe] == -errno.E2BIG


def test_pin_get_close_and_open_or_create():
    path = bpf.MapPath("test_pin_map")
    fd, new = bpf.OpenOrCreateMap(path, 1, 8, 24, 100, 0)
    assert new and fd > 0
    bpf.UpdateElement(fd, b"k" * 8, b"v" * 24)
    fd2, new2 = bpf.OpenOrCreateMap(path, 1, 8, 24, 100, 0)
    assert not new2 and bpf.LookupElement(fd2, b"k" * 8, 24) == b"v" * 24
    fd3, new3 = bpf.OpenOrCreateMap(path, 1, 8, 24, 200, 0)   # property mismatch -> recreated, data lost
    assert new3
    with pytest.raises(bpf.BPFError):
        bpf.LookupElement(fd3, b"k" * 8, 24)
    bpf.ObjClose(fd2)
    with pytest.raises(bpf.BPFError):
        bpf.ObjGet("/sys/fs/bpf/tc/globals/does_not_exist")


def test_policymap_wrapper():
    pm, _ = policymap.OpenMap(bpf.MapPath("cilium_policy_t1"))
    pm.AllowIdentity(300)
    pm.AllowL4(301, 80, 6)
    pm.AllowL4(302, 443, 6, proxy_port=15001)
    assert pm.IdentityExists(300) and pm.L4Exists(301, 80, 6) and not pm.L4Exists(301, 81, 6)
    d = {(e.Identity, e.DestPort, e.Nexthdr): e.ProxyPort for e in pm.DumpToSlice()}
    assert d[(301, 0x5000, 6)] == 0 and d[(302, 0xbb01, 6)] == 0x993a
    pm.DeleteL4(301, 80, 6)
    assert not pm.L4Exists(301, 80, 6)
    pm.Flush()
    assert pm.DumpToSlice() == []


def test_lbmap_add_svc_layout():
    lb = lbmap.LBMaps(prefix="t2_")
    lb.AddSVC2BPFMap("10.96.0.10", 80, [("10.0.0.1", 8080, 0), ("10.0.0.2", 80, 0)], True, 7)
    master = bpf.LookupElement(lb.s4, lbmap.LBMaps.service4_key("10.96.0.10", 80, 0), 12)
    assert struct.unpack("<4sHHHH", master)[2] == 2          # count, host order
    be2 = bpf.LookupElement(lb.s4, lbmap.LBMaps.service4_key("10.96.0.10", 80, 2), 12)
    assert be2[:4] == bytes([10, 0, 0, 2]) and struct.unpack_from("<H", be2, 4)[0] == 0x5000
    assert struct.unpack_from("<H", be2, 8)[0] == 0x0700                # rev_nat in network order
    rn = bpf.LookupElement(lb.r4, struct.pack("<H", 0x0700), 6)
    assert rn == bytes([10, 96, 0, 10, 0, 80])


def test_lxcmap_and_ctmap_wrappers():
    lx = lxcmap.LXCMap(path=bpf.MapPath("lxc_t3"))
    lx.WriteEndpoint(["10.1.0.5", "f00d::5"], lxcmap.endpoint_info(ifindex=7, lxc_id=99))
    lx.AddHostEntry("10.0.0.1")
    assert bpf.LookupElement(lx.fd, lxcmap.endpoint_key("10.1.0.5"), 112)[:4] == struct.pack("<I", 7)
    fd, _ = ctmap.OpenMap(bpf.MapPath("ct4_t3"), max_entries=1000)
    bpf.UpdateElement(fd, ctmap.ct_key4(1, 2, 3, 4, 6, 1), ctmap.ct_entry(lifetime=50))
    bpf.UpdateElement(fd, ctmap.ct_key4(1, 2, 3, 5, 6, 1), ctmap.ct_entry(lifetime=500))
    assert ctmap.GC(fd, 100) == 1
    assert len(ctmap.Dump(fd)) == 1


def test_batch_update_matches_sequential():
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 256, (500, 14), dtype=np.uint8)
    vals = rng.integers(0, 256, (500, 48), dtype=np.uint8)
    a = bpf.CreateMap(1, 14, 48, 1000)
    b = bpf.CreateMap(1, 14, 48, 1000)
    bpf.UpdateBatch(a, keys.ctypes.data, vals.ctypes.data, 500)
    for i in range(500):
        bpf.UpdateElement(b, keys[i].tobytes(), vals[i].tobytes())
    ma, mb = bpf.Map("a", 1, 14, 48, 1000), bpf.Map("b", 1, 14, 48, 1000)
    ma.fd, mb.fd = a, b
    assert ma.Dump() == mb.Dump()


@pytest.mark.parametrize("v6", [False, True])
def test_ctmap_gc_and_flush_host_shadow(v6):
    """ctmap.GC (GCFilterByTime: lifetime < now) and Flush through gf_ct_gc on a
    host-authoritative map, against the oracle's restatement of doGC4/doGC6."""
    rng = random.Random(7 + v6)
    fd, _ = ctmap.OpenMap(bpf.MapPath(f"test_gc_{int(v6)}"), v6=v6, max_entries=5000)
    om = O.OMap(9, 40 if v6 else 14, 48, 5000)
    for i in range(3000):
        if v6:
            k = ctmap.ct_key6(rng.randbytes(16), rng.randbytes(16), rng.getrandbits(16), rng.getrandbits(16), 6, i & 1)
        else:
            k = ctmap.ct_key4(rng.getrandbits(32), rng.getrandbits(32), rng.getrandbits(16), rng.getrandbits(16), 6,
                              i & 3)
        v = ctmap.ct_entry(rx_packets=i, lifetime=rng.choice([0, 5, 99, 100, 101, 43300]), flags=16)
        bpf.UpdateElement(fd, k, v)
        assert om.update(k, v) == 0
    want = O.lib.o_ct_gc(om.ptr, 100)
    got = ctmap.GC(fd, 100, v6=v6)
    assert got == want > 0
    left = dict(ctmap.Dump(fd, v6))
    assert set(left) == set(om.dump())
    assert all(e.lifetime >= 100 for e in left.values())
    assert ctmap.Flush(fd, v6=v6) == len(left)
    assert ctmap.Dump(fd, v6) == []
    bpf.ObjClose(fd)


def test_ct_map_names_global_and_local():
    """pkg/endpoint/bpf.go:268-276: CT_MAP4/6 are the global maps unless the endpoint
    has ConntrackLocal, which gives it cilium_ct4_<id> / cilium_ct6_<id> of
    MapNumEntriesLocal entries (pkg/maps/ctmap/ctmap.go:34-41)."""
    assert ctmap.MapNames() == ("cilium_ct6_global", "cilium_ct4_global", 1000000)
    assert ctmap.MapNames(111, local=True) == ("cilium_ct6_111", "cilium_ct4_111", 64000)
    with pytest.raises(ValueError):
        ctmap.MapNames(local=True)
