"""Golden fixtures (tests/golden/, made by tests/golden/make_golden.py):
the reference's own known answers as data, and a seeded frame scenario with
the outputs every program must give.  CPU: the oracle reproduces them (its
behaviour is frozen).  GPU: the HIP path reproduces the same bytes without
consulting the oracle."""
import ctypes as C
import json
import os
import struct

import numpy as np
import pytest

from cilium_amd import synth

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KATS = json.load(open(os.path.join(HERE, "unit_test_kats.json")))
META = json.load(open(os.path.join(HERE, "fuzz21.json")))
GOLD = np.load(os.path.join(HERE, "fuzz21.npz"))

from golden.make_golden import input_digest, dump_digest, state_maps   # noqa: E402


def _scenario():
    sc = synth.fuzz(**META["args"])
    assert input_digest(sc) == META["input_sha256"], "scenario generator drifted from the fixture"
    return sc


@pytest.mark.parametrize("case", KATS["ipv6_addr_clear_suffix"], ids=lambda c: str(c["prefix"]))
def test_unit_test_c_clear_suffix(case):
    from oracle import oracle as O
    a = (C.c_uint8 * 16)(*([0xff] * 16))
    O.lib.o_ipv6_addr_clear_suffix(a, case["prefix"])
    assert list(struct.unpack(">4I", bytes(a))) == case["words"]


def test_unit_test_c_lpm_iteration():
    from oracle import oracle as O
    htonl = lambda x: struct.unpack("<I", struct.pack(">I", x))[0]
    for c in KATS["lpm4_prefix_iteration"]:
        arr = (C.c_int * len(c["prefixes"]))(*c["prefixes"])
        got = bool(O.lib.o_lpm4_iter_lookup(htonl(c["stored"]), arr, len(c["prefixes"]), htonl(c["addr"])))
        assert got == c["hit"], c


def test_oracle_reproduces_golden_fuzz():
    from oracle.scenario import OracleDP
    sc = _scenario()
    ref = OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        assert np.array_equal(ref.xdp(pk), GOLD[f"xdp_{bi}"])
        lo, nd6 = ref.lb(pk)
        assert np.array_equal(lo.view(np.uint8).reshape(len(lo), -1), GOLD[f"lb_{bi}"])
        assert np.array_equal(nd6, GOLD[f"lb_nd6_{bi}"])
        io = ref.ingress(pk, sc.now + bi)
        assert np.array_equal(io.view(np.uint8).reshape(len(io), -1), GOLD[f"ingress_{bi}"])
    for n in state_maps(sc):
        assert dump_digest(ref.dump(n)) == META["state_sha256"][n], n


@pytest.mark.gpu
def test_hip_reproduces_golden_fuzz():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    from cilium_amd.datapath import Datapath, DeviceBatch, LB_OUT, ING_OUT, to_numpy
    sc = _scenario()
    dp = Datapath(sc, pin_prefix=None)
    for bi, pk in enumerate(sc.batches):
        b = DeviceBatch(pk)
        v, (lo, nd6), io = dp.xdp(b), dp.lb(b), dp.ingress(b, sc.now + bi)
        torch.cuda.synchronize()
        assert np.array_equal(v.cpu().numpy(), GOLD[f"xdp_{bi}"]), f"xdp b{bi}"
        assert np.array_equal(to_numpy(lo, LB_OUT).view(np.uint8).reshape(len(lo), -1), GOLD[f"lb_{bi}"]), f"lb b{bi}"
        assert np.array_equal(nd6.cpu().numpy(), GOLD[f"lb_nd6_{bi}"]), f"lb nd6 b{bi}"
        got = to_numpy(io, ING_OUT)
        assert np.array_equal(got.view(np.uint8).reshape(len(got), -1), GOLD[f"ingress_{bi}"]), f"ingress b{bi}"
    for n in state_maps(sc):
        assert dump_digest(dp.dump_map(n)) == META["state_sha256"][n], n
