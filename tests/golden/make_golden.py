"""Generates the committed golden fixtures of tests/golden/ — run from the repo
root:  python tests/golden/make_golden.py

* unit_test_kats.json — the only per-function known answers the reference's
  own tests hold for this path, transcribed as data from
  test/bpf/unit-test.c:20-58 (ipv6_addr_clear_suffix) and :60-102 (the
  prefix-iterating LPM lookup, LPM_LOOKUP_FN of bpf/lib/maps.h:147-160).
* fuzz<seed>.npz / .json — a seeded multi-batch frame scenario
  (cilium_amd.synth.fuzz: weird IHL, truncation, IPv6 extension chains,
  replies, related ICMP, deletes on deny, proxies, rev-NAT ...) with the
  oracle's outputs for every program (XDP verdicts, LB records, ingress
  records) and digests of the device-authoritative map state afterwards.
  The reference BPF programs cannot be run here; these vectors
  come from the CPU restatement (oracle/), which the KATs pin.  They freeze
  its behaviour so any later drift — in the oracle or in the HIP path, which
  tests/test_golden.py checks against the same file on the GPU — is caught.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

FUZZ = dict(seed=21, n_packets=3000, n_batches=3)

KATS = {
    "source": "reference test/bpf/unit-test.c",
    # test_ipv6_addr_clear_suffix (:20-58): all-ones address, prefix -> 4 big-endian words
    "ipv6_addr_clear_suffix": [
        {"prefix": 128, "words": [0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff]},
        {"prefix": 127, "words": [0xffffffff, 0xffffffff, 0xffffffff, 0xfffffffe]},
        {"prefix": 95, "words": [0xffffffff, 0xffffffff, 0xfffffffe, 0x00000000]},
        {"prefix": 1, "words": [0x80000000, 0x00000000, 0x00000000, 0x00000000]},
        {"prefix": -1, "words": [0x00000000, 0x00000000, 0x00000000, 0x00000000]},
    ],
    # test_lpm_lookup (:60-102): stored prefix (host order), prefix list, address, expected hit
    "lpm4_prefix_iteration": [
        {"stored": 0xFFFFFFFF, "prefixes": [32], "addr": 0xFFFFFFFF, "hit": True},
        {"stored": 0xFFFFFFFF, "prefixes": [32], "addr": 0xFFF00000, "hit": False},
        {"stored": 0xFFFFFFFE, "prefixes": [31], "addr": 0xFFFFFFFE, "hit": True},
        {"stored": 0xFFFFFFFE, "prefixes": [31], "addr": 0xFFFFFFFF, "hit": True},
        {"stored": 0xFFFFFFFE, "prefixes": [31], "addr": 0xFFF00000, "hit": False},
        {"stored": 0xFFFFFC00, "prefixes": [22], "addr": 0xFFFFFC00, "hit": True},
        {"stored": 0xFFFFFC00, "prefixes": [22], "addr": 0xFFFFFFFF, "hit": True},
        {"stored": 0xFFFFFC00, "prefixes": [22], "addr": 0xFFF00000, "hit": False},
        {"stored": 0xFFE00000, "prefixes": [11], "addr": 0xFFE00000, "hit": True},
        {"stored": 0xFFE00000, "prefixes": [11], "addr": 0xFFFFFFFF, "hit": True},
        {"stored": 0xFFE00000, "prefixes": [11], "addr": 0xFFF00000, "hit": True},
        {"stored": 0xF0000000, "prefixes": [11], "addr": 0xF0000000, "hit": True},
        {"stored": 0x00000000, "prefixes": [0], "addr": 0x00000000, "hit": True},
        {"stored": 0x00000000, "prefixes": [0], "addr": 0xFFFFFFFF, "hit": True},
    ],
}


def input_digest(sc):
    """sha256 over every table and every batch column of a scenario."""
    h = hashlib.sha256()
    for name in sorted(sc.maps):
        m = sc.maps[name]
        h.update(name.encode())
        h.update(np.ascontiguousarray(m.keys).tobytes())
        h.update(np.ascontiguousarray(m.vals).tobytes())
    for pk in sc.batches:
        for a in (pk.frames, pk.lens, pk.src_identity, pk.ifindex, pk.lxc_id, pk.tc_index, pk.flow_hash):
            h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def dump_digest(entries):
    h = hashlib.sha256()
    for k, v in sorted(entries.items()):
        h.update(bytes(k)); h.update(bytes(v))
    return h.hexdigest()


def state_maps(sc):
    return [n for n in sorted(sc.maps) if n.startswith("ct") or n.startswith("pol")]


def main():
    from cilium_amd import synth
    from oracle.scenario import OracleDP
    with open(os.path.join(HERE, "unit_test_kats.json"), "w") as f:
        json.dump(KATS, f, indent=1)
    sc = synth.fuzz(**FUZZ)
    ref = OracleDP(sc)
    arrays = {}
    for bi, pk in enumerate(sc.batches):
        arrays[f"xdp_{bi}"] = ref.xdp(pk)
        lo, nd6 = ref.lb(pk)
        arrays[f"lb_{bi}"] = lo.view(np.uint8).reshape(len(lo), -1)
        arrays[f"lb_nd6_{bi}"] = nd6
        io = ref.ingress(pk, sc.now + bi)
        arrays[f"ingress_{bi}"] = io.view(np.uint8).reshape(len(io), -1)
    tag = f"fuzz{FUZZ['seed']}"
    np.savez_compressed(os.path.join(HERE, tag + ".npz"), **arrays)
    meta = {"generator": "cilium_amd.synth.fuzz", "args": FUZZ, "input_sha256": input_digest(sc),
            "state_sha256": {n: dump_digest(ref.dump(n)) for n in state_maps(sc)},
            "state_entries": {n: len(ref.dump(n)) for n in state_maps(sc)}}
    with open(os.path.join(HERE, tag + ".json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", tag, meta["state_entries"])


if __name__ == "__main__":
    main()
