"""pkg/maps/policymap mirror (/root/reference/pkg/maps/policymap/policymap.go).

policyKey  {u32 Identity; u16 DestPort (network order); u8 Nexthdr; u8 TrafficDirection}  8 B
PolicyEntry {u16 ProxyPort (network order); u16 pad[3]; u64 Packets; u64 Bytes}          24 B
"""
import errno
import socket
import struct

from .. import bpf

MapName = "cilium_policy_"
MaxEntries = 16384
Ingress, Egress = 0, 1          # trafficdirection.go:21-28
KEY = struct.Struct("<IHBB")
ENTRY = struct.Struct("<HHHHQQ")


def htons(p):
    return socket.htons(p)


def policy_key(identity, dport_be=0, proto=0, direction=Ingress):
    return KEY.pack(identity, dport_be, proto, direction)


def policy_entry(proxy_port_be=0, packets=0, nbytes=0):
    return ENTRY.pack(proxy_port_be, 0, 0, 0, packets, nbytes)


class PolicyEntryDump:
    def __init__(self, key, val):
        self.Identity, self.DestPort, self.Nexthdr, self.TrafficDirection = KEY.unpack(key)
        pp, _, _, _, self.Packets, self.Bytes = ENTRY.unpack(val)
        self.ProxyPort = pp
        self.Key = key


class PolicyMap:
    def __init__(self, path, fd):
        self.path, self.Fd = path, fd

    def AllowIdentity(self, id_, direction=Ingress):
        bpf.UpdateElement(self.Fd, policy_key(id_, 0, 0, direction), policy_entry(), 0)

    def AllowL4(self, id_, dport, proto, direction=Ingress, proxy_port=0):
        bpf.UpdateElement(self.Fd, policy_key(id_, htons(dport), proto, direction),
                          policy_entry(htons(proxy_port) if proxy_port else 0), 0)

    def _exists(self, key):
        try:
            bpf.LookupElement(self.Fd, key, ENTRY.size)
            return True
        except bpf.BPFError:
            return False

    def IdentityExists(self, id_, direction=Ingress):
        return self._exists(policy_key(id_, 0, 0, direction))

    def L4Exists(self, id_, dport, proto, direction=Ingress):
        return self._exists(policy_key(id_, htons(dport), proto, direction))

    def DeleteIdentity(self, id_, direction=Ingress):
        bpf.DeleteElement(self.Fd, policy_key(id_, 0, 0, direction))

    def DeleteL4(self, id_, dport, proto, direction=Ingress):
        bpf.DeleteElement(self.Fd, policy_key(id_, htons(dport), proto, direction))

    def DeleteEntry(self, entry):
        bpf.DeleteElement(self.Fd, entry.Key)

    def DumpToSlice(self):
        out = []
        key = None
        while True:
            try:
                nk = bpf.GetNextKey(self.Fd, key, KEY.size)
            except bpf.BPFError as e:
                if e.errno == errno.ENOENT:
                    return out
                raise
            out.append(PolicyEntryDump(nk, bpf.LookupElement(self.Fd, nk, ENTRY.size)))
            key = nk

    def Flush(self):
        for e in self.DumpToSlice():
            bpf.DeleteElement(self.Fd, e.Key)

    def Close(self):
        bpf.ObjClose(self.Fd)


def OpenMap(path, max_entries=MaxEntries):
    fd, new = bpf.OpenOrCreateMap(path, bpf.BPF_MAP_TYPE_HASH, KEY.size, ENTRY.size, max_entries, 0)
    return PolicyMap(path, fd), new
