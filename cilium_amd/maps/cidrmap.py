"""pkg/maps/cidrmap mirror (/root/reference/pkg/maps/cidrmap/cidrmap.go:30-220).

Key: ``struct {u32 prefixlen; u8 net[AddrSize]}`` (cidrKey, :52-55), value 1 B.
"""
import ipaddress
import struct

from .. import bpf

MapName = "cilium_cidr_"
MaxEntries = 16384
LPM_MAP_VALUE_SIZE = 1


class CIDRMap:
    def __init__(self, path, fd, addr_size, prefixlen, dynamic):
        self.path, self.Fd, self.AddrSize = path, fd, addr_size
        self.Prefixlen, self.PrefixIsDynamic = prefixlen, dynamic

    def key_size(self):
        return 4 + self.AddrSize

    def cidrKeyInit(self, cidr):
        net = ipaddress.ip_network(cidr, strict=False)
        raw = net.network_address.packed
        return struct.pack("<I", net.prefixlen) + raw[len(raw) - self.AddrSize:]

    def keyCidrInit(self, key):
        plen = struct.unpack_from("<I", key)[0]
        addr = key[4:4 + self.AddrSize]
        ip = ipaddress.ip_address(addr)
        return ipaddress.ip_network(f"{ip}/{plen}", strict=False)

    def checkPrefixlen(self, key, operation):
        plen = struct.unpack_from("<I", key)[0]
        if self.Prefixlen != 0 and ((self.PrefixIsDynamic and self.Prefixlen < plen) or
                                    (not self.PrefixIsDynamic and self.Prefixlen != plen)):
            raise ValueError(f"Unable to {operation} element with dynamic prefix length "
                             f"cm.Prefixlen={self.Prefixlen} key.Prefixlen={plen}")

    def InsertCIDR(self, cidr):
        key = self.cidrKeyInit(cidr)
        self.checkPrefixlen(key, "update")
        bpf.UpdateElement(self.Fd, key, b"\x00", 0)

    def DeleteCIDR(self, cidr):
        key = self.cidrKeyInit(cidr)
        self.checkPrefixlen(key, "delete")
        bpf.DeleteElement(self.Fd, key)

    def CIDRExists(self, cidr):
        try:
            bpf.LookupElement(self.Fd, self.cidrKeyInit(cidr), LPM_MAP_VALUE_SIZE)
            return True
        except bpf.BPFError:
            return False

    def CIDRNext(self, cidr):
        key = self.cidrKeyInit(cidr) if cidr is not None else b"\x00" * self.key_size()
        try:
            nk = bpf.GetNextKey(self.Fd, key, self.key_size())
        except bpf.BPFError:
            return None
        return self.keyCidrInit(nk)

    def CIDRDump(self, to=None):
        to = [] if to is None else to
        key = None
        while True:
            nk = self.CIDRNext(key)
            if nk is None:
                return to
            key = nk
            to.append(str(key))

    def Close(self):
        bpf.ObjClose(self.Fd)


def OpenMapElems(path, prefixlen, prefixdyn, maxelem):
    """cidrmap.OpenMapElems (:166-220): LPM trie if the prefix is dynamic, else hash."""
    if prefixlen <= 0:
        raise ValueError("prefixlen must be > 0")
    typ = bpf.BPF_MAP_TYPE_LPM_TRIE if prefixdyn else bpf.BPF_MAP_TYPE_HASH
    prefix = 0 if prefixdyn else prefixlen
    nbytes = (prefixlen - 1) // 8 + 1
    fd, new = bpf.OpenOrCreateMap(path, typ, 4 + nbytes, LPM_MAP_VALUE_SIZE, maxelem, bpf.BPF_F_NO_PREALLOC)
    return CIDRMap(path, fd, nbytes, prefix, prefixdyn), new


def OpenMap(path, prefixlen, prefixdyn):
    return OpenMapElems(path, prefixlen, prefixdyn, MaxEntries)
