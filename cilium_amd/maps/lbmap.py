"""pkg/maps/lbmap mirror (/root/reference/pkg/maps/lbmap/{lbmap,ipv4,ipv6}.go).

Service4Key {IPv4 Address; u16 Port; u16 Slave}           8 B  (Port -> network order)
Service4Value {IPv4 Address; u16 Port; u16 Count; u16 RevNat; u16 Weight} 12 B
  (ToNetwork converts Port, RevNat, Weight; Count stays host order)
RevNat4Key u16 (network order) -> RevNat4Value {IPv4 Address; u16 Port}  6 B
Service6*/RevNat6*: 16-byte addresses.
"""
import ipaddress
import socket
import struct

from .. import bpf

MaxEntries = 65536
MaxSeq = 31
S4K = struct.Struct("<4sHH")
S4V = struct.Struct("<4sHHHH")
S6K = struct.Struct("<16sHH")
S6V = struct.Struct("<16sHHHH")
R4V = struct.Struct("<4sH")
R6V = struct.Struct("<16sH")


def _a(ip, n):
    return ipaddress.ip_address(ip).packed if not isinstance(ip, bytes) else ip[:n]


class LBMaps:
    """The four service/revNAT maps of one node (lbmap/ipv4.go:27-76)."""

    def __init__(self, max_entries=MaxEntries, prefix=""):
        self.s4, _ = bpf.OpenOrCreateMap(bpf.MapPath(prefix + "cilium_lb4_services"), bpf.BPF_MAP_TYPE_HASH,
                                         S4K.size, S4V.size, max_entries, 0)
        self.r4, _ = bpf.OpenOrCreateMap(bpf.MapPath(prefix + "cilium_lb4_reverse_nat"), bpf.BPF_MAP_TYPE_HASH,
                                         2, R4V.size, max_entries, 0)
        self.s6, _ = bpf.OpenOrCreateMap(bpf.MapPath(prefix + "cilium_lb6_services"), bpf.BPF_MAP_TYPE_HASH,
                                         S6K.size, S6V.size, max_entries, 0)
        self.r6, _ = bpf.OpenOrCreateMap(bpf.MapPath(prefix + "cilium_lb6_reverse_nat"), bpf.BPF_MAP_TYPE_HASH,
                                         2, R6V.size, max_entries, 0)

    # ---- host-order constructors + ToNetwork, as in the Go code ----
    @staticmethod
    def service4_key(ip, port, slave):
        return S4K.pack(_a(ip, 4), socket.htons(port), slave)

    @staticmethod
    def service4_value(count, target, port, revnat, weight=0):
        return S4V.pack(_a(target, 4), socket.htons(port), count, socket.htons(revnat), socket.htons(weight))

    @staticmethod
    def service6_key(ip, port, slave):
        return S6K.pack(_a(ip, 16), socket.htons(port), slave)

    @staticmethod
    def service6_value(count, target, port, revnat, weight=0):
        return S6V.pack(_a(target, 16), socket.htons(port), count, socket.htons(revnat), socket.htons(weight))

    def UpdateService(self, key, value, v6=False):
        bpf.UpdateElement(self.s6 if v6 else self.s4, key, value, 0)

    def UpdateRevNat(self, revnat_id, ip, port, v6=False):
        if revnat_id == 0:
            raise ValueError("invalid RevNat ID (0)")
        k = struct.pack("<H", socket.htons(revnat_id))
        v = R6V.pack(_a(ip, 16), socket.htons(port)) if v6 else R4V.pack(_a(ip, 4), socket.htons(port))
        bpf.UpdateElement(self.r6 if v6 else self.r4, k, v, 0)

    def AddSVC2BPFMap(self, fe_ip, fe_port, backends, add_revnat, revnat_id, v6=False):
        """lbmap.AddSVC2BPFMap (lbmap.go:320-371): backends as slaves 1..N,
        then revNAT, then the master slot 0 with count = N.
        backends: list of (target_ip, port, weight)."""
        keyf = self.service6_key if v6 else self.service4_key
        valf = self.service6_value if v6 else self.service4_value
        nnz = 0
        for i, (ip, port, weight) in enumerate(backends, start=1):
            if revnat_id == 0:
                raise ValueError("invalid RevNat ID (0) in the Service Value")
            nnz += 1 if weight else 0
            self.UpdateService(keyf(fe_ip, fe_port, i), valf(0, ip, port, revnat_id, weight), v6)
        if add_revnat:
            self.UpdateRevNat(revnat_id, fe_ip, fe_port, v6)
        zero = "::" if v6 else "0.0.0.0"
        self.UpdateService(keyf(fe_ip, fe_port, 0), valf(len(backends), zero, 0, 0, nnz), v6)
