"""pkg/maps/lxcmap mirror (/root/reference/pkg/maps/lxcmap/lxcmap.go:100-200).

EndpointKey (pkg/bpf/endpoint.go:33-38): {u8 IP[16]; u8 Family; u8 Pad4; u16 Pad5}  20 B
EndpointInfo: {u32 IfIndex; u16 SecLabelID; u16 LxcID; u32 Flags; u32 pad; u64 MAC;
               u64 NodeMAC; u32 Pad[4]; PortMap[16] {u16 From; u16 To}}                112 B
"""
import ipaddress
import struct

from .. import bpf

MapName = "cilium_lxc"
MaxEntries = 65535
EndpointFlagHost = 1
KEY = struct.Struct("<16sBBH")
INFO = struct.Struct("<IHHIIQQ16s64s")


def endpoint_key(ip):
    a = ipaddress.ip_address(ip)
    raw = a.packed
    if a.version == 4:
        return KEY.pack(raw + b"\x00" * 12, 1, 0, 0)
    return KEY.pack(raw, 2, 0, 0)


def endpoint_info(ifindex=0, sec_label=0, lxc_id=0, flags=0, mac=0, node_mac=0, portmap=b""):
    return INFO.pack(ifindex, sec_label, lxc_id, flags, 0, mac, node_mac, b"\x00" * 16,
                     portmap.ljust(64, b"\x00"))


class LXCMap:
    def __init__(self, path=None, max_entries=MaxEntries):
        self.fd, _ = bpf.OpenOrCreateMap(path or bpf.MapPath(MapName), bpf.BPF_MAP_TYPE_HASH,
                                         KEY.size, INFO.size, max_entries, 0)

    def WriteEndpoint(self, ips, info):
        for ip in ips:
            bpf.UpdateElement(self.fd, endpoint_key(ip), info, 0)

    def AddHostEntry(self, ip):
        bpf.UpdateElement(self.fd, endpoint_key(ip), endpoint_info(flags=EndpointFlagHost), 0)

    def DeleteEntry(self, ip):
        bpf.DeleteElement(self.fd, endpoint_key(ip))
