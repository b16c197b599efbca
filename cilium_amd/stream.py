"""Steady-state packet stream for BASELINE config 2, generated on the GPU.

Benchmark input only (not part of the classifier).  Flows start at a fixed
rate; every flow has 4 packets sent in 4 consecutive steps (SYN/first,
ACK, ACK, FIN-or-RST; UDP and ICMP-echo flows likewise), so a step mixes
new, established and closing flows.  5% of flows are replies to
connections the endpoint opened (their egress CT entries are pre-inserted
through the map API), 1% of those end with an ICMP DEST_UNREACH that hits
the related entry; 0.5% unknown-protocol and 0.5% truncated packets; 1% of
packets carry TC_INDEX_F_SKIP_PROXY.

Sharding (multi-GPU): a rank owns the address pairs whose unordered-pair
hash maps to it (RSS-style); its flows only use those pairs, so each GPU's
CT partition sees every packet of its flow groups.

Columns are emitted exactly as gf_parse_frames would produce them from the
corresponding frames (see to_frames(), used for the CPU-baseline sample).
"""
import numpy as np

from . import synth

TCP, UDP, ICMP = 6, 17, 1


def _bswap16(x):
    return ((x & 0xff) << 8) | ((x >> 8) & 0xff)


def _bswap32(x):
    return ((x & 0xff) << 24) | ((x & 0xff00) << 8) | ((x >> 8) & 0xff00) | ((x >> 24) & 0xff)


def _h(torch, x, k):
    """64-bit mix of int64 tensor x with salt k (splitmix-style, wraps mod 2^64)."""
    x = x * -7046029254386353131 + k               # 0x9E3779B97F4A7C15 as signed
    x = (x ^ (x >> 30)) * -4658895280553007687     # 0xbf58476d1ce4e5b9 as signed
    x = (x ^ (x >> 27)) * -7723592293110705685     # 0x94d049bb133111eb
    return (x ^ (x >> 31)) & 0x7FFFFFFFFFFFFFFF


def pair_rank(raddr, ep_ip, world):
    a, b = np.minimum(raddr, ep_ip).astype(np.uint64), np.maximum(raddr, ep_ip).astype(np.uint64)
    return (synth.mix32((b << np.uint64(32)) | a) % np.uint32(world)).astype(np.int64)


class Stream:
    def __init__(self, pairs, rank=0, world=1, flows_per_step=4 << 20, device="cuda", seed=0xC1D40002,
                 reply_frac=0.05, related_frac=0.20, unk_frac=0.005, trunc_frac=0.005, skip_proxy_frac=0.01,
                 vip_ip=None, vip_frac=0.3):
        import torch
        self.torch = torch
        self.device = device
        self.F = int(flows_per_step)
        self.seed = seed + 7919 * rank
        own = np.nonzero(pair_rank(pairs["raddr"], pairs["ep_ip"][pairs["pe"]], world) == rank)[0]
        self.own = own
        T = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).to(device)
        pe = pairs["pe"][own]
        self.p_saddr = T(_bswap32(pairs["raddr"][own].astype(np.int64)), np.int64)
        self.p_daddr = T(_bswap32(pairs["ep_ip"][pe].astype(np.int64)), np.int64)
        self.p_id = T(pairs["pid"][own], np.int64)
        self.p_ifx = T(pairs["ifidx"][pe], np.int64)
        self.p_lxc = T(pairs["lxc_id"][pe], np.int64)
        self.p_port1 = T(pairs["port1"][own], np.int64)
        self.p_port2 = T(pairs["port2"][own], np.int64)
        self.np_ = len(own)
        # config 4: pairs whose flows address the endpoint's service VIP (bpf_lb translates it back)
        self.p_vip = None
        if vip_ip is not None:
            self.p_vip = T(_bswap32(np.asarray(vip_ip)[pe].astype(np.int64)), np.int64)
            self.p_usevip = T((synth.mix32(own.astype(np.uint64) * np.uint64(2654435761)) % 1000) < int(vip_frac * 1000),
                              np.bool_)
        self.fr = (int(reply_frac * 1000), int(related_frac * 1000), int(unk_frac * 10000), int(trunc_frac * 10000),
                   int(skip_proxy_frac * 1000))

    # ---- flow attributes --------------------------------------------------
    def _flows(self, f):
        torch = self.torch
        s = self.seed
        p = _h(torch, f, s + 1) % self.np_
        u = _h(torch, f, s + 2) % 1000
        proto = torch.where(u < 700, TCP, torch.where(u < 950, UDP, ICMP))
        sport = 32768 + _h(torch, f, s + 3) % 28232
        dport = torch.where(_h(torch, f, s + 4) % 10 < 8, self.p_port1[p], self.p_port2[p])
        reply = (_h(torch, f, s + 5) % 1000) < self.fr[0]
        related = reply & ((_h(torch, f, s + 6) % 1000) < self.fr[1])
        rst = (_h(torch, f, s + 7) % 10) < 2
        return p, proto, sport, dport, reply, related, rst

    def reply_ct_entries(self, n_steps):
        """Egress-created CT entries (tuple + ICMP related) for every reply flow
        of steps [0, n_steps): keys/values in ipv4_ct_tuple / ct_entry layout."""
        torch = self.torch
        f = torch.arange(0, n_steps * self.F, device=self.device, dtype=torch.int64)
        p, proto, sport, dport, reply, related, rst = self._flows(f)
        m = reply & (proto != ICMP)
        p, proto, sport, dport = p[m], proto[m], sport[m], dport[m]
        E, R = self.p_daddr[p].cpu().numpy(), self.p_saddr[p].cpu().numpy()
        E, R = _bswap32(E), _bswap32(R)                      # host order for synth helpers
        sp, dp, pr = sport.cpu().numpy(), dport.cpu().numpy(), proto.cpu().numpy()
        n = len(E)
        k = synth.ct4_keys(E, R, synth.raw16(sp), synth.raw16(dp), pr, np.zeros(n))
        rk = synth.ct4_keys(E, R, np.zeros(n), np.zeros(n), np.full(n, ICMP), np.full(n, 2))
        v = synth.ct_vals(n, 100_000 + 43200, 16, 0, 0, tx=(1, 100))
        return synth.dedup(np.concatenate([k, rk]), np.concatenate([v, v]))

    # ---- one step -----------------------------------------------------------
    def step(self, s):
        """Packets of step s as device columns (dict of tensors) + the pair index per packet."""
        torch = self.torch
        dev = self.device
        fs, js = [], []
        for j in range(4):
            st = s - j
            if st < 0:
                continue
            fs.append(torch.arange(st * self.F, (st + 1) * self.F, device=dev, dtype=torch.int64))
            js.append(torch.full((self.F,), j, device=dev, dtype=torch.int64))
        f = torch.cat(fs)
        j = torch.cat(js)
        g = torch.Generator(device=dev)
        g.manual_seed(self.seed * 1000003 + s)
        perm = torch.randperm(len(f), device=dev, generator=g)
        f, j = f[perm], j[perm]
        p, proto, sport, dport, reply, related, rst = self._flows(f)
        last = j == 3
        icmp_t = torch.where(related & last, 3, 8)
        proto = torch.where(related & last, ICMP, proto)
        flags = torch.where(j == 0, torch.where(reply, 0x10, 0x02),
                            torch.where(last & ~reply, torch.where(rst, 0x04, 0x11), 0x10))
        n = len(f)
        ph = _h(torch, f * 4 + j, self.seed + 11)
        unk = (ph % 10000) < self.fr[2]
        trunc = ((ph // 10000) % 10000) < self.fr[3]
        proto = torch.where(unk, 47, proto)
        l4h = torch.where(proto == TCP, 20, torch.where(proto == UDP, 8, torch.where(proto == ICMP, 8, 0)))
        length = 34 + l4h + (ph // 100000000) % 1400
        length = torch.where(trunc, 14 + (ph >> 40) % 36, length)
        is_tu = (proto == TCP) | (proto == UDP)
        l4w0 = torch.where(is_tu, _bswap16(sport) | (_bswap16(dport) << 16), torch.where(proto == ICMP, icmp_t, 0))
        l4w3 = torch.where(proto == TCP, 0x50 | (flags << 8), 0)
        # columns beyond len are 0-filled by the parser
        l4w0 = torch.where(length >= 34 + 4, l4w0, torch.where(length >= 35, l4w0 & ((1 << (8 * (length - 34).clamp(0, 4))) - 1), 0))
        l4w3 = torch.where(length >= 48, l4w3, torch.where(length == 47, l4w3 & 0xff, 0))
        hdr_ok = length >= 34
        daddr = self.p_daddr[p]
        if self.p_vip is not None:
            daddr = torch.where(self.p_usevip[p] & is_tu, self.p_vip[p], daddr)
        i32 = lambda x: x.to(torch.int64).where(x < (1 << 31), x - (1 << 32)).to(torch.int32)
        cols = {
            "len": length.to(torch.int32),
            "ethertype": torch.where(length >= 14, 0x0800, 0).to(torch.int16),
            "saddr4": i32(torch.where(hdr_ok, self.p_saddr[p], 0)),
            "daddr4": i32(torch.where(hdr_ok, daddr, 0)),
            "proto": torch.where(hdr_ok, proto, 0).to(torch.uint8),
            "l4_off": torch.where(hdr_ok, 34, 0).to(torch.int16),
            "l4w0": i32(torch.where(hdr_ok, l4w0, 0)),
            "l4w3": torch.where(hdr_ok, l4w3, 0).to(torch.int32).to(torch.int16),
            "src_identity": self.p_id[p].to(torch.int32),
            "ifindex": self.p_ifx[p].to(torch.int32),
            "lxc_id": self.p_lxc[p].to(torch.int16),
            "tc_index": ((ph >> 20) % 1000 < self.fr[4]).to(torch.uint8),
        }
        return cols, p, n


def to_frames(cols_np, stride=64):
    """Raw Ethernet/IPv4 frames whose parse yields exactly these columns."""
    n = len(cols_np["len"])
    lens = cols_np["len"].astype(np.uint32)
    f = np.zeros((n, stride), np.uint8)
    f[:, 12], f[:, 13] = 0x08, 0x00
    f[:, 14] = 0x45
    f[:, 23] = cols_np["proto"]
    f[:, 26:30] = cols_np["saddr4"].astype(np.uint32).view(np.uint8).reshape(n, 4)
    f[:, 30:34] = cols_np["daddr4"].astype(np.uint32).view(np.uint8).reshape(n, 4)
    f[:, 34:38] = cols_np["l4w0"].astype(np.uint32).view(np.uint8).reshape(n, 4)
    f[:, 46:48] = cols_np["l4w3"].astype(np.uint16).view(np.uint8).reshape(n, 2)
    return f, lens


def device_frames(cols, stride=64, ttl=64):
    """Raw Ethernet/IPv4 frames on the device whose parse yields exactly these
    columns (torch twin of to_frames, TTL set): the input of the full pipeline."""
    import torch
    n = cols["len"].shape[0]
    f = torch.zeros((n, stride // 4), dtype=torch.int32, device=cols["len"].device)
    u = lambda t: t.to(torch.int64) & 0xFFFFFFFF
    i32 = lambda x: torch.where(x >= (1 << 31), x - (1 << 32), x).to(torch.int32)
    sa, da, w0 = u(cols["saddr4"]), u(cols["daddr4"]), u(cols["l4w0"])
    w3 = cols["l4w3"].to(torch.int64) & 0xFFFF
    pr = cols["proto"].to(torch.int64)
    f[:, 3] = 0x00450008                                           # ethertype 0x0800, ver/IHL 0x45
    f[:, 5] = i32((ttl << 16) | (pr << 24))                        # TTL, protocol
    f[:, 6] = i32((sa & 0xFFFF) << 16)                             # saddr bytes 26..27
    f[:, 7] = i32((sa >> 16) | ((da & 0xFFFF) << 16))
    f[:, 8] = i32((da >> 16) | ((w0 & 0xFFFF) << 16))
    f[:, 9] = i32(w0 >> 16)
    f[:, 11] = i32(w3 << 16)                                       # TCP flags word (bytes 46..47)
    return f.view(torch.uint8).reshape(n, stride), cols["len"]


class Stream6(Stream):
    """Config 5: the same flow model over IPv6 (remote 2001:db8::<v4 remote>,
    endpoints f00d::<v4 endpoint>; ICMP flows are ICMPv6 echo / DEST_UNREACH),
    no pre-inserted reply entries."""

    def __init__(self, pairs, **kw):
        kw.setdefault("reply_frac", 0.0)
        super().__init__(pairs, **kw)

    def step(self, s):
        torch = self.torch
        cols, p, n = super().step(s)
        length = cols["len"].to(torch.int64) + 20                     # 40-B header instead of 20
        proto = cols["proto"].to(torch.int64)
        w0 = cols["l4w0"].to(torch.int64) & 0xFFFFFFFF
        icmp = proto == ICMP
        # ICMP echo (8) -> ICMPv6 echo request (128), DEST_UNREACH (3) -> ICMPv6 DEST_UNREACH (1)
        w0 = torch.where(icmp, torch.where((w0 & 0xff) == 3, 1, 128), w0)
        proto = torch.where(icmp, 58, proto)
        hdr_ok = length >= 54
        avail = (length - 54).clamp(0, 4)                             # the parser zero-fills past len
        w0 = torch.where(hdr_ok, w0 & ((1 << (8 * avail)) - 1), 0)
        w3 = cols["l4w3"].to(torch.int64) & 0xFFFF
        w3 = torch.where(length >= 68, w3, torch.where(length == 67, w3 & 0xff, 0))
        s6 = torch.zeros((n, 4), dtype=torch.int32, device=self.device)
        d6 = torch.zeros((n, 4), dtype=torch.int32, device=self.device)
        s6[:, 0] = 0xb80d0120 - (1 << 32)                            # 2001:db8::
        s6[:, 3] = self.p_saddr[p].to(torch.int64).where(self.p_saddr[p] < (1 << 31), self.p_saddr[p] - (1 << 32)).to(torch.int32)
        d6[:, 0] = 0x00000df0                                        # f00d::
        d6[:, 3] = self.p_daddr[p].to(torch.int64).where(self.p_daddr[p] < (1 << 31), self.p_daddr[p] - (1 << 32)).to(torch.int32)
        z = lambda t: torch.where(hdr_ok[:, None], t, 0)
        i32 = lambda x: torch.where(x >= (1 << 31), x - (1 << 32), x).to(torch.int32)
        cols.update({
            "len": length.to(torch.int32),
            "ethertype": torch.where(length >= 14, 0x86DD - (1 << 16), 0).to(torch.int16),
            "saddr4": torch.zeros(n, dtype=torch.int32, device=self.device),
            "daddr4": torch.zeros(n, dtype=torch.int32, device=self.device),
            "proto": torch.where(hdr_ok, proto, 0).to(torch.uint8),
            "l4_off": torch.where(hdr_ok, 54, 0).to(torch.int16),
            "l4w0": i32(w0),
            "l4w3": torch.where(w3 >= (1 << 15), w3 - (1 << 16), w3).to(torch.int16),
            "saddr6": z(s6).view(torch.uint8).reshape(n, 16),
            "daddr6": z(d6).view(torch.uint8).reshape(n, 16),
        })
        return cols, p, n


def to_frames6(cols_np, stride=96):
    """Raw Ethernet/IPv6 frames whose parse yields exactly these Stream6 columns."""
    n = len(cols_np["len"])
    lens = cols_np["len"].astype(np.uint32)
    f = np.zeros((n, stride), np.uint8)
    f[:, 12], f[:, 13] = 0x86, 0xDD
    f[:, 14] = 0x60
    f[:, 20] = cols_np["proto"]
    f[:, 21] = 64
    f[:, 22:38] = cols_np["saddr6"]
    f[:, 38:54] = cols_np["daddr6"]
    f[:, 54:58] = cols_np["l4w0"].astype(np.uint32).view(np.uint8).reshape(n, 4)
    f[:, 66:68] = cols_np["l4w3"].astype(np.uint16).view(np.uint8).reshape(n, 2)
    return f, lens


class Stream6Frames(Stream):
    """Config 5: the flow model over IPv6 raw frames (80-B snaps) for the full
    pipeline.  A pair's remote end is a cluster source (ROUTER_IP's /64, its
    identity in the flow label) or, for the CIDR class, a NAT64 world source;
    the endpoint end is its IPv6 address.  5% of flows answer connections the
    endpoint opened (their egress CT entries are in the pre-fill)."""

    def __init__(self, pairs, meta, **kw):
        super().__init__(pairs, **kw)
        import torch
        own = self.own
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)
        self.src6 = T(meta["src6"][own])
        self.dst6 = T(meta["dst6"][own])
        world = pairs["cls"][own] == 2
        self.flabel = T(np.where(world, 0, pairs["pid"][own]).astype(np.int64))
        self._s6, self._d6 = meta["src6"][own], meta["dst6"][own]

    def pair_addrs6(self):
        return self._s6, self._d6

    def reply_ct6_entries(self, n_steps):
        """Egress-created CT6 entries (tuple + ICMPv6 related) of every reply flow
        of steps [0, n_steps), in ipv6_ct_tuple / ct_entry layout."""
        torch = self.torch
        f = torch.arange(0, n_steps * self.F, device=self.device, dtype=torch.int64)
        p, proto, sport, dport, reply, related, rst = self._flows(f)
        m = reply & (proto != ICMP)
        p, proto, sport, dport = p[m].cpu().numpy(), proto[m].cpu().numpy(), sport[m].cpu().numpy(), dport[m].cpu().numpy()
        E, R = self._d6[p], self._s6[p]
        n = len(p)
        k = synth.ct6_keys(E, R, synth.raw16(sport), synth.raw16(dport), proto, np.zeros(n))
        rk = synth.ct6_keys(E, R, np.zeros(n), np.zeros(n), np.full(n, 58), np.full(n, 2))
        v = synth.ct_vals(n, 100_000 + 43200, 16, 0, 0, tx=(1, 100))
        return synth.dedup(np.concatenate([k, rk]), np.concatenate([v, v]))

    def step(self, s):
        """Frames of step s: (frames uint8[n, 80], len int32[n], pair index)."""
        torch = self.torch
        cols, p, n = Stream.step(self, s)
        length = cols["len"].to(torch.int64) + 20                     # 40-B header instead of 20
        proto = cols["proto"].to(torch.int64)
        w0 = cols["l4w0"].to(torch.int64) & 0xFFFFFFFF
        icmp = proto == ICMP
        # ICMP echo (8) -> ICMPv6 echo request (128), DEST_UNREACH (3) -> ICMPv6 DEST_UNREACH (1)
        w0 = torch.where(icmp, torch.where((w0 & 0xff) == 3, 1, 128), w0)
        proto = torch.where(icmp, 58, proto)
        w3 = cols["l4w3"].to(torch.int64) & 0xFFFF
        fl = self.flabel[p]
        f = torch.zeros((n, 80), dtype=torch.uint8, device=self.device)
        f[:, 12], f[:, 13] = 0x86, 0xDD
        f[:, 14] = 0x60
        f[:, 15] = ((fl >> 16) & 0xF).to(torch.uint8)
        f[:, 16] = ((fl >> 8) & 0xFF).to(torch.uint8)
        f[:, 17] = (fl & 0xFF).to(torch.uint8)
        pl = (length - 54).clamp(0, 0xFFFF)
        f[:, 18] = (pl >> 8).to(torch.uint8)
        f[:, 19] = (pl & 0xFF).to(torch.uint8)
        f[:, 20] = proto.to(torch.uint8)
        f[:, 21] = 64
        f[:, 22:38] = self.src6[p]
        f[:, 38:54] = self.dst6[p]
        for b in range(4):
            f[:, 54 + b] = ((w0 >> (8 * b)) & 0xFF).to(torch.uint8)
        f[:, 66] = (w3 & 0xFF).to(torch.uint8)
        f[:, 67] = (w3 >> 8).to(torch.uint8)
        return f, length.to(torch.int32), p
