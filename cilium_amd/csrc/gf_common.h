// gf_common.h — table layouts shared by the host shadow (gf_maps.cpp) and the
// HIP kernels (gf_kernels.hip) of libgpuflow.
//
// Exact-match hash maps (kernel BPF_MAP_TYPE_HASH / LRU_HASH semantics, see
// DESIGN.md) use open addressing with linear probing over fixed-size slots:
//
//   inline layout (slot <= 128 B, never straddles a 128-B L2 line):
//     [ key (ksz B) | state (1 B) | pad | value (vsz B) at voff | pad ]
//   split layout (key+value > 128 B, e.g. endpoint_info 112 B):
//     slots: [ key | state | pad ]  (pow2 stride)   vals: vsz B per slot
//   hot-split layout (CT maps, value codec GF_VCODEC_CT): the first 16 value
//     bytes (what an ingress hit reads and writes) stay in the slot, the other
//     32 go to vals, so a CT4 slot is 32 B — one memory sector — and a probe
//     step of 2 slots is one 64-B request:
//     slots: [ key | state | pad | hot 16 B at voff ]   vals: 32 B per slot
//   policy layout (policy maps, codec GF_VCODEC_POL): 16-B slots
//     [ key 8 | state | pad | proxy_port 2 at voff 10 | pad 4 ], so one 64-B
//     request reads the 4 slots an identity's L3/L4 keys cluster in;
//     vals: 24 B per slot (packets, bytes, the reference's pad bytes)
//
// state: 0 empty, 1 full, 2 deleted (tombstone), 3 busy (device insert in
// flight), 4 free (a slot the LRU eviction pass emptied between two classify
// calls, with its key bytes zeroed).  Probes walk past tombstones and free slots
// alike and end at an EMPTY one.  Device inserts claim EMPTY and FREE slots, never
// a tombstone (a key deleted inside the running launch may still be re-probed by
// its own lane); tombstones turn FREE or EMPTY in the eviction pass and the GC
// sweep, or are reused by host-side rebuilds (the CT concurrency note in DESIGN.md).
//
// The hash is a murmur3-style mix over the key as little-endian u32 words
// (zero-padded), identical on host and device.
//
// LPM tries (kernel BPF_MAP_TYPE_LPM_TRIE) are only ever queried by the
// datapath for membership ("is there a stored prefix covering addr"):
// bpf_xdp.c:112 and maps.h:129,139 test the lookup result against NULL.  The
// device form is therefore a coverage trie: a 2^R-entry root table followed by
// 8-bit-stride 128-B nodes of four 32-B groups {full word, child word, first
// child} (one group per 64 values of the byte; layout below, GF_TRIE_GROUP_BYTES).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define GF_HD __host__ __device__ __forceinline__
#else
#define GF_HD inline
#endif

enum : uint8_t { GF_SLOT_EMPTY = 0, GF_SLOT_FULL = 1, GF_SLOT_TOMB = 2, GF_SLOT_BUSY = 3, GF_SLOT_FREE = 4 };

struct gf_htab_desc {
    uint8_t  *slots;       // nslots * slot_size (hash mode: see gf_key_hash)
    uint8_t  *vals;        // split layout only (nslots * vsz), else nullptr
    uint32_t *count;       // device element counter (inserts / deletes)
    uint64_t  mask;        // nslots - 1 (0 with slots == nullptr => empty map)
    uint32_t  ksz, vsz, slot_size, voff;
    uint32_t  split, max_entries;
    uint32_t  vin;         // value bytes inline in the slot (at voff); the rest is in vals
    uint32_t  sstride;     // bytes per slot in vals (0: no side array)
};

struct gf_trie_desc {
    const uint32_t *root;  // 2^root_bits entries: 0 empty, ~0u full, else node+1
    const uint8_t  *nodes; // 128-B nodes, four 32-B groups (GF_TRIE_GROUP_BYTES)
    uint32_t root_bits;    // 8 or 16; 0 => map absent/empty (never matches)
    uint32_t addr_bytes;   // 4 or 16
    const uint64_t *rsum;  // root_bits 16: the root as two 2^16-bit maps (covered | has a node), else null
};
#define GF_TRIE_RSUM_BYTES 16384u
#define GF_TRIE_NODE_BYTES 128u
// A node: for each 64 values of its byte (group w = byte >> 6, at 32 * w) the
// full-coverage word, the child word (u64 LE each), then the node index of the
// group's first child (u32: the children are contiguous, in byte order), 12 B pad.
#define GF_TRIE_GROUP_BYTES 32u
// Compact IPv4 address sets (Map::addr_set): 2^bits u32 slots, 0 = empty (address 0
// is a flag of its own), linear probing from a Fibonacci hash of the raw address.
GF_HD uint32_t gf_aset_home(uint32_t a, uint32_t bits) { return (a * 0x9E3779B1u) >> (32 - bits); }
#define GF_TRIE_FULL 0xFFFFFFFFu

GF_HD uint32_t gf_rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

GF_HD uint32_t gf_hash_words(const uint32_t *w, int nw, uint32_t nbytes) {
    uint32_t h = 0x9747b28cu ^ nbytes;
    for (int i = 0; i < nw; i++) {
        uint32_t k = w[i] * 0xcc9e2d51u;
        k = gf_rotl32(k, 15);
        k *= 0x1b873593u;
        h ^= k;
        h = gf_rotl32(h, 13);
        h = h * 5u + 0xe6546b64u;
    }
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

// Hash modes: a map's role picks how its keys are hashed (host and device agree).
//  PLAIN  : all key words.
//  CT     : the canonical tuple (unordered addresses, unordered ports, flags
//           without TUPLE_F_IN), so a tuple and its reverse share a home line —
//           ct_lookup's reverse-then-forward probe touches one line.
//  POLICY : identity only for identity != 0, so an identity's L3 and L4 entries
//           share a home line (the L4 miss -> L3 hit sequence of
//           __policy_can_access touches one line); identity 0 (L4 wildcard)
//           hashes the full key.
enum { GF_HASH_PLAIN = 0, GF_HASH_CT = 1, GF_HASH_POLICY = 2 };

GF_HD uint32_t gf_key_hash(const uint32_t *w, uint32_t ksz, uint32_t mode) {
    if (mode == GF_HASH_CT && ksz == 14) {
        uint32_t a = w[0], b = w[1];
        uint32_t p0 = w[2] & 0xffffu, p1 = w[2] >> 16;
        uint32_t c[4] = {a < b ? a : b, a < b ? b : a,
                         (p0 < p1 ? p0 : p1) | ((p0 < p1 ? p1 : p0) << 16),
                         (w[3] & 0xffu) | (((w[3] >> 8) & 0xfeu) << 8)};
        return gf_hash_words(c, 4, 14);
    }
    if (mode == GF_HASH_CT && ksz == 40) {
        // less: the first address is the smaller (word-wise compare); selects per
        // word, not a pointer into w (which would put w in scratch on the device)
        const bool less = w[0] != w[4] ? w[0] < w[4] : w[1] != w[5] ? w[1] < w[5]
                        : w[2] != w[6] ? w[2] < w[6] : w[3] < w[7];
        uint32_t p0 = w[8] & 0xffffu, p1 = w[8] >> 16;
        uint32_t c[10] = {less ? w[0] : w[4], less ? w[1] : w[5], less ? w[2] : w[6], less ? w[3] : w[7],
                          less ? w[4] : w[0], less ? w[5] : w[1], less ? w[6] : w[2], less ? w[7] : w[3],
                          (p0 < p1 ? p0 : p1) | ((p0 < p1 ? p1 : p0) << 16),
                          (w[9] & 0xffu) | (((w[9] >> 8) & 0xfeu) << 8)};
        return gf_hash_words(c, 10, 40);
    }
    if (mode == GF_HASH_POLICY && ksz == 8 && w[0] != 0) return gf_hash_words(w, 1, 4);
    return gf_hash_words(w, (int)((ksz + 3) / 4), ksz);
}

// First slot probed: the first slot of the home 128-B line (lines hold
// 128/slot_size slots), then linear.
GF_HD uint64_t gf_home_slot(uint32_t h, uint64_t mask, uint32_t slot_size) {
    uint64_t spl = slot_size >= 128 ? 1 : 128 / slot_size;
    return ((uint64_t)h & mask) & ~(spl - 1);
}

// Value codecs: how a map's value bytes are laid out in its slots (host shadow
// and HBM replica alike).  The ABI always sees the reference layout.
//  IDENT : the reference struct as is.
//  CT    : struct ct_entry (bpf/lib/common.h:359-374) reordered so that what an
//          ingress hit reads and writes sits in the 16 B right after the key,
//          i.e. in the key's own 32-B sector:
//            +0 lifetime  +4 flags u16 | rev_nat_index u16  +8 rx_packets lo32
//            +12 rx_bytes lo32  +16 rx_packets hi32  +20 rx_bytes hi32
//            +24 tx_packets  +32 tx_bytes  +40 unused, pad  +44 src_sec_id
//          (reference offsets: rx_packets 0, rx_bytes 8, tx_packets 16,
//          tx_bytes 24, lifetime 32, flags 36, rev_nat_index 38, 40.., 44).
//  POL   : struct policy_entry (common.h:192-197: proxy_port, pad[3], packets,
//          bytes) reordered as proxy_port | packets | bytes | pad: proxy_port
//          stays in a 16-B slot with the key, the counters start the side
//          array entry 8-aligned for the device's 64-bit atomics.
enum { GF_VCODEC_IDENT = 0, GF_VCODEC_CT = 1, GF_VCODEC_POL = 2 };
#define GF_POL_VSZ 24u
GF_HD void gf_pol_encode(const uint8_t *ext, uint8_t *in) {
    __builtin_memcpy(in, ext, 2);
    __builtin_memcpy(in + 2, ext + 8, 16);
    __builtin_memcpy(in + 18, ext + 2, 6);
}
GF_HD void gf_pol_decode(const uint8_t *in, uint8_t *ext) {
    __builtin_memcpy(ext, in, 2);
    __builtin_memcpy(ext + 8, in + 2, 16);
    __builtin_memcpy(ext + 2, in + 18, 6);
}
#define GF_CT_VSZ 48u
// CT maps (the datapath inserts into them) get a fixed slot array of a power of two
// >= factor x max_entries slots: 8 for ipv4_ct_tuple (a 1/8-loaded table: HBM is
// plentiful, and the hit path's probes stay in the home line as the table fills —
// DESIGN.md, round 5), 4 for ipv6_ct_tuple (64-B slots; the LRU hand walks twice
// the lines at 8, and config 5 evicts on most calls).
#ifndef GF_CT4_SLOT_FACTOR
#define GF_CT4_SLOT_FACTOR 8
#endif
#ifndef GF_CT6_SLOT_FACTOR
#define GF_CT6_SLOT_FACTOR 4
#endif
GF_HD uint32_t gf_ct_slot_factor(uint32_t ksz) { return ksz == 14 ? GF_CT4_SLOT_FACTOR : GF_CT6_SLOT_FACTOR; }
GF_HD void gf_ct_encode(const uint8_t *ext, uint8_t *in) {
    const int map[12] = {8, 9, 0, 2, 1, 3, 4, 5, 6, 7, 10, 11};   // internal word k <- reference word map[k]
    uint32_t w[12];
    for (int k = 0; k < 12; k++) { uint32_t v; __builtin_memcpy(&v, ext + 4 * map[k], 4); w[k] = v; }
    __builtin_memcpy(in, w, 48);
}
GF_HD void gf_ct_decode(const uint8_t *in, uint8_t *ext) {
    const int map[12] = {8, 9, 0, 2, 1, 3, 4, 5, 6, 7, 10, 11};
    uint32_t w[12];
    __builtin_memcpy(w, in, 48);
    for (int k = 0; k < 12; k++) __builtin_memcpy(ext + 4 * map[k], &w[k], 4);
}

// Layout rule (host decides, device reads from the descriptor).
GF_HD uint32_t gf_pow2ceil32(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}
GF_HD void gf_htab_layout(uint32_t ksz, uint32_t vsz, uint32_t *slot_size, uint32_t *voff,
                          uint32_t *split) {
    uint32_t hdr = ksz + 1;
    uint32_t align = vsz >= 8 ? 8u : (vsz >= 4 ? 4u : 1u);
    uint32_t vo = (hdr + align - 1) / align * align;
    uint32_t inl = gf_pow2ceil32(vo + vsz);
    if (inl < 16) inl = 16;
    if (inl <= 128) { *slot_size = inl; *voff = vo; *split = 0; return; }
    uint32_t ks = gf_pow2ceil32(hdr);
    if (ks < 16) ks = 16;
    *slot_size = ks; *voff = 0; *split = 1;
}

// Unordered-address-pair group hash (flow group of the CT ordering rule).
GF_HD uint32_t gf_pair_hash4(uint32_t a, uint32_t b) {
    uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
    uint32_t w[2] = {lo, hi};
    return gf_hash_words(w, 2, 8);
}
// Connection group hash (IPv4): the unordered pair of (address, port)
// endpoints plus the protocol, so a connection's two directions share it.
// Ports are the raw be16 values of the CT tuple (0 for portless protocols).
GF_HD uint32_t gf_conn_hash4(uint32_t a, uint32_t pa, uint32_t b, uint32_t pb, uint32_t nh) {
    const bool sw = a > b || (a == b && pa > pb);
    uint32_t w[4] = {sw ? b : a, sw ? a : b, sw ? (pb | (pa << 16)) : (pa | (pb << 16)), nh | 0x5a00u};
    return gf_hash_words(w, 4, 16);
}
GF_HD uint32_t gf_pair_hash6(const uint32_t *a, const uint32_t *b) {
    // lexicographic byte compare of the two 16-byte addresses
    int less = 0;
    for (int i = 0; i < 4; i++) {
        uint32_t x = a[i], y = b[i];
        if (x != y) {
            // compare as big-endian bytes
            uint32_t xb = ((x & 0xff) << 24) | ((x & 0xff00) << 8) | ((x >> 8) & 0xff00) | (x >> 24);
            uint32_t yb = ((y & 0xff) << 24) | ((y & 0xff00) << 8) | ((y >> 8) & 0xff00) | (y >> 24);
            less = xb < yb;
            break;
        }
    }
    const uint32_t *lo = less ? a : b, *hi = less ? b : a;
    uint32_t w[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return gf_hash_words(w, 8, 32);
}

// Packed per-packet record used by the ingress kernel after grouping
// (32 B, one dwordx4 x2 load).  cls: bits0-1 L3 class (0 other, 1 v4, 2 v6),
// bit 2 TC_INDEX_F_SKIP_PROXY, bit 3 the pipeline packet ended before the tail
// call, bits 4-6 the pipeline front's GF_PIPE_F_* flags (flags byte bits 5-7).
struct __attribute__((aligned(16))) gf_rec {
    uint32_t saddr, daddr, len, l4w0, src_identity, ifindex;
    uint16_t ep;           // cilium_policy slot of the packet's lxc_id: program index + 1, 0 = empty
    int16_t  l4_off;
    uint16_t l4w3;
    uint8_t  proto, cls;
};
static_assert(sizeof(gf_rec) == 32, "gf_rec must be 32 bytes");

// Device-side endpoint program (lxc) configuration.
#define GF_MAX_L4 64
struct gf_l4_allow_dev { uint16_t port, proxy; uint8_t nexthdr, pad[3]; };
struct gf_lxc_dev {
    uint32_t flags, lxc_id, seclabel, n_l4;
    gf_htab_desc policy, ct4, ct6, revnat4, revnat6;
    gf_trie_desc cidr4, cidr6;
    gf_l4_allow_dev l4[GF_MAX_L4];
    // the from-container section (bpf_lxc.c:427-658)
    uint32_t lxc_mac[2], node_mac[2];  // 6 B each, LE words (upper half of word 1 zero)
    uint32_t lxc_ipv4, n_portmap, n_l4e, pad;
    gf_htab_desc lb4, ipcache;
    gf_trie_desc cidr4e;
    uint32_t portmap[16];              // from | to << 16 (raw be16 each)
    gf_l4_allow_dev l4e[GF_MAX_L4];
    uint32_t lxc_ip6[4];               // LXC_IP (LE words)
    gf_htab_desc lb6;
    gf_trie_desc cidr6e;
};
