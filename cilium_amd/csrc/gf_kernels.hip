// gf_kernels.hip — gfx950 kernels of libgpuflow and the program/classify C ABI.
//
//   k_parse     raw frames -> SoA header columns   (skb_load_bytes rules)
//   k_xdp       bpf/bpf_xdp.c:88-184               one packet per lane
//   k_lb        bpf/bpf_lb.c:58-212 + lib/lb.h      one packet per lane
//   k_ing_pack  columns -> 32-B records + flow-group key (unordered addr pair)
//   (rocPRIM stable radix sort of (group, index) + exclusive scan)
//   k_bucket_*  bucket-size histogram + count-descending bucket order
//   k_ing_level bpf/bpf_lxc.c:745-1024 handle_policy, level-synchronous: launch k
//               runs the k-th packet of every flow-group bucket (CT ordering rule)
//   k_ing_tail  the remaining ranks of the few deepest buckets, sequentially
#include "gf_internal.h"
#include "gf_device.h"
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_run_length_encode.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/discard_iterator.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <errno.h>
#include <stdlib.h>
#include <stdio.h>
#include <functional>
#include <unordered_set>
#include <chrono>
#include <algorithm>
#include <array>
#include <atomic>
#include <string.h>

using namespace gf;
using namespace gfd;

#define BLOCK 256
#ifndef GF_DIAG
#define GF_DIAG 0      // diagnostic ablations (tools/diag.sh); 0 in the product build
#endif
// Tuning knobs of the flow-group kernel (tools/variants.sh sweeps them).
#ifndef GF_KEY_BITS
#define GF_KEY_BITS 32      // bucket key: family bit + (GF_KEY_BITS-1) bits of the group hash
#endif
#define GF_KEY_FAM (1u << (GF_KEY_BITS - 1))
#define GF_KEY_HASH (GF_KEY_FAM - 1u)
// The key of every packet the handle_policy pass skips (a pipeline packet that
// ended before the tail call, an egress packet that was not delivered locally):
// they sort into one run, which the bucket schedule leaves out, so no lane reads
// their records.  Group keys never take this value (gf_key_live).
#define GF_KEY_SKIP GF_KEY_HASH
__device__ __forceinline__ uint32_t gf_key_live(uint32_t k) { return (k & GF_KEY_HASH) == GF_KEY_SKIP ? k - 1u : k; }
#ifndef GF_ING_MINW
#define GF_ING_MINW 4       // __launch_bounds__ min waves per SIMD (register budget)
#endif
#ifndef GF_ING_MINW6
#define GF_ING_MINW6 3      // IPv6 buckets: the lane state (RelCache<10>) keeps the block at 3 per CU by LDS
#endif
#ifndef GF_ING_BINS_WAVE
#define GF_ING_BINS_WAVE 0  // k_ing_groups: reason / action bins aggregated over the active lanes (no effect: 2.728 ms both)
#endif
#ifndef GF_PERM_VEC
#define GF_PERM_VEC 1       // k_ing_groups: the bucket's indices read four at a time (16-B loads; 2.625 -> 2.615 ms)
#endif
#ifndef GF_EG_MINW
#define GF_EG_MINW 3        // k_eg_groups: min waves per SIMD (4 spills: 1.65 vs 1.60 ms, egress leg)
#endif
#ifndef GF_CT_COOP
#define GF_CT_COOP 1        // CT4 home lines read by complete lane quads together (ProbeLine::load_quad)
#endif
#ifndef GF_EG_COOP
#define GF_EG_COOP 1        // k_eg_groups: the CT4 home line read by complete lane quads (load_quad)
#endif
#ifndef GF_FRONT_MINW
#define GF_FRONT_MINW 8     // k_pipe_front: __launch_bounds__ min waves per SIMD (64 VGPRs: 1.294 vs 1.410 ms, config 4)
#endif
#ifndef GF_EG_DYN
#define GF_EG_DYN 1         // k_eg_front: LDS rows sized by the snap stride (64-B snaps: half the LDS; 0.586 vs 0.622 ms)
#endif
#ifndef GF_EG_LEAN
#define GF_EG_LEAN 1        // egress: the deferred-entry sets sized by the logged count, empty-family and no-IPv6 blocks skipped
#endif
#define GF_RUN_ITEMS 4096u  // keys per tile of the run-start / single-bucket count-scan-write passes
// Buckets per lane per queue grab once a wave reaches the single-packet buckets
// (the lists are longest first, so from there on every bucket is one packet): one
// queue atomic per 64 x GF_GRAB_* buckets instead of per 64, and a lane runs several
// independent packets back to back.  Longer buckets keep one per lane per grab (a
// lane holding four long buckets would stretch the tail: config 2 4.8 vs 2.4 ms).
#ifndef GF_GRAB_ING
#define GF_GRAB_ING 4       // k_ing_groups
#endif
#ifndef GF_GRAB_EG
#define GF_GRAB_EG 2        // k_eg_groups
#endif
#ifndef GF_SINGLE_ORDER
#define GF_SINGLE_ORDER 1   // egress passes: single-packet buckets scheduled in packet-index order
#endif
#ifndef GF_REC_NT
#define GF_REC_NT 0         // k_ing_groups: packet records read with nontemporal loads
#endif
#ifndef GF_CT_COOP6
#define GF_CT_COOP6 1       // the same for CT6 (168 VGPRs: fits the 3 waves the LDS allows; 1.242 vs 1.252 ms)
#endif
#ifndef GF_MEMO4
#define GF_MEMO4 2          // policy decisions memoised per lane, IPv4 buckets
#endif
#ifndef GF_MEMO6
#define GF_MEMO6 2          // IPv6 buckets (1 fits 4 blocks' lane state in LDS, but the 128-VGPR
                            // budget that occupancy 4 then imposes spills: 1.93 vs 1.20 ms, config 5)
#endif

// ---------------------------------------------------------------- constants
enum {
    TC_OK = 0, TC_SHOT = 2, TC_REDIRECT = 7, XDP_DROP_ = 1, XDP_PASS_ = 2,
    D_POLICY = -133, D_INVALID = -134, D_CT_INVALID_HDR = -135, D_CT_UNKNOWN_PROTO = -137,
    D_UNKNOWN_L3 = -139, D_MISSED_TAIL_CALL = -140, D_WRITE_ERROR = -141, D_UNKNOWN_L4 = -142,
    D_CSUM_L4 = -154, D_CT_CREATE_FAILED = -155, D_NO_SERVICE = -158, D_POLICY_L4 = -159,
};
enum { CT_NEW = 0, CT_ESTABLISHED = 1, CT_REPLY = 2, CT_RELATED = 3 };
enum { ACT_UNSPEC = 0, ACT_CREATE = 1, ACT_CLOSE = 2 };
#define F_RX_CLOSING 1u
#define F_TX_CLOSING 2u
#define F_LB_LOOPBACK 8u
#define F_SEEN_NON_SYN 16u

// ---------------------------------------------------------------- stats
struct Stats {
    uint32_t *lds;
    __device__ void init() {
        for (int k = threadIdx.x; k < 272; k += blockDim.x) lds[k] = 0;
        __syncthreads();
    }
    __device__ void add(uint32_t bin) { atomicAdd(&lds[bin], 1u); }
    __device__ void add_n(uint32_t bin, uint32_t v) { if (v) atomicAdd(&lds[bin], v); }
    // one packet: reason/action bins + packets, wire bytes, algorithmic bytes
    __device__ void pkt(uint32_t reason, uint32_t action, uint32_t len, uint32_t ab) {
        add(reason); add(256 + action); add(268); add_n(269, len); add_n(270, ab);
    }
    // pkt() aggregated over the wave: one LDS atomic per distinct (reason,
    // action) pair and one per sum instead of five per lane.  Every lane of the
    // wave must call it (act = the lane counts a packet; ab is summed over every
    // lane, so a lane without a packet passes 0).
    __device__ void pkt_wave(bool act, uint32_t reason, uint32_t action, uint32_t len, uint32_t ab) {
        uint32_t n = act ? 1u : 0u, l = act ? len : 0u, a = ab;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            n += __shfl_xor(n, o); l += __shfl_xor(l, o); a += __shfl_xor(a, o);
        }
        const uint32_t lane = threadIdx.x & 63u, key = (reason & 0xffu) | (action << 8);
        uint64_t rem = __ballot(act);
        while (rem) {
            const uint32_t lead = (uint32_t)__ffsll((unsigned long long)rem) - 1u;
            const uint32_t k = __shfl(key, (int)lead);
            const uint64_t m = __ballot(act && key == k) & rem;
            if (lane == lead) {
                atomicAdd(&lds[k & 0xffu], (uint32_t)__popcll(m));
                atomicAdd(&lds[256 + (k >> 8)], (uint32_t)__popcll(m));
            }
            rem &= ~m;
        }
        if (lane == 0) { if (n) { atomicAdd(&lds[268], n); atomicAdd(&lds[269], l); } if (a) atomicAdd(&lds[270], a); }
    }
    // pkt_wave's (reason, action) bins alone: for grid-stride loops that keep the
    // packet count and the byte sums per lane and hand them to sums() once
    __device__ void bins_wave(bool act, uint32_t reason, uint32_t action) {
        const uint32_t lane = threadIdx.x & 63u, key = (reason & 0xffu) | (action << 8);
        uint64_t rem = __ballot(act);
        while (rem) {
            const uint32_t lead = (uint32_t)__ffsll((unsigned long long)rem) - 1u;
            const uint32_t k = __shfl(key, (int)lead);
            const uint64_t m = __ballot(act && key == k) & rem;
            if (lane == lead) {
                atomicAdd(&lds[k & 0xffu], (uint32_t)__popcll(m));
                atomicAdd(&lds[256 + (k >> 8)], (uint32_t)__popcll(m));
            }
            rem &= ~m;
        }
    }
    __device__ void sums(uint32_t n, uint32_t len, uint32_t ab) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) { n += __shfl_xor(n, o); len += __shfl_xor(len, o); ab += __shfl_xor(ab, o); }
        if ((threadIdx.x & 63u) == 0) { add_n(268, n); add_n(269, len); add_n(270, ab); }
    }
    // XDP verdict counts (reason 1 / XDP_DROP, reason 0 / XDP_PASS) and sums, summed
    // per lane over a whole grid-stride loop: one wave reduction (every lane calls it)
    __device__ void xdp_sums(uint32_t drop, uint32_t pass, uint32_t len, uint32_t ab) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            drop += __shfl_xor(drop, o); pass += __shfl_xor(pass, o);
            len += __shfl_xor(len, o); ab += __shfl_xor(ab, o);
        }
        if ((threadIdx.x & 63u) == 0) {
            add_n(1, drop); add_n(256 + 1, drop); add_n(0, pass); add_n(256 + 2, pass);
            add_n(268, drop + pass); add_n(269, len); add_n(270, ab);
        }
    }
    __device__ void flush(unsigned long long *g) {
        __syncthreads();
        for (int k = threadIdx.x; k < 272; k += blockDim.x)
            if (lds[k]) atomicAdd(&g[k], (unsigned long long)lds[k]);
    }
};

// ================================================================ parse
__device__ __forceinline__ uint32_t fbyte(const uint8_t *f, uint32_t cap, uint32_t off) {
    return off < cap ? f[off] : 0u;
}

// Header values of one frame, as the BPF programs hold them after their loads
// (the rules of gf_parse_frames; oracle.c o_parse_batch).
struct PktHdr {
    uint32_t et, sa, da, w0, w3, proto;
    int l4;
    uint32_t s6[4], d6[4];
};
__device__ __forceinline__ void parse_row(const uint8_t *f, uint32_t cap, uint32_t len, PktHdr &h) {
    h.et = len >= 14 ? ((fbyte(f, cap, 12) << 8) | fbyte(f, cap, 13)) : 0u;
    h.sa = h.da = h.w0 = h.w3 = h.proto = 0;
    h.l4 = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) h.s6[k] = h.d6[k] = 0;
    bool have = false;
    if (h.et == 0x0800 && len >= 34) {
        for (int k = 0; k < 4; k++) { h.sa |= fbyte(f, cap, 26 + k) << (8 * k); h.da |= fbyte(f, cap, 30 + k) << (8 * k); }
        h.proto = fbyte(f, cap, 23);
        h.l4 = 14 + (int)(fbyte(f, cap, 14) & 0xf) * 4;
        have = true;
    } else if (h.et == 0x86DD && len >= 54) {
        for (int k = 0; k < 16; k++) {
            h.s6[k >> 2] |= fbyte(f, cap, 22 + k) << (8 * (k & 3));
            h.d6[k >> 2] |= fbyte(f, cap, 38 + k) << (8 * (k & 3));
        }
        // ipv6_hdrlen, bpf/lib/ipv6.h:61-98 (AUTH length chosen by the NEXT header, as written)
        uint32_t nh = fbyte(f, cap, 20);
        int hl = 40, res = -156;
        for (int it = 0; it < 4; it++) {
            if (nh == 59) { res = -156; goto done; }
            if (nh == 44) { res = -157; goto done; }
            if (nh == 0 || nh == 43 || nh == 51 || nh == 60) {
                int off = 14 + hl;
                if (!skb_ok(off, 2, len)) { res = -134; goto done; }
                uint32_t onh = fbyte(f, cap, off), ohl = fbyte(f, cap, off + 1);
                nh = onh;
                if (nh == 51) hl += (int)(ohl + 2) << 2; else hl += (int)(ohl + 1) << 3;
                continue;
            }
            res = hl;
            h.proto = nh;
            goto done;
        }
        res = -156;
    done:
        if (res < 0) h.proto = fbyte(f, cap, 20);
        h.l4 = 14 + res;
        have = true;
    }
    if (have) {
        for (int k = 0; k < 4; k++) {
            int64_t off = (int64_t)h.l4 + k;
            if (off >= 0 && off < (int64_t)len) h.w0 |= fbyte(f, cap, (uint32_t)off) << (8 * k);
        }
        for (int k = 0; k < 2; k++) {
            int64_t off = (int64_t)h.l4 + 12 + k;
            if (off >= 0 && off < (int64_t)len) h.w3 |= fbyte(f, cap, (uint32_t)off) << (8 * k);
        }
    }
}

__global__ __launch_bounds__(BLOCK) void k_parse(gf_frames fr, gf_pkt_cols_out o) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < fr.n; i += gridDim.x * blockDim.x) {
        const uint8_t *f = fr.snap + (size_t)i * fr.snap_stride;
        uint32_t len = fr.len[i];
        uint32_t cap = fr.snap_stride < len ? fr.snap_stride : len;
        PktHdr h;
        parse_row(f, cap, len, h);
        o.ethertype[i] = (uint16_t)h.et; o.saddr4[i] = h.sa; o.daddr4[i] = h.da; o.proto[i] = (uint8_t)h.proto;
        o.l4_off[i] = (int16_t)h.l4; o.l4w0[i] = h.w0; o.l4w3[i] = (uint16_t)h.w3;
        if (o.saddr6) reinterpret_cast<uint4 *>(o.saddr6)[i] = make_uint4(h.s6[0], h.s6[1], h.s6[2], h.s6[3]);
        if (o.daddr6) reinterpret_cast<uint4 *>(o.daddr6)[i] = make_uint4(h.d6[0], h.d6[1], h.d6[2], h.d6[3]);
    }
}

// Header access for the per-packet programs: packet i of a column batch, or
// the values a lane parsed itself (the fused pipeline front).
struct ColA {
    const gf_pkt_cols &c;
    uint32_t i;
    __device__ __forceinline__ uint32_t saddr4() const { return c.saddr4[i]; }
    __device__ __forceinline__ uint32_t daddr4() const { return c.daddr4[i]; }
    __device__ __forceinline__ uint32_t proto() const { return c.proto[i]; }
    __device__ __forceinline__ int l4_off() const { return c.l4_off[i]; }
    __device__ __forceinline__ uint32_t l4w0() const { return c.l4w0[i]; }
    __device__ __forceinline__ uint32_t fhash() const { return c.flow_hash ? c.flow_hash[i] : 0u; }
    __device__ __forceinline__ bool has6() const { return c.saddr6 && c.daddr6; }
    __device__ __forceinline__ uint4 saddr6() const { return reinterpret_cast<const uint4 *>(c.saddr6)[i]; }
    __device__ __forceinline__ uint4 daddr6() const { return gload<uint4>(c.daddr6 + 16 * (size_t)i); }
};
struct PktHdrA {
    const PktHdr &h;
    uint32_t fh;
    __device__ __forceinline__ uint32_t saddr4() const { return h.sa; }
    __device__ __forceinline__ uint32_t daddr4() const { return h.da; }
    __device__ __forceinline__ uint32_t proto() const { return h.proto; }
    __device__ __forceinline__ int l4_off() const { return h.l4; }
    __device__ __forceinline__ uint32_t l4w0() const { return h.w0; }
    __device__ __forceinline__ uint32_t fhash() const { return fh; }
    __device__ __forceinline__ bool has6() const { return true; }
    __device__ __forceinline__ uint4 saddr6() const { return make_uint4(h.s6[0], h.s6[1], h.s6[2], h.s6[3]); }
    __device__ __forceinline__ uint4 daddr6() const { return make_uint4(h.d6[0], h.d6[1], h.d6[2], h.d6[3]); }
};

// The lane's frame copy.  Reads past the snap (or len) are 0, writes past the
// snap are dropped (the snap holds every header byte the programs touch).
struct Row {
    uint8_t *p;
    uint32_t cap;
    __device__ __forceinline__ uint32_t b(uint32_t off) const { return off < cap ? (uint32_t)p[off] : 0u; }
    __device__ __forceinline__ uint32_t r16(uint32_t off) const { return b(off) | (b(off + 1) << 8); }
    __device__ __forceinline__ uint32_t r32(uint32_t off) const { return r16(off) | (r16(off + 2) << 16); }
    __device__ __forceinline__ void w8(uint32_t off, uint32_t v) { if (off < cap) p[off] = (uint8_t)v; }
    __device__ __forceinline__ void w16(uint32_t off, uint32_t v) { w8(off, v & 0xffu); w8(off + 1, (v >> 8) & 0xffu); }
    __device__ __forceinline__ void w32(uint32_t off, uint32_t v) { w16(off, v & 0xffffu); w16(off + 2, v >> 16); }
};

// Checksum arithmetic of bpf_l3_csum_replace / bpf_l4_csum_replace /
// bpf_csum_diff (Linux net/core/filter.c over include/net/checksum.h; the skb is
// a received frame, not CHECKSUM_PARTIAL).  Operands are raw LE loads of the
// network-order bytes, as the programs pass them.
#define GF_F_PSEUDO_HDR (1u << 4)
#define GF_F_MANGLED_0 (1u << 5)
__device__ __forceinline__ uint32_t ck_add(uint32_t a, uint32_t b) { uint32_t r = a + b; return r + (r < b ? 1u : 0u); }
__device__ __forceinline__ uint32_t ck_fold(uint32_t x) {
    x = (x & 0xffffu) + (x >> 16);
    x = (x & 0xffffu) + (x >> 16);
    return ~x & 0xffffu;
}
__device__ __forceinline__ uint32_t ck16_add(uint32_t a, uint32_t b) {
    uint32_t r = (a + b) & 0xffffu;
    return (r + (r < b ? 1u : 0u)) & 0xffffu;
}
// bpf_l3_csum_replace: size 0 = by diff, 2 = csum_replace2, 4 = csum_replace4
__device__ int l3_csum(Row &w, uint32_t len, int32_t off, uint32_t from, uint32_t to, uint32_t size) {
    if (!l4csum_ok(off, len)) return -GF_EFAULT;
    uint32_t sum = w.r16((uint32_t)off);
    if (size == 0) sum = ck_fold(ck_add(to, ~sum));
    else if (size == 2) sum = ~ck16_add(ck16_add(~sum & 0xffffu, ~from & 0xffffu), to & 0xffffu) & 0xffffu;
    else sum = ck_fold(ck_add(ck_add(~sum, ~from), to));
    w.w16((uint32_t)off, sum);
    return 0;
}
// bpf_l4_csum_replace (inet_proto_csum_replace4 / _by_diff, BPF_F_MARK_MANGLED_0)
__device__ int l4_csum(Row &w, uint32_t len, int32_t off, uint32_t from, uint32_t to, uint32_t flags) {
    if (!l4csum_ok(off, len)) return -GF_EFAULT;
    uint32_t sum = w.r16((uint32_t)off);
    const bool mmzero = (flags & GF_F_MANGLED_0) != 0;
    if (mmzero && !sum) return 0;
    if ((flags & 0xfu) == 0) sum = ck_fold(ck_add(to, ~sum));
    else sum = ck_fold(ck_add(ck_add(~sum, ~from), to));
    if (mmzero && !sum) sum = 0xffffu;                  // CSUM_MANGLED_0
    w.w16((uint32_t)off, sum);
    return 0;
}

// ================================================================ XDP
struct XdpDev {
    gf_htab_desc h4, h6, lxc;
    gf_trie_desc l4, l6;
    uint32_t has_h4, has_h6;
    // optional: the /32 map's and cilium_lxc's IPv4 keys as compact address sets
    // (Map::addr_set) probed in place of their hash tables (IPv4 only)
    const uint32_t *h4set, *lxset;
    uint32_t h4bits, lxbits, h4zero, lxzero;
    // optional (GF_XDP_DIR24, Map::dir24): the v4 prefixes as DIR-24-8 tables, read
    // in place of the trie walk below a root-summary "has a node" bit
    const uint16_t *d24;
    const uint32_t *d8;
};
// DIR-24-8 coverage of an IPv4 source (raw network-order word): one 2-B read of
// tbl24, one 4-B read of the /24's group when it holds longer prefixes.
__device__ __forceinline__ bool dir24_cov(const uint16_t *t24, const uint32_t *t8, uint32_t sa) {
    const uint32_t i24 = ((sa & 0xffu) << 16) | (sa & 0xff00u) | ((sa >> 16) & 0xffu), b = sa >> 24;
    const uint32_t e = gload<uint16_t>(t24 + i24);
    if (e == 0xffffu) return true;
    return e && ((gload<uint32_t>(t8 + (e - 1u) * 8u + (b >> 5)) >> (b & 31u)) & 1u);
}
// The table slot of an address in an endpoint-key set (its second array), or -1.
__device__ __forceinline__ int64_t aset_slot(const uint32_t *t, uint32_t bits, uint32_t zero, uint32_t a) {
    if (!a) return (int64_t)zero - 1;
    const uint32_t m = (1u << bits) - 1u;
    for (uint32_t k = gf_aset_home(a, bits);; k = (k + 1) & m) {
        const uint32_t v = t[k];
        if (v == a) return (int64_t)t[(1u << bits) + k];
        if (!v) return -1;
    }
}
// Membership in a compact IPv4 address set (gf_aset_home; <= 1/2 load), in LDS
// (k_xdp_lds) or in HBM / L2.
__device__ __forceinline__ bool aset_has(const uint32_t *t, uint32_t bits, uint32_t zero, uint32_t a) {
    if (!a) return zero != 0;
    const uint32_t m = (1u << bits) - 1u;
    for (uint32_t k = gf_aset_home(a, bits);; k = (k + 1) & m) {
        const uint32_t v = t[k];
        if (v == a) return true;
        if (!v) return false;
    }
}

__device__ __forceinline__ bool lxc_has4(const gf_htab_desc &lxc, uint32_t daddr) {
    uint32_t kw[5] = {daddr, 0, 0, 0, 1u};          // endpoint_key {ip4, pad.., family=1}
    return ht_find<20>(lxc, kw, key_hash<20>(kw)) >= 0;
}
__device__ __forceinline__ bool lxc_has6(const gf_htab_desc &lxc, const uint32_t *d) {
    uint32_t kw[5] = {d[0], d[1], d[2], d[3], 2u};
    return ht_find<20>(lxc, kw, key_hash<20>(kw)) >= 0;
}

// xdp_start -> check_filters -> check_v4 / check_v6 (bpf/bpf_xdp.c:97-184) for
// packet i; ab accumulates the algorithmic bytes.  The three lookups (the LPM
// trie, the /32 or /128 hash, the cilium_lxc endpoint) have no side effects, so
// GF_XDP_PRE can load the hash probes' home lines before the trie walk (all in
// flight together; the verdict still combines them in the reference's order).
// Measured on config 1 (r2): 0.080 ms with both lines preloaded, 0.076 with the
// prefix hash only, 0.075 with none — k_xdp is bound by the request rate of its
// L2-resident tables, not by the latency of the chain, so the default issues
// each probe only when the reference would.
#define GF_XDP_U 2
#ifndef GF_XDP_PRE
#define GF_XDP_PRE 0      // home lines loaded before the trie walk: 0 none, 1 the prefix hash, 2 + cilium_lxc
#endif
template <class A>
__device__ __forceinline__ uint8_t xdp_verdict(const XdpDev &x, const A &a, uint32_t len, uint32_t et, uint32_t &ab) {
    if (len < 14) return XDP_DROP_;
    if (et == 0x0800) {
        if (len < 34) return XDP_DROP_;
        uint32_t sa = a.saddr4();
        const uint32_t kw[2] = {32u, sa};
        const uint32_t lk[5] = {a.daddr4(), 0, 0, 0, 1u};     // endpoint_key {ip4, pad.., family=1}
        ProbeLine<20, GF_XDP_U> ll;
        if (GF_XDP_PRE >= 2) ll.load(x.lxc, key_hash<20>(lk));
        ProbeLine<8, GF_XDP_U> hl;
        if (GF_XDP_PRE >= 1 && x.has_h4) hl.load(x.h4, key_hash<8>(kw));
        bool drop = false;
        ab += 10;
        if (x.has_h4) {
            ab += 9;
            bool cov;
            if (x.l4.rsum) {                            // the root summary: covered / has a node / neither
                const uint32_t idx = ((sa & 0xffu) << 8) | ((sa >> 8) & 0xffu);
                cov = (gload<uint64_t>(x.l4.rsum + (idx >> 6)) >> (idx & 63)) & 1ull;
                if (!cov && ((gload<uint64_t>(x.l4.rsum + 1024 + (idx >> 6)) >> (idx & 63)) & 1ull))
                    cov = x.d24 ? dir24_cov(x.d24, x.d8, sa)
                                : trie_nodes<1>(x.l4, AddrBytes<1>(&sa), gload<uint32_t>(x.l4.root + idx) - 1u);
            } else {
                cov = trie_lookup<1>(x.l4, &sa);
            }
            if (cov) drop = true;
            else {
                ab += 9;
                if (x.h4set) drop = aset_has(x.h4set, x.h4bits, x.h4zero, sa);
                else {
                    if (GF_XDP_PRE < 1) hl.load(x.h4, key_hash<8>(kw));
                    drop = probe2<8, GF_XDP_U, 0>(x.h4, kw, kw, hl, false).f >= 0;
                }
            }
        }
        if (drop) return XDP_DROP_;
        ab += 20;
        if (x.lxset) return aset_has(x.lxset, x.lxbits, x.lxzero, lk[0]) ? XDP_PASS_ : XDP_DROP_;
        if (GF_XDP_PRE < 2) ll.load(x.lxc, key_hash<20>(lk));
        return probe2<20, GF_XDP_U, 0>(x.lxc, lk, lk, ll, false).f >= 0 ? XDP_PASS_ : XDP_DROP_;
    }
    if (et == 0x86DD) {
        if (len < 54 || !a.has6()) return XDP_DROP_;
        uint4 s = a.saddr6();
        uint32_t sw[4] = {s.x, s.y, s.z, s.w};
        const uint32_t kw[5] = {128u, s.x, s.y, s.z, s.w};
        const uint4 d = a.daddr6();
        const uint32_t lk[5] = {d.x, d.y, d.z, d.w, 2u};
        ProbeLine<20, GF_XDP_U> ll;
        if (GF_XDP_PRE >= 2) ll.load(x.lxc, key_hash<20>(lk));
        ProbeLine<20, GF_XDP_U> hl;
        if (GF_XDP_PRE >= 1 && x.has_h6) hl.load(x.h6, key_hash<20>(kw));
        bool drop = false;
        ab += 34;
        if (x.has_h6) {
            ab += 21;
            if (trie_lookup<4>(x.l6, sw)) drop = true;
            else {
                ab += 21;
                if (GF_XDP_PRE < 1) hl.load(x.h6, key_hash<20>(kw));
                drop = probe2<20, GF_XDP_U, 0>(x.h6, kw, kw, hl, false).f >= 0;
            }
        }
        if (drop) return XDP_DROP_;
        ab += 20;
        if (GF_XDP_PRE < 2) ll.load(x.lxc, key_hash<20>(lk));
        return probe2<20, GF_XDP_U, 0>(x.lxc, lk, lk, ll, false).f >= 0 ? XDP_PASS_ : XDP_DROP_;
    }
    return XDP_PASS_;
}

__global__ __launch_bounds__(BLOCK) void k_xdp(gf_pkt_cols c, XdpDev x, uint8_t *verdict,
                                               unsigned long long *stats) {
    __shared__ uint32_t sl[272];
    Stats st{sl};
    if (stats) st.init();
    uint32_t n_drop = 0, n_pass = 0, s_len = 0, s_ab = 0;      // the lane's counter sums (Stats::xdp_sums)
    for (uint32_t b = blockIdx.x * blockDim.x; b < c.n; b += gridDim.x * blockDim.x) {
        const uint32_t i = b + threadIdx.x;
        if (i < c.n) {
            uint32_t ab = 1;                               // output record
            const uint32_t len = c.len[i];
            const uint8_t v = xdp_verdict(x, ColA{c, i}, len, c.ethertype[i], ab);
            verdict[i] = v;
            n_drop += v == XDP_DROP_; n_pass += v == XDP_PASS_; s_len += len; s_ab += ab;
        }
    }
    if (stats) { st.xdp_sums(n_drop, n_pass, s_len, s_ab); st.flush(stats); }
}

// check_v4 with the prefilter's hot levels in LDS (k_xdp_lds): the trie's
// 2^16-entry root as two bitmaps (covered: drop at once / has a node: walk on in
// HBM), and — when they fit — the /32 hash's slot array and cilium_lxc's key
// slots, staged once per block (one or two 1024-lane blocks per CU, grid-stride
// over the batch).  The lookups and their order are xdp_verdict's; IPv6 and
// other frames take xdp_verdict as it is.
struct XdpLds {
    uint32_t h4_bytes, lxc_bytes;                  // slot arrays staged as they are (0: not staged)
    const uint32_t *h4set, *lxset;                 // or the tables' compact address sets (Map::addr_set)
    uint32_t h4bits, lxbits, h4zero, lxzero;
};

// Exact-match probe over a slot array held in LDS (layout as in HBM).
template <int KSZ>
__device__ __forceinline__ bool lds_has(const uint8_t *slots, uint64_t mask, uint32_t slot_size, const uint32_t *kw,
                                        uint32_t h) {
    constexpr int SW = KSZ / 4;
    static_assert(KSZ % 4 == 0, "word keys");
    const uint32_t m = (uint32_t)mask, i = (uint32_t)gf_home_slot(h, mask, slot_size);   // LDS tables: < 2^32 slots
    for (uint32_t p = 0; p <= m; p++) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(slots + ((i + p) & m) * slot_size);
        const uint32_t st = w[SW] & 0xffu;
        if (st == GF_SLOT_EMPTY) return false;
        if (st == GF_SLOT_FULL) {
            bool e = true;
#pragma unroll
            for (int k = 0; k < SW; k++) e &= w[k] == kw[k];
            if (e) return true;
        }
    }
    return false;
}
__global__ __launch_bounds__(1024) void k_xdp_lds(gf_pkt_cols c, XdpDev x, XdpLds L, uint8_t *verdict,
                                                  unsigned long long *stats) {
    extern __shared__ uint4 xl[];
    __shared__ uint32_t sl[272];
    Stats st{sl};
    const uint64_t *rs = reinterpret_cast<const uint64_t *>(xl);
    const uint32_t h4b = L.h4set ? 4u << L.h4bits : L.h4_bytes, lxb = L.lxset ? 4u << L.lxbits : L.lxc_bytes;
    const uint8_t *h4s = reinterpret_cast<const uint8_t *>(xl) + GF_TRIE_RSUM_BYTES;
    const uint8_t *lxs = h4s + h4b;
    {
        uint4 *d = xl;
        const uint4 *src = reinterpret_cast<const uint4 *>(x.l4.rsum);
        for (uint32_t k = threadIdx.x; k < GF_TRIE_RSUM_BYTES / 16; k += blockDim.x) d[k] = src[k];
        d += GF_TRIE_RSUM_BYTES / 16;
        src = reinterpret_cast<const uint4 *>(L.h4set ? (const void *)L.h4set : (const void *)x.h4.slots);
        for (uint32_t k = threadIdx.x; k < h4b / 16; k += blockDim.x) d[k] = src[k];
        d += h4b / 16;
        src = reinterpret_cast<const uint4 *>(L.lxset ? (const void *)L.lxset : (const void *)x.lxc.slots);
        for (uint32_t k = threadIdx.x; k < lxb / 16; k += blockDim.x) d[k] = src[k];
    }
    if (stats) st.init(); else __syncthreads();
    uint32_t n_drop = 0, n_pass = 0, s_len = 0, s_ab = 0;      // the lane's counter sums, reduced once at the end
    for (uint32_t b = blockIdx.x * blockDim.x; b < c.n; b += gridDim.x * blockDim.x) {   // wave-uniform trips
        const uint32_t i = b + threadIdx.x;
        const bool act = i < c.n;
        uint32_t len = 0, ab = 1;
        uint8_t v = 0;
        if (act) {
            len = c.len[i];
            const uint32_t et = c.ethertype[i];
            if (et != 0x0800 || len < 34) {
                v = xdp_verdict(x, ColA{c, i}, len, et, ab);
            } else {
                const uint32_t sa = c.saddr4[i];
                bool drop = false;
                ab += 10;
                if (x.has_h4) {
                    ab += 9;
                    const uint32_t idx = ((sa & 0xffu) << 8) | ((sa >> 8) & 0xffu);   // the first two address bytes
                    if ((rs[idx >> 6] >> (idx & 63)) & 1ull) drop = true;
                    else if ((rs[1024 + (idx >> 6)] >> (idx & 63)) & 1ull)
                        drop = x.d24 ? dir24_cov(x.d24, x.d8, sa)
                                     : trie_nodes<1>(x.l4, AddrBytes<1>(&sa), gload<uint32_t>(x.l4.root + idx) - 1u);
                    if (!drop) {
                        ab += 9;
                        const uint32_t kw[2] = {32u, sa};
                        drop = L.h4set ? aset_has(reinterpret_cast<const uint32_t *>(h4s), L.h4bits, L.h4zero, sa)
                             : L.h4_bytes ? lds_has<8>(h4s, x.h4.mask, x.h4.slot_size, kw, key_hash<8>(kw))
                                          : ht_find<8>(x.h4, kw, key_hash<8>(kw)) >= 0;
                    }
                }
                if (drop) {
                    v = XDP_DROP_;
                } else {
                    ab += 20;
                    const uint32_t lk[5] = {c.daddr4[i], 0, 0, 0, 1u};
                    const bool ep = L.lxset ? aset_has(reinterpret_cast<const uint32_t *>(lxs), L.lxbits, L.lxzero, lk[0])
                                  : L.lxc_bytes ? lds_has<20>(lxs, x.lxc.mask, x.lxc.slot_size, lk, key_hash<20>(lk))
                                                : ht_find<20>(x.lxc, lk, key_hash<20>(lk)) >= 0;
                    v = ep ? XDP_PASS_ : XDP_DROP_;
                }
            }
            verdict[i] = v;
            n_drop += v == XDP_DROP_; n_pass += v == XDP_PASS_; s_len += len; s_ab += ab;
        }
    }
    if (stats) {
        st.xdp_sums(n_drop, n_pass, s_len, s_ab);
        st.flush(stats);
    }
}

// ================================================================ LB
struct LbDev {
    gf_htab_desc s4, s6;
    uint32_t flags;
};

__device__ __forceinline__ int lb_checks(const LbDev &L, uint32_t len, int l4_off, uint32_t nh,
                                         uint32_t key_dport, uint32_t svc_port, bool v6, uint16_t *new_dport) {
    uint32_t co = csum_l4_offset(nh);
    if ((co || v6) && !l4csum_ok(l4_off + (int)co, len)) return D_CSUM_L4;
    if ((L.flags & GF_LB_F_L4) && svc_port && key_dport != svc_port && (nh == 6 || nh == 17)) {
        if (!l4csum_ok(l4_off + (int)co, len)) return D_CSUM_L4;
        if (!skb_ok(l4_off + 2, 2, len)) return D_WRITE_ERROR;
        *new_dport = (uint16_t)svc_port;
    }
    return TC_OK;
}

// returns program result (TC_OK pass / TC_REDIRECT translated / negative error)
template <class A>
__device__ int lb_v4(const LbDev &L, const A &a, uint32_t len, gf_lb_out &o, uint32_t &ab, uint32_t &key_dport) {
    if (len < 34) return D_INVALID;
    uint32_t nh = a.proto(), daddr = a.daddr4();
    int l4_off = a.l4_off();
    uint32_t dport = 0;
    if (L.flags & GF_LB_F_L4) {
        if (nh == 6 || nh == 17) {
            if (!skb_ok(l4_off + 2, 2, len)) return -GF_EFAULT;
            dport = a.l4w0() >> 16;
        } else if (nh != 1 && nh != 58) return TC_OK;     // DROP_UNKNOWN_L4 -> pass
    }
    const uint8_t *svc = nullptr;
    if ((L.flags & GF_LB_F_L4) && dport) {
        uint32_t kw[2] = {daddr, dport};
        int64_t f = ht_find<8>(L.s4, kw, key_hash<8>(kw));
        ab += 20;
        if (f >= 0) { const uint8_t *v = ht_val(L.s4, f); if (gload<uint16_t>(v + 6)) svc = v; }
        if (!svc) dport = 0;
    }
    if (!svc && (L.flags & GF_LB_F_L3)) {
        uint32_t kw[2] = {daddr, dport};
        int64_t f = ht_find<8>(L.s4, kw, key_hash<8>(kw));
        ab += 20;
        if (f >= 0) { const uint8_t *v = ht_val(L.s4, f); if (gload<uint16_t>(v + 6)) svc = v; }
    }
    if (!svc) return TC_OK;
    uint32_t count = gload<uint16_t>(svc + 6);
    uint32_t slave = (a.fhash() % count + 1u) & 0xffffu;
    uint32_t kw[2] = {daddr, dport | (slave << 16)};
    int64_t f = ht_find<8>(L.s4, kw, key_hash<8>(kw));
    ab += 20;
    if (f < 0) return D_NO_SERVICE;
    const uint8_t *be = ht_val(L.s4, f);
    uint32_t target = gload<uint32_t>(be);
    uint32_t port = gload<uint16_t>(be + 4);
    uint32_t rn = gload<uint16_t>(be + 8);
    uint16_t nd = 0;
    int r = lb_checks(L, len, l4_off, nh, dport, port, false, &nd);
    if (r < 0) return r;
    key_dport = dport;
    o.slave = (uint16_t)slave; o.new_dport = nd; o.rev_nat = (uint16_t)rn; o.new_daddr4 = target;
    return TC_REDIRECT;
}

template <class A>
__device__ int lb_v6(const LbDev &L, const A &a, uint32_t len, gf_lb_out &o, uint32_t *nd6, uint32_t &ab,
                     uint32_t &key_dport) {
    if (len < 54 || !a.has6()) return D_INVALID;
    uint32_t nh = a.proto();
    int l4_off = a.l4_off();
    uint4 d = a.daddr6();
    uint32_t dport = 0;
    if (L.flags & GF_LB_F_L4) {
        if (nh == 6 || nh == 17) {
            if (!skb_ok(l4_off + 2, 2, len)) return -GF_EFAULT;
            dport = a.l4w0() >> 16;
        } else if (nh != 1 && nh != 58) return TC_OK;
    }
    const uint8_t *svc = nullptr;
    if ((L.flags & GF_LB_F_L4) && dport) {
        uint32_t kw[5] = {d.x, d.y, d.z, d.w, dport};
        int64_t f = ht_find<20>(L.s6, kw, key_hash<20>(kw));
        ab += 44;
        if (f >= 0) { const uint8_t *v = ht_val(L.s6, f); if (gload<uint16_t>(v + 18)) svc = v; }
        if (!svc) dport = 0;
    }
    if (!svc && (L.flags & GF_LB_F_L3)) {
        uint32_t kw[5] = {d.x, d.y, d.z, d.w, dport};
        int64_t f = ht_find<20>(L.s6, kw, key_hash<20>(kw));
        ab += 44;
        if (f >= 0) { const uint8_t *v = ht_val(L.s6, f); if (gload<uint16_t>(v + 18)) svc = v; }
    }
    if (!svc) return TC_OK;
    uint32_t count = gload<uint16_t>(svc + 18);
    uint32_t slave = (a.fhash() % count + 1u) & 0xffffu;
    uint32_t kw[5] = {d.x, d.y, d.z, d.w, dport | (slave << 16)};
    int64_t f = ht_find<20>(L.s6, kw, key_hash<20>(kw));
    ab += 44;
    if (f < 0) return D_NO_SERVICE;
    const uint8_t *be = ht_val(L.s6, f);
    uint32_t t[4];
    for (int k = 0; k < 4; k++) t[k] = gload<uint32_t>(be + 4 * k);
    uint32_t port = gload<uint16_t>(be + 16);
    uint32_t rn = gload<uint16_t>(be + 20);
    if (rn) t[3] |= rn;
    uint16_t ndp = 0;
    int r = lb_checks(L, len, l4_off, nh, dport, port, true, &ndp);
    if (r < 0) return r;
    key_dport = dport;
    o.slave = (uint16_t)slave; o.new_dport = ndp; o.rev_nat = (uint16_t)rn;
    for (int k = 0; k < 4; k++) nd6[k] = t[k];
    return TC_REDIRECT;
}

__global__ __launch_bounds__(BLOCK) void k_lb(gf_pkt_cols c, LbDev L, gf_lb_out *out, uint8_t *nd6,
                                              unsigned long long *stats) {
    __shared__ uint32_t sl[272];
    Stats st{sl};
    if (stats) st.init();
    uint32_t s_n = 0, s_len = 0, s_ab = 0;              // the lane's packet count and sums (Stats::sums)
    // wave-uniform trip count (the stats aggregation is a wave collective)
    for (uint32_t b = blockIdx.x * blockDim.x; b < c.n; b += gridDim.x * blockDim.x) {
      const uint32_t i = b + threadIdx.x;
      const bool act = i < c.n;
      gf_lb_out o{};
      uint32_t len = 0;
      uint32_t ab = 12 + 12;                              // header columns + output record
      if (act) {
        uint32_t n6[4] = {0, 0, 0, 0};
        len = c.len[i];
        const uint32_t et = c.ethertype[i];
        int ret = TC_OK;
        bool v6 = false;
        uint32_t kd = 0;
        if (et == 0x86DD) { if (!(L.flags & GF_LB_F_NO_IPV6)) { v6 = true; ab += 28; ret = lb_v6(L, ColA{c, i}, len, o, n6, ab, kd); } }
        else if (et == 0x0800) { if (!(L.flags & GF_LB_F_NO_IPV4)) ret = lb_v4(L, ColA{c, i}, len, o, ab, kd); }
        if (ret < 0 || ret == TC_SHOT) {
            o = gf_lb_out{};
            o.action = TC_SHOT; o.reason = (uint8_t)(-ret);
            n6[0] = n6[1] = n6[2] = n6[3] = 0;
        } else {
            o.action = ((L.flags & GF_LB_F_REDIRECT) && ret == TC_REDIRECT) ? TC_REDIRECT : TC_OK;
        }
        out[i] = o;
        if (nd6 && v6) reinterpret_cast<uint4 *>(nd6)[i] = make_uint4(n6[0], n6[1], n6[2], n6[3]);
        else if (nd6) reinterpret_cast<uint4 *>(nd6)[i] = make_uint4(0, 0, 0, 0);
      }
      if (act) { s_n++; s_len += len; s_ab += ab; }
      if (stats) st.bins_wave(act, o.reason, o.action);
    }
    if (stats) { st.sums(s_n, s_len, s_ab); st.flush(stats); }
}

// ================================================================ ingress (handle_policy)
// Device-only program flags (high bits of gf_lxc_dev.flags): the program binds
// the CT map of that family (all programs share one per family, X.ct4 / X.ct6).
#define GF_LXC_DEV_HAS_CT4 (1u << 30)
#define GF_LXC_DEV_HAS_CT6 (1u << 31)

#ifndef GF_POUT_WO
#define GF_POUT_WO 1        // gf_pipeline_classify: complete the records without reading them (IngCtx::pout_wo)
#endif
#ifndef GF_EG_RSET
#define GF_EG_RSET 1        // egress connection groups: related entries through RelSet (0: the r5 write log)
#endif
// The ICMP-related entries of an egress connection-group run: the
// only CT keys two connections of one address pair share, written (BPF_ANY) by every
// new connection of the pair in both passes and read by nothing in the run.  Only the
// last write of each key in batch order survives, so each write enters its key here
// instead of a log: the key {daddr, saddr} of the related tuple (its ports are 0 and
// its flags byte is 2 | direction, which picks one of the slot's two words) claims a
// slot (open addressing, 0 = empty; key 0 has the extra slot mask + 1), and the word
// keeps 1 + the highest order written (2i: packet i's from-container create, 2i + 1:
// its delivery's).  k_rset_apply rebuilds each winner's value from its packet.
struct RelSet {
    unsigned long long *slot;          // mask + 2 slots of 16 B: the key, then its two words
    uint32_t *list, *list_n;           // the claimed slots, for the apply
    uint32_t mask;
};
struct IngCtx {
    const gf_lxc_dev *cfgs;
    const uint8_t *saddr6, *daddr6;
    uint32_t a6_stride;      // bytes between two packets' v6 addresses: 16 (the caller's columns) or 32 (the
                             // pipeline / egress deliveries: both addresses of a packet in one 32-B piece)
    gf_htab_desc ct4, ct6;   // cilium_ct4_global / cilium_ct6_global (shared by every program)
    uint32_t now, host_ifindex;
    uint32_t strict;   // bit0 / bit1: CT4 / CT6 inserts check max_entries with atomics
    uint8_t *pout;     // pipeline records (gf_pipeline_out) to complete instead of gf_ingress_out
    uint32_t pout_wo;  // gf_pipeline_classify: the record's first 10 bytes are written without reading them
    uint32_t pol_wave; // policy counter adds summed per wave first (pol_count_add): the egress deliveries' pass
                       // (stage POLICY, the front's GF_PIPE_F_* bits 5-7 in gf_rec.cls bits 4-6)
    uint8_t *snap;     // pipeline: the frames as rewritten so far (handle_policy's writes land here)
    uint32_t snap_stride;
    uint32_t *plog, *plog_n;   // cilium_proxy{4,6} update log (16 words per redirect) and its length
    uint32_t gw, host6[4];     // IPV4_GATEWAY, HOST_IP (node_config.h)
    uint8_t *tmark, *tcap;     // trace notifications: per-packet GF_TR_* marks, 128-B captures (null: off)
    uint32_t *rlog, *rlog_n;   // egress connection groups: ct_create4's related entries logged (null: written)
    const uint32_t *rlog_off;  // device word: nonzero = the run fell back to pair groups (entries written inline)
    RelSet rs;                 // GF_EG_RSET: the related entries' set (rlog non-null: in use)
};

// ---- handle_policy's own header writes (kept out of line: cold paths of the
// hot kernel) and the proxy-map log ----
// The IngCtx fields the writers read, passed by value to the out-of-line copies:
// a reference (or a pointer to a local tuple) would keep the whole context (or
// the tuple) in scratch for the entire IPv6 kernel.
struct PolCtx {
    uint8_t *snap;
    uint32_t *plog, *plog_n;
    uint32_t snap_stride, now, gw, host6[4];
};
__device__ __forceinline__ PolCtx pol_ctx(const IngCtx &X) {
    PolCtx c;
    c.snap = X.snap; c.plog = X.plog; c.plog_n = X.plog_n;
    c.snap_stride = X.snap_stride; c.now = X.now; c.gw = X.gw;
    for (int k = 0; k < 4; k++) c.host6[k] = X.host6[k];
    return c;
}
template <class XC>
__device__ __forceinline__ Row pol_row(const XC &X, uint32_t i, uint32_t len) {
    return Row{X.snap + (size_t)i * X.snap_stride, X.snap_stride < len ? X.snap_stride : len};
}
// Trace notifications (bpf/lib/trace.h:59-106).  The records themselves are
// written after the launches by the event pass (k_ev_*), from the verdict
// records; the kernels only leave what the records cannot tell: a per-packet
// mark byte and, for TRACE_TO_PROXY, the frame as it was when the redirect sent
// it (before its own rewrites, lib/lxc.h:115-117 / 167-169).
#define GF_TR_PX_EGRESS 1u    // from-container ipv{4,6}_redirect_to_host_port entered (TRACE_TO_PROXY)
#define GF_TR_PX_POLICY 2u    // handle_policy's ipv{4,6}_redirect_to_host_port entered (TRACE_TO_PROXY)
#define GF_TR_CLUSTER   4u    // from-container dstID == CLUSTER_ID (TRACE_TO_STACK's dst_label)
#define GF_TR_CAPTURED 16u    // tcap holds the TO_PROXY capture
// f: the frame in HBM; a/na: header bytes a kernel holds in an LDS copy (they
// replace the frame's first na bytes); cap = min(len, stride, TRACE_PAYLOAD_LEN).
__device__ __forceinline__ void trace_proxy(uint8_t *tmark, uint8_t *tcap, const uint8_t *f, const uint8_t *a,
                                            uint32_t na, uint32_t cap, uint32_t i, uint32_t bit) {
    uint32_t m = tmark[i] | bit;
    if (f) {
        uint8_t *d = tcap + (size_t)i * GF_TRACE_PAYLOAD_LEN;
        for (uint32_t k = 0; k < GF_TRACE_PAYLOAD_LEN; k += 4) {
            uint32_t v = 0;
            for (uint32_t b = 0; b < 4; b++) {
                const uint32_t o = k + b;
                if (o < cap) v |= (uint32_t)(o < na ? a[o] : f[o]) << (8 * b);
            }
            *reinterpret_cast<uint32_t *>(d + k) = v;
        }
        m |= GF_TR_CAPTURED;
    }
    tmark[i] = (uint8_t)m;
}
__device__ __forceinline__ uint32_t trace_cap_len(uint32_t len, uint32_t stride) {
    const uint32_t c = len < stride ? len : stride;
    return c < GF_TRACE_PAYLOAD_LEN ? c : GF_TRACE_PAYLOAD_LEN;
}
// reverse_map_l4_port (bpf/lib/lb.h:217-251) + __lb4_rev_nat / __lb6_rev_nat
// (lb.h:253-293, 447-512; v4 with REV_NAT_F_TUPLE_SADDR: the old address is the
// tuple's, v6 with flags 0: the frame's)
template <class XC>
__device__ __forceinline__ void pol_rev_nat_write(const XC &X, uint32_t i, uint32_t len, int l4_off,
                                                            uint32_t nh, const uint8_t *nat, bool v6,
                                                            uint32_t old_sip4) {
    Row w = pol_row(X, i, len);
    const uint32_t co = csum_l4_offset(nh), fl = nh == 17 ? GF_F_MANGLED_0 : 0u;
    const uint32_t port = gload<uint16_t>(nat + (v6 ? 16 : 4));
    if (port && (nh == 6 || nh == 17)) {
        const uint32_t old = w.r16((uint32_t)l4_off);
        if (port != old) {
            l4_csum(w, len, l4_off + (int)co, old, port, 2u | fl);
            w.w16((uint32_t)l4_off, port);
        }
    }
    uint32_t sum = 0;
    if (!v6) {
        const uint32_t nw = gload<uint32_t>(nat);
        w.w32(26, nw);
        sum = ck_add(ck_add(0u, ~old_sip4), nw);
        l3_csum(w, len, 24, 0, sum, 0);
        if (co) l4_csum(w, len, l4_off + (int)co, 0, sum, GF_F_PSEUDO_HDR | fl);
    } else {
        for (int k = 0; k < 4; k++) {
            const uint32_t od = w.r32(22 + 4 * k), nw = gload<uint32_t>(nat + 4 * k);
            w.w32(22 + 4 * k, nw);
            sum = ck_add(ck_add(sum, ~od), nw);
        }
        l4_csum(w, len, l4_off + (int)co, 0, sum, GF_F_PSEUDO_HDR | fl);
    }
}
// ipv6_policy's "derive reverse NAT index and zero it" (bpf_lxc.c:774-790)
template <class XC>
__device__ __forceinline__ void pol_v6_zero_rn(const XC &X, uint32_t i, uint32_t len, int l4_off,
                                                         uint32_t nh, uint32_t rn) {
    Row w = pol_row(X, i, len);
    w.w16(38 + 12, 0);
    const uint32_t co = csum_l4_offset(nh);
    if (co) l4_csum(w, len, l4_off + (int)co, 0, ck_add(ck_add(0u, ~rn), 0u),
                    GF_F_PSEUDO_HDR | (nh == 17 ? GF_F_MANGLED_0 : 0u));
}
// ipv{4,6}_redirect_to_host_port writes (lib/lxc.h:96-205) after their checks,
// and the cilium_proxy{4,6} entry, logged for the in-order apply after the launch.
// t: the CT tuple words as ct_lookup left them; od: the original daddr.
template <class XC>
__device__ __forceinline__ void pol_redirect(const XC &X, uint32_t i, uint32_t len, int l4_off,
                                                       uint32_t nh, const uint32_t *t, bool v6, uint32_t new_port,
                                                       const uint32_t *od, uint32_t identity, uint32_t egress = 0) {
    const uint32_t pw = v6 ? t[8] : t[2];
    const uint32_t old_port = pw & 0xffffu, sport = pw >> 16;
    if (X.snap) {
        Row w = pol_row(X, i, len);
        const uint32_t co = csum_l4_offset(nh), fl = nh == 17 ? GF_F_MANGLED_0 : 0u;
        l4_csum(w, len, l4_off + (int)co, old_port, new_port, 2u | fl);     // l4_modify_port
        w.w16((uint32_t)(l4_off + 2), new_port);
        if (!v6) {
            w.w32(30, X.gw);
            l3_csum(w, len, 24, od[0], X.gw, 4);
            if (co) l4_csum(w, len, l4_off + (int)co, od[0], X.gw, 4u | GF_F_PSEUDO_HDR | fl);
        } else {
            uint32_t sum = 0;
            for (int k = 0; k < 4; k++) {
                w.w32(38 + 4 * k, X.host6[k]);
                sum = ck_add(ck_add(sum, ~od[k]), X.host6[k]);
            }
            if (co) l4_csum(w, len, l4_off + (int)co, 0, sum, GF_F_PSEUDO_HDR | fl);
        }
    }
    if (X.plog) {
        uint32_t *e = X.plog + 16ull * atomicAdd(X.plog_n, 1u);
        uint32_t q[16] = {0};
        q[0] = i; q[1] = v6 ? 6u : 4u;
        const int a = v6 ? 4 : 1;                       // key: .saddr = tuple->daddr, .dport, .sport, .nexthdr
        for (int k = 0; k < a; k++) q[2 + k] = t[k];
        q[2 + a] = new_port | (sport << 16);
        q[3 + a] = nh;
        for (int k = 0; k < a; k++) q[8 + k] = od[k];  // value: orig_daddr, orig_dport, identity, lifetime
        q[8 + a] = old_port;
        q[9 + a] = identity;
        q[10 + a] = X.now + 720u;                       // PROXY_DEFAULT_LIFETIME
        q[15] = egress;                                 // from-container entry: no handle_policy MAC stores
        for (int k = 0; k < 16; k += 4) *reinterpret_cast<uint4 *>(e + k) = make_uint4(q[k], q[k + 1], q[k + 2], q[k + 3]);
    }
}

struct CtState { uint32_t rev_nat, loopback, carry; };

// Slot headers fetched per probe step.  CT maps use the hot-split layout
// (gf_common.h): CT4 slots are 32 B (2 per step = one 64-B request), CT6 64 B;
// policy maps the 16-B policy layout (4 per step = one 64-B request).
// Results do not depend on these.
#ifndef GF_CT4_U
#define GF_CT4_U 2
#endif
#define GF_CT6_U 1
#ifndef GF_POL_U
#define GF_POL_U 4
#endif
#define GF_POL_SLOT 16u    // policy layout (GF_VCODEC_POL, gf_common.h): key | state | pad | proxy_port
#define GF_POL_VOFF 10u
#define GF_POL_SIDE 24u    // side array: packets, bytes, pad

// The endpoint program of the lane's current packet, kept in registers while
// consecutive packets of the lane's bucket target the same endpoint.
struct Ep {
    uint32_t sl;                     // program slot + 1 (0: none loaded)
    uint32_t flags;
    uint8_t *pol;                    // policy map slots / side array / mask (< 2^32 slots)
    uint8_t *pol_side;
    uint32_t pol_mask;
    uint32_t next;                   // round-robin bits: bit0 counter sums (PolAcc), bit1 decisions (PolMemo)
    __device__ __forceinline__ void init() { sl = 0; flags = 0; pol = pol_side = nullptr; pol_mask = 0; next = 0; }
    __device__ __forceinline__ void use(const IngCtx &X, uint32_t s) {
        if (s == sl) return;
        sl = s;
        const gf_lxc_dev *c = X.cfgs + (s - 1);
        flags = gload<uint32_t>(&c->flags);
        // (diagnosis GF_DIAG & 32: every endpoint reads program 0's policy map — one
        // L2-resident table instead of 256 in the MALL; verdicts differ)
        const gf_lxc_dev *pc = (GF_DIAG & 32) ? X.cfgs : c;
        pol = gload<uint8_t *>(&pc->policy.slots);
        pol_side = gload<uint8_t *>(&c->policy.vals);
        pol_mask = (uint32_t)gload<uint64_t>(&pc->policy.mask);
    }
    __device__ __forceinline__ const gf_lxc_dev *cfg(const IngCtx &X) const { return X.cfgs + (sl - 1); }
    __device__ __forceinline__ gf_htab_desc pdesc() const {
        gf_htab_desc d{};
        d.slots = pol; d.vals = pol_side; d.mask = pol_mask; d.ksz = 8; d.vsz = 24;
        d.slot_size = GF_POL_SLOT; d.voff = GF_POL_VOFF; d.vin = 2; d.split = 1; d.sstride = GF_POL_SIDE;
        return d;
    }
};

// The CT map a packet's program binds (CT_MAP4 / CT_MAP6 of its endpoint).
// PCT = false: every program binds the global map (cilium_ct4_global /
// cilium_ct6_global), passed once in the launch context.  PCT = true: the
// ConntrackLocal layout (pkg/endpoint/bpf.go:268-276, cilium_ct4_<id>): each
// program's own map, read from the program table per packet.
template <int FAM, bool PCT>
__device__ __forceinline__ gf_htab_desc ing_ct(const IngCtx &X, const Ep &ep) {
    constexpr uint32_t has = FAM == 6 ? GF_LXC_DEV_HAS_CT6 : GF_LXC_DEV_HAS_CT4;
    if (!(ep.flags & has)) return gf_htab_desc{};
    if constexpr (PCT) return gload<gf_htab_desc>(FAM == 6 ? &ep.cfg(X)->ct6 : &ep.cfg(X)->ct4);
    else return FAM == 6 ? X.ct6 : X.ct4;
}

// The ICMP-related entry ct_create writes for every new flow of a group
// (conntrack.h:563-577) is the same key for the whole group: a lane keeps
// where it lives.  Only this lane changes keys of its group; a delete by the
// lane clears the cache.
// IPv4 (GF_REL_DEFER): the lane also keeps the entry's last hot-part rewrite
// pending instead of storing each one — the value of an ingress create's related
// entry is fixed by now (per launch), the protocol's timeout and the packet's
// length — in the spare high bits of the cached key's last word (bits 16-31: the
// length, bit 15: TCP), and writes it once: before a packet that could read it (an
// ICMP packet of the lane: only ct_lookup4's related probe matches the key),
// before the cache moves to another entry and at the end of the launch.  A group
// creating 4 flows a step then writes its related entry once instead of 4 times.
#ifndef GF_REL_DEFER
#define GF_REL_DEFER 1
#endif
template <int TW>
struct RelCache {
    uint32_t k[TW];
    uint32_t slot;           // ~0u: none (tables of >= 2^32 slots are not cached)
    uint32_t sec;            // src_sec_id of the cold value part this lane wrote there
    __device__ __forceinline__ void init() { slot = ~0u; sec = 0; k[TW - 1] = 0; }
};
// The pending hot-part write of the IPv4 related entry (RelCache<4>::k[3] >> 15), if any.
__device__ __forceinline__ void rel_flush4(const gf_htab_desc &d, RelCache<4> &rc, uint32_t now) {
    const uint32_t p = rc.k[3] >> 15;
    if (!p) return;
    rc.k[3] &= 0x7fffu;
    if (rc.slot == ~0u || !d.slots) return;
    const uint32_t v[4] = {now + ((p & 1u) ? 300u : 43200u), F_SEEN_NON_SYN, 1u, p >> 1};
    store_words<4>(d.slots + (uint64_t)rc.slot * d.slot_size + d.voff, v);
    GF_WR(WR_REL_HOT);
}
template <int TW>
__device__ __forceinline__ void rel_drop(const gf_htab_desc &d, RelCache<TW> &rc, uint32_t now) {
    if constexpr (TW == 4) rel_flush4(d, rc, now);
    rc.slot = ~0u;
}

// __ct_lookup, bpf/lib/conntrack.h:75-135 (dir = CT_INGRESS), hit part.  CT
// values use the GF_VCODEC_CT layout: `hot` = the entry's first 16 B
// (lifetime, flags | rev_nat_index, rx_packets lo32, rx_bytes lo32), loaded
// with the key; the update is one 16-B store into the key's sector (the high
// halves of the rx counters are touched only on a 32-bit carry).
__device__ __forceinline__ void ct_hit(const gf_htab_desc &d, int64_t f, uint4 hot, int action, bool syn,
                                       uint32_t len, uint32_t now, bool acct, CtState &st, uint32_t &ab) {
    ab += 96;                                           // entry RMW: 48 B read + 48 B written
    uint8_t *e = ht_val(d, (uint64_t)f);
    uint32_t life = hot.x, fl = hot.y & 0xffffu, rn = hot.y >> 16;
    if (!(fl & F_RX_CLOSING) || !(fl & F_TX_CLOSING)) {  // ct_entry_alive -> ct_update_timeout
        if (!syn) fl |= F_SEEN_NON_SYN;
        life = now + ((fl & F_SEEN_NON_SYN) ? 43200u : 300u);
    }
    st.rev_nat = rn;
    st.loopback = (fl >> 3) & 1u;
    if (acct) {                                         // rx_packets += 1, rx_bytes += len (exclusive lane)
        uint32_t pk = hot.z + 1u, by = hot.w + len;
        uint8_t *hi = d.sstride ? ht_side(d, (uint64_t)f) : e + 16;
        if (pk == 0u) { gstore<uint32_t>(hi, gload<uint32_t>(hi) + 1u); st.carry = 1; GF_WR(WR_CARRY); }
        if (by < hot.w) { gstore<uint32_t>(hi + 4, gload<uint32_t>(hi + 4) + 1u); st.carry = 1; GF_WR(WR_CARRY); }
        hot.z = pk; hot.w = by;
    }
    if (action == ACT_CREATE) {
        if (fl & (F_RX_CLOSING | F_TX_CLOSING)) {
            fl &= ~(F_RX_CLOSING | F_TX_CLOSING);
            if (!syn) fl |= F_SEEN_NON_SYN;
            life = now + ((fl & F_SEEN_NON_SYN) ? 43200u : 300u);
        }
    } else if (action == ACT_CLOSE) {
        fl |= F_RX_CLOSING;
        if ((fl & F_RX_CLOSING) && (fl & F_TX_CLOSING)) life = now + 10u;
    }
    hot.x = life;
    hot.y = (hot.y & 0xffff0000u) | fl;
    gstore<uint4>(e, hot);
    GF_WR(WR_HIT);
}

// ct_lookup4/6 (conntrack.h:310-437, dir = CT_INGRESS), resolve part: the home
// line of t (shared by the reverse-direction tuple t and the forward tuple tf
// under GF_HASH_CT) was loaded by the caller.  Reverse probe of t, then forward
// probe of tf, answered by one walk.  On return t holds the tuple the reference
// leaves in *tuple (tf unless the first probe hit), *tfl its flags, and pr the
// walk (its EMPTY slot is where ct_create inserts).
template <int KSZ, int TW, int U>
__device__ __forceinline__ int ct_lookup(const gf_htab_desc &d, ProbeLine<KSZ, U, 4> &L, uint32_t *t, uint32_t nh,
                                         uint32_t &tfl, int action, bool syn, uint32_t len, uint32_t now, bool acct,
                                         CtState &st, ProbeRes &pr, uint32_t &ab) {
    constexpr int AW = (TW - 2) / 2;                   // address words per side
    uint32_t tf[TW];
#pragma unroll
    for (int k = 0; k < AW; k++) { tf[k] = t[AW + k]; tf[AW + k] = t[k]; }
    tf[TW - 2] = (t[TW - 2] >> 16) | (t[TW - 2] << 16);
    tf[TW - 1] = nh | ((tfl ^ 1u) << 8);
    pr = probe2<KSZ, U, 4>(d, t, tf, L);
    ab += KSZ;
    uint4 hot = make_uint4(0, 0, 0, 0);
    if (pr.f >= 0) {
        constexpr int NW = Hdr<KSZ, 4>::NW;
        if (pr.u >= 0) {
#pragma unroll
            for (int u = 0; u < U; u++)
                if (u == pr.u) hot = make_uint4(L.hd[u].w[NW - 4], L.hd[u].w[NW - 3], L.hd[u].w[NW - 2], L.hd[u].w[NW - 1]);
        } else {
            hot = gload<uint4>(ht_val(d, (uint64_t)pr.f));
        }
    }
    if (pr.f >= 0 && !pr.is_b) {
        ct_hit(d, pr.f, hot, action, syn, len, now, acct, st, ab);
        return (tfl & 2u) ? CT_RELATED : CT_REPLY;
    }
    ab += KSZ;
#pragma unroll
    for (int k = 0; k < TW; k++) t[k] = tf[k];
    tfl ^= 1u;
    if (pr.f < 0) return CT_NEW;
    ct_hit(d, pr.f, hot, action, syn, len, now, acct, st, ab);
    return CT_ESTABLISHED;
}

// A slot in a log shared by many lanes: one atomic per wave (the active lanes'
// count), each lane its rank among them.
__device__ __forceinline__ uint32_t wave_reserve(uint32_t *ctr) {
    const uint64_t m = __ballot(1);
    const uint32_t lane = threadIdx.x & 63u, lead = (uint32_t)__ffsll((unsigned long long)m) - 1u;
    uint32_t base = 0;
    if (lane == lead) base = atomicAdd(ctr, (uint32_t)__popcll(m));
    base = __shfl(base, (int)lead);
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}
// One related-entry write into the run's set (RelSet).
__device__ __forceinline__ void rset_put(const RelSet &R, uint32_t w0, uint32_t w1, uint32_t side, uint32_t order) {
    const unsigned long long k = ((unsigned long long)w0 << 32) | w1;
    uint32_t p;
    const uint32_t want = order + 1u;
    uint32_t seen = 0;                                  // the key's word as last read (stale: lower)
    if (k == 0ull) {
        p = R.mask + 1u;
        if (atomicCAS(&R.slot[2ull * p], 0ull, 1ull) == 0ull) R.list[atomicAdd(R.list_n, 1u)] = p;
    } else {
        const uint32_t w[2] = {w0, w1};
        p = gf_hash_words(w, 2, 8) & R.mask;
        for (;;) {
            // plain read first (key and words together): within a run a key only goes
            // from 0 to its value and a word only up, so a stale read only makes the
            // CAS fail or costs the atomicMax it would have skipped
            const uint4 sl = *reinterpret_cast<const uint4 *>(R.slot + 2ull * p);
            unsigned long long cur = ((unsigned long long)sl.y << 32) | sl.x;
            if (cur == 0ull) {
                cur = atomicCAS(&R.slot[2ull * p], 0ull, k);
                if (cur == 0ull) { R.list[atomicAdd(R.list_n, 1u)] = p; break; }
            }
            if (cur == k) { seen = side ? sl.w : sl.z; break; }
            p = (p + 1u) & R.mask;
        }
    }
    if (seen < want) atomicMax(reinterpret_cast<uint32_t *>(R.slot + 2ull * p + 1u) + side, want);
}

// ct_create4/6 (conntrack.h:446-580) for ingress (ct_state->addr == 0).  The
// tuple goes to the EMPTY slot the lookup walk ended on (one CAS), the related
// entry to its cached slot when this lane wrote it before — or, with connection
// groups (rlog), to the log applied after the run.

template <int KSZ, int TW, int U>
__device__ __forceinline__ int ct_create(const gf_htab_desc &d, uint32_t *t, uint32_t rev_nat, uint32_t src_sec,
                                         uint32_t len, uint32_t now, bool strict, const ProbeRes &pr, int *added,
                                         RelCache<TW> &rc, uint32_t &ab, uint32_t *rlog = nullptr,
                                         uint32_t *rlog_n = nullptr, uint32_t order = 0, const RelSet *rs = nullptr) {
    constexpr int NHW = TW - 1;                         // word holding nexthdr | flags << 8
    ab += 2 * (KSZ + 48);                               // tuple + ICMP-related entry written
    uint32_t nh = t[NHW] & 0xffu, tfl = (t[NHW] >> 8) & 0xffu;
    uint32_t fl = (nh == 6) ? 0u : F_SEEN_NON_SYN;      // ct_update_timeout(syn = nexthdr == TCP)
    uint32_t life = now + ((fl & F_SEEN_NON_SYN) ? 43200u : 300u);
    // GF_VCODEC_CT: lifetime, flags|rev_nat, rx_packets/bytes lo, hi, tx, unused, src_sec_id
    uint32_t v[12] = {life, fl | (rev_nat << 16), 1u, len, 0u, 0u, 0u, 0u, 0u, 0u, 0u, src_sec};
    if (ht_upsert<KSZ, 12, GF_HASH_CT, U>(d, t, v, strict, added, true, pr.empty, pr.empty_word) < 0)
        return D_CT_CREATE_FAILED;
    uint32_t it[TW];
#pragma unroll
    for (int k = 0; k < TW; k++) it[k] = t[k];
    it[NHW - 1] = 0;                                    // sport = dport = 0
    it[NHW] = (KSZ == 40 ? 58u : 1u) | ((tfl | 2u) << 8);
    v[1] = (fl | F_SEEN_NON_SYN) | (rev_nat << 16);
    if constexpr (KSZ == 14) if (rlog) {                // connection groups: applied after the run, in order
        GF_WR(WR_RLOG);
        if (GF_EG_RSET && rs->slot) {
            rset_put(*rs, it[0], it[1], (it[NHW] >> 8) & 1u, order);
            return 0;
        }
        uint32_t *lg = rlog + (size_t)20 * wave_reserve(rlog_n);
        lg[0] = order;
#pragma unroll
        for (int k = 0; k < TW; k++) lg[1 + k] = it[k];
#pragma unroll
        for (int k = 0; k < 12; k++) lg[5 + k] = v[k];
        return 0;
    }
    bool same = rc.slot != ~0u;
#pragma unroll
    for (int k = 0; k < TW; k++) same &= ((k == TW - 1 ? rc.k[k] & 0x7fffu : rc.k[k]) == it[k]);
    if (same) {                                         // BPF_ANY over the entry this lane wrote
        if (d.vin == 16 && rc.sec == src_sec) {         // cold part (rx hi, tx, src_sec_id) unchanged
            if constexpr (TW == 4 && GF_REL_DEFER) {    // (rev_nat is 0 on the ingress path)
                rc.k[3] = (rc.k[3] & 0x7fffu) | (((len << 1) | (nh == 6 ? 1u : 0u)) << 15);
            } else {
                store_words<4>(d.slots + (uint64_t)rc.slot * d.slot_size + d.voff, v);
                GF_WR(WR_REL_HOT);
            }
        } else {
            if constexpr (TW == 4) rc.k[3] &= 0x7fffu;  // superseded
            store_value<12>(d, (uint64_t)rc.slot, v);
            GF_WR(WR_REL_FULL);
        }
        rc.sec = src_sec;
        return 0;
    }
    if constexpr (TW == 4) rel_flush4(d, rc, now);      // the previous entry's pending write
    GF_WR(WR_REL_NEW);
    int64_t s = ht_upsert<KSZ, 12, GF_HASH_CT, U>(d, it, v, strict, added);
    if (s < 0) return D_CT_CREATE_FAILED;
#pragma unroll
    for (int k = 0; k < TW; k++) rc.k[k] = it[k];
    rc.slot = (uint64_t)s < 0xffffffffull ? (uint32_t)s : ~0u;
    rc.sec = src_sec;
    return 0;
}

// l4_proxy_lookup (ingress) + BPF_L4_MAP semantics, bpf/lib/l4.h:151-217, common.h:105-127
__device__ __forceinline__ int l4_proxy_lookup(const gf_lxc_dev *c, uint32_t nh, uint32_t dport) {
    if (nh != 6 && nh != 17) return 0;
    uint32_t n = gload<uint32_t>(&c->n_l4);
    if (!n) return 0;
    for (uint32_t k = 0; k < n; k++) {
        gf_l4_allow_dev a = gload<gf_l4_allow_dev>(&c->l4[k]);
        if (a.port && a.port == dport) {
            if (a.nexthdr && a.nexthdr == nh) return a.proxy;   // first match decides
        }
    }
    return 0;
}

// policy_entry packets/bytes counters (policy.h:67-68,79-80,91-92).  The
// reference adds them per packet; nothing reads them inside a batch (the host
// sees them after classify returns), so a lane sums the increments of its
// consecutive packets that hit the same entry in registers and applies them
// with one pair of atomics when the entry changes and at the end — the same
// totals with a fraction of the memory-side atomics.
// policy_entry packets += pk, bytes += by at c (two u64 atomics; agent-scope atomics
// go to the memory side, ~17 G/s on MI355X).  wave (IngCtx::pol_wave): the active
// lanes that add to the same entry as the first active lane sum their counts in
// registers first and that lane adds once; the other lanes add their own.  It pays
// on the egress deliveries' pass, whose lanes take neighbouring packets of few
// endpoints (deliveries' k_ing_groups 0.662 -> 0.625 ms), and costs the ingress
// configurations, whose lanes rarely share an entry (config 2 2.535 -> 2.565 ms,
// config 4 1.902 -> 1.957: profiles/r5q_*.json).  Counter sums commute: the final
// values are the reference's.
#ifndef GF_POL_WAVE
#define GF_POL_WAVE 1
#endif
__device__ __forceinline__ void pol_count_add(uint8_t *c, uint32_t pk, uint32_t by, bool wave) {
#if GF_POL_WAVE
  if (wave) {
    const uint64_t act = __ballot(1);
    const uint32_t lane = threadIdx.x & 63u, lead = (uint32_t)__ffsll((unsigned long long)act) - 1u;
    const uint64_t lc = (uint64_t)(uintptr_t)c;
    const uint32_t clo = (uint32_t)__shfl((int)(uint32_t)lc, (int)lead);
    const uint32_t chi = (uint32_t)__shfl((int)(uint32_t)(lc >> 32), (int)lead);
    const bool same = (uint32_t)lc == clo && (uint32_t)(lc >> 32) == chi;
    const uint64_t m = __ballot(same) & act;
    if (same) {                                         // (only the lanes of m run this: sources active)
        unsigned long long sp = 0, sb = 0;
        for (uint64_t mm = m; mm; mm &= mm - 1ull) {
            const int l = __ffsll((unsigned long long)mm) - 1;
            sp += (uint32_t)__shfl((int)pk, l);
            sb += (uint32_t)__shfl((int)by, l);
        }
        if (lane == lead) { gadd64(c, sp); gadd64(c + 8, sb); }
        return;
    }
  }
#endif
    gadd64(c, (unsigned long long)pk);
    gadd64(c + 8, (unsigned long long)by);
}
struct PolAcc {
    uint32_t f[2];                           // policy slots of the open sums
    uint16_t sl[2];                          // their program slot + 1 (0: sum not open)
    uint32_t pk[2], by[2];                   // flushed before a 32-bit sum could wrap
    __device__ __forceinline__ void init() {
        for (int j = 0; j < 2; j++) { f[j] = 0; sl[j] = 0; pk[j] = 0; by[j] = 0; }
    }
    __device__ __forceinline__ void flush_one(const IngCtx &X, int j) {
        if (sl[j]) {
            uint8_t *side = gload<uint8_t *>(&X.cfgs[sl[j] - 1].policy.vals);
            // (GF_DIAG & 32: the slot came from program 0's map; counted in the endpoint's own array)
            const uint32_t fj = (GF_DIAG & 32) ? f[j] & (uint32_t)gload<uint64_t>(&X.cfgs[sl[j] - 1].policy.mask) : f[j];
            uint8_t *c = side + (uint64_t)fj * GF_POL_SIDE;
            if (!(GF_DIAG & 256)) pol_count_add(c, pk[j], by[j], X.pol_wave != 0);   // (GF_DIAG & 256: ablation)
            GF_WR(WR_POLCNT); GF_WR(WR_POLCNT);
        }
        sl[j] = 0; pk[j] = 0; by[j] = 0;
    }
    __device__ __forceinline__ void flush(const IngCtx &X) { flush_one(X, 0); flush_one(X, 1); }
    __device__ __forceinline__ void add(const IngCtx &X, uint32_t s, uint32_t slot, uint32_t len, uint32_t &next) {
        int j = (sl[0] == s && f[0] == slot) ? 0 : ((sl[1] == s && f[1] == slot) ? 1 : -1);
        if (j < 0) { j = (int)(next & 1u); next ^= 1u; flush_one(X, j); sl[j] = (uint16_t)s; f[j] = slot; }
        else if (by[j] + len < by[j] || pk[j] == 0xffffffffu) { flush_one(X, j); sl[j] = (uint16_t)s; f[j] = slot; }
        pk[j] += 1u; by[j] += len;
    }
};

// policy_entry packets/bytes of slot f of the program's policy map (policy maps
// hold < 2^32 slots: max_entries is u32 and the load is <= 1/2)
__device__ __forceinline__ void policy_count(const IngCtx &X, Ep &ep, int64_t f, uint32_t len, PolAcc &acc) {
    acc.add(X, ep.sl, (uint32_t)f, len, ep.next);
}

// A policy slot is 16 B with proxy_port inside, so an L4 hit needs no second load.
typedef ProbeLine<8, GF_POL_U, 0> PolLine;

__device__ __forceinline__ uint32_t pol_home(uint32_t identity, uint32_t dport, uint32_t proto) {
    uint32_t kw[2] = {identity, dport | (proto << 16)};
    return key_hash<8, GF_HASH_POLICY>(kw);
}

// The lane's last policy decision.  __policy_can_access + the reserved-identity
// CIDR check are a pure function of (program, identity, dport, proto, source
// address for reserved identities) while a batch runs: the device never changes
// policy keys, proxy ports, CIDR tries or L4 lists, only the entry counters —
// which stay per packet.  Consecutive packets of a lane's flow group mostly ask
// the same question, so the answer (and the entry to count) is kept.
struct PolDecision {          // 24 B (kept in LDS with the rest of the lane state)
    uint32_t id, sip, pk;
    uint32_t slab;           // program slot + 1 | algorithmic bytes of the decision << 16 (0: empty)
    uint32_t f;              // policy slot counted by the decision, ~0u: none
    int verdict;
};
template <int N>
struct PolMemo {             // N decisions (a group's flows use a couple of ports)
    PolDecision d[N];
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int j = 0; j < N; j++) d[j].slab = 0;
    }
    __device__ __forceinline__ int find(uint32_t s, uint32_t identity, uint32_t k, uint32_t a) const {
#pragma unroll
        for (int j = 0; j < N; j++)
            if ((d[j].slab & 0xffffu) == s && d[j].id == identity && d[j].pk == k && (identity >= 256 || d[j].sip == a))
                return j;
        return -1;
    }
    __device__ __forceinline__ bool hit(uint32_t s, uint32_t identity, uint32_t k, uint32_t a) const {
        return find(s, identity, k, a) >= 0;
    }
    // the slot a new decision replaces: round-robin on bit 1 of the endpoint's bits
    __device__ __forceinline__ PolDecision &victim(uint32_t &next) {
        if constexpr (N == 1) return d[0];
        PolDecision &v = d[(next >> 1) & 1u];
        next ^= 2u;
        return v;
    }
};

// __policy_can_access (policy.h:42-113) + policy_can_access_ingress (:133-168),
// without the counter update: *fc = the entry the reference counts (or -1).
// pl: the home line of (identity, *) if pl_loaded (identity != 0 hashes by
// identity only, so the L4 and the L3 key of the identity share it).
__device__ int policy_lookup(const IngCtx &X, const Ep &ep, PolLine &pl, bool pl_loaded, uint32_t identity, uint32_t dport,
                             uint32_t proto, bool v6, const uint32_t *cidr_addr, uint32_t &ab, int64_t &fc) {
    const uint32_t flags = ep.flags;
    fc = -1;
    if (flags & GF_LXC_F_DROP_ALL) return D_POLICY;
    if (!(flags & GF_LXC_F_POLICY_INGRESS)) return TC_OK;
    const gf_htab_desc pd = ep.pdesc();
    int64_t f;
    uint32_t pp = 0;
    {
        uint32_t k4[2] = {identity, dport | (proto << 16)}, k3[2] = {identity, 0u};
        if (!pl_loaded) pl.load(pd, identity ? pol_home(identity, 0u, 0u) : pol_home(0u, dport, proto));
        if (flags & GF_LXC_F_HAVE_L4_POLICY) {
            ProbeRes r = probe2<8, GF_POL_U, 0>(pd, k4, k3, pl, identity != 0);
            ab += 8;
            if (r.f >= 0 && !r.is_b) {
                pp = 0xffffffffu;
#pragma unroll
                for (int u = 0; u < GF_POL_U; u++)
                    if (u == r.u) pp = pl.hd[u].w[2] >> 16;          // proxy_port at slot byte 10
                f = r.f;
                goto proxy;
            }
            ab += 8;
            if (!identity) {                                // L3 key {0,0,0}: its own home line
                f = ht_find<8, GF_POL_U>(pd, k3, key_hash<8, GF_HASH_POLICY>(k3));
            } else f = r.f;
            if (f >= 0) { ab += 40; fc = f; return TC_OK; }
        } else {
            if (identity) { ProbeRes r = probe2<8, GF_POL_U, 0>(pd, k3, k3, pl, false); f = r.f; }
            else f = ht_find<8, GF_POL_U>(pd, k3, key_hash<8, GF_HASH_POLICY>(k3));
            ab += 8;
            if (f >= 0) { ab += 40; fc = f; return TC_OK; }
        }
    }
    if (flags & GF_LXC_F_HAVE_L4_POLICY) {
        uint32_t kw[2] = {0u, dport | (proto << 16)};
        f = ht_find<8, GF_POL_U>(pd, kw, key_hash<8, GF_HASH_POLICY>(kw));
        ab += 8;
        if (f >= 0) { pp = 0xffffffffu; goto proxy; }
    }
    goto deny;
proxy: {
        ab += 40;                                       // entry read + counters written
        fc = f;
        if (pp == 0xffffffffu) pp = gload<uint16_t>(ht_val(pd, (uint64_t)f));
        if (pp) return (int)pp;
        return l4_proxy_lookup(ep.cfg(X), proto, dport);
    }
deny:
    if (identity < 256) {                               // identity_is_reserved
        const gf_lxc_dev *c = ep.cfg(X);
        if (v6) { const gf_trie_desc tr = gload<gf_trie_desc>(&c->cidr6); if (tr.root_bits) ab += 21; if (trie_lookup<4>(tr, cidr_addr)) return TC_OK; }
        else { const gf_trie_desc tr = gload<gf_trie_desc>(&c->cidr4); if (tr.root_bits) ab += 9; if (trie_lookup<1>(tr, cidr_addr)) return TC_OK; }
    }
    return D_POLICY;
}

// policy_can_access_ingress with the counter update (policy.h:67-92), through the
// lane's decision memo (IPv4, or any non-reserved identity).
template <int N>
__device__ __forceinline__ int policy_ingress(const IngCtx &X, Ep &ep, PolLine &pl, bool pl_loaded, uint32_t identity,
                                              uint32_t dport, uint32_t proto, uint32_t len, bool v6,
                                              const uint32_t *cidr_addr, uint32_t &ab, PolAcc &acc, PolMemo<N> &m) {
    const uint32_t pk = dport | (proto << 16), sip = v6 ? 0u : cidr_addr[0];
#if GF_DIAG & 16
    // diagnosis (ceiling of any policy-map staging): no policy-map read, the counter
    // update kept on a pseudo-random slot of the endpoint's map; verdicts differ
    policy_count(X, ep, (int64_t)((identity * 0x9E3779B1u + pk) & ep.pol_mask), len, acc);
    return TC_OK;
#endif
    const bool memo_ok = !v6 || identity >= 256;
    const int j = memo_ok ? m.find(ep.sl, identity, pk, sip) : -1;
    if (j >= 0) {
        const PolDecision &d = m.d[j];
        ab += d.slab >> 16;
        if (d.f != ~0u) policy_count(X, ep, (int64_t)d.f, len, acc);
        return d.verdict;
    }
    uint32_t ab0 = ab;
    int64_t fc;
    int v = policy_lookup(X, ep, pl, pl_loaded, identity, dport, proto, v6, cidr_addr, ab, fc);
    if (fc >= 0) policy_count(X, ep, fc, len, acc);
    if (memo_ok) {
        PolDecision &d = m.victim(ep.next);
        d.id = identity; d.pk = pk; d.sip = sip; d.verdict = v;
        d.f = fc >= 0 ? (uint32_t)fc : ~0u;    // policy maps hold < 2^32 slots (max_entries is u32)
        d.slab = ep.sl | ((ab - ab0) << 16);
    }
    return v;
}

// __lb{4,6}_rev_nat verdict-affecting checks (lb.h:217-293, 447-512)
__device__ __forceinline__ int rev_nat_checks(uint32_t len, int l4_off, uint32_t nh, uint32_t nat_port,
                                              uint32_t l4w0, bool v6) {
    uint32_t co = csum_l4_offset(nh);
    if (nat_port) {
        if (nh == 6 || nh == 17) {
            if (!skb_ok(l4_off, 2, len)) return -GF_EFAULT;
            if (nat_port != (l4w0 & 0xffffu)) {
                if (!l4csum_ok(l4_off + (int)co, len)) return D_CSUM_L4;
                if (!skb_ok(l4_off, 2, len)) return D_WRITE_ERROR;
            }
        } else if (nh != 1 && nh != 58) return D_UNKNOWN_L4;
    }
    if (v6) { if (!l4csum_ok(l4_off + (int)co, len)) return D_CSUM_L4; }
    else if (co && !l4csum_ok(l4_off + (int)co, len)) return D_CSUM_L4;
    return 0;
}

// ipv{4,6}_redirect_to_host_port verdict-affecting checks (lib/lxc.h:96-205)
__device__ __forceinline__ int redirect_checks(uint32_t len, int l4_off, uint32_t nh) {
    uint32_t co = csum_l4_offset(nh);
    if (!l4csum_ok(l4_off + (int)co, len)) return D_WRITE_ERROR;
    if (!skb_ok(l4_off + 2, 2, len)) return D_WRITE_ERROR;
    return 0;
}

// ct_lookup4/6 header part: fills tuple port/flag words, returns action or error
__device__ __forceinline__ int ct_l4(uint32_t nh, bool v6, const gf_rec &r, uint32_t &pw, uint32_t &tfl,
                                     int &action, bool &syn) {
    uint32_t len = r.len;
    int off = r.l4_off;
    action = ACT_UNSPEC; syn = false;
    if ((!v6 && nh == 1) || (v6 && nh == 58)) {
        if (!skb_ok(off, 1, len)) return D_CT_INVALID_HDR;
        uint32_t type = r.l4w0 & 0xffu;
        pw = 0;
        if (!v6) {
            if (type == 3 || type == 11 || type == 12) tfl |= 2u;
            else if (type == 0) pw = 8u;                         // dport = ICMP_ECHO
            else { if (type == 8) pw = 8u << 16; action = ACT_CREATE; }
        } else {
            if (type >= 1 && type <= 4) tfl |= 2u;
            else if (type == 129) pw = 128u;
            else { if (type == 128) pw = 128u << 16; action = ACT_CREATE; }
        }
        return 0;
    }
    if (nh == 6) {
        if (!skb_ok(off + 12, 2, len)) return D_CT_INVALID_HDR;
        uint32_t w = r.l4w3;
        bool fin = (w >> 8) & 1, sy = (w >> 9) & 1, rst = (w >> 10) & 1;
        action = (rst || fin) ? ACT_CLOSE : ACT_CREATE;
        syn = sy;
        if (!skb_ok(off, 4, len)) return D_CT_INVALID_HDR;
        pw = r.l4w0;
        return 0;
    }
    if (nh == 17) {
        if (!skb_ok(off, 4, len)) return D_CT_INVALID_HDR;
        pw = r.l4w0;
        action = ACT_CREATE;
        return 0;
    }
    return D_CT_UNKNOWN_PROTO;
}

// Out-of-line copies for the IPv6 kernel, whose register budget the inlined
// cold paths would cut to 2 waves/SIMD (the IPv4 kernel keeps them inline).
__device__ __attribute__((noinline)) void pol_rev_nat_write_ol(PolCtx X, uint32_t i, uint32_t len, int l4_off,
                                                               uint32_t nh, const uint8_t *nat) {
    pol_rev_nat_write(X, i, len, l4_off, nh, nat, true, 0u);
}
__device__ __attribute__((noinline)) void pol_v6_zero_rn_ol(PolCtx X, uint32_t i, uint32_t len, int l4_off,
                                                            uint32_t nh, uint32_t rn) {
    pol_v6_zero_rn(X, i, len, l4_off, nh, rn);
}
struct V6Tuple { uint32_t w[10]; };
__device__ __attribute__((noinline)) void pol_redirect_ol(PolCtx X, uint32_t i, uint32_t len, int l4_off,
                                                          uint32_t nh, V6Tuple t, uint32_t new_port,
                                                          uint4 od, uint32_t identity) {
    const uint32_t odw[4] = {od.x, od.y, od.z, od.w};
    pol_redirect(X, i, len, l4_off, nh, t.w, true, new_port, odw, identity);
}

// ipv4_policy, bpf/bpf_lxc.c:865-970
// rlog: X.rlog unless the run fell back to pair groups (read once per kernel, k_ing_groups);
// RL: the instance has the egress connection groups' related-entry path at all (the
// egress deliveries' pass), kept out of the others' registers
template <bool PCT, bool RL = false>
__device__ int ipv4_policy(const IngCtx &X, Ep &ep, const gf_rec &r, uint32_t i, int &fwd, uint8_t &ofl, uint16_t &proxy,
                           uint32_t &ifindex, int *added, uint32_t &ab, PolAcc &acc, RelCache<4> &rc, PolMemo<GF_MEMO4> &pm,
                           uint32_t *rlog) {
    uint32_t len = r.len;
    if (len < 34) return D_INVALID;
    const uint32_t flags = ep.flags;
    uint32_t nh = r.proto;
    uint32_t t[4] = {r.daddr, r.saddr, 0u, nh};
    uint32_t tfl = 0;                                   // TUPLE_F_OUT (ingress)
    if (nh == 1) {                                      // its related probe may read the pending entry
        if constexpr (PCT) rel_flush4(ing_ct<4, true>(X, ep), rc, X.now);   // (the lane's cache is this map's)
        else rel_flush4(X.ct4, rc, X.now);
    }
    int action; bool syn;
    int e = ct_l4(nh, false, r, t[2], tfl, action, syn);
    if (e < 0) return e;
    t[3] = nh | (tfl << 8);
    const gf_htab_desc ct = ing_ct<4, PCT>(X, ep);
    // the CT home line and the policy home line of the source identity go out together
    ProbeLine<14, GF_CT4_U, 4> cl;
#if GF_CT_COOP
    cl.load_quad(ct, key_hash<14, GF_HASH_CT>(t));
#else
    cl.load(ct, key_hash<14, GF_HASH_CT>(t));
#endif
    // (unless the lane's policy memo already answers the NEW/ESTABLISHED question)
    PolLine pl;
    const bool pre = r.src_identity &&
                     (flags & (GF_LXC_F_POLICY_INGRESS | GF_LXC_F_DROP_ALL)) == GF_LXC_F_POLICY_INGRESS &&
                     !pm.hit(ep.sl, r.src_identity, (t[2] >> 16) | (nh << 16), r.saddr) && !(GF_DIAG & (4 | 16));
    if (pre) pl.load(ep.pdesc(), pol_home(r.src_identity, 0u, 0u));
    bool acct = (flags & GF_LXC_F_CT_ACCOUNTING) != 0;
    CtState st{0, 0, 0};
    ProbeRes pr;
    int ret = ct_lookup<14, 4, GF_CT4_U>(ct, cl, t, nh, tfl, action, syn, len, X.now, acct, st, pr, ab);
    fwd = ret;
    if (st.carry) rel_drop(PCT ? ct : X.ct4, rc, X.now);   // a counter carry touched a cold value part
    if (ret == CT_REPLY && st.rev_nat && !st.loopback) {
        const gf_htab_desc rn = gload<gf_htab_desc>(&ep.cfg(X)->revnat4);
        uint32_t kw[1] = {st.rev_nat};
        int64_t f = ht_find<2>(rn, kw, key_hash<2>(kw));
        ab += 8;
        if (f >= 0) {
            const uint8_t *nat = ht_val(rn, f);
            int r2 = rev_nat_checks(len, r.l4_off, nh, gload<uint16_t>(nat + 4), r.l4w0, false);
            if (r2 < 0) return r2;
            if (X.snap) pol_rev_nat_write(X, i, len, r.l4_off, nh, nat, false, t[1]);
            t[1] = gload<uint32_t>(nat);                       // tuple->saddr = nat->address
        }
    }
    uint32_t orig_sip = r.saddr;
    int verdict = (GF_DIAG & 4) ? 0 : policy_ingress(X, ep, pl, pre, r.src_identity, t[2] & 0xffffu, nh, len, false,
                                                     &orig_sip, ab, acc, pm);
    if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
        if (ret == CT_ESTABLISHED) {
            ab += 14;
            ht_delete<14, GF_HASH_CT, GF_CT4_U>(ct, t, X.strict & 1, added);
            rel_drop(PCT ? ct : X.ct4, rc, X.now);
        }
        return D_POLICY;
    }
    if (r.cls & 4) verdict = 0;                         // skip_proxy
    if (ret == CT_NEW && !(GF_DIAG & 8)) {
        ret = ct_create<14, 4, GF_CT4_U>(ct, t, 0u, r.src_identity, len, X.now, X.strict & 1, pr, added, rc, ab,
                                         RL ? rlog : nullptr, X.rlog_n, 2u * i + 1u, &X.rs);
        if (ret < 0) return ret;
        ofl |= GF_INGRESS_F_CREATED;
    }
    if (verdict > 0 && (ret == CT_NEW || ret == CT_ESTABLISHED)) {
        if (X.tmark)
            trace_proxy(X.tmark, X.tcap, X.snap ? X.snap + (size_t)i * X.snap_stride : nullptr, nullptr, 0,
                        trace_cap_len(len, X.snap_stride), i, GF_TR_PX_POLICY);
        int r3 = redirect_checks(len, r.l4_off, nh);
        if (r3 < 0) return r3;
        if (X.snap || X.plog) { const uint32_t od[1] = {r.daddr}; pol_redirect(X, i, len, r.l4_off, nh, t, false, (uint32_t)verdict & 0xffffu, od, r.src_identity); }
        ifindex = X.host_ifindex;
        ofl |= GF_INGRESS_F_PROXY;
        proxy = (uint16_t)verdict;
    }
    return 0;
}

// ipv6_policy, bpf/bpf_lxc.c:745-862
template <bool PCT>
__device__ int ipv6_policy(const IngCtx &X, Ep &ep, const gf_rec &r, uint32_t i, int &fwd, uint8_t &ofl,
                           uint16_t &proxy, uint32_t &ifindex, int *added, uint32_t &ab, PolAcc &acc,
                           RelCache<10> &rc, PolMemo<GF_MEMO6> &pm) {
    uint32_t len = r.len;
    if (len < 54) return D_INVALID;
    if (!X.daddr6 || !X.saddr6) return D_INVALID;      // batch built without IPv6 columns
    const uint32_t flags = ep.flags;
    uint32_t nh = r.proto;
    uint4 d = gload<uint4>(X.daddr6 + (size_t)X.a6_stride * i);
    uint4 s = gload<uint4>(X.saddr6 + (size_t)X.a6_stride * i);
    uint32_t t[10] = {d.x, d.y, d.z, d.w, s.x, s.y, s.z, s.w, 0u, nh};
    uint32_t co = csum_l4_offset(nh);
    uint32_t rn_new = d.w & 0xffffu;                    // ip6->daddr.s6_addr32[3] & 0xFFFF
    if (rn_new) {
        if (X.snap) pol_v6_zero_rn_ol(pol_ctx(X), i, len, r.l4_off, nh, rn_new);
        if (co && !l4csum_ok(r.l4_off + (int)co, len)) return D_CSUM_L4;
    }
    uint32_t tfl = 0;
    int action; bool syn;
    int e = ct_l4(nh, true, r, t[8], tfl, action, syn);
    if (e < 0) return e;
    t[9] = nh | (tfl << 8);
    const gf_htab_desc ct = ing_ct<6, PCT>(X, ep);
    ProbeLine<40, GF_CT6_U, 4> cl;
#if GF_CT_COOP6
    cl.load_quad(ct, key_hash<40, GF_HASH_CT>(t));
#else
    cl.load(ct, key_hash<40, GF_HASH_CT>(t));
#endif
    PolLine pl;
    const bool pre = r.src_identity &&
                     (flags & (GF_LXC_F_POLICY_INGRESS | GF_LXC_F_DROP_ALL)) == GF_LXC_F_POLICY_INGRESS &&
                     !(r.src_identity >= 256 && pm.hit(ep.sl, r.src_identity, (t[8] >> 16) | (nh << 16), 0u));
    if (pre) pl.load(ep.pdesc(), pol_home(r.src_identity, 0u, 0u));
    bool acct = (flags & GF_LXC_F_CT_ACCOUNTING) != 0;
    CtState st{0, 0, 0};
    ProbeRes pr;
    int ret = ct_lookup<40, 10, GF_CT6_U>(ct, cl, t, nh, tfl, action, syn, len, X.now, acct, st, pr, ab);
    fwd = ret;
    if (st.carry) rc.slot = ~0u;
    if (st.rev_nat) {
        const gf_htab_desc rn = gload<gf_htab_desc>(&ep.cfg(X)->revnat6);
        uint32_t kw[1] = {st.rev_nat};
        int64_t f = ht_find<2>(rn, kw, key_hash<2>(kw));
        ab += 20;
        if (f >= 0) {
            const uint8_t *nat = ht_val(rn, f);
            int r2 = rev_nat_checks(len, r.l4_off, nh, gload<uint16_t>(nat + 16), r.l4w0, true);
            if (r2 < 0) return r2;
            if (X.snap) pol_rev_nat_write_ol(pol_ctx(X), i, len, r.l4_off, nh, nat);
        }
    }
    int verdict = policy_ingress(X, ep, pl, pre, r.src_identity, t[8] & 0xffffu, nh, len, true, t + 4, ab, acc, pm);
    if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
        if (ret == CT_ESTABLISHED) {
            ab += 40;
            ht_delete<40, GF_HASH_CT, GF_CT6_U>(ct, t, (X.strict & 2) != 0, added);
            rc.slot = ~0u;
        }
        return D_POLICY;
    }
    if (r.cls & 4) verdict = 0;
    if (ret == CT_NEW) {
        ret = ct_create<40, 10, GF_CT6_U>(ct, t, rn_new, r.src_identity, len, X.now, (X.strict & 2) != 0, pr, added, rc, ab);
        if (ret < 0) return ret;
        ofl |= GF_INGRESS_F_CREATED;
    }
    if (verdict > 0 && (ret == CT_NEW || ret == CT_ESTABLISHED)) {
        if (X.tmark)
            trace_proxy(X.tmark, X.tcap, X.snap ? X.snap + (size_t)i * X.snap_stride : nullptr, nullptr, 0,
                        trace_cap_len(len, X.snap_stride), i, GF_TR_PX_POLICY);
        int r3 = redirect_checks(len, r.l4_off, nh);
        if (r3 < 0) return r3;
        if (X.snap || X.plog) {
            V6Tuple tv;
#pragma unroll
            for (int k = 0; k < 10; k++) tv.w[k] = t[k];
            pol_redirect_ol(pol_ctx(X), i, len, r.l4_off, nh, tv, (uint32_t)verdict & 0xffffu, d, r.src_identity);
        }
        ifindex = X.host_ifindex;
        ofl |= GF_INGRESS_F_PROXY;
        proxy = (uint16_t)verdict;
    }
    return 0;
}

// Per-lane state carried across the packets of the lane's buckets.  It lives in
// LDS (one record per thread, k_ing_groups) so that registers hold only the
// state of the packet in flight: the register budget is what bounds waves per
// SIMD, and waves in flight are what hide the probes' memory latency.
// The lane's share of the counter block: wire / algorithmic byte sums and the
// four CT-result counts (16 bits each; the packet count is their sum), kept per
// lane so the common bins take no same-address LDS atomics; folded into the
// block's bins before a field could wrap and at the end of the launch.
struct LaneCnt {
    uint32_t len, ab, c01, c23;
    __device__ __forceinline__ void init() { len = ab = c01 = c23 = 0; }
    __device__ __forceinline__ void fold(Stats &st) {
        const uint32_t a = c01 & 0xffffu, b = c01 >> 16, c = c23 & 0xffffu, d = c23 >> 16;
        st.add_n(264, a); st.add_n(265, b); st.add_n(266, c); st.add_n(267, d);
        st.add_n(268, a + b + c + d); st.add_n(269, len); st.add_n(270, ab);
        init();
    }
    __device__ __forceinline__ void add(uint32_t l, uint32_t a, uint32_t ct, Stats &st) {
        len += l; ab += a;
        const uint32_t sh = 16u * (ct & 1u);
        uint32_t &w = ct < 2 ? c01 : c23;
        w += 1u << sh;
        if (((w >> sh) & 0xffffu) == 0xffffu || len >= 0xf0000000u || ab >= 0xf0000000u) fold(st);
    }
};

template <int FAM>
struct Lane {
    Ep ep;
    PolAcc acc;
    PolMemo<FAM == 6 ? GF_MEMO6 : GF_MEMO4> pm;
    RelCache<FAM == 6 ? 10 : 4> rc;
    int added;
    LaneCnt sc;
    __device__ __forceinline__ void init() { ep.init(); acc.init(); pm.init(); rc.init(); added = 0; sc.init(); }
};
// Per-endpoint CT maps, non-strict accounting: the lane's net inserts belong to its
// current program's map, added to that map's count (no return value) when the lane
// moves to another program and at the end of the launch.
template <int FAM, bool PCT>
__device__ __forceinline__ void lane_flush_added(const IngCtx &X, Lane<FAM> &ln) {
    if constexpr (PCT) {
        if (ln.added && ln.ep.sl && !(X.strict & (FAM == 6 ? 2u : 1u)))
            atomicAdd(ing_ct<FAM, true>(X, ln.ep).count, (uint32_t)ln.added);
        ln.added = 0;
    }
}
// The lane's pending related-entry write (IPv4), to its map, and the cache dropped.
template <int FAM, bool PCT>
__device__ __forceinline__ void lane_rel_drop(const IngCtx &X, Lane<FAM> &ln) {
    if constexpr (PCT) {
        if (ln.ep.sl) rel_drop(ing_ct<FAM, true>(X, ln.ep), ln.rc, X.now);
        else ln.rc.slot = ~0u;                          // (nothing is pending before a program ran)
    } else {
        rel_drop(X.ct4, ln.rc, X.now);
    }
}

// handle_policy, bpf/bpf_lxc.c:980-1024.  FAM selects the CT path compiled in:
// 4 = the IPv4 path plus every packet that cannot reach conntrack (no IP
// header: their early returns need no CT code), 6 = IPv6 packets that reach
// conntrack.  The sort key keeps the two sets in different buckets.
template <int FAM, bool PCT, bool RL>
__device__ __forceinline__ gf_ingress_out handle_policy(const IngCtx &X, const gf_rec &r, uint32_t i, Lane<FAM> &ln,
                                                       uint32_t &ab, uint32_t *rlog) {
    gf_ingress_out o{};
    uint32_t sl = r.ep;
    if (!sl) { o.action = TC_SHOT; o.reason = 140; return o; }   // missed tail call (DROP_MISSED_TAIL_CALL)
    ln.ep.use(X, sl);
    uint32_t flags = ln.ep.flags;
    int fwd = 0, ret;
    uint8_t fl = 0;
    uint16_t proxy = 0;
    uint32_t ifindex = r.ifindex;
    uint32_t cls = r.cls & 3u;
    if (flags & GF_LXC_F_DROP_ALL) ret = D_POLICY;
    else if (cls == 2) {
        ab += 47;
        if constexpr (FAM == 6) ret = ipv6_policy<PCT>(X, ln.ep, r, i, fwd, fl, proxy, ifindex, &ln.added, ab, ln.acc, ln.rc, ln.pm);
        else ret = D_INVALID;                       // ipv6_policy: short frame or batch without v6 columns
    }
    else if (cls == 1 && (flags & GF_LXC_F_LXC_IPV4)) {
        ab += 23;
        if constexpr (FAM == 4) ret = ipv4_policy<PCT, RL>(X, ln.ep, r, i, fwd, fl, proxy, ifindex, &ln.added, ab, ln.acc, ln.rc, ln.pm,
                                                  rlog);
        else ret = D_INVALID;                       // (not reached: v4 packets sort into FAM 4 buckets)
    }
    else ret = D_UNKNOWN_L3;
    o.ct_ret = (uint8_t)fwd;
    if (ret < 0 || ret == TC_SHOT) {
        o.action = TC_SHOT; o.reason = (uint8_t)(-ret); o.flags = fl & GF_INGRESS_F_CREATED;
        return o;
    }
    o.flags = fl;
    o.proxy_port = proxy;
    o.ifindex_lo = (uint16_t)ifindex;
    o.action = ifindex ? TC_REDIRECT : TC_OK;
    return o;
}

// The 32-B record handle_policy reads and the packet's flow-group bucket key.
// Only packets that can reach conntrack (an IP header is present) are bound to
// their flow group; the rest carry no ordering constraint and are spread out.
// GF_KEY_BITS-1 bits of the group hash are the sort key: groups that collide
// share a bucket (always safe: a bucket is serialized as a whole), and a
// shorter key is one radix pass less.  The top key bit is the family of the CT
// path (1: IPv6 reaching conntrack).  skipped: a pipeline packet that ended
// before the cilium_policy tail call (cls bit 3; left untouched).
__device__ __forceinline__ uint32_t pack_rec(uint32_t i, uint32_t et, uint32_t len, uint32_t sa, uint32_t da,
                                             uint32_t w0, uint32_t w3, int l4, uint32_t proto, uint32_t sid,
                                             uint32_t ifx, uint16_t ep, uint32_t tci, bool skipped, bool have6,
                                             const uint32_t *s6, const uint32_t *d6, gf_rec &r) {
    r.len = len;
    r.saddr = sa; r.daddr = da;
    r.l4w0 = w0; r.l4w3 = (uint16_t)w3;
    r.src_identity = sid;
    r.ifindex = ifx;
    r.ep = ep;                                          // tail_call(cilium_policy, lxc_id) target
    r.l4_off = (int16_t)l4;
    r.proto = (uint8_t)proto;
    uint32_t cls = et == 0x0800 ? 1u : et == 0x86DD ? 2u : 0u;
    if (tci & 1) cls |= 4u;
    if (skipped) cls |= 8u;
    r.cls = (uint8_t)cls;
    if (skipped) return GF_KEY_SKIP;
    const bool ct_ok = ((cls & 3) == 1 && len >= 34) || ((cls & 3) == 2 && len >= 54 && have6);
    if (!ct_ok) return gf_key_live(gf_hash_words(&i, 1, 4) & GF_KEY_HASH);
    if ((cls & 3) == 2) return gf_key_live(gf_pair_hash6(s6, d6) & GF_KEY_HASH) | GF_KEY_FAM;
    return gf_key_live(gf_pair_hash4(sa, da) & GF_KEY_HASH);
}

__global__ __launch_bounds__(BLOCK) void k_ing_pack(gf_pkt_cols c, const uint16_t *slot_of, gf_rec *rec,
                                                    uint32_t *keys) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= c.n) return;
    const uint32_t et = c.ethertype[i], len = c.len[i];
    uint32_t s6[4] = {0, 0, 0, 0}, d6[4] = {0, 0, 0, 0};
    if (et == 0x86DD && len >= 54 && c.saddr6) {
        uint4 sv = reinterpret_cast<const uint4 *>(c.saddr6)[i];
        uint4 dv = gload<uint4>(c.daddr6 + 16 * (size_t)i);
        s6[0] = sv.x; s6[1] = sv.y; s6[2] = sv.z; s6[3] = sv.w;
        d6[0] = dv.x; d6[1] = dv.y; d6[2] = dv.z; d6[3] = dv.w;
    }
    gf_rec r;
    keys[i] = pack_rec(i, et, len, c.saddr4[i], c.daddr4[i], c.l4w0[i], c.l4w3[i], c.l4_off[i], c.proto[i],
                       c.src_identity ? c.src_identity[i] : 0u, c.ifindex ? c.ifindex[i] : 0u,
                       slot_of[c.lxc_id ? c.lxc_id[i] : 0], c.tc_index ? c.tc_index[i] : 0u, false,
                       c.saddr6 != nullptr, s6, d6, r);
    rec[i] = r;
}

// Flow-group schedule.  A bucket is a run of equal 32-bit group hash in the
// stably sorted batch, so it holds whole flow groups with their packets in batch
// order.  One lane runs one bucket to completion, packet after packet — the
// order BPF would see them on one CPU — while different buckets (disjoint CT
// keys) run concurrently.  Buckets are handed out longest first
// (LPT): k_bucket_order lists them by packet count, descending, and waves take
// the next 64 entries of that list from a device queue, so the lanes of a wave
// carry equal work and the deepest buckets start first.
template <int FAM, bool PCT, bool RL>
__device__ __forceinline__ void ing_one(const IngCtx &X, uint32_t i, const gf_rec &r, gf_ingress_out *out,
                                        Stats &st, bool stats, Lane<FAM> &ln, uint32_t *rlog) {
    if (r.cls & 8) return;                              // pipeline: ended before the tail call
    uint32_t ab = 8;                                    // output record
    if constexpr (PCT) {
        // per-endpoint CT maps: the lane's related-entry cache belongs to its current
        // program's map; a packet of another program writes the pending entry first
        if (r.ep != ln.ep.sl) { lane_rel_drop<FAM, true>(X, ln); lane_flush_added<FAM, true>(X, ln); }
    }
    gf_ingress_out o = handle_policy<FAM, PCT, RL>(X, r, i, ln, ab, rlog);
    if (X.pout && X.pout_wo) {                          // complete the pipeline record: stores only
        uint8_t *q = X.pout + 24 * (size_t)i;
        const uint32_t ff = ((uint32_t)(r.cls >> 4) & 7u) << 5;   // the front's whole GF_PIPE_F_* byte
        *reinterpret_cast<uint32_t *>(q) = GF_STAGE_POLICY | ((uint32_t)o.action << 8) | ((uint32_t)o.reason << 16) |
                                           ((uint32_t)o.ct_ret << 24);
        *reinterpret_cast<uint32_t *>(q + 4) = (ff | o.flags) | ((uint32_t)o.proxy_port << 16);
        *reinterpret_cast<uint16_t *>(q + 8) = o.ifindex_lo;
    } else if (X.pout) {                                // complete the pipeline / egress record
        uint8_t *q = X.pout + 24 * (size_t)i;
        // (GF_DIAG & 128: ablation, the record's kept bytes not read — records wrong)
        uint2 a = (GF_DIAG & 128) ? make_uint2(0u, 0u) : *reinterpret_cast<const uint2 *>(q);
        uint2 b = (GF_DIAG & 128) ? make_uint2(0u, 0u) : *reinterpret_cast<const uint2 *>(q + 8);
        a.x = (a.x & 0xffu) | ((uint32_t)o.action << 8) | ((uint32_t)o.reason << 16) | ((uint32_t)o.ct_ret << 24);
        a.y = ((a.y & 0xffu) | o.flags) | (a.y & 0xff00u) | ((uint32_t)o.proxy_port << 16);
        b.x = (b.x & 0xffff0000u) | o.ifindex_lo;
        *reinterpret_cast<uint2 *>(q) = a;
        *reinterpret_cast<uint2 *>(q + 8) = b;
    } else if (!(GF_DIAG & 1)) {
        out[i] = o;
        GF_WR(WR_OUT);
    }
    if (stats && !(GF_DIAG & 2)) {
#if GF_ING_BINS_WAVE
        st.bins_wave(true, o.reason, o.action);         // the active lanes' bins, one LDS atomic per distinct pair
#else
        st.add(o.reason); st.add(256 + o.action);
#endif
        ln.sc.add(r.len, ab, o.ct_ret & 3u, st);
    }
}

__device__ __forceinline__ gf_rec ld_rec(const gf_rec *rec, uint32_t i) {
    if constexpr (GF_REC_NT) {
        const uint4 a = gload_nt16(rec + i), b = gload_nt16(reinterpret_cast<const uint8_t *>(rec + i) + 16);
        gf_rec r;
        __builtin_memcpy(&r, &a, 16);
        __builtin_memcpy(reinterpret_cast<uint8_t *>(&r) + 16, &b, 16);
        return r;
    } else {
        return rec[i];
    }
}
__device__ __forceinline__ void flush_added(const IngCtx &X, uint32_t fam_bit, int added, uint32_t *ct_count,
                                            uint32_t *lds_added) {
    if (X.strict & fam_bit) return;
    if (added) atomicAdd(lds_added, (uint32_t)added);
    __syncthreads();
    if (threadIdx.x == 0 && *lds_added && ct_count) atomicAdd(ct_count, *lds_added);
}

// Bucket lists: family (IPv4 / IPv6 CT path) x endpoint class.  A bucket's class
// is its first packet's endpoint slot mod GF_NCLS (a scheduling hint only: a bucket
// is still one lane's, whole); the lanes of workgroup b start on the lists of class
// b mod GF_NCLS — the XCD the workgroup runs on, dispatch being round-robin over the
// 8 XCDs — and move to the other classes' lists when theirs is drained, so that an
// XCD's L2 would hold the policy maps of its class of endpoints only.  Measured with
// 8 classes: k_ing_groups 2.90 vs 2.40 ms on config 2 — most likely because a
// wave's 64 buckets are no longer neighbours in key order, so their CT home lines
// (placed by the same pair hash) no longer share pages — so one class (the plain
// longest-first list) stays.
#ifndef GF_NCLS
#define GF_NCLS 1u
#endif
#define GF_NL (2u * GF_NCLS)
// Schedule words (device): hist[GF_NL][GF_LCAP+1] | base[..] | cursor[..] | nruns |
// queue[GF_NL] | nfam[2] | lcnt[GF_NL] | lstart[GF_NL] (lists in order: family 0's
// classes, then family 1's; each list by bucket size, descending).
#define GF_LCAP 1024u
#define GF_SCHED_HIST(p) (p)
#define GF_SCHED_BASE(p) ((p) + GF_NL * (GF_LCAP + 1))
#define GF_SCHED_CURSOR(p) ((p) + 2 * GF_NL * (GF_LCAP + 1))
#define GF_SCHED_NRUNS(p) ((p) + 3 * GF_NL * (GF_LCAP + 1))
#define GF_SCHED_QUEUE(p) (GF_SCHED_NRUNS(p) + 1)
#define GF_SCHED_NFAM(p) (GF_SCHED_QUEUE(p) + GF_NL)
#define GF_SCHED_LCNT(p) (GF_SCHED_NFAM(p) + 2)
#define GF_SCHED_LSTART(p) (GF_SCHED_LCNT(p) + GF_NL)
#define GF_SCHED_WORDS (3 * GF_NL * (GF_LCAP + 1) + 1 + GF_NL + 2 + 2 * GF_NL)
#define GF_SCHED_HBYTES (GF_NL * (GF_LCAP + 1) * 4)    // the block-local bins of k_bucket_hist / order (dynamic LDS)
// The list of a bucket: family from its key, class from its first packet's record.
__device__ __forceinline__ uint32_t sched_list(uint32_t key, const gf_rec *rec, const uint32_t *perm, uint32_t b) {
    const uint32_t f = key >> (GF_KEY_BITS - 1);
    const uint32_t x = rec ? (uint32_t)rec[perm[b]].ep % GF_NCLS : 0u;
    return f * GF_NCLS + x;
}

// GRAB: buckets per lane per queue grab in the single-packet tail (GF_GRAB_ING for the
// egress deliveries' pass, whose buckets are mostly single packets; 1 elsewhere,
// where the extra state costs the kernel registers it cannot spare)
template <int FAM, int GRAB = 1, bool PCT = false, bool RL = false>
__global__ __launch_bounds__(BLOCK, FAM == 6 ? GF_ING_MINW6 : GF_ING_MINW) void k_ing_groups(IngCtx X, uint32_t *sched, const uint2 *order,
                                                      const uint32_t *perm,
                                                      const gf_rec *rec, gf_ingress_out *out, uint32_t *ct_count,
                                                      unsigned long long *stats) {
    constexpr int F = FAM == 6 ? 1 : 0;
    const uint32_t *nfam = GF_SCHED_NFAM(sched);
    if (nfam[F] == 0) return;                          // no bucket of this family (nothing to count either)
    __shared__ uint32_t sl[272];
    __shared__ uint32_t sadd;
    Stats st{sl};
    if (threadIdx.x == 0) sadd = 0;
    if (stats) st.init(); else __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t *lcnt = GF_SCHED_LCNT(sched), *lstart = GF_SCHED_LSTART(sched);
    __shared__ Lane<FAM> lanes[BLOCK];
    Lane<FAM> &ln = lanes[threadIdx.x];
    ln.init();
    uint32_t *const rlog = RL && X.rlog && !(X.rlog_off && *X.rlog_off) ? X.rlog : nullptr;
    const uint32_t x0 = blockIdx.x % GF_NCLS;           // this workgroup's XCD class first
    for (uint32_t xi = 0; xi < GF_NCLS; xi++) {
    const uint32_t L = F * GF_NCLS + (x0 + xi) % GF_NCLS;
    uint32_t *queue = GF_SCHED_QUEUE(sched) + L;
    const uint32_t nb = lcnt[L];
    const uint2 *lorder = order + lstart[L];
    // the wave's grab: [base, base + 64 * left) of the list, one 64-bucket round at a
    // time (wave-uniform values); grab = buckets per lane of the next grab
    uint32_t grab = 1, gbase = 0, left = 0;
    for (;;) {
        uint32_t t;
        bool first = false;
        if constexpr (GRAB == 1) {
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(queue, 64u);
            base = __shfl(base, 0);
            if (base >= nb) break;
            t = base + lane;
        } else {
            if (!left) {
                uint32_t b0 = 0;
                if (lane == 0) b0 = atomicAdd(queue, 64u * grab);
                gbase = (uint32_t)__builtin_amdgcn_readfirstlane((int)b0);
                left = grab;
            }
            if (gbase >= nb) break;
            t = gbase + lane;
            first = left == grab;
            gbase += 64u; left--;
        }
        if (t >= nb) continue;
        const uint2 oc = lorder[t];
        if (GRAB > 1 && first && (uint32_t)__builtin_amdgcn_readfirstlane((int)oc.y) == 1u) grab = GRAB;   // single-packet tail
        const uint32_t b = oc.x, c = oc.y;
        uint32_t i = perm[b];
        uint32_t inx = c > 1 ? perm[b + 1] : 0u;
        gf_rec r = ld_rec(rec, i);
        lane_rel_drop<FAM, PCT>(X, ln);                  // a new bucket: new flow groups
#if GF_PERM_VEC
        uint4 pw = make_uint4(0, 0, 0, 0);               // perm[j & ~3 .. +3], j = b + k + 2
        if (c > 2) pw = *reinterpret_cast<const uint4 *>(perm + ((b + 2) & ~3u));
#endif
        for (uint32_t k = 0; k < c; k++) {
            // the next record and the index after it are in flight while packet k runs
            uint32_t in2 = 0;
#if GF_PERM_VEC
            if (k + 2 < c) {
                const uint32_t j = b + k + 2;
                if (!(j & 3u) && k) pw = *reinterpret_cast<const uint4 *>(perm + j);
                const uint32_t q = j & 3u;
                in2 = q == 0 ? pw.x : q == 1 ? pw.y : q == 2 ? pw.z : pw.w;
            }
#else
            if (k + 2 < c) in2 = perm[b + k + 2];
#endif
            ing_one<FAM, PCT, RL>(X, i, r, out, st, stats != nullptr, ln, rlog);
            i = inx; inx = in2;
            if (k + 1 < c) r = ld_rec(rec, i);
        }
    }
    }
    ln.acc.flush(X);
    lane_rel_drop<FAM, PCT>(X, ln);                     // the pending related-entry write (IPv4)
    lane_flush_added<FAM, PCT>(X, ln);                  // (per-endpoint maps: the lane's own count add)
    if (stats) ln.sc.fold(st);
    flush_added(X, F ? 2u : 1u, ln.added, ct_count, &sadd);
    if (stats) st.flush(stats);
}

#define GF_LCAP 1024u
// Bucket-size histogram per family (bit 31 of the bucket's sorted key):
// block-local LDS bins, one global add per non-empty bin.
#define GF_SCHED_ITEMS 4096
// off[q]: the start of run q in the sorted keys (nruns of them); its length is
// the distance to the next start (or to n).
__global__ __launch_bounds__(BLOCK) void k_bucket_hist(uint32_t n, const uint32_t *off, const uint32_t *skeys,
                                                       const gf_rec *rec, const uint32_t *perm, uint32_t *sched) {
    extern __shared__ uint32_t h[];                     // GF_SCHED_HBYTES
    for (uint32_t k = threadIdx.x; k < GF_NL * (GF_LCAP + 1); k += blockDim.x) h[k] = 0;
    __syncthreads();
    uint32_t nq = *GF_SCHED_NRUNS(sched);
    uint32_t b0 = blockIdx.x * GF_SCHED_ITEMS;
    for (uint32_t q = b0 + threadIdx.x; q < b0 + GF_SCHED_ITEMS && q < nq; q += blockDim.x) {
        const uint32_t key = skeys[off[q]];
        uint32_t c = (q + 1 < nq ? off[q + 1] : n) - off[q];
        if (c && key != GF_KEY_SKIP)
            atomicAdd(&h[sched_list(key, rec, perm, off[q]) * (GF_LCAP + 1) + (c < GF_LCAP ? c : GF_LCAP)], 1u);
    }
    __syncthreads();
    uint32_t *hist = GF_SCHED_HIST(sched);
    for (uint32_t k = threadIdx.x; k < GF_NL * (GF_LCAP + 1); k += blockDim.x)
        if (h[k]) atomicAdd(&hist[k], h[k]);
}

// base[l][c] = start of (list l, count c) in the order array: the lists one after
// the other, each by count descending.  One block of GF_LCAP threads (thread k owns
// bin c = GF_LCAP - k); also clears the cursors and the work queues and writes each
// list's count and start and each family's total.
__global__ __launch_bounds__(GF_LCAP) void k_bucket_base(uint32_t *sched) {
    __shared__ uint32_t s[GF_LCAP];
    __shared__ uint32_t tot;
    const uint32_t k = threadIdx.x, c = GF_LCAP - k;
    const uint32_t *hist = GF_SCHED_HIST(sched);
    uint32_t *base = GF_SCHED_BASE(sched), *cursor = GF_SCHED_CURSOR(sched);
    if (k == 0) { tot = 0; GF_SCHED_NFAM(sched)[0] = GF_SCHED_NFAM(sched)[1] = 0; }
    __syncthreads();
    for (uint32_t l = 0; l < GF_NL; l++) {
        const uint32_t *hf = hist + l * (GF_LCAP + 1);
        s[k] = hf[c];
        __syncthreads();
        for (uint32_t d = 1; d < GF_LCAP; d <<= 1) {    // inclusive scan over bins GF_LCAP .. 1
            uint32_t v = k >= d ? s[k - d] : 0u;
            __syncthreads();
            s[k] += v;
            __syncthreads();
        }
        const uint32_t add = tot;
        base[l * (GF_LCAP + 1) + c] = add + s[k] - hf[c];
        cursor[l * (GF_LCAP + 1) + c] = 0;
        if (k == 0) { base[l * (GF_LCAP + 1)] = add; cursor[l * (GF_LCAP + 1)] = 0; }
        __syncthreads();
        if (k == GF_LCAP - 1) {
            GF_SCHED_LCNT(sched)[l] = s[k];
            GF_SCHED_LSTART(sched)[l] = add;
            GF_SCHED_NFAM(sched)[l / GF_NCLS] += s[k];
            GF_SCHED_QUEUE(sched)[l] = 0;
            tot = add + s[k];
        }
        __syncthreads();
    }
}

// order[] = {first sorted position, packet count} of the non-empty buckets,
// family 0 then 1, each by count descending (ties in any order): block-local
// counts per bin, one global reservation per (block, bin).
__global__ __launch_bounds__(BLOCK) void k_bucket_order(uint32_t n, const uint32_t *off, const uint32_t *skeys,
                                                        const gf_rec *rec, const uint32_t *perm, uint32_t *sched,
                                                        uint2 *order, uint32_t skip1) {
    extern __shared__ uint32_t h[];                     // GF_SCHED_HBYTES
    for (uint32_t k = threadIdx.x; k < GF_NL * (GF_LCAP + 1); k += blockDim.x) h[k] = 0;
    __syncthreads();
    uint32_t nq = *GF_SCHED_NRUNS(sched);
    const uint32_t *base = GF_SCHED_BASE(sched);
    uint32_t *cursor = GF_SCHED_CURSOR(sched);
    uint32_t b0 = blockIdx.x * GF_SCHED_ITEMS;
    for (uint32_t q = b0 + threadIdx.x; q < b0 + GF_SCHED_ITEMS && q < nq; q += blockDim.x) {
        const uint32_t key = skeys[off[q]];
        uint32_t c = (q + 1 < nq ? off[q + 1] : n) - off[q];
        if (c && key != GF_KEY_SKIP && !(skip1 && c == 1))
            atomicAdd(&h[sched_list(key, rec, perm, off[q]) * (GF_LCAP + 1) + (c < GF_LCAP ? c : GF_LCAP)], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < GF_NL * (GF_LCAP + 1); k += blockDim.x)
        if (h[k]) h[k] = base[k] + atomicAdd(&cursor[k], h[k]);
    __syncthreads();
    for (uint32_t q = b0 + threadIdx.x; q < b0 + GF_SCHED_ITEMS && q < nq; q += blockDim.x) {
        const uint32_t key = skeys[off[q]];
        uint32_t c = (q + 1 < nq ? off[q + 1] : n) - off[q];
        if (c && key != GF_KEY_SKIP && !(skip1 && c == 1))
            order[atomicAdd(&h[sched_list(key, rec, perm, off[q]) * (GF_LCAP + 1) + (c < GF_LCAP ? c : GF_LCAP)], 1u)] =
                make_uint2(off[q], c);
    }
}
// Single-packet buckets in packet-index order (GF_SINGLE_ORDER, the egress passes,
// whose connection groups are mostly one packet a step): the tail of each family's
// list (bin c = 1) is filled by packet index, so a wave's lanes read neighbouring
// records, frames and output rows instead of 64 random ones.  k_single_mark writes
// each such packet's word sw[i] = (bucket start + 1) << 1 | family (one 4-B store;
// 0 = not a single-packet bucket); k_single_count / k_run_scan / k_single_write
// rank them per family in index order.
__global__ __launch_bounds__(BLOCK) void k_single_mark(uint32_t n, const uint32_t *off, const uint32_t *skeys,
                                                       const uint32_t *perm, const uint32_t *sched, uint32_t *sw) {
    const uint32_t nq = *GF_SCHED_NRUNS(sched);
    for (uint32_t q = blockIdx.x * BLOCK + threadIdx.x; q < nq; q += gridDim.x * BLOCK) {
        const uint32_t b = off[q], key = skeys[b];
        if ((q + 1 < nq ? off[q + 1] : n) - b != 1u || key == GF_KEY_SKIP) continue;
        sw[perm[b]] = ((b + 1u) << 1) | (key >> (GF_KEY_BITS - 1));
    }
}
// the family of a packet's single-bucket word: 1 / 2, 0 = none
__device__ __forceinline__ uint32_t single_fam(uint32_t w) { return w ? 1u + (w & 1u) : 0u; }
__global__ __launch_bounds__(BLOCK) void k_single_count(uint32_t n, const uint32_t *sw, uint32_t *t0, uint32_t *t1) {
    __shared__ uint32_t wc[2][BLOCK / 64];
    const uint32_t b0 = blockIdx.x * GF_RUN_ITEMS, lane = threadIdx.x & 63u;
    uint32_t c0 = 0, c1 = 0;
    for (uint32_t k = 0; k < GF_RUN_ITEMS / BLOCK; k++) {
        const uint32_t j = b0 + k * BLOCK + threadIdx.x;
        const uint32_t f = j < n ? single_fam(sw[j]) : 0u;
        c0 += (uint32_t)__popcll(__ballot(f == 1u));
        c1 += (uint32_t)__popcll(__ballot(f == 2u));
    }
    if (lane == 0) { wc[0][threadIdx.x >> 6] = c0; wc[1][threadIdx.x >> 6] = c1; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t a = 0, z = 0;
        for (uint32_t w = 0; w < BLOCK / 64; w++) { a += wc[0][w]; z += wc[1][w]; }
        t0[blockIdx.x] = a; t1[blockIdx.x] = z;
    }
}
__global__ __launch_bounds__(BLOCK) void k_single_write(uint32_t n, const uint32_t *sw, const uint32_t *t0,
                                                        const uint32_t *t1, const uint32_t *sched, uint2 *order) {
    __shared__ uint32_t wc[2][BLOCK / 64];
    const uint32_t b0 = blockIdx.x * GF_RUN_ITEMS, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t *base = GF_SCHED_BASE(sched);         // bin c = 1 of family f's list (GF_NCLS == 1)
    uint32_t p0 = base[0 * (GF_LCAP + 1) + 1] + t0[blockIdx.x], p1 = base[1 * (GF_LCAP + 1) + 1] + t1[blockIdx.x];
    for (uint32_t k = 0; k < GF_RUN_ITEMS / BLOCK; k++) {
        const uint32_t j = b0 + k * BLOCK + threadIdx.x;
        const uint32_t w = j < n ? sw[j] : 0u, f = single_fam(w);
        const uint64_t m0 = __ballot(f == 1u), m1 = __ballot(f == 2u);
        if (lane == 0) { wc[0][wv] = (uint32_t)__popcll(m0); wc[1][wv] = (uint32_t)__popcll(m1); }
        __syncthreads();
        uint32_t e0 = 0, e1 = 0, a0 = 0, a1 = 0;
        for (uint32_t q = 0; q < BLOCK / 64; q++) {
            e0 += q < wv ? wc[0][q] : 0u; e1 += q < wv ? wc[1][q] : 0u;
            a0 += wc[0][q]; a1 += wc[1][q];
        }
        const uint64_t below = (1ull << lane) - 1ull;
        if (f == 1u) order[p0 + e0 + (uint32_t)__popcll(m0 & below)] = make_uint2((w >> 1) - 1u, 1u);
        if (f == 2u) order[p1 + e1 + (uint32_t)__popcll(m1 & below)] = make_uint2((w >> 1) - 1u, 1u);
        p0 += a0; p1 += a1;
        __syncthreads();
    }
}

// ================================================================ pipeline (config 4)
// bpf_xdp -> bpf_lb from-netdev -> bpf_netdev from-netdev -> cilium_policy tail
// call, each program seeing the frame as the previous one rewrote it.
// k_pipe_front stages a block's frames in LDS and runs the first three on one
// packet per lane over its frame there (the rewrites and their checksum updates
// are applied to that copy), re-parses the rewritten header and writes the
// packet's handle_policy record and flow-group key directly (k_ing_pack fused);
// the ingress machinery then runs handle_policy on the packets that reached the
// tail call and completes their pipeline records in place.
struct NetdevDev {
    gf_htab_desc lxc;
    const uint32_t *lxset;         // cilium_lxc's IPv4 keys: address set + slots (Map::addr_set), or null
    uint32_t lxbits, lxzero;
    uint32_t flags, fixed_secctx;
    uint32_t router6[2];           // first 8 bytes of ROUTER_IP (LE words)
};
struct PipeDev {
    XdpDev x;
    LbDev L;
    NetdevDev nd;
    uint32_t has_xdp, has_lb, lb_redirect_ifindex, vec_copy;
    uint8_t *tcap_in;              // TRACE_FROM_STACK captures (128 B per packet; null: the netdev does not trace)
};
// lb4_xlate / lb6_xlate writes (bpf/lib/lb.h:615-659, 397-423) of a translation
// lb_v4/lb_v6 accepted (their checks passed, so every helper succeeds).
__device__ void pipe_lb_rewrite(Row &w, uint32_t len, const PktHdr &h, bool v6, const gf_lb_out &o,
                                const uint32_t *n6, uint32_t key_dport, uint32_t &ab) {
    const uint32_t nh = h.proto;
    const int l4_off = h.l4;
    uint32_t sum = 0;
    if (!v6) {
        const uint32_t old = h.da, nw = o.new_daddr4;
        w.w32(30, nw);
        sum = ck_add(ck_add(0u, ~old), nw);             // csum_diff(&key->address, 4, new_daddr, 4, 0)
        l3_csum(w, len, 24, 0, sum, 0);
        ab += 4 + 2;
    } else {
        const uint32_t *od = h.d6;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            w.w32(38 + 4 * k, n6[k]);                   // ipv6_store_daddr
            sum = ck_add(ck_add(sum, ~od[k]), n6[k]);
        }
        ab += 16;
    }
    const uint32_t co = csum_l4_offset(nh), fl = nh == 17 ? GF_F_MANGLED_0 : 0u;
    if (co || v6) { l4_csum(w, len, l4_off + (int)co, 0, sum, GF_F_PSEUDO_HDR | fl); ab += 2; }
    if (o.new_dport) {                                  // l4_modify_port, bpf/lib/l4.h:50-60
        l4_csum(w, len, l4_off + (int)co, key_dport, o.new_dport, 2u | fl);
        w.w16((uint32_t)(l4_off + 2), o.new_dport);
        ab += 4;
    }
}

enum { ND_TAILCALL = 1000, ND_ICMP6_TE = 1001 };

// The common tail of ipv{4,6}_local_delivery (bpf/lib/l3.h:106-168): MACs,
// map_lxc_in (l3.h:71-104 + l4_port_map_in, bpf/lib/l4.h:62-88: every portmap
// entry is compared with the dport loaded once), cb[], tail call.
__device__ int delivery_tail(Row &w, uint32_t len, int l4_off, uint32_t nh, const uint8_t *ep, uint32_t &ifx,
                             uint32_t &lxc, uint32_t &mapped, uint32_t &ndport, uint32_t &ab) {
    const uint32_t m0 = gload<uint32_t>(ep + 16), m1 = gload<uint32_t>(ep + 20);
    const uint32_t r0 = gload<uint32_t>(ep + 24), r1 = gload<uint32_t>(ep + 28);
    w.w32(6, r0); w.w16(10, r1 & 0xffffu);              // eth_store_saddr(node_mac)
    w.w32(0, m0); w.w16(4, m1 & 0xffffu);               // eth_store_daddr(mac)
    ab += 16 + 12;
    const uint32_t pm0 = gload<uint32_t>(ep + 48);
    ab += 4;
    if ((pm0 >> 16) && (nh == 6 || nh == 17)) {
        if (!skb_ok(l4_off + 2, 2, len)) return D_INVALID;
        const uint32_t dport = w.r16((uint32_t)(l4_off + 2));
        const uint32_t co = csum_l4_offset(nh), fl = nh == 17 ? GF_F_MANGLED_0 : 0u;
        for (int k = 0; k < 16; k++) {                  // PORTMAP_MAX
            const uint32_t pm = k ? gload<uint32_t>(ep + 48 + 4 * k) : pm0;
            const uint32_t from = pm & 0xffffu, to = pm >> 16;
            if (k) ab += 4;
            if (!to || !from) break;
            if (from != dport) continue;
            if (l4_csum(w, len, l4_off + (int)co, dport, to, 2u | fl) < 0) return D_CSUM_L4;
            if (!skb_ok(l4_off + 2, 2, len)) return D_WRITE_ERROR;
            w.w16((uint32_t)(l4_off + 2), to);
            mapped = 1; ndport = to;
            ab += 4;
        }
    }
    ifx = gload<uint32_t>(ep);                          // cb[CB_IFINDEX] = ep->ifindex
    lxc = gload<uint16_t>(ep + 6);                      // tail_call(cilium_policy, ep->lxc_id)
    return ND_TAILCALL;
}

// from_netdev of bpf/bpf_netdev.c:395-460 -> handle_ipv4 (:326-393) / handle_ipv6
// (:160-247), without FROM_HOST, ENCAP_IFINDEX or HANDLE_NS.
__device__ int pipe_netdev(const NetdevDev &N, Row &w, const PktHdr &h, uint32_t et, uint32_t len,
                           uint32_t &sec, uint32_t &ifx, uint32_t &lxc, uint32_t &mapped, uint32_t &ndport,
                           uint32_t &ab) {
    if (et == 0x0800) {
        if (len < 34) return D_INVALID;                 // revalidate_data
        sec = (N.flags & GF_NETDEV_F_FIXED_SECCTX) ? N.fixed_secctx : 2u;   // derive_ipv4_sec_ctx: WORLD_ID
        uint32_t kw[5] = {w.r32(30), 0, 0, 0, 1u};      // lookup_ip4_endpoint (post-LB daddr)
        const int64_t f = N.lxset ? aset_slot(N.lxset, N.lxbits, N.lxzero, kw[0]) : ht_find<20>(N.lxc, kw, key_hash<20>(kw));
        ab += 20;
        if (f < 0) return TC_OK;
        const uint8_t *ep = ht_val(N.lxc, f);
        ab += 8;
        if (gload<uint32_t>(ep + 8) & 1u) return TC_OK; // ENDPOINT_F_HOST
        const uint32_t ttl = w.b(22);                   // ipv4_dec_ttl, bpf/lib/ipv4.h:30-43
        if (ttl <= 1) return D_INVALID;
        l3_csum(w, len, 24, ttl, ttl - 1, 2);
        w.w8(22, ttl - 1);
        ab += 3;
        return delivery_tail(w, len, h.l4, h.proto, ep, ifx, lxc, mapped, ndport, ab);
    }
    if (et == 0x86DD) {
        if (len < 54) return D_INVALID;
        sec = 2u;                                       // derive_sec_ctx (bpf_netdev.c:50-64)
        if (N.flags & GF_NETDEV_F_FIXED_SECCTX) sec = N.fixed_secctx;
        else if (w.r32(22) == N.router6[0] && w.r32(26) == N.router6[1])
            sec = __builtin_bswap32(w.r32(14) & __builtin_bswap32(0x000FFFFFu));
        uint32_t kw[5] = {w.r32(38), w.r32(42), w.r32(46), w.r32(50), 2u};
        const int64_t f = ht_find<20>(N.lxc, kw, key_hash<20>(kw));
        ab += 20 + 8;
        if (f < 0) return TC_OK;
        const uint8_t *ep = ht_val(N.lxc, f);
        ab += 8;
        if (gload<uint32_t>(ep + 8) & 1u) return TC_OK;
        const uint32_t hl = w.b(21);                    // ipv6_dec_hoplimit, bpf/lib/ipv6.h:178-193
        if (hl <= 1) return ND_ICMP6_TE;
        w.w8(21, hl - 1);
        ab += 1;
        return delivery_tail(w, len, h.l4, h.proto, ep, ifx, lxc, mapped, ndport, ab);
    }
    return TC_OK;                                       // unknown traffic to the stack
}

// One packet per lane; the block's frames are staged in LDS (BLOCK * snap_stride
// bytes of dynamic shared memory) and copied back out only when the caller
// asked for the rewritten frames.
template <int NT>
__global__ __launch_bounds__(NT, GF_FRONT_MINW) void k_pipe_front(gf_frames fr, const uint8_t *tc_index, const uint32_t *flow_hash,
                                                      PipeDev P, const uint16_t *slot_of, gf_rec *rec, uint32_t *keys,
                                                      uint8_t *s6out, uint8_t *d6out, gf_pipeline_out *out,
                                                      uint8_t *nd6, uint8_t *snap_out, unsigned long long *stats) {
    extern __shared__ uint4 lds_rows[];
    uint8_t *rows = reinterpret_cast<uint8_t *>(lds_rows);
    __shared__ uint32_t sl[272];
    Stats st{sl};
    if (stats) st.init();
    const uint32_t S = fr.snap_stride;
    const uint32_t b0 = blockIdx.x * NT;
    const uint32_t nb = fr.n - b0 < NT ? fr.n - b0 : NT;
    const size_t bytes = (size_t)nb * S;
    {
        const uint8_t *src = fr.snap + (size_t)b0 * S;
        size_t k0 = 0;
        if (P.vec_copy) {
            const size_t nv = bytes / 16;
            for (size_t k = threadIdx.x; k < nv; k += NT) lds_rows[k] = reinterpret_cast<const uint4 *>(src)[k];
            k0 = nv * 16;
        }
        for (size_t k = k0 + threadIdx.x; k < bytes; k += NT) rows[k] = src[k];
    }
    __syncthreads();
    const uint32_t i = b0 + threadIdx.x;
    bool scnt = false;                                  // the lane's counter-block entry
    uint32_t sreason = 0, saction = 0, slen = 0, sab = 0;
    if (i < fr.n) {
        const uint32_t len = fr.len[i];
        const uint32_t cap = S < len ? S : len;
        Row w{rows + (size_t)threadIdx.x * S, cap};
        PktHdr h;
        parse_row(w.p, cap, len, h);
        const uint32_t et = h.et;
        const PktHdrA ha{h, flow_hash ? flow_hash[i] : 0u};
        gf_pipeline_out o{};
        uint32_t n6[4] = {0, 0, 0, 0};
        uint32_t sec = 0, ifx = 0, lxc = 0, mapped = 0, ndport = 0;
        uint32_t ab = 24 + 34;                          // output record, header bytes parsed
        bool tail = false;
        do {
            if (P.has_xdp && xdp_verdict(P.x, ha, len, et, ab) == XDP_DROP_) {
                o.stage = GF_STAGE_XDP; o.action = XDP_DROP_;
                break;
            }
            if (P.has_lb) {
                gf_lb_out lo{};
                uint32_t kd = 0;
                int ret = TC_OK;
                bool v6 = false;
                ab += 12;
                if (et == 0x86DD) {
                    if (!(P.L.flags & GF_LB_F_NO_IPV6)) { v6 = true; ab += 28; ret = lb_v6(P.L, ha, len, lo, n6, ab, kd); }
                } else if (et == 0x0800) {
                    if (!(P.L.flags & GF_LB_F_NO_IPV4)) ret = lb_v4(P.L, ha, len, lo, ab, kd);
                }
                if (ret < 0 || ret == TC_SHOT) {
                    o.stage = GF_STAGE_LB; o.action = TC_SHOT; o.reason = (uint8_t)(-ret);
                    n6[0] = n6[1] = n6[2] = n6[3] = 0;
                    break;
                }
                if (ret == TC_REDIRECT) {
                    pipe_lb_rewrite(w, len, h, v6, lo, n6, kd, ab);
                    o.slave = lo.slave; o.rev_nat = lo.rev_nat; o.dport = lo.new_dport;
                    o.daddr4 = v6 ? 0u : lo.new_daddr4;
                    o.flags |= GF_PIPE_F_LB;
                    if (P.L.flags & GF_LB_F_REDIRECT) {
                        o.stage = GF_STAGE_LB; o.action = TC_REDIRECT; o.ifindex_lo = (uint16_t)P.lb_redirect_ifindex;
                        break;
                    }
                } else {
                    n6[0] = n6[1] = n6[2] = n6[3] = 0;
                }
            }
            if (P.tcap_in) {                            // from_netdev's send_trace_notify (bpf_netdev.c:436)
                uint8_t *d = P.tcap_in + (size_t)i * GF_TRACE_PAYLOAD_LEN;
                const uint32_t cb = S < GF_TRACE_PAYLOAD_LEN ? S : GF_TRACE_PAYLOAD_LEN;
                if (P.vec_copy) {
                    for (uint32_t k = 0; k < cb; k += 16)
                        *reinterpret_cast<uint4 *>(d + k) = *reinterpret_cast<const uint4 *>(w.p + k);
                } else {
                    for (uint32_t k = 0; k < cb; k++) d[k] = w.p[k];
                }
            }
            const int r = pipe_netdev(P.nd, w, h, et, len, sec, ifx, lxc, mapped, ndport, ab);
            if (mapped) { o.flags |= GF_PIPE_F_PORTMAP; o.dport = (uint16_t)ndport; }
            o.stage = GF_STAGE_NETDEV;
            if (r == ND_TAILCALL) { o.stage = GF_STAGE_POLICY; o.lxc_id = (uint16_t)lxc; tail = true; }
            else if (r == ND_ICMP6_TE) { o.action = TC_REDIRECT; o.flags |= GF_PIPE_F_ICMP6_TE; }
            else if (r < 0 || r == TC_SHOT) { o.action = TC_SHOT; o.reason = (uint8_t)(-r); }
            else o.action = (uint8_t)r;
        } while (0);
        // handle_policy's input: the rewritten header, re-parsed (k_ing_pack fused)
        gf_rec rr;
        uint32_t key;
        const uint32_t tci = tc_index ? tc_index[i] : 0u;
        if (tail) {
            PktHdr h2;
            parse_row(w.p, cap, len, h2);
            key = pack_rec(i, h2.et, len, h2.sa, h2.da, h2.w0, h2.w3, h2.l4, h2.proto, sec, ifx, slot_of[lxc & 0xffffu],
                           tci, false, true, h2.s6, h2.d6, rr);
            // the front's record flags (every GF_PIPE_F_* bit: the top three of the byte)
            // ride along in cls bits 4-6 for k_ing_groups' write-only completion (IngCtx::pout_wo)
            static_assert(((GF_PIPE_F_ICMP6_TE | GF_PIPE_F_LB | GF_PIPE_F_PORTMAP) & ~0xE0u) == 0,
                          "the pipeline's front flags must fit the top three bits of the flags byte");
            rr.cls |= (uint8_t)(((o.flags & 0xE0u) >> 5) << 4);
            if (h2.et == 0x86DD) {                       // both addresses in one 32-B piece (a6_stride 32)
                reinterpret_cast<uint4 *>(s6out)[2 * (size_t)i] = make_uint4(h2.s6[0], h2.s6[1], h2.s6[2], h2.s6[3]);
                reinterpret_cast<uint4 *>(d6out)[2 * (size_t)i] = make_uint4(h2.d6[0], h2.d6[1], h2.d6[2], h2.d6[3]);
            }
        } else {
            key = pack_rec(i, et, len, 0, 0, 0, 0, 0, 0, 0, 0, 0, tci, true, true, h.s6, h.d6, rr);
        }
        rec[i] = rr;
        keys[i] = key;
        out[i] = o;
        if (nd6) reinterpret_cast<uint4 *>(nd6)[i] = make_uint4(n6[0], n6[1], n6[2], n6[3]);
        sab = ab;                                       // a tail-called packet: handle_policy counts it
        if (!tail) { scnt = true; sreason = o.reason; saction = o.action; slen = len; }
    }
    if (stats) st.pkt_wave(scnt, sreason, saction, slen, sab);
    if (snap_out) {
        __syncthreads();
        uint8_t *dst = snap_out + (size_t)b0 * S;
        size_t k0 = 0;
        if (P.vec_copy) {
            const size_t nv = bytes / 16;
            for (size_t k = threadIdx.x; k < nv; k += NT) reinterpret_cast<uint4 *>(dst)[k] = lds_rows[k];
            k0 = nv * 16;
        }
        for (size_t k = k0 + threadIdx.x; k < bytes; k += NT) dst[k] = rows[k];
    }
    if (stats) st.flush(stats);
}

// ---- ingest re-partition (real traffic on N GPUs): the owner rank of each
// frame is the rank of its flow group, the unordered address pair that the
// CT of handle_policy sees, i.e. after bpf_lb's translation (stateless, so it
// can run before the exchange).  Same rule as the synthetic stream's
// (cilium_amd/stream.py pair_rank): fmix64 of (max << 32 | min) of the
// host-order addresses, mod the rank count.  Frames that cannot reach
// conntrack stay on their rank.
__device__ __forceinline__ uint32_t pair_rank4(uint32_t sa_raw, uint32_t da_raw, uint32_t world) {
    const uint64_t a = __builtin_bswap32(sa_raw), b = __builtin_bswap32(da_raw);
    uint64_t x = ((a < b ? b : a) << 32) | (a < b ? a : b);
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)(x & 0xffffffffull) % world;
}
// lb_v6's translated address (d6 unchanged unless it translates); kept out of
// line: inlined into k_partition, the hipcc of this image merged the target's
// third word with the lookup key's (observed on gfx950, the parity test pins it)
__device__ __attribute__((noinline)) void lb_v6_daddr(const LbDev &L, const PktHdr &h, uint32_t fh, uint32_t len,
                                                      uint32_t *d6) {
    const PktHdrA ha{h, fh};
    gf_lb_out lo{};
    uint32_t n6[4], ab = 0, kd = 0;
    if (lb_v6(L, ha, len, lo, n6, ab, kd) == TC_REDIRECT)
        for (int k = 0; k < 4; k++) d6[k] = n6[k];
}
__global__ __launch_bounds__(BLOCK) void k_partition(gf_frames fr, const uint32_t *flow_hash, PipeDev P, uint32_t self,
                                                     uint32_t world, uint32_t *owner, uint32_t *counts) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= fr.n) return;
    const uint32_t len = fr.len[i], S = fr.snap_stride;
    const uint32_t cap = S < len ? S : len;
    PktHdr h;
    parse_row(fr.snap + (size_t)i * S, cap, len, h);
    const PktHdrA ha{h, flow_hash ? flow_hash[i] : 0u};
    uint32_t r = self, ab = 0, kd = 0;
    if (h.et == 0x0800 && len >= 34) {
        uint32_t da = h.da;
        if (P.has_lb && !(P.L.flags & GF_LB_F_NO_IPV4)) {
            gf_lb_out lo{};
            if (lb_v4(P.L, ha, len, lo, ab, kd) == TC_REDIRECT) da = lo.new_daddr4;
        }
        r = pair_rank4(h.sa, da, world);
    } else if (h.et == 0x86DD && len >= 54) {
        // lb_v6 leaves d6 alone unless it translates (then it writes all four words)
        uint32_t d6[4] = {h.d6[0], h.d6[1], h.d6[2], h.d6[3]};
        if (P.has_lb && !(P.L.flags & GF_LB_F_NO_IPV6)) lb_v6_daddr(P.L, h, ha.fh, len, d6);
        r = gf_pair_hash6(h.s6, d6) % world;
    }
    owner[i] = r;
    atomicAdd(&counts[r], 1u);
}

// ================================================================ CT garbage collection / LRU eviction
// ctmap.GC / Flush (pkg/maps/ctmap/ctmap.go:277-368, GCFilterByTime): delete every
// entry with lifetime < filter_time.  The LRU stand-in (below) deletes by the same
// sweep with two cutoffs: closing entries (rx_closing or tx_closing set) with
// lifetime < cut_c, the others with lifetime < cut_o.  On the device the sweep
// also compacts each probe cluster (a maximal run of non-EMPTY slots) in place,
// so deleted entries and the tombstones of ct_delete leave EMPTY slots behind:
// k_gc_starts marks the cluster starts (a non-EMPTY slot after an EMPTY one) on
// the unmodified table, then k_gc_clusters walks each cluster with one lane,
// dropping deleted entries and tombstones and moving every live entry to the
// first EMPTY slot at or after its home — the invariant lookups rely on (no
// EMPTY slot between a key's home and the key) holds after the move.
// Cutoffs live in device memory so an eviction decided on the device (no host
// round trip) runs the same two kernels; active == 0 makes them no-ops.
struct GcCut {
    unsigned long long c, o;      // closing / other entries: deleted iff their age key < cut
    uint32_t active;
    uint32_t lru;                 // age key: 0 = lifetime (ctmap.GC), 1 = last use (the LRU stand-in)
};
__global__ __launch_bounds__(BLOCK) void k_gc_starts(gf_htab_desc d, uint32_t *bits, const GcCut *cut) {
    if (!cut->active) return;
    const uint64_t nw = (d.mask + 1 + 31) / 32;
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t m = 0;
        uint64_t i0 = w * 32;
        uint32_t prev = d.slots[((i0 - 1) & d.mask) * d.slot_size + d.ksz];
        for (int k = 0; k < 32; k++) {
            uint64_t i = i0 + k;
            if (i > d.mask) break;
            uint32_t st = d.slots[i * d.slot_size + d.ksz];
            if (st != GF_SLOT_EMPTY && prev == GF_SLOT_EMPTY) m |= 1u << k;
            prev = st;
        }
        bits[w] = m;
    }
}

__device__ __forceinline__ void gc_move(const gf_htab_desc &d, uint64_t from, uint64_t to, uint32_t vstride) {
    uint8_t *a = d.slots + from * d.slot_size, *b = d.slots + to * d.slot_size;
    for (uint32_t k = 0; k < d.slot_size; k += 16) *reinterpret_cast<uint4 *>(b + k) = *reinterpret_cast<const uint4 *>(a + k);
    if (vstride) {
        uint8_t *va = d.vals + from * vstride, *vb = d.vals + to * vstride;
        if (vstride % 16 == 0)
            for (uint32_t k = 0; k < vstride; k += 16) *reinterpret_cast<uint4 *>(vb + k) = *reinterpret_cast<const uint4 *>(va + k);
        else
            for (uint32_t k = 0; k < vstride; k += 4) *reinterpret_cast<uint32_t *>(vb + k) = *reinterpret_cast<const uint32_t *>(va + k);
    }
    a[d.ksz] = GF_SLOT_EMPTY;
}

// lt_off: byte offset of ct_entry.lifetime within the value bytes ht_val points at
// (0 in the CT codec's hot block, 32 in the reference layout); the flags word
// follows it in both.  res[0] += deleted entries, res[1] += tombstones cleared.
// The time of an entry's last update: every writer of ct_entry.lifetime sets it to
// now + the timeout its flags select (conntrack.h:47-62, 127, 527): CT_CLOSE_TIMEOUT
// once both directions close, CT_DEFAULT_LIFETIME after a non-SYN packet, else
// CT_SYN_TIMEOUT.  lifetime - that timeout is exact to the second.
__device__ __forceinline__ long long ct_last_use(uint32_t lt, uint32_t fl) {
    const uint32_t to = ((fl & F_RX_CLOSING) && (fl & F_TX_CLOSING)) ? 10u : ((fl & F_SEEN_NON_SYN) ? 43200u : 300u);
    return (long long)lt - (long long)to;
}
__device__ __forceinline__ bool gc_kill(uint32_t lt, uint32_t fl, const GcCut &c) {
    const long long k = c.lru ? ct_last_use(lt, fl) : (long long)lt;
    const unsigned long long cut = (fl & (F_RX_CLOSING | F_TX_CLOSING)) ? c.c : c.o;
    return k < 0 || (unsigned long long)k < cut;
}
__global__ __launch_bounds__(BLOCK) void k_gc_clusters(gf_htab_desc d, uint32_t mode, uint32_t lt_off, const GcCut *cutp,
                                                       const uint32_t *bits, unsigned long long *res) {
    if (!cutp->active) return;
    const GcCut cut = *cutp;
    const uint64_t nw = (d.mask + 1 + 31) / 32;
    const uint32_t vstride = d.vals ? (d.sstride ? d.sstride : d.vsz) : 0u;
    uint32_t dead = 0, tombs = 0;
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t m = bits[w];
        while (m) {
            const int k = __builtin_ctz(m);
            m &= m - 1;
            uint64_t j = w * 32 + k;
            // hole: a slot of this cluster before j was emptied by this walk.  Until
            // then every slot from the cluster start to j is occupied, so the entry
            // at j (whose home lies in that range) cannot move: no rehash needed.
            bool hole = false;
            for (;;) {
                uint8_t *sl = d.slots + j * d.slot_size;
                const uint32_t st = sl[d.ksz];
                if (st == GF_SLOT_EMPTY) break;
                if (st == GF_SLOT_TOMB || st == GF_SLOT_FREE) {
                    sl[d.ksz] = GF_SLOT_EMPTY;
                    tombs++;
                    hole = true;
                } else {
                    const uint8_t *v = ht_val(d, j) + lt_off;
                    const uint32_t lt = *reinterpret_cast<const uint32_t *>(v);
                    const uint32_t fl = *reinterpret_cast<const uint16_t *>(v + 4);
                    if (gc_kill(lt, fl, cut)) {
                        sl[d.ksz] = GF_SLOT_EMPTY;
                        dead++;
                        hole = true;
                    } else if (hole) {
                        uint32_t kw[10];
                        for (uint32_t q = 0; q < 10; q++) kw[q] = 0;
                        for (uint32_t q = 0; q < d.ksz; q += 4) {       // slots are 4-B aligned
                            const uint32_t x = *reinterpret_cast<const uint32_t *>(sl + q);
                            kw[q >> 2] = d.ksz - q >= 4 ? x : (x & ((1u << (8 * (d.ksz - q))) - 1u));
                        }
                        const uint64_t home = gf_home_slot(gf_key_hash(kw, d.ksz, mode), d.mask, d.slot_size);
                        for (uint64_t p = home; p != j; p = (p + 1) & d.mask) {
                            if (d.slots[p * d.slot_size + d.ksz] == GF_SLOT_EMPTY) { gc_move(d, j, p, vstride); break; }
                        }
                    }
                }
                j = (j + 1) & d.mask;
            }
        }
    }
    if (dead) atomicAdd(&res[0], (unsigned long long)dead);
    if (tombs) atomicAdd(&res[1], (unsigned long long)tombs);
}

// ---- LRU stand-in (CT maps are BPF_MAP_TYPE_LRU_HASH, bpf/bpf_lxc.c:53-75;
// ctmap.go:38-39).  The kernel never fails an LRU insert: it evicts from per-CPU
// LRU lists, taking entries off the tail of an inactive list it keeps about as
// long as the active one (kernel/bpf/bpf_lru_list.c, not in /root/reference) — in
// effect from the older half of the entries, in an order nothing reproduces.
// Here an LRU CT map may exceed max_entries inside a batch (the slot array has
// room); at the end of every classify call that inserts into it, once the device
// count exceeds the high-water mark HW = max_entries - max_entries / 8, a
// deterministic *hand* evicts (the oracle restates it, o_ct_lru_evict):
//  * age key of an entry: 0 if its last use (ct_last_use) lies before time 0,
//    else closing entries (rx_closing | tx_closing) in [0, 65536) and the others
//    in [65536, 131072), each by last use in one-second bins relative to now (bin
//    0 = last used 65535 s or more ago);
//  * home line of an entry: its key's home slot in this table (gf_home_slot of the
//    CT hash) / slots per 128-B line; NL lines in all;
//  * the sample: the entries homed in the SL lines from where the hand stands (SL
//    = NL when NL <= 65536, else max(65536, NL >> 10)), the lines it passes next.  K = the smallest age key covering half of
//    the sample (its older half is eligible); es = the sample entries with age key
//    <= K.  A window that holds no entry (only keys chosen to avoid those lines)
//    is replaced by the whole table (SL = NL);
//  * the lines for q entries: ceil(q * SL / es);
//  * round 0 (count > HW): q = count - HW; round 1 (only while count >
//    max_entries): q = count - HW again, for what round 0's estimate left; round 2
//    (only while count > max_entries still): the rest of the table.  Each round
//    passes its lines (at most NL - the lines already passed) from where the hand
//    stands and deletes every entry with age key <= K homed in them.
// A map that runs at HW deletes in each call about what the call inserted, so
// the work per call follows the call's inserts, not the table; the count is back
// at <= max_entries after every call unless fewer than count - max_entries
// entries are eligible in the whole table (documented bound, include/gpuflow.h).
// A deleted slot turns EMPTY when every slot after it up to the end of its probe
// cluster is gone too (the probe invariant holds), else FREE (claimed by later
// device inserts, gf_common.h); tombstones the hand passes are cleared the same
// way.  Key bytes of the cleared slots are zeroed.  Every eviction is logged
// (gf_ct_evict_log: batch number, now, K, the hand's first line, lines passed,
// entries deleted).
#ifndef GF_LRU_NT
#define GF_LRU_NT 0         // the eviction passes' slot loads nontemporal (same-box A/B r6e: the hand 7-12 % slower,
                            // the next k_ing_groups unchanged: off)
#endif
#define GF_LRU_BINS 65536u
#define GF_LRU_LOGCAP 4096u
#define GF_LRU_SAMPLE_SHIFT 10
#define GF_LRU_SAMPLE_MIN 65536ull
#define GF_LRU_ROUNDS 3u
#define GF_LRU_HT 256u                  // k_lru_hand block
#define GF_LRU_CHUNK 1024u              // k_lru_hand: slots a block decides together (CT6; CT4 twice that)
struct LruLog { uint32_t seq, now, age_cut, pad; unsigned long long hand, lines, evicted; };
#define GF_LRU_GROUPS (2u * GF_LRU_BINS / 64u)
struct LruDev {
    uint32_t hist[2 * GF_LRU_BINS];     // the sample's age histogram
    uint32_t coarse[GF_LRU_GROUPS];     // its sums per group of 64 bins (k_lru_plan reads these first)
    GcCut cut;                          // gf_ct_gc (k_gc_*)
    unsigned long long res[2];          // gf_ct_gc: entries deleted, tombstones cleared
    uint32_t flag;                      // this call evicts (count > HW)
    uint32_t K;                         // age keys [0, K] are eligible
    unsigned long long es;              // eligible sample entries (0: empty sample, age-blind)
    unsigned long long hand;            // the hand's next home line (kept across calls)
    unsigned long long cnt0;            // the count when this call's eviction began
    unsigned long long sl;              // the lines the sample covered (the window, or the table)
    uint32_t wide, pad1;                // the window held no entry: sample the whole table
    unsigned long long kills[GF_LRU_ROUNDS];   // entries deleted by each round
    unsigned long long cleared;         // tombstones / FREE slots rewritten (diagnostics)
    uint32_t nlog, pad;
    LruLog log[GF_LRU_LOGCAP];
};
// The sampled home lines of a table of nl lines.
__host__ __device__ __forceinline__ uint64_t lru_sample_lines(uint64_t nl) {
    if (nl <= GF_LRU_SAMPLE_MIN) return nl;
    const uint64_t s = nl >> GF_LRU_SAMPLE_SHIFT;
    return s > GF_LRU_SAMPLE_MIN ? s : GF_LRU_SAMPLE_MIN;
}
__host__ __device__ __forceinline__ unsigned long long lru_high_water(uint32_t max_entries) {
    return (unsigned long long)(max_entries - max_entries / 8u);
}
// Round r of this call: the hand's first line and the lines it passes, from the
// call's state (count at the start, K / es, the earlier rounds' deletions).  Every
// block of a round's launches computes the same values; nothing is written.
struct LruRound { unsigned long long h0, lines; };
__device__ __forceinline__ LruRound lru_round(const LruDev *L, uint32_t r, uint32_t max_entries, uint64_t nl) {
    const unsigned long long hw = lru_high_water(max_entries), es = L->es, sl = L->sl;
    unsigned long long c = L->cnt0, passed = 0, h = L->hand;
    LruRound o{h, 0ull};
    if (!L->flag) return o;
    for (uint32_t j = 0; j <= r; j++) {
        if (j) c -= L->kills[j - 1];
        unsigned long long ln = 0;
        if ((j == 0 ? c > hw : c > (unsigned long long)max_entries) && passed < nl) {
            if (j + 1 < GF_LRU_ROUNDS) {
                const unsigned long long q = c - hw;
                ln = es ? (q * sl + es - 1) / es : nl;  // es >= 1: the sample holds entries
                if (ln > nl - passed) ln = nl - passed;
            } else {
                ln = nl - passed;
            }
        }
        if (j == r) { o.h0 = h; o.lines = ln; return o; }
        h = (h + ln) % nl;
        passed += ln;
    }
    return o;
}
__device__ __forceinline__ uint32_t lru_age_key(uint32_t lt, uint32_t fl, uint32_t now) {
    const long long lu = ct_last_use(lt, fl);
    if (lu < 0) return 0u;
    long long b = lu - ((long long)now - (long long)(GF_LRU_BINS - 1));
    b = b < 0 ? 0 : (b > (long long)(GF_LRU_BINS - 1) ? (long long)(GF_LRU_BINS - 1) : b);
    return ((fl & (F_RX_CLOSING | F_TX_CLOSING)) ? 0u : GF_LRU_BINS) + (uint32_t)b;
}
// One CT slot as the eviction pass reads it.  KIND 1: the CT v4 slot (32 B: key
// 14, state at 14, hot value at 16 with the lifetime first) as two 16-B loads;
// KIND 2: the CT v6 slot (64 B: key 40, state at 40, hot value at 48) as four.
template <int KIND>
struct LruSlot {
    static constexpr uint32_t SZ = KIND == 2 ? 64u : 32u, SPL = 128u / SZ, KW = KIND == 2 ? 10 : 4;
    uint32_t kw[KW];
    uint32_t st = GF_SLOT_EMPTY, lt = 0, fl = 0;
    // nontemporal loads: the eviction passes stream GBs of slots per call, which must
    // not push the policy maps and hot CT lines of the next launch out of L2 / MALL
    __device__ __forceinline__ static uint4 ld(const uint8_t *p) { return GF_LRU_NT ? gload_nt16(p) : gload<uint4>(p); }
    __device__ __forceinline__ void load(const gf_htab_desc &d, uint64_t i) {
        const uint8_t *p = d.slots + i * SZ;
        if constexpr (KIND == 2) {
            const uint4 a = ld(p), b = ld(p + 16), c = ld(p + 32), e = ld(p + 48);
            kw[0] = a.x; kw[1] = a.y; kw[2] = a.z; kw[3] = a.w; kw[4] = b.x; kw[5] = b.y; kw[6] = b.z; kw[7] = b.w;
            kw[8] = c.x; kw[9] = c.y;
            st = c.z & 0xffu; lt = e.x; fl = e.y & 0xffffu;
        } else {
            const uint4 a = ld(p), b = ld(p + 16);
            kw[0] = a.x; kw[1] = a.y; kw[2] = a.z; kw[3] = a.w & 0xffffu;
            st = (a.w >> 16) & 0xffu; lt = b.x; fl = b.y & 0xffffu;
        }
    }
    __device__ __forceinline__ uint64_t home_line(const gf_htab_desc &d, uint32_t mode) const {
        return gf_home_slot(gf_key_hash(kw, KIND == 2 ? 40u : 14u, mode), d.mask, SZ) / SPL;
    }
};
// A deleted / cleared slot: key bytes zeroed, state EMPTY or FREE (16-B stores).
template <int KIND>
__device__ __forceinline__ void lru_clear_slot(const gf_htab_desc &d, uint64_t j, uint32_t st) {
    uint8_t *p = d.slots + j * LruSlot<KIND>::SZ;
    if constexpr (KIND == 2) {
        gstore<uint4>(p + 32, make_uint4(0u, 0u, st, 0u));
        gstore<uint4>(p, make_uint4(0u, 0u, 0u, 0u));
        gstore<uint4>(p + 16, make_uint4(0u, 0u, 0u, 0u));
    } else {
        gstore<uint4>(p, make_uint4(0u, 0u, 0u, st << 16));
    }
}
// The chain after a classify call: k_lru_sample, k_lru_plan, k_lru_hand x 2 per
// round (GF_LRU_ROUNDS), k_lru_end.  Each launch exits at once unless the count
// exceeds HW (and a round's, unless the round passes lines).  The histogram is zero
// between calls (cleared by k_lru_plan after its scan; zero at allocation).
// Age histogram of the sample: wave-aggregated (a wave's entries mostly share a
// bin), then counted per block in LDS and flushed with one global add per
// non-zero bin.  The last GF_LRU_WIN seconds of each class are counted directly
// (one LDS slot per bin, no collisions): a steady stream's live entries were all
// last used within its flows' lifetimes.  Older bins go through a block-local
// LDS cache: a 64-bit {bin, count} word per line (Fibonacci-hashed), updated by
// CAS; a bin that misses takes the line over and flushes the previous bin's
// count with one global add.  (An XOR-folded index once mapped a closing bin and
// the non-closing bin 32 s from it to one line: every wave alternated them and
// sent a global add to a few hot addresses.)
#define GF_LRU_LDS 2048u
#define GF_LRU_WIN 4096u
#define GF_LRU_HB 1024u                 // k_lru_sample block: 16 waves share the LDS bins
// One histogram add; its group's sum goes to the block's LDS copy of the sums
// (flushed once per block: a sample's entries fall in a few groups, whose global
// words every block would otherwise hit for each of its bins).
__device__ __forceinline__ void lru_hist_put(LruDev *L, uint32_t *cg, uint32_t bin, uint32_t c) {
    atomicAdd(&L->hist[bin], c);
    atomicAdd(&cg[bin >> 6], c);
}
// key: the entry's age key, ~0u for none.  Wave-uniform call.
__device__ __forceinline__ void lru_hist_add(LruDev *L, unsigned long long *line, uint32_t *win, uint32_t *cg,
                                             uint32_t key) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t kb = key & (GF_LRU_BINS - 1u);
    const bool inwin = key != ~0u && kb >= GF_LRU_BINS - GF_LRU_WIN;
    if (inwin) atomicAdd(&win[(key >> 16) * GF_LRU_WIN + kb - (GF_LRU_BINS - GF_LRU_WIN)], 1u);
    uint64_t rem = __ballot(key != ~0u && !inwin);
    while (rem) {
        const uint32_t lead = (uint32_t)__ffsll((unsigned long long)rem) - 1u;
        const uint32_t k = __shfl(key, (int)lead);
        const uint64_t m = __ballot(key == k) & rem;
        if (lane == lead) {
            const uint32_t n = (uint32_t)__popcll(m), h = (k * 0x9E3779B1u) >> (32 - 11);
            unsigned long long cur = line[h];
            for (;;) {
                const uint32_t ck = (uint32_t)(cur >> 32);
                const unsigned long long want = ck == k ? cur + n : (((unsigned long long)k << 32) | n);
                const unsigned long long seen = atomicCAS(&line[h], cur, want);
                if (seen == cur) {
                    if (ck != k && ck != ~0u && (uint32_t)cur) lru_hist_put(L, cg, ck, (uint32_t)cur);
                    break;
                }
                cur = seen;
            }
        }
        rem &= ~m;
    }
}
// The sample: the sl home lines just ahead of the hand (the lines it passes next,
// so their density is the one its rounds are planned with; the whole table when
// sl = nl): slots [hand * SPL, (hand + sl) * SPL) mod NS and the rest of the probe
// cluster running past them (entries homed in the window; one wave walks it, at
// most to where the window starts again).
// wide: the whole table (launched after k_lru_plan found the window empty).
template <int KIND>
__device__ __forceinline__ void lru_sample_body(const gf_htab_desc &d, uint32_t mode, uint32_t now, LruDev *L,
                                                uint64_t sl, uint32_t max_entries, uint32_t wide) {
    if (wide ? !L->wide : (unsigned long long)*d.count <= lru_high_water(max_entries)) return;
    __shared__ unsigned long long line[GF_LRU_LDS];    // bin << 32 | count; bin ~0 = empty
    __shared__ uint32_t win[2 * GF_LRU_WIN];           // class * WIN + bin - (BINS - WIN)
    __shared__ uint32_t cg[GF_LRU_GROUPS];             // the block's group sums
    for (uint32_t k = threadIdx.x; k < GF_LRU_LDS; k += blockDim.x) line[k] = 0xffffffff00000000ull;
    for (uint32_t k = threadIdx.x; k < 2 * GF_LRU_WIN; k += blockDim.x) win[k] = 0;
    for (uint32_t k = threadIdx.x; k < GF_LRU_GROUPS; k += blockDim.x) cg[k] = 0;
    __syncthreads();
    constexpr uint32_t SPL = LruSlot<KIND>::SPL;
    const uint64_t ns = d.mask + 1, nl = ns / SPL;
    if (wide) sl = nl;
    const uint64_t n = sl * SPL, h0 = sl >= nl ? 0 : L->hand, P0 = h0 * SPL;
    auto in_window = [&](const LruSlot<KIND> &s) { return (s.home_line(d, mode) + nl - h0) % nl < sl; };
    for (uint64_t b0 = (uint64_t)blockIdx.x * GF_LRU_HB; b0 < n; b0 += (uint64_t)gridDim.x * GF_LRU_HB) {  // uniform trips
        const uint64_t i = b0 + threadIdx.x;
        uint32_t key = ~0u;
        if (i < n) {
            LruSlot<KIND> s;
            s.load(d, (P0 + i) & d.mask);
            if (s.st == GF_SLOT_FULL && in_window(s)) key = lru_age_key(s.lt, s.fl, now);
        }
        lru_hist_add(L, line, win, cg, key);
    }
    if (blockIdx.x == 0 && threadIdx.x < 64 && n < ns) {
        for (uint64_t q = n;; q += 64) {
            const uint64_t i = q + threadIdx.x;
            LruSlot<KIND> s;
            if (i < ns) s.load(d, (P0 + i) & d.mask);
            const uint64_t em = __ballot(s.st == GF_SLOT_EMPTY);
            const uint32_t stop = em ? (uint32_t)__ffsll((unsigned long long)em) - 1u : 64u;
            uint32_t key = ~0u;
            if (threadIdx.x < stop && s.st == GF_SLOT_FULL && in_window(s)) key = lru_age_key(s.lt, s.fl, now);
            lru_hist_add(L, line, win, cg, key);
            if (em || q + 64 >= ns) break;
        }
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < GF_LRU_LDS; k += blockDim.x) {
        const unsigned long long v = line[k];
        if ((uint32_t)(v >> 32) != ~0u && (uint32_t)v) lru_hist_put(L, cg, (uint32_t)(v >> 32), (uint32_t)v);
    }
    for (uint32_t k = threadIdx.x; k < 2 * GF_LRU_WIN; k += blockDim.x)
        if (win[k]) lru_hist_put(L, cg, (k / GF_LRU_WIN) * GF_LRU_BINS + GF_LRU_BINS - GF_LRU_WIN + k % GF_LRU_WIN, win[k]);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < GF_LRU_GROUPS; k += blockDim.x)
        if (cg[k]) atomicAdd(&L->coarse[k], cg[k]);
}
template <int KIND>
__global__ __launch_bounds__(GF_LRU_HB) void k_lru_sample(gf_htab_desc d, uint32_t mode, uint32_t now, LruDev *L,
                                                          uint64_t sl, uint32_t max_entries, uint32_t wide) {
    lru_sample_body<KIND>(d, mode, now, L, sl, max_entries, wide);
}
// K and es from the sample's histogram, the count the call starts from, and the
// histogram cleared for the next call (one block).
// wide = 0: the window's sample; an empty one (sl < nl) sets L->wide for the
// whole-table sample and its plan (wide = 1) instead of planning.
__device__ __forceinline__ void lru_plan_body(const uint32_t *count, uint32_t max_entries, LruDev *L, uint64_t sl,
                                              uint64_t nl, uint32_t wide) {
    const uint32_t c = *count;
    const uint32_t t = threadIdx.x;
    if (wide) {
        if (!L->wide) return;
        sl = nl;
    } else if ((unsigned long long)c <= lru_high_water(max_entries)) {
        if (t == 0) L->flag = 0u;
        return;
    }
    // the 2048 group sums (two per thread), a block scan, then one wave finds the
    // median's bin among its group's 64; only the groups that hold entries are cleared
    constexpr uint32_t NB = 2 * GF_LRU_BINS;
    __shared__ unsigned long long part[1024];
    __shared__ uint32_t s_k, s_g;
    __shared__ unsigned long long s_es, s_before;
    const uint32_t g0 = L->coarse[2 * t], g1 = L->coarse[2 * t + 1];
    if (t == 0) { s_k = NB - 1; s_es = 0; s_g = ~0u; s_before = 0; }
    {                                                   // inclusive scan: in each wave, then over the 16 waves
        const uint32_t lane = t & 63u, wv = t >> 6;
        unsigned long long v = (unsigned long long)g0 + g1;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long u = __shfl_up(v, o);
            if (lane >= (uint32_t)o) v += u;
        }
        __shared__ unsigned long long wsum[16];
        if (lane == 63) wsum[wv] = v;
        __syncthreads();
        unsigned long long off = 0;
        for (uint32_t q = 0; q < wv; q++) off += wsum[q];
        part[t] = v + off;
        __syncthreads();
    }
    const unsigned long long total = part[1023], need = (total + 1) / 2, before = t ? part[t - 1] : 0ull;
    if (!total && sl < nl) {                            // no entry in the window (histogram still all zero)
        if (t == 0) { L->wide = 1u; L->flag = 0u; }
        return;
    }
    if (total && before < need && part[t] >= need) {    // the median lies in group 2t or 2t + 1
        const bool first = before + g0 >= need;
        s_g = first ? 2 * t : 2 * t + 1;
        s_before = first ? before : before + g0;
    }
    __syncthreads();
    if (t < 64 && s_g != ~0u) {                          // wave 0: the median group's bins, one per lane
        const uint32_t v = L->hist[s_g * 64u + t];
        uint32_t inc = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(inc, o);
            if (t >= (uint32_t)o) inc += u;
        }
        const uint64_t hit = __ballot(s_before + inc >= need);
        if (t == (uint32_t)__ffsll((unsigned long long)hit) - 1u) { s_k = s_g * 64u + t; s_es = s_before + inc; }
    }
    __syncthreads();
    // clear for the next sample: the bins of the groups that hold entries, and the sums
    for (uint32_t q = 0; q < 2; q++) {
        const uint32_t g = 2 * t + q;
        if (!(q ? g1 : g0)) continue;
        uint4 *hb = reinterpret_cast<uint4 *>(L->hist + g * 64u);
#pragma unroll
        for (uint32_t k = 0; k < 16; k++) hb[k] = make_uint4(0u, 0u, 0u, 0u);
        L->coarse[g] = 0u;
    }
    if (t == 0) {
        L->K = s_k; L->es = s_es; L->cnt0 = c; L->sl = sl; L->wide = 0u; L->flag = 1u; L->cleared = 0;
        for (uint32_t r = 0; r < GF_LRU_ROUNDS; r++) L->kills[r] = 0;
    }
}
__global__ __launch_bounds__(1024) void k_lru_plan(const uint32_t *count, uint32_t max_entries, LruDev *L, uint64_t sl,
                                                   uint64_t nl, uint32_t wide) {
    lru_plan_body(count, max_entries, L, sl, nl, wide);
}
// The hand over this round's lines: the slots from the first line's first slot,
// lines * SPL of them, in chunks (GF_LRU_CHUNK slots, twice that for CT4), plus the cluster running past
// the last one (entries homed in the range).  Launched twice, PAR = 0 for the
// even chunks and 1 for the odd ones: a chunk's last slots turn EMPTY only if the
// slots after it, up to the cluster's end, are all gone too, which the block
// reads from the next chunk (at most one chunk ahead, else it keeps them FREE) —
// untouched in the even launch, final in the odd one, so no read races a write.
// The slots past the last chunk are read and written by its block alone (there
// deleted entries turn FREE).  Codes: 0 EMPTY, 1 kept, 2 deleted now, 3 a
// tombstone or FREE slot (cleared).
template <int KIND, int PAR>
__device__ __forceinline__ void lru_hand_body(const gf_htab_desc &d, uint32_t mode, uint32_t now, LruDev *L,
                                              uint64_t nl, uint64_t sl, uint32_t max_entries, uint32_t round) {
    if (!L->flag) return;
    const LruRound R = lru_round(L, round, max_entries, nl);
    const unsigned long long lines = R.lines;
    if (!lines) return;
    using S = LruSlot<KIND>;
    // slots a block decides together: 8 per thread for the 32-B CT4 slots, 4 for the
    // 64-B CT6 slots (the same 64 KB of loads in flight per block)
    constexpr uint32_t CH = KIND == 2 ? GF_LRU_CHUNK : 2 * GF_LRU_CHUNK, U = CH / GF_LRU_HT;
    const uint32_t K = L->K;
    const unsigned long long h0 = R.h0;
    const uint64_t ns = d.mask + 1, P0 = h0 * S::SPL, NP = lines * S::SPL;
    const bool whole = NP >= ns;
    const uint64_t nch = (NP + CH - 1) / CH;
    __shared__ uint8_t code[2 * GF_LRU_CHUNK];
    __shared__ uint32_t s_ef, s_kills, s_clr;
    auto code_of = [&](const S &s) -> uint32_t {
        if (s.st == GF_SLOT_EMPTY) return 0u;
        if (s.st == GF_SLOT_TOMB || s.st == GF_SLOT_FREE) return 3u;
        if (s.st != GF_SLOT_FULL || lru_age_key(s.lt, s.fl, now) > K) return 1u;
        const uint64_t hl = s.home_line(d, mode);
        return (hl + nl - h0) % nl < lines ? 2u : 1u;
    };
    if (threadIdx.x == 0) { s_kills = 0; s_clr = 0; }
    uint32_t kills = 0, clr = 0;
    const uint32_t lane = threadIdx.x & 63u;
    for (uint64_t c = 2 * (uint64_t)blockIdx.x + PAR; c < nch; c += 2 * (uint64_t)gridDim.x) {
        const uint64_t base = c * CH;
        const uint32_t cnt = (uint32_t)(NP - base < CH ? NP - base : CH);
        const bool last = base + cnt == NP;
        uint32_t mine[U], ost[U];
        // wave 0 also loads the first 64 slots after the chunk with the chunk's own
        // loads (at low load they decide the chunk's trailing run): one round trip
        // less per chunk.  Nothing writes them during this launch before wave 0 reads
        // them below (the next chunk is the other launch's, and past the last chunk
        // only this block writes, after reading).
        S la;
        const bool look = threadIdx.x < 64 && !(last && whole);
        const uint64_t o0 = base + cnt + lane;
        if (look && o0 < ns) la.load(d, (P0 + o0) & d.mask);
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t off = u * GF_LRU_HT + threadIdx.x;
            mine[u] = 1u; ost[u] = GF_SLOT_FULL;
            if (off < cnt) {
                S s;
                s.load(d, (P0 + base + off) & d.mask);
                mine[u] = code_of(s);
                ost[u] = s.st;
                code[off] = (uint8_t)mine[u];
            }
        }
        __syncthreads();
        if (threadIdx.x < 64) {                          // wave 0: the slots after the chunk
            bool ef = false, decided = false;
            if (look) {
                for (uint64_t q = 0;; q += 64) {
                    if (!last && q >= CH) break;                           // undecided: the chunk's run stays FREE
                    const uint64_t o = base + cnt + q + lane;              // offset from P0
                    uint32_t cd = 0;
                    if (o < ns) {                                          // never back into the range
                        const uint64_t j = (P0 + o) & d.mask;
                        if (q) la.load(d, j);
                        cd = code_of(la);
                        if (last && cd == 2) { lru_clear_slot<KIND>(d, j, GF_SLOT_FREE); kills++; }
                    }
                    const uint64_t stop_m = __ballot(cd <= 1u);
                    if (!decided && stop_m) {
                        ef = __shfl(cd, (int)((uint32_t)__ffsll((unsigned long long)stop_m) - 1u)) == 0u;
                        decided = true;
                    }
                    if (!last && decided) break;
                    if (last && __ballot(cd == 0u)) break;                 // the cluster past the range ends
                }
            }
            if (lane == 0) s_ef = decided && ef ? 1u : 0u;
        }
        __syncthreads();
        const bool ef = s_ef != 0;
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t off = u * GF_LRU_HT + threadIdx.x;
            if (off >= cnt || mine[u] < 2u) continue;
            bool to_empty = ef;
            for (uint32_t k = off + 1; k < cnt; k++) {
                const uint32_t x = code[k];
                if (x <= 1u) { to_empty = x == 0u; break; }
            }
            const uint32_t nst = to_empty ? GF_SLOT_EMPTY : GF_SLOT_FREE;
            if (mine[u] == 2u) kills++;
            else if (ost[u] != nst) clr++;
            if (mine[u] == 2u || ost[u] != nst) lru_clear_slot<KIND>(d, (P0 + base + off) & d.mask, nst);
        }
        __syncthreads();                                 // code[] is the next chunk's
    }
    if (kills) atomicAdd(&s_kills, kills);
    if (clr) atomicAdd(&s_clr, clr);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_kills) atomicAdd(&L->kills[round], (unsigned long long)s_kills);
        if (s_clr) atomicAdd(&L->cleared, (unsigned long long)s_clr);
    }
}
template <int KIND, int PAR>
__global__ __launch_bounds__(GF_LRU_HT) void k_lru_hand(gf_htab_desc d, uint32_t mode, uint32_t now, LruDev *L,
                                                        uint64_t nl, uint64_t sl, uint32_t max_entries, uint32_t round) {
    lru_hand_body<KIND, PAR>(d, mode, now, L, nl, sl, max_entries, round);
}
// After the last round: the count, the hand, the log (hcount: the count for the
// host's bound, pinned host memory, may be null).
__device__ __forceinline__ void lru_end_body(uint32_t *count, uint32_t seq, uint32_t now, LruDev *L,
                                             uint32_t max_entries, uint64_t nl, uint32_t *hcount) {
    if (!L->flag) {
        if (hcount) *hcount = *count;
        return;
    }
    unsigned long long killed = 0, lines = 0;
    for (uint32_t r = 0; r < GF_LRU_ROUNDS; r++) {
        lines += lru_round(L, r, max_entries, nl).lines;
        killed += L->kills[r];
    }
    *count = (uint32_t)(*count - killed);
    const uint32_t n = L->nlog;
    if (n < GF_LRU_LOGCAP) {
        LruLog &g = L->log[n];
        g.seq = seq; g.now = now; g.age_cut = L->K; g.pad = 0;
        g.hand = L->hand; g.lines = lines; g.evicted = killed;
    }
    L->nlog = n + 1;
    L->hand = (L->hand + lines) % nl;
    L->flag = 0;
    if (hcount) *hcount = *count;
}
__global__ void k_lru_end(uint32_t *count, uint32_t seq, uint32_t now, LruDev *L, uint32_t max_entries, uint64_t nl,
                          uint32_t *hcount) {
    lru_end_body(count, seq, now, L, max_entries, nl, hcount);
}

// The same chain over several maps of one slot kind at once (per-endpoint CT maps,
// the ConntrackLocal option): one launch per phase for up to GF_LRU_MULTI maps, each
// block running every map's share in turn (the plan and the end: one block / one
// thread per map).  The maps travel in the kernel arguments.
#define GF_LRU_MULTI 32u
struct LruMap {
    gf_htab_desc d;
    LruDev *L;
    uint64_t nl, sl;
    uint32_t mode, max_entries, seq, pad;
    uint32_t *hcount;
    unsigned long long *stamp;          // multi-map pass: seq << 32 | count after the pass (pinned), or null
};
struct LruBatch { LruMap m[GF_LRU_MULTI]; uint32_t n; };
static_assert(GF_LRU_MULTI <= 32, "lru_active keeps one bit per map in a 32-bit mask");
static_assert(sizeof(LruBatch) + 64 <= 4096, "the maps travel in the kernel arguments");
// The batch's maps a phase has work for, read by one lane per map at once (a block
// would otherwise pay one dependent round trip per map): what 0 = over the high-water
// mark (the sample; wide: the window was empty), 1 = evicting this call (the hand).
__device__ __forceinline__ uint32_t lru_active(const LruBatch &B, uint32_t what, uint32_t wide) {
    __shared__ uint32_t s_mask;
    if (threadIdx.x < 64) {
        bool a = false;
        if (threadIdx.x < B.n) {
            const LruMap &M = B.m[threadIdx.x];
            if (what) a = M.L->flag != 0u;
            else a = wide ? M.L->wide != 0u : (unsigned long long)*M.d.count > lru_high_water(M.max_entries);
        }
        const uint64_t b = __ballot(a);
        if (threadIdx.x == 0) s_mask = (uint32_t)b;
    }
    __syncthreads();
    return s_mask;
}
template <int KIND>
__global__ __launch_bounds__(GF_LRU_HB) void k_lru_sample_multi(LruBatch B, uint32_t now, uint32_t wide) {
    const uint32_t act = lru_active(B, 0u, wide);
    for (uint32_t k = 0; k < B.n; k++) {
        if (!((act >> k) & 1u)) continue;
        const LruMap &M = B.m[k];
        lru_sample_body<KIND>(M.d, M.mode, now, M.L, M.sl, M.max_entries, wide);
        __syncthreads();                                // the LDS bins are the next map's
    }
}
__global__ __launch_bounds__(1024) void k_lru_plan_multi(LruBatch B, uint32_t wide) {
    const LruMap &M = B.m[blockIdx.x];
    lru_plan_body(M.d.count, M.max_entries, M.L, M.sl, M.nl, wide);
}
template <int KIND, int PAR>
__global__ __launch_bounds__(GF_LRU_HT) void k_lru_hand_multi(LruBatch B, uint32_t now, uint32_t round) {
    const uint32_t act = lru_active(B, 1u, 0u);
    for (uint32_t k = 0; k < B.n; k++) {
        if (!((act >> k) & 1u)) continue;
        const LruMap &M = B.m[k];
        lru_hand_body<KIND, PAR>(M.d, M.mode, now, M.L, M.nl, M.sl, M.max_entries, round);
        __syncthreads();                                // code[] and the block's counts are the next map's
    }
}
__global__ void k_lru_end_multi(LruBatch B, uint32_t now) {
    if (threadIdx.x >= B.n) return;
    const LruMap &M = B.m[threadIdx.x];
    lru_end_body(M.d.count, M.seq, now, M.L, M.max_entries, M.nl, M.hcount);
    if (M.stamp) *M.stamp = ((unsigned long long)M.seq << 32) | *M.d.count;
}

// ================================================================ drop notifications
// send_drop_notify / __send_drop_notify (bpf/lib/drop.h:47-107, DROP_NOTIFY): one
// struct drop_notify (32 B, pkg/monitor DropNotify) + up to TRACE_PAYLOAD_LEN
// captured bytes per dropped packet, appended to the event ring in batch order
// (per-block counts, an exclusive scan, then a block-local scan for the slots).
struct EvSrc {
    const uint8_t *recs;      // per-packet verdict records
    uint32_t stride, act_off; // record stride, offset of action (reason, ct_ret, flags follow)
    int32_t stage_off;        // pipeline / egress: offset of the stage byte (-1: ingress records)
    const gf_rec *prec;       // handle_policy inputs (src_identity, ifindex, program slot)
    const gf_lxc_dev *cfgs;   // endpoint programs (LXC_ID, SECLABEL)
    const uint32_t *len, *flow_hash;
    const uint8_t *snap;      // frames to capture from (may be null)
    uint32_t snap_stride, n;
    // trace notifications (trace.h:59-106); trace == 0: drop records only
    uint32_t trace, kind;     // kind: 0 ingress, 1 pipeline, 2 egress
    const uint8_t *tmark;     // GF_TR_* per packet
    const uint8_t *tcap_px;   // TO_PROXY captures (GF_TR_CAPTURED)
    const uint8_t *tcap_in;   // pipeline: TRACE_FROM_STACK captures
    const uint8_t *orig;      // egress: the frames as sent (TRACE_FROM_LXC), snap_stride apart
    const uint16_t *lxc_id, *slot_of;   // egress: the sender's program
    uint32_t host_ifindex, encap_ifindex, nd_trace, nd_ifindex;
};
// One notification: the 8 header words of struct drop_notify / trace_notify and
// where its captured bytes come from.
struct EvOne {
    uint32_t w[8];
    const uint8_t *pay;       // frame bytes (null: zeros)
    uint32_t pstride;         // bytes present at pay
};
__device__ __forceinline__ EvOne ev_trace(uint32_t obs, uint32_t source, uint32_t hash, uint32_t len, uint32_t src,
                                          uint32_t dst, uint32_t dst_id, uint32_t ifindex, uint32_t reason,
                                          const uint8_t *pay, uint32_t pstride) {
    EvOne e;
    const uint32_t cap = len < GF_TRACE_PAYLOAD_LEN ? len : GF_TRACE_PAYLOAD_LEN;
    e.w[0] = 4u /* CILIUM_NOTIFY_TRACE */ | (obs << 8) | ((source & 0xffffu) << 16);
    e.w[1] = hash; e.w[2] = len; e.w[3] = cap; e.w[4] = src; e.w[5] = dst;
    e.w[6] = (dst_id & 0xffffu) | ((reason & 0xffu) << 16);
    e.w[7] = ifindex;
    e.pay = pay; e.pstride = pstride;
    return e;
}
enum { TR_TO_LXC = 0, TR_TO_PROXY = 1, TR_TO_HOST = 2, TR_TO_STACK = 3, TR_TO_OVERLAY = 4, TR_FROM_LXC = 5,
       TR_FROM_STACK = 8 };
// The notifications of packet i in the order the programs send them (k < 0:
// just count them).  Drops: send_drop_notify / __send_drop_notify (drop.h:47-107)
// after handle_policy (src_label, SECLABEL, LXC_ID, ifindex), the sender's
// (SECLABEL, 0, 0, 0) after the from-container program, zeros for the callers'
// send_drop_notify_error.  Traces: from_netdev's TRACE_FROM_STACK
// (bpf_netdev.c:436), handle_ingress's TRACE_FROM_LXC (bpf_lxc.c:705), the
// redirects' TRACE_TO_PROXY (lxc.h:116/168), TO_HOST / TO_STACK / TO_OVERLAY
// of the from-container exits (bpf_lxc.c:364,381,650,669, encap.h:67) and
// handle_policy's TRACE_TO_LXC when it did not redirect (bpf_lxc.c:1013-1016).
__device__ uint32_t ev_list(const EvSrc &E, uint32_t i, int k, EvOne &out) {
    const uint8_t *r = E.recs + (size_t)i * E.stride;
    const uint32_t act = r[E.act_off], reason = r[E.act_off + 1], ct_ret = r[E.act_off + 2], ofl = r[E.act_off + 3];
    const uint32_t stage = E.stage_off < 0 ? (uint32_t)GF_STAGE_POLICY : r[E.stage_off];
    const uint32_t len = E.len[i], hash = E.flow_hash ? E.flow_hash[i] : 0u;
    const uint8_t *fin = E.snap ? E.snap + (size_t)i * E.snap_stride : nullptr;
    const uint32_t mark = E.tmark ? E.tmark[i] : 0u;
    const uint8_t *pxc = (mark & GF_TR_CAPTURED) ? E.tcap_px + (size_t)i * GF_TRACE_PAYLOAD_LEN : fin;
    const uint32_t pxs = (mark & GF_TR_CAPTURED) ? GF_TRACE_PAYLOAD_LEN : E.snap_stride;
    uint32_t n = 0;
    auto put = [&](const EvOne &e) { if ((int)n == k) out = e; n++; };
    if (E.trace) {
        if (E.kind == 1 && E.nd_trace && (stage == GF_STAGE_NETDEV || stage == GF_STAGE_POLICY))
            put(ev_trace(TR_FROM_STACK, 0, hash, len, 0, 0, 0, E.nd_ifindex, 0,
                         E.tcap_in + (size_t)i * GF_TRACE_PAYLOAD_LEN, GF_TRACE_PAYLOAD_LEN));
        if (E.kind == 2) {
            const uint32_t sl = E.slot_of[E.lxc_id ? E.lxc_id[i] : 0];
            const gf_lxc_dev *sc = sl ? E.cfgs + (sl - 1) : nullptr;
            if (sc && (gload<uint32_t>(&sc->flags) & GF_LXC_F_TRACE_NOTIFY)) {
                const uint32_t lid = gload<uint32_t>(&sc->lxc_id), sec = gload<uint32_t>(&sc->seclabel);
                const uint32_t fwd = r[5];                 // gf_egress_out.eg_ct_ret
                const uint32_t ef = *reinterpret_cast<const uint16_t *>(r + 14);
                put(ev_trace(TR_FROM_LXC, lid, hash, len, sec, 0, 0, 0, 0, E.orig + (size_t)i * E.snap_stride,
                             E.snap_stride));
                if (mark & GF_TR_PX_EGRESS)
                    put(ev_trace(TR_TO_PROXY, lid, hash, len, sec, 0, 0, E.host_ifindex, fwd, pxc, pxs));
                if (stage == GF_STAGE_FROM_LXC && act != TC_SHOT) {
                    if (ef & GF_EG_F_TO_HOST)
                        put(ev_trace(TR_TO_HOST, lid, hash, len, sec, 1u /* HOST_ID */, 0, E.host_ifindex, fwd, fin,
                                     E.snap_stride));
                    else if (ef & GF_EG_F_TO_STACK)
                        put(ev_trace(TR_TO_STACK, lid, hash, len, sec, (mark & GF_TR_CLUSTER) ? 3u : 2u, 0, 0, fwd, fin,
                                     E.snap_stride));
                    else if (ef & GF_EG_F_ENCAP)
                        put(ev_trace(TR_TO_OVERLAY, lid, hash, len, sec, 0, 0, E.encap_ifindex, 0, fin, E.snap_stride));
                }
            }
        }
        if (stage == GF_STAGE_POLICY) {                    // handle_policy of the destination
            const gf_rec pr = E.prec[i];
            const gf_lxc_dev *dc = pr.ep ? E.cfgs + (pr.ep - 1) : nullptr;
            if (dc && (gload<uint32_t>(&dc->flags) & GF_LXC_F_TRACE_NOTIFY)) {
                const uint32_t lid = gload<uint32_t>(&dc->lxc_id), sec = gload<uint32_t>(&dc->seclabel);
                if (mark & GF_TR_PX_POLICY)
                    put(ev_trace(TR_TO_PROXY, lid, hash, len, sec, 0, 0, E.host_ifindex, ct_ret, pxc, pxs));
                if (act != TC_SHOT && !((ofl & GF_INGRESS_F_PROXY) && pr.ifindex != E.host_ifindex))
                    put(ev_trace(TR_TO_LXC, lid, hash, len, pr.src_identity, sec, lid, pr.ifindex, ct_ret, fin,
                                 E.snap_stride));
            }
        }
    }
    if (act == TC_SHOT && stage != GF_STAGE_XDP && (int)n == k) {
        uint32_t src = 0, dst = 0, dst_id = 0, ifx = 0, source = 0;
        if (stage == GF_STAGE_FROM_LXC) {
            const gf_rec pr = E.prec[i];                // send_drop_notify(skb, SECLABEL, 0, 0, 0, ret) of the sender
            if (pr.ep) { const gf_lxc_dev &cf = E.cfgs[pr.ep - 1]; src = cf.seclabel & 0xffffu; source = cf.lxc_id & 0xffffu; }
        } else if (stage == GF_STAGE_POLICY) {
            const gf_rec pr = E.prec[i];
            if (pr.ep) {                                // handle_policy: send_drop_notify(src_label, SECLABEL, LXC_ID, ifindex)
                const gf_lxc_dev &cf = E.cfgs[pr.ep - 1];
                src = pr.src_identity & 0xffffu; dst = cf.seclabel & 0xffffu;
                dst_id = cf.lxc_id; ifx = pr.ifindex; source = cf.lxc_id & 0xffffu;
            }                                           // else the caller's send_drop_notify_error: zeros
        }
        out.w[0] = 1u /* CILIUM_NOTIFY_DROP */ | (reason << 8) | (source << 16);
        out.w[1] = hash;
        out.w[2] = len; out.w[3] = len < GF_TRACE_PAYLOAD_LEN ? len : GF_TRACE_PAYLOAD_LEN;
        out.w[4] = src; out.w[5] = dst; out.w[6] = dst_id; out.w[7] = ifx;
        out.pay = fin; out.pstride = E.snap_stride;
    }
    if (act == TC_SHOT && stage != GF_STAGE_XDP) n++;
    return n;
}
__global__ __launch_bounds__(BLOCK) void k_ev_count(EvSrc E, uint32_t *blk) {
    __shared__ uint32_t c;
    if (threadIdx.x == 0) c = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    EvOne e;
    if (i < E.n) { const uint32_t m = ev_list(E, i, -1, e); if (m) atomicAdd(&c, m); }
    __syncthreads();
    if (threadIdx.x == 0) blk[blockIdx.x] = c;
}
__global__ __launch_bounds__(BLOCK) void k_ev_write(EvSrc E, const uint32_t *boff, gf_event_ring R) {
    __shared__ uint32_t sc[BLOCK];
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    EvOne e;
    const uint32_t m = i < E.n ? ev_list(E, i, -1, e) : 0u;
    sc[threadIdx.x] = m;
    __syncthreads();
    for (uint32_t o = 1; o < BLOCK; o <<= 1) {          // inclusive scan
        uint32_t v = threadIdx.x >= o ? sc[threadIdx.x - o] : 0u;
        __syncthreads();
        sc[threadIdx.x] += v;
        __syncthreads();
    }
    for (uint32_t k = 0; k < m; k++) {
        const uint64_t pos = (uint64_t)*R.count + boff[blockIdx.x] + sc[threadIdx.x] - m + k;
        if (pos >= R.capacity) return;                  // ring full: the record is lost
        ev_list(E, i, (int)k, e);
        uint32_t *w = reinterpret_cast<uint32_t *>(R.records + pos * GF_EVENT_RECORD);
        for (int q = 0; q < 8; q++) w[q] = e.w[q];
        const uint32_t cap = e.w[3];
        for (uint32_t q = 0; q < GF_TRACE_PAYLOAD_LEN / 4; q++) {
            uint32_t v = 0;
            for (uint32_t b = 0; b < 4; b++) {
                const uint32_t off = 4 * q + b;
                if (e.pay && off < cap && off < e.pstride) v |= (uint32_t)e.pay[off] << (8 * b);
            }
            w[8 + q] = v;
        }
    }
}
__global__ void k_ev_commit(const uint32_t *boff, const uint32_t *blk, uint32_t nb, gf_event_ring R) {
    *R.count += boff[nb - 1] + blk[nb - 1];
}

// ================================================================ cilium_proxy{4,6} updates
// The redirects of a launch are logged (pol_redirect) and applied here in batch
// order.  The proxy maps change only through these updates while a batch runs,
// so applying them after the launch gives every update the outcome sequential
// execution gives it.  Parallel path (the maps cannot fill): the log is sorted by
// (key hash, packet index); an entry is applied only if no later entry of the
// batch has the same key (the last writer wins, as in order), and distinct keys
// insert concurrently.  Sequential path (a map could fill): one lane applies the
// log in packet order with exact max_entries accounting; a failed update turns
// the packet into DROP_PROXYMAP_CREATE_FAILED (lxc.h:137/199).  Successful
// redirects get ipv{4,6}_policy's MAC stores (bpf_lxc.c:840-846, 955-961).
struct PxDev {
    gf_htab_desc d4, d6;
    uint8_t *snap;              // writable frames (pipeline) or null
    const uint32_t *len;
    uint32_t snap_stride;
    uint32_t host_mac[2], node_mac[2];
};
__device__ __forceinline__ bool px_same(const uint32_t *a, const uint32_t *b) {
    if (a[1] != b[1]) return false;
    const int nw = a[1] == 6 ? 6 : 3;
    for (int k = 0; k < nw; k++) if (a[2 + k] != b[2 + k]) return false;
    return true;
}
__device__ __forceinline__ void px_macs(const PxDev &P, uint32_t i) {
    if (!P.snap) return;
    const uint32_t len = P.len[i];
    Row w{P.snap + (size_t)i * P.snap_stride, P.snap_stride < len ? P.snap_stride : len};
    w.w32(6, P.node_mac[0]); w.w16(10, P.node_mac[1]);     // eth_store_saddr(NODE_MAC)
    w.w32(0, P.host_mac[0]); w.w16(4, P.host_mac[1]);      // eth_store_daddr(HOST_IFINDEX_MAC)
}
__device__ __forceinline__ int64_t px_upsert(const PxDev &P, const uint32_t *e, bool strict, int *added) {
    if (e[1] == 6) return P.d6.slots ? ht_upsert<22, 7, GF_HASH_PLAIN>(P.d6, e + 2, e + 8, strict, added) : 0;
    return P.d4.slots ? ht_upsert<10, 4, GF_HASH_PLAIN>(P.d4, e + 2, e + 8, strict, added) : 0;
}
// Without proxy maps the updates are no-ops: only the redirects' MAC stores (frames written)
__global__ __launch_bounds__(BLOCK) void k_px_macs(const uint32_t *plog, const uint32_t *n_, PxDev P) {
    const uint32_t n = *n_;
    for (uint32_t j = blockIdx.x * BLOCK + threadIdx.x; j < n; j += gridDim.x * BLOCK) {
        const uint32_t *e = plog + 16ull * j;
        if (!e[15]) px_macs(P, e[0]);
    }
}
__global__ __launch_bounds__(BLOCK) void k_px_keys(const uint32_t *plog, uint32_t n, bool by_index,
                                                   unsigned long long *key, uint32_t *val) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= n) return;
    const uint32_t *e = plog + 16ull * j;
    uint32_t h = 0;
    if (!by_index) h = e[1] == 6 ? key_hash<22>(e + 2) : key_hash<10>(e + 2);
    key[j] = ((unsigned long long)h << 32) | e[0];
    val[j] = j;
}
__global__ __launch_bounds__(BLOCK) void k_px_apply(const uint32_t *plog, uint32_t n, const unsigned long long *key,
                                                    const uint32_t *perm, PxDev P) {
    const uint32_t p = blockIdx.x * BLOCK + threadIdx.x;
    if (p >= n) return;
    const uint32_t *e = plog + 16ull * perm[p];
    if (!e[15]) px_macs(P, e[0]);
    const uint32_t h = (uint32_t)(key[p] >> 32);
    for (uint32_t q = p + 1; q < n && (uint32_t)(key[q] >> 32) == h; q++)
        if (px_same(e, plog + 16ull * perm[q])) return;     // a later update of the same key wins
    int added = 0;
    px_upsert(P, e, false, &added);
    if (added) atomicAdd(e[1] == 6 ? P.d6.count : P.d4.count, (uint32_t)added);
}
__global__ void k_px_apply_seq(const uint32_t *plog, uint32_t n, const uint32_t *perm, PxDev P, uint8_t *recs,
                               uint32_t stride, uint32_t act_off, unsigned long long *stats) {
    for (uint32_t p = 0; p < n; p++) {
        const uint32_t *e = plog + 16ull * perm[p];
        const uint32_t i = e[0];
        if (px_upsert(P, e, true, nullptr) >= 0) { if (!e[15]) px_macs(P, i); continue; }
        uint8_t *r = recs + (size_t)i * stride;             // DROP_PROXYMAP_CREATE_FAILED
        const uint32_t old_action = r[act_off];
        r[act_off] = TC_SHOT; r[act_off + 1] = 161;
        if (stride == 8) { r[3] &= 2; r[4] = r[5] = r[6] = r[7] = 0; }
        else { r[4] &= ~1u; r[6] = r[7] = r[8] = r[9] = 0; }
        if (stats) {
            atomicAdd(&stats[0], ~0ull); atomicAdd(&stats[161], 1ull);
            atomicAdd(&stats[256 + old_action], ~0ull); atomicAdd(&stats[256 + TC_SHOT], 1ull);
        }
    }
}

// ================================================================ endpoint egress (from-container)
// handle_ingress (bpf/bpf_lxc.c:685-738) -> tail_handle_ipv4 -> handle_ipv4_from_lxc
// (:427-658) over frames sent by local endpoints.  k_eg_front runs the stateless
// part on one packet per lane (checks, lb4_local with its lb4_xlate rewrites,
// map_lxc_out) and keys the packet by the flow group of its CT tuple; the
// schedule of the ingress path orders the groups; k_eg_groups runs the CT /
// policy part of each bucket on one lane in batch order, ending in a verdict or
// in ipv4_local_delivery, whose handle_policy runs in the ingress pass after it.
// ct_create4's service entry (conntrack.h:533-561) has the pair {target, target}
// or {IPV4_LOOPBACK, sender}, outside the packet's group: it is logged and
// applied after the launch in batch order (last writer wins, as in order).  No
// packet of the batch reads such a key unless its own tuple has that shape
// (saddr == daddr, or IPV4_LOOPBACK in it); k_eg_front flags those batches and
// they run as a single bucket with the entry written inline.
enum {
    D_INVALID_SMAC = -130, D_INVALID_DMAC = -131, D_INVALID_SIP = -132, D_NO_LXC = -152, D_CSUM_L3 = -153,
    D_POLICY_CIDR = -162,
};
#define GF_EGR_FINAL 1u                 // EgRec.st: the verdict was written by k_eg_front
struct __attribute__((aligned(16))) EgRec {   // 32 B: what the CT part needs from the front
    uint32_t t_daddr, t_saddr;          // CT tuple addresses after lb4_local
    uint32_t len, orig_dip;             // skb->len; orig_dip (tuple.daddr after lb4_local)
    uint32_t ct_addr;                   // ct_state_new.addr (0: not load balanced)
    uint16_t rev_nat, ep;               // ct_state_new.rev_nat_index; program slot + 1
    int16_t  l4_off;
    uint8_t  nh, st;
    uint16_t slave, eflags;             // lb4_local's slave; GF_EG_F_* so far
};
static_assert(sizeof(EgRec) == 32, "EgRec must be 32 bytes");
struct EgDev {
    const gf_lxc_dev *cfgs;
    uint8_t *v6blk;                     // per front block: holds an IPv6 frame (k_eg_front<4> writes, <6> reads), or null
    const uint16_t *slot_of;
    gf_htab_desc ct4, ct6, lxc, tunnel;
    const uint32_t *lxset, *tnset;      // cilium_lxc's / the tunnel map's IPv4 keys: address set + slots
    uint32_t lxbits, lxzero, tnbits, tnzero;   // (Map::addr_set), or null
    uint8_t *snap;                      // the frames, rewritten in place
    uint8_t *s6out, *d6out;             // IPv6 addresses of the local deliveries (handle_policy's columns)
    uint32_t stride, now, host_ifindex, encap_ifindex;
    uint32_t cluster_range, cluster_mask, loopback, ipv4_mask;
    uint32_t host_mac[2];
    uint32_t router6[4], host6[4];      // ROUTER_IP, HOST_IP (LE words)
    uint32_t strict;                    // bit0: CT4 inserts check max_entries (forces the single bucket); bit1: CT6
    uint32_t *seq;                      // device word: 1 = single-bucket batch (written by k_eg_front)
    uint32_t *ctlog, *ctlog_n;          // deferred service entries {i, key[4], value[12], pad[3]}; [n, v6 deliveries]
    IngCtx X;                           // redirect writes + cilium_proxy4 log (pol_redirect)
    uint64_t *hz_k;                     // per packet, GF_HZ_NK keys (hz_key order below), n apart
    const uint32_t *vip4;               // the rev-NAT addresses of the programs' revNAT maps (open addressing,
    const uint4 *vip6;                  //   0 = empty), vip*_mask + 1 slots; null: none
    uint32_t vip4_mask, vip6_mask;
    uint8_t *hz_fl;                     // per packet: GF_HZ_* (null: no ordering check)
    uint32_t *hz;                       // device words: [0] 1 = ordering hazard (k_eg_groups idles), [1] GF_HZ_* kinds seen
    // Connection groups (IPv4): conn = 1 keys IPv4 packets by their
    // connection and logs the ICMP-related entries ct_create4 writes (the only CT key
    // two connections of a pair share, read only by ICMP errors); an IPv4 ICMP packet
    // in the run sets *cflag and the run falls back to address-pair groups.
    uint32_t conn;
    uint32_t *cflag;                    // device word: 1 = pair groups (an IPv4 ICMP packet reaches conntrack)
    uint32_t *keysP, *key2P;            // the pair keys of the front / of the deliveries (fallback)
    uint32_t *rlog, *rlog_n;            // logged related entries {order, key[4], value[12], pad[3]}
    RelSet rs;                          // GF_EG_RSET: their set instead
    gf_rec *rec2;                       // the handle_policy pass's records: the front writes every packet's
    uint32_t *key2;                     //   as "not delivered" in batch order, k_eg_groups only the deliveries
};
// The ordering check.  The reference runs a local delivery's
// handle_policy right after its from-container program, before the next packet;
// the batch runs every from-container part first, then every handle_policy.  The
// two orders differ only when a packet's from-container part touches a CT entry an
// earlier packet's handle_policy touches.  The CT keys a packet can touch follow
// from its tuples (conntrack.h:170-289 lookups, :446-580 creates):
//  * handle_policy: its tuple (the frame after the from-container rewrites) and
//    the reverse, for ICMP the related entry of the address pair;
//  * from-container: its CT tuple (after lb4_local) and the reverse, the related
//    entry of the pair for ICMP, and lb4_local's loopback service entry (the frame
//    pair after the SNAT).
// A handle_policy tuple and a later from-container tuple share an entry only in
// opposite directions (the lookups differ in TUPLE_F_IN); so the front keys each
// packet by the connection of its frame tuple and of its CT tuple (unordered 5-tuple,
// ICMP ports 0, + direction), their address pairs, and its two addresses:
//   a later packet whose CT connection equals an earlier frame connection in the
//     other direction (a reply in the same batch);
//   an ICMP packet after any packet of its CT pair, any packet after an ICMP packet
//     of its pair (the related entries);
//   a loopback packet whose frame connection appeared earlier (its service entry);
//   a packet to a rev-NAT address without translation after any packet with its
//     source address (a reply rev-NATed by lb4/6_rev_nat reaches handle_policy as
//     {service address, one of its own addresses});
// flags the batch, which then runs in contiguous runs free of these, in order.
#define GF_HZ_NK      6u                // keys per packet: conn(frame), conn(CT), pair(frame), pair(CT), src, dst
#define GF_HZ_VALID   1u                // continues past the front
#define GF_HZ_DIRI    2u                // direction of the frame tuple within its connection
#define GF_HZ_DIRE    4u                // direction of the CT tuple within its connection
#define GF_HZ_ICMP    8u                // ICMP / ICMPv6
#define GF_HZ_VIP    16u                // to a rev-NAT address without lb4/6_local translation
#define GF_HZ_LOOP   32u                // lb4_local back to the sender (loopback SNAT)
#define GF_HZ_V6     64u                // the IPv6 path
#define GF_HZ_DLV   128u                // may reach ipv4/6_local_delivery (daddr an endpoint, or IPV4_LOOPBACK
                                        // whose rev-NAT restores the sender): only these enter handle_policy
// A CT map that could fill during the batch (strict accounting) makes every
// insert order-dependent (E2BIG for whichever comes last): a batch with a
// continuing packet of that family is flagged 2 and runs one packet at a time.
#define GF_HZ_ICMPSALT 0x6a09e667f3bcc908ull   // the related-entry space of ICMP packets' pairs
#define GF_CTLOG_WORDS 20u

// The header bytes the IPv4 egress programs touch (< l4_off + 18 <= 92) are staged
// per lane in LDS: one vector load per row instead of a global access per byte.
#define GF_EG_STAGE 128u
GF_HD uint32_t eg_stage_bytes(uint32_t S) { return S < GF_EG_STAGE ? S : GF_EG_STAGE; }
#ifndef GF_EG_GROUPS_DYN
#define GF_EG_GROUPS_DYN 1  // k_eg_groups: LDS rows sized by the snap stride (0: GF_EG_STAGE-byte rows)
#endif
GF_HD uint32_t eg_row_bytes(uint32_t S) {           // k_eg_groups' LDS row
    return GF_EG_GROUPS_DYN ? (eg_stage_bytes(S) + 15u) & ~15u : GF_EG_STAGE;
}
__device__ __forceinline__ void eg_copy(uint8_t *dst, const uint8_t *src, uint32_t n) {
    if (!(n & 15u) && !(((uintptr_t)src | (uintptr_t)dst) & 15u)) {
        for (uint32_t k = 0; k < n; k += 16) *reinterpret_cast<uint4 *>(dst + k) = *reinterpret_cast<const uint4 *>(src + k);
    } else {
        for (uint32_t k = 0; k < n; k++) dst[k] = src[k];
    }
}
__device__ __forceinline__ bool mac_eq(const Row &w, uint32_t off, const uint32_t *m) {
    return w.r32(off) == m[0] && w.r16(off + 4) == (m[1] & 0xffffu);
}
// ipv4_l3 (bpf/lib/l3.h:54-70) + ipv4_dec_ttl (bpf/lib/ipv4.h:30-43); smac may be null
__device__ __forceinline__ int eg_ipv4_l3(Row &w, uint32_t len, const uint32_t *smac, const uint32_t *dmac) {
    const uint32_t ttl = w.b(22);
    if (ttl <= 1) return D_INVALID;
    l3_csum(w, len, 24, ttl, ttl - 1, 2);
    w.w8(22, ttl - 1);
    if (smac) { w.w32(6, smac[0]); w.w16(10, smac[1] & 0xffffu); }
    w.w32(0, dmac[0]); w.w16(4, dmac[1] & 0xffffu);
    return TC_OK;
}

// handle_ipv6 (bpf_lxc.c:388-416) + the stateless head of ipv6_l3_from_lxc (:120-185):
// icmp6_handle's responders, the source checks, ipv6_hdrlen, lb6_extract_key +
// lb6_lookup_service + lb6_local (lb6_xlate: daddr, the L4 checksum at l4_off + its
// offset even when that offset is 0, the port), map_lxc_out.  TC_OK: continue in
// k_eg_groups (r.st = 0); a stage-NONE responder returns TC_OK with r.st set.
__device__ __forceinline__ int eg_front6(const EgDev &E, const gf_lxc_dev *c, Row &w, uint32_t len, uint32_t fh,
                                         EgRec &r, gf_egress_out &o, uint32_t &ab) {
    r.eflags = GF_EG_F_IPV6;
    if (len < 54) return D_INVALID;
    if (w.b(20) == 58) {                                // icmp6_handle (bpf/lib/icmp6.h:380-401)
        if (len < 62) return D_INVALID;
        const uint32_t type = w.b(54);
        bool to_router = true;
        for (int k = 0; k < 4; k++) to_router &= w.r32(38 + 4 * k) == E.router6[k];
        if (type == 135 || (type == 128 && to_router)) {
            o.stage = GF_STAGE_NONE; o.eg_flags = GF_EG_F_IPV6 | GF_EG_F_RESPONDER;
            return TC_OK;
        }
    }
    uint32_t m[2];
    m[0] = gload<uint32_t>(&c->lxc_mac[0]); m[1] = gload<uint32_t>(&c->lxc_mac[1]);
    if (!mac_eq(w, 6, m)) return D_INVALID_SMAC;
    m[0] = gload<uint32_t>(&c->node_mac[0]); m[1] = gload<uint32_t>(&c->node_mac[1]);
    if (!mac_eq(w, 0, m)) return D_INVALID_DMAC;
    for (int k = 0; k < 4; k++)
        if (w.r32(22 + 4 * k) != gload<uint32_t>(&c->lxc_ip6[k])) return D_INVALID_SIP;
    PktHdr h;
    parse_row(w.p, w.cap, len, h);                      // nexthdr / l4_off after ipv6_hdrlen (negative: added as is)
    const uint32_t nh = h.proto;
    const int l4_off = h.l4;
    r.nh = (uint8_t)nh; r.l4_off = (int16_t)l4_off;
    ab += 34 + 28;
    const uint32_t co = csum_l4_offset(nh), fl = nh == 17 ? GF_F_MANGLED_0 : 0u;
    bool lb_try = true;
    uint32_t kport = 0;
    if (nh == 6 || nh == 17) {
        if (!skb_ok(l4_off + 2, 2, len)) return -GF_EFAULT;
        kport = w.r16((uint32_t)(l4_off + 2));
    } else if (nh != 1 && nh != 58) lb_try = false;
    const gf_htab_desc lb = gload<gf_htab_desc>(&c->lb6);
    if (lb_try && lb.slots) {
        const uint8_t *svc = nullptr;
        if (kport) {
            uint32_t kw[5] = {h.d6[0], h.d6[1], h.d6[2], h.d6[3], kport};
            const int64_t f = ht_find<20>(lb, kw, key_hash<20>(kw));
            ab += 44;
            if (f >= 0) { const uint8_t *v = ht_val(lb, f); if (gload<uint16_t>(v + 18)) svc = v; }
            if (!svc) kport = 0;
        }
        if (!svc) {
            uint32_t kw[5] = {h.d6[0], h.d6[1], h.d6[2], h.d6[3], kport};
            const int64_t f = ht_find<20>(lb, kw, key_hash<20>(kw));
            ab += 44;
            if (f >= 0) { const uint8_t *v = ht_val(lb, f); if (gload<uint16_t>(v + 18)) svc = v; }
        }
        if (svc) {                                      // lb6_local, lb.h:425-445
            const uint32_t count = gload<uint16_t>(svc + 18);
            const uint32_t slave = (fh % count + 1u) & 0xffffu;
            uint32_t kw[5] = {h.d6[0], h.d6[1], h.d6[2], h.d6[3], kport | (slave << 16)};
            const int64_t f = ht_find<20>(lb, kw, key_hash<20>(kw));
            ab += 44;
            if (f < 0) return D_NO_SERVICE;
            const uint8_t *be = ht_val(lb, f);
            r.slave = (uint16_t)slave; r.eflags |= GF_EG_F_LB;
            r.rev_nat = gload<uint16_t>(be + 20);
            uint32_t sum = 0;
            for (int k = 0; k < 4; k++) {               // lb6_xlate: ipv6_store_daddr + csum_diff
                const uint32_t nw = gload<uint32_t>(be + 4 * k);
                w.w32(38 + 4 * k, nw);
                sum = ck_add(ck_add(sum, ~h.d6[k]), nw);
            }
            if (l4_csum(w, len, l4_off + (int)co, 0, sum, GF_F_PSEUDO_HDR | fl) < 0) return D_CSUM_L4;
            const uint32_t sp = gload<uint16_t>(be + 16);
            if (sp && kport != sp && (nh == 6 || nh == 17)) {
                if (l4_csum(w, len, l4_off + (int)co, kport, sp, 2u | fl) < 0) return D_CSUM_L4;
                if (!skb_ok(l4_off + 2, 2, len)) return D_WRITE_ERROR;
                w.w16((uint32_t)(l4_off + 2), sp);
            }
            ab += 24;
        }
    }
    const uint32_t npm = gload<uint32_t>(&c->n_portmap);          // map_lxc_out
    if (npm && (nh == 6 || nh == 17)) {
        if (!skb_ok(l4_off, 2, len)) return D_INVALID;
        const uint32_t sp = w.r16((uint32_t)l4_off);
        for (uint32_t k = 0; k < npm && k < 16; k++) {
            const uint32_t pm = gload<uint32_t>(&c->portmap[k]);
            const uint32_t from = pm & 0xffffu, to = pm >> 16;
            if (to != sp) continue;
            if (l4_csum(w, len, l4_off + (int)co, sp, from, 2u | fl) < 0) return D_CSUM_L4;
            if (!skb_ok(l4_off, 2, len)) return D_WRITE_ERROR;
            w.w16((uint32_t)l4_off, from);
            r.eflags |= GF_EG_F_PORTMAP;
        }
    }
    r.st = 0;
    return TC_OK;
}

// handle_ingress + the stateless head of handle_ipv4_from_lxc, one packet per lane
// FAM 6 takes the IPv6 frames, FAM 4 every other frame (two launches: the IPv6
// path's registers and stack stay out of the IPv4 kernel).
// the slot of a rev-NAT address (fmix32: raw be32 addresses share their low bytes)
GF_HD uint32_t vip_slot(uint32_t x) {
    x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ bool vip4_has(const EgDev &E, uint32_t a) {
    if (!E.vip4 || !a) return false;
    uint32_t slot = vip_slot(a) & E.vip4_mask;
    for (uint32_t k = 0; k <= E.vip4_mask; k++) {
        const uint32_t v = E.vip4[slot];
        if (v == a) return true;
        if (!v) return false;
        slot = (slot + 1u) & E.vip4_mask;
    }
    return false;
}
__device__ __forceinline__ bool vip6_has(const EgDev &E, const uint32_t *a) {
    if (!E.vip6 || !(a[0] | a[1] | a[2] | a[3])) return false;
    uint32_t slot = vip_slot(a[0] ^ vip_slot(a[1] ^ vip_slot(a[2] ^ vip_slot(a[3])))) & E.vip6_mask;
    for (uint32_t k = 0; k <= E.vip6_mask; k++) {
        const uint4 v = E.vip6[slot];
        if (v.x == a[0] && v.y == a[1] && v.z == a[2] && v.w == a[3]) return true;
        if (!(v.x | v.y | v.z | v.w)) return false;
        slot = (slot + 1u) & E.vip6_mask;
    }
    return false;
}
__device__ __forceinline__ uint64_t hz_mix(uint64_t h, uint64_t v) {
    h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
    h *= 0xff51afd7ed558ccdull;
    return h ^ (h >> 31);
}
// Connection key of a tuple: order-free hash of {(sa, sp), (da, dp)} + nexthdr;
// dir = the (sa, sp) side sorts second.
__device__ __forceinline__ uint64_t hz_key(const uint32_t *sa, const uint32_t *da, int nw, uint32_t sp, uint32_t dp,
                                           uint32_t nh, bool &dir) {
    int c = 0;
    for (int k = 0; k < nw && !c; k++) c = sa[k] < da[k] ? -1 : (sa[k] > da[k] ? 1 : 0);
    if (!c) c = sp < dp ? -1 : (sp > dp ? 1 : 0);
    dir = c > 0;
    const uint32_t *lo = dir ? da : sa, *hi = dir ? sa : da;
    uint64_t h = 0x5eed0000ull | (uint64_t)nw;
    for (int k = 0; k < nw; k++) h = hz_mix(h, lo[k]);
    h = hz_mix(h, dir ? dp : sp);
    for (int k = 0; k < nw; k++) h = hz_mix(h, hi[k]);
    h = hz_mix(h, ((dir ? sp : dp) << 8) | nh);
    return h | 1ull;
}

template <int FAM>
__global__ __launch_bounds__(BLOCK) void k_eg_front(gf_frames fr, const uint16_t *lxc_id, const uint32_t *fhash, EgDev E,
                                                    EgRec *erec, uint32_t *keys, gf_egress_out *out,
                                                    unsigned long long *stats) {
    if (FAM == 6 && E.v6blk && !E.v6blk[blockIdx.x]) return;   // no IPv6 frame in this block
    __shared__ uint32_t sl[272];
    extern __shared__ uint4 lds[];                      // BLOCK * eg_stage_bytes(S) (FAM 6: none)
    Stats st{sl};
    if (stats) st.init();
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t S = fr.snap_stride;
    const uint32_t len = i < fr.n ? fr.len[i] : 0u;
    const uint8_t *src = fr.snap + (size_t)i * S;
    const uint32_t cap0 = S < len ? S : len;
    // IPv4 frames that fit a row (and 16-B aligned): the block stages its frames
    // with coalesced 16-B loads and stores them back the same way at the end
    // (block-uniform); otherwise each lane stages its own header.
    const bool coop = FAM == 4 && S <= GF_EG_STAGE && !(S & 15u) &&
                      !(((uintptr_t)fr.snap | (uintptr_t)E.snap) & 15u);
    const uint32_t b0 = blockIdx.x * BLOCK;
    const uint32_t nv = b0 < fr.n ? ((fr.n - b0 < BLOCK ? fr.n - b0 : BLOCK) * S) / 16 : 0u;
    if (coop) {
        const uint4 *g = reinterpret_cast<const uint4 *>(fr.snap + (size_t)b0 * S);
        for (uint32_t k = threadIdx.x; k < nv; k += BLOCK) lds[k] = g[k];
        __syncthreads();
    }
    uint8_t *row = reinterpret_cast<uint8_t *>(lds) + (FAM == 6 ? 0 : threadIdx.x * (coop ? S : eg_stage_bytes(S)));
    const uint8_t *hdr = coop ? row : src;
    const bool v6 = i < fr.n && len >= 14 && fbyte(hdr, cap0, 12) == 0x86 && fbyte(hdr, cap0, 13) == 0xDD;
    if (FAM == 4 && E.v6blk) {                                // tells k_eg_front<6> which blocks to run
        const int any6 = __syncthreads_or(v6 ? 1 : 0);
        if (threadIdx.x == 0) E.v6blk[blockIdx.x] = any6 ? 1u : 0u;
    }
    bool scnt = false;                                        // the lane's counter-block entry
    uint32_t sreason = 0, saction = 0, slen = 0, sab = 0;
    if (i < fr.n && v6 == (FAM == 6)) {
        const uint32_t K = eg_stage_bytes(S);
        uint8_t *dst = E.snap + (size_t)i * S;
        if (FAM == 6) {                                       // extension headers: the whole snap, in HBM
            if (src != dst) eg_copy(dst, src, S);
        } else if (!coop) {
            eg_copy(row, src, K);                             // the header, staged
            if (S > K && src != dst) eg_copy(dst + K, src + K, S - K);   // the rest of the snap, as is
        }
        Row w{row, K < len ? K : len};                        // IPv4: the LDS copy (ds_* accesses)
        Row wg{dst, cap0};                                    // IPv6: the frame in HBM
        gf_egress_out o{};
        EgRec r{};
        r.len = len;
        uint32_t ab = 24 + 34;                            // output record, header bytes parsed
        const uint32_t sl_ = E.slot_of[lxc_id ? lxc_id[i] : 0];
        r.ep = (uint16_t)sl_;
        r.st = GF_EGR_FINAL;
        int ret = TC_OK;
        o.stage = GF_STAGE_FROM_LXC;
        const uint32_t et = len >= 14 ? ((fbyte(src, cap0, 12) << 8) | fbyte(src, cap0, 13)) : 0u;
        do {
            if (!sl_) { ret = D_MISSED_TAIL_CALL; break; }
            const gf_lxc_dev *c = E.cfgs + (sl_ - 1);
            const uint32_t flags = gload<uint32_t>(&c->flags);
            if (et == 0x0806) { o.stage = GF_STAGE_NONE; o.eg_flags = GF_EG_F_ARP; break; }
            if (flags & GF_LXC_F_DROP_ALL) { ret = D_POLICY; break; }
            if constexpr (FAM == 6) { ret = eg_front6(E, c, wg, len, fhash ? fhash[i] : 0u, r, o, ab); break; }
            if (et != 0x0800) { ret = D_UNKNOWN_L3; break; }
            if (len < 34) { ret = D_INVALID; break; }
            const uint32_t nh = w.b(23);
            uint32_t m[2];
            m[0] = gload<uint32_t>(&c->lxc_mac[0]); m[1] = gload<uint32_t>(&c->lxc_mac[1]);
            if (!mac_eq(w, 6, m)) { ret = D_INVALID_SMAC; break; }
            m[0] = gload<uint32_t>(&c->node_mac[0]); m[1] = gload<uint32_t>(&c->node_mac[1]);
            if (!mac_eq(w, 0, m)) { ret = D_INVALID_DMAC; break; }
            const uint32_t saddr = w.r32(26), daddr = w.r32(30);
            if (!(flags & GF_LXC_F_LXC_IPV4) || saddr != gload<uint32_t>(&c->lxc_ipv4)) { ret = D_INVALID_SIP; break; }
            const int l4_off = 14 + (int)(w.b(14) & 0xfu) * 4;
            const uint32_t co = csum_l4_offset(nh), fl = nh == 17 ? GF_F_MANGLED_0 : 0u;
            r.t_daddr = daddr; r.t_saddr = saddr; r.nh = (uint8_t)nh; r.l4_off = (int16_t)l4_off;
            // lb4_extract_key (CT_EGRESS: key.address = daddr) + extract_l4_port (lb.h:191-215, 552-564)
            bool lb_try = true;
            uint32_t kport = 0;
            if (nh == 6 || nh == 17) {
                if (!skb_ok(l4_off + 2, 2, len)) { ret = -GF_EFAULT; break; }
                kport = w.r16((uint32_t)(l4_off + 2));
            } else if (nh != 1 && nh != 58) lb_try = false;     // DROP_UNKNOWN_L4: skip_service_lookup
            const gf_htab_desc lb = gload<gf_htab_desc>(&c->lb4);
            if (lb_try && lb.slots) {
                // lb4_lookup_service (lb.h:566-597), LB_L4 then LB_L3
                const uint8_t *svc = nullptr;
                ab += 12;
                if (kport) {
                    uint32_t kw[2] = {daddr, kport};
                    const int64_t f = ht_find<8>(lb, kw, key_hash<8>(kw));
                    ab += 20;
                    if (f >= 0) { const uint8_t *v = ht_val(lb, f); if (gload<uint16_t>(v + 6)) svc = v; }
                    if (!svc) kport = 0;
                }
                if (!svc) {
                    uint32_t kw[2] = {daddr, kport};
                    const int64_t f = ht_find<8>(lb, kw, key_hash<8>(kw));
                    ab += 20;
                    if (f >= 0) { const uint8_t *v = ht_val(lb, f); if (gload<uint16_t>(v + 6)) svc = v; }
                }
                if (svc) {                                    // lb4_local, lb.h:662-699
                    const uint32_t count = gload<uint16_t>(svc + 6);
                    const uint32_t slave = ((fhash ? fhash[i] : 0u) % count + 1u) & 0xffffu;
                    uint32_t kw[2] = {daddr, kport | (slave << 16)};
                    const int64_t f = ht_find<8>(lb, kw, key_hash<8>(kw));
                    ab += 20;
                    if (f < 0) { ret = D_NO_SERVICE; break; }
                    const uint8_t *be = ht_val(lb, f);
                    const uint32_t target = gload<uint32_t>(be), sport_ = gload<uint16_t>(be + 4);
                    r.slave = (uint16_t)slave; r.eflags |= GF_EG_F_LB;
                    r.rev_nat = gload<uint16_t>(be + 8);
                    r.ct_addr = target;
                    uint32_t new_saddr = 0;
                    if (saddr == target) {                    // loopback back to the sender
                        new_saddr = E.loopback; r.ct_addr = new_saddr; r.eflags |= GF_EG_F_LOOPBACK;
                    } else r.t_daddr = target;
                    // lb4_xlate (lb.h:615-659)
                    w.w32(30, target);
                    uint32_t sum = ck_add(ck_add(0u, ~daddr), target);
                    if (new_saddr) {
                        w.w32(26, new_saddr);
                        sum = ck_add(sum, ck_add(ck_add(0u, ~saddr), new_saddr));
                    }
                    l3_csum(w, len, 24, 0, sum, 0);
                    if (co && l4_csum(w, len, l4_off + (int)co, 0, sum, GF_F_PSEUDO_HDR | fl) < 0) { ret = D_CSUM_L4; break; }
                    if (sport_ && kport != sport_ && (nh == 6 || nh == 17)) {   // l4_modify_port
                        if (l4_csum(w, len, l4_off + (int)co, kport, sport_, 2u | fl) < 0) { ret = D_CSUM_L4; break; }
                        if (!skb_ok(l4_off + 2, 2, len)) { ret = D_WRITE_ERROR; break; }
                        w.w16((uint32_t)(l4_off + 2), sport_);
                    }
                    ab += 12;
                }
            }
            r.orig_dip = r.t_daddr;
            // map_lxc_out (bpf_lxc.c:80-108) + l4_port_map_out (l4.h:107-118)
            const uint32_t npm = gload<uint32_t>(&c->n_portmap);
            if (npm && (nh == 6 || nh == 17)) {
                if (!skb_ok(l4_off, 2, len)) { ret = D_INVALID; break; }
                const uint32_t sp = w.r16((uint32_t)l4_off);
                bool bad = false;
                for (uint32_t k = 0; k < npm && k < 16; k++) {
                    const uint32_t pm = gload<uint32_t>(&c->portmap[k]);
                    const uint32_t from = pm & 0xffffu, to = pm >> 16;
                    if (to != sp) continue;
                    if (l4_csum(w, len, l4_off + (int)co, sp, from, 2u | fl) < 0) { ret = D_CSUM_L4; bad = true; break; }
                    if (!skb_ok(l4_off, 2, len)) { ret = D_WRITE_ERROR; bad = true; break; }
                    w.w16((uint32_t)l4_off, from);
                    r.eflags |= GF_EG_F_PORTMAP;
                }
                if (bad) break;
            }
            r.st = 0;                                       // continue in k_eg_groups
        } while (0);
        uint32_t key;
        if (E.hz_fl) {
            uint64_t K[GF_HZ_NK] = {0, 0, 0, 0, 0, 0};
            uint32_t hfl = 0;
            if (r.st == 0) {
                const int lo4 = r.l4_off;
                const bool tu = (r.nh == 6 || r.nh == 17) && skb_ok(lo4 + 0, 4, len);
                bool di = false, de = false, pd;
                if (FAM == 6) {
                    const uint32_t sp = tu ? wg.r16((uint32_t)lo4) : 0u, dp = tu ? wg.r16((uint32_t)lo4 + 2u) : 0u;
                    uint32_t s6[4], d6[4];
                    for (int k = 0; k < 4; k++) { s6[k] = wg.r32(22 + 4 * k); d6[k] = wg.r32(38 + 4 * k); }
                    K[0] = K[1] = hz_key(s6, d6, 4, sp, dp, r.nh, di);           // the IPv6 path keeps its addresses
                    de = di;
                    K[2] = K[3] = hz_key(s6, d6, 4, 0u, 0u, 0x1ffu, pd);
                    K[4] = hz_key(s6, s6, 4, 0u, 0u, 0x2ffu, pd);
                    K[5] = hz_key(d6, d6, 4, 0u, 0u, 0x2ffu, pd);
                    const bool vip = !(r.eflags & GF_EG_F_LB) && vip6_has(E, d6);
                    const bool dlv = E.lxc.slots && lxc_has6(E.lxc, d6);
                    hfl = (r.nh == 58 ? GF_HZ_ICMP : 0u) | (vip ? GF_HZ_VIP : 0u) | GF_HZ_V6 | (dlv ? GF_HZ_DLV : 0u);
                } else {
                    const uint32_t sp = tu ? w.r16((uint32_t)lo4) : 0u, dp = tu ? w.r16((uint32_t)lo4 + 2u) : 0u;
                    const uint32_t fs = w.r32(26), fd = w.r32(30), ts = r.t_saddr, td = r.t_daddr;
                    K[0] = hz_key(&fs, &fd, 1, sp, dp, r.nh, di);
                    K[1] = hz_key(&ts, &td, 1, sp, dp, r.nh, de);
                    K[2] = hz_key(&fs, &fd, 1, 0u, 0u, 0x1ffu, pd);
                    K[3] = hz_key(&ts, &td, 1, 0u, 0u, 0x1ffu, pd);
                    K[4] = hz_key(&fs, &fs, 1, 0u, 0u, 0x2ffu, pd);
                    K[5] = hz_key(&fd, &fd, 1, 0u, 0u, 0x2ffu, pd);
                    const bool vip = !(r.eflags & GF_EG_F_LB) && vip4_has(E, fd);
                    const bool dlv = (E.lxc.slots && (E.lxset ? aset_has(E.lxset, E.lxbits, E.lxzero, fd) : lxc_has4(E.lxc, fd))) ||
                                     (E.loopback && fd == E.loopback);
                    hfl = (r.nh == 1 ? GF_HZ_ICMP : 0u) | (vip ? GF_HZ_VIP : 0u) |
                          ((r.eflags & GF_EG_F_LOOPBACK) ? GF_HZ_LOOP : 0u) | (dlv ? GF_HZ_DLV : 0u);
                }
                hfl |= GF_HZ_VALID | (di ? GF_HZ_DIRI : 0u) | (de ? GF_HZ_DIRE : 0u);
            }
            for (uint32_t k = 0; k < GF_HZ_NK; k++) E.hz_k[(size_t)k * fr.n + i] = K[k];
            E.hz_fl[i] = (uint8_t)hfl;
            if (hfl & (GF_HZ_ICMP | GF_HZ_VIP)) atomicOr(E.hz + 1, hfl);   // the batch's kinds
        }
        if (r.st == 0 && FAM == 6) {
            uint32_t s6[4], d6[4];
            for (int k = 0; k < 4; k++) { s6[k] = wg.r32(22 + 4 * k); d6[k] = wg.r32(38 + 4 * k); }
            key = gf_key_live(gf_pair_hash6(s6, d6) & GF_KEY_HASH) | GF_KEY_FAM;   // the IPv6 family of the schedule
        } else if (r.st == 0) {
            key = gf_key_live(gf_pair_hash4(r.t_saddr, r.t_daddr) & GF_KEY_HASH);
            if (E.conn) {
                E.keysP[i] = key;
                const bool tu = (r.nh == 6 || r.nh == 17) && skb_ok(r.l4_off, 4, len);
                const uint32_t sp = tu ? w.r16((uint32_t)r.l4_off) : 0u, dp = tu ? w.r16((uint32_t)r.l4_off + 2u) : 0u;
                key = gf_key_live(gf_conn_hash4(r.t_saddr, sp, r.t_daddr, dp, r.nh) & GF_KEY_HASH);
                if (r.nh == 1) atomicOr(E.cflag, 1u);
            }
            const uint32_t lo = E.loopback;
            if (r.t_saddr == r.t_daddr || (lo && (r.t_saddr == lo || r.t_daddr == lo)) || (E.strict & 1u)) *E.seq = 1u;
        } else {
            key = GF_KEY_SKIP;                        // final in the front: k_eg_groups has nothing to do
            if (E.conn) E.keysP[i] = key;
            if (o.stage == GF_STAGE_FROM_LXC) {
                if (ret < 0 || ret == TC_SHOT) {
                    o.action = TC_SHOT; o.reason = (uint8_t)(-ret);
                    o.eg_flags = r.eflags & (GF_EG_F_LB | GF_EG_F_LOOPBACK | GF_EG_F_PORTMAP | GF_EG_F_IPV6);
                    o.slave = r.slave; o.rev_nat = r.rev_nat;
                } else o.action = (uint8_t)ret;
            }
            out[i] = o;
            scnt = true; sreason = o.reason; saction = o.action; slen = len; sab = ab;
        }
        erec[i] = r;
        keys[i] = key;
        {                                                     // not (yet) a local delivery: skipped by the
            gf_rec rr;                                        // handle_policy pass (coalesced writes here,
            const uint32_t k2 = pack_rec(i, 0, len, 0, 0, 0, 0, 0, 0, 0, 0, r.ep, 0, true, false, nullptr, nullptr, rr);
            E.rec2[i] = rr;                                   // none for most packets in k_eg_groups)
            E.key2[i] = k2;
            if (E.conn) E.key2P[i] = k2;
        }
        if (FAM == 4 && !coop) eg_copy(dst, row, K);         // the frame as the front left it
    }
    if (coop) {             // every row of the block (IPv6 rows unchanged: k_eg_front<6> rewrites them after)
        __syncthreads();
        uint4 *g = reinterpret_cast<uint4 *>(E.snap + (size_t)b0 * S);
        for (uint32_t k = threadIdx.x; k < nv; k += BLOCK) g[k] = lds[k];
    }
    if (stats) { st.pkt_wave(scnt, sreason, saction, slen, sab); st.flush(stats); }
}

// After the front: a flagged batch runs as one bucket per family (every IPv4
// key equal; the IPv6 path writes no service entries and keeps its own bucket).
// With connection groups and an IPv4 ICMP packet in the run: the pair keys.
// The deliveries' keys of a run that fell back to pair groups (*cflag): their pair keys.
__global__ __launch_bounds__(BLOCK) void k_eg_pick_keys(const uint32_t *cflag, const uint32_t *key2P, uint32_t n,
                                                        uint32_t *keys) {
    if (!*cflag) return;
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) keys[i] = key2P[i];
}
__global__ __launch_bounds__(BLOCK) void k_eg_seq_keys(const uint32_t *seq, const uint32_t *cflag,
                                                       const uint32_t *keysP, uint32_t n, uint32_t *keys) {
    if (*seq) {
        for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) keys[i] &= GF_KEY_FAM;
    } else if (cflag && *cflag) {
        for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK)
            if (!(keys[i] & GF_KEY_FAM)) keys[i] = keysP[i];
    }
}

// The ordering check: every continuing packet records the first batch index of
// its connection key per direction (open addressing, key 0 = empty)...
__device__ __forceinline__ void hz_put(unsigned long long k, uint32_t half, uint32_t i, unsigned long long *tkey,
                                       uint32_t *tfirst, uint32_t mask) {
    uint32_t slot = (uint32_t)(k >> 32) & mask;
    for (uint32_t probe = 0; probe <= mask; probe++) {
        const unsigned long long old = atomicCAS(&tkey[slot], 0ull, k);
        if (old == 0ull || old == k) { atomicMin(&tfirst[2 * slot + half], i); return; }
        slot = (slot + 1u) & mask;
    }
}
__device__ __forceinline__ uint32_t hz_get(unsigned long long k, uint32_t half, const unsigned long long *tkey,
                                           const uint32_t *tfirst, uint32_t mask) {
    uint32_t slot = (uint32_t)(k >> 32) & mask;
    for (uint32_t probe = 0; probe <= mask; probe++) {
        const unsigned long long t = tkey[slot];
        if (t == k) return tfirst[2 * slot + half];
        if (t == 0ull) break;
        slot = (slot + 1u) & mask;
    }
    return 0xffffffffu;
}
struct HzTab { unsigned long long *key; uint32_t *first; uint32_t mask; };
// The connection table is never cleared: a slot belongs to the current call when
// its key word carries the call's 16-bit generation (key = gen << 48 | 48 hash
// bits), and a first-index word is (gen << 32 | ~index), kept by atomicMax.  The
// host clears it when the generation wraps or the table is reallocated.
struct HzGen { unsigned long long *key; unsigned long long *first; uint32_t mask; uint32_t gen; };
__device__ __forceinline__ void hzg_put(const HzGen &T, unsigned long long k, uint32_t half, uint32_t i) {
    const unsigned long long want = ((unsigned long long)T.gen << 48) | (k & 0xffffffffffffull);
    uint32_t slot = (uint32_t)(k >> 32) & T.mask;
    for (uint32_t probe = 0; probe <= T.mask;) {
        unsigned long long cur = T.key[slot];
        if ((uint32_t)(cur >> 48) != T.gen) {          // a stale slot: claim it
            const unsigned long long old = atomicCAS(&T.key[slot], cur, want);
            if (old != cur) continue;                   // changed under us: look again
            cur = want;
        }
        if (cur == want) {
            atomicMax(&T.first[2 * slot + half], ((unsigned long long)T.gen << 32) | (0xffffffffull - i));
            return;
        }
        slot = (slot + 1u) & T.mask;
        probe++;
    }
}
__device__ __forceinline__ uint32_t hzg_get(const HzGen &T, unsigned long long k, uint32_t half) {
    const unsigned long long want = ((unsigned long long)T.gen << 48) | (k & 0xffffffffffffull);
    uint32_t slot = (uint32_t)(k >> 32) & T.mask;
    for (uint32_t probe = 0; probe <= T.mask; probe++) {
        const unsigned long long cur = T.key[slot];
        if ((uint32_t)(cur >> 48) != T.gen) break;
        if (cur == want) {
            const unsigned long long w = T.first[2 * slot + half];
            return (uint32_t)(w >> 32) == T.gen ? 0xffffffffu - (uint32_t)w : 0xffffffffu;
        }
        slot = (slot + 1u) & T.mask;
    }
    return 0xffffffffu;
}
// The pair / address keys live in a second table, cleared (here, on the device)
// only for a batch with ICMP or GF_HZ_VIP packets.
__global__ __launch_bounds__(BLOCK) void k_hz_clear(HzTab A, const uint32_t *hz) {
    if (!(hz[1] & (GF_HZ_ICMP | GF_HZ_VIP))) return;
    for (uint64_t k = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; k <= A.mask; k += (uint64_t)gridDim.x * BLOCK) {
        A.key[k] = 0ull;
        A.first[2 * k] = A.first[2 * k + 1] = 0xffffffffu;
    }
}
__global__ __launch_bounds__(BLOCK) void k_hz_insert(const uint64_t *K, const uint8_t *fl, uint32_t n,
                                                     const uint32_t *hz, HzGen C, HzTab A) {
    const uint32_t kinds = hz[1];                       // pair / address keys only when a packet probes them
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) {
        const uint32_t f = fl[i];
        if (!(f & GF_HZ_VALID)) continue;
        if (f & GF_HZ_DLV) hzg_put(C, K[i], (f & GF_HZ_DIRI) ? 1u : 0u, i);
        if (kinds & GF_HZ_ICMP) {
            hz_put(K[2ull * n + i], 0u, i, A.key, A.first, A.mask);
            if (f & GF_HZ_ICMP) hz_put(K[2ull * n + i] ^ GF_HZ_ICMPSALT, 0u, i, A.key, A.first, A.mask);
        }
        if (kinds & GF_HZ_VIP) {
            hz_put(K[4ull * n + i], 0u, i, A.key, A.first, A.mask);
            hz_put(K[5ull * n + i], 0u, i, A.key, A.first, A.mask);
        }
    }
}
// ... then each packet probes what its from-container part touches; a hit on an
// earlier index flags the batch.
__global__ __launch_bounds__(BLOCK) void k_hz_probe(const uint64_t *K, const uint8_t *fl, uint32_t n, HzGen C,
                                                    HzTab A, uint32_t strict, uint32_t *hz) {
    const uint32_t kinds = hz[1];
    bool hit = false, each = false;
    uint32_t first = 0xffffffffu;
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) {
        const uint32_t f = fl[i];
        if (!(f & GF_HZ_VALID)) continue;
        each |= (strict & ((f & GF_HZ_V6) ? 2u : 1u)) != 0;
        hit |= hzg_get(C, K[1ull * n + i], (f & GF_HZ_DIRE) ? 0u : 1u) < i;
        if (kinds & GF_HZ_ICMP) {
            if (f & GF_HZ_ICMP) hit |= hz_get(K[3ull * n + i], 0u, A.key, A.first, A.mask) < i;
            hit |= hz_get(K[3ull * n + i] ^ GF_HZ_ICMPSALT, 0u, A.key, A.first, A.mask) < i;
        }
        if (f & GF_HZ_LOOP)
            hit |= hzg_get(C, K[i], 0u) < i || hzg_get(C, K[i], 1u) < i;
        if (f & GF_HZ_VIP) hit |= hz_get(K[4ull * n + i], 0u, A.key, A.first, A.mask) < i;
        if (hit && first == 0xffffffffu) first = i;
    }
    // the earliest flagged packet: everything before it is a run without a hazard
    uint32_t m = first;
    for (int o = 32; o > 0; o >>= 1) m = min(m, (uint32_t)__shfl_xor(m, o));
    if ((threadIdx.x & 63u) == 0 && m != 0xffffffffu) atomicMin(hz + 2, m);
    if (__any(each) && (threadIdx.x & 63u) == 0) atomicOr(hz, 2u);
    else if (__any(hit) && (threadIdx.x & 63u) == 0) atomicOr(hz, 1u);
}

// Adds a call's counter block to the registered sink.
__global__ void k_stats_fold(const unsigned long long *src, unsigned long long *dst) {
    for (int k = threadIdx.x; k < 272; k += blockDim.x)
        if (src[k]) atomicAdd(&dst[k], src[k]);
}

// __ct_lookup hit part for CT_EGRESS (conntrack.h:75-135): tx accounting (the
// cold part of the value), TX_CLOSING on close.
__device__ __forceinline__ void ct_hit_eg(const gf_htab_desc &d, int64_t f, int action, bool syn, uint32_t len,
                                          uint32_t now, bool acct, CtState &st) {
    uint8_t *e = ht_val(d, (uint64_t)f);
    uint4 hot = gload<uint4>(e);
    uint32_t life = hot.x, fl = hot.y & 0xffffu;
    if (!(fl & F_RX_CLOSING) || !(fl & F_TX_CLOSING)) {
        if (!syn) fl |= F_SEEN_NON_SYN;
        life = now + ((fl & F_SEEN_NON_SYN) ? 43200u : 300u);
    }
    st.rev_nat = hot.y >> 16;
    st.loopback = (fl >> 3) & 1u;
    if (acct && !(GF_DIAG & 64)) {                      // tx_packets += 1, tx_bytes += len (GF_DIAG & 64: ablation)
        uint8_t *base = d.sstride ? ht_side(d, (uint64_t)f) - 16 : e;   // internal value word k at base + 4k
        gstore<unsigned long long>(base + 24, gload<unsigned long long>(base + 24) + 1ull);
        gstore<unsigned long long>(base + 32, gload<unsigned long long>(base + 32) + (unsigned long long)len);
    }
    if (action == ACT_CREATE) {
        if (fl & (F_RX_CLOSING | F_TX_CLOSING)) {
            fl &= ~(F_RX_CLOSING | F_TX_CLOSING);
            if (!syn) fl |= F_SEEN_NON_SYN;
            life = now + ((fl & F_SEEN_NON_SYN) ? 43200u : 300u);
        }
    } else if (action == ACT_CLOSE) {
        fl |= F_TX_CLOSING;
        if ((fl & F_RX_CLOSING) && (fl & F_TX_CLOSING)) life = now + 10u;
    }
    hot.x = life;
    hot.y = (hot.y & 0xffff0000u) | fl;
    gstore<uint4>(e, hot);
    GF_WR(WR_HIT);
}

// policy_can_egress4 (policy.h:241-264 with POLICY_EGRESS, else :282-289):
// ipcache identity, __policy_can_access(dir = CT_EGRESS: key.egress = 1, the
// CFG_L3L4_EGRESS list), reserved identities through CIDR4_EGRESS_MAP.
__device__ __forceinline__ int eg_policy(const gf_lxc_dev *c, uint32_t flags, uint32_t dst_id, const uint32_t *da, bool v6,
                         uint32_t dport, uint32_t proto, uint32_t len, uint32_t &ab) {
    if (flags & GF_LXC_F_DROP_ALL) return D_POLICY;
    if (!(flags & GF_LXC_F_POLICY_EGRESS)) return TC_OK;
    uint32_t identity = dst_id;
    const gf_htab_desc ic = gload<gf_htab_desc>(&c->ipcache);
    if (ic.slots) {
        uint32_t kw[5] = {da[0], v6 ? da[1] : 0u, v6 ? da[2] : 0u, v6 ? da[3] : 0u, v6 ? 2u : 1u};
        const int64_t f = ht_find<20>(ic, kw, key_hash<20>(kw));
        ab += 20;
        if (f >= 0) { identity = gload<uint16_t>(ht_val(ic, f)); ab += 8; }
    }
    const gf_htab_desc pd = gload<gf_htab_desc>(&c->policy);
    int verdict = D_POLICY;
    int64_t f = -1;
    bool l4hit = false;
    if (flags & GF_LXC_F_HAVE_L4_POLICY) {
        uint32_t kw[2] = {identity, dport | (proto << 16) | (1u << 24)};
        f = ht_find<8, GF_POL_U>(pd, kw, key_hash<8, GF_HASH_POLICY>(kw));
        ab += 8;
        l4hit = f >= 0;
    }
    if (f < 0) {
        uint32_t kw[2] = {identity, 1u << 24};
        f = ht_find<8, GF_POL_U>(pd, kw, key_hash<8, GF_HASH_POLICY>(kw));
        ab += 8;
        if (f >= 0) verdict = TC_OK;
    }
    if (f < 0 && (flags & GF_LXC_F_HAVE_L4_POLICY)) {
        uint32_t kw[2] = {0u, dport | (proto << 16) | (1u << 24)};
        f = ht_find<8, GF_POL_U>(pd, kw, key_hash<8, GF_HASH_POLICY>(kw));
        ab += 8;
        l4hit = f >= 0;
    }
    if (f >= 0) {
        uint8_t *cnt = pd.vals + (uint64_t)f * GF_POL_SIDE;          // packets / bytes (policy.h:67-92)
        pol_count_add(cnt, 1u, len, false);
        ab += 40;
        if (l4hit) {
            const uint32_t pp = gload<uint16_t>(ht_val(pd, (uint64_t)f));
            verdict = 0;
            if (pp) verdict = (int)pp;
            else if (proto == 6 || proto == 17) {         // l4_egress_proxy_lookup (l4.h:178-188)
                const uint32_t n = gload<uint32_t>(&c->n_l4e);
                for (uint32_t k = 0; k < n; k++) {
                    const gf_l4_allow_dev a = gload<gf_l4_allow_dev>(&c->l4e[k]);
                    if (a.port && a.port == dport) { if (a.nexthdr && a.nexthdr == proto) { verdict = a.proxy; break; } }
                }
            }
        }
    }
    if (identity < 256 && verdict < 0) {               // identity_is_reserved -> lpm{4,6}_egress_lookup
        const gf_trie_desc tr = gload<gf_trie_desc>(v6 ? &c->cidr6e : &c->cidr4e);
        if (tr.root_bits) ab += v6 ? 21 : 9;
        verdict = (v6 ? trie_lookup<4>(tr, da) : trie_lookup<1>(tr, da)) ? 0 : D_POLICY_CIDR;
    }
    return verdict;
}

// The from-container program's CT map (CT_MAP4 / CT_MAP6 of the sending endpoint):
// the global one of the launch, or (PCT, ConntrackLocal) the program's own.
template <int FAM, bool PCT>
__device__ __forceinline__ gf_htab_desc eg_ct(const EgDev &E, const gf_lxc_dev *c) {
    if constexpr (PCT) return gload<gf_htab_desc>(FAM == 6 ? &c->ct6 : &c->ct4);
    else return FAM == 6 ? E.ct6 : E.ct4;
}

// The CT / policy part of handle_ipv4_from_lxc (bpf_lxc.c:499-658) for packet i.
// Returns TC_OK / TC_REDIRECT / ND_TAILCALL (local delivery; ifx, lxc, mapped
// filled) or an error.
template <bool PCT>
__device__ __forceinline__ int eg_ct_part(const EgDev &E, const EgRec &r, uint32_t i, Row &w, gf_egress_out &o, uint32_t &ifx,
                          uint32_t &lxc, int *added, bool seq, bool rlog, uint32_t &ab) {
    const uint32_t len = r.len, nh = r.nh;
    const int l4_off = r.l4_off;
    const gf_lxc_dev *c = E.cfgs + (r.ep - 1);
    const uint32_t flags = gload<uint32_t>(&c->flags);
    const uint32_t co = csum_l4_offset(nh), fl = nh == 17 ? GF_F_MANGLED_0 : 0u;
    // ct_lookup4(CT_EGRESS): the L4 words as the frame holds them now
    gf_rec hr{};
    hr.len = len; hr.l4_off = (int16_t)l4_off;
    for (int k = 0; k < 4; k++) { const int64_t off = (int64_t)l4_off + k; if (off >= 0 && off < (int64_t)len) hr.l4w0 |= w.b((uint32_t)off) << (8 * k); }
    {
        uint32_t w3 = 0;
        for (int k = 0; k < 2; k++) { const int64_t off = (int64_t)l4_off + 12 + k; if (off >= 0 && off < (int64_t)len) w3 |= w.b((uint32_t)off) << (8 * k); }
        hr.l4w3 = (uint16_t)w3;
    }
    uint32_t t[4] = {r.t_daddr, r.t_saddr, 0u, nh};
    uint32_t tfl = 1u;                                  // TUPLE_F_IN (egress)
    int action; bool syn;
    int e = ct_l4(nh, false, hr, t[2], tfl, action, syn);
    if (e < 0) return e;
    t[3] = nh | (tfl << 8);
    if (!(flags & GF_LXC_DEV_HAS_CT4)) return D_CT_CREATE_FAILED;   // (no CT map bound: never in a valid config)
    const gf_htab_desc ct = eg_ct<4, PCT>(E, c);
    const bool acct = (flags & GF_LXC_F_CT_ACCOUNTING) != 0;
    uint32_t tf[4] = {t[1], t[0], (t[2] >> 16) | (t[2] << 16), nh | ((tfl ^ 1u) << 8)};
    bool isb = false;
#if GF_EG_COOP
    // the home line read by the lane quad together (the egress CT4 holds 2^28 slots, 8 GB)
    ProbeLine<14, GF_CT4_U, 4> cl;
    cl.load_quad(ct, key_hash<14, GF_HASH_CT>(t));
    const ProbeRes pr = probe2<14, GF_CT4_U, 4>(ct, t, tf, cl, true);
    const int64_t f = pr.f;
    isb = pr.is_b;
#else
    const int64_t f = ht_find2<14, GF_CT4_U>(ct, t, tf, key_hash<14, GF_HASH_CT>(t), &isb);
#endif
    ab += 14;
    CtState st{0, 0, 0};
    int ret;
    if (f >= 0 && !isb) {
        ab += 96;
        ct_hit_eg(ct, f, action, syn, len, E.now, acct, st);
        ret = (tfl & 2u) ? CT_RELATED : CT_REPLY;
    } else {
        ab += 14;
        for (int k = 0; k < 4; k++) t[k] = tf[k];
        tfl ^= 1u;
        if (f >= 0) { ab += 96; ct_hit_eg(ct, f, action, syn, len, E.now, acct, st); ret = CT_ESTABLISHED; }
        else ret = CT_NEW;
    }
    o.eg_ct_ret = (uint8_t)ret;
    const uint32_t dst_id = ((r.orig_dip & E.cluster_mask) == E.cluster_range) ? 3u : 2u;   // CLUSTER_ID / WORLD_ID
    if (E.X.tmark && dst_id == 3u) E.X.tmark[i] |= GF_TR_CLUSTER;
    const int verdict = eg_policy(c, flags, dst_id, &t[1], false, t[2] & 0xffffu, nh, len, ab);
    if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
        if (ret == CT_ESTABLISHED) {
            ab += 14;
            ht_delete<14, GF_HASH_CT, GF_CT4_U>(ct, t, (E.strict & 1) != 0, added);
            o.eg_flags |= GF_EG_F_DELETED;
        }
        return verdict;
    }
    if (ret == CT_NEW) {                                // ct_create4(CT_EGRESS), conntrack.h:503-580
        ab += 3 * (14 + 48);
        const uint32_t loop = (r.eflags & GF_EG_F_LOOPBACK) ? 1u : 0u;
        uint32_t efl = (nh == 6) ? 0u : F_SEEN_NON_SYN;
        efl |= loop ? F_LB_LOOPBACK : 0u;
        const uint32_t life = E.now + ((efl & F_SEEN_NON_SYN) ? 43200u : 300u);
        const uint32_t seclabel = gload<uint32_t>(&c->seclabel);
        // GF_VCODEC_CT: lifetime, flags|rev_nat, rx lo x2, rx hi x2, tx_packets, tx_bytes, unused, src_sec_id
        uint32_t v[12] = {life, efl | ((uint32_t)r.rev_nat << 16), 0u, 0u, 0u, 0u, 1u, 0u, len, 0u, 0u, seclabel};
        const bool strict = (E.strict & 1) != 0;
        if (ht_upsert<14, 12, GF_HASH_CT, GF_CT4_U>(ct, t, v, strict, added) < 0) return D_CT_CREATE_FAILED;
        if (r.ct_addr) {
            uint32_t t2[4] = {r.ct_addr, t[1], t[2], t[3]};          // dir EGRESS: tuple->daddr = ct_state->addr
            if (loop) { t2[3] = nh | (1u << 8); t2[1] = r.t_saddr; }  // TUPLE_F_IN, tuple->saddr = svc_addr
            if (seq) {
                if (ht_upsert<14, 12, GF_HASH_CT, GF_CT4_U>(ct, t2, v, strict, added) < 0) return D_CT_CREATE_FAILED;
            } else {
                uint32_t *lg = E.ctlog + (size_t)GF_CTLOG_WORDS * atomicAdd(E.ctlog_n, 1u);
                lg[0] = i;
                for (int k = 0; k < 4; k++) lg[1 + k] = t2[k];
                for (int k = 0; k < 12; k++) lg[5 + k] = v[k];
                if constexpr (PCT) {                    // the entry's map: its program and its slot array
                    lg[17] = r.ep;
                    lg[18] = (uint32_t)(uintptr_t)ct.slots; lg[19] = (uint32_t)((uintptr_t)ct.slots >> 32);
                }
            }
        }
        uint32_t it[4] = {t[0], t[1], 0u, 1u | ((((t[3] >> 8) & 0xffu) | 2u) << 8)};
        v[1] |= F_SEEN_NON_SYN;
        if (rlog && GF_EG_RSET && E.rs.slot) {          // the run's set (RelSet), applied after the run
            rset_put(E.rs, it[0], it[1], (it[3] >> 8) & 1u, 2u * i);
        } else if (rlog) {                              // applied after the run, in packet order (the pair's
            uint32_t *lg = E.rlog + (size_t)GF_CTLOG_WORDS * wave_reserve(E.rlog_n);   // other connections
            lg[0] = 2u * i;                                                             // never read it)
            for (int k = 0; k < 4; k++) lg[1 + k] = it[k];
            for (int k = 0; k < 12; k++) lg[5 + k] = v[k];
        } else if (ht_upsert<14, 12, GF_HASH_CT, GF_CT4_U>(ct, it, v, strict, added) < 0) {
            return D_CT_CREATE_FAILED;
        }
        o.eg_flags |= GF_EG_F_CREATED;
    } else if (ret == CT_REPLY || ret == CT_RELATED) {
        if (st.rev_nat) {                               // lb4_rev_nat(flags 0), lb.h:447-534
            const gf_htab_desc rn = gload<gf_htab_desc>(&c->revnat4);
            uint32_t kw[1] = {st.rev_nat};
            const int64_t fr_ = ht_find<2>(rn, kw, key_hash<2>(kw));
            ab += 8;
            if (fr_ >= 0) {
                const uint8_t *nat = ht_val(rn, fr_);
                const uint32_t port = gload<uint16_t>(nat + 4);
                if (port) {                             // reverse_map_l4_port
                    if (nh == 6 || nh == 17) {
                        if (!skb_ok(l4_off, 2, len)) return -GF_EFAULT;
                        const uint32_t old = w.r16((uint32_t)l4_off);
                        if (port != old) {
                            if (l4_csum(w, len, l4_off + (int)co, old, port, 2u | fl) < 0) return D_CSUM_L4;
                            if (!skb_ok(l4_off, 2, len)) return D_WRITE_ERROR;
                            w.w16((uint32_t)l4_off, port);
                        }
                    } else if (nh != 1 && nh != 58) return D_UNKNOWN_L4;
                }
                const uint32_t old_sip = w.r32(26), new_sip = gload<uint32_t>(nat);
                uint32_t sum = 0;
                if (st.loopback) {
                    const uint32_t old_dip = w.r32(30);
                    w.w32(30, old_sip);
                    sum = ck_add(ck_add(0u, ~old_dip), old_sip);
                    t[1] = old_sip;
                }
                w.w32(26, new_sip);
                sum = ck_add(sum, ck_add(ck_add(0u, ~old_sip), new_sip));
                l3_csum(w, len, 24, 0, sum, 0);
                if (co && l4_csum(w, len, l4_off + (int)co, 0, sum, GF_F_PSEUDO_HDR | fl) < 0) return D_CSUM_L4;
                ab += 16;
            }
            o.eg_flags |= GF_EG_F_REVNAT;
        }
    }
    uint32_t nm[2] = {gload<uint32_t>(&c->node_mac[0]), gload<uint32_t>(&c->node_mac[1])};
    if (verdict > 0) {                                  // ipv4_redirect_to_host_port + ipv4_l3 -> HOST_IFINDEX
        if (E.X.tmark)
            trace_proxy(E.X.tmark, E.X.tcap, E.snap + (size_t)i * E.stride, w.p, w.cap, trace_cap_len(len, E.stride), i,
                        GF_TR_PX_EGRESS);
        const int r3 = redirect_checks(len, l4_off, nh);
        if (r3 < 0) return r3;
        const uint32_t od[1] = {r.orig_dip};
        const uint32_t np = (uint32_t)verdict & 0xffffu, gw = E.X.gw;
        l4_csum(w, len, l4_off + (int)co, t[2] & 0xffffu, np, 2u | fl);   // l4_modify_port (lxc.h:124)
        w.w16((uint32_t)(l4_off + 2), np);
        w.w32(30, gw);                                                    // daddr = IPV4_GATEWAY
        l3_csum(w, len, 24, r.orig_dip, gw, 4);
        if (co) l4_csum(w, len, l4_off + (int)co, r.orig_dip, gw, 4u | GF_F_PSEUDO_HDR | fl);
        pol_redirect(E.X, i, len, l4_off, nh, t, false, np, od, gload<uint32_t>(&c->seclabel), 1u);
        o.eg_flags |= GF_EG_F_PROXY;
        o.proxy_port = (uint16_t)verdict;
        const int r4 = eg_ipv4_l3(w, len, nm, E.host_mac);
        if (r4 != TC_OK) return r4;
        ifx = E.host_ifindex;
        return TC_REDIRECT;
    }
    const uint32_t dip = w.r32(30);
    if (E.lxc.slots) {                                  // lookup_ip4_endpoint
        uint32_t kw[5] = {dip, 0, 0, 0, 1u};
        const int64_t fe = E.lxset ? aset_slot(E.lxset, E.lxbits, E.lxzero, dip) : ht_find<20>(E.lxc, kw, key_hash<20>(kw));
        ab += 20;
        if (fe >= 0) {
            const uint8_t *ep = ht_val(E.lxc, fe);
            ab += 8;
            if (gload<uint32_t>(ep + 8) & 1u) {         // ENDPOINT_F_HOST -> to_host
                if (!E.host_ifindex) return D_NO_LXC;
                const int r4 = eg_ipv4_l3(w, len, nm, E.host_mac);
                if (r4 != TC_OK) return r4;
                o.eg_flags |= GF_EG_F_TO_HOST;
                ifx = E.host_ifindex;
                return TC_REDIRECT;
            }
            // ipv4_local_delivery (l3.h:136-168): ipv4_l3(node_mac, mac), map_lxc_in, tail call
            const uint32_t ttl = w.b(22);
            if (ttl <= 1) return D_INVALID;
            l3_csum(w, len, 24, ttl, ttl - 1, 2);
            w.w8(22, ttl - 1);
            o.eg_flags |= GF_EG_F_LOCAL;
            uint32_t mapped = 0, ndport = 0;
            return delivery_tail(w, len, l4_off, nh, ep, ifx, lxc, mapped, ndport, ab);
        }
    }
    if (E.encap_ifindex && E.tunnel.slots) {            // encap_and_redirect (lib/encap.h)
        uint32_t kw[5] = {dip & E.ipv4_mask, 0, 0, 0, 1u};
        const int64_t ft = E.tnset ? aset_slot(E.tnset, E.tnbits, E.tnzero, kw[0]) : ht_find<20>(E.tunnel, kw, key_hash<20>(kw));
        ab += 20;
        if (ft >= 0) {
            o.tunnel_ip = __builtin_bswap32(gload<uint32_t>(ht_val(E.tunnel, ft)));
            o.eg_flags |= GF_EG_F_ENCAP;
            ifx = E.encap_ifindex;
            ab += 20;
            return TC_REDIRECT;
        }
    }
    const int r4 = eg_ipv4_l3(w, len, nullptr, nm);    // pass_to_stack
    if (r4 != TC_OK) return r4;
    o.eg_flags |= GF_EG_F_TO_STACK;
    return TC_OK;
}

// ipv6_l3 (bpf/lib/l3.h:31-52) + ipv6_dec_hoplimit (bpf/lib/ipv6.h:178-193); smac may
// be null.  ND_ICMP6_TE: the hop limit ran out (icmp6_send_time_exceeded).
__device__ __forceinline__ int eg_ipv6_l3(Row &w, const uint32_t *smac, const uint32_t *dmac) {
    const uint32_t hl = w.b(21);
    if (hl <= 1) return ND_ICMP6_TE;
    w.w8(21, hl - 1);
    if (smac) { w.w32(6, smac[0]); w.w16(10, smac[1] & 0xffffu); }
    w.w32(0, dmac[0]); w.w16(4, dmac[1] & 0xffffu);
    return TC_OK;
}

// The CT / policy part of ipv6_l3_from_lxc (bpf_lxc.c:186-386) for packet i, on
// the frame in HBM (extension headers may put the L4 header anywhere in the snap).
template <bool PCT>
__device__ __forceinline__ int eg_ct_part6(const EgDev &E, const EgRec &r, uint32_t i, Row &w, gf_egress_out &o,
                                           uint32_t &ifx, uint32_t &lxc, int *added, uint32_t &ab) {
    const uint32_t len = r.len, nh = r.nh;
    const int l4_off = r.l4_off;
    const gf_lxc_dev *c = E.cfgs + (r.ep - 1);
    const uint32_t flags = gload<uint32_t>(&c->flags);
    const uint32_t co = csum_l4_offset(nh), fl = nh == 17 ? GF_F_MANGLED_0 : 0u;
    gf_rec hr{};
    hr.len = len; hr.l4_off = (int16_t)l4_off;
    for (int k = 0; k < 4; k++) { const int64_t off = (int64_t)l4_off + k; if (off >= 0 && off < (int64_t)len) hr.l4w0 |= w.b((uint32_t)off) << (8 * k); }
    {
        uint32_t w3 = 0;
        for (int k = 0; k < 2; k++) { const int64_t off = (int64_t)l4_off + 12 + k; if (off >= 0 && off < (int64_t)len) w3 |= w.b((uint32_t)off) << (8 * k); }
        hr.l4w3 = (uint16_t)w3;
    }
    uint32_t t[10];
    for (int k = 0; k < 4; k++) { t[k] = w.r32(38 + 4 * k); t[4 + k] = w.r32(22 + 4 * k); }
    const uint32_t od[4] = {t[0], t[1], t[2], t[3]};   // orig_dip (after lb6_local)
    t[8] = 0; t[9] = nh;
    uint32_t tfl = 1u;                                  // TUPLE_F_IN (egress)
    int action; bool syn;
    int e = ct_l4(nh, true, hr, t[8], tfl, action, syn);
    if (e < 0) return e;
    t[9] = nh | (tfl << 8);
    if (!(flags & GF_LXC_DEV_HAS_CT6)) return D_CT_CREATE_FAILED;
    const gf_htab_desc ct = eg_ct<6, PCT>(E, c);
    const bool acct = (flags & GF_LXC_F_CT_ACCOUNTING) != 0;
    uint32_t tf[10];
    for (int k = 0; k < 4; k++) { tf[k] = t[4 + k]; tf[4 + k] = t[k]; }
    tf[8] = (t[8] >> 16) | (t[8] << 16);
    tf[9] = nh | ((tfl ^ 1u) << 8);
    bool isb = false;
    const int64_t f = ht_find2<40, GF_CT6_U>(ct, t, tf, key_hash<40, GF_HASH_CT>(t), &isb);
    ab += 40;
    CtState st{0, 0, 0};
    int ret;
    if (f >= 0 && !isb) {
        ab += 96;
        ct_hit_eg(ct, f, action, syn, len, E.now, acct, st);
        ret = (tfl & 2u) ? CT_RELATED : CT_REPLY;
    } else {
        ab += 40;
        for (int k = 0; k < 10; k++) t[k] = tf[k];
        tfl ^= 1u;
        if (f >= 0) { ab += 96; ct_hit_eg(ct, f, action, syn, len, E.now, acct, st); ret = CT_ESTABLISHED; }
        else ret = CT_NEW;
    }
    o.eg_ct_ret = (uint8_t)ret;
    const uint32_t dst_id = (w.r32(38) == E.router6[0] && w.r32(42) == E.router6[1]) ? 3u : 2u;
    if (E.X.tmark && dst_id == 3u) E.X.tmark[i] |= GF_TR_CLUSTER;
    const int verdict = eg_policy(c, flags, dst_id, &t[4], true, t[8] & 0xffffu, nh, len, ab);
    const bool strict = (E.strict & 2) != 0;
    if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
        if (ret == CT_ESTABLISHED) {
            ab += 40;
            ht_delete<40, GF_HASH_CT, GF_CT6_U>(ct, t, strict, added);
            o.eg_flags |= GF_EG_F_DELETED;
        }
        return verdict;
    }
    if (ret == CT_NEW) {                                // ct_create6(CT_EGRESS), conntrack.h:446-493
        ab += 2 * (40 + 48);
        const uint32_t efl = (nh == 6) ? 0u : F_SEEN_NON_SYN;
        const uint32_t life = E.now + ((efl & F_SEEN_NON_SYN) ? 43200u : 300u);
        uint32_t v[12] = {life, efl | ((uint32_t)r.rev_nat << 16), 0u, 0u, 0u, 0u, 1u, 0u, len, 0u, 0u,
                          gload<uint32_t>(&c->seclabel)};
        if (ht_upsert<40, 12, GF_HASH_CT, GF_CT6_U>(ct, t, v, strict, added) < 0) return D_CT_CREATE_FAILED;
        uint32_t it[10];
        for (int k = 0; k < 8; k++) it[k] = t[k];
        it[8] = 0;
        it[9] = 58u | ((((t[9] >> 8) & 0xffu) | 2u) << 8);
        v[1] |= F_SEEN_NON_SYN;
        if (ht_upsert<40, 12, GF_HASH_CT, GF_CT6_U>(ct, it, v, strict, added) < 0) return D_CT_CREATE_FAILED;
        o.eg_flags |= GF_EG_F_CREATED;
    } else if ((ret == CT_REPLY || ret == CT_RELATED) && st.rev_nat) {   // lb6_rev_nat(flags 0)
        const gf_htab_desc rn = gload<gf_htab_desc>(&c->revnat6);
        uint32_t kw[1] = {st.rev_nat};
        const int64_t fr_ = ht_find<2>(rn, kw, key_hash<2>(kw));
        ab += 20;
        if (fr_ >= 0) {
            const uint8_t *nat = ht_val(rn, fr_);
            const uint32_t port = gload<uint16_t>(nat + 16);
            if (port) {
                if (nh == 6 || nh == 17) {
                    if (!skb_ok(l4_off, 2, len)) return -GF_EFAULT;
                    const uint32_t old = w.r16((uint32_t)l4_off);
                    if (port != old) {
                        if (l4_csum(w, len, l4_off + (int)co, old, port, 2u | fl) < 0) return D_CSUM_L4;
                        if (!skb_ok(l4_off, 2, len)) return D_WRITE_ERROR;
                        w.w16((uint32_t)l4_off, port);
                    }
                } else if (nh != 1 && nh != 58) return D_UNKNOWN_L4;
            }
            uint32_t sum = 0;
            for (int k = 0; k < 4; k++) {
                const uint32_t os = w.r32(22 + 4 * k), nw = gload<uint32_t>(nat + 4 * k);
                w.w32(22 + 4 * k, nw);
                sum = ck_add(ck_add(sum, ~os), nw);
            }
            if (l4_csum(w, len, l4_off + (int)co, 0, sum, GF_F_PSEUDO_HDR | fl) < 0) return D_CSUM_L4;
        }
        o.eg_flags |= GF_EG_F_REVNAT;
    }
    uint32_t nm[2] = {gload<uint32_t>(&c->node_mac[0]), gload<uint32_t>(&c->node_mac[1])};
    if (verdict > 0) {                                  // ipv6_redirect_to_host_port + ipv6_l3 -> HOST_IFINDEX
        if (E.X.tmark)
            trace_proxy(E.X.tmark, E.X.tcap, w.p, nullptr, 0, trace_cap_len(len, E.stride), i, GF_TR_PX_EGRESS);
        const int r3 = redirect_checks(len, l4_off, nh);
        if (r3 < 0) return r3;
        const uint32_t np = (uint32_t)verdict & 0xffffu;
        l4_csum(w, len, l4_off + (int)co, t[8] & 0xffffu, np, 2u | fl);   // l4_modify_port
        w.w16((uint32_t)(l4_off + 2), np);
        uint32_t sum = 0;
        for (int k = 0; k < 4; k++) { w.w32(38 + 4 * k, E.host6[k]); sum = ck_add(ck_add(sum, ~od[k]), E.host6[k]); }
        if (co) l4_csum(w, len, l4_off + (int)co, 0, sum, GF_F_PSEUDO_HDR | fl);
        pol_redirect(E.X, i, len, l4_off, nh, t, true, np, od, gload<uint32_t>(&c->seclabel), 1u);
        o.eg_flags |= GF_EG_F_PROXY;
        o.proxy_port = (uint16_t)verdict;
        const int r4 = eg_ipv6_l3(w, nm, E.host_mac);
        if (r4 != TC_OK) return r4;
        ifx = E.host_ifindex;
        return TC_REDIRECT;
    }
    uint32_t d6[4];
    for (int k = 0; k < 4; k++) d6[k] = w.r32(38 + 4 * k);
    if (E.lxc.slots) {                                  // lookup_ip6_endpoint
        uint32_t kw[5] = {d6[0], d6[1], d6[2], d6[3], 2u};
        const int64_t fe = ht_find<20>(E.lxc, kw, key_hash<20>(kw));
        ab += 20;
        if (fe >= 0) {
            const uint8_t *ep = ht_val(E.lxc, fe);
            ab += 8;
            if (gload<uint32_t>(ep + 8) & 1u) {         // ENDPOINT_F_HOST -> to_host
                if (!E.host_ifindex) return D_NO_LXC;
                const int r4 = eg_ipv6_l3(w, nm, E.host_mac);
                if (r4 != TC_OK) return r4;
                o.eg_flags |= GF_EG_F_TO_HOST;
                ifx = E.host_ifindex;
                return TC_REDIRECT;
            }
            uint32_t emac[2] = {gload<uint32_t>(ep + 16), gload<uint32_t>(ep + 20)};
            uint32_t rmac[2] = {gload<uint32_t>(ep + 24), gload<uint32_t>(ep + 28)};
            const int r4 = eg_ipv6_l3(w, rmac, emac);   // ipv6_local_delivery (l3.h:106-134)
            if (r4 != TC_OK) return r4;
            o.eg_flags |= GF_EG_F_LOCAL;
            uint32_t mapped = 0, ndport = 0;
            return delivery_tail(w, len, l4_off, nh, ep, ifx, lxc, mapped, ndport, ab);
        }
    }
    if (E.encap_ifindex && E.tunnel.slots) {            // encap_and_redirect, key daddr/96
        uint32_t kw[5] = {d6[0], d6[1], d6[2], 0u, 2u};
        const int64_t ft = ht_find<20>(E.tunnel, kw, key_hash<20>(kw));
        ab += 20;
        if (ft >= 0) {
            o.tunnel_ip = __builtin_bswap32(gload<uint32_t>(ht_val(E.tunnel, ft)));
            o.eg_flags |= GF_EG_F_ENCAP;
            ifx = E.encap_ifindex;
            return TC_REDIRECT;
        }
    }
    const int r4 = eg_ipv6_l3(w, nullptr, nm);         // pass_to_stack
    if (r4 != TC_OK) return r4;
    {                                                   // ipv6_store_flowlabel(SECLABEL_NB), ipv6.h:245-260
        const uint32_t old = w.r32(14) & __builtin_bswap32(0x0FF00000u);
        w.w32(14, __builtin_bswap32(0x60000000u) | __builtin_bswap32(gload<uint32_t>(&c->seclabel)) | old);
    }
    o.eg_flags |= GF_EG_F_TO_STACK;
    return TC_OK;
}

// One bucket per lane from the longest-first queue (the ingress schedule), in
// batch order.  Writes each packet's verdict, and for local deliveries the
// handle_policy record + flow-group key of the ingress pass (rec2 / key2).
// FAM 4 runs the schedule's family 0 (IPv4 buckets and every packet the front
// finished), FAM 6 family 1 (IPv6); the two touch disjoint state.
// PCT: per-endpoint CT maps (ConntrackLocal): each packet's net element change goes
// to its own program's map as the packet ends (ct_count unused).
template <int FAM, bool PCT = false>
__global__ __launch_bounds__(BLOCK, GF_EG_MINW) void k_eg_groups(EgDev E, uint32_t *sched, const uint2 *order, const uint32_t *perm,
                                                     const EgRec *erec, gf_egress_out *out, gf_rec *rec2, uint32_t *key2,
                                                     uint32_t *ct_count, unsigned long long *stats) {
    if (E.hz && *E.hz) return;                          // hazard: the batch reruns in ordered runs
    if (GF_EG_LEAN && !GF_SCHED_NFAM(sched)[FAM == 6 ? 1 : 0]) return;   // no bucket of this family (nothing to count)
    __shared__ uint32_t sl[272];
    __shared__ uint32_t sadd;
    // FAM 4: one LDS row per lane of the staged header bytes, sized by the snap
    // (eg_row_bytes: 64-B snaps take half the LDS of 128-B rows, so more blocks
    // fit a CU — the LDS, not the registers, bounded the waves); FAM 6: unused
    extern __shared__ uint4 lds[];
    __shared__ uint32_t lsum[3 * BLOCK];                // the lane's packets / wire bytes / algorithmic bytes
    Stats st{sl};
    uint32_t *ls = lsum + 3 * threadIdx.x;
    ls[0] = ls[1] = ls[2] = 0;
    auto fold = [&]() { st.add_n(268, ls[0]); st.add_n(269, ls[1]); st.add_n(270, ls[2]); ls[0] = ls[1] = ls[2] = 0; };
    if (threadIdx.x == 0) sadd = 0;
    if (stats) st.init(); else __syncthreads();
    const uint32_t K = eg_stage_bytes(E.stride);
    uint8_t *row = reinterpret_cast<uint8_t *>(lds) + (FAM == 6 ? 0 : threadIdx.x * eg_row_bytes(E.stride));
    constexpr int F = FAM == 6 ? 1 : 0;
    // the from-container pass schedules without records: every bucket is in class 0
    const uint32_t nb = GF_SCHED_LCNT(sched)[F * GF_NCLS], lane = threadIdx.x & 63u;
    uint32_t *queue = GF_SCHED_QUEUE(sched) + F * GF_NCLS;
    order += GF_SCHED_LSTART(sched)[F * GF_NCLS];
    const bool seq = *E.seq != 0;
    const bool rlog = FAM == 4 && E.conn && !seq && !*E.cflag;   // connection groups: related entries logged
    int added = 0;
    // the wave's grab: [base, base + 64 * left) of the list, one 64-bucket round at a
    // time (wave-uniform values); grab = buckets per lane of the next grab
    uint32_t grab = 1, base = 0, left = 0;
    for (;;) {
        if (!left) {
            uint32_t b0 = 0;
            if (lane == 0) b0 = atomicAdd(queue, 64u * grab);
            base = (uint32_t)__builtin_amdgcn_readfirstlane((int)b0);
            left = grab;
        }
        if (base >= nb) break;
        const uint32_t tq = base + lane;
        const bool first = left == grab;
        base += 64u; left--;
        if (tq >= nb) continue;
        const uint2 oc = order[tq];
        if (first && (uint32_t)__builtin_amdgcn_readfirstlane((int)oc.y) == 1u) grab = GF_GRAB_EG;   // single-packet tail
        for (uint32_t k = 0; k < oc.y; k++) {
            const uint32_t i = perm[oc.x + k];
            const EgRec r = erec[i];
            gf_rec rr;
            if (r.st) continue;                         // final in the front (its pass-2 record is written)
            gf_egress_out o{};
            o.stage = GF_STAGE_FROM_LXC;
            o.slave = r.slave; o.rev_nat = r.rev_nat; o.eg_flags = r.eflags;
            uint32_t ifx = 0, lxc = 0, ab = 24 + 34 + 32;
            uint8_t *g = E.snap + (size_t)i * E.stride;
            constexpr bool v6 = FAM == 6;
            int ret;
            PktHdr h2;                                  // the delivered header, re-parsed (local deliveries)
            if constexpr (v6) {                         // the frame in HBM
                Row w{g, E.stride < r.len ? E.stride : r.len};
                ret = eg_ct_part6<PCT>(E, r, i, w, o, ifx, lxc, &added, ab);
                if (ret == ND_TAILCALL) parse_row(w.p, w.cap, r.len, h2);
            } else {                                    // the LDS copy of the header bytes
                eg_copy(row, g, K);
                Row w{row, K < r.len ? K : r.len};
                ret = eg_ct_part<PCT>(E, r, i, w, o, ifx, lxc, &added, seq, rlog, ab);
                if (ret == ND_TAILCALL) parse_row(w.p, w.cap, r.len, h2);
                eg_copy(g, row, K);
            }
            o.ct_ret = o.eg_ct_ret;
            if constexpr (PCT) {
                if (added && !(E.strict & (FAM == 6 ? 2u : 1u))) {
                    const gf_lxc_dev *c = E.cfgs + (r.ep - 1);
                    atomicAdd(gload<uint32_t *>(FAM == 6 ? &c->ct6.count : &c->ct4.count), (uint32_t)added);
                }
                added = 0;
            }
            if (ret == ND_ICMP6_TE) {                   // ipv6_l3 -> icmp6_send_time_exceeded: the reply goes out
                ret = TC_REDIRECT; ifx = 0;
                o.eg_flags |= GF_EG_F_ICMP6_TE;
            }
            if (ret == ND_TAILCALL) {                   // handle_policy of the destination, next pass
                o.stage = GF_STAGE_POLICY; o.lxc_id = (uint16_t)lxc; o.ct_ret = 0;
                const gf_lxc_dev *c = E.cfgs + (r.ep - 1);
                uint32_t kk = pack_rec(i, h2.et, r.len, h2.sa, h2.da, h2.w0, h2.w3, h2.l4, h2.proto,
                                       gload<uint32_t>(&c->seclabel), ifx, E.slot_of[lxc & 0xffffu], 0, false, true,
                                       h2.s6, h2.d6, rr);
                if (E.conn) {                           // the delivery's connection (handle_policy's CT tuple)
                    E.key2P[i] = kk;
                    if (h2.et == 0x0800 && r.len >= 34) {
                        const bool tu = h2.proto == 6 || h2.proto == 17;
                        kk = gf_key_live(gf_conn_hash4(h2.sa, tu ? (h2.w0 & 0xffffu) : 0u, h2.da, tu ? (h2.w0 >> 16) : 0u,
                                                       h2.proto) & GF_KEY_HASH);
                    }
                }
                key2[i] = kk;
                rec2[i] = rr;
                if constexpr (v6) {
                    reinterpret_cast<uint4 *>(E.s6out)[2 * (size_t)i] = make_uint4(h2.s6[0], h2.s6[1], h2.s6[2], h2.s6[3]);
                    reinterpret_cast<uint4 *>(E.d6out)[2 * (size_t)i] = make_uint4(h2.d6[0], h2.d6[1], h2.d6[2], h2.d6[3]);
                    atomicAdd(E.ctlog_n + 1, 1u);       // the ingress pass needs its IPv6 kernel
                }
                if (stats) { ls[2] += ab; if (ls[2] >= 0xf0000000u) fold(); }
            } else {
                if (ret < 0 || ret == TC_SHOT) {
                    o.action = TC_SHOT; o.reason = (uint8_t)(-ret);
                    o.eg_flags &= (GF_EG_F_CREATED | GF_EG_F_DELETED | GF_EG_F_LB | GF_EG_F_LOOPBACK | GF_EG_F_PORTMAP |
                                   GF_EG_F_REVNAT | GF_EG_F_IPV6);
                    o.proxy_port = 0; o.tunnel_ip = 0;
                } else {
                    o.action = (uint8_t)ret;
                    o.ifindex_lo = (uint16_t)ifx;
                }
                if (stats) {
                    st.add(o.reason); st.add(256 + o.action);
                    ls[0] += 1; ls[1] += r.len; ls[2] += ab;
                    if (ls[1] >= 0xf0000000u || ls[2] >= 0xf0000000u) fold();
                }
            }
            out[i] = o;
        }
    }
    if (!(E.strict & (FAM == 6 ? 2u : 1u))) {       // strict maps counted each insert inline
        if (added) atomicAdd(&sadd, (uint32_t)added);
        __syncthreads();
        if (threadIdx.x == 0 && sadd && ct_count) atomicAdd(ct_count, sadd);
    }
    if (stats) { fold(); st.flush(stats); }
}

// The deferred service entries of a launch, in batch order (k_px_apply's rule):
// sorted by (key hash, packet index), an entry is applied only if no later
// entry of the batch has the same key.
// The logged ct_create entries (service entries of the from-container pass,
// related entries of connection groups), applied last-writer-wins per CT key:
// k_ctlog_max enters every entry into a scratch open-addressing set keyed by the
// logged tuple.  A slot is one u64: (1 + the highest order entered for its key)
// << 32 | that entry's index, 0 = empty; the key of a slot is its current entry's
// (every entry ever held by a slot has the slot's key).  A key's first entry
// claims a slot with one CAS, a later one raises it with atomicMax (the order in
// the high half), so a key logged once — most of them — costs one atomic.
// k_ctlog_apply walks the set's slots and upserts each key's winning entry.  Log
// entry: [0] order, [1..4] the 14-B key, [5..16] the 48-B value.
template <bool PCT = false>
__device__ __forceinline__ bool ctlog_same(const uint32_t *a, const uint32_t *b) {
    if (PCT && (a[18] != b[18] || a[19] != b[19])) return false;   // per-endpoint maps: the same map too
    return a[1] == b[1] && a[2] == b[2] && a[3] == b[3] && (a[4] & 0xffffu) == (b[4] & 0xffffu);
}
// The set is sized for the entries actually logged (<= 1/2 load; the count is on
// the device) inside an allocation made for the call's upper bound: both kernels
// derive the mask from the count themselves, and k_ctlog_apply leaves every slot it
// walks zero again — the set is all zero between applies (zeroed once when it is
// allocated), so no launch of its own clears it.
__device__ __forceinline__ uint32_t ctlog_mask(uint32_t n, uint32_t cap_mask) {
    const uint64_t want = GF_EG_LEAN ? 2ull * n : (uint64_t)cap_mask + 1;
    uint32_t t = 1023u;
    while ((uint64_t)t + 1 < want && t < cap_mask) t = t * 2 + 1;
    return t < cap_mask ? t : cap_mask;
}
template <bool PCT = false>
__global__ __launch_bounds__(BLOCK) void k_ctlog_max(const uint32_t *lg, const uint32_t *n_, unsigned long long *tab,
                                                     uint32_t cap_mask) {
    const uint32_t n = *n_, tmask = ctlog_mask(n, cap_mask);
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= n) return;
    const uint32_t *e = lg + (size_t)GF_CTLOG_WORDS * j;
    const unsigned long long want = ((unsigned long long)(e[0] + 1u) << 32) | j;
    uint32_t h0 = key_hash<14, GF_HASH_CT>(e + 1);
    if constexpr (PCT) h0 ^= gf_hash_words(e + 18, 2, 8);   // (the same tuple in two maps: two keys)
    for (uint32_t p = h0 & tmask;; p = (p + 1) & tmask) {
        // plain read first: a stale 0 only makes the CAS fail, a stale value only
        // costs the atomicMax it would have skipped
        unsigned long long cur = tab[p];
        if (cur == 0ull) {
            cur = atomicCAS(&tab[p], 0ull, want);
            if (cur == 0ull) return;                    // claimed for this key
        }
        if (ctlog_same<PCT>(lg + (size_t)GF_CTLOG_WORDS * (uint32_t)cur, e)) {
            if (cur < want) atomicMax(&tab[p], want);
            return;
        }
    }
}
// PCT: each entry into its program's own map (cfgs; ct, ct_count unused).
template <bool PCT = false>
__global__ __launch_bounds__(BLOCK) void k_ctlog_apply(const uint32_t *lg, const uint32_t *n_, unsigned long long *tab,
                                                       uint32_t cap_mask, gf_htab_desc ct, uint32_t *ct_count,
                                                       const gf_lxc_dev *cfgs = nullptr) {
    const uint32_t tmask = ctlog_mask(*n_, cap_mask);
    int added = 0;
    for (uint64_t p = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; p <= tmask; p += (uint64_t)gridDim.x * BLOCK) {
        const unsigned long long t = tab[p];
        if (t == 0ull) continue;                        // an empty slot
        tab[p] = 0ull;                                  // the set is clean for its next use
        const uint32_t *e = lg + (size_t)GF_CTLOG_WORDS * (uint32_t)t;   // the key's last entry in order
        if constexpr (PCT) {
            const gf_htab_desc d = gload<gf_htab_desc>(&cfgs[e[17] - 1].ct4);
            int a = 0;
            ht_upsert<14, 12, GF_HASH_CT, GF_CT4_U>(d, e + 1, e + 5, false, &a);
            if (a) atomicAdd(d.count, (uint32_t)a);
        } else {
            ht_upsert<14, 12, GF_HASH_CT, GF_CT4_U>(ct, e + 1, e + 5, false, &added);
        }
    }
    if (!ct_count || !__any(added != 0)) return;
    uint32_t tot = (uint32_t)added;                     // one count add per wave
    for (int d = 32; d >= 1; d >>= 1) tot += (uint32_t)__shfl_xor((int)tot, d);
    if ((threadIdx.x & 63u) == 0u) atomicAdd(ct_count, tot);
}

// The winners of a connection-group run's related-entry set (RelSet), written after
// the run: each claimed slot's one or two keys get the value their last writer's
// ct_create4 builds (conntrack.h:563-577) — order 2i: packet i's from-container create
// (the sender's SECLABEL and tx counters, bpf_lxc.c:534), 2i + 1: its delivery's
// handle_policy create (src_sec_id the source identity, rx counters, bpf_lxc.c:941) —
// and the slot is left zero for the next run.
__global__ __launch_bounds__(BLOCK) void k_rset_apply(RelSet R, const EgRec *erec, const gf_rec *rec,
                                                      const gf_lxc_dev *cfgs, gf_htab_desc ct, uint32_t *ct_count,
                                                      uint32_t now) {
    const uint32_t n = *R.list_n;
    int added = 0;
    for (uint32_t j = blockIdx.x * BLOCK + threadIdx.x; j < n; j += gridDim.x * BLOCK) {
        const uint32_t p = R.list[j];
        const uint4 sl = *reinterpret_cast<const uint4 *>(R.slot + 2ull * p);
        const unsigned long long k = p == R.mask + 1u ? 0ull : ((unsigned long long)sl.y << 32) | sl.x;
        for (uint32_t side = 0; side < 2; side++) {
            const uint32_t w = side ? sl.w : sl.z;
            if (!w) continue;
            const uint32_t o = w - 1u, i = o >> 1;
            const uint32_t it[4] = {(uint32_t)(k >> 32), (uint32_t)k, 0u, 1u | ((2u | side) << 8)};
            uint32_t v[12] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
            if (o & 1u) {                               // handle_policy (rev_nat 0 on ingress)
                const gf_rec r = rec[i];
                const uint32_t fl = r.proto == 6 ? 0u : F_SEEN_NON_SYN;
                v[0] = now + ((fl & F_SEEN_NON_SYN) ? 43200u : 300u);
                v[1] = fl | F_SEEN_NON_SYN;
                v[2] = 1u; v[3] = r.len; v[11] = r.src_identity;
            } else {                                    // from-container
                const EgRec r = erec[i];
                uint32_t efl = r.nh == 6 ? 0u : F_SEEN_NON_SYN;
                if (r.eflags & GF_EG_F_LOOPBACK) efl |= F_LB_LOOPBACK;
                v[0] = now + ((efl & F_SEEN_NON_SYN) ? 43200u : 300u);
                v[1] = efl | F_SEEN_NON_SYN | ((uint32_t)r.rev_nat << 16);
                v[6] = 1u; v[8] = r.len; v[11] = gload<uint32_t>(&cfgs[r.ep - 1].seclabel);
            }
            ht_upsert<14, 12, GF_HASH_CT, GF_CT4_U>(ct, it, v, false, &added);
        }
        *reinterpret_cast<uint4 *>(R.slot + 2ull * p) = make_uint4(0u, 0u, 0u, 0u);
    }
    if (!ct_count || !__any(added != 0)) return;
    uint32_t tot = (uint32_t)added;                     // one count add per wave
    for (int d = 32; d >= 1; d >>= 1) tot += (uint32_t)__shfl_xor((int)tot, d);
    if ((threadIdx.x & 63u) == 0u) atomicAdd(ct_count, tot);
}

// ================================================================ host: programs
namespace {

// ---- launch profiler: HIP events on the launch stream around each kernel ----
struct ProfEntry { std::string name; hipEvent_t a, b; };
struct Prof {
    bool on = false;
    std::mutex mu;                     // concurrent classify calls record launches
    std::vector<ProfEntry> pending;
    std::map<std::string, std::pair<uint32_t, double>> acc;
};
Prof &prof() { static Prof p; return p; }
struct ProfScope {
    ProfEntry e{};
    bool on;
    hipStream_t s;
    ProfScope(const char *n, hipStream_t s_) : on(prof().on), s(s_) {
        if (!on) return;
        e.name = n;
        // timing only: no system-scope fence (an L2 writeback) at each launch boundary
        (void)hipEventCreateWithFlags(&e.a, hipEventDisableSystemFence);
        (void)hipEventCreateWithFlags(&e.b, hipEventDisableSystemFence);
        (void)hipEventRecord(e.a, s);
    }
    ~ProfScope() {
        if (!on) return;
        (void)hipEventRecord(e.b, s);
        std::lock_guard<std::mutex> g(prof().mu);
        prof().pending.push_back(e);
    }
};
void prof_drain() {
    std::lock_guard<std::mutex> g(prof().mu);
    for (auto &e : prof().pending) {
        float ms = 0;
        if (hipEventSynchronize(e.b) == hipSuccess && hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess) {
            auto &a = prof().acc[e.name];
            a.first++;
            a.second += ms;
        }
        (void)hipEventDestroy(e.a);
        (void)hipEventDestroy(e.b);
    }
    prof().pending.clear();
}

struct Workspace {
    DevBuf rec, keys, skeys, perm, tcnt, off, tmp, sched, order;
    DevBuf sb, st0, st1;               // single-packet buckets in index order (GF_SINGLE_ORDER)
};
// GF_HOST_PROF (diagnosis): the host time of a classify call's phases, one line
// per call on stderr (where a call waits on the device, or spends its launches).
struct HostMarks {
    using clk = std::chrono::steady_clock;
    bool on;
    clk::time_point t0, last;
    char buf[768];
    int len = 0;
    HostMarks *prev;
    static HostMarks *&cur() { static thread_local HostMarks *c = nullptr; return c; }
    HostMarks() : on(getenv("GF_HOST_PROF") != nullptr), prev(cur()) {
        buf[0] = 0;
        if (on) { t0 = last = clk::now(); cur() = this; }
    }
    static double us(clk::duration d) { return std::chrono::duration<double, std::micro>(d).count(); }
    void mark(const char *what) {
        if (!on) return;
        const auto t = clk::now();
        if (len < (int)sizeof buf - 40) len += snprintf(buf + len, sizeof buf - len, " %s %.0f", what, us(t - last));
        last = t;
    }
    ~HostMarks() {
        if (!on) return;
        cur() = prev;
        fprintf(stderr, "[gf] host us:%s | total %.0f\n", buf, us(clk::now() - t0));
    }
};
void host_mark(const char *what) { if (HostMarks *m = HostMarks::cur()) m->mark(what); }
// ---- call contexts: the device workspaces of one classify call.  Each HIP
// stream has its own, so calls on different streams (over disjoint programs and
// maps, see CallOrder) run concurrently, host and device; calls on one stream
// take its context one at a time.  Workspace accessors keep one instance of
// their type per context (CallCtx::get).
}  // namespace
namespace gf {
struct CallCtx {
    std::mutex mu;
    hipEvent_t ev = nullptr;       // recorded at the end of every call in this context (made with the context)
    std::atomic<bool> have{false}; // ev has been recorded once (read by other contexts' CallOrder)
    int ws_slot = 0;      // gf_policy_ingress_classify_batches: schedule k+1 builds in one while k runs
    std::map<const void *, std::shared_ptr<void>> bag;
    template <class T> T &get(const void *tag) {
        auto &p = bag[tag];
        if (!p) p = std::make_shared<T>();
        return *static_cast<T *>(p.get());
    }
};
}  // namespace gf
namespace {
thread_local CallCtx *t_ctx = nullptr;
CallCtx &ctx_for(hipStream_t s) {
    static std::mutex mu;
    static std::map<hipStream_t, std::unique_ptr<CallCtx>> all;
    std::lock_guard<std::mutex> g(mu);
    auto &c = all[s];
    if (!c) {
        c = std::make_unique<CallCtx>();
        // the call-order event exists before any other thread can see the context
        // (device-scope release: the event orders device work between streams)
        if (hipEventCreateWithFlags(&c->ev, hipEventDisableTiming | hipEventReleaseToDevice) != hipSuccess) c->ev = nullptr;
    }
    return *c;
}
// The calling thread's context (map API paths outside a classify call: the
// null stream's).
CallCtx &cur_ctx() { return t_ctx ? *t_ctx : ctx_for(nullptr); }
struct CtxScope {
    CallCtx *prev, *c;
    std::unique_lock<std::mutex> l;
    explicit CtxScope(hipStream_t s) : prev(t_ctx), c(&ctx_for(s)), l(c->mu) { t_ctx = c; }
    ~CtxScope() { t_ctx = prev; }
};
Workspace &ws() {
    static const char tag = 0;
    CallCtx &c = cur_ctx();
    struct Two { Workspace w[2]; };
    return c.get<Two>(&tag).w[c.ws_slot];
}
gf_event_ring &event_ring() { static gf_event_ring r{}; return r; }
struct PipeWs {
    DevBuf s6, d6;             // IPv6 addresses of the rewritten frames (read by handle_policy)
};
PipeWs &pipe_ws() { static const char tag = 0; return cur_ctx().get<PipeWs>(&tag); }

int check_cols(const gf_pkt_cols *p) {
    if (!p) return -EFAULT;
    if (p->n == 0) return 0;
    if (!p->len || !p->ethertype || !p->saddr4 || !p->daddr4 || !p->proto || !p->l4_off || !p->l4w0 || !p->l4w3)
        return -EFAULT;
    return 1;
}

uint32_t grid_for(uint32_t n) {
    uint32_t g = (n + BLOCK - 1) / BLOCK;
    return g < 1 ? 1 : (g > 65535u * 8 ? 65535u * 8 : g);
}
// Grid of the one-packet-per-lane stream kernels (k_xdp, k_lb): capped at
// GF_STREAM_GRID blocks (grid-stride beyond) so the per-block counter flush
// stays a few thousand atomics per bin; 0 = one lane per packet.  Measured
// (config 3, k_lb, 16M packets): uncapped 0.86 ms, 2k 0.85, 4k 0.72, 16k 0.68.
#ifndef GF_STREAM_GRID
#define GF_STREAM_GRID 16384
#endif
// GPUFLOW_STREAM_GRID overrides the cap (the GPU tests force a few blocks so
// every block runs several tiles of the grid-stride loop).
uint32_t stream_grid_cap() {
    const char *e = getenv("GPUFLOW_STREAM_GRID");
    return e ? (uint32_t)strtoul(e, nullptr, 10) : (uint32_t)GF_STREAM_GRID;
}
uint32_t stream_grid(uint32_t n, uint32_t per_block = BLOCK) {
    const uint32_t g = n == 0 ? 1u : (n + per_block - 1) / per_block, cap = stream_grid_cap();
    const uint32_t lim = cap ? cap : 65535u * 8;      // grid-stride covers the rest
    return g > lim ? lim : g;
}

int push_map(const std::shared_ptr<Map> &m, hipStream_t s) { return m ? m->push(s) : 0; }
// The v4 prefixes as DIR-24-8 tables for XdpDev (GF_XDP_DIR24=1: the A/B against
// the trie walk), when they build.
void xdp_dir(const std::shared_ptr<Map> &l4, XdpDev &x, hipStream_t s) {
    const char *e = getenv("GF_XDP_DIR24");       // read per call: a test flips it in-process
    const bool on = e && atoi(e) != 0;
    x.d24 = nullptr; x.d8 = nullptr;
    if (on && l4 && l4->dir24(s, &x.d24, &x.d8)) { x.d24 = nullptr; x.d8 = nullptr; }
}
// The prefilter's compact address sets (Map::addr_set) for XdpDev, when they build.
void xdp_sets(const std::shared_ptr<Map> &h4, const std::shared_ptr<Map> &lxc, XdpDev &x, hipStream_t s) {
    static const bool no_sets = getenv("GF_XDP_NOSETS") != nullptr;     // diagnosis: the hash tables
    if (no_sets) return;
    if (h4 && h4->addr_set(8, 8192, s, &x.h4set, &x.h4bits, &x.h4zero)) x.h4set = nullptr;
    if (lxc && lxc->addr_set(20, 8192, s, &x.lxset, &x.lxbits, &x.lxzero)) x.lxset = nullptr;
}

// ---- device-side order of the calls that share an object.  Every map a call
// binds and the cilium_policy array it runs remember the call context (stream)
// of the last call that used them (OrderPt): a call first waits on the end event
// of each other context found there (one wait per context, on its latest call —
// a conservative bound), so a kernel still reading or writing a map replica (or a
// program table) finishes before this call pushes into it or runs over it; at its
// end the call records its context's event once and marks every object with its
// context (under the objects' locks).  The workspaces are per stream (CallCtx), so
// calls over disjoint objects on different streams do not wait on each other.
// With an event ring set, calls append to it in turn.
std::mutex &ring_mu() { static std::mutex m; return m; }
OrderPt &ring_ord() { static OrderPt o; return o; }
struct CallOrder {
    hipStream_t s;
    CallCtx *me;
    std::vector<OrderPt *> pts;
    std::unique_lock<std::mutex> ring;
    CallOrder(hipStream_t s_, std::vector<OrderPt *> p) : s(s_), me(&cur_ctx()), pts(std::move(p)) {
        if (event_ring().records) {
            ring = std::unique_lock<std::mutex>(ring_mu());
            pts.push_back(&ring_ord());
        }
        CallCtx *waited[8];
        int nw = 0;
        for (OrderPt *o : pts) {
            CallCtx *c = o->last;
            if (!c || c == me || !c->have.load(std::memory_order_acquire)) continue;
            bool seen = false;
            for (int k = 0; k < nw; k++) seen |= waited[k] == c;
            if (seen) continue;
            (void)hipStreamWaitEvent(s, c->ev, 0);
            if (nw < 8) waited[nw++] = c;
        }
    }
    CallOrder(hipStream_t s_, const MapLocks &L, PolicyArray *a = nullptr) : CallOrder(s_, order_pts(L, a)) {}
    static std::vector<OrderPt *> order_pts(const MapLocks &L, PolicyArray *a) {
        std::vector<OrderPt *> v;
        for (Map *m : L.held) v.push_back(&m->ord);
        if (a) v.push_back(&a->ord);
        return v;
    }
    ~CallOrder() {
        if (!me->ev || hipEventRecord(me->ev, s) != hipSuccess) return;
        me->have.store(true, std::memory_order_release);
        for (OrderPt *o : pts) o->last = me;
    }
};
void lock_lxc_maps(MapLocks &L, const std::shared_ptr<ProgLxc> &p) {
    for (auto m : {p->policy, p->ct4, p->ct6, p->cidr4, p->cidr6, p->revnat4, p->revnat6, p->lb4, p->ipcache,
                   p->cidr4e, p->lb6, p->cidr6e})
        L.add(m);
}
void lock_array_maps(MapLocks &L, const std::shared_ptr<PolicyArray> &a) {
    for (auto &kv : a->slots) lock_lxc_maps(L, kv.second);
    L.add(proxy_map(4)); L.add(proxy_map(6)); L.add(node_map(1)); L.add(node_map(2));
}
void lock_xdp_maps(MapLocks &L, const ProgXdp &x) { L.add(x.m4h); L.add(x.m4l); L.add(x.m6h); L.add(x.m6l); L.add(x.lxc); }


// blocks of BLOCK threads that fill the device at `per_cu` blocks per CU
uint32_t resident_blocks(uint32_t per_cu) {
    static const int cus = [] {                   // thread-safe one-time init (concurrent calls)
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            c = 256;
        return c;
    }();
    return (uint32_t)cus * per_cu;
}

}  // namespace

extern "C" {

int gf_parse_frames(const gf_frames *fr, gf_pkt_cols_out *o, void *stream) {
    if (!fr || !o) return -EFAULT;
    if (fr->n == 0) return 0;
    if (!fr->snap || !fr->len || !o->ethertype || !o->saddr4 || !o->daddr4 || !o->proto || !o->l4_off ||
        !o->l4w0 || !o->l4w3)
        return -EFAULT;
    if (fr->snap_stride < 14) return -EINVAL;
    ProfScope ps("k_parse", (hipStream_t)stream);
    hipLaunchKernelGGL(k_parse, dim3(grid_for(fr->n)), dim3(BLOCK), 0, (hipStream_t)stream, *fr, *o);
    return hip_ok(hipGetLastError(), "k_parse");
}

int gf_xdp_prog_load(const gf_xdp_cfg *cfg) {
    std::unique_lock<std::shared_mutex> g(prog_lock());
    if (!cfg) return -EFAULT;
    auto p = std::make_shared<ProgXdp>();
    p->cfg = *cfg;
    auto bind = [](int h, uint32_t ksz, bool lpm, std::shared_ptr<Map> &out) -> int {
        if (!h) return 0;
        auto m = get_map(h);
        if (!m) return -EBADF;
        if (m->ksz != ksz || m->is_lpm() != lpm) return -EINVAL;
        out = m;
        return 0;
    };
    int r;
    if ((r = bind(cfg->cidr4_hmap, 8, false, p->m4h))) return r;
    if ((r = bind(cfg->cidr4_lmap, 8, true, p->m4l))) return r;
    if ((r = bind(cfg->cidr6_hmap, 20, false, p->m6h))) return r;
    if ((r = bind(cfg->cidr6_lmap, 20, true, p->m6l))) return r;
    if ((r = bind(cfg->lxc_map, 20, false, p->lxc))) return r;
    if (!p->lxc) return -EINVAL;
    return new_handle(p);
}

int gf_xdp_classify(int prog, const gf_pkt_cols *pkts, uint8_t *verdict, void *stream) {
    std::shared_lock<std::shared_mutex> g(prog_lock());
    auto o = get_obj(prog);
    if (!o || o->kind != ObjKind::ProgXdp) return -EBADF;
    auto p = std::static_pointer_cast<ProgXdp>(o);
    int c = check_cols(pkts);
    if (c <= 0) return c;
    if (!verdict) return -EFAULT;
    hipStream_t s = (hipStream_t)stream;
    CtxScope cx(s);
    MapLocks L;
    lock_xdp_maps(L, *p);
    L.lock();
    CallOrder co(s, L);
    int r;
    if ((r = push_map(p->m4h, s)) || (r = push_map(p->m4l, s)) || (r = push_map(p->m6h, s)) ||
        (r = push_map(p->m6l, s)) || (r = push_map(p->lxc, s)))
        return r;
    XdpDev x{};
    xdp_sets(p->m4h, p->lxc, x, s);
    if (p->m4h) { x.h4 = p->m4h->hdesc(); x.has_h4 = 1; }
    if (p->m6h) { x.h6 = p->m6h->hdesc(); x.has_h6 = 1; }
    if (p->m4l) x.l4 = p->m4l->tdesc();
    if (p->m6l) x.l6 = p->m6l->tdesc();
    xdp_dir(p->m4l, x, s);
    x.lxc = p->lxc->hdesc();
    ProfScope ps("k_xdp", s);
    // The LDS variant when the LPM map has a 16-bit root (its summary is 16 KB);
    // the /32 hash and the endpoint keys join it while they fit.
    static const bool no_lds = getenv("GF_XDP_NOLDS") != nullptr;     // diagnosis: the HBM-only kernel
    if (!no_lds && x.l4.rsum && x.has_h4 && x.l4.addr_bytes == 4) {
        static const uint32_t cap = getenv("GF_XDP_LDS_KB") ? 1024u * (uint32_t)atoi(getenv("GF_XDP_LDS_KB")) : 48u * 1024u;
        XdpLds L{};
        // the /32 hash and the endpoint keys as compact address sets (4 B a slot), else
        // their slot arrays when those fit the budget
        L.h4set = x.h4set; L.h4bits = x.h4bits; L.h4zero = x.h4zero;
        L.lxset = x.lxset; L.lxbits = x.lxbits; L.lxzero = x.lxzero;
        const uint64_t hb = (uint64_t)(x.h4.mask + 1) * x.h4.slot_size, lb = (uint64_t)(x.lxc.mask + 1) * x.lxc.slot_size;
        if (!L.h4set && x.h4.slots && x.h4.ksz == 8 && hb % 16 == 0 && GF_TRIE_RSUM_BYTES + hb <= std::min(cap, 96u * 1024u))
            L.h4_bytes = (uint32_t)hb;
        const uint32_t h4b = L.h4set ? 4u << L.h4bits : L.h4_bytes;
        if (!L.lxset && x.lxc.slots && x.lxc.ksz == 20 && lb % 16 == 0 && GF_TRIE_RSUM_BYTES + h4b + lb <= cap)
            L.lxc_bytes = (uint32_t)lb;
        const uint32_t lds = GF_TRIE_RSUM_BYTES + h4b + (L.lxset ? 4u << L.lxbits : L.lxc_bytes);
        // the address sets count against the budget too: larger maps take k_xdp,
        // which reads the same sets and the root summary through L2
        static std::atomic<uint32_t> lds_set{0};
        bool fits = lds <= std::max(cap, GF_TRIE_RSUM_BYTES);
        if (fits && lds > lds_set.load()) {
            fits = hipFuncSetAttribute((const void *)k_xdp_lds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) ==
                   hipSuccess;
            if (fits) {
                uint32_t cur = lds_set.load();
                while (lds > cur && !lds_set.compare_exchange_weak(cur, lds)) {}
            } else {
                (void)hipGetLastError();
            }
        }
        if (fits) {
        const uint32_t per_cu = lds <= 78u * 1024u ? 2u : 1u;
        static const uint32_t grid_env = getenv("GF_XDP_GRID") ? (uint32_t)atoi(getenv("GF_XDP_GRID")) : 0u;   // diagnosis
        const uint32_t grid = grid_env ? grid_env
                                       : std::max<uint32_t>(1u, std::min<uint32_t>(resident_blocks(per_cu), (pkts->n + 1023) / 1024));
        hipLaunchKernelGGL(k_xdp_lds, dim3(grid), dim3(1024), lds, s, *pkts, x, L, verdict,
                           (unsigned long long *)stats_sink());
        return hip_ok(hipGetLastError(), "k_xdp_lds");
        }
    }
    hipLaunchKernelGGL(k_xdp, dim3(stream_grid(pkts->n)), dim3(BLOCK), 0, s, *pkts, x, verdict,
                       (unsigned long long *)stats_sink());
    return hip_ok(hipGetLastError(), "k_xdp");
}

int gf_lb_prog_load(const gf_lb_cfg *cfg) {
    std::unique_lock<std::shared_mutex> g(prog_lock());
    if (!cfg) return -EFAULT;
    auto p = std::make_shared<ProgLb>();
    p->cfg = *cfg;
    if (cfg->lb4_services) {
        p->lb4 = get_map(cfg->lb4_services);
        if (!p->lb4) return -EBADF;
        if (p->lb4->ksz != 8 || p->lb4->vsz != 12 || p->lb4->is_lpm()) return -EINVAL;
    }
    if (cfg->lb6_services) {
        p->lb6 = get_map(cfg->lb6_services);
        if (!p->lb6) return -EBADF;
        if (p->lb6->ksz != 20 || p->lb6->vsz != 24 || p->lb6->is_lpm()) return -EINVAL;
    }
    return new_handle(p);
}

int gf_lb_classify(int prog, const gf_pkt_cols *pkts, gf_lb_out *out, uint8_t *nd6, void *stream) {
    std::shared_lock<std::shared_mutex> g(prog_lock());
    auto o = get_obj(prog);
    if (!o || o->kind != ObjKind::ProgLb) return -EBADF;
    auto p = std::static_pointer_cast<ProgLb>(o);
    int c = check_cols(pkts);
    if (c <= 0) return c;
    if (!out) return -EFAULT;
    hipStream_t s = (hipStream_t)stream;
    CtxScope cx(s);
    MapLocks ML;
    ML.add(p->lb4); ML.add(p->lb6);
    ML.lock();
    CallOrder co(s, ML);
    int r;
    if ((r = push_map(p->lb4, s)) || (r = push_map(p->lb6, s))) return r;
    LbDev L{};
    if (p->lb4) L.s4 = p->lb4->hdesc();
    if (p->lb6) L.s6 = p->lb6->hdesc();
    L.flags = p->cfg.flags;
    ProfScope ps("k_lb", s);
    hipLaunchKernelGGL(k_lb, dim3(stream_grid(pkts->n)), dim3(BLOCK), 0, s, *pkts, L, out, nd6,
                       (unsigned long long *)stats_sink());
    return hip_ok(hipGetLastError(), "k_lb");
}

int gf_lxc_prog_load(const gf_lxc_cfg *cfg) {
    std::unique_lock<std::shared_mutex> g(prog_lock());
    if (!cfg) return -EFAULT;
    if (cfg->n_l4_ingress > GF_MAX_L4_INGRESS || cfg->n_l4_egress > GF_MAX_L4_INGRESS ||
        cfg->n_portmap > GF_MAX_PORTMAP)
        return -E2BIG;
    auto p = std::make_shared<ProgLxc>();
    p->cfg = *cfg;
    struct B { int h; uint32_t k, v; bool lpm; std::shared_ptr<Map> *out; };
    B binds[] = {
        {cfg->policy_map, 8, 24, false, &p->policy}, {cfg->ct_map4, 14, 48, false, &p->ct4},
        {cfg->ct_map6, 40, 48, false, &p->ct6},      {cfg->cidr4_ingress_map, 8, 0, true, &p->cidr4},
        {cfg->cidr6_ingress_map, 20, 0, true, &p->cidr6}, {cfg->revnat4_map, 2, 6, false, &p->revnat4},
        {cfg->revnat6_map, 2, 18, false, &p->revnat6},
        {cfg->lb4_services, 8, 12, false, &p->lb4},      {cfg->ipcache_map, 20, 8, false, &p->ipcache},
        {cfg->cidr4_egress_map, 8, 0, true, &p->cidr4e}, {cfg->lb6_services, 20, 24, false, &p->lb6},
        {cfg->cidr6_egress_map, 20, 0, true, &p->cidr6e},
    };
    for (auto &b : binds) {
        if (!b.h) continue;
        auto m = get_map(b.h);
        if (!m) return -EBADF;
        if (m->ksz != b.k || m->is_lpm() != b.lpm || (!b.lpm && m->vsz != b.v)) return -EINVAL;
        *b.out = m;
    }
    MapLocks L;
    lock_lxc_maps(L, p);
    L.lock();
    if (p->ct4) { p->ct4->set_hash_mode(GF_HASH_CT); p->ct4->set_value_codec(GF_VCODEC_CT); p->ct4->make_fixed_capacity(gf_ct_slot_factor(p->ct4->ksz)); }
    if (p->ct6) { p->ct6->set_hash_mode(GF_HASH_CT); p->ct6->set_value_codec(GF_VCODEC_CT); p->ct6->make_fixed_capacity(gf_ct_slot_factor(p->ct6->ksz)); }
    if (p->policy) { p->policy->set_hash_mode(GF_HASH_POLICY); p->policy->set_value_codec(GF_VCODEC_POL); }
    return new_handle(p);
}

int gf_set_event_ring(const gf_event_ring *ring) {
    std::unique_lock<std::shared_mutex> g(prog_lock());
    if (!ring) { event_ring() = gf_event_ring{}; return 0; }
    if (!ring->records || !ring->count) return -EFAULT;
    event_ring() = *ring;
    return 0;
}

int gf_prof_enable(int on) {
    std::unique_lock<std::shared_mutex> g(prog_lock());
    prof_drain();
    prof().acc.clear();
    prof().on = on != 0;
    return 0;
}

int gf_prof_read(gf_prof_rec *out, int max) {
    std::unique_lock<std::shared_mutex> g(prog_lock());
    if (max < 0 || (max > 0 && !out)) return -EFAULT;
    prof_drain();
    int k = 0;
    for (auto &kv : prof().acc) {
        if (k >= max) break;
        memset(&out[k], 0, sizeof out[k]);
        strncpy(out[k].name, kv.first.c_str(), sizeof(out[k].name) - 1);
        out[k].count = kv.second.first;
        out[k].total_ms = kv.second.second;
        k++;
    }
    return k;
}

int gf_policy_array_create(void) {
    std::unique_lock<std::shared_mutex> g(prog_lock());
    return new_handle(std::make_shared<PolicyArray>());
}

int gf_policy_array_update(int array, uint32_t lxc_id, int prog) {
    std::unique_lock<std::shared_mutex> g(prog_lock());
    auto o = get_obj(array);
    if (!o || o->kind != ObjKind::PolicyArray) return -EBADF;
    if (lxc_id > 0xffff) return -E2BIG;
    auto a = std::static_pointer_cast<PolicyArray>(o);
    if (!prog) { a->slots.erase(lxc_id); a->dirty = true; return 0; }
    auto po = get_obj(prog);
    if (!po || po->kind != ObjKind::ProgLxc) return -EINVAL;
    a->slots[lxc_id] = std::static_pointer_cast<ProgLxc>(po);
    a->dirty = true;
    return 0;
}

}  // extern "C"

// handle_policy over a batch (caller holds prog_lock and the maps' locks, and checked the columns).
// skip (DEVICE, may be null): packets a pipeline ended before the tail call.
// Trace notifications of a call: per-packet marks and captures (GF_TR_*),
// allocated and the marks cleared by the caller before its first kernel.
struct TraceWs { DevBuf mark, px, in; };
static TraceWs &trace_ws() { static const char tag = 0; return cur_ctx().get<TraceWs>(&tag); }
struct PassArgs {                  // what the pipeline / egress callers pass to their handle_policy pass
    uint32_t kind;                 // 1 pipeline, 2 egress
    uint32_t *rlog, *rlog_n;       // egress connection groups: the related-entry log (null: written inline)
    const uint32_t *rlog_off;      // device word: the run fell back to pair groups (the log is not used)
    RelSet rs;                     // GF_EG_RSET: the related entries' set (rlog then only marks it in use)
    bool on;                       // this call traces (a ring is set and a program / the netdev traces)
    uint32_t nd_trace, nd_ifindex; // pipeline: GF_NETDEV_F_TRACE_NOTIFY, skb->ingress_ifindex
    const uint8_t *orig;           // egress: the frames as sent
    const uint16_t *lxc_id;        // egress: the senders
};
static bool array_traces(const std::shared_ptr<PolicyArray> &a) {
    if (!a) return false;
    for (auto &kv : a->slots)
        if (kv.second->cfg.flags & GF_LXC_F_TRACE_NOTIFY) return true;
    return false;
}
static int trace_prepare(uint32_t n, bool with_in, hipStream_t s) {
    TraceWs &t = trace_ws();
    auto grow = [](DevBuf &d, size_t want) -> int { return d.bytes >= want ? 0 : d.ensure(want); };
    int r;
    if ((r = grow(t.mark, (size_t)n + 16)) || (r = grow(t.px, (size_t)n * GF_TRACE_PAYLOAD_LEN)) ||
        (with_in && (r = grow(t.in, (size_t)n * GF_TRACE_PAYLOAD_LEN))))
        return r;
    return hip_ok(hipMemsetAsync(t.mark.p, 0, n, s), "trace marks");
}

// Drop (and trace) notifications of one classify call (no-op without an event ring).
static int emit_drop_events(EvSrc E, hipStream_t s) {
    gf_event_ring R = event_ring();
    if (!R.records || !R.count || !R.capacity || E.n == 0) return 0;
    struct EvWs { DevBuf blk, boff, tmp; };
    static const char tag = 0;
    EvWs &ew = cur_ctx().get<EvWs>(&tag);
    DevBuf &blk = ew.blk, &boff = ew.boff, &tmp = ew.tmp;
    const uint32_t nb = (E.n + BLOCK - 1) / BLOCK;
    auto grow = [](DevBuf &d, size_t want) -> int { return d.bytes >= want ? 0 : d.ensure(want); };
    int r;
    if ((r = grow(blk, (size_t)nb * 4)) || (r = grow(boff, (size_t)nb * 4))) return r;
    size_t tb = 0;
    (void)rocprim::exclusive_scan(nullptr, tb, (uint32_t *)blk.p, (uint32_t *)boff.p, 0u, nb, rocprim::plus<uint32_t>(), s);
    if ((r = grow(tmp, tb + 256))) return r;
    ProfScope ps("k_drop_events", s);
    hipLaunchKernelGGL(k_ev_count, dim3(nb), dim3(BLOCK), 0, s, E, (uint32_t *)blk.p);
    tb = tmp.bytes;
    if (hip_ok(rocprim::exclusive_scan(tmp.p, tb, (uint32_t *)blk.p, (uint32_t *)boff.p, 0u, nb,
                                       rocprim::plus<uint32_t>(), s), "event scan"))
        return -EIO;
    hipLaunchKernelGGL(k_ev_write, dim3(nb), dim3(BLOCK), 0, s, E, (const uint32_t *)boff.p, R);
    hipLaunchKernelGGL(k_ev_commit, dim3(1), dim3(1), 0, s, (const uint32_t *)boff.p, (const uint32_t *)blk.p, nb, R);
    return hip_ok(hipGetLastError(), "k_drop_events");
}

// Per-batch workspace of the flow-group schedule (records, keys, sort, runs, order).
static int ws_grow(uint32_t n) {
    Workspace &w = ws();
    auto grow = [](DevBuf &b, size_t want) -> int { return b.bytes >= want ? 0 : b.ensure(want); };
    int r;
    if ((r = grow(w.rec, (size_t)n * sizeof(gf_rec))) || (r = grow(w.keys, (size_t)n * 4)) ||
        (r = grow(w.skeys, (size_t)n * 4)) || (r = grow(w.perm, (size_t)n * 4 + 16)) ||
        (r = grow(w.off, (size_t)n * 4)) || (r = grow(w.order, (size_t)n * 8)) ||
        (r = grow(w.sched, GF_SCHED_WORDS * 4)))
        return r;
    return 0;
}

// The flow-group schedule of ws().keys[0..n): stable radix sort of (32-bit group
// hash, index), the start of every run of equal hashes (one bucket per run: a
// select of the positions whose key differs from the one before), then the
// longest-first bucket order per family, built on the device (no host round
// trip): ws().perm / order / sched.
#ifndef GF_SORT_RADIX
#define GF_SORT_RADIX 8                // digit bits of the onesweep passes (rocPRIM's gfx950 default)
#endif
#ifndef GF_SORT_IPT
#define GF_SORT_IPT 16
#endif
#if GF_SORT_RADIX == 8 && GF_SORT_IPT == 16
using GfSortCfg = rocprim::default_config;
#else
using GfSortCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, GF_SORT_IPT>, rocprim::kernel_config<1024, GF_SORT_IPT>,
                                        GF_SORT_RADIX, rocprim::block_radix_rank_algorithm::match>>;
#endif
// Run starts of the sorted keys in three passes over GF_RUN_ITEMS-key tiles:
// count the starts per tile, scan the tile counts (one block), write each
// tile's starts at its offset in position order (wave ballots + LDS scan).
__device__ __forceinline__ bool run_start(const uint32_t *k, uint32_t j) { return j == 0 || k[j] != k[j - 1]; }
// zero: n words to clear on the way (the single-bucket words of an egress schedule,
// k_single_mark: one launch fewer than a fill of their own), or null
__global__ __launch_bounds__(BLOCK) void k_run_count(uint32_t n, const uint32_t *skeys, uint32_t *tcnt,
                                                     uint32_t *zero = nullptr) {
    __shared__ uint32_t wc[BLOCK / 64];
    const uint32_t b0 = blockIdx.x * GF_RUN_ITEMS, lane = threadIdx.x & 63u;
    uint32_t c = 0;
    for (uint32_t k = 0; k < GF_RUN_ITEMS / BLOCK; k++) {
        const uint32_t j = b0 + k * BLOCK + threadIdx.x;
        c += (uint32_t)__popcll(__ballot(j < n && run_start(skeys, j)));
        if (zero && j < n) zero[j] = 0u;
    }
    if (lane == 0) wc[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < BLOCK / 64; w++) t += wc[w];
        tcnt[blockIdx.x] = t;
    }
}
// zero / nzero: words to clear on the way (the schedule's bucket histogram: one
// launch fewer than a fill of its own)
__global__ __launch_bounds__(1024) void k_run_scan(uint32_t nt, uint32_t *tcnt, uint32_t *nruns, uint32_t *zero = nullptr,
                                                   uint32_t nzero = 0) {
    __shared__ uint32_t part[1024];
    __shared__ uint32_t carry;
    for (uint32_t k = threadIdx.x; k < nzero; k += 1024) zero[k] = 0;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t c0 = 0; c0 < nt; c0 += 1024) {         // exclusive scan in place, 1024 tiles at a time
        const uint32_t t = c0 + threadIdx.x;
        const uint32_t v = t < nt ? tcnt[t] : 0u;
        part[threadIdx.x] = v;
        __syncthreads();
        for (uint32_t o = 1; o < 1024; o <<= 1) {
            const uint32_t x = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
            __syncthreads();
            part[threadIdx.x] += x;
            __syncthreads();
        }
        if (t < nt) tcnt[t] = carry + part[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += part[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *nruns = carry;
}
__global__ __launch_bounds__(BLOCK) void k_run_write(uint32_t n, const uint32_t *skeys, const uint32_t *toff,
                                                     uint32_t *off) {
    __shared__ uint32_t wc[BLOCK / 64];
    const uint32_t b0 = blockIdx.x * GF_RUN_ITEMS, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t base = toff[blockIdx.x];
    for (uint32_t k = 0; k < GF_RUN_ITEMS / BLOCK; k++) {
        const uint32_t j = b0 + k * BLOCK + threadIdx.x;
        const bool f = j < n && run_start(skeys, j);
        const uint64_t m = __ballot(f);
        if (lane == 0) wc[wv] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t before = 0, all = 0;
        for (uint32_t w = 0; w < BLOCK / 64; w++) { before += w < wv ? wc[w] : 0u; all += wc[w]; }
        if (f) off[base + before + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = j;
        base += all;
        __syncthreads();
    }
}
// rec: the packets' handle_policy records (the bucket's endpoint class), or null
// (every bucket in class 0: the egress from-container pass).
// single: single-packet buckets in packet-index order (the egress passes).
static int schedule_groups(uint32_t n, hipStream_t s, const gf_rec *rec = nullptr, bool single = false) {
    Workspace &w = ws();
    auto grow = [](DevBuf &b, size_t want) -> int { return b.bytes >= want ? 0 : b.ensure(want); };
    int r;
    uint32_t *d_sched = (uint32_t *)w.sched.p, *d_nruns = GF_SCHED_NRUNS(d_sched);
    size_t sort_bytes = 0;
    (void)rocprim::radix_sort_pairs<GfSortCfg>(nullptr, sort_bytes, (uint32_t *)w.keys.p, (uint32_t *)w.skeys.p,
                                               rocprim::counting_iterator<uint32_t>(0u), (uint32_t *)w.perm.p, n, 0,
                                               GF_KEY_BITS, s);
    const uint32_t nt = (n + GF_RUN_ITEMS - 1) / GF_RUN_ITEMS;
    if ((r = grow(w.tmp, sort_bytes + 256)) || (r = grow(w.tcnt, (size_t)nt * 4 + 16))) return r;
    single = single && GF_SINGLE_ORDER && GF_NCLS == 1;
    if (single && ((r = grow(w.sb, (size_t)n * 4)) || (r = grow(w.st0, (size_t)nt * 4 + 16)) ||
                   (r = grow(w.st1, (size_t)nt * 4 + 16))))
        return r;
    size_t tb = w.tmp.bytes;
    {
        ProfScope ps("rocprim_radix_sort", s);
        if (hip_ok(rocprim::radix_sort_pairs<GfSortCfg>(w.tmp.p, tb, (uint32_t *)w.keys.p, (uint32_t *)w.skeys.p,
                                                        rocprim::counting_iterator<uint32_t>(0u), (uint32_t *)w.perm.p,
                                                        n, 0, GF_KEY_BITS, s), "radix_sort_pairs"))
            return -EIO;
    }
    {
        ProfScope ps("bucket_runs", s);
        if (nt) hipLaunchKernelGGL(k_run_count, dim3(nt), dim3(BLOCK), 0, s, n, (const uint32_t *)w.skeys.p,
                                   (uint32_t *)w.tcnt.p, single ? (uint32_t *)w.sb.p : nullptr);
        hipLaunchKernelGGL(k_run_scan, dim3(1), dim3(1024), 0, s, nt, (uint32_t *)w.tcnt.p, d_nruns,
                           GF_SCHED_HIST(d_sched), GF_SCHED_HBYTES / 4u);   // (+ the bucket histogram cleared)
        if (nt) hipLaunchKernelGGL(k_run_write, dim3(nt), dim3(BLOCK), 0, s, n, (const uint32_t *)w.skeys.p,
                                   (const uint32_t *)w.tcnt.p, (uint32_t *)w.off.p);
        if ((r = hip_ok(hipGetLastError(), "run starts"))) return r;
    }
    {
        ProfScope ps("k_bucket_sched", s);
        static const bool lds_ok = [] {                  // the bins are > 64 KB of dynamic LDS
            return hipFuncSetAttribute((const void *)k_bucket_hist, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)GF_SCHED_HBYTES) == hipSuccess &&
                   hipFuncSetAttribute((const void *)k_bucket_order, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)GF_SCHED_HBYTES) == hipSuccess;
        }();
        if (!lds_ok) return hip_ok(hipErrorInvalidValue, "k_bucket_sched LDS");
        uint32_t g = (n + GF_SCHED_ITEMS - 1) / GF_SCHED_ITEMS;
        const gf_rec *lrec = GF_NCLS > 1 ? rec : nullptr;
        hipLaunchKernelGGL(k_bucket_hist, dim3(g), dim3(BLOCK), GF_SCHED_HBYTES, s, n, (const uint32_t *)w.off.p,
                           (const uint32_t *)w.skeys.p, lrec, (const uint32_t *)w.perm.p, d_sched);
        hipLaunchKernelGGL(k_bucket_base, dim3(1), dim3(GF_LCAP), 0, s, d_sched);
        hipLaunchKernelGGL(k_bucket_order, dim3(g), dim3(BLOCK), GF_SCHED_HBYTES, s, n, (const uint32_t *)w.off.p,
                           (const uint32_t *)w.skeys.p, lrec, (const uint32_t *)w.perm.p, d_sched, (uint2 *)w.order.p,
                           single ? 1u : 0u);
        if (single) {                                   // (the words were cleared by k_run_count)
            hipLaunchKernelGGL(k_single_mark, dim3(std::min<uint32_t>((n + BLOCK - 1) / BLOCK, 8192u)), dim3(BLOCK), 0, s, n,
                               (const uint32_t *)w.off.p, (const uint32_t *)w.skeys.p, (const uint32_t *)w.perm.p,
                               (const uint32_t *)d_sched, (uint32_t *)w.sb.p);
            hipLaunchKernelGGL(k_single_count, dim3(nt), dim3(BLOCK), 0, s, n, (const uint32_t *)w.sb.p,
                               (uint32_t *)w.st0.p, (uint32_t *)w.st1.p);
            hipLaunchKernelGGL(k_run_scan, dim3(1), dim3(1024), 0, s, nt, (uint32_t *)w.st0.p, (uint32_t *)w.st0.p + nt,
                               nullptr, 0u);
            hipLaunchKernelGGL(k_run_scan, dim3(1), dim3(1024), 0, s, nt, (uint32_t *)w.st1.p, (uint32_t *)w.st1.p + nt,
                               nullptr, 0u);
            hipLaunchKernelGGL(k_single_write, dim3(nt), dim3(BLOCK), 0, s, n, (const uint32_t *)w.sb.p,
                               (const uint32_t *)w.st0.p, (const uint32_t *)w.st1.p, (const uint32_t *)d_sched,
                               (uint2 *)w.order.p);
        }
    }
    return hip_ok(hipGetLastError(), "k_bucket_sched");
}

// cilium_proxy{4,6} update log of one launch (pol_redirect) and its in-order
// apply after the launch (see k_px_apply).
struct PxWs {
    DevBuf plog, plog_n, pkey, pkey2, pval, pperm, ptmp;
    bool live = false;         // a log was begun in this call (its count is valid)
};
static PxWs &px_ws() { static const char tag = 0; return cur_ctx().get<PxWs>(&tag); }
// keep: continue the log the from-container pass of the same egress call wrote
// (each packet logs at most one update: an egress redirect is never delivered).
// Without proxy maps the updates are no-ops that succeed (the reference's maps
// always exist), but a redirect still gets the MAC stores that follow it in
// ipv{4,6}_policy when the call writes frames: the log is kept for those.
static int px_log_begin(uint32_t n, hipStream_t s, IngCtx &X, bool keep = false) {
    auto px4 = proxy_map(4), px6 = proxy_map(6);
    X.plog = nullptr; X.plog_n = nullptr;
    PxWs &w = px_ws();
    if (!px4 && !px6 && !X.snap && !(keep && w.live)) { w.live = keep && w.live; return 0; }
    int r;
    auto grow = [](DevBuf &b, size_t want) -> int { return b.bytes >= want ? 0 : b.ensure(want); };
    if ((r = grow(w.plog, (size_t)n * 64)) || (r = grow(w.plog_n, 4))) return r;
    if ((!keep || !w.live) && hip_ok(hipMemsetAsync(w.plog_n.p, 0, 4, s), "plog_n")) return -EIO;
    w.live = true;
    for (auto &m : {px4, px6})
        if (m && (r = push_map(m, s))) return r;
    X.plog = (uint32_t *)w.plog.p; X.plog_n = (uint32_t *)w.plog_n.p;
    return 0;
}
// recs: the launch's verdict records (24-B pipeline/egress layout when wide, else gf_ingress_out)
static int px_log_apply(const IngCtx &X, hipStream_t s, uint8_t *wsnap, const uint32_t *len, uint32_t stride,
                        uint8_t *recs, bool wide, uint32_t n) {
    if (!X.plog) return 0;
    px_ws().live = false;
    auto px4 = proxy_map(4), px6 = proxy_map(6);
    const gf_node_cfg &node = node_cfg();
    PxWs &w = px_ws();
    int r;
    if (!px4 && !px6) {                               // the MAC stores alone: the count stays on the device
        if (!wsnap) return 0;
        PxDev P{};
        P.snap = wsnap; P.len = len; P.snap_stride = stride;
        memcpy(P.host_mac, node.host_mac, 6); memcpy(P.node_mac, node.node_mac, 6);
        ProfScope ps("k_proxy_apply", s);
        hipLaunchKernelGGL(k_px_macs, dim3(grid_for(n)), dim3(BLOCK), 0, s, (const uint32_t *)X.plog,
                           (const uint32_t *)X.plog_n, P);
        return hip_ok(hipGetLastError(), "k_px_macs");
    }
    uint32_t cnt = 0;
    if (hip_ok(hipMemcpyAsync(&cnt, X.plog_n, 4, hipMemcpyDeviceToHost, s), "plog count") ||
        hip_ok(hipStreamSynchronize(s), "plog sync"))
        return -EIO;
    if (!cnt) return 0;
    PxDev P{};
    bool seq = false;
    for (auto &m : {px4, px6}) {
        if (!m) continue;
        if (m->host_valid) m->dev_count_hi = m->ht.count;
        if (m->dev_count_hi + cnt > m->max_entries) seq = true;
    }
    if (px4) P.d4 = px4->hdesc();
    if (px6) P.d6 = px6->hdesc();
    P.snap = wsnap; P.len = len; P.snap_stride = stride;
    memcpy(P.host_mac, node.host_mac, 6); memcpy(P.node_mac, node.node_mac, 6);
    auto grow = [](DevBuf &b, size_t want) -> int { return b.bytes >= want ? 0 : b.ensure(want); };
    if ((r = grow(w.pkey, (size_t)cnt * 8)) || (r = grow(w.pkey2, (size_t)cnt * 8)) || (r = grow(w.pval, (size_t)cnt * 4)) ||
        (r = grow(w.pperm, (size_t)cnt * 4)))
        return r;
    size_t tb = 0;
    (void)rocprim::radix_sort_pairs(nullptr, tb, (unsigned long long *)w.pkey.p, (unsigned long long *)w.pkey2.p,
                                    (uint32_t *)w.pval.p, (uint32_t *)w.pperm.p, cnt, 0, 64, s);
    if ((r = grow(w.ptmp, tb + 256))) return r;
    ProfScope ps("k_proxy_apply", s);
    const uint32_t g = (cnt + BLOCK - 1) / BLOCK;
    hipLaunchKernelGGL(k_px_keys, dim3(g), dim3(BLOCK), 0, s, (const uint32_t *)w.plog.p, cnt, seq,
                       (unsigned long long *)w.pkey.p, (uint32_t *)w.pval.p);
    tb = w.ptmp.bytes;
    if (hip_ok(rocprim::radix_sort_pairs(w.ptmp.p, tb, (unsigned long long *)w.pkey.p, (unsigned long long *)w.pkey2.p,
                                         (uint32_t *)w.pval.p, (uint32_t *)w.pperm.p, cnt, 0, 64, s), "proxy sort"))
        return -EIO;
    if (seq)
        hipLaunchKernelGGL(k_px_apply_seq, dim3(1), dim3(1), 0, s, (const uint32_t *)w.plog.p, cnt,
                           (const uint32_t *)w.pperm.p, P, recs, wide ? 24u : 8u, wide ? 1u : 0u,
                           (unsigned long long *)stats_sink());
    else
        hipLaunchKernelGGL(k_px_apply, dim3(g), dim3(BLOCK), 0, s, (const uint32_t *)w.plog.p, cnt,
                           (const unsigned long long *)w.pkey2.p, (const uint32_t *)w.pperm.p, P);
    if ((r = hip_ok(hipGetLastError(), "k_proxy_apply"))) return r;
    for (auto &m : {px4, px6}) if (m) { m->device_modified(); m->dev_count_hi += cnt; }
    return 0;
}

// A CT map's launch descriptor: an LRU conntrack map's inserts are limited by its
// slot array (dev_insert_limit), not by max_entries (the eviction pass after the
// call brings the count back).
static gf_htab_desc ct_dev_desc(Map &m) {
    gf_htab_desc d = m.hdesc();
    if (m.type == GF_MAP_TYPE_LRU_HASH) d.max_entries = (uint32_t)std::min<uint64_t>(dev_insert_limit(m), 0xffffffffu);
    return d;
}

// The device program table of a cilium_policy array (every bound map pushed to
// HBM first); uploaded only when it changed (programs, bindings, or a map's
// device storage moved).  progs: the distinct programs, slot k+1 = progs[k].
static int prog_table(const std::shared_ptr<PolicyArray> &a, hipStream_t s,
                      std::vector<std::shared_ptr<ProgLxc>> &progs) {
    int r;
    std::map<ProgLxc *, uint32_t> index;
    std::vector<uint16_t> slot_of(65536, 0);
    for (auto &kv : a->slots) {
        auto &p = kv.second;
        auto it = index.find(p.get());
        if (it == index.end()) {
            if (progs.size() >= 65535) return -E2BIG;
            it = index.emplace(p.get(), (uint32_t)progs.size()).first;
            progs.push_back(p);
        }
        slot_of[kv.first] = (uint16_t)(it->second + 1);
    }
    std::vector<gf_lxc_dev> cfgs(progs.size());
    for (size_t k = 0; k < progs.size(); k++) {
        auto &p = progs[k];
        for (auto m : {p->policy, p->ct4, p->ct6, p->cidr4, p->cidr6, p->revnat4, p->revnat6, p->lb4, p->ipcache,
                       p->cidr4e, p->lb6, p->cidr6e})
            if ((r = push_map(m, s))) return r;
        gf_lxc_dev &d = cfgs[k];
        memset(&d, 0, sizeof d);
        d.flags = p->cfg.flags; d.lxc_id = p->cfg.lxc_id; d.seclabel = p->cfg.seclabel;
        d.n_l4 = p->cfg.n_l4_ingress;
        for (uint32_t j = 0; j < d.n_l4; j++) {
            d.l4[j].port = p->cfg.l4_ingress[j].port; d.l4[j].proxy = p->cfg.l4_ingress[j].proxy;
            d.l4[j].nexthdr = p->cfg.l4_ingress[j].nexthdr;
        }
        if (p->policy) d.policy = p->policy->hdesc();
        if (p->ct4) { d.ct4 = ct_dev_desc(*p->ct4); d.flags |= GF_LXC_DEV_HAS_CT4; }
        if (p->ct6) { d.ct6 = ct_dev_desc(*p->ct6); d.flags |= GF_LXC_DEV_HAS_CT6; }
        if (p->cidr4) d.cidr4 = p->cidr4->tdesc();
        if (p->cidr6) d.cidr6 = p->cidr6->tdesc();
        if (p->revnat4) d.revnat4 = p->revnat4->hdesc();
        if (p->revnat6) d.revnat6 = p->revnat6->hdesc();
        memcpy(d.lxc_mac, p->cfg.lxc_mac, 6);
        memcpy(d.node_mac, p->cfg.node_mac, 6);
        d.lxc_ipv4 = p->cfg.lxc_ipv4;
        d.n_portmap = p->cfg.n_portmap;
        for (uint32_t j = 0; j < d.n_portmap; j++)
            d.portmap[j] = p->cfg.portmap[j].from | ((uint32_t)p->cfg.portmap[j].to << 16);
        d.n_l4e = p->cfg.n_l4_egress;
        for (uint32_t j = 0; j < d.n_l4e; j++) {
            d.l4e[j].port = p->cfg.l4_egress[j].port; d.l4e[j].proxy = p->cfg.l4_egress[j].proxy;
            d.l4e[j].nexthdr = p->cfg.l4_egress[j].nexthdr;
        }
        if (p->lb4) d.lb4 = p->lb4->hdesc();
        if (p->ipcache) d.ipcache = p->ipcache->hdesc();
        if (p->cidr4e) d.cidr4e = p->cidr4e->tdesc();
        memcpy(d.lxc_ip6, p->cfg.lxc_ip6, 16);
        if (p->lb6) d.lb6 = p->lb6->hdesc();
        if (p->cidr6e) d.cidr6e = p->cidr6e->tdesc();
    }
    size_t cb = cfgs.size() * sizeof(gf_lxc_dev);
    bool changed = a->dirty || a->h_cfgs.size() != cb || a->h_slot_of.size() != slot_of.size() ||
                   (cb && memcmp(a->h_cfgs.data(), cfgs.data(), cb)) ||
                   memcmp(a->h_slot_of.data(), slot_of.data(), slot_of.size() * 2);
    if (changed) {
        if (getenv("GF_SYNC_DEBUG")) fprintf(stderr, "[gf] program table upload (dirty %d)\n", (int)a->dirty);
        if ((r = a->d_slot_of_lxc.ensure(65536 * 2))) return r;
        if ((r = a->d_cfgs.ensure(std::max<size_t>(1, cb)))) return r;
        a->h_cfgs.assign((const uint8_t *)cfgs.data(), (const uint8_t *)cfgs.data() + cb);
        a->h_slot_of = slot_of;
        if (hip_ok(hipMemcpyAsync(a->d_slot_of_lxc.p, a->h_slot_of.data(), 65536 * 2, hipMemcpyHostToDevice, s), "slots"))
            return -EIO;
        if (cb && hip_ok(hipMemcpyAsync(a->d_cfgs.p, a->h_cfgs.data(), cb, hipMemcpyHostToDevice, s), "cfgs"))
            return -EIO;
        if (hip_ok(hipStreamSynchronize(s), "cfg sync")) return -EIO;
        a->dirty = false;
    }
    return 0;
}

// The host's bound of a CT map's device count (ct_limits, lru_evict) tightened
// from the counts the recent eviction chains wrote to pinned host memory: the
// newest one whose event has fired (a query, never a wait), plus what the calls
// enqueued since may have added.  A ring of events, so a host that runs several
// calls ahead of the device still finds a fired one.
// wait: block on the oldest pending event instead (the device only has to reach
// that earlier call, not drain the queue) — ct_limits' alternative to a readback.
static void ct_count_refresh(Map &m, bool wait = false) {
    if (m.h_stamp) {                                    // the multi-map pass's stamp (no wait: read as it is)
        const unsigned long long v = *reinterpret_cast<volatile unsigned long long *>(m.h_stamp);
        const uint32_t seq = (uint32_t)(v >> 32), j = seq % Map::GF_STRING;
        if (seq > m.st_floor && m.st_seq[j] == seq)
            m.dev_count_hi = std::min<uint64_t>(m.dev_count_hi, (uint64_t)(uint32_t)v + (m.cnt_add - m.st_add[j]));
    }
    if (!m.ev_pending || !m.h_evcount) return;
    if (wait)
        for (uint32_t k = Map::GF_EVRING; k >= 1; k--) {
            const uint32_t j = (m.ev_head + Map::GF_EVRING - k) % Map::GF_EVRING;
            if (m.ev_pending & (1u << j)) { (void)hipEventSynchronize(m.ev_count[j]); break; }
        }
    for (uint32_t k = 1; k <= Map::GF_EVRING; k++) {
        const uint32_t j = (m.ev_head + Map::GF_EVRING - k) % Map::GF_EVRING;
        if (!(m.ev_pending & (1u << j))) continue;
        if (hipEventQuery(m.ev_count[j]) != hipSuccess) continue;
        m.dev_count_hi = std::min<uint64_t>(m.dev_count_hi, (uint64_t)m.h_evcount[j] + (m.cnt_add - m.ev_add[j]));
        // this slot and every older one are used up
        for (uint32_t q = k; q <= Map::GF_EVRING; q++) m.ev_pending &= ~(1u << ((m.ev_head + Map::GF_EVRING - q) % Map::GF_EVRING));
        return;
    }
}
// Element accounting mode of the CT maps for a batch of n packets inserting at
// most per_pkt entries each (see ingress_run); fills the launch descriptors.
static int ct_limits(const std::shared_ptr<Map> &ct4m, const std::shared_ptr<Map> &ct6m, uint32_t n, uint32_t per_pkt,
                     hipStream_t s, uint32_t &strict, gf_htab_desc &cfg_ct4, gf_htab_desc &cfg_ct6) {
    strict = 0;
    if (ct4m) cfg_ct4 = ct_dev_desc(*ct4m);
    if (ct6m) cfg_ct6 = ct_dev_desc(*ct6m);
    for (auto &m : {ct4m, ct6m}) {
        if (!m) continue;
        // LRU: never fails in the kernel (it evicts); here no eviction inside a classify
        // call, the entries stay until the eviction pass after it (lru_evict), bounded by
        // the slot array (7/8 load = 3.5 x max_entries)
        const uint64_t limit = dev_insert_limit(*m);
        if (m->host_valid) { m->dev_count_hi = m->ht.count; m->ev_pending = 0; m->st_floor = m->lru_seq; }
        ct_count_refresh(*m);
        // near the limit: the count of an eviction chain a few calls back first (no
        // queue drain), then, if that is not enough, a readback
        if (m->dev_count_hi + (uint64_t)per_pkt * n > limit && (uint64_t)per_pkt * n <= limit && !m->host_valid)
            ct_count_refresh(*m, true);
        // (no readback when the batch alone could exceed the limit: strict either way)
        if (m->dev_count_hi + (uint64_t)per_pkt * n > limit && (uint64_t)per_pkt * n <= limit && !m->host_valid) {
            if (getenv("GF_SYNC_DEBUG"))
                fprintf(stderr, "[gf] CT count readback (bound %llu + %u x %u > %llu)\n", (unsigned long long)m->dev_count_hi,
                        per_pkt, n, (unsigned long long)limit);
            uint32_t dc = 0;
            if (hip_ok(hipStreamSynchronize(s), "ct count sync") ||
                hip_ok(hipMemcpy(&dc, m->d_count.p, 4, hipMemcpyDeviceToHost), "read ct count"))
                return -EIO;
            m->dev_count_hi = dc;
            m->ev_pending = 0;
            m->st_floor = m->lru_seq;
        }
        if (m->dev_count_hi + (uint64_t)per_pkt * n > limit) strict |= m == ct4m ? 1u : 2u;
        m->dev_count_hi += (uint64_t)per_pkt * n;
        m->cnt_add += (uint64_t)per_pkt * n;
    }
    return 0;
}

// The CT maps the programs of a call bind, per family, each once.  pct: some family
// has more than one (endpoints with the ConntrackLocal option, cilium_ct4_<id>,
// pkg/endpoint/bpf.go:268-276) — the per-endpoint kernels (ing_ct<FAM, true>).
struct CtMaps {
    std::vector<std::shared_ptr<Map>> m4, m6;
    bool pct = false;
    std::shared_ptr<Map> one(int fam) const {
        const auto &v = fam == 6 ? m6 : m4;
        return v.empty() ? nullptr : v[0];
    }
};
static int ct_maps_of(const std::vector<std::shared_ptr<ProgLxc>> &progs, CtMaps &cm) {
    std::set<const Map *> s4, s6;
    for (auto &p : progs) {
        if (p->ct4 && s4.insert(p->ct4.get()).second) cm.m4.push_back(p->ct4);
        if (p->ct6 && s6.insert(p->ct6.get()).second) cm.m6.push_back(p->ct6);
    }
    for (auto *m : s4)
        if (s6.count(m)) return -EINVAL;                // one map bound as both families' CT map
    cm.pct = cm.m4.size() > 1 || cm.m6.size() > 1;
    return 0;
}
// Per-endpoint maps: each map's host bound moves as if the whole batch could insert
// into it; a family whose maps could any of them fill counts every insert exactly
// (strict: the count and insert limit the program table's descriptor carries,
// ct_dev_desc), else each lane adds its net inserts to its program's map
// (lane_flush_added).
static int ct_limits_pct(const CtMaps &cm, uint32_t n, uint32_t per_pkt, hipStream_t s, uint32_t &strict) {
    gf_htab_desc d4{}, d6{};
    int r;
    strict = 0;
    for (auto &m : cm.m4) {
        uint32_t st = 0;
        if ((r = ct_limits(m, nullptr, n, per_pkt, s, st, d4, d6))) return r;
        strict |= st;
    }
    for (auto &m : cm.m6) {
        uint32_t st = 0;
        if ((r = ct_limits(nullptr, m, n, per_pkt, s, st, d4, d6))) return r;
        strict |= st;
    }
    return 0;
}

// ---- CT sweeps on the device: per-map LRU state (histogram, cutoffs, log) and
// the cluster-start bits of the GC sweep.
static int ct_sweep_bufs(Map &m, LruDev *&L, uint32_t *&bits) {
    if (!m.d_lru.p) {
        if (m.d_lru.ensure(sizeof(LruDev))) return -ENOMEM;
        if (hip_ok(hipMemset(m.d_lru.p, 0, sizeof(LruDev)), "lru init")) return -EIO;
    }
    const size_t nw = (m.ht.nslots + 31) / 32;
    if (m.d_gcbits.bytes < nw * 4 && m.d_gcbits.ensure(nw * 4)) return -ENOMEM;
    L = (LruDev *)m.d_lru.p;
    bits = (uint32_t *)m.d_gcbits.p;
    return 0;
}
static void ct_sweep_launch(Map &m, LruDev *L, uint32_t *bits, hipStream_t s) {
    const gf_htab_desc d = m.hdesc();
    const uint32_t lt_off = m.ht.codec == GF_VCODEC_CT ? 0u : 32u;
    const uint64_t nw = (d.mask + 1 + 31) / 32;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((nw + BLOCK - 1) / BLOCK, 65535u * 8);
    hipLaunchKernelGGL(k_gc_starts, dim3(grid), dim3(BLOCK), 0, s, d, bits, (const GcCut *)&L->cut);
    hipLaunchKernelGGL(k_gc_clusters, dim3(grid), dim3(BLOCK), 0, s, d, m.ht.mode, lt_off, (const GcCut *)&L->cut,
                       (const uint32_t *)bits, L->res);
}
// The LRU stand-in after a classify call (k_lru_*: see the kernels): fully on the
// device, a chain of launches that exit at once unless the map's count exceeds its
// high-water mark; not launched at all while the host's bound of the count is at or
// below it.
// One map's part of an eviction pass: its state, this call's count word, and the
// descriptor the kernels read (kind 0: nothing to launch for it).
struct LruPrep { Map *m = nullptr; int kind = 0; uint32_t slot = 0; LruMap lm{}; };
// track: the chain writes the count to the map's pinned ring behind an event, for the
// host's bound (the multi-map pass does not: one event record per map per call costs
// more host time than the bound saves there).
static int lru_prepare(const std::shared_ptr<Map> &m, LruPrep &P, bool track = true) {
    P = LruPrep{};
    if (!m || m->type != GF_MAP_TYPE_LRU_HASH || !m->d_slots.p) return 0;
    m->lru_seq++;
    ct_count_refresh(*m);
    if (m->dev_count_hi <= lru_high_water(m->max_entries)) return 0;   // cannot have crossed HW
    if (!m->d_lru.p) {
        if (m->d_lru.ensure(sizeof(LruDev))) return -ENOMEM;
        if (hip_ok(hipMemset(m->d_lru.p, 0, sizeof(LruDev)), "lru init")) return -EIO;
    }
    const gf_htab_desc d = m->hdesc();
    const int kind = d.slot_size == 32 && d.ksz == 14 && d.vin == 16 && d.voff == 16 ? 1
                   : d.slot_size == 64 && d.ksz == 40 && d.vin == 16 && d.voff == 48 ? 2 : 0;
    if (!kind) return -EIO;                              // the CT codec's layouts only
    if (!m->h_evcount) {
        // every event first, the count words last: a failure leaves nothing half made
        hipEvent_t ev[Map::GF_EVRING] = {};
        bool ok = true;
        for (auto &e : ev)
            if (ok && hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "lru count event")) ok = false;
        void *p = nullptr;
        if (ok && hip_ok(hipHostMalloc(&p, 4 * Map::GF_EVRING, hipHostMallocMapped | hipHostMallocCoherent),
                         "lru count words"))
            ok = false;
        if (!ok) {
            for (auto &e : ev)
                if (e) (void)hipEventDestroy(e);
            return -ENOMEM;
        }
        uint32_t *dp = nullptr;
        if (hip_ok(hipHostGetDevicePointer((void **)&dp, p, 0), "lru count words")) {
            for (auto &e : ev) (void)hipEventDestroy(e);
            (void)hipHostFree(p);
            return -EIO;
        }
        for (uint32_t k = 0; k < Map::GF_EVRING; k++) m->ev_count[k] = ev[k];
        m->h_evcount = (uint32_t *)p;
        m->d_evcount = dp;
    }
    if (!track && !m->h_stamp) {
        void *p = nullptr;
        unsigned long long *dp = nullptr;
        if (hip_ok(hipHostMalloc(&p, 8, hipHostMallocMapped | hipHostMallocCoherent), "lru stamp")) return -ENOMEM;
        *(unsigned long long *)p = 0ull;
        if (hip_ok(hipHostGetDevicePointer((void **)&dp, p, 0), "lru stamp")) { (void)hipHostFree(p); return -EIO; }
        m->h_stamp = (unsigned long long *)p;
        m->d_stamp = dp;
    }
    P.m = m.get(); P.kind = kind; P.slot = m->ev_head;
    LruMap &M = P.lm;
    M.hcount = track ? m->d_evcount + P.slot : nullptr;
    M.stamp = track ? nullptr : m->d_stamp;
    if (!track) {                                       // the stamp's reference point: cnt_add at this call
        const uint32_t j = m->lru_seq % Map::GF_STRING;
        m->st_seq[j] = m->lru_seq;
        m->st_add[j] = m->cnt_add;
    }
    const uint64_t ns = d.mask + 1, spl = 128 / d.slot_size;
    M.d = d; M.L = (LruDev *)m->d_lru.p; M.nl = ns / spl; M.sl = lru_sample_lines(M.nl);
    M.mode = m->ht.mode; M.max_entries = m->max_entries; M.seq = m->lru_seq;
    return 0;
}
// After the chain: the count word's event, for the host's bound (ct_count_refresh).
static int lru_post(const LruPrep &P, uint32_t now, hipStream_t s) {
    Map *m = P.m;
    if (hip_ok(hipEventRecord(m->ev_count[P.slot], s), "lru count event")) return -EIO;
    m->ev_pending |= 1u << P.slot;
    m->ev_add[P.slot] = m->cnt_add;
    m->ev_head = (P.slot + 1) % Map::GF_EVRING;
    static const bool stats = getenv("GF_LRU_STATS") != nullptr;   // diagnostics: syncs the stream
    if (stats) {
        LruDev h;
        LruDev *L = P.lm.L;
        if (!hip_ok(hipMemcpyAsync(&h, L, offsetof(LruDev, log), hipMemcpyDeviceToHost, s), "lru stats") &&
            !hip_ok(hipStreamSynchronize(s), "lru stats") && h.nlog) {
            uint32_t n = h.nlog;
            LruLog g{};
            if (!hip_ok(hipMemcpy(&g, &L->log[std::min(n, GF_LRU_LOGCAP) - 1], sizeof g, hipMemcpyDeviceToHost),
                        "lru stats log") && g.seq == m->lru_seq)
                fprintf(stderr, "[lru] seq %u now %u: K %u es %llu lines %llu of %llu (hand %llu) evicted %llu "
                        "(rounds %llu / %llu / %llu), cleared %llu\n", g.seq, now, g.age_cut, h.es, g.lines,
                        (unsigned long long)P.lm.nl, g.hand, g.evicted, h.kills[0], h.kills[1], h.kills[2], h.cleared);
        }
    }
    return 0;
}
// The LRU stand-in after a classify call (k_lru_*: see the kernels): fully on the
// device, a chain of launches that exit at once unless the map's count exceeds its
// high-water mark; not launched at all while the host's bound of the count is at or
// below it.
static int lru_evict(const std::shared_ptr<Map> &m, uint32_t now, hipStream_t s) {
    LruPrep P;
    int r;
    if ((r = lru_prepare(m, P)) || !P.kind) return r;
    const LruMap &M = P.lm;
    const gf_htab_desc &d = M.d;
    LruDev *L = M.L;
    const int kind = P.kind;
    const uint64_t spl = 128 / d.slot_size, nl = M.nl, sl = M.sl;
    const uint32_t gs = (uint32_t)std::min<uint64_t>((sl * spl + GF_LRU_HB - 1) / GF_LRU_HB, resident_blocks(2));
    const uint32_t gh = resident_blocks(8);
    const uint32_t *cnt = (const uint32_t *)d.count;
    const uint32_t mx = M.max_entries, mode = M.mode;
    {
        ProfScope ps("k_lru_evict", s);
        // the window's sample and plan, then (large tables only) the whole-table
        // pair, which runs only when the window held no entry
        for (uint32_t wide = 0; wide < (sl < nl ? 2u : 1u); wide++) {
            const dim3 g(wide ? gh : gs);
            if (kind == 1)
                hipLaunchKernelGGL(k_lru_sample<1>, g, dim3(GF_LRU_HB), 0, s, d, mode, now, L, sl, mx, wide);
            else
                hipLaunchKernelGGL(k_lru_sample<2>, g, dim3(GF_LRU_HB), 0, s, d, mode, now, L, sl, mx, wide);
            hipLaunchKernelGGL(k_lru_plan, dim3(1), dim3(1024), 0, s, cnt, mx, L, sl, nl, wide);
        }
        for (uint32_t round = 0; round < GF_LRU_ROUNDS; round++) {
            // round 1 is rare and short (what round 0's estimate left): a smaller grid, the same chunks
            const dim3 g(round == 1 ? gh / 8 : gh);
            if (kind == 1) {
                hipLaunchKernelGGL((k_lru_hand<1, 0>), g, dim3(GF_LRU_HT), 0, s, d, mode, now, L, nl, sl, mx, round);
                hipLaunchKernelGGL((k_lru_hand<1, 1>), g, dim3(GF_LRU_HT), 0, s, d, mode, now, L, nl, sl, mx, round);
            } else {
                hipLaunchKernelGGL((k_lru_hand<2, 0>), g, dim3(GF_LRU_HT), 0, s, d, mode, now, L, nl, sl, mx, round);
                hipLaunchKernelGGL((k_lru_hand<2, 1>), g, dim3(GF_LRU_HT), 0, s, d, mode, now, L, nl, sl, mx, round);
            }
        }
        hipLaunchKernelGGL(k_lru_end, dim3(1), dim3(1), 0, s, d.count, M.seq, now, L, mx, nl, M.hcount);
    }
    if ((r = lru_post(P, now, s))) return r;
    return hip_ok(hipGetLastError(), "k_lru_evict");
}
// The pass over several maps (per-endpoint CT maps): the maps that may be above their
// high-water marks, GF_LRU_MULTI of one slot kind per chain of launches (a single one
// takes the one-map chain).  Each map's rounds, cutoffs and log are its own, exactly
// as with its own chain.
static int lru_evict_maps(const std::vector<std::shared_ptr<Map>> &ms, uint32_t now, hipStream_t s) {
    if (ms.empty()) return 0;
    if (ms.size() == 1) return lru_evict(ms[0], now, s);
    std::vector<LruPrep> ps;
    int r;
    for (auto &m : ms) {
        LruPrep P;
        if ((r = lru_prepare(m, P, false))) return r;
        if (P.kind) ps.push_back(P);
    }
    if (ps.empty()) return 0;
    const uint32_t gh = resident_blocks(8);
    ProfScope prof("k_lru_evict", s);
    for (int kind = 1; kind <= 2; kind++) {
        std::vector<const LruPrep *> ks;
        for (auto &P : ps)
            if (P.kind == kind) ks.push_back(&P);
        for (size_t b = 0; b < ks.size(); b += GF_LRU_MULTI) {
            LruBatch B{};
            B.n = (uint32_t)std::min<size_t>(GF_LRU_MULTI, ks.size() - b);
            uint64_t gs = 1;
            bool big = false;
            for (uint32_t k = 0; k < B.n; k++) {
                B.m[k] = ks[b + k]->lm;
                const uint64_t spl = 128 / B.m[k].d.slot_size;
                gs = std::max<uint64_t>(gs, (B.m[k].sl * spl + GF_LRU_HB - 1) / GF_LRU_HB);
                big |= B.m[k].sl < B.m[k].nl;
            }
            const dim3 g1((uint32_t)std::min<uint64_t>(gs, resident_blocks(2)));
            for (uint32_t wide = 0; wide < (big ? 2u : 1u); wide++) {
                // (the whole-table pass runs only for a map whose window held no entry: a
                // smaller grid, which costs little on the many calls where it has no work)
                const dim3 g(wide ? std::max<uint32_t>(gh / 8, 1) : g1.x);
                if (kind == 1) hipLaunchKernelGGL(k_lru_sample_multi<1>, g, dim3(GF_LRU_HB), 0, s, B, now, wide);
                else hipLaunchKernelGGL(k_lru_sample_multi<2>, g, dim3(GF_LRU_HB), 0, s, B, now, wide);
                hipLaunchKernelGGL(k_lru_plan_multi, dim3(B.n), dim3(1024), 0, s, B, wide);
            }
            for (uint32_t round = 0; round < GF_LRU_ROUNDS; round++) {
                // rounds 1 and 2 run only for what round 0's estimate left: smaller grids
                const dim3 g(round ? std::max<uint32_t>(gh / 8, 1) : gh);
                if (kind == 1) {
                    hipLaunchKernelGGL((k_lru_hand_multi<1, 0>), g, dim3(GF_LRU_HT), 0, s, B, now, round);
                    hipLaunchKernelGGL((k_lru_hand_multi<1, 1>), g, dim3(GF_LRU_HT), 0, s, B, now, round);
                } else {
                    hipLaunchKernelGGL((k_lru_hand_multi<2, 0>), g, dim3(GF_LRU_HT), 0, s, B, now, round);
                    hipLaunchKernelGGL((k_lru_hand_multi<2, 1>), g, dim3(GF_LRU_HT), 0, s, B, now, round);
                }
            }
            hipLaunchKernelGGL(k_lru_end_multi, dim3(1), dim3(64), 0, s, B, now);
            if ((r = hip_ok(hipGetLastError(), "k_lru_*_multi"))) return r;
        }
    }
    return 0;
}

// pack (may be empty): fills the records and bucket keys itself (the fused
// pipeline front) instead of k_ing_pack; pout: pipeline records to complete.
using PackFn = std::function<int(const uint16_t *slot_of, gf_rec *rec, uint32_t *keys)>;
static int ingress_run(const std::shared_ptr<PolicyArray> &a, const gf_pkt_cols *pkts, uint32_t now_sec,
                       gf_ingress_out *out, hipStream_t s, const PackFn &pack = PackFn(), uint8_t *pout = nullptr,
                       const uint32_t *ev_len = nullptr, const uint8_t *ev_snap = nullptr, uint32_t ev_stride = 0,
                       uint8_t *wsnap = nullptr, bool lru = true, bool px_keep = false, bool prepared = false,
                       const PassArgs *ta = nullptr) {
    int r;
    // trace notifications: the plain ingress call decides here, the pipeline and
    // egress callers (whose earlier kernels mark packets) pass their decision
    const bool tracing = ta ? ta->on : (event_ring().records && array_traces(a));
    if (tracing && !ta && (r = trace_prepare(pkts->n, false, s))) return r;
    // 1. sync tables, build the device program table
    std::vector<std::shared_ptr<ProgLxc>> progs;
    host_mark("ing");
    if ((r = prog_table(a, s, progs))) return r;
    host_mark("prog");
    // CT maps: the global layout (every program binds cilium_ct4_global / ct6_global)
    // or per-endpoint maps (ConntrackLocal, ct_maps_of: the PCT kernels)
    CtMaps cm;
    if ((r = ct_maps_of(progs, cm))) return r;
    std::shared_ptr<Map> ct4m = cm.pct ? nullptr : cm.one(4), ct6m = cm.pct ? nullptr : cm.one(6);
    // Strict (exact, atomic per insert) element accounting only when this batch could
    // reach the limit.  HASH maps are limited by max_entries (E2BIG).  LRU maps never
    // fail in the kernel (they evict); here they keep entries past max_entries until
    // GC and are bounded only by the slot array (7/8 load), see DESIGN.md.
    // The decision uses a host-side upper bound of the device element count (each
    // packet inserts at most 2 entries), read back from the device only when the
    // bound gets near the limit — steady-state batches never wait on the GPU here.
    // Per-endpoint maps: the same per family, over every map of it (ct_limits_pct).
    uint32_t strict = 0;
    gf_htab_desc cfg_ct4{}, cfg_ct6{};
    if ((r = ct_limits(ct4m, ct6m, pkts->n, 2, s, strict, cfg_ct4, cfg_ct6))) return r;
    if (cm.pct && (r = ct_limits_pct(cm, pkts->n, 2, s, strict))) return r;
    host_mark("ctlim");
    // 2. group by flow group (records and keys first), 3. longest-first bucket order
    uint32_t n = pkts->n;
    Workspace &w = ws();
    if (prepared) {
        // pack + schedule already built in ws() (ingress_prepare)
    } else if ((r = ws_grow(n))) {
        return r;
    } else if (pack) {
        if ((r = pack((const uint16_t *)a->d_slot_of_lxc.p, (gf_rec *)w.rec.p, (uint32_t *)w.keys.p))) return r;
    } else {
        ProfScope ps("k_ing_pack", s);
        hipLaunchKernelGGL(k_ing_pack, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, *pkts,
                           (const uint16_t *)a->d_slot_of_lxc.p, (gf_rec *)w.rec.p,
                           (uint32_t *)w.keys.p);
        if ((r = hip_ok(hipGetLastError(), "k_ing_pack"))) return r;
    }
    host_mark("pack");
    if (!prepared && (r = schedule_groups(n, s, (const gf_rec *)w.rec.p, ta && ta->kind == 2))) return r;
    host_mark("sched");
    uint32_t *d_sched = (uint32_t *)w.sched.p;
    // 4. handle_policy: one bucket per lane, buckets from the longest-first queue
    IngCtx X{};
    X.cfgs = (const gf_lxc_dev *)a->d_cfgs.p;
    X.saddr6 = pkts->saddr6; X.daddr6 = pkts->daddr6;
    X.a6_stride = ta ? 32u : 16u;                       // the pipeline's / egress' interleaved addresses
    if (ct4m) X.ct4 = cfg_ct4;
    if (ct6m) X.ct6 = cfg_ct6;
    X.now = now_sec; X.host_ifindex = host_ifindex();
    X.strict = strict;
    X.pout = pout;
    X.pout_wo = GF_POUT_WO && pout && ta && ta->kind == 1 ? 1u : 0u;
    X.pol_wave = ta && ta->kind == 2 ? 1u : 0u;
    X.snap = wsnap; X.snap_stride = ev_stride;
    const gf_node_cfg &node = node_cfg();
    X.gw = node.ipv4_gateway;
    memcpy(X.host6, node.host_ip6, 16);
    if (tracing) { X.tmark = (uint8_t *)trace_ws().mark.p; X.tcap = (uint8_t *)trace_ws().px.p; }
    if (ta) { X.rlog = ta->rlog; X.rlog_n = ta->rlog_n; X.rlog_off = ta->rlog_off; X.rs = ta->rs; }
    if ((r = px_log_begin(n, s, X, px_keep))) return r;
    // Non-strict mode accounts each kernel's net element change into its family's map.
    uint32_t *cnt4 = ct4m ? (uint32_t *)ct4m->d_count.p : nullptr, *cnt6 = ct6m ? (uint32_t *)ct6m->d_count.p : nullptr;
    unsigned long long *sink = (unsigned long long *)stats_sink();
    {
        // resident-grid launches: every wave loops on its family's queue until it is drained
        uint32_t grid = resident_blocks(8);
        uint32_t need = (n + BLOCK - 1) / BLOCK;
        if (grid > need) grid = need;
        {
            ProfScope ps("k_ing_groups", s);
            if (cm.pct)                                 // per-endpoint CT maps (ConntrackLocal)
                hipLaunchKernelGGL((k_ing_groups<4, 1, true>), dim3(grid), dim3(BLOCK), 0, s, X, d_sched,
                                   (const uint2 *)w.order.p, (const uint32_t *)w.perm.p, (const gf_rec *)w.rec.p, out,
                                   nullptr, sink);
            else if (X.pol_wave)                        // the egress deliveries' pass (single-packet buckets)
                hipLaunchKernelGGL((k_ing_groups<4, GF_GRAB_ING, false, true>), dim3(grid), dim3(BLOCK), 0, s, X, d_sched,
                                   (const uint2 *)w.order.p, (const uint32_t *)w.perm.p, (const gf_rec *)w.rec.p, out, cnt4,
                                   sink);
            else
                hipLaunchKernelGGL(k_ing_groups<4>, dim3(grid), dim3(BLOCK), 0, s, X, d_sched, (const uint2 *)w.order.p,
                                   (const uint32_t *)w.perm.p,
                                   (const gf_rec *)w.rec.p, out, cnt4, sink);
        }
        if (pkts->saddr6) {    // IPv6 packets reach conntrack only with v6 columns
            ProfScope ps("k_ing_groups6", s);
            if (cm.pct)
                hipLaunchKernelGGL((k_ing_groups<6, 1, true>), dim3(grid), dim3(BLOCK), 0, s, X, d_sched,
                                   (const uint2 *)w.order.p, (const uint32_t *)w.perm.p, (const gf_rec *)w.rec.p, out,
                                   nullptr, sink);
            else
                hipLaunchKernelGGL(k_ing_groups<6>, dim3(grid), dim3(BLOCK), 0, s, X, d_sched, (const uint2 *)w.order.p,
                                   (const uint32_t *)w.perm.p,
                                   (const gf_rec *)w.rec.p, out, cnt6, sink);
        }
    }
    if ((r = hip_ok(hipGetLastError(), "k_ing_groups"))) return r;
    host_mark("groups");
    if ((r = px_log_apply(X, s, wsnap, ev_len ? ev_len : pkts->len, ev_stride, pout ? pout : (uint8_t *)out,
                          pout != nullptr, n)))
        return r;
    {
        EvSrc E{};
        E.recs = pout ? pout : (const uint8_t *)out;
        E.stride = pout ? 24u : 8u; E.act_off = pout ? 1u : 0u; E.stage_off = pout ? 0 : -1;
        E.prec = (const gf_rec *)w.rec.p; E.cfgs = (const gf_lxc_dev *)a->d_cfgs.p;
        E.len = ev_len ? ev_len : pkts->len; E.flow_hash = pkts->flow_hash; E.n = n;
        E.snap = ev_snap; E.snap_stride = ev_stride;
        if (tracing) {
            const TraceWs &t = trace_ws();
            E.trace = 1; E.kind = ta ? ta->kind : 0u;
            E.tmark = (const uint8_t *)t.mark.p; E.tcap_px = (const uint8_t *)t.px.p;
            E.tcap_in = (const uint8_t *)t.in.p;
            E.host_ifindex = host_ifindex(); E.encap_ifindex = node.encap_ifindex;
            if (ta) {
                E.nd_trace = ta->nd_trace; E.nd_ifindex = ta->nd_ifindex;
                E.orig = ta->orig; E.lxc_id = ta->lxc_id;
                E.slot_of = (const uint16_t *)a->d_slot_of_lxc.p;
            }
        }
        if ((r = emit_drop_events(E, s))) return r;
    }
    host_mark("px+ev");
    for (auto &p : progs) {
        if (p->policy) p->policy->device_modified();
    }
    if (lru && ((r = lru_evict_maps(cm.m4, now_sec, s)) || (r = lru_evict_maps(cm.m6, now_sec, s)))) return r;
    host_mark("lru");
    for (auto *v : {&cm.m4, &cm.m6})
        for (auto &m : *v) m->device_modified();
    return 0;
}

// The stateless half of ingress_run (k_ing_pack + the flow-group schedule) into ws().
static int ingress_prepare(const std::shared_ptr<PolicyArray> &a, const gf_pkt_cols *pkts, hipStream_t s) {
    const uint32_t n = pkts->n;
    Workspace &w = ws();
    int r;
    if ((r = ws_grow(n))) return r;
    {
        ProfScope ps("k_ing_pack", s);
        hipLaunchKernelGGL(k_ing_pack, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, *pkts,
                           (const uint16_t *)a->d_slot_of_lxc.p, (gf_rec *)w.rec.p, (uint32_t *)w.keys.p);
        if ((r = hip_ok(hipGetLastError(), "k_ing_pack"))) return r;
    }
    return schedule_groups(n, s, (const gf_rec *)w.rec.p);
}

// The stream that builds the next batch's schedule, and the events between the two.
struct PipeSync {
    hipStream_t aux = nullptr;
    hipEvent_t ready = nullptr, built[2] = {nullptr, nullptr}, done[2] = {nullptr, nullptr};
    int init() {
        if (aux) return 0;
        if (hip_ok(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking), "aux stream")) return -EIO;
        for (hipEvent_t *e : {&ready, &built[0], &built[1], &done[0], &done[1]})
            if (hip_ok(hipEventCreateWithFlags(e, hipEventDisableTiming), "pipe event")) return -EIO;
        return 0;
    }
};
static PipeSync &pipe_sync() { static const char tag = 0; return cur_ctx().get<PipeSync>(&tag); }

extern "C" {

int gf_policy_ingress_classify_batches(int array, uint32_t nb, const gf_pkt_cols *const *batches,
                                       const uint32_t *now_sec, gf_ingress_out *const *outs, void *stream) {
    std::shared_lock<std::shared_mutex> g(prog_lock());
    auto o = get_obj(array);
    if (!o || o->kind != ObjKind::PolicyArray) return -EBADF;
    auto a = std::static_pointer_cast<PolicyArray>(o);
    if (nb && (!batches || !now_sec || !outs)) return -EFAULT;
    for (uint32_t k = 0; k < nb; k++) {
        const int c = check_cols(batches[k]);
        if (c < 0) return c;
        if (c && !outs[k]) return -EFAULT;
        if (batches[k]->n > (1u << 30)) return -E2BIG;
    }
    hipStream_t s = (hipStream_t)stream;
    CtxScope cx(s);
    std::lock_guard<std::mutex> ag(a->mu);
    MapLocks L;
    lock_array_maps(L, a);
    L.lock();
    CallOrder co(s, L, a.get());
    PipeSync &P = pipe_sync();
    int r;
    if ((r = P.init())) return r;
    std::vector<std::shared_ptr<ProgLxc>> progs;
    if ((r = prog_table(a, s, progs))) return r;          // the program table k_ing_pack reads, on s
    if (hip_ok(hipEventRecord(P.ready, s), "ready") || hip_ok(hipStreamWaitEvent(P.aux, P.ready, 0), "aux wait"))
        return -EIO;
    auto prep = [&](uint32_t k) -> int {                  // batch k's schedule on the aux stream, workspace k & 1
        const int slot = (int)(k & 1u);
        if (k >= 2 && hip_ok(hipStreamWaitEvent(P.aux, P.done[slot], 0), "aux wait done")) return -EIO;
        cur_ctx().ws_slot = slot;
        int rr = batches[k]->n ? ingress_prepare(a, batches[k], P.aux) : 0;
        cur_ctx().ws_slot = 0;
        if (rr) return rr;
        return hip_ok(hipEventRecord(P.built[slot], P.aux), "built") ? -EIO : 0;
    };
    if (nb && (r = prep(0))) return r;
    for (uint32_t k = 0; k < nb; k++) {
        if (k + 1 < nb && (r = prep(k + 1))) return r;    // overlaps handle_policy of batch k
        const int slot = (int)(k & 1u);
        if (hip_ok(hipStreamWaitEvent(s, P.built[slot], 0), "wait built")) return -EIO;
        if (batches[k]->n) {
            cur_ctx().ws_slot = slot;
            r = ingress_run(a, batches[k], now_sec[k], outs[k], s, PackFn(), nullptr, nullptr, nullptr, 0, nullptr,
                            true, false, true);
            cur_ctx().ws_slot = 0;
            if (r) return r;
        }
        if (hip_ok(hipEventRecord(P.done[slot], s), "done")) return -EIO;
    }
    return 0;
}

int gf_policy_ingress_classify(int array, const gf_pkt_cols *pkts, uint32_t now_sec, gf_ingress_out *out,
                               void *stream) {
    std::shared_lock<std::shared_mutex> g(prog_lock());
    auto o = get_obj(array);
    if (!o || o->kind != ObjKind::PolicyArray) return -EBADF;
    auto a = std::static_pointer_cast<PolicyArray>(o);
    int c = check_cols(pkts);
    if (c <= 0) return c;
    if (!out) return -EFAULT;
    if (pkts->n > (1u << 30)) return -E2BIG;
    CtxScope cx((hipStream_t)stream);
    std::lock_guard<std::mutex> ag(a->mu);
    MapLocks L;
    lock_array_maps(L, a);
    L.lock();
    CallOrder co((hipStream_t)stream, L, a.get());
    return ingress_run(a, pkts, now_sec, out, (hipStream_t)stream);
}

// ---- full pipeline ----
int gf_pipeline_load(const gf_pipeline_cfg *cfg) {
    std::unique_lock<std::shared_mutex> g(prog_lock());
    if (!cfg) return -EFAULT;
    auto p = std::make_shared<ProgPipe>();
    p->cfg = *cfg;
    if (cfg->xdp_prog) {
        auto o = get_obj(cfg->xdp_prog);
        if (!o || o->kind != ObjKind::ProgXdp) return -EBADF;
        p->xdp = std::static_pointer_cast<ProgXdp>(o);
    }
    if (cfg->lb_prog) {
        auto o = get_obj(cfg->lb_prog);
        if (!o || o->kind != ObjKind::ProgLb) return -EBADF;
        p->lb = std::static_pointer_cast<ProgLb>(o);
    }
    auto m = get_map(cfg->netdev.lxc_map);
    if (!m) return -EBADF;
    if (m->ksz != 20 || m->vsz != 112 || m->is_lpm()) return -EINVAL;
    p->lxc = m;
    auto a = get_obj(cfg->policy_array);
    if (!a || a->kind != ObjKind::PolicyArray) return -EBADF;
    p->policy = std::static_pointer_cast<PolicyArray>(a);
    return new_handle(p);
}

int gf_pipeline_classify(int pipe, const gf_pipe_batch *b, uint32_t now_sec, gf_pipeline_out *out,
                         uint8_t *nd6, uint8_t *snap_out, void *stream) {
    std::shared_lock<std::shared_mutex> g(prog_lock());
    auto o = get_obj(pipe);
    if (!o || o->kind != ObjKind::ProgPipe) return -EBADF;
    auto p = std::static_pointer_cast<ProgPipe>(o);
    if (!b) return -EFAULT;
    const gf_frames &fr = b->frames;
    if (fr.n == 0) return 0;
    if (!fr.snap || !fr.len || !out) return -EFAULT;
    if (fr.snap_stride < 14) return -EINVAL;
    if (fr.n > (1u << 30)) return -E2BIG;
    hipStream_t s = (hipStream_t)stream;
    HostMarks hm;
    CtxScope cx(s);
    std::lock_guard<std::mutex> ag(p->policy->mu);
    MapLocks L;
    if (p->xdp) lock_xdp_maps(L, *p->xdp);
    if (p->lb) { L.add(p->lb->lb4); L.add(p->lb->lb6); }
    L.add(p->lxc);
    lock_array_maps(L, p->policy);
    L.lock();
    CallOrder co(s, L, p->policy.get());
    int r;
    const uint32_t n = fr.n;
    PipeDev P{};
    if (p->xdp) {
        auto &x = *p->xdp;
        if ((r = push_map(x.m4h, s)) || (r = push_map(x.m4l, s)) || (r = push_map(x.m6h, s)) ||
            (r = push_map(x.m6l, s)) || (r = push_map(x.lxc, s)))
            return r;
        if (x.m4h) { P.x.h4 = x.m4h->hdesc(); P.x.has_h4 = 1; }
        if (x.m6h) { P.x.h6 = x.m6h->hdesc(); P.x.has_h6 = 1; }
        if (x.m4l) P.x.l4 = x.m4l->tdesc();
        if (x.m6l) P.x.l6 = x.m6l->tdesc();
        P.x.lxc = x.lxc->hdesc();
        xdp_sets(x.m4h, x.lxc, P.x, s);
        xdp_dir(x.m4l, P.x, s);
        P.has_xdp = 1;
    }
    if (p->lb) {
        if ((r = push_map(p->lb->lb4, s)) || (r = push_map(p->lb->lb6, s))) return r;
        if (p->lb->lb4) P.L.s4 = p->lb->lb4->hdesc();
        if (p->lb->lb6) P.L.s6 = p->lb->lb6->hdesc();
        P.L.flags = p->lb->cfg.flags;
        P.lb_redirect_ifindex = p->lb->cfg.redirect_ifindex;
        P.has_lb = 1;
    }
    if ((r = push_map(p->lxc, s))) return r;
    P.nd.lxc = p->lxc->hdesc();
    if (getenv("GF_XDP_NOSETS") || p->lxc->addr_set(20, 8192, s, &P.nd.lxset, &P.nd.lxbits, &P.nd.lxzero))
        P.nd.lxset = nullptr;
    P.nd.flags = p->cfg.netdev.flags;
    P.nd.fixed_secctx = p->cfg.netdev.fixed_secctx;
    memcpy(P.nd.router6, p->cfg.netdev.router_ip6, 8);
    // LDS staging of the block's frames (one row per lane)
    // (256 lanes per block up to 128-B snaps, 128 lanes up to 256 B: <= 32 KiB)
    if (fr.snap_stride > 256) return -EINVAL;          // not a header snap
    const uint32_t nt = fr.snap_stride <= 128 ? 256u : 128u;
    const size_t lds = (size_t)nt * fr.snap_stride;
    PipeWs &w = pipe_ws();
    auto grow = [](DevBuf &d, size_t want) -> int { return d.bytes >= want ? 0 : d.ensure(want); };
    if ((r = grow(w.s6, (size_t)n * 32))) return r;    // saddr6 | daddr6 per packet (IngCtx::a6_stride 32)
    P.vec_copy = (fr.snap_stride % 16 == 0) && (((uintptr_t)fr.snap | (uintptr_t)snap_out) & 15u) == 0;
    PassArgs ta{};
    ta.kind = 1;
    ta.nd_trace = (p->cfg.netdev.flags & GF_NETDEV_F_TRACE_NOTIFY) ? 1u : 0u;
    ta.nd_ifindex = p->cfg.netdev.ingress_ifindex;
    ta.on = event_ring().records && (ta.nd_trace || array_traces(p->policy));
    if (ta.on && (r = trace_prepare(n, ta.nd_trace != 0, s))) return r;
    if (ta.on && ta.nd_trace) P.tcap_in = (uint8_t *)trace_ws().in.p;
    unsigned long long *sink = (unsigned long long *)stats_sink();
    const uint32_t grid = (n + nt - 1) / nt;         // one NT-frame tile per block
    gf_pkt_cols c2{};
    c2.n = n;
    c2.saddr6 = (const uint8_t *)w.s6.p; c2.daddr6 = (const uint8_t *)w.s6.p + 16;
    auto front = [&](const uint16_t *slot_of, gf_rec *rec, uint32_t *keys) -> int {
        ProfScope ps("k_pipe_front", s);
        if (nt == 256)
            hipLaunchKernelGGL(k_pipe_front<256>, dim3(grid), dim3(256), lds, s, fr, b->tc_index, b->flow_hash, P,
                               slot_of, rec, keys, (uint8_t *)w.s6.p, (uint8_t *)w.s6.p + 16, out, nd6, snap_out, sink);
        else
            hipLaunchKernelGGL(k_pipe_front<128>, dim3(grid), dim3(128), lds, s, fr, b->tc_index, b->flow_hash, P,
                               slot_of, rec, keys, (uint8_t *)w.s6.p, (uint8_t *)w.s6.p + 16, out, nd6, snap_out, sink);
        return hip_ok(hipGetLastError(), "k_pipe_front");
    };
    c2.flow_hash = b->flow_hash;
    return ingress_run(p->policy, &c2, now_sec, nullptr, s, front, (uint8_t *)out, fr.len,
                       snap_out ? snap_out : fr.snap, fr.snap_stride, snap_out, true, false, false, &ta);
}

// ---- ingest re-partition ----
int gf_pipeline_partition(int pipe, const gf_pipe_batch *b, uint32_t self_rank, uint32_t nranks, uint32_t *owner,
                          uint32_t *order, uint32_t *counts, void *stream) {
    std::shared_lock<std::shared_mutex> g(prog_lock());
    auto o = get_obj(pipe);
    if (!o || o->kind != ObjKind::ProgPipe) return -EBADF;
    auto p = std::static_pointer_cast<ProgPipe>(o);
    if (!b || !owner || !order || !counts) return -EFAULT;
    if (nranks == 0 || nranks > 65536 || self_rank >= nranks) return -EINVAL;
    const gf_frames &fr = b->frames;
    hipStream_t s = (hipStream_t)stream;
    CtxScope cx(s);
    MapLocks L;
    if (p->lb) { L.add(p->lb->lb4); L.add(p->lb->lb6); }
    L.lock();
    CallOrder co(s, L);
    if (hip_ok(hipMemsetAsync(counts, 0, (size_t)nranks * 4, s), "partition counts")) return -EIO;
    if (fr.n == 0) return 0;
    if (!fr.snap || !fr.len) return -EFAULT;
    if (fr.snap_stride < 14) return -EINVAL;
    if (fr.n > (1u << 30)) return -E2BIG;
    int r;
    PipeDev P{};
    if (p->lb) {
        if ((r = push_map(p->lb->lb4, s)) || (r = push_map(p->lb->lb6, s))) return r;
        if (p->lb->lb4) P.L.s4 = p->lb->lb4->hdesc();
        if (p->lb->lb6) P.L.s6 = p->lb->lb6->hdesc();
        P.L.flags = p->lb->cfg.flags;
        P.has_lb = 1;
    }
    const uint32_t n = fr.n;
    struct PartWs { DevBuf keys, tmp; };
    static const char tag = 0;
    PartWs &pw = cur_ctx().get<PartWs>(&tag);
    DevBuf &keys = pw.keys, &tmp = pw.tmp;
    auto grow = [](DevBuf &d, size_t want) -> int { return d.bytes >= want ? 0 : d.ensure(want); };
    if ((r = grow(keys, (size_t)n * 4))) return r;
    {
        ProfScope ps("k_partition", s);
        hipLaunchKernelGGL(k_partition, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, fr, b->flow_hash, P, self_rank,
                           nranks, owner, counts);
        if ((r = hip_ok(hipGetLastError(), "k_partition"))) return r;
    }
    // stable counting order by owner: radix sort of (owner, index) over the owner's bits
    int bits = 1;
    while ((1u << bits) < nranks) bits++;
    size_t tb = 0;
    (void)rocprim::radix_sort_pairs(nullptr, tb, owner, (uint32_t *)keys.p, rocprim::counting_iterator<uint32_t>(0u), order,
                                    n, 0, bits, s);
    if ((r = grow(tmp, tb + 256))) return r;
    tb = tmp.bytes;
    if (hip_ok(rocprim::radix_sort_pairs(tmp.p, tb, owner, (uint32_t *)keys.p, rocprim::counting_iterator<uint32_t>(0u),
                                         order, n, 0, bits, s), "partition sort"))
        return -EIO;
    return 0;
}

// ---- conntrack GC ----
int gf_ct_gc(int map, uint32_t filter_time, void *stream) {
    std::shared_lock<std::shared_mutex> g(prog_lock());
    auto m = get_map(map);
    if (!m) return -EBADF;
    if (m->is_lpm() || (m->ksz != 14 && m->ksz != 40) || m->vsz != 48) return -EINVAL;
    hipStream_t s = (hipStream_t)stream;
    CtxScope cx(s);
    std::lock_guard<std::recursive_mutex> mg(m->mu);
    CallOrder co(s, std::vector<OrderPt *>{&m->ord});
    const uint32_t lt_off = m->ht.codec == GF_VCODEC_CT ? 0u : 32u;
    if (m->host_valid || !m->dev_valid || !m->d_slots.p) {
        // host shadow authoritative: delete there, the replica is rebuilt on the next push
        if (m->ht.slots.empty()) return 0;              // never materialised: no entries
        uint64_t dead = 0;
        std::vector<std::string> keys;
        uint8_t v[GF_CT_VSZ];
        for (uint64_t i = 0; i < m->ht.nslots; i++) {
            if (m->ht.state(i) != GF_SLOT_FULL) continue;
            m->ht.get_val(i, v);
            uint32_t lt;
            memcpy(&lt, v + lt_off, 4);
            if (lt < filter_time) keys.emplace_back((const char *)m->ht.key(i), m->ksz);
        }
        for (auto &k : keys) if (m->erase((const uint8_t *)k.data()) == 0) dead++;
        return (int)std::min<uint64_t>(dead, 0x7fffffff);
    }
    LruDev *L;
    uint32_t *bits;
    int rr;
    if ((rr = ct_sweep_bufs(*m, L, bits))) return rr;
    GcCut cut{filter_time, filter_time, 1u, 0u};             // lifetime < filter_time
    const unsigned long long zero2[2] = {0, 0};
    if (hip_ok(hipMemcpyAsync(&L->cut, &cut, sizeof cut, hipMemcpyHostToDevice, s), "gc cut") ||
        hip_ok(hipMemcpyAsync(L->res, zero2, sizeof zero2, hipMemcpyHostToDevice, s), "gc res"))
        return -EIO;
    {
        ProfScope ps("k_gc", s);
        ct_sweep_launch(*m, L, bits, s);
    }
    if (hip_ok(hipGetLastError(), "k_gc")) return -EIO;
    unsigned long long r[2] = {0, 0};
    const GcCut off{0, 0, 0u, 0u};
    if (hip_ok(hipMemcpyAsync(r, L->res, 16, hipMemcpyDeviceToHost, s), "gc result") ||
        hip_ok(hipMemcpyAsync(&L->cut, &off, sizeof off, hipMemcpyHostToDevice, s), "gc cut off") ||
        hip_ok(hipStreamSynchronize(s), "gc sync"))
        return -EIO;
    // device element count: entries are deleted, tombstones were already uncounted
    uint32_t cnt = 0;
    if (hip_ok(hipMemcpy(&cnt, m->d_count.p, 4, hipMemcpyDeviceToHost), "gc count")) return -EIO;
    cnt = cnt >= r[0] ? cnt - (uint32_t)r[0] : 0u;
    if (hip_ok(hipMemcpy(m->d_count.p, &cnt, 4, hipMemcpyHostToDevice), "gc count")) return -EIO;
    m->dev_count_hi = cnt;
    m->ev_pending = 0;
    m->st_floor = m->lru_seq;
    m->device_modified();
    return (int)std::min<unsigned long long>(r[0], 0x7fffffff);
}

#if GF_WRSTATS
// Diagnostic builds only: the write-source counters (gf_device.h WR_*), read and cleared.
int gf_diag_wrstats(unsigned long long *out, uint32_t n) {
    if (hip_ok(hipDeviceSynchronize(), "wrstats sync")) return -EIO;
    unsigned long long v[WR_N] = {0};
    if (hip_ok(hipMemcpyFromSymbol(v, HIP_SYMBOL(g_wrstat), sizeof v), "wrstats")) return -EIO;
    const unsigned long long z[WR_N] = {0};
    if (hip_ok(hipMemcpyToSymbol(HIP_SYMBOL(g_wrstat), z, sizeof z), "wrstats clear")) return -EIO;
    for (uint32_t k = 0; k < n && k < WR_N; k++) out[k] = v[k];
    return WR_N;
}
#endif

int gf_ct_evict_log(int map, gf_ct_evict_rec *out, uint32_t max) {
    auto m = get_map(map);
    if (!m) return -EBADF;
    if (max && !out) return -EFAULT;
    std::lock_guard<std::recursive_mutex> mg(m->mu);
    if (!m->d_lru.p) return 0;
    static_assert(sizeof(LruLog) == sizeof(gf_ct_evict_rec), "log record layout");
    if (hip_ok(hipDeviceSynchronize(), "evict log sync")) return -EIO;
    uint32_t n = 0;
    LruDev *L = (LruDev *)m->d_lru.p;
    if (hip_ok(hipMemcpy(&n, &L->nlog, 4, hipMemcpyDeviceToHost), "evict log count")) return -EIO;
    const uint32_t k = std::min(std::min(n, GF_LRU_LOGCAP), max);
    if (k && hip_ok(hipMemcpy(out, L->log, (size_t)k * sizeof(LruLog), hipMemcpyDeviceToHost), "evict log")) return -EIO;
    return (int)std::min<uint32_t>(n, 0x7fffffffu);
}

}  // extern "C"


// ================================================================ bulk insert (gf_map_update_batch)
// A batch of distinct keys loaded straight into a fixed-capacity table in HBM:
// one lane per element walks the key's probe sequence, overwrites the key's slot
// (BPF_ANY) or claims the first EMPTY slot with a CAS on its state word (BUSY),
// fills key and value and publishes FULL with a release store; readers acquire
// the state word first.  Keys are distinct (checked first), so the outcome is
// that of the sequential updates.
__device__ __forceinline__ void bulk_key_words(const uint8_t *k, uint32_t ksz, uint32_t *kw) {
    for (int q = 0; q < 16; q++) kw[q] = 0;
    for (uint32_t b = 0; b < ksz; b++) kw[b >> 2] |= (uint32_t)k[b] << (8 * (b & 3));
}
__device__ __forceinline__ bool bulk_eq(const uint8_t *a, const uint8_t *b, uint32_t n) {
    for (uint32_t q = 0; q < n; q++) if (a[q] != b[q]) return false;
    return true;
}
__global__ __launch_bounds__(BLOCK) void k_bulk_hash(const uint8_t *keys, uint32_t ksz, uint32_t mode, uint32_t n, uint32_t *h) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint32_t kw[16];
        bulk_key_words(keys + (size_t)i * ksz, ksz, kw);
        h[i] = gf_key_hash(kw, ksz, mode);
    }
}
// flag[0]: two equal keys in the batch (equal keys have equal hashes: adjacent runs after the sort)
__global__ __launch_bounds__(BLOCK) void k_bulk_dups(const uint32_t *hs, const uint32_t *idx, const uint8_t *keys,
                                                     uint32_t ksz, uint32_t n, uint32_t *flag) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x)
        for (int64_t k = (int64_t)j - 1; k >= 0 && hs[k] == hs[j]; k--)
            if (bulk_eq(keys + (size_t)idx[k] * ksz, keys + (size_t)idx[j] * ksz, ksz)) atomicOr(&flag[0], 1u);
}
__device__ __forceinline__ uint32_t bulk_state_word(const gf_htab_desc &d, uint64_t j) {
    const uint32_t *sw = reinterpret_cast<const uint32_t *>(d.slots + j * d.slot_size + (d.ksz & ~3u));
    return __hip_atomic_load(sw, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
// flag[1]: a key of the batch is already in the table
__global__ __launch_bounds__(BLOCK) void k_bulk_probe(gf_htab_desc d, const uint8_t *keys, const uint32_t *h, uint32_t n,
                                                      uint32_t *flag) {
    const uint32_t sb = 8 * (d.ksz & 3u);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint8_t *k = keys + (size_t)i * d.ksz;
        uint64_t j = gf_home_slot(h[i], d.mask, d.slot_size);
        for (uint64_t p = 0; p <= d.mask; p++, j = (j + 1) & d.mask) {
            const uint32_t st = (bulk_state_word(d, j) >> sb) & 0xffu;
            if (st == GF_SLOT_EMPTY) break;
            if (st == GF_SLOT_FULL && bulk_eq(d.slots + j * d.slot_size, k, d.ksz)) { atomicOr(&flag[1], 1u); break; }
        }
    }
}
__global__ __launch_bounds__(BLOCK) void k_bulk_insert(gf_htab_desc d, uint32_t codec, const uint8_t *keys,
                                                       const uint8_t *vals, const uint32_t *h, uint32_t n) {
    const uint32_t sb = 8 * (d.ksz & 3u), kw0 = d.ksz & ~3u;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint8_t *k = keys + (size_t)i * d.ksz, *ext = vals + (size_t)i * d.vsz;
        uint8_t in[128];
        if (codec == GF_VCODEC_CT) gf_ct_encode(ext, in);
        else if (codec == GF_VCODEC_POL) gf_pol_encode(ext, in);
        else for (uint32_t b = 0; b < d.vsz; b++) in[b] = ext[b];
        uint32_t keep = 0;
        for (uint32_t b = kw0; b < d.ksz; b++) keep |= (uint32_t)k[b] << (8 * (b - kw0));
        auto put_val = [&](uint64_t j) {
            uint8_t *sl = d.slots + j * d.slot_size;
            for (uint32_t b = 0; b < d.vin; b++) sl[d.voff + b] = in[b];
            for (uint32_t b = d.vin; b < d.vsz; b++) d.vals[j * d.sstride + (b - d.vin)] = in[b];
        };
        uint64_t j = gf_home_slot(h[i], d.mask, d.slot_size);
        for (uint64_t p = 0; p <= d.mask;) {
            uint32_t *sw = reinterpret_cast<uint32_t *>(d.slots + j * d.slot_size + kw0);
            uint32_t w = bulk_state_word(d, j);
            const uint32_t st = (w >> sb) & 0xffu;
            if (st == GF_SLOT_FULL && bulk_eq(d.slots + j * d.slot_size, k, d.ksz)) { put_val(j); break; }
            if (st == GF_SLOT_EMPTY) {
                const uint32_t busy = keep | ((uint32_t)GF_SLOT_BUSY << sb);
                uint32_t seen = w;
                __hip_atomic_compare_exchange_strong(sw, &seen, busy, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                if (seen != w) continue;                       // lost the slot: look at it again
                uint8_t *sl = d.slots + j * d.slot_size;
                for (uint32_t b = 0; b < kw0; b++) sl[b] = k[b];
                put_val(j);
                __hip_atomic_store(sw, keep | ((uint32_t)GF_SLOT_FULL << sb), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                atomicAdd(d.count, 1u);
                break;
            }
            p++;
            j = (j + 1) & d.mask;
        }
    }
}

namespace gf {
int dev_bulk_insert(Map &m, const uint8_t *keys, const uint8_t *vals, uint32_t n, uint64_t flags, bool &fallback) {
    fallback = true;
    int dc = 0;
    if (hipGetDeviceCount(&dc) != hipSuccess || dc == 0 || m.vsz > 128 || m.ksz > 64) return 0;
    const bool had = m.dev_auth();
    uint64_t before = 0;
    if (had) { uint32_t c; if (m.dev_count(c)) return 0; before = c; }
    if (before + n > dev_insert_limit(m)) return 0;     // the host path reports E2BIG at the exact element
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    static DevBuf dk, dv, dh, dhs, didx, tmp, dflag;
    auto grow = [](DevBuf &b, size_t want) -> int { return b.bytes >= want ? 0 : b.ensure(want); };
    int r;
    if ((r = grow(dk, (size_t)n * m.ksz)) || (r = grow(dv, (size_t)n * m.vsz)) || (r = grow(dh, (size_t)n * 4)) ||
        (r = grow(dhs, (size_t)n * 4)) || (r = grow(didx, (size_t)n * 4)) || (r = grow(dflag, 8)))
        return r;
    if (!had) {                                          // create the (empty) replica
        m.dev_valid = false;
        if ((r = m.push((hipStream_t)0))) return r;
    }
    const hipStream_t s = (hipStream_t)0;
    if (hip_ok(hipMemcpy(dk.p, keys, (size_t)n * m.ksz, hipMemcpyHostToDevice), "bulk keys") ||
        hip_ok(hipMemcpy(dv.p, vals, (size_t)n * m.vsz, hipMemcpyHostToDevice), "bulk vals") ||
        hip_ok(hipMemset(dflag.p, 0, 8), "bulk flags"))
        return -EIO;
    m.xfer_h2d += (size_t)n * (m.ksz + m.vsz);
    const gf_htab_desc d = m.hdesc();
    const uint32_t g = std::min<uint32_t>((n + BLOCK - 1) / BLOCK, 65535u);
    hipLaunchKernelGGL(k_bulk_hash, dim3(g), dim3(BLOCK), 0, s, (const uint8_t *)dk.p, m.ksz, m.ht.mode, n, (uint32_t *)dh.p);
    size_t tb = 0;
    (void)rocprim::radix_sort_pairs(nullptr, tb, (uint32_t *)dh.p, (uint32_t *)dhs.p, rocprim::counting_iterator<uint32_t>(0u),
                                    (uint32_t *)didx.p, n, 0, 32, s);
    if ((r = grow(tmp, tb + 256))) return r;
    tb = tmp.bytes;
    if (hip_ok(rocprim::radix_sort_pairs(tmp.p, tb, (uint32_t *)dh.p, (uint32_t *)dhs.p, rocprim::counting_iterator<uint32_t>(0u),
                                         (uint32_t *)didx.p, n, 0, 32, s), "bulk sort"))
        return -EIO;
    hipLaunchKernelGGL(k_bulk_dups, dim3(g), dim3(BLOCK), 0, s, (const uint32_t *)dhs.p, (const uint32_t *)didx.p,
                       (const uint8_t *)dk.p, m.ksz, n, (uint32_t *)dflag.p);
    if (had && flags == GF_NOEXIST)
        hipLaunchKernelGGL(k_bulk_probe, dim3(g), dim3(BLOCK), 0, s, d, (const uint8_t *)dk.p, (const uint32_t *)dh.p, n,
                           (uint32_t *)dflag.p);
    uint32_t fl[2] = {0, 0};
    if (hip_ok(hipGetLastError(), "bulk check") || hip_ok(hipMemcpy(fl, dflag.p, 8, hipMemcpyDeviceToHost), "bulk flags"))
        return -EIO;
    if (fl[0] || fl[1]) return 0;                        // duplicates / EEXIST: the sequential host path
    hipLaunchKernelGGL(k_bulk_insert, dim3(g), dim3(BLOCK), 0, s, d, m.ht.codec, (const uint8_t *)dk.p,
                       (const uint8_t *)dv.p, (const uint32_t *)dh.p, n);
    if (hip_ok(hipGetLastError(), "k_bulk_insert") || hip_ok(hipDeviceSynchronize(), "bulk sync")) return -EIO;
    m.host_valid = false;
    m.dev_gen++;
    m.dev_count_hi = before + n;
    m.ev_pending = 0;
    m.st_floor = m.lru_seq;
    fallback = false;
    return 0;
}
}  // namespace gf

// ================================================================ chunked dump (gf_map_lookup_batch)
// The FULL slots of a range of a device-authoritative hash map, compacted in
// slot order on the device (rocPRIM select over the slot indices), their keys
// and reference-layout values gathered into a staging buffer: only the entries
// cross PCIe, a 64M-entry CT dumps without its 16 GB slot arrays moving.
struct SlotFull {
    const uint8_t *slots;
    uint64_t base;
    uint32_t ss, ksz;
    __device__ bool operator()(uint32_t j) const { return slots[(base + j) * ss + ksz] == GF_SLOT_FULL; }
};
__global__ __launch_bounds__(BLOCK) void k_dump_gather(gf_htab_desc d, uint32_t codec, uint64_t base, const uint32_t *sel,
                                                       const uint32_t *nsel, uint32_t cap, uint8_t *keys, uint8_t *vals) {
    const uint32_t n = min(*nsel, cap);
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        const uint64_t i = base + sel[t];
        const uint8_t *sl = d.slots + i * d.slot_size;
        for (uint32_t b = 0; b < d.ksz; b++) keys[(size_t)t * d.ksz + b] = sl[b];
        uint8_t in[128], ext[128];
        for (uint32_t b = 0; b < d.vin; b++) in[b] = sl[d.voff + b];
        for (uint32_t b = d.vin; b < d.vsz; b++) in[b] = d.vals[i * d.sstride + (b - d.vin)];
        if (codec == GF_VCODEC_CT) gf_ct_decode(in, ext);
        else if (codec == GF_VCODEC_POL) gf_pol_decode(in, ext);
        else for (uint32_t b = 0; b < d.vsz; b++) ext[b] = in[b];
        for (uint32_t b = 0; b < d.vsz; b++) vals[(size_t)t * d.vsz + b] = ext[b];
    }
}

namespace gf {
int dev_dump(Map &m, uint64_t start, uint32_t max, uint8_t *keys, uint8_t *vals, uint32_t *n, uint64_t *next) {
    static std::mutex mu;                                // the staging buffers below
    std::lock_guard<std::mutex> g(mu);
    static DevBuf sel, nsel, tmp, dk, dv;
    *n = 0; *next = start;
    if (!max || start >= m.ht.nslots) { *next = m.ht.nslots; return 0; }
    if (m.vsz > 128) return -EOPNOTSUPP;
    const uint64_t R = std::min<uint64_t>(m.ht.nslots - start, std::min<uint64_t>(1ull << 24, std::max<uint64_t>(1ull << 16, 4ull * max)));
    const uint32_t cap = (uint32_t)std::min<uint64_t>(max, R);
    auto grow = [](DevBuf &b, size_t want) -> int { return b.bytes >= want ? 0 : b.ensure(want); };
    int r;
    if ((r = grow(sel, R * 4)) || (r = grow(nsel, 8)) || (r = grow(dk, (size_t)cap * m.ksz)) || (r = grow(dv, (size_t)cap * m.vsz)))
        return r;
    gf_htab_desc d = m.hdesc();
    SlotFull pred{d.slots, start, d.slot_size, d.ksz};
    size_t tb = 0;
    (void)rocprim::select(nullptr, tb, rocprim::counting_iterator<uint32_t>(0u), (uint32_t *)sel.p, (uint32_t *)nsel.p,
                          (size_t)R, pred, (hipStream_t)0);
    if ((r = grow(tmp, tb + 256))) return r;
    tb = tmp.bytes;
    if (hip_ok(rocprim::select(tmp.p, tb, rocprim::counting_iterator<uint32_t>(0u), (uint32_t *)sel.p, (uint32_t *)nsel.p,
                               (size_t)R, pred, (hipStream_t)0), "dump select"))
        return -EIO;
    const uint32_t g2 = (uint32_t)std::min<uint64_t>((cap + BLOCK - 1) / BLOCK, 65535u);
    hipLaunchKernelGGL(k_dump_gather, dim3(g2 ? g2 : 1), dim3(BLOCK), 0, (hipStream_t)0, d, m.ht.codec, start,
                       (const uint32_t *)sel.p, (const uint32_t *)nsel.p, cap, (uint8_t *)dk.p, (uint8_t *)dv.p);
    if (hip_ok(hipGetLastError(), "k_dump_gather")) return -EIO;
    uint32_t ns = 0;
    if (hip_ok(hipMemcpy(&ns, nsel.p, 4, hipMemcpyDeviceToHost), "dump count")) return -EIO;
    const uint32_t got = std::min(ns, cap);
    m.xfer_d2h += 4 + (size_t)got * (m.ksz + m.vsz);
    if (got && (hip_ok(hipMemcpy(keys, dk.p, (size_t)got * m.ksz, hipMemcpyDeviceToHost), "dump keys") ||
                hip_ok(hipMemcpy(vals, dv.p, (size_t)got * m.vsz, hipMemcpyDeviceToHost), "dump vals")))
        return -EIO;
    if (ns > cap) {                                      // stopped inside the range: resume after the last one
        uint32_t last = 0;
        if (hip_ok(hipMemcpy(&last, (const uint32_t *)sel.p + (cap - 1), 4, hipMemcpyDeviceToHost), "dump last")) return -EIO;
        *next = start + last + 1;
    } else {
        *next = start + R;
    }
    *n = got;
    return 0;
}
}  // namespace gf

// ---- endpoint egress (from-container) ----
namespace {
struct EgWs { DevBuf erec, rec2, key2, seq, ctlog, ctlog_n, snap, ckey, s6, d6,
             hzk, hzfl, hztk, hztf, hzak, hzaf, hzst, vip4, vip6, keysP, key2P, rlog, rlog_n, v6blk,
             rsslot, rslist;
             uint32_t hz_gen = 0, hz_cap = 0;
             uint32_t *h_hz = nullptr;          // pinned: the ordering check's words, read back without a stream sync
             hipEvent_t ev_hz = nullptr;
             std::vector<std::pair<const Map *, uint64_t>> vip_stamp;
             uint32_t vip4_mask = 0, vip6_mask = 0; bool vip4_any = false, vip6_any = false; };
EgWs &eg_ws() { static const char tag = 0; return cur_ctx().get<EgWs>(&tag); }
}  // namespace

static int egress_ordered(const std::shared_ptr<PolicyArray> &a, const gf_lxc_batch *b, uint32_t now_sec,
                          gf_egress_out *out, uint8_t *snap_out, hipStream_t s, bool lru, uint32_t first, uint32_t depth);
static int egress_runs(const std::shared_ptr<PolicyArray> &a, const gf_lxc_batch *b, uint32_t now_sec,
                       gf_egress_out *out, uint8_t *snap_out, hipStream_t s, bool lru, const std::vector<uint32_t> &cut);
static int egress_each(const std::shared_ptr<PolicyArray> &a, const gf_lxc_batch *b, uint32_t now_sec,
                       gf_egress_out *out, uint8_t *snap_out, hipStream_t s, bool lru) {
    std::vector<uint32_t> cut(b->frames.n + 1);
    for (uint32_t j = 0; j <= b->frames.n; j++) cut[j] = j;
    return egress_runs(a, b, now_sec, out, snap_out, s, lru, cut);
}
// The rev-NAT addresses of the programs' revNAT maps as device sets (the ordering
// check's GF_HZ_VIP), rebuilt when a map changed through the API.
static int vip_sets(const std::vector<std::shared_ptr<ProgLxc>> &progs, EgWs &ew, hipStream_t s) {
    std::vector<std::pair<const Map *, uint64_t>> stamp;
    std::vector<Map *> m4, m6;
    for (auto &p : progs) {
        if (p->revnat4 && std::find(m4.begin(), m4.end(), p->revnat4.get()) == m4.end()) m4.push_back(p->revnat4.get());
        if (p->revnat6 && std::find(m6.begin(), m6.end(), p->revnat6.get()) == m6.end()) m6.push_back(p->revnat6.get());
    }
    for (Map *m : m4) stamp.push_back({m, m->host_gen * 2});
    for (Map *m : m6) stamp.push_back({m, m->host_gen * 2 + 1});
    if (stamp == ew.vip_stamp) return 0;                // (no maps and nothing built compare equal too)
    std::vector<uint32_t> a4;
    std::vector<std::array<uint32_t, 4>> a6;
    std::vector<uint8_t> v(32);
    for (int fam = 4; fam <= 6; fam += 2) {
        for (Map *m : fam == 4 ? m4 : m6) {
            std::lock_guard<std::recursive_mutex> g(m->mu);
            int r = m->pull();
            if (r) return r;
            for (uint64_t i = 0; i < m->ht.nslots; i++) {
                if (m->ht.state(i) != GF_SLOT_FULL) continue;
                m->ht.get_val(i, v.data());
                if (fam == 4) { uint32_t x; memcpy(&x, v.data(), 4); if (x) a4.push_back(x); }
                else { std::array<uint32_t, 4> x; memcpy(x.data(), v.data(), 16); if (x[0] | x[1] | x[2] | x[3]) a6.push_back(x); }
            }
        }
    }
    auto build = [&](size_t cnt, uint32_t &mask) { mask = 15; while ((uint64_t)mask + 1 < 4ull * cnt) mask = mask * 2 + 1; };
    ew.vip4_any = !a4.empty(); ew.vip6_any = !a6.empty();
    if (ew.vip4_any) {
        build(a4.size(), ew.vip4_mask);
        std::vector<uint32_t> t(ew.vip4_mask + 1, 0);
        for (uint32_t x : a4) {
            uint32_t slot = vip_slot(x) & ew.vip4_mask;
            while (t[slot] && t[slot] != x) slot = (slot + 1u) & ew.vip4_mask;
            t[slot] = x;
        }
        if (ew.vip4.ensure(t.size() * 4) ||
            hip_ok(hipMemcpyAsync(ew.vip4.p, t.data(), t.size() * 4, hipMemcpyHostToDevice, s), "vip4") ||
            hip_ok(hipStreamSynchronize(s), "vip4 sync"))
            return -EIO;
    }
    if (ew.vip6_any) {
        build(a6.size(), ew.vip6_mask);
        std::vector<std::array<uint32_t, 4>> t(ew.vip6_mask + 1, std::array<uint32_t, 4>{0, 0, 0, 0});
        for (auto &x : a6) {
            uint32_t slot = vip_slot(x[0] ^ vip_slot(x[1] ^ vip_slot(x[2] ^ vip_slot(x[3])))) & ew.vip6_mask;
            while ((t[slot][0] | t[slot][1] | t[slot][2] | t[slot][3]) && t[slot] != x) slot = (slot + 1u) & ew.vip6_mask;
            t[slot] = x;
        }
        if (ew.vip6.ensure(t.size() * 16) ||
            hip_ok(hipMemcpyAsync(ew.vip6.p, t.data(), t.size() * 16, hipMemcpyHostToDevice, s), "vip6") ||
            hip_ok(hipStreamSynchronize(s), "vip6 sync"))
            return -EIO;
    }
    ew.vip_stamp = stamp;
    return 0;
}
// The per-call words of egress_call in one launch instead of four fills: the
// sequence words (seq[1] the ordering check's flag, seq[3] its first hazard,
// ~0 = none), both log counts and the front's scratch counter block.
__global__ __launch_bounds__(256) void k_eg_init(uint32_t *seq, uint32_t *ctlog_n, uint32_t *rlog_n,
                                                 unsigned long long *hzst) {
    const uint32_t t = threadIdx.x;
    if (t < 3) seq[t] = 0u;
    if (t == 3) seq[3] = ~0u;
    if (t < 2) ctlog_n[t] = 0u;
    if (t < 2 && rlog_n) rlog_n[t] = 0u;
    if (hzst)
        for (uint32_t k = t; k < 272; k += 256) hzst[k] = 0ull;
}
// A log of deferred CT4 writes {order, key[4], value[12], pad[3]} applied in
// order (k_ctlog_max / k_ctlog_apply: the last writer of a key wins).
// nlog: an upper bound of the entry count (*d_n, read by the kernels): no host
// round trip for the count.
// cfgs (per-endpoint CT maps): each entry into its program's own map instead of ct.
static int ctlog_apply(EgWs &ew, const uint32_t *lg, const uint32_t *d_n, uint32_t nlog, const gf_htab_desc &ct,
                       uint32_t *ct_count, hipStream_t s, const gf_lxc_dev *cfgs = nullptr) {
    if (!nlog) return 0;
    uint32_t cap = 1023;                               // the set for the bound, at <= 1/2 load
    while ((uint64_t)cap + 1 < 2ull * nlog) cap = cap * 2 + 1;
    const size_t tb = (size_t)(cap + 1) * 8;
    if (ew.ckey.bytes < tb) {                           // a new set: zero once (k_ctlog_apply keeps it zero)
        if (ew.ckey.ensure(tb)) return -ENOMEM;
        if (hip_ok(hipMemsetAsync(ew.ckey.p, 0, tb, s), "ct log set")) return -EIO;
    }
    ProfScope ps("k_ctlog_apply", s);
    const uint32_t gs = std::min<uint32_t>((cap + BLOCK) / BLOCK, 2048u);   // grid-stride over the set
    const uint32_t gl = (nlog + BLOCK - 1) / BLOCK;
    if (cfgs) {
        hipLaunchKernelGGL(k_ctlog_max<true>, dim3(gl), dim3(BLOCK), 0, s, lg, d_n, (unsigned long long *)ew.ckey.p, cap);
        hipLaunchKernelGGL(k_ctlog_apply<true>, dim3(gs), dim3(BLOCK), 0, s, lg, d_n, (unsigned long long *)ew.ckey.p, cap,
                           gf_htab_desc{}, nullptr, cfgs);
    } else {
        hipLaunchKernelGGL(k_ctlog_max<false>, dim3(gl), dim3(BLOCK), 0, s, lg, d_n, (unsigned long long *)ew.ckey.p, cap);
        hipLaunchKernelGGL(k_ctlog_apply<false>, dim3(gs), dim3(BLOCK), 0, s, lg, d_n, (unsigned long long *)ew.ckey.p,
                           cap, ct, ct_count, nullptr);
    }
    return hip_ok(hipGetLastError(), "k_ctlog_apply");
}
// One ordered run of an egress batch: check = run the ordering check first (a
// flagged batch is split into runs, each through this function again); lru = the
// LRU stand-in after it (once per classify call).
static int egress_call(const std::shared_ptr<PolicyArray> &a, const gf_lxc_batch *b, uint32_t now_sec,
                       gf_egress_out *out, uint8_t *snap_out, hipStream_t s, bool check, bool lru, uint32_t depth = 0) {
    const gf_frames &fr = b->frames;
    const uint32_t n = fr.n, S = fr.snap_stride;
    if (n == 0) return 0;
    check = check && n > 1;
    int r;
    std::vector<std::shared_ptr<ProgLxc>> progs;
    if ((r = prog_table(a, s, progs))) return r;
    CtMaps cm;
    if ((r = ct_maps_of(progs, cm))) return r;
    const bool pct = cm.pct;                           // per-endpoint CT maps (ConntrackLocal)
    std::shared_ptr<Map> ct4m = pct ? nullptr : cm.one(4), ct6m = pct ? nullptr : cm.one(6);
    uint32_t strict = 0;
    gf_htab_desc cfg_ct4{}, cfg_ct6{};
    if ((r = ct_limits(ct4m, ct6m, n, 3, s, strict, cfg_ct4, cfg_ct6))) return r;
    if (pct) {                                          // a family's bit: one of its maps could fill
        gf_htab_desc d4{}, d6{};
        for (auto &m : cm.m4) {
            uint32_t st = 0;
            if ((r = ct_limits(m, nullptr, n, 3, s, st, d4, d6))) return r;
            strict |= st;
        }
        for (auto &m : cm.m6) {
            uint32_t st = 0;
            if ((r = ct_limits(nullptr, m, n, 3, s, st, d4, d6))) return r;
            strict |= st;
        }
    }
    auto lxc = node_map(1), tun = node_map(2);
    if ((r = push_map(lxc, s)) || (r = push_map(tun, s))) return r;
    EgWs &ew = eg_ws();
    auto grow = [](DevBuf &d, size_t want) -> int { return d.bytes >= want ? 0 : d.ensure(want); };
    uint32_t hmask = 1023, amask = 1023;                 // conn keys at <= 1/2 load, up to 4 aux keys at <= 1/2
    while (check && (uint64_t)hmask + 1 < 2ull * n) hmask = hmask * 2 + 1;
    while (check && (uint64_t)amask + 1 < 8ull * n) amask = amask * 2 + 1;
    if ((r = grow(ew.erec, (size_t)n * sizeof(EgRec))) || (r = grow(ew.rec2, (size_t)n * sizeof(gf_rec))) ||
        (r = grow(ew.key2, (size_t)n * 4)) || (r = grow(ew.seq, 16)) || (r = grow(ew.ctlog_n, 8)) ||
        (r = grow(ew.ctlog, (size_t)n * GF_CTLOG_WORDS * 4)) || (r = grow(ew.s6, (size_t)n * 32)) || (r = grow(ew.hzst, 272 * 8)) || (r = ws_grow(n)))
        return r;
    if (check && ((r = grow(ew.hzk, (size_t)n * 8 * GF_HZ_NK)) || (r = grow(ew.hzfl, (size_t)n)) ||
                  (r = grow(ew.hztk, (size_t)(hmask + 1) * 8)) || (r = grow(ew.hztf, (size_t)(hmask + 1) * 16)) ||
                  (r = grow(ew.hzak, (size_t)(amask + 1) * 8)) || (r = grow(ew.hzaf, (size_t)(amask + 1) * 8))))
        return r;
    // In place (snap_out == the frames) with the check: the flagged pass must leave
    // the frames as they came, so the rewrites go to scratch and are copied at the end
    // (also when tracing: TRACE_FROM_LXC captures the frames as sent).
    PassArgs ta{};
    ta.kind = 2;
    ta.on = event_ring().records && array_traces(a);
    ta.orig = fr.snap; ta.lxc_id = b->lxc_id;
    if (ta.on && (r = trace_prepare(n, false, s))) return r;
    const bool inplace = (check || ta.on) && snap_out == fr.snap;
    uint8_t *wsnap = inplace ? nullptr : snap_out;
    if (!wsnap) {
        if ((r = grow(ew.snap, (size_t)n * S))) return r;
        wsnap = (uint8_t *)ew.snap.p;
    }
    const gf_node_cfg &node = node_cfg();
    EgDev E{};
    E.cfgs = (const gf_lxc_dev *)a->d_cfgs.p;
    E.slot_of = (const uint16_t *)a->d_slot_of_lxc.p;
    E.ct4 = cfg_ct4; E.ct6 = cfg_ct6;
    if ((r = grow(ew.v6blk, (n + BLOCK - 1) / BLOCK))) return r;
    E.v6blk = GF_EG_LEAN ? (uint8_t *)ew.v6blk.p : nullptr;
    E.s6out = (uint8_t *)ew.s6.p; E.d6out = (uint8_t *)ew.s6.p + 16;   // interleaved (IngCtx::a6_stride 32)
    memcpy(E.router6, node.router_ip6, 16); memcpy(E.host6, node.host_ip6, 16);
    if (lxc) {
        E.lxc = lxc->hdesc();
        if (getenv("GF_XDP_NOSETS") || lxc->addr_set(20, 8192, s, &E.lxset, &E.lxbits, &E.lxzero)) E.lxset = nullptr;
    }
    if (tun) {
        E.tunnel = tun->hdesc();
        if (getenv("GF_XDP_NOSETS") || tun->addr_set(20, 8192, s, &E.tnset, &E.tnbits, &E.tnzero)) E.tnset = nullptr;
    }
    E.snap = wsnap; E.stride = S; E.now = now_sec; E.host_ifindex = host_ifindex();
    E.encap_ifindex = node.encap_ifindex;
    E.cluster_range = node.ipv4_cluster_range; E.cluster_mask = node.ipv4_cluster_mask;
    E.loopback = node.ipv4_loopback; E.ipv4_mask = node.ipv4_mask;
    memcpy(E.host_mac, node.host_mac, 6);
    E.strict = strict;
    E.seq = (uint32_t *)ew.seq.p;
    E.ctlog = (uint32_t *)ew.ctlog.p; E.ctlog_n = (uint32_t *)ew.ctlog_n.p;
    E.rec2 = (gf_rec *)ew.rec2.p; E.key2 = (uint32_t *)ew.key2.p;
    // Connection groups for IPv4 (EgDev::conn): off when CT4 inserts are counted
    // exactly (strict: the batch runs as one bucket anyway).
    static const bool no_conn = getenv("GF_EG_PAIRS") != nullptr;   // diagnosis: address-pair groups only
    const bool conn = ct4m && !(strict & 1u) && !no_conn;
    uint32_t *d_rn = nullptr;                          // [0] related entries logged, [1] pair-group fallback
    if (conn) {
        // the related entries' set (GF_EG_RSET): 4n slots keep it at most half full (<= 2n
        // writes, one per new connection in each pass); batches too large for 32-bit slot
        // numbers keep the write log
        uint64_t ns = 1024;
        while (ns < 4ull * n) ns *= 2;
        const bool rset = GF_EG_RSET && ns <= (1ull << 31);
        if ((r = grow(ew.keysP, (size_t)n * 4)) || (r = grow(ew.key2P, (size_t)n * 4)) || (r = grow(ew.rlog_n, 8)) ||
            (!rset && (r = grow(ew.rlog, (size_t)2 * n * GF_CTLOG_WORDS * 4))))
            return r;
        d_rn = (uint32_t *)ew.rlog_n.p;
        E.conn = 1; E.cflag = d_rn + 1;
        E.keysP = (uint32_t *)ew.keysP.p; E.key2P = (uint32_t *)ew.key2P.p;
        E.rlog = (uint32_t *)ew.rlog.p; E.rlog_n = d_rn;
        if (rset) {
            // zeroed when allocated, and left zero by k_rset_apply, which clears every
            // slot a run claimed
            const size_t sb = (size_t)(ns + 1) * 16;
            if (ew.rsslot.bytes < sb) {
                if (ew.rsslot.ensure(sb)) return -ENOMEM;
                if (hip_ok(hipMemsetAsync(ew.rsslot.p, 0, sb, s), "related set")) return -EIO;
            }
            if ((r = grow(ew.rslist, (size_t)2 * n * 4 + 4))) return r;
            E.rs.slot = (unsigned long long *)ew.rsslot.p;
            E.rs.list = (uint32_t *)ew.rslist.p; E.rs.list_n = d_rn; E.rs.mask = (uint32_t)(ns - 1);
            E.rlog = E.rs.list;                          // (marks the set in use for the deliveries' pass)
        }
    }
    uint32_t *d_hz = (uint32_t *)ew.seq.p + 1;           // word 1 of the seq buffer: the hazard flag
    if (check) {
        E.hz_k = (uint64_t *)ew.hzk.p; E.hz_fl = (uint8_t *)ew.hzfl.p; E.hz = d_hz;
        if ((r = vip_sets(progs, ew, s))) return r;
        if (ew.vip4_any) { E.vip4 = (const uint32_t *)ew.vip4.p; E.vip4_mask = ew.vip4_mask; }
        if (ew.vip6_any) { E.vip6 = (const uint4 *)ew.vip6.p; E.vip6_mask = ew.vip6_mask; }
    }
    E.X.snap = nullptr; E.X.snap_stride = S; E.X.now = now_sec; E.X.gw = node.ipv4_gateway;   // writes: k_eg_groups
    memcpy(E.X.host6, node.host_ip6, 16);
    if (ta.on) { E.X.tmark = (uint8_t *)trace_ws().mark.p; E.X.tcap = (uint8_t *)trace_ws().px.p; }
    if ((r = px_log_begin(n, s, E.X))) return r;
    unsigned long long *sink = (unsigned long long *)stats_sink();
    // With the check, the front counts into a scratch block folded into the sink
    // only when the batch runs as it is (a flagged batch's runs count themselves).
    unsigned long long *fsink = sink;
    if (check && sink) fsink = (unsigned long long *)ew.hzst.p;
    hipLaunchKernelGGL(k_eg_init, dim3(1), dim3(256), 0, s, (uint32_t *)ew.seq.p, (uint32_t *)ew.ctlog_n.p, d_rn,
                       fsink != sink ? fsink : nullptr);
    Workspace &w = ws();
    {
        ProfScope ps("k_eg_front", s);
        // the IPv4 kernel's LDS rows: one per lane, the staged header bytes (<= GF_EG_STAGE)
        const uint32_t eg_lds = GF_EG_DYN ? BLOCK * std::min<uint32_t>(S, GF_EG_STAGE) : BLOCK * GF_EG_STAGE;
        hipLaunchKernelGGL(k_eg_front<4>, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), eg_lds, s, fr, b->lxc_id, b->flow_hash,
                           E, (EgRec *)ew.erec.p, (uint32_t *)w.keys.p, out, fsink);
        hipLaunchKernelGGL(k_eg_front<6>, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 16, s, fr, b->lxc_id, b->flow_hash,
                           E, (EgRec *)ew.erec.p, (uint32_t *)w.keys.p, out, fsink);
        hipLaunchKernelGGL(k_eg_seq_keys, dim3(grid_for(n)), dim3(BLOCK), 0, s, (const uint32_t *)ew.seq.p,
                           (const uint32_t *)E.cflag, (const uint32_t *)E.keysP, n, (uint32_t *)w.keys.p);
        if ((r = hip_ok(hipGetLastError(), "k_eg_front"))) return r;
    }
    if (check) {
        ProfScope ps("k_hz_check", s);
        if (ew.hz_cap != hmask + 1 || ew.hz_gen >= 0xffffu) {   // new table or wrapped generation
            if (hip_ok(hipMemsetAsync(ew.hztk.p, 0, (size_t)(hmask + 1) * 8, s), "hz keys") ||
                hip_ok(hipMemsetAsync(ew.hztf.p, 0, (size_t)(hmask + 1) * 16, s), "hz first"))
                return -EIO;
            ew.hz_cap = hmask + 1; ew.hz_gen = 0;
        }
        const HzGen C{(unsigned long long *)ew.hztk.p, (unsigned long long *)ew.hztf.p, hmask, ++ew.hz_gen};
        const HzTab A{(unsigned long long *)ew.hzak.p, (uint32_t *)ew.hzaf.p, amask};
        hipLaunchKernelGGL(k_hz_clear, dim3(std::min<uint32_t>((amask + 1) / BLOCK, 8192)), dim3(BLOCK), 0, s, A,
                           (const uint32_t *)d_hz);
        hipLaunchKernelGGL(k_hz_insert, dim3(grid_for(n)), dim3(BLOCK), 0, s, (const uint64_t *)ew.hzk.p,
                           (const uint8_t *)ew.hzfl.p, n, (const uint32_t *)d_hz, C, A);
        hipLaunchKernelGGL(k_hz_probe, dim3(grid_for(n)), dim3(BLOCK), 0, s, (const uint64_t *)ew.hzk.p,
                           (const uint8_t *)ew.hzfl.p, n, C, A, strict, d_hz);
        if ((r = hip_ok(hipGetLastError(), "k_hz_check"))) return r;
        // the check's verdict goes to pinned host memory behind an event: the host
        // reads it while the device already builds the schedule (no stream sync)
        if (!ew.h_hz && (hip_ok(hipHostMalloc((void **)&ew.h_hz, 16, hipHostMallocDefault), "hz host") ||
                         hip_ok(hipEventCreateWithFlags(&ew.ev_hz, hipEventDisableTiming), "hz event")))
            return -EIO;
        if (hip_ok(hipMemcpyAsync(ew.h_hz, d_hz, 12, hipMemcpyDeviceToHost, s), "hz flag") ||
            hip_ok(hipEventRecord(ew.ev_hz, s), "hz record"))
            return -EIO;
    }
    if ((r = schedule_groups(n, s, nullptr, true))) return r;   // (reads only the front's keys: harmless on a flagged batch)
    host_mark("front+sched");
    // k_eg_groups is queued before the host looks at the ordering check: it reads the
    // check's flag itself and idles on a flagged batch (no map state changes then), so
    // the device has the schedule and the groups to run while the host waits for the
    // check's verdict and enqueues the rest of the call behind them
    {
        uint32_t grid = resident_blocks(8), need = (n + BLOCK - 1) / BLOCK;
        if (grid > need) grid = need;
        ProfScope ps("k_eg_groups", s);
        if (pct) {
            hipLaunchKernelGGL((k_eg_groups<4, true>), dim3(grid), dim3(BLOCK), BLOCK * eg_row_bytes(S), s, E,
                               (uint32_t *)w.sched.p, (const uint2 *)w.order.p, (const uint32_t *)w.perm.p,
                               (const EgRec *)ew.erec.p, out, (gf_rec *)ew.rec2.p, (uint32_t *)ew.key2.p, nullptr, sink);
            hipLaunchKernelGGL((k_eg_groups<6, true>), dim3(grid), dim3(BLOCK), 16, s, E, (uint32_t *)w.sched.p,
                               (const uint2 *)w.order.p, (const uint32_t *)w.perm.p, (const EgRec *)ew.erec.p, out,
                               (gf_rec *)ew.rec2.p, (uint32_t *)ew.key2.p, nullptr, sink);
        } else {
            hipLaunchKernelGGL(k_eg_groups<4>, dim3(grid), dim3(BLOCK), BLOCK * eg_row_bytes(S), s, E,
                               (uint32_t *)w.sched.p, (const uint2 *)w.order.p, (const uint32_t *)w.perm.p,
                               (const EgRec *)ew.erec.p, out, (gf_rec *)ew.rec2.p, (uint32_t *)ew.key2.p,
                               ct4m ? (uint32_t *)ct4m->d_count.p : nullptr, sink);
            hipLaunchKernelGGL(k_eg_groups<6>, dim3(grid), dim3(BLOCK), 16, s, E, (uint32_t *)w.sched.p,
                               (const uint2 *)w.order.p, (const uint32_t *)w.perm.p, (const EgRec *)ew.erec.p, out,
                               (gf_rec *)ew.rec2.p, (uint32_t *)ew.key2.p, ct6m ? (uint32_t *)ct6m->d_count.p : nullptr,
                               sink);
        }
        if ((r = hip_ok(hipGetLastError(), "k_eg_groups"))) return r;
    }
    uint32_t hz = 0, hz_first = 0;
    if (check) {
        if (hip_ok(hipEventSynchronize(ew.ev_hz), "hz sync")) return -EIO;
        host_mark("hzwait");
        hz = ew.h_hz[0]; hz_first = ew.h_hz[2];
    }
    if (hz & 2u) {
        if (getenv("GF_HZ_DEBUG")) fprintf(stderr, "[gf] egress n=%u: a CT map could fill, one packet at a time\n", n);
        return egress_each(a, b, now_sec, out, snap_out, s, lru);
    }
    if (hz) return egress_ordered(a, b, now_sec, out, snap_out, s, lru, hz_first, depth);
    // ct_create4's deferred service entries, in batch order; every count from here
    // on is read on the device (no host round trip inside the call)
    if (check && sink) {
        hipLaunchKernelGGL(k_stats_fold, dim3(1), dim3(256), 0, s, (const unsigned long long *)fsink, sink);
        if ((r = hip_ok(hipGetLastError(), "k_stats_fold"))) return r;
    }
    if (ct4m && (r = ctlog_apply(ew, (const uint32_t *)ew.ctlog.p, (const uint32_t *)ew.ctlog_n.p, n, cfg_ct4,
                                 (uint32_t *)ct4m->d_count.p, s)))
        return r;
    if (pct && !cm.m4.empty() &&
        (r = ctlog_apply(ew, (const uint32_t *)ew.ctlog.p, (const uint32_t *)ew.ctlog_n.p, n, gf_htab_desc{}, nullptr, s,
                         (const gf_lxc_dev *)a->d_cfgs.p)))
        return r;
    for (auto *v : {&cm.m4, &cm.m6})
        for (auto &m : *v) m->device_modified();
    // The egress redirects' cilium_proxy{4,6} updates stay in the log: the
    // deliveries' handle_policy appends theirs and the whole log is applied in
    // packet order after it (nothing on these paths reads the proxy maps).
    // handle_policy of the local deliveries (the tail calls of ipv4_local_delivery)
    gf_pkt_cols c2{};
    c2.n = n;
    c2.len = fr.len;
    c2.flow_hash = b->flow_hash;
    c2.saddr6 = (const uint8_t *)ew.s6.p; c2.daddr6 = (const uint8_t *)ew.s6.p + 16;   // IPv6 deliveries (if any)
    // the deliveries' keys: their connections, or address pairs when the run fell back
    // k_eg_groups wrote them in batch order: they become the workspace's records and
    // keys by exchanging the buffers (the workspace's old ones are the next call's
    // pass-2 buffers), not by copying n records; a fallen-back run takes the pair
    // keys on the device (k_eg_seq_keys' rule, *cflag)
    auto pack = [&](const uint16_t *, gf_rec *, uint32_t *) -> int {
        Workspace &w = ws();
        std::swap(w.rec.p, ew.rec2.p); std::swap(w.rec.bytes, ew.rec2.bytes);
        std::swap(w.keys.p, ew.key2.p); std::swap(w.keys.bytes, ew.key2.bytes);
        if (conn) {
            hipLaunchKernelGGL(k_eg_pick_keys, dim3(grid_for(n)), dim3(BLOCK), 0, s, (const uint32_t *)E.cflag,
                               (const uint32_t *)ew.key2P.p, n, (uint32_t *)w.keys.p);
            return hip_ok(hipGetLastError(), "k_eg_pick_keys");
        }
        return 0;
    };
    if (conn) { ta.rlog = E.rlog; ta.rlog_n = d_rn; ta.rlog_off = E.cflag; ta.rs = E.rs; }
    if ((r = ingress_run(a, &c2, now_sec, nullptr, s, pack, (uint8_t *)out, fr.len, wsnap, S, wsnap, lru && !conn, true,
                         false, &ta)))
        return r;
    if (conn && E.rs.slot) {                           // both passes' related entries: each key's last writer
        ProfScope ps("k_ctlog_apply", s);
        // the deliveries' records are the workspace's now (the pack swap above)
        hipLaunchKernelGGL(k_rset_apply, dim3(std::min<uint32_t>(grid_for(2 * n), 2048u)), dim3(BLOCK), 0, s, E.rs,
                           (const EgRec *)ew.erec.p, (const gf_rec *)ws().rec.p, E.cfgs, cfg_ct4,
                           (uint32_t *)ct4m->d_count.p, now_sec);
        if ((r = hip_ok(hipGetLastError(), "k_rset_apply"))) return r;
    } else if (conn) {                                 // both passes' related entries, in packet order
        if ((r = ctlog_apply(ew, (const uint32_t *)ew.rlog.p, d_rn, 2 * n, cfg_ct4, (uint32_t *)ct4m->d_count.p, s)))
            return r;
    }
    if (conn) {
        ct4m->device_modified();
        if (lru && ((r = lru_evict(ct4m, now_sec, s)) || (r = lru_evict(ct6m, now_sec, s)))) return r;
    }
    static const bool logstats = getenv("GF_EG_LOGSTATS") != nullptr;   // diagnostics: syncs the stream
    if (logstats) {
        uint32_t c[2] = {0, 0}, rc[2] = {0, 0};
        if (!hip_ok(hipStreamSynchronize(s), "logstats") &&
            !hip_ok(hipMemcpy(c, ew.ctlog_n.p, 8, hipMemcpyDeviceToHost), "logstats") &&
            (!conn || !hip_ok(hipMemcpy(rc, d_rn, 8, hipMemcpyDeviceToHost), "logstats")))
            fprintf(stderr, "[gf] egress n=%u: service-entry log %u, related-entry log %u (fallback %u)\n", n, c[0], rc[0],
                    rc[1]);
    }
    if (inplace && hip_ok(hipMemcpyAsync(snap_out, wsnap, (size_t)n * S, hipMemcpyDeviceToDevice, s), "snap copy"))
        return -EIO;
    return 0;
}

// A flagged batch: the cut points (a new run starts at a packet whose reverse
// direction is in the current run, and around every single-bucket tuple), then
// every run through egress_call in order.  Nothing of the flagged pass changed
// the maps: k_eg_groups idled, and the front only reads them.
static int egress_greedy(const std::shared_ptr<PolicyArray> &a, const gf_lxc_batch *b, uint32_t now_sec,
                         gf_egress_out *out, uint8_t *snap_out, hipStream_t s, bool lru);
static int egress_ordered(const std::shared_ptr<PolicyArray> &a, const gf_lxc_batch *b, uint32_t now_sec,
                          gf_egress_out *out, uint8_t *snap_out, hipStream_t s, bool lru, uint32_t first, uint32_t depth) {
    const uint32_t n = b->frames.n;
    if (getenv("GF_HZ_DEBUG")) fprintf(stderr, "[gf] egress n=%u: ordering hazard at %u (run %u)\n", n, first, depth + 1);
    if (first == 0 || first >= n || depth >= 32) return egress_greedy(a, b, now_sec, out, snap_out, s, lru);
    // [0, first) has no hazard; the rest runs after it, checked again
    std::vector<uint32_t> cut{0, first};
    int r = egress_runs(a, b, now_sec, out, snap_out, s, false, cut);
    if (r) return r;
    const uint32_t S = b->frames.snap_stride;
    gf_lxc_batch rest = *b;
    rest.frames.n = n - first;
    rest.frames.snap = b->frames.snap + (size_t)first * S;
    rest.frames.len = b->frames.len + first;
    if (b->lxc_id) rest.lxc_id = b->lxc_id + first;
    if (b->flow_hash) rest.flow_hash = b->flow_hash + first;
    return egress_call(a, &rest, now_sec, out + first, snap_out ? snap_out + (size_t)first * S : nullptr, s, true, lru,
                       depth + 1);
}
// Many runs: the cut points on the host, in one pass over the batch's keys.
static int egress_greedy(const std::shared_ptr<PolicyArray> &a, const gf_lxc_batch *b, uint32_t now_sec,
                         gf_egress_out *out, uint8_t *snap_out, hipStream_t s, bool lru) {
    EgWs &ew = eg_ws();
    const uint32_t n = b->frames.n;
    std::vector<uint64_t> K((size_t)n * GF_HZ_NK);
    std::vector<uint8_t> fl(n);
    if (hip_ok(hipMemcpyAsync(K.data(), ew.hzk.p, K.size() * 8, hipMemcpyDeviceToHost, s), "hz keys") ||
        hip_ok(hipMemcpyAsync(fl.data(), ew.hzfl.p, n, hipMemcpyDeviceToHost, s), "hz fl") ||
        hip_ok(hipStreamSynchronize(s), "hz sync"))
        return -EIO;
    // the rules of k_hz_insert / k_hz_probe over the current run (keys are odd:
    // bit 0 carries a connection key's direction)
    std::vector<uint32_t> cut{0};
    std::unordered_set<uint64_t> seen;
    const uint64_t D = 1ull;
    uint32_t why[5] = {0, 0, 0, 0, 0};
    auto k = [&](uint32_t which, uint32_t j) { return K[(size_t)which * n + j] & ~D; };
    for (uint32_t j = 0; j < n; j++) {
        const uint32_t f = fl[j];
        if (!(f & GF_HZ_VALID)) continue;
        const bool h0 = seen.count(k(1, j) | ((f & GF_HZ_DIRE) ? 0ull : D)) != 0;
        const bool h1 = (f & GF_HZ_ICMP) && seen.count(k(3, j) ^ 2ull) != 0;
        const bool h2 = seen.count((k(3, j) ^ GF_HZ_ICMPSALT) & ~D) != 0;
        const bool h3 = (f & GF_HZ_LOOP) && (seen.count(k(0, j)) || seen.count(k(0, j) | D));
        const bool h4 = (f & GF_HZ_VIP) && seen.count(k(4, j) ^ 2ull) != 0;
        why[0] += h0; why[1] += h1; why[2] += h2; why[3] += h3; why[4] += h4;
        if (h0 || h1 || h2 || h3 || h4) { cut.push_back(j); seen.clear(); }
        if (f & GF_HZ_DLV) seen.insert(k(0, j) | ((f & GF_HZ_DIRI) ? D : 0ull));
        seen.insert(k(2, j) ^ 2ull);
        if (f & GF_HZ_ICMP) seen.insert((k(2, j) ^ GF_HZ_ICMPSALT) & ~D);
        seen.insert(k(4, j) ^ 2ull);
        seen.insert(k(5, j) ^ 2ull);
    }
    if (cut.back() != n) cut.push_back(n);
    if (getenv("GF_HZ_DEBUG"))
        fprintf(stderr, "[gf] egress n=%u: %zu ordered runs (reply %u, icmp-after %u, after-icmp %u, loopback %u, vip %u)\n",
                n, cut.size() - 1, why[0], why[1], why[2], why[3], why[4]);
    return egress_runs(a, b, now_sec, out, snap_out, s, lru, cut);
}

// The runs [cut[k], cut[k+1]) of a batch through egress_call, in order; the LRU
// stand-in after the last.
static int egress_runs(const std::shared_ptr<PolicyArray> &a, const gf_lxc_batch *b, uint32_t now_sec,
                       gf_egress_out *out, uint8_t *snap_out, hipStream_t s, bool lru, const std::vector<uint32_t> &cut) {
    const uint32_t S = b->frames.snap_stride;
    for (size_t k = 0; k + 1 < cut.size(); k++) {
        const uint32_t lo = cut[k], hi = cut[k + 1];
        gf_lxc_batch sub = *b;
        sub.frames.n = hi - lo;
        sub.frames.snap = b->frames.snap + (size_t)lo * S;
        sub.frames.len = b->frames.len + lo;
        if (b->lxc_id) sub.lxc_id = b->lxc_id + lo;
        if (b->flow_hash) sub.flow_hash = b->flow_hash + lo;
        int r = egress_call(a, &sub, now_sec, out + lo, snap_out ? snap_out + (size_t)lo * S : nullptr, s, false,
                            lru && k + 2 == cut.size());
        if (r) return r;
    }
    return 0;
}

extern "C" int gf_lxc_egress_classify(int array, const gf_lxc_batch *b, uint32_t now_sec, gf_egress_out *out,
                                      uint8_t *snap_out, void *stream) {
    std::shared_lock<std::shared_mutex> g(prog_lock());
    auto o = get_obj(array);
    if (!o || o->kind != ObjKind::PolicyArray) return -EBADF;
    auto a = std::static_pointer_cast<PolicyArray>(o);
    if (!b) return -EFAULT;
    const gf_frames &fr = b->frames;
    if (fr.n == 0) return 0;
    if (!fr.snap || !fr.len || !out) return -EFAULT;
    if (fr.snap_stride < 34) return -EINVAL;           // an Ethernet + IPv4 header at least
    if (fr.n > (1u << 30)) return -E2BIG;
    hipStream_t s = (hipStream_t)stream;
    HostMarks hm;
    CtxScope cx(s);
    std::lock_guard<std::mutex> ag(a->mu);
    MapLocks L;
    lock_array_maps(L, a);
    L.lock();
    CallOrder co(s, L, a.get());
    host_mark("locks");
    static const bool nocheck = getenv("GF_EG_NOCHECK") != nullptr;     // diagnosis only: the unordered schedule
    static const bool dbg = getenv("GF_HZ_DEBUG") != nullptr;
    if (!dbg) return egress_call(a, b, now_sec, out, snap_out, s, !nocheck, true);
    (void)hipStreamSynchronize(s);
    auto t0 = std::chrono::steady_clock::now();
    int r = egress_call(a, b, now_sec, out, snap_out, s, !nocheck, true);
    (void)hipStreamSynchronize(s);
    fprintf(stderr, "[gf] egress n=%u: %.3f ms\n", fr.n,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    return r;
}
