/*
 * oracle.c — CPU restatement of the Cilium 1.0.0-rc9 verdict path.
 * TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline), see oracle.h.
 *
 * Byte layouts (little-endian host, as the BPF programs see them):
 *   struct ipv4_ct_tuple  14 B packed  bpf/lib/common.h:338-346
 *   struct ipv6_ct_tuple  40 B         bpf/lib/common.h:317-325
 *   struct ct_entry       48 B         bpf/lib/common.h:359-374
 *   struct policy_key      8 B         bpf/lib/common.h:184-190
 *   struct policy_entry   24 B         bpf/lib/common.h:192-197
 *   struct lb4_key/lb4_service/lb4_reverse_nat 8/12/6 B  common.h:395-412
 *   struct lb6_key/lb6_service/lb6_reverse_nat 20/24/18 B common.h:376-393
 *   struct endpoint_key   20 B packed  common.h:150-163
 *   struct endpoint_info 112 B         common.h:168-177
 *   struct lpm_v4_key / lpm_v6_key 8/20 B  bpf/lib/xdp.h:23-31
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include <pthread.h>
#include <sys/mman.h>

/* ------------------------------------------------------------------ */
/* kernel-side constants                                               */
/* ------------------------------------------------------------------ */
#define ETH_HLEN 14
#define IPPROTO_ICMP 1
#define IPPROTO_TCP 6
#define IPPROTO_UDP 17
#define IPPROTO_ICMPV6 58

#define TC_ACT_OK 0
#define TC_ACT_SHOT 2
#define TC_ACT_REDIRECT 7
#define XDP_DROP 1
#define XDP_PASS 2

#define DROP_POLICY -133
#define DROP_INVALID -134
#define DROP_CT_INVALID_HDR -135
#define DROP_CT_UNKNOWN_PROTO -137
#define DROP_UNKNOWN_L3 -139
#define DROP_MISSED_TAIL_CALL -140
#define DROP_WRITE_ERROR -141
#define DROP_UNKNOWN_L4 -142
#define DROP_CSUM_L3 -153
#define DROP_CSUM_L4 -154
#define DROP_CT_CREATE_FAILED -155
#define DROP_INVALID_EXTHDR -156
#define DROP_FRAG_NOSUPPORT -157
#define DROP_NO_SERVICE -158
#define DROP_POLICY_L4 -159
#define DROP_PROXYMAP_CREATE_FAILED -161

#define CT_EGRESS 0
#define CT_INGRESS 1
#define CT_NEW 0
#define CT_ESTABLISHED 1
#define CT_REPLY 2
#define CT_RELATED 3
#define TUPLE_F_OUT 0
#define TUPLE_F_IN 1
#define TUPLE_F_RELATED 2
#define ACTION_UNSPEC 0
#define ACTION_CREATE 1
#define ACTION_CLOSE 2
#define CT_DEFAULT_LIFETIME 43200
#define CT_SYN_TIMEOUT 300
#define CT_CLOSE_TIMEOUT 10

/* include/gpuflow.h flag values (kept in sync by tests) */
#define LB_F_L3 (1u << 0)
#define LB_F_L4 (1u << 1)
#define LB_F_REDIRECT (1u << 2)
#define LB_F_NO_IPV4 (1u << 3)
#define LB_F_NO_IPV6 (1u << 4)
#define LXC_F_DROP_ALL (1u << 0)
#define LXC_F_POLICY_INGRESS (1u << 1)
#define LXC_F_HAVE_L4_POLICY (1u << 2)
#define LXC_F_CT_ACCOUNTING (1u << 3)
#define LXC_F_LXC_IPV4 (1u << 4)

/* IS_ERR, bpf/lib/common.h:221 */
#define IS_ERR(x) (((x) < 0) || ((x) == TC_ACT_SHOT))

/* ------------------------------------------------------------------ */
/* maps: exact-match hash (kernel htab) and LPM trie                   */
/* ------------------------------------------------------------------ */
/* A shard's slots are records [state | key | pad | value | pad] (one cache line
 * for the CT shapes), so a probe step touches one line, not three arrays. */
typedef struct om_shard {
    uint8_t *rec;                   /* cap records of om_map.rs bytes; state: 0 empty, 1 full, 2 deleted */
    uint64_t cap, used, tomb;
    pthread_mutex_t mu;
} om_shard;

struct om_map {
    uint32_t type, ksz, vsz, max_entries, nshards;
    uint32_t koff, rs;              /* value offset in a record, record stride */
    uint32_t count;                 /* total elements (atomic across shards) */
    uint64_t lru_hand;              /* LRU CT maps: the eviction hand's next home line */
    uint8_t lens_present[129];      /* LPM: prefix lengths present (count) */
    uint32_t lens_cnt[129];
    om_shard *sh;
};

static uint64_t fnv1a(const uint8_t *p, uint32_t n) {
    uint64_t h = 1469598103934665603ull;
    for (uint32_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ull; }
    return h ^ (h >> 29);
}

static int is_lpm(const om_map *m) { return m->type == OM_LPM_TRIE; }
#define SH_ST(m, h, i) ((h)->rec[(uint64_t)(i) * (m)->rs])
#define SH_KEY(m, h, i) ((h)->rec + (uint64_t)(i) * (m)->rs + 1)
#define SH_VAL(m, h, i) ((h)->rec + (uint64_t)(i) * (m)->rs + (m)->koff)
/* zeroed record storage; large arrays are asked for transparent huge pages (the
 * bench's CT shards reach gigabytes: fewer TLB misses per probe) */
static uint8_t *sh_alloc(uint64_t bytes) {
    if (bytes < (4u << 20)) return (uint8_t *)calloc(1, bytes);
    void *p = NULL;
    const uint64_t al = 2u << 20, sz = (bytes + al - 1) / al * al;
    if (posix_memalign(&p, al, sz)) return NULL;
#ifdef MADV_HUGEPAGE
    madvise(p, sz, MADV_HUGEPAGE);
#endif
    memset(p, 0, sz);
    return (uint8_t *)p;
}
static uint32_t lpm_bits(const om_map *m) { return (m->ksz - 4) * 8; }

/* LPM keys are stored normalized: data bits beyond prefixlen cleared. */
static void lpm_normalize(const om_map *m, const uint8_t *key, uint8_t *out) {
    uint32_t plen; memcpy(&plen, key, 4);
    memcpy(out, key, m->ksz);
    uint32_t nbytes = m->ksz - 4;
    for (uint32_t i = 0; i < nbytes; i++) {
        int keep = (int)plen - (int)(i * 8);
        uint8_t mask = keep >= 8 ? 0xff : keep <= 0 ? 0 : (uint8_t)(0xff << (8 - keep));
        out[4 + i] &= mask;
    }
}

static uint32_t shard_of(const om_map *m, const uint8_t *key);

om_map *om_create(uint32_t type, uint32_t key_size, uint32_t value_size,
                  uint32_t max_entries, uint32_t shards) {
    if (!key_size || !value_size || !max_entries) return NULL;
    if (type == OM_LPM_TRIE && (key_size < 5 || key_size > 4 + 16)) return NULL;
    om_map *m = (om_map *)calloc(1, sizeof(*m));
    m->type = type; m->ksz = key_size; m->vsz = value_size; m->max_entries = max_entries;
    m->koff = (1 + key_size + 7) / 8 * 8;
    m->rs = m->koff + (value_size + 7) / 8 * 8;
    m->nshards = shards ? shards : 1;
    m->sh = (om_shard *)calloc(m->nshards, sizeof(om_shard));
    for (uint32_t s = 0; s < m->nshards; s++) {
        om_shard *h = &m->sh[s];
        h->cap = 64;
        h->rec = sh_alloc(h->cap * m->rs);
        pthread_mutex_init(&h->mu, NULL);
    }
    return m;
}

void om_destroy(om_map *m) {
    if (!m) return;
    for (uint32_t s = 0; s < m->nshards; s++) {
        free(m->sh[s].rec);
        pthread_mutex_destroy(&m->sh[s].mu);
    }
    free(m->sh); free(m);
}

static int64_t sh_find(const om_map *m, const om_shard *h, const uint8_t *key) {
    uint64_t mask = h->cap - 1, i = fnv1a(key, m->ksz) & mask;
    for (;;) {
        uint8_t st = SH_ST(m, h, i);
        if (st == 0) return -1;
        if (st == 1 && memcmp(SH_KEY(m, h, i), key, m->ksz) == 0) return (int64_t)i;
        i = (i + 1) & mask;
    }
}

static void sh_grow(const om_map *m, om_shard *h) {
    uint64_t ncap = h->cap;
    while ((h->used + 1) * 2 > ncap) ncap *= 2;
    uint8_t *old = h->rec; uint64_t ocap = h->cap;
    h->cap = ncap;
    h->rec = sh_alloc(ncap * m->rs);
    h->tomb = 0;
    for (uint64_t j = 0; j < ocap; j++) {
        const uint8_t *o = old + j * m->rs;
        if (o[0] != 1) continue;
        uint64_t i = fnv1a(o + 1, m->ksz) & (ncap - 1);
        while (SH_ST(m, h, i)) i = (i + 1) & (ncap - 1);
        memcpy(h->rec + i * m->rs, o, m->rs);
    }
    free(old);
}

/* Element lookup returning a pointer into the shard (NULL if absent). For
 * LPM maps: exact (normalized) match — used by update/delete. */
static uint8_t *om_ptr_exact(om_map *m, const uint8_t *key) {
    uint8_t nk[64];
    const uint8_t *k = key;
    if (is_lpm(m)) { lpm_normalize(m, key, nk); k = nk; }
    om_shard *h = &m->sh[shard_of(m, k)];
    int64_t i = sh_find(m, h, k);
    return i < 0 ? NULL : SH_VAL(m, h, i);
}

/* kernel trie_lookup_elem: longest stored prefix with len <= key.prefixlen
 * whose bits match the key data (kernel/bpf/lpm_trie.c). */
static uint8_t *om_lpm_lookup_ptr(om_map *m, const uint8_t *key) {
    uint32_t plen; memcpy(&plen, key, 4);
    uint32_t maxb = lpm_bits(m);
    if (plen > maxb) plen = maxb;
    uint8_t probe[64];
    for (int l = (int)plen; l >= 0; l--) {
        if (!m->lens_cnt[l]) continue;
        uint32_t ul = (uint32_t)l;
        memcpy(probe, key, m->ksz);
        memcpy(probe, &ul, 4);
        uint8_t *v = om_ptr_exact(m, probe);
        if (v) return v;
    }
    return NULL;
}

/* datapath map_lookup_elem() */
static uint8_t *om_lookup_ptr(om_map *m, const void *key) {
    if (!m) return NULL;
    if (is_lpm(m)) return om_lpm_lookup_ptr(m, (const uint8_t *)key);
    om_shard *h = &m->sh[shard_of(m, (const uint8_t *)key)];
    int64_t i = sh_find(m, h, (const uint8_t *)key);
    return i < 0 ? NULL : SH_VAL(m, h, i);
}

int om_lookup(om_map *m, const void *key, void *value_out) {
    uint8_t *v = om_lookup_ptr(m, key);
    if (!v) return -ENOENT;
    if (value_out) memcpy(value_out, v, m->vsz);
    return 0;
}

/* Element ceiling of an insert.  HASH / LPM: max_entries (E2BIG / ENOSPC).
 * LRU_HASH: the kernel never fails an LRU insert (it evicts).  libgpuflow evicts
 * only the conntrack maps (ipv4/ipv6_ct_tuple -> ct_entry, the maps a classify
 * call binds, LRU stand-in above): those may exceed max_entries inside a batch, up
 * to the 7/8 load of their slot array (ct_slots: 8 x max_entries for ipv4_ct_tuple,
 * 4 x for ipv6_ct_tuple, rounded up to a power of 2, gf_common.h
 * gf_ct_slot_factor).  Any other LRU map has no eviction path there and stops at
 * max_entries. */
static uint64_t ct_slots(const om_map *m) {
    uint64_t want = (m->ksz == 14 ? 8ull : 4ull) * m->max_entries, p = 64;
    while (p < want) p <<= 1;
    return p;
}
static uint32_t om_insert_limit(const om_map *m) {
    if (m->type != OM_LRU_HASH || !((m->ksz == 14 || m->ksz == 40) && m->vsz == 48)) return m->max_entries;
    uint64_t p = ct_slots(m);
    return (uint32_t)(p / 8 * 7 > 0xffffffffull ? 0xffffffffu : p / 8 * 7);
}

/* map_update_elem(): kernel htab_map_update_elem / trie_update_elem. */
int om_update(om_map *m, const void *key_, const void *value, uint64_t flags) {
    if (flags > 2) return -EINVAL;
    uint8_t nk[64];
    const uint8_t *key = (const uint8_t *)key_;
    if (is_lpm(m)) {
        uint32_t plen; memcpy(&plen, key, 4);
        if (plen > lpm_bits(m)) return -EINVAL;
        lpm_normalize(m, key, nk); key = nk;
    }
    om_shard *h = &m->sh[shard_of(m, key)];
    int64_t i = sh_find(m, h, key);
    if (i >= 0) {
        if (flags == 1) return -EEXIST;
        memcpy(SH_VAL(m, h, i), value, m->vsz);
        return 0;
    }
    if (flags == 2) return -ENOENT;
    uint32_t c = __atomic_add_fetch(&m->count, 1, __ATOMIC_RELAXED);
    if (c > om_insert_limit(m)) {
        __atomic_sub_fetch(&m->count, 1, __ATOMIC_RELAXED);
        return is_lpm(m) ? -ENOSPC : -E2BIG;
    }
    if ((h->used + h->tomb + 1) * 2 > h->cap) sh_grow(m, h);
    uint64_t mask = h->cap - 1, j = fnv1a(key, m->ksz) & mask;
    while (SH_ST(m, h, j) == 1) j = (j + 1) & mask;
    if (SH_ST(m, h, j) == 2) h->tomb--;
    SH_ST(m, h, j) = 1;
    memcpy(SH_KEY(m, h, j), key, m->ksz);
    memcpy(SH_VAL(m, h, j), value, m->vsz);
    h->used++;
    if (is_lpm(m)) { uint32_t plen; memcpy(&plen, key, 4); m->lens_cnt[plen]++; }
    return 0;
}

/* n sequential om_update calls; stops at the first error (returns it, *done = applied). */
int om_update_many(om_map *m, const void *keys, const void *values, uint32_t n, uint64_t flags, uint32_t *done) {
    for (uint32_t i = 0; i < n; i++) {
        int r = om_update(m, (const uint8_t *)keys + (size_t)i * m->ksz, (const uint8_t *)values + (size_t)i * m->vsz, flags);
        if (r) { if (done) *done = i; return r; }
    }
    if (done) *done = n;
    return 0;
}

int om_delete(om_map *m, const void *key_) {
    uint8_t nk[64];
    const uint8_t *key = (const uint8_t *)key_;
    if (is_lpm(m)) {
        uint32_t plen; memcpy(&plen, key, 4);
        if (plen > lpm_bits(m)) return -EINVAL;
        lpm_normalize(m, key, nk); key = nk;
    }
    om_shard *h = &m->sh[shard_of(m, key)];
    int64_t i = sh_find(m, h, key);
    if (i < 0) return -ENOENT;
    SH_ST(m, h, i) = 2; h->used--; h->tomb++;
    __atomic_sub_fetch(&m->count, 1, __ATOMIC_RELAXED);
    if (is_lpm(m)) { uint32_t plen; memcpy(&plen, key, 4); m->lens_cnt[plen]--; }
    return 0;
}

uint32_t om_count(om_map *m) { return m->count; }

uint32_t om_foreach(om_map *m, om_visit_fn fn, void *ctx) {
    uint32_t n = 0;
    for (uint32_t s = 0; s < m->nshards; s++) {
        om_shard *h = &m->sh[s];
        for (uint64_t i = 0; i < h->cap; i++)
            if (SH_ST(m, h, i) == 1) { fn(SH_KEY(m, h, i), SH_VAL(m, h, i), ctx); n++; }
    }
    return n;
}

typedef struct dump_ctx { om_map *m; uint8_t *k, *v; uint32_t cap, n; } dump_ctx;
static void dump_visit(const void *k, const void *v, void *c_) {
    dump_ctx *c = (dump_ctx *)c_;
    if (c->n < c->cap) {
        memcpy(c->k + (size_t)c->n * c->m->ksz, k, c->m->ksz);
        memcpy(c->v + (size_t)c->n * c->m->vsz, v, c->m->vsz);
    }
    c->n++;
}
uint32_t om_dump(om_map *m, void *keys, void *values, uint32_t capacity) {
    dump_ctx c = { m, (uint8_t *)keys, (uint8_t *)values, capacity, 0 };
    om_foreach(m, dump_visit, &c);
    return c.n;
}

/* CT shard selection: unordered address pair of the tuple. */
uint32_t o_ct_pair_hash4(uint32_t a, uint32_t b) {
    uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
    uint64_t x = ((uint64_t)hi << 32) | lo;
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)x;
}
uint32_t o_ct_pair_hash6(const uint8_t *a, const uint8_t *b) {
    const uint8_t *lo = memcmp(a, b, 16) <= 0 ? a : b, *hi = lo == a ? b : a;
    uint8_t buf[32]; memcpy(buf, lo, 16); memcpy(buf + 16, hi, 16);
    return (uint32_t)fnv1a(buf, 32);
}
static uint32_t shard_of(const om_map *m, const uint8_t *key) {
    if (m->nshards <= 1) return 0;
    if (m->ksz == 14) { uint32_t a, b; memcpy(&a, key, 4); memcpy(&b, key + 4, 4);
        return o_ct_pair_hash4(a, b) % m->nshards; }
    if (m->ksz == 40) return o_ct_pair_hash6(key, key + 16) % m->nshards;
    return (uint32_t)(fnv1a(key, m->ksz) % m->nshards);
}

/* ------------------------------------------------------------------ */
/* skb access emulation                                                */
/* ------------------------------------------------------------------ */
typedef struct skb {
    const uint8_t *data; uint32_t len, cap;   /* cap = snap bytes present */
    uint32_t cb[5];
    uint32_t tc_index, hash;
    uint16_t protocol;                        /* host order ethertype */
    uint32_t idx;                             /* packet index in the batch (trace sink slot) */
} skb_t;

static inline uint8_t skb_byte(const skb_t *s, uint32_t off) { return off < s->cap ? s->data[off] : 0; }

/* bpf_skb_load_bytes(): offset > 0xffff (incl. negative) or past len -> -EFAULT */
static int skb_load_bytes(const skb_t *s, int32_t off, void *to, uint32_t n) {
    uint8_t *d = (uint8_t *)to;
    if ((uint32_t)off > 0xffff || (uint64_t)(uint32_t)off + n > s->len) {
        memset(d, 0, n);
        return -EFAULT;
    }
    for (uint32_t i = 0; i < n; i++) d[i] = skb_byte(s, (uint32_t)off + i);
    return 0;
}
/* bpf_skb_store_bytes()/bpf_l{3,4}_csum_replace() writability checks:
 * offset > 0xffff -> -EFAULT; offset + n past len -> -EFAULT. */
static int skb_writable(const skb_t *s, int32_t off, uint32_t n) {
    if ((uint32_t)off > 0xffff || (uint64_t)(uint32_t)off + n > s->len) return -EFAULT;
    return 0;
}
static int l4_csum_replace_chk(const skb_t *s, int32_t off) {
    if ((uint32_t)off > 0xffff || (off & 1)) return -EFAULT;
    return skb_writable(s, off, 2);
}
static inline uint16_t rd16(const skb_t *s, uint32_t off) {
    return (uint16_t)(skb_byte(s, off) | (skb_byte(s, off + 1) << 8));
}
static inline uint32_t rd32(const skb_t *s, uint32_t off) {
    return (uint32_t)rd16(s, off) | ((uint32_t)rd16(s, off + 2) << 16);
}
static inline uint16_t bswap16(uint16_t x) { return (uint16_t)((x >> 8) | (x << 8)); }

/* csum_l4_offset_and_flags, bpf/lib/csum.h:45-67 (offset part) */
static uint16_t csum_l4_offset(uint8_t nexthdr) {
    switch (nexthdr) {
    case IPPROTO_TCP: return 16;
    case IPPROTO_UDP: return 6;
    case IPPROTO_ICMPV6: return 2;
    default: return 0;
    }
}

/* ------------------------------------------------------------------ */
/* KAT helpers, bpf/lib/ipv6.h:136-150, bpf/lib/maps.h:147-160          */
/* ------------------------------------------------------------------ */
static inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
uint32_t o_get_prefix(int prefix) {
    uint32_t v = prefix <= 0 ? 0 : prefix < 32 ? ((1u << prefix) - 1) << (32 - prefix) : 0xFFFFFFFFu;
    return bswap32(v);   /* bpf_htonl */
}
void o_ipv6_addr_clear_suffix(uint8_t addr[16], int prefix) {
    for (int w = 0; w < 4; w++) {
        uint32_t p; memcpy(&p, addr + 4 * w, 4);
        p &= o_get_prefix(prefix);
        memcpy(addr + 4 * w, &p, 4);
        prefix -= 32;
    }
}
int o_lpm4_iter_lookup(uint32_t stored_net, const int *prefixes, int n, uint32_t addr) {
    for (int i = 0; i < n; i++)
        if ((addr & o_get_prefix(prefixes[i])) == stored_net) return 1;
    return 0;
}

/* ------------------------------------------------------------------ */
/* header parse (the rules gf_parse_frames implements)                 */
/* ------------------------------------------------------------------ */

/* ipv6_hdrlen, bpf/lib/ipv6.h:61-98.  NB: the AUTH length formula is chosen
 * by the NEXT header value (nh is reassigned before the test), reproduced. */
static int ipv6_hdrlen(const skb_t *s, int l3_off, uint8_t *nexthdr) {
    int len = 40;
    uint8_t nh = *nexthdr;
    for (int i = 0; i < 4; i++) {
        switch (nh) {
        case 59: return DROP_INVALID_EXTHDR;      /* NEXTHDR_NONE */
        case 44: return DROP_FRAG_NOSUPPORT;      /* NEXTHDR_FRAGMENT */
        case 0: case 43: case 51: case 60: {      /* HOP, ROUTING, AUTH, DEST */
            uint8_t opt[2];
            if (skb_load_bytes(s, l3_off + len, opt, 2) < 0) return DROP_INVALID;
            nh = opt[0];
            if (nh == 51) len += (opt[1] + 2) << 2;   /* ipv6_authlen */
            else len += (opt[1] + 1) << 3;            /* ipv6_optlen */
            break;
        }
        default:
            *nexthdr = nh;
            return len;
        }
    }
    return DROP_INVALID_EXTHDR;
}

static void skb_init(skb_t *s, const o_batch *b, uint32_t i) {
    memset(s, 0, sizeof(*s));
    s->data = b->snap + (size_t)i * b->snap_stride;
    s->len = b->len[i];
    s->cap = b->snap_stride < s->len ? b->snap_stride : s->len;
    s->protocol = s->len >= 14 ? (uint16_t)((s->data[12] << 8) | s->data[13]) : 0;
    if (b->tc_index) s->tc_index = b->tc_index[i];
    if (b->flow_hash) s->hash = b->flow_hash[i];
    s->idx = i;
}

static void l4_bytes(const skb_t *s, int l4_off, uint32_t *w0, uint16_t *w3) {
    uint8_t b[4] = {0, 0, 0, 0}, c[2] = {0, 0};
    for (int k = 0; k < 4; k++) {
        int64_t o = (int64_t)l4_off + k;
        if (o >= 0 && o < s->len) b[k] = skb_byte(s, (uint32_t)o);
    }
    for (int k = 0; k < 2; k++) {
        int64_t o = (int64_t)l4_off + 12 + k;
        if (o >= 0 && o < s->len) c[k] = skb_byte(s, (uint32_t)o);
    }
    memcpy(w0, b, 4); memcpy(w3, c, 2);
}

void o_parse_batch(const o_batch *b, o_cols *o) {
    for (uint32_t i = 0; i < b->n; i++) {
        skb_t s; skb_init(&s, b, i);
        uint16_t et = s.protocol;
        uint32_t sa = 0, da = 0, w0 = 0; uint16_t w3 = 0; uint8_t proto = 0; int l4 = 0;
        uint8_t s6[16] = {0}, d6[16] = {0};
        if (et == 0x0800 && s.len >= 34) {
            sa = rd32(&s, 26); da = rd32(&s, 30); proto = skb_byte(&s, 23);
            l4 = ETH_HLEN + (skb_byte(&s, 14) & 0xf) * 4;
            l4_bytes(&s, l4, &w0, &w3);
        } else if (et == 0x86DD && s.len >= 54) {
            for (int k = 0; k < 16; k++) { s6[k] = skb_byte(&s, 22 + k); d6[k] = skb_byte(&s, 38 + k); }
            proto = skb_byte(&s, 20);
            l4 = ETH_HLEN + ipv6_hdrlen(&s, ETH_HLEN, &proto);
            l4_bytes(&s, l4, &w0, &w3);
        }
        o->ethertype[i] = et; o->saddr4[i] = sa; o->daddr4[i] = da; o->proto[i] = proto;
        o->l4_off[i] = (int16_t)l4; o->l4w0[i] = w0; o->l4w3[i] = w3;
        if (o->saddr6) memcpy(o->saddr6 + 16 * (size_t)i, s6, 16);
        if (o->daddr6) memcpy(o->daddr6 + 16 * (size_t)i, d6, 16);
    }
}

/* ------------------------------------------------------------------ */
/* XDP prefilter, bpf/bpf_xdp.c:88-184                                 */
/* ------------------------------------------------------------------ */
/* lookup_ip4_endpoint / lookup_ip6_endpoint, bpf/lib/eps.h:26-46 */
static int lookup_ip4_endpoint(om_map *lxc, uint32_t daddr) {
    uint8_t key[20] = {0};
    memcpy(key, &daddr, 4); key[16] = 1;   /* ENDPOINT_KEY_IPV4 */
    return om_lookup_ptr(lxc, key) != NULL;
}
static int lookup_ip6_endpoint(om_map *lxc, const uint8_t *daddr) {
    uint8_t key[20] = {0};
    memcpy(key, daddr, 16); key[16] = 2;   /* ENDPOINT_KEY_IPV6 */
    return om_lookup_ptr(lxc, key) != NULL;
}

static int xdp_check_v4(const o_xdp_cfg *c, const skb_t *s) {
    if (s->len < ETH_HLEN + 20) return XDP_DROP;          /* xdp_no_room */
    uint32_t saddr = rd32(s, 26), daddr = rd32(s, 30);
    if (c->cidr4_hmap) {                                   /* CIDR4_FILTER */
        uint8_t pfx[8]; uint32_t pl = 32;
        memcpy(pfx, &pl, 4); memcpy(pfx + 4, &saddr, 4);
        if (c->cidr4_lmap && om_lookup_ptr(c->cidr4_lmap, pfx)) return XDP_DROP;
        return om_lookup_ptr(c->cidr4_hmap, pfx) ? XDP_DROP
               : (lookup_ip4_endpoint(c->lxc_map, daddr) ? XDP_PASS : XDP_DROP);
    }
    return lookup_ip4_endpoint(c->lxc_map, daddr) ? XDP_PASS : XDP_DROP;
}
static int xdp_check_v6(const o_xdp_cfg *c, const skb_t *s) {
    if (s->len < ETH_HLEN + 40) return XDP_DROP;
    uint8_t saddr[16], daddr[16];
    for (int k = 0; k < 16; k++) { saddr[k] = skb_byte(s, 22 + k); daddr[k] = skb_byte(s, 38 + k); }
    if (c->cidr6_hmap) {                                   /* CIDR6_FILTER */
        uint8_t pfx[20]; uint32_t pl = 128;
        memcpy(pfx, &pl, 4); memcpy(pfx + 4, saddr, 16);
        if (c->cidr6_lmap && om_lookup_ptr(c->cidr6_lmap, pfx)) return XDP_DROP;
        return om_lookup_ptr(c->cidr6_hmap, pfx) ? XDP_DROP
               : (lookup_ip6_endpoint(c->lxc_map, daddr) ? XDP_PASS : XDP_DROP);
    }
    return lookup_ip6_endpoint(c->lxc_map, daddr) ? XDP_PASS : XDP_DROP;
}
static int xdp_start(const o_xdp_cfg *c, const skb_t *s) {
    if (s->len < ETH_HLEN) return XDP_DROP;
    if (s->protocol == 0x0800) return xdp_check_v4(c, s);
    if (s->protocol == 0x86DD) return xdp_check_v6(c, s);
    return XDP_PASS;
}

void o_xdp_batch(const o_xdp_cfg *cfg, const o_batch *b, uint8_t *verdict) {
    for (uint32_t i = 0; i < b->n; i++) { skb_t s; skb_init(&s, b, i); verdict[i] = (uint8_t)xdp_start(cfg, &s); }
}

/* ------------------------------------------------------------------ */
/* Standalone LB, bpf/bpf_lb.c:58-212 + bpf/lib/lb.h                   */
/* ------------------------------------------------------------------ */
typedef struct lb_res { uint16_t slave, new_dport, rev_nat, key_dport; uint32_t new_daddr4; uint8_t nd6[16]; } lb_res;

/* extract_l4_port, bpf/lib/lb.h:191-215 */
static int extract_l4_port(const skb_t *s, uint8_t nexthdr, int l4_off, uint16_t *port) {
    switch (nexthdr) {
    case IPPROTO_TCP: case IPPROTO_UDP: {
        int ret = skb_load_bytes(s, l4_off + 2, port, 2);   /* l4_load_port, TCP_DPORT_OFF */
        if (IS_ERR(ret)) return ret;
        break;
    }
    case IPPROTO_ICMPV6: case IPPROTO_ICMP: break;
    default: return DROP_UNKNOWN_L4;
    }
    return 0;
}

/* lb4_lookup_service, bpf/lib/lb.h:566-597 ; key = {be32 address, be16 dport, u16 slave} */
static uint8_t *lb4_lookup_service(const o_lb_cfg *c, uint8_t *key) {
    uint16_t dport; memcpy(&dport, key + 4, 2);
    if ((c->flags & LB_F_L4) && dport) {
        uint8_t *svc = om_lookup_ptr(c->lb4_services, key);
        if (svc) { uint16_t cnt; memcpy(&cnt, svc + 6, 2); if (cnt) return svc; }
        memset(key + 4, 0, 2);                                 /* key->dport = 0 */
    }
    if (c->flags & LB_F_L3) {
        uint8_t *svc = om_lookup_ptr(c->lb4_services, key);
        if (svc) { uint16_t cnt; memcpy(&cnt, svc + 6, 2); if (cnt) return svc; }
    }
    return NULL;
}
/* lb6_lookup_service, bpf/lib/lb.h:350-379 ; lb6_key = {addr[16], be16 dport, u16 slave} */
static uint8_t *lb6_lookup_service(const o_lb_cfg *c, uint8_t *key) {
    uint16_t dport; memcpy(&dport, key + 16, 2);
    if ((c->flags & LB_F_L4) && dport) {
        uint8_t *svc = om_lookup_ptr(c->lb6_services, key);
        if (svc) { uint16_t cnt; memcpy(&cnt, svc + 18, 2); if (cnt) return svc; }
        memset(key + 16, 0, 2);
    }
    if (c->flags & LB_F_L3) {
        uint8_t *svc = om_lookup_ptr(c->lb6_services, key);
        if (svc) { uint16_t cnt; memcpy(&cnt, svc + 18, 2); if (cnt) return svc; }
    }
    return NULL;
}

/* shared tail of lb4_xlate / lb6_xlate (bpf/lib/lb.h:615-659, 397-423):
 * verdict-affecting checks of the checksum/port rewrites. */
static int lb_xlate_checks(const o_lb_cfg *c, const skb_t *s, uint8_t nexthdr, int l4_off,
                           uint16_t key_dport, uint16_t svc_port, int v6, uint16_t *new_dport) {
    uint16_t csum_off = csum_l4_offset(nexthdr);
    if ((csum_off || v6) && l4_csum_replace_chk(s, l4_off + csum_off) < 0) return DROP_CSUM_L4;
    if ((c->flags & LB_F_L4) && svc_port && key_dport != svc_port &&
        (nexthdr == IPPROTO_TCP || nexthdr == IPPROTO_UDP)) {
        /* l4_modify_port: csum_l4_replace then skb_store_bytes(l4_off+2) */
        if (l4_csum_replace_chk(s, l4_off + csum_off) < 0) return DROP_CSUM_L4;
        if (skb_writable(s, l4_off + 2, 2) < 0) return DROP_WRITE_ERROR;
        *new_dport = svc_port;
    }
    return TC_ACT_OK;
}

static int lb_handle_ipv4(const o_lb_cfg *c, const skb_t *s, lb_res *r) {
    if (s->len < ETH_HLEN + 20) return DROP_INVALID;             /* revalidate_data */
    uint8_t nexthdr = skb_byte(s, 23);
    uint8_t key[8] = {0};
    uint32_t daddr = rd32(s, 30);
    memcpy(key, &daddr, 4);
    int l4_off = ETH_HLEN + (skb_byte(s, 14) & 0xf) * 4;        /* ipv4_hdrlen */
    int ret;
    if (c->flags & LB_F_L4) {
        ret = extract_l4_port(s, nexthdr, l4_off, (uint16_t *)(key + 4));
        if (IS_ERR(ret)) return ret == DROP_UNKNOWN_L4 ? TC_ACT_OK : ret;
    }
    uint8_t *svc = lb4_lookup_service(c, key);
    if (!svc) return TC_ACT_OK;
    uint16_t count; memcpy(&count, svc + 6, 2);
    uint16_t slave = (uint16_t)((s->hash % count) + 1);           /* lb4_select_slave */
    memcpy(key + 6, &slave, 2);                                  /* lb4_lookup_slave */
    svc = om_lookup_ptr(c->lb4_services, key);
    if (!svc) return DROP_NO_SERVICE;
    uint16_t key_dport, svc_port; memcpy(&key_dport, key + 4, 2); memcpy(&svc_port, svc + 4, 2);
    ret = lb_xlate_checks(c, s, nexthdr, l4_off, key_dport, svc_port, 0, &r->new_dport);
    if (IS_ERR(ret)) return ret;
    r->slave = slave; r->key_dport = key_dport;
    memcpy(&r->new_daddr4, svc, 4);
    memcpy(&r->rev_nat, svc + 8, 2);
    return TC_ACT_REDIRECT;
}

static int lb_handle_ipv6(const o_lb_cfg *c, const skb_t *s, lb_res *r) {
    if (s->len < ETH_HLEN + 40) return DROP_INVALID;
    uint8_t nexthdr = skb_byte(s, 20);
    uint8_t key[20] = {0};
    for (int k = 0; k < 16; k++) key[k] = skb_byte(s, 38 + k);
    int l4_off = ETH_HLEN + ipv6_hdrlen(s, ETH_HLEN, &nexthdr);
    int ret;
    if (c->flags & LB_F_L4) {
        ret = extract_l4_port(s, nexthdr, l4_off, (uint16_t *)(key + 16));
        if (IS_ERR(ret)) return ret == DROP_UNKNOWN_L4 ? TC_ACT_OK : ret;
    }
    uint8_t *svc = lb6_lookup_service(c, key);
    if (!svc) return TC_ACT_OK;
    uint16_t count; memcpy(&count, svc + 18, 2);
    uint16_t slave = (uint16_t)((s->hash % count) + 1);
    memcpy(key + 18, &slave, 2);
    svc = om_lookup_ptr(c->lb6_services, key);
    if (!svc) return DROP_NO_SERVICE;
    uint8_t nd[16]; memcpy(nd, svc, 16);
    uint16_t rn; memcpy(&rn, svc + 20, 2);
    if (rn) { uint32_t p4; memcpy(&p4, nd + 12, 4); p4 |= rn; memcpy(nd + 12, &p4, 4); }
    uint16_t key_dport, svc_port; memcpy(&key_dport, key + 16, 2); memcpy(&svc_port, svc + 16, 2);
    ret = lb_xlate_checks(c, s, nexthdr, l4_off, key_dport, svc_port, 1, &r->new_dport);
    if (IS_ERR(ret)) return ret;
    r->slave = slave; r->rev_nat = rn; r->key_dport = key_dport;
    memcpy(r->nd6, nd, 16);
    return TC_ACT_REDIRECT;
}

/* from_netdev, bpf/bpf_lb.c:169-212.  The output reports what the
 * translation changed: slave/new_daddr/rev_nat when lb*_xlate ran, new_dport
 * when the L4 port was rewritten; zero otherwise. */
static void lb_one_res(const o_lb_cfg *c, const skb_t *s, o_lb_out *o, uint8_t *nd6, lb_res *rout) {
    lb_res r; memset(&r, 0, sizeof(r));
    if (rout) memset(rout, 0, sizeof *rout);
    memset(o, 0, sizeof *o);
    if (nd6) memset(nd6, 0, 16);
    int ret, v6 = 0;
    switch (s->protocol) {
    case 0x86DD:
        if (c->flags & LB_F_NO_IPV6) return;
        v6 = 1; ret = lb_handle_ipv6(c, s, &r); break;
    case 0x0800:
        if (c->flags & LB_F_NO_IPV4) return;
        ret = lb_handle_ipv4(c, s, &r); break;
    default:
        return;                                           /* TC_ACT_OK */
    }
    if (IS_ERR(ret)) {                                    /* send_drop_notify_error */
        o->action = TC_ACT_SHOT; o->reason = (uint8_t)(-ret);
        return;
    }
    o->action = ((c->flags & LB_F_REDIRECT) && ret == TC_ACT_REDIRECT) ? TC_ACT_REDIRECT : TC_ACT_OK;
    if (ret == TC_ACT_REDIRECT) {
        o->slave = r.slave; o->new_dport = r.new_dport; o->rev_nat = r.rev_nat;
        if (v6) { if (nd6) memcpy(nd6, r.nd6, 16); }
        else o->new_daddr4 = r.new_daddr4;
        if (rout) *rout = r;
    }
}
static void lb_one(const o_lb_cfg *c, const skb_t *s, o_lb_out *o, uint8_t *nd6) { lb_one_res(c, s, o, nd6, NULL); }

void o_lb_batch(const o_lb_cfg *cfg, const o_batch *b, o_lb_out *out, uint8_t *nd6) {
    for (uint32_t i = 0; i < b->n; i++) {
        skb_t s; skb_init(&s, b, i);
        lb_one(cfg, &s, &out[i], nd6 ? nd6 + 16 * (size_t)i : NULL);
    }
}

/* ------------------------------------------------------------------ */
/* Conntrack, bpf/lib/conntrack.h:47-580                               */
/* ------------------------------------------------------------------ */
/* ct_entry byte offsets */
#define CTE_RX_PKTS 0
#define CTE_RX_BYTES 8
#define CTE_TX_PKTS 16
#define CTE_TX_BYTES 24
#define CTE_LIFETIME 32
#define CTE_FLAGS 36
#define CTE_REVNAT 38
#define CTE_SRCSEC 44
#define CTF_RX_CLOSING 1u
#define CTF_TX_CLOSING 2u
#define CTF_LB_LOOPBACK 8u
#define CTF_SEEN_NON_SYN 16u

typedef struct ct_state { uint16_t rev_nat_index; uint8_t loopback; uint16_t orig_dport;
                          uint32_t addr, svc_addr, src_sec_id; } ct_state_t;

static inline uint16_t ge16(const uint8_t *p, int o) { uint16_t v; memcpy(&v, p + o, 2); return v; }
static inline void se16(uint8_t *p, int o, uint16_t v) { memcpy(p + o, &v, 2); }
static inline uint32_t ge32(const uint8_t *p, int o) { uint32_t v; memcpy(&v, p + o, 4); return v; }
static inline void se32(uint8_t *p, int o, uint32_t v) { memcpy(p + o, &v, 4); }
static inline uint64_t ge64(const uint8_t *p, int o) { uint64_t v; memcpy(&v, p + o, 8); return v; }
static inline void se64(uint8_t *p, int o, uint64_t v) { memcpy(p + o, &v, 8); }

/* ct_update_timeout / __ct_update_timeout (NEEDS_TIMEOUT), conntrack.h:47-62 */
static void ct_update_timeout(uint8_t *e, int syn, uint32_t now) {
    uint16_t f = ge16(e, CTE_FLAGS);
    if (!syn) f |= CTF_SEEN_NON_SYN;
    se16(e, CTE_FLAGS, f);
    se32(e, CTE_LIFETIME, now + ((f & CTF_SEEN_NON_SYN) ? CT_DEFAULT_LIFETIME : CT_SYN_TIMEOUT));
}
static int ct_entry_alive(const uint8_t *e) {
    uint16_t f = ge16(e, CTE_FLAGS);
    return !(f & CTF_RX_CLOSING) || !(f & CTF_TX_CLOSING);
}

typedef struct ctx {
    uint32_t now;
    const o_lxc_cfg *lxc;
} ctx_t;

/* __ct_lookup, conntrack.h:75-135 */
static int __ct_lookup(om_map *map, const skb_t *s, const void *tuple, int action, int dir,
                       ct_state_t *st, int syn, uint32_t now, int accounting) {
    uint8_t *e = om_lookup_ptr(map, tuple);
    if (!e) return CT_NEW;
    if (ct_entry_alive(e)) ct_update_timeout(e, syn, now);
    if (st) {
        st->rev_nat_index = ge16(e, CTE_REVNAT);
        st->loopback = (ge16(e, CTE_FLAGS) & CTF_LB_LOOPBACK) ? 1 : 0;
    }
    if (accounting) {
        if (dir == CT_INGRESS) {
            se64(e, CTE_RX_PKTS, ge64(e, CTE_RX_PKTS) + 1);
            se64(e, CTE_RX_BYTES, ge64(e, CTE_RX_BYTES) + s->len);
        } else {
            se64(e, CTE_TX_PKTS, ge64(e, CTE_TX_PKTS) + 1);
            se64(e, CTE_TX_BYTES, ge64(e, CTE_TX_BYTES) + s->len);
        }
    }
    uint16_t f = ge16(e, CTE_FLAGS);
    switch (action) {
    case ACTION_CREATE:
        if (((f & CTF_RX_CLOSING) ? 1 : 0) + ((f & CTF_TX_CLOSING) ? 1 : 0) >= 1) {
            se16(e, CTE_FLAGS, (uint16_t)(f & ~(CTF_RX_CLOSING | CTF_TX_CLOSING)));
            ct_update_timeout(e, syn, now);
        }
        break;
    case ACTION_CLOSE:
        f |= (dir == CT_INGRESS) ? CTF_RX_CLOSING : CTF_TX_CLOSING;
        se16(e, CTE_FLAGS, f);
        if (ct_entry_alive(e)) break;
        se32(e, CTE_LIFETIME, now + CT_CLOSE_TIMEOUT);
        break;
    }
    return CT_ESTABLISHED;
}

/* tuple4 offsets: daddr 0, saddr 4, dport 8, sport 10, nexthdr 12, flags 13 */
static void ipv4_ct_tuple_reverse(uint8_t *t) {                 /* conntrack.h:291-308 */
    uint8_t tmp[4]; memcpy(tmp, t + 4, 4); memcpy(t + 4, t, 4); memcpy(t, tmp, 4);
    uint16_t sp = ge16(t, 10), dp = ge16(t, 8); se16(t, 10, dp); se16(t, 8, sp);
    t[13] = (t[13] & TUPLE_F_IN) ? (uint8_t)(t[13] & ~TUPLE_F_IN) : (uint8_t)(t[13] | TUPLE_F_IN);
}
/* tuple6 offsets: daddr 0, saddr 16, dport 32, sport 34, nexthdr 36, flags 37 */
static void ipv6_ct_tuple_reverse(uint8_t *t) {                 /* conntrack.h:147-167 */
    uint8_t tmp[16]; memcpy(tmp, t + 16, 16); memcpy(t + 16, t, 16); memcpy(t, tmp, 16);
    uint16_t sp = ge16(t, 34), dp = ge16(t, 32); se16(t, 34, dp); se16(t, 32, sp);
    t[37] = (t[37] & TUPLE_F_IN) ? (uint8_t)(t[37] & ~TUPLE_F_IN) : (uint8_t)(t[37] | TUPLE_F_IN);
}

/* ct_lookup4 / ct_lookup6 (conntrack.h:170-289, 319-435).  v6 selects the
 * tuple layout and the ICMPv6 type table. */
static int ct_lookup(om_map *map, uint8_t *t, const skb_t *s, int off, int dir,
                     ct_state_t *st, int v6, uint32_t now, int accounting) {
    int action = ACTION_UNSPEC, syn = 0, ret;
    int o_dport = v6 ? 32 : 8, o_sport = v6 ? 34 : 10, o_nh = v6 ? 36 : 12, o_fl = v6 ? 37 : 13;
    t[o_fl] = dir == CT_INGRESS ? TUPLE_F_OUT : TUPLE_F_IN;
    uint8_t nh = t[o_nh];
    if ((!v6 && nh == IPPROTO_ICMP) || (v6 && nh == IPPROTO_ICMPV6)) {
        uint8_t type;
        if (skb_load_bytes(s, off, &type, 1) < 0) return DROP_CT_INVALID_HDR;
        se16(t, o_sport, 0); se16(t, o_dport, 0);
        if (!v6) {
            switch (type) {
            case 3: case 11: case 12: t[o_fl] |= TUPLE_F_RELATED; break;   /* DEST_UNREACH, TIME_EXCEEDED, PARAMETERPROB */
            case 0: se16(t, o_dport, 8); break;                             /* ECHOREPLY -> dport = ICMP_ECHO */
            case 8: se16(t, o_sport, type); /* fallthrough */               /* ECHO */
            default: action = ACTION_CREATE; break;
            }
        } else {
            switch (type) {
            case 1: case 2: case 3: case 4: t[o_fl] |= TUPLE_F_RELATED; break;
            case 129: se16(t, o_dport, 128); break;                         /* ECHO_REPLY */
            case 128: se16(t, o_sport, type); /* fallthrough */
            default: action = ACTION_CREATE; break;
            }
        }
    } else if (nh == IPPROTO_TCP) {
        uint16_t fl;
        if (skb_load_bytes(s, off + 12, &fl, 2) < 0) return DROP_CT_INVALID_HDR;
        int fin = (fl >> 8) & 1, sy = (fl >> 9) & 1, rst = (fl >> 10) & 1;   /* struct tcp_flags, LE bitfield */
        action = (rst || fin) ? ACTION_CLOSE : ACTION_CREATE;
        syn = sy;
        if (skb_load_bytes(s, off, t + o_dport, 4) < 0) return DROP_CT_INVALID_HDR;
    } else if (nh == IPPROTO_UDP) {
        if (skb_load_bytes(s, off, t + o_dport, 4) < 0) return DROP_CT_INVALID_HDR;
        action = ACTION_CREATE;
    } else {
        return DROP_CT_UNKNOWN_PROTO;
    }
    ret = __ct_lookup(map, s, t, action, dir, st, syn, now, accounting);
    if (ret != CT_NEW) {
        if (ret == CT_ESTABLISHED) ret = (t[o_fl] & TUPLE_F_RELATED) ? CT_RELATED : CT_REPLY;
        return ret;
    }
    if (v6) ipv6_ct_tuple_reverse(t); else ipv4_ct_tuple_reverse(t);
    return __ct_lookup(map, s, t, action, dir, st, syn, now, accounting);
}

/* ct_create4 (conntrack.h:503-580) / ct_create6 (:446-493).  The second
 * (service / loopback) entry exists only on the v4 egress path, where
 * lb4_local sets ct_state->addr. */
static int ct_create(om_map *map, uint8_t *t, const skb_t *s, int dir, const ct_state_t *st,
                     int v6, uint32_t now) {
    uint8_t e[48]; memset(e, 0, sizeof e);
    int o_nh = v6 ? 36 : 12, o_fl = v6 ? 37 : 13, ksz = v6 ? 40 : 14;
    se16(e, CTE_REVNAT, st->rev_nat_index);
    if (st->loopback) se16(e, CTE_FLAGS, CTF_LB_LOOPBACK);
    ct_update_timeout(e, t[o_nh] == IPPROTO_TCP, now);
    if (dir == CT_INGRESS) { se64(e, CTE_RX_PKTS, 1); se64(e, CTE_RX_BYTES, s->len); }
    else { se64(e, CTE_TX_PKTS, 1); se64(e, CTE_TX_BYTES, s->len); }
    se32(e, CTE_SRCSEC, st->src_sec_id);
    if (om_update(map, t, e, 0) < 0) return DROP_CT_CREATE_FAILED;
    if (!v6 && st->addr) {                              /* conntrack.h:533-561 (lb4_local set ct_state->addr) */
        uint8_t sv[14]; memcpy(sv, t, 14);
        if (dir == CT_INGRESS) se32(t, 4, st->addr); else se32(t, 0, st->addr);
        if (st->loopback) {
            t[13] = TUPLE_F_IN;
            if (dir == CT_INGRESS) se32(t, 0, st->svc_addr); else se32(t, 4, st->svc_addr);
        }
        int r = om_update(map, t, e, 0);
        memcpy(t, sv, 14);
        if (r < 0) return DROP_CT_CREATE_FAILED;
    }
    uint8_t it[40]; memset(it, 0, sizeof it);
    if (v6) { memcpy(it, t, 32); it[36] = IPPROTO_ICMPV6; }
    else { memcpy(it, t, 8); it[12] = IPPROTO_ICMP; }
    it[o_fl] = t[o_fl] | TUPLE_F_RELATED;
    se16(e, CTE_FLAGS, (uint16_t)(ge16(e, CTE_FLAGS) | CTF_SEEN_NON_SYN));
    if (om_update(map, it, e, 0) < 0) return DROP_CT_CREATE_FAILED;
    (void)ksz;
    return 0;
}

/* ------------------------------------------------------------------ */
/* Policy, bpf/lib/policy.h:42-168 + bpf/lib/l4.h:151-217              */
/* ------------------------------------------------------------------ */
/* l4_ingress_proxy_lookup via BPF_L4_MAP/F (bpf/lib/common.h:105-127) */
static int l4_ingress_proxy_lookup(const o_lxc_cfg *c, uint16_t dport, uint8_t nexthdr) {
    if (!c->n_l4_ingress) return 0;                 /* CFG_L3L4_INGRESS undefined */
    int allowed = DROP_POLICY_L4;
    for (uint32_t i = 0; i < c->n_l4_ingress; i++) {
        const o_l4_allow *a = &c->l4_ingress[i];
        allowed = allowed > -1 ? allowed
                : ((a->port && a->port == dport) ? ((a->nexthdr && a->nexthdr == nexthdr) ? (int)a->proxy
                                                                                     : DROP_POLICY_L4)
                                                  : DROP_POLICY_L4);
    }
    return allowed > 0 ? allowed : 0;
}
static int l4_proxy_lookup(const o_lxc_cfg *c, uint8_t nh, uint16_t dport) {   /* dir = INGRESS */
    int proxy_port = 0;
    if (nh == IPPROTO_UDP || nh == IPPROTO_TCP) {
        proxy_port = l4_ingress_proxy_lookup(c, dport, nh);
        if (proxy_port < 0) return proxy_port;
    }
    return proxy_port;
}

static void policy_count(uint8_t *p, uint32_t len) {            /* __sync_fetch_and_add x2 */
    __atomic_fetch_add((uint64_t *)(p + 8), 1, __ATOMIC_RELAXED);
    __atomic_fetch_add((uint64_t *)(p + 16), (uint64_t)len, __ATOMIC_RELAXED);
}

/* l4_egress_proxy_lookup via BPF_L4_MAP (bpf/lib/l4.h:178-188, CFG_L3L4_EGRESS) */
static int l4_egress_proxy_lookup(const o_lxc_cfg *c, uint16_t dport, uint8_t nexthdr) {
    if (!c->n_l4_egress) return 0;
    int allowed = DROP_POLICY_L4;
    for (uint32_t i = 0; i < c->n_l4_egress; i++) {
        const o_l4_allow *a = &c->l4_egress[i];
        allowed = allowed > -1 ? allowed
                : ((a->port && a->port == dport) ? ((a->nexthdr && a->nexthdr == nexthdr) ? (int)a->proxy
                                                                                     : DROP_POLICY_L4)
                                                  : DROP_POLICY_L4);
    }
    return allowed > 0 ? allowed : 0;
}

/* __policy_can_access, policy.h:42-113; dir CT_INGRESS (key.egress = 0) or
 * CT_EGRESS (key.egress = 1, l4_proxy_lookup's egress list, l4.h:192-217) */
static int __policy_can_access_dir(const o_lxc_cfg *c, const skb_t *s, uint32_t identity,
                                   uint16_t dport, uint8_t proto, int dir) {
    if (c->flags & LXC_F_DROP_ALL) return DROP_POLICY;
    uint8_t key[8];
    se32(key, 0, identity); se16(key, 4, dport); key[6] = proto; key[7] = (uint8_t)!dir;   /* egress = !dir */
    uint8_t *p;
    if (c->flags & LXC_F_HAVE_L4_POLICY) {
        p = om_lookup_ptr(c->policy_map, key);
        if (p) { policy_count(p, s->len); goto get_proxy_port; }
    }
    se16(key, 4, 0); key[6] = 0;
    p = om_lookup_ptr(c->policy_map, key);
    if (p) { policy_count(p, s->len); return TC_ACT_OK; }
    if (c->flags & LXC_F_HAVE_L4_POLICY) {
        se32(key, 0, 0); se16(key, 4, dport); key[6] = proto;
        p = om_lookup_ptr(c->policy_map, key);
        if (p) { policy_count(p, s->len); goto get_proxy_port; }
    }
    if (s->cb[2]) return TC_ACT_OK;                   /* cb[CB_POLICY], cleared by policy_clear_mark */
    return DROP_POLICY;
get_proxy_port: {
        uint16_t pp = ge16(p, 0);
        if (pp) return pp;
        if (dir == CT_INGRESS) return l4_proxy_lookup(c, proto, dport);
        if (proto == IPPROTO_UDP || proto == IPPROTO_TCP) return l4_egress_proxy_lookup(c, dport, proto);
        return 0;
    }
}
static int __policy_can_access(const o_lxc_cfg *c, const skb_t *s, uint32_t identity,
                               uint16_t dport, uint8_t proto) {
    return __policy_can_access_dir(c, s, identity, dport, proto, CT_INGRESS);
}

/* policy_can_access_ingress, policy.h:133-168 */
static int policy_can_access_ingress(const o_lxc_cfg *c, const skb_t *s, uint32_t src_identity,
                                     uint16_t dport, uint8_t proto, int v6, const uint8_t *cidr_addr) {
    if (c->flags & LXC_F_DROP_ALL) return DROP_POLICY;
    if (!(c->flags & LXC_F_POLICY_INGRESS)) return TC_ACT_OK;
    int ret = __policy_can_access(c, s, src_identity, dport, proto);
    if (ret >= TC_ACT_OK) return ret;
    if (src_identity < 256) {                          /* identity_is_reserved */
        if (v6 && c->cidr6_ingress_map) {
            uint8_t k[20]; uint32_t pl = 128; memcpy(k, &pl, 4); memcpy(k + 4, cidr_addr, 16);
            if (om_lookup_ptr(c->cidr6_ingress_map, k)) return TC_ACT_OK;
        }
        if (!v6 && c->cidr4_ingress_map) {
            uint8_t k[8]; uint32_t pl = 32; memcpy(k, &pl, 4); memcpy(k + 4, cidr_addr, 4);
            if (om_lookup_ptr(c->cidr4_ingress_map, k)) return TC_ACT_OK;
        }
    }
    return DROP_POLICY;
}

/* __lb4_rev_nat / __lb6_rev_nat verdict-affecting steps (lb.h:447-512,
 * 253-293): reverse_map_l4_port + checksum writability. */
static int lb_rev_nat_checks(const skb_t *s, int l4_off, uint8_t nexthdr, uint16_t nat_port, int v6) {
    uint16_t csum_off = csum_l4_offset(nexthdr);
    if (nat_port) {
        switch (nexthdr) {                             /* reverse_map_l4_port, lb.h:217-251 */
        case IPPROTO_TCP: case IPPROTO_UDP: {
            uint16_t old;
            int ret = skb_load_bytes(s, l4_off, &old, 2);   /* TCP_SPORT_OFF */
            if (IS_ERR(ret)) return ret;
            if (nat_port != old) {
                if (l4_csum_replace_chk(s, l4_off + csum_off) < 0) return DROP_CSUM_L4;
                if (skb_writable(s, l4_off, 2) < 0) return DROP_WRITE_ERROR;
            }
            break;
        }
        case IPPROTO_ICMPV6: case IPPROTO_ICMP: break;
        default: return DROP_UNKNOWN_L4;
        }
    }
    if (v6) {
        if (l4_csum_replace_chk(s, l4_off + csum_off) < 0) return DROP_CSUM_L4;
    } else {
        if (csum_off && l4_csum_replace_chk(s, l4_off + csum_off) < 0) return DROP_CSUM_L4;
    }
    return 0;
}

/* header-write helpers (defined with the pipeline section below); w == NULL:
 * the checks only (column batches carry no frame to rewrite) */
static void wbytes(const skb_t *s, uint8_t *w, uint32_t off, const void *from, uint32_t n);
static int l3_csum_replace(const skb_t *s, uint8_t *w, int32_t off, uint32_t from, uint32_t to, uint32_t flags);
static int l4_csum_replace(const skb_t *s, uint8_t *w, int32_t off, uint32_t from, uint32_t to, uint32_t flags);
static uint32_t ck_diff(const uint8_t *from, const uint8_t *to, int n);
static uint32_t csum_l4_flags(uint8_t nexthdr);
#define BPF_F_PSEUDO_HDR (1u << 4)
#define PROXY_DEFAULT_LIFETIME 720                     /* bpf/lib/common.h:433 */
#define DROP_PROXYMAP_CREATE_FAILED_ -161

/* The policy-stage context of one packet: the writable frame (pipeline) and
 * its proxy-map log entry (applied in batch order after the batch, see
 * proxy_apply).  Log entry: [0] family 4/6, key at +4, value at +28. */
#define O_PLOG 64
/* w: writable frame; plog: this packet's proxy-log entry; mark: its "entry written"
 * byte (ingress batches: the log's pages are touched only by redirecting packets,
 * proxy_apply scans the marks), NULL where the caller clears the entry itself */
typedef struct pol_ctx { uint8_t *w; uint8_t *plog; uint8_t *mark; } pol_ctx;

/* reverse_map_l4_port (bpf/lib/lb.h:217-251) + the address part of
 * __lb4_rev_nat / __lb6_rev_nat (lb.h:253-293, 447-512) */
static void rev_nat_write(const skb_t *s, uint8_t *w, int l4_off, uint8_t nh, const uint8_t *nat_addr,
                          uint16_t nat_port, const uint8_t *old_saddr, int v6) {
    uint16_t co = csum_l4_offset(nh);
    uint32_t fl = csum_l4_flags(nh);
    if (nat_port && (nh == IPPROTO_TCP || nh == IPPROTO_UDP)) {
        uint16_t old = rd16(s, (uint32_t)l4_off);
        if (nat_port != old) {
            l4_csum_replace(s, w, l4_off + co, old, nat_port, 2 | fl);
            wbytes(s, w, (uint32_t)l4_off, &nat_port, 2);
        }
    }
    int n = v6 ? 16 : 4;
    wbytes(s, w, v6 ? 22 : 26, nat_addr, n);
    uint32_t sum = ck_diff(old_saddr, nat_addr, n);
    if (!v6) {
        l3_csum_replace(s, w, ETH_HLEN + 10, 0, sum, 0);
        if (co) l4_csum_replace(s, w, l4_off + co, 0, sum, BPF_F_PSEUDO_HDR | fl);
    } else {
        l4_csum_replace(s, w, l4_off + co, 0, sum, BPF_F_PSEUDO_HDR | fl);
    }
}

/* ipv4_redirect_to_host_port / ipv6_... verdict-affecting steps (lib/lxc.h:96-205) */
static int redirect_to_host_port_checks(const skb_t *s, int l4_off, uint8_t nexthdr) {
    uint16_t csum_off = csum_l4_offset(nexthdr);
    if (l4_csum_replace_chk(s, l4_off + csum_off) < 0) return DROP_WRITE_ERROR;  /* l4_modify_port */
    if (skb_writable(s, l4_off + 2, 2) < 0) return DROP_WRITE_ERROR;
    return 0;                                          /* cilium_proxy{4,6} update: §8(f) */
}

/* per thread: several oracle instances may run side by side (bench.py egress leg);
 * run_mt hands the caller's copy to its workers */
static __thread o_node_cfg g_node = {1, NULL, NULL, 0, {0}, {0}, {0}, NULL, 0, 0, 0, 0, 0, NULL, {0}};   /* bpf/node_config.h */
#define g_host_ifindex (g_node.host_ifindex)
void o_set_node(const o_node_cfg *node) { g_node = *node; }

/* send_trace_notify (bpf/lib/trace.h:59-106, TRACE_NOTIFY): struct trace_notify
 * (32 B: type CILIUM_NOTIFY_TRACE=4, subtype = observation point, source =
 * EVENT_SOURCE, hash, len_orig, len_cap, src_label, dst_label, dst_id, reason,
 * pad, ifindex) followed by the first len_cap (<= TRACE_PAYLOAD_LEN) bytes of
 * the skb as it is at the call.  Events go to a per-packet list (the sink):
 * packet i's events in emission order at ev + (i * per + k) * 160, the count in
 * cnt[i]; the drop notification of a dropped packet is appended last by the
 * batch drivers.  Per thread, like g_node (run_mt hands it to its workers). */
#define O_EVENT_RECORD 160
enum { TRACE_TO_LXC, TRACE_TO_PROXY, TRACE_TO_HOST, TRACE_TO_STACK, TRACE_TO_OVERLAY, TRACE_FROM_LXC,
       TRACE_FROM_PROXY, TRACE_FROM_HOST, TRACE_FROM_STACK, TRACE_FROM_OVERLAY };
#define LXC_F_TRACE_NOTIFY (1u << 6)
#define NETDEV_F_TRACE_NOTIFY (1u << 1)
typedef struct o_trace_sink { uint8_t *ev; uint8_t *cnt; uint32_t per; int capture; } o_trace_sink;
static __thread o_trace_sink g_tr = {NULL, NULL, 0, 0};
void o_set_trace_sink(uint8_t *ev, uint8_t *cnt, uint32_t per_pkt, int capture) {
    g_tr.ev = ev; g_tr.cnt = cnt; g_tr.per = per_pkt; g_tr.capture = capture;
}
static uint8_t *ev_slot(uint32_t i) {
    if (!g_tr.ev || g_tr.cnt[i] >= g_tr.per) return NULL;
    return g_tr.ev + ((size_t)i * g_tr.per + g_tr.cnt[i]++) * O_EVENT_RECORD;
}
static void trace_event(const skb_t *s, uint8_t obs, uint16_t source, uint32_t src, uint32_t dst, uint16_t dst_id,
                        uint32_t ifindex, uint8_t reason) {
    uint8_t *ev = ev_slot(s->idx);
    if (!ev) return;
    memset(ev, 0, O_EVENT_RECORD);
    uint32_t cap = s->len < 128 ? s->len : 128;          /* min(TRACE_PAYLOAD_LEN, skb->len) */
    uint32_t f[4] = {s->len, cap, src, dst};
    ev[0] = 4;                                           /* CILIUM_NOTIFY_TRACE */
    ev[1] = obs;
    memcpy(ev + 2, &source, 2);
    memcpy(ev + 4, &s->hash, 4);                         /* get_hash_recalc(skb) */
    memcpy(ev + 8, f, 16);
    memcpy(ev + 24, &dst_id, 2);
    ev[26] = reason;
    memcpy(ev + 28, &ifindex, 4);
    if (g_tr.capture) memcpy(ev + 32, s->data, cap < s->cap ? cap : s->cap);
}

/* ipv{4,6}_redirect_to_host_port writes (lib/lxc.h:96-205) once its checks
 * passed, and the cilium_proxy{4,6} entry it creates (logged, see proxy_apply) */
static void redirect_write(const skb_t *s, pol_ctx *x, int l4_off, const uint8_t *t, int v6, uint16_t new_port,
                           const uint8_t *orig_dip, uint32_t identity, uint32_t now) {
    uint8_t nh = v6 ? t[36] : t[12];
    uint16_t old_port; memcpy(&old_port, t + (v6 ? 32 : 8), 2);
    uint16_t sport; memcpy(&sport, t + (v6 ? 34 : 10), 2);
    if (x->w) {
        uint16_t co = csum_l4_offset(nh);
        uint32_t fl = csum_l4_flags(nh);
        uint8_t *w = x->w;
        l4_csum_replace(s, w, l4_off + co, old_port, new_port, 2 | fl);      /* l4_modify_port */
        wbytes(s, w, (uint32_t)l4_off + 2, &new_port, 2);
        if (!v6) {
            uint32_t gw = g_node.ipv4_gateway, od; memcpy(&od, orig_dip, 4);
            wbytes(s, w, 30, &gw, 4);
            l3_csum_replace(s, w, ETH_HLEN + 10, od, gw, 4);
            if (co) l4_csum_replace(s, w, l4_off + co, od, gw, 4 | BPF_F_PSEUDO_HDR | fl);
        } else {
            wbytes(s, w, 38, g_node.host_ip6, 16);                           /* ipv6_store_daddr */
            if (co) l4_csum_replace(s, w, l4_off + co, 0, ck_diff(orig_dip, g_node.host_ip6, 16), BPF_F_PSEUDO_HDR | fl);
        }
    }
    uint8_t *e = x->plog;
    if (!e) return;
    memset(e, 0, O_PLOG);
    e[0] = v6 ? 6 : 4;
    if (x->mark) *x->mark = 1;
    uint8_t *k = e + 4, *v = e + 28;
    int a = v6 ? 16 : 4;
    memcpy(k, t, a);                                  /* .saddr = tuple->daddr */
    memcpy(k + a, &new_port, 2);                      /* .dport = new_port */
    memcpy(k + a + 2, &sport, 2);                     /* .sport = tuple->sport */
    k[a + 4] = nh;
    uint32_t lt = now + PROXY_DEFAULT_LIFETIME;       /* proxy{4,6}_update_timeout */
    memcpy(v, orig_dip, a);
    memcpy(v + a, &old_port, 2);
    memcpy(v + a + 4, &identity, 4);
    memcpy(v + a + 8, &lt, 4);
}

/* The logged cilium_proxy{4,6} updates of a batch, in batch order: each is the
 * map_update_elem(BPF_ANY) of lxc.h:137/:199.  The maps change only through
 * these updates while a batch runs, so the outcome of update i (E2BIG ->
 * DROP_PROXYMAP_CREATE_FAILED) is the one sequential execution gives.  A failed
 * packet's verdict is patched; a successful one gets the MAC stores of
 * ipv{4,6}_policy that follow the redirect (bpf_lxc.c:840-846, 955-961). */
static void proxy_apply_one(const o_batch *b, const uint8_t *plog, o_ingress_out *out, uint8_t *wsnap, uint32_t i) {
    const uint8_t *e = plog + (size_t)i * O_PLOG;
    if (!e[0]) return;
    om_map *m = e[0] == 4 ? g_node.proxy4_map : g_node.proxy6_map;
    int r = m ? om_update(m, e + 4, e + 28, 0) : 0;
    if (r < 0) {
        out[i].action = TC_ACT_SHOT; out[i].reason = (uint8_t)(-DROP_PROXYMAP_CREATE_FAILED_);
        out[i].flags &= 2; out[i].proxy_port = 0; out[i].ifindex_lo = 0;
    } else if (wsnap) {
        skb_t s; skb_init(&s, b, i);
        uint8_t *w = wsnap + (size_t)i * b->snap_stride;
        wbytes(&s, w, 6, g_node.node_mac, 6);      /* eth_store_saddr(NODE_MAC) */
        wbytes(&s, w, 0, g_node.host_mac, 6);      /* eth_store_daddr(HOST_IFINDEX_MAC) */
    }
}
static void proxy_apply(const o_batch *b, const uint8_t *plog, const uint8_t *mark, o_ingress_out *out, uint8_t *wsnap) {
    for (uint32_t i = 0; i < b->n; i++) if (mark[i]) proxy_apply_one(b, plog, out, wsnap, i);
}
/* a batch's proxy log: n zeroed O_PLOG entries (mapped on first write) + n marks */
typedef struct plog_t { uint8_t *log, *mark; } plog_t;
static plog_t plog_new(uint32_t n) {
    plog_t p = {(uint8_t *)calloc((size_t)n + 1, O_PLOG), (uint8_t *)calloc((size_t)n + 1, 1)};
    return p;
}
static void plog_free(plog_t p) { free(p.log); free(p.mark); }

/* ipv4_policy, bpf/bpf_lxc.c:865-970 */
static int ipv4_policy(const o_lxc_cfg *c, skb_t *s, uint32_t src_label, int *fwd, uint32_t now, uint8_t *oflags,
                       uint16_t *proxy, pol_ctx *x) {
    if (s->len < ETH_HLEN + 20) return DROP_INVALID;
    s->cb[2] = 0;                                      /* policy_clear_mark */
    uint8_t t[14]; memset(t, 0, sizeof t);
    t[12] = skb_byte(s, 23);
    int skip_proxy = s->tc_index & 1;
    uint32_t daddr = rd32(s, 30), saddr = rd32(s, 26);
    se32(t, 0, daddr); se32(t, 4, saddr);
    uint32_t orig_sip = saddr;
    int l4_off = ETH_HLEN + (skb_byte(s, 14) & 0xf) * 4;
    ct_state_t st; memset(&st, 0, sizeof st);
    int acct = (c->flags & LXC_F_CT_ACCOUNTING) != 0;
    int ret = ct_lookup(c->ct_map4, t, s, l4_off, CT_INGRESS, &st, 0, now, acct);
    if (ret < 0) return ret;
    *fwd = ret;
    if (ret == CT_REPLY && st.rev_nat_index && !st.loopback) {
        uint8_t *nat = om_lookup_ptr(c->revnat4_map, &st.rev_nat_index);
        if (nat) {
            int r2 = lb_rev_nat_checks(s, l4_off, t[12], ge16(nat, 4), 0);
            if (IS_ERR(r2)) return r2;
            if (x->w) rev_nat_write(s, x->w, l4_off, t[12], nat, ge16(nat, 4), t + 4, 0);
            memcpy(t + 4, nat, 4);                     /* tuple->saddr = nat->address */
        }
    }
    int verdict = policy_can_access_ingress(c, s, src_label, ge16(t, 8), t[12], 0, (const uint8_t *)&orig_sip);
    if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
        if (ret == CT_ESTABLISHED) om_delete(c->ct_map4, t);   /* ct_delete4 */
        return DROP_POLICY;
    }
    if (skip_proxy) verdict = 0;
    if (ret == CT_NEW) {
        ct_state_t sn; memset(&sn, 0, sizeof sn);
        sn.orig_dport = ge16(t, 8); sn.src_sec_id = src_label;
        ret = ct_create(c->ct_map4, t, s, CT_INGRESS, &sn, 0, now);
        if (IS_ERR(ret)) return ret;
        *oflags |= 2;
    }
    if (verdict > 0 && (ret == CT_NEW || ret == CT_ESTABLISHED)) {
        /* ipv4_redirect_to_host_port: traced before its rewrites (lib/lxc.h:115-117) */
        if (c->flags & LXC_F_TRACE_NOTIFY)
            trace_event(s, TRACE_TO_PROXY, (uint16_t)c->lxc_id, c->seclabel, 0, 0, g_host_ifindex, (uint8_t)*fwd);
        ret = redirect_to_host_port_checks(s, l4_off, t[12]);
        if (IS_ERR(ret)) return ret;
        redirect_write(s, x, l4_off, t, 0, (uint16_t)verdict, (const uint8_t *)&daddr, src_label, now);
        s->cb[1] = g_host_ifindex;
        *oflags |= 1;
        *proxy = (uint16_t)verdict;
    }
    return 0;
}

/* ipv6_policy, bpf/bpf_lxc.c:745-862 */
static int ipv6_policy(const o_lxc_cfg *c, skb_t *s, uint32_t src_label, int *fwd, uint32_t now, uint8_t *oflags,
                       uint16_t *proxy, pol_ctx *x) {
    if (s->len < ETH_HLEN + 40) return DROP_INVALID;
    s->cb[2] = 0;
    uint8_t t[40]; memset(t, 0, sizeof t);
    t[36] = skb_byte(s, 20);
    for (int k = 0; k < 16; k++) { t[k] = skb_byte(s, 38 + k); t[16 + k] = skb_byte(s, 22 + k); }
    int skip_proxy = s->tc_index & 1;
    int l4_off = ETH_HLEN + ipv6_hdrlen(s, ETH_HLEN, &t[36]);
    uint16_t csum_off = csum_l4_offset(t[36]);
    ct_state_t st, sn; memset(&st, 0, sizeof st); memset(&sn, 0, sizeof sn);
    uint32_t p4 = ge32(t, 12);                         /* ip6->daddr.s6_addr32[3] */
    sn.rev_nat_index = (uint16_t)(p4 & 0xFFFF);
    uint8_t orig_dip[16]; memcpy(orig_dip, t, 16);
    if (sn.rev_nat_index) {                            /* dip.p4 &= ~0xFFFF; ipv6_store_daddr */
        static const uint8_t z2[2] = {0, 0};
        wbytes(s, x->w, 38 + 12, z2, 2);
        if (csum_off && l4_csum_replace_chk(s, l4_off + csum_off) < 0) return DROP_CSUM_L4;
        if (csum_off) {                                /* csum_diff(&rev_nat_index, 4, &zero_nat, 4) */
            uint32_t rn = sn.rev_nat_index, zero = 0;
            l4_csum_replace(s, x->w, l4_off + csum_off, 0, ck_diff((const uint8_t *)&rn, (const uint8_t *)&zero, 4),
                            BPF_F_PSEUDO_HDR | csum_l4_flags(t[36]));
        }
    }
    int acct = (c->flags & LXC_F_CT_ACCOUNTING) != 0;
    int ret = ct_lookup(c->ct_map6, t, s, l4_off, CT_INGRESS, &st, 1, now, acct);
    if (ret < 0) return ret;
    *fwd = ret;
    if (st.rev_nat_index) {
        uint8_t *nat = om_lookup_ptr(c->revnat6_map, &st.rev_nat_index);
        if (nat) {
            int r2 = lb_rev_nat_checks(s, l4_off, t[36], ge16(nat, 16), 1);
            if (IS_ERR(r2)) return r2;
            if (x->w) {                                /* flags 0: the old saddr is the frame's */
                uint8_t os[16];
                for (int k = 0; k < 16; k++) os[k] = skb_byte(s, 22 + k);
                rev_nat_write(s, x->w, l4_off, t[36], nat, ge16(nat, 16), os, 1);
            }
        }
    }
    int verdict = policy_can_access_ingress(c, s, src_label, ge16(t, 32), t[36], 1, t + 16);
    if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
        if (ret == CT_ESTABLISHED) om_delete(c->ct_map6, t);
        return DROP_POLICY;
    }
    if (skip_proxy) verdict = 0;
    if (ret == CT_NEW) {
        sn.orig_dport = ge16(t, 32); sn.src_sec_id = src_label;
        ret = ct_create(c->ct_map6, t, s, CT_INGRESS, &sn, 1, now);
        if (IS_ERR(ret)) return ret;
        *oflags |= 2;
    }
    if (verdict > 0 && (ret == CT_NEW || ret == CT_ESTABLISHED)) {
        if (c->flags & LXC_F_TRACE_NOTIFY)                 /* lib/lxc.h:167-169 */
            trace_event(s, TRACE_TO_PROXY, (uint16_t)c->lxc_id, c->seclabel, 0, 0, g_host_ifindex, (uint8_t)*fwd);
        ret = redirect_to_host_port_checks(s, l4_off, t[36]);
        if (IS_ERR(ret)) return ret;
        redirect_write(s, x, l4_off, t, 1, (uint16_t)verdict, orig_dip, src_label, now);
        s->cb[1] = g_host_ifindex;
        *oflags |= 1;
        *proxy = (uint16_t)verdict;
    }
    return 0;
}

/* handle_policy, bpf/bpf_lxc.c:980-1024 */
static void handle_policy_skb(const o_prog_array *a, skb_t s, uint32_t lxc_id, uint32_t now, o_ingress_out *o,
                              pol_ctx *x) {
    memset(o, 0, sizeof *o);
    const o_lxc_cfg *c = a->slot[lxc_id & 0xffff];
    if (!c) {                                          /* tail_call miss -> caller's DROP_MISSED_TAIL_CALL */
        o->action = TC_ACT_SHOT; o->reason = (uint8_t)(-DROP_MISSED_TAIL_CALL);
        return;
    }
    uint32_t src_label = s.cb[0], entry_ifindex = s.cb[1];
    int fwd = 0, ret;
    uint8_t fl = 0;
    uint16_t proxy = 0;
    if (c->flags & LXC_F_DROP_ALL) ret = DROP_POLICY;
    else if (s.protocol == 0x86DD) ret = ipv6_policy(c, &s, src_label, &fwd, now, &fl, &proxy, x);
    else if (s.protocol == 0x0800 && (c->flags & LXC_F_LXC_IPV4)) ret = ipv4_policy(c, &s, src_label, &fwd, now, &fl, &proxy, x);
    else ret = DROP_UNKNOWN_L3;
    o->ct_ret = (uint8_t)fwd;
    o->flags = fl;
    if (ret < 0 || ret == TC_ACT_SHOT) {                /* IS_ERR */
        o->action = TC_ACT_SHOT; o->reason = (uint8_t)(-ret); o->flags = fl & 2;
        if (x->mark) { if (*x->mark) { x->plog[0] = 0; *x->mark = 0; } }   /* no proxy entry for a dropped packet */
        else if (x->plog) x->plog[0] = 0;
        return;
    }
    o->proxy_port = proxy;
    if ((c->flags & LXC_F_TRACE_NOTIFY) && entry_ifindex == s.cb[1])   /* not redirected to host / proxy */
        trace_event(&s, TRACE_TO_LXC, (uint16_t)c->lxc_id, src_label, c->seclabel, (uint16_t)c->lxc_id, entry_ifindex,
                    (uint8_t)fwd);
    uint32_t ifindex = s.cb[1];
    o->ifindex_lo = (uint16_t)ifindex;
    o->action = ifindex ? TC_ACT_REDIRECT : TC_ACT_OK;
}
/* plog: the batch's proxy log (n * O_PLOG); wsnap: writable frames (pipeline) */
static void handle_policy(const o_prog_array *a, const o_batch *b, uint32_t i, uint32_t now, o_ingress_out *o,
                          plog_t plog, uint8_t *wsnap) {
    skb_t s; skb_init(&s, b, i);
    s.cb[0] = b->src_identity ? b->src_identity[i] : 0;
    s.cb[1] = b->ifindex ? b->ifindex[i] : 0;
    pol_ctx x = {wsnap ? wsnap + (size_t)i * b->snap_stride : NULL, plog.log + (size_t)i * O_PLOG, plog.mark + i};
    handle_policy_skb(a, s, b->lxc_id ? b->lxc_id[i] : 0, now, o, &x);
}

o_prog_array *o_prog_array_create(void) { return (o_prog_array *)calloc(1, sizeof(o_prog_array)); }
void o_prog_array_destroy(o_prog_array *a) { free(a); }
void o_prog_array_set(o_prog_array *a, uint32_t lxc_id, const o_lxc_cfg *cfg) { a->slot[lxc_id & 0xffff] = cfg; }

void o_ingress_batch(const o_prog_array *a, const o_batch *b, uint32_t now, o_ingress_out *out) {
    plog_t plog = plog_new(b->n);
    for (uint32_t i = 0; i < b->n; i++) handle_policy(a, b, i, now, &out[i], plog, NULL);
    proxy_apply(b, plog.log, plog.mark, out, NULL);
    plog_free(plog);
}

/* ------------------------------------------------------------------ */
/* multi-threaded drivers (CPU baseline)                               */
/* ------------------------------------------------------------------ */
typedef struct mt_arg {
    const o_prog_array *a; const o_batch *b; uint32_t now; o_ingress_out *out;
    const o_xdp_cfg *xc; uint8_t *verdict; const o_lb_cfg *lc; o_lb_out *lo; uint8_t *nd6;
    uint32_t tid, nthreads; int kind;
    /* ingress partition (RSS-style): owner[], per-slice counts, per-owner lists */
    uint32_t *owner, *cnt, *list, *start;
    int phase;
    const uint8_t *skip;                /* pipeline: packets that never reach handle_policy */
    plog_t plog;                        /* proxy log */
    uint8_t *wsnap;                     /* writable frames (pipeline) */
    /* pipeline front pass (kind 3) */
    const o_pipeline_cfg *pc; o_pipeline_out *po; uint8_t *snap_out, *skip_w;
    uint32_t *secctx, *ifx; uint16_t *lxcid;
    o_node_cfg node;                    /* the caller's node config (thread-local g_node) */
    o_trace_sink tr;                    /* the caller's trace sink (thread-local g_tr) */
} mt_arg;

static void pipeline_front(const o_pipeline_cfg *c, const o_batch *b, uint32_t i, uint8_t *row, o_pipeline_out *o,
                           uint8_t *nd6, uint32_t *secctx, uint32_t *ifx, uint16_t *lxcid, uint8_t *skip);

/* send_drop_notify + __send_drop_notify, bpf/lib/drop.h:47-107: the 32-B struct
 * drop_notify followed by the first len_cap (<= TRACE_PAYLOAD_LEN) frame bytes. */
static void drop_event(uint8_t *ev, int reason, uint32_t source, uint32_t hash, uint32_t len, uint32_t src,
                       uint32_t dst, uint32_t dst_id, uint32_t ifindex, const uint8_t *frame, uint32_t frame_bytes) {
    memset(ev, 0, O_EVENT_RECORD);
    uint32_t cb1 = (src << 16) | (dst & 0xFFFF);        /* skb->cb[1] */
    uint32_t cap = len < 128 ? len : 128;                /* min(TRACE_PAYLOAD_LEN, skb->len) */
    int error = reason < 0 ? -reason : reason;
    uint16_t src16 = (uint16_t)source;
    uint32_t f[6] = {len, cap, cb1 >> 16, cb1 & 0xFFFF, dst_id, ifindex};
    ev[0] = 1;                                           /* CILIUM_NOTIFY_DROP */
    ev[1] = (uint8_t)error;
    memcpy(ev + 2, &src16, 2);
    memcpy(ev + 4, &hash, 4);
    memcpy(ev + 8, f, 24);
    if (frame) memcpy(ev + 32, frame, cap < frame_bytes ? cap : frame_bytes);
}

static uint32_t pkt_group(const o_batch *b, uint32_t i) {
    const uint8_t *d = b->snap + (size_t)i * b->snap_stride;
    uint32_t len = b->len[i], cap = b->snap_stride < len ? b->snap_stride : len;
    if (cap >= 34 && d[12] == 0x08 && d[13] == 0x00) {
        uint32_t sa, da; memcpy(&sa, d + 26, 4); memcpy(&da, d + 30, 4);
        return o_ct_pair_hash4(sa, da);
    }
    if (cap >= 54 && d[12] == 0x86 && d[13] == 0xDD) return o_ct_pair_hash6(d + 22, d + 38);
    return i * 2654435761u;              /* no CT access: no ordering constraint */
}

static void *mt_worker(void *p) {
    mt_arg *m = (mt_arg *)p;
    g_node = m->node;
    g_tr = m->tr;
    const o_batch *b = m->b;
    uint32_t T = m->nthreads, t = m->tid;
    uint32_t lo = (uint32_t)((uint64_t)b->n * t / T), hi = (uint32_t)((uint64_t)b->n * (t + 1) / T);
    if (m->kind == 0) {
        if (m->phase == 0) {                 /* group -> owner thread, counts per (slice, owner) */
            uint32_t *c = m->cnt + (size_t)t * T;
            for (uint32_t i = lo; i < hi; i++) { uint32_t o = pkt_group(b, i) % T; m->owner[i] = o; c[o]++; }
        } else if (m->phase == 1) {          /* stable scatter into per-owner lists */
            uint32_t pos[1024];
            for (uint32_t u = 0; u < T; u++) pos[u] = m->start[(size_t)t * T + u];
            for (uint32_t i = lo; i < hi; i++) m->list[pos[m->owner[i]]++] = i;
        } else {                             /* each owner runs its flow groups in batch order */
            uint32_t a0 = m->start[t], a1 = m->start[T * T + t];
            for (uint32_t k = a0; k < a1; k++) {
                uint32_t i = m->list[k];
                if (m->skip && m->skip[i]) continue;
                handle_policy(m->a, b, i, m->now, &m->out[i], m->plog, m->wsnap);
            }
        }
    } else if (m->kind == 3) {
        for (uint32_t i = lo; i < hi; i++)
            pipeline_front(m->pc, b, i, m->snap_out + (size_t)i * b->snap_stride, &m->po[i],
                           m->nd6 ? m->nd6 + 16 * (size_t)i : NULL, &m->secctx[i], &m->ifx[i], &m->lxcid[i],
                           &m->skip_w[i]);
    } else {
        for (uint32_t i = lo; i < hi; i++) {
            skb_t s; skb_init(&s, b, i);
            if (m->kind == 1) m->verdict[i] = (uint8_t)xdp_start(m->xc, &s);
            else lb_one(m->lc, &s, &m->lo[i], m->nd6 ? m->nd6 + 16 * (size_t)i : NULL);
        }
    }
    return NULL;
}

static void run_mt(mt_arg *tmpl, uint32_t threads) {
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)calloc(threads, sizeof(pthread_t));
    mt_arg *args = (mt_arg *)calloc(threads, sizeof(mt_arg));
    tmpl->node = g_node;
    tmpl->tr = g_tr;
    for (uint32_t t = 0; t < threads; t++) {
        args[t] = *tmpl; args[t].tid = t; args[t].nthreads = threads;
        pthread_create(&th[t], NULL, mt_worker, &args[t]);
    }
    for (uint32_t t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th); free(args);
}

static void ingress_mt(const o_prog_array *a, const o_batch *b, uint32_t now, o_ingress_out *out, uint32_t threads,
                       const uint8_t *skip, plog_t plog, uint8_t *wsnap) {
    if (threads < 1) threads = 1;
    if (threads > 1024) threads = 1024;
    uint32_t T = threads;
    mt_arg m; memset(&m, 0, sizeof m);
    m.a = a; m.b = b; m.now = now; m.out = out; m.kind = 0; m.skip = skip; m.plog = plog; m.wsnap = wsnap;
    m.owner = (uint32_t *)malloc((size_t)b->n * 4 + 4);
    m.list = (uint32_t *)malloc((size_t)b->n * 4 + 4);
    m.cnt = (uint32_t *)calloc((size_t)T * T, 4);
    /* start: [slice t][owner u] write offsets, then row T*T.. : owner begin/end */
    m.start = (uint32_t *)calloc((size_t)T * T + T + 1, 4);
    m.phase = 0; run_mt(&m, T);
    uint32_t acc = 0;
    for (uint32_t u = 0; u < T; u++) {
        for (uint32_t t = 0; t < T; t++) { m.start[(size_t)t * T + u] = acc; acc += m.cnt[(size_t)t * T + u]; }
    }
    /* owner ranges: begin = start[0*T+u] (slice 0 offset), end = begin of owner u+1 */
    uint32_t *beg = (uint32_t *)malloc((T + 1) * 4);
    for (uint32_t u = 0; u < T; u++) beg[u] = m.start[u];
    beg[T] = acc;
    m.phase = 1; run_mt(&m, T);
    for (uint32_t u = 0; u < T; u++) { m.start[u] = beg[u]; m.start[(size_t)T * T + u] = beg[u + 1]; }
    m.phase = 2; run_mt(&m, T);
    free(beg); free(m.owner); free(m.list); free(m.cnt); free(m.start);
}
void o_ingress_batch_mt(const o_prog_array *a, const o_batch *b, uint32_t now, o_ingress_out *out, uint32_t threads) {
    plog_t plog = plog_new(b->n);
    ingress_mt(a, b, now, out, threads, NULL, plog, NULL);
    proxy_apply(b, plog.log, plog.mark, out, NULL);
    plog_free(plog);
}
void o_xdp_batch_mt(const o_xdp_cfg *cfg, const o_batch *b, uint8_t *verdict, uint32_t threads) {
    mt_arg m; memset(&m, 0, sizeof m);
    m.b = b; m.xc = cfg; m.verdict = verdict; m.kind = 1;
    run_mt(&m, threads);
}
void o_lb_batch_mt(const o_lb_cfg *cfg, const o_batch *b, o_lb_out *out, uint8_t *nd6, uint32_t threads) {
    mt_arg m; memset(&m, 0, sizeof m);
    m.b = b; m.lc = cfg; m.lo = out; m.nd6 = nd6; m.kind = 2;
    run_mt(&m, threads);
}

/* ------------------------------------------------------------------ */
/* Checksum arithmetic of the helpers the header rewrites call: Linux   */
/* net/core/filter.c bpf_l3_csum_replace / bpf_l4_csum_replace /        */
/* bpf_csum_diff over include/net/checksum.h (generic forms; not in     */
/* /root/reference).  Operands are the raw little-endian loads of the   */
/* network-order bytes, exactly what the BPF programs pass.  The skb is */
/* taken as not CHECKSUM_PARTIAL (a received frame).                    */
/* ------------------------------------------------------------------ */
#define BPF_F_MARK_MANGLED_0 (1u << 5)
#define ENDPOINT_F_HOST 1u
#define WORLD_ID 2u
#define O_NETDEV_TAILCALL 1000
#define O_NETDEV_ICMP6_TE 1001
#define O_PIPE_F_ICMP6_TE 0x20
#define O_PIPE_F_LB 0x40
#define O_PIPE_F_PORTMAP 0x80

static inline uint32_t ck_add(uint32_t a, uint32_t b) { uint32_t r = a + b; return r + (r < b); }   /* csum_add */
static inline uint32_t ck_sub(uint32_t a, uint32_t b) { return ck_add(a, ~b); }                   /* csum_sub */
static inline uint16_t ck_fold(uint32_t x) {                                                      /* csum_fold */
    x = (x & 0xffff) + (x >> 16); x = (x & 0xffff) + (x >> 16); return (uint16_t)~x;
}
static inline uint16_t ck16_add(uint16_t a, uint16_t b) { uint16_t r = (uint16_t)(a + b); return (uint16_t)(r + (r < b)); }
/* bpf_csum_diff(from, n, to, n, 0): ones' complement sum of ~from and to words */
static uint32_t ck_diff(const uint8_t *from, const uint8_t *to, int n) {
    uint32_t x = 0;
    for (int k = 0; k < n; k += 4) {
        uint32_t f, t; memcpy(&f, from + k, 4); memcpy(&t, to + k, 4);
        x = ck_add(x, ~f); x = ck_add(x, t);
    }
    return x;
}
static uint32_t csum_l4_flags(uint8_t nexthdr) { return nexthdr == IPPROTO_UDP ? BPF_F_MARK_MANGLED_0 : 0; }  /* csum.h:52-55 */

/* writes into the frame copy w (bytes past the snap are not kept) */
static void wbytes(const skb_t *s, uint8_t *w, uint32_t off, const void *from, uint32_t n) {
    if (!w) return;
    for (uint32_t k = 0; k < n; k++) if (off + k < s->cap) w[off + k] = ((const uint8_t *)from)[k];
}
/* bpf_skb_store_bytes */
static int skb_store_bytes(const skb_t *s, uint8_t *w, int32_t off, const void *from, uint32_t n) {
    if (skb_writable(s, off, n) < 0) return -EFAULT;
    wbytes(s, w, (uint32_t)off, from, n);
    return 0;
}
/* bpf_l3_csum_replace */
static int l3_csum_replace(const skb_t *s, uint8_t *w, int32_t off, uint32_t from, uint32_t to, uint32_t flags) {
    if (l4_csum_replace_chk(s, off) < 0) return -EFAULT;      /* offset > 0xffff || odd || past len */
    uint16_t sum = rd16(s, (uint32_t)off);
    switch (flags & 0xf) {
    case 0: if (from) return -EINVAL; sum = ck_fold(ck_add(to, ~(uint32_t)sum)); break;          /* csum_replace_by_diff */
    case 2: sum = (uint16_t)~ck16_add(ck16_add((uint16_t)~sum, (uint16_t)~(uint16_t)from), (uint16_t)to); break; /* csum_replace2 */
    case 4: sum = ck_fold(ck_add(ck_sub(~(uint32_t)sum, from), to)); break;                     /* csum_replace4 */
    default: return -EINVAL;
    }
    wbytes(s, w, (uint32_t)off, &sum, 2);
    return 0;
}
/* bpf_l4_csum_replace (inet_proto_csum_replace{4,2,_by_diff}) */
static int l4_csum_replace(const skb_t *s, uint8_t *w, int32_t off, uint32_t from, uint32_t to, uint32_t flags) {
    if (l4_csum_replace_chk(s, off) < 0) return -EFAULT;
    uint16_t sum = rd16(s, (uint32_t)off);
    int mmzero = (flags & BPF_F_MARK_MANGLED_0) != 0;
    if (mmzero && !sum) return 0;
    switch (flags & 0xf) {
    case 0: if (from) return -EINVAL; sum = ck_fold(ck_add(to, ~(uint32_t)sum)); break;
    case 2: case 4: sum = ck_fold(ck_add(ck_sub(~(uint32_t)sum, from), to)); break;
    default: return -EINVAL;
    }
    if (mmzero && !sum) sum = 0xffff;                         /* CSUM_MANGLED_0 */
    wbytes(s, w, (uint32_t)off, &sum, 2);
    return 0;
}

/* lb4_xlate / lb6_xlate writes (bpf/lib/lb.h:615-659, 397-423) for a
 * translation lb_one_res accepted (its checks already passed, so every
 * helper below succeeds). */
static void lb_rewrite(const skb_t *s, uint8_t *w, const lb_res *r, int v6) {
    uint8_t nexthdr;
    int l4_off;
    uint8_t old[16], nw[16];
    uint32_t sum;
    if (!v6) {
        nexthdr = skb_byte(s, 23);
        l4_off = ETH_HLEN + (skb_byte(s, 14) & 0xf) * 4;
        for (int k = 0; k < 4; k++) old[k] = skb_byte(s, 30 + k);
        memcpy(nw, &r->new_daddr4, 4);
        wbytes(s, w, 30, nw, 4);                                        /* daddr */
        sum = ck_diff(old, nw, 4);
        l3_csum_replace(s, w, ETH_HLEN + 10, 0, sum, 0);
    } else {
        nexthdr = skb_byte(s, 20);
        l4_off = ETH_HLEN + ipv6_hdrlen(s, ETH_HLEN, &nexthdr);
        for (int k = 0; k < 16; k++) old[k] = skb_byte(s, 38 + k);
        memcpy(nw, r->nd6, 16);
        wbytes(s, w, 38, nw, 16);                                       /* ipv6_store_daddr */
        sum = ck_diff(old, nw, 16);
    }
    uint16_t co = csum_l4_offset(nexthdr);
    uint32_t fl = csum_l4_flags(nexthdr);
    if (co || v6) l4_csum_replace(s, w, l4_off + co, 0, sum, BPF_F_PSEUDO_HDR | fl);
    if (r->new_dport) {                                                 /* l4_modify_port, bpf/lib/l4.h:50-60 */
        l4_csum_replace(s, w, l4_off + co, r->key_dport, r->new_dport, 2 | fl);
        wbytes(s, w, (uint32_t)l4_off + 2, &r->new_dport, 2);
    }
}

/* map_lxc_in, bpf/lib/l3.h:71-104, with l4_port_map_in (bpf/lib/l4.h:62-88):
 * every entry is compared against the dport loaded once at the start. */
static int map_lxc_in(const skb_t *s, uint8_t *w, int l4_off, const uint8_t *ep, uint8_t nexthdr, int *mapped,
                      uint16_t *new_dport) {
    uint16_t to0; memcpy(&to0, ep + 48 + 2, 2);
    if (!to0) return 0;
    if (nexthdr != IPPROTO_TCP && nexthdr != IPPROTO_UDP) return 0;
    uint16_t dport;
    if (skb_load_bytes(s, l4_off + 2, &dport, 2) < 0) return DROP_INVALID;
    uint16_t co = csum_l4_offset(nexthdr);
    uint32_t fl = csum_l4_flags(nexthdr);
    for (int i = 0; i < 16; i++) {                                      /* PORTMAP_MAX */
        uint16_t from, to;
        memcpy(&from, ep + 48 + 4 * i, 2); memcpy(&to, ep + 48 + 4 * i + 2, 2);
        if (!to || !from) break;
        if (from != dport) continue;
        if (l4_csum_replace(s, w, l4_off + co, dport, to, 2 | fl) < 0) return DROP_CSUM_L4;
        if (skb_store_bytes(s, w, l4_off + 2, &to, 2) < 0) return DROP_WRITE_ERROR;
        *mapped = 1; *new_dport = to;
    }
    return 0;
}

static const uint8_t *endpoint_val4(om_map *lxc, uint32_t daddr) {
    uint8_t key[20] = {0};
    memcpy(key, &daddr, 4); key[16] = 1;
    return om_lookup_ptr(lxc, key);
}
static const uint8_t *endpoint_val6(om_map *lxc, const uint8_t *daddr) {
    uint8_t key[20] = {0};
    memcpy(key, daddr, 16); key[16] = 2;
    return om_lookup_ptr(lxc, key);
}

typedef struct nd_res { uint32_t secctx, ifindex; uint16_t lxc_id, new_dport; int mapped; } nd_res;

/* the common tail of ipv{4,6}_local_delivery, bpf/lib/l3.h:106-168: MACs, port map, cb[], tail call */
static int local_delivery_tail(const skb_t *s, uint8_t *w, int l4_off, const uint8_t *ep, uint8_t nexthdr,
                               uint32_t seclabel, nd_res *r) {
    if (skb_store_bytes(s, w, 6, ep + 24, 6) < 0) return DROP_WRITE_ERROR;   /* eth_store_saddr(node_mac) */
    if (skb_store_bytes(s, w, 0, ep + 16, 6) < 0) return DROP_WRITE_ERROR;   /* eth_store_daddr(mac) */
    int ret = map_lxc_in(s, w, l4_off, ep, nexthdr, &r->mapped, &r->new_dport);
    if (IS_ERR(ret)) return ret;
    r->secctx = seclabel;                                                   /* cb[CB_SRC_LABEL] */
    memcpy(&r->ifindex, ep, 4);                                             /* cb[CB_IFINDEX] */
    memcpy(&r->lxc_id, ep + 6, 2);                                          /* tail_call(cilium_policy, lxc_id) */
    return O_NETDEV_TAILCALL;
}

/* handle_ipv4 of bpf/bpf_netdev.c:326-393 (no FROM_HOST, no ENCAP_IFINDEX)
 * + ipv4_local_delivery (bpf/lib/l3.h:136-168) + ipv4_l3 / ipv4_dec_ttl
 * (l3.h:54-70, bpf/lib/ipv4.h:30-43) */
static int netdev_ipv4(const o_netdev_cfg *c, const skb_t *s, uint8_t *w, nd_res *r) {
    if (s->len < ETH_HLEN + 20) return DROP_INVALID;
    int l4_off = ETH_HLEN + (skb_byte(s, 14) & 0xf) * 4;
    uint32_t secctx = (c->flags & O_NETDEV_F_FIXED_SECCTX) ? c->fixed_secctx : WORLD_ID;  /* derive_ipv4_sec_ctx */
    uint8_t nexthdr = skb_byte(s, 23);
    const uint8_t *ep = endpoint_val4(c->lxc_map, rd32(s, 30));
    if (!ep) return TC_ACT_OK;
    uint32_t epf; memcpy(&epf, ep + 8, 4);
    if (epf & ENDPOINT_F_HOST) return TC_ACT_OK;
    uint8_t ttl = skb_byte(s, 22);
    if (ttl <= 1) return DROP_INVALID;
    uint8_t nt = (uint8_t)(ttl - 1);
    l3_csum_replace(s, w, ETH_HLEN + 10, ttl, nt, 2);
    skb_store_bytes(s, w, ETH_HLEN + 8, &nt, 1);
    return local_delivery_tail(s, w, l4_off, ep, nexthdr, secctx, r);
}

/* handle_ipv6 of bpf/bpf_netdev.c:160-247 (no HANDLE_NS, FROM_HOST,
 * ENCAP_IFINDEX) + derive_sec_ctx (:50-64) + ipv6_local_delivery
 * (bpf/lib/l3.h:106-134) + ipv6_l3 / ipv6_dec_hoplimit (l3.h:31-52,
 * bpf/lib/ipv6.h:178-193) */
static int netdev_ipv6(const o_netdev_cfg *c, const skb_t *s, uint8_t *w, nd_res *r) {
    if (s->len < ETH_HLEN + 40) return DROP_INVALID;
    uint8_t nexthdr = skb_byte(s, 20);
    int l4_off = ETH_HLEN + ipv6_hdrlen(s, ETH_HLEN, &nexthdr);
    uint32_t fl = WORLD_ID;
    if (c->flags & O_NETDEV_F_FIXED_SECCTX) fl = c->fixed_secctx;
    else {
        int match = 1;
        for (int k = 0; k < 8; k++) if (skb_byte(s, 22 + k) != c->router_ip6[k]) match = 0;  /* ipv6_match_prefix_64 */
        if (match) fl = bswap32(rd32(s, 14) & bswap32(0x000FFFFFu));                           /* flow label */
    }
    uint8_t d6[16];
    for (int k = 0; k < 16; k++) d6[k] = skb_byte(s, 38 + k);
    const uint8_t *ep = endpoint_val6(c->lxc_map, d6);
    if (!ep) return TC_ACT_OK;
    uint32_t epf; memcpy(&epf, ep + 8, 4);
    if (epf & ENDPOINT_F_HOST) return TC_ACT_OK;
    uint8_t hl = skb_byte(s, ETH_HLEN + 7);
    if (hl <= 1) return O_NETDEV_ICMP6_TE;              /* icmp6_send_time_exceeded, bpf/lib/icmp6.h:313-322 */
    uint8_t nh = (uint8_t)(hl - 1);
    if (skb_store_bytes(s, w, ETH_HLEN + 7, &nh, 1) < 0) return DROP_WRITE_ERROR;
    return local_delivery_tail(s, w, l4_off, ep, nexthdr, fl, r);
}

/* One packet through bpf_xdp -> bpf_lb from-netdev -> bpf_netdev from-netdev
 * up to the cilium_policy tail call.  row receives the frame as rewritten. */
static void pipeline_front(const o_pipeline_cfg *c, const o_batch *b, uint32_t i, uint8_t *row, o_pipeline_out *o,
                           uint8_t *nd6, uint32_t *secctx, uint32_t *ifx, uint16_t *lxcid, uint8_t *skip) {
    skb_t s; skb_init(&s, b, i);
    memcpy(row, s.data, b->snap_stride);
    s.data = row;
    memset(o, 0, sizeof *o);
    if (nd6) memset(nd6, 0, 16);
    *skip = 1; *secctx = 0; *ifx = 0; *lxcid = 0;
    if (c->xdp && xdp_start(c->xdp, &s) == XDP_DROP) { o->stage = 1; o->action = XDP_DROP; return; }
    if (c->lb) {
        o_lb_out lo; lb_res r; uint8_t n6[16];
        lb_one_res(c->lb, &s, &lo, n6, &r);
        if (lo.action == TC_ACT_SHOT) { o->stage = 2; o->action = TC_ACT_SHOT; o->reason = lo.reason; return; }
        if (lo.slave) {
            int v6 = s.protocol == 0x86DD;
            lb_rewrite(&s, row, &r, v6);
            o->slave = lo.slave; o->rev_nat = lo.rev_nat; o->dport = lo.new_dport; o->daddr4 = lo.new_daddr4;
            o->flags |= O_PIPE_F_LB;
            if (v6 && nd6) memcpy(nd6, n6, 16);
        }
        if (lo.action == TC_ACT_REDIRECT) {
            o->stage = 2; o->action = TC_ACT_REDIRECT; o->ifindex_lo = (uint16_t)c->lb->redirect_ifindex;
            return;
        }
    }
    nd_res nr; memset(&nr, 0, sizeof nr);
    int ret;
    if (c->netdev->flags & NETDEV_F_TRACE_NOTIFY)           /* from_netdev, bpf_netdev.c:436 */
        trace_event(&s, TRACE_FROM_STACK, 0, 0, 0, 0, c->netdev->ingress_ifindex, 0);
    if (s.protocol == 0x86DD) ret = netdev_ipv6(c->netdev, &s, row, &nr);
    else if (s.protocol == 0x0800) ret = netdev_ipv4(c->netdev, &s, row, &nr);   /* tail_handle_ipv4 */
    else ret = TC_ACT_OK;
    if (nr.mapped) { o->flags |= O_PIPE_F_PORTMAP; o->dport = nr.new_dport; }
    o->stage = 3;
    if (ret == O_NETDEV_TAILCALL) {
        o->stage = 4; o->lxc_id = nr.lxc_id;
        *skip = 0; *secctx = nr.secctx; *ifx = nr.ifindex; *lxcid = nr.lxc_id;
    } else if (ret == O_NETDEV_ICMP6_TE) {              /* the reply goes back out: redirect */
        o->action = TC_ACT_REDIRECT; o->flags |= O_PIPE_F_ICMP6_TE;
    } else if (IS_ERR(ret)) {
        o->action = TC_ACT_SHOT; o->reason = (uint8_t)(-ret);
    } else {
        o->action = (uint8_t)ret;
    }
}

void o_pipeline_batch_mt(const o_pipeline_cfg *c, const o_batch *b, uint32_t now, o_pipeline_out *out,
                         uint8_t *nd6, uint8_t *snap_out, uint32_t threads, uint8_t *events) {
    if (threads < 1) threads = 1;
    uint32_t n = b->n;
    uint8_t *snap = snap_out ? snap_out : (uint8_t *)malloc((size_t)n * b->snap_stride + 1);
    uint8_t *skip = (uint8_t *)malloc((size_t)n + 1);
    uint32_t *secctx = (uint32_t *)malloc((size_t)n * 4 + 4), *ifx = (uint32_t *)malloc((size_t)n * 4 + 4);
    uint16_t *lxcid = (uint16_t *)malloc((size_t)n * 2 + 2);
    o_ingress_out *ing = (o_ingress_out *)calloc((size_t)n + 1, sizeof(o_ingress_out));
    mt_arg m; memset(&m, 0, sizeof m);
    m.b = b; m.kind = 3; m.pc = c; m.po = out; m.nd6 = nd6; m.snap_out = snap; m.skip_w = skip;
    m.secctx = secctx; m.ifx = ifx; m.lxcid = lxcid;
    run_mt(&m, threads);
    if (c->policy) {
        /* handle_policy over the rewritten frames, flow groups of the rewritten addresses */
        o_batch b2 = *b;
        b2.snap = snap; b2.src_identity = secctx; b2.ifindex = ifx; b2.lxc_id = lxcid; b2.flow_hash = b->flow_hash;   /* the skb's hash (trace records) */
        plog_t plog = plog_new(n);
        if (threads == 1) {
            for (uint32_t i = 0; i < n; i++) if (!skip[i]) handle_policy(c->policy, &b2, i, now, &ing[i], plog, snap);
        } else {
            ingress_mt(c->policy, &b2, now, ing, threads, skip, plog, snap);
        }
        proxy_apply(&b2, plog.log, plog.mark, ing, snap);
        plog_free(plog);
    }
    for (uint32_t i = 0; i < n; i++) {
        o_pipeline_out *o = &out[i];
        if (!skip[i]) {
            if (!c->policy) { o->action = TC_ACT_SHOT; o->reason = (uint8_t)(-DROP_MISSED_TAIL_CALL); }
            else {
                o->action = ing[i].action; o->reason = ing[i].reason; o->ct_ret = ing[i].ct_ret;
                o->flags |= ing[i].flags; o->proxy_port = ing[i].proxy_port; o->ifindex_lo = ing[i].ifindex_lo;
            }
        }
        if (!events && !g_tr.ev) continue;
        uint8_t tmp[O_EVENT_RECORD];
        uint8_t *e = events ? events + (size_t)i * O_EVENT_RECORD : tmp;
        memset(e, 0, O_EVENT_RECORD);
        if (o->action != TC_ACT_SHOT || o->stage == 1) continue;
        const uint8_t *row = snap + (size_t)i * b->snap_stride;
        uint32_t hash = b->flow_hash ? b->flow_hash[i] : 0, len = b->len[i];
        const o_lxc_cfg *lc = (o->stage == 4 && c->policy) ? c->policy->slot[lxcid[i]] : NULL;
        if (lc) drop_event(e, o->reason, lc->lxc_id, hash, len, secctx[i], lc->seclabel, lc->lxc_id, ifx[i], row,
                           b->snap_stride);
        else drop_event(e, o->reason, 0, hash, len, 0, 0, 0, 0, row, b->snap_stride);
        uint8_t *t = ev_slot(i);
        if (t) memcpy(t, e, O_EVENT_RECORD);
    }
    if (!snap_out) free(snap);
    free(skip); free(secctx); free(ifx); free(lxcid); free(ing);
}
void o_pipeline_batch(const o_pipeline_cfg *c, const o_batch *b, uint32_t now, o_pipeline_out *out,
                      uint8_t *nd6, uint8_t *snap_out) {
    o_pipeline_batch_mt(c, b, now, out, nd6, snap_out, 1, NULL);
}

/* ------------------------------------------------------------------ */
/* ctmap.GC / Flush, pkg/maps/ctmap/ctmap.go:277-368 (GCFilterByTime): */
/* delete every entry whose ct_entry.lifetime (offset 32) < t.          */
/* ------------------------------------------------------------------ */
typedef struct gc_ctx { uint32_t t, n, cap, ksz; uint8_t *keys; } gc_ctx;
static void gc_visit(const void *k, const void *v, void *c_) {
    gc_ctx *c = (gc_ctx *)c_;
    uint32_t lt; memcpy(&lt, (const uint8_t *)v + 32, 4);
    if (lt >= c->t) return;
    if (c->n == c->cap) { c->cap = c->cap ? 2 * c->cap : 1024; c->keys = (uint8_t *)realloc(c->keys, (size_t)c->cap * c->ksz); }
    memcpy(c->keys + (size_t)c->n * c->ksz, k, c->ksz);
    c->n++;
}
uint32_t o_ct_gc(om_map *m, uint32_t filter_time) {
    gc_ctx c = {filter_time, 0, 0, m->ksz, NULL};
    om_foreach(m, gc_visit, &c);
    uint32_t dead = 0;
    for (uint32_t i = 0; i < c.n; i++) if (om_delete(m, c.keys + (size_t)i * c.ksz) == 0) dead++;
    free(c.keys);
    return dead;
}

/* ------------------------------------------------------------------ */
/* LRU stand-in (the CT maps are BPF_MAP_TYPE_LRU_HASH, bpf/bpf_lxc.c:  */
/* 53-75).  The kernel evicts from per-CPU LRU lists — the tail of an   */
/* inactive list kept about as long as the active one — in an order    */
/* that is not reproducible; libgpuflow and this restatement share one  */
/* deterministic rule instead (include/gpuflow.h):        */
/* after a batch, if count > HW = max_entries - max_entries / 8, a hand */
/* sweeping the home lines of libgpuflow's slot array deletes the       */
/* entries of the older half homed in the lines it passes:              */
/*  * age key: 0 if the last use lies before time 0, else closing       */
/*    entries (rx_closing | tx_closing) in [0, 65536), the others in    */
/*    [65536, 131072), by last use in one-second bins relative to now   */
/*    (bin 0 = last used 65535 s or more ago).  Last use = lifetime     */
/*    minus the timeout the entry's flags select (every lifetime writer */
/*    sets it to now + that timeout, conntrack.h:47-62,127,527);        */
/*  * home line: (CT hash of the key & (NS - 1)) / SPL, NS = the slot   */
/*    array (ct_slots: pow2ceil(max(64, 8 or 4 x max_entries))), SPL  */
/*    = 128-B line /                                                    */
/*    slot (4 for ipv4_ct_tuple, 2 for ipv6_ct_tuple); NL = NS / SPL;   */
/*  * sample = entries homed in [hand, hand + SL) (mod NL), SL =        */
/*    max(65536, NL >> 10) (NL when NL <= 65536), the lines the hand    */
/*    passes next; K = the smallest age key with at least half of the  */
/*    sample at or below it, es = the sample's entries with age key     */
/*    <= K; a window holding no entry is replaced by the whole table    */
/*    (SL = NL, hand 0);                                                */
/*  * lines for q entries: ceil(q SL / es);                             */
/*  * round 0 (count > HW): q = count - HW; round 1 (count still >      */
/*    max_entries): q = count - HW; round 2 (count still > max_entries):*/
/*    the rest of the table; each round at most NL - lines so far,      */
/*    deleting every entry with age key <= K homed in [hand, hand +     */
/*    lines) (mod NL); hand += lines.                                   */
/* ------------------------------------------------------------------ */
#define LRU_BINS 65536u
static int64_t ct_last_use(uint32_t lt, uint16_t fl) {
    const uint32_t to = ((fl & 1u) && (fl & 2u)) ? CT_CLOSE_TIMEOUT : ((fl & 16u) ? CT_DEFAULT_LIFETIME : CT_SYN_TIMEOUT);
    return (int64_t)lt - (int64_t)to;
}
static uint32_t lru_age_key(const uint8_t *v, uint32_t now) {
    uint32_t lt; uint16_t fl;
    memcpy(&lt, v + 32, 4); memcpy(&fl, v + 36, 2);
    const int64_t lu = ct_last_use(lt, fl);
    if (lu < 0) return 0u;
    int64_t b = lu - ((int64_t)now - (int64_t)(LRU_BINS - 1));
    b = b < 0 ? 0 : (b > (int64_t)(LRU_BINS - 1) ? (int64_t)(LRU_BINS - 1) : b);
    return ((fl & 3u) ? 0u : LRU_BINS) + (uint32_t)b;
}
/* libgpuflow's CT hash (gf_common.h gf_key_hash, mode CT): a murmur3-style mix
 * of the canonical tuple — addresses and ports unordered, flags without
 * TUPLE_F_IN — as little-endian u32 words. */
static uint32_t gfh_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static uint32_t gfh_words(const uint32_t *w, int nw, uint32_t nbytes) {
    uint32_t h = 0x9747b28cu ^ nbytes;
    for (int i = 0; i < nw; i++) {
        uint32_t k = w[i] * 0xcc9e2d51u;
        k = gfh_rotl(k, 15);
        k *= 0x1b873593u;
        h ^= k;
        h = gfh_rotl(h, 13);
        h = h * 5u + 0xe6546b64u;
    }
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}
static uint32_t gf_ct_hash(const uint8_t *key, uint32_t ksz) {
    uint32_t w[10] = {0};
    memcpy(w, key, ksz);
    if (ksz == 14) {
        const uint32_t a = w[0], b = w[1], p0 = w[2] & 0xffffu, p1 = w[2] >> 16;
        const uint32_t c[4] = {a < b ? a : b, a < b ? b : a, (p0 < p1 ? p0 : p1) | ((p0 < p1 ? p1 : p0) << 16),
                               (w[3] & 0xffu) | (((w[3] >> 8) & 0xfeu) << 8)};
        return gfh_words(c, 4, 14);
    }
    int less = 0;                                   /* word-wise compare of the two addresses */
    for (int i = 0; i < 4; i++) if (w[i] != w[4 + i]) { less = w[i] < w[4 + i]; break; }
    const uint32_t p0 = w[8] & 0xffffu, p1 = w[8] >> 16;
    uint32_t c[10];
    for (int i = 0; i < 4; i++) { c[i] = less ? w[i] : w[4 + i]; c[4 + i] = less ? w[4 + i] : w[i]; }
    c[8] = (p0 < p1 ? p0 : p1) | ((p0 < p1 ? p1 : p0) << 16);
    c[9] = (w[9] & 0xffu) | (((w[9] >> 8) & 0xfeu) << 8);
    return gfh_words(c, 10, 40);
}
typedef struct lru_geo { uint64_t ns, nl, sl; uint32_t spl; } lru_geo;
static lru_geo lru_geometry(const om_map *m) {
    lru_geo g;
    g.ns = ct_slots(m);
    g.spl = m->ksz == 14 ? 4u : 2u;
    g.nl = g.ns / g.spl;
    g.sl = g.nl <= 65536 ? g.nl : ((g.nl >> 10) > 65536 ? (g.nl >> 10) : 65536);
    return g;
}
static uint64_t lru_home_line(const om_map *m, const lru_geo *g, const uint8_t *key) {
    return ((uint64_t)gf_ct_hash(key, m->ksz) & (g->ns - 1)) / g->spl;
}
/* the passes run one thread per shard group */
typedef struct lru_job {
    om_map *m; const lru_geo *g; uint32_t now, s0, s1, K;
    int kill;                                       /* 0: sample histogram, 1: delete */
    uint64_t h0, lines, done;
    uint64_t *hist;
} lru_job;
static void *lru_worker(void *a_) {
    lru_job *a = (lru_job *)a_;
    om_map *m = a->m;
    for (uint32_t s = a->s0; s < a->s1; s++) {
        om_shard *h = &m->sh[s];
        for (uint64_t i = 0; i < h->cap; i++) {
            if (SH_ST(m, h, i) != 1) continue;
            const uint8_t *k = SH_KEY(m, h, i);
            if (!a->kill) {
                const uint64_t hl = lru_home_line(m, a->g, k);
                if ((hl + a->g->nl - a->h0) % a->g->nl < a->lines) a->hist[lru_age_key(SH_VAL(m, h, i), a->now)]++;
                continue;
            }
            if (lru_age_key(SH_VAL(m, h, i), a->now) > a->K) continue;
            const uint64_t hl = lru_home_line(m, a->g, k);
            if ((hl + a->g->nl - a->h0) % a->g->nl >= a->lines) continue;
            SH_ST(m, h, i) = 2; h->used--; h->tomb++;
            a->done++;
        }
    }
    return NULL;
}
static uint64_t lru_pass(om_map *m, const lru_geo *g, uint32_t now, int kill, uint32_t K, uint64_t h0, uint64_t lines,
                         uint64_t *hist) {
    uint32_t nt = m->nshards < 64 ? m->nshards : 64;
    lru_job jobs[64];
    pthread_t th[64];
    for (uint32_t t = 0; t < nt; t++) {
        jobs[t] = (lru_job){m, g, now, m->nshards * t / nt, m->nshards * (t + 1) / nt, K, kill, h0, lines, 0,
                            kill ? NULL : (uint64_t *)calloc(2 * LRU_BINS, sizeof(uint64_t))};
        if (nt > 1) pthread_create(&th[t], NULL, lru_worker, &jobs[t]);
        else lru_worker(&jobs[t]);
    }
    uint64_t done = 0;
    for (uint32_t t = 0; t < nt; t++) {
        if (nt > 1) pthread_join(th[t], NULL);
        done += jobs[t].done;
        if (!kill) {
            for (uint32_t k = 0; k < 2 * LRU_BINS; k++) hist[k] += jobs[t].hist[k];
            free(jobs[t].hist);
        }
    }
    if (kill) __atomic_sub_fetch(&m->count, (uint32_t)done, __ATOMIC_RELAXED);
    return done;
}
/* The hand after a batch: 1 and the log record (age_cut, first line, lines,
 * evicted) if it evicted, else 0.  The hand's position lives in the map. */
int o_ct_lru_evict(om_map *m, uint32_t now, uint32_t *age_cut, uint64_t *hand, uint64_t *lines, uint64_t *evicted) {
    const uint64_t hw = m->max_entries - m->max_entries / 8u;
    if (m->count <= hw) return 0;
    const lru_geo g = lru_geometry(m);
    uint64_t *hist = (uint64_t *)calloc(2 * LRU_BINS, sizeof(uint64_t));
    /* the sample: the window of SL lines ahead of the hand (the histogram pass's
     * "lines" argument is the window size); if no entry is homed there, the
     * whole table */
    uint64_t sl = g.sl, total = 0, acc = 0, es = 0;
    lru_pass(m, &g, now, 0, 0, sl >= g.nl ? 0 : m->lru_hand, sl, hist);
    for (uint32_t k = 0; k < 2 * LRU_BINS; k++) total += hist[k];
    if (!total && sl < g.nl) {
        sl = g.nl;
        lru_pass(m, &g, now, 0, 0, 0, sl, hist);
        for (uint32_t k = 0; k < 2 * LRU_BINS; k++) total += hist[k];
    }
    uint32_t K = 2 * LRU_BINS - 1;
    const uint64_t need = (total + 1) / 2;
    if (total)
        for (uint32_t k = 0; k < 2 * LRU_BINS; k++) { acc += hist[k]; if (acc >= need) { K = k; es = acc; break; } }
    free(hist);
    *age_cut = K; *hand = m->lru_hand; *lines = 0; *evicted = 0;
    for (int round = 0; round < 3; round++) {
        const uint64_t c = m->count;
        if (!(round == 0 ? c > hw : c > m->max_entries) || *lines >= g.nl) continue;
        uint64_t l;
        if (round < 2) {
            const uint64_t q = c - hw;
            l = es ? (q * sl + es - 1) / es : g.nl;         /* es >= 1: the table holds entries */
            if (l > g.nl - *lines) l = g.nl - *lines;
        } else {
            l = g.nl - *lines;
        }
        *evicted += lru_pass(m, &g, now, 1, K, m->lru_hand, l, NULL);
        m->lru_hand = (m->lru_hand + l) % g.nl;
        *lines += l;
    }
    return 1;
}
/* The device's logged eviction replayed (a sampled oracle cannot derive K and
 * the lines from the whole table): deletes entries with age key <= age_cut homed
 * in [hand, hand + lines); returns how many. */
uint64_t o_ct_lru_replay(om_map *m, uint32_t now, uint32_t age_cut, uint64_t hand, uint64_t lines) {
    const lru_geo g = lru_geometry(m);
    const uint64_t ev = lru_pass(m, &g, now, 1, age_cut, hand, lines, NULL);
    m->lru_hand = (hand + lines) % g.nl;
    return ev;
}

/* Drop notifications of an ingress batch: one record per dropped packet, in
 * the packet's slot (ev: n * O_EVENT_RECORD, zero for the others).  Column
 * batches carry no frame bytes to capture. */
void o_ingress_events(const o_prog_array *a, const o_batch *b, const o_ingress_out *out, uint8_t *ev) {
    uint8_t tmp[O_EVENT_RECORD];
    for (uint32_t i = 0; i < b->n; i++) {
        uint8_t *e = ev ? ev + (size_t)i * O_EVENT_RECORD : tmp;
        memset(e, 0, O_EVENT_RECORD);
        if (out[i].action != TC_ACT_SHOT) continue;
        uint32_t hash = b->flow_hash ? b->flow_hash[i] : 0, len = b->len[i];
        const o_lxc_cfg *c = a->slot[(b->lxc_id ? b->lxc_id[i] : 0) & 0xffff];
        if (c) drop_event(e, out[i].reason, c->lxc_id, hash, len, b->src_identity ? b->src_identity[i] : 0,
                          c->seclabel, c->lxc_id, b->ifindex ? b->ifindex[i] : 0, NULL, 0);
        else drop_event(e, out[i].reason, 0, hash, len, 0, 0, 0, 0, NULL, 0);   /* caller's send_drop_notify_error */
        uint8_t *t = ev_slot(i);                         /* after the packet's traces */
        if (t) memcpy(t, e, O_EVENT_RECORD);
    }
}

/* ------------------------------------------------------------------ */
/* Endpoint egress: the from-container program, bpf/bpf_lxc.c:427-738  */
/* ------------------------------------------------------------------ */
#define DROP_INVALID_SMAC -130
#define DROP_INVALID_DMAC -131
#define DROP_INVALID_SIP -132
#define DROP_NO_LXC -152
#define DROP_POLICY_CIDR -162
#define CLUSTER_ID 3u
#define HOST_ID 1u
#define EG_F_CREATED 0x0001
#define EG_F_PROXY 0x0002
#define EG_F_LB 0x0004
#define EG_F_LOOPBACK 0x0008
#define EG_F_REVNAT 0x0010
#define EG_F_PORTMAP 0x0020
#define EG_F_ENCAP 0x0040
#define EG_F_TO_HOST 0x0080
#define EG_F_TO_STACK 0x0100
#define EG_F_LOCAL 0x0200
#define EG_F_DELETED 0x0400
#define EG_F_ARP 0x0800
#define EG_F_IPV6 0x1000
#define O_STAGE_POLICY 4
#define O_STAGE_FROM_LXC 5
#define LXC_F_POLICY_EGRESS (1u << 5)

/* ipv4_l3 (bpf/lib/l3.h:54-70) with ipv4_dec_ttl (bpf/lib/ipv4.h:30-43) */
static int ipv4_l3(const skb_t *s, uint8_t *w, const uint8_t *smac, const uint8_t *dmac) {
    uint8_t ttl = skb_byte(s, 22);
    if (ttl <= 1) return DROP_INVALID;
    uint8_t nt = (uint8_t)(ttl - 1);
    l3_csum_replace(s, w, ETH_HLEN + 10, ttl, nt, 2);
    skb_store_bytes(s, w, ETH_HLEN + 8, &nt, 1);
    if (smac && skb_store_bytes(s, w, 6, smac, 6) < 0) return DROP_WRITE_ERROR;     /* eth_store_saddr */
    if (skb_store_bytes(s, w, 0, dmac, 6) < 0) return DROP_WRITE_ERROR;             /* eth_store_daddr */
    return TC_ACT_OK;
}

/* policy_can_egress4 (bpf/lib/policy.h:241-264 with POLICY_EGRESS, else
 * :282-289) + lookup_ip4_remote_endpoint (bpf/lib/eps.h:60-69) +
 * lpm4_egress_lookup (bpf/lib/maps.h:218-270) */
static int policy_can_egress4(const o_lxc_cfg *c, const skb_t *s, const uint8_t *t, uint16_t dst_id,
                              uint32_t daddr) {
    if (c->flags & LXC_F_DROP_ALL) return DROP_POLICY;
    if (!(c->flags & LXC_F_POLICY_EGRESS)) return TC_ACT_OK;
    uint16_t identity = dst_id;
    if (c->ipcache_map) {
        uint8_t k[20] = {0}; memcpy(k, &daddr, 4); k[16] = 1;
        const uint8_t *info = om_lookup_ptr(c->ipcache_map, k);
        if (info) identity = ge16(info, 0);
    }
    int verdict = __policy_can_access_dir(c, s, identity, ge16(t, 8), t[12], CT_EGRESS);
    if (verdict < 0) verdict = DROP_POLICY;                         /* policy_can_egress */
    if (identity < 256 && verdict < 0) {                             /* identity_is_reserved */
        int hit = 0;
        if (c->cidr4_egress_map) {
            uint8_t k[8]; uint32_t pl = 32; memcpy(k, &pl, 4); memcpy(k + 4, &daddr, 4);
            hit = om_lookup_ptr(c->cidr4_egress_map, k) != NULL;
        }
        verdict = hit ? 0 : DROP_POLICY_CIDR;
    }
    return verdict;
}

/* lb4_rev_nat / __lb4_rev_nat with flags 0 (bpf/lib/lb.h:447-534): the old
 * source address is the frame's; a looped-back flow also restores daddr. */
static int lb4_rev_nat_eg(const o_lxc_cfg *c, const skb_t *s, uint8_t *w, int l4_off, uint8_t *t,
                          const ct_state_t *st) {
    const uint8_t *nat = c->revnat4_map ? om_lookup_ptr(c->revnat4_map, &st->rev_nat_index) : NULL;
    if (!nat) return 0;
    uint8_t nh = t[12];
    uint16_t co = csum_l4_offset(nh);
    uint32_t fl = csum_l4_flags(nh);
    uint16_t port = ge16(nat, 4);
    if (port) {                                                   /* reverse_map_l4_port, lb.h:217-251 */
        switch (nh) {
        case IPPROTO_TCP: case IPPROTO_UDP: {
            uint16_t old;
            int ret = skb_load_bytes(s, l4_off, &old, 2);
            if (IS_ERR(ret)) return ret;
            if (port != old) {
                if (l4_csum_replace(s, w, l4_off + co, old, port, 2 | fl) < 0) return DROP_CSUM_L4;
                if (skb_store_bytes(s, w, l4_off, &port, 2) < 0) return DROP_WRITE_ERROR;
            }
            break;
        }
        case IPPROTO_ICMPV6: case IPPROTO_ICMP: break;
        default: return DROP_UNKNOWN_L4;
        }
    }
    uint32_t old_sip = rd32(s, 26), new_sip = ge32(nat, 0), sum = 0;
    if (st->loopback) {
        uint32_t old_dip = rd32(s, 30);
        if (skb_store_bytes(s, w, 30, &old_sip, 4) < 0) return DROP_WRITE_ERROR;
        sum = ck_diff((const uint8_t *)&old_dip, (const uint8_t *)&old_sip, 4);
        se32(t, 4, old_sip);                                      /* tuple->saddr = old_sip */
    }
    if (skb_store_bytes(s, w, 26, &new_sip, 4) < 0) return DROP_WRITE_ERROR;
    sum = ck_add(sum, ck_diff((const uint8_t *)&old_sip, (const uint8_t *)&new_sip, 4));
    if (l3_csum_replace(s, w, ETH_HLEN + 10, 0, sum, 0) < 0) return DROP_CSUM_L3;
    if (co && l4_csum_replace(s, w, l4_off + co, 0, sum, BPF_F_PSEUDO_HDR | fl) < 0) return DROP_CSUM_L4;
    return 0;
}

typedef struct eg_res { uint32_t ifindex, tunnel_ip; uint16_t proxy, eg_flags, slave, rev_nat; uint8_t ct_ret; } eg_res;

/* handle_ipv4_from_lxc, bpf/bpf_lxc.c:427-658.  w is the frame (s->data == w).
 * Returns TC_ACT_OK / TC_ACT_REDIRECT / O_NETDEV_TAILCALL (ipv4_local_delivery's
 * tail call into cilium_policy, nr filled) or an error. */
static int from_lxc_ipv4(const o_lxc_cfg *c, skb_t *s, uint8_t *w, uint32_t now, eg_res *r, uint8_t *plog,
                         nd_res *nr) {
    if (s->len < ETH_HLEN + 20) return DROP_INVALID;                  /* revalidate_data */
    uint8_t t[14]; memset(t, 0, sizeof t);
    t[12] = skb_byte(s, 23);
    for (int k = 0; k < 6; k++) if (skb_byte(s, 6 + k) != c->lxc_mac[k]) return DROP_INVALID_SMAC;
    for (int k = 0; k < 6; k++) if (skb_byte(s, k) != c->node_mac[k]) return DROP_INVALID_DMAC;
    uint32_t saddr = rd32(s, 26), daddr = rd32(s, 30);
    if (!(c->flags & LXC_F_LXC_IPV4) || saddr != c->lxc_ipv4) return DROP_INVALID_SIP;
    se32(t, 0, daddr); se32(t, 4, saddr);
    int l4_off = ETH_HLEN + (skb_byte(s, 14) & 0xf) * 4;                /* ipv4_hdrlen */
    const uint8_t nh = t[12];
    const uint16_t co = csum_l4_offset(nh);
    const uint32_t fl = csum_l4_flags(nh);
    ct_state_t sn; memset(&sn, 0, sizeof sn);
    uint8_t key[8] = {0}; memcpy(key, &daddr, 4);                      /* lb4_extract_key(CT_EGRESS) */
    int ret = extract_l4_port(s, nh, l4_off, (uint16_t *)(key + 4));   /* LB_L4 */
    if (IS_ERR(ret)) {
        if (ret != DROP_UNKNOWN_L4) return ret;
        goto skip_service_lookup;
    }
    sn.orig_dport = ge16(key, 4);
    if (c->lb4_services) {
        o_lb_cfg lc; memset(&lc, 0, sizeof lc);
        lc.lb4_services = c->lb4_services; lc.flags = LB_F_L3 | LB_F_L4;
        uint8_t *svc = lb4_lookup_service(&lc, key);
        if (svc) {                                                      /* lb4_local, lb.h:662-699 */
            uint16_t count = ge16(svc, 6);
            uint16_t slave = (uint16_t)((s->hash % count) + 1);
            se16(key, 6, slave);
            const uint8_t *be = om_lookup_ptr(c->lb4_services, key);
            if (!be) return DROP_NO_SERVICE;
            r->slave = slave; r->eg_flags |= EG_F_LB;
            sn.rev_nat_index = ge16(be, 8); r->rev_nat = sn.rev_nat_index;
            uint32_t target = ge32(be, 0), new_saddr = 0;
            sn.addr = target;
            if (saddr == target) {                                       /* !DISABLE_LOOPBACK_LB */
                new_saddr = g_node.ipv4_loopback;
                sn.loopback = 1; sn.addr = new_saddr; sn.svc_addr = saddr;
                r->eg_flags |= EG_F_LOOPBACK;
            }
            if (!sn.loopback) se32(t, 0, target);
            /* lb4_xlate, lb.h:615-659 */
            if (skb_store_bytes(s, w, 30, &target, 4) < 0) return DROP_WRITE_ERROR;
            uint32_t sum = ck_diff(key, (const uint8_t *)&target, 4);
            if (new_saddr) {
                if (skb_store_bytes(s, w, 26, &new_saddr, 4) < 0) return DROP_WRITE_ERROR;
                sum = ck_add(sum, ck_diff((const uint8_t *)&saddr, (const uint8_t *)&new_saddr, 4));
            }
            if (l3_csum_replace(s, w, ETH_HLEN + 10, 0, sum, 0) < 0) return DROP_CSUM_L3;
            if (co && l4_csum_replace(s, w, l4_off + co, 0, sum, BPF_F_PSEUDO_HDR | fl) < 0) return DROP_CSUM_L4;
            uint16_t sp = ge16(be, 4), kd = ge16(key, 4);
            if (sp && kd != sp && (nh == IPPROTO_TCP || nh == IPPROTO_UDP)) {   /* l4_modify_port */
                if (l4_csum_replace(s, w, l4_off + co, kd, sp, 2 | fl) < 0) return DROP_CSUM_L4;
                if (skb_store_bytes(s, w, l4_off + 2, &sp, 2) < 0) return DROP_WRITE_ERROR;
            }
        }
    }
skip_service_lookup: ;
    uint32_t orig_dip = ge32(t, 0);
    /* map_lxc_out, bpf_lxc.c:80-108 + l4_port_map_out (bpf/lib/l4.h:107-118) */
    if (c->n_portmap && (nh == IPPROTO_TCP || nh == IPPROTO_UDP)) {
        uint16_t sport;
        if (skb_load_bytes(s, l4_off, &sport, 2) < 0) return DROP_INVALID;
        for (uint32_t k = 0; k < c->n_portmap && k < 16; k++) {
            if (c->portmap[k].to != sport) continue;
            uint16_t from = c->portmap[k].from;
            if (l4_csum_replace(s, w, l4_off + co, sport, from, 2 | fl) < 0) return DROP_CSUM_L4;
            if (skb_store_bytes(s, w, l4_off, &from, 2) < 0) return DROP_WRITE_ERROR;
            r->eg_flags |= EG_F_PORTMAP;
        }
    }
    ct_state_t st; memset(&st, 0, sizeof st);
    const int acct = (c->flags & LXC_F_CT_ACCOUNTING) != 0;
    ret = ct_lookup(c->ct_map4, t, s, l4_off, CT_EGRESS, &st, 0, now, acct);
    if (ret < 0) return ret;
    const int fwd = ret;
    r->ct_ret = (uint8_t)fwd;
    uint16_t dst_id = ((orig_dip & g_node.ipv4_cluster_mask) == g_node.ipv4_cluster_range) ? CLUSTER_ID : WORLD_ID;
    int verdict = policy_can_egress4(c, s, t, dst_id, ge32(t, 4));   /* ipv4_ct_tuple_get_daddr = tuple->saddr */
    if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
        if (ret == CT_ESTABLISHED) { om_delete(c->ct_map4, t); r->eg_flags |= EG_F_DELETED; }
        return verdict;
    }
    switch (ret) {
    case CT_NEW:
        sn.src_sec_id = c->seclabel;
        ret = ct_create(c->ct_map4, t, s, CT_EGRESS, &sn, 0, now);
        if (IS_ERR(ret)) return ret;
        r->eg_flags |= EG_F_CREATED;
        break;
    case CT_ESTABLISHED:
        break;
    case CT_RELATED: case CT_REPLY:
        s->cb[2] = 1;                                                    /* policy_mark_skip */
        if (st.rev_nat_index) {
            ret = lb4_rev_nat_eg(c, s, w, l4_off, t, &st);
            if (IS_ERR(ret)) return ret;
            r->eg_flags |= EG_F_REVNAT;
        }
        break;
    default:
        return DROP_POLICY;
    }
    const int tr = (c->flags & LXC_F_TRACE_NOTIFY) != 0;
    if (verdict > 0) {                                                   /* redirect_to_proxy */
        if (tr) trace_event(s, TRACE_TO_PROXY, (uint16_t)c->lxc_id, c->seclabel, 0, 0, g_node.host_ifindex, (uint8_t)fwd);
        ret = redirect_to_host_port_checks(s, l4_off, nh);
        if (IS_ERR(ret)) return ret;
        pol_ctx x = {w, plog, NULL};
        redirect_write(s, &x, l4_off, t, 0, (uint16_t)verdict, (const uint8_t *)&orig_dip, c->seclabel, now);
        if (plog) plog[1] = 1;                                          /* egress entry: no policy MAC stores */
        r->eg_flags |= EG_F_PROXY; r->proxy = (uint16_t)verdict;
        ret = ipv4_l3(s, w, c->node_mac, g_node.host_mac);
        if (ret != TC_ACT_OK) return ret;
        r->ifindex = g_node.host_ifindex;
        return TC_ACT_REDIRECT;
    }
    orig_dip = rd32(s, 30);
    const uint8_t *ep = g_node.lxc_map ? endpoint_val4(g_node.lxc_map, orig_dip) : NULL;
    if (ep) {
        uint32_t epf; memcpy(&epf, ep + 8, 4);
        if (epf & ENDPOINT_F_HOST) {
            if (!g_node.host_ifindex) return DROP_NO_LXC;
            goto to_host;
        }
        s->cb[2] = 0;                                                    /* policy_clear_mark */
        ret = ipv4_l3(s, w, ep + 24, ep + 16);                           /* ipv4_local_delivery, l3.h:136-168 */
        if (ret != TC_ACT_OK) return ret;
        r->eg_flags |= EG_F_LOCAL;
        return local_delivery_tail(s, w, l4_off, ep, nh, c->seclabel, nr);
    }
    if (g_node.encap_ifindex) {                                          /* encap_and_redirect, lib/encap.h */
        uint8_t k[20] = {0};
        uint32_t a = orig_dip & g_node.ipv4_mask;
        memcpy(k, &a, 4); k[16] = 1;
        const uint8_t *tun = g_node.tunnel_map ? om_lookup_ptr(g_node.tunnel_map, k) : NULL;
        if (tun) {
            r->tunnel_ip = bswap32(ge32(tun, 0));                        /* bpf_htonl(tunnel->ip4) */
            if (tr) trace_event(s, TRACE_TO_OVERLAY, (uint16_t)c->lxc_id, c->seclabel, 0, 0, g_node.encap_ifindex, 0);
            r->ifindex = g_node.encap_ifindex;
            r->eg_flags |= EG_F_ENCAP;
            return TC_ACT_REDIRECT;
        }
    }
    if (dst_id == CLUSTER_ID) s->cb[2] = 1;                              /* policy_mark_skip */
    ret = ipv4_l3(s, w, NULL, c->node_mac);                              /* pass_to_stack */
    if (ret != TC_ACT_OK) return ret;
    if (tr) trace_event(s, TRACE_TO_STACK, (uint16_t)c->lxc_id, c->seclabel, dst_id, 0, 0, (uint8_t)fwd);   /* :669 */
    r->eg_flags |= EG_F_TO_STACK;
    return TC_ACT_OK;
to_host:
    ret = ipv4_l3(s, w, c->node_mac, g_node.host_mac);
    if (ret != TC_ACT_OK) return ret;
    if (tr) trace_event(s, TRACE_TO_HOST, (uint16_t)c->lxc_id, c->seclabel, HOST_ID, 0, g_node.host_ifindex,
                        (uint8_t)fwd);                                   /* :650 */
    r->eg_flags |= EG_F_TO_HOST;
    r->ifindex = g_node.host_ifindex;
    return TC_ACT_REDIRECT;
}

#define EG_F_ICMP6_TE 0x2000
#define EG_F_RESPONDER 0x4000
#define O_EG_RESPONDER 1001
#define O_EG_ICMP6_TE 1002

/* ipv6_l3 (bpf/lib/l3.h:31-52) + ipv6_dec_hoplimit (bpf/lib/ipv6.h:178-193) */
static int ipv6_l3(const skb_t *s, uint8_t *w, const uint8_t *smac, const uint8_t *dmac) {
    uint8_t hl = skb_byte(s, ETH_HLEN + 7);
    if (hl <= 1) return O_EG_ICMP6_TE;                 /* icmp6_send_time_exceeded (a responder) */
    uint8_t nh = (uint8_t)(hl - 1);
    if (skb_store_bytes(s, w, ETH_HLEN + 7, &nh, 1) < 0) return DROP_WRITE_ERROR;
    if (smac && skb_store_bytes(s, w, 6, smac, 6) < 0) return DROP_WRITE_ERROR;
    if (skb_store_bytes(s, w, 0, dmac, 6) < 0) return DROP_WRITE_ERROR;
    return TC_ACT_OK;
}

/* policy_can_egress6 (bpf/lib/policy.h:214-239 with POLICY_EGRESS, else :268-278) */
static int policy_can_egress6(const o_lxc_cfg *c, const skb_t *s, const uint8_t *t, uint16_t dst_id,
                              const uint8_t *daddr) {
    if (c->flags & LXC_F_DROP_ALL) return DROP_POLICY;
    if (!(c->flags & LXC_F_POLICY_EGRESS)) return TC_ACT_OK;
    uint16_t identity = dst_id;
    if (c->ipcache_map) {
        uint8_t k[20] = {0}; memcpy(k, daddr, 16); k[16] = 2;
        const uint8_t *info = om_lookup_ptr(c->ipcache_map, k);
        if (info) identity = ge16(info, 0);
    }
    int verdict = __policy_can_access_dir(c, s, identity, ge16(t, 32), t[36], CT_EGRESS);
    if (verdict < 0) verdict = DROP_POLICY;
    if (identity < 256 && verdict < 0) {
        int hit = 0;
        if (c->cidr6_egress_map) {
            uint8_t k[20]; uint32_t pl = 128; memcpy(k, &pl, 4); memcpy(k + 4, daddr, 16);
            hit = om_lookup_ptr(c->cidr6_egress_map, k) != NULL;
        }
        verdict = hit ? 0 : DROP_POLICY_CIDR;
    }
    return verdict;
}

/* handle_ipv6 (bpf_lxc.c:388-416) -> ipv6_l3_from_lxc (:120-386) */
static int from_lxc_ipv6(const o_lxc_cfg *c, skb_t *s, uint8_t *w, uint32_t now, eg_res *r, uint8_t *plog,
                         nd_res *nr) {
    if (s->len < ETH_HLEN + 40) return DROP_INVALID;
    uint8_t d6[16];
    for (int k = 0; k < 16; k++) d6[k] = skb_byte(s, 38 + k);
    if (skb_byte(s, 20) == IPPROTO_ICMPV6) {
        if (s->len < ETH_HLEN + 40 + 8) return DROP_INVALID;
        uint8_t type = skb_byte(s, ETH_HLEN + 40);              /* icmp6_handle, bpf/lib/icmp6.h:380-401 */
        if (type == 135) return O_EG_RESPONDER;                   /* icmp6_handle_ns (tail call) */
        if (type == 128 && !memcmp(d6, g_node.router_ip6, 16)) return O_EG_RESPONDER;   /* echo reply */
    }
    for (int k = 0; k < 6; k++) if (skb_byte(s, 6 + k) != c->lxc_mac[k]) return DROP_INVALID_SMAC;
    for (int k = 0; k < 6; k++) if (skb_byte(s, k) != c->node_mac[k]) return DROP_INVALID_DMAC;
    for (int k = 0; k < 16; k++) if (skb_byte(s, 22 + k) != c->lxc_ip6[k]) return DROP_INVALID_SIP;
    uint8_t t[40]; memset(t, 0, sizeof t);
    t[36] = skb_byte(s, 20);
    memcpy(t, d6, 16);
    for (int k = 0; k < 16; k++) t[16 + k] = skb_byte(s, 22 + k);
    int l4_off = ETH_HLEN + ipv6_hdrlen(s, ETH_HLEN, &t[36]);    /* added unchecked (bpf_lxc.c:145) */
    const uint8_t nh = t[36];
    const uint16_t co = csum_l4_offset(nh);
    const uint32_t fl = csum_l4_flags(nh);
    ct_state_t sn; memset(&sn, 0, sizeof sn);
    uint8_t key[20] = {0}; memcpy(key, t, 16);                   /* lb6_extract_key(CT_EGRESS) */
    int ret = extract_l4_port(s, nh, l4_off, (uint16_t *)(key + 16));
    if (IS_ERR(ret)) {
        if (ret != DROP_UNKNOWN_L4) return ret;
        goto skip_service_lookup;
    }
    if (c->lb6_services) {
        o_lb_cfg lc; memset(&lc, 0, sizeof lc);
        lc.lb6_services = c->lb6_services; lc.flags = LB_F_L3 | LB_F_L4;
        uint8_t *svc = lb6_lookup_service(&lc, key);
        if (svc) {                                               /* lb6_local, lb.h:425-445 */
            uint16_t count = ge16(svc, 18);
            uint16_t slave = (uint16_t)((s->hash % count) + 1);
            se16(key, 18, slave);
            const uint8_t *be = om_lookup_ptr(c->lb6_services, key);
            if (!be) return DROP_NO_SERVICE;
            r->slave = slave; r->eg_flags |= EG_F_LB;
            memcpy(t, be, 16);                                   /* tuple->daddr = svc->target */
            sn.rev_nat_index = ge16(be, 20); r->rev_nat = sn.rev_nat_index;
            wbytes(s, w, 38, be, 16);                            /* lb6_xlate: ipv6_store_daddr */
            uint32_t sum = ck_diff(key, be, 16);
            if (l4_csum_replace(s, w, l4_off + co, 0, sum, BPF_F_PSEUDO_HDR | fl) < 0) return DROP_CSUM_L4;
            uint16_t sp = ge16(be, 16), kd = ge16(key, 16);
            if (sp && kd != sp && (nh == IPPROTO_TCP || nh == IPPROTO_UDP)) {
                if (l4_csum_replace(s, w, l4_off + co, kd, sp, 2 | fl) < 0) return DROP_CSUM_L4;
                if (skb_store_bytes(s, w, l4_off + 2, &sp, 2) < 0) return DROP_WRITE_ERROR;
            }
        }
    }
skip_service_lookup: ;
    uint8_t orig_dip[16]; memcpy(orig_dip, t, 16);
    if (c->n_portmap && (nh == IPPROTO_TCP || nh == IPPROTO_UDP)) {    /* map_lxc_out */
        uint16_t sport;
        if (skb_load_bytes(s, l4_off, &sport, 2) < 0) return DROP_INVALID;
        for (uint32_t k = 0; k < c->n_portmap && k < 16; k++) {
            if (c->portmap[k].to != sport) continue;
            uint16_t from = c->portmap[k].from;
            if (l4_csum_replace(s, w, l4_off + co, sport, from, 2 | fl) < 0) return DROP_CSUM_L4;
            if (skb_store_bytes(s, w, l4_off, &from, 2) < 0) return DROP_WRITE_ERROR;
            r->eg_flags |= EG_F_PORTMAP;
        }
    }
    ct_state_t st; memset(&st, 0, sizeof st);
    ret = ct_lookup(c->ct_map6, t, s, l4_off, CT_EGRESS, &st, 1, now, (c->flags & LXC_F_CT_ACCOUNTING) != 0);
    if (ret < 0) return ret;
    r->ct_ret = (uint8_t)ret;
    for (int k = 0; k < 16; k++) d6[k] = skb_byte(s, 38 + k);
    uint16_t dst_id = !memcmp(d6, g_node.router_ip6, 8) ? CLUSTER_ID : WORLD_ID;   /* ipv6_match_prefix_64 */
    int verdict = policy_can_egress6(c, s, t, dst_id, t + 16);   /* ipv6_ct_tuple_get_daddr = &tuple->saddr */
    if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
        if (ret == CT_ESTABLISHED) { om_delete(c->ct_map6, t); r->eg_flags |= EG_F_DELETED; }
        return verdict;
    }
    switch (ret) {
    case CT_NEW:
        sn.src_sec_id = c->seclabel;
        ret = ct_create(c->ct_map6, t, s, CT_EGRESS, &sn, 1, now);
        if (IS_ERR(ret)) return ret;
        r->eg_flags |= EG_F_CREATED;
        break;
    case CT_ESTABLISHED:
        break;
    case CT_RELATED: case CT_REPLY:
        s->cb[2] = 1;
        if (st.rev_nat_index) {                                 /* lb6_rev_nat(flags 0), lb.h:253-316 */
            const uint8_t *nat = c->revnat6_map ? om_lookup_ptr(c->revnat6_map, &st.rev_nat_index) : NULL;
            if (nat) {
                uint16_t port = ge16(nat, 16);
                if (port) {
                    switch (nh) {
                    case IPPROTO_TCP: case IPPROTO_UDP: {
                        uint16_t old;
                        int rr = skb_load_bytes(s, l4_off, &old, 2);
                        if (IS_ERR(rr)) return rr;
                        if (port != old) {
                            if (l4_csum_replace(s, w, l4_off + co, old, port, 2 | fl) < 0) return DROP_CSUM_L4;
                            if (skb_store_bytes(s, w, l4_off, &port, 2) < 0) return DROP_WRITE_ERROR;
                        }
                        break;
                    }
                    case IPPROTO_ICMPV6: case IPPROTO_ICMP: break;
                    default: return DROP_UNKNOWN_L4;
                    }
                }
                uint8_t os[16];
                for (int k = 0; k < 16; k++) os[k] = skb_byte(s, 22 + k);
                wbytes(s, w, 22, nat, 16);                       /* ipv6_store_saddr */
                if (l4_csum_replace(s, w, l4_off + co, 0, ck_diff(os, nat, 16), BPF_F_PSEUDO_HDR | fl) < 0)
                    return DROP_CSUM_L4;
            }
            r->eg_flags |= EG_F_REVNAT;
        }
        break;
    default:
        return DROP_POLICY;
    }
    const int tr = (c->flags & LXC_F_TRACE_NOTIFY) != 0;
    const uint8_t fwd = r->ct_ret;                               /* forwarding_reason */
    if (verdict > 0) {                                           /* ipv6_redirect_to_host_port + ipv6_l3 */
        if (tr) trace_event(s, TRACE_TO_PROXY, (uint16_t)c->lxc_id, c->seclabel, 0, 0, g_node.host_ifindex, fwd);
        ret = redirect_to_host_port_checks(s, l4_off, nh);
        if (IS_ERR(ret)) return ret;
        pol_ctx x = {w, plog, NULL};
        redirect_write(s, &x, l4_off, t, 1, (uint16_t)verdict, orig_dip, c->seclabel, now);
        if (plog) plog[1] = 1;
        r->eg_flags |= EG_F_PROXY; r->proxy = (uint16_t)verdict;
        ret = ipv6_l3(s, w, c->node_mac, g_node.host_mac);
        if (ret != TC_ACT_OK) return ret;
        r->ifindex = g_node.host_ifindex;
        return TC_ACT_REDIRECT;
    }
    for (int k = 0; k < 16; k++) d6[k] = skb_byte(s, 38 + k);
    const uint8_t *ep = g_node.lxc_map ? endpoint_val6(g_node.lxc_map, d6) : NULL;
    if (ep) {
        uint32_t epf; memcpy(&epf, ep + 8, 4);
        if (epf & ENDPOINT_F_HOST) {
            if (!g_node.host_ifindex) return DROP_NO_LXC;
            goto to_host;
        }
        s->cb[2] = 0;
        ret = ipv6_l3(s, w, ep + 24, ep + 16);                   /* ipv6_local_delivery, l3.h:106-134 */
        if (ret != TC_ACT_OK) return ret;
        r->eg_flags |= EG_F_LOCAL;
        return local_delivery_tail(s, w, l4_off, ep, nh, c->seclabel, nr);
    }
    if (g_node.encap_ifindex) {                                  /* encap_and_redirect, key daddr/96 */
        uint8_t k[20] = {0};
        memcpy(k, d6, 12); k[16] = 2;
        const uint8_t *tun = g_node.tunnel_map ? om_lookup_ptr(g_node.tunnel_map, k) : NULL;
        if (tun) {
            r->tunnel_ip = bswap32(ge32(tun, 0));
            if (tr) trace_event(s, TRACE_TO_OVERLAY, (uint16_t)c->lxc_id, c->seclabel, 0, 0, g_node.encap_ifindex, 0);
            r->ifindex = g_node.encap_ifindex;
            r->eg_flags |= EG_F_ENCAP;
            return TC_ACT_REDIRECT;
        }
    }
    if (dst_id == CLUSTER_ID) s->cb[2] = 1;
    ret = ipv6_l3(s, w, NULL, c->node_mac);                      /* pass_to_stack */
    if (ret != TC_ACT_OK) return ret;
    {                                                            /* ipv6_store_flowlabel(SECLABEL_NB) */
        uint32_t old;
        if (skb_load_bytes(s, ETH_HLEN, &old, 4) < 0) return DROP_INVALID;
        old &= bswap32(0x0FF00000u);
        old = bswap32(0x60000000u) | bswap32(c->seclabel) | old;
        if (skb_store_bytes(s, w, ETH_HLEN, &old, 4) < 0) return DROP_WRITE_ERROR;
    }
    if (tr) trace_event(s, TRACE_TO_STACK, (uint16_t)c->lxc_id, c->seclabel, dst_id, 0, 0, fwd);   /* :381 */
    r->eg_flags |= EG_F_TO_STACK;
    return TC_ACT_OK;
to_host:
    ret = ipv6_l3(s, w, c->node_mac, g_node.host_mac);
    if (ret != TC_ACT_OK) return ret;
    if (tr) trace_event(s, TRACE_TO_HOST, (uint16_t)c->lxc_id, c->seclabel, HOST_ID, 0, g_node.host_ifindex, fwd);  /* :364 */
    r->eg_flags |= EG_F_TO_HOST;
    r->ifindex = g_node.host_ifindex;
    return TC_ACT_REDIRECT;
}

/* handle_ingress (from-container, bpf_lxc.c:685-738) + tail_handle_ipv4 (:659-668) */
static void from_container(const o_prog_array *a, const o_batch *b, uint32_t i, uint32_t now, o_egress_out *o,
                           uint8_t *row, uint8_t *plog, uint8_t *skip, uint32_t *secctx, uint32_t *ifx,
                           uint16_t *lxcid) {
    skb_t s; skb_init(&s, b, i);
    memcpy(row, s.data, b->snap_stride);
    s.data = row;
    memset(o, 0, sizeof *o);
    *skip = 1; *secctx = 0; *ifx = 0; *lxcid = 0;
    if (plog) memset(plog, 0, O_PLOG);
    const o_lxc_cfg *c = a->slot[(b->lxc_id ? b->lxc_id[i] : 0) & 0xffff];
    o->stage = O_STAGE_FROM_LXC;
    if (!c) { o->action = TC_ACT_SHOT; o->reason = (uint8_t)(-DROP_MISSED_TAIL_CALL); return; }
    if (c->flags & LXC_F_TRACE_NOTIFY)                   /* handle_ingress, bpf_lxc.c:705 */
        trace_event(&s, TRACE_FROM_LXC, (uint16_t)c->lxc_id, c->seclabel, 0, 0, 0, 0);
    int ret;
    eg_res r; memset(&r, 0, sizeof r);
    nd_res nr; memset(&nr, 0, sizeof nr);
    if (s.protocol == 0x0806) {                  /* tail_handle_arp: the ARP responder (out of scope) */
        o->stage = 0; o->eg_flags = EG_F_ARP; return;
    }
    if (c->flags & LXC_F_DROP_ALL) ret = DROP_POLICY;
    else if (s.protocol == 0x86DD) { r.eg_flags = EG_F_IPV6; ret = from_lxc_ipv6(c, &s, row, now, &r, plog, &nr); }
    else if (s.protocol == 0x0800) ret = from_lxc_ipv4(c, &s, row, now, &r, plog, &nr);
    else ret = DROP_UNKNOWN_L3;
    if (ret == O_EG_RESPONDER) { o->stage = 0; o->eg_flags = EG_F_IPV6 | EG_F_RESPONDER; return; }
    if (ret == O_EG_ICMP6_TE) {                  /* ipv6_l3 -> icmp6_send_time_exceeded: the reply goes back out */
        r.eg_flags |= EG_F_ICMP6_TE; r.eg_flags &= (uint16_t)~(EG_F_LOCAL | EG_F_TO_STACK | EG_F_TO_HOST);
        ret = TC_ACT_REDIRECT; r.ifindex = 0;
    }
    o->eg_ct_ret = r.ct_ret; o->ct_ret = r.ct_ret;
    o->slave = r.slave; o->rev_nat = r.rev_nat; o->eg_flags = r.eg_flags;
    if (ret == O_NETDEV_TAILCALL) {
        o->stage = O_STAGE_POLICY; o->lxc_id = nr.lxc_id; o->ct_ret = 0;
        *skip = 0; *secctx = nr.secctx; *ifx = nr.ifindex; *lxcid = nr.lxc_id;
        if (plog) plog[0] = 0;
        return;
    }
    if (IS_ERR(ret)) {                           /* send_drop_notify(SECLABEL, 0, 0, 0, ret, TC_ACT_SHOT) */
        o->action = TC_ACT_SHOT; o->reason = (uint8_t)(-ret);
        /* a cilium_proxy4 entry written by ipv4_redirect_to_host_port stays when
         * the ipv4_l3 that follows it drops the packet (lxc.h:137 before l3.h:54) */
        if (plog && !(r.eg_flags & EG_F_PROXY)) plog[0] = 0;
        o->eg_flags &= (uint16_t)(EG_F_CREATED | EG_F_DELETED | EG_F_LB | EG_F_LOOPBACK | EG_F_PORTMAP | EG_F_REVNAT |
                                  EG_F_IPV6);
        return;
    }
    o->action = (uint8_t)ret;
    o->proxy_port = r.proxy; o->ifindex_lo = (uint16_t)r.ifindex; o->tunnel_ip = r.tunnel_ip;
}

void o_egress_batch(const o_prog_array *a, const o_batch *b, uint32_t now, o_egress_out *out, uint8_t *snap_out,
                    uint8_t *events) {
    const uint32_t n = b->n;
    uint8_t *snap = snap_out ? snap_out : (uint8_t *)malloc((size_t)n * b->snap_stride + 1);
    uint8_t *skip = (uint8_t *)malloc((size_t)n + 1);
    uint32_t *secctx = (uint32_t *)malloc((size_t)n * 4 + 4), *ifx = (uint32_t *)malloc((size_t)n * 4 + 4);
    uint16_t *lxcid = (uint16_t *)malloc((size_t)n * 2 + 2);
    uint8_t *plog = (uint8_t *)calloc((size_t)n + 1, O_PLOG);
    plog_t plog2 = plog_new(n);
    o_ingress_out *ing = (o_ingress_out *)calloc((size_t)n + 1, sizeof(o_ingress_out));
    o_batch b2 = *b;                                   /* the local deliveries, over the rewritten frames */
    b2.snap = snap; b2.src_identity = secctx; b2.ifindex = ifx; b2.lxc_id = lxcid; b2.flow_hash = b->flow_hash;   /* the skb's hash (trace records) */
    /* One packet at a time, as on one CPU: the from-container program, its
     * cilium_proxy{4,6} update (lxc.h:137), then — for a local delivery — the
     * destination's handle_policy (the tail call of ipv4_local_delivery) and its
     * proxy update, before the next packet. */
    for (uint32_t i = 0; i < n; i++) {
        from_container(a, b, i, now, &out[i], snap + (size_t)i * b->snap_stride, plog + (size_t)i * O_PLOG, &skip[i],
                       &secctx[i], &ifx[i], &lxcid[i]);
        const uint8_t *e = plog + (size_t)i * O_PLOG;
        if (e[0]) {
            om_map *m = e[0] == 4 ? g_node.proxy4_map : g_node.proxy6_map;
            if (m && om_update(m, e + 4, e + 28, 0) < 0) {
                o_egress_out *o = &out[i];
                o->action = TC_ACT_SHOT; o->reason = (uint8_t)(-DROP_PROXYMAP_CREATE_FAILED_);
                o->flags &= (uint8_t)~1u; o->proxy_port = 0; o->ifindex_lo = 0;
            }
        }
        if (skip[i]) continue;
        handle_policy(a, &b2, i, now, &ing[i], plog2, snap);
        proxy_apply_one(&b2, plog2.log, ing, snap, i);
        o_egress_out *o = &out[i];
        o->action = ing[i].action; o->reason = ing[i].reason; o->ct_ret = ing[i].ct_ret;
        o->flags = ing[i].flags; o->proxy_port = ing[i].proxy_port; o->ifindex_lo = ing[i].ifindex_lo;
    }
    /* drop notifications: the sender's send_drop_notify(SECLABEL, 0, 0, 0, ret) for
     * from-container drops (bpf_lxc.c:659-668), handle_policy's for local deliveries */
    for (uint32_t i = 0; (events || g_tr.ev) && i < n; i++) {
        uint8_t tmp[O_EVENT_RECORD];
        uint8_t *e = events ? events + (size_t)i * O_EVENT_RECORD : tmp;
        memset(e, 0, O_EVENT_RECORD);
        const o_egress_out *o = &out[i];
        if (o->action != TC_ACT_SHOT) continue;
        const uint8_t *row = snap + (size_t)i * b->snap_stride;
        uint32_t hash = b->flow_hash ? b->flow_hash[i] : 0, len = b->len[i];
        const o_lxc_cfg *c = o->stage == O_STAGE_POLICY ? a->slot[lxcid[i]]
                                                         : a->slot[(b->lxc_id ? b->lxc_id[i] : 0) & 0xffff];
        if (!c) drop_event(e, o->reason, 0, hash, len, 0, 0, 0, 0, row, b->snap_stride);
        else if (o->stage == O_STAGE_POLICY)
            drop_event(e, o->reason, c->lxc_id, hash, len, secctx[i], c->seclabel, c->lxc_id, ifx[i], row, b->snap_stride);
        else drop_event(e, o->reason, c->lxc_id, hash, len, c->seclabel, 0, 0, 0, row, b->snap_stride);
        uint8_t *t = ev_slot(i);
        if (t) memcpy(t, e, O_EVENT_RECORD);
    }
    plog_free(plog2); free(ing); free(plog);
    if (!snap_out) free(snap);
    free(skip); free(secctx); free(ifx); free(lxcid);
}

/* ------------------------------------------------------------------ */
/* Parity helper (checker only): a 64-bit fingerprint of each (key, value) row of */
/* a table dump, so two dumps of ~10^8 entries compare as sorted u64 arrays      */
/* (oracle/parity.py compare_tables) instead of a lexicographic row sort.        */
static uint64_t o_fmix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
void o_rows_fp(const uint8_t *keys, const uint8_t *vals, uint64_t n, uint32_t ksz, uint32_t vsz, uint64_t *out) {
    for (uint64_t i = 0; i < n; i++) {
        uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)ksz << 32) ^ vsz;
        const uint8_t *rows[2] = {keys + i * ksz, vals + i * vsz};
        const uint32_t len[2] = {ksz, vsz};
        for (int r = 0; r < 2; r++) {
            for (uint32_t o = 0; o < len[r]; o += 8) {
                uint64_t w = 0;
                memcpy(&w, rows[r] + o, len[r] - o < 8 ? len[r] - o : 8);
                h = o_fmix64(h ^ w) + 0x632BE59BD9B4E019ull * (uint64_t)(r + 1);
            }
        }
        out[i] = h;
    }
}
