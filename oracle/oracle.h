/*
 * oracle.h — CPU restatement of Cilium's per-packet verdict path
 * (carlanton/cilium 1.0.0-rc9), used ONLY as the parity checker and the
 * CPU baseline.  TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product (libgpuflow)
 * never links or calls it.
 *
 * Written line-by-line from the reference text (read, never compiled):
 * each function cites the file:line it restates.  Kernel map semantics
 * (htab exact match over key_size bytes, LPM trie longest-prefix match,
 * E2BIG/ENOSPC at max_entries) follow the Linux kernel's published
 * behaviour (kernel/bpf/hashtab.c, kernel/bpf/lpm_trie.c), which are not in
 * /root/reference; see DESIGN.md "Oracle".
 *
 * Inputs are raw frames (Ethernet header first) plus the skb metadata the
 * calling programs provide, so every skb_load_bytes()/revalidate_data()
 * bound check of the reference is exercised on real bytes.
 */
#ifndef GF_ORACLE_H
#define GF_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- maps ---------------- */
#define OM_HASH 1
#define OM_LRU_HASH 9
#define OM_LPM_TRIE 11

typedef struct om_map om_map;
/* shards > 1 partitions a CT map by unordered address pair (used by the
 * multi-threaded baseline; semantics identical to one map). */
om_map *om_create(uint32_t type, uint32_t key_size, uint32_t value_size,
                  uint32_t max_entries, uint32_t shards);
void    om_destroy(om_map *m);
int     om_update(om_map *m, const void *key, const void *value, uint64_t flags);
int     om_lookup(om_map *m, const void *key, void *value_out); /* 0 / -ENOENT */
int     om_delete(om_map *m, const void *key);
int     om_update_many(om_map *m, const void *keys, const void *values, uint32_t n, uint64_t flags, uint32_t *done);
uint32_t om_count(om_map *m);
/* Iterate all entries (order unspecified). Returns number visited. */
typedef void (*om_visit_fn)(const void *key, const void *value, void *ctx);
uint32_t om_foreach(om_map *m, om_visit_fn fn, void *ctx);
/* Dump all entries into flat arrays (capacity in entries); returns count. */
uint32_t om_dump(om_map *m, void *keys, void *values, uint32_t capacity);

/* ---------------- programs ---------------- */
typedef struct o_xdp_cfg {
    om_map *cidr4_hmap, *cidr4_lmap, *cidr6_hmap, *cidr6_lmap, *lxc_map;
} o_xdp_cfg;

typedef struct o_lb_cfg {
    om_map *lb4_services, *lb6_services;
    uint32_t flags;             /* GF_LB_F_* of include/gpuflow.h */
    uint32_t redirect_ifindex;
} o_lb_cfg;

typedef struct o_l4_allow { uint16_t port, proxy; uint8_t nexthdr, pad[3]; } o_l4_allow;

typedef struct o_lxc_cfg {
    uint32_t lxc_id, seclabel;
    om_map *policy_map, *ct_map4, *ct_map6, *cidr4_ingress_map, *cidr6_ingress_map;
    om_map *revnat4_map, *revnat6_map;
    uint32_t flags;             /* GF_LXC_F_* */
    uint32_t n_l4_ingress;
    o_l4_allow l4_ingress[64];
    /* from-container section (== gf_lxc_cfg) */
    uint8_t lxc_mac[6], node_mac[6];
    uint32_t lxc_ipv4;
    om_map *lb4_services, *ipcache_map, *cidr4_egress_map;
    uint32_t n_portmap;
    struct { uint16_t from, to; } portmap[16];
    uint32_t n_l4_egress;
    o_l4_allow l4_egress[64];
    uint8_t lxc_ip6[16];
    om_map *lb6_services, *cidr6_egress_map;
} o_lxc_cfg;

typedef struct o_node_cfg {       /* == gf_node_cfg (bpf/node_config.h values on the path) */
    uint32_t host_ifindex;        /* HOST_IFINDEX */
    om_map *proxy4_map, *proxy6_map;  /* cilium_proxy4 / cilium_proxy6 (NULL: not installed) */
    uint32_t ipv4_gateway;        /* IPV4_GATEWAY (raw be32) */
    uint8_t host_ip6[16];         /* HOST_IP */
    uint8_t host_mac[6];          /* HOST_IFINDEX_MAC */
    uint8_t node_mac[6];          /* NODE_MAC */
    om_map *lxc_map;              /* cilium_lxc (egress endpoint lookup) */
    uint32_t ipv4_cluster_range, ipv4_cluster_mask, ipv4_loopback, ipv4_mask, encap_ifindex;
    om_map *tunnel_map;           /* cilium_tunnel_map */
    uint8_t router_ip6[16];       /* ROUTER_IP */
} o_node_cfg;

/* Per-packet metadata of a batch (host arrays, may be NULL where unused). */
typedef struct o_batch {
    uint32_t n, snap_stride;
    const uint8_t  *snap;       /* n * snap_stride */
    const uint32_t *len;
    const uint32_t *src_identity, *ifindex, *flow_hash;
    const uint16_t *lxc_id;
    const uint8_t  *tc_index;
} o_batch;

typedef struct o_lb_out {       /* == gf_lb_out */
    uint8_t action, reason; uint16_t slave, new_dport, rev_nat; uint32_t new_daddr4;
} o_lb_out;

typedef struct o_ingress_out {  /* == gf_ingress_out */
    uint8_t action, reason, ct_ret, flags; uint16_t proxy_port, ifindex_lo;
} o_ingress_out;

/* Parsed columns (== gf_pkt_cols_out rules), host arrays. */
typedef struct o_cols {
    uint16_t *ethertype; uint32_t *saddr4, *daddr4; uint8_t *proto;
    int16_t *l4_off; uint32_t *l4w0; uint16_t *l4w3; uint8_t *saddr6, *daddr6;
} o_cols;

void o_parse_batch(const o_batch *b, o_cols *out);
void o_xdp_batch(const o_xdp_cfg *cfg, const o_batch *b, uint8_t *verdict);
void o_lb_batch(const o_lb_cfg *cfg, const o_batch *b, o_lb_out *out, uint8_t *new_daddr6);

/* Prog array for handle_policy tail calls: index lxc_id (0..65535). */
typedef struct o_prog_array { const o_lxc_cfg *slot[65536]; } o_prog_array;
o_prog_array *o_prog_array_create(void);
void o_prog_array_destroy(o_prog_array *a);
void o_prog_array_set(o_prog_array *a, uint32_t lxc_id, const o_lxc_cfg *cfg);
void o_set_node(const o_node_cfg *node);

/* Sequential handle_policy over the batch in order (one CPU). */
void o_ingress_batch(const o_prog_array *a, const o_batch *b, uint32_t now_sec,
                     o_ingress_out *out);
/* T threads, packets partitioned by unordered address pair (RSS-like);
 * CT maps must have been created with shards == T. */
void o_ingress_batch_mt(const o_prog_array *a, const o_batch *b, uint32_t now_sec,
                        o_ingress_out *out, uint32_t threads);
void o_xdp_batch_mt(const o_xdp_cfg *cfg, const o_batch *b, uint8_t *verdict, uint32_t threads);
void o_lb_batch_mt(const o_lb_cfg *cfg, const o_batch *b, o_lb_out *out, uint8_t *nd6, uint32_t threads);

/* ---------------- full pipeline (BASELINE config 4) ----------------
 * bpf_xdp -> bpf_lb from-netdev -> bpf_netdev from-netdev (endpoint
 * delivery) -> cilium_policy tail call (handle_policy), each stage on the
 * frame as the previous one rewrote it (== gf_pipeline_classify). */
#define O_NETDEV_F_FIXED_SECCTX 1u
typedef struct o_netdev_cfg {
    om_map *lxc_map;
    uint32_t flags, fixed_secctx;   /* flags: bit 0 FIXED_SRC_SECCTX, bit 1 TRACE_NOTIFY */
    uint8_t router_ip6[16];
    uint32_t ingress_ifindex;       /* skb->ingress_ifindex of the batch (TRACE_FROM_STACK) */
} o_netdev_cfg;
typedef struct o_pipeline_cfg {
    const o_xdp_cfg *xdp;           /* NULL: no XDP stage */
    const o_lb_cfg *lb;             /* NULL: no LB stage */
    const o_netdev_cfg *netdev;
    const o_prog_array *policy;
} o_pipeline_cfg;
typedef struct o_pipeline_out {     /* == gf_pipeline_out (24 B) */
    uint8_t stage, action, reason, ct_ret, flags, pad0;
    uint16_t proxy_port, ifindex_lo, slave, rev_nat, dport;
    uint32_t daddr4;
    uint16_t lxc_id, pad1;
} o_pipeline_out;
/* snap_out (n * snap_stride, may be NULL) receives each frame as rewritten
 * before handle_policy; nd6 (16 B per packet, may be NULL) the LB v6 address. */
void o_pipeline_batch(const o_pipeline_cfg *c, const o_batch *b, uint32_t now_sec, o_pipeline_out *out,
                      uint8_t *nd6, uint8_t *snap_out);
void o_pipeline_batch_mt(const o_pipeline_cfg *c, const o_batch *b, uint32_t now_sec, o_pipeline_out *out,
                         uint8_t *nd6, uint8_t *snap_out, uint32_t threads, uint8_t *events);
/* Drop notifications (bpf/lib/drop.h:47-107): events holds n records of 160 B
 * (struct drop_notify + up to 128 captured bytes), a packet's record in its
 * slot, zero where the packet was not dropped. */
void o_ingress_events(const o_prog_array *a, const o_batch *b, const o_ingress_out *out, uint8_t *events);
/* Trace notifications (bpf/lib/trace.h:59-106, per program with o_lxc_cfg.flags
 * bit 6 / o_netdev_cfg.flags bit 1 = TRACE_NOTIFY): while a sink is set, every
 * batch call of this thread appends each packet's trace records in emission
 * order, then its drop record, to that packet's list: ev holds n * per_pkt
 * records of 160 B, cnt[i] (zeroed by the caller) counts packet i's.  capture = 0
 * leaves the payload zero (column batches, whose frames the GPU path never
 * sees).  NULL ev disables. */
void o_set_trace_sink(uint8_t *ev, uint8_t *cnt, uint32_t per_pkt, int capture);

/* ---------------- endpoint egress (== gf_lxc_egress_classify) ----------------
 * The from-container program of endpoint lxc_id[i] over each frame, in batch
 * order (bpf/bpf_lxc.c:685-738, 427-658), its proxy-map log applied in batch
 * order, then handle_policy over the local deliveries in batch order. */
typedef struct o_egress_out {       /* == gf_egress_out (24 B) */
    uint8_t stage, action, reason, ct_ret, flags, eg_ct_ret;
    uint16_t proxy_port, ifindex_lo, slave, rev_nat, eg_flags;
    uint32_t tunnel_ip;
    uint16_t lxc_id, pad;
} o_egress_out;
void o_egress_batch(const o_prog_array *a, const o_batch *b, uint32_t now_sec, o_egress_out *out,
                    uint8_t *snap_out, uint8_t *events);   /* events: n * 160 B (drop_notify), may be NULL */

/* ctmap.GC (GCFilterByTime): deletes entries with lifetime < filter_time. */
uint32_t o_ct_gc(om_map *m, uint32_t filter_time);
/* LRU stand-in (== libgpuflow): after a batch, 1 and the eviction's
 * log record if count > max_entries (the map keeps the hand's position). */
int o_ct_lru_evict(om_map *m, uint32_t now, uint32_t *age_cut, uint64_t *hand, uint64_t *lines, uint64_t *evicted);
/* A logged eviction replayed: entries with age key <= age_cut homed in [hand, hand + lines). */
uint64_t o_ct_lru_replay(om_map *m, uint32_t now, uint32_t age_cut, uint64_t hand, uint64_t lines);
void o_rows_fp(const uint8_t *keys, const uint8_t *vals, uint64_t n, uint32_t ksz, uint32_t vsz, uint64_t *out);

/* Shard of a CT key (unordered address pair), exposed for pre-population. */
uint32_t o_ct_pair_hash4(uint32_t a, uint32_t b);
uint32_t o_ct_pair_hash6(const uint8_t *a, const uint8_t *b);

/* Helpers restated for the reference's own KATs (test/bpf/unit-test.c). */
uint32_t o_get_prefix(int prefix);                       /* GET_PREFIX, bpf/lib/ipv6.h:136-138 */
void     o_ipv6_addr_clear_suffix(uint8_t addr[16], int prefix); /* bpf/lib/ipv6.h:140-150 */
/* LPM_LOOKUP_FN over an explicit prefix list against a single stored net
 * (test/bpf/unit-test.c:60-102 harness). */
int      o_lpm4_iter_lookup(uint32_t stored_net, const int *prefixes, int n, uint32_t addr);

#ifdef __cplusplus
}
#endif
#endif
