/*
 * gpuflow.h — C ABI of libgpuflow, the MI355X-native replacement for the
 * kernel side of Cilium's BPF map syscalls and its per-packet verdict
 * programs (reference: carlanton/cilium 1.0.0-rc9, /root/reference).
 *
 * Plain C: pointers, sizes and integer handles only.  Every entry point
 * returns 0 / a positive handle on success and -errno on failure, the way
 * the bpf(2) syscall wrappers in pkg/bpf/bpf.go see the kernel.
 *
 * Two groups of entry points:
 *
 *  1. Map API (drop-in for pkg/bpf/bpf.go) — host shadow + HBM replica.
 *     gf_map_create        <- bpf.CreateMap        pkg/bpf/bpf.go:84-112
 *     gf_map_update_elem   <- bpf.UpdateElement    pkg/bpf/bpf.go:129-149
 *     gf_map_lookup_elem   <- bpf.LookupElement    pkg/bpf/bpf.go:153-172
 *     gf_map_delete_elem   <- bpf.DeleteElement    pkg/bpf/bpf.go:175-192
 *     gf_map_get_next_key  <- bpf.GetNextKey       pkg/bpf/bpf.go:195-213
 *     gf_obj_pin           <- bpf.ObjPin           pkg/bpf/bpf.go:224-243
 *     gf_obj_get           <- bpf.ObjGet           pkg/bpf/bpf.go:246-266
 *     gf_obj_close         <- bpf.ObjClose         pkg/bpf/bpf.go:269-274
 *     gf_map_get_info      <- bpf.GetMapInfo       pkg/bpf/map.go:171-209 (fdinfo parse)
 *     gf_map_lookup_batch  <- the GetNextKey + LookupElement loop of bpf.Map.DumpWithCallback
 *                             pkg/bpf/map.go:319-369, in chunks
 *     gf_now_sec           <- bpf.GetMtime()/1e9   pkg/bpf/bpf.go:426-435, bpf/lib/utils.h:58-64
 *
 *  2. Program API (replaces the BPF programs of the hot path).  A "program"
 *     binds map handles the way the compile-time #defines of the generated
 *     headers do (pkg/endpoint/bpf.go:156-330, bpf/filter_config.h,
 *     bpf/lxc_config.h, bpf/netdev_config.h); a classify call runs the
 *     program over one batch of packets that is resident in HBM.
 *     gf_xdp_classify            <- xdp_start/check_filters   bpf/bpf_xdp.c:88-184
 *     gf_lb_classify             <- from_netdev (bpf_lb)      bpf/bpf_lb.c:58-212
 *     gf_policy_ingress_classify <- handle_policy/ipv{4,6}_policy bpf/bpf_lxc.c:745-1024
 *     gf_lxc_egress_classify     <- from-container handle_ingress bpf/bpf_lxc.c:427-738
 *     gf_pipeline_classify       <- bpf_xdp -> bpf_lb -> bpf_netdev -> cilium_policy tail call
 *     gf_parse_frames            <- the skb_load_bytes()/revalidate_data() header
 *                                   accesses of those programs (bpf/lib/common.h:67-87,
 *                                   bpf/lib/ipv4.h:45-48, bpf/lib/ipv6.h:61-98)
 *
 * Host/device contract: map updates go to the host shadow and are pushed to
 * the HBM replica at the next classify call (batch boundary; a documented
 * relaxation of the kernel's per-element RCU visibility).  Maps the
 * datapath writes (CT entries, policy counters) are device-authoritative:
 * host-side lookups, updates, deletes and get_next_key then walk the key's
 * probe sequence in HBM with small reads / writes, and dumps stream in chunks
 * selected on the device; no call copies a whole table.  Each map has its own
 * lock; a classify call holds the locks of the maps its programs bind.
 *
 * All batch/column/output pointers passed to classify calls are DEVICE
 * pointers (hipMalloc / torch CUDA tensors).  `stream` is a hipStream_t
 * (NULL = default stream).  Classify calls are asynchronous w.r.t. the host
 * except for the table sync they may perform before launching.
 */
#ifndef GPUFLOW_H
#define GPUFLOW_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- map types (enum bpf_map_type subset, pkg/bpf/bpf.go:38-52) ---- */
#define GF_MAP_TYPE_HASH      1
#define GF_MAP_TYPE_ARRAY     2
#define GF_MAP_TYPE_PROG_ARRAY 3
#define GF_MAP_TYPE_LRU_HASH  9
#define GF_MAP_TYPE_LPM_TRIE  11

/* update flags (pkg/bpf/bpf.go:73-75) */
#define GF_ANY     0
#define GF_NOEXIST 1
#define GF_EXIST   2

/* map flags (pkg/bpf/bpf.go:77-78) */
#define GF_F_NO_PREALLOC   (1u << 0)
#define GF_F_NO_COMMON_LRU (1u << 1)

/* ---- return codes of the datapath (bpf/include/bpf/api.h:17-25,
 *      bpf/include/linux/bpf.h:622-624) ---- */
#define GF_TC_ACT_OK        0
#define GF_TC_ACT_SHOT      2
#define GF_TC_ACT_REDIRECT  7
#define GF_XDP_DROP         1
#define GF_XDP_PASS         2

/* CT lookup results (bpf/lib/common.h:310-315) */
#define GF_CT_NEW         0
#define GF_CT_ESTABLISHED 1
#define GF_CT_REPLY       2
#define GF_CT_RELATED     3

/* drop reasons are reported as u8 = -DROP_* (bpf/lib/common.h:224-256) */
#define GF_DROP_INVALID            134
#define GF_DROP_POLICY             133
#define GF_DROP_CT_INVALID_HDR     135
#define GF_DROP_CT_UNKNOWN_PROTO   137
#define GF_DROP_UNKNOWN_L3         139
#define GF_DROP_MISSED_TAIL_CALL   140
#define GF_DROP_WRITE_ERROR        141
#define GF_DROP_UNKNOWN_L4         142
#define GF_DROP_CSUM_L3            153
#define GF_DROP_CSUM_L4            154
#define GF_DROP_CT_CREATE_FAILED   155
#define GF_DROP_INVALID_EXTHDR     156
#define GF_DROP_FRAG_NOSUPPORT     157
#define GF_DROP_NO_SERVICE         158
#define GF_DROP_POLICY_L4          159

/* ======================= 1. Map API ======================= */

/* bpf.CreateMap: returns handle > 0 or -errno.  key/value sizes are the
 * byte sizes of the reference C structs (bpf/lib/common.h). */
int gf_map_create(uint32_t map_type, uint32_t key_size, uint32_t value_size,
                  uint32_t max_entries, uint32_t map_flags);
/* bpf.UpdateElement: flags GF_ANY/GF_NOEXIST/GF_EXIST.  -E2BIG when a
 * hash map is full, -ENOSPC for a full LPM trie, -EEXIST/-ENOENT under
 * NOEXIST/EXIST, -EINVAL for bad flags or an LPM prefixlen > max. */
int gf_map_update_elem(int map, const void *key, const void *value, uint64_t flags);
/* bpf.LookupElement: copies the value; -ENOENT if absent.  LPM tries use
 * longest-prefix semantics on key->prefixlen (kernel trie_lookup_elem). */
int gf_map_lookup_elem(int map, const void *key, void *value);
/* bpf.DeleteElement: -ENOENT if absent. */
int gf_map_delete_elem(int map, const void *key);
/* bpf.GetNextKey: key == NULL or an absent key -> first key; -ENOENT at end. */
int gf_map_get_next_key(int map, const void *key, void *next_key);
/* Batched update (same semantics as n sequential gf_map_update_elem calls;
 * stops at the first error and returns it, *n_done = entries applied). */
int gf_map_update_batch(int map, const void *keys, const void *values,
                        uint32_t n, uint64_t flags, uint32_t *n_done);

/* Chunked dump (what bpf.Map.DumpWithCallback, pkg/bpf/map.go:319-369, gets
 * from one GetNextKey + LookupElement pair per entry; the kernel's later
 * BPF_MAP_LOOKUP_BATCH contract): copies up to *count entries after the
 * opaque cursor *in_batch (NULL = from the start) into keys / values (host
 * arrays, reference layouts), sets *count to the number copied and *out_batch
 * to the cursor to resume from.  Returns 0, or -ENOENT once the map holds no
 * entry past the cursor (*count may still be > 0).  Device-authoritative maps
 * are compacted on the device; only the entries cross PCIe. */
int gf_map_lookup_batch(int map, const uint64_t *in_batch, uint64_t *out_batch,
                        void *keys, void *values, uint32_t *count);

typedef struct gf_map_info {
    uint32_t map_type, key_size, value_size, max_entries, map_flags;
    uint32_t n_entries;        /* current element count */
    uint64_t device_bytes;     /* HBM bytes of the replica (0 if never synced) */
    uint64_t xfer_d2h;         /* bytes the map API has copied device -> host (element walks, */
    uint64_t xfer_h2d;         /* dumps, pulls) and host -> device (element writes, pushes) */
} gf_map_info;
int gf_map_get_info(int map, gf_map_info *info);

/* bpf.ObjPin / ObjGet / ObjClose.  Pin paths are names in a process-wide
 * registry that stands in for /sys/fs/bpf (pkg/bpf/bpffs.go:35-38). */
int gf_obj_pin(int handle, const char *path);
int gf_obj_get(const char *path);          /* new handle referring to the object */
int gf_obj_close(int handle);
int gf_obj_unpin(const char *path);        /* os.Remove(path) of a pinned map */

/* CLOCK_MONOTONIC seconds, the clock bpf_ktime_get_sec() reads. */
uint32_t gf_now_sec(void);

/* ======================= 2. Programs ======================= */

/* Parsed header columns.  One element per packet; all DEVICE pointers.
 * Produced from raw frames by gf_parse_frames (or by a NIC/ingest stage
 * with the same rules).  "be16"/"be32" fields hold the raw network-order
 * bytes of the frame loaded little-endian, exactly what the BPF programs
 * hold in their registers after skb_load_bytes(). */
typedef struct gf_pkt_cols {
    uint32_t n;
    const uint32_t *len;        /* skb->len (linear == data_end - data) */
    const uint16_t *ethertype;  /* host order: 0x0800 / 0x86DD / other; 0 if len < 14 */
    const uint32_t *saddr4;     /* iphdr.saddr (raw be32), v4 only */
    const uint32_t *daddr4;     /* iphdr.daddr (raw be32), v4 only */
    const uint8_t  *proto;      /* v4: protocol; v6: nexthdr after ipv6_hdrlen() (unchanged on error) */
    const int16_t  *l4_off;     /* v4: 14 + ihl*4; v6: 14 + ipv6_hdrlen() (negative DROP_* on error) */
    const uint32_t *l4w0;       /* frame bytes [l4_off, l4_off+4) (0-filled past len) */
    const uint16_t *l4w3;       /* frame bytes [l4_off+12, l4_off+14) (TCP flags word) */
    const uint8_t  *saddr6;     /* 16 B per packet, v6 (may be NULL if no IPv6 in batch) */
    const uint8_t  *daddr6;     /* 16 B per packet, v6 */
    /* skb metadata the calling programs provide */
    const uint32_t *src_identity; /* cb[CB_SRC_LABEL] (bpf/lib/l3.h:160) */
    const uint32_t *ifindex;      /* cb[CB_IFINDEX]  (bpf/lib/l3.h:161) */
    const uint16_t *lxc_id;       /* tail-call slot into cilium_policy (bpf/lib/l3.h:163) */
    const uint8_t  *tc_index;     /* skb->tc_index (TC_INDEX_F_SKIP_PROXY = bit 0) */
    const uint32_t *flow_hash;    /* get_hash_recalc(skb) (bpf/lib/lb.h:109-121) */
} gf_pkt_cols;

/* Raw frames: snap_stride bytes per packet starting at the Ethernet header. */
typedef struct gf_frames {
    uint32_t n;
    uint32_t snap_stride;       /* >= all header bytes the programs read */
    const uint8_t  *snap;       /* n * snap_stride bytes */
    const uint32_t *len;        /* wire length of each frame */
} gf_frames;

/* Writable column storage for gf_parse_frames (DEVICE pointers, n elements;
 * saddr6/daddr6 16*n bytes, may be NULL to skip IPv6 address extraction). */
typedef struct gf_pkt_cols_out {
    uint16_t *ethertype; uint32_t *saddr4; uint32_t *daddr4; uint8_t *proto;
    int16_t *l4_off; uint32_t *l4w0; uint16_t *l4w3; uint8_t *saddr6; uint8_t *daddr6;
} gf_pkt_cols_out;
int gf_parse_frames(const gf_frames *frames, gf_pkt_cols_out *out, void *stream);

/* ---- XDP prefilter (bpf/bpf_xdp.c, bpf/filter_config.h) ----
 * A zero handle means the corresponding #define is absent. */
typedef struct gf_xdp_cfg {
    int cidr4_hmap;   /* CIDR4_FILTER + CIDR4_HMAP_NAME (v4_fix, HASH, key lpm_v4_key) */
    int cidr4_lmap;   /* CIDR4_LPM_PREFILTER + CIDR4_LMAP_NAME (v4_dyn, LPM_TRIE) */
    int cidr6_hmap;   /* CIDR6_FILTER + v6_fix */
    int cidr6_lmap;   /* CIDR6_LPM_PREFILTER + v6_dyn */
    int lxc_map;      /* cilium_lxc (bpf/lib/maps.h:27-33) */
} gf_xdp_cfg;
int gf_xdp_prog_load(const gf_xdp_cfg *cfg);
/* verdict[i] = GF_XDP_DROP / GF_XDP_PASS. */
int gf_xdp_classify(int prog, const gf_pkt_cols *pkts, uint8_t *verdict, void *stream);

/* ---- standalone LB (bpf/bpf_lb.c, bpf/netdev_config.h) ---- */
#define GF_LB_F_L3       (1u << 0)   /* LB_L3 */
#define GF_LB_F_L4       (1u << 1)   /* LB_L4 */
#define GF_LB_F_REDIRECT (1u << 2)   /* LB_REDIRECT defined */
#define GF_LB_F_NO_IPV4  (1u << 3)   /* LB_DISABLE_IPV4 */
#define GF_LB_F_NO_IPV6  (1u << 4)   /* LB_DISABLE_IPV6 */
typedef struct gf_lb_cfg {
    int lb4_services;  /* cilium_lb4_services (key lb4_key 8 B, value lb4_service 12 B) */
    int lb6_services;  /* cilium_lb6_services (key lb6_key 20 B, value lb6_service 24 B) */
    uint32_t flags;
    uint32_t redirect_ifindex; /* LB_REDIRECT */
} gf_lb_cfg;
int gf_lb_prog_load(const gf_lb_cfg *cfg);
/* Output record per packet (12 B). */
typedef struct gf_lb_out {
    uint8_t  action;     /* GF_TC_ACT_OK / SHOT / REDIRECT */
    uint8_t  reason;     /* -DROP_* (or errno for helper failures) when SHOT, else 0 */
    uint16_t slave;      /* selected slave index (0 = not load balanced) */
    uint16_t new_dport;  /* raw be16 destination port after lb*_xlate */
    uint16_t rev_nat;    /* slave's rev_nat_index (raw) */
    uint32_t new_daddr4; /* raw be32 (v4) */
} gf_lb_out;
/* new_daddr6 (16 B per packet, may be NULL) receives the v6 translated address. */
int gf_lb_classify(int prog, const gf_pkt_cols *pkts, gf_lb_out *out,
                   uint8_t *new_daddr6, void *stream);

/* ---- endpoint ingress policy (bpf/bpf_lxc.c handle_policy) ---- */
#define GF_LXC_F_DROP_ALL        (1u << 0)  /* DROP_ALL */
#define GF_LXC_F_POLICY_INGRESS  (1u << 1)  /* POLICY_INGRESS */
#define GF_LXC_F_HAVE_L4_POLICY  (1u << 2)  /* HAVE_L4_POLICY */
#define GF_LXC_F_CT_ACCOUNTING   (1u << 3)  /* CONNTRACK_ACCOUNTING */
#define GF_LXC_F_LXC_IPV4        (1u << 4)  /* LXC_IPV4 */
#define GF_LXC_F_POLICY_EGRESS   (1u << 5)  /* POLICY_EGRESS (pkg/endpoint/endpoint.go:153-156, emitted when egress
                                               is enforced, pkg/endpoint/policy.go:820-839) */
#define GF_LXC_F_TRACE_NOTIFY    (1u << 6)  /* TRACE_NOTIFY (pkg/endpoint/endpoint.go:131-134, on by default:
                                               daemon/main.go:629): send_trace_notify records, see below */
#define GF_MAX_L4_INGRESS 64
#define GF_MAX_PORTMAP 16
typedef struct gf_portmap {    /* struct portmap (bpf/lib/common.h), LXC_PORT_MAPPINGS entries */
    uint16_t from;             /* raw be16 */
    uint16_t to;               /* raw be16 */
} gf_portmap;
typedef struct gf_l4_allow {   /* struct l4_allow, bpf/lib/l4.h:126-136 */
    uint16_t port;             /* raw be16 */
    uint16_t proxy;            /* raw be16 */
    uint8_t  nexthdr;
    uint8_t  pad[3];
} gf_l4_allow;
typedef struct gf_lxc_cfg {
    uint32_t lxc_id;           /* LXC_ID */
    uint32_t seclabel;         /* SECLABEL */
    int policy_map;            /* POLICY_MAP (key policy_key 8 B, value policy_entry 24 B) */
    int ct_map4;               /* CT_MAP4 (key ipv4_ct_tuple 14 B, value ct_entry 48 B) */
    int ct_map6;               /* CT_MAP6 (key ipv6_ct_tuple 40 B, value ct_entry 48 B).  Either every
                                  program binds the same map per family (the agent's default,
                                  cilium_ct4_global / cilium_ct6_global) or programs bind maps of their own
                                  (the ConntrackLocal option, cilium_ct4_<id>, pkg/endpoint/bpf.go:268-276),
                                  mixed freely in one array.  With more than one map per family a call runs
                                  the per-endpoint kernels: each packet's program's own map, inserts counted
                                  into that map, the LRU eviction pass on each map after the call.  One map
                                  bound as both a CT_MAP4 and a CT_MAP6: -EINVAL. */
    int cidr4_ingress_map;     /* CIDR4_INGRESS_MAP (LPM_TRIE), 0 = undefined */
    int cidr6_ingress_map;     /* CIDR6_INGRESS_MAP (LPM_TRIE), 0 = undefined */
    int revnat4_map;           /* cilium_lb4_reverse_nat (key u16, value 6 B) */
    int revnat6_map;           /* cilium_lb6_reverse_nat (key u16, value 18 B) */
    uint32_t flags;            /* GF_LXC_F_* */
    uint32_t n_l4_ingress;     /* CFG_L3L4_INGRESS entries */
    gf_l4_allow l4_ingress[GF_MAX_L4_INGRESS];
    /* ---- the from-container section of the same object (bpf_lxc.c:427-738) ---- */
    uint8_t  lxc_mac[6];       /* LXC_MAC (is_valid_lxc_src_mac) */
    uint8_t  node_mac[6];      /* NODE_MAC (is_valid_gw_dst_mac, router MAC of ipv4_l3) */
    uint32_t lxc_ipv4;         /* LXC_IPV4 value (raw be32, is_valid_lxc_src_ipv4) */
    int lb4_services;          /* cilium_lb4_services (LB_L3 + LB_L4: lb4_lookup_service / lb4_local), 0 = none */
    int ipcache_map;           /* cilium_ipcache (endpoint_key 20 B -> remote_endpoint_info 8 B), POLICY_EGRESS */
    int cidr4_egress_map;      /* CIDR4_EGRESS_MAP (LPM_TRIE), 0 = undefined (deny) */
    uint32_t n_portmap;        /* LXC_PORT_MAPPINGS entries (map_lxc_out) */
    gf_portmap portmap[GF_MAX_PORTMAP];
    uint32_t n_l4_egress;      /* CFG_L3L4_EGRESS entries (l4_egress_proxy_lookup) */
    gf_l4_allow l4_egress[GF_MAX_L4_INGRESS];
    uint8_t  lxc_ip6[16];      /* LXC_IP (is_valid_lxc_src_ip) */
    int lb6_services;          /* cilium_lb6_services (lb6_lookup_service / lb6_local), 0 = none */
    int cidr6_egress_map;      /* CIDR6_EGRESS_MAP (LPM_TRIE), 0 = undefined (deny) */
} gf_lxc_cfg;
int gf_lxc_prog_load(const gf_lxc_cfg *cfg);

/* The cilium_policy prog array (bpf/lib/maps.h:36-43): slot lxc_id -> program. */
int gf_policy_array_create(void);
int gf_policy_array_update(int array, uint32_t lxc_id, int prog);  /* prog 0 = delete */

typedef struct gf_node_cfg {   /* node_config.h values used on the path */
    uint32_t host_ifindex;     /* HOST_IFINDEX */
    int      proxy4_map;       /* cilium_proxy4 (proxy4_tbl_key 10 B -> proxy4_tbl_value 16 B), 0 = none */
    int      proxy6_map;       /* cilium_proxy6 (proxy6_tbl_key 22 B -> proxy6_tbl_value 28 B), 0 = none */
    uint32_t ipv4_gateway;     /* IPV4_GATEWAY (raw be32), the proxy redirect's new daddr */
    uint8_t  host_ip6[16];     /* HOST_IP, the IPv6 proxy redirect's new daddr */
    uint8_t  host_mac[6];      /* HOST_IFINDEX_MAC */
    uint8_t  node_mac[6];      /* NODE_MAC */
    /* the from-container path (bpf_lxc.c:427-658) */
    int      lxc_map;          /* cilium_lxc (lookup_ip4_endpoint of the egress path), 0 = none */
    uint32_t ipv4_cluster_range; /* IPV4_CLUSTER_RANGE (raw be32) */
    uint32_t ipv4_cluster_mask;  /* IPV4_CLUSTER_MASK (raw be32) */
    uint32_t ipv4_loopback;    /* IPV4_LOOPBACK (raw be32), lb4_local's loopback SNAT source */
    uint32_t ipv4_mask;        /* IPV4_MASK (raw be32), the tunnel map key of encap_and_redirect */
    uint32_t encap_ifindex;    /* ENCAP_IFINDEX, 0 = undefined (no tunnel) */
    int      tunnel_map;       /* cilium_tunnel_map (endpoint_key 20 B -> endpoint_key 20 B) */
    uint8_t  router_ip6[16];   /* ROUTER_IP (the IPv6 egress path's CLUSTER_ID test) */
} gf_node_cfg;
int gf_node_config(const gf_node_cfg *cfg);

/* Output record per packet (8 B). */
typedef struct gf_ingress_out {
    uint8_t  action;      /* TC_ACT_OK / SHOT / REDIRECT (handle_policy return) */
    uint8_t  reason;      /* cb[2] = -ret when SHOT (bpf/lib/drop.h:92-107) */
    uint8_t  ct_ret;      /* forwarding_reason: CT_NEW/ESTABLISHED/REPLY/RELATED */
    uint8_t  flags;       /* bit0: redirected to proxy, bit1: CT entry created */
    uint16_t proxy_port;  /* raw be16 policy verdict > 0 */
    uint16_t ifindex_lo;  /* low 16 bits of the redirect ifindex */
} gf_ingress_out;
#define GF_INGRESS_F_PROXY    1
#define GF_INGRESS_F_CREATED  2

/* Runs handle_policy over the batch, in batch order per flow group
 * (unordered address pair): packets of one group see each other's CT
 * updates in batch order, as on one CPU of the reference.  now_sec
 * replaces bpf_ktime_get_sec() for the whole batch. */
int gf_policy_ingress_classify(int policy_array, const gf_pkt_cols *pkts,
                               uint32_t now_sec, gf_ingress_out *out, void *stream);
/* nb consecutive gf_policy_ingress_classify calls on `stream` (batch k with
 * now_sec[k] into outs[k]), with identical results.  The stateless half of a
 * batch (record pack, flow-group sort and schedule: no map state) is built on an
 * internal second stream while handle_policy of the previous batch runs, so the
 * schedule leaves the critical path of a stream of batches. */
int gf_policy_ingress_classify_batches(int policy_array, uint32_t nb, const gf_pkt_cols *const *batches,
                                       const uint32_t *now_sec, gf_ingress_out *const *outs, void *stream);

/* ---- endpoint egress: the from-container program (bpf/bpf_lxc.c:685-738
 * handle_ingress -> tail_handle_ipv4 -> handle_ipv4_from_lxc :427-658) ----
 * Frames sent by local endpoints; packet i runs the program of endpoint
 * lxc_id[i] (its bpf_lxc object = the cilium_policy slot's program).  Local
 * deliveries (ipv4_local_delivery, bpf/lib/l3.h:136-168) continue into the
 * destination's handle_policy (tail call into cilium_policy) in a second pass
 * over the batch, as gf_pipeline_classify does: every from-container effect
 * of the batch (CT, proxy map) precedes every handle_policy effect of its
 * deliveries.  IPv6 frames run tail_handle_ipv6 -> ipv6_l3_from_lxc
 * (:120-416).  Frames for the ARP / ICMPv6 responders (tail_handle_arp,
 * icmp6_handle's NS and echo-to-router) are reported as stage GF_STAGE_NONE. */
typedef struct gf_lxc_batch {
    gf_frames frames;          /* DEVICE frames (snap_stride >= every header byte touched, <= 256) */
    const uint16_t *lxc_id;    /* DEVICE: the sending endpoint (whose from-container program runs) */
    const uint32_t *flow_hash; /* DEVICE get_hash_recalc(skb) (lb4_select_slave), may be NULL */
} gf_lxc_batch;
#define GF_STAGE_NONE     0    /* not classified: ARP / ICMPv6 responders */
#define GF_STAGE_FROM_LXC 5    /* the from-container verdict is final */
/* GF_STAGE_POLICY (4): delivered locally, handle_policy of endpoint lxc_id */
#define GF_EG_F_CREATED   0x0001  /* ct_create4(CT_EGRESS) */
#define GF_EG_F_PROXY     0x0002  /* ipv4_redirect_to_host_port */
#define GF_EG_F_LB        0x0004  /* lb4_local translated the destination */
#define GF_EG_F_LOOPBACK  0x0008  /* ... back to the sender: source SNAT to IPV4_LOOPBACK */
#define GF_EG_F_REVNAT    0x0010  /* lb4_rev_nat of a reply */
#define GF_EG_F_PORTMAP   0x0020  /* map_lxc_out rewrote the source port */
#define GF_EG_F_ENCAP     0x0040  /* encap_and_redirect: tunnel_ip holds the remote node */
#define GF_EG_F_TO_HOST   0x0080  /* to_host: redirect(HOST_IFINDEX) */
#define GF_EG_F_TO_STACK  0x0100  /* pass_to_stack: TC_ACT_OK */
#define GF_EG_F_LOCAL     0x0200  /* ipv4_local_delivery (stage GF_STAGE_POLICY) */
#define GF_EG_F_DELETED   0x0400  /* ct_delete4 of an ESTABLISHED flow the policy now denies */
#define GF_EG_F_ARP       0x0800  /* stage NONE: ARP (tail_handle_arp, the responder) */
#define GF_EG_F_IPV6      0x1000  /* the IPv6 path (ipv6_l3_from_lxc) */
#define GF_EG_F_ICMP6_TE  0x2000  /* hop limit reached in ipv6_l3: icmp6_send_time_exceeded (action
                                     REDIRECT; the reply itself is not built) */
#define GF_EG_F_RESPONDER 0x4000  /* stage NONE: icmp6_handle's NS / echo-to-router responders */
typedef struct gf_egress_out {   /* 24 B; bytes 0-9 as gf_pipeline_out */
    uint8_t  stage;       /* GF_STAGE_FROM_LXC / GF_STAGE_POLICY / GF_STAGE_NONE */
    uint8_t  action;      /* final TC_ACT_* */
    uint8_t  reason;      /* drop reason when SHOT */
    uint8_t  ct_ret;      /* stage FROM_LXC: the egress ct_lookup4 result; POLICY: handle_policy's */
    uint8_t  flags;       /* stage POLICY: gf_ingress_out.flags */
    uint8_t  eg_ct_ret;   /* egress ct_lookup4 result (forwarding_reason) */
    uint16_t proxy_port;  /* raw be16 proxy port of the final redirect */
    uint16_t ifindex_lo;  /* redirect target (HOST_IFINDEX, ENCAP_IFINDEX, or handle_policy's) */
    uint16_t slave;       /* lb4_local: selected slave */
    uint16_t rev_nat;     /* lb4_local: rev_nat_index (raw) */
    uint16_t eg_flags;    /* GF_EG_F_* */
    uint32_t tunnel_ip;   /* ENCAP: bpf_tunnel_key.remote_ipv4 */
    uint16_t lxc_id;      /* stage POLICY: destination endpoint */
    uint16_t pad;
} gf_egress_out;
/* snap_out (n * snap_stride, may be NULL): the frames as the programs left them. */
int gf_lxc_egress_classify(int policy_array, const gf_lxc_batch *batch, uint32_t now_sec,
                           gf_egress_out *out, uint8_t *snap_out, void *stream);

/* ---- full pipeline (BASELINE config 4) ----
 * One frame through the programs a node attaches in order, each seeing the
 * frame as the previous one rewrote it:
 *   bpf_xdp (prefilter)          bpf/bpf_xdp.c:158-184
 *   bpf_lb  from-netdev          bpf/bpf_lb.c:169-212 (lb4_xlate/lb6_xlate rewrites + checksums)
 *   bpf_netdev from-netdev       bpf/bpf_netdev.c:160-247, 326-393 (endpoint lookup,
 *                                ipv{4,6}_local_delivery: TTL/hop limit, MACs, port map)
 *   cilium_policy[ep->lxc_id]    bpf/bpf_lxc.c:980-1024 handle_policy (as gf_policy_ingress_classify)
 * The pipeline replaces the per-program entry points of a node for traffic
 * arriving on the netdev; it has no equivalent call in the reference (the
 * kernel chains the programs), see DESIGN.md. */
#define GF_NETDEV_F_FIXED_SECCTX (1u << 0)  /* FIXED_SRC_SECCTX defined */
#define GF_NETDEV_F_TRACE_NOTIFY (1u << 1)  /* TRACE_NOTIFY: TRACE_FROM_STACK at from_netdev (bpf_netdev.c:436) */
typedef struct gf_netdev_cfg {
    int lxc_map;               /* cilium_lxc (endpoint_key 20 B -> endpoint_info 112 B) */
    uint32_t flags;            /* GF_NETDEV_F_* */
    uint32_t fixed_secctx;     /* FIXED_SRC_SECCTX */
    uint8_t  router_ip6[16];   /* ROUTER_IP (node_config.h), derive_sec_ctx() */
    uint32_t ingress_ifindex;  /* skb->ingress_ifindex of the frames (the netdev's ifindex) */
} gf_netdev_cfg;
typedef struct gf_pipeline_cfg {
    int xdp_prog;              /* gf_xdp_prog_load handle, 0 = no XDP program attached */
    int lb_prog;               /* gf_lb_prog_load handle, 0 = no LB program attached */
    gf_netdev_cfg netdev;
    int policy_array;          /* cilium_policy prog array */
} gf_pipeline_cfg;
int gf_pipeline_load(const gf_pipeline_cfg *cfg);

typedef struct gf_pipe_batch {
    gf_frames frames;          /* DEVICE frames; snap_stride must hold every header byte the
                                  programs read or write (>= l4_off + 18) */
    const uint8_t  *tc_index;  /* skb->tc_index (DEVICE, may be NULL) */
    const uint32_t *flow_hash; /* get_hash_recalc(skb) (DEVICE, may be NULL) */
} gf_pipe_batch;

#define GF_STAGE_XDP    1      /* dropped by bpf_xdp (action = XDP_DROP) */
#define GF_STAGE_LB     2      /* bpf_lb verdict is final (SHOT, or REDIRECT with LB_REDIRECT) */
#define GF_STAGE_NETDEV 3      /* bpf_netdev verdict is final (to the stack, SHOT, ICMPv6 reply) */
#define GF_STAGE_POLICY 4      /* tail-called into cilium_policy: handle_policy's verdict */
#define GF_PIPE_F_ICMP6_TE  0x20  /* hop limit reached: icmp6_send_time_exceeded (bpf/lib/icmp6.h:313-322);
                                     action REDIRECT, the reply frame itself is not built */
#define GF_PIPE_F_LB        0x40  /* translated by lb*_xlate */
#define GF_PIPE_F_PORTMAP   0x80  /* dport rewritten by map_lxc_in */
typedef struct gf_pipeline_out {   /* 24 B */
    uint8_t  stage;       /* GF_STAGE_* */
    uint8_t  action;      /* XDP_DROP at stage XDP, else TC_ACT_* */
    uint8_t  reason;      /* drop reason (cb[2]) when SHOT */
    uint8_t  ct_ret;      /* stage POLICY: CT_NEW/ESTABLISHED/REPLY/RELATED */
    uint8_t  flags;       /* gf_ingress_out.flags | GF_PIPE_F_* */
    uint8_t  pad0;
    uint16_t proxy_port;  /* stage POLICY: raw be16 */
    uint16_t ifindex_lo;  /* redirect target (LB_REDIRECT ifindex, or handle_policy's) */
    uint16_t slave;       /* LB: selected slave */
    uint16_t rev_nat;     /* LB: slave's rev_nat_index */
    uint16_t dport;       /* raw be16 dport written by lb*_xlate / map_lxc_in (0 = unchanged) */
    uint32_t daddr4;      /* raw be32 daddr written by lb4_xlate (0 = unchanged) */
    uint16_t lxc_id;      /* stage POLICY: endpoint tail-called into */
    uint16_t pad1;
} gf_pipeline_out;
/* new_daddr6 (16 B per packet, may be NULL): lb6_xlate's address.  snap_out
 * (n * snap_stride, may be NULL): every frame as rewritten before handle_policy
 * (MACs, TTL/hop limit, daddr, dport, IPv4 + L4 checksums). */
int gf_pipeline_classify(int pipe, const gf_pipe_batch *batch, uint32_t now_sec, gf_pipeline_out *out,
                         uint8_t *new_daddr6, uint8_t *snap_out, void *stream);

/* ---- ingest re-partition for N GPUs (real traffic) ----
 * owner[i] = the rank owning packet i's flow group: the unordered address pair
 * handle_policy's conntrack sees (after bpf_lb's translation, which is
 * stateless), fmix64-hashed mod nranks (frames that cannot reach conntrack
 * stay on self_rank); order = the packet indices stably grouped by owner;
 * counts[r] = packets for rank r.  All DEVICE pointers (n, n, nranks
 * elements).  The caller exchanges the frames (cilium_amd.shard: one RCCL
 * all-to-all) and classifies what it receives. */
int gf_pipeline_partition(int pipe, const gf_pipe_batch *batch, uint32_t self_rank, uint32_t nranks,
                          uint32_t *owner, uint32_t *order, uint32_t *counts, void *stream);

/* ---- conntrack garbage collection ----
 * ctmap.GC(m, name, GCFilterByTime) / ctmap.Flush (pkg/maps/ctmap/ctmap.go:277-368):
 * deletes every entry of a CT map (key ipv4_ct_tuple 14 B or ipv6_ct_tuple 40 B,
 * value ct_entry 48 B) whose lifetime < filter_time (Flush: 0xFFFFFFFF) and
 * returns how many were deleted (or -errno).  Runs on the device replica when the
 * datapath owns the map (compacting probe clusters in the same sweep), else on the
 * host shadow.  Synchronous on `stream`. */
int gf_ct_gc(int map, uint32_t filter_time, void *stream);

/* ---- LRU CT maps (BPF_MAP_TYPE_LRU_HASH, bpf/bpf_lxc.c:53-75) ----
 * The kernel evicts from per-CPU LRU lists (the tail of an inactive list kept
 * about as long as the active one) in a nondeterministic order and never fails
 * an insert.  libgpuflow's deterministic stand-in: inside a batch an
 * LRU CT map may exceed max_entries (up to the 7/8 load of its slot array: a power
 * of two >= 8 x max_entries for ipv4_ct_tuple, 4 x for ipv6_ct_tuple).  At the end
 * of every classify call that uses it, once the count exceeds the high-water mark
 * HW = max_entries - max_entries/8, a hand sweeping the table's home lines deletes
 * the entries of the older half (age key <= age_cut: the median age of a sample —
 * the max(65536, lines/1024) home lines just ahead of the hand, or the whole table if
 * no entry is homed there; closing entries older than all others, then by last use
 * in one-second bins) homed in the lines it passes, as many lines as bring the count
 * back to HW by the sample's density.  A map running at HW so deletes in each call
 * about what the call inserted: the eviction's work per call follows the call's
 * inserts, not the table.  If the count is still above max_entries, a second round
 * passes more lines by the same estimate and a third the rest of the table.
 * Bound: after a call the count is <= max_entries unless the whole table held
 * fewer than count - max_entries entries of the sample's older half (a single call
 * inserting more than about half of max_entries beyond HW); it never falls below
 * the entries younger than age_cut.  Every eviction is logged: */
typedef struct gf_ct_evict_rec {
    uint32_t seq;              /* the map's classify call (1 = first call that used the map) */
    uint32_t now_sec;          /* that call's now_sec */
    uint32_t age_cut;          /* entries with age key <= age_cut were eligible */
    uint32_t pad;
    uint64_t hand_line;        /* the first home line the hand passed */
    uint64_t lines;            /* home lines passed (from hand_line, wrapping) */
    uint64_t evicted;          /* entries deleted */
} gf_ct_evict_rec;
/* Copies up to max records (oldest first) and returns the number logged. */
int gf_ct_evict_log(int map, gf_ct_evict_rec *out, uint32_t max);

/* ---- drop notifications (bpf/lib/drop.h:38-107, DROP_NOTIFY) ----
 * With a ring set, gf_policy_ingress_classify and gf_pipeline_classify append
 * one record per dropped packet (TC_ACT_SHOT; XDP drops send none), in batch
 * order: struct drop_notify (32 B: type CILIUM_NOTIFY_DROP=1, subtype = drop
 * reason, source = EVENT_SOURCE, hash, len_orig, len_cap, src_label, dst_label,
 * dst_id, ifindex — the layout pkg/monitor/datapath_drop.go DropNotify decodes)
 * followed by GF_TRACE_PAYLOAD_LEN bytes holding the first len_cap bytes of the
 * frame (the pipeline's frames; zeros for column batches, which carry none).
 * *count accumulates across calls; records past `capacity` are lost (a perf ring
 * overrun). */
/* ---- trace notifications (bpf/lib/trace.h:59-106, TRACE_NOTIFY) ----
 * Programs loaded with GF_LXC_F_TRACE_NOTIFY (and a pipeline whose netdev has
 * GF_NETDEV_F_TRACE_NOTIFY) also append struct trace_notify records to the same
 * ring (type CILIUM_NOTIFY_TRACE=4, subtype = observation point TRACE_TO_LXC 0,
 * TO_PROXY 1, TO_HOST 2, TO_STACK 3, TO_OVERLAY 4, FROM_LXC 5, FROM_STACK 8;
 * source = EVENT_SOURCE, hash, len_orig, len_cap, src_label, dst_label, dst_id
 * (u16), reason (the CT result that forwarded it), pad, ifindex — the layout
 * pkg/monitor/datapath_trace.go TraceNotify decodes), followed by the first
 * len_cap bytes of the frame as it was at the call.  Per packet the records are
 * in the order the programs send them (from_netdev / handle_ingress first, the
 * drop record last), packets in batch order.  Call sites: bpf_lxc.c:364,381,
 * 650,669,705,1014, lib/lxc.h:116,168, lib/encap.h:67, bpf_netdev.c:436. */
#define GF_TRACE_PAYLOAD_LEN 128u   /* TRACE_PAYLOAD_LEN, bpf/lib/common.h:213-215 */
#define GF_EVENT_RECORD 160u
typedef struct gf_event_ring {
    uint8_t  *records;         /* DEVICE, capacity * GF_EVENT_RECORD bytes */
    uint32_t  capacity;        /* records */
    uint32_t *count;           /* DEVICE u32: records appended so far */
} gf_event_ring;
int gf_set_event_ring(const gf_event_ring *ring);   /* NULL disables */

/* ---- per-call statistics (device counter block) ---- */
#define GF_STATS_WORDS 512
/* Adds the counters of the next classify calls into `dev_counters`
 * (GF_STATS_WORDS u64 in DEVICE memory; NULL disables). Layout:
 * [0..255] drop-reason histogram (reason 0 = not dropped), [256..263]
 * action counts, [264..267] CT ret counts, [268] packets, [269] wire bytes,
 * [270] algorithmic bytes touched (per-probe costs of SURVEY.md §8(d)). */
int gf_set_stats_sink(uint64_t *dev_counters);

/* ---- launch profiler (HIP events recorded on the launch stream) ---- */
typedef struct gf_prof_rec {
    char     name[32];     /* kernel / primitive name */
    uint32_t count;        /* launches since gf_prof_enable */
    uint32_t pad;
    double   total_ms;     /* summed event-measured duration */
} gf_prof_rec;
int gf_prof_enable(int on);                       /* clears accumulators */
int gf_prof_read(gf_prof_rec *out, int max);      /* returns records written */

/* ---- device memory helpers for hosts without a GPU runtime binding ---- */
void *gf_dev_alloc(size_t bytes);
int   gf_dev_free(void *p);
int   gf_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream);
int   gf_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream);
int   gf_stream_sync(void *stream);
/* Number of visible GPUs; a library built without a device returns 0. */
int   gf_device_count(void);
const char *gf_version(void);
/* sha256 prefix of the sources (cilium_amd/csrc, include/gpuflow.h) this library
 * was compiled from ("unknown" for builds outside __graft_entry__.build()). */
const char *gf_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* GPUFLOW_H */
