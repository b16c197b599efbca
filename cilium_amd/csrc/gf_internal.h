// gf_internal.h — host-side objects of libgpuflow (maps, programs, registry).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include "gf_common.h"
#include "../../include/gpuflow.h"

namespace gf {

// Locking (the reference: one RWMutex per bpf.Map, pkg/bpf/map.go:121, and
// per-element RCU in the kernel; its programs run concurrently on every CPU):
//  * every map operation holds that map's own mutex (Map::mu);
//  * loading / changing program objects, cilium_policy arrays and the node
//    config holds prog_lock() exclusively; classify calls hold it shared, so
//    calls run concurrently with each other but never with a reconfiguration;
//  * a classify call holds its stream's call context (the device workspaces
//    of one call: CallCtx, gf_kernels.hip), the mutex of the cilium_policy array
//    it runs and the mutex of every map it binds (MapLocks, address order, so two
//    classify calls or a classify and a map operation never deadlock); on the
//    device it is ordered after the last call that used any of those objects on
//    another stream (OrderPt), so calls over disjoint programs and maps on
//    different streams overlap;
//  * the object registry (handles, pins) has its own short lock.
// Lock order: prog_lock -> call context -> policy array -> maps -> registry.
std::shared_mutex &prog_lock();

// The device-side order of the calls that use one object (map, policy array):
// the call context (one per stream, gf_kernels.hip) of the last such call.
struct CallCtx;
struct OrderPt {
    CallCtx *last = nullptr;
};
std::mutex &reg_lock();

// ---- device buffer ----
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    ~DevBuf();
    int ensure(size_t n);   // (re)allocate to exactly n bytes, contents undefined
    void release();
};

int hip_ok(hipError_t e, const char *what);

// ---- LPM key ordering (kernel trie post-order, kernel/bpf/lpm_trie.c) ----
struct LpmKeyLess {
    uint32_t data_bytes;
    bool operator()(const std::string &a, const std::string &b) const;
};

// ---- exact-match hash table (host shadow, same layout as the device) ----
// Host shadow storage: calloc'd (large blocks come from mmap as untouched zero
// pages) and not value-initialised by the vector, so a table of gigabytes costs
// host memory only in the pages an update or a pull writes.
template <class T>
struct ZeroAlloc {
    using value_type = T;
    ZeroAlloc() = default;
    template <class U> ZeroAlloc(const ZeroAlloc<U> &) {}
    T *allocate(size_t n) {
        void *p = calloc(n, sizeof(T));
        if (!p) throw std::bad_alloc();
        return (T *)p;
    }
    void deallocate(T *p, size_t) { free(p); }
    template <class U> void construct(U *) noexcept {}            // calloc'd: already zero
    template <class U, class... A> void construct(U *p, A &&...a) { ::new ((void *)p) U(std::forward<A>(a)...); }
    template <class U> bool operator==(const ZeroAlloc<U> &) const { return true; }
    template <class U> bool operator!=(const ZeroAlloc<U> &) const { return false; }
};
using ZBytes = std::vector<uint8_t, ZeroAlloc<uint8_t>>;
// n zero bytes in a fresh allocation (never the old one's contents)
inline void zbytes_reset(ZBytes &v, size_t n) { ZBytes().swap(v); v.resize(n); }

struct HTab {
    uint32_t ksz = 0, vsz = 0, slot_size = 0, voff = 0, split = 0, mode = GF_HASH_PLAIN;
    uint32_t codec = GF_VCODEC_IDENT;   // value layout in the slots (gf_common.h)
    uint32_t hot_split = 0;             // 1: hot-split layout (CT maps, gf_common.h)
    uint32_t vin = 0, sstride = 0;      // inline value bytes / side-array bytes per slot
    uint64_t nslots = 0;
    ZBytes slots, vals;
    uint64_t count = 0, tombs = 0;
    void init(uint32_t k, uint32_t v, uint64_t n);
    uint32_t hash(const uint8_t *key) const;
    int64_t find(const uint8_t *key) const;
    void relayout();                    // slot_size/voff/split/vin/sstride from ksz, vsz, hot_split
    void get_val(uint64_t i, uint8_t *out) const;
    void put_val(uint64_t i, const uint8_t *in);
    const uint8_t *key(uint64_t i) const { return &slots[i * slot_size]; }
    uint8_t state(uint64_t i) const { return slots[i * slot_size + ksz]; }
    void set_state(uint64_t i, uint8_t s) { slots[i * slot_size + ksz] = s; }
    int64_t insert_new(const uint8_t *key, const uint8_t *value);  // caller checked absence
    void erase(uint64_t i);
    void rehash(uint64_t new_nslots);
};

enum class ObjKind { Map, ProgXdp, ProgLb, ProgLxc, PolicyArray, ProgPipe };

struct Obj {
    ObjKind kind;
    explicit Obj(ObjKind k) : kind(k) {}
    virtual ~Obj() {}
};

struct Map : Obj {
    uint32_t type, ksz, vsz, max_entries, flags;
    std::recursive_mutex mu;    // this map's lock (pkg/bpf/map.go:121)
    OrderPt ord;                // device order of the classify calls that bind it
    // hash types
    HTab ht;
    bool host_valid = true;     // host shadow up to date
    bool dev_valid = false;     // HBM replica up to date
    bool fixed_capacity = false; // device inserts into this map (CT): nslots sized by max_entries
    uint64_t dev_count_hi = 0;  // upper bound of the device element count (classify bookkeeping)
    uint64_t dev_gen = 0;       // bumped on every device-side change (invalidates nk_cache)
    uint64_t host_gen = 0;      // bumped on every update / delete through the map API
    uint64_t xfer_d2h = 0, xfer_h2d = 0;   // bytes the map API moved over PCIe (gf_map_info)
    DevBuf d_slots, d_vals, d_count;
    DevBuf d_lru, d_gcbits;     // CT maps: LRU stand-in state + eviction log, GC cluster-start bits
    uint32_t lru_seq = 0;       // classify calls that used this map (the eviction log's batch number)
    // LRU CT maps: the counts the last GF_EVRING eviction chains left, written by the
    // device to pinned host memory, each behind its own event; cnt_add sums the
    // increments of dev_count_hi (ct_limits), ev_add[k] its value when event k was
    // recorded; ev_pending: the slots recorded since the bound was last set directly
    static constexpr uint32_t GF_EVRING = 8;
    uint32_t *h_evcount = nullptr;
    uint32_t *d_evcount = nullptr;    // its device address (hipHostGetDevicePointer, once)
    hipEvent_t ev_count[GF_EVRING] = {};
    uint64_t ev_add[GF_EVRING] = {};
    uint32_t ev_head = 0, ev_pending = 0;
    uint64_t cnt_add = 0;
    // The multi-map eviction pass (per-endpoint CT maps) records no events: its end
    // kernel stamps the map's count with the call's lru_seq (seq << 32 | count) in
    // pinned memory, st_add[] keeps cnt_add per recent seq, and stamps of calls at or
    // before st_floor (the last time the bound was set directly) are ignored.
    static constexpr uint32_t GF_STRING = 8;
    unsigned long long *h_stamp = nullptr, *d_stamp = nullptr;
    uint32_t st_seq[GF_STRING] = {};
    uint64_t st_add[GF_STRING] = {};
    uint32_t st_floor = 0;
    // get_next_key over a device-authoritative map: a host copy of one chunk of
    // slot headers, and the slot of the key returned last (the dump loop's next
    // argument) so a walk is not needed to resume.
    std::vector<uint8_t> nk_cache;
    uint64_t nk_base = 0, nk_n = 0, nk_gen = ~0ull;
    std::string nk_last_key;
    int64_t nk_last_slot = -1;
    uint64_t nk_last_gen = ~0ull;
    // LPM
    std::map<std::string, std::string, LpmKeyLess> lpm;   // orig key bytes -> value
    uint32_t lpm_len_cnt[129] = {0};
    bool trie_dirty = true;
    DevBuf d_root, d_nodes, d_rsum;   // coverage trie (+ root summary, root_bits 16)
    uint32_t trie_root_bits = 0;
    uint64_t trie_gen = 0;            // trie rebuilds (derived DIR-24-8 tables follow it)
    // IPv4 LPM coverage as DIR-24-8 tables (GF_XDP_DIR24 A/B): tbl24 = 2^24 u16
    // (0 none, 0xffff covered, else 1 + the /24's 256-bit group in tbl8); rebuilt
    // after the trie.  -E2BIG past 65534 groups, -EINVAL for another key size.
    int dir24(hipStream_t s, const uint16_t **t24, const uint32_t **t8);
    DevBuf d_dir24, d_dir8;
    uint64_t dir_gen = ~0ull;
    bool dir_big = false;

    Map(uint32_t t, uint32_t k, uint32_t v, uint32_t m, uint32_t f);
    ~Map();
    bool is_lpm() const { return type == GF_MAP_TYPE_LPM_TRIE; }
    uint32_t lpm_bits() const { return (ksz - 4) * 8; }
    uint32_t n_entries() const { return is_lpm() ? (uint32_t)lpm.size() : (uint32_t)ht.count; }

    // host ops (kernel syscall semantics)
    int update(const uint8_t *key, const uint8_t *value, uint64_t flags);
    int lookup(const uint8_t *key, uint8_t *value);
    int erase(const uint8_t *key);
    int next_key(const uint8_t *key, uint8_t *next);

    // coherence
    int pull();                       // device -> host if !host_valid
    int push(hipStream_t s);          // host -> device if !dev_valid / trie dirty
    // The IPv4 addresses of the keys as a compact open-addressing set for a
    // kernel's LDS (kind 8: {prefixlen 32, addr} keys; kind 20: endpoint keys
    // {addr, 0, 0, 0, family 1}, followed by a second array: each address's slot
    // in the table); rebuilt when the map changed.  zero: address 0's slot + 1
    // (0: absent).  -E2BIG past max_slots, -EINVAL for another key size.
    int addr_set(uint32_t kind, uint32_t max_slots, hipStream_t s, const uint32_t **set, uint32_t *bits, uint32_t *zero);
    DevBuf d_aset;
    uint64_t aset_gen = ~0ull;
    uint32_t aset_kind = 0, aset_bits = 0, aset_zero = 0;
    bool aset_big = false;             // the last build at aset_gen did not fit max_slots
    void device_modified() { host_valid = false; dev_gen++; }
    // Element access on the HBM replica of a device-authoritative hash map (the
    // datapath wrote it last): walks the key's probe sequence with small reads
    // instead of pulling the whole table back (a CT map is tens of GB).
    bool dev_auth() const { return !is_lpm() && !host_valid && dev_valid && d_slots.p; }
    int dev_find(const uint8_t *key, int64_t &slot, int64_t &ins);   // slot: -1 absent; ins: first TOMB/EMPTY
    int dev_get_val(uint64_t i, uint8_t *ext);                       // reference layout
    int dev_put_val(uint64_t i, const uint8_t *ext);
    int dev_count(uint32_t &c);
    int dev_set_count(uint32_t c);
    int dev_next_full(uint64_t start, int64_t &slot);                // first FULL slot >= start, or -1
    void make_fixed_capacity(uint32_t factor = 2);
    void set_hash_mode(uint32_t mode);   // role-specific hashing (gf_key_hash), rehashes
    void set_value_codec(uint32_t codec); // role-specific value layout, converts stored values
    gf_htab_desc hdesc();             // requires push() done
    gf_trie_desc tdesc();             // requires push() done
    uint64_t device_bytes() const { return d_slots.bytes + d_vals.bytes + d_root.bytes + d_nodes.bytes; }
};

struct ProgXdp : Obj {
    gf_xdp_cfg cfg{};
    std::shared_ptr<Map> m4h, m4l, m6h, m6l, lxc;
    ProgXdp() : Obj(ObjKind::ProgXdp) {}
};
struct ProgLb : Obj {
    gf_lb_cfg cfg{};
    std::shared_ptr<Map> lb4, lb6;
    ProgLb() : Obj(ObjKind::ProgLb) {}
};
struct ProgLxc : Obj {
    gf_lxc_cfg cfg{};
    std::shared_ptr<Map> policy, ct4, ct6, cidr4, cidr6, revnat4, revnat6;
    std::shared_ptr<Map> lb4, ipcache, cidr4e, lb6, cidr6e;   // from-container section
    ProgLxc() : Obj(ObjKind::ProgLxc) {}
};
struct PolicyArray : Obj {
    std::map<uint32_t, std::shared_ptr<ProgLxc>> slots;   // lxc_id -> prog
    // device image
    DevBuf d_slot_of_lxc;      // uint16[65536]: 0 = empty, else cfg index + 1
    DevBuf d_cfgs;             // gf_lxc_dev[]
    std::vector<uint8_t> h_cfgs;       // last uploaded program table (change detection)
    std::vector<uint16_t> h_slot_of;
    bool dirty = true;
    std::mutex mu;             // one classify call at a time per array (its device image)
    OrderPt ord;
    PolicyArray() : Obj(ObjKind::PolicyArray) {}
};

struct ProgPipe : Obj {
    gf_pipeline_cfg cfg{};
    std::shared_ptr<ProgXdp> xdp;
    std::shared_ptr<ProgLb> lb;
    std::shared_ptr<Map> lxc;
    std::shared_ptr<PolicyArray> policy;
    ProgPipe() : Obj(ObjKind::ProgPipe) {}
};

// Element ceiling of an insert through the map API (single updates, the host
// path and the device bulk load alike): HASH maps end at max_entries (-E2BIG).
// LRU conntrack maps (which the kernel never lets fail: it evicts) take entries
// up to the slot array's 7/8 load and are brought back under max_entries by the
// eviction sweep of the next classify call that binds them (lru_evict); other
// LRU maps have no eviction path here and end at max_entries like HASH maps.
inline uint64_t dev_insert_limit(const Map &m) {
    return m.type == GF_MAP_TYPE_LRU_HASH && m.ht.codec == GF_VCODEC_CT ? m.ht.nslots / 8 * 7 : m.max_entries;
}

std::shared_ptr<Obj> get_obj(int handle);
std::shared_ptr<Map> get_map(int handle);
int new_handle(std::shared_ptr<Obj> o);
uint32_t host_ifindex();
const gf_node_cfg &node_cfg();
std::shared_ptr<Map> proxy_map(int fam);   // cilium_proxy4 (4) / cilium_proxy6 (6), may be null
std::shared_ptr<Map> node_map(int which);  // 1: cilium_lxc, 2: cilium_tunnel_map (gf_node_cfg), may be null
uint64_t *stats_sink();

// trie builder (host)
void build_trie(const Map &m, std::vector<uint32_t> &root, std::vector<uint8_t> &nodes,
                uint32_t &root_bits);

// Chunked dump of a device-authoritative hash map (gf_kernels.hip): the FULL
// slots of [start, start + range) in slot order, at most `max` of them, keys and
// reference-layout values copied to the host arrays; *next = the slot after the
// last one examined.
int dev_dump(Map &m, uint64_t start, uint32_t max, uint8_t *keys, uint8_t *vals, uint32_t *n, uint64_t *next);

// Bulk insert into a fixed-capacity hash map on the device (gf_map_update_batch
// of >= 4096 entries into an empty or device-authoritative CT-like map), exactly
// the outcome of the sequential updates: *fallback when it cannot guarantee that
// (duplicate keys in the batch, NOEXIST over an existing key, a batch that could
// exceed the element ceiling, no GPU), in which case nothing was written.
int dev_bulk_insert(Map &m, const uint8_t *keys, const uint8_t *vals, uint32_t n, uint64_t flags, bool &fallback);

// Locks the mutexes of a set of maps in address order (deadlock-free), for the
// duration of a classify call's host part.
struct MapLocks {
    std::vector<Map *> held;
    bool locked = false;
    void add(const std::shared_ptr<Map> &m) { if (m && !locked) held.push_back(m.get()); }
    void lock();
    ~MapLocks();
};

}  // namespace gf
