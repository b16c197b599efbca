// gf_maps.cpp — host side of libgpuflow: object registry, the map API that
// replaces the bpf(2) syscall under pkg/bpf (pkg/bpf/bpf.go:84-274), host
// shadows of every map, their HBM replicas, and the coverage-trie builder.
//
// Kernel semantics restated (Linux 6.x kernel/bpf/hashtab.c, lpm_trie.c; the
// kernel is not part of /root/reference, see DESIGN.md "Oracle"):
//   htab: exact match over key_size bytes; update flags ANY/NOEXIST/EXIST
//         (-EINVAL otherwise, -EEXIST/-ENOENT by flag); a NEW key when
//         count == max_entries -> -E2BIG (replacing an existing key is fine);
//         get_next_key: absent/NULL key -> first key, -ENOENT at the end.
//   trie: prefixlen > max -> -EINVAL; NEW key when full -> -ENOSPC; lookup =
//         longest stored prefix with len <= key.prefixlen that matches;
//         get_next_key in post-order (more specific prefixes first).
//   LRU_HASH never fails an insert (the kernel evicts instead).  The conntrack
//   maps (CT key/value shape, GF_VCODEC_CT) accept inserts through the API or the
//   datapath up to the slot array's 7/8 load, and the deterministic LRU stand-in
//   (gf_kernels.hip lru_evict) brings such a map back under
//   max_entries after the next classify call that binds it as ct4 / ct6; between
//   an API insert and that call GetMapInfo may report more than max_entries
//   entries.  Every other LRU map has no eviction path and stops at max_entries
//   with E2BIG (documented deviations; tests/test_maps.py).
#include "gf_internal.h"
#include <string.h>
#include <errno.h>
#include <time.h>
#include <algorithm>
#include <deque>
#include <unordered_map>

namespace gf {

std::shared_mutex &prog_lock() {
    static std::shared_mutex m;
    return m;
}
std::mutex &reg_lock() {
    static std::mutex m;
    return m;
}

void MapLocks::lock() {
    std::sort(held.begin(), held.end());
    held.erase(std::unique(held.begin(), held.end()), held.end());
    for (Map *m : held) m->mu.lock();
    locked = true;
}
MapLocks::~MapLocks() {
    if (!locked) return;
    for (auto it = held.rbegin(); it != held.rend(); ++it) (*it)->mu.unlock();
}

int hip_ok(hipError_t e, const char *what) {
    if (e == hipSuccess) return 0;
    fprintf(stderr, "gpuflow: %s failed: %s\n", what, hipGetErrorString(e));
    return -EIO;
}

DevBuf::~DevBuf() { release(); }
void DevBuf::release() {
    if (p) (void)hipFree(p);
    p = nullptr; bytes = 0;
}
int DevBuf::ensure(size_t n) {
    if (n == bytes && p) return 0;
    release();
    if (n == 0) return 0;
    if (hip_ok(hipMalloc(&p, n), "hipMalloc")) { p = nullptr; return -ENOMEM; }
    bytes = n;
    return 0;
}

// ------------------------------------------------------------------ HTab
void HTab::relayout() {
    if (hot_split == 2) {                       // policy layout (gf_common.h)
        vin = 2;
        voff = ksz + 2;
        slot_size = std::max<uint32_t>(16, gf_pow2ceil32(voff + vin));
        split = 1;
        sstride = (vsz - vin + 7) / 8 * 8;
        return;
    }
    if (hot_split) {
        voff = (ksz + 1 + 15) / 16 * 16;
        vin = 16;
        slot_size = std::max<uint32_t>(16, gf_pow2ceil32(voff + vin));
        split = 1;
        sstride = vsz - vin;
        return;
    }
    gf_htab_layout(ksz, vsz, &slot_size, &voff, &split);
    vin = split ? 0 : vsz;
    sstride = split ? vsz : 0;
}

void HTab::init(uint32_t k, uint32_t v, uint64_t n) {
    ksz = k; vsz = v;
    relayout();
    nslots = n;
    zbytes_reset(slots, nslots * slot_size);
    if (sstride) zbytes_reset(vals, nslots * sstride); else ZBytes().swap(vals);
    count = 0; tombs = 0;
}

void HTab::get_val(uint64_t i, uint8_t *out) const {
    if (vin) memcpy(out, &slots[i * slot_size + voff], vin);
    if (vin < vsz) memcpy(out + vin, &vals[i * sstride], vsz - vin);
}

void HTab::put_val(uint64_t i, const uint8_t *in) {
    if (vin) memcpy(&slots[i * slot_size + voff], in, vin);
    if (vin < vsz) memcpy(&vals[i * sstride], in + vin, vsz - vin);
}

uint32_t HTab::hash(const uint8_t *key) const {
    uint32_t w[16] = {0};
    memcpy(w, key, ksz);
    return gf_key_hash(w, ksz, mode);
}

int64_t HTab::find(const uint8_t *key) const {
    if (!nslots) return -1;
    uint64_t mask = nslots - 1, i = gf_home_slot(hash(key), mask, slot_size);
    for (uint64_t p = 0; p < nslots; p++) {
        uint8_t st = state(i);
        if (st == GF_SLOT_EMPTY) return -1;
        if (st == GF_SLOT_FULL && memcmp(this->key(i), key, ksz) == 0) return (int64_t)i;
        i = (i + 1) & mask;
    }
    return -1;
}

int64_t HTab::insert_new(const uint8_t *key, const uint8_t *value) {
    uint64_t mask = nslots - 1, i = gf_home_slot(hash(key), mask, slot_size);
    for (uint64_t p = 0; p < nslots; p++) {
        uint8_t st = state(i);
        if (st == GF_SLOT_EMPTY || st == GF_SLOT_TOMB || st == GF_SLOT_FREE) {
            if (st != GF_SLOT_EMPTY) tombs--;
            uint8_t *s = &slots[i * slot_size];
            memset(s, 0, slot_size);
            memcpy(s, key, ksz);
            s[ksz] = GF_SLOT_FULL;
            put_val(i, value);
            count++;
            return (int64_t)i;
        }
        i = (i + 1) & mask;
    }
    return -1;
}

void HTab::erase(uint64_t i) {
    set_state(i, GF_SLOT_TOMB);
    count--; tombs++;
}

void HTab::rehash(uint64_t n) {
    if (slots.empty()) { relayout(); nslots = n; count = 0; tombs = 0; return; }   // not materialised: all-empty
    HTab old;
    old.ksz = ksz; old.vsz = vsz; old.slot_size = slot_size; old.voff = voff; old.vin = vin;
    old.sstride = sstride; old.nslots = nslots;
    old.slots.swap(slots); old.vals.swap(vals);
    init(ksz, vsz, n);
    std::vector<uint8_t> v(vsz);
    for (uint64_t i = 0; i < old.nslots; i++) {
        if (old.state(i) != GF_SLOT_FULL) continue;
        old.get_val(i, v.data());
        insert_new(old.key(i), v.data());
    }
}

// ------------------------------------------------------------------ LPM order
static inline int key_bit(const std::string &k, uint32_t bit) {
    return (((uint8_t)k[4 + bit / 8]) >> (7 - bit % 8)) & 1;
}
bool LpmKeyLess::operator()(const std::string &a, const std::string &b) const {
    uint32_t la, lb, maxb = data_bytes * 8;
    memcpy(&la, a.data(), 4); memcpy(&lb, b.data(), 4);
    if (la > maxb) la = maxb;
    if (lb > maxb) lb = maxb;
    uint32_t m = std::min(la, lb);
    for (uint32_t k = 0; k < m; k++) {
        int ba = key_bit(a, k), bb = key_bit(b, k);
        if (ba != bb) return ba < bb;
    }
    if (la == lb) return false;
    return la > lb;   // post-order: the more specific prefix first
}

static uint64_t pow2ceil64(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// ------------------------------------------------------------------ Map
Map::Map(uint32_t t, uint32_t k, uint32_t v, uint32_t m, uint32_t f)
    : Obj(ObjKind::Map), type(t), ksz(k), vsz(v), max_entries(m), flags(f),
      lpm(LpmKeyLess{k > 4 ? k - 4 : 0}) {
    if (!is_lpm()) {
        // LRU maps: a fixed slot array of 4 x max_entries (CT-shaped ones take theirs below), whose
        // 7/8 load bounds inserts between two eviction sweeps (dev_insert_limit)
        if (type == GF_MAP_TYPE_LRU_HASH) { fixed_capacity = true; ht.init(k, v, 0); ht.nslots = pow2ceil64(std::max<uint64_t>(64, 4ull * m)); }
        else ht.init(k, v, 64);
        // Maps of the CT shape (ipv4_ct_tuple / ipv6_ct_tuple -> ct_entry) and of the policy
        // shape (policy_key -> policy_entry) take their datapath layout at creation, while
        // they are empty: it is invisible through the API (the codecs convert) and saves the
        // re-layout of a filled table when a program binds the map later.
        if ((k == 14 || k == 40) && v == GF_CT_VSZ) {
            set_hash_mode(GF_HASH_CT); set_value_codec(GF_VCODEC_CT); make_fixed_capacity(gf_ct_slot_factor(k));
        } else if (k == 8 && v == GF_POL_VSZ) {
            set_hash_mode(GF_HASH_POLICY); set_value_codec(GF_VCODEC_POL);
        }
    }
}

Map::~Map() {
    for (auto &e : ev_count) if (e) (void)hipEventDestroy(e);
    if (h_evcount) (void)hipHostFree(h_evcount);
    if (h_stamp) (void)hipHostFree(h_stamp);
}

// Fixed-capacity maps are materialized lazily: slots.size()==0 means all-empty.
static void materialize(HTab &h) {
    if (h.slots.empty() && h.nslots) {
        zbytes_reset(h.slots, h.nslots * h.slot_size);
        if (h.sstride) zbytes_reset(h.vals, h.nslots * h.sstride);
    }
}

static void codec_encode(uint32_t c, const uint8_t *ext, uint8_t *in) {
    if (c == GF_VCODEC_CT) gf_ct_encode(ext, in);
    else gf_pol_encode(ext, in);
}
static void codec_decode(uint32_t c, const uint8_t *in, uint8_t *ext) {
    if (c == GF_VCODEC_CT) gf_ct_decode(in, ext);
    else gf_pol_decode(in, ext);
}

void Map::set_value_codec(uint32_t c) {
    if (is_lpm() || ht.codec == c) return;
    if (c == GF_VCODEC_CT && vsz != GF_CT_VSZ) return;
    if (c == GF_VCODEC_POL && (vsz != GF_POL_VSZ || ksz != 8)) return;
    pull();
    uint8_t v[GF_CT_VSZ], tmp[GF_CT_VSZ];
    for (uint64_t i = 0; i < (ht.slots.empty() ? 0 : ht.nslots); i++) {
        if (ht.state(i) != GF_SLOT_FULL) continue;
        ht.get_val(i, v);
        if (ht.codec != GF_VCODEC_IDENT) { codec_decode(ht.codec, v, tmp); memcpy(v, tmp, vsz); }
        if (c != GF_VCODEC_IDENT) { codec_encode(c, v, tmp); memcpy(v, tmp, vsz); }
        ht.put_val(i, v);
    }
    ht.codec = c;
    uint32_t hs = c == GF_VCODEC_CT ? 1u : (c == GF_VCODEC_POL ? 2u : 0u);
    if (hs != ht.hot_split) { ht.hot_split = hs; ht.rehash(ht.nslots); }
    host_gen++;                 // a re-layout moves slots: derived caches (addr_set's slot indices) rebuild
    dev_valid = false;
}

void Map::set_hash_mode(uint32_t m) {
    if (is_lpm() || ht.mode == m) return;
    pull();
    ht.mode = m;
    if (!ht.slots.empty()) ht.rehash(ht.nslots);
    host_gen++;
    dev_valid = false;
}


// Maps the device inserts into (CT) get a slot array sized from max_entries
// once, never rehashed by the device.  `factor` slots per entry (gf_ct_slot_factor:
// HBM is plentiful on MI355X; a lightly loaded table resolves almost every probe
// in the home line).  A map already at that capacity is left alone:
// binding a program to it must not pull the table into host memory (tens of GB
// for the bench's CT) nor invalidate the device copy.
void Map::make_fixed_capacity(uint32_t factor) {
    if (is_lpm()) return;
    uint64_t want = pow2ceil64(std::max<uint64_t>(64, (uint64_t)factor * max_entries));
    if (fixed_capacity && want == ht.nslots) return;
    pull();
    fixed_capacity = true;
    if (want != ht.nslots) ht.rehash(want);
    host_gen++;
    dev_valid = false;
}

int Map::pull() {
    if (is_lpm() || host_valid) return 0;
    materialize(ht);
    if (hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize")) return -EIO;
    xfer_d2h += ht.slots.size() + (ht.sstride ? ht.vals.size() : 0);
    if (d_slots.p && hip_ok(hipMemcpy(ht.slots.data(), d_slots.p, ht.slots.size(), hipMemcpyDeviceToHost), "pull slots")) return -EIO;
    if (ht.sstride && d_vals.p && hip_ok(hipMemcpy(ht.vals.data(), d_vals.p, ht.vals.size(), hipMemcpyDeviceToHost), "pull vals")) return -EIO;
    // recount (device inserts/deletes)
    uint64_t c = 0, t = 0;
    for (uint64_t i = 0; i < ht.nslots; i++) {
        uint8_t st = ht.state(i);
        if (st == GF_SLOT_FULL) c++;
        else if (st == GF_SLOT_TOMB || st == GF_SLOT_FREE) t++;
    }
    ht.count = c; ht.tombs = t;
    host_valid = true;
    return 0;
}

int Map::push(hipStream_t s) {
    if (is_lpm()) {
        if (!trie_dirty && d_root.p) return 0;
        std::vector<uint32_t> root; std::vector<uint8_t> nodes; uint32_t rb = 0;
        build_trie(*this, root, nodes, rb);
        int r;
        if ((r = d_root.ensure(root.size() * 4))) return r;
        if ((r = d_nodes.ensure(std::max<size_t>(nodes.size(), GF_TRIE_NODE_BYTES)))) return r;
        if (hip_ok(hipMemcpy(d_root.p, root.data(), root.size() * 4, hipMemcpyHostToDevice), "push trie root")) return -EIO;
        if (!nodes.empty() && hip_ok(hipMemcpy(d_nodes.p, nodes.data(), nodes.size(), hipMemcpyHostToDevice), "push trie nodes")) return -EIO;
        if (rb == 16) {                                // the root summary a kernel can keep in LDS
            std::vector<uint64_t> sum(2 * 1024, 0);
            for (size_t k = 0; k < root.size(); k++) {
                if (root[k] == GF_TRIE_FULL) sum[k >> 6] |= 1ull << (k & 63);
                else if (root[k]) sum[1024 + (k >> 6)] |= 1ull << (k & 63);
            }
            if ((r = d_rsum.ensure(GF_TRIE_RSUM_BYTES))) return r;
            if (hip_ok(hipMemcpy(d_rsum.p, sum.data(), GF_TRIE_RSUM_BYTES, hipMemcpyHostToDevice), "push trie summary"))
                return -EIO;
        }
        trie_root_bits = rb;
        trie_dirty = false;
        trie_gen++;
        return 0;
    }
    if (dev_valid) return 0;
    int r;
    if ((r = d_slots.ensure(ht.nslots * ht.slot_size))) return r;
    if (ht.sstride && (r = d_vals.ensure(ht.nslots * ht.sstride))) return r;
    if ((r = d_count.ensure(8))) return r;
    if (ht.slots.empty()) {
        if (hip_ok(hipMemsetAsync(d_slots.p, 0, d_slots.bytes, s), "memset slots")) return -EIO;
        if (ht.sstride && hip_ok(hipMemsetAsync(d_vals.p, 0, d_vals.bytes, s), "memset vals")) return -EIO;
    } else {
        xfer_h2d += ht.slots.size() + (ht.sstride ? ht.vals.size() : 0);
        if (hip_ok(hipMemcpyAsync(d_slots.p, ht.slots.data(), ht.slots.size(), hipMemcpyHostToDevice, s), "push slots")) return -EIO;
        if (ht.sstride && hip_ok(hipMemcpyAsync(d_vals.p, ht.vals.data(), ht.vals.size(), hipMemcpyHostToDevice, s), "push vals")) return -EIO;
    }
    uint32_t cnt[2] = {(uint32_t)ht.count, 0};
    if (hip_ok(hipMemcpyAsync(d_count.p, cnt, 8, hipMemcpyHostToDevice, s), "push count")) return -EIO;
    if (hip_ok(hipStreamSynchronize(s), "push sync")) return -EIO;
    dev_valid = true;
    return 0;
}

int Map::addr_set(uint32_t kind, uint32_t max_slots, hipStream_t s, const uint32_t **set, uint32_t *bits, uint32_t *zero) {
    std::lock_guard<std::recursive_mutex> g(mu);
    if (is_lpm() || ksz != kind || (kind != 8 && kind != 20)) return -EINVAL;
    if (aset_gen == host_gen && aset_kind == kind && aset_big) return -E2BIG;   // this generation did not fit
    if (aset_gen != host_gen || aset_kind != kind || !d_aset.p) {
        int r;
        if ((r = pull())) return r;
        std::vector<std::pair<uint32_t, uint32_t>> a;   // (address, slot)
        uint32_t z = 0;
        uint32_t w[5];
        for (uint64_t i = 0; i < (ht.slots.empty() ? 0 : ht.nslots); i++) {
            if (ht.state(i) != GF_SLOT_FULL) continue;
            memcpy(w, &ht.slots[i * ht.slot_size], kind);
            uint32_t x;
            if (kind == 8) { if (w[0] != 32u) continue; x = w[1]; }
            else { if (w[1] | w[2] | w[3] || w[4] != 1u) continue; x = w[0]; }
            if (x) a.push_back({x, (uint32_t)i}); else z = (uint32_t)i + 1;
        }
        uint32_t b = 4;                                  // load <= 1/2
        while ((1ull << b) < 2ull * a.size()) b++;
        if ((1ull << b) > max_slots || ht.nslots > 0xffffffffull) {
            aset_gen = host_gen; aset_kind = kind; aset_big = true;
            return -E2BIG;
        }
        // addresses, then (endpoint keys) the slot of each address in the table
        std::vector<uint32_t> t((kind == 20 ? 2u : 1u) << b, 0u);
        for (auto &e : a) {
            uint32_t k = gf_aset_home(e.first, b);
            while (t[k] && t[k] != e.first) k = (k + 1) & ((1u << b) - 1);
            t[k] = e.first;
            if (kind == 20) t[(1u << b) + k] = e.second;
        }
        if ((r = d_aset.ensure(t.size() * 4))) return r;
        // on the call's stream: ordered after the previous call's kernels (CallOrder)
        if (hip_ok(hipMemcpyAsync(d_aset.p, t.data(), t.size() * 4, hipMemcpyHostToDevice, s), "push address set") ||
            hip_ok(hipStreamSynchronize(s), "address set sync"))
            return -EIO;
        aset_gen = host_gen; aset_kind = kind; aset_bits = b; aset_zero = z; aset_big = false;
    }
    *set = (const uint32_t *)d_aset.p; *bits = aset_bits; *zero = aset_zero;
    return 0;
}

int Map::dir24(hipStream_t s, const uint16_t **t24, const uint32_t **t8) {
    std::lock_guard<std::recursive_mutex> g(mu);
    if (!is_lpm() || ksz != 8) return -EINVAL;
    if (dir_gen == trie_gen && dir_big) return -E2BIG;
    if (dir_gen != trie_gen || !d_dir24.p) {
        std::vector<uint16_t> t(1u << 24, 0);
        std::vector<uint32_t> grp;                       // 8 words a group
        // prefixes up to /24 first (whole /24 ranges), then the longer ones as
        // byte ranges in their /24's group (a covered /24 needs none)
        for (auto &kv : lpm) {
            uint32_t L; memcpy(&L, kv.first.data(), 4);
            if (L > 24) continue;
            const uint8_t *a = (const uint8_t *)kv.first.data() + 4;
            const uint32_t i24 = ((uint32_t)a[0] << 16) | ((uint32_t)a[1] << 8) | a[2];
            const uint32_t span = 1u << (24 - L), st = i24 & ~(span - 1);
            std::fill(t.begin() + st, t.begin() + st + span, (uint16_t)0xffff);
        }
        for (auto &kv : lpm) {
            uint32_t L; memcpy(&L, kv.first.data(), 4);
            if (L <= 24) continue;
            const uint8_t *a = (const uint8_t *)kv.first.data() + 4;
            const uint32_t i24 = ((uint32_t)a[0] << 16) | ((uint32_t)a[1] << 8) | a[2];
            if (t[i24] == 0xffff) continue;
            if (!t[i24]) {
                if (grp.size() / 8 >= 65534) { dir_gen = trie_gen; dir_big = true; return -E2BIG; }
                grp.resize(grp.size() + 8, 0u);
                t[i24] = (uint16_t)(grp.size() / 8);
            }
            uint32_t *w = &grp[(t[i24] - 1u) * 8];
            const uint32_t span = 1u << (32 - L), st = a[3] & ~(span - 1);
            for (uint32_t b = st; b < st + span; b++) w[b >> 5] |= 1u << (b & 31);
        }
        if (grp.empty()) grp.assign(8, 0u);
        int r;
        if ((r = d_dir24.ensure(t.size() * 2)) || (r = d_dir8.ensure(grp.size() * 4))) return r;
        if (hip_ok(hipMemcpyAsync(d_dir24.p, t.data(), t.size() * 2, hipMemcpyHostToDevice, s), "push tbl24") ||
            hip_ok(hipMemcpyAsync(d_dir8.p, grp.data(), grp.size() * 4, hipMemcpyHostToDevice, s), "push tbl8") ||
            hip_ok(hipStreamSynchronize(s), "dir24 sync"))
            return -EIO;
        dir_gen = trie_gen; dir_big = false;
    }
    *t24 = (const uint16_t *)d_dir24.p; *t8 = (const uint32_t *)d_dir8.p;
    return 0;
}

gf_htab_desc Map::hdesc() {
    gf_htab_desc d{};
    d.slots = (uint8_t *)d_slots.p;
    d.vals = (uint8_t *)d_vals.p;
    d.count = (uint32_t *)d_count.p;
    d.mask = ht.nslots ? ht.nslots - 1 : 0;
    d.ksz = ksz; d.vsz = vsz; d.slot_size = ht.slot_size; d.voff = ht.voff;
    d.split = ht.split; d.max_entries = max_entries;
    d.vin = ht.vin; d.sstride = ht.sstride;
    return d;
}

gf_trie_desc Map::tdesc() {
    gf_trie_desc d{};
    d.root = (const uint32_t *)d_root.p;
    d.nodes = (const uint8_t *)d_nodes.p;
    d.root_bits = lpm.empty() ? 0 : trie_root_bits;
    d.addr_bytes = ksz - 4;
    d.rsum = (d.root_bits == 16 && d_rsum.p) ? (const uint64_t *)d_rsum.p : nullptr;
    return d;
}


// ------------------------------------------------------------------ device-side element access
// A map the datapath wrote last (CT entries, policy counters, proxy entries) is
// authoritative in HBM.  The map API reaches its elements there directly: the
// key's probe sequence is read in 512-B pieces, values and state bytes are
// written in place, and the element count is the device counter (exact between
// classify calls).  The whole-table pull is kept only for re-layouts.
static int dev_rd(Map &m, void *dst, const void *src, size_t n) {
    m.xfer_d2h += n;
    return hip_ok(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost), "map read") ? -EIO : 0;
}
static int dev_wr(Map &m, void *dst, const void *src, size_t n) {
    m.xfer_h2d += n;
    return hip_ok(hipMemcpy(dst, src, n, hipMemcpyHostToDevice), "map write") ? -EIO : 0;
}

int Map::dev_find(const uint8_t *key, int64_t &slot, int64_t &ins) {
    slot = -1; ins = -1;
    if (hip_ok(hipDeviceSynchronize(), "map sync")) return -EIO;   // kernels that write the map are done
    const uint64_t mask = ht.nslots - 1;
    const uint32_t ss = ht.slot_size, per = std::max<uint32_t>(1, 512 / ss);
    std::vector<uint8_t> buf((size_t)per * ss);
    uint64_t i = gf_home_slot(ht.hash(key), mask, ss);
    for (uint64_t p = 0; p < ht.nslots;) {
        const uint64_t nr = std::min<uint64_t>(per, ht.nslots - i);      // a piece never wraps
        int r = dev_rd(*this, buf.data(), (const uint8_t *)d_slots.p + i * ss, nr * ss);
        if (r) return r;
        for (uint64_t k = 0; k < nr; k++) {
            const uint8_t *sl = &buf[k * ss];
            const uint8_t st = sl[ksz];
            if (st == GF_SLOT_EMPTY) { if (ins < 0) ins = (int64_t)(i + k); return 0; }
            if (st == GF_SLOT_TOMB || st == GF_SLOT_FREE) { if (ins < 0) ins = (int64_t)(i + k); continue; }
            if (st == GF_SLOT_FULL && memcmp(sl, key, ksz) == 0) { slot = (int64_t)(i + k); return 0; }
        }
        p += nr;
        i = (i + nr) & mask;
    }
    return 0;
}

int Map::dev_get_val(uint64_t i, uint8_t *ext) {
    std::vector<uint8_t> inb(vsz);
    uint8_t *in = inb.data();
    int r;
    if (ht.vin && (r = dev_rd(*this, in, (const uint8_t *)d_slots.p + i * ht.slot_size + ht.voff, ht.vin))) return r;
    if (ht.vin < vsz && (r = dev_rd(*this, in + ht.vin, (const uint8_t *)d_vals.p + i * ht.sstride, vsz - ht.vin))) return r;
    if (ht.codec != GF_VCODEC_IDENT) codec_decode(ht.codec, in, ext);
    else memcpy(ext, in, vsz);
    return 0;
}

int Map::dev_put_val(uint64_t i, const uint8_t *ext) {
    std::vector<uint8_t> inb(vsz);
    uint8_t *in = inb.data();
    if (ht.codec != GF_VCODEC_IDENT) codec_encode(ht.codec, ext, in);
    else memcpy(in, ext, vsz);
    int r;
    if (ht.vin && (r = dev_wr(*this, (uint8_t *)d_slots.p + i * ht.slot_size + ht.voff, in, ht.vin))) return r;
    if (ht.vin < vsz && (r = dev_wr(*this, (uint8_t *)d_vals.p + i * ht.sstride, in + ht.vin, vsz - ht.vin))) return r;
    dev_gen++;
    return 0;
}

int Map::dev_count(uint32_t &c) {
    c = 0;
    if (hip_ok(hipDeviceSynchronize(), "map sync")) return -EIO;
    return dev_rd(*this, &c, d_count.p, 4);
}

int Map::dev_set_count(uint32_t c) {
    dev_count_hi = c;
    ev_pending = 0;
    st_floor = lru_seq;
    return dev_wr(*this, d_count.p, &c, 4);
}

// First FULL slot at or after `start` (chunks of slot headers cached on the
// host until the device changes), for get_next_key.
int Map::dev_next_full(uint64_t start, int64_t &slot) {
    slot = -1;
    const uint64_t CH = 65536;
    const uint32_t ss = ht.slot_size;
    for (uint64_t c = start; c < ht.nslots;) {
        const uint64_t base = c / CH * CH;
        if (nk_gen != dev_gen || nk_base != base || nk_n == 0) {
            if (hip_ok(hipDeviceSynchronize(), "map sync")) return -EIO;
            nk_n = std::min<uint64_t>(CH, ht.nslots - base);
            nk_cache.resize(nk_n * ss);
            int r = dev_rd(*this, nk_cache.data(), (const uint8_t *)d_slots.p + base * ss, nk_n * ss);
            if (r) { nk_n = 0; return r; }
            nk_base = base;
            nk_gen = dev_gen;
        }
        for (uint64_t j = c - base; j < nk_n; j++)
            if (nk_cache[j * ss + ksz] == GF_SLOT_FULL) { slot = (int64_t)(base + j); return 0; }
        c = base + nk_n;
    }
    return 0;
}

static int dev_update(Map &m, const uint8_t *key, const uint8_t *value, uint64_t fl, bool &fallback) {
    fallback = false;
    int64_t s, ins;
    int r = m.dev_find(key, s, ins);
    if (r) return r;
    if (s >= 0) {
        if (fl == GF_NOEXIST) return -EEXIST;
        return m.dev_put_val((uint64_t)s, value);
    }
    if (fl == GF_EXIST) return -ENOENT;
    uint32_t c;
    if ((r = m.dev_count(c))) return r;
    if (c >= dev_insert_limit(m)) return -E2BIG;
    // a map the host sizes by element count (load <= 1/2) grows on the host
    if (ins < 0 || (!m.fixed_capacity && ((uint64_t)c + 1) * 2 > m.ht.nslots)) { fallback = true; return 0; }
    const uint32_t ss = m.ht.slot_size;
    std::vector<uint8_t> sl(ss, 0), inb(m.vsz);
    uint8_t *in = inb.data();
    if (m.ht.codec != GF_VCODEC_IDENT) codec_encode(m.ht.codec, value, in);
    else memcpy(in, value, m.vsz);
    memcpy(sl.data(), key, m.ksz);
    sl[m.ksz] = GF_SLOT_FULL;
    if (m.ht.vin) memcpy(&sl[m.ht.voff], in, m.ht.vin);
    if (m.ht.vin < m.vsz && (r = dev_wr(m, (uint8_t *)m.d_vals.p + (uint64_t)ins * m.ht.sstride, in + m.ht.vin,
                                       m.vsz - m.ht.vin)))
        return r;
    if ((r = dev_wr(m, (uint8_t *)m.d_slots.p + (uint64_t)ins * ss, sl.data(), ss))) return r;
    m.dev_gen++;
    return m.dev_set_count(c + 1);
}

// A large table the datapath inserts into (fixed capacity, >= 64 MB of slots) that
// holds nothing yet is written in HBM from its first element on: its replica is
// created there (zeroed) and made authoritative, instead of building a host shadow
// of the whole slot array for a few host writes.  Needs a GPU; without one the host
// path is taken.
static bool go_device(Map &m) {
    if (m.dev_auth() || !m.fixed_capacity || m.is_lpm() || !m.ht.slots.empty() || m.ht.count != 0 || m.ht.tombs != 0)
        return m.dev_auth();
    if (m.ht.nslots * m.ht.slot_size < (64ull << 20)) return false;
    int dc = 0;
    if (hipGetDeviceCount(&dc) != hipSuccess || dc == 0) return false;
    m.dev_valid = false;
    if (m.push((hipStream_t)0)) return false;          // memset replica, count 0
    m.host_valid = false;
    return m.dev_auth();
}

int Map::update(const uint8_t *key, const uint8_t *value, uint64_t fl) {
    host_gen++;
    if (fl > GF_EXIST) return -EINVAL;
    if (is_lpm()) {
        uint32_t plen; memcpy(&plen, key, 4);
        if (plen > lpm_bits()) return -EINVAL;
        std::string k((const char *)key, ksz);
        auto it = lpm.find(k);
        if (it != lpm.end()) {
            if (fl == GF_NOEXIST) return -EEXIST;
            lpm.erase(it);
            lpm.emplace(k, std::string((const char *)value, vsz));
            trie_dirty = true;
            return 0;
        }
        if (fl == GF_EXIST) return -ENOENT;
        if (lpm.size() >= max_entries) return -ENOSPC;
        lpm.emplace(k, std::string((const char *)value, vsz));
        lpm_len_cnt[plen]++;
        trie_dirty = true;
        return 0;
    }
    if (go_device(*this)) {
        bool fallback;
        int r = dev_update(*this, key, value, fl, fallback);
        if (!fallback) return r;
    }
    int r = pull(); if (r) return r;
    materialize(ht);
    uint8_t enc[GF_CT_VSZ];
    if (ht.codec != GF_VCODEC_IDENT) { codec_encode(ht.codec, value, enc); value = enc; }
    int64_t i = ht.find(key);
    if (i >= 0) {
        if (fl == GF_NOEXIST) return -EEXIST;
        ht.put_val((uint64_t)i, value);
        dev_valid = false;
        return 0;
    }
    if (fl == GF_EXIST) return -ENOENT;
    if (ht.count >= dev_insert_limit(*this)) return -E2BIG;
    if (fixed_capacity) {
        if (ht.tombs && (ht.count + ht.tombs + 1) * 4 > ht.nslots * 3) ht.rehash(ht.nslots);   // drop tombstones
    } else if ((ht.count + ht.tombs + 1) * 2 > ht.nslots) {
        ht.rehash(std::max<uint64_t>(64, gf_pow2ceil32((uint32_t)((ht.count + 1) * 4))));
    }
    if (ht.insert_new(key, value) < 0) return -E2BIG;
    dev_valid = false;
    return 0;
}

int Map::lookup(const uint8_t *key, uint8_t *value) {
    if (is_lpm()) {
        uint32_t plen; memcpy(&plen, key, 4);
        if (plen > lpm_bits()) plen = lpm_bits();
        std::string probe((const char *)key, ksz);
        for (int l = (int)plen; l >= 0; l--) {
            if (!lpm_len_cnt[l]) continue;
            uint32_t ul = (uint32_t)l;
            memcpy(&probe[0], &ul, 4);
            auto it = lpm.find(probe);
            if (it != lpm.end()) { memcpy(value, it->second.data(), vsz); return 0; }
        }
        return -ENOENT;
    }
    if (dev_auth()) {
        int64_t s, ins;
        int r = dev_find(key, s, ins);
        if (r) return r;
        if (s < 0) return -ENOENT;
        return dev_get_val((uint64_t)s, value);
    }
    int r = pull(); if (r) return r;
    if (ht.slots.empty()) return -ENOENT;
    int64_t i = ht.find(key);
    if (i < 0) return -ENOENT;
    if (ht.codec != GF_VCODEC_IDENT) { uint8_t v[GF_CT_VSZ]; ht.get_val((uint64_t)i, v); codec_decode(ht.codec, v, value); }
    else ht.get_val((uint64_t)i, value);
    return 0;
}

int Map::erase(const uint8_t *key) {
    host_gen++;
    if (is_lpm()) {
        uint32_t plen; memcpy(&plen, key, 4);
        if (plen > lpm_bits()) return -EINVAL;
        auto it = lpm.find(std::string((const char *)key, ksz));
        if (it == lpm.end()) return -ENOENT;
        lpm.erase(it);
        lpm_len_cnt[plen]--;
        trie_dirty = true;
        return 0;
    }
    if (dev_auth()) {
        int64_t s, ins;
        int r = dev_find(key, s, ins);
        if (r) return r;
        if (s < 0) return -ENOENT;
        const uint8_t tomb = GF_SLOT_TOMB;
        if ((r = dev_wr(*this, (uint8_t *)d_slots.p + (uint64_t)s * ht.slot_size + ksz, &tomb, 1))) return r;
        dev_gen++;
        uint32_t c;
        if ((r = dev_count(c))) return r;
        return dev_set_count(c ? c - 1 : 0);
    }
    int r = pull(); if (r) return r;
    if (ht.slots.empty()) return -ENOENT;
    int64_t i = ht.find(key);
    if (i < 0) return -ENOENT;
    ht.erase((uint64_t)i);
    dev_valid = false;
    return 0;
}

int Map::next_key(const uint8_t *key, uint8_t *next) {
    if (is_lpm()) {
        if (lpm.empty()) return -ENOENT;
        auto it = lpm.end();
        if (key) {
            uint32_t plen; memcpy(&plen, key, 4);
            if (plen <= lpm_bits()) {
                auto f = lpm.find(std::string((const char *)key, ksz));
                if (f != lpm.end()) { it = f; ++it; if (it == lpm.end()) return -ENOENT;
                    memcpy(next, it->first.data(), ksz); return 0; }
            }
        }
        memcpy(next, lpm.begin()->first.data(), ksz);
        return 0;
    }
    if (dev_auth()) {
        uint64_t start = 0;
        int r;
        if (key) {
            if (nk_last_gen == dev_gen && nk_last_slot >= 0 && nk_last_key.size() == ksz &&
                memcmp(nk_last_key.data(), key, ksz) == 0) {
                start = (uint64_t)nk_last_slot + 1;
            } else {
                int64_t s, ins;
                if ((r = dev_find(key, s, ins))) return r;
                if (s >= 0) start = (uint64_t)s + 1;
            }
        }
        int64_t s;
        if ((r = dev_next_full(start, s))) return r;
        if (s < 0) return -ENOENT;
        memcpy(next, &nk_cache[((uint64_t)s - nk_base) * ht.slot_size], ksz);
        nk_last_key.assign((const char *)next, ksz);
        nk_last_slot = s;
        nk_last_gen = dev_gen;
        return 0;
    }
    int r = pull(); if (r) return r;
    if (ht.slots.empty() || ht.count == 0) return -ENOENT;
    uint64_t start = 0;
    if (key) {
        int64_t i = ht.find(key);
        if (i >= 0) start = (uint64_t)i + 1;
    }
    for (uint64_t i = start; i < ht.nslots; i++)
        if (ht.state(i) == GF_SLOT_FULL) { memcpy(next, ht.key(i), ksz); return 0; }
    return -ENOENT;
}

// ------------------------------------------------------------------ trie build
struct BNode {
    uint64_t full[4] = {0, 0, 0, 0};
    BNode *child[256];
    BNode() { memset(child, 0, sizeof child); }
    ~BNode() { for (auto c : child) delete c; }
};

static inline uint32_t addr_bits(const uint8_t *a, uint32_t from, uint32_t n) {
    uint32_t v = 0;
    for (uint32_t k = 0; k < n; k++) v = (v << 1) | ((a[(from + k) / 8] >> (7 - (from + k) % 8)) & 1);
    return v;
}

void build_trie(const Map &m, std::vector<uint32_t> &root, std::vector<uint8_t> &nodes, uint32_t &root_bits) {
    const uint32_t W = m.lpm_bits();
    const uint32_t R = m.lpm.size() > 256 ? 16 : 8;
    root_bits = R;
    std::vector<uint8_t> rfull(1u << R, 0);
    std::vector<BNode *> rchild(1u << R, nullptr);
    for (auto &kv : m.lpm) {
        uint32_t L; memcpy(&L, kv.first.data(), 4);
        const uint8_t *a = (const uint8_t *)kv.first.data() + 4;
        if (L <= R) {
            uint32_t start = L ? addr_bits(a, 0, L) << (R - L) : 0, cnt = 1u << (R - L);
            for (uint32_t e = start; e < start + cnt; e++) { rfull[e] = 1; delete rchild[e]; rchild[e] = nullptr; }
            continue;
        }
        uint32_t idx = addr_bits(a, 0, R);
        if (rfull[idx]) continue;
        if (!rchild[idx]) rchild[idx] = new BNode();
        BNode *n = rchild[idx];
        uint32_t d = R;
        for (;;) {
            uint32_t b = addr_bits(a, d, 8);
            if (L <= d + 8) {
                uint32_t span = 1u << (d + 8 - L), st = b & ~(span - 1);
                for (uint32_t e = st; e < st + span; e++) {
                    n->full[e >> 6] |= 1ull << (e & 63);
                    delete n->child[e]; n->child[e] = nullptr;
                }
                break;
            }
            if ((n->full[b >> 6] >> (b & 63)) & 1) break;
            if (!n->child[b]) n->child[b] = new BNode();
            n = n->child[b];
            d += 8;
        }
        (void)W;
    }
    // BFS serialization: children of a node are contiguous, in byte order.
    root.assign(1u << R, 0);
    std::vector<BNode *> order;
    std::deque<BNode *> q;
    for (uint32_t e = 0; e < (1u << R); e++) {
        if (rfull[e]) root[e] = GF_TRIE_FULL;
        else if (rchild[e]) { root[e] = (uint32_t)order.size() + 1; order.push_back(rchild[e]); q.push_back(rchild[e]); }
    }
    std::unordered_map<BNode *, uint32_t> base;
    size_t head = 0;
    while (head < order.size()) {
        BNode *n = order[head++];
        base[n] = (uint32_t)order.size();
        for (int b = 0; b < 256; b++)
            if (n->child[b] && !((n->full[b >> 6] >> (b & 63)) & 1)) order.push_back(n->child[b]);
    }
    nodes.assign(order.size() * GF_TRIE_NODE_BYTES, 0);
    for (size_t i = 0; i < order.size(); i++) {
        BNode *n = order[i];
        uint8_t *o = &nodes[i * GF_TRIE_NODE_BYTES];
        uint64_t ch[4] = {0, 0, 0, 0};
        for (int b = 0; b < 256; b++)
            if (n->child[b] && !((n->full[b >> 6] >> (b & 63)) & 1)) ch[b >> 6] |= 1ull << (b & 63);
        uint32_t cb = base[n];                       // the node's first child
        for (int w = 0; w < 4; w++) {                // group w: full, child, first child of the group
            uint8_t *g = o + GF_TRIE_GROUP_BYTES * w;
            memcpy(g, &n->full[w], 8);
            memcpy(g + 8, &ch[w], 8);
            memcpy(g + 16, &cb, 4);
            cb += (uint32_t)__builtin_popcountll(ch[w]);
        }
    }
    for (auto c : rchild) delete c;
}

// ------------------------------------------------------------------ registry
struct Registry {
    std::map<int, std::shared_ptr<Obj>> handles;
    std::map<std::string, std::shared_ptr<Obj>> pins;
    int next = 3;      // like fds: 0/1/2 are never handed out
    uint32_t host_ifindex = 1;
    uint64_t *stats = nullptr;
    gf_node_cfg node{};
    std::shared_ptr<Map> px4, px6, lxc, tunnel;
};
static Registry &reg() { static Registry r; return r; }

std::shared_ptr<Obj> get_obj(int h) {
    std::lock_guard<std::mutex> g(reg_lock());
    auto &r = reg();
    auto it = r.handles.find(h);
    return it == r.handles.end() ? nullptr : it->second;
}
std::shared_ptr<Map> get_map(int h) {
    auto o = get_obj(h);
    if (!o || o->kind != ObjKind::Map) return nullptr;
    return std::static_pointer_cast<Map>(o);
}
int new_handle(std::shared_ptr<Obj> o) {
    std::lock_guard<std::mutex> g(reg_lock());
    auto &r = reg();
    int h = r.next++;
    r.handles[h] = std::move(o);
    return h;
}
uint32_t host_ifindex() { return reg().host_ifindex; }
const gf_node_cfg &node_cfg() { return reg().node; }
std::shared_ptr<Map> proxy_map(int fam) { return fam == 6 ? reg().px6 : reg().px4; }
std::shared_ptr<Map> node_map(int which) { return which == 1 ? reg().lxc : reg().tunnel; }
uint64_t *stats_sink() { return reg().stats; }

}  // namespace gf

using namespace gf;

// ================================================================== C ABI
extern "C" {

int gf_map_create(uint32_t map_type, uint32_t key_size, uint32_t value_size,
                  uint32_t max_entries, uint32_t map_flags) {
    if (!key_size || !value_size || !max_entries) return -EINVAL;
    switch (map_type) {
    case GF_MAP_TYPE_HASH:
    case GF_MAP_TYPE_LRU_HASH:
        if (map_flags & ~(GF_F_NO_PREALLOC | GF_F_NO_COMMON_LRU)) return -EINVAL;
        if (key_size > 512) return -E2BIG;
        if (key_size > 64) return -EINVAL;          /* libgpuflow limit (all path keys <= 40 B) */
        break;
    case GF_MAP_TYPE_LPM_TRIE:
        /* trie_alloc checks (kernel/bpf/lpm_trie.c) */
        if (!(map_flags & GF_F_NO_PREALLOC) || (map_flags & ~GF_F_NO_PREALLOC)) return -EINVAL;
        if (key_size < 5 || key_size > 4 + 16) return -EINVAL;  /* libgpuflow: IPv4/IPv6 tries */
        if (value_size > 4096) return -EINVAL;
        break;
    default:
        return -EINVAL;
    }
    auto m = std::make_shared<Map>(map_type, key_size, value_size, max_entries, map_flags);
    return new_handle(m);
}

int gf_map_update_elem(int h, const void *key, const void *value, uint64_t flags) {
    auto m = get_map(h);
    if (!m) return -EBADF;
    std::lock_guard<std::recursive_mutex> g(m->mu);
    if (!key || !value) return -EFAULT;
    return m->update((const uint8_t *)key, (const uint8_t *)value, flags);
}

int gf_map_update_batch(int h, const void *keys, const void *values, uint32_t n,
                        uint64_t flags, uint32_t *n_done) {
    auto m = get_map(h);
    if (n_done) *n_done = 0;
    if (!m) return -EBADF;
    std::lock_guard<std::recursive_mutex> g(m->mu);
    if (n && (!keys || !values)) return -EFAULT;
    m->host_gen++;
    if (n >= 4096 && m->fixed_capacity && !m->is_lpm() && (flags == GF_ANY || flags == GF_NOEXIST) &&
        (m->dev_auth() || (m->ht.slots.empty() && m->ht.count == 0))) {
        // a table the datapath inserts into, filled in bulk (the agent restoring a CT,
        // a benchmark's pre-population): loaded in HBM directly, no host shadow built
        bool fallback = false;
        int r = dev_bulk_insert(*m, (const uint8_t *)keys, (const uint8_t *)values, n, flags, fallback);
        if (!fallback) {
            if (!r && n_done) *n_done = n;
            return r;
        }
    }
    for (uint32_t i = 0; i < n; i++) {
        int r = m->update((const uint8_t *)keys + (size_t)i * m->ksz,
                          (const uint8_t *)values + (size_t)i * m->vsz, flags);
        if (r) return r;
        if (n_done) *n_done = i + 1;
    }
    return 0;
}

int gf_map_lookup_elem(int h, const void *key, void *value) {
    auto m = get_map(h);
    if (!m) return -EBADF;
    std::lock_guard<std::recursive_mutex> g(m->mu);
    if (!key || !value) return -EFAULT;
    return m->lookup((const uint8_t *)key, (uint8_t *)value);
}

int gf_map_delete_elem(int h, const void *key) {
    auto m = get_map(h);
    if (!m) return -EBADF;
    std::lock_guard<std::recursive_mutex> g(m->mu);
    if (!key) return -EFAULT;
    return m->erase((const uint8_t *)key);
}

int gf_map_get_next_key(int h, const void *key, void *next_key) {
    auto m = get_map(h);
    if (!m) return -EBADF;
    std::lock_guard<std::recursive_mutex> g(m->mu);
    if (!next_key) return -EFAULT;
    return m->next_key((const uint8_t *)key, (uint8_t *)next_key);
}

// Chunked dump: what DumpWithCallback (pkg/bpf/map.go:319-369) obtains with one
// GetNextKey + LookupElement pair per entry, a chunk of entries per call (the
// kernel's later BPF_MAP_LOOKUP_BATCH contract).  Cursor = slot index (hash
// maps) or ordinal (LPM tries, post-order).
int gf_map_lookup_batch(int h, const uint64_t *in_batch, uint64_t *out_batch, void *keys, void *values,
                        uint32_t *count) {
    auto m = get_map(h);
    if (!m) return -EBADF;
    if (!out_batch || !count || (*count && (!keys || !values))) return -EFAULT;
    std::lock_guard<std::recursive_mutex> g(m->mu);
    const uint32_t want = *count;
    uint64_t cur = in_batch ? *in_batch : 0;
    uint8_t *ko = (uint8_t *)keys, *vo = (uint8_t *)values;
    uint32_t n = 0;
    *count = 0;
    if (m->is_lpm()) {
        uint64_t k = 0;
        auto it = m->lpm.begin();
        for (; it != m->lpm.end() && k < cur; ++it, ++k) {}
        for (; it != m->lpm.end() && n < want; ++it, ++k, ++n) {
            memcpy(ko + (size_t)n * m->ksz, it->first.data(), m->ksz);
            memcpy(vo + (size_t)n * m->vsz, it->second.data(), m->vsz);
        }
        *count = n; *out_batch = k;
        return it == m->lpm.end() ? -ENOENT : 0;
    }
    if (m->dev_auth()) {
        if (hip_ok(hipDeviceSynchronize(), "map sync")) return -EIO;
        while (n < want && cur < m->ht.nslots) {
            uint32_t got = 0;
            uint64_t next = cur;
            int r = dev_dump(*m, cur, want - n, ko + (size_t)n * m->ksz, vo + (size_t)n * m->vsz, &got, &next);
            if (r) return r;
            n += got; cur = next;
        }
        *count = n; *out_batch = cur;
        return cur >= m->ht.nslots ? -ENOENT : 0;
    }
    int r = m->pull();
    if (r) return r;
    const HTab &t = m->ht;
    if (t.slots.empty()) { *out_batch = t.nslots; return -ENOENT; }
    std::vector<uint8_t> v(m->vsz);
    for (; cur < t.nslots && n < want; cur++) {
        if (t.state(cur) != GF_SLOT_FULL) continue;
        memcpy(ko + (size_t)n * m->ksz, t.key(cur), m->ksz);
        t.get_val(cur, v.data());
        if (t.codec != GF_VCODEC_IDENT) codec_decode(t.codec, v.data(), vo + (size_t)n * m->vsz);
        else memcpy(vo + (size_t)n * m->vsz, v.data(), m->vsz);
        n++;
    }
    while (cur < t.nslots && t.state(cur) != GF_SLOT_FULL) cur++;     // ENOENT as soon as nothing is left
    *count = n; *out_batch = cur;
    return cur >= t.nslots ? -ENOENT : 0;
}

int gf_map_get_info(int h, gf_map_info *info) {
    auto m = get_map(h);
    if (!m) return -EBADF;
    std::lock_guard<std::recursive_mutex> g(m->mu);
    if (!info) return -EFAULT;
    info->map_type = m->type; info->key_size = m->ksz; info->value_size = m->vsz;
    info->max_entries = m->max_entries; info->map_flags = m->flags;
    info->n_entries = m->n_entries();
    if (m->dev_auth()) {                 // the device counter (exact between classify calls)
        uint32_t c;
        int r = m->dev_count(c);
        if (r) return r;
        info->n_entries = c;
    } else if (!m->host_valid) {
        int r = m->pull();
        if (r) return r;
        info->n_entries = m->n_entries();
    }
    info->device_bytes = m->device_bytes();
    info->xfer_d2h = m->xfer_d2h;
    info->xfer_h2d = m->xfer_h2d;
    return 0;
}

int gf_obj_pin(int h, const char *path) {
    auto o = get_obj(h);
    if (!o) return -EBADF;
    if (!path || !*path) return -EINVAL;
    std::lock_guard<std::mutex> g(reg_lock());
    auto &r = reg();
    if (r.pins.count(path)) return -EEXIST;
    r.pins[path] = o;
    return 0;
}

int gf_obj_get(const char *path) {
    if (!path) return -EFAULT;
    std::shared_ptr<Obj> o;
    {
        std::lock_guard<std::mutex> g(reg_lock());
        auto &r = reg();
        auto it = r.pins.find(path);
        if (it == r.pins.end()) return -ENOENT;
        o = it->second;
    }
    return new_handle(o);
}

int gf_obj_unpin(const char *path) {
    if (!path) return -EFAULT;
    std::lock_guard<std::mutex> g(reg_lock());
    return reg().pins.erase(path) ? 0 : -ENOENT;
}

int gf_obj_close(int h) {
    std::shared_ptr<Obj> o;              // released outside the registry lock
    std::lock_guard<std::mutex> g(reg_lock());
    auto it = reg().handles.find(h);
    if (it == reg().handles.end()) return -EBADF;
    o = std::move(it->second);
    reg().handles.erase(it);
    return 0;
}

uint32_t gf_now_sec(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint32_t)((uint64_t)ts.tv_sec + (uint64_t)ts.tv_nsec / 1000000000ull);
}

int gf_node_config(const gf_node_cfg *cfg) {
    std::unique_lock<std::shared_mutex> g(prog_lock());
    if (!cfg) return -EFAULT;
    std::shared_ptr<Map> m4, m6;
    if (cfg->proxy4_map) {
        m4 = get_map(cfg->proxy4_map);
        if (!m4) return -EBADF;
        if (m4->ksz != 10 || m4->vsz != 16 || m4->is_lpm()) return -EINVAL;
    }
    if (cfg->proxy6_map) {
        m6 = get_map(cfg->proxy6_map);
        if (!m6) return -EBADF;
        if (m6->ksz != 22 || m6->vsz != 28 || m6->is_lpm()) return -EINVAL;
    }
    std::shared_ptr<Map> lxc, tun;
    if (cfg->lxc_map) {
        lxc = get_map(cfg->lxc_map);
        if (!lxc) return -EBADF;
        if (lxc->ksz != 20 || lxc->vsz != 112 || lxc->is_lpm()) return -EINVAL;
    }
    if (cfg->tunnel_map) {
        tun = get_map(cfg->tunnel_map);
        if (!tun) return -EBADF;
        if (tun->ksz != 20 || tun->vsz != 20 || tun->is_lpm()) return -EINVAL;
    }
    // the datapath inserts into the proxy maps: fixed slot arrays (1/2 load at max_entries)
    for (auto &m : {m4, m6}) if (m) { std::lock_guard<std::recursive_mutex> mg(m->mu); m->make_fixed_capacity(2); }
    reg().host_ifindex = cfg->host_ifindex;
    reg().node = *cfg;
    reg().px4 = m4; reg().px6 = m6;
    reg().lxc = lxc; reg().tunnel = tun;
    return 0;
}

int gf_set_stats_sink(uint64_t *dev_counters) {
    std::unique_lock<std::shared_mutex> g(prog_lock());
    reg().stats = dev_counters;
    return 0;
}

void *gf_dev_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    return p;
}
int gf_dev_free(void *p) { return hip_ok(hipFree(p), "hipFree"); }
int gf_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream) {
    return hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream), "h2d");
}
int gf_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream) {
    return hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream), "d2h");
}
int gf_stream_sync(void *stream) { return hip_ok(hipStreamSynchronize((hipStream_t)stream), "sync"); }
int gf_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
const char *gf_version(void) { return "gpuflow 0.1 (gfx950)"; }
#ifndef GF_SRC_SHA
#define GF_SRC_SHA "unknown"
#endif
const char *gf_build_id(void) { return GF_SRC_SHA; }

}  // extern "C"
