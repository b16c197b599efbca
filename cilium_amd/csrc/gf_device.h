// gf_device.h — device-side table probes for gfx950 (one packet per lane).
//
// Every probe is a plain global load of the slot header (dwordx4 where the
// slot allows it), compare, and linear step; the table descriptor lives in
// kernel arguments (SGPRs).  Values are read/written in place.
#pragma once
#include "gf_common.h"

#define GF_EFAULT 14

namespace gfd {

// Diagnostic build only (GF_WRSTATS=1, tools/variant.sh): every global write of
// the handle_policy path counted by its source, one wave-aggregated add per write
// site (gf_diag_wrstats reads them).  The product build compiles GF_WR away.
#ifndef GF_WRSTATS
#define GF_WRSTATS 0
#endif
enum { WR_OUT = 0, WR_HIT = 1, WR_CARRY = 2, WR_CAS = 3, WR_HDR = 4, WR_HOT = 5, WR_COLD = 6, WR_REL_HOT = 7,
       WR_REL_FULL = 8, WR_REL_NEW = 9, WR_DEL = 10, WR_POLCNT = 11, WR_RLOG = 12, WR_STRICT = 13, WR_N = 16 };
#if GF_WRSTATS
__device__ unsigned long long g_wrstat[WR_N];
__device__ __forceinline__ void wr_count(int k) {
    const uint64_t m = __ballot(1);
    if ((threadIdx.x & 63u) == (uint32_t)__ffsll((unsigned long long)m) - 1u)
        atomicAdd(&g_wrstat[k], (unsigned long long)__popcll(m));
}
#define GF_WR(k) wr_count(k)
#else
#define GF_WR(k) ((void)0)
#endif

// Table pointers reach the kernels inside descriptor structs (kernel arguments
// passed by value, or loaded from the program table), where the compiler can no
// longer see that they point to global memory and would emit flat_* accesses.
// Flat accesses count against both vmcnt and lgkmcnt, so every wait on one also
// drains the LDS traffic of the lane state (and vice versa).  All table accesses
// go through these global-address-space views instead.
#define GF_GLOBAL __attribute__((address_space(1)))
typedef unsigned int gf_u32x4 __attribute__((ext_vector_type(4)));
// Scalars load/store directly; aggregates (uint4, descriptors) move as words.
template <class T>
__device__ __forceinline__ T gload(const void *p) {
    if constexpr (__is_scalar(T)) {
        return *(const GF_GLOBAL T *)p;
    } else if constexpr (sizeof(T) % 16 == 0 && alignof(T) >= 16) {
        gf_u32x4 w[sizeof(T) / 16];
#pragma unroll
        for (unsigned k = 0; k < sizeof(T) / 16; k++) w[k] = ((const GF_GLOBAL gf_u32x4 *)p)[k];
        T v;
        __builtin_memcpy(&v, w, sizeof(T));
        return v;
    } else if constexpr (sizeof(T) % 8 == 0 && alignof(T) >= 8) {
        unsigned long long w[sizeof(T) / 8];
#pragma unroll
        for (unsigned k = 0; k < sizeof(T) / 8; k++) w[k] = ((const GF_GLOBAL unsigned long long *)p)[k];
        T v;
        __builtin_memcpy(&v, w, sizeof(T));
        return v;
    } else if constexpr (sizeof(T) % 4 == 0 && alignof(T) >= 4) {
        unsigned w[sizeof(T) / 4];
#pragma unroll
        for (unsigned k = 0; k < sizeof(T) / 4; k++) w[k] = ((const GF_GLOBAL unsigned *)p)[k];
        T v;
        __builtin_memcpy(&v, w, sizeof(T));
        return v;
    } else {
        static_assert(sizeof(T) % 2 == 0 && alignof(T) >= 2, "gload: half-word aggregates at least");
        unsigned short w[sizeof(T) / 2];
#pragma unroll
        for (unsigned k = 0; k < sizeof(T) / 2; k++) w[k] = ((const GF_GLOBAL unsigned short *)p)[k];
        T v;
        __builtin_memcpy(&v, w, sizeof(T));
        return v;
    }
}
template <class T>
__device__ __forceinline__ void gstore(void *p, T v) {
    if constexpr (__is_scalar(T)) {
        *(GF_GLOBAL T *)p = v;
    } else {
        static_assert(sizeof(T) == 16 && alignof(T) >= 16, "gstore: 16-B aggregates only");
        gf_u32x4 w;
        __builtin_memcpy(&w, &v, 16);
        *(GF_GLOBAL gf_u32x4 *)p = w;
    }
}
// Nontemporal 16-B load (global_load_dwordx4 ... nt): a random line read this
// way ran at 54 G lines/s over a 16-GB table against 39 G/s plain
// (profiles/r4_primbench.txt, "cache policies").
__device__ __forceinline__ uint4 gload_nt16(const void *p) {
    const gf_u32x4 v = __builtin_nontemporal_load((const GF_GLOBAL gf_u32x4 *)p);
    return make_uint4(v[0], v[1], v[2], v[3]);
}
#ifndef GF_CT_NT
#define GF_CT_NT 0          // coop_line64 reads with nontemporal loads
#endif
#ifndef GF_HDR_NT
#define GF_HDR_NT 0         // every probe header load (Hdr::load) nontemporal
#endif
#ifndef GF_CAS_SCOPE
#define GF_CAS_SCOPE __HIP_MEMORY_SCOPE_AGENT
#endif
__device__ __forceinline__ uint32_t gcas(void *p, uint32_t expect, uint32_t want) {
    __hip_atomic_compare_exchange_strong((GF_GLOBAL uint32_t *)p, &expect, want, __ATOMIC_RELAXED,
                                         __ATOMIC_RELAXED, GF_CAS_SCOPE);
    return expect;                                   // the value seen (== expect on success)
}
__device__ __forceinline__ uint32_t gadd32(void *p, uint32_t v) {
    return __hip_atomic_fetch_add((GF_GLOBAL uint32_t *)p, v, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gadd64(void *p, unsigned long long v) {
    (void)__hip_atomic_fetch_add((GF_GLOBAL unsigned long long *)p, v, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gstore_relaxed(void *p, uint32_t v) {
    __hip_atomic_store((GF_GLOBAL uint32_t *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NW>
__device__ __forceinline__ void load_words(const uint8_t *p, uint32_t (&w)[NW]) {
    int k = 0;
#pragma unroll
    for (; k + 4 <= NW; k += 4) {
        uint4 v = *reinterpret_cast<const uint4 *>(p + 4 * k);
        w[k] = v.x; w[k + 1] = v.y; w[k + 2] = v.z; w[k + 3] = v.w;
    }
    if (NW - k >= 2) {
        uint2 v = *reinterpret_cast<const uint2 *>(p + 4 * k);
        w[k] = v.x; w[k + 1] = v.y;
        k += 2;
    }
    if (NW - k == 1) w[k] = *reinterpret_cast<const uint32_t *>(p + 4 * k);
}

template <int KSZ, int MODE = GF_HASH_PLAIN>
__device__ __forceinline__ uint32_t key_hash(const uint32_t *kw) {
    return gf_key_hash(kw, KSZ, MODE);
}

// Slot header = key words + the word holding the state byte, loaded as whole
// dwordx4s (every slot is >= 16 B and a pow2 >= the header, so the rounded-up
// header never leaves the slot).  XW extra words (a multiple of 4) load the
// start of the value with the header (e.g. the policy proxy_port).
template <int KSZ, int XW = 0>
struct Hdr {
    static constexpr int SW = KSZ / 4, SB = KSZ % 4, NW = (SW + 1 + 3) / 4 * 4 + XW;
    uint32_t w[NW];
    __device__ __forceinline__ void load(const uint8_t *s) {
#pragma unroll
        for (int k = 0; k < NW; k += 4) {
            uint4 v = GF_HDR_NT ? gload_nt16(s + 4 * k) : gload<uint4>(s + 4 * k);
            w[k] = v.x; w[k + 1] = v.y; w[k + 2] = v.z; w[k + 3] = v.w;
        }
    }
    __device__ __forceinline__ uint32_t state() const { return (w[SW] >> (8 * SB)) & 0xffu; }
    __device__ __forceinline__ bool eq(const uint32_t *kw) const {
        bool e = true;
#pragma unroll
        for (int k = 0; k < SW; k++) e &= (w[k] == kw[k]);
        if (SB) e &= ((w[SW] & ((1u << (8 * SB)) - 1u)) == kw[SW]);
        return e;
    }
};

// Exact-match probe; returns slot index or -1.  U slot headers are loaded
// together per step (U = slots per 128-B line for the map's layout), so a
// probe that resolves inside its home line costs one memory round trip.
template <int KSZ, int U = 1>
__device__ __forceinline__ int64_t ht_find(const gf_htab_desc &d, const uint32_t *kw, uint32_t h) {
    if (!d.slots) return -1;
    uint64_t i = gf_home_slot(h, d.mask, d.slot_size);
    for (uint64_t p = 0; p <= d.mask; p += U) {
        Hdr<KSZ> hd[U];
#pragma unroll
        for (int u = 0; u < U; u++) hd[u].load(d.slots + ((i + u) & d.mask) * d.slot_size);
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint32_t st = hd[u].state();
            if (st == GF_SLOT_EMPTY) return -1;
            if (st == GF_SLOT_FULL && hd[u].eq(kw)) return (int64_t)((i + u) & d.mask);
        }
        i = (i + U) & d.mask;
    }
    return -1;
}

// Two keys with the same hash (hence the same probe sequence): the CT reverse
// and forward tuples under GF_HASH_CT, the L4 and L3 policy keys of one
// identity under GF_HASH_POLICY.  Key A has priority: returns A's slot if A is
// present, else B's slot (*is_b = true), else -1 — exactly the outcome of
// probing A and then B, with the home line fetched once.
template <int KSZ, int U = 1>
__device__ __forceinline__ int64_t ht_find2(const gf_htab_desc &d, const uint32_t *ka, const uint32_t *kb, uint32_t h,
                                            bool *is_b) {
    *is_b = false;
    if (!d.slots) return -1;
    int64_t fb = -1;
    uint64_t i = gf_home_slot(h, d.mask, d.slot_size);
    for (uint64_t p = 0; p <= d.mask; p += U) {
        Hdr<KSZ> hd[U];
#pragma unroll
        for (int u = 0; u < U; u++) hd[u].load(d.slots + ((i + u) & d.mask) * d.slot_size);
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint32_t st = hd[u].state();
            if (st == GF_SLOT_EMPTY) goto done;
            if (st == GF_SLOT_FULL) {
                if (hd[u].eq(ka)) return (int64_t)((i + u) & d.mask);
                if (fb < 0 && hd[u].eq(kb)) fb = (int64_t)((i + u) & d.mask);
            }
        }
        i = (i + U) & d.mask;
    }
done:
    *is_b = fb >= 0;
    return fb;
}

// The home line of a key, loaded ahead of its use so that probes of different
// tables (CT and policy) are in flight together: U slot headers from the
// first slot of the home line.
template <int KSZ, int U, int XW = 0>
struct ProbeLine {
    Hdr<KSZ, XW> hd[U];
    uint64_t i;
    __device__ __forceinline__ void load(const gf_htab_desc &d, uint32_t h) {
        i = gf_home_slot(h, d.mask, d.slot_size);
        if (!d.slots) return;
#pragma unroll
        for (int u = 0; u < U; u++) hd[u].load(d.slots + ((i + u) & d.mask) * d.slot_size);
    }
    // load() with the home line read by the lane's quad together (coop_line64)
    // when all four lanes of the quad are here; otherwise each lane reads its own.
    // For the layouts whose home step is one 64-B line (CT4: 2 x 32 B, CT6: 64 B).
    __device__ __forceinline__ void load_quad(const gf_htab_desc &d, uint32_t h);
};

// ---- cooperative line loads (the quad of lanes 4q..4q+3 together) ----
// A lane that reads its own 64-B line with four 16-B loads makes four
// wave-instructions that each touch 64 different lines; over a table larger
// than the GPU's page-translation reach (~2-4 GB on MI355X) those run at 16.5 G
// lines/s, against 48 G/s when four lanes read one line with one 16-B load each
// (16 lines per wave-instruction) — profiles/r4_primbench.txt, "tlb".  The CT
// slot arrays are 4-32 GB.  So the quad reads its four lanes' lines together and
// a 4 x 4 transpose over DPP quad permutes hands every lane its own line.
// quad_perm dpp_ctrl: lane i of each quad reads quad lane p_i (p0 | p1 << 2 | ...)
template <int CTRL>
__device__ __forceinline__ uint32_t quad_dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ uint4 quad_dpp4(uint4 v) {
    return make_uint4(quad_dpp<CTRL>(v.x), quad_dpp<CTRL>(v.y), quad_dpp<CTRL>(v.z), quad_dpp<CTRL>(v.w));
}
template <int Q>
__device__ __forceinline__ const uint8_t *quad_bcast_ptr(const uint8_t *p) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = quad_dpp<Q * 0x55>((uint32_t)a), hi = quad_dpp<Q * 0x55>((uint32_t)(a >> 32));
    return (const uint8_t *)(((uint64_t)hi << 32) | lo);
}
// Every lane of each quad must be active (convergent call).  p: the lane's 64-B
// line (16-B aligned), nullptr for none (its words are then zero).
__device__ __forceinline__ void coop_line64(const uint8_t *p, uint32_t (&w)[16]) {
    const uint32_t j = threadIdx.x & 3u;
    uint4 v[4];
    const uint8_t *pq[4] = {quad_bcast_ptr<0>(p), quad_bcast_ptr<1>(p), quad_bcast_ptr<2>(p), quad_bcast_ptr<3>(p)};
#pragma unroll
    for (int q = 0; q < 4; q++)
        v[q] = pq[q] ? (GF_CT_NT ? gload_nt16(pq[q] + 16 * j) : gload<uint4>(pq[q] + 16 * j)) : make_uint4(0, 0, 0, 0);
    // lane j holds chunk j of quad lane q's line in v[q]; wanted: chunk k of its own
    // line in v[k], i.e. out[j][k] = in[k][j].  Stage b (b = 1, 2): keep v[k] where
    // bit b of k equals that of j, else take lane j^b's v[k^b].
    uint4 t[4];
    t[0] = quad_dpp4<0xB1>(v[1]); t[1] = quad_dpp4<0xB1>(v[0]);     // [1,0,3,2]: lane j ^ 1
    t[2] = quad_dpp4<0xB1>(v[3]); t[3] = quad_dpp4<0xB1>(v[2]);
#pragma unroll
    for (int k = 0; k < 4; k++) if (((uint32_t)k ^ j) & 1u) v[k] = t[k];
    t[0] = quad_dpp4<0x4E>(v[2]); t[1] = quad_dpp4<0x4E>(v[3]);     // [2,3,0,1]: lane j ^ 2
    t[2] = quad_dpp4<0x4E>(v[0]); t[3] = quad_dpp4<0x4E>(v[1]);
#pragma unroll
    for (int k = 0; k < 4; k++) if (((uint32_t)k ^ j) & 2u) v[k] = t[k];
#pragma unroll
    for (int k = 0; k < 4; k++) { w[4 * k] = v[k].x; w[4 * k + 1] = v[k].y; w[4 * k + 2] = v[k].z; w[4 * k + 3] = v[k].w; }
}
template <int KSZ, int U, int XW>
__device__ __forceinline__ void ProbeLine<KSZ, U, XW>::load_quad(const gf_htab_desc &d, uint32_t h) {
    constexpr int NW = Hdr<KSZ, XW>::NW;
    static_assert(U * NW == 16, "load_quad: the home step must be one 64-B line");
    const uint64_t here = __ballot(1);
    if (((here >> (threadIdx.x & 60u)) & 0xFull) != 0xFull) { load(d, h); return; }
    i = gf_home_slot(h, d.mask, d.slot_size);
    uint32_t w[16];
    coop_line64(d.slots ? d.slots + i * d.slot_size : nullptr, w);
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int k = 0; k < NW; k++) hd[u].w[k] = w[u * NW + k];
}

// Outcome of a probe walk: the slot of key A, else of key B (is_b), else -1;
// plus where an absent key is inserted — the first FREE slot the walk passed,
// else the EMPTY slot that ended it — and the header word holding its state
// byte as it was observed.
struct ProbeRes {
    int64_t f, empty;
    uint32_t empty_word;
    bool is_b;
    int u;                 // index of the found slot in L.hd (headers still loaded), or -1
};

// ht_find2 continuing from a preloaded home line (key B only when has_b).  The
// walk ends at the first EMPTY slot, as in ht_find2; the first FREE slot before
// it (the LRU eviction pass's reusable slots, gf_common.h) is the insert slot.
template <int KSZ, int U, int XW>
__device__ __forceinline__ ProbeRes probe2(const gf_htab_desc &d, const uint32_t *ka, const uint32_t *kb,
                                           ProbeLine<KSZ, U, XW> &L, bool has_b = true) {
    constexpr int SW = Hdr<KSZ, XW>::SW;
    ProbeRes r{-1, -1, 0u, false, -1};
    if (!d.slots) return r;
    int64_t fb = -1;
    int ub = -1;
    uint64_t i = L.i;
    for (uint64_t p = 0; p <= d.mask; p += U) {
        if (p) {
            ub = -1;                                   // headers of B's line are replaced
#pragma unroll
            for (int u = 0; u < U; u++) L.hd[u].load(d.slots + ((i + u) & d.mask) * d.slot_size);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint32_t st = L.hd[u].state();
            int64_t slot = (int64_t)((i + u) & d.mask);
            if (st == GF_SLOT_EMPTY) {
                if (r.empty < 0) { r.empty = slot; r.empty_word = L.hd[u].w[SW]; }
                goto done;
            }
            if (st == GF_SLOT_FREE && r.empty < 0) { r.empty = slot; r.empty_word = L.hd[u].w[SW]; }
            if (st == GF_SLOT_FULL) {
                if (L.hd[u].eq(ka)) { r.f = slot; r.u = u; return r; }
                if (has_b && fb < 0 && L.hd[u].eq(kb)) { fb = slot; ub = u; }
            }
        }
        i = (i + U) & d.mask;
    }
done:
    r.f = fb;
    r.is_b = fb >= 0;
    r.u = ub;
    return r;
}

// VW value words to p (16-B aligned for every device-written layout: CT values
// sit at voff 16 / 48).
template <int VW>
__device__ __forceinline__ void store_words(uint8_t *p, const uint32_t *v) {
    if ((VW % 4) == 0 && ((uintptr_t)p & 15u) == 0) {
#pragma unroll
        for (int k = 0; k < VW; k += 4) gstore<uint4>(p + 4 * k, make_uint4(v[k], v[k + 1], v[k + 2], v[k + 3]));
    } else {
#pragma unroll
        for (int k = 0; k < VW; k++) gstore<uint32_t>(p + 4 * k, v[k]);
    }
}

// Value bytes of slot i held in the slot (all of them for inline maps, the hot
// 16 B for hot-split CT maps), or the side-array value of a full-split map.
__device__ __forceinline__ uint8_t *ht_val(const gf_htab_desc &d, uint64_t i) {
    return d.vin ? d.slots + i * d.slot_size + d.voff : d.vals + i * d.vsz;
}
// The side-array part of a hot-split value (value bytes vin..vsz).
__device__ __forceinline__ uint8_t *ht_side(const gf_htab_desc &d, uint64_t i) {
    return d.vals + i * d.sstride;
}

// A whole value of VW words into slot i in the map's layout.
template <int VW>
__device__ __forceinline__ void store_value(const gf_htab_desc &d, uint64_t i, const uint32_t *vw) {
    if (!d.sstride) { store_words<VW>(ht_val(d, i), vw); return; }
    if (d.vin == 16 && VW > 4) {                        // hot-split: 4 words inline, the rest aside
        store_words<4>(d.slots + i * d.slot_size + d.voff, vw);
        store_words<VW - 4>(ht_side(d, i), vw + 4);
        GF_WR(WR_HOT); GF_WR(WR_COLD);
        return;
    }
    store_words<VW>(d.vals + i * d.vsz, vw);            // full split
}

// Insert-or-replace (map_update_elem BPF_ANY) for keys owned by the calling
// lane (flow-group exclusivity).  VW = value words.  Returns the
// slot written, or -7 (E2BIG) when a new key would exceed max_entries (strict
// mode) or no empty slot is left.  *added is incremented for a new key.
// hint/hint_word: an EMPTY slot observed by this lane's lookup walk of the same
// home (and the header word seen there), tried first with one CAS.
template <int KSZ, int VW, int MODE, int U = 1>
__device__ __forceinline__ int64_t ht_upsert(const gf_htab_desc &d, const uint32_t *kw, const uint32_t *vw,
                                             bool strict, int *added, bool known_absent = false,
                                             int64_t hint = -1, uint32_t hint_word = 0) {
    constexpr int SW = KSZ / 4, SB = KSZ % 4;
    if (!d.slots) return -7;
    uint32_t h = key_hash<KSZ, MODE>(kw);
    int64_t f = -1;
    if (!known_absent) {                               // lookup walk; its EMPTY slot is the insert hint
        ProbeLine<KSZ, U> L;
        L.load(d, h);
        ProbeRes r = probe2<KSZ, U, 0>(d, kw, kw, L, false);
        f = r.f;
        hint = r.empty;
        hint_word = r.empty_word;
    }
    if (f >= 0) {
        store_value<VW>(d, (uint64_t)f, vw);
        return f;
    }
    if (strict) {
        GF_WR(WR_STRICT);
        uint32_t old = gadd32(d.count, 1u);
        if (old >= d.max_entries) { gadd32(d.count, ~0u); return -7; }
    }
    const uint32_t keep = SB ? (kw[SW] & ((1u << (8 * SB)) - 1u)) : 0u;
    const uint32_t busy = keep | ((uint32_t)GF_SLOT_BUSY << (8 * SB));
    // The claimed (BUSY) slot is this lane's: key, state FULL and value are plain
    // stores (other lanes only ever test the slot for EMPTY, and their claims go
    // through the CAS; the host reads after the kernel).  The header goes out as
    // whole 16-B words when the value starts after the padded header.
    auto fill = [&](uint64_t i) {
        uint8_t *s = d.slots + i * d.slot_size;
        constexpr int NW = Hdr<KSZ>::NW;
        if (d.voff >= 4u * NW) {
            uint32_t h[NW];
#pragma unroll
            for (int k = 0; k < NW; k++) h[k] = k < SW ? kw[k] : 0u;
            h[SW] = keep | ((uint32_t)GF_SLOT_FULL << (8 * SB));
#pragma unroll
            for (int k = 0; k < NW; k += 4) gstore<uint4>(s + 4 * k, make_uint4(h[k], h[k + 1], h[k + 2], h[k + 3]));
            GF_WR(WR_HDR);
        } else {
#pragma unroll
            for (int k = 0; k < SW; k++) gstore<uint32_t>(s + 4 * k, kw[k]);
            gstore<uint32_t>(s + 4 * SW, keep | ((uint32_t)GF_SLOT_FULL << (8 * SB)));
        }
        store_value<VW>(d, i, vw);
        if (!strict) (*added)++;
    };
    // EMPTY or FREE (reusable between launches, gf_common.h) slots are claimed;
    // the key is absent from the whole walk, so any of them keeps every probe exact
    auto claimable = [&](uint32_t w) {
        const uint32_t st = (w >> (8 * SB)) & 0xffu;
        return st == GF_SLOT_EMPTY || st == GF_SLOT_FREE;
    };
    if (hint >= 0 && claimable(hint_word)) {
        uint8_t *sw = d.slots + (uint64_t)hint * d.slot_size + 4 * SW;
        GF_WR(WR_CAS);
        if (gcas(sw, hint_word, busy) == hint_word) { fill((uint64_t)hint); return hint; }
    }
    uint64_t i = gf_home_slot(h, d.mask, d.slot_size);
    for (uint64_t p = 0; p <= d.mask; p++) {
        uint8_t *sw = d.slots + i * d.slot_size + 4 * SW;
        uint32_t cur = gload<uint32_t>(sw);            // a stale view only makes the CAS fail and retry
        for (;;) {
            if (!claimable(cur)) break;
            GF_WR(WR_CAS);
            uint32_t seen = gcas(sw, cur, busy);
            if (seen == cur) { fill(i); return (int64_t)i; }
            cur = seen;
        }
        i = (i + 1) & d.mask;
    }
    if (strict) gadd32(d.count, ~0u);
    return -7;
}

template <int KSZ, int MODE, int U = 1>
__device__ __forceinline__ void ht_delete(const gf_htab_desc &d, const uint32_t *kw, bool strict, int *added) {
    constexpr int SW = KSZ / 4, SB = KSZ % 4;
    int64_t f = ht_find<KSZ, U>(d, kw, key_hash<KSZ, MODE>(kw));
    if (f < 0) return;
    uint8_t *sw = d.slots + (uint64_t)f * d.slot_size + 4 * SW;
    uint32_t cur = gload<uint32_t>(sw);
    uint32_t nv = (cur & ~(0xffu << (8 * SB))) | ((uint32_t)GF_SLOT_TOMB << (8 * SB));
    gstore<uint32_t>(sw, nv);                          // the key is this lane's (group exclusivity)
    GF_WR(WR_DEL);
    if (strict) gadd32(d.count, ~0u);
    else (*added)--;
}

// Coverage-trie membership of an address given as NW raw (LE-loaded) words.
// The words are copied to registers and a byte picked by selects: a dynamic
// index into the caller's array would put that array in scratch.
template <int NW>
struct AddrBytes {
    uint32_t a[NW];
    __device__ __forceinline__ AddrBytes(const uint32_t *aw) {
#pragma unroll
        for (int j = 0; j < NW; j++) a[j] = aw[j];
    }
    __device__ __forceinline__ uint32_t operator()(uint32_t k) const {
        uint32_t w = a[0];
#pragma unroll
        for (int j = 1; j < NW; j++) w = (k >> 2) == (uint32_t)j ? a[j] : w;
        return (w >> (8 * (k & 3))) & 0xffu;
    }
};
// The node levels below the root, from `node` (the root entry - 1).  A node is
// four 32-B groups, one per 64 values of the level's byte (gf_common.h): the
// byte's group alone answers the level — its full and child words in one 16-B
// load and the index of the group's first child in one 4-B load, issued together.
template <int NW>
__device__ __forceinline__ bool trie_nodes(const gf_trie_desc &t, const AddrBytes<NW> &byte_at, uint32_t node) {
    for (uint32_t k = t.root_bits / 8; k < t.addr_bytes; k++) {
        const uint32_t b = byte_at(k);
        const uint8_t *g = t.nodes + (uint64_t)node * GF_TRIE_NODE_BYTES + GF_TRIE_GROUP_BYTES * (b >> 6);
        const uint4 fc = gload<uint4>(g);
        const uint32_t base = gload<uint32_t>(g + 16);
        const uint32_t bit = b & 63u;
        const uint64_t full = fc.x | ((uint64_t)fc.y << 32), child = fc.z | ((uint64_t)fc.w << 32);
        if ((full >> bit) & 1ull) return true;
        if (!((child >> bit) & 1ull)) return false;
        node = base + (uint32_t)__popcll(child & ((1ull << bit) - 1ull));
    }
    return false;
}
template <int NW>
__device__ __forceinline__ bool trie_lookup(const gf_trie_desc &t, const uint32_t *aw) {
    if (!t.root_bits) return false;
    const AddrBytes<NW> byte_at(aw);
    uint32_t idx = t.root_bits == 16 ? ((byte_at(0) << 8) | byte_at(1)) : byte_at(0);
    uint32_t e = gload<uint32_t>(t.root + idx);
    if (e == 0) return false;
    if (e == GF_TRIE_FULL) return true;
    return trie_nodes<NW>(t, byte_at, e - 1);
}

// skb_load_bytes / store / csum_replace bound rules (see oracle.c).
__device__ __forceinline__ bool skb_ok(int32_t off, uint32_t n, uint32_t len) {
    return (uint32_t)off <= 0xffffu && (uint64_t)(uint32_t)off + n <= len;
}
__device__ __forceinline__ bool l4csum_ok(int32_t off, uint32_t len) {
    return (uint32_t)off <= 0xffffu && !(off & 1) && (uint64_t)(uint32_t)off + 2 <= len;
}
__device__ __forceinline__ uint32_t csum_l4_offset(uint32_t nexthdr) {
    return nexthdr == 6 ? 16u : nexthdr == 17 ? 6u : nexthdr == 58 ? 2u : 0u;
}

}  // namespace gfd
