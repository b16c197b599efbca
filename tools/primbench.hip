// primbench.hip — rates of the memory primitives the flow-group kernels are built
// from, on MI355X.  Two parts:
//
//   legacy   (r1, profiles/r1_primbench.txt): random 16-B loads from an 8 GB
//            table, slot RMW, u64 atomics, hot-address atomics, 8-B scatter.
//   matrix   (r4, profiles/r4_primbench.txt): the random-request ceiling as a
//            function of what k_ing_groups actually does —
//     rd  <W,L>   flooded grid, every lane L independent random W-byte reads
//                 (W = 16: one 16-B load into a random 64-B line; 64 / 128: the
//                 whole line with 4 / 8 16-B loads), footprints 128 MB (fits
//                 the 256-MB Infinity Cache), 2 GB, 16 GB
//     chain<L>    persistent grid of WPS waves per SIMD (1..8), every lane a
//                 dependent chain: L independent random 16-B loads whose
//                 addresses come from the previous step's data (the shape of a
//                 lane running its bucket packet after packet)
//     st  <W>     random W-byte stores (4, 8, 16, 32, 64, 128) into random lines
//     at  <K>     K u64 atomicAdds per lane into one random 16-B pair (K = 1, 2)
//     mix         one random 16-B read + one independent random 16-B store
//     rmw         16-B read + 8-B store into the same random 64-B line
//     seq         coalesced 16-B/lane streaming read / write (PMC byte calibration)
//   Each kernel is its own template instance, so a rocprofv3 --pmc pass gives its
//   requests per access (TCC_EA0_RDREQ / _32B / _128B, WRREQ / _64B, ATOMIC).
//
//   hipcc -O3 --offload-arch=gfx950 tools/primbench.hip -o tools/_bin/primbench
//   tools/_bin/primbench [matrix|legacy|all|tlb|pol]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

// ---------------------------------------------------------------- legacy (r1)
__global__ void k_rd(const uint8_t *buf, uint64_t nslots, uint32_t *out, uint32_t salt) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint4 v = *reinterpret_cast<const uint4 *>(buf + (mix(t + salt) % nslots) * 64);
    if (v.x == 0x12345678u) out[t & 1023] = v.y;
}
__global__ void k_rmw(uint8_t *buf, uint64_t nslots, uint32_t salt) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint8_t *s = buf + (mix(t + salt) % nslots) * 64;
    uint4 v = *reinterpret_cast<const uint4 *>(s + 32);
    *reinterpret_cast<uint2 *>(s + 32) = make_uint2(v.x + 1, v.y ^ 3);
}
__global__ void k_rmw_acct(uint8_t *buf, uint64_t nslots, uint32_t salt) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint8_t *s = buf + (mix(t + salt) % nslots) * 64;
    uint4 v = *reinterpret_cast<const uint4 *>(s + 32);
    uint4 c = *reinterpret_cast<const uint4 *>(s);
    *reinterpret_cast<uint2 *>(s + 32) = make_uint2(v.x + 1, v.y ^ 3);
    *reinterpret_cast<uint4 *>(s) = make_uint4(c.x + 1, c.y, c.z + 100, c.w);
}
__global__ void k_atom(unsigned long long *buf, uint64_t nslots, uint32_t salt) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    unsigned long long *p = buf + (mix(t + salt) % nslots) * 8;
    atomicAdd(&p[0], 1ull);
    atomicAdd(&p[1], 100ull);
}
__global__ void k_atom_hot(unsigned long long *buf, uint32_t nhot, uint32_t salt) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    atomicAdd(&buf[(mix(t + salt) % nhot) * 8], 1ull);
}
__global__ void k_scatter(const uint32_t *perm, uint2 *out, uint32_t n) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) out[perm[t]] = make_uint2(t, t ^ 7);
}
__global__ void k_coal(uint2 *out, uint32_t n) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) out[t] = make_uint2(t, t ^ 7);
}
__global__ void k_blockflush(unsigned long long *ctr, uint32_t nbins) {
    __shared__ uint32_t s;
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    atomicAdd(&s, 1u);
    __syncthreads();
    if (threadIdx.x < nbins) atomicAdd(&ctr[threadIdx.x], (unsigned long long)s);
}
// a bijective multiplicative permutation mod 2^k
__global__ void k_perm_mul(uint32_t *perm, uint32_t n) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) perm[t] = (uint32_t)(((uint64_t)t * 2654435761ull + 12345) & (n - 1));
}

static double timeit(hipEvent_t a, hipEvent_t b) {
    float ms; CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b)); return ms;
}

static void legacy(uint8_t *big, uint64_t big_bytes) {
    const uint64_t CT = 8ull << 30, POL = 256ull << 20;
    const uint32_t N = 1u << 24;              // 16.8M packets
    uint8_t *ct = big, *pol = big + CT; uint32_t *out, *perm; uint2 *o8; unsigned long long *hot;
    if (big_bytes < CT + POL) { printf("legacy: table too small\n"); return; }
    CK(hipMalloc(&out, 4096)); CK(hipMalloc(&perm, N * 4ull)); CK(hipMalloc(&o8, N * 8ull));
    CK(hipMalloc(&hot, 1 << 20)); CK(hipMemset(hot, 0, 1 << 20));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    dim3 B(256), G(N / 256);
    double ms;
    CK(hipEventRecord(a)); hipLaunchKernelGGL(k_rd, G, B, 0, 0, ct, CT / 64, out, 0); CK(hipEventRecord(b));
    ms = timeit(a, b); printf("legacy random 16B load, 8GB table      : %7.3f ms per 16.8M  %6.2f G/s\n", ms, N / ms / 1e6);
    CK(hipEventRecord(a)); hipLaunchKernelGGL(k_rmw, G, B, 0, 0, ct, CT / 64, 0); CK(hipEventRecord(b));
    ms = timeit(a, b); printf("legacy random slot RMW (16B ld+8B st)  : %7.3f ms per 16.8M  %6.2f G/s\n", ms, N / ms / 1e6);
    CK(hipEventRecord(a)); hipLaunchKernelGGL(k_rmw_acct, G, B, 0, 0, ct, CT / 64, 0); CK(hipEventRecord(b));
    ms = timeit(a, b); printf("legacy random slot RMW + acct (2x16B)  : %7.3f ms per 16.8M  %6.2f G/s\n", ms, N / ms / 1e6);
    CK(hipEventRecord(a)); hipLaunchKernelGGL(k_atom, G, B, 0, 0, (unsigned long long *)pol, POL / 64, 0); CK(hipEventRecord(b));
    ms = timeit(a, b); printf("legacy 2x atomicAdd u64, 256MB random  : %7.3f ms per 16.8M  %6.2f G pkt/s\n", ms, N / ms / 1e6);
    for (uint32_t nh : {1u, 32u, 1024u}) {
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_atom_hot, G, B, 0, 0, hot, nh, 0); CK(hipEventRecord(b));
        ms = timeit(a, b); printf("legacy atomicAdd u64 into %5u hot     : %7.3f ms per 16.8M  %6.2f G/s\n", nh, ms, N / ms / 1e6);
    }
    hipLaunchKernelGGL(k_perm_mul, G, B, 0, 0, perm, N);
    CK(hipEventRecord(a)); hipLaunchKernelGGL(k_scatter, G, B, 0, 0, perm, o8, N); CK(hipEventRecord(b));
    ms = timeit(a, b); printf("legacy 8B scatter via permutation 134MB: %7.3f ms per 16.8M  %6.2f G/s\n", ms, N / ms / 1e6);
    CK(hipEventRecord(a)); hipLaunchKernelGGL(k_coal, G, B, 0, 0, o8, N); CK(hipEventRecord(b));
    ms = timeit(a, b); printf("legacy 8B coalesced store 134MB        : %7.3f ms per 16.8M  %6.2f G/s\n", ms, N / ms / 1e6);
    CK(hipFree(out)); CK(hipFree(perm)); CK(hipFree(o8)); CK(hipFree(hot));
    fflush(stdout);
}

// ---------------------------------------------------------------- matrix (r4)
// A line is 64 B; a "128-B" access reads the line pair [2k, 2k+1].
// rd<W, L>: each lane L independent accesses, W bytes each
template <int W, int L>
__global__ __launch_bounds__(256) void k_mrd(const uint4 *__restrict__ tab, uint64_t lmask, uint32_t *sink, uint32_t salt) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    constexpr int V = W >= 32 ? W / 16 : 1;             // 16-B loads per access
    uint4 v[L][V];
#pragma unroll
    for (int k = 0; k < L; k++) {
        uint64_t line = mix(t * L + k + salt) & lmask;
        if (W == 128) line &= ~1ull;
#pragma unroll
        for (int j = 0; j < V; j++) v[k][j] = tab[line * 4 + j];
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < L; k++)
#pragma unroll
        for (int j = 0; j < V; j++) acc ^= v[k][j].x + v[k][j].w;
    if (acc == 0x9e3779b9u) sink[t & 1023] = acc;
}
// xcd: the table split into 8 slices, block b reading only slice b % 8 — the XCD the
// dispatcher places it on — so each XCD's L2 holds one slice (an endpoint-partitioned
// policy layout's best case).
__global__ __launch_bounds__(256) void k_mrd_xcd(const uint4 *__restrict__ tab, uint64_t slice_mask, uint32_t *sink,
                                                 uint32_t salt) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t line = (mix(t + salt) & slice_mask) + (uint64_t)(blockIdx.x & 7u) * (slice_mask + 1);
    const uint4 v = tab[line * 4];
    const uint32_t acc = v.x + v.w;
    if (acc == 0x9e3779b9u) sink[t & 1023] = acc;
}
// coop: the 64-B line read cooperatively, 4 consecutive lanes per line and one
// 16-B load each (16 lines per wave-instruction instead of 64)
__global__ __launch_bounds__(256) void k_mrd_coop(const uint4 *__restrict__ tab, uint64_t lmask, uint32_t *sink, uint32_t salt) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t line = mix((t >> 2) + salt) & lmask;
    const uint4 v = tab[line * 4 + (t & 3)];
    if ((v.x ^ v.w) == 0x9e3779b9u) sink[t & 1023] = v.y;
}
typedef unsigned int vu4 __attribute__((ext_vector_type(4)));
// request size of a random 16-B read under each cache policy: plain, nontemporal
// (nt), agent-coherent (sc1), system-coherent (sc0 sc1), and the same on an
// uncached (hipDeviceMallocUncached) allocation
template <int POL>
__global__ __launch_bounds__(256) void k_mrd_pol(const uint4 *__restrict__ tab, uint64_t lmask, uint32_t *sink, uint32_t salt) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint4 *p = tab + (mix(t + salt) & lmask) * 4;
    uint4 v;
    if constexpr (POL == 0) v = *p;
    else if constexpr (POL == 1) { const vu4 x = __builtin_nontemporal_load((const vu4 *)p); v = make_uint4(x[0], x[1], x[2], x[3]); }
    else if constexpr (POL == 2) { vu4 x; asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(p) : "memory"); v = make_uint4(x[0], x[1], x[2], x[3]); }
    else { vu4 x; asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(p) : "memory"); v = make_uint4(x[0], x[1], x[2], x[3]); }
    if ((v.x ^ v.w) == 0x9e3779b9u) sink[t & 1023] = v.y;
}
// the same four policies on the cooperative 64-B line read
template <int POL>
__global__ __launch_bounds__(256) void k_mrd_coop_pol(const uint4 *__restrict__ tab, uint64_t lmask, uint32_t *sink, uint32_t salt) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint4 *p = tab + (mix((t >> 2) + salt) & lmask) * 4 + (t & 3);
    uint4 v;
    if constexpr (POL == 0) v = *p;
    else if constexpr (POL == 1) { const vu4 x = __builtin_nontemporal_load((const vu4 *)p); v = make_uint4(x[0], x[1], x[2], x[3]); }
    else if constexpr (POL == 2) { vu4 x; asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(p) : "memory"); v = make_uint4(x[0], x[1], x[2], x[3]); }
    else { vu4 x; asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(p) : "memory"); v = make_uint4(x[0], x[1], x[2], x[3]); }
    if ((v.x ^ v.w) == 0x9e3779b9u) sink[t & 1023] = v.y;
}
// partial 16-B and full 64-B stores, nontemporal, and the cooperative full-line store
template <int POL>
__global__ __launch_bounds__(256) void k_mst_pol(uint4 *__restrict__ tab, uint64_t lmask, uint32_t salt) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const vu4 v = {(uint32_t)t, 1u, 2u, 3u};
    if constexpr (POL == 0) __builtin_nontemporal_store(v, (vu4 *)(tab + (mix(t + salt) & lmask) * 4));
    else if constexpr (POL == 1) *(vu4 *)(tab + (mix((t >> 2) + salt) & lmask) * 4 + (t & 3)) = v;     // 4 lanes: one full line
    else __builtin_nontemporal_store(v, (vu4 *)(tab + (mix((t >> 2) + salt) & lmask) * 4 + (t & 3)));
}
// a CT hit's shape: the 64-B line read cooperatively (4 lanes), then written back:
// MODE 0 read only, 1 one 16-B partial store into it, 2 the whole line (4 lanes x 16 B)
template <int MODE>
__global__ __launch_bounds__(256) void k_mhit(uint4 *__restrict__ tab, uint64_t lmask, uint32_t *sink, uint32_t salt) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint4 *p = tab + (mix((t >> 2) + salt) & lmask) * 4 + (t & 3);
    uint4 v = *p;
    if (MODE == 1 && (t & 3) == 1) *p = make_uint4(v.x + 1, v.y, v.z + 64, v.w);
    if (MODE == 2) *p = make_uint4(v.x + 1, v.y, v.z + 64, v.w);
    if ((v.x ^ v.w) == 0x9e3779b9u) sink[t & 1023] = v.y;
}
// chain<L>: persistent lanes, L dependent streams per lane
template <int L>
__global__ __launch_bounds__(256) void k_mchain(const uint4 *__restrict__ tab, uint64_t lmask, uint32_t iters,
                                                uint32_t *sink, uint32_t salt) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t h[L];
#pragma unroll
    for (int k = 0; k < L; k++) h[k] = mix(t * L + k + salt);
    for (uint32_t it = 0; it < iters; it++) {
        uint4 v[L];
#pragma unroll
        for (int k = 0; k < L; k++) v[k] = tab[(h[k] & lmask) * 4];
#pragma unroll
        for (int k = 0; k < L; k++) h[k] = mix(h[k] + v[k].x + it + 1);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < L; k++) acc ^= (uint32_t)h[k];
    if (acc == 0x9e3779b9u) sink[t & 1023] = acc;
}
// chain with the k_ing_groups write mix: per step a 16-B store back into the
// line just read (CT hot block) and an 8-B store into a random output line
template <int L>
__global__ __launch_bounds__(256) void k_mchain_w(uint4 *__restrict__ tab, uint64_t lmask, uint2 *__restrict__ outp,
                                                  uint64_t omask, uint32_t iters, uint32_t *sink, uint32_t salt) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t h[L];
#pragma unroll
    for (int k = 0; k < L; k++) h[k] = mix(t * L + k + salt);
    for (uint32_t it = 0; it < iters; it++) {
        uint4 v[L];
        uint64_t ln[L];
#pragma unroll
        for (int k = 0; k < L; k++) { ln[k] = h[k] & lmask; v[k] = tab[ln[k] * 4]; }
#pragma unroll
        for (int k = 0; k < L; k++) {
            tab[ln[k] * 4 + 2] = make_uint4(v[k].x + 1, v[k].y, v[k].z + 64, (uint32_t)it);
            outp[(mix(h[k] ^ 0x55) & omask) * 8] = make_uint2(v[k].x, (uint32_t)it);
            h[k] = mix(h[k] + v[k].x + it + 1);
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < L; k++) acc ^= (uint32_t)h[k];
    if (acc == 0x9e3779b9u) sink[t & 1023] = acc;
}
// st<W>: one W-byte store per lane at the start of a random 64-B line (128: a line pair)
template <int W>
__global__ __launch_bounds__(256) void k_mst(uint8_t *__restrict__ tab, uint64_t lmask, uint32_t salt) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t line = mix(t + salt) & lmask;
    if (W == 128) line &= ~1ull;
    uint8_t *p = tab + line * 64;
    const uint32_t x = (uint32_t)t;
    if constexpr (W == 4) *reinterpret_cast<uint32_t *>(p) = x;
    else if constexpr (W == 8) *reinterpret_cast<uint2 *>(p) = make_uint2(x, x ^ 1);
    else {
#pragma unroll
        for (int j = 0; j < W / 16; j++) reinterpret_cast<uint4 *>(p)[j] = make_uint4(x, x + j, x ^ 3, x + 9);
    }
}
// at<K>: K u64 atomicAdds per lane into one random 16-B pair
template <int K>
__global__ __launch_bounds__(256) void k_mat(unsigned long long *__restrict__ tab, uint64_t lmask, uint32_t salt) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    unsigned long long *p = tab + (mix(t + salt) & lmask) * 8;
    atomicAdd(&p[0], 1ull);
    if (K > 1) atomicAdd(&p[1], 100ull);
}
// one random 16-B read + one independent random 16-B store (different lines)
__global__ __launch_bounds__(256) void k_mmix(uint4 *__restrict__ tab, uint64_t lmask, uint32_t *sink, uint32_t salt) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint4 v = tab[(mix(t + salt) & lmask) * 4];
    tab[(mix(t ^ 0xabcdefull + salt) & lmask) * 4 + 1] = make_uint4((uint32_t)t, 1, 2, 3);
    if (v.x == 0x9e3779b9u) sink[t & 1023] = v.y;
}
// 16-B read + 8-B store into the same random 64-B line
__global__ __launch_bounds__(256) void k_mrmw(uint4 *__restrict__ tab, uint64_t lmask, uint32_t salt) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint4 *s = tab + (mix(t + salt) & lmask) * 4;
    const uint4 v = s[2];
    *reinterpret_cast<uint2 *>(s + 2) = make_uint2(v.x + 1, v.y ^ 3);
}
// streaming, coalesced: 16 B per lane (byte calibration of FETCH/WRITE counters)
__global__ __launch_bounds__(256) void k_mseq_rd(const uint4 *__restrict__ tab, uint64_t n16, uint32_t *sink) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (; t < n16; t += (uint64_t)gridDim.x * blockDim.x) { const uint4 v = tab[t]; acc ^= v.x + v.w; }
    if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;
}
__global__ __launch_bounds__(256) void k_mseq_wr(uint4 *__restrict__ tab, uint64_t n16) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (; t < n16; t += (uint64_t)gridDim.x * blockDim.x) tab[t] = make_uint4((uint32_t)t, 1, 2, 3);
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    template <class F>
    double best(F launch, int reps = 3) {     // min over reps (the first launch warms the TLB)
        double m = 1e30;
        for (int r = 0; r < reps; r++) {
            CK(hipEventRecord(a)); launch(r); CK(hipEventRecord(b));
            CK(hipGetLastError());
            m = std::min(m, timeit(a, b));
        }
        return m;
    }
};

static const char *fp_name(uint64_t bytes) {
    static char s[8][16]; static int i = 0;
    i = (i + 1) & 7;
    if (bytes >= (1ull << 30)) snprintf(s[i], 16, "%lluGB", (unsigned long long)(bytes >> 30));
    else snprintf(s[i], 16, "%lluMB", (unsigned long long)(bytes >> 20));
    return s[i];
}

// rate line: accesses (or lane-steps) per second and the 64-B line requests they imply
static void line(const char *what, uint64_t fp, double ms, double accesses, double req_per_access) {
    printf("%-34s %6s  %8.3f ms  %7.2f G acc/s  %7.2f G 64B-req/s\n", what, fp_name(fp), ms, accesses / ms / 1e6,
           accesses * req_per_access / ms / 1e6);
    fflush(stdout);
}

template <int W, int L>
static void run_rd(Timer &T, const uint4 *tab, uint64_t fp, uint32_t *sink) {
    const uint64_t acc = 1ull << 24, threads = acc / L;
    const uint64_t lmask = fp / 64 - 1;
    double ms = T.best([&](int r) { hipLaunchKernelGGL((k_mrd<W, L>), dim3(threads / 256), dim3(256), 0, 0, tab, lmask, sink, 1000u * r); });
    char n[64]; snprintf(n, 64, "rd  W=%3dB L=%d (flooded)", W, L);
    line(n, fp, ms, (double)acc, W <= 64 ? 1.0 : W / 64.0);
}
template <int L>
static void run_chain(Timer &T, const uint4 *tab, uint64_t fp, uint32_t *sink, int wps, int cus) {
    const uint64_t lanes = (uint64_t)cus * wps * 256, acc_target = 1ull << 24;
    uint32_t iters = (uint32_t)std::max<uint64_t>(8, acc_target / (lanes * L));
    double ms = T.best([&](int r) { hipLaunchKernelGGL((k_mchain<L>), dim3(cus * wps), dim3(256), 0, 0, tab, fp / 64 - 1, iters, sink, 77u * r); });
    char n[64]; snprintf(n, 64, "chain L=%d WPS=%d", L, wps);
    const double acc = (double)lanes * iters * L;
    line(n, fp, ms, acc, 1.0);
    printf("%-34s %6s  latency/step %.2f us (lanes %llu, steps %u)\n", "", "", ms * 1e3 / iters, (unsigned long long)lanes, iters);
}
template <int L>
static void run_chain_w(Timer &T, uint4 *tab, uint64_t fp, uint2 *outp, uint64_t ofp, uint32_t *sink, int wps, int cus) {
    const uint64_t lanes = (uint64_t)cus * wps * 256, acc_target = 1ull << 24;
    uint32_t iters = (uint32_t)std::max<uint64_t>(8, acc_target / (lanes * L));
    double ms = T.best([&](int r) {
        hipLaunchKernelGGL((k_mchain_w<L>), dim3(cus * wps), dim3(256), 0, 0, tab, fp / 64 - 1, outp, ofp / 64 - 1, iters, sink, 91u * r);
    });
    char n[64]; snprintf(n, 64, "chain+2st L=%d WPS=%d", L, wps);
    const double steps = (double)lanes * iters * L;
    line(n, fp, ms, steps, 3.0);      // 1 read + 2 store requests per step
}
template <int W>
static void run_st(Timer &T, uint8_t *tab, uint64_t fp) {
    const uint64_t acc = 1ull << 24;
    double ms = T.best([&](int r) { hipLaunchKernelGGL((k_mst<W>), dim3(acc / 256), dim3(256), 0, 0, tab, fp / 64 - 1, 31u * r); });
    char n[64]; snprintf(n, 64, "st  W=%3dB (flooded)", W);
    line(n, fp, ms, (double)acc, W <= 64 ? 1.0 : W / 64.0);
}
template <int K>
static void run_at(Timer &T, unsigned long long *tab, uint64_t fp) {
    const uint64_t acc = 1ull << 24;
    double ms = T.best([&](int r) { hipLaunchKernelGGL((k_mat<K>), dim3(acc / 256), dim3(256), 0, 0, tab, fp / 64 - 1, 17u * r); });
    char n[64]; snprintf(n, 64, "at  u64 x%d per lane (flooded)", K);
    line(n, fp, ms, (double)acc * K, 1.0);
}

// footprint sweep of the one-load and the four-load line read (where page
// translation starts to cost), the cooperative form, and a contiguous allocation
static void tlb(int cus) {
    Timer T;
    uint32_t *sink; CK(hipMalloc(&sink, 4096));
    const uint64_t BIG = 32ull << 30;
    uint8_t *big; CK(hipMalloc(&big, BIG)); CK(hipMemset(big, 0, BIG));
    uint4 *tab = reinterpret_cast<uint4 *>(big);
    printf("# page-translation sweep: 16.8M line reads per launch (hipMalloc)\n");
    for (uint64_t gb : {1ull, 2ull, 4ull, 8ull, 16ull, 32ull}) {
        const uint64_t fp = gb << 30;
        run_rd<16, 1>(T, tab, fp, sink);
        run_rd<32, 1>(T, tab, fp, sink);
        run_rd<64, 1>(T, tab, fp, sink);
        const uint64_t acc = 1ull << 24;
        double ms = T.best([&](int r) { hipLaunchKernelGGL(k_mrd_coop, dim3(acc * 4 / 256), dim3(256), 0, 0, tab, fp / 64 - 1, sink, 100u * r); });
        line("rd  W= 64B coop (4 lanes/line)", fp, ms, (double)acc, 1.0);
    }
    for (int wps : {2, 4}) for (uint64_t gb : {2ull, 8ull, 32ull}) run_chain<1>(T, tab, gb << 30, sink, wps, cus);
    CK(hipFree(big));
    uint8_t *cg = nullptr;
    const uint64_t CB = 16ull << 30;
    if (hipExtMallocWithFlags((void **)&cg, CB, hipDeviceMallocContiguous) == hipSuccess && cg) {
        CK(hipMemset(cg, 0, CB));
        printf("# the same on a 16-GB hipDeviceMallocContiguous allocation\n");
        uint4 *ct = reinterpret_cast<uint4 *>(cg);
        run_rd<16, 1>(T, ct, CB, sink); run_rd<64, 1>(T, ct, CB, sink);
        const uint64_t acc = 1ull << 24;
        double ms = T.best([&](int r) { hipLaunchKernelGGL(k_mrd_coop, dim3(acc * 4 / 256), dim3(256), 0, 0, ct, CB / 64 - 1, sink, 100u * r); });
        line("rd  W= 64B coop (4 lanes/line)", CB, ms, (double)acc, 1.0);
        CK(hipFree(cg));
    } else {
        (void)hipGetLastError();
        printf("# hipDeviceMallocContiguous 16 GB: not available\n");
    }
    CK(hipFree(sink));
}

// request sizes and rates by cache policy (random 16-B reads, cooperative 64-B
// line reads, stores) at 2 GB and 16 GB, and on an uncached allocation
static void policies(int cus) {
    Timer T;
    uint32_t *sink; CK(hipMalloc(&sink, 4096));
    const uint64_t BIG = 16ull << 30, acc = 1ull << 24;
    uint8_t *big; CK(hipMalloc(&big, BIG)); CK(hipMemset(big, 0, BIG));
    uint4 *tab = reinterpret_cast<uint4 *>(big);
    const char *pn[4] = {"plain", "nt", "sc1", "sc0 sc1"};
    printf("# cache policies: 16.8M random reads per launch\n");
    for (uint64_t fp : {2ull << 30, 16ull << 30}) {
        double ms;
        char n[64];
#define POLRD(P) ms = T.best([&](int r) { hipLaunchKernelGGL(k_mrd_pol<P>, dim3(acc / 256), dim3(256), 0, 0, tab, fp / 64 - 1, sink, 7u * r); }); \
        snprintf(n, 64, "rd  W= 16B %s", pn[P]); line(n, fp, ms, (double)acc, 1.0);
        POLRD(0) POLRD(1) POLRD(2) POLRD(3)
#define POLCO(P) ms = T.best([&](int r) { hipLaunchKernelGGL(k_mrd_coop_pol<P>, dim3(acc * 4 / 256), dim3(256), 0, 0, tab, fp / 64 - 1, sink, 9u * r); }); \
        snprintf(n, 64, "rd  W= 64B coop %s", pn[P]); line(n, fp, ms, (double)acc, 1.0);
        POLCO(0) POLCO(1) POLCO(2) POLCO(3)
        ms = T.best([&](int r) { hipLaunchKernelGGL(k_mst_pol<0>, dim3(acc / 256), dim3(256), 0, 0, tab, fp / 64 - 1, 3u * r); });
        line("st  W= 16B nt", fp, ms, (double)acc, 1.0);
        ms = T.best([&](int r) { hipLaunchKernelGGL(k_mhit<0>, dim3(acc * 4 / 256), dim3(256), 0, 0, tab, fp / 64 - 1, sink, 5u * r); });
        line("hit: coop 64B read", fp, ms, (double)acc, 1.0);
        ms = T.best([&](int r) { hipLaunchKernelGGL(k_mhit<1>, dim3(acc * 4 / 256), dim3(256), 0, 0, tab, fp / 64 - 1, sink, 5u * r); });
        line("hit: coop read + 16B partial store", fp, ms, (double)acc, 2.0);
        ms = T.best([&](int r) { hipLaunchKernelGGL(k_mhit<2>, dim3(acc * 4 / 256), dim3(256), 0, 0, tab, fp / 64 - 1, sink, 5u * r); });
        line("hit: coop read + 64B line store", fp, ms, (double)acc, 2.0);
        ms = T.best([&](int r) { hipLaunchKernelGGL(k_mst_pol<1>, dim3(acc * 4 / 256), dim3(256), 0, 0, tab, fp / 64 - 1, 3u * r); });
        line("st  W= 64B coop (full line)", fp, ms, (double)acc, 1.0);
        ms = T.best([&](int r) { hipLaunchKernelGGL(k_mst_pol<2>, dim3(acc * 4 / 256), dim3(256), 0, 0, tab, fp / 64 - 1, 3u * r); });
        line("st  W= 64B coop nt (full line)", fp, ms, (double)acc, 1.0);
    }
    CK(hipFree(big));
    uint8_t *ub = nullptr;
    const uint64_t UB = 2ull << 30;
    if (hipExtMallocWithFlags((void **)&ub, UB, hipDeviceMallocUncached) == hipSuccess && ub) {
        CK(hipMemset(ub, 0, UB));
        uint4 *ut = reinterpret_cast<uint4 *>(ub);
        printf("# the same on a 2-GB hipDeviceMallocUncached allocation\n");
        double ms = T.best([&](int r) { hipLaunchKernelGGL(k_mrd_pol<0>, dim3(acc / 256), dim3(256), 0, 0, ut, UB / 64 - 1, sink, 7u * r); });
        line("rd  W= 16B plain (uncached mem)", UB, ms, (double)acc, 1.0);
        ms = T.best([&](int r) { hipLaunchKernelGGL(k_mrd_coop_pol<0>, dim3(acc * 4 / 256), dim3(256), 0, 0, ut, UB / 64 - 1, sink, 9u * r); });
        line("rd  W= 64B coop (uncached mem)", UB, ms, (double)acc, 1.0);
        CK(hipFree(ub));
    } else {
        (void)hipGetLastError();
        printf("# hipDeviceMallocUncached: not available\n");
    }
    CK(hipFree(sink));
}

static void matrix(uint8_t *big, uint64_t big_bytes, int cus) {
    Timer T;
    uint32_t *sink; CK(hipMalloc(&sink, 4096));
    uint4 *tab = reinterpret_cast<uint4 *>(big);
    printf("# random-request matrix: 16.8M accesses per launch, min of 3 launches; 1 access = 1 64-B line request\n");
    printf("# (W=128: 2 requests); chain lines count lane-steps; 'G 64B-req/s' = the request rate the access count implies\n");
    const uint64_t fps[3] = {128ull << 20, 2ull << 30, 16ull << 30};
    for (uint64_t fp : fps) {
        if (fp > big_bytes) continue;
        run_rd<16, 1>(T, tab, fp, sink); run_rd<16, 2>(T, tab, fp, sink); run_rd<16, 4>(T, tab, fp, sink); run_rd<16, 8>(T, tab, fp, sink);
        run_rd<64, 1>(T, tab, fp, sink); run_rd<64, 2>(T, tab, fp, sink); run_rd<64, 4>(T, tab, fp, sink);
        run_rd<128, 1>(T, tab, fp, sink); run_rd<128, 2>(T, tab, fp, sink);
    }
    for (uint64_t fp : {2ull << 30, 16ull << 30}) {
        if (fp > big_bytes) continue;
        for (int wps : {1, 2, 4, 8}) {
            run_chain<1>(T, tab, fp, sink, wps, cus);
            run_chain<2>(T, tab, fp, sink, wps, cus);
            run_chain<4>(T, tab, fp, sink, wps, cus);
        }
    }
    {
        const uint64_t fp = 16ull << 30, ofp = 128ull << 20;
        if (fp + ofp <= big_bytes) {
            uint2 *outp = reinterpret_cast<uint2 *>(big + fp);
            for (int wps : {2, 4, 8}) { run_chain_w<1>(T, tab, fp, outp, ofp, sink, wps, cus); run_chain_w<2>(T, tab, fp, outp, ofp, sink, wps, cus); }
        }
    }
    for (uint64_t fp : fps) {
        if (fp > big_bytes) continue;
        run_st<4>(T, big, fp); run_st<8>(T, big, fp); run_st<16>(T, big, fp); run_st<32>(T, big, fp);
        run_st<64>(T, big, fp); run_st<128>(T, big, fp);
    }
    for (uint64_t fp : fps) {
        if (fp > big_bytes) continue;
        run_at<1>(T, reinterpret_cast<unsigned long long *>(big), fp);
        run_at<2>(T, reinterpret_cast<unsigned long long *>(big), fp);
    }
    for (uint64_t fp : fps) {
        if (fp > big_bytes) continue;
        const uint64_t acc = 1ull << 24;
        double ms = T.best([&](int r) { hipLaunchKernelGGL(k_mmix, dim3(acc / 256), dim3(256), 0, 0, tab, fp / 64 - 1, sink, 5u * r); });
        line("mix 16B rd + 16B st (2 lines)", fp, ms, (double)acc, 2.0);
        ms = T.best([&](int r) { hipLaunchKernelGGL(k_mrmw, dim3(acc / 256), dim3(256), 0, 0, tab, fp / 64 - 1, 3u * r); });
        line("rmw 16B rd + 8B st (same line)", fp, ms, (double)acc, 2.0);
    }
    {
        const uint64_t bytes = 4ull << 30;
        double ms = T.best([&](int) { hipLaunchKernelGGL(k_mseq_rd, dim3(cus * 8), dim3(256), 0, 0, tab, bytes / 16, sink); });
        printf("%-34s %6s  %8.3f ms  %7.2f TB/s\n", "seq 16B/lane coalesced read", fp_name(bytes), ms, bytes / ms / 1e9);
        ms = T.best([&](int) { hipLaunchKernelGGL(k_mseq_wr, dim3(cus * 8), dim3(256), 0, 0, tab, bytes / 16); });
        printf("%-34s %6s  %8.3f ms  %7.2f TB/s\n", "seq 16B/lane coalesced write", fp_name(bytes), ms, bytes / ms / 1e9);
    }
    CK(hipFree(sink));
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "matrix";
    hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("# %s, %d CUs\n", p.name, cus);
    if (!strcmp(mode, "tlb")) { tlb(cus); return 0; }
    if (!strcmp(mode, "pol")) { policies(cus); return 0; }
    const uint64_t BIG = (16ull << 30) + (256ull << 20);
    uint8_t *big; CK(hipMalloc(&big, BIG)); CK(hipMemset(big, 0, BIG));
    if (!strcmp(mode, "legacy") || !strcmp(mode, "all")) legacy(big, BIG);
    if (!strcmp(mode, "matrix") || !strcmp(mode, "all")) matrix(big, BIG, cus);
    if (!strcmp(mode, "xcd")) {        // per-XCD slices against one shared table of the same size
        Timer T;
        uint32_t *sink; CK(hipMalloc(&sink, 4096));
        printf("# random 16-B reads, 16.8M per launch: whole table per block vs 1/8 slice per XCD (block %% 8)\n");
        const uint64_t acc = 1ull << 24;
        for (uint64_t fp = 8ull << 20; fp <= (128ull << 20); fp <<= 1) {
            run_rd<16, 1>(T, reinterpret_cast<const uint4 *>(big), fp, sink);
            const uint64_t sm = fp / 8 / 64 - 1;
            double ms = T.best([&](int r) { hipLaunchKernelGGL(k_mrd_xcd, dim3(acc / 256), dim3(256), 0, 0,
                                                               reinterpret_cast<const uint4 *>(big), sm, sink, 1000u * r); });
            line("rd  W= 16B per-XCD slice", fp, ms, (double)acc, 1.0);
        }
        CK(hipFree(sink));
    }
    if (!strcmp(mode, "foot")) {       // random-read rate against footprint: the L2 and MALL steps
        Timer T;
        uint32_t *sink; CK(hipMalloc(&sink, 4096));
        printf("# random 16-B / 64-B reads (1 and 4 loads per lane) against table footprint; 16.8M accesses per launch\n");
        for (uint64_t fp = 1ull << 20; fp <= (16ull << 30); fp <<= 1) {
            run_rd<16, 1>(T, reinterpret_cast<const uint4 *>(big), fp, sink);
            run_rd<16, 4>(T, reinterpret_cast<const uint4 *>(big), fp, sink);
            run_rd<64, 1>(T, reinterpret_cast<const uint4 *>(big), fp, sink);
        }
        CK(hipFree(sink));
    }
    CK(hipDeviceSynchronize());
    CK(hipFree(big));
    return 0;
}
