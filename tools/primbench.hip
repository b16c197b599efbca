// primbench.hip — rates of the memory primitives the ingress kernel is built
// from, on MI355X, at the footprints of BASELINE config 2:
//   * random 16-B loads from an 8 GB table (CT home line probe)
//   * random line RMW: 16-B load + 8-B store into the same 64-B slot (CT hit update)
//   * random 64-bit atomicAdd into a 256 MB table (policy counters)
//   * 64-bit atomicAdd into 32 / 1 hot addresses (contended policy entries / stats bins)
//   * scattered 8-B stores through a permutation into 134 MB (output records)
//   * one atomicAdd per workgroup into one address (block-level counter flush)
//   hipcc -O3 --offload-arch=gfx950 tools/primbench.hip -o tools/_bin/primbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

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
__global__ void k_perm_init(uint32_t *perm, uint32_t n) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) perm[t] = t;
}
// Fisher-Yates is sequential; a bijective multiplicative permutation mod 2^k is enough here
__global__ void k_perm_mul(uint32_t *perm, uint32_t n) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) perm[t] = (uint32_t)(((uint64_t)t * 2654435761ull + 12345) & (n - 1));
}

static double timeit(hipEvent_t a, hipEvent_t b) {
    float ms; CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b)); return ms;
}

int main() {
    const uint64_t CT = 8ull << 30, POL = 256ull << 20;
    const uint32_t N = 1u << 24;              // 16.8M packets
    uint8_t *ct, *pol; uint32_t *out, *perm; uint2 *o8; unsigned long long *hot;
    CK(hipMalloc(&ct, CT)); CK(hipMemset(ct, 0, CT));
    CK(hipMalloc(&pol, POL)); CK(hipMemset(pol, 0, POL));
    CK(hipMalloc(&out, 4096)); CK(hipMalloc(&perm, N * 4ull)); CK(hipMalloc(&o8, N * 8ull));
    CK(hipMalloc(&hot, 1 << 20)); CK(hipMemset(hot, 0, 1 << 20));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    dim3 B(256), G(N / 256);
    for (int rep = 0; rep < 2; rep++) {
        double ms;
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_rd, G, B, 0, 0, ct, CT / 64, out, rep); CK(hipEventRecord(b));
        ms = timeit(a, b); printf("random 16B load, 8GB table      : %7.3f ms per 16.8M  %6.2f G/s\n", ms, N / ms / 1e6);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_rmw, G, B, 0, 0, ct, CT / 64, rep); CK(hipEventRecord(b));
        ms = timeit(a, b); printf("random slot RMW (16B ld+8B st)  : %7.3f ms per 16.8M  %6.2f G/s\n", ms, N / ms / 1e6);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_rmw_acct, G, B, 0, 0, ct, CT / 64, rep); CK(hipEventRecord(b));
        ms = timeit(a, b); printf("random slot RMW + acct (2x16B)  : %7.3f ms per 16.8M  %6.2f G/s\n", ms, N / ms / 1e6);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_atom, G, B, 0, 0, (unsigned long long *)pol, POL / 64, rep); CK(hipEventRecord(b));
        ms = timeit(a, b); printf("2x atomicAdd u64, 256MB random  : %7.3f ms per 16.8M  %6.2f G pkt/s\n", ms, N / ms / 1e6);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_atom, G, B, 0, 0, (unsigned long long *)ct, CT / 64, rep); CK(hipEventRecord(b));
        ms = timeit(a, b); printf("2x atomicAdd u64, 8GB random    : %7.3f ms per 16.8M  %6.2f G pkt/s\n", ms, N / ms / 1e6);
        for (uint32_t nh : {1u, 32u, 1024u, 65536u}) {
            CK(hipEventRecord(a)); hipLaunchKernelGGL(k_atom_hot, G, B, 0, 0, hot, nh > 2048 ? 2048 : nh, rep); CK(hipEventRecord(b));
            ms = timeit(a, b); printf("atomicAdd u64 into %5u hot     : %7.3f ms per 16.8M  %6.2f G/s\n", nh > 2048 ? 2048 : nh, ms, N / ms / 1e6);
        }
        hipLaunchKernelGGL(k_perm_mul, G, B, 0, 0, perm, N);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_scatter, G, B, 0, 0, perm, o8, N); CK(hipEventRecord(b));
        ms = timeit(a, b); printf("8B scatter via permutation 134MB: %7.3f ms per 16.8M  %6.2f G/s\n", ms, N / ms / 1e6);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_coal, G, B, 0, 0, o8, N); CK(hipEventRecord(b));
        ms = timeit(a, b); printf("8B coalesced store 134MB        : %7.3f ms per 16.8M  %6.2f G/s\n", ms, N / ms / 1e6);
        for (uint32_t nb : {1u, 12u}) {
            CK(hipEventRecord(a)); hipLaunchKernelGGL(k_blockflush, dim3(4096), B, 0, 0, hot, nb); CK(hipEventRecord(b));
            ms = timeit(a, b); printf("4096 blocks x %2u-bin flush      : %7.3f ms\n", nb, ms);
        }
        fflush(stdout);
    }
    return 0;
}
