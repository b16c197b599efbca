// membench.hip — random-access latency / throughput of MI355X HBM vs footprint.
// Characterises the regime of the CT / policy probes (one random line per
// lane, dependent chains per packet).  Build + run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 tools/membench.hip -o /tmp/membench && /tmp/membench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

// Dependent chain: each lane hops `hops` times; next address depends on loaded value.
__global__ void k_chase(const uint32_t *buf, uint64_t nlines, int hops, uint32_t *out) {
    uint64_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t x = mix(t + 1);
    uint32_t acc = 0;
    for (int h = 0; h < hops; h++) {
        uint64_t line = (x + acc) % nlines;
        acc += buf[line * 32];           // 128-B lines, first dword
        x = mix(x);
    }
    out[t] = acc;
}

// Independent random 16-B loads, `per` per lane, all issued before use.
template <int PER>
__global__ void k_rand(const uint4 *buf, uint64_t nlines, uint32_t *out, uint32_t salt) {
    uint64_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint4 v[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
        uint64_t line = mix(t * PER + k + salt) % nlines;
        v[k] = buf[line * 8];
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) acc += v[k].x ^ v[k].w;
    out[t] = acc;
}

// Random atomics (no return), one per lane.
__global__ void k_atom(unsigned long long *buf, uint64_t nlines, uint32_t salt) {
    uint64_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t line = mix(t + salt) % nlines;
    atomicAdd(&buf[line * 16], 1ull);
}

int main() {
    size_t maxb = 16ull << 30;
    uint8_t *buf;
    CK(hipMalloc(&buf, maxb));
    CK(hipMemset(buf, 0, maxb));
    uint32_t *out;
    CK(hipMalloc(&out, 64 << 20));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    size_t sizes[] = {16ull << 20, 256ull << 20, 1ull << 30, 4ull << 30, 8ull << 30, 16ull << 30};
    for (size_t S : sizes) {
        uint64_t nl = S / 128;
        float ms;
        // latency: 64 lanes (one wave) x 200 hops
        hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, (const uint32_t *)buf, nl, 50, out);
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, (const uint32_t *)buf, nl, 200, out);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        double lat_ns = ms * 1e6 / 200;
        // loaded latency: 512K lanes x 20 hops
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_chase, dim3(2048), dim3(256), 0, 0, (const uint32_t *)buf, nl, 20, out);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        double chase_rate = 2048.0 * 256 * 20 / (ms * 1e-3) / 1e9;
        // throughput: 4M lanes x 4 independent loads
        hipLaunchKernelGGL(k_rand<4>, dim3(16384), dim3(256), 0, 0, (const uint4 *)buf, nl, out, 1);
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_rand<4>, dim3(16384), dim3(256), 0, 0, (const uint4 *)buf, nl, out, 2);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        double rnd = 16384.0 * 256 * 4 / (ms * 1e-3) / 1e9;
        // atomics
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_atom, dim3(65536), dim3(256), 0, 0, (unsigned long long *)buf, nl, 3);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        double at = 65536.0 * 256 / (ms * 1e-3) / 1e9;
        printf("footprint %6zu MB: idle dep latency %7.0f ns | loaded chase %6.2f G/s | random 16B loads %6.2f G/s | random atomics %6.2f G/s\n",
               S >> 20, lat_ns, chase_rate, rnd, at);
        fflush(stdout);
    }
    CK(hipFree(buf));
    return 0;
}
