// The flow-group sort's cost against the key bits it sorts (for DESIGN §8's "the
// sort's 0.36 of streaming rate"): rocPRIM radix_sort_pairs of n u32 keys with the
// packet index as value (counting iterator -> u32), as schedule_groups calls it, for
// end_bit 32 / 28 / 24 / 20 / 16 and the default vs the onesweep 11-bit config.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/sortbench.hip -o tools/_bin/sortbench
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_fill(uint32_t *k, uint32_t n, uint32_t salt) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint32_t x = (i / 16u) * 0x9E3779B1u ^ salt;     // 16 packets per flow group, like config 2
        x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
        k[i] = x;
    }
}

using Onesweep11 = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 16>, rocprim::kernel_config<1024, 16>, 11,
                                        rocprim::block_radix_rank_algorithm::match>>;

template <class Cfg>
static float run(const char *name, uint32_t *keys, uint32_t *skeys, uint32_t *perm, uint32_t n, int bits, void *&tmp,
                 size_t &tmpb) {
    size_t need = 0;
    CK(rocprim::radix_sort_pairs<Cfg>(nullptr, need, keys, skeys, rocprim::counting_iterator<uint32_t>(0u), perm, n,
                                      0, bits, 0));
    if (need > tmpb) { if (tmp) CK(hipFree(tmp)); CK(hipMalloc(&tmp, need)); tmpb = need; }
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 6; r++) {
        CK(hipEventRecord(a, 0));
        CK(rocprim::radix_sort_pairs<Cfg>(tmp, need, keys, skeys, rocprim::counting_iterator<uint32_t>(0u), perm, n,
                                          0, bits, 0));
        CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        if (r && ms < best) best = ms;
    }
    // sortedness of the low `bits` bits, and perm a permutation check by key gather
    std::vector<uint32_t> hk(n), hs(n), hp(n);
    CK(hipMemcpy(hk.data(), keys, n * 4ull, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hs.data(), skeys, n * 4ull, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hp.data(), perm, n * 4ull, hipMemcpyDeviceToHost));
    const uint32_t m = bits == 32 ? 0xffffffffu : ((1u << bits) - 1u);
    bool ok = true;
    for (uint32_t i = 0; i < n && ok; i++) {
        ok = hp[i] < n && hs[i] == hk[hp[i]];
        if (i) ok = ok && ((hs[i - 1] & m) < (hs[i] & m) || ((hs[i - 1] & m) == (hs[i] & m) && hp[i - 1] < hp[i]));
    }
    const double bytes = (double)n * 16.0;    // keys + values in and out, once
    printf("%-22s bits %2d  %7.3f ms  %6.2f TB/s (one read + one write of keys and values)  %s\n", name, bits, best,
           bytes / best / 1e9, ok ? "sorted+stable" : "WRONG");
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
    return best;
}

int main() {
    const uint32_t n = 1u << 24;
    uint32_t *keys, *skeys, *perm;
    CK(hipMalloc(&keys, n * 4ull)); CK(hipMalloc(&skeys, n * 4ull)); CK(hipMalloc(&perm, n * 4ull));
    k_fill<<<4096, 256>>>(keys, n, 0x1234567u);
    CK(hipDeviceSynchronize());
    void *tmp = nullptr; size_t tmpb = 0;
    printf("# rocPRIM radix_sort_pairs, n = %u u32 keys (16 per flow group) + counting-iterator values\n", n);
    for (int bits : {32, 28, 24, 20, 16}) run<rocprim::default_config>("default (8-bit onesweep)", keys, skeys, perm, n, bits, tmp, tmpb);
    for (int bits : {32, 22}) run<Onesweep11>("onesweep 11-bit", keys, skeys, perm, n, bits, tmp, tmpb);
    CK(hipFree(tmp)); CK(hipFree(keys)); CK(hipFree(skeys)); CK(hipFree(perm));
    return 0;
}
