// write_probe.hip -- what limits a kernel that writes one small field per
// packet at packet-header positions (the tx fill's stores)?
// Standalone measurement (not product code).  A 4.75 GB buffer; "headers" at
// i * stride (+10); pure write kernels (no read stream) in several shapes and
// orders, and the rate in writes per second:
//   u16      one lane per header, a 2-byte store (the fill's field)
//   u16 perm the same, headers visited in a random permutation
//   line     one 128-B line per header written whole (8 lanes x 16 B)
//   rmw      one lane per header reads its 16-B chunk (default policy) and
//            writes it back with the field changed
//   sec32/64 the aligned 32-/64-B sector holding the field, written whole
//            (rmw: read first, the sector's own bytes written back)
//   dense    2 bytes per header into a dense array (the write bytes alone)
// Build: hipcc --offload-arch=gfx950 -O3 -o build/write_probe scripts/write_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                                     \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

__global__ __launch_bounds__(256) void k_u16(uint8_t *a, uint64_t stride, uint32_t n, const uint32_t *perm,
                                             uint16_t v)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t p = perm ? perm[i] : i;
    *(uint16_t *)(a + (uint64_t)p * stride + 10) = (uint16_t)(v + p);
}

__global__ __launch_bounds__(256) void k_line(uint8_t *a, uint64_t stride, uint32_t n, const uint32_t *perm,
                                              uint16_t v)
{
    const uint32_t i = blockIdx.x * 32u + threadIdx.x / 8u;
    if (i >= n)
        return;
    const uint32_t p = perm ? perm[i] : i;
    u32x4 *l = (u32x4 *)((uintptr_t)(a + (uint64_t)p * stride) & ~(uintptr_t)127);
    l[threadIdx.x & 7u] = u32x4(v + p);
}

__global__ __launch_bounds__(256) void k_rmw(uint8_t *a, uint64_t stride, uint32_t n, const uint32_t *perm,
                                             uint16_t v)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t p = perm ? perm[i] : i;
    u32x4 *c = (u32x4 *)((uintptr_t)(a + (uint64_t)p * stride + 10) & ~(uintptr_t)15);
    u32x4 x = *c;
    x.x ^= v;
    *c = x;
}

// one aligned S-byte sector per header (S/16 lanes x 16 B), written whole;
// RMW: read first (the sector's own bytes back, one field changed)
template <int S, bool RMW>
__global__ __launch_bounds__(256) void k_sector(uint8_t *a, uint64_t stride, uint32_t n, const uint32_t *perm,
                                                uint16_t v)
{
    constexpr uint32_t L = S / 16;
    const uint32_t i = blockIdx.x * (256u / L) + threadIdx.x / L;
    if (i >= n)
        return;
    const uint32_t p = perm ? perm[i] : i;
    u32x4 *c = (u32x4 *)((uintptr_t)(a + (uint64_t)p * stride + 10) & ~(uintptr_t)(S - 1)) + (threadIdx.x % L);
    if constexpr (RMW) {
        u32x4 x = *c;
        x.x ^= v;
        *c = x;
    } else {
        *c = u32x4(v + p);
    }
}

__global__ __launch_bounds__(256) void k_dense(uint8_t *a, uint64_t stride, uint32_t n, const uint32_t *perm,
                                               uint16_t v)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n)
        return;
    ((uint16_t *)a)[i] = (uint16_t)(v + i);
}

// streams `n16` 16-B chunks (default policy): pushes the Infinity Cache's
// contents out before a timed write launch
__global__ __launch_bounds__(256) void k_evict(const u32x4 *__restrict__ b, uint64_t n16, uint32_t *sink)
{
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256u) {
        const u32x4 x = b[i];
        acc ^= x.x ^ x.y ^ x.z ^ x.w;
    }
    if (acc == 0x9E3779B9u)
        sink[0] = acc;
}

typedef void (*kfn)(uint8_t *, uint64_t, uint32_t, const uint32_t *, uint16_t);

int main(int argc, char **argv)
{
    const uint64_t total = 4752ull << 20;
    std::vector<uint64_t> strides = {64, 128, 256, 512, 1024, 2048, 4096, 4532, 8192, 16384};
    if (argc > 2)
        strides = {strtoull(argv[2], 0, 0)};
    uint8_t *a;
    CHECK(hipMalloc(&a, total + 4096));
    CHECK(hipMemset(a, 0x11, total + 4096));
    uint32_t *dperm;
    CHECK(hipMalloc(&dperm, (total / 64 + 64) * 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::mt19937 rng(7);
    const uint32_t nmax = 1u << 20; // a million headers at most (the mixed config's count)
    const bool cold = argc > 1 && argv[1][0] == 'c';
    const uint64_t evict_bytes = 1ull << 30; // 4x the Infinity Cache
    printf("%s\n", cold ? "cold: time of [write launch + 1 GiB read] minus [1 GiB read], caches evicted before"
                          : "warm: 10 launches back to back");
    for (uint64_t stride : strides) {
        uint32_t n = (uint32_t)std::min<uint64_t>(total / stride, nmax);
        std::vector<uint32_t> perm(n);
        for (uint32_t i = 0; i < n; ++i)
            perm[i] = i;
        std::shuffle(perm.begin(), perm.end(), rng);
        CHECK(hipMemcpy(dperm, perm.data(), n * 4ull, hipMemcpyHostToDevice));
        struct V {
            const char *name;
            kfn k;
            bool perm;
            uint32_t per_block;
        } vs[] = {{"u16", k_u16, false, 256}, {"u16 perm", k_u16, true, 256}, {"line", k_line, false, 32},
                  {"line perm", k_line, true, 32}, {"rmw", k_rmw, false, 256}, {"rmw perm", k_rmw, true, 256},
                  {"sec32", k_sector<32, false>, false, 128}, {"sec32 rmw", k_sector<32, true>, false, 128},
                  {"sec64", k_sector<64, false>, false, 64}, {"sec64 rmw", k_sector<64, true>, false, 64},
                  {"dense", k_dense, false, 256}};
        constexpr int NV = sizeof(vs) / sizeof(vs[0]);
        std::vector<float> t[NV];
        for (int round = 0; round < 5; ++round)
            for (int v = 0; v < NV; ++v) {
                const dim3 grid((n + vs[v].per_block - 1) / vs[v].per_block);
                const uint32_t *pp = vs[v].perm ? dperm : nullptr;
                hipLaunchKernelGGL(vs[v].k, grid, dim3(256), 0, 0, a, stride, n, pp, (uint16_t)round);
                float ms = 0;
                if (cold) {
                    // cold: [evict] then timed [write, evict] minus timed [evict, evict]: the write launch
                    // plus whatever the dirty lines cost the read stream that pushes them out to HBM
                    auto evict = [&]() {
                        hipLaunchKernelGGL(k_evict, dim3(4096), dim3(256), 0, 0,
                                           (const u32x4 *)(a + total - evict_bytes), evict_bytes / 16, dperm);
                    };
                    float base = 0;
                    for (int r = 0; r < 4; ++r) {
                        float m;
                        evict();
                        CHECK(hipEventRecord(e0, 0));
                        hipLaunchKernelGGL(vs[v].k, grid, dim3(256), 0, 0, a, stride, n, pp, (uint16_t)(r + round));
                        evict();
                        CHECK(hipEventRecord(e1, 0));
                        CHECK(hipEventSynchronize(e1));
                        CHECK(hipEventElapsedTime(&m, e0, e1));
                        ms += m * 250.f; // us (x1000 / 4)
                        evict();
                        CHECK(hipEventRecord(e0, 0));
                        evict();
                        CHECK(hipEventRecord(e1, 0));
                        CHECK(hipEventSynchronize(e1));
                        CHECK(hipEventElapsedTime(&m, e0, e1));
                        base += m * 250.f;
                    }
                    t[v].push_back((ms - base) / 10.f); // printed x10 below
                    continue;
                }
                CHECK(hipEventRecord(e0, 0));
                for (int r = 0; r < 10; ++r)
                    hipLaunchKernelGGL(vs[v].k, grid, dim3(256), 0, 0, a, stride, n, pp, (uint16_t)(r + round));
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipEventSynchronize(e1));
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                t[v].push_back(ms * 10.f); // us per launch, /10 at the print
            }
        for (int v = 0; v < NV; ++v) {
            std::sort(t[v].begin(), t[v].end());
            const double us = t[v][2] * 10.0;
            printf("stride %6llu n %8u  %-10s %8.1f us  %6.2f G writes/s  %6.3f ns/write\n",
                   (unsigned long long)stride, n, vs[v].name, us, n / us / 1e3, us * 1e3 / n);
        }
        fflush(stdout);
    }
    return 0;
}
