// store_probe.hip -- what do the tx fill's two 2-byte field writes per packet
// cost beside a nontemporal read stream, and does the write SHAPE matter?
// Standalone measurement (not product code): packets of `stride` bytes back to
// back in one buffer, 32 lanes per packet read every byte (nt dwordx4, 4 loads
// in flight per lane, the k_ipv4 shape for the mixed config), then write:
//   V0 nothing                      V1 four byte stores (the kernel today)
//   V2 two u16 stores               V3 two 16-B chunk stores (16-B aligned)
//   V4 the 64-B aligned sector(s) holding the fields, whole
//   V5 the 128-B aligned line(s) holding the fields, whole
//   V6 4 B per packet into a dense side array (no writes into the packets)
//   V7 V6, then a second kernel scatters the side array into the fields
//   V8 two u16 nontemporal stores   V9 V4 with nontemporal stores
// Build: hipcc --offload-arch=gfx950 -O3 -o build/store_probe scripts/store_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
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

template <int V>
__global__ __launch_bounds__(256) void k_probe(uint8_t *__restrict__ a, uint64_t stride, uint32_t n,
                                               uint32_t *__restrict__ side)
{
    constexpr int G = 32, U = 4;
    const uint32_t gl = threadIdx.x & (G - 1);
    const uint32_t pk = blockIdx.x * (256u / G) + threadIdx.x / G;
    const bool live = pk < n;
    uint8_t *start = a + (uint64_t)(live ? pk : 0u) * stride;
    const uint32_t s0 = (uint32_t)((uintptr_t)start & 15u);
    const u32x4 *base = (const u32x4 *)(start - s0);
    const uint32_t nch = live ? (uint32_t)((stride + s0 + 15) >> 4) : 0u;
    uint32_t acc = 0;
    for (uint32_t b0 = 0; b0 < nch; b0 += G * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = b0 + u * G + gl;
            v[u] = __builtin_nontemporal_load(base + (i < nch ? i : nch - 1));
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
#pragma unroll
    for (int m = 1; m < G; m <<= 1)
        acc += __shfl_xor(acc, m, 64);
    if (!live)
        return;
    uint8_t *f1 = start + 10, *f2 = start + 36;
    if constexpr (V == 0) {
        if (acc == 0x9E3779B9u)
            side[0] = acc;
    } else if constexpr (V == 1) {
        if (gl == 0) {
            f1[0] = (uint8_t)acc;
            f1[1] = (uint8_t)(acc >> 8);
            f2[0] = (uint8_t)(acc >> 16);
            f2[1] = (uint8_t)(acc >> 24);
        }
    } else if constexpr (V == 2) {
        if (gl == 0) {
            *(uint16_t *)f1 = (uint16_t)acc;
            *(uint16_t *)f2 = (uint16_t)(acc >> 16);
        }
    } else if constexpr (V == 3) {
        if (gl < 2) {
            u32x4 *c = (u32x4 *)((uintptr_t)(gl ? f2 : f1) & ~(uintptr_t)15);
            *c = u32x4(acc);
        }
    } else if constexpr (V == 4 || V == 5) {
        constexpr uintptr_t S = V == 4 ? 64 : 128;
        constexpr uint32_t L = S / 16;
        const uintptr_t s1 = (uintptr_t)f1 & ~(S - 1), s2 = (uintptr_t)f2 & ~(S - 1);
        if (gl < L) {
            *((u32x4 *)s1 + gl) = u32x4(acc);
        } else if (gl < 2 * L && s2 != s1) {
            *((u32x4 *)s2 + (gl - L)) = u32x4(acc);
        }
    } else if constexpr (V == 8) {
        if (gl == 0) {
            __builtin_nontemporal_store((uint16_t)acc, (uint16_t *)f1);
            __builtin_nontemporal_store((uint16_t)(acc >> 16), (uint16_t *)f2);
        }
    } else if constexpr (V == 9) {
        const uintptr_t s1 = (uintptr_t)f1 & ~(uintptr_t)63, s2 = (uintptr_t)f2 & ~(uintptr_t)63;
        if (gl < 4)
            __builtin_nontemporal_store(u32x4(acc), (u32x4 *)s1 + gl);
        else if (gl < 8 && s2 != s1)
            __builtin_nontemporal_store(u32x4(acc), (u32x4 *)s2 + (gl - 4));
    } else {
        if (gl == 0)
            side[pk] = acc;
    }
}

__global__ __launch_bounds__(256) void k_scatter(uint8_t *__restrict__ a, uint64_t stride, uint32_t n,
                                                 const uint32_t *__restrict__ side)
{
    const uint32_t pk = blockIdx.x * 256u + threadIdx.x;
    if (pk >= n)
        return;
    const uint32_t v = side[pk];
    uint8_t *start = a + (uint64_t)pk * stride;
    *(uint16_t *)(start + 10) = (uint16_t)v;
    *(uint16_t *)(start + 36) = (uint16_t)(v >> 16);
}

typedef void (*kfn)(uint8_t *, uint64_t, uint32_t, uint32_t *);

int main(int argc, char **argv)
{
    const uint64_t total = argc > 1 ? strtoull(argv[1], 0, 0) : (4752ull << 20);
    const int nstrides = argc > 2 ? argc - 2 : 0;
    std::vector<uint64_t> strides;
    for (int i = 0; i < nstrides; ++i)
        strides.push_back(strtoull(argv[2 + i], 0, 0));
    if (strides.empty())
        strides = {4532, 1500, 65536};
    uint8_t *a;
    uint32_t *side;
    CHECK(hipMalloc(&a, total + 4096));
    CHECK(hipMemset(a, 0x11, total + 4096));
    CHECK(hipMalloc(&side, (total / 64 + 64) * 4));
    constexpr int NV = 10;
    const kfn ks[NV] = {k_probe<0>, k_probe<1>, k_probe<2>, k_probe<3>, k_probe<4>,
                        k_probe<5>, k_probe<6>, k_probe<6>, k_probe<8>, k_probe<9>};
    const char *names[NV] = {"none",       "4 byte",      "2 u16",     "2 x 16B",   "64B sector",
                             "128B line",  "dense side",  "side+scat", "2 u16 nt",  "64B nt"};
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (uint64_t stride : strides) {
        const uint32_t n = (uint32_t)(total / stride);
        const dim3 grid((n + 7) / 8);
        std::vector<float> t[NV];
        for (int round = 0; round < 5; ++round)
            for (int v = 0; v < NV; ++v) {
                hipLaunchKernelGGL(ks[v], grid, dim3(256), 0, 0, a, stride, n, side);
                CHECK(hipEventRecord(e0, 0));
                for (int r = 0; r < 10; ++r) {
                    hipLaunchKernelGGL(ks[v], grid, dim3(256), 0, 0, a, stride, n, side);
                    if (v == 7)
                        hipLaunchKernelGGL(k_scatter, dim3((n + 255) / 256), dim3(256), 0, 0, a, stride, n, side);
                }
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                t[v].push_back(ms * 100.f); // us per launch
            }
        for (int v = 0; v < NV; ++v) {
            std::sort(t[v].begin(), t[v].end());
            const double us = t[v][2];
            printf("stride %6llu n %8u  %-11s %9.1f us  %7.1f GB/s read\n", (unsigned long long)stride, n,
                   names[v], us, (double)n * stride / us / 1e3);
        }
        fflush(stdout);
    }
    return 0;
}
