// pingpong_probe.hip -- host <-> resident-wave round-trip latency by where the
// doorbell lives (measurement, not product code).
//   A: doorbell in pinned host memory (hipHostMalloc coherent), the wave polls
//      it over PCIe; ack in pinned host memory (what the queue server does);
//   B: doorbell in fine-grained DEVICE memory written by the host through the
//      BAR (hipExtMallocWithFlags hipDeviceMallocFinegrained), the wave polls
//      HBM; ack in pinned host memory.
// One wave polls with vector atomics (system scope) and s_sleep; the host
// spins on the ack.  Every wait on either side is bounded.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/pingpong_probe scripts/pingpong_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CHECK(x)                                                                                     \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

// Serve `rounds` pings: wait for bell == k, then ack = k.  Gives up after
// ~`limit_ticks` of the 100 MHz clock without a ping, so the wave always ends.
__global__ void k_pong(uint32_t *bell, uint32_t *ack, uint32_t rounds, uint64_t limit_ticks, int sleep)
{
    if (threadIdx.x != 0)
        return;
    for (uint32_t k = 1; k <= rounds; ++k) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(bell, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != k) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > limit_ticks)
                return;
            if (sleep)
                __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(ack, k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double run(const char *name, uint32_t *bell_host_view, uint32_t *bell_dev_view, uint32_t *ack_host,
                  uint32_t *ack_dev, int sleep)
{
    const uint32_t rounds = 20000;
    *reinterpret_cast<volatile uint32_t *>(bell_host_view) = 0;
    *reinterpret_cast<volatile uint32_t *>(ack_host) = 0;
    hipLaunchKernelGGL(k_pong, dim3(1), dim3(64), 0, 0, bell_dev_view, ack_dev, rounds, 200000000ull, sleep);
    CHECK(hipGetLastError());
    std::vector<double> us;
    us.reserve(rounds);
    bool lost = false;
    for (uint32_t k = 1; k <= rounds && !lost; ++k) {
        const auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(bell_host_view, k, __ATOMIC_RELEASE);
        while (__atomic_load_n(reinterpret_cast<volatile uint32_t *>(ack_host), __ATOMIC_ACQUIRE) != k) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(500)) {
                lost = true;
                break;
            }
        }
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    CHECK(hipDeviceSynchronize());
    if (lost) {
        printf("%-44s lost a ping after %zu rounds\n", name, us.size());
        return -1;
    }
    std::sort(us.begin() + 100, us.end());
    const double med = us[100 + (us.size() - 100) / 2], p10 = us[100 + (us.size() - 100) / 10],
                 p90 = us[100 + (us.size() - 100) * 9 / 10];
    printf("%-44s round trip median %6.2f us  p10 %6.2f  p90 %6.2f\n", name, med, p10, p90);
    return med;
}

int main()
{
    CHECK(hipSetDevice(0));
    uint32_t *ack_h = nullptr, *ack_d = nullptr, *bell_h = nullptr, *bell_hd = nullptr;
    CHECK(hipHostMalloc(reinterpret_cast<void **>(&ack_h), 4096, hipHostMallocCoherent));
    CHECK(hipHostGetDevicePointer(reinterpret_cast<void **>(&ack_d), ack_h, 0));
    CHECK(hipHostMalloc(reinterpret_cast<void **>(&bell_h), 4096, hipHostMallocCoherent));
    CHECK(hipHostGetDevicePointer(reinterpret_cast<void **>(&bell_hd), bell_h, 0));
    for (int sleep = 0; sleep < 2; ++sleep) {
        char name[96];
        snprintf(name, sizeof name, "A bell in pinned host memory, sleep=%d", sleep);
        run(name, bell_h, bell_hd, ack_h, ack_d, sleep);
    }

    // B: fine-grained device memory; is it host-visible?
    uint32_t *bell_dev = nullptr;
    hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void **>(&bell_dev), 4096, hipDeviceMallocFinegrained);
    if (e != hipSuccess) {
        printf("B hipExtMallocWithFlags(Finegrained): %s\n", hipGetErrorString(e));
        return 0;
    }
    hipPointerAttribute_t a{};
    CHECK(hipPointerGetAttributes(&a, bell_dev));
    printf("B fine-grained device memory: type %d device %d hostPointer %p devicePointer %p\n", (int)a.type,
           a.device, a.hostPointer, a.devicePointer);
    if (!a.hostPointer) {
        printf("B not host-mapped: skipped\n");
        return 0;
    }
    uint32_t *bell_dh = static_cast<uint32_t *>(a.hostPointer);
    for (int sleep = 0; sleep < 2; ++sleep) {
        char name[96];
        snprintf(name, sizeof name, "B bell in device memory (BAR), sleep=%d", sleep);
        run(name, bell_dh, bell_dev, ack_h, ack_d, sleep);
    }
    return 0;
}
