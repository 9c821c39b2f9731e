// lasterror_probe.hip -- what the HIP runtime leaves in the calling thread's
// last-error slot (hipGetLastError / hipPeekAtLastError) after the calls
// libtcsum.so makes that may answer with something other than hipSuccess
// (DESIGN.md §5, round 4's intermittent TCSUM_ERR_SYS).  Measurement only.
//   hipcc --offload-arch=gfx950 -O2 scripts/lasterror_probe.hip -o lasterror_probe
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

// Keeps the stream busy for about `ticks` of the 100 MHz real-time clock.
__global__ void k_spin(uint64_t ticks, uint32_t *sink)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks)
        __builtin_amdgcn_s_sleep(8);
    if (threadIdx.x == 0 && ticks == 7)
        sink[0] = 1u;
}

__global__ void k_noop(uint32_t *sink)
{
    if (threadIdx.x == 1000)
        sink[0] = 2u;
}

static void show(const char *what, hipError_t ret)
{
    const hipError_t peek = hipPeekAtLastError();
    printf("%-58s returned %3d (%s); last-error slot now %3d (%s)\n", what, (int)ret, hipGetErrorName(ret),
           (int)peek, hipGetErrorName(peek));
}

int main()
{
    uint32_t *sink = nullptr;
    hipStream_t s;
    if (hipMalloc(&sink, 64) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        fprintf(stderr, "no device\n");
        return 2;
    }
    (void)hipGetLastError();
    int rtv = 0, drv = 0;
    (void)hipRuntimeGetVersion(&rtv);
    (void)hipDriverGetVersion(&drv);
    printf("HIP runtime %d, driver %d\n", rtv, drv);

    // 1. hipStreamQuery on a busy stream
    k_spin<<<1, 64, 0, s>>>(5000000ull, sink); // ~50 ms
    show("launch k_spin (50 ms)", hipSuccess);
    show("hipStreamQuery(busy stream)", hipStreamQuery(s));
    // 2. does a later successful launch read back as failed?
    k_noop<<<1, 64, 0, s>>>(sink);
    const hipError_t after = hipGetLastError();
    printf("%-58s %3d (%s)\n", "hipGetLastError() right after a good launch", (int)after, hipGetErrorName(after));
    (void)hipStreamSynchronize(s);
    (void)hipGetLastError();
    // 3. hipEventQuery on a pending event
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    k_spin<<<1, 64, 0, s>>>(5000000ull, sink);
    (void)hipEventRecord(ev, s);
    show("hipEventQuery(pending event)", hipEventQuery(ev));
    (void)hipStreamSynchronize(s);
    (void)hipGetLastError();
    // 4. hipPointerGetAttributes on pageable memory
    void *pg = malloc(1 << 20);
    memset(pg, 1, 1 << 20);
    hipPointerAttribute_t a{};
    show("hipPointerGetAttributes(pageable)", hipPointerGetAttributes(&a, pg));
    printf("    type = %d\n", (int)a.type);
    (void)hipGetLastError();
    // 5. hipMemcpyAsync H2D from pageable memory, then sync
    void *d = nullptr;
    (void)hipMalloc(&d, 1 << 20);
    show("hipMemcpyAsync H2D from pageable (1 MiB)", hipMemcpyAsync(d, pg, 1 << 20, hipMemcpyHostToDevice, s));
    show("hipStreamSynchronize after it", hipStreamSynchronize(s));
    (void)hipGetLastError();
    // 6. a real error: hipSetDevice(out of range), then a good launch
    int n = 0;
    (void)hipGetDeviceCount(&n);
    show("hipSetDevice(device count) -- invalid", hipSetDevice(n));
    show("hipSetDevice(0)", hipSetDevice(0));
    k_noop<<<1, 64, 0, s>>>(sink);
    const hipError_t after2 = hipGetLastError();
    printf("%-58s %3d (%s)\n", "hipGetLastError() after that, and a good launch", (int)after2, hipGetErrorName(after2));
    // 7. hipLaunchKernel's own status with a stale error in the slot
    (void)hipSetDevice(n);
    void *args[] = {&sink};
    show("hipLaunchKernel(k_noop) with an invalid-device error pending",
         hipLaunchKernel(reinterpret_cast<const void *>(&k_noop), dim3(1), dim3(64), args, 0, s));
    (void)hipStreamSynchronize(s);
    (void)hipGetLastError();
    return 0;
}
