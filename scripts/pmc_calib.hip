// pmc_calib.hip -- what FETCH_SIZE / WRITE_SIZE report for each access class
// the checksum kernels use, on known byte counts (MI355X_MICROARCH.md: the
// counters are calibrated only for 16-B-per-lane streaming reads (x2) and
// stores; "other access widths are uncalibrated").  Standalone measurement,
// not product code; run under rocprofv3 --pmc by scripts/pmc_calib.py, which
// pairs each kernel's counter with the byte count printed here.
//
// Every class kernel runs after a 1 GiB streaming read of another buffer
// (k_flush), so none of its lines is in L2 when it starts; FETCH_SIZE counts
// L2 -> fabric requests (Infinity-Cache hits included), so the class's own
// request sizes are what is measured.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/build/pmc_calib scripts/pmc_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                                     \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

static constexpr uint32_t kPkts = 1u << 20;     // packets per class launch (configs[1] / [3] count)
static constexpr uint64_t kStride = 4532;       // configs[3]'s mean packet spacing

__device__ __forceinline__ void sink_it(uint32_t x, uint32_t *sink)
{
    if (x == 0x9E3779B9u)
        sink[0] = x;
}

// 1 GiB streaming read: evicts every L2 between class launches
__global__ __launch_bounds__(256) void k_flush(const u32x4 *__restrict__ p, uint64_t nchunks, uint32_t *sink)
{
    u32x4 x = u32x4(0u);
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nchunks; i += (uint64_t)gridDim.x * 256u)
        x ^= __builtin_nontemporal_load(p + i);
    sink_it(x.x ^ x.y ^ x.z ^ x.w, sink);
}

// wide streaming read, 16 B per lane, NT (the data pass) or default policy
template <bool NT>
__global__ __launch_bounds__(256) void k_stream(const u32x4 *__restrict__ p, uint64_t nchunks, uint32_t *sink)
{
    u32x4 x = u32x4(0u);
    const uint64_t i0 = (blockIdx.x * 256ull) * 4 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint64_t i = i0 + u * 256u;
        if (i < nchunks)
            x ^= NT ? __builtin_nontemporal_load(p + i) : p[i];
    }
    sink_it(x.x ^ x.y ^ x.z ^ x.w, sink);
}

// descriptors read by 16-lane groups: every lane of a group loads the same
// 16-B record (k_ipv4 / k_segments MODE_SEG), or 16 + 8 B (MODE_PESO's 24 B)
template <int DSZ>
__global__ __launch_bounds__(256) void k_desc(const uint8_t *__restrict__ d, uint32_t n, uint32_t *sink)
{
    const uint32_t i = blockIdx.x * 16u + threadIdx.x / 16u;
    if (i >= n)
        return;
    const uint8_t *r = d + (uint64_t)DSZ * i;
    u32x4 a = *reinterpret_cast<const u32x4 *>(r);
    uint32_t x = a.x ^ a.y ^ a.z ^ a.w;
    if constexpr (DSZ == 24) {
        const uint2 b = *reinterpret_cast<const uint2 *>(r + 16);
        x ^= b.x ^ b.y;
    }
    sink_it(x, sink);
}

// k_segments_pk's descriptor pattern (K = 8 ranges of 24 B per 4-wave
// workgroup): every wave scalar-loads the first and the last descriptor's
// offset and length (desc_span: a workgroup-uniform index, so s_load), and
// lanes 0..7 of wave 0 then vector-load all eight (load_desc).  SCALAR_ONLY:
// the scalar loads alone; VECTOR_ONLY: the vector loads alone.
template <int MODE>
__global__ __launch_bounds__(256) void k_pkdesc(const uint8_t *__restrict__ d, uint32_t n, uint32_t *sink)
{
    constexpr uint32_t K = 8;
    const uint32_t first = blockIdx.x * K;
    uint32_t x = 0;
    if (MODE != 2) { // scalar: offset (8 B) and length (4 B) of the first and last descriptor
        const uint8_t *a = d + 24ull * first, *b = d + 24ull * (first + K - 1u);
        const uint2 oa = *reinterpret_cast<const uint2 *>(a), ob = *reinterpret_cast<const uint2 *>(b);
        x ^= oa.x ^ oa.y ^ ob.x ^ ob.y ^ *reinterpret_cast<const uint32_t *>(a + 8) ^
             *reinterpret_cast<const uint32_t *>(b + 8);
    }
    if (MODE != 1 && threadIdx.x < K) { // vector: lane r loads descriptor first + r (16 + 8 B)
        const uint8_t *r = d + 24ull * (first + threadIdx.x);
        const u32x4 v = *reinterpret_cast<const u32x4 *>(r);
        const uint2 w = *reinterpret_cast<const uint2 *>(r + 16);
        x ^= v.x ^ v.y ^ v.z ^ v.w ^ w.x ^ w.y;
    }
    sink_it(x, sink);
}

// one default-policy 16-B chunk per packet (the edge / header chunks)
__global__ __launch_bounds__(256) void k_sparse16(const uint8_t *__restrict__ a, uint32_t n, uint64_t stride,
                                                  uint32_t *sink)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n)
        return;
    const u32x4 v = *reinterpret_cast<const u32x4 *>(a + ((i * stride) & ~15ull));
    sink_it(v.x ^ v.y ^ v.z ^ v.w, sink);
}

// dense loads of T per lane (k_tx_scatter's value / position arrays), and
// 8 B per lane at a 16-B stride (its descriptor offsets)
template <typename T, int STRIDE>
__global__ __launch_bounds__(256) void k_load(const uint8_t *__restrict__ a, uint32_t n, uint32_t *sink)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n)
        return;
    const T v = *reinterpret_cast<const T *>(a + (uint64_t)STRIDE * i);
    sink_it((uint32_t)v ^ (uint32_t)((uint64_t)v >> 16 >> 16), sink);
}

// dense stores of T per lane (results: u8 verdicts, u16 sums, u32 pairs, 8-B scratch)
template <typename T>
__global__ __launch_bounds__(256) void k_store_dense(T *__restrict__ o, uint32_t n)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n)
        o[i] = (T)(i * 2654435761u);
}

// one u16 per workgroup (k_segments_wg's result: lane 0 of each range's workgroup)
__global__ __launch_bounds__(256) void k_store_wg16(uint16_t *__restrict__ o, uint32_t n)
{
    if (threadIdx.x == 0 && blockIdx.x < n)
        o[blockIdx.x] = (uint16_t)blockIdx.x;
}

// scattered u16 field stores at packet-header positions (the tx fill's
// fields: the IPv4 checksum at +10 and, FIELDS == 2, a TCP one at +36)
template <int FIELDS>
__global__ __launch_bounds__(256) void k_store_field(uint8_t *__restrict__ a, uint32_t n, uint64_t stride)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n)
        return;
    uint8_t *p = a + i * stride;
    p[10] = (uint8_t)i;
    p[11] = (uint8_t)(i >> 8);
    if (FIELDS == 2) {
        p[36] = (uint8_t)(i >> 3);
        p[37] = (uint8_t)(i >> 11);
    }
}

int main()
{
    const uint64_t flush_bytes = 1ull << 30, stream_bytes = 1ull << 31;
    const uint64_t pkt_bytes = (uint64_t)kPkts * kStride + 4096;
    u32x4 *flush, *stream;
    uint8_t *pkts, *desc, *dense;
    uint32_t *sink;
    CHECK(hipMalloc(&flush, flush_bytes));
    CHECK(hipMalloc(&stream, stream_bytes));
    CHECK(hipMalloc(&pkts, pkt_bytes));
    CHECK(hipMalloc(&desc, 24ull * kPkts));
    CHECK(hipMalloc(&dense, 8ull * kPkts));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMemset(flush, 1, flush_bytes));
    CHECK(hipMemset(stream, 2, stream_bytes));
    CHECK(hipMemset(pkts, 3, pkt_bytes));
    CHECK(hipMemset(desc, 4, 24ull * kPkts));
    CHECK(hipDeviceSynchronize());
    auto flush_l2 = [&] {
        hipLaunchKernelGGL(k_flush, dim3(8192), dim3(256), 0, 0, flush, flush_bytes / 16, sink);
    };
    const uint32_t pblocks = (kPkts + 255) / 256;
    // name, algorithmic bytes of one launch, read (0) or write (1)
    printf("[\n");
    bool first = true;
    auto note = [&](const char *kernel, const char *cls, double bytes, int write) {
        printf("%s{\"kernel\": \"%s\", \"class\": \"%s\", \"bytes\": %.0f, \"write\": %d}\n", first ? "" : ",",
               kernel, cls, bytes, write);
        first = false;
    };
    for (int rep = 0; rep < 3; ++rep) {
        flush_l2();
        hipLaunchKernelGGL(k_stream<true>, dim3((uint32_t)(stream_bytes / 16 / 1024)), dim3(256), 0, 0, stream,
                           stream_bytes / 16, sink);
        flush_l2();
        hipLaunchKernelGGL(k_stream<false>, dim3((uint32_t)(stream_bytes / 16 / 1024)), dim3(256), 0, 0, stream,
                           stream_bytes / 16, sink);
        flush_l2();
        hipLaunchKernelGGL(k_desc<16>, dim3(kPkts / 16), dim3(256), 0, 0, desc, kPkts, sink);
        flush_l2();
        hipLaunchKernelGGL(k_desc<24>, dim3(kPkts / 16), dim3(256), 0, 0, desc, kPkts, sink);
        flush_l2();
        hipLaunchKernelGGL(k_pkdesc<0>, dim3(kPkts / 8), dim3(256), 0, 0, desc, kPkts, sink);
        flush_l2();
        hipLaunchKernelGGL(k_pkdesc<1>, dim3(kPkts / 8), dim3(256), 0, 0, desc, kPkts, sink);
        flush_l2();
        hipLaunchKernelGGL(k_pkdesc<2>, dim3(kPkts / 8), dim3(256), 0, 0, desc, kPkts, sink);
        flush_l2();
        hipLaunchKernelGGL(k_sparse16, dim3(pblocks), dim3(256), 0, 0, pkts, kPkts, (uint64_t)1500, sink);
        flush_l2();
        hipLaunchKernelGGL(k_sparse16, dim3(pblocks), dim3(256), 0, 0, pkts, kPkts, kStride, sink);
        flush_l2();
        hipLaunchKernelGGL((k_load<uint32_t, 4>), dim3(pblocks), dim3(256), 0, 0, dense, kPkts, sink);
        flush_l2();
        hipLaunchKernelGGL((k_load<uint64_t, 16>), dim3(pblocks), dim3(256), 0, 0, desc, kPkts, sink);
        flush_l2();
        hipLaunchKernelGGL(k_store_dense<uint8_t>, dim3(pblocks), dim3(256), 0, 0, dense, kPkts);
        flush_l2();
        hipLaunchKernelGGL(k_store_dense<uint16_t>, dim3(pblocks), dim3(256), 0, 0, (uint16_t *)dense, kPkts);
        flush_l2();
        hipLaunchKernelGGL(k_store_dense<uint32_t>, dim3(pblocks), dim3(256), 0, 0, (uint32_t *)dense, kPkts);
        flush_l2();
        hipLaunchKernelGGL(k_store_dense<uint64_t>, dim3(pblocks), dim3(256), 0, 0, (uint64_t *)dense, kPkts);
        flush_l2();
        hipLaunchKernelGGL(k_store_wg16, dim3(kPkts / 4), dim3(256), 0, 0, (uint16_t *)dense, kPkts / 4);
        flush_l2();
        hipLaunchKernelGGL(k_store_field<1>, dim3(pblocks), dim3(256), 0, 0, pkts, kPkts, kStride);
        flush_l2();
        hipLaunchKernelGGL(k_store_field<2>, dim3(pblocks), dim3(256), 0, 0, pkts, kPkts, kStride);
        flush_l2();
        CHECK(hipDeviceSynchronize());
    }
    note("k_stream<true>", "streaming read, 16 B/lane, nontemporal", (double)stream_bytes, 0);
    note("k_stream<false>", "streaming read, 16 B/lane, default policy", (double)stream_bytes, 0);
    note("k_desc<16>", "16-B descriptor per 16-lane group", 16.0 * kPkts, 0);
    note("k_desc<24>", "24-B descriptor (16 + 8 B loads) per 16-lane group", 24.0 * kPkts, 0);
    note("k_pkdesc<0>", "k_segments_pk's descriptors: scalar first/last + vector all (24 B x 8 per workgroup)",
         24.0 * kPkts, 0);
    note("k_pkdesc<1>", "the same, scalar first/last only (algorithmic: every descriptor line)", 24.0 * kPkts, 0);
    note("k_pkdesc<2>", "the same, vector loads only", 24.0 * kPkts, 0);
    note("k_sparse16@1500", "one default-policy 16-B chunk per packet, stride 1500", 16.0 * kPkts, 0);
    note("k_sparse16@4532", "one default-policy 16-B chunk per packet, stride 4532", 16.0 * kPkts, 0);
    note("k_load<unsigned int, 4>", "dense u32 load per lane", 4.0 * kPkts, 0);
    note("k_load<unsigned long, 16>", "8-B load per lane at a 16-B stride", 8.0 * kPkts, 0);
    note("k_store_dense<unsigned char>", "dense u8 per lane", 1.0 * kPkts, 1);
    note("k_store_dense<unsigned short>", "dense u16 per lane", 2.0 * kPkts, 1);
    note("k_store_dense<unsigned int>", "dense u32 per lane", 4.0 * kPkts, 1);
    note("k_store_dense<unsigned long>", "dense 8 B per lane", 8.0 * kPkts, 1);
    note("k_store_wg16", "one u16 per workgroup (lane 0)", 2.0 * (kPkts / 4), 1);
    note("k_store_field<1>", "one scattered 2-B field per packet (stride 4532)", 2.0 * kPkts, 1);
    note("k_store_field<2>", "two scattered 2-B fields per packet (+10, +36)", 4.0 * kPkts, 1);
    printf("]\n");
    return 0;
}
