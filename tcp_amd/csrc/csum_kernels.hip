// csum_kernels.hip -- gfx950 kernels for the Internet checksum (RFC 1071 sum as
// the wj9806/tcp stack computes it: net/src/tools.c:24-75, pktbuf.c:646-670).
//
// libtcsum.so's kernels: the device code of csum_device.h instantiated in
// the shapes the router (pick_geometry) can choose, the resident servers,
// and the launch functions csum_api.cpp calls.  Measurement kernels (load
// probes, synthetic data) live in libtcsum_bench.so (bench_kernels.hip).
#include "csum_device.h"

#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>

namespace tcsum {

// ---------------------------------------------------------------- queue server
//
// A resident grid that serves small host-queue batches without a launch and
// a stream sync per batch (tcsum_queue_server, include/tcsum.h).  The host
// posts one job at a time into pinned, coherent memory (SrvHost: job fields,
// then `req`); workgroup 0 polls `req` over PCIe with one lane and s_sleep,
// copies the job into device memory (SrvCtl, agent-scope atomics) and bumps
// SrvCtl::seq; the other workgroups poll that word (relaxed, s_sleep), take
// ONE system-scope acquire (their L1/L2 may hold host lines from the last
// job), and every workgroup sums its share of the packets.  Each workgroup
// drains its stores, releases them at system scope (results and tx bytes live
// in host memory) and adds to SrvCtl::arrivals; the last arriver writes
// SrvHost::done.  Exit: workgroup 0 alone decides -- host `quit`, or no job
// for `idle_ticks` of the 100 MHz real-time clock -- and publishes
// SrvCtl::quit; every other workgroup also gives up after 8x that without a
// word, so every wave reaches an exit.  A job posted while the grid is
// leaving is never lost: the host sees the stream idle with done != req and
// relaunches (csum_api.cpp).
template <int G, int U>
__global__ __launch_bounds__(256) void k_server(SrvHost *__restrict__ h, SrvCtl *__restrict__ d, uint32_t last,
                                                uint64_t idle_ticks)
{
    __shared__ uint32_t s_go;
    const bool lead = threadIdx.x == 0;
    uint32_t jobs = 0;
    uint64_t t_last = __builtin_amdgcn_s_memrealtime();
    // phase stamps (100 MHz) of job j in tr[(j % 256) * 8 + k], measurement only
    uint64_t *tr = reinterpret_cast<uint64_t *>(__hip_atomic_load(&h->trace, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    auto stamp = [&](int k) {
        if (tr)
            __hip_atomic_store(tr + (jobs % 256u) * 8u + k, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    };
    for (;;) {
        if (lead) {
            uint32_t go = 0;
            if (blockIdx.x == 0) {
                for (;;) {
                    const uint32_t r = __hip_atomic_load(&h->req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    if (r != last) {
                        stamp(0);
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); // system: the host's job and data
                        // all job words in flight together: one PCIe round trip, not seven
                        const uint32_t jop = __hip_atomic_load(&h->op, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        const uint32_t jn = __hip_atomic_load(&h->n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        uint64_t jp[5];
#pragma unroll
                        for (int k = 0; k < 5; ++k)
                            jp[k] = __hip_atomic_load(&h->ptr[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        __hip_atomic_store(&d->op, jop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&d->n, jn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                        for (int k = 0; k < 5; ++k)
                            __hip_atomic_store(&d->ptr[k], jp[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        __hip_atomic_store(&d->seq, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        stamp(1);
                        go = r;
                        break;
                    }
                    if (__hip_atomic_load(&h->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ||
                        __builtin_amdgcn_s_memrealtime() - t_last > idle_ticks) {
                        __hip_atomic_store(&d->quit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(4);
                }
            } else {
                for (;;) {
                    const uint32_t sq = __hip_atomic_load(&d->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (sq != 0u && sq != last) { // 0: zeroed at launch, nothing posted yet
                        if (blockIdx.x == 1)
                            stamp(2);
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); // system: SrvCtl + the host's data
                        go = sq;
                        break;
                    }
                    if (__hip_atomic_load(&d->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                        __builtin_amdgcn_s_memrealtime() - t_last > 8 * idle_ticks)
                        break;
                    __builtin_amdgcn_s_sleep(8);
                }
            }
            s_go = go;
        }
        __syncthreads();
        const uint32_t go = s_go;
        if (!go)
            return;
        const uint32_t op = __hip_atomic_load(&d->op, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t n = __hip_atomic_load(&d->n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint64_t q[5];
#pragma unroll
        for (int k = 0; k < 5; ++k)
            q[k] = __hip_atomic_load(&d->ptr[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint8_t *arena = reinterpret_cast<uint8_t *>(q[0]);
        const tcsum_pkt_t *pkts = reinterpret_cast<const tcsum_pkt_t *>(q[1]);
        uint32_t *out = reinterpret_cast<uint32_t *>(q[2]);
        uint8_t *flags = reinterpret_cast<uint8_t *>(q[3]);
        int8_t *verdict = reinterpret_cast<int8_t *>(q[4]);
        constexpr uint32_t PER = 256u / G;
        const uint32_t stride = gridDim.x * PER;
        for (uint32_t first = blockIdx.x * PER; first < n; first += stride) { // workgroup-uniform
            const uint32_t pk = first + threadIdx.x / G;
            if (op == IP_TX)
                ipv4_packet<G, U, IP_TX>(arena, pkts, pk, n, out, flags, verdict, 0u);
            else if (op == IP_RX)
                ipv4_packet<G, U, IP_RX>(arena, pkts, pk, n, out, flags, verdict, 0u);
            else
                ipv4_packet<G, U, IP_SUMS>(arena, pkts, pk, n, out, flags, verdict, 0u);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // every storing wave drains
        __syncthreads();
        if (lead) {
            if (blockIdx.x == 0)
                stamp(3);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); // system: this workgroup's results / tx bytes
            if (blockIdx.x == 0)
                stamp(4);
            const uint32_t old = __hip_atomic_fetch_add(&d->arrivals, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old == (jobs + 1u) * gridDim.x - 1u) {
                stamp(5);
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");
                __hip_atomic_store(&h->done, go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                stamp(6);
            }
            ++jobs;
        }
        last = go;
        t_last = __builtin_amdgcn_s_memrealtime();
    }
}

// ---------------------------------------------------------------- call server
//
// One resident wave serving the synchronous drop-in calls (csum_api.cpp,
// tcsum_call_server): instead of a kernel launch plus a stream sync per call
// (~17 us), the host copies the call's bytes into pinned staging, writes the
// job into a pinned CallBox and spins on the result word; the wave polls the
// box (both 16-byte job words in one PCIe round trip, s_sleep between polls),
// sums the range with all 64 lanes exactly like k_segments, and stores
// result << 32 | seq with one system-scope release.  A job is taken only when
// both job words carry its sequence number: the host stores them last, w1
// before w0, so a read that sees the new number in both saw every field.
// Exit: a QUIT job, or no job for idle_ticks of the 100 MHz clock -- every
// path leaves the loop, so the wave always finishes.

// The box's four 16-byte job words, system-scope loads all in flight (one
// PCIe round trip)
__device__ __forceinline__ void load_job(const CallBox *p, u32x4 &a, u32x4 &b, u32x4 &c, u32x4 &e)
{
    asm volatile("global_load_dwordx4 %0, %4, off sc0 sc1\n\t"
                 "global_load_dwordx4 %1, %4, off offset:16 sc0 sc1\n\t"
                 "global_load_dwordx4 %2, %4, off offset:32 sc0 sc1\n\t"
                 "global_load_dwordx4 %3, %4, off offset:48 sc0 sc1\n\t"
                 "s_waitcnt vmcnt(0)"
                 : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(e)
                 : "v"(p)
                 : "memory");
}

__global__ __launch_bounds__(64) void k_call(CallBox *__restrict__ box, const uint8_t *__restrict__ stage,
                                             uint32_t last, uint64_t idle_ticks)
{
    constexpr int G = 64, U = 16; // 16 KiB per pass: a 1500-B call is one PCIe round trip
    const uint32_t gl = threadIdx.x;
    uint64_t t_last = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        u32x4 a, b, c, e;
        for (;;) {
            load_job(box, a, b, c, e);
            const uint32_t sa = __builtin_amdgcn_readfirstlane(a.x), sb = __builtin_amdgcn_readfirstlane(b.w),
                           sc = __builtin_amdgcn_readfirstlane(c.w), se = __builtin_amdgcn_readfirstlane(e.w);
            if (sa != last && sa != 0u && sa == sb && sa == sc && sa == se)
                break;
            if (__builtin_amdgcn_s_memrealtime() - t_last > idle_ticks)
                return;
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); // system: the staged bytes
        last = __builtin_amdgcn_readfirstlane(a.x);
        const uint32_t ctl = __builtin_amdgcn_readfirstlane(a.y);
        if (ctl & CALL_QUIT)
            return;
        SegDesc d;
        d.off = (ctl & CALL_ODD) ? 1u : 0u;
        d.len = __builtin_amdgcn_readfirstlane(a.z);
        d.pre = __builtin_amdgcn_readfirstlane(a.w);
        d.src = __builtin_amdgcn_readfirstlane(b.x);
        d.dst = __builtin_amdgcn_readfirstlane(b.y);
        d.proto = __builtin_amdgcn_readfirstlane(b.z) & 0xFFu;
        const uint32_t mode = ctl & CALL_MODE_MASK;
        uint32_t acc;
        uintptr_t start = reinterpret_cast<uintptr_t>(stage + d.off);
        if (ctl & CALL_INLINE) {
            // <= 24 bytes that came with the job: the host zeroed the rest of
            // w2/w3 and put the bytes at offset (ctl & CALL_ODD), so the
            // exact word sum of the six dwords is the range's (no PCIe trip)
            acc = 0;
            acc = dot_halves(acc, __builtin_amdgcn_readfirstlane(c.x), 0x00010001u);
            acc = dot_halves(acc, __builtin_amdgcn_readfirstlane(c.y), 0x00010001u);
            acc = dot_halves(acc, __builtin_amdgcn_readfirstlane(c.z), 0x00010001u);
            acc = dot_halves(acc, __builtin_amdgcn_readfirstlane(e.x), 0x00010001u);
            acc = dot_halves(acc, __builtin_amdgcn_readfirstlane(e.y), 0x00010001u);
            acc = dot_halves(acc, __builtin_amdgcn_readfirstlane(e.z), 0x00010001u);
            start = d.off; // the byte parity the sum was taken at
        } else {
            if (mode == MODE_EXACT)
                acc = sum_range<G, U, true>(stage, d.off, d.len, gl, [] {});
            else
                acc = sum_range<G, U, false>(stage, d.off, d.len, gl, [] {});
            acc = group_sum<G>(acc);
        }
        if (gl == 0) {
            const uint32_t comp = (ctl & CALL_COMPLEMENT) ? 1u : 0u;
            uint16_t r;
            if (mode == MODE_EXACT)
                r = finalize<MODE_EXACT>(acc, start, d, comp | ((uint32_t)d.off << 1), 0u);
            else if (mode == MODE_PESO)
                r = finalize<MODE_PESO>(acc, start, d, 0u, peso_pseudo16(d));
            else
                r = finalize<MODE_SEG>(acc, start, d, comp, 0u);
            __hip_atomic_store(&box->res, ((uint64_t)r << 32) | last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        t_last = __builtin_amdgcn_s_memrealtime();
    }
}

// ---------------------------------------------------------------- dispatch

// A shape or size a launcher refuses without calling the runtime: the
// status is the library's own, so it never touches the caller's last-error
// slot (rc_of, csum_api.cpp, asks which it was).
static thread_local bool t_refused = false;

hipError_t refused()
{
    t_refused = true;
    return hipErrorInvalidValue;
}

bool take_refused()
{
    const bool r = t_refused;
    t_refused = false;
    return r;
}

// Test and measurement overrides (include/tcsum_debug.h): set only by an
// explicit tcsum_debug_set call -- nothing in the environment changes a route.
static std::atomic<int64_t> g_knobs[KNOB_COUNT] = {};
static std::once_flag g_knobs_once;

static void knobs_init()
{
    std::call_once(g_knobs_once, [] {
        for (auto &k : g_knobs)
            k.store(-1, std::memory_order_relaxed);
    });
}

int64_t knob(Knob k)
{
    knobs_init();
    return g_knobs[k].load(std::memory_order_relaxed);
}

void set_knob(Knob k, int64_t v)
{
    knobs_init();
    g_knobs[k].store(v, std::memory_order_relaxed);
}

// Measured on MI355X (scripts/tune.py; profiles/r01/tune*.txt, one process,
// interleaved rounds).  Interior chunks per range c (edges excluded):
//   c <= ~136 (<= ~2 KiB, e.g. MTU): 16 lanes, U = ceil(c/16) loads -> one
//       pass with almost no idle slots (1500 B: G=16, U=6, 95% of the read
//       probe on the same bytes);
//   ~2 KiB .. 32 KiB (mixed 64-9000 B, mean 4.5 KiB): 32 lanes x 6 loads,
//       several passes (95-97% of the probe; re-measured with the XCD order);
//   >= 32 KiB (TSO): one range per WORKGROUP (16 loads per lane, or 16 waves
//       x 4 loads from 48 KiB; profiles/r03/ab_tso_shapes2*.txt).
// Round 1-3's resident-grid variants measured slower on all three and are gone.
Geometry pick_geometry(uint64_t mean_len)
{
    // xcd: 64 workgroups per XCD run (scripts/xcd_tune.py, profiles/r01/xcd_tune.txt:
    // 2-4 % on every config, flat from 32 to 512)
    Geometry g{32, 4, 64, 0, 0};
    const uint64_t chunks = mean_len / 16 + 1;
    const uint64_t interior = chunks > 2 ? chunks - 2 : 0;
    g.interior = (int)(interior < 65536 ? interior : 65536);
    if (chunks >= 3072) {
        // >= 48 KiB (TSO): one range per 16-wave workgroup, 32-lane groups on
        // 2-KiB sub-ranges, 4 loads per lane: a 64-KiB range is one pass of
        // the workgroup -- 3.6 % faster than k_segments_wg on configs[2]
        // (profiles/r03/ab_tso_shapes2*.txt: 2,242 against 2,326 us)
        g.lanes = 1024;
        g.loads = 4;
    } else if (chunks >= 2048) {
        g.lanes = 256; // one range per workgroup (k_segments_wg): 1.8 % over G=64 on configs[2]
        g.loads = 16;
    } else if (interior > 128) {
        g.lanes = 32;
        g.loads = 6; // 1.0-1.5 % over 4 and 8 on every mixed variant (profiles/r01/geom_tune_mixed.txt)
    } else if (interior > 32) {
        g.lanes = 16;
        const uint64_t u = (interior + 15) / 16; // 3..8
        g.loads = u <= 3 ? 3 : u <= 4 ? 4 : u <= 6 ? 6 : 8;
    } else if (interior > 8) {
        g.lanes = 8;
        g.loads = 4;
    } else {
        g.lanes = 4;
        g.loads = interior > 4 ? 2 : 1;
    }
    const int64_t kl = knob(KNOB_LANES), ku = knob(KNOB_LOADS), kx = knob(KNOB_XCD), kp = knob(KNOB_PACKED);
    if (kl >= 0)
        g.lanes = (int)kl;
    if (ku >= 0)
        g.loads = (int)ku;
    if (kx >= 0)
        g.xcd = (int)kx;
    // packed stream (k_segments_pk) for checksum_peso / pktbuf_checksum16
    // batches of ranges up to ~4 KiB: K ranges of this mean length fill one
    // 12-KiB pass of a 4-wave workgroup (1500 B: K = 8).  One-process A/Bs on
    // 1.5-GB batches (profiles/r03/packed/ab_pk_layouts_default.txt, measured
    // with this 4-wave x 3-load shape): packed 1500-B ranges 0.98 of
    // k_segments<16,6>'s time, 576 B 0.73, 200 B 0.48, 64 B 0.70, 4000 B 0.94,
    // ragged 64..2936 B 0.96, with 0..63-B gaps 1.00; with K < 3 (mean > ~4
    // KiB) it lost (9000 B 1.04, ragged 64..9000 B 1.20).  A forced per-range
    // geometry (debug lanes / loads) keeps it off unless debug "packed" = 1.
    const bool forced = kl >= 0 || ku >= 0;
    if ((kp >= 0 ? kp != 0 : !forced) && mean_len > 0) {
        const uint64_t pass = 16ull * 64u * kPkWaves * kPkLoads;
        const uint64_t k = (pass - 15u) / mean_len;
        const uint64_t kmax = (uint64_t)kPkMaxRanges * kPkWaves;
        if (k >= 3)
            g.packed = (int)(k > kmax ? kmax : k);
        if (kp > 1) // measurement: K itself
            g.packed = (int)((uint64_t)kp > kmax ? kmax : (uint64_t)kp);
    }
    return g;
}

// Descriptor prefetch distance of k_segments_pk's range-by-range path, in
// workgroups (in aux >> 8): 2048 -- 1024 / 2048 / 4096 measured alike on a
// shuffled configs[1] batch (profiles/r05/pk_layouts_pf.txt); debug knob
// "pf_dist" overrides, 0 = off.  Off by default above K = 32 ranges per
// workgroup: there the descriptors
// are a large share of the bytes (24 of every 88 for 64-B ranges), and the
// prefetch's own touches cost more than they save (shuffled 64-B ranges
// 909 -> 888 us, 200-B 635 -> 628 us without it; 576-B, K = 21, 325 -> 349
// us: profiles/r06/ab15/pk_pf_ab.txt).
static uint32_t pf_dist(uint32_t K)
{
    const int64_t v = knob(KNOB_PF_DIST);
    if (v < 0)
        return K <= 32u ? 2048u : 0u;
    return (uint32_t)(v < (1 << 23) ? v : (1 << 23) - 1);
}

// k_segments_pk's range-by-range path reads its descriptors with scalar
// loads (debug knob "pk_early", on unless 0): one-box A/B, descriptors
// shuffled, against the vector loads: 1500-B ranges 0.940x, ragged
// 64..2936 B 0.939x, 4000 B 0.960x, 576 B 0.977x; packed layouts 1.000-1.004x
// (profiles/r05/pk_early/pk_early6.txt)
bool pk_early()
{
    return knob(KNOB_PK_EARLY) != 0;
}

// The per-range kernel's descriptor prefetch distance (debug knob
// "pf_range"; 0 = off, the default while unmeasured)
static uint32_t pf_range()
{
    const int64_t v = knob(KNOB_PF_RANGE);
    return v <= 0 ? 0u : (uint32_t)(v < (1 << 23) ? v : (1 << 23) - 1);
}

// The shapes the router can pick for the per-range kernels (and only those:
// a debug override naming another shape is refused).
template <int MODE>
static hipError_t seg_u(int G, int U, uint32_t xg, uint32_t n, const void *arena, const void *descs, uint16_t *out,
                        uint32_t aux, hipStream_t s)
{
    const uint8_t *a = static_cast<const uint8_t *>(arena);
#define TCSUM_SEG(GG, UU)                                                                                     \
    if (G == GG && U == UU) {                                                                               \
        return launch(k_segments<GG, UU, MODE>, dim3((n + 256u / GG - 1) / (256u / GG)), dim3(256), 0, s, a,     \
                      descs, n, out, aux | (pf_range() << 8) | (knob(KNOB_SEG_SDESC) != 0 ? kSegScalarDesc : 0u), \
                      xg);                                                                                    \
    }
    TCSUM_SEG(4, 1) TCSUM_SEG(4, 2) TCSUM_SEG(4, 3) TCSUM_SEG(8, 3) TCSUM_SEG(8, 4) TCSUM_SEG(16, 3) TCSUM_SEG(16, 4)
    TCSUM_SEG(16, 6) TCSUM_SEG(16, 8) TCSUM_SEG(32, 6)
#undef TCSUM_SEG
    if (G == 1024 && U == 4) { // one range per 16-wave workgroup, 2 KiB sub-ranges (TSO)
        return launch(k_segments_wgx<16, 32, 4, MODE>, dim3(n), dim3(1024), 0, s, a, descs, n, out, aux, xg);
    }
    if (G == 256 && U == 16) { // one range per workgroup
        return launch(k_segments_wg<16, MODE>, dim3(n), dim3(256), 0, s, a, descs, n, out, aux, xg);
    }
    return refused();
}

// The AQL dispatch packet counts work-items in 32 bits: one launch may carry
// at most 2^24 - 1 workgroups of 256 threads.  Larger batches are split into
// several launches over consecutive descriptor ranges.
static constexpr uint64_t kMaxBlocks = (1u << 24) - 1;

hipError_t launch_segments(Mode mode, Geometry g, const void *arena, const void *descs, uint32_t n,
                           uint16_t *out, uint32_t aux, hipStream_t stream)
{
    if (n == 0)
        return hipSuccess;
    {
        const uint32_t lanes = mode == MODE_EXACT ? 64u : (uint32_t)g.lanes;
        // ranges per launch: 2^32 - 1 work-items (256 / G ranges per 256-thread
        // block; one range per block of 256 or 1024 threads)
        const uint64_t per_launch = g.packed > 0 && mode != MODE_EXACT ? ((1ull << 22) - 1) * (uint64_t)g.packed
                                    : lanes >= 1024 ? (1ull << 22) - 1
                                    : lanes >= 256 ? kMaxBlocks
                                                   : kMaxBlocks * (256u / (lanes ? lanes : 64u));
        if (n > per_launch) {
            const size_t dsz = mode == MODE_PESO ? sizeof(tcsum_peso_t) : sizeof(tcsum_seg_t);
            for (uint64_t i0 = 0; i0 < n; i0 += per_launch) {
                const uint32_t m = (uint32_t)(n - i0 < per_launch ? n - i0 : per_launch);
                const hipError_t e = launch_segments(mode, g, arena, static_cast<const uint8_t *>(descs) + i0 * dsz,
                                                     m, out + i0, aux, stream);
                if (e != hipSuccess)
                    return e;
            }
            return hipSuccess;
        }
    }
    if (g.packed > 0 && mode != MODE_EXACT) {
        const uint32_t K = (uint32_t)g.packed < kPkMaxRanges * kPkWaves ? (uint32_t)g.packed
                                                                          : kPkMaxRanges * kPkWaves;
        const uint8_t *a = static_cast<const uint8_t *>(arena);
        const dim3 gr((n + K - 1) / K), bl(kPkWaves * 64);
        const uint32_t ax = aux | (pf_dist(K) << 8) | (pk_early() ? kPkEarly : 0u);
        if (mode == MODE_SEG)
            return launch(k_segments_pk<MODE_SEG>, gr, bl, 0, stream, a, descs, n, out, ax, (uint32_t)g.xcd, K);
        return launch(k_segments_pk<MODE_PESO>, gr, bl, 0, stream, a, descs, n, out, ax, (uint32_t)g.xcd, K);
    }
    if (mode != MODE_EXACT && g.lanes == 8 && g.loads == 4 && g.interior >= 9 && g.interior <= 24 &&
        knob(KNOB_LANES) < 0 && knob(KNOB_LOADS) < 0) {
        // the per-range kernel for ranges of ~144-415 B (SHUFFLED hint, or a
        // packed batch's K < 3: never at these lengths): fewer load slots than
        // the 8 x 4 the IPv4 kernels keep from pick_geometry -- shuffled 160-B
        // ranges 702 -> 559 us at 4 x 2, 200-B 607 -> 533 at 4 x 3, 250-400-B
        // 7-8 % faster at 8 x 3 (profiles/r06/ab18/seg_shapes.txt)
        if (g.interior <= 10) {
            g.lanes = 4;
            g.loads = 2;
        } else if (g.interior <= 12) {
            g.lanes = 4;
            g.loads = 3;
        } else {
            g.loads = 3;
        }
    }
    if (mode == MODE_EXACT) {
        return launch(k_segments<64, 8, MODE_EXACT>, dim3((n + 3) / 4), dim3(256), 0, stream,
                      static_cast<const uint8_t *>(arena), descs, n, out, aux, 1u);
    }
    if (mode == MODE_SEG)
        return seg_u<MODE_SEG>(g.lanes, g.loads, (uint32_t)g.xcd, n, arena, descs, out, aux, stream);
    return seg_u<MODE_PESO>(g.lanes, g.loads, (uint32_t)g.xcd, n, arena, descs, out, aux, stream);
}

// k_ipv4 in the shapes launch_ipv4's rules make of pick_geometry's (lanes
// clamped to 16..64, rx at 16 where the others take 32).
template <int IPM>
static hipError_t ipv4_u(int G, int U, dim3 grid, uint8_t *arena, const tcsum_pkt_t *pkts, uint32_t n,
                         uint32_t *out, uint8_t *flags, int8_t *verdict, uint32_t opts, uint32_t xg,
                         hipStream_t s)
{
#define TCSUM_IP(GG, UU)                                                                             \
    if (G == GG && U == UU) {                                                                      \
        return launch(k_ipv4<GG, UU, IPM>, grid, dim3(256), 0, s, arena, pkts, n, out, flags, verdict, opts, \
                      xg);                                                                           \
    }
    TCSUM_IP(2, 4) TCSUM_IP(4, 4) TCSUM_IP(8, 3) TCSUM_IP(8, 4) TCSUM_IP(8, 6)
    TCSUM_IP(16, 1) TCSUM_IP(16, 2) TCSUM_IP(16, 3) TCSUM_IP(16, 4) TCSUM_IP(16, 6) TCSUM_IP(16, 8)
    TCSUM_IP(32, 6) TCSUM_IP(64, 4) TCSUM_IP(64, 16)
#undef TCSUM_IP
    return refused();
}


// Stream-ordered scratch for the deferred tx fill, from a pool of the
// library's own per device that keeps up to 1 GiB between calls: the default
// pool hands its memory back at every synchronization, and mapping it again
// cost a synchronized 1M-packet fill ~190 us (profiles/r02/tx_sync_probe.txt).
// The pool is the one of the device the caller's stream belongs to (the
// calling thread's current device only for the null stream).
static std::mutex g_scratch_mu;
static hipMemPool_t g_scratch_pools[64] = {};

static hipError_t scratch_alloc(void **p, size_t bytes, hipStream_t stream)
{
    int dev = 0;
    hipError_t e = stream ? hipStreamGetDevice(stream, &dev) : hipGetDevice(&dev);
    if (e != hipSuccess)
        return e;
    hipMemPool_t pool = nullptr;
    if (dev >= 0 && dev < 64) {
        std::lock_guard<std::mutex> lk(g_scratch_mu);
        if (!g_scratch_pools[dev]) {
            hipMemPoolProps props = {};
            props.allocType = hipMemAllocationTypePinned;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = dev;
            if (quiet(hipMemPoolCreate(&g_scratch_pools[dev], &props)) == hipSuccess) {
                uint64_t keep = 1ull << 30;
                (void)quiet(hipMemPoolSetAttribute(g_scratch_pools[dev], hipMemPoolAttrReleaseThreshold, &keep));
            } else {
                g_scratch_pools[dev] = nullptr;
            }
        }
        pool = g_scratch_pools[dev];
    }
    return pool ? hipMallocFromPoolAsync(p, bytes, pool, stream) : hipMallocAsync(p, bytes, stream);
}

// Bytes the tx fill's scratch pool of device dev holds (tcsum_debug_get
// "scratch_reserved"); 0 before its first deferred fill.
uint64_t scratch_reserved(int dev)
{
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    uint64_t v = 0;
    if (dev >= 0 && dev < 64 && g_scratch_pools[dev])
        (void)quiet(hipMemPoolGetAttribute(g_scratch_pools[dev], hipMemPoolAttrReservedMemCurrent, &v));
    return v;
}

// tcsum_release: hand the pool's kept memory back (the caller has synchronized
// every stream that allocated from it).
hipError_t scratch_trim(int dev)
{
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    if (dev < 0 || dev >= 64 || !g_scratch_pools[dev])
        return hipSuccess;
    return hipMemPoolTrimTo(g_scratch_pools[dev], 0);
}

// The tx fill with its stores deferred (IP_OPT_DEFER + k_tx_scatter): the
// values are computed from `arena` and stored into `store`, the same packets
// at another address (the same arena, or the host memory an HBM copy was
// made from: the scatter's stores then cross PCIe as posted writes).
// `side`: 8 * n bytes of scratch (positions [n], then the values [n] when the
// caller wants no `out`).
static hipError_t tx_split_in(Geometry g, dim3 grid, uint32_t xg, uint8_t *arena, uint8_t *store,
                              const tcsum_pkt_t *pkts, uint32_t n, uint32_t *out, uint8_t *flags, uint32_t *side,
                              hipStream_t stream)
{
    uint32_t *vals = out ? out : side + n;
    hipError_t e = ipv4_u<IP_TX>(g.lanes, g.loads, grid, arena, pkts, n, vals, flags,
                                 reinterpret_cast<int8_t *>(side), IP_OPT_DEFER, xg, stream);
    if (e == hipSuccess) {
        // the warming loads only where the packets sit in device memory
        hipPointerAttribute_t at{};
        const bool hbm = quiet(hipPointerGetAttributes(&at, store)) == hipSuccess && at.type == hipMemoryTypeDevice;
        if (hbm && knob(KNOB_TX_WARM) != 0)
            e = launch(k_tx_scatter<true>, dim3((n + 255) / 256), dim3(256), 0, stream, store, pkts, n, vals, side);
        else
            e = launch(k_tx_scatter<false>, dim3((n + 255) / 256), dim3(256), 0, stream, store, pkts, n, vals, side);
    }
    return e;
}

static hipError_t tx_split(Geometry g, dim3 grid, uint32_t xg, uint8_t *arena, uint8_t *store,
                           const tcsum_pkt_t *pkts, uint32_t n, uint32_t *out, uint8_t *flags, hipStream_t stream)
{
    uint32_t *side = nullptr;
    hipError_t e = scratch_alloc(reinterpret_cast<void **>(&side), (size_t)n * (out ? 4u : 8u), stream);
    if (e != hipSuccess)
        return e;
    e = tx_split_in(g, grid, xg, arena, store, pkts, n, out, flags, side, stream);
    const hipError_t f = hipFreeAsync(side, stream);
    return e != hipSuccess ? e : f;
}

hipError_t launch_ipv4_tx_scratch(Geometry g, uint8_t *arena, const tcsum_pkt_t *pkts, uint32_t n, uint32_t *out,
                                  uint8_t *flags, uint32_t *scratch, hipStream_t stream)
{
    if (n == 0)
        return hipSuccess;
    ipv4_geometry(g, IP_TX); // launch_ipv4's rules
    const uint64_t per_launch = kMaxBlocks * (256u / (uint32_t)g.lanes);
    if (n > per_launch) { // each part uses the scratch of its own packets
        for (uint64_t i0 = 0; i0 < n; i0 += per_launch) {
            const uint32_t m = (uint32_t)(n - i0 < per_launch ? n - i0 : per_launch);
            const hipError_t e = launch_ipv4_tx_scratch(g, arena, pkts + i0, m, out ? out + i0 : nullptr,
                                                        flags ? flags + i0 : nullptr, scratch + 2 * i0, stream);
            if (e != hipSuccess)
                return e;
        }
        return hipSuccess;
    }
    const uint64_t per_block = 256u / (uint32_t)g.lanes;
    return tx_split_in(g, dim3((uint32_t)((n + per_block - 1) / per_block)), (uint32_t)g.xcd, arena, arena, pkts,
                       n, out, flags, scratch, stream);
}

hipError_t launch_ipv4_tx_to(Geometry g, uint8_t *arena, uint8_t *store, const tcsum_pkt_t *pkts, uint32_t n,
                             uint32_t *out, uint8_t *flags, hipStream_t stream)
{
    if (n == 0)
        return hipSuccess;
    ipv4_geometry(g, IP_TX); // launch_ipv4's rules
    const uint64_t per_launch = kMaxBlocks * (256u / (uint32_t)g.lanes);
    if (n > per_launch) {
        for (uint64_t i0 = 0; i0 < n; i0 += per_launch) {
            const uint32_t m = (uint32_t)(n - i0 < per_launch ? n - i0 : per_launch);
            const hipError_t e = launch_ipv4_tx_to(g, arena, store, pkts + i0, m, out ? out + i0 : nullptr,
                                                   flags ? flags + i0 : nullptr, stream);
            if (e != hipSuccess)
                return e;
        }
        return hipSuccess;
    }
    const uint64_t per_block = 256u / (uint32_t)g.lanes;
    return tx_split(g, dim3((uint32_t)((n + per_block - 1) / per_block)), (uint32_t)g.xcd, arena, store, pkts, n,
                    out, flags, stream);
}

// k_ipv4's shape for geometry g: short packets by ipv4_short_shape (unless
// a debug knob forces lanes or loads; a forced shape k_ipv4 is not built in
// is refused), the rest with lanes clamped to 16..64.
void ipv4_geometry(Geometry &g, int ip_mode)
{
    const bool forced = knob(KNOB_LANES) >= 0 || knob(KNOB_LOADS) >= 0;
    if (!forced && ipv4_short_shape(g, ip_mode == IP_RX ? 2 : 0, (uint64_t)g.interior))
        return;
    if (g.lanes < (forced ? 2 : 16))
        g.lanes = forced ? 2 : 16;
    if (g.lanes > 64) // k_ipv4 keeps a packet inside one wave (no workgroup-per-packet form)
        g.lanes = 64;
    // rx keeps more registers live through the data pass (the gate codes, the
    // field sum): with 16 lanes per packet instead of 32 it measured 3.8 %
    // faster on configs[3] (profiles/r02/geom_rx.txt); the other modes keep 32
    if (ip_mode == IP_RX && g.lanes == 32 && knob(KNOB_LANES) < 0)
        g.lanes = 16;
}

hipError_t launch_ipv4(int ip_mode, Geometry g, uint8_t *arena, const tcsum_pkt_t *pkts, uint32_t n,
                       uint32_t *out, uint8_t *flags, int8_t *verdict, hipStream_t stream)
{
    if (n == 0)
        return hipSuccess;
    ipv4_geometry(g, ip_mode);
    const uint64_t per_launch = kMaxBlocks * (256u / (uint32_t)g.lanes);
    if (n > per_launch) { // see kMaxBlocks
        for (uint64_t i0 = 0; i0 < n; i0 += per_launch) {
            const uint32_t m = (uint32_t)(n - i0 < per_launch ? n - i0 : per_launch);
            const hipError_t e = launch_ipv4(ip_mode, g, arena, pkts + i0, m, out ? out + i0 : nullptr,
                                             flags ? flags + i0 : nullptr, verdict ? verdict + i0 : nullptr, stream);
            if (e != hipSuccess)
                return e;
        }
        return hipSuccess;
    }
    const uint64_t per_block = 256u / (uint32_t)g.lanes;
    const dim3 grid((uint32_t)((n + per_block - 1) / per_block));
    const uint32_t xg = (uint32_t)g.xcd;
    switch (ip_mode) {
    case IP_TX:
        return ipv4_u<IP_TX>(g.lanes, g.loads, grid, arena, pkts, n, out, flags, verdict, 0u, xg, stream);
    case IP_TX_SPLIT: // the fill with its stores deferred to k_tx_scatter
        return tx_split(g, grid, xg, arena, arena, pkts, n, out, flags, stream);
    case IP_TX_OFFLOAD: // the tx values into `out` only; the packets are not written
        return ipv4_u<IP_TX>(g.lanes, g.loads, grid, arena, pkts, n, out, flags, verdict, IP_OPT_NO_STORE, xg,
                             stream);
    case IP_RX:
        return ipv4_u<IP_RX>(g.lanes, g.loads, grid, arena, pkts, n, out, flags, verdict, 0u, xg, stream);
    default:
        return ipv4_u<IP_SUMS>(g.lanes, g.loads, grid, arena, pkts, n, out, flags, verdict, 0u, xg, stream);
    }
}

hipError_t launch_server(SrvHost *h, SrvCtl *d, uint32_t last, uint64_t idle_ticks, int wgs, hipStream_t stream)
{
    hipError_t e = hipMemsetAsync(d, 0, sizeof(SrvCtl), stream); // re-initialise every polled word
    if (e != hipSuccess)
        return e;
    // 64 lanes x 16 loads per frame: a frame of up to 16 KiB is one pass -- one
    // PCIe round trip for its bytes (the server's frames live in host memory)
    return launch(k_server<64, 16>, dim3((uint32_t)(wgs > 0 ? wgs : 1)), dim3(256), 0, stream, h, d, last, idle_ticks);
}

// checksum16 on <= kCallInline bytes with the bytes in the kernel arguments
// (the call server's inline job, as a one-shot launch): no PCIe read of a
// descriptor or of staged bytes before the sum -- ipv4.c:243,656's 20-byte
// header checks.  w: the bytes at offset `odd`, zero-padded to 24.
template <int MODE>
__global__ __launch_bounds__(64) void k_inline16(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4,
                                                 uint32_t w5, uint32_t odd, uint32_t len, uint32_t pre,
                                                 uint32_t comp, uint16_t *__restrict__ out)
{
    if (threadIdx.x != 0)
        return;
    uint32_t acc = 0; // the exact word sum of the six dwords is the range's
    acc = dot_halves(acc, w0, 0x00010001u);
    acc = dot_halves(acc, w1, 0x00010001u);
    acc = dot_halves(acc, w2, 0x00010001u);
    acc = dot_halves(acc, w3, 0x00010001u);
    acc = dot_halves(acc, w4, 0x00010001u);
    acc = dot_halves(acc, w5, 0x00010001u);
    SegDesc d;
    d.off = odd;
    d.len = len;
    d.pre = pre;
    d.src = d.dst = d.proto = 0u;
    if constexpr (MODE == MODE_EXACT)
        *out = finalize<MODE_EXACT>(acc, odd, d, comp | (odd << 1), 0u);
    else
        *out = finalize<MODE_SEG>(acc, odd, d, comp, 0u);
}

// One staged range (the drop-in symbols' launch path) with its descriptor in
// the kernel arguments instead of pinned memory: one PCIe read less before
// the bytes.  The call server's staged job as a one-shot launch.
template <int MODE>
__global__ __launch_bounds__(64) void k_once(const uint8_t *__restrict__ stage, uint32_t off, uint32_t len,
                                             uint32_t pre, uint32_t src, uint32_t dst, uint32_t proto, uint32_t comp,
                                             uint16_t *__restrict__ out)
{
    constexpr int G = 64, U = 16; // 16 KiB per pass
    const uint32_t gl = threadIdx.x;
    SegDesc d;
    d.off = off;
    d.len = len;
    d.pre = pre;
    d.src = src;
    d.dst = dst;
    d.proto = proto;
    uint32_t acc = sum_range<G, U, MODE == MODE_EXACT>(stage, off, len, gl, [] {});
    acc = group_sum<G>(acc);
    if (gl == 0) {
        const uintptr_t start = reinterpret_cast<uintptr_t>(stage + off);
        if constexpr (MODE == MODE_EXACT)
            *out = finalize<MODE_EXACT>(acc, start, d, comp | ((off & 1u) << 1), 0u);
        else if constexpr (MODE == MODE_PESO)
            *out = finalize<MODE_PESO>(acc, start, d, 0u, peso_pseudo16(d));
        else
            *out = finalize<MODE_SEG>(acc, start, d, comp, 0u);
    }
}

hipError_t launch_once(Mode mode, const uint8_t *stage, uint32_t off, uint32_t len, uint32_t pre, uint32_t src,
                       uint32_t dst, uint32_t proto, int complement, uint16_t *out, hipStream_t stream)
{
    const uint32_t comp = complement ? 1u : 0u;
    if (mode == MODE_EXACT)
        return launch(k_once<MODE_EXACT>, dim3(1), dim3(64), 0, stream, stage, off, len, pre, src, dst, proto, comp,
                      out);
    if (mode == MODE_PESO)
        return launch(k_once<MODE_PESO>, dim3(1), dim3(64), 0, stream, stage, off, len, pre, src, dst, proto, comp,
                      out);
    return launch(k_once<MODE_SEG>, dim3(1), dim3(64), 0, stream, stage, off, len, pre, src, dst, proto, comp, out);
}

hipError_t launch_inline16(Mode mode, const void *bytes, uint32_t len, uint32_t odd, uint32_t pre, int complement,
                           uint16_t *out, hipStream_t stream)
{
    if (len + odd > kCallInline || (mode != MODE_EXACT && mode != MODE_SEG))
        return refused();
    uint32_t w[6] = {0u, 0u, 0u, 0u, 0u, 0u};
    if (len)
        memcpy(reinterpret_cast<uint8_t *>(w) + odd, bytes, len);
    if (mode == MODE_EXACT)
        return launch(k_inline16<MODE_EXACT>, dim3(1), dim3(64), 0, stream, w[0], w[1], w[2], w[3], w[4], w[5], odd,
                      len, pre, complement ? 1u : 0u, out);
    return launch(k_inline16<MODE_SEG>, dim3(1), dim3(64), 0, stream, w[0], w[1], w[2], w[3], w[4], w[5], odd, len,
                  pre, complement ? 1u : 0u, out);
}

hipError_t launch_call_server(CallBox *box, const uint8_t *stage, uint32_t last, uint64_t idle_ticks,
                              hipStream_t stream)
{
    return launch(k_call, dim3(1), dim3(64), 0, stream, box, stage, last, idle_ticks);
}

} // namespace tcsum
