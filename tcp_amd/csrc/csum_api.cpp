// csum_api.cpp -- the C ABI of libtcsum.so (include/tcsum.h, tcsum_legacy.h,
// tcsum_debug.h): argument checks, per-device context, pinned staging, and
// the legacy drop-in entry points.  Every checksum is computed by the gfx950
// kernels in csum_kernels.hip; nothing here sums bytes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <future>
#include <chrono>
#include <mutex>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <thread>
#include <vector>

#include "csum_launch.h"
#include "tcsum.h"
#include "tcsum_legacy.h"
#include "tcsum_debug.h"

// The drop-in symbols are called with the reference's own structs: the
// mirror types must have the reference's LP64 layout (net/net/list.h:9-34,
// net/net/pktbuf.h:15-41, net/net/ipaddr.h:12-22).
static_assert(sizeof(tcsum_node_t) == 16, "node_t");
static_assert(sizeof(tcsum_list_t) == 24, "list_t");
static_assert(offsetof(tcsum_pktblk_t, size) == 16 && offsetof(tcsum_pktblk_t, data) == 24,
              "pktblk_t");
static_assert(offsetof(tcsum_pktbuf_t, blk_list) == 8 && offsetof(tcsum_pktbuf_t, ref) == 32 &&
                  offsetof(tcsum_pktbuf_t, pos) == 56 && offsetof(tcsum_pktbuf_t, curr_blk) == 64 &&
                  offsetof(tcsum_pktbuf_t, blk_offset) == 72 && sizeof(tcsum_pktbuf_t) == 80,
              "pktbuf_t");
static_assert(offsetof(tcsum_ipaddr_t, addr) == 4 && sizeof(tcsum_ipaddr_t) == 8, "ipaddr_t");
static_assert(sizeof(tcsum_seg_t) == 16 && sizeof(tcsum_peso_t) == 24 && sizeof(tcsum_pkt_t) == 16,
              "descriptors");

namespace {

using tcsum::Geometry;

constexpr int kMaxDev = 16;
constexpr int kHostStreams = 2; // host batches: one copy stream, one kernel stream
constexpr int kHostEvents = 8; // ring of copy-done events (host batches)
constexpr int kPageSlots = 3;  // pinned staging slots of a pageable tcsum_host_batch_peso arena
constexpr uint64_t kPageSlot = 32ull << 20;

// Grow-only pinned, coherent host buffer with its device-side address.
struct Pinned {
    uint8_t *h = nullptr;
    uint8_t *d = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t bytes)
    {
        if (bytes <= cap)
            return hipSuccess;
        size_t c = 1 << 16;
        while (c < bytes)
            c <<= 1;
        if (h)
            (void)tcsum::quiet(hipHostFree(h));
        h = d = nullptr;
        cap = 0;
        hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&h), c, hipHostMallocCoherent);
        if (e != hipSuccess) {
            h = nullptr;
            return e;
        }
        if ((e = hipHostGetDevicePointer(reinterpret_cast<void **>(&d), h, 0)) != hipSuccess) {
            (void)tcsum::quiet(hipHostFree(h));
            h = d = nullptr;
            return e;
        }
        cap = c;
        return hipSuccess;
    }
};

struct Ctx {
    std::mutex mu;
    // set last by ctx_init under mu; legacy_ctx reads it before taking mu
    std::atomic<bool> ready{false};
    int device = -1;
    hipStream_t stream = nullptr; // legacy (synchronous) calls
    // pinned, fine-grained staging the kernel reads/writes directly
    uint8_t *stage = nullptr;
    size_t stage_cap = 0;
    void *desc = nullptr;       // one tcsum_seg_t / tcsum_peso_t
    uint16_t *result = nullptr; // one u16
    uint8_t *d_stage = nullptr; // device-side addresses of the three above
    void *d_desc = nullptr;
    uint16_t *d_result = nullptr;
    uint32_t sync_seq = 0; // run_sync's completion word
    // host-resident batches
    hipStream_t hs[kHostStreams] = {};
    hipEvent_t hev[kHostEvents] = {};
    uint8_t *d_arena = nullptr;
    size_t d_arena_cap = 0;
    uint8_t *d_lead = nullptr; // the first chunk's bytes, copied before the rest is known
    size_t d_lead_cap = 0;
    tcsum_seg_t *d_descs = nullptr;
    size_t d_descs_cap = 0;
    uint16_t *d_out = nullptr;
    size_t d_out_cap = 0;
    // host-queue batches: pinned, fine-grained descriptors / results / a copy
    // of a pageable arena, all read and written by the kernel over PCIe
    Pinned q_desc, q_res, q_arena;
    // tcsum_host_batch_peso from pageable memory: pinned slots the bytes pass
    // through on their way to the copy engine, each with its copy-done event
    Pinned q_page[kPageSlots];
    hipEvent_t pev[kPageSlots] = {};
    bool pev_ok = false;
    // queue server (tcsum_queue_server): a resident grid serving host-queue
    // jobs posted through pinned memory, instead of a launch + wait per job
    bool srv_on = false;      // enabled for this device
    bool srv_running = false; // a grid was launched and not yet seen to finish
    hipStream_t srv_stream = nullptr;
    tcsum::SrvHost *srv_h = nullptr;  // pinned, coherent: host address
    tcsum::SrvHost *srv_hd = nullptr; // ... and the device's address of it
    tcsum::SrvCtl *srv_d = nullptr;
    uint32_t srv_seq = 0; // last job posted (0 = none)
    uint64_t *srv_trace = nullptr; // debug knob "server_trace": phase stamps (host address)
    // call server (tcsum_call_server): one resident wave serving the three
    // synchronous drop-in symbols, instead of a launch + wait per call
    bool cs_on = false;      // enabled for this device
    bool cs_running = false; // the wave was launched and not yet seen to finish
    hipStream_t cs_stream = nullptr;
    tcsum::CallBox *cs_h = nullptr;  // pinned, coherent: host address
    tcsum::CallBox *cs_hd = nullptr; // ... and the device's address of it
    uint8_t *cs_stage = nullptr;     // pinned staging for the call's bytes
    uint8_t *cs_stage_d = nullptr;
    uint32_t cs_seq = 0; // last job posted (0 = none)
};

// Bytes one served call may carry (checksum16's len is a u16; longer pktbuf
// ranges take the launch path).
constexpr size_t kCallStageMax = 1u << 16;

// Launch-path drop-in calls up to this many bytes pass their descriptor (and
// up to kCallInline bytes) in the kernel arguments: one wave, one pass
// (k_once / k_inline16).  Debug knob "args_launch" = 0: the descriptor in pinned
// memory, as before (debug knob "args_launch", include/tcsum_debug.h; read per
// call so one process can run both, tests/test_gpu_parity.py).
constexpr size_t kOnceMax = 16u << 10;
bool args_launch() { return tcsum::knob(tcsum::KNOB_ARGS_LAUNCH) != 0; }

Ctx g_ctx[kMaxDev];
std::mutex g_default_mu;
int g_default_dev = -1;

[[noreturn]] void die(const char *what, hipError_t e)
{
    fprintf(stderr, "tcsum: %s failed: %s -- no CPU fallback, aborting\n", what,
            hipGetErrorString(e));
    abort();
}

// The last failed HIP call of a batch, init or release path:
// step * 1000 + the hipError_t (tcsum_debug_get "last_sys_error"; 0 = none
// yet).  Steps: include/tcsum_debug.h.  Returns `rc`.
std::atomic<int64_t> g_last_sys{0};
// `from_runtime`: e is what a runtime call just returned.  A code the
// library makes up itself (a refused shape, its own time-out) is recorded
// only: the caller's last-error slot may hold the same code as the caller's
// own error, and that stays.
int note_err(int step, hipError_t e, int rc, bool from_runtime = true)
{
    g_last_sys.store((int64_t)step * 1000 + (int64_t)e, std::memory_order_relaxed);
    // the failed call's error is returned as rc: it must not also reach the
    // caller's next hipGetLastError() as an error of the caller's own
    if (from_runtime)
        (void)tcsum::quiet(e);
    return rc;
}
int note_sys(int step, hipError_t e) { return note_err(step, e, TCSUM_ERR_SYS); }
int note_mem(int step, hipError_t e) { return note_err(step, e, TCSUM_ERR_MEM); }

// hipStreamQuery for a poll: hipErrorNotReady is an answer there, not a
// failure.  ROCm 7.2's runtime does not store it in the calling thread's
// last-error slot (scripts/lasterror_probe.hip, profiles/r05/); a runtime
// that did would hand it to the caller's next hipGetLastError() (PyTorch
// checks every kernel launch that way), so a NotReady this poll left in a
// slot that was clear before it is taken out again.
hipError_t poll_stream(hipStream_t s)
{
    const hipError_t before = hipPeekAtLastError();
    const hipError_t q = hipStreamQuery(s);
    if (q == hipErrorNotReady && before == hipSuccess)
        (void)tcsum::quiet(q);
    return q;
}

bool is_gfx950(int dev)
{
    hipDeviceProp_t p;
    if (tcsum::quiet(hipGetDeviceProperties(&p, dev)) != hipSuccess)
        return false;
    return strncmp(p.gcnArchName, "gfx950", 6) == 0;
}

// Initialise ctx for `dev`; returns a net_err_t-style code.
int ctx_init(Ctx &c, int dev)
{
    if (c.ready)
        return TCSUM_OK;
    int count = 0;
    if (tcsum::quiet(hipGetDeviceCount(&count)) != hipSuccess || dev < 0 || dev >= count)
        return TCSUM_ERR_NOT_SUPPORT;
    if (!is_gfx950(dev))
        return TCSUM_ERR_NOT_SUPPORT;
    hipError_t e = hipSetDevice(dev);
    if (e != hipSuccess)
        return note_sys(20, e);
    // a failure part-way leaves what was made so far: the next call resumes
    if (!c.stream && (e = hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking)) != hipSuccess)
        return note_sys(21, e);
    for (auto &s : c.hs)
        if (!s && (e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess)
            return note_sys(22, e);
    for (auto &ev : c.hev)
        if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess)
            return note_sys(23, e);
    if (!c.desc && (e = hipHostMalloc(&c.desc, 64, hipHostMallocCoherent)) != hipSuccess) {
        c.desc = nullptr;
        return note_mem(24, e);
    }
    if (!c.result && (e = hipHostMalloc(reinterpret_cast<void **>(&c.result), 64, hipHostMallocCoherent)) != hipSuccess) {
        c.result = nullptr;
        return note_mem(24, e);
    }
    if ((e = hipHostGetDevicePointer(&c.d_desc, c.desc, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer(reinterpret_cast<void **>(&c.d_result), c.result, 0)) != hipSuccess)
        return note_sys(25, e);
    c.device = dev;
    c.ready = true;
    return TCSUM_OK;
}

int default_device()
{
    std::lock_guard<std::mutex> lk(g_default_mu);
    if (g_default_dev < 0) {
        const char *s = getenv("TCSUM_DEVICE");
        g_default_dev = s ? atoi(s) : 0;
    }
    return g_default_dev;
}

// Legacy context: initialised or abort (the three drop-in symbols have no
// error channel -- SURVEY §8(b)).
Ctx &legacy_ctx()
{
    const int dev = default_device();
    if (dev < 0 || dev >= kMaxDev)
        die("TCSUM_DEVICE", hipErrorInvalidDevice);
    Ctx &c = g_ctx[dev];
    if (!c.ready) {
        std::lock_guard<std::mutex> lk(c.mu);
        const int rc = ctx_init(c, dev);
        if (rc != TCSUM_OK)
            die(rc == TCSUM_ERR_NOT_SUPPORT ? "finding a gfx950 device" : "device init",
                rc == TCSUM_ERR_NOT_SUPPORT ? hipErrorNoDevice : hipErrorOutOfMemory);
        const char *cs = getenv("TCSUM_CALL_SERVER"); // drop-in users: no code change needed
        if (cs && atoi(cs) != 0)
            c.cs_on = true;
    }
    const hipError_t e = hipSetDevice(c.device); // HIP's current device is per thread
    if (e != hipSuccess)
        die("hipSetDevice", e);
    return c;
}

void ensure_stage(Ctx &c, size_t bytes)
{
    bytes += 32; // parity slot + 16-byte tail
    if (bytes <= c.stage_cap)
        return;
    size_t cap = 1 << 16;
    while (cap < bytes)
        cap <<= 1;
    if (c.stage)
        (void)tcsum::quiet(hipHostFree(c.stage));
    c.stage = nullptr;
    c.stage_cap = 0;
    hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&c.stage), cap, hipHostMallocCoherent);
    if (e != hipSuccess)
        die("hipHostMalloc(staging)", e);
    e = hipHostGetDevicePointer(reinterpret_cast<void **>(&c.d_stage), c.stage, 0);
    if (e != hipSuccess)
        die("hipHostGetDevicePointer(staging)", e);
    c.stage_cap = cap;
}

// Wait for everything queued on c.stream.  The stream writes a sequence
// number into pinned memory behind the last kernel and the host spins on that
// word: 13.5-15.5 us per drop-in call against 16.9-17.6 us blocking in
// hipStreamSynchronize (profiles/r02/legacy_latency_poll.txt).
// Debug knob "sync_block" = 1: the latter.  The spin is only the fast path: after 10 s
// (a contended GPU, a profiler serialising kernels) the wait continues in
// hipStreamSynchronize, so a caller never gets control back while its kernels
// may still read or write its buffers; only a real device error is returned.
hipError_t stream_wait(Ctx &c)
{
    if (tcsum::knob(tcsum::KNOB_SYNC_BLOCK) > 0)
        return hipStreamSynchronize(c.stream);
    uint32_t *flag = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(c.result) + 32);
    void *dflag = reinterpret_cast<uint8_t *>(c.d_result) + 32;
    const uint32_t seq = ++c.sync_seq ? c.sync_seq : ++c.sync_seq;
    hipError_t e = hipStreamWriteValue32(c.stream, dflag, seq, 0);
    if (e != hipSuccess)
        return e;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spins = 1; __atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq; ++spins) {
        if ((spins & 4095u) == 0) {
            e = poll_stream(c.stream);
            if (e != hipSuccess && e != hipErrorNotReady)
                return e;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10))
                return hipStreamSynchronize(c.stream); // drains the stream, whatever it takes
        }
        __builtin_ia32_pause();
    }
    return hipSuccess;
}

void run_sync(Ctx &c, hipError_t launched)
{
    if (launched != hipSuccess)
        die("kernel launch", launched);
    const hipError_t e = stream_wait(c);
    if (e != hipSuccess)
        die("waiting for the kernel", e);
}

// ---- pktbuf cursor, restated from net/src/pktbuf.c:153-170, 446-483 ----

inline tcsum_pktblk_t *blk_next(tcsum_pktblk_t *b)
{
    tcsum_node_t *n = b->node.next;
    return n ? reinterpret_cast<tcsum_pktblk_t *>(n) : nullptr; // node is the first member
}

inline int curr_blk_remain(const tcsum_pktbuf_t *buf) // pktbuf.c:162-170
{
    const tcsum_pktblk_t *b = buf->curr_blk;
    return b ? (int)(b->data + b->size - buf->blk_offset) : 0;
}

inline void move_forward(tcsum_pktbuf_t *buf, int size) // pktbuf.c:463-483
{
    buf->pos += size;
    buf->blk_offset += size;
    tcsum_pktblk_t *cur = buf->curr_blk;
    if (buf->blk_offset >= cur->data + cur->size) {
        buf->curr_blk = blk_next(cur);
        buf->blk_offset = buf->curr_blk ? buf->curr_blk->data : nullptr;
    }
}

inline void reset_access(tcsum_pktbuf_t *buf) // pktbuf.c:446-458
{
    buf->pos = 0;
    tcsum_node_t *first = buf->blk_list.first;
    buf->curr_blk = first ? reinterpret_cast<tcsum_pktblk_t *>(first) : nullptr;
    buf->blk_offset = buf->curr_blk ? buf->curr_blk->data : nullptr;
}

void check_ref(const tcsum_pktbuf_t *buf)
{
    if (buf->ref == 0) { // pktbuf.c:648 assert
        fprintf(stderr, "tcsum: pktbuf ref == 0 (assert in pktbuf.c:648), aborting\n");
        abort();
    }
}

// Walk `len` bytes from the cursor the way pktbuf.c:659-668 does, copying
// them into the staging buffer at `dst` and advancing the cursor.
void gather(tcsum_pktbuf_t *buf, int len, uint8_t *dst)
{
    while (len > 0) {
        const int blk = curr_blk_remain(buf);
        const int take = blk > len ? len : blk;
        if (!buf->curr_blk)
            break; // inconsistent total_size; the reference would fault here
        if (take > 0)
            memcpy(dst, buf->blk_offset, (size_t)take);
        dst += take;
        move_forward(buf, take);
        len -= take;
    }
}

} // namespace

// ===================================================================== ABI

extern "C" {

const char *tcsum_version(void) { return "tcsum 0.1 (gfx950, hand-written HIP)"; }

int tcsum_device_count(void)
{
    int count = 0;
    if (tcsum::quiet(hipGetDeviceCount(&count)) != hipSuccess)
        return 0;
    int ok = 0;
    for (int d = 0; d < count; ++d)
        ok += is_gfx950(d) ? 1 : 0;
    return ok;
}

void tcsum_pick_geometry(uint64_t mean_len, int *lanes, int *loads)
{
    const Geometry g = tcsum::pick_geometry(mean_len);
    if (lanes)
        *lanes = g.lanes;
    if (loads)
        *loads = g.loads;
}

int tcsum_plat_init(int device)
{
    if (device < 0 || device >= kMaxDev)
        return TCSUM_ERR_PARAM;
    {
        std::lock_guard<std::mutex> lk(g_default_mu);
        g_default_dev = device;
    }
    Ctx &c = g_ctx[device];
    std::lock_guard<std::mutex> lk(c.mu);
    return ctx_init(c, device);
}

void *tcsum_host_alloc(size_t bytes)
{
    void *p = nullptr;
    // portable: a multi-device host batch reads it from every GPU's link
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable) != hipSuccess)
        return nullptr;
    return p;
}

void tcsum_host_free(void *p)
{
    if (p)
        (void)tcsum::quiet(hipHostFree(p));
}

int tcsum_host_register(void *p, size_t bytes)
{
    if (!p || bytes == 0)
        return TCSUM_ERR_PARAM;
    // portable + mapped, like tcsum_host_alloc: every GPU of a *_multi batch maps it
    if (const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable);
        e != hipSuccess)
        return note_sys(60, e);
    return TCSUM_OK;
}

int tcsum_host_unregister(void *p)
{
    if (!p)
        return TCSUM_ERR_PARAM;
    if (const hipError_t e = hipHostUnregister(p); e != hipSuccess)
        return note_sys(61, e);
    return TCSUM_OK;
}

// ------------------------------------------------------------ debug knobs

static const struct {
    const char *key;
    tcsum::Knob k;
} kKnobs[] = {
    {"lanes", tcsum::KNOB_LANES},         {"loads", tcsum::KNOB_LOADS},
    {"xcd", tcsum::KNOB_XCD},             {"packed", tcsum::KNOB_PACKED},
    {"tx_split", tcsum::KNOB_TX_SPLIT},
    {"args_launch", tcsum::KNOB_ARGS_LAUNCH}, {"sync_block", tcsum::KNOB_SYNC_BLOCK},
    {"e2e_trace", tcsum::KNOB_E2E_TRACE}, {"e2e_chunk_mb", tcsum::KNOB_E2E_CHUNK_MB},
    {"server_max", tcsum::KNOB_SERVER_MAX}, {"server_trace", tcsum::KNOB_SERVER_TRACE},
    {"server_idle_ms", tcsum::KNOB_SERVER_IDLE_MS}, {"server_wgs", tcsum::KNOB_SERVER_WGS},
    {"hostq_dma_kb", tcsum::KNOB_HOSTQ_DMA_KB}, {"hostq_dma_keep_mb", tcsum::KNOB_HOSTQ_DMA_KEEP_MB},
    {"copy_threads", tcsum::KNOB_COPY_THREADS}, {"pf_dist", tcsum::KNOB_PF_DIST}, {"pf_range", tcsum::KNOB_PF_RANGE},
    {"pk_early", tcsum::KNOB_PK_EARLY}, {"page_stage", tcsum::KNOB_PAGE_STAGE},
    {"seg_sdesc", tcsum::KNOB_SEG_SDESC}, {"tx_warm", tcsum::KNOB_TX_WARM},
};

static int knob_of(const char *key)
{
    if (key)
        for (const auto &e : kKnobs)
            if (strcmp(e.key, key) == 0)
                return e.k;
    return -1;
}

int tcsum_debug_set(const char *key, int64_t value)
{
    const int k = knob_of(key);
    if (k < 0 || value < -1)
        return TCSUM_ERR_PARAM;
    tcsum::set_knob((tcsum::Knob)k, value);
    return TCSUM_OK;
}

int64_t tcsum_debug_get(const char *key)
{
    if (key && strcmp(key, "last_sys_error") == 0)
        return g_last_sys.load(std::memory_order_relaxed);
    if (key && strcmp(key, "scratch_reserved") == 0) { // the calling thread's current device
        int dev = 0;
        return tcsum::quiet(hipGetDevice(&dev)) == hipSuccess ? (int64_t)tcsum::scratch_reserved(dev) : -2;
    }
    const int k = knob_of(key);
    return k < 0 ? -2 : tcsum::knob((tcsum::Knob)k);
}

void tcsum_debug_ipv4_route(uint64_t mean_len, int ip_mode, int32_t out[2])
{
    Geometry g = tcsum::pick_geometry(mean_len);
    tcsum::ipv4_geometry(g, ip_mode);
    if (out) {
        out[0] = g.lanes;
        out[1] = g.loads;
    }
}

void tcsum_debug_route(uint64_t mean_len, int32_t out[5])
{
    const Geometry g = tcsum::pick_geometry(mean_len);
    if (out) {
        out[0] = g.lanes;
        out[1] = g.loads;
        out[2] = g.xcd;
        out[3] = g.packed;
        Geometry s = g; // what a SHUFFLED batch (or a host chunk out of offset order) takes
        tcsum::shuffled_route(s, tcsum::knob(tcsum::KNOB_PACKED));
        out[4] = s.packed;
    }
}

// hipErrorInvalidValue from a launcher: a shape or size it refuses
static int rc_of(hipError_t e)
{
    if (e == hipSuccess)
        return TCSUM_OK;
    const bool mine = tcsum::take_refused() && e == hipErrorInvalidValue;
    return e == hipErrorInvalidValue ? note_err(70, e, TCSUM_ERR_PARAM, !mine) : note_sys(70, e);
}

static uint64_t mean_of(uint64_t total, uint32_t n) { return total && n ? total / n : 1500; }

// device tx fills of at least this many packets, of at least this mean
// length, defer their stores (mode 4).  Shorter packets keep the stores in
// the kernel: equal 100-B packets 3,451 against 5,852 us deferred, 300-B
// 1,794 / 2,801, 1,000-B 1,077 / 1,200, 2,500-B 895 / 919; 3,000-B 891 /
// 838 (profiles/r06/ab24/tx_short*.txt) -- millions of scattered field
// writes in a second launch cost more than the in-kernel stores save there.
static constexpr uint32_t kTxSplitMin = 131072;
static constexpr uint64_t kTxSplitMinLen = 2800;

// The route for a batch and what its caller knows of the layout
// (tcsum_hint_t): SHUFFLED skips the stream kernel where its workgroups,
// finding out one by one, would be slower than the per-range kernel
// (tcsum::shuffled_route: ranges under ~1.5 KiB); the debug knob "packed" set
// to 1 keeps it on regardless.
static Geometry route_for(uint64_t total, uint32_t n, uint32_t layout)
{
    Geometry g = tcsum::pick_geometry(mean_of(total, n));
    if (layout == TCSUM_LAYOUT_SHUFFLED)
        tcsum::shuffled_route(g, tcsum::knob(tcsum::KNOB_PACKED));
    return g;
}

int tcsum_batch(int op, void *arena, const void *descs, uint32_t n, void *out, uint8_t *flags, int8_t *verdict,
                const tcsum_hint_t *hint, void *stream)
{
    if (n == 0)
        return TCSUM_OK;
    const uint64_t total = hint ? hint->total_bytes : 0;
    const uint32_t layout = hint ? hint->layout : TCSUM_LAYOUT_UNKNOWN;
    if (!arena || !descs || layout > TCSUM_LAYOUT_SHUFFLED || (hint && hint->rsv != 0))
        return TCSUM_ERR_PARAM;
    const Geometry g = route_for(total, n, layout);
    const hipStream_t st = static_cast<hipStream_t>(stream);
    uint8_t *a = static_cast<uint8_t *>(arena);
    const tcsum_pkt_t *pk = static_cast<const tcsum_pkt_t *>(descs);
    switch (op) {
    case TCSUM_OP_SEGMENTS:
    case TCSUM_OP_SEGMENTS_COMP:
    case TCSUM_OP_PESO:
        if (!out)
            return TCSUM_ERR_PARAM;
        return rc_of(tcsum::launch_segments(op == TCSUM_OP_PESO ? tcsum::MODE_PESO : tcsum::MODE_SEG, g, arena,
                                            descs, n, static_cast<uint16_t *>(out),
                                            op == TCSUM_OP_SEGMENTS_COMP ? 1u : 0u, st));
    case TCSUM_OP_IPV4:
        if (!out)
            return TCSUM_ERR_PARAM;
        return rc_of(tcsum::launch_ipv4(0, g, a, pk, n, static_cast<uint32_t *>(out), flags, nullptr, st));
    case TCSUM_OP_IPV4_TX_FILL: {
        // Large batches: every packet's values and store positions first, then
        // all the field stores in one short second launch (mode 4) -- 4-6 %
        // faster on configs[3] than storing each packet's fields as its sums
        // finish, which trickles a million isolated writes through the read
        // stream (profiles/history/DESIGN_rounds1-5.md §6, tx fill).  Small batches keep one launch.
        // Debug knob "tx_split" forces.  Under hipGraph capture the
        // single-launch form is taken: it allocates nothing (tcsum.h).
        const int64_t ks = tcsum::knob(tcsum::KNOB_TX_SPLIT);
        bool split = ks >= 0 ? ks != 0 : n >= kTxSplitMin && mean_of(total, n) >= kTxSplitMinLen;
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        if (split && tcsum::quiet(hipStreamIsCapturing(st, &cap)) == hipSuccess && cap != hipStreamCaptureStatusNone)
            split = false;
        return rc_of(tcsum::launch_ipv4(split ? 4 : 1, g, a, pk, n, static_cast<uint32_t *>(out), flags, nullptr, st));
    }
    case TCSUM_OP_IPV4_TX_OFFLOAD:
        if (!out || !flags)
            return TCSUM_ERR_PARAM;
        // the kernel never writes the arena in this mode
        return rc_of(tcsum::launch_ipv4(3, g, a, pk, n, static_cast<uint32_t *>(out), flags, nullptr, st));
    case TCSUM_OP_IPV4_RX_VERIFY:
        if (!verdict)
            return TCSUM_ERR_PARAM;
        // the kernel never writes the arena in this mode
        return rc_of(tcsum::launch_ipv4(2, g, a, pk, n, static_cast<uint32_t *>(out), flags, verdict, st));
    default:
        return TCSUM_ERR_PARAM;
    }
}

static int batch_unknown(int op, const void *arena, const void *descs, uint32_t n, void *out, uint8_t *flags,
                         int8_t *verdict, uint64_t total_bytes_hint, void *stream)
{
    const tcsum_hint_t h{total_bytes_hint, TCSUM_LAYOUT_UNKNOWN, 0u};
    return tcsum_batch(op, const_cast<void *>(arena), descs, n, out, flags, verdict, &h, stream);
}

int tcsum_batch_segments(const void *arena, const tcsum_seg_t *segs, uint32_t n, uint16_t *out,
                         int complement, uint64_t total_bytes_hint, void *stream)
{
    return batch_unknown(complement ? TCSUM_OP_SEGMENTS_COMP : TCSUM_OP_SEGMENTS, arena, segs, n, out, nullptr,
                         nullptr, total_bytes_hint, stream);
}

int tcsum_batch_peso(const void *arena, const tcsum_peso_t *segs, uint32_t n, uint16_t *out,
                     uint64_t total_bytes_hint, void *stream)
{
    return batch_unknown(TCSUM_OP_PESO, arena, segs, n, out, nullptr, nullptr, total_bytes_hint, stream);
}

int tcsum_batch_ipv4(const void *arena, const tcsum_pkt_t *pkts, uint32_t n, uint32_t *out,
                     uint8_t *flags, uint64_t total_bytes_hint, void *stream)
{
    return batch_unknown(TCSUM_OP_IPV4, arena, pkts, n, out, flags, nullptr, total_bytes_hint, stream);
}

int tcsum_batch_ipv4_tx_fill(void *arena, const tcsum_pkt_t *pkts, uint32_t n, uint32_t *out, uint8_t *flags,
                             uint64_t total_bytes_hint, void *stream)
{
    return batch_unknown(TCSUM_OP_IPV4_TX_FILL, arena, pkts, n, out, flags, nullptr, total_bytes_hint, stream);
}

int tcsum_batch_ipv4_tx_fill_scratch(void *arena, const tcsum_pkt_t *pkts, uint32_t n, uint32_t *out,
                                     uint8_t *flags, void *scratch, uint64_t scratch_bytes, uint64_t total_bytes_hint,
                                     void *stream)
{
    if (n == 0)
        return TCSUM_OK;
    if (!arena || !pkts || !scratch || (reinterpret_cast<uintptr_t>(scratch) & 3u) || scratch_bytes < 8ull * n)
        return TCSUM_ERR_PARAM;
    const hipError_t e = tcsum::launch_ipv4_tx_scratch(tcsum::pick_geometry(mean_of(total_bytes_hint, n)),
                                                       static_cast<uint8_t *>(arena), pkts, n, out, flags,
                                                       static_cast<uint32_t *>(scratch),
                                                       static_cast<hipStream_t>(stream));
    return rc_of(e);
}

int tcsum_batch_ipv4_tx_offload(const void *arena, const tcsum_pkt_t *pkts, uint32_t n, uint32_t *out,
                                uint8_t *flags, uint64_t total_bytes_hint, void *stream)
{
    return batch_unknown(TCSUM_OP_IPV4_TX_OFFLOAD, arena, pkts, n, out, flags, nullptr, total_bytes_hint, stream);
}

// Host side of the offload contract: the stores k_ipv4<IP_TX> makes, driven
// by the flags it computed (so no header gate is restated here).
int tcsum_tx_apply(void *frame, uint32_t len, uint32_t csums, uint8_t flags)
{
    if (!frame)
        return TCSUM_ERR_PARAM;
    if (flags & (TCSUM_PKT_SHORT | TCSUM_PKT_BAD_VERSION | TCSUM_PKT_BAD_HDRLEN | TCSUM_PKT_BAD_TOTLEN))
        return TCSUM_OK; // the fill writes nothing into a rejected packet
    if (len < 20)
        return TCSUM_ERR_PARAM; // flags that do not belong to this frame
    uint8_t *p = static_cast<uint8_t *>(frame);
    p[10] = (uint8_t)csums; // ipv4.c:643,656, host order like the struct field
    p[11] = (uint8_t)(csums >> 8);
    if (flags & (TCSUM_PKT_FRAGMENT | TCSUM_PKT_L4_SHORT | TCSUM_PKT_PROTO_OTHER))
        return TCSUM_OK;
    const uint32_t hl = (uint32_t)(p[0] & 0xFu) << 2;
    const uint32_t fld = p[9] == 6 ? 16u : p[9] == 17 ? 6u : p[9] == 1 ? 2u : 0u; // tcp.h:71 udp.h:24 icmpv4.h:28
    if (!fld || hl + fld + 2 > len)
        return TCSUM_ERR_PARAM;
    p[hl + fld] = (uint8_t)(csums >> 16); // tcp_out.c:19-20 / udp.c:320-321 / icmpv4.c:45-58
    p[hl + fld + 1] = (uint8_t)(csums >> 24);
    return TCSUM_OK;
}

int tcsum_tx_apply_batch(void *arena, uint64_t arena_bytes, const tcsum_pkt_t *pkts, uint32_t n,
                         const uint32_t *csums, const uint8_t *flags)
{
    if (n == 0)
        return TCSUM_OK;
    if (!arena || !pkts || !csums || !flags)
        return TCSUM_ERR_PARAM;
    for (uint32_t i = 0; i < n; ++i)
        if (pkts[i].offset > arena_bytes || pkts[i].len > arena_bytes - pkts[i].offset)
            return TCSUM_ERR_PARAM;
    int rc = TCSUM_OK;
    for (uint32_t i = 0; i < n; ++i) {
        const int r = tcsum_tx_apply(static_cast<uint8_t *>(arena) + pkts[i].offset, pkts[i].len, csums[i], flags[i]);
        rc = rc == TCSUM_OK ? r : rc;
    }
    return rc;
}

int tcsum_batch_ipv4_rx_verify(const void *arena, const tcsum_pkt_t *pkts, uint32_t n, int8_t *verdict,
                               uint32_t *out, uint8_t *flags, uint64_t total_bytes_hint, void *stream)
{
    return batch_unknown(TCSUM_OP_IPV4_RX_VERIFY, arena, pkts, n, out, flags, verdict, total_bytes_hint, stream);
}

// ------------------------------------------------------------ host batches

namespace { // defined with the host-queue batches below
uint8_t *mapped_host(const void *p);
void par_memcpy(uint8_t *dst, const uint8_t *src, size_t n);
extern "C++" {
template <class F>
void parallel_for(size_t n, size_t min_per, F &&f);
}

// Byte span [lo, hi) and byte count of a run of segments.
// `ordered`: the non-empty segments' offsets never decrease (first / last:
// the first and last such offset); merged in segment order.
struct HostSpan {
    uint64_t lo = UINT64_MAX, hi = 0, bytes = 0;
    uint64_t first = UINT64_MAX, last = 0;
    bool bad = false, ordered = true;
    void merge(const HostSpan &o)
    {
        lo = o.lo < lo ? o.lo : lo;
        hi = o.hi > hi ? o.hi : hi;
        bytes += o.bytes;
        bad |= o.bad;
        if (o.first != UINT64_MAX) {
            ordered = ordered && o.ordered && (first == UINT64_MAX || o.first >= last);
            first = first == UINT64_MAX ? o.first : first;
            last = o.last;
        }
    }
};

extern "C++" { // (inside the extern "C" block: C++ linkage for these helpers)
// ---- tcsum_host_batch_peso's plan: which bytes go where, which kernels
// run on which descriptors.  Host arithmetic only (no HIP call), so the plan
// of any batch can be checked without a device (tcsum_debug_plan_host_peso,
// tests/test_abi.py): every copy inside the caller's arena and its device
// buffer, every byte a kernel reads copied before it.

constexpr uint32_t kSpanBlock = 4096; // segments per span block

// The device buffer bytes a span needs: its 16-byte chunks from the one
// holding lo, plus a 16-byte tail so the last aligned chunk is in bounds.
uint64_t span_bytes(const HostSpan &sp)
{
    return sp.hi > sp.lo ? (((sp.hi - (sp.lo & ~uint64_t(15))) + 15) & ~uint64_t(15)) + 16 : 16;
}

// The host bytes [lo, hi) a span's copy moves (whole 16-byte chunks, cut at
// the arena's end); empty when the span is.
void span_copy(const HostSpan &sp, uint64_t arena_bytes, uint64_t &lo, uint64_t &hi)
{
    lo = hi = 0;
    if (sp.hi <= sp.lo)
        return;
    lo = sp.lo & ~uint64_t(15);
    hi = std::min(arena_bytes, (sp.hi + 15) & ~uint64_t(15));
}

struct PesoChunk {
    uint32_t b0, b1; // span blocks [b0, b1)
    HostSpan sp;
    int buf;         // 0: the lead's buffer, 1: the arena buffer
};

struct PesoPlan {
    uint32_t n = 0, nblk = 0;
    uint32_t m = 0;      // blocks of the lead
    bool early = false;  // the lead's copy starts before the rest is looked at
    uint64_t target = 0; // chunk size in packet bytes
    HostSpan lead, rest; // the lead's span; the span of the blocks after it (all of them if !early)
    std::vector<HostSpan> blk;
    std::vector<PesoChunk> ch;
    uint32_t r0() const { return early ? m : 0u; }
    // device buffer sizes and where arena offset 0 sits in each (offset of
    // arena byte x in buffer b: x - base[b])
    uint64_t lead_base() const { return lead.hi ? lead.lo & ~uint64_t(15) : 0; }
    uint64_t rest_base() const { return rest.hi ? rest.lo & ~uint64_t(15) : 0; }
};

HostSpan span_of_block(const tcsum_peso_t *segs, uint32_t n, uint64_t arena_bytes, size_t k)
{
    HostSpan sp;
    const uint32_t i1 = (uint32_t)std::min<uint64_t>(n, (k + 1) * (uint64_t)kSpanBlock);
    for (uint32_t i = (uint32_t)k * kSpanBlock; i < i1; ++i) {
        const uint64_t o = segs[i].offset, l = segs[i].len;
        sp.bad |= o > arena_bytes || l > arena_bytes - o;
        if (l) {
            sp.lo = o < sp.lo ? o : sp.lo;
            sp.hi = o + l > sp.hi ? o + l : sp.hi;
            sp.bytes += l;
            sp.ordered &= sp.first == UINT64_MAX || o >= sp.last;
            sp.first = sp.first == UINT64_MAX ? o : sp.first;
            sp.last = o;
        }
    }
    return sp;
}

// Stage 1, on the calling thread before anything else: the chunk size and
// the lead -- the first blocks, up to 64 MiB of packet bytes.  When they are
// dense (their span at most 1.25x their bytes) their copy starts at once,
// into a buffer of their own, and the rest of the descriptors are looked at
// while it runs (the whole pass first kept the link idle for 420-635 us of a
// 29-ms batch).  false: a lead segment lies outside the arena.
bool peso_plan_lead(PesoPlan &pl, const tcsum_peso_t *segs, uint32_t n, uint64_t arena_bytes)
{
    pl.n = n;
    pl.nblk = (n + kSpanBlock - 1) / kSpanBlock;
    pl.blk.assign(pl.nblk, HostSpan());
    // Chunks of >= `target` packet bytes (whole span blocks).  All copies go
    // in order on ONE copy stream, so the host link never idles between
    // chunks and no two copies compete for it; each chunk's kernel waits on
    // its copy's event on the kernel stream and runs under the next copy.
    // Every copy costs ~18 us of link idle before it (rocprofv3
    // --memory-copy-trace, profiles/r02/e2e_phase.txt), so chunks are large:
    // a quarter of the batch, at least 64 MiB (debug knob "e2e_chunk_mb": fixed size).
    const uint32_t step = std::max<uint32_t>(1, n / 64); // the batch's bytes, estimated from 64 segments
    uint64_t sampled = 0, taken = 0;
    for (uint32_t i = 0; i < n; i += step, ++taken)
        sampled += segs[i].len;
    const uint64_t total_hint = sampled / taken * (uint64_t)n;
    pl.target = std::max<uint64_t>(64ull << 20, total_hint / 4);
    if (const int64_t v = tcsum::knob(tcsum::KNOB_E2E_CHUNK_MB); v > 0)
        pl.target = (uint64_t)v << 20;
    const uint64_t lead_target = std::min<uint64_t>(pl.target, 64ull << 20);
    pl.m = 0;
    while (pl.m < pl.nblk && pl.lead.bytes < lead_target) {
        pl.blk[pl.m] = span_of_block(segs, n, arena_bytes, pl.m);
        pl.lead.merge(pl.blk[pl.m]);
        ++pl.m;
    }
    if (pl.lead.bad)
        return false;
    pl.early = pl.m < pl.nblk && pl.lead.hi > pl.lead.lo && pl.lead.hi - pl.lead.lo <= pl.lead.bytes + pl.lead.bytes / 4;
    return true;
}

// Stage 2 (while the lead's bytes cross): the other blocks' spans, in
// parallel, and the chunks: [the lead], then the rest in `target`-byte
// chunks.  false: a segment lies outside the arena.
bool peso_plan_rest(PesoPlan &pl, const tcsum_peso_t *segs, uint64_t arena_bytes)
{
    const uint32_t m = pl.m, nblk = pl.nblk, r0 = pl.r0(), n = pl.n;
    parallel_for(nblk - m, 16, [&](size_t b, size_t e) {
        for (size_t k = m + b; k < m + e; ++k)
            pl.blk[k] = span_of_block(segs, n, arena_bytes, k);
    });
    for (uint32_t k = r0; k < nblk; ++k)
        pl.rest.merge(pl.blk[k]);
    if (pl.rest.bad)
        return false;
    pl.ch.clear();
    if (pl.early)
        pl.ch.push_back({0u, m, pl.lead, 0});
    const size_t first_rest = pl.ch.size();
    for (uint32_t k = r0; k < nblk; ++k) {
        if (pl.ch.size() == first_rest || pl.ch.back().sp.bytes >= pl.target)
            pl.ch.push_back({k, k, HostSpan(), 1});
        pl.ch.back().sp.merge(pl.blk[k]);
        pl.ch.back().b1 = k + 1;
    }
    // segments in no particular order: every chunk's span covers most of the
    // batch's, so copy the batch's span once and run one kernel on it
    uint64_t spans = 0;
    for (size_t k = first_rest; k < pl.ch.size(); ++k)
        spans += pl.ch[k].sp.hi > pl.ch[k].sp.lo ? pl.ch[k].sp.hi - pl.ch[k].sp.lo : 0;
    const uint64_t rest_span = pl.rest.hi > pl.rest.lo ? pl.rest.hi - pl.rest.lo : 0;
    if (pl.ch.size() > first_rest + 1 && spans > rest_span + rest_span / 4) {
        pl.ch.resize(first_rest);
        pl.ch.push_back({r0, nblk, pl.rest, 1});
    }
    return true;
}
} // extern "C++"
} // namespace

int tcsum_host_batch_peso(int device, const void *host_arena, uint64_t arena_bytes,
                          const tcsum_peso_t *segs, uint32_t n, uint16_t *out)
{
    if (n == 0)
        return TCSUM_OK;
    // debug knob "e2e_trace" = 1: host-side phase times of this call on stderr (measurement)
    const bool trace = tcsum::knob(tcsum::KNOB_E2E_TRACE) > 0;
    const auto t_start = std::chrono::steady_clock::now();
    auto stamp = [&](const char *what) {
        if (trace)
            fprintf(stderr, "e2e %-16s %9.1f us\n", what,
                    std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_start).count());
    };
    if (!host_arena || !segs || !out || device < 0 || device >= kMaxDev)
        return TCSUM_ERR_PARAM;
    PesoPlan pl;
    if (!peso_plan_lead(pl, segs, n, arena_bytes))
        return TCSUM_ERR_PARAM;
    stamp("lead");

    Ctx &c = g_ctx[device];
    std::lock_guard<std::mutex> lk(c.mu);
    int rc = ctx_init(c, device); // a failing HIP call is recorded there (steps 20-25)
    if (rc != TCSUM_OK)
        return rc;
    if (const hipError_t e = hipSetDevice(device); e != hipSuccess)
        return note_sys(1, e);
    const uint8_t *h = static_cast<const uint8_t *>(host_arena);
    hipStream_t cs = c.hs[0], ks = c.hs[1];
    // device buffers (grow-only) hold only the spans the segments touch (a
    // shard of a multi-device batch holds its own part only)
    auto grow = [](uint8_t *&buf, size_t &cap, size_t need) {
        if (need <= cap)
            return hipSuccess;
        if (buf)
            (void)tcsum::quiet(hipFree(buf));
        buf = nullptr;
        cap = 0;
        const hipError_t e = hipMalloc(reinterpret_cast<void **>(&buf), need);
        if (e != hipSuccess) {
            buf = nullptr;
            return e;
        }
        cap = need;
        return hipSuccess;
    };
    // Pageable caller memory passes through the context's pinned slots (host
    // threads fill one while the copy engine drains the others): every DMA
    // reads memory the library owns.  Round 5 moved off the runtime's own
    // pageable path after two suites stopped at this call's first copy; round
    // 6 found the runtime's path clean on its own and the fault's cause
    // elsewhere unrecorded.  Debug knob "page_stage" = 0: the
    // runtime's path (measurement: 50.5 against 49.6 GiB/s,
    // profiles/r06/ab/e2e_pageable.txt).
    const bool pageable = tcsum::knob(tcsum::KNOB_PAGE_STAGE) != 0 && mapped_host(host_arena) == nullptr;
    if (pageable && !c.pev_ok) {
        for (auto &e : c.pev) // a failure part-way keeps those made: the next call makes only the rest
            if (!e)
                if (const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming); r != hipSuccess) {
                    e = nullptr;
                    return note_sys(17, r);
                }
        c.pev_ok = true;
    }
    bool slot_busy[kPageSlots] = {};
    int slot_turn = 0;
    auto copy_staged = [&](uint8_t *dst, const uint8_t *src, uint64_t bytes) -> hipError_t {
        for (uint64_t o = 0; o < bytes; o += kPageSlot) {
            const int s = slot_turn;
            slot_turn = (slot_turn + 1) % kPageSlots;
            if (slot_busy[s])
                if (const hipError_t e = hipEventSynchronize(c.pev[s]); e != hipSuccess)
                    return e;
            const uint64_t len = std::min(kPageSlot, bytes - o);
            if (const hipError_t e = c.q_page[s].reserve(kPageSlot); e != hipSuccess)
                return e;
            par_memcpy(c.q_page[s].h, src + o, len);
            if (const hipError_t e = hipMemcpyAsync(dst + o, c.q_page[s].h, len, hipMemcpyHostToDevice, cs);
                e != hipSuccess)
                return e;
            if (const hipError_t e = hipEventRecord(c.pev[s], cs); e != hipSuccess)
                return e;
            slot_busy[s] = true;
        }
        return hipSuccess;
    };
    // copy a span into buffer `buf` of the plan
    uint8_t *base[2] = {nullptr, nullptr}; // device address arena offset 0 has in each buffer
    auto copy_span = [&](int buf, const HostSpan &sp) {
        uint64_t lo, hi;
        span_copy(sp, arena_bytes, lo, hi);
        if (hi <= lo)
            return hipSuccess;
        if (pageable)
            return copy_staged(base[buf] + lo, h + lo, hi - lo);
        return hipMemcpyAsync(base[buf] + lo, h + lo, hi - lo, hipMemcpyHostToDevice, cs);
    };
    // once a copy is queued, an error return first drains both streams: no
    // copy may still read the caller's memory after the call returns
    auto fail = [&](int code) {
        (void)tcsum::quiet(hipStreamSynchronize(ks));
        (void)tcsum::quiet(hipStreamSynchronize(cs));
        return code;
    };
    // (a pinned staging slot that cannot be allocated is TCSUM_ERR_MEM)
    auto fail_sys = [&](int step, hipError_t e) {
        return fail(e == hipErrorOutOfMemory ? note_mem(step, e) : note_sys(step, e));
    };
    if (pl.early) {
        if (const hipError_t e = grow(c.d_lead, c.d_lead_cap, span_bytes(pl.lead)); e != hipSuccess)
            return note_mem(13, e);
        base[0] = c.d_lead - pl.lead_base();
        if (const hipError_t e = copy_span(0, pl.lead); e != hipSuccess)
            return fail_sys(2, e);
        stamp("lead copy");
    }
    if (!peso_plan_rest(pl, segs, arena_bytes))
        return fail(TCSUM_ERR_PARAM);
    stamp("span pass");
    if (const hipError_t e = grow(c.d_arena, c.d_arena_cap, span_bytes(pl.rest)); e != hipSuccess)
        return fail(note_mem(14, e));
    base[1] = c.d_arena - pl.rest_base();
    if (n > c.d_descs_cap) {
        if (c.d_descs)
            (void)tcsum::quiet(hipFree(c.d_descs));
        if (c.d_out)
            (void)tcsum::quiet(hipFree(c.d_out));
        c.d_descs = nullptr;
        c.d_out = nullptr;
        c.d_descs_cap = c.d_out_cap = 0;
        hipError_t e = hipMalloc(reinterpret_cast<void **>(&c.d_descs), sizeof(tcsum_seg_t) * n);
        if (e == hipSuccess)
            e = hipMalloc(reinterpret_cast<void **>(&c.d_out), sizeof(uint16_t) * n);
        if (e != hipSuccess) {
            if (c.d_descs)
                (void)tcsum::quiet(hipFree(c.d_descs)); // both or neither: the caps below describe both
            c.d_descs = nullptr;
            c.d_out = nullptr;
            return fail(note_mem(15, e));
        }
        c.d_descs_cap = c.d_out_cap = n;
    }
    const std::vector<PesoChunk> &ch = pl.ch;
    // a hipMemcpyAsync from pageable memory is staged by the runtime per call
    // (~100 us per chunk), so descriptors and results go through pinned
    // staging.  The descriptors cross the link as tcsum_seg_t (16 B, not 24):
    // checksum_peso is pktbuf_checksum16 over the segment with the folded
    // pseudo-header as pre_sum (tools.c:58-73), so the pseudo-header is folded
    // here, in the staging pass, and the kernels run as pktbuf_checksum16
    const bool stage_out = !mapped_host(out);
    if (const hipError_t e = c.q_desc.reserve(sizeof(tcsum_seg_t) * n); e != hipSuccess)
        return fail(note_mem(16, e));
    if (const hipError_t e = stage_out ? c.q_res.reserve(sizeof(uint16_t) * n + 64) : hipSuccess; e != hipSuccess)
        return fail(note_mem(16, e));
    uint16_t *hout = stage_out ? reinterpret_cast<uint16_t *>(c.q_res.h) : out;
    // The first chunk's bytes cross while the host stages the descriptors.
    // From pinned memory its copy is queued and returns at once; a pageable
    // arena's goes slot by slot through host copies that wait on the copy
    // engine, so a large one (a shuffled batch collapses to ONE chunk, the
    // whole span) runs on a thread of its own beside the descriptor pass.
    std::future<hipError_t> first_copy;
    if (!pl.early) {
        uint64_t lo, hi;
        span_copy(ch[0].sp, arena_bytes, lo, hi);
        if (pageable && hi > lo && hi - lo >= kPageSlot) {
            first_copy = std::async(std::launch::async, [&, device] {
                const hipError_t e = hipSetDevice(device); // HIP's current device is per thread
                return e != hipSuccess ? e : copy_span(ch[0].buf, ch[0].sp);
            });
        } else if (const hipError_t e = copy_span(ch[0].buf, ch[0].sp); e != hipSuccess) {
            return fail_sys(3, e);
        }
    }
    tcsum_seg_t *hseg = reinterpret_cast<tcsum_seg_t *>(c.q_desc.h);
    parallel_for(n, size_t(1) << 16, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; ++i) {
            const tcsum_peso_t &d = segs[i];
            uint32_t src, dst;
            memcpy(&src, d.src, 4);
            memcpy(&dst, d.dst, 4);
            // memory-order words of src, dst, {0, proto}, htons((u16)len)
            uint64_t q = (src & 0xFFFFu) + (src >> 16) + (dst & 0xFFFFu) + (dst >> 16) + ((uint32_t)d.protocol << 8) +
                         (((d.len & 0xFFu) << 8) | ((d.len >> 8) & 0xFFu));
            while (q >> 16)
                q = (q & 0xFFFFu) + (q >> 16);
            hseg[i].offset = d.offset;
            hseg[i].len = d.len;
            hseg[i].pre_sum = (uint32_t)q;
        }
    });
    if (first_copy.valid())
        if (const hipError_t e = first_copy.get(); e != hipSuccess)
            return fail_sys(3, e);
    if (const hipError_t e = hipMemcpyAsync(c.d_descs, hseg, sizeof(tcsum_seg_t) * n, hipMemcpyHostToDevice, cs);
        e != hipSuccess)
        return fail_sys(4, e);
    stamp("descs staged");
    for (size_t k = 0; k < ch.size(); ++k) {
        if (const hipError_t e = k ? copy_span(ch[k].buf, ch[k].sp) : hipSuccess; e != hipSuccess)
            return fail_sys(5, e);
        hipEvent_t ev = c.hev[k % kHostEvents];
        if (const hipError_t e = hipEventRecord(ev, cs); e != hipSuccess)
            return fail_sys(6, e);
        if (const hipError_t e = hipStreamWaitEvent(ks, ev, 0); e != hipSuccess)
            return fail_sys(7, e);
        const uint32_t i0 = ch[k].b0 * kSpanBlock;
        const uint32_t i1 = (uint32_t)std::min<uint64_t>(n, (uint64_t)ch[k].b1 * kSpanBlock);
        if (i1 <= i0)
            continue;
        // the host saw the order: segments out of offset order take
        // tcsum_batch's SHUFFLED route (the per-range kernel unless the
        // packed kernel's range-by-range path is the faster)
        tcsum::Geometry g = tcsum::pick_geometry(mean_of(ch[k].sp.bytes, i1 - i0));
        if (!ch[k].sp.ordered)
            tcsum::shuffled_route(g, tcsum::knob(tcsum::KNOB_PACKED));
        const hipError_t e = tcsum::launch_segments(tcsum::MODE_SEG, g, base[ch[k].buf], c.d_descs + i0, i1 - i0,
                                                    c.d_out + i0, 1u, ks);
        if (e != hipSuccess)
            return fail_sys(8, e);
    }
    if (const hipError_t e = hipMemcpyAsync(hout, c.d_out, sizeof(uint16_t) * n, hipMemcpyDeviceToHost, ks);
        e != hipSuccess)
        return fail_sys(9, e);
    stamp("all issued");
    if (const hipError_t e = hipStreamSynchronize(ks); e != hipSuccess)
        return fail_sys(10, e);
    if (const hipError_t e = hipStreamSynchronize(cs); e != hipSuccess)
        return note_sys(11, e);
    stamp("synced");
    if (hout != out)
        memcpy(out, hout, sizeof(uint16_t) * n);
    stamp("done");
    return TCSUM_OK;
}

// The plan tcsum_host_batch_peso makes for a batch, as rows of 5 u64
// (tcsum_debug.h): no device is touched.
int64_t tcsum_debug_plan_host_peso(const tcsum_peso_t *segs, uint32_t n, uint64_t arena_bytes, uint64_t *rows,
                                   uint32_t max_rows, uint64_t *buf_bytes)
{
    if (!segs || n == 0 || !buf_bytes || (max_rows && !rows))
        return TCSUM_ERR_PARAM;
    PesoPlan pl;
    if (!peso_plan_lead(pl, segs, n, arena_bytes) || !peso_plan_rest(pl, segs, arena_bytes))
        return TCSUM_ERR_PARAM;
    buf_bytes[0] = pl.early ? span_bytes(pl.lead) : 0;
    buf_bytes[1] = span_bytes(pl.rest);
    const uint64_t bases[2] = {pl.lead_base(), pl.rest_base()};
    uint32_t k = 0;
    auto row = [&](uint64_t a, uint64_t b, uint64_t c, uint64_t d, uint64_t e) {
        if (k < max_rows) {
            uint64_t *r = rows + 5ull * k;
            r[0] = a, r[1] = b, r[2] = c, r[3] = d, r[4] = e;
        }
        ++k;
    };
    for (const PesoChunk &c : pl.ch) { // in queue order: chunk k's copy, then its kernel
        uint64_t lo, hi;
        span_copy(c.sp, arena_bytes, lo, hi);
        if (hi > lo) // copy: buffer, host [lo, hi), buffer offset of lo
            row(0, (uint64_t)c.buf, lo, hi, lo - bases[c.buf]);
        const uint32_t i0 = c.b0 * kSpanBlock, i1 = (uint32_t)std::min<uint64_t>(n, (uint64_t)c.b1 * kSpanBlock);
        if (i1 > i0) // kernel (2: the segments are out of offset order), buffer, segments [i0, i1), arena base
            row(c.sp.ordered ? 1 : 2, (uint64_t)c.buf, i0, i1, bases[c.buf]);
    }
    return (int64_t)k;
}

extern "C++" {
// Contiguous shards of a descriptor array balanced by bytes:
// shard d is [cut[d], cut[d+1]).
// Shard k starts after the first segment whose inclusive byte prefix reaches
// quantile k.  Block sums in parallel first (a serial pass over 8M
// descriptors would hold every device's copies back by milliseconds), then
// each cut is found inside the one block where the prefix crosses it.
template <class D>
std::vector<uint32_t> byte_shards(const D *descs, uint32_t n, int ndev)
{
    constexpr uint32_t kB = 1u << 16;
    const uint32_t nb = (n + kB - 1) / kB;
    std::vector<uint64_t> pre((size_t)nb + 1, 0); // pre[b]: bytes of blocks < b
    parallel_for(nb, 1, [&](size_t b, size_t e) {
        for (size_t k = b; k < e; ++k) {
            uint64_t t = 0;
            const uint32_t i1 = (uint32_t)std::min<uint64_t>(n, (k + 1) * (uint64_t)kB);
            for (uint32_t i = (uint32_t)k * kB; i < i1; ++i)
                t += descs[i].len;
            pre[k + 1] = t;
        }
    });
    for (uint32_t b = 0; b < nb; ++b)
        pre[b + 1] += pre[b];
    const uint64_t total = pre[nb];
    std::vector<uint32_t> cut((size_t)ndev + 1, n);
    cut[0] = 0;
    uint32_t b = 0;
    for (int k = 1; k < ndev; ++k) {
        auto reached = [&](uint64_t acc) { return acc * (uint64_t)ndev >= total * (uint64_t)k; };
        while (b < nb && !reached(pre[b + 1])) // the first block whose end reaches quantile k
            ++b;
        if (b == nb)
            break; // never reached: this and every later shard start at n
        uint64_t acc = pre[b];
        const uint32_t i0 = std::max<uint32_t>(b * kB, k > 1 ? cut[k - 1] - 1 : 0u);
        for (uint32_t i = b * kB; i < i0; ++i)
            acc += descs[i].len;
        for (uint32_t i = i0;; ++i) {
            acc += descs[i].len;
            if (reached(acc)) {
                cut[k] = i + 1;
                break;
            }
        }
    }
    return cut;
}

// Per shard of the last multi-device host batch (tcsum_debug_shards): which
// device took which descriptors, how many bytes, its return code and its
// wall time -- so a slow host link or GPU shows on its own.
std::mutex g_shards_mu;
std::vector<tcsum_shard_stat_t> g_shards;

// Run `one(device, i0, i1)` on contiguous shards of descs[0, n) balanced by
// bytes, one host thread per entry of devices[] (the calling thread when
// there is one), and record every shard.  Returns the first failing shard's
// code.
template <class D, class F>
int run_shards(const int *devices, int ndev, const D *descs, uint32_t n, F &&one)
{
    const std::vector<uint32_t> cut = ndev > 1 ? byte_shards(descs, n, ndev) : std::vector<uint32_t>{0u, n};
    std::vector<tcsum_shard_stat_t> st((size_t)ndev);
    auto shard = [&](int d) {
        tcsum_shard_stat_t &s = st[d];
        const auto t0 = std::chrono::steady_clock::now();
        if (s.count)
            s.rc = one(devices[d], cut[d], cut[d + 1]);
        s.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        for (uint32_t i = cut[d]; i < cut[d + 1]; ++i)
            s.bytes += descs[i].len;
    };
    for (int d = 0; d < ndev; ++d)
        st[d] = tcsum_shard_stat_t{devices[d], TCSUM_OK, cut[d], cut[d + 1] - cut[d], 0u, 0.0};
    if (ndev == 1) {
        shard(0);
    } else {
        std::vector<std::thread> th;
        for (int d = 0; d < ndev; ++d)
            if (cut[d + 1] > cut[d])
                th.emplace_back([&shard, d] { shard(d); });
        for (auto &t : th)
            t.join();
    }
    {
        std::lock_guard<std::mutex> lk(g_shards_mu);
        g_shards = st;
    }
    for (const auto &s : st)
        if (s.rc != TCSUM_OK)
            return s.rc;
    return TCSUM_OK;
}

}

// One host batch over several GPUs: contiguous shards balanced by bytes
// (SURVEY §8(e)), one host thread per device, each shard through its own
// device's host link and HBM; no collective.
int tcsum_host_batch_peso_multi(const int *devices, int ndev, const void *host_arena, uint64_t arena_bytes,
                                const tcsum_peso_t *segs, uint32_t n, uint16_t *out)
{
    if (n == 0)
        return TCSUM_OK;
    if (!devices || ndev <= 0 || ndev > kMaxDev || !host_arena || !segs || !out)
        return TCSUM_ERR_PARAM;
    for (int d = 0; d < ndev; ++d)
        if (devices[d] < 0 || devices[d] >= kMaxDev)
            return TCSUM_ERR_PARAM;
    return run_shards(devices, ndev, segs, n, [&](int dev, uint32_t i0, uint32_t i1) {
        return tcsum_host_batch_peso(dev, host_arena, arena_bytes, segs + i0, i1 - i0, out + i0);
    });
}

int tcsum_debug_shards(tcsum_shard_stat_t *out, int max)
{
    std::lock_guard<std::mutex> lk(g_shards_mu);
    const int k = (int)g_shards.size();
    for (int i = 0; i < k && i < max && out; ++i)
        out[i] = g_shards[i];
    return k;
}

// ------------------------------------------------------ host-queue batches

namespace {

// Device-side address of host memory the kernel may read/write in place
// (pinned by hipHostMalloc / hipHostRegister), or nullptr for pageable memory.
uint8_t *mapped_host(const void *p)
{
    hipPointerAttribute_t a{};
    if (tcsum::quiet(hipPointerGetAttributes(&a, p)) != hipSuccess) // unknown to the runtime: pageable
        return nullptr;
    if (a.type != hipMemoryTypeHost)
        return nullptr;
    void *d = nullptr;
    if (tcsum::quiet(hipHostGetDevicePointer(&d, const_cast<void *>(p), 0)) != hipSuccess)
        return nullptr;
    return static_cast<uint8_t *>(d);
}

// Host worker threads, started on first use and kept for the life of the
// process (never joined: nothing waits on them at exit).  parallel_for on
// freshly created std::threads paid ~35 us per thread: the span pass of a
// 1M-segment host batch took 635 us, most of it thread creation, before its
// first byte could be copied (profiles/r02/e2e_phase.txt).  Callers from
// several threads at once (the *_multi batches) share the pool; a caller
// runs its own job's tasks too until none is left unclaimed, so a job always
// completes even when every worker is busy (or absent, after a fork).
struct PoolJob {
    std::function<void(size_t)> fn;
    size_t k = 0;
    std::atomic<size_t> next{0}; // next task index to claim
    size_t left = 0;             // tasks not finished (under mu)
    std::mutex mu;
    std::condition_variable cv;
    // run claimed task i and count it done
    void finish(size_t i)
    {
        fn(i);
        std::lock_guard<std::mutex> l(mu); // the owner can only see 0 once this is released
        if (--left == 0)
            cv.notify_all();
    }
    // claim and run one task; false when every task is claimed
    bool run_one()
    {
        const size_t i = next.fetch_add(1);
        if (i >= k)
            return false;
        finish(i);
        return true;
    }
};

class HostPool {
  public:
    explicit HostPool(unsigned workers)
    {
        for (unsigned i = 0; i < workers; ++i)
            std::thread([this] { loop(); }).detach();
    }
    void submit(PoolJob *j)
    {
        {
            std::lock_guard<std::mutex> l(mu_);
            q_.push_back(j);
        }
        cv_.notify_all();
    }
    void retire(PoolJob *j) // the owner's job is done: drop it if still queued
    {
        std::lock_guard<std::mutex> l(mu_);
        q_.erase(std::remove(q_.begin(), q_.end(), j), q_.end());
    }

  private:
    void loop()
    {
        for (;;) {
            PoolJob *j = nullptr;
            size_t i = 0;
            {
                std::unique_lock<std::mutex> l(mu_);
                for (;;) {
                    cv_.wait(l, [&] { return !q_.empty(); });
                    j = q_.front();
                    // claim under the queue lock: the task is then counted in
                    // the job's `left`, so its owner (which retires the job
                    // under this lock, after `left` reaches 0) keeps it alive
                    i = j->next.fetch_add(1);
                    if (i < j->k)
                        break;
                    q_.pop_front();
                }
            }
            j->finish(i);
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<PoolJob *> q_;
};

extern "C++" {
// Host threads a parallel pass may use: 16 (the box's CPU share; debug knob
// copy_threads), at most the machine's.
unsigned host_threads()
{
    static const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int64_t k = tcsum::knob(tcsum::KNOB_COPY_THREADS);
    const unsigned v = k > 0 ? (unsigned)std::min<int64_t>(k, 4096) : 16u;
    return std::max(1u, std::min(hw, v));
}

// The one pool of the process (every parallel_for instantiation shares it).
HostPool &host_pool()
{
    static HostPool *pool = new HostPool(host_threads() - 1); // kept: see HostPool
    return *pool;
}
}

// f(begin, end) over [0, n) split across host threads, at least `min_per`
// items each (one core moves ~10-20 GB/s through memcpy; the PCIe link takes
// ~55).
extern "C++" {
template <class F>
void parallel_for(size_t n, size_t min_per, F &&f)
{
    const unsigned cap = host_threads();
    size_t k = std::min<size_t>(cap, min_per ? n / min_per : cap);
    if (k <= 1) {
        f(size_t(0), n);
        return;
    }
    HostPool *pool = &host_pool();
    const size_t per = (n + k - 1) / k;
    PoolJob job;
    job.fn = [&f, n, per](size_t i) {
        const size_t b = std::min(n, i * per), e = std::min(n, b + per);
        if (e > b)
            f(b, e);
    };
    job.k = k;
    job.left = k;
    pool->submit(&job);
    while (job.run_one()) {
    }
    {
        std::unique_lock<std::mutex> l(job.mu);
        job.cv.wait(l, [&] { return job.left == 0; });
    }
    pool->retire(&job);
}
}

void par_memcpy(uint8_t *dst, const uint8_t *src, size_t n)
{
    parallel_for(n, size_t(8) << 20, [=](size_t b, size_t e) { memcpy(dst + b, src + b, e - b); });
}

// The bytes of a packet a tx fill may write: the IPv4 header checksum at
// 10..11 and the L4 checksum at hl + fld .. +1 with hl <= 60 (IHL <= 15) and
// fld <= 16 (tcp.h:71): all below byte 78 of the packet.
constexpr uint64_t kTxWindow = 78;

// ---- queue server (k_server, csum_kernels.hip) ----

// a debug knob's value, or the default while it is unset (-1)
int knob_or(tcsum::Knob k, int dflt)
{
    const int64_t v = tcsum::knob(k);
    return v >= 0 ? (int)v : dflt;
}

// Largest host-queue batch handed to the server (bigger ones are bandwidth
// work: a launch per batch costs nothing there).
uint32_t srv_max_packets() { return (uint32_t)knob_or(tcsum::KNOB_SERVER_MAX, 65536); }

int srv_setup(Ctx &c)
{
    if (c.srv_h)
        return TCSUM_OK;
    hipError_t e;
    if (!c.srv_stream && (e = hipStreamCreateWithFlags(&c.srv_stream, hipStreamNonBlocking)) != hipSuccess) {
        c.srv_stream = nullptr;
        return note_sys(40, e);
    }
    if ((e = hipHostMalloc(reinterpret_cast<void **>(&c.srv_h), sizeof(tcsum::SrvHost), hipHostMallocCoherent)) !=
            hipSuccess ||
        (e = hipHostGetDevicePointer(reinterpret_cast<void **>(&c.srv_hd), c.srv_h, 0)) != hipSuccess ||
        (e = hipMalloc(reinterpret_cast<void **>(&c.srv_d), sizeof(tcsum::SrvCtl))) != hipSuccess) {
        c.srv_h = nullptr;
        return note_mem(41, e);
    }
    memset(c.srv_h, 0, sizeof(tcsum::SrvHost));
    if (knob_or(tcsum::KNOB_SERVER_TRACE, 0)) { // phase stamps, printed by srv_stop (measurement only)
        uint64_t *t = nullptr, *td = nullptr;
        if (hipHostMalloc(reinterpret_cast<void **>(&t), 256 * 8 * sizeof(uint64_t), hipHostMallocCoherent) ==
                hipSuccess &&
            hipHostGetDevicePointer(reinterpret_cast<void **>(&td), t, 0) == hipSuccess) {
            memset(t, 0, 256 * 8 * sizeof(uint64_t));
            c.srv_trace = t;
            c.srv_h->trace = reinterpret_cast<uint64_t>(td);
        }
    }
    return TCSUM_OK;
}

// Mean phase durations over the traced jobs (debug knob "server_trace" = 1), in us.
void srv_print_trace(const Ctx &c)
{
    const uint64_t *t = c.srv_trace;
    if (!t)
        return;
    static const char *names[6] = {"seen->bcast", "bcast->wg1 seen", "bcast->wg0 summed", "wg0 release fence",
                                   "wg0 release->last arrival", "last arrival->done stored"};
    const int from[6] = {0, 1, 1, 3, 4, 5}, to[6] = {1, 2, 3, 4, 5, 6};
    double sum[6] = {0};
    int cnt[6] = {0};
    for (int j = 0; j < 256; ++j)
        for (int k = 0; k < 6; ++k) {
            const uint64_t a = t[j * 8 + from[k]], b = t[j * 8 + to[k]];
            if (a && b && b >= a && b - a < 100000000ull) {
                sum[k] += (double)(b - a) / 100.0;
                ++cnt[k];
            }
        }
    for (int k = 0; k < 6; ++k)
        if (cnt[k])
            fprintf(stderr, "tcsum server trace: %-28s %8.2f us (%d jobs)\n", names[k], sum[k] / cnt[k], cnt[k]);
}

void reap_at_exit();

int srv_launch(Ctx &c, uint32_t last)
{
    reap_at_exit();
    const uint64_t idle_ticks = 100000ull * (uint64_t)std::max(1, knob_or(tcsum::KNOB_SERVER_IDLE_MS, 10)); // 100 MHz
    if (const hipError_t e = tcsum::launch_server(c.srv_hd, c.srv_d, last, idle_ticks,
                                                  std::max(1, knob_or(tcsum::KNOB_SERVER_WGS, 64)), c.srv_stream);
        e != hipSuccess)
        return note_sys(42, e);
    c.srv_running = true;
    return TCSUM_OK;
}

// Ask the grid to leave and wait (bounded) until its stream is idle.
int srv_stop(Ctx &c)
{
    if (!c.srv_h)
        return TCSUM_OK;
    __atomic_store_n(&c.srv_h->quit, 1u, __ATOMIC_SEQ_CST);
    int rc = TCSUM_OK;
    if (c.srv_running) {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t q = poll_stream(c.srv_stream);
            if (q == hipSuccess)
                break;
            if (q != hipErrorNotReady || std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
                rc = note_sys(43, q);
                break;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
        if (rc == TCSUM_OK)
            c.srv_running = false;
    }
    if (rc == TCSUM_OK)
        __atomic_store_n(&c.srv_h->quit, 0u, __ATOMIC_SEQ_CST);
    srv_print_trace(c);
    return rc;
}

// Post one job and wait for it.  A grid that left (idle, or a job posted
// while it was leaving) is relaunched; it serves any job with req != last.
int srv_submit(Ctx &c, int op, uint8_t *d_arena, const tcsum_pkt_t *d_pkts, uint32_t n, uint32_t *d_out,
               uint8_t *d_flags, int8_t *d_verdict)
{
    int rc = srv_setup(c);
    if (rc != TCSUM_OK)
        return rc;
    tcsum::SrvHost *h = c.srv_h;
    const uint32_t prev = c.srv_seq;
    const uint32_t seq = prev + 1u ? prev + 1u : 1u; // never 0
    h->op = (uint32_t)op;
    h->n = n;
    h->ptr[0] = reinterpret_cast<uint64_t>(d_arena);
    h->ptr[1] = reinterpret_cast<uint64_t>(d_pkts);
    h->ptr[2] = reinterpret_cast<uint64_t>(d_out);
    h->ptr[3] = reinterpret_cast<uint64_t>(d_flags);
    h->ptr[4] = reinterpret_cast<uint64_t>(d_verdict);
    __atomic_store_n(&h->req, seq, __ATOMIC_SEQ_CST); // after the job fields
    c.srv_seq = seq;
    if (!c.srv_running && (rc = srv_launch(c, prev)) != TCSUM_OK)
        return rc;
    // spin on `done`; only every 100 us ask the runtime whether the grid left
    // (a hipStreamQuery in the spin loop itself delays noticing `done`)
    const auto t0 = std::chrono::steady_clock::now();
    auto check = t0 + std::chrono::microseconds(100);
    for (unsigned spins = 1;; ++spins) {
        if (__atomic_load_n(&h->done, __ATOMIC_ACQUIRE) == seq)
            return TCSUM_OK;
        if ((spins & 1023u) == 0) {
            const auto now = std::chrono::steady_clock::now();
            if (now >= check) {
                if (c.srv_running) {
                    const hipError_t q = poll_stream(c.srv_stream);
                    if (q == hipSuccess)
                        c.srv_running = false;
                    else if (q != hipErrorNotReady)
                        return note_sys(44, q);
                }
                if (!c.srv_running) {
                    if (__atomic_load_n(&h->done, __ATOMIC_ACQUIRE) == seq)
                        return TCSUM_OK;
                    if ((rc = srv_launch(c, prev)) != TCSUM_OK)
                        return rc;
                }
                if (now - t0 > std::chrono::seconds(10))
                    return note_err(45, hipErrorLaunchTimeOut, TCSUM_ERR_SYS, false); // the library's own time-out
                check = now + std::chrono::microseconds(100);
            }
        }
        __builtin_ia32_pause();
    }
}

// ---- call server (k_call, csum_kernels.hip) ----

int cs_setup(Ctx &c)
{
    if (c.cs_h)
        return TCSUM_OK;
    hipError_t e;
    if (!c.cs_stream && (e = hipStreamCreateWithFlags(&c.cs_stream, hipStreamNonBlocking)) != hipSuccess) {
        c.cs_stream = nullptr;
        return note_sys(49, e);
    }
    tcsum::CallBox *h = nullptr, *hd = nullptr;
    uint8_t *st = nullptr, *std_ = nullptr;
    if ((e = hipHostMalloc(reinterpret_cast<void **>(&h), sizeof(tcsum::CallBox), hipHostMallocCoherent)) !=
            hipSuccess ||
        (e = hipHostGetDevicePointer(reinterpret_cast<void **>(&hd), h, 0)) != hipSuccess ||
        (e = hipHostMalloc(reinterpret_cast<void **>(&st), kCallStageMax + 64, hipHostMallocCoherent)) !=
            hipSuccess ||
        (e = hipHostGetDevicePointer(reinterpret_cast<void **>(&std_), st, 0)) != hipSuccess)
        return note_mem(49, e);
    memset(h, 0, sizeof(tcsum::CallBox));
    memset(st, 0, kCallStageMax + 64);
    c.cs_stage = st;
    c.cs_stage_d = std_;
    c.cs_hd = hd;
    c.cs_h = h;
    return TCSUM_OK;
}

void cs_launch(Ctx &c, uint32_t last)
{
    reap_at_exit();
    const uint64_t idle_ticks = 100000ull * (uint64_t)std::max(1, knob_or(tcsum::KNOB_SERVER_IDLE_MS, 10)); // 100 MHz
    const hipError_t e = tcsum::launch_call_server(c.cs_hd, c.cs_stage_d, last, idle_ticks, c.cs_stream);
    if (e != hipSuccess)
        die("call server launch", e);
    c.cs_running = true;
}

// Post one job (its bytes already in cs_stage) and spin until the wave has
// answered; a wave that left (idle, or leaving while the job was posted) is
// relaunched and serves the job (it takes any seq != last).
// `small`: the call's bytes (len + parity <= kCallInline) travel in the job
// line itself instead of cs_stage -- one PCIe round trip less for the
// 20-byte IPv4 header checks (ipv4.c:243, 656).
uint32_t cs_post(Ctx &c, uint32_t ctl, uint32_t len, uint32_t pre, uint32_t src, uint32_t dst, uint32_t proto,
                 const uint8_t *small = nullptr)
{
    tcsum::CallBox *h = c.cs_h;
    const uint32_t prev = c.cs_seq;
    const uint32_t seq = prev + 1u ? prev + 1u : 1u; // never 0
    if (small) {
        uint8_t b[tcsum::kCallInline] = {};
        if (len)
            memcpy(b + ((ctl & tcsum::CALL_ODD) ? 1 : 0), small, len);
        memcpy(h->w2, b, 12);
        memcpy(h->w3, b + 12, 12);
        ctl |= tcsum::CALL_INLINE;
    }
    h->w0[1] = ctl;
    h->w0[2] = len;
    h->w0[3] = pre;
    h->w1[0] = src;
    h->w1[1] = dst;
    h->w1[2] = proto;
    __atomic_thread_fence(__ATOMIC_SEQ_CST); // the staged bytes and fields before the sequence words
    __atomic_store_n(&h->w3[3], seq, __ATOMIC_RELEASE);
    __atomic_store_n(&h->w2[3], seq, __ATOMIC_RELEASE);
    __atomic_store_n(&h->w1[3], seq, __ATOMIC_RELEASE);
    __atomic_store_n(&h->w0[0], seq, __ATOMIC_RELEASE);
    c.cs_seq = seq;
    if (!c.cs_running)
        cs_launch(c, prev);
    const auto t0 = std::chrono::steady_clock::now();
    auto check = t0 + std::chrono::microseconds(100);
    for (unsigned spins = 1;; ++spins) {
        const uint64_t r = __atomic_load_n(&h->res, __ATOMIC_ACQUIRE);
        if ((uint32_t)r == seq)
            return (uint32_t)(r >> 32);
        if ((spins & 1023u) == 0) {
            const auto now = std::chrono::steady_clock::now();
            if (now >= check) {
                if (c.cs_running) {
                    const hipError_t q = poll_stream(c.cs_stream);
                    if (q == hipSuccess)
                        c.cs_running = false;
                    else if (q != hipErrorNotReady)
                        die("call server", q);
                }
                if (!c.cs_running && (uint32_t)__atomic_load_n(&h->res, __ATOMIC_ACQUIRE) != seq)
                    cs_launch(c, prev);
                if (now - t0 > std::chrono::seconds(10))
                    die("call server (no answer in 10 s)", hipErrorLaunchTimeOut);
                check = now + std::chrono::microseconds(100);
            }
        }
        __builtin_ia32_pause();
    }
}

// Ask the wave to leave and wait (bounded) until its stream is idle.
int cs_stop(Ctx &c)
{
    if (!c.cs_h || !c.cs_running)
        return TCSUM_OK;
    tcsum::CallBox *h = c.cs_h;
    const uint32_t seq = c.cs_seq + 1u ? c.cs_seq + 1u : 1u;
    h->w0[1] = tcsum::CALL_QUIT;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    __atomic_store_n(&h->w3[3], seq, __ATOMIC_RELEASE);
    __atomic_store_n(&h->w2[3], seq, __ATOMIC_RELEASE);
    __atomic_store_n(&h->w1[3], seq, __ATOMIC_RELEASE);
    __atomic_store_n(&h->w0[0], seq, __ATOMIC_RELEASE);
    c.cs_seq = seq;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = poll_stream(c.cs_stream);
        if (q == hipSuccess)
            break;
        if (q != hipErrorNotReady || std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5))
            return note_sys(46, q);
        std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    c.cs_running = false;
    return TCSUM_OK;
}

// At exit: ask every live server grid / wave to leave (bounded wait) while
// the HIP runtime is still up -- registered with atexit at the first server
// launch, i.e. after the runtime's own initialisation, so it runs before the
// runtime's teardown; the static destructor below is the fallback for a
// dlclose'd library.
void reap_servers()
{
    for (auto &c : g_ctx) {
        if (c.srv_running)
            (void)srv_stop(c);
        if (c.cs_running)
            (void)cs_stop(c);
    }
}
struct SrvReaper {
    ~SrvReaper() { reap_servers(); }
} g_srv_reaper;
std::once_flag g_reap_once;
void reap_at_exit() { std::call_once(g_reap_once, [] { atexit(reap_servers); }); }

// Give back every cached batch buffer of a device (tcsum_release): the HBM
// copy of host spans and descriptors, and the pinned host-queue staging.  The
// servers go first: their next job would name the freed buffers.
// The calling thread's current device is restored on return (release may
// run on a thread that works on another device).
struct KeepDevice {
    int dev = -1;
    KeepDevice()
    {
        if (tcsum::quiet(hipGetDevice(&dev)) != hipSuccess)
            dev = -1;
    }
    ~KeepDevice()
    {
        if (dev >= 0)
            (void)tcsum::quiet(hipSetDevice(dev));
    }
};

int release_ctx(Ctx &c, int dev)
{
    std::lock_guard<std::mutex> lk(c.mu);
    const KeepDevice keep;
    if (!c.ready) {
        // no context (only device-resident batch calls on caller streams ran
        // here): the tx fill's scratch pool may still hold memory.  Its
        // blocks are stream-ordered: the device is synchronized (tcsum.h)
        if (!tcsum::scratch_reserved(dev))
            return TCSUM_OK;
        hipError_t e = hipSetDevice(dev);
        if (e == hipSuccess)
            e = hipDeviceSynchronize();
        if (e == hipSuccess)
            e = tcsum::scratch_trim(dev);
        return e == hipSuccess ? TCSUM_OK : note_sys(50, e);
    }
    if (const hipError_t e = hipSetDevice(c.device); e != hipSuccess)
        return note_sys(51, e);
    if ((c.srv_running && srv_stop(c) != TCSUM_OK) || (c.cs_running && cs_stop(c) != TCSUM_OK))
        return TCSUM_ERR_SYS;
    // a stream that does not drain (a faulted device) is the caller's to
    // know: nothing is freed under work that may still be reading it
    for (hipStream_t st : c.hs)
        if (st)
            if (const hipError_t e = hipStreamSynchronize(st); e != hipSuccess)
                return note_sys(53, e);
    if (const hipError_t e = hipStreamSynchronize(c.stream); e != hipSuccess)
        return note_sys(53, e);
    for (void *p : {(void *)c.d_arena, (void *)c.d_lead, (void *)c.d_descs, (void *)c.d_out})
        if (p)
            (void)tcsum::quiet(hipFree(p));
    c.d_arena = nullptr;
    c.d_lead = nullptr;
    c.d_lead_cap = 0;
    c.d_descs = nullptr;
    c.d_out = nullptr;
    c.d_arena_cap = c.d_descs_cap = c.d_out_cap = 0;
    for (Pinned *q : {&c.q_desc, &c.q_res, &c.q_arena, &c.q_page[0], &c.q_page[1], &c.q_page[2]}) {
        if (q->h)
            (void)tcsum::quiet(hipHostFree(q->h));
        q->h = q->d = nullptr;
        q->cap = 0;
    }
    // the tx fill's pooled scratch (every stream of this context is idle;
    // a caller's own stream on this device must be too, tcsum.h)
    if (const hipError_t e = hipDeviceSynchronize(); e != hipSuccess)
        return note_sys(54, e);
    if (const hipError_t e = tcsum::scratch_trim(c.device); e != hipSuccess)
        return note_sys(52, e);
    return TCSUM_OK;
}

// IPv4 batch over packets in host memory (the stack's netif queues): pinned
// arenas are read -- and for tx written -- in place by the kernel over PCIe;
// a pageable arena is first copied into pinned staging (and copied back after
// a tx fill).  Descriptors and results travel through pinned staging too.
int host_ipv4(int ip_mode, int device, uint8_t *host_arena, uint64_t arena_bytes, const tcsum_pkt_t *pkts,
              uint32_t n, int8_t *verdict, uint32_t *out, uint8_t *flags)
{
    if (n == 0)
        return TCSUM_OK;
    if (!host_arena || !pkts || device < 0 || device >= kMaxDev || (ip_mode == 2 && !verdict))
        return TCSUM_ERR_PARAM;
    // one pass over the descriptors (in parallel for large queues: a serial
    // pass over 1M descriptors kept the link idle for milliseconds): validity,
    // the byte span [lo, hi), the bytes, and whether the non-empty packets are
    // in offset order
    struct QSpan {
        uint64_t lo = UINT64_MAX, hi = 0, total = 0, first = UINT64_MAX, last = 0;
        bool bad = false, ordered = true;
    };
    constexpr uint32_t kQBlock = 4096;
    const uint32_t nqb = (n + kQBlock - 1) / kQBlock;
    std::vector<QSpan> qb(nqb);
    parallel_for(nqb, 16, [&](size_t b, size_t e) {
        for (size_t k = b; k < e; ++k) {
            QSpan q;
            const uint32_t i1 = (uint32_t)std::min<uint64_t>(n, (k + 1) * (uint64_t)kQBlock);
            for (uint32_t i = (uint32_t)k * kQBlock; i < i1; ++i) {
                const uint64_t o = pkts[i].offset, l = pkts[i].len;
                q.bad |= o > arena_bytes || l > arena_bytes - o;
                if (l == 0)
                    continue;
                q.lo = o < q.lo ? o : q.lo;
                q.hi = o + l > q.hi ? o + l : q.hi;
                q.total += l;
                q.ordered &= q.first == UINT64_MAX || o >= q.last;
                q.first = q.first == UINT64_MAX ? o : q.first;
                q.last = o;
            }
            qb[k] = q;
        }
    });
    uint64_t lo = UINT64_MAX, hi = 0, total = 0, prev_last = 0;
    bool any = false, in_order = true;
    for (const QSpan &q : qb) {
        if (q.bad)
            return TCSUM_ERR_PARAM;
        lo = q.lo < lo ? q.lo : lo;
        hi = q.hi > hi ? q.hi : hi;
        total += q.total;
        if (q.first != UINT64_MAX) {
            in_order = in_order && q.ordered && (!any || q.first >= prev_last);
            prev_last = q.last;
            any = true;
        }
    }
    Ctx &c = g_ctx[device];
    std::lock_guard<std::mutex> lk(c.mu);
    int rc = ctx_init(c, device); // a failing HIP call is recorded there (steps 20-25)
    if (rc != TCSUM_OK)
        return rc;
    if (const hipError_t se = hipSetDevice(device); se != hipSuccess)
        return note_sys(31, se);

    uint8_t *d_arena = mapped_host(host_arena);
    const bool staged = d_arena == nullptr;
    constexpr uint64_t kPad = 16; // aligned over-reads around [lo, hi) stay inside the staging buffer
    if (staged) {
        if (hi <= lo)
            lo = hi = 0;
        if (const hipError_t me = c.q_arena.reserve(hi - lo + 2 * kPad); me != hipSuccess)
            return note_mem(32, me);
        d_arena = reinterpret_cast<uint8_t *>(reinterpret_cast<uintptr_t>(c.q_arena.d) + kPad - lo);
    }
    if (const hipError_t me = c.q_desc.reserve(sizeof(tcsum_pkt_t) * n); me != hipSuccess)
        return note_mem(33, me);
    if (const hipError_t me = c.q_res.reserve(6ull * n + 64); me != hipSuccess)
        return note_mem(33, me);
    par_memcpy(c.q_desc.h, reinterpret_cast<const uint8_t *>(pkts), sizeof(tcsum_pkt_t) * n);
    // results: out u32[n] | flags u8[n] | verdict i8[n]
    uint32_t *d_out = out ? reinterpret_cast<uint32_t *>(c.q_res.d) : nullptr;
    uint8_t *d_flags = flags ? c.q_res.d + 4ull * n : nullptr;
    int8_t *d_verdict = verdict ? reinterpret_cast<int8_t *>(c.q_res.d + 5ull * n) : nullptr;
    const tcsum_pkt_t *d_pkts = reinterpret_cast<const tcsum_pkt_t *>(c.q_desc.d);
    auto launch = [&](uint32_t i0, uint32_t i1, uint64_t bytes) {
        return tcsum::launch_ipv4(ip_mode, tcsum::pick_geometry(mean_of(bytes, i1 - i0)), d_arena, d_pkts + i0,
                                  i1 - i0, d_out ? d_out + i0 : nullptr, d_flags ? d_flags + i0 : nullptr,
                                  d_verdict ? d_verdict + i0 : nullptr, c.stream);
    };
    hipError_t e = hipSuccess;
    uint8_t *const st = c.q_arena.h + kPad; // staging byte of arena offset x: st[x - lo]
    if (c.srv_on && n <= srv_max_packets()) { // small queue: the resident grid, no launch
        if (staged)
            par_memcpy(st, host_arena + lo, hi - lo);
        rc = srv_submit(c, ip_mode, d_arena, d_pkts, n, d_out, d_flags, d_verdict);
        if (rc != TCSUM_OK)
            return rc;
        goto results;
    }
    {
    // Large pinned batches go through the copy engine instead of the kernel's
    // own PCIe reads: pieces copied in order on
    // one copy stream into HBM, each piece's kernel behind its copy's event
    // (tcsum_host_batch_peso's pipeline): 50.7 against 49.3 GiB/s for 1M
    // mixed frames (profiles/r01/hostq_dma.txt).  Debug knob "hostq_dma_kb": the
    // span from which it is used (0 = never).  Only for DENSE batches -- the
    // packets cover at least 3/4 of their span: a few frames spread over a big
    // pinned pool would otherwise move gigabytes to sum kilobytes, where the
    // in-place path reads only the packets' own bytes.
    // A pageable batch takes the same path, each piece staged into
    // pinned memory by the host threads just before its copy (the staging of
    // piece k+1 overlaps the copy of piece k) instead of being read in place
    // from the staging by the kernel.
    const uint64_t dma_min = (uint64_t)knob_or(tcsum::KNOB_HOSTQ_DMA_KB, 256 << 10) << 10;
    const uint64_t alo = lo & ~uint64_t(15), ahi = std::min<uint64_t>(arena_bytes, (hi + 15) & ~uint64_t(15));
    // A tx fill takes it too: the packets are read from the HBM copy and the
    // fields stored straight into the frames in host memory (or the staging)
    // by k_tx_scatter, over PCIe as posted writes.
    // A pinned tx fill only from 4x that span: its last piece's field stores
    // trail the copies, and at 298 MB the in-place fill was 3.6 % faster
    // (4.7 GB: 3.3 % slower; profiles/r02/hostq_ab_pieces.txt).
    bool dma = in_order && dma_min && hi > lo && hi - lo >= dma_min && total * 4 >= (hi - lo) * 3 &&
               (ip_mode != 1 || staged || hi - lo >= 4 * dma_min);
    if (dma && (size_t)(ahi - alo) + 32 > c.d_arena_cap) {
        // no room in HBM for the span: the in-place path below needs none
        if (c.d_arena)
            (void)tcsum::quiet(hipFree(c.d_arena));
        c.d_arena = nullptr;
        c.d_arena_cap = 0;
        if (tcsum::quiet(hipMalloc(reinterpret_cast<void **>(&c.d_arena), (size_t)(ahi - alo) + 32)) == hipSuccess) {
            c.d_arena_cap = (size_t)(ahi - alo) + 32;
        } else {
            c.d_arena = nullptr;
            dma = false; // not an error: the in-place path needs no HBM copy
        }
    }
    if (dma) {
        uint8_t *const dbase = c.d_arena + 16 - alo;
        hipStream_t cs = c.hs[0], ks = c.hs[1];
        // Pinned: pieces growing from 64 MiB to a quarter of the span (an
        // eighth for tx, whose last piece's field stores trail the copies):
        // every copy costs ~18 us of idle link before it
        // (tcsum_host_batch_peso).  Pageable: the host's staging copy is the
        // slower side, so pieces stay small (1/16 of the span, 32..128 MiB)
        // and the link waits for little more than the first one.
        const uint64_t span = hi - lo;
        const uint64_t kPieceMax =
            staged ? std::min<uint64_t>(128ull << 20, std::max<uint64_t>(32ull << 20, span / 16))
                   : std::max<uint64_t>(64ull << 20, span / (ip_mode == 1 ? 8 : 4));
        uint64_t piece = std::min<uint64_t>(64ull << 20, kPieceMax);
        // host address of arena offset x: `src + x` (the staging when pageable;
        // it covers [lo - kPad, hi + kPad), which holds every aligned piece)
        const uintptr_t src = staged ? reinterpret_cast<uintptr_t>(st) - lo : reinterpret_cast<uintptr_t>(host_arena);
        uint64_t copied_hi = alo;
        size_t k = 0;
        for (uint32_t i0 = 0; i0 < n && e == hipSuccess; ++k, piece = std::min(kPieceMax, piece * 2)) {
            uint32_t i1 = i0;
            uint64_t bytes = 0, end = copied_hi, first = UINT64_MAX;
            while (i1 < n && (i1 == i0 || bytes < piece)) {
                if (pkts[i1].len) {
                    bytes += pkts[i1].len;
                    first = std::min<uint64_t>(first, pkts[i1].offset);
                    end = std::max<uint64_t>(end, pkts[i1].offset + pkts[i1].len);
                }
                ++i1;
            }
            end = std::min<uint64_t>(arena_bytes, (end + 15) & ~uint64_t(15));
            // this piece's own span (the 16-byte chunks its packets touch), not
            // the gap before it
            const uint64_t from = std::max<uint64_t>(copied_hi, first == UINT64_MAX ? end : first & ~uint64_t(15));
            if (end > from) {
                if (staged)
                    par_memcpy(reinterpret_cast<uint8_t *>(src + from), host_arena + from, end - from);
                e = hipMemcpyAsync(dbase + from, reinterpret_cast<const void *>(src + from), end - from,
                                   hipMemcpyHostToDevice, cs);
                copied_hi = end;
            }
            hipEvent_t ev = c.hev[k % kHostEvents];
            if (e == hipSuccess)
                e = hipEventRecord(ev, cs);
            if (e == hipSuccess)
                e = hipStreamWaitEvent(ks, ev, 0);
            const Geometry g = tcsum::pick_geometry(mean_of(bytes, i1 - i0));
            if (e == hipSuccess && ip_mode == 1) // values from HBM, fields into the frames where they live
                e = tcsum::launch_ipv4_tx_to(g, dbase, d_arena, d_pkts + i0, i1 - i0, d_out ? d_out + i0 : nullptr,
                                             d_flags ? d_flags + i0 : nullptr, ks);
            else if (e == hipSuccess)
                e = tcsum::launch_ipv4(ip_mode, g, dbase, d_pkts + i0, i1 - i0, d_out ? d_out + i0 : nullptr,
                                       d_flags ? d_flags + i0 : nullptr, d_verdict ? d_verdict + i0 : nullptr, ks);
            i0 = i1;
        }
        const hipError_t s1 = hipStreamSynchronize(ks), s2 = hipStreamSynchronize(cs);
        // the HBM copy of the span is cached for the next batch only up to
        // debug knob "hostq_dma_keep_mb" (default 256): a one-off multi-GiB verify
        // does not keep its span allocated for the life of the process
        if (c.d_arena_cap > ((size_t)knob_or(tcsum::KNOB_HOSTQ_DMA_KEEP_MB, 256) << 20)) {
            (void)tcsum::quiet(hipFree(c.d_arena));
            c.d_arena = nullptr;
            c.d_arena_cap = 0;
        }
        if (e != hipSuccess)
            return note_sys(34, e);
        if (s1 != hipSuccess || s2 != hipSuccess)
            return note_sys(35, s1 != hipSuccess ? s1 : s2);
        goto results;
    }
    if (!staged) {
        e = launch(0, n, total);
    } else if (!in_order) {
        par_memcpy(st, host_arena + lo, hi - lo);
        e = launch(0, n, total);
    } else {
        // packets in offset order: stage 1/16 of the bytes (32..256 MiB) at a time and launch
        // on each piece as soon as it is staged, so the host copy of the next
        // piece overlaps the kernel's PCIe reads of this one.  `staged_hi`: every
        // byte below it is in staging; no byte is copied twice (a tx fill may
        // already have written it).
        const uint64_t kPiece = std::min<uint64_t>(256ull << 20, std::max<uint64_t>(32ull << 20, (hi - lo) / 16));
        uint64_t staged_hi = lo;
        for (uint32_t i0 = 0; i0 < n && e == hipSuccess;) {
            uint32_t i1 = i0;
            uint64_t bytes = 0, end = staged_hi;
            while (i1 < n && (i1 == i0 || bytes < kPiece)) {
                if (pkts[i1].len) {
                    bytes += pkts[i1].len;
                    end = std::max<uint64_t>(end, pkts[i1].offset + pkts[i1].len);
                }
                ++i1;
            }
            if (end > staged_hi) {
                par_memcpy(st + (staged_hi - lo), host_arena + staged_hi, end - staged_hi);
                staged_hi = end;
            }
            e = launch(i0, i1, bytes);
            i0 = i1;
        }
    }
    // on a failed launch the pieces already launched still read the arena
    // (and the staging the next call reuses): drain them before returning
    const hipError_t se = e == hipSuccess ? stream_wait(c) : hipStreamSynchronize(c.stream);
    if (e != hipSuccess)
        return note_sys(36, e);
    if (se != hipSuccess)
        return note_sys(37, se);
    }
results:
    if (out)
        memcpy(out, c.q_res.h, 4ull * n);
    if (flags)
        memcpy(flags, c.q_res.h + 4ull * n, n);
    if (verdict)
        memcpy(verdict, c.q_res.h + 5ull * n, n);
    if (staged && ip_mode == 1) {
        // copy back only what the fill may have written: each packet's first
        // kTxWindow bytes (staging holds the final state of every byte, so
        // overlapping packets copy consistent values)
        parallel_for(n, size_t(1) << 16, [=](size_t b, size_t e) {
            for (size_t i = b; i < e; ++i) {
                const uint64_t w = pkts[i].len < kTxWindow ? pkts[i].len : kTxWindow;
                if (w)
                    memcpy(host_arena + pkts[i].offset, st + (pkts[i].offset - lo), w);
            }
        });
    }
    return TCSUM_OK;
}

} // namespace

int tcsum_host_batch_ipv4(int device, const void *host_arena, uint64_t arena_bytes, const tcsum_pkt_t *pkts,
                          uint32_t n, uint32_t *out, uint8_t *flags)
{
    if (n && !out)
        return TCSUM_ERR_PARAM;
    return host_ipv4(0, device, const_cast<uint8_t *>(static_cast<const uint8_t *>(host_arena)), arena_bytes,
                     pkts, n, nullptr, out, flags);
}

int tcsum_host_batch_ipv4_tx_fill(int device, void *host_arena, uint64_t arena_bytes, const tcsum_pkt_t *pkts,
                                  uint32_t n, uint32_t *out, uint8_t *flags)
{
    return host_ipv4(1, device, static_cast<uint8_t *>(host_arena), arena_bytes, pkts, n, nullptr, out, flags);
}

int tcsum_host_batch_ipv4_rx_verify(int device, const void *host_arena, uint64_t arena_bytes,
                                    const tcsum_pkt_t *pkts, uint32_t n, int8_t *verdict, uint32_t *out,
                                    uint8_t *flags)
{
    // the kernel never writes the arena in this mode
    return host_ipv4(2, device, const_cast<uint8_t *>(static_cast<const uint8_t *>(host_arena)), arena_bytes,
                     pkts, n, verdict, out, flags);
}

// The host-queue batches over several GPUs (tcsum_host_batch_peso_multi's
// split): each shard is an ordinary host batch on its device -- pinned
// frames read (and, tx, written) in place over that GPU's own host link,
// pageable ones staged by that device's context.
static int host_ipv4_multi(int ip_mode, const int *devices, int ndev, uint8_t *host_arena, uint64_t arena_bytes,
                           const tcsum_pkt_t *pkts, uint32_t n, int8_t *verdict, uint32_t *out, uint8_t *flags)
{
    if (n == 0)
        return TCSUM_OK;
    if (!devices || ndev <= 0 || ndev > kMaxDev || !host_arena || !pkts)
        return TCSUM_ERR_PARAM;
    for (int d = 0; d < ndev; ++d)
        if (devices[d] < 0 || devices[d] >= kMaxDev)
            return TCSUM_ERR_PARAM;
    return run_shards(devices, ndev, pkts, n, [&](int dev, uint32_t i0, uint32_t i1) {
        return host_ipv4(ip_mode, dev, host_arena, arena_bytes, pkts + i0, i1 - i0, verdict ? verdict + i0 : nullptr,
                         out ? out + i0 : nullptr, flags ? flags + i0 : nullptr);
    });
}

int tcsum_host_batch_ipv4_multi(const int *devices, int ndev, const void *host_arena, uint64_t arena_bytes,
                                const tcsum_pkt_t *pkts, uint32_t n, uint32_t *out, uint8_t *flags)
{
    if (n && !out)
        return TCSUM_ERR_PARAM;
    return host_ipv4_multi(0, devices, ndev, const_cast<uint8_t *>(static_cast<const uint8_t *>(host_arena)),
                           arena_bytes, pkts, n, nullptr, out, flags);
}

int tcsum_host_batch_ipv4_tx_fill_multi(const int *devices, int ndev, void *host_arena, uint64_t arena_bytes,
                                        const tcsum_pkt_t *pkts, uint32_t n, uint32_t *out, uint8_t *flags)
{
    return host_ipv4_multi(1, devices, ndev, static_cast<uint8_t *>(host_arena), arena_bytes, pkts, n, nullptr, out,
                           flags);
}

int tcsum_host_batch_ipv4_rx_verify_multi(const int *devices, int ndev, const void *host_arena,
                                          uint64_t arena_bytes, const tcsum_pkt_t *pkts, uint32_t n,
                                          int8_t *verdict, uint32_t *out, uint8_t *flags)
{
    if (n && !verdict)
        return TCSUM_ERR_PARAM;
    return host_ipv4_multi(2, devices, ndev, const_cast<uint8_t *>(static_cast<const uint8_t *>(host_arena)),
                           arena_bytes, pkts, n, verdict, out, flags);
}

int tcsum_queue_server(int device, int enable)
{
    if (device < 0 || device >= kMaxDev)
        return TCSUM_ERR_PARAM;
    Ctx &c = g_ctx[device];
    std::lock_guard<std::mutex> lk(c.mu);
    int rc = ctx_init(c, device);
    if (rc != TCSUM_OK)
        return rc;
    if (const hipError_t e = hipSetDevice(device); e != hipSuccess)
        return note_sys(47, e);
    if (enable) {
        rc = srv_setup(c);
        if (rc == TCSUM_OK)
            c.srv_on = true;
        return rc;
    }
    c.srv_on = false;
    return srv_stop(c);
}

int tcsum_call_server(int device, int enable)
{
    if (device < 0 || device >= kMaxDev)
        return TCSUM_ERR_PARAM;
    Ctx &c = g_ctx[device];
    std::lock_guard<std::mutex> lk(c.mu);
    int rc = ctx_init(c, device);
    if (rc != TCSUM_OK)
        return rc;
    if (const hipError_t e = hipSetDevice(device); e != hipSuccess)
        return note_sys(48, e);
    if (enable) {
        rc = cs_setup(c);
        if (rc == TCSUM_OK)
            c.cs_on = true;
        return rc;
    }
    c.cs_on = false;
    return cs_stop(c);
}

// ================================================== drop-in legacy symbols

// net/src/tools.c:24-54
uint16_t checksum16(int offset, void *buf, uint16_t len, uint32_t pre_sum, int complement)
{
    Ctx &c = legacy_ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    // place the bytes so that address parity == logical parity: the kernel
    // then has the exact u32 word sum for the reference's u32 wrap
    const uint32_t par = (uint32_t)offset & 1u;
    if (c.cs_on && cs_setup(c) == TCSUM_OK) {
        const uint32_t ctl = tcsum::MODE_EXACT | (complement ? tcsum::CALL_COMPLEMENT : 0u) |
                             (par ? tcsum::CALL_ODD : 0u);
        if (len + par <= tcsum::kCallInline)
            return (uint16_t)cs_post(c, ctl, len, pre_sum, 0u, 0u, 0u, static_cast<const uint8_t *>(buf));
        memcpy(c.cs_stage + par, buf, len);
        return (uint16_t)cs_post(c, ctl, len, pre_sum, 0u, 0u, 0u);
    }
    if (len + par <= tcsum::kCallInline && args_launch()) { // the bytes travel in the kernel arguments
        run_sync(c, tcsum::launch_inline16(tcsum::MODE_EXACT, buf, len, par, pre_sum, complement, c.d_result,
                                           c.stream));
        return *c.result;
    }
    ensure_stage(c, len);
    uint8_t *dst = c.stage + par;
    if (len)
        memcpy(dst, buf, len);
    if (len <= kOnceMax && args_launch()) { // the descriptor travels in the kernel arguments
        run_sync(c, tcsum::launch_once(tcsum::MODE_EXACT, c.d_stage, par, len, pre_sum, 0u, 0u, 0u, complement,
                                       c.d_result, c.stream));
        return *c.result;
    }
    tcsum_seg_t *d = static_cast<tcsum_seg_t *>(c.desc);
    d->offset = par;
    d->len = len;
    d->pre_sum = pre_sum;
    const hipError_t e = tcsum::launch_segments(tcsum::MODE_EXACT, Geometry{64, 8, 1, 0} /* unused for MODE_EXACT */, c.d_stage, c.d_desc,
                                                1, c.d_result, (complement ? 1u : 0u) | (par << 1), c.stream);
    run_sync(c, e);
    return *c.result;
}

// net/src/pktbuf.c:646-670
uint16_t pktbuf_checksum16(tcsum_pktbuf_t *buf, int len, int pre_sum, int complement)
{
    check_ref(buf);
    const int remain = buf->total_size - buf->pos; // total_blk_remain, pktbuf.c:153-156
    if (remain < len)
        return 0; // pktbuf.c:650-655
    if (len < 0)
        len = 0; // loop not entered: the kernel returns (uint16_t)pre_sum, complemented or not
    Ctx &c = legacy_ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    if (c.cs_on && (size_t)len <= kCallStageMax && cs_setup(c) == TCSUM_OK) {
        const uint32_t ctl = tcsum::MODE_SEG | (complement ? tcsum::CALL_COMPLEMENT : 0u);
        if ((uint32_t)len <= tcsum::kCallInline) {
            uint8_t small[tcsum::kCallInline];
            gather(buf, len, small);
            return (uint16_t)cs_post(c, ctl, (uint32_t)len, (uint32_t)pre_sum, 0u, 0u, 0u, small);
        }
        gather(buf, len, c.cs_stage);
        return (uint16_t)cs_post(c, ctl, (uint32_t)len, (uint32_t)pre_sum, 0u, 0u, 0u);
    }
    if ((uint32_t)len <= tcsum::kCallInline && args_launch()) { // the bytes travel in the kernel arguments
        uint8_t small[tcsum::kCallInline];
        gather(buf, len, small);
        run_sync(c, tcsum::launch_inline16(tcsum::MODE_SEG, small, (uint32_t)len, 0u, (uint32_t)pre_sum, complement,
                                           c.d_result, c.stream));
        return *c.result;
    }
    ensure_stage(c, (size_t)len);
    gather(buf, len, c.stage);
    if ((size_t)len <= kOnceMax && args_launch()) { // the descriptor travels in the kernel arguments
        run_sync(c, tcsum::launch_once(tcsum::MODE_SEG, c.d_stage, 0u, (uint32_t)len, (uint32_t)pre_sum, 0u, 0u, 0u,
                                       complement, c.d_result, c.stream));
        return *c.result;
    }
    tcsum_seg_t *d = static_cast<tcsum_seg_t *>(c.desc);
    d->offset = 0;
    d->len = (uint32_t)len;
    d->pre_sum = (uint32_t)pre_sum;
    const hipError_t e = tcsum::launch_segments(tcsum::MODE_SEG, tcsum::pick_geometry((uint64_t)len), c.d_stage,
                                                c.d_desc, 1, c.d_result, complement ? 1u : 0u, c.stream);
    run_sync(c, e);
    return *c.result;
}

// net/src/tools.c:56-75
uint16_t checksum_peso(tcsum_pktbuf_t *buf, const tcsum_ipaddr_t *dest, const tcsum_ipaddr_t *src,
                       uint8_t protocol)
{
    check_ref(buf);
    reset_access(buf); // tools.c:72
    const int total = buf->total_size;
    Ctx &c = legacy_ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    if (c.cs_on && (total <= 0 || (size_t)total <= kCallStageMax) && cs_setup(c) == TCSUM_OK) {
        if (total > 0)
            gather(buf, total, c.cs_stage); // leaves the cursor at the end, like tools.c:73
        uint32_t s32, d32;
        memcpy(&s32, src->addr, 4);
        memcpy(&d32, dest->addr, 4);
        return (uint16_t)cs_post(c, tcsum::MODE_PESO, total > 0 ? (uint32_t)total : 0u, 0u, s32, d32, protocol);
    }
    ensure_stage(c, total > 0 ? (size_t)total : 0);
    if (total > 0)
        gather(buf, total, c.stage); // leaves the cursor at the end, like tools.c:73
    if ((total <= 0 || (size_t)total <= kOnceMax) && args_launch()) { // the descriptor in the kernel arguments
        uint32_t s32, d32;
        memcpy(&s32, src->addr, 4);
        memcpy(&d32, dest->addr, 4);
        run_sync(c, tcsum::launch_once(tcsum::MODE_PESO, c.d_stage, 0u, total > 0 ? (uint32_t)total : 0u, 0u, s32,
                                       d32, protocol, 0, c.d_result, c.stream));
        return *c.result;
    }
    tcsum_peso_t *d = static_cast<tcsum_peso_t *>(c.desc);
    d->offset = 0;
    d->len = total > 0 ? (uint32_t)total : 0;
    memcpy(d->src, src->addr, 4);
    memcpy(d->dst, dest->addr, 4);
    d->protocol = protocol;
    d->rsv[0] = d->rsv[1] = d->rsv[2] = 0;
    const hipError_t e = tcsum::launch_segments(tcsum::MODE_PESO, tcsum::pick_geometry((uint64_t)d->len),
                                                c.d_stage, c.d_desc, 1, c.d_result, 0u, c.stream);
    run_sync(c, e);
    return *c.result;
}

int tcsum_release(int device)
{
    if (device < 0 || device >= kMaxDev)
        return TCSUM_ERR_PARAM;
    return release_ctx(g_ctx[device], device);
}

} // extern "C"
