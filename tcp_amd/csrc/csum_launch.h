// csum_launch.h -- internal interface between the C ABI (csum_api.cpp) and the
// gfx950 kernels (csum_kernels.hip).  Not installed; not part of include/.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tcsum.h"

namespace tcsum {

// A failed runtime call whose failure this library handles itself (a
// cleanup free, a fallback): its error must not stay in the calling thread's
// last-error slot, where the caller's next hipGetLastError() -- PyTorch
// checks every kernel launch that way -- would take it for its own.  The slot
// is cleared only when it holds this call's error, so an error of the
// caller's stays for the caller.  (No launch of the library reads the slot:
// launch(), csum_device.h, returns each launch's own status.)
inline hipError_t quiet(hipError_t e)
{
    if (e != hipSuccess && hipPeekAtLastError() == e)
        (void)hipGetLastError();
    return e;
}

// hipErrorInvalidValue for a shape or size a launcher refuses itself (no
// runtime call made); take_refused(): whether the last such status of this
// thread was one, clearing the mark.
hipError_t refused();
bool take_refused();

// What a segment kernel computes per range (see csum_kernels.hip).
enum Mode : int {
    MODE_SEG = 0,   // pktbuf_checksum16: u16 pre_sum, optional complement
    MODE_EXACT = 1, // checksum16: u32 pre_sum with the reference's u32 wrap
    MODE_PESO = 2,  // checksum_peso: pseudo-header built in-kernel
};

struct Geometry {
    int lanes;  // G: lanes that share one packet (4..64, power of two; 256 / 1024: one range per workgroup)
    int loads;  // U: 16-byte loads in flight per lane per pass
    int xcd;    // consecutive workgroups kept on one XCD (1: dispatch order)
    int packed; // K > 0: checksum_peso / pktbuf_checksum16 batches as a packed
                // stream, K consecutive ranges per 4-wave workgroup (k_segments_pk)
    int interior; // a mean-length range's interior 16-B chunks (0: unknown), for the per-range shape
};

// Test and measurement overrides (include/tcsum_debug.h): -1 = the router's
// own choice.  Read on launch paths; set only by tcsum_debug_set.
enum Knob : int {
    KNOB_LANES = 0,  // per-range lanes (G)
    KNOB_LOADS,      // per-range loads per lane (U)
    KNOB_XCD,        // XCD run length
    KNOB_PACKED,     // 0 / 1: k_segments_pk off / on
    KNOB_TX_SPLIT,   // 0 / 1: tx fill stores in the kernel / deferred to k_tx_scatter
    KNOB_ARGS_LAUNCH, // 0: drop-in launch path with its descriptor in pinned memory
    KNOB_SYNC_BLOCK, // 1: drop-in calls block in hipStreamSynchronize instead of spinning
    KNOB_E2E_TRACE,  // 1: tcsum_host_batch_peso prints phase stamps
    KNOB_E2E_CHUNK_MB, // tcsum_host_batch_peso chunk size
    KNOB_SERVER_MAX,   // largest host-queue batch handed to the queue server (65536)
    KNOB_SERVER_TRACE, // 1: the queue server prints its phase stamps when stopped
    KNOB_SERVER_IDLE_MS, // resident servers stop after this long without a job (10)
    KNOB_SERVER_WGS,   // queue server workgroups (64)
    KNOB_HOSTQ_DMA_KB, // host-queue batches from this span on go through the copy engine (262144)
    KNOB_HOSTQ_DMA_KEEP_MB, // device arena kept between host-queue calls up to this size (256)
    KNOB_COPY_THREADS, // host threads of a parallel gather / scatter pass (16)
    KNOB_PF_DIST,      // descriptor prefetch distance of k_segments_pk's range-by-range path (2048)
    KNOB_PF_RANGE,     // descriptor prefetch distance of the per-range kernels k_segments (0)
    KNOB_PK_EARLY,     // 0 / 1: k_segments_pk's range-by-range path reads its descriptors with scalar loads (1)
    KNOB_PAGE_STAGE,   // 0 / 1: tcsum_host_batch_peso copies a pageable arena through its own pinned slots (1)
    KNOB_SEG_SDESC,    // 0 / 1: the per-range kernel (8-16 lanes per range) reads its descriptors with scalar loads (1)
    KNOB_TX_WARM,      // 0 / 1: the deferred tx scatter loads each field's dword before storing it (1, HBM only)
    KNOB_COUNT
};
int64_t knob(Knob k);
void set_knob(Knob k, int64_t v);

Geometry pick_geometry(uint64_t mean_len);

// Whether k_segments_pk's range-by-range path reads its descriptors with
// scalar loads (debug knob "pk_early"; on by default).
bool pk_early();

// The route for ranges known to be out of offset order: the packed kernel
// only where its range-by-range path beats the per-range kernels (K <= 8,
// i.e. ranges of ~1.5 KiB and up, with pk_early), else the per-range kernel.
inline void shuffled_route(Geometry &g, int64_t packed_knob)
{
    if (packed_knob != 1 && !(g.packed > 0 && g.packed <= 8 && pk_early()))
        g.packed = 0;
}

// k_ipv4's lane groups for packets of mean length ~16 * (interior + 1) B when
// no debug knob forces one (launch_ipv4 and the bench lib's probe).  Short
// packets take narrow groups: the header parse, the gates and the result
// are per-lane work every lane of a group repeats, and a 16-lane group on a
// 100-B packet repeats it 16 times for 7 chunks.  Equal-length batches,
// one process (profiles/r06/ab21/ipv4_narrow*.txt), route against 16 x 2..8:
// sums 40-64 B 1.3-1.5x faster again at 2 x 4 than at 4 x 4 (ab26/; rx 40-100 B
// 1.2-1.3x), 100 B 2.44x at 4 x 4, 200 B 1.9x, 300 B 1.66x at 8 x 4, 600 B
// 1.37x at 8 x 6, 1,000 B 1.23x at 8 x 3, 1,500-3,000 B 3-7 % at 16 x 4 /
// 16 x 3 / 16 x 6; rx 100-300 B 1.8-2.3x at 4 x 4, 600 B 1.35x at 8 x 6,
// 1,000 B 1.35x at 8 x 3, 1,500 B 1.22x, 2,000 B 1.14x (ab25/).  Longer
// packets keep pick_geometry's lanes (>= 16; rx at 16 where the others take
// 32).  Returns false when nothing changed.
inline bool ipv4_short_shape(Geometry &g, int ip_mode, uint64_t interior)
{
    const bool rx = ip_mode == 2;
    int G = 0, U = 0;
    if (interior == 0 || interior > 246) // unknown, or ~4 KiB and longer
        return false;
    if (interior <= (rx ? 6u : 4u)) { // < ~96 B (rx: < ~128 B): two lanes a packet
        G = 2, U = 4;
    } else if (interior <= 14) { // < ~250 B
        G = 4, U = 4;
    } else if (interior <= 27) { // ~250-450 B
        G = rx ? 4 : 8, U = 4;
    } else if (interior <= 48) { // ~450-800 B
        G = 8, U = 6;
    } else if (interior <= 80) { // ~800-1300 B
        G = 8, U = 3;
    } else if (rx) { // ~1300-2500 B: 8 x 3, then 16 x 3 (1,500-B 1.22x, 2,000-B 1.14x); longer: the old rule
        if (interior > 155)
            return false;
        G = interior <= 111 ? 8 : 16, U = 3;
    } else if (interior <= 111) { // ~1300-1800 B
        G = 16, U = 4;
    } else if (interior <= 155) { // ~1800-2500 B
        G = 16, U = 3;
    } else { // ~2500-4000 B
        G = 16, U = 6;
    }
    g.lanes = G;
    g.loads = U;
    return true;
}

// The k_ipv4 shape launch_ipv4 takes for geometry g and ip_mode (below):
// ipv4_short_shape unless a debug knob forces lanes / loads, else lanes
// clamped to 16..64 (forced: 2..64), rx at 16 where the others take 32.
void ipv4_geometry(Geometry &g, int ip_mode);

// aux: MODE_SEG -> complement; MODE_EXACT -> complement | (offset parity << 1).
hipError_t launch_segments(Mode mode, Geometry g, const void *arena, const void *descs,
                           uint32_t n, uint16_t *out, uint32_t aux, hipStream_t stream);

// ip_mode: 0 sums, 1 tx fill (writes into arena), 2 rx verify (verdict required),
//          3 tx offload (the tx fill's values into out only; out required),
//          4 tx fill with its stores deferred to a second launch (k_tx_scatter)
hipError_t launch_ipv4(int ip_mode, Geometry g, uint8_t *arena, const tcsum_pkt_t *pkts, uint32_t n,
                       uint32_t *out, uint8_t *flags, int8_t *verdict, hipStream_t stream);

// The tx fill (deferred stores) reading `arena` and storing the fields into
// `store` (the same packets at another device-visible address).
hipError_t launch_ipv4_tx_to(Geometry g, uint8_t *arena, uint8_t *store, const tcsum_pkt_t *pkts, uint32_t n,
                             uint32_t *out, uint8_t *flags, hipStream_t stream);

// The tx fill with its stores deferred, in scratch the caller owns (8 * n
// bytes): no allocation, so it can be captured in a hipGraph.
// give back the tx fill's pooled scratch of device dev (tcsum_release)
hipError_t scratch_trim(int dev);
uint64_t scratch_reserved(int dev);

hipError_t launch_ipv4_tx_scratch(Geometry g, uint8_t *arena, const tcsum_pkt_t *pkts, uint32_t n, uint32_t *out,
                                  uint8_t *flags, uint32_t *scratch, hipStream_t stream);

// Queue server (k_server): one job at a time.  SrvHost lives in pinned,
// coherent host memory (the host writes the job, then `req`, and reads `done`);
// SrvCtl in device memory (zeroed before every launch).
struct SrvHost {
    uint32_t req;  // host: sequence number of the posted job (never 0)
    uint32_t quit; // host: ask the grid to leave
    uint32_t op;   // IP_SUMS / IP_TX / IP_RX
    uint32_t n;    // packets
    uint64_t ptr[5]; // device-visible: arena, pkts, out, flags, verdict (0 = none)
    uint64_t trace;  // device-visible u64[256 * 8] of phase stamps, or 0 (debug knob "server_trace")
    uint32_t pad[2];
    alignas(64) uint32_t done; // device: last completed job
};
struct SrvCtl {
    uint32_t seq, quit, op, n;
    uint64_t ptr[5];
    uint32_t arrivals;
    uint32_t pad;
};
static_assert(sizeof(SrvCtl) % 16 == 0, "SrvCtl is memset whole");

hipError_t launch_server(SrvHost *h /*device-visible address*/, SrvCtl *d, uint32_t last, uint64_t idle_ticks,
                         int wgs, hipStream_t stream);

// Call server (k_call): one resident wave serving the synchronous drop-in
// calls (checksum16 / pktbuf_checksum16 / checksum_peso) posted through
// pinned, coherent host memory.  The wave reads the four 16-byte job words in
// one poll and takes the job only when all carry the new sequence number
// (the host stores every field, then w3[3], w2[3], w1[3] and w0[0] last).
enum CallCtl : uint32_t {
    CALL_MODE_MASK = 3u,    // a Mode
    CALL_COMPLEMENT = 4u,   // MODE_SEG / MODE_EXACT: complement the result
    CALL_ODD = 8u,          // MODE_EXACT: the bytes start at stage + 1 (offset parity)
    CALL_INLINE = 16u,      // the bytes are in w2/w3 (<= kCallInline with the parity byte), not in stage
    CALL_QUIT = 1u << 31,   // leave
};
constexpr uint32_t kCallInline = 24; // bytes carried in the job line itself
struct CallBox {
    uint32_t w0[4]; // seq, ctl, len, pre_sum
    uint32_t w1[4]; // src, dst (as in memory), protocol, seq
    uint32_t w2[4]; // inline bytes 0..11, seq
    uint32_t w3[4]; // inline bytes 12..23, seq
    alignas(64) uint64_t res; // device: result << 32 | seq of the finished job
};
static_assert(sizeof(CallBox) == 128, "CallBox: job line + result line");

// MODE_EXACT (checksum16) or MODE_SEG (pktbuf_checksum16) on len + odd <=
// kCallInline bytes passed in the kernel arguments; the u16 result into *out.
hipError_t launch_inline16(Mode mode, const void *bytes, uint32_t len, uint32_t odd, uint32_t pre, int complement,
                           uint16_t *out, hipStream_t stream);

// One range of staged bytes at stage + off, its descriptor in the kernel
// arguments (src/dst/proto: MODE_PESO only); the u16 result into *out.
hipError_t launch_once(Mode mode, const uint8_t *stage, uint32_t off, uint32_t len, uint32_t pre, uint32_t src,
                       uint32_t dst, uint32_t proto, int complement, uint16_t *out, hipStream_t stream);

hipError_t launch_call_server(CallBox *box /*device-visible address*/, const uint8_t *stage /*device-visible*/,
                              uint32_t last, uint64_t idle_ticks, hipStream_t stream);

} // namespace tcsum
