/*
 * tcsum.h -- MI355X Internet-checksum engine: C ABI.
 *
 * This library replaces one leaf of the wj9806/tcp stack: the one's-complement
 * 16-bit folding sum over IPv4 headers and TCP/UDP pseudo-header + payload.
 *
 *   Legacy, drop-in (same names and signatures as the reference): see
 *   tcsum_legacy.h -- checksum16 / checksum_peso / pktbuf_checksum16.
 *
 *   Batched, device-resident (this header): packets sit contiguously in HBM
 *   (an "arena") and are described by an offset/length array; one launch
 *   checksums the whole batch with hand-written gfx950 kernels.
 *
 * Conventions
 *   - All pointers marked [dev] are device (HBM) pointers; [host] are host.
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream).
 *     Batch calls are asynchronous on that stream; nothing is allocated or
 *     freed inside them (they are safe to capture in a hipGraph) -- except
 *     the stream-ordered scratch of a large tcsum_batch_ipv4_tx_fill outside
 *     capture (see there).
 *   - Results are the u16 exactly as the reference returns it: the value as it
 *     sits in little-endian host memory, so storing it into the header field
 *     yields network-order bytes (net/src/tools.c:24-54).
 *   - Return codes are the reference's net_err_t values
 *     (net/net/net_err.h:8-29): 0 = OK, negative = error.
 *   - One arena per batch: every byte from a batch's lowest range start to
 *     its highest range end must be readable device memory (one
 *     allocation).  The stream kernels read the bytes between neighbouring
 *     ranges -- padding, gaps -- and discard them; ranges may sit anywhere
 *     in that span, in any order, overlap or repeat.
 */
#ifndef TCSUM_H
#define TCSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TCSUM_OK 0               /* NET_ERR_OK */
#define TCSUM_ERR_SYS (-1)       /* NET_ERR_SYS: HIP runtime failure */
#define TCSUM_ERR_MEM (-2)       /* NET_ERR_MEM: allocation failed */
#define TCSUM_ERR_SIZE (-5)      /* NET_ERR_SIZE */
#define TCSUM_ERR_PARAM (-7)     /* NET_ERR_PARAM: bad argument */
#define TCSUM_ERR_BROKEN (-13)   /* NET_ERR_BROKEN: checksum mismatch (rx verdicts) */
#define TCSUM_ERR_UNREACHABLE (-14) /* NET_ERR_UNREACHABLE: rx verdict, UDP to port 0 */
#define TCSUM_ERR_NOT_SUPPORT (-11) /* NET_ERR_NOT_SUPPORT: no usable gfx950 device */

/* ------------------------------------------------------------ descriptors */

/* A byte range with a caller-supplied partial sum: one pktbuf_checksum16 call
 * (net/src/pktbuf.c:646-670).  pre_sum is truncated to 16 bits exactly like
 * `uint16_t sum = pre_sum` (pktbuf.c:657); byte parity counts from `offset`. */
typedef struct tcsum_seg {
    uint64_t offset; /* byte offset of the range in the arena (any alignment) */
    uint32_t len;    /* bytes; may exceed 65535 (chained like the pktbuf walk) */
    uint32_t pre_sum;
} tcsum_seg_t;

/* A TCP/UDP segment: one checksum_peso call (net/src/tools.c:56-75).  The
 * pseudo-header (src, dst, {0,protocol}, htons((uint16_t)len)) is built
 * in-kernel. */
typedef struct tcsum_peso {
    uint64_t offset;  /* L4 header start in the arena */
    uint32_t len;     /* L4 header + payload bytes (buf->total_size) */
    uint8_t src[4];   /* ipaddr_t.addr of the source, network order */
    uint8_t dst[4];   /* ipaddr_t.addr of the destination */
    uint8_t protocol; /* 6 (TCP) or 17 (UDP); any value is summed as given */
    uint8_t rsv[3];
} tcsum_peso_t;

/* A captured IPv4 packet (header + L4) for tcsum_batch_ipv4. */
typedef struct tcsum_pkt {
    uint64_t offset; /* first byte of the IPv4 header in the arena */
    uint32_t len;    /* captured frame length from the IPv4 header on */
    uint32_t rsv;
} tcsum_pkt_t;

/* tcsum_batch_ipv4 flag bits: what is_pkt_ok (net/src/ipv4.c:220-239) would
 * reject, plus protocols with no L4 checksum here. */
#define TCSUM_PKT_BAD_VERSION 0x01u /* version != 4                   (ipv4.c:222) */
#define TCSUM_PKT_BAD_HDRLEN 0x02u  /* ihl*4 < 20 or > len            (ipv4.c:229) */
#define TCSUM_PKT_BAD_TOTLEN 0x04u  /* total_len < 20, > len, < ihl*4 (ipv4.c:236) */
#define TCSUM_PKT_PROTO_OTHER 0x08u /* not TCP/UDP/ICMP: l4 result is 0 */
#define TCSUM_PKT_SHORT 0x10u       /* len < 20: both results are 0 */
#define TCSUM_PKT_FRAGMENT 0x20u    /* MF or fragment offset: the L4 checksum spans the
                                       datagram, so tx fill / rx verify leave it (ipv4.c:506) */
#define TCSUM_PKT_L4_SHORT 0x40u    /* L4 shorter than its header (TCP 20, UDP 8, ICMP 4 B) */

/* ------------------------------------------------ device-resident batches */

/* What a caller knows of where its ranges lie (tcsum_batch's hint). */
#define TCSUM_LAYOUT_UNKNOWN 0  /* the calls below: the stream kernels check per workgroup */
#define TCSUM_LAYOUT_ORDERED 1  /* descriptors in arena order, ranges disjoint (gaps allowed) */
#define TCSUM_LAYOUT_SHUFFLED 2 /* no order to exploit: the per-range / per-packet kernels (ranges of
                                 * ~1.5 KiB and up: the packed kernel's range-by-range path, faster) */

typedef struct tcsum_hint {
    uint64_t total_bytes; /* sum of the lengths; 0 = unknown (read as 1500-B ranges) */
    uint32_t layout;      /* TCSUM_LAYOUT_* */
    uint32_t rsv;         /* 0 */
} tcsum_hint_t;

/* tcsum_batch operations: the same computations as the named calls below. */
#define TCSUM_OP_SEGMENTS 0        /* tcsum_batch_segments, complement 0: out u16[n], descs tcsum_seg_t */
#define TCSUM_OP_SEGMENTS_COMP 1   /* tcsum_batch_segments, complement 1 */
#define TCSUM_OP_PESO 2            /* tcsum_batch_peso: out u16[n], descs tcsum_peso_t */
#define TCSUM_OP_IPV4 3            /* tcsum_batch_ipv4: out u32[n], flags (or NULL) */
#define TCSUM_OP_IPV4_TX_FILL 4    /* tcsum_batch_ipv4_tx_fill: out (or NULL), flags (or NULL) */
#define TCSUM_OP_IPV4_TX_OFFLOAD 5 /* tcsum_batch_ipv4_tx_offload: out and flags required */
#define TCSUM_OP_IPV4_RX_VERIFY 6  /* tcsum_batch_ipv4_rx_verify: verdict required, out / flags or NULL */

/* Every device-resident batch in one call, with the caller's layout hint
 * (hint NULL: total unknown, layout UNKNOWN -- exactly the named calls).
 * Results are the same whatever the hint.  ORDERED is routed as UNKNOWN
 * today (the stream kernels check the order per workgroup either way; a
 * batch that breaks the promise is still summed exactly).  SHUFFLED skips
 * the stream kernels, which a batch in no particular order would only leave
 * again.  hint->rsv must be 0 (TCSUM_ERR_PARAM otherwise).  arena is written
 * only by TCSUM_OP_IPV4_TX_FILL. */
int tcsum_batch(int op, void *arena /*[dev]*/, const void *descs /*[dev]*/, uint32_t n, void *out /*[dev]*/,
                uint8_t *flags /*[dev] or NULL*/, int8_t *verdict /*[dev] or NULL*/, const tcsum_hint_t *hint /*[host]*/,
                void *stream);

/* out[i] = pktbuf_checksum16 over segs[i] with complement (0/1).
 * total_bytes_hint = sum of lens if known, else 0 (read as 1500-B ranges): the
 * mean length selects the kernel -- up to ~4 KiB, ranges listed in arena order
 * are streamed as one region per workgroup (k_segments_pk), any order exact. */
int tcsum_batch_segments(const void *arena /*[dev]*/, const tcsum_seg_t *segs /*[dev]*/,
                         uint32_t n, uint16_t *out /*[dev]*/, int complement,
                         uint64_t total_bytes_hint, void *stream);

/* out[i] = checksum_peso over segs[i]: the value tcp_out.c:20 / udp.c:321
 * store, or 0 on rx for a segment whose stored checksum is right
 * (tcp_in.c:80, udp.c:410). */
int tcsum_batch_peso(const void *arena /*[dev]*/, const tcsum_peso_t *segs /*[dev]*/,
                     uint32_t n, uint16_t *out /*[dev]*/, uint64_t total_bytes_hint,
                     void *stream);

/* Both checksums of each IPv4 packet, pseudo-header taken from the packet:
 *   out[i] & 0xFFFF = checksum16(0, hdr, ihl*4, 0, 1)                (ipv4.c:243, 656)
 *   out[i] >> 16    = checksum_peso(l4, dst, src, proto) for TCP/UDP (tcp_in.c:80, udp.c:410)
 *                   = pktbuf_checksum16(l4, l4len, 0, 1) for ICMP    (icmpv4.c:36)
 *                   = 0 otherwise
 * with l4 = [ihl*4, total_len).  On a rejected packet the ranges are clamped
 * to [20 .. len] and flags[i] says why; flags may be NULL. */
int tcsum_batch_ipv4(const void *arena /*[dev]*/, const tcsum_pkt_t *pkts /*[dev]*/,
                     uint32_t n, uint32_t *out /*[dev]*/, uint8_t *flags /*[dev] or NULL*/,
                     uint64_t total_bytes_hint, void *stream);

/* Batched tx fill, in place in the arena: for every
 * well-formed packet the checksum fields are read as zero and the values the
 * stack's tx path stores are written into them:
 *   IPv4 header checksum (bytes 10-11)      ipv4.c:643,656 (fragments too)
 *   TCP checksum (L4 + 16)                  tcp_out.c:19-20
 *   UDP checksum (L4 + 6; 0 is stored as 0) udp.c:320-321
 *   ICMP checksum (L4 + 2)                  icmpv4.c:45-58
 * L4 fields are left alone for fragments and short L4s; nothing is written
 * for SHORT / BAD_* packets.  out (ip | l4 << 16) and flags may be NULL.
 * From 131,072 packets of a mean length of 2,800 B or more (total_bytes_hint
 * / n; 1,500 B when the hint is 0) the stores are deferred (tests and
 * measurement force either form with tcsum_debug_set("tx_split", 0 / 1),
 * tcsum_debug.h): one launch computes every packet's values and field
 * positions into stream-ordered scratch (4-8 B per packet, from a memory
 * pool the library keeps per device, up to 1 GiB retained between calls;
 * freed on the stream), a second short launch writes all the fields.  Same
 * bytes either way; the batch is complete when the stream reaches the end.
 * On a stream under hipGraph capture the fill is one launch that allocates
 * nothing, like every other batch call. */
int tcsum_batch_ipv4_tx_fill(void *arena /*[dev]*/, const tcsum_pkt_t *pkts /*[dev]*/, uint32_t n,
                             uint32_t *out /*[dev] or NULL*/, uint8_t *flags /*[dev] or NULL*/,
                             uint64_t total_bytes_hint, void *stream);

/* tcsum_batch_ipv4_tx_fill in its deferred-store form (the faster one for
 * large batches) with scratch the caller owns: scratch_bytes >= 8 * n,
 * 4-byte aligned, device memory, not touched by anything else until the
 * stream passes the call.  Nothing is allocated, so unlike the plain call's
 * deferred form it can be captured in a hipGraph (replays of one graph must
 * not run concurrently: they share the scratch).  Same bytes as
 * tcsum_batch_ipv4_tx_fill. */
int tcsum_batch_ipv4_tx_fill_scratch(void *arena /*[dev]*/, const tcsum_pkt_t *pkts /*[dev]*/, uint32_t n,
                                     uint32_t *out /*[dev] or NULL*/, uint8_t *flags /*[dev] or NULL*/,
                                     void *scratch /*[dev]*/, uint64_t scratch_bytes, uint64_t total_bytes_hint,
                                     void *stream);

/* Batched tx offload (NIC checksum-offload style): the
 * values tcsum_batch_ipv4_tx_fill would store -- out[i] = ip | l4 << 16, with
 * the checksum fields read as zero -- and flags[i], WITHOUT writing the
 * packets (the arena is read-only here).  The host applies them with
 * tcsum_tx_apply where it touches the frame anyway (the pcap tx thread's copy
 * of each frame, netif_pcap.c:42-67), which skips the scattered in-place
 * writes of the fill.  tcsum_tx_apply on every packet of a batch leaves the
 * bytes tcsum_batch_ipv4_tx_fill leaves.  out and flags are required. */
int tcsum_batch_ipv4_tx_offload(const void *arena /*[dev]*/, const tcsum_pkt_t *pkts /*[dev]*/, uint32_t n,
                                uint32_t *out /*[dev]*/, uint8_t *flags /*[dev]*/,
                                uint64_t total_bytes_hint, void *stream);

/* Host side of the offload: store csums (one out[] word) into the IPv4 frame
 * of len bytes at `frame` [host] exactly as the fill would -- header checksum
 * always, the TCP/UDP/ICMP field unless flags says fragment / short L4 /
 * other protocol, nothing for a SHORT / BAD_* packet.  Plain CPU stores. */
int tcsum_tx_apply(void *frame /*[host]*/, uint32_t len, uint32_t csums, uint8_t flags);
/* tcsum_tx_apply over a batch in a host arena (bounds checked first). */
int tcsum_tx_apply_batch(void *arena /*[host]*/, uint64_t arena_bytes, const tcsum_pkt_t *pkts /*[host]*/,
                         uint32_t n, const uint32_t *csums /*[host]*/, const uint8_t *flags /*[host]*/);

/* Batched rx verify: verdict[i] = the net_err_t the
 * reference's receive path returns, gate by gate in its order, up to (not
 * including) socket lookup and routing:
 *   frame < 20                               SIZE        ipv4.c:475 (pktbuf_set_cont)
 *   version != 4                             NOT_SUPPORT ipv4.c:222-226
 *   IHL*4 < 20, total_len < 20 or > frame    SIZE        ipv4.c:228-240
 *   stored header checksum != 0 and wrong    BROKEN      ipv4.c:241-249
 *   fragment (MF or offset)                  OK          ipv4.c:506-509 (reassembly)
 *   TCP  (after pktbuf_remove_header, ipv4.c:450-452)
 *     segment < 20 bytes                     -1 (SYS)    tcp_in.c:70-74
 *     stored checksum != 0 and wrong         BROKEN      tcp_in.c:77-85
 *     segment < data offset * 4              SIZE        tcp_in.c:87-91
 *     source or destination port 0           BROKEN      tcp_in.c:93-97
 *     flag word (offset+flags) 0             BROKEN      tcp_in.c:99-103
 *   UDP  datagram < 8 bytes                  SIZE        udp.c:386-391
 *        destination port 0                  UNREACHABLE udp.c:337-340, 399-403
 *        stored checksum != 0 and wrong      BROKEN      udp.c:407-415
 *   ICMP message < 4 bytes                   SIZE        icmpv4.c:68-73 (its checksum
 *                                                        test cannot fail, A10)
 *   otherwise OK (other protocols: raw_in, no checksum).
 * The verdicts equal the reference stack's own on every packet of
 * tests/golden/ipv4_rx_* (oracle/stack_gen.c runs its ipv4_in/tcp_in/udp_in/
 * icmpv4_in/raw_in) with a UDP socket bound to each port and the netif owning
 * each destination.  Defined here where the reference is not: TCP with
 * IHL*4 > total_len -> SIZE (the reference dereferences NULL in
 * pktbuf_remove_header); a nonzero header checksum with IHL*4 past the frame
 * is checked over the captured bytes only (the reference reads past them).
 * out and flags may be NULL. */
int tcsum_batch_ipv4_rx_verify(const void *arena /*[dev]*/, const tcsum_pkt_t *pkts /*[dev]*/,
                               uint32_t n, int8_t *verdict /*[dev]*/, uint32_t *out /*[dev] or NULL*/,
                               uint8_t *flags /*[dev] or NULL*/, uint64_t total_bytes_hint, void *stream);

/* --------------------------------------------------- host-resident batches */

/* End to end: host arena -> hipMemcpyAsync H2D (chunks in order on one copy
 * stream; each chunk's kernel on a second stream behind that chunk's copy) ->
 * tcsum_batch_peso -> D2H of the results; returns after the results are in
 * host_out.  host_arena should come from tcsum_host_alloc (pinned) for full
 * PCIe rate; a pageable host_arena crosses through the library's own pinned
 * slots (the host threads copy, the copy engine reads only memory the
 * library owns: ~0.96 of the pinned rate).  Segments may be in any order (in offset order the copies and
 * kernels pipeline; otherwise the batch's byte span is copied once).  The
 * first ~64 MiB of segments are checked before anything else; a bad segment
 * after them is found while their copy runs (the call drains it and returns
 * NET_ERR_PARAM), so on a host without a usable device such a batch reports
 * the device error first. */
int tcsum_host_batch_peso(int device, const void *host_arena, uint64_t arena_bytes,
                          const tcsum_peso_t *segs /*[host]*/, uint32_t n,
                          uint16_t *out /*[host]*/);

/* tcsum_host_batch_peso over several GPUs of this node: the segments are cut
 * into contiguous shards balanced by bytes, one per entry of devices[] (a
 * device may repeat; its shards then run one after the other), each shard
 * moved over its own GPU's host link and summed in its HBM by one host thread
 * per device.  Results land in out[] in segment order.  No collective. */
int tcsum_host_batch_peso_multi(const int *devices, int ndev, const void *host_arena, uint64_t arena_bytes,
                                const tcsum_peso_t *segs /*[host]*/, uint32_t n, uint16_t *out /*[host]*/);

/* Host-queue IPv4 batches: the frames of a netif
 * in_q / out_q (net/src/netif.c:339-349, exmsg.c:89-112) as they sit in host
 * memory.  Same semantics as the device-resident calls above; every pointer
 * is [host] and the calls return when the results are in place.
 *   - host_arena from tcsum_host_alloc (or any pinned memory) is read -- and
 *     by tx fill written -- IN PLACE by the kernel over PCIe: no staging copy,
 *     the "DMA-able pktbuf storage" of plat/ (pktbuf.c:13).
 *   - a pageable host_arena is copied into pinned staging first (and, for tx
 *     fill, copied back afterwards).
 *   - every [offset, offset+len) must lie inside [0, arena_bytes) ->
 *     otherwise TCSUM_ERR_PARAM and nothing is touched.
 * out / flags may be NULL except out for tcsum_host_batch_ipv4. */
int tcsum_host_batch_ipv4(int device, const void *host_arena, uint64_t arena_bytes,
                          const tcsum_pkt_t *pkts /*[host]*/, uint32_t n, uint32_t *out /*[host]*/,
                          uint8_t *flags /*[host] or NULL*/);
int tcsum_host_batch_ipv4_tx_fill(int device, void *host_arena, uint64_t arena_bytes,
                                  const tcsum_pkt_t *pkts /*[host]*/, uint32_t n,
                                  uint32_t *out /*[host] or NULL*/, uint8_t *flags /*[host] or NULL*/);
int tcsum_host_batch_ipv4_rx_verify(int device, const void *host_arena, uint64_t arena_bytes,
                                    const tcsum_pkt_t *pkts /*[host]*/, uint32_t n, int8_t *verdict /*[host]*/,
                                    uint32_t *out /*[host] or NULL*/, uint8_t *flags /*[host] or NULL*/);

/* (Capture files: include/tcsum_pcap.h, a separate host-only helper library.) */

/* The three host-queue batches over several GPUs of this node: contiguous
 * shards balanced by bytes, one per entry of devices[] (a device may repeat;
 * its shards then run one after the other), each an ordinary host batch on
 * its device -- pinned frames (tcsum_host_alloc is portable: every GPU maps
 * it) read and, tx, written in place over that GPU's own host link.  Same
 * results, in packet order, as the one-device calls.  For the tx fill, packets
 * of different shards must not overlap. */
int tcsum_host_batch_ipv4_multi(const int *devices, int ndev, const void *host_arena, uint64_t arena_bytes,
                                const tcsum_pkt_t *pkts /*[host]*/, uint32_t n, uint32_t *out /*[host]*/,
                                uint8_t *flags /*[host] or NULL*/);
int tcsum_host_batch_ipv4_tx_fill_multi(const int *devices, int ndev, void *host_arena, uint64_t arena_bytes,
                                        const tcsum_pkt_t *pkts /*[host]*/, uint32_t n,
                                        uint32_t *out /*[host] or NULL*/, uint8_t *flags /*[host] or NULL*/);
int tcsum_host_batch_ipv4_rx_verify_multi(const int *devices, int ndev, const void *host_arena,
                                          uint64_t arena_bytes, const tcsum_pkt_t *pkts /*[host]*/, uint32_t n,
                                          int8_t *verdict /*[host]*/, uint32_t *out /*[host] or NULL*/,
                                          uint8_t *flags /*[host] or NULL*/);

/* Queue server for small host-queue batches (the stack's <= 50-frame netif
 * queues, NETIF_INQ_SIZE net_cfg.h:39): with enable != 0, the
 * tcsum_host_batch_ipv4* calls on `device` with n <= 65,536 frames are
 * served by a resident grid that polls pinned memory for the next job,
 * instead of one kernel launch and one stream sync per call (same results,
 * same arguments).  The grid leaves by itself after 10 ms without a job and
 * is relaunched by the next call (both limits: tcsum_debug_set "server_max"
 * / "server_idle_ms", tcsum_debug.h; nothing in the environment sets them); while it is up, a device-wide synchronisation
 * (hipDeviceSynchronize) waits for it to leave.  enable == 0 stops it (bounded
 * wait).  Returns TCSUM_OK, TCSUM_ERR_NOT_SUPPORT without a gfx950 device. */
int tcsum_queue_server(int device, int enable);

/* Call server for the three synchronous drop-in symbols (checksum16,
 * pktbuf_checksum16, checksum_peso; tcsum_legacy.h): with enable != 0 their
 * calls on `device` (the legacy device, tcsum_plat_init / $TCSUM_DEVICE) are
 * served by one resident wave that polls a pinned job box, instead of one
 * kernel launch and one stream sync per call (same results, same side
 * effects).  Ranges over 64 KiB still take the launch path.  The wave leaves
 * by itself after 10 ms without a call ("server_idle_ms", tcsum_debug.h) and
 * the next call relaunches it; while it is up, a device-wide synchronisation
 * waits for it to leave.  $TCSUM_CALL_SERVER=1 turns it on at the first
 * legacy call without a code change.  enable == 0 stops it (bounded wait).
 * Returns TCSUM_OK, TCSUM_ERR_NOT_SUPPORT without a gfx950 device. */
int tcsum_call_server(int device, int enable);

/* ------------------------------------------------------------ platform */

/* HIP device init for the stack's net_plat_init hook (plat/net_plat.c:7):
 * selects `device`, creates the legacy-call stream and its pinned staging.
 * Optional -- the first checksum call does it lazily on device 0 (or
 * $TCSUM_DEVICE). */
int tcsum_plat_init(int device);

/* Pinned host memory (hipHostMalloc) for packet arenas: the "pinned host
 * buffer pool" that plat/ gains.  Returns NULL on failure. */
void *tcsum_host_alloc(size_t bytes);
void tcsum_host_free(void *p);

/* Pin memory the stack already owns, in place (hipHostRegister, mapped): a
 * frame ring the capture path fills (a libpcap / PACKET_MMAP ring, the tx
 * arena of INTEGRATION.md §4a, or the reference's static block pool
 * `block_buffer`, net/src/pktbuf.c:13) becomes DMA-able without moving it,
 * and the host-queue batches then read -- and tx fill writes -- its frames in
 * place instead of staging them.  Returns TCSUM_OK, TCSUM_ERR_PARAM, or
 * TCSUM_ERR_SYS when the runtime refuses.  Unregister before the memory goes
 * away. */
int tcsum_host_register(void *p, size_t bytes);
int tcsum_host_unregister(void *p);

/* Free every buffer the batch calls cache on `device` between calls: the
 * HBM copy of host spans (tcsum_host_batch_peso, the copy-engine path of the
 * host-queue batches), descriptors, the pinned host-queue staging, and the
 * memory the tx fill's scratch pool keeps (up to 1 GiB); a running queue /
 * call server is stopped first and the device is synchronized, so no work of
 * the caller's may still be queued on it.  The next call allocates again.
 * (The copy-engine path keeps at most 256 MiB between calls by itself;
 * "hostq_dma_keep_mb", tcsum_debug.h.)  Returns TCSUM_OK, TCSUM_ERR_PARAM, or
 * TCSUM_ERR_SYS. */
int tcsum_release(int device);

/* Number of usable gfx950 devices (0 when none); never aborts. */
int tcsum_device_count(void);

/* Kernel geometry the batch calls choose for a mean length: lanes per packet
 * (G) and 16-byte loads in flight per lane (U).  Exposed for tests/tuning;
 * tcsum_debug_set("lanes" / "loads") overrides the choice (tcsum_debug.h). */
void tcsum_pick_geometry(uint64_t mean_len, int *lanes_per_packet, int *loads_per_lane);

/* Library identification string. */
const char *tcsum_version(void);

#ifdef __cplusplus
}
#endif
#endif /* TCSUM_H */
