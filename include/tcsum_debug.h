/*
 * tcsum_debug.h -- test and measurement controls of libtcsum.so.
 *
 * NOT for production callers.  These calls force which kernel the batch calls
 * of this PROCESS launch, so that the parity tests can run every shape the
 * router can pick and the measurement scripts can A/B them in one process.
 * Nothing in the environment changes a route: a stack process that inherits
 * stray variables runs exactly the router's choice.
 */
#ifndef TCSUM_DEBUG_H
#define TCSUM_DEBUG_H

#include <stdint.h>

#include "tcsum.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Set a knob; value -1 gives the choice back to the router.  Keys:
 *   "pf_dist"         descriptor prefetch distance, in workgroups, of the
 *                     packed kernel's range-by-range path (2048; 0 = off)
 *   "pf_range"        the same for the per-range kernels (0 = off)
 *   "page_stage"      0 / 1 (default 1): tcsum_host_batch_peso copies a
 *                     pageable arena through the context's pinned slots (0:
 *                     the runtime's own pageable copy, measurement only)
 *   "seg_sdesc"       0 / 1 (default 1): the per-range kernel with 8 or 16
 *                     lanes per range reads its wave's descriptors with
 *                     scalar loads, each lane group picking its own
 *   "pk_early"        0 / 1 (default 1): the packed kernel's range-by-range
 *                     path (a workgroup whose ranges are not one region, up
 *                     to 32 of them) reads its descriptors with scalar loads
 *                     -- lines its span check just cached -- instead of
 *                     vector loads through the L2; with 0, SHUFFLED batches
 *                     always take the per-range kernel
 *   "lanes", "loads"  per-range kernel shape (lanes per range x 16-B loads per
 *                     lane): one of the shapes the router picks -- 4x1, 4x2,
 *                     4x3, 8x3, 8x4, 16x3, 16x4, 16x6, 16x8, 32x6, 256x16,
 *                     1024x4; IPv4 calls: 2x4, 4x4, 8x3, 8x4, 8x6, 16x1..16x8,
 *                     32x6, 64x4, 64x16 (lanes clamped to 2..64); another
 *                     shape makes the batch call return TCSUM_ERR_PARAM
 *   "xcd"             workgroups per XCD run (1 = dispatch order)
 *   "packed"          0 / 1: checksum_peso / pktbuf_checksum16 batches on the
 *                     packed-stream kernel (k_segments_pk) off / on; K > 1: on,
 *                     with K ranges per workgroup (measurement)
 *   "tx_split"        0 / 1: the tx fill's stores in the kernel / deferred
 *   "tx_warm"         0 / 1: the deferred stores load each field's dword
 *                     first (packets in device memory; default 1)
 *   "args_launch"     0: drop-in calls pass their descriptor in pinned memory
 *   "sync_block"      1: drop-in calls block in hipStreamSynchronize
 *   "e2e_trace"       1: tcsum_host_batch_peso prints phase times on stderr
 *   "e2e_chunk_mb"    tcsum_host_batch_peso's copy chunk size
 *   "server_max"      largest host-queue batch the queue server takes (65536)
 *   "server_trace"    1: the queue server prints its phase stamps when stopped
 *   "server_idle_ms"  the resident servers stop after this long idle (10)
 *   "server_wgs"      queue server workgroups (64)
 *   "hostq_dma_kb"    host-queue batches spanning this much go through the
 *                     copy engine (262144)
 *   "hostq_dma_keep_mb" device arena kept between host-queue calls (256)
 *   "copy_threads"    host threads of a parallel gather / scatter (16; the
 *                     worker pool is sized once, at first use)
 * Only TCSUM_DEVICE and TCSUM_CALL_SERVER are read from the environment
 * (deployment choices for an unmodified drop-in stack); nothing there changes
 * a route or a tuning.
 * Returns TCSUM_OK, or TCSUM_ERR_PARAM for an unknown key. */
int tcsum_debug_set(const char *key, int64_t value);

/* The knob's value (-1 = the router's choice; -2 = unknown key).  Two
 * read-only keys: "scratch_reserved" (bytes the tx fill's scratch pool holds on
 * the calling thread's device) and "last_sys_error": the last HIP call that
 * failed under any TCSUM_ERR_SYS / TCSUM_ERR_MEM return of the library, as
 * step * 1000 + its hipError_t (0 = none yet).  Steps:
 *    1-17  tcsum_host_batch_peso (1 set device, 2-5 copies, 6-7 events,
 *          8 launch, 9 results copy, 10-11 stream syncs, 13-16 allocations,
 *          17 the pageable staging slots' events)
 *   20-25  device context init (any entry point that creates it)
 *   31-37  host-queue IPv4 batches (31 set device, 32-33 pinned staging,
 *          34-35 copy-engine pieces, 36 launch, 37 wait)
 *   40-49  queue / call server set-up, launch, stop
 *   50-54  tcsum_release (53: a stream did not drain, 54: the device sync);
 *          60-61 tcsum_host_register / unregister
 *   70     a device-resident batch call's launch */
int64_t tcsum_debug_get(const char *key);

/* The plan tcsum_host_batch_peso makes for a batch of n segments in an
 * arena of arena_bytes, without touching a device (host arithmetic only):
 * the copies and kernel launches it would queue, in queue order, as rows of
 * five u64 -- {0, buffer, host lo, host hi, buffer offset of lo} for a copy
 * of host bytes [lo, hi) into device buffer 0 (the lead's) or 1 (the
 * arena's), {1, buffer, i0, i1, arena offset of the buffer's byte 0} for a
 * kernel over segments [i0, i1) reading that buffer ({2, ...}: the same, the
 * segments out of offset order, so tcsum_batch's SHUFFLED route) -- at most max_rows of
 * them written; buf_bytes[0..1]: the two buffers' sizes (0: unused).  Uses
 * the "e2e_chunk_mb" knob like the call.  Returns the row count, or
 * TCSUM_ERR_PARAM (a segment outside the arena, as the call would). */
int64_t tcsum_debug_plan_host_peso(const tcsum_peso_t *segs, uint32_t n, uint64_t arena_bytes, uint64_t *rows,
                                   uint32_t max_rows, uint64_t *buf_bytes);

/* One shard of a multi-device host batch (tcsum_host_batch_peso_multi,
 * tcsum_host_batch_ipv4*_multi). */
typedef struct tcsum_shard_stat {
    int32_t device;  /* the devices[] entry that took it */
    int32_t rc;      /* its return code */
    uint32_t first;  /* descriptors [first, first + count) */
    uint32_t count;
    uint64_t bytes;  /* the shard's packet bytes */
    double ms;       /* wall time of the shard's call on its host thread */
} tcsum_shard_stat_t;

/* The shards of the last multi-device host batch of this process (any
 * thread), in devices[] order: up to max written to out; returns how many
 * there were (0 before the first). */
int tcsum_debug_shards(tcsum_shard_stat_t *out, int max);

/* The route a batch call would take for a mean range length, with the knobs
 * applied: out[0] lanes, out[1] loads, out[2] xcd, out[3] packed K (0 = off),
 * out[4] the packed K a TCSUM_LAYOUT_SHUFFLED batch of that mean takes (0:
 * the per-range kernel).  libtcsum_bench.so's probes follow it. */
void tcsum_debug_route(uint64_t mean_len, int32_t out[5]);

/* The k_ipv4 lane group an IPv4 batch of that mean packet length takes, with
 * the knobs applied: out[0] lanes per packet, out[1] loads per lane.
 * ip_mode: 0 sums, 1 tx fill, 2 rx verify, 3 tx offload. */
void tcsum_debug_ipv4_route(uint64_t mean_len, int ip_mode, int32_t out[2]);

#ifdef __cplusplus
}
#endif
#endif /* TCSUM_DEBUG_H */
