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

#ifdef __cplusplus
extern "C" {
#endif

/* Set a knob; value -1 gives the choice back to the router.  Keys:
 *   "lanes", "loads"  per-range kernel shape (lanes per range x 16-B loads per
 *                     lane): one of the shapes the router picks -- 4x1, 4x2,
 *                     8x4, 16x3, 16x4, 16x6, 16x8, 32x6, 256x16, 1024x4 (IPv4
 *                     calls: lanes clamped to 16..64); another shape makes the
 *                     batch call return TCSUM_ERR_PARAM
 *   "xcd"             workgroups per XCD run (1 = dispatch order)
 *   "packed"          0 / 1: checksum_peso / pktbuf_checksum16 batches on the
 *                     packed-stream kernel (k_segments_pk) off / on
 *   "flat"            0 / 1: the byte-window stream (k_flat_*) off / on
 *   "tx_split"        0 / 1: the tx fill's stores in the kernel / deferred
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
 * the calling thread's device) and "last_sys_error" (the last TCSUM_ERR_SYS
 * of tcsum_host_batch_peso: step * 1000 + the hipError_t; 0 = none). */
int64_t tcsum_debug_get(const char *key);

/* The route a batch call would take for a mean range length, with the knobs
 * applied: out[0] lanes, out[1] loads, out[2] xcd, out[3] packed K (0 = off),
 * out[4] flat (0/1).  libtcsum_bench.so's probes follow it. */
void tcsum_debug_route(uint64_t mean_len, int32_t out[5]);

#ifdef __cplusplus
}
#endif
#endif /* TCSUM_DEBUG_H */
