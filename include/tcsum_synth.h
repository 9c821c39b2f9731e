/*
 * tcsum_synth.h -- libtcsum_bench.so: on-device synthetic packet batches and
 * the load probes, for tests and bench.py.
 *
 * Not part of the checksum path: a separate library (tcp_amd/csrc/
 * bench_kernels.hip), so that libtcsum.so holds only the kernels its router
 * launches.  The byte stream is the one the CPU oracle
 * reproduces (oracle/csum_oracle.c: orc_synth_fill): byte p of the stream is
 * byte (p & 7) of splitmix64(seed + (p >> 3)), so host and device see the same
 * packets without a transfer.
 */
#ifndef TCSUM_SYNTH_H
#define TCSUM_SYNTH_H

#include <stdint.h>

#include "tcsum.h"

#ifdef __cplusplus
extern "C" {
#endif

/* arena[0 .. nbytes) := stream bytes [byte_base, byte_base + nbytes).
 * arena must be 16-byte aligned and byte_base a multiple of 16. */
int tcsum_synth_fill(void *arena /*[dev]*/, uint64_t nbytes, uint64_t byte_base,
                     uint64_t seed, void *stream);

/* Overwrite the first 20 bytes of every packet with an IPv4 header:
 * version 4, IHL 5, total_len = pkts[i].len, TTL 64, protocol TCP or UDP
 * (from the hash of seed and i), header checksum 0 (tx form), random src/dst;
 * and, in packets of >= 40 bytes, the L4 fields the receive gates read:
 * nonzero ports, TCP data offset 5 with ACK (PSH half the time), UDP length.
 * Checksum fields are left as stream bytes (the tx fill zeroes them).
 * Packets shorter than 20 bytes are left alone. */
int tcsum_synth_ipv4(void *arena /*[dev]*/, const tcsum_pkt_t *pkts /*[dev]*/, uint32_t n,
                     uint64_t seed, void *stream);

/* Stream-read nbytes (rounded down to 16) with the checksum kernels' load
 * shape and nothing else: the measured "achievable" HBM read rate for the
 * roofline.  sink: one device u32 (written only on a 2^-32 fluke). */
int tcsum_probe_read(const void *p /*[dev]*/, uint64_t nbytes, uint32_t *sink /*[dev]*/, void *stream);

/* The same plain read in the product kernels' own tile shape: `lanes` lanes
 * share a unit of lanes*loads consecutive 16-B chunks (lane l loads chunks
 * u*lanes + l), 256/lanes units per workgroup, workgroups in the product's
 * XCD-grouped order (k_segments / k_ipv4 / k_segments_wg minus descriptors,
 * masking and sums).  dep != 0: each unit's loads wait behind one dependent
 * 16-B read, as the product's wait for their descriptor.  lanes x loads in
 * {16,32} x {4,6,8}, 64 x {4,8}, 256 x {4,8,16}; otherwise TCSUM_ERR_PARAM. */
int tcsum_probe_tile(const void *p /*[dev]*/, uint64_t nbytes, int lanes, int loads, int dep,
                     uint32_t *sink /*[dev]*/, void *stream);

/* tcsum_batch_peso's loads and nothing else: the same descriptors, lanes,
 * edge / interior cache policies and workgroup order, with the sums, the
 * reduction and the result store replaced by an XOR fold -- the rate the
 * checksum kernel would run at if its arithmetic were free.  It follows the
 * route libtcsum.so's router takes (tcsum_debug_route): the packed stream,
 * the TSO workgroup shape or a per-range shape. */
int tcsum_probe_segments(const void *arena /*[dev]*/, const tcsum_peso_t *segs /*[dev]*/, uint32_t n,
                         uint64_t total_bytes_hint, uint32_t *sink /*[dev]*/, void *stream);

/* The same for the IPv4 batch calls: tcsum_batch_ipv4's descriptor, header
 * and line-aligned data loads, XOR-folded, nothing stored but the fluke sink
 * (mode 0).  mode 1: tcsum_batch_ipv4_rx_verify's (two more header chunks,
 * its lane count).  mode 2, the ceiling for the tx fill, which must write:
 * mode 0's loads plus exactly the deferred fill's writes -- 8 bytes of scratch
 * per packet (a value and the field positions, derived from the header by the
 * fill's own rules) and then the fill's k_tx_scatter storing the fields; the
 * stored values are the XOR fold, so every IPv4 / L4 checksum field of the
 * batch is left holding junk (the arena is written despite the const).
 * The per-packet shape k_ipv4 takes for the mean length. */
int tcsum_probe_ipv4(const void *arena /*[dev]*/, const tcsum_pkt_t *pkts /*[dev]*/, uint32_t n,
                     uint64_t total_bytes_hint, int mode, uint32_t *sink /*[dev]*/, void *stream);

/* The byte-window stream (k_flat_plan + k_flat_ipv4, tcsum_batch_ipv4's
 * sums) in a workgroup shape of `waves` x `loads` (4x3, 8x3, 8x4, 16x4, 16x2),
 * for A/Bs: variant 0 = the product's arithmetic (out/flags as
 * tcsum_batch_ipv4); 1 = the plan and the windows' loads only; 2 = + the
 * prefix scans into LDS; 3 = everything but the combine of packets that
 * cross windows (their values are then wrong).  out: out_words u32, at
 * least n for variants 0 and 3 (they write every packet's word; fewer:
 * TCSUM_ERR_PARAM), a one-word sink for 1 and 2; flags may be NULL. */
int tcsum_probe_flat(const void *arena /*[dev]*/, const tcsum_pkt_t *pkts /*[dev]*/, uint32_t n,
                     uint64_t total_bytes, int variant, int waves, int loads, uint32_t *out /*[dev]*/,
                     uint64_t out_words, uint8_t *flags /*[dev] or NULL*/, void *stream);

/* The byte-window stream (k_flat_plan + k_flat_ipv4, 4 waves x 3 loads: 12-KiB
 * windows) in every IPv4 mode -- round 4's candidate for configs[3], exact
 * but slower than the route (k_ipv4), kept here for A/Bs and its parity tests
 * (tests/test_gpu_flat.py).  mode: 0 sums (out required, flags or NULL), 1 tx
 * fill in place, 2 rx verify (verdict required), 3 tx offload (out and flags
 * required), 4 tx fill with deferred stores -- the arguments of the matching
 * tcsum_batch_ipv4* call.  total_bytes (the sum of the lengths) sizes the
 * windows; a batch that is not a stream (descriptors out of arena order,
 * overlaps, a span the total does not cover) is summed packet by packet in
 * the same launch.  Allocates its plan with hipMallocAsync on the stream. */
int tcsum_flat_ipv4(int mode, void *arena /*[dev]*/, const tcsum_pkt_t *pkts /*[dev]*/, uint32_t n,
                    uint64_t total_bytes, uint32_t *out /*[dev] or NULL*/, uint8_t *flags /*[dev] or NULL*/,
                    int8_t *verdict /*[dev] or NULL*/, void *stream);

/* The tx fill's design-independent floor: read every byte of arena[0,
 * nbytes) once and write each packet's two 2-byte checksum fields at the
 * addresses the fill writes, with no descriptors, parse or sums.
 * tcsum_probe_txfloor_prepare (outside any measurement) derives them with
 * the fill's field rules: side = 2n u32 scratch (values, then positions),
 * fpos = 2n u64 field offsets from the arena (~0: none), ffirst =
 * tcsum_probe_txfloor_windows(nbytes) + 1 u32 (first packet of each 16-KiB
 * window; pkts in arena order).  tcsum_probe_txfloor: variant 0 = the stores
 * in-stream (each window's workgroup writes its packets' fields after its
 * loads), 1 = deferred (the plain read, then one dense scatter of side's
 * values).  The fields are left junk. */
/* An IPv4 batch in launch forms the route does not take (measurement): mode 0
 * = tcsum_batch_ipv4's sums by k_ipv4<32, 6> (out), mode 2 = rx verify by
 * k_ipv4<16, 6> (verdict, and the sums into out), in wg = 256 / 512 / 1024
 * thread workgroups (rx: 256 / 1024), or with wg = 256 held to occ waves per
 * SIMD (sums: 8; rx: 7 or 8; 0 = as built), or (occ = 100 + s, wg = 256)
 * with its data pass starting s bytes past a 128-B line instead of on one
 * (sums: s = 16, 64; rx: 16), or (occ = 200) two data passes in flight, or
 * (occ = 300 + M, wg = 256; sums M = 2, 4, 8, 16, rx 2, 4, 8) M packets per
 * lane group handed out inside the workgroup (k_ipv4_dyn), or (occ = 500 +
 * v) the rolling load slots (each slot reissued for the next pass as soon as
 * its chunk is taken): v = 0 the mode's shape, 4 = 4 loads, sums 8 = 8 loads,
 * 16 = 16 lanes x 6, rx 32 = 32 lanes x 6, sums 7 / rx 6 = the mode's shape
 * held to that many waves per SIMD; or (occ = 600) no header loads, the
 * header chunks shuffled from the first data pass, or (occ = 700) the
 * descriptors by scalar loads.  Others:
 * TCSUM_ERR_PARAM. */
int tcsum_probe_ipv4_shape(void *arena /*[dev]*/, const tcsum_pkt_t *pkts /*[dev]*/, uint32_t n, int mode, int wg,
                           int occ, uint32_t *out /*[dev]*/, int8_t *verdict /*[dev] or NULL*/, void *stream);

/* The byte-window stream's load phase alone (measurement): waves x loads in
 * {16x4, 8x4, 4x3}, one window per workgroup, XOR-folded into sink; dep = what
 * the loads wait for: 0 nothing, 1 one shared scalar word, 2 two dependent
 * shared 16-B loads (word[0..3], all 0), 3 a 24-B descriptor per
 * workgroup (descs: ndescs >= the grid's count, offsets < 2^63); 4 the
 * window's chunks shifted 16 B past its boundary, 5 default-policy loads of
 * its first and last chunk beside them, 6 both, 7 both behind the descriptor
 * (k_segments_wgx's own pattern). */
int tcsum_probe_window(const void *p /*[dev]*/, uint64_t nbytes, int waves, int loads, int dep,
                       const uint64_t *word /*[dev]*/, const void *descs /*[dev]*/, uint64_t ndescs,
                       uint32_t *sink /*[dev]*/, void *stream);

uint32_t tcsum_probe_txfloor_windows(uint64_t nbytes);
int tcsum_probe_txfloor_prepare(const void *arena /*[dev]*/, uint64_t nbytes, const tcsum_pkt_t *pkts /*[dev]*/,
                                uint32_t n, uint64_t total_bytes_hint, uint32_t *side /*[dev]*/, uint64_t side_words,
                                uint64_t *fpos /*[dev]*/, uint64_t fpos_words, uint32_t *ffirst /*[dev]*/,
                                uint64_t ffirst_words, void *stream);
int tcsum_probe_txfloor(void *arena /*[dev]*/, uint64_t nbytes, const uint64_t *fpos /*[dev]*/,
                        const uint32_t *side /*[dev]*/, uint32_t n, const uint32_t *ffirst /*[dev]*/, int variant,
                        uint32_t *sink /*[dev]*/, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* TCSUM_SYNTH_H */
