/*
 * tcsum_synth.h -- on-device synthetic packet batches and a read probe, for
 * tests and bench.py.
 *
 * Not part of the checksum path.  The byte stream is the one the CPU oracle
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
 * masking and sums).  lanes x loads in {16,32} x {4,6,8}, 64 x {4,8},
 * 256 x {4,8,16}; otherwise TCSUM_ERR_PARAM. */
int tcsum_probe_tile(const void *p /*[dev]*/, uint64_t nbytes, int lanes, int loads, uint32_t *sink /*[dev]*/,
                     void *stream);

#ifdef __cplusplus
}
#endif
#endif /* TCSUM_SYNTH_H */
