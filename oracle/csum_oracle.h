/*
 * csum_oracle.h -- CPU restatement of the reference's Internet-checksum path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is linked into, loaded by,
 * or called from the product library (tcp_amd/libtcsum.so).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as
 * the checker / the timed CPU baseline.
 *
 * Parity is PINNED: tests/test_oracle_golden.py checks every function below
 * against fixtures produced by the reference's own checksum16 / pktbuf_checksum16
 * / checksum_peso, compiled from /root/reference (oracle/Makefile, target
 * `golden`, generator oracle/golden_gen.c).
 *
 * Reference anchors (paths relative to the wj9806/tcp tree):
 *   checksum16          net/src/tools.c:24-54   (decl net/net/tools.h:45)
 *   checksum_peso       net/src/tools.c:56-75   (decl net/net/tools.h:47)
 *   pktbuf_checksum16   net/src/pktbuf.c:646-670 (decl net/net/pktbuf.h:229)
 *   IPv4 header verify  net/src/ipv4.c:220-250  (is_pkt_ok)
 */
#ifndef TCSUM_ORACLE_H
#define TCSUM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The block size of the reference's chained packet buffer (net/net/net_cfg.h:31). */
#define ORC_PKTBUF_BLK_SIZE 127

/* tools.c:24-54: one's-complement 16-bit sum of a flat range, u32 accumulator,
 * byte parity taken from `offset`, end-around-carry fold, optional complement. */
uint16_t orc_checksum16(int offset, const void *buf, uint16_t len,
                        uint32_t pre_sum, int complement);

/* One piece of a scatter-gather packet: the range a pktbuf block exposes. */
typedef struct orc_piece {
    const uint8_t *data;
    int size;
} orc_piece_t;

/* pktbuf.c:646-670 over an explicit piece list that starts at the cursor.
 * Returns 0 when len exceeds the bytes available (pktbuf.c:650-655). */
uint16_t orc_pieces_checksum16(const orc_piece_t *pieces, int npieces, int len,
                               int pre_sum, int complement);

/* pktbuf_checksum16 semantics over a contiguous range: the range is walked in
 * ORC_PKTBUF_BLK_SIZE pieces exactly as the reference stack walks its blocks
 * (the result does not depend on the split; the loop shape is kept for the
 * CPU baseline).  len may exceed 65535. */
uint16_t orc_flat_checksum16(const uint8_t *buf, uint64_t len, int pre_sum,
                             int complement);

/* tools.c:56-75: the pseudo-header partial (src, dst, {0,proto}, htons(len))
 * folded the way checksum_peso builds it.  len is truncated to 16 bits exactly
 * like x_htons(buf->total_size) (tools.c:69). */
uint16_t orc_pseudo_sum(const uint8_t src[4], const uint8_t dst[4],
                        uint8_t protocol, uint32_t len);

/* tools.c:56-75: checksum_peso over a contiguous L4 segment. */
uint16_t orc_checksum_peso(const uint8_t *seg, uint32_t len,
                           const uint8_t dest[4], const uint8_t src[4],
                           uint8_t protocol);

/* Batch descriptors shared with the product ABI (include/tcsum.h). */
typedef struct orc_seg {
    uint64_t offset;
    uint32_t len;
    uint32_t pre_sum;
} orc_seg_t;

typedef struct orc_peso {
    uint64_t offset;
    uint32_t len;
    uint8_t src[4];
    uint8_t dst[4];
    uint8_t protocol;
    uint8_t rsv[3];
} orc_peso_t;

typedef struct orc_pkt {
    uint64_t offset;
    uint32_t len;
    uint32_t rsv;
} orc_pkt_t;

/* Per-packet IPv4 result pair, as defined for tcsum_batch_ipv4 (include/tcsum.h):
 *   ip  = checksum16(0, hdr, ihl*4, 0, 1)                        (ipv4.c:243)
 *   l4  = checksum_peso(l4, dst, src, proto)  for TCP(6)/UDP(17)  (tcp_in.c:80, udp.c:410)
 *       = pktbuf_checksum16(l4, l4len, 0, 1)  for ICMP(1)          (icmpv4.c:36)
 *       = 0                                   for other protocols
 * flags: TCSUM_PKT_* bits (see include/tcsum.h) for what is_pkt_ok
 * (ipv4.c:220-239) would have rejected; lengths are clamped as documented. */
void orc_ipv4_pair(const uint8_t *pkt, uint32_t frame_len, uint16_t *ip_out,
                   uint16_t *l4_out, uint8_t *flags_out);

/* Batched tx fill of one packet, in place: zero the
 * checksum fields and store the values the stack's tx path stores:
 *   IPv4 header  ipv4.c:643,656  (every packet, fragments included)
 *   TCP          tcp_out.c:19-20 (non-fragments, L4 >= 20 B)
 *   UDP          udp.c:320-321   (non-fragments, L4 >= 8 B; 0 stays 0)
 *   ICMP         icmpv4.c:45-52  (non-fragments, L4 >= 4 B)
 * Nothing is written for a packet with SHORT/BAD_* flags.  Returns flags. */
uint8_t orc_ipv4_tx_fill(uint8_t *pkt, uint32_t frame_len);

/* Batched rx verify of one packet: the net_err_t the
 * reference's receive path returns from its size and checksum gates, in its
 * order -- ipv4_in/is_pkt_ok (ipv4.c:475-249), then for non-fragments
 * tcp_in (tcp_in.c:69-85), udp_in (udp.c:386-415, socket lookup not modelled),
 * icmpv4_in (icmpv4.c:29-43,71-77: its checksum test never fails, A10). */
int8_t orc_ipv4_rx_verify(const uint8_t *pkt, uint32_t frame_len, uint8_t *flags_out);

/* Batch forms over an arena; nthreads <= 1 runs on the calling thread. */
void orc_batch_segments(const uint8_t *arena, const orc_seg_t *segs, uint32_t n,
                        uint16_t *out, int complement, int nthreads);
void orc_batch_peso(const uint8_t *arena, const orc_peso_t *segs, uint32_t n,
                    uint16_t *out, int nthreads);
void orc_batch_ipv4(const uint8_t *arena, const orc_pkt_t *pkts, uint32_t n,
                    uint32_t *out, uint8_t *flags, int nthreads);
void orc_batch_ipv4_tx_fill(uint8_t *arena, const orc_pkt_t *pkts, uint32_t n,
                            uint8_t *flags, int nthreads);
void orc_batch_ipv4_rx_verify(const uint8_t *arena, const orc_pkt_t *pkts, uint32_t n,
                              int8_t *verdict, uint8_t *flags, int nthreads);

/* Synthetic data shared with the device generator (tcsum_synth_fill):
 * 64-bit word w of the stream is splitmix64(seed + w), stored little-endian. */
uint64_t orc_splitmix64(uint64_t x);
void orc_synth_fill(uint8_t *dst, uint64_t byte_offset, uint64_t nbytes,
                    uint64_t seed);

/* CPU baseline timer used by bench.py: runs `fn` (a checksum_peso-shaped
 * routine) over the segments with nthreads pthreads for at least min_seconds,
 * returns bytes/second (payload bytes only). */
typedef uint16_t (*orc_peso_fn)(const uint8_t *seg, uint32_t len,
                                const uint8_t dest[4], const uint8_t src[4],
                                uint8_t protocol);
double orc_time_peso(orc_peso_fn fn, const uint8_t *arena, const orc_peso_t *segs,
                     uint32_t n, int nthreads, double min_seconds,
                     uint64_t *checksum_of_checksums);
/* orc_time_peso, and each thread's own rate (bytes / its seconds) into
 * thread_rates[0..nthreads) when not NULL. */
double orc_time_peso_rates(orc_peso_fn fn, const uint8_t *arena, const orc_peso_t *segs,
                           uint32_t n, int nthreads, double min_seconds,
                           uint64_t *checksum_of_checksums, double *thread_rates);

#ifdef __cplusplus
}
#endif
#endif /* TCSUM_ORACLE_H */
