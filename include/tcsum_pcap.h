/*
 * tcsum_pcap.h -- capture-file helper, libtcsum_pcap.so.  NOT part of the
 * checksum path: host-only C++ (no GPU code), built
 * beside libtcsum.so so that frames recorded from the pcap driver's recv_thread
 * (plat/netif_pcap.c:9-38) can be handed to the host-queue batches of
 * include/tcsum.h in place.  Link with -ltcsum_pcap (and -ltcsum for the
 * batches).
 */
#ifndef TCSUM_PCAP_H
#define TCSUM_PCAP_H

#include "tcsum.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A libpcap savefile -- classic, or pcapng (Enhanced / Simple / obsolete
 * Packet Blocks; link type and FCS length per interface; any number of
 * sections, each in its own byte order) -- already in memory (mmap'd, read,
 * or copied to HBM as is) indexed into IPv4 batch descriptors that point INTO
 * the file:
 * the file is the arena, no bytes move.  Host code, no GPU needed.
 *   pkts[i]       frame i's IPv4 packet: offset = record data + link header,
 *                 len = captured bytes after it (an FCS the file declares is
 *                 not counted); len 0 when the frame is not for ipv4_in
 *   l2_verdict[i] (may be NULL) what the stack's rx front end does with the
 *                 frame before ipv4_in (plat/netif_pcap.c:9-38,
 *                 net/src/ether.c:14-25,62-101): TCSUM_OK -> ipv4_in;
 *                 TCSUM_PCAP_ARP -> arp_in (not this path); TCSUM_ERR_SIZE
 *                 (is_pkt_ok: < 14 or > 14 + 1500 bytes); TCSUM_ERR_NOT_SUPPORT
 *                 (other ethertype / family); raw-IP links hand every frame
 *                 to ipv4_in, whose gates judge it (SIZE, NOT_SUPPORT ...)
 * Link types: Ethernet (1, what netif_pcap captures), raw IPv4 (101, 228),
 * BSD loopback (0, AF_INET), Linux cooked (113); either byte order, us or ns
 * timestamps.  A record is the captured bytes (caplen): where the reference
 * copies pkthdr->len bytes (netif_pcap.c:23-30) from a shorter record, rx
 * verify sees the short frame (TCSUM_ERR_SIZE once total_len > captured).
 * *n_frames = records in the file.  Returns TCSUM_OK; TCSUM_ERR_MEM when
 * max_frames < records (the first max_frames are indexed; max_frames 0 and
 * pkts NULL = count only); TCSUM_ERR_SIZE when the file ends inside a record
 * (the whole records before it are indexed); TCSUM_ERR_PARAM for a file that
 * is not a savefile (or a corrupt pcapng block); TCSUM_ERR_NOT_SUPPORT for
 * another link type (pcapng: that interface's frames get it as l2_verdict). */
#define TCSUM_PCAP_ARP 1
int tcsum_pcap_index(const void *file /*[host]*/, uint64_t file_bytes, tcsum_pkt_t *pkts /*[host]*/,
                     int8_t *l2_verdict /*[host] or NULL*/, uint32_t max_frames, uint32_t *n_frames);

#ifdef __cplusplus
}
#endif
#endif /* TCSUM_PCAP_H */
