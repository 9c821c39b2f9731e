// Capture-file side of the rx path: a classic libpcap savefile in memory ->
// IPv4 batch descriptors that point INTO the file, so the file's bytes are
// the arena (mmap it and hand it to tcsum_host_batch_ipv4_rx_verify, or copy
// it to HBM as is and call tcsum_batch_ipv4_rx_verify).
//
// The stack's own rx front end this replaces for offline work:
//   plat/netif_pcap.c:9-38   recv_thread: pcap_next_ex, one pktbuf per frame
//   net/src/ether.c:14-25    is_pkt_ok: 14 <= size <= 14 + ETHER_MTU (1500)
//   net/src/ether.c:62-101   ether_in: 0x0806 -> arp_in, 0x0800 -> ipv4_in
//                            (header removed), anything else NOT_SUPPORT
// Host code only (no device work): the index is a sequential walk over the
// record headers, one pass, ~16 B touched per frame.
#include <stdint.h>
#include <string.h>

#include "tcsum.h"

namespace {

constexpr uint32_t kMagicUs = 0xA1B2C3D4u;
constexpr uint32_t kMagicNs = 0xA1B23C4Du;
constexpr uint64_t kFileHdr = 24;
constexpr uint64_t kRecHdr = 16;
constexpr uint32_t kEtherHdr = 14;   // ether_hdr_t (ether.h:20-25)
constexpr uint32_t kEtherMtu = 1500; // ETHER_MTU (ether.h:14)

inline uint32_t rd32(const uint8_t *p, bool swap)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return swap ? __builtin_bswap32(v) : v;
}

inline uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }

} // namespace

extern "C" int tcsum_pcap_index(const void *file, uint64_t file_bytes, tcsum_pkt_t *pkts, int8_t *l2_verdict,
                                uint32_t max_frames, uint32_t *n_frames)
{
    if (n_frames)
        *n_frames = 0;
    if (!file || !n_frames || (max_frames && !pkts))
        return TCSUM_ERR_PARAM;
    const uint8_t *f = static_cast<const uint8_t *>(file);
    if (file_bytes < kFileHdr)
        return TCSUM_ERR_PARAM;
    uint32_t magic;
    memcpy(&magic, f, 4);
    const bool swap = magic == __builtin_bswap32(kMagicUs) || magic == __builtin_bswap32(kMagicNs);
    if (!swap && magic != kMagicUs && magic != kMagicNs)
        return TCSUM_ERR_PARAM; // not a classic savefile (pcapng is not read here)
    // LinkType and FCS information (bits 0-15 type, 26 F, 28-31 FCS length
    // in 16-bit units)
    const uint32_t link = rd32(f + 20, swap);
    const uint32_t type = link & 0xFFFFu;
    const uint32_t fcs = (link & (1u << 26)) ? 2u * (link >> 28) : 0u;
    enum { ETHER, RAW, NUL, SLL } kind;
    if (type == 1)
        kind = ETHER; // LINKTYPE_ETHERNET: what netif_pcap opens (pcap_open_live on a NIC)
    else if (type == 101 || type == 228)
        kind = RAW; // LINKTYPE_RAW / LINKTYPE_IPV4: the IPv4 header is the first byte
    else if (type == 0)
        kind = NUL; // LINKTYPE_NULL: 4-byte address family in the writer's byte order
    else if (type == 113)
        kind = SLL; // LINKTYPE_LINUX_SLL: 16-byte cooked header, protocol at 14..15
    else
        return TCSUM_ERR_NOT_SUPPORT;

    uint64_t pos = kFileHdr;
    uint32_t i = 0;
    int rc = TCSUM_OK;
    while (pos < file_bytes) {
        if (file_bytes - pos < kRecHdr) {
            rc = TCSUM_ERR_SIZE; // a partial record header at the end
            break;
        }
        const uint32_t caplen = rd32(f + pos + 8, swap);
        const uint64_t data = pos + kRecHdr;
        if (caplen > file_bytes - data) {
            rc = TCSUM_ERR_SIZE; // the last record's bytes are cut short
            break;
        }
        pos = data + caplen;
        if (i >= max_frames) { // count only
            ++i;
            continue;
        }
        // the frame as the capture holds it (recv_thread copies pkthdr->len
        // bytes, netif_pcap.c:23-30; only caplen of them exist in a record)
        const uint32_t frame = caplen >= fcs ? caplen - fcs : 0u;
        const uint8_t *p = f + data;
        uint32_t l2 = 0;
        int v = TCSUM_OK;
        switch (kind) {
        case ETHER:
            l2 = kEtherHdr;
            if (frame < kEtherHdr || frame > kEtherHdr + kEtherMtu)
                v = TCSUM_ERR_SIZE; // is_pkt_ok, ether.c:14-25
            else if (be16(p + 12) == 0x0806)
                v = TCSUM_PCAP_ARP; // arp_in, ether.c:76-84: not this path
            else if (be16(p + 12) != 0x0800)
                v = TCSUM_ERR_NOT_SUPPORT; // ether.c:95-97
            break;
        case RAW: // every frame goes to ipv4_in, whose gates sort out short
            break; // frames (SIZE) and IPv6 (NOT_SUPPORT, ipv4.c:222)
        case NUL:
            l2 = 4;
            if (frame < 4)
                v = TCSUM_ERR_SIZE;
            else if (rd32(p, swap) != 2u) // AF_INET
                v = TCSUM_ERR_NOT_SUPPORT;
            break;
        case SLL:
            l2 = 16;
            if (frame < 16)
                v = TCSUM_ERR_SIZE;
            else if (be16(p + 14) == 0x0806)
                v = TCSUM_PCAP_ARP;
            else if (be16(p + 14) != 0x0800)
                v = TCSUM_ERR_NOT_SUPPORT;
            break;
        }
        tcsum_pkt_t &d = pkts[i];
        d.offset = data + (v == TCSUM_OK ? l2 : 0u);
        d.len = v == TCSUM_OK ? frame - l2 : 0u;
        d.rsv = 0;
        if (l2_verdict)
            l2_verdict[i] = (int8_t)v;
        ++i;
    }
    *n_frames = i;
    if (rc == TCSUM_OK && i > max_frames)
        rc = TCSUM_ERR_MEM; // *n_frames = records in the file; max_frames of them indexed
    return rc;
}
