// Capture-file side of the rx path: a libpcap savefile (classic or pcapng) in memory ->
// IPv4 batch descriptors that point INTO the file, so the file's bytes are
// the arena (mmap it and hand it to tcsum_host_batch_ipv4_rx_verify, or copy
// it to HBM as is and call tcsum_batch_ipv4_rx_verify).
//
// The stack's own rx front end this replaces for offline work:
//   plat/netif_pcap.c:9-38   recv_thread: pcap_next_ex, one pktbuf per frame
//   net/src/ether.c:14-25    is_pkt_ok: 14 <= size <= 14 + ETHER_MTU (1500)
//   net/src/ether.c:62-101   ether_in: 0x0806 -> arp_in, 0x0800 -> ipv4_in
//                            (header removed), anything else NOT_SUPPORT
// Host code only (no device work): a walk over the record headers, ~16 B
// touched per frame, in parallel pieces for large files (see below).
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "tcsum_pcap.h"

namespace {

constexpr uint32_t kMagicUs = 0xA1B2C3D4u;
constexpr uint32_t kMagicNs = 0xA1B23C4Du;
constexpr uint64_t kFileHdr = 24;
constexpr uint64_t kRecHdr = 16;
constexpr uint32_t kEtherHdr = 14;   // ether_hdr_t (ether.h:20-25)
constexpr uint32_t kEtherMtu = 1500; // ETHER_MTU (ether.h:14)
constexpr uint32_t kMaxCap = 262144;  // libpcap's largest snapshot length
constexpr int kSyncRun = 8;           // consecutive plausible headers that make a sync point
constexpr uint64_t kPieceMin = 16ull << 20; // bytes per piece, at least
constexpr unsigned kChains = 4;             // pieces one walker thread interleaves

inline uint32_t rd32(const uint8_t *p, bool swap)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return swap ? __builtin_bswap32(v) : v;
}

inline uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }

inline uint16_t rd16(const uint8_t *p, bool swap)
{
    uint16_t v;
    memcpy(&v, p, 2);
    return swap ? __builtin_bswap16(v) : v;
}

enum Link { L_ETHER, L_RAW, L_NULL, L_SLL, L_OTHER };

// LINKTYPE_* value -> the kinds read here
Link link_kind(uint32_t type)
{
    switch (type) {
    case 1: // LINKTYPE_ETHERNET: what netif_pcap opens (pcap_open_live on a NIC)
        return L_ETHER;
    case 101: // LINKTYPE_RAW
    case 228: // LINKTYPE_IPV4: the IPv4 header is the first byte
        return L_RAW;
    case 0: // LINKTYPE_NULL: 4-byte address family in the writer's byte order
        return L_NULL;
    case 113: // LINKTYPE_LINUX_SLL: 16-byte cooked header, protocol at 14..15
        return L_SLL;
    default:
        return L_OTHER;
    }
}

// One captured frame (`caplen` bytes at file offset `data`, `fcs` trailing
// FCS bytes) -> its IPv4 descriptor and the rx front end's decision.
int8_t classify(const uint8_t *f, uint64_t data, uint32_t caplen, Link kind, uint32_t fcs, bool swap,
                tcsum_pkt_t &d)
{
    // the frame as the capture holds it (recv_thread copies pkthdr->len
    // bytes, netif_pcap.c:23-30; only caplen of them exist in a record)
    const uint32_t frame = caplen >= fcs ? caplen - fcs : 0u;
    const uint8_t *p = f + data;
    uint32_t l2 = 0;
    int v = TCSUM_OK;
    switch (kind) {
    case L_ETHER:
        l2 = kEtherHdr;
        if (frame < kEtherHdr || frame > kEtherHdr + kEtherMtu)
            v = TCSUM_ERR_SIZE; // is_pkt_ok, ether.c:14-25
        else if (be16(p + 12) == 0x0806)
            v = TCSUM_PCAP_ARP; // arp_in, ether.c:76-84: not this path
        else if (be16(p + 12) != 0x0800)
            v = TCSUM_ERR_NOT_SUPPORT; // ether.c:95-97
        break;
    case L_RAW: // every frame goes to ipv4_in, whose gates sort out short
        break;  // frames (SIZE) and IPv6 (NOT_SUPPORT, ipv4.c:222)
    case L_NULL:
        l2 = 4;
        if (frame < 4)
            v = TCSUM_ERR_SIZE;
        else if (rd32(p, swap) != 2u) // AF_INET
            v = TCSUM_ERR_NOT_SUPPORT;
        break;
    case L_SLL:
        l2 = 16;
        if (frame < 16)
            v = TCSUM_ERR_SIZE;
        else if (be16(p + 14) == 0x0806)
            v = TCSUM_PCAP_ARP;
        else if (be16(p + 14) != 0x0800)
            v = TCSUM_ERR_NOT_SUPPORT;
        break;
    case L_OTHER: // a pcapng interface of a link type not read here
        v = TCSUM_ERR_NOT_SUPPORT;
        break;
    }
    d.offset = data + (v == TCSUM_OK ? l2 : 0u);
    d.len = v == TCSUM_OK ? frame - l2 : 0u;
    d.rsv = 0;
    return (int8_t)v;
}

// ------------------------------------------------------------ parallel walk
//
// A capture is a chain of records (classic) or blocks (pcapng): each header
// gives the next one's position, and walking it is one dependent cache + TLB
// miss per record (~0.45 us over a multi-GiB file).  Large files are cut into
// K pieces, kChains of them per walker thread, walked with their chains
// interleaved (their misses overlap); the walker of piece t > 0 first finds a
// record boundary at or after the piece's start by looking for kSyncRun
// consecutive plausible headers.  The stitch accepts a piece only if its sync
// point is exactly where the exact walk of the pieces before it ended, and
// re-walks it from there otherwise, so the result is the sequential walk's.
enum StepResult { S_FRAME, S_SKIP, S_TRUNC, S_BAD, S_SEQ };

struct Frame {
    uint64_t data = 0, next = 0;
    uint32_t caplen = 0, iface = 0;
};

constexpr int kNeedSeq = 100; // a piece met a block only a sequential walk may interpret

// Step:      StepResult(uint64_t pos, Frame &)   one record at pos
// Plausible: bool(uint64_t pos, uint64_t &next)   could a record start at pos?
// Classify:  int8_t(const Frame &, tcsum_pkt_t &) descriptor + front-end verdict
template <class Step, class Plausible, class Classify>
struct Walker {
    const uint8_t *f;
    uint64_t file_bytes, body; // records start at `body`
    Step step;
    Plausible plausible;
    Classify classify;

    struct Piece {
        uint64_t begin = 0, end = 0; // first record walked / first record at or past the piece end
        std::vector<tcsum_pkt_t> pk;
        std::vector<int8_t> v;
        int rc = TCSUM_OK;
        bool synced = false;
    };

    // Walk pieces [a, b) to their ends, one record of each per round.
    void walk(Piece *pcs, const uint64_t *start, const uint64_t *stop, unsigned a, unsigned b) const
    {
        uint64_t pos[kChains];
        bool live[kChains];
        unsigned left = 0;
        for (unsigned j = a; j < b; ++j) {
            Piece &pc = pcs[j];
            pc.begin = pos[j - a] = start[j];
            pc.pk.clear();
            pc.v.clear();
            pc.rc = TCSUM_OK;
            live[j - a] = pc.synced;
            left += pc.synced;
            if (!pc.synced)
                pc.end = pc.begin;
        }
        while (left) {
            for (unsigned j = a; j < b; ++j) {
                if (!live[j - a])
                    continue;
                Piece &pc = pcs[j];
                uint64_t &q = pos[j - a];
                bool done = q >= stop[j] || q >= file_bytes;
                if (!done) {
                    Frame fr;
                    const StepResult r = step(q, fr);
                    if (r == S_FRAME || r == S_SKIP) {
                        if (r == S_FRAME) {
                            tcsum_pkt_t d;
                            pc.v.push_back(classify(fr, d));
                            pc.pk.push_back(d);
                        }
                        q = fr.next;
                        __builtin_prefetch(f + std::min(q + 8, file_bytes - 1));
                    } else {
                        pc.rc = r == S_TRUNC ? TCSUM_ERR_SIZE : r == S_BAD ? TCSUM_ERR_PARAM : kNeedSeq;
                        done = true;
                    }
                }
                if (done) {
                    pc.end = q;
                    live[j - a] = false;
                    --left;
                }
            }
        }
    }

    bool sync(uint64_t from, uint64_t limit, uint64_t &at) const
    {
        for (uint64_t p = from; p < limit && p < file_bytes; ++p) {
            uint64_t q = p, next = 0;
            int k = 0;
            while (k < kSyncRun && q < file_bytes && plausible(q, next)) {
                q = next;
                ++k;
            }
            if (k == kSyncRun || (k > 0 && q == file_bytes)) {
                at = p;
                return true;
            }
        }
        return false;
    }

    int run(tcsum_pkt_t *pkts, int8_t *l2_verdict, uint32_t max_frames, uint32_t *n_frames) const
    {
        const uint64_t span = file_bytes > body ? file_bytes - body : 0;
        uint64_t piece_min = kPieceMin; // TCSUM_PCAP_PIECE_KB overrides (tests: many pieces on small files)
        if (const char *e = getenv("TCSUM_PCAP_PIECE_KB"))
            piece_min = std::max<uint64_t>(1, strtoull(e, nullptr, 10)) << 10;
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        const unsigned T0 = std::min(16u, hw);
        const unsigned K = (unsigned)std::min<uint64_t>(T0 * kChains, std::max<uint64_t>(1, span / piece_min));
        const unsigned T = (K + kChains - 1) / kChains; // walker threads, kChains pieces each
        std::vector<uint64_t> cut(K + 1), start(K, body);
        for (unsigned t = 0; t <= K; ++t)
            cut[t] = body + span * t / K;
        std::vector<Piece> pcs(K);
        {
            std::vector<std::thread> th;
            for (unsigned t = 0; t < T; ++t) {
                auto job = [&, t] {
                    const unsigned a = t * kChains, b = std::min(K, a + kChains);
                    for (unsigned j = a; j < b; ++j)
                        pcs[j].synced = j == 0 || sync(cut[j], cut[j + 1], start[j]);
                    walk(pcs.data(), start.data(), cut.data() + 1, a, b);
                };
                if (t + 1 < T)
                    th.emplace_back(job);
                else
                    job();
            }
            for (auto &x : th)
                x.join();
        }
        // stitch: piece 0 is exact; each later piece must start where the
        // exact walk so far ended
        uint64_t pos = pcs[0].end;
        int rc = pcs[0].rc;
        for (unsigned t = 1; t < K && rc == TCSUM_OK; ++t) {
            Piece &pc = pcs[t];
            if (!(pc.synced && pc.begin == pos)) { // a false or missing sync point: walk it exactly
                pc.synced = true;
                start[t] = pos;
                walk(pcs.data(), start.data(), cut.data() + 1, t, t + 1);
            }
            pos = pc.end;
            rc = pc.rc;
        }
        if (rc == TCSUM_ERR_PARAM || rc == kNeedSeq)
            return rc;
        uint64_t count = 0;
        unsigned last = K;
        for (unsigned t = 0; t < K; ++t) {
            count += pcs[t].pk.size();
            if (pcs[t].rc != TCSUM_OK) {
                last = t + 1; // the file ends inside this piece's last record
                break;
            }
        }
        uint64_t i = 0;
        for (unsigned t = 0; t < last && i < max_frames; ++t) {
            const Piece &pc = pcs[t];
            const size_t m = (size_t)std::min<uint64_t>(pc.pk.size(), max_frames - i);
            if (!m)
                continue;
            memcpy(pkts + i, pc.pk.data(), m * sizeof(tcsum_pkt_t));
            if (l2_verdict)
                memcpy(l2_verdict + i, pc.v.data(), m);
            i += m;
        }
        *n_frames = (uint32_t)std::min<uint64_t>(count, UINT32_MAX);
        if (rc == TCSUM_OK && count > max_frames)
            rc = TCSUM_ERR_MEM; // *n_frames = records in the file; max_frames of them indexed
        return rc;
    }
};

template <class S, class P, class C>
Walker<S, P, C> make_walker(const uint8_t *f, uint64_t file_bytes, uint64_t body, S step, P plausible, C classify)
{
    return Walker<S, P, C>{f, file_bytes, body, step, plausible, classify};
}

// pcapng (block types: pcapng spec) -- one sequential walk over the blocks:
// a Section Header Block sets the byte order and clears the interface table,
// Interface Description Blocks add link type + FCS length, and Enhanced /
// Simple / obsolete Packet Blocks are frames; other blocks are skipped.
constexpr uint32_t kShb = 0x0A0D0D0Au, kIdb = 1, kPb = 2, kSpb = 3, kEpb = 6;

struct Iface {
    Link kind;
    uint32_t fcs, snaplen;
};

int pcapng_index_seq(const uint8_t *f, uint64_t file_bytes, tcsum_pkt_t *pkts, int8_t *l2_verdict,
                     uint32_t max_frames, uint32_t *n_frames)
{
    bool swap = false;
    std::vector<Iface> ifs;
    uint64_t pos = 0, count = 0;
    int rc = TCSUM_OK;
    while (pos < file_bytes) {
        if (file_bytes - pos < 12) {
            rc = TCSUM_ERR_SIZE; // the file ends inside a block header
            break;
        }
        uint32_t type;
        memcpy(&type, f + pos, 4); // the SHB type is a palindrome: no byte order needed
        if (type == kShb) {
            const uint32_t bom = rd32(f + pos + 8, false);
            if (bom == 0x1A2B3C4Du)
                swap = false;
            else if (bom == 0x4D3C2B1Au)
                swap = true;
            else
                return TCSUM_ERR_PARAM;
            ifs.clear();
        } else if (pos == 0) {
            return TCSUM_ERR_PARAM;
        }
        type = rd32(f + pos, swap);
        const uint32_t len = rd32(f + pos + 4, swap);
        if (len < 12 || (len & 3u))
            return TCSUM_ERR_PARAM; // not a pcapng block
        if (len > file_bytes - pos) {
            rc = TCSUM_ERR_SIZE; // the file ends inside this block
            break;
        }
        if (rd32(f + pos + len - 4, swap) != len)
            return TCSUM_ERR_PARAM; // leading and trailing lengths differ: corrupt
        const uint8_t *b = f + pos;
        if (type == kIdb && len >= 20) {
            Iface in{link_kind(rd16(b + 8, swap)), 0, rd32(b + 12, swap)};
            for (uint64_t o = 16; o + 4 <= (uint64_t)len - 4;) { // options: code, length, value (4-byte padded)
                const uint16_t code = rd16(b + o, swap), olen = rd16(b + o + 2, swap);
                if (code == 0)
                    break;
                if (code == 13 && olen >= 1 && o + 4 + olen <= (uint64_t)len - 4) // if_fcslen: bits in
                    in.fcs = b[o + 4] >= 8 ? b[o + 4] / 8u : b[o + 4]; // the spec (16, 32); writers using bytes give 2, 4
                o += 4 + ((olen + 3u) & ~3u);
            }
            ifs.push_back(in);
        } else if (type == kEpb || type == kPb || type == kSpb) {
            uint32_t iface = 0, caplen;
            uint64_t data;
            if (type == kSpb) {
                data = pos + 12;
                const uint32_t orig = len >= 16 ? rd32(b + 8, swap) : 0u;
                caplen = std::min<uint32_t>(orig, len - 16);
                if (!ifs.empty() && ifs[0].snaplen)
                    caplen = std::min(caplen, ifs[0].snaplen);
            } else {
                if (len < 32)
                    return TCSUM_ERR_PARAM;
                iface = type == kEpb ? rd32(b + 8, swap) : rd16(b + 8, swap);
                caplen = rd32(b + 20, swap);
                data = pos + 28;
                if (caplen > len - 32)
                    return TCSUM_ERR_PARAM;
            }
            if (count < max_frames) {
                const Iface in = iface < ifs.size() ? ifs[iface] : Iface{L_OTHER, 0, 0};
                const int8_t v = classify(f, data, caplen, in.kind, in.fcs, swap, pkts[count]);
                if (l2_verdict)
                    l2_verdict[count] = v;
            }
            ++count;
        }
        pos += len;
    }
    *n_frames = (uint32_t)std::min<uint64_t>(count, UINT32_MAX);
    if (rc == TCSUM_OK && count > max_frames)
        rc = TCSUM_ERR_MEM;
    return rc;
}

// Large single-section files: the header blocks (SHB, IDBs) are read first;
// from the first packet block on, the blocks are walked in parallel pieces
// (a block's leading and trailing lengths must agree, so a sync point is
// hard to fake).  A piece that meets another SHB or IDB hands the whole file
// to the sequential walk, which interprets them in order.
int pcapng_index(const uint8_t *f, uint64_t file_bytes, tcsum_pkt_t *pkts, int8_t *l2_verdict,
                 uint32_t max_frames, uint32_t *n_frames)
{
    if (file_bytes < 28)
        return pcapng_index_seq(f, file_bytes, pkts, l2_verdict, max_frames, n_frames);
    const uint32_t bom = rd32(f + 8, false);
    if (bom != 0x1A2B3C4Du && bom != 0x4D3C2B1Au)
        return TCSUM_ERR_PARAM;
    const bool swap = bom == 0x4D3C2B1Au;
    std::vector<Iface> ifs;
    uint64_t body = 0;
    for (;;) { // header region: the SHB, then blocks up to the first packet block
        if (file_bytes - body < 12)
            return pcapng_index_seq(f, file_bytes, pkts, l2_verdict, max_frames, n_frames);
        const uint32_t type = rd32(f + body, swap), len = rd32(f + body + 4, swap);
        if (len < 12 || (len & 3u) || len > file_bytes - body || (body > 0 && type == kShb) ||
            rd32(f + body + len - 4, swap) != len) // the walk's own checks decide (ERR_PARAM, SIZE)
            return pcapng_index_seq(f, file_bytes, pkts, l2_verdict, max_frames, n_frames);
        if (type == kEpb || type == kPb || type == kSpb)
            break;
        if (type == kIdb && len >= 20) {
            Iface in{link_kind(rd16(f + body + 8, swap)), 0, rd32(f + body + 12, swap)};
            for (uint64_t o = 16; o + 4 <= (uint64_t)len - 4;) { // options: code, length, value (4-byte padded)
                const uint16_t code = rd16(f + body + o, swap), olen = rd16(f + body + o + 2, swap);
                if (code == 0)
                    break;
                if (code == 13 && olen >= 1 && o + 4 + olen <= (uint64_t)len - 4) // if_fcslen, as in the walk
                    in.fcs = f[body + o + 4] >= 8 ? f[body + o + 4] / 8u : f[body + o + 4];
                o += 4 + ((olen + 3u) & ~3u);
            }
            ifs.push_back(in);
        }
        body += len;
    }
    uint64_t piece_min = kPieceMin;
    if (const char *e = getenv("TCSUM_PCAP_PIECE_KB"))
        piece_min = std::max<uint64_t>(1, strtoull(e, nullptr, 10)) << 10;
    if (file_bytes - body < 2 * piece_min) // small: one walk
        return pcapng_index_seq(f, file_bytes, pkts, l2_verdict, max_frames, n_frames);
    auto step = [=](uint64_t q, Frame &fr) {
        if (file_bytes - q < 12)
            return S_TRUNC;
        uint32_t raw;
        memcpy(&raw, f + q, 4);
        const uint32_t type = rd32(f + q, swap), len = rd32(f + q + 4, swap);
        if (len < 12 || (len & 3u))
            return S_BAD;
        if (len > file_bytes - q)
            return S_TRUNC;
        if (rd32(f + q + len - 4, swap) != len)
            return S_BAD;
        if (raw == kShb || type == kIdb)
            return S_SEQ;
        fr.next = q + len;
        if (type == kSpb) {
            fr.data = q + 12;
            // as the one-piece walk: an SPB too short for its length word is an empty frame
            fr.caplen = len < 16 ? 0u : std::min<uint32_t>(rd32(f + q + 8, swap), len - 16);
            if (!ifs.empty() && ifs[0].snaplen)
                fr.caplen = std::min(fr.caplen, ifs[0].snaplen);
            fr.iface = 0;
            return S_FRAME;
        }
        if (type == kEpb || type == kPb) {
            if (len < 32)
                return S_BAD;
            fr.iface = type == kEpb ? rd32(f + q + 8, swap) : rd16(f + q + 8, swap);
            fr.caplen = rd32(f + q + 20, swap);
            fr.data = q + 28;
            return fr.caplen > len - 32 ? S_BAD : S_FRAME;
        }
        return S_SKIP;
    };
    auto plausible = [=](uint64_t q, uint64_t &next) {
        if (file_bytes - q < 12)
            return false;
        const uint32_t type = rd32(f + q, swap), len = rd32(f + q + 4, swap);
        if (!(type == kEpb || type == kSpb || type == kPb || type == 4 || type == 5) || len < 16 || (len & 3u) ||
            len > file_bytes - q || rd32(f + q + len - 4, swap) != len)
            return false;
        if ((type == kEpb || type == kPb) && (len < 32 || rd32(f + q + 20, swap) > len - 32))
            return false;
        next = q + len;
        return true;
    };
    auto cls = [&](const Frame &fr, tcsum_pkt_t &d) {
        const Iface in = fr.iface < ifs.size() ? ifs[fr.iface] : Iface{L_OTHER, 0, 0};
        return classify(f, fr.data, fr.caplen, in.kind, in.fcs, swap, d);
    };
    const int rc = make_walker(f, file_bytes, body, step, plausible, cls).run(pkts, l2_verdict, max_frames, n_frames);
    if (rc == kNeedSeq)
        return pcapng_index_seq(f, file_bytes, pkts, l2_verdict, max_frames, n_frames);
    return rc;
}

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
    if (magic == kShb)
        return pcapng_index(f, file_bytes, pkts, l2_verdict, max_frames, n_frames);
    const bool swap = magic == __builtin_bswap32(kMagicUs) || magic == __builtin_bswap32(kMagicNs);
    const bool ns = magic == kMagicNs || magic == __builtin_bswap32(kMagicNs);
    if (!swap && magic != kMagicUs && magic != kMagicNs)
        return TCSUM_ERR_PARAM; // not a classic savefile (pcapng is not read here)
    // LinkType and FCS information (bits 0-15 type, 26 F, 28-31 FCS length
    // in 16-bit units)
    const uint32_t link = rd32(f + 20, swap);
    const uint32_t type = link & 0xFFFFu;
    const uint32_t fcs = (link & (1u << 26)) ? 2u * (link >> 28) : 0u;
    const Link kind = link_kind(type);
    if (kind == L_OTHER)
        return TCSUM_ERR_NOT_SUPPORT;
    const uint32_t frac_max = ns ? 1000000000u : 1000000u;
    auto step = [=](uint64_t q, Frame &fr) {
        if (file_bytes - q < kRecHdr)
            return S_TRUNC; // a partial record header at the end
        const uint32_t caplen = rd32(f + q + 8, swap);
        if (caplen > file_bytes - q - kRecHdr)
            return S_TRUNC; // the last record's bytes are cut short
        fr.data = q + kRecHdr;
        fr.caplen = caplen;
        fr.next = fr.data + caplen;
        return S_FRAME;
    };
    auto plausible = [=](uint64_t q, uint64_t &next) {
        if (file_bytes - q < kRecHdr)
            return false;
        const uint32_t frac = rd32(f + q + 4, swap), cap = rd32(f + q + 8, swap), orig = rd32(f + q + 12, swap);
        // cap >= 1: runs of zero bytes (padding, zeroed payloads) would
        // otherwise read as chains of empty records
        next = q + kRecHdr + cap;
        return frac < frac_max && cap >= 1 && cap <= kMaxCap && orig >= cap && orig <= kMaxCap &&
               cap <= file_bytes - q - kRecHdr;
    };
    auto cls = [=](const Frame &fr, tcsum_pkt_t &d) { return classify(f, fr.data, fr.caplen, kind, fcs, swap, d); };
    return make_walker(f, file_bytes, kFileHdr, step, plausible, cls).run(pkts, l2_verdict, max_frames, n_frames);
}
