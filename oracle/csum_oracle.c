/*
 * csum_oracle.c -- CPU restatement of the reference's checksum path.
 *
 * TEST INFRASTRUCTURE ONLY (see csum_oracle.h).  Pinned against fixtures that
 * the reference's own routines produced (tests/golden/, oracle/golden_gen.c).
 *
 * The scalar loops deliberately keep the reference's loop shape -- 16-bit
 * loads into a 32-bit accumulator, one fold per call, 127-byte block chaining
 * -- so that this file is also a faithful CPU baseline ("kind": "port").
 */
#define _GNU_SOURCE
#include "csum_oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <unistd.h>
#include <string.h>
#include <time.h>

/* Fold a 32-bit partial sum to 16 bits by end-around carry (tools.c:47-51). */
static inline uint32_t fold32(uint32_t s)
{
    while (s >> 16)
        s = (s & 0xFFFFu) + (s >> 16);
    return s;
}

/* tools.c:24-54.  A byte at logical position (offset + i) is the high byte of
 * its 16-bit word when that position is odd.  The reference walks the buffer
 * as host (little-endian) u16 words; so does this. */
uint16_t orc_checksum16(int offset, const void *buf, uint16_t len,
                        uint32_t pre_sum, int complement)
{
    const uint8_t *p = (const uint8_t *)buf;
    uint32_t acc = pre_sum;
    uint32_t left = len;

    if ((offset & 1) && left > 0) { /* tools.c:29-35 (len==0 is a no-op here) */
        acc += (uint32_t)p[0] << 8;
        p++;
        left--;
    }
    while (left > 1) { /* tools.c:36-40 */
        uint16_t w;
        memcpy(&w, p, 2);
        acc += w;
        p += 2;
        left -= 2;
    }
    if (left) /* tools.c:42-45: trailing byte is a low byte */
        acc += p[0];

    acc = fold32(acc);
    return complement ? (uint16_t)~acc : (uint16_t)acc;
}

/* pktbuf.c:646-670.  `offset` counts bytes from the start of this call, the
 * running sum is kept in a uint16_t (pktbuf.c:657) and folded per block. */
uint16_t orc_pieces_checksum16(const orc_piece_t *pieces, int npieces, int len,
                               int pre_sum, int complement)
{
    long avail = 0;
    for (int i = 0; i < npieces; i++)
        avail += pieces[i].size;
    if (avail < len) /* pktbuf.c:650-655 */
        return 0;

    uint16_t sum = (uint16_t)pre_sum;
    uint32_t offset = 0;
    for (int i = 0; len > 0 && i < npieces; i++) {
        int take = pieces[i].size < len ? pieces[i].size : len;
        if (take <= 0)
            continue;
        sum = orc_checksum16((int)offset, pieces[i].data, (uint16_t)take, sum, 0);
        len -= take;
        offset += (uint32_t)take;
    }
    return complement ? (uint16_t)~sum : sum;
}

uint16_t orc_flat_checksum16(const uint8_t *buf, uint64_t len, int pre_sum,
                             int complement)
{
    uint16_t sum = (uint16_t)pre_sum;
    uint64_t offset = 0;
    while (len > 0) {
        uint32_t take = len > ORC_PKTBUF_BLK_SIZE ? ORC_PKTBUF_BLK_SIZE : (uint32_t)len;
        sum = orc_checksum16((int)(offset & 1), buf + offset, (uint16_t)take, sum, 0);
        len -= take;
        offset += take;
    }
    return complement ? (uint16_t)~sum : sum;
}

/* tools.c:58-70: src, dst, {0, proto}, htons((uint16_t)len), in memory order,
 * each through checksum16 with the running offset. */
uint16_t orc_pseudo_sum(const uint8_t src[4], const uint8_t dst[4],
                        uint8_t protocol, uint32_t len)
{
    uint8_t zp[2] = {0, protocol};
    uint16_t l16 = (uint16_t)len;
    uint8_t lbe[2] = {(uint8_t)(l16 >> 8), (uint8_t)(l16 & 0xFF)}; /* x_htons on LE */
    uint32_t s = orc_checksum16(0, src, 4, 0, 0);
    s = orc_checksum16(4, dst, 4, s, 0);
    s = orc_checksum16(8, zp, 2, s, 0);
    s = orc_checksum16(10, lbe, 2, s, 0);
    return (uint16_t)s;
}

/* tools.c:56-75 (argument order dest, src as in the reference). */
uint16_t orc_checksum_peso(const uint8_t *seg, uint32_t len,
                           const uint8_t dest[4], const uint8_t src[4],
                           uint8_t protocol)
{
    uint16_t pre = orc_pseudo_sum(src, dest, protocol, len);
    return orc_flat_checksum16(seg, len, (int)pre, 1);
}

/* Flag bits, identical to TCSUM_PKT_* in include/tcsum.h. */
#define F_BAD_VERSION 0x01u
#define F_BAD_HDRLEN 0x02u
#define F_BAD_TOTLEN 0x04u
#define F_PROTO_OTHER 0x08u
#define F_SHORT 0x10u
#define F_FRAGMENT 0x20u
#define F_L4_SHORT 0x40u

/* net_err_t values (net/net/net_err.h) */
#define E_SYS (-1)
#define E_SIZE (-5)
#define E_NOT_SUPPORT (-11)
#define E_BROKEN (-13)
#define E_UNREACHABLE (-14)

/* L4 checksum field offset and minimum header, by protocol. */
static int l4_field(uint8_t proto, uint32_t *field, uint32_t *min_len)
{
    switch (proto) {
    case 6: *field = 16; *min_len = 20; return 1;  /* tcp_hdr_t.checksum, tcp.h:71 */
    case 17: *field = 6; *min_len = 8; return 1;   /* udp_hdr_t.checksum, udp.h:24 */
    case 1: *field = 2; *min_len = 4; return 1;    /* icmpv4_hdr_t.checksum, icmpv4.h:28 */
    default: return 0;
    }
}

static int is_fragment(const uint8_t *pkt)
{
    /* frag_all after ntohs: offset = low 13 bits, more = bit 13 (ipv4.h:42-56) */
    return (pkt[6] & 0x20) || (((pkt[6] & 0x1F) << 8) | pkt[7]);
}

void orc_ipv4_pair(const uint8_t *pkt, uint32_t frame_len, uint16_t *ip_out,
                   uint16_t *l4_out, uint8_t *flags_out)
{
    uint8_t flags = 0;
    if (frame_len < 20) {
        *ip_out = 0;
        *l4_out = 0;
        *flags_out = F_SHORT;
        return;
    }
    uint32_t version = pkt[0] >> 4;
    uint32_t ihl4 = (uint32_t)(pkt[0] & 0x0F) * 4u;
    uint32_t tl = ((uint32_t)pkt[2] << 8) | pkt[3];
    uint8_t proto = pkt[9];

    if (version != 4) /* ipv4.c:222 */
        flags |= F_BAD_VERSION;
    if (ihl4 < 20 || ihl4 > frame_len) /* ipv4.c:229 */
        flags |= F_BAD_HDRLEN;
    if (tl < 20 || tl > frame_len || tl < ihl4) /* ipv4.c:236 */
        flags |= F_BAD_TOTLEN;
    if (is_fragment(pkt))
        flags |= F_FRAGMENT;

    uint32_t hl = ihl4 < 20 ? 20 : ihl4;
    if (hl > frame_len)
        hl = frame_len;
    uint32_t end = tl < hl ? hl : tl;
    if (end > frame_len)
        end = frame_len;

    *ip_out = orc_checksum16(0, pkt, (uint16_t)hl, 0, 1); /* ipv4.c:243 */

    const uint8_t *l4 = pkt + hl;
    uint32_t l4len = end - hl;
    uint32_t fld, minl;
    if (l4_field(proto, &fld, &minl) && l4len < minl)
        flags |= F_L4_SHORT;
    if (proto == 6 || proto == 17) { /* tcp_in.c:80 / udp.c:410 */
        *l4_out = orc_checksum_peso(l4, l4len, pkt + 16, pkt + 12, proto);
    } else if (proto == 1) { /* icmpv4.c:36 */
        *l4_out = orc_flat_checksum16(l4, l4len, 0, 1);
    } else {
        *l4_out = 0;
        flags |= F_PROTO_OTHER;
    }
    *flags_out = flags;
}

uint8_t orc_ipv4_tx_fill(uint8_t *pkt, uint32_t frame_len)
{
    uint16_t ip, l4;
    uint8_t flags;
    orc_ipv4_pair(pkt, frame_len, &ip, &l4, &flags); /* for the flags */
    if (flags & (F_SHORT | F_BAD_VERSION | F_BAD_HDRLEN | F_BAD_TOTLEN))
        return flags;
    uint32_t hl = (uint32_t)(pkt[0] & 0x0F) * 4u;
    uint32_t tl = ((uint32_t)pkt[2] << 8) | pkt[3];
    uint8_t proto = pkt[9];
    uint32_t fld, minl;
    /* L4 first, as the stack does (send_out/udp_out run before ipv4_out) */
    if (!(flags & (F_FRAGMENT | F_L4_SHORT)) && l4_field(proto, &fld, &minl)) {
        uint8_t *l4p = pkt + hl;
        uint32_t l4len = tl - hl;
        l4p[fld] = l4p[fld + 1] = 0; /* tcp_out.c:19, udp.c:320, icmpv4.c:58 */
        uint16_t v = proto == 1 ? orc_flat_checksum16(l4p, l4len, 0, 1)
                                : orc_checksum_peso(l4p, l4len, pkt + 16, pkt + 12, proto);
        memcpy(l4p + fld, &v, 2); /* stored in host order, like the struct field */
    }
    pkt[10] = pkt[11] = 0; /* ipv4.c:643 */
    uint16_t h = orc_checksum16(0, pkt, (uint16_t)hl, 0, 1);
    memcpy(pkt + 10, &h, 2); /* ipv4.c:656 */
    return flags;
}

/* The receive path's verdict: the net_err_t of the first gate that rejects
 * the packet, in the reference's order -- ipv4_in / is_pkt_ok, then the L4
 * input function ip_normal_in dispatches to (ipv4.c:420-470) -- up to, not
 * including, socket lookup and routing.  Pinned by tests/golden/ipv4_rx_*,
 * the return values of the reference stack's own code (oracle/stack_gen.c). */
int8_t orc_ipv4_rx_verify(const uint8_t *pkt, uint32_t frame_len, uint8_t *flags_out)
{
    uint16_t ip, l4;
    uint8_t flags;
    orc_ipv4_pair(pkt, frame_len, &ip, &l4, &flags);
    *flags_out = flags;
    if (frame_len < 20) /* pktbuf_set_cont(buf, 20), ipv4.c:475 */
        return E_SIZE;
    uint32_t ihl4 = (uint32_t)(pkt[0] & 0x0F) * 4u;
    uint32_t tl = ((uint32_t)pkt[2] << 8) | pkt[3];
    if ((pkt[0] >> 4) != 4) /* ipv4.c:222 */
        return E_NOT_SUPPORT;
    if (ihl4 < 20) /* ipv4.c:229 */
        return E_SIZE;
    if (tl < 20 || frame_len < tl) /* ipv4.c:236 */
        return E_SIZE;
    /* ipv4.c:241-249 (IHL*4 past the frame: the reference sums bytes it was
     * not given; here only the captured ones count) */
    if ((pkt[10] | pkt[11]) && ip != 0)
        return E_BROKEN;
    if (flags & F_FRAGMENT) /* ipv4.c:506-509: reassembly first, ipv4_in returns OK */
        return 0;
    uint8_t proto = pkt[9];
    const uint8_t *l4p = pkt + ihl4;
    if (proto == 6) { /* ip_normal_in -> pktbuf_remove_header + tcp_in (ipv4.c:450-452) */
        if (ihl4 > tl) /* the reference runs off the block list (pktbuf.c:264-281); defined here */
            return E_SIZE;
        uint32_t seg = tl - ihl4;
        if (seg < 20) /* pktbuf_set_cont(buf, 20) fails: tcp_in returns -1, tcp_in.c:70-74 */
            return E_SYS;
        if ((l4p[16] | l4p[17]) && l4 != 0) /* tcp_in.c:77-85 */
            return E_BROKEN;
        if (seg < (uint32_t)(l4p[12] >> 4) * 4u) /* tcp_in.c:87-91 */
            return E_SIZE;
        if (!(l4p[0] | l4p[1]) || !(l4p[2] | l4p[3])) /* tcp_in.c:93-97 */
            return E_BROKEN;
        if (!(l4p[12] | l4p[13])) /* tcp_in.c:99-103 */
            return E_BROKEN;
        return 0; /* socket lookup (tcp_in.c:115) */
    }
    if (proto == 17) { /* udp_in (ipv4.c:436) */
        if (tl < ihl4 + 8) /* pktbuf_set_cont(buf, 8 + ihl), udp.c:386-391 */
            return E_SIZE;
        if (!(l4p[2] | l4p[3])) /* port 0 matches no socket: udp.c:337-340, :399-403 */
            return E_UNREACHABLE;
        if ((l4p[6] | l4p[7]) && l4 != 0) /* udp.c:407-415 */
            return E_BROKEN;
        return 0; /* udp.c:373 cannot fail past the set_cont above */
    }
    if (proto == 1) { /* icmpv4_in (ipv4.c:427) */
        if (tl < ihl4 + 4) /* pktbuf_set_cont(buf, ihl + 4), icmpv4.c:68-73 */
            return E_SIZE;
        /* icmpv4.c:31 (total <= 21) cannot fire past that, and the checksum
         * test cannot fail (A10: len > remain, pktbuf.c:650-655) */
        return 0;
    }
    return 0; /* raw_in: no checksum (ipv4.c:460-469) */
}

/* ---------------------------------------------------------------- batches */

typedef struct job {
    int kind; /* 0 seg, 1 peso, 2 ipv4 */
    const uint8_t *arena;
    const void *descs;
    uint32_t lo, hi;
    void *out;
    uint8_t *flags;
    int complement;
} job_t;

static void run_range(const job_t *j)
{
    for (uint32_t i = j->lo; i < j->hi; i++) {
        if (j->kind == 0) {
            const orc_seg_t *d = (const orc_seg_t *)j->descs + i;
            ((uint16_t *)j->out)[i] =
                orc_flat_checksum16(j->arena + d->offset, d->len, (int)d->pre_sum,
                                    j->complement);
        } else if (j->kind == 1) {
            const orc_peso_t *d = (const orc_peso_t *)j->descs + i;
            ((uint16_t *)j->out)[i] = orc_checksum_peso(j->arena + d->offset, d->len,
                                                        d->dst, d->src, d->protocol);
        } else if (j->kind == 2) {
            const orc_pkt_t *d = (const orc_pkt_t *)j->descs + i;
            uint16_t ip, l4;
            uint8_t fl;
            orc_ipv4_pair(j->arena + d->offset, d->len, &ip, &l4, &fl);
            ((uint32_t *)j->out)[i] = (uint32_t)ip | ((uint32_t)l4 << 16);
            if (j->flags)
                j->flags[i] = fl;
        } else if (j->kind == 3) {
            const orc_pkt_t *d = (const orc_pkt_t *)j->descs + i;
            uint8_t fl = orc_ipv4_tx_fill((uint8_t *)j->arena + d->offset, d->len);
            if (j->flags)
                j->flags[i] = fl;
        } else {
            const orc_pkt_t *d = (const orc_pkt_t *)j->descs + i;
            uint8_t fl;
            ((int8_t *)j->out)[i] = orc_ipv4_rx_verify(j->arena + d->offset, d->len, &fl);
            if (j->flags)
                j->flags[i] = fl;
        }
    }
}

static void *job_thread(void *arg)
{
    run_range((const job_t *)arg);
    return NULL;
}

static void run_batch(job_t base, uint32_t n, int nthreads)
{
    if (nthreads <= 1 || n < 2) {
        base.lo = 0;
        base.hi = n;
        run_range(&base);
        return;
    }
    if (nthreads > 256)
        nthreads = 256;
    pthread_t th[256];
    job_t jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = base;
        jobs[t].lo = (uint32_t)((uint64_t)n * t / nthreads);
        jobs[t].hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
        pthread_create(&th[t], NULL, job_thread, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
}

void orc_batch_segments(const uint8_t *arena, const orc_seg_t *segs, uint32_t n,
                        uint16_t *out, int complement, int nthreads)
{
    job_t j = {0, arena, segs, 0, 0, out, NULL, complement};
    run_batch(j, n, nthreads);
}

void orc_batch_peso(const uint8_t *arena, const orc_peso_t *segs, uint32_t n,
                    uint16_t *out, int nthreads)
{
    job_t j = {1, arena, segs, 0, 0, out, NULL, 0};
    run_batch(j, n, nthreads);
}

void orc_batch_ipv4(const uint8_t *arena, const orc_pkt_t *pkts, uint32_t n,
                    uint32_t *out, uint8_t *flags, int nthreads)
{
    job_t j = {2, arena, pkts, 0, 0, out, flags, 0};
    run_batch(j, n, nthreads);
}

void orc_batch_ipv4_tx_fill(uint8_t *arena, const orc_pkt_t *pkts, uint32_t n,
                            uint8_t *flags, int nthreads)
{
    job_t j = {3, arena, pkts, 0, 0, NULL, flags, 0};
    run_batch(j, n, nthreads);
}

void orc_batch_ipv4_rx_verify(const uint8_t *arena, const orc_pkt_t *pkts, uint32_t n,
                              int8_t *verdict, uint8_t *flags, int nthreads)
{
    job_t j = {4, arena, pkts, 0, 0, verdict, flags, 0};
    run_batch(j, n, nthreads);
}

/* ---------------------------------------------------------- synthetic data */

uint64_t orc_splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

void orc_synth_fill(uint8_t *dst, uint64_t byte_offset, uint64_t nbytes,
                    uint64_t seed)
{
    for (uint64_t i = 0; i < nbytes; i++) {
        uint64_t pos = byte_offset + i;
        uint64_t w = orc_splitmix64(seed + (pos >> 3));
        dst[i] = (uint8_t)(w >> (8 * (pos & 7)));
    }
}

/* ------------------------------------------------------------ CPU baseline */

typedef struct tjob {
    orc_peso_fn fn;
    const uint8_t *arena;
    const orc_peso_t *segs;
    uint32_t lo, hi;
    double min_seconds;
    pthread_barrier_t *bar;
    uint64_t bytes;
    uint64_t csum;
    double secs;
    int cpu; /* pin to this logical CPU, or -1 */
} tjob_t;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *time_thread(void *arg)
{
    tjob_t *j = (tjob_t *)arg;
    /* Pin the thread to one logical CPU and give it its own copy of its
     * segments' bytes, first touched here: the pages land on this thread's
     * NUMA node.  (A sample first touched by the calling thread sits on one
     * socket of a 2-socket host, and the all-core rate then moved by 2x from
     * run to run: VERDICT r03, weak 7.) */
    if (j->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(j->cpu, &set);
        (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    }
    uint64_t lo = UINT64_MAX, hi = 0, own = 0;
    for (uint32_t i = j->lo; i < j->hi; i++) {
        const orc_peso_t *d = j->segs + i;
        if (d->offset < lo)
            lo = d->offset;
        if (d->offset + d->len > hi)
            hi = d->offset + d->len;
        own += d->len;
    }
    uint8_t *local = NULL;
    const uint8_t *src = j->arena;
    /* a slice whose segments are spread over much more than their own bytes
     * (descriptors in no particular order) reads the shared sample instead */
    if (hi > lo && hi - lo <= 2 * own + (1u << 20)) {
        local = (uint8_t *)malloc(hi - lo + 64);
        if (local) {
            memcpy(local, j->arena + lo, hi - lo);
            src = local - lo; /* segment offsets index the copy */
        }
    }
    pthread_barrier_wait(j->bar);
    double t0 = now_s(), t1;
    uint64_t bytes = 0, csum = 0;
    do {
        csum = 0;
        for (uint32_t i = j->lo; i < j->hi; i++) {
            const orc_peso_t *d = j->segs + i;
            csum += j->fn(src + d->offset, d->len, d->dst, d->src, d->protocol);
            bytes += d->len;
        }
        t1 = now_s();
    } while (t1 - t0 < j->min_seconds);
    j->bytes = bytes;
    j->csum = csum;
    j->secs = t1 - t0;
    free(local);
    return NULL;
}

double orc_time_peso(orc_peso_fn fn, const uint8_t *arena, const orc_peso_t *segs,
                     uint32_t n, int nthreads, double min_seconds,
                     uint64_t *checksum_of_checksums)
{
    return orc_time_peso_rates(fn, arena, segs, n, nthreads, min_seconds, checksum_of_checksums, NULL);
}

double orc_time_peso_rates(orc_peso_fn fn, const uint8_t *arena, const orc_peso_t *segs,
                           uint32_t n, int nthreads, double min_seconds,
                           uint64_t *checksum_of_checksums, double *thread_rates)
{
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    pthread_t th[256];
    tjob_t jobs[256];
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
    /* the CPUs this process may run on, in order: thread t on the t-th */
    int allowed[1024], nallowed = 0;
    cpu_set_t mask;
    CPU_ZERO(&mask);
    if (sched_getaffinity(0, sizeof(mask), &mask) == 0)
        for (int c = 0; c < CPU_SETSIZE && nallowed < 1024; c++)
            if (CPU_ISSET(c, &mask))
                allowed[nallowed++] = c;
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (tjob_t){fn, arena, segs,
                           (uint32_t)((uint64_t)n * t / nthreads),
                           (uint32_t)((uint64_t)n * (t + 1) / nthreads),
                           min_seconds, &bar, 0, 0, 0.0,
                           nthreads > 1 && nallowed >= nthreads ? allowed[t] : -1};
        pthread_create(&th[t], NULL, time_thread, &jobs[t]);
    }
    double rate = 0.0, max_secs = 0.0;
    uint64_t total = 0, csum = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        total += jobs[t].bytes;
        csum += jobs[t].csum;
        if (thread_rates) /* each thread's own bytes / its own seconds */
            thread_rates[t] = jobs[t].secs > 0 ? (double)jobs[t].bytes / jobs[t].secs : 0.0;
        if (jobs[t].secs > max_secs)
            max_secs = jobs[t].secs;
    }
    pthread_barrier_destroy(&bar);
    if (max_secs > 0)
        rate = (double)total / max_secs;
    if (checksum_of_checksums)
        *checksum_of_checksums = csum;
    return rate;
}
