/*
 * pcap_wire.c -- the reference's own pcap driver (plat/netif_pcap.c, with
 * integration/net_checksum_gpu.patch) run for real over the libpcap test
 * double (integration/pcap_double.c).  TEST PROGRAM, built by
 * integration/Makefile:
 *   _build/pcap_wire        the patched stack + libtcsum.so (checksums on the GPU)
 *   _build/pcap_wire_cpu    the same stack + tcsum_cpu_double.c (oracle; no GPU)
 *   _build/pcap_wire_tsan   the CPU form under ThreadSanitizer
 * Usage: pcap_wire GOLDEN_DIR [--max N] [--skip-concurrent]
 *
 * The netif is opened the way the reference's app opens its pcap netif
 * (app/test/main.c netdev_init: netif_open with netdev_ops and a pcap_data_t,
 * then netif_set_addr / netif_set_active): pcap_device_open (sys_plat.c:540-618)
 * finds the double's device by IP, and netif_pcap_open starts the reference's
 * recv_thread and xmit_thread (netif_pcap.c:84-85).  Phases, each ending in
 * one "phase NAME: ok ..." or "phase NAME: FAIL ..." line (exit 0 iff all ok):
 *
 *   tx   every frame of tests/golden/stack_tx_in.bin (frames the reference
 *        stack transmitted, with the checksum fields it filled set to junk)
 *        behind an Ethernet header goes on the netif's out_q with
 *        netif_put_out, where ether_raw_out puts frames (netif.c:339-349);
 *        xmit_thread drains it, fills the batch in pinned staging and
 *        pcap_injects from there.  Every injected frame must equal the same
 *        header + the stack_tx_out.bin frame, byte for byte.
 *   rx   every non-fragment frame of ipv4_rx_pool.bin that fits the Ethernet
 *        MTU (ether.c:14-25 drops longer ones before ipv4_in) goes on the wire;
 *        recv_thread reads it (pcap_next_ex), do_netif_in sums its drained
 *        in_q as one batch and the unchanged per-packet path decides.  The
 *        decision -- the return of tcp_in / udp_in / icmpv4_in / raw_in when
 *        one ran, else ipv4_in's, i.e. exactly oracle/stack_gen.c's verdict --
 *        is read through link-time taps (--wrap) and must equal the fixture's.
 *        The per-frame state stack_gen assumes is set by the ipv4_in tap (the
 *        netif's address = the frame's destination, a UDP socket bound to its
 *        port, a raw socket of protocol 0; their receive lists emptied after
 *        each frame).  The replies the stack sends meanwhile (TCP resets, ICMP
 *        echo replies and port unreachables) leave through the batch fill too:
 *        each must equal its own oracle tx fill (orc_ipv4_tx_fill).
 *   faults  one tx fill made to fail (the engine call, through --wrap): logged,
 *        counted (tx_fail_batches / tx_dropped) and its frames dropped, the
 *        frames after it sent intact; one rx batch made to fail: logged,
 *        counted, and every verdict still equal (the checksum tests sum through
 *        the drop-in symbols); one pcap_inject failure: the reference's own
 *        log line (netif_pcap.c:62-65), the other frames sent.
 *   concurrent  a UDP echo over the loop netif (loop_xmit: the batch fill on
 *        the work thread) while the tx fixtures leave through the pcap
 *        xmit_thread: two threads inside net_csum_gpu_tx at once.
 *
 * sys_mutex_create is made recursive (the Makefile weakens the Linux one):
 * pktbuf_free takes the pktbuf lock twice (pktbuf.c:203 -> :44).
 */
#include <pthread.h>
#include <signal.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "exmsg.h"
#include "icmpv4.h"
#include "ipv4.h"
#include "net.h"
#include "net_api.h"
#include "net_csum_gpu.h"
#include "netif.h"
#include "netif_pcap.h"
#include "pktbuf.h"
#include "raw.h"
#include "sys_plat.h"
#include "tcp_in.h"
#include "udp.h"

#include "csum_oracle.h"
#include "pcap_double.h"
#include "tcsum.h"

sys_mutex_t sys_mutex_create(void)
{
    pthread_mutex_t *m = (pthread_mutex_t *)malloc(sizeof *m);
    pthread_mutexattr_t a;
    pthread_mutexattr_init(&a);
    pthread_mutexattr_settype(&a, PTHREAD_MUTEX_RECURSIVE);
    pthread_mutex_init(m, &a);
    pthread_mutexattr_destroy(&a);
    return m;
}

#define GATE_FRAG 2u /* oracle/stack_gen.h TAP_GATE_FRAG */
#define GATE_L4 3u   /* oracle/stack_gen.h TAP_GATE_L4 */
#define ETH 14
#define ETHER_MTU_BYTES 1500

static const uint8_t our_mac[6] = {0x02, 0x00, 0x5e, 0x00, 0x00, 0x01};
static const uint8_t peer_mac[6] = {0x02, 0x00, 0x5e, 0x10, 0x00, 0x01};
static netif_t *wire;
static udp_t *udp_sock;
static raw_t *raw_sock;
static int failures;

static const char *volatile stage = "start";
static void watchdog(int sig)
{
    printf("watchdog: no progress at stage '%s'\n", stage);
    fflush(stdout);
    _exit(3);
}

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void phase(const char *name, int ok, const char *fmt, ...)
{
    char msg[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(msg, sizeof msg, fmt, ap);
    va_end(ap);
    printf("\nphase %s: %s %s\n", name, ok ? "ok" : "FAIL", msg); /* the stack prints lines without an end */
    fflush(stdout);
    if (!ok)
        failures++;
}

/* ------------------------------------------------------------ fixtures */

static uint8_t *slurp(const char *dir, const char *name, size_t *len)
{
    char path[1024];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE *f = fopen(path, "rb");
    if (!f) {
        perror(path);
        exit(2);
    }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *p = (uint8_t *)malloc(n > 0 ? (size_t)n : 1u);
    if (!p || fread(p, 1, (size_t)n, f) != (size_t)n) {
        fprintf(stderr, "%s: read failed\n", path);
        exit(2);
    }
    fclose(f);
    *len = (size_t)n;
    return p;
}

typedef struct {
    uint32_t at, len;
} span_t;

static uint8_t *tx_in, *tx_out, *rx_pool;
static span_t *tx_cases;
static uint32_t n_tx;
static struct {
    uint32_t at, len;
    int32_t verdict;
    uint32_t gate;
} * rx_cases;
static uint32_t n_rx;

/* The reference's receive path over its pcap driver leaves the pktbuf
 * cursor stale: netif_get_in resets it (netif.c:326-331), then ether_in /
 * arp_update_from_ipbuf / ipv4_in / icmpv4_in move the first block's bytes
 * with pktbuf_set_cont (pktbuf.c:394-444) and pktbuf_remove_header
 * (pktbuf.c:259-286) without resetting it, and icmpv4_in then walks it
 * (pktbuf_seek, icmpv4.c:76 -> pktbuf.c:545-580).  When the walk runs off the
 * block list, move_forward dereferences NULL (pktbuf.c:470): the reference
 * crashes there, with or without this patch -- a frame with no defined
 * behaviour, skipped like oracle/stack_gen.c's ref_defined skips its own.
 * This replays those calls on the block sizes alone: pktbuf_alloc's layout
 * for the frame recv_thread writes (head insertion, the partial block first,
 * pktbuf.c:62-110,172-199), each set_cont / remove_header / resize on it, and
 * the seek from the stale offset.  1 = the walk stays on the list. */
static int icmp_seek_defined(uint32_t L, uint32_t ihl4, uint32_t tl)
{
    enum { B = PKTBUF_BLK_SIZE };
    int off[64], size[64], nb, total = ETH + (int)L;
    const int r = total % B ? total % B : B;
    nb = (total - r) / B + 1;
    for (int i = 0; i < nb; i++)
        off[i] = i ? 0 : B - r, size[i] = i ? B : r;
    const int cursor = off[0]; /* netif_get_in's reset; never moved again */
#define CONT(n)                                                                                                        \
    do {                                                                                                               \
        if (size[0] < (n)) {                                                                                           \
            off[0] = 0;                                                                                                \
            int need = (n)-size[0];                                                                                    \
            while (need && nb > 1) {                                                                                   \
                int take = size[1] < need ? size[1] : need;                                                            \
                off[1] += take, size[1] -= take, size[0] += take, need -= take;                                        \
                if (!size[1]) {                                                                                        \
                    for (int j = 1; j + 1 < nb; j++)                                                                   \
                        off[j] = off[j + 1], size[j] = size[j + 1];                                                    \
                    nb--;                                                                                              \
                }                                                                                                      \
            }                                                                                                          \
        }                                                                                                              \
    } while (0)
    CONT(ETH);                        /* ether_in (ether.c:67) */
    CONT(ETH + 20);                   /* arp_update_from_ipbuf (arp.c:481) */
    off[0] += ETH, size[0] -= ETH;    /* pktbuf_remove_header (ether.c:87); size[0] >= 20 */
    total -= ETH;
    CONT(20);                         /* ipv4_in (ipv4.c:475) */
    if ((int)tl < total) {            /* pktbuf_resize (ipv4.c:490) */
        int acc = 0, k = 0;
        while (k < nb && (acc += size[k]) < (int)tl)
            k++;
        int freed = 0;
        for (int j = k + 1; j < nb; j++)
            freed += size[j];
        size[k] -= total - freed - (int)tl;
        nb = k + 1;
        total = (int)tl;
    }
    if ((int)ihl4 + 4 > total)
        return 1;                     /* icmpv4_in's set_cont fails: no walk */
    CONT((int)ihl4 + 4);              /* icmpv4.c:68 */
#undef CONT
    if ((int)ihl4 >= total)
        return 1;                     /* pktbuf_seek refuses it */
    int cb = 0, at = cursor, move = (int)ihl4;
    while (move) {
        if (cb >= nb)
            return 0;                 /* move_forward on a NULL block */
        const int rem = off[cb] + size[cb] - at, cm = move > rem ? rem : move;
        at += cm, move -= cm;
        if (at >= off[cb] + size[cb]) {
            cb++;
            at = cb < nb ? off[cb] : 0;
        }
    }
    return 1;
}

static uint32_t n_rx_undefined;

static void load_fixtures(const char *dir, uint32_t max)
{
    size_t n;
    uint32_t *c = (uint32_t *)slurp(dir, "stack_tx_cases.bin", &n);
    n_tx = (uint32_t)(n / 16);
    tx_cases = (span_t *)malloc(n_tx * sizeof *tx_cases);
    for (uint32_t i = 0; i < n_tx; i++)
        tx_cases[i].at = c[4 * i], tx_cases[i].len = c[4 * i + 1];
    free(c);
    tx_in = slurp(dir, "stack_tx_in.bin", &n);
    tx_out = slurp(dir, "stack_tx_out.bin", &n);
    rx_pool = slurp(dir, "ipv4_rx_pool.bin", &n);
    c = (uint32_t *)slurp(dir, "ipv4_rx_cases.bin", &n);
    uint32_t all = (uint32_t)(n / 20);
    rx_cases = malloc(all * sizeof *rx_cases);
    n_rx = 0;
    for (uint32_t i = 0; i < all; i++) {
        uint32_t len = c[5 * i + 1], gate = c[5 * i + 4] & 255u;
        if (gate == GATE_FRAG || len > ETHER_MTU_BYTES)
            continue; /* reassembly state / dropped by ether_in: not a per-frame verdict */
        const uint8_t *p = rx_pool + c[5 * i];
        if (gate == GATE_L4 && p[9] == 1 &&
            !icmp_seek_defined(len, (uint32_t)(p[0] & 15) * 4, ((uint32_t)p[2] << 8) | p[3])) {
            n_rx_undefined++;
            continue;
        }
        rx_cases[n_rx].at = c[5 * i];
        rx_cases[n_rx].len = len;
        rx_cases[n_rx].verdict = (int32_t)c[5 * i + 2];
        rx_cases[n_rx].gate = gate;
        n_rx++;
    }
    free(c);
    if (max) {
        n_tx = n_tx < max ? n_tx : max;
        n_rx = n_rx < max ? n_rx : max;
    }
}

/* ------------------------------------------------------------ taps (--wrap) */

/* the verdict of each IPv4 frame the pcap netif received, in order */
#define VLOG_MAX 16384
static int32_t vlog[VLOG_MAX];
static uint32_t vn;
static int l4_called;   /* work thread only */
static uint64_t leaks_freed;
static net_err_t l4_ret;

static uint32_t verdicts(void) { return __atomic_load_n(&vn, __ATOMIC_ACQUIRE); }

static int peek(pktbuf_t *buf, uint8_t *to, int max) /* the first bytes, cursor untouched */
{
    int n = 0;
    pktblk_t *b = pktbuf_first_blk(buf);
    for (int left = buf->total_size; b && n < max && left > 0; b = pktblk_blk_next(b)) {
        int k = b->size < max - n ? b->size : max - n;
        k = k < left ? k : left;
        memcpy(to + n, b->data, (size_t)k);
        n += k;
        left -= k;
    }
    return n;
}

static void drain(list_t *l)
{
    node_t *nd;
    while ((nd = list_remove_first(l)) != (node_t *)0)
        pktbuf_free(list_node_parent(nd, pktbuf_t, node));
}

net_err_t __real_ipv4_in(netif_t *netif, pktbuf_t *buf);
net_err_t __wrap_ipv4_in(netif_t *netif, pktbuf_t *buf)
{
    if (netif != wire)
        return __real_ipv4_in(netif, buf);
    uint8_t h[64];
    const int n = peek(buf, h, (int)sizeof h);
    if (n >= 20) { /* the state oracle/stack_gen.c's rx_buf sets */
        memcpy(&wire->ipaddr.q_addr, h + 16, 4);
        const uint32_t ihl4 = (uint32_t)(h[0] & 15) * 4, tl = ((uint32_t)h[2] << 8) | h[3];
        if (ihl4 + 4 <= tl && tl <= (uint32_t)buf->total_size && ihl4 + 4 <= (uint32_t)n)
            udp_sock->base.local_port = (uint16_t)(((uint32_t)h[ihl4 + 2] << 8) | h[ihl4 + 3]);
    }
    static int trace = -1;
    if (trace < 0)
        trace = getenv("PCAP_WIRE_TRACE") != NULL;
    if (trace)
        fprintf(stderr, "trace: frame %u len %d ihl4 %d proto %d first block %d\n", vn, buf->total_size,
                n ? (h[0] & 15) * 4 : -1, n >= 10 ? h[9] : -1, pktbuf_first_blk(buf)->size);
    l4_called = 0;
    const net_err_t err = __real_ipv4_in(netif, buf);
    const uint32_t k = vn;
    if (k < VLOG_MAX)
        vlog[k] = l4_called ? (int32_t)l4_ret : (int32_t)err;
    /* The reference leaks this frame's buffer: ipv4_in returns OK whatever
     * ip_normal_in returned (ipv4.c:506-514), and an error is the caller's
     * only cue to free it (exmsg.c do_netif_in frees on err < 0; every L4
     * function leaves the buffer to its caller when it fails).  One packet
     * buffer per frame the L4 layer rejects would run the 100-block pool
     * (net_cfg.h PKTBUF_BLK_CNT) dry after a few dozen bad frames, so the tap
     * frees it where the reference's caller would have. */
    if (l4_called && l4_ret < 0 && err == NET_ERR_OK) {
        pktbuf_free(buf);
        __atomic_fetch_add(&leaks_freed, 1, __ATOMIC_RELAXED);
    }
    __atomic_store_n(&vn, k + 1, __ATOMIC_RELEASE);
    drain(&udp_sock->recv_list);
    drain(&raw_sock->recv_list);
    return err;
}

#define L4_TAP(name, params, args)                                                                                    \
    net_err_t __real_##name params;                                                                                    \
    net_err_t __wrap_##name params                                                                                     \
    {                                                                                                                  \
        net_err_t e = __real_##name args;                                                                              \
        l4_called = 1;                                                                                                 \
        l4_ret = e;                                                                                                    \
        return e;                                                                                                      \
    }
L4_TAP(tcp_in, (pktbuf_t * buf, ipaddr_t *src, ipaddr_t *dst), (buf, src, dst))
L4_TAP(udp_in, (pktbuf_t * buf, ipaddr_t *src, ipaddr_t *dst), (buf, src, dst))
L4_TAP(icmpv4_in, (ipaddr_t * src, ipaddr_t *netif_ip, pktbuf_t *buf), (src, netif_ip, buf))
L4_TAP(raw_in, (pktbuf_t * buf), (buf))

/* engine failures on demand */
static int fail_tx, fail_rx;
static int take(int *n)
{
    int v = __atomic_load_n(n, __ATOMIC_ACQUIRE);
    while (v > 0 && !__atomic_compare_exchange_n(n, &v, v - 1, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE))
        ;
    return v > 0;
}
int __real_tcsum_host_batch_ipv4_tx_fill(int, void *, uint64_t, const tcsum_pkt_t *, uint32_t, uint32_t *, uint8_t *);
int __wrap_tcsum_host_batch_ipv4_tx_fill(int d, void *a, uint64_t b, const tcsum_pkt_t *p, uint32_t n, uint32_t *o,
                                         uint8_t *f)
{
    return take(&fail_tx) ? TCSUM_ERR_SYS : __real_tcsum_host_batch_ipv4_tx_fill(d, a, b, p, n, o, f);
}
int __real_tcsum_host_batch_ipv4(int, const void *, uint64_t, const tcsum_pkt_t *, uint32_t, uint32_t *, uint8_t *);
int __wrap_tcsum_host_batch_ipv4(int d, const void *a, uint64_t b, const tcsum_pkt_t *p, uint32_t n, uint32_t *o,
                                 uint8_t *f)
{
    return take(&fail_rx) ? TCSUM_ERR_SYS : __real_tcsum_host_batch_ipv4(d, a, b, p, n, o, f);
}

/* ------------------------------------------------------------ helpers */

static int blocks_of(uint32_t bytes) { return (int)((bytes + PKTBUF_BLK_SIZE - 1) / PKTBUF_BLK_SIZE) + 1; }

static void eth_hdr(uint8_t *h, const uint8_t *dst, const uint8_t *src)
{
    memcpy(h, dst, 6);
    memcpy(h + 6, src, 6);
    h[12] = 0x08, h[13] = 0x00;
}

/* one frame onto the pcap netif's out_q, as ether_raw_out queues it */
static int put_out(const uint8_t *frame, uint32_t len)
{
    pktbuf_t *b = (pktbuf_t *)0;
    for (int tries = 0; !(b = pktbuf_alloc((int)(ETH + len))) && tries < 5000; tries++)
        usleep(1000);
    if (!b) {
        printf("put_out: no packet buffer for %u bytes\n", ETH + len);
        return -1;
    }
    uint8_t h[ETH];
    eth_hdr(h, peer_mac, our_mac);
    pktbuf_reset_access(b);
    if (pktbuf_write(b, h, ETH) != NET_ERR_OK || (len && pktbuf_write(b, (uint8_t *)frame, (int)len) != NET_ERR_OK)) {
        printf("put_out: pktbuf_write failed\n");
        pktbuf_free(b);
        return -1;
    }
    return netif_put_out(wire, b, 0) == NET_ERR_OK ? 0 : -1;
}

/* injected frame i == Ethernet header + expected */
static int same_frame(uint32_t i, const uint8_t *expect, uint32_t len, uint32_t *at)
{
    uint32_t got_len;
    const uint8_t *got = pcapd_injected(i, &got_len);
    uint8_t h[ETH];
    eth_hdr(h, peer_mac, our_mac);
    *at = 0;
    if (!got || got_len != ETH + len)
        return 0;
    if (memcmp(got, h, ETH) != 0)
        return 0;
    for (uint32_t k = 0; k < len; k++)
        if (got[ETH + k] != expect[k]) {
            *at = k;
            return 0;
        }
    return 1;
}

static int is_ipv4(uint32_t i)
{
    uint32_t len;
    const uint8_t *f = pcapd_injected(i, &len);
    return f && len >= ETH && f[12] == 0x08 && f[13] == 0x00;
}

/* send tx cases [c0, c1) through the pcap netif and check what comes out */
static int run_tx(uint32_t c0, uint32_t c1, const char *name)
{
    uint32_t base = pcapd_injected_count();
    uint32_t sent = 0;
    double t0 = now_s();
    for (uint32_t i = c0; i < c1;) {
        int blocks = 0, k = 0;
        while (i < c1 && k < 40 && blocks + blocks_of(ETH + tx_cases[i].len) <= 60) {
            blocks += blocks_of(ETH + tx_cases[i].len);
            if (put_out(tx_in + tx_cases[i].at, tx_cases[i].len) != 0)
                return 0;
            i++, k++, sent++;
        }
        /* the frames of this group are injected before the next group is
         * queued, so the packet pool (PKTBUF_BLK_CNT blocks) never runs dry */
        uint32_t need = sent, seen = 0;
        for (double t1 = now_s(); now_s() - t1 < 20.0;) {
            seen = 0;
            const uint32_t tot = pcapd_injected_count();
            for (uint32_t j = base; j < tot; j++)
                seen += is_ipv4(j);
            if (seen >= need)
                break;
            usleep(200);
        }
        if (seen < need) {
            phase(name, 0, "%u of %u frames injected after 20 s", seen, need);
            return 0;
        }
    }
    const double dt = now_s() - t0;
    uint32_t k = c0, bad = 0, first_bad = 0, first_at = 0;
    const uint32_t tot = pcapd_injected_count();
    for (uint32_t j = base; j < tot && k < c1; j++) {
        if (!is_ipv4(j))
            continue;
        uint32_t at;
        if (!same_frame(j, tx_out + tx_cases[k].at, tx_cases[k].len, &at)) {
            if (!bad++)
                first_bad = k, first_at = at;
        }
        k++;
    }
    phase(name, bad == 0 && k == c1, "%u frames injected through the batched fill, %u differ from stack_tx_out%s "
          "(first: case %u byte %u); %.1f ms", k - c0, bad, bad ? "" : "", first_bad, first_at, dt * 1e3);
    return bad == 0 && k == c1;
}

/* feed rx cases [c0, c1); check the verdicts; replies checked against the oracle fill */
/* Until no frame has been injected for quiet_s (at most max_s): the replies
 * the stack sends to received frames leave through xmit_thread after the
 * receive phase that caused them has returned, and a fault phase that counts
 * the frames injected since its start must not count them. */
static void wait_tx_quiet(double quiet_s, double max_s)
{
    uint32_t last = pcapd_injected_count();
    double t_last = now_s();
    for (double t0 = now_s(); now_s() - t0 < max_s; usleep(1000)) {
        const uint32_t c = pcapd_injected_count();
        if (c != last) {
            last = c;
            t_last = now_s();
        } else if (now_s() - t_last >= quiet_s) {
            return;
        }
    }
}

static int run_rx(uint32_t c0, uint32_t c1, const char *name)
{
    uint32_t v0 = verdicts(), fed = 0;
    static uint8_t frame[ETH + 65536];
    double t0 = now_s();
    for (uint32_t i = c0; i < c1;) {
        int blocks = 0, k = 0;
        while (i < c1 && k < 40 && blocks + blocks_of(ETH + rx_cases[i].len) <= 50) {
            blocks += blocks_of(ETH + rx_cases[i].len);
            eth_hdr(frame, our_mac, peer_mac);
            memcpy(frame + ETH, rx_pool + rx_cases[i].at, rx_cases[i].len);
            pcapd_feed(frame, ETH + rx_cases[i].len);
            i++, k++, fed++;
        }
        double t1 = now_s();
        while (verdicts() < v0 + fed && now_s() - t1 < 20.0)
            usleep(200);
        if (verdicts() < v0 + fed) {
            phase(name, 0, "%u of %u frames reached ipv4_in after 20 s (a packet buffer ran out?)", verdicts() - v0,
                  fed);
            return 0;
        }
        /* the replies this group caused hold pool blocks until xmit_thread has
         * sent them: let them leave before the next group needs blocks, or
         * recv_thread's pktbuf_alloc fails and drops a frame (the reference's
         * pool is 100 blocks, net_cfg.h) */
        for (double tq = now_s(); fixq_count(&wire->out_q) > 0 && now_s() - tq < 5.0;)
            usleep(200);
        wait_tx_quiet(0.003, 2.0);
    }
    const double dt = now_s() - t0;
    uint32_t bad = 0, first = 0, hist[32] = {0};
    for (uint32_t k = 0; k < fed; k++) {
        const int32_t want = rx_cases[c0 + k].verdict, got = vlog[(v0 + k) % VLOG_MAX];
        if (got != want && !bad++)
            first = c0 + k;
        hist[(-want) & 31]++;
    }
    char h[256] = "";
    for (int e = 0; e < 32; e++)
        if (hist[e])
            snprintf(h + strlen(h), sizeof h - strlen(h), " %d:%u", -e, hist[e]);
    if (bad)
        phase(name, 0, "%u of %u verdicts differ from ipv4_rx_cases (first: case at %u, want %d got %d)", bad, fed,
              rx_cases[first].at, rx_cases[first].verdict, vlog[(v0 + first - c0) % VLOG_MAX]);
    else
        phase(name, 1, "%u frames through recv_thread -> batched do_netif_in, every verdict equal "
              "(net_err_t:count%s); %.1f ms; %llu rejected frames' buffers freed for the reference (its ipv4_in "
              "drops the error that would free them)", fed, h, dt * 1e3,
              (unsigned long long)__atomic_load_n(&leaks_freed, __ATOMIC_RELAXED));
    return bad == 0;
}

/* every IPv4 frame injected from index i0 on must equal its own oracle fill */
static int check_replies(uint32_t i0, const char *name)
{
    static uint8_t copy[ETH + 65536];
    uint32_t n = 0, bad = 0;
    const uint32_t tot = pcapd_injected_count();
    for (uint32_t j = i0; j < tot; j++) {
        uint32_t len;
        const uint8_t *f = pcapd_injected(j, &len);
        if (!is_ipv4(j) || len <= ETH)
            continue;
        memcpy(copy, f, len);
        orc_ipv4_tx_fill(copy + ETH, len - ETH);
        bad += memcmp(copy, f, len) != 0;
        n++;
    }
    phase(name, bad == 0 && n > 0, "%u replies the stack sent (TCP resets, ICMP echo replies / unreachables), "
          "%u differ from the oracle's fill", n, bad);
    return bad == 0;
}

static void stats(net_csum_gpu_stats_t *st) { net_csum_gpu_stats(st); }

static void print_stats(const char *when)
{
    net_csum_gpu_stats_t st;
    stats(&st);
    printf("engine %s: tx %llu frames in %llu batches; rx %llu frames in %llu batches, %llu tests answered from a "
           "batch; failures: tx %llu batches (%llu frames dropped), rx %llu batches; pcap double: %llu ARP replies, "
           "%llu frames filtered, %llu inject failures\n",
           when, (unsigned long long)st.tx_frames, (unsigned long long)st.tx_batches,
           (unsigned long long)st.rx_frames, (unsigned long long)st.rx_batches, (unsigned long long)st.rx_used,
           (unsigned long long)st.tx_fail_batches, (unsigned long long)st.tx_dropped,
           (unsigned long long)st.rx_fail_batches, (unsigned long long)pcapd_arp_replies(),
           (unsigned long long)pcapd_filtered(), (unsigned long long)pcapd_inject_failures());
    // frames per batch (tx coalescing, net_csum_gpu.h): 1, 2-3, 4-7, 8-15, 16-31, >= 32
    printf("batch sizes %s: tx [1 %llu | 2-3 %llu | 4-7 %llu | 8-15 %llu | 16-31 %llu | 32+ %llu], "
           "rx [1 %llu | 2-3 %llu | 4-7 %llu | 8-15 %llu | 16-31 %llu | 32+ %llu]\n", when,
           (unsigned long long)st.tx_hist[0], (unsigned long long)st.tx_hist[1], (unsigned long long)st.tx_hist[2],
           (unsigned long long)st.tx_hist[3], (unsigned long long)st.tx_hist[4], (unsigned long long)st.tx_hist[5],
           (unsigned long long)st.rx_hist[0], (unsigned long long)st.rx_hist[1], (unsigned long long)st.rx_hist[2],
           (unsigned long long)st.rx_hist[3], (unsigned long long)st.rx_hist[4], (unsigned long long)st.rx_hist[5]);
    fflush(stdout);
}

/* ------------------------------------------------------------ faults */

static int wait_until(int (*cond)(void *), void *arg, double s)
{
    for (double t0 = now_s(); now_s() - t0 < s; usleep(500))
        if (cond(arg))
            return 1;
    return cond(arg);
}

typedef struct {
    uint32_t base, want;
    uint64_t dropped0;
} tx_wait_t;

static uint32_t ipv4_since(uint32_t base)
{
    uint32_t n = 0;
    const uint32_t tot = pcapd_injected_count();
    for (uint32_t j = base; j < tot; j++)
        n += is_ipv4(j);
    return n;
}

static int tx_accounted(void *a)
{
    tx_wait_t *w = (tx_wait_t *)a;
    net_csum_gpu_stats_t st;
    stats(&st);
    return ipv4_since(w->base) + (st.tx_dropped - w->dropped0) + pcapd_inject_failures() >= w->want;
}

static void run_faults(void)
{
    const uint32_t G = n_tx < 12 ? n_tx : 12;
    net_csum_gpu_stats_t s0, s1;

    /* (1) the engine fails one tx fill */
    wait_tx_quiet(0.2, 10.0);
    stats(&s0);
    uint64_t inj_fail0 = pcapd_inject_failures();
    tx_wait_t w = {pcapd_injected_count(), G + (uint32_t)inj_fail0, s0.tx_dropped};
    __atomic_store_n(&fail_tx, 1, __ATOMIC_RELEASE);
    for (uint32_t i = 0; i < G; i++)
        put_out(tx_in + tx_cases[i].at, tx_cases[i].len);
    wait_until(tx_accounted, &w, 20.0);
    stats(&s1);
    const uint32_t dropped = (uint32_t)(s1.tx_dropped - s0.tx_dropped), sent = ipv4_since(w.base);
    uint32_t bad = 0, k = dropped;
    for (uint32_t j = w.base; j < pcapd_injected_count() && k < G; j++) {
        uint32_t at;
        if (!is_ipv4(j))
            continue;
        bad += !same_frame(j, tx_out + tx_cases[k].at, tx_cases[k].len, &at);
        k++;
    }
    phase("fault_tx", s1.tx_fail_batches == s0.tx_fail_batches + 1 && dropped >= 1 && dropped + sent == G && !bad,
          "one fill failed: %llu failed batch logged and counted, %u frames dropped with it, the other %u sent "
          "intact (%u differ)", (unsigned long long)(s1.tx_fail_batches - s0.tx_fail_batches), dropped, sent, bad);

    /* (2) the engine fails one rx batch: the tests then sum per call */
    stats(&s0);
    const uint32_t R = n_rx < 30 ? n_rx : 30;
    __atomic_store_n(&fail_rx, 1, __ATOMIC_RELEASE);
    int ok = run_rx(0, R, "fault_rx_verdicts");
    stats(&s1);
    phase("fault_rx", ok && s1.rx_fail_batches == s0.rx_fail_batches + 1,
          "one rx batch failed: %llu logged and counted, its frames' checksum tests summed by the drop-in "
          "symbols, all %u verdicts equal", (unsigned long long)(s1.rx_fail_batches - s0.rx_fail_batches), R);

    /* (3) one pcap_inject fails: the reference's own handling (logged, frame lost) */
    wait_tx_quiet(0.2, 10.0); /* the replies to the fault_rx frames leave first */
    stats(&s0);
    w.base = pcapd_injected_count();
    w.dropped0 = s0.tx_dropped;
    inj_fail0 = pcapd_inject_failures();
    w.want = G + (uint32_t)inj_fail0;
    pcapd_fail_inject(1);
    for (uint32_t i = 0; i < G; i++)
        put_out(tx_in + tx_cases[i].at, tx_cases[i].len);
    wait_until(tx_accounted, &w, 20.0);
    const uint32_t got = ipv4_since(w.base);
    bad = 0, k = 1;
    for (uint32_t j = w.base; j < pcapd_injected_count() && k < G; j++) {
        uint32_t at;
        if (!is_ipv4(j))
            continue;
        bad += !same_frame(j, tx_out + tx_cases[k].at, tx_cases[k].len, &at);
        k++;
    }
    phase("fault_inject", pcapd_inject_failures() == inj_fail0 + 1 && got == G - 1 && !bad,
          "one pcap_inject failed: %u of %u frames sent, the rest intact (%u differ)", got, G, bad);
}

/* ------------------------------------------------------------ concurrent */

#define ECHO_PORT 7
#define ECHO_ROUNDS 200
static volatile int echo_rc = -1;

static void echo_server(void *arg)
{
    int s = socket(AF_INET, SOCK_DGRAM, 0);
    struct sockaddr_in a;
    memset(&a, 0, sizeof a);
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = INADDR_ANY;
    a.sin_port = htons(ECHO_PORT);
    if (s < 0 || bind(s, (const struct sockaddr *)&a, sizeof a) < 0)
        return;
    for (;;) {
        static char buf[2048];
        struct sockaddr_in c;
        x_socklen_t len = sizeof c;
        ssize_t n = recvfrom(s, buf, sizeof buf, 0, (struct sockaddr *)&c, &len);
        if (n > 0)
            sendto(s, buf, (size_t)n, 0, (struct sockaddr *)&c, len);
    }
}

static void *echo_client(void *arg)
{
    int s = socket(AF_INET, SOCK_DGRAM, 0);
    struct x_timeval tv = {2, 0};
    setsockopt(s, SOL_SOCKET, SO_RCVTIMEO, (const char *)&tv, sizeof tv);
    struct sockaddr_in to;
    memset(&to, 0, sizeof to);
    to.sin_family = AF_INET;
    to.sin_addr.s_addr = inet_addr("127.0.0.1");
    to.sin_port = htons(ECHO_PORT);
    static uint8_t out[1500], in[2048];
    int rc = 0;
    for (int r = 0; r < ECHO_ROUNDS && !rc; r++) {
        int n = 1 + (r * 53) % 1400;
        for (int i = 0; i < n; i++)
            out[i] = (uint8_t)(r * 31 + i * 7);
        if (sendto(s, out, (size_t)n, 0, (const struct sockaddr *)&to, sizeof to) != n)
            rc = 1;
        struct sockaddr_in from;
        x_socklen_t len = sizeof from;
        ssize_t got = recvfrom(s, in, sizeof in, 0, (struct sockaddr *)&from, &len);
        if (got != n || memcmp(in, out, (size_t)n) != 0)
            rc = 2;
    }
    echo_rc = rc;
    return (void *)0;
}

static net_err_t restore_addr(func_msg_t *m) /* on the work thread, like every stack state change */
{
    ipaddr_from_str(&wire->ipaddr, "10.0.0.1");
    udp_sock->base.local_port = 0;
    return NET_ERR_OK;
}

int main(int argc, char **argv)
{
    setvbuf(stdout, NULL, _IOLBF, 0);
    if (argc < 2)
        return fprintf(stderr, "usage: %s GOLDEN_DIR [--max N] [--skip-concurrent]\n", argv[0]), 2;
    uint32_t max = 0;
    int concurrent = 1;
    for (int i = 2; i < argc; i++) {
        if (!strcmp(argv[i], "--max") && i + 1 < argc)
            max = (uint32_t)atoi(argv[++i]);
        else if (!strcmp(argv[i], "--skip-concurrent"))
            concurrent = 0;
    }
    signal(SIGALRM, watchdog);
    alarm(300);
    load_fixtures(argv[1], max);
    if (tcsum_device_count() < 1)
        return fprintf(stderr, "no gfx950 device for the checksum engine\n"), 2;

    stage = "net_init";
    pcapd_setup("192.168.74.2", peer_mac);
    if (net_init() != NET_ERR_OK) /* net_plat_init -> net_csum_gpu_init */
        return fprintf(stderr, "net_init failed\n"), 2;
    udp_sock = (udp_t *)udp_create(AF_INET, IPPROTO_UDP);
    raw_sock = (raw_t *)raw_create(AF_INET, 0);
    if (!udp_sock || !raw_sock)
        return fprintf(stderr, "socket create failed\n"), 2;

    stage = "netif_open";
    static pcap_data_t data = {.ip = "192.168.74.2", .hwaddr = our_mac};
    wire = netif_open("netif 0", &netdev_ops, &data); /* pcap_device_open, recv_thread, xmit_thread */
    if (!wire)
        return fprintf(stderr, "netif_open over the pcap double failed\n"), 2;
    ipaddr_t ip, mask, gw;
    ipaddr_from_str(&ip, "10.0.0.1");
    ipaddr_from_str(&mask, "255.255.255.0");
    ipaddr_from_str(&gw, "10.0.0.254");
    netif_set_addr(wire, &ip, &mask, &gw);
    netif_set_active(wire); /* gratuitous ARP out (ether_open); default route via gw */
    net_start();
    if (pcapd_wait_injected(1, 10000) != 0)
        return fprintf(stderr, "the gratuitous ARP never left xmit_thread\n"), 3;
    printf("pcap netif '%s' up over the double: %u tx fixtures, %u rx fixtures (non-fragment, <= %d B; %u ICMP "
           "frames skipped: the reference walks a stale cursor off their block list)\n",
           wire->name, n_tx, n_rx, ETHER_MTU_BYTES, n_rx_undefined);

    stage = "tx";
    run_tx(0, n_tx, "tx");
    print_stats("after tx");

    stage = "rx";
    uint32_t reply0 = pcapd_injected_count();
    run_rx(0, n_rx, "rx");
    usleep(200000); /* the last replies leave */
    check_replies(reply0, "rx_replies");
    print_stats("after rx");

    stage = "faults";
    run_faults();
    print_stats("after faults");

    if (concurrent) {
        stage = "concurrent";
        exmsg_func_exec(restore_addr, (void *)0);
        sys_thread_create(echo_server, (void *)0);
        sys_sleep(50);
        net_csum_gpu_stats_t s0, s1;
        stats(&s0);
        pthread_t cl;
        pthread_create(&cl, NULL, echo_client, NULL);
        int ok = run_tx(0, n_tx, "concurrent_tx");
        pthread_join(cl, NULL);
        stats(&s1);
        phase("concurrent", ok && echo_rc == 0,
              "loop echo (%d datagrams, rc %d) while the pcap xmit_thread sent %u frames: %llu tx batches "
              "from both threads",
              ECHO_ROUNDS, echo_rc, n_tx, (unsigned long long)(s1.tx_batches - s0.tx_batches));
    }
    print_stats("final");
    alarm(0);
    printf("pcap_wire: %s\n", failures ? "FAIL" : "all phases ok");
    fflush(stdout);
    _exit(failures ? 1 : 0); /* the stack's threads never return */
}
