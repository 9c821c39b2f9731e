/*
 * stack_gen.c -- IPv4 tx/rx fixtures taken from the REFERENCE STACK's own
 * transmit and receive code.  TEST INFRASTRUCTURE ONLY.
 *
 * Built by `make -C oracle stack` in the build container: every file of the
 * reference's net/src plus plat/sys_plat.c and plat/net_plat.c is compiled in
 * place under /root/reference (ipv4.c, tcp_out.c and icmpv4.c through the
 * stack_tap_*.c units, which #include them to reach their static functions),
 * and linked with this driver.  The binary goes to oracle/_ref/; only the data
 * files it writes are committed (tests/golden/).
 *
 * What it writes
 *   stack_tx_{cases,in,out}.bin  frames the reference's transmit path built
 *       and checksummed: udp_out (udp.c:295-330), send_out (tcp_out.c:10-31),
 *       icmpv4_out (icmpv4.c:45-52), ipv4_out for other protocols
 *       (ipv4.c:594-665) and ip_frag_out (ipv4.c:517-591), captured where the
 *       stack hands them to its netif driver (netif_out -> ops->xmit,
 *       netif.c:364-386).  `out` is the frame as the reference sent it; `in`
 *       is the same frame with the checksum fields the reference filled set to
 *       junk (the IPv4 header checksum always; the L4 field unless the frame
 *       is a fragment -- ip_frag_out copies the L4 bytes checksummed over the
 *       whole datagram and fills only the header, ipv4.c:574).
 *   ipv4_rx_{cases,pool}.bin  frames and the net_err_t the reference's receive
 *       path returns for each: tap_ipv4_rx (stack_tap_ipv4.c) runs ipv4_in's
 *       own steps and keeps ip_normal_in's return -- tcp_in (tcp_in.c:54-124),
 *       udp_in (udp.c:382-447), icmpv4_in (icmpv4.c:62-103), raw_in
 *       (raw.c:214-236).  Each verdict is cross-checked against the real
 *       ipv4_in (ipv4.c:472) on the same frame.
 *
 * The stack state the verdicts assume (socket lookup and routing are not
 * what the checksum path decides): the netif's address is each packet's
 * destination (ipv4.c:501 matches), a UDP socket is bound to each datagram's
 * destination port on any address (udp.c:335-369 finds it unless the port is
 * 0), a raw socket of protocol 0 is open (raw.c:188-211 takes every
 * protocol), no TCP connection exists (tcp_in.c:117-124: tcp_closed_in, OK),
 * and a default route leads to the capture netif (replies go out there).
 *
 * Two platform details, both about the reference on Linux:
 *  - sys_mutex_create makes a default (non-recursive) pthread mutex
 *    (sys_plat.c:399-407) and pktbuf_free takes the pktbuf lock twice
 *    (pktbuf.c:203 -> :44): the first free deadlocks.  On the reference's
 *    primary platform CreateMutex is recursive (sys_plat.c:215-221).  The
 *    Makefile weakens the Linux definition and this file supplies a recursive
 *    one; no other platform function is replaced.
 *  - is_pkt_ok sums hdr_len bytes from a pointer made contiguous for 20 only
 *    (ipv4.c:243 vs :475).  Frames are therefore built the way the pcap driver
 *    builds them (pktbuf_alloc + pktbuf_write, netif_pcap.c:23-30) and the
 *    header is then made contiguous with the reference's pktbuf_set_cont, the
 *    layout in which that read stays inside the packet.
 * Frames on which the reference has no defined behaviour are not emitted
 * (see ref_defined): a nonzero header checksum with IHL*4 past the captured
 * bytes (the sum reads beyond the frame), and TCP with IHL*4 > total_len
 * (pktbuf_remove_header runs off the block list, pktbuf.c:264-281, a NULL
 * dereference).  include/tcsum.h documents the value returned for them.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "exmsg.h"
#include "icmpv4.h"
#include "ipv4.h"
#include "net_cfg.h"
#include "netif.h"
#include "pktbuf.h"
#include "raw.h"
#include "sock.h"
#include "tcp.h"
#include "timer.h"
#include "tools.h"
#include "udp.h"

#include "stack_gen.h"

/* ------------------------------------------------------------ platform */

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

/* ------------------------------------------------------------ helpers */

static uint64_t rng_state = 0x57AC4B17ull;
static uint64_t sm64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static uint64_t rnd(void) { return sm64(rng_state++); }
static uint32_t rnd_below(uint32_t n) { return n ? (uint32_t)(rnd() % n) : 0; }
static void rnd_fill(uint8_t *p, uint32_t n)
{
    for (uint32_t i = 0; i < n; i++)
        p[i] = (uint8_t)rnd();
}

static const char *outdir;
static FILE *open_out(const char *name)
{
    char path[1024];
    snprintf(path, sizeof path, "%s/%s", outdir, name);
    FILE *f = fopen(path, "wb");
    if (!f) {
        perror(path);
        exit(2);
    }
    return f;
}
static void put_u32(FILE *f, uint32_t v) { fwrite(&v, 4, 1, f); }

static void die(const char *what, long a, long b)
{
    fprintf(stderr, "stack_gen: %s (%ld, %ld)\n", what, a, b);
    exit(3);
}

/* The batch API's flag classification (TCSUM_PKT_* in include/tcsum.h): a
 * builder-defined description of the packet, not a reference output. */
#define F_BAD_VERSION 0x01u
#define F_BAD_HDRLEN 0x02u
#define F_BAD_TOTLEN 0x04u
#define F_PROTO_OTHER 0x08u
#define F_SHORT 0x10u
#define F_FRAGMENT 0x20u
#define F_L4_SHORT 0x40u

static uint32_t l4_min(uint8_t proto) { return proto == 6 ? 20 : proto == 17 ? 8 : proto == 1 ? 4 : 0; }
static uint32_t l4_fld(uint8_t proto) { return proto == 6 ? 16 : proto == 17 ? 6 : proto == 1 ? 2 : 0; }
static uint32_t ihl4_of(const uint8_t *p) { return (uint32_t)(p[0] & 15) * 4; }
static uint32_t tl_of(const uint8_t *p) { return ((uint32_t)p[2] << 8) | p[3]; }
static int frag_of(const uint8_t *p) { return (p[6] & 0x20) || (((p[6] & 0x1F) << 8) | p[7]); }

static uint32_t api_flags(const uint8_t *p, uint32_t frame)
{
    if (frame < 20)
        return F_SHORT;
    uint32_t fl = 0, ihl4 = ihl4_of(p), tl = tl_of(p);
    if ((p[0] >> 4) != 4)
        fl |= F_BAD_VERSION;
    if (ihl4 < 20 || ihl4 > frame)
        fl |= F_BAD_HDRLEN;
    if (tl < 20 || tl > frame || tl < ihl4)
        fl |= F_BAD_TOTLEN;
    if (frag_of(p))
        fl |= F_FRAGMENT;
    uint32_t hl = ihl4 < 20 ? 20 : ihl4;
    hl = hl > frame ? frame : hl;
    uint32_t end = tl < hl ? hl : tl;
    end = end > frame ? frame : end;
    uint8_t proto = p[9];
    if (l4_min(proto) && end - hl < l4_min(proto))
        fl |= F_L4_SHORT;
    if (proto != 6 && proto != 17 && proto != 1)
        fl |= F_PROTO_OTHER;
    return fl;
}

/* ------------------------------------------------------------ the stack */

static netif_t *cap;
static udp_t *udp_sock;
static raw_t *raw_sock;

#define CAP_BYTES (8u << 20)
#define CAP_MAX 16384
static uint8_t cap_bytes[CAP_BYTES];
static uint32_t cap_used, ncap, cap_off[CAP_MAX], cap_len[CAP_MAX];
static int capturing;

/* A loopback-type netif (no link layer, like loop.c:7-11), so ipv4_out's
 * frames reach the driver as IPv4 packets (netif.c:377-385). */
static net_err_t cap_open(struct netif_t *netif, void *data)
{
    netif->type = NETIF_TYPE_LOOP;
    return NET_ERR_OK;
}
static void cap_close(struct netif_t *netif) {}
/* The driver end of the stack (netif.c:380-384 calls it after netif_put_out):
 * every frame the stack transmits is copied out here, as netif_pcap.c's
 * xmit_thread copies it for pcap_inject (netif_pcap.c:42-67). */
static net_err_t cap_xmit(struct netif_t *netif)
{
    pktbuf_t *b;
    while ((b = netif_get_out(netif, -1)) != (pktbuf_t *)0) {
        if (capturing && b->total_size > 0 && ncap < CAP_MAX && cap_used + b->total_size <= CAP_BYTES) {
            if (pktbuf_read(b, cap_bytes + cap_used, b->total_size) != NET_ERR_OK)
                die("pktbuf_read", b->total_size, 0);
            cap_off[ncap] = cap_used;
            cap_len[ncap++] = (uint32_t)b->total_size;
            cap_used += (uint32_t)b->total_size;
        }
        pktbuf_free(b);
    }
    return NET_ERR_OK;
}
static const netif_ops_t cap_ops = {cap_open, cap_close, cap_xmit};

static void stack_init(void)
{
    tools_init();
    exmsg_init();
    pktbuf_init();
    netif_init();
    net_timer_init();
    ipv4_init();
    icmpv4_init();
    socket_init();
    raw_init();
    udp_init();
    tcp_init();
    cap = netif_open("cap", &cap_ops, (void *)0);
    if (!cap)
        die("netif_open", 0, 0);
    ipaddr_t ip, mask, gw;
    ipaddr_from_str(&ip, "10.0.0.1");
    ipaddr_from_str(&mask, "255.255.255.0");
    ipaddr_from_str(&gw, "10.0.0.254");
    netif_set_addr(cap, &ip, &mask, &gw);
    if (netif_set_active(cap) != NET_ERR_OK)
        die("netif_set_active", 0, 0);
    rt_add(ipaddr_get_any(), ipaddr_get_any(), &gw, cap); /* a default route, as netif_set_default adds */
    udp_sock = (udp_t *)udp_create(AF_INET, IPPROTO_UDP);
    raw_sock = (raw_t *)raw_create(AF_INET, 0);
    if (!udp_sock || !raw_sock)
        die("socket create", 0, 0);
}

/* A fresh packet pool per case: buffers the stack keeps (socket receive
 * lists) are dropped with it. */
static void fresh(void)
{
    pktbuf_init();
    list_init(&udp_sock->recv_list);
    list_init(&raw_sock->recv_list);
    cap->mtu = 0;
}

static pktbuf_t *make_buf(const uint8_t *bytes, uint32_t len)
{
    pktbuf_t *b = pktbuf_alloc((int)len);
    if (!b)
        die("pktbuf_alloc", len, 0);
    if (len && pktbuf_write(b, bytes, (int)len) != NET_ERR_OK)
        die("pktbuf_write", len, 0);
    pktbuf_reset_access(b);
    return b;
}

static ipaddr_t rnd_addr(void)
{
    ipaddr_t a;
    memset(&a, 0, sizeof a);
    a.type = IPADDR_V4;
    do
        a.q_addr = (uint32_t)rnd();
    while (a.q_addr == 0);
    return a;
}

/* ------------------------------------------------------------ transmit */

/* ip_frag_out writes a 20-byte header through pktbuf_data of a fresh
 * pktbuf_alloc(curr + 20) (ipv4.c:533-548), whose first block holds only
 * ((curr + 20 - 1) % 127) + 1 bytes: below 20 the header runs past that
 * block.  Skip datagram sizes that make the reference do that. */
static int frag_safe(uint32_t total, uint32_t mtu)
{
    if (!mtu || total + 20 <= mtu)
        return 1;
    while (total) {
        uint32_t curr = total + 20 > mtu ? mtu - 20 : total;
        if (((curr + 20 - 1) % PKTBUF_BLK_SIZE) + 1 < 20)
            return 0;
        total -= curr;
    }
    return 1;
}

static uint32_t pick_mtu(void)
{
    uint32_t r = rnd_below(100);
    return r < 78 ? 0 : r < 86 ? 1500 : r < 94 ? 576 : r < 98 ? 1006 : 68;
}

static uint8_t scratch[16384];

static void tx_udp(uint32_t plen, uint32_t mtu)
{
    if (!frag_safe(plen + 8, mtu))
        return;
    fresh();
    cap->mtu = (int)mtu;
    rnd_fill(scratch, plen);
    pktbuf_t *b = make_buf(scratch, plen);
    ipaddr_t d = rnd_addr(), s = rnd_addr();
    uint16_t sport = (uint16_t)rnd(), dport = (uint16_t)rnd();
    capturing = 1;
    net_err_t e = udp_out(&d, dport, &s, sport, b); /* udp.c:295 */
    capturing = 0;
    if (e != NET_ERR_OK)
        die("udp_out", e, plen);
}

static void tx_tcp(uint32_t plen, uint32_t mtu)
{
    uint32_t hdr = rnd_below(100) < 70 ? 20 : 20 + 4 * (1 + rnd_below(10));
    if (!frag_safe(hdr + plen, mtu))
        return;
    fresh();
    cap->mtu = (int)mtu;
    memset(scratch, 0, hdr);
    rnd_fill(scratch + hdr, plen);
    if (hdr > 20) { /* an MSS option, then NOPs, as tcp_out writes on SYN */
        scratch[20] = 2;
        scratch[21] = 4;
        scratch[22] = (uint8_t)rnd();
        scratch[23] = (uint8_t)rnd();
        memset(scratch + 24, 1, hdr - 24);
    }
    pktbuf_t *b = make_buf(scratch, hdr + plen);
    if (pktbuf_set_cont(b, (int)hdr) != NET_ERR_OK)
        die("set_cont tcp", hdr, plen);
    tcp_hdr_t *h = (tcp_hdr_t *)pktbuf_data(b);
    h->sport = (uint16_t)(1 + rnd_below(65535));
    h->dport = (uint16_t)(1 + rnd_below(65535));
    h->seq = (uint32_t)rnd();
    h->ack = (uint32_t)rnd();
    h->flag = 0;
    tcp_set_hdr_size(h, (int)hdr);
    ((uint8_t *)h)[13] = (uint8_t)(rnd_below(4) ? (0x10 | (rnd() & 0x0F)) : rnd()); /* ACK + some, or any */
    h->win = (uint16_t)rnd();
    h->urg_ptr = (uint16_t)(rnd_below(4) ? 0 : rnd());
    ipaddr_t d = rnd_addr(), s = rnd_addr();
    capturing = 1;
    net_err_t e = tap_tcp_send_out(h, b, &d, &s); /* tcp_out.c:10 */
    capturing = 0;
    if (e != NET_ERR_OK)
        die("send_out", e, plen);
}

static void tx_icmp(uint32_t plen, uint32_t mtu)
{
    if (!frag_safe(8 + plen, mtu))
        return;
    fresh();
    cap->mtu = (int)mtu;
    static const uint8_t types[] = {0, 3, 8, 11, 13, 0, 8};
    scratch[0] = types[rnd_below(sizeof types)];
    scratch[1] = (uint8_t)rnd_below(16);
    scratch[2] = scratch[3] = 0; /* the callers zero it: icmpv4.c:58, :123 */
    rnd_fill(scratch + 4, 4 + plen);
    pktbuf_t *b = make_buf(scratch, 8 + plen);
    if (pktbuf_set_cont(b, 8) != NET_ERR_OK)
        die("set_cont icmp", plen, 0);
    ipaddr_t d = rnd_addr(), s = rnd_addr();
    capturing = 1;
    net_err_t e = tap_icmpv4_out(&d, &s, b); /* icmpv4.c:45 */
    capturing = 0;
    if (e != NET_ERR_OK)
        die("icmpv4_out", e, plen);
}

static void tx_raw(uint32_t plen, uint32_t mtu)
{
    if (!frag_safe(plen, mtu))
        return;
    fresh();
    cap->mtu = (int)mtu;
    uint8_t proto;
    do
        proto = (uint8_t)rnd();
    while (proto == 1 || proto == 6 || proto == 17);
    rnd_fill(scratch, plen);
    pktbuf_t *b = make_buf(scratch, plen);
    ipaddr_t d = rnd_addr(), s = rnd_addr();
    capturing = 1;
    net_err_t e = ipv4_out(proto, &d, &s, b); /* ipv4.c:594, as raw_sendto calls it */
    capturing = 0;
    if (e != NET_ERR_OK)
        die("ipv4_out", e, plen);
}

static uint32_t pick_plen(uint32_t cap_len_)
{
    uint32_t r = rnd_below(100);
    uint32_t v = r < 5 ? 1 + rnd_below(8) : r < 30 ? 1 + rnd_below(200) : 1 + rnd_below(cap_len_);
    return v;
}

static void gen_tx(int rounds)
{
    for (int i = 0; i < rounds; i++) {
        uint32_t k = rnd_below(100), mtu = pick_mtu();
        if (k < 35)
            tx_udp(pick_plen(2900), mtu);
        else if (k < 75)
            tx_tcp(rnd_below(10) == 0 ? 0 : pick_plen(2900), mtu);
        else if (k < 90)
            tx_icmp(pick_plen(2900), mtu);
        else
            tx_raw(pick_plen(2900), mtu);
    }
}

/* ------------------------------------------------------------ receive */

/* Frames on which the reference's receive path has defined behaviour. */
static int ref_defined(const uint8_t *p, uint32_t frame)
{
    if (frame < 20 || (p[0] >> 4) != 4)
        return 1;
    uint32_t ihl4 = ihl4_of(p), tl = tl_of(p);
    if (ihl4 < 20 || tl < 20 || frame < tl)
        return 1;
    if ((p[10] | p[11]) && ihl4 > frame) /* ipv4.c:243 sums past the captured bytes */
        return 0;
    if (!frag_of(p) && p[9] == 6 && ihl4 > tl) /* ipv4.c:451 -> pktbuf.c:264-281 NULL deref */
        return 0;
    return 1;
}

static pktbuf_t *rx_buf(const uint8_t *f, uint32_t len)
{
    pktbuf_t *b = make_buf(f, len);
    if (len >= 20) {
        uint32_t hc = ihl4_of(f);
        hc = hc < 20 ? 20 : hc;
        hc = hc > len ? len : hc;
        if (pktbuf_set_cont(b, (int)hc) != NET_ERR_OK)
            die("set_cont rx", hc, len);
        pktbuf_reset_access(b); /* the cursor netif_get_in hands over (netif.c:327) */
        memcpy(&cap->ipaddr.q_addr, f + 16, 4); /* the netif is every packet's destination */
        uint32_t ihl4 = ihl4_of(f), tl = tl_of(f);
        if (ihl4 + 4 <= tl && tl <= len) /* the bound UDP socket's port */
            udp_sock->base.local_port = (uint16_t)(((uint32_t)f[ihl4 + 2] << 8) | f[ihl4 + 3]);
    }
    return b;
}

static int32_t ref_rx(const uint8_t *f, uint32_t len, uint32_t *gate)
{
    fresh();
    pktbuf_t *b = rx_buf(f, len);
    unsigned g;
    net_err_t e = tap_ipv4_rx(cap, b, &g);
    *gate = g;
    if (g != TAP_GATE_FRAG) { /* cross-check with the real ipv4_in (fragments would stay queued) */
        fresh();
        pktbuf_t *b2 = rx_buf(f, len);
        net_err_t e2 = ipv4_in(cap, b2);
        if (e2 != (g == TAP_GATE_IPV4 ? e : NET_ERR_OK))
            die("ipv4_in disagrees with tap_ipv4_rx", e2, e);
    }
    return e;
}

/* Checksums refilled with the reference's own routines after a header edit
 * (L4 first, then the IPv4 header, the order the tx path stores them). */
static uint16_t ref_l4_sum(const uint8_t *p, uint32_t ihl4, uint32_t tl)
{
    pktbuf_init();
    pktbuf_t *b = make_buf(p + ihl4, tl - ihl4);
    if (p[9] == 1)
        return pktbuf_checksum16(b, b->total_size, 0, 1); /* icmpv4.c:49 */
    ipaddr_t d, s;
    ipaddr_from_buf(&d, p + 16);
    ipaddr_from_buf(&s, p + 12);
    return checksum_peso(b, &d, &s, p[9]); /* tcp_out.c:20, udp.c:321 */
}

static void refill(uint8_t *p, uint32_t frame, int l4)
{
    uint32_t ihl4 = ihl4_of(p), tl = tl_of(p);
    if (ihl4 < 20 || ihl4 > frame)
        return;
    uint8_t proto = p[9];
    if (l4 && !frag_of(p) && l4_fld(proto) && tl <= frame && tl >= ihl4 + l4_min(proto)) {
        uint8_t *fp = p + ihl4 + l4_fld(proto);
        fp[0] = fp[1] = 0;
        uint16_t v = ref_l4_sum(p, ihl4, tl);
        memcpy(fp, &v, 2);
    }
    p[10] = p[11] = 0;
    uint16_t h = checksum16(0, p, (uint16_t)ihl4, 0, 1); /* ipv4.c:656 */
    memcpy(p + 10, &h, 2);
}

/* A random packet: mostly well formed, with the odd broken field. */
static uint32_t make_packet(uint8_t *p, uint32_t max_frame)
{
    uint32_t fr = rnd_below(100);
    uint32_t frame = fr < 2 ? rnd_below(20) : fr < 12 ? 20 + rnd_below(100) : 64 + rnd_below(max_frame - 64 + 1);
    rnd_fill(p, frame);
    if (frame < 20)
        return frame;
    uint32_t ihl = rnd_below(100) < 80 ? 5 : 5 + rnd_below(11);
    if (ihl * 4 > frame)
        ihl = 5;
    uint32_t vr = rnd_below(100);
    uint32_t ver = vr < 96 ? 4 : vr < 98 ? 6 : rnd_below(16);
    if (rnd_below(100) < 2)
        ihl = rnd_below(5);
    p[0] = (uint8_t)((ver << 4) | ihl);
    uint32_t tr = rnd_below(100), tl;
    if (tr < 85)
        tl = frame;
    else if (tr < 93)
        tl = ihl * 4 + rnd_below(frame - ihl * 4 + 1);
    else
        tl = rnd_below(0x10000);
    p[2] = (uint8_t)(tl >> 8);
    p[3] = (uint8_t)tl;
    uint32_t fg = rnd_below(100);
    p[6] = fg < 85 ? 0x40 : (uint8_t)rnd();
    p[7] = fg < 85 ? 0 : (uint8_t)rnd();
    uint32_t pr = rnd_below(100);
    p[9] = pr < 42 ? 6 : pr < 84 ? 17 : pr < 92 ? 1 : (uint8_t)rnd();
    p[10] = p[11] = 0;
    if (rnd_below(3))
        refill(p, frame, 1);
    return frame;
}

static void set_tl(uint8_t *p, uint32_t tl)
{
    p[2] = (uint8_t)(tl >> 8);
    p[3] = (uint8_t)tl;
}

/* Edits that reach the L4 gates behind the checksum test (tcp_in.c:87-103,
 * udp.c:337-340): TCP ports / flag word zeroed or the data offset past the
 * segment, UDP destination port 0; checksums refilled (mostly), so the gate
 * itself decides.  0 when the frame is not an unfragmented TCP/UDP one. */
static int gate_edit(uint8_t *p, uint32_t frame)
{
    uint32_t ihl4 = ihl4_of(p), tl = tl_of(p);
    uint8_t proto = p[9];
    if (frag_of(p) || (proto != 6 && proto != 17) || tl > frame || tl < ihl4 + l4_min(proto))
        return 0;
    uint8_t *t = p + ihl4;
    if (proto == 17) {
        t[2] = t[3] = 0;
        if (rnd_below(3) == 0)
            t[0] = t[1] = 0; /* source port 0 is no gate */
    } else {
        uint32_t w = rnd_below(5);
        if (w == 0)
            t[0] = t[1] = 0;
        else if (w == 1)
            t[2] = t[3] = 0;
        else if (w == 2)
            t[12] = t[13] = 0;
        else if (w == 3)
            t[13] = 0; /* flags only: the data offset keeps the word nonzero */
        else {
            uint32_t seg = tl - ihl4, doff = 6 + rnd_below(10);
            t[12] = (uint8_t)((doff << 4) | (t[12] & 15));
            if (doff * 4 <= seg) /* cut the segment to 20..doff*4-1 bytes */
                set_tl(p, ihl4 + 20 + rnd_below(doff * 4 - 20));
        }
    }
    refill(p, frame, rnd_below(6) != 0); /* sometimes a stale checksum too */
    return 1;
}

/* One receive case derived from a frame the reference transmitted: damaged
 * the way a receiver meets frames, or edited to reach a particular gate
 * (then refilled, so the checksum gates pass and the later gate decides). */
static uint32_t damage(uint8_t *p, uint32_t frame, uint32_t room)
{
    uint32_t ihl4 = ihl4_of(p), tl = tl_of(p);
    uint8_t proto = p[9];
    uint32_t k = rnd_below(100);
    if (k < 20) /* clean */
        return frame;
    if (k < 32) { /* payload bit flip */
        if (tl > ihl4)
            p[ihl4 + rnd_below(tl - ihl4)] ^= (uint8_t)(1u << rnd_below(8));
        return frame;
    }
    if (k < 40) { /* header bit flip, any bit */
        p[rnd_below(ihl4)] ^= (uint8_t)(1u << rnd_below(8));
        return frame;
    }
    if (k < 45) { /* zeroed header checksum + a flip in the addresses */
        p[10] = p[11] = 0;
        p[12 + rnd_below(8)] ^= 1;
        return frame;
    }
    if (k < 52) { /* zeroed L4 checksum + payload flip: skipped (tcp_in.c:77, udp.c:407) */
        if (l4_fld(proto) && !frag_of(p) && tl >= ihl4 + l4_min(proto)) {
            p[ihl4 + l4_fld(proto)] = p[ihl4 + l4_fld(proto) + 1] = 0;
            p[ihl4 + rnd_below(tl - ihl4)] ^= 0x10;
        }
        return frame;
    }
    if (k < 57) /* captured short: frame < total_len */
        return rnd_below(frame);
    if (k < 61) { /* trailing bytes after total_len (Ethernet padding) */
        uint32_t extra = 1 + rnd_below(46);
        if (frame + extra > room)
            return frame;
        rnd_fill(p + frame, extra);
        return frame + extra;
    }
    if (k < 70 && gate_edit(p, frame))
        return frame;
    if (k < 77) { /* L4 shorter than its header: total_len = IHL*4 + 0..min-1 */
        uint32_t m = l4_min(proto) ? l4_min(proto) : 8;
        uint32_t ntl = ihl4 + rnd_below(m);
        set_tl(p, ntl);
        refill(p, frame, 0);
        return rnd_below(2) ? ntl : frame;
    }
    if (k < 85) { /* IPv4 options inserted: IHL 6..15, L4 unchanged */
        uint32_t opt = 4 * (1 + rnd_below(10));
        if (frame + opt > room || ihl4 != 20)
            return frame;
        memmove(p + 20 + opt, p + 20, frame - 20);
        memset(p + 20, 1, opt); /* NOPs */
        if (rnd_below(2))
            p[20 + opt - 1] = 0; /* end of options */
        p[0] = (uint8_t)(0x40 | ((20 + opt) / 4));
        set_tl(p, tl + opt);
        refill(p, frame + opt, 0);
        return frame + opt;
    }
    if (k < 90) { /* IHL*4 beyond total_len (still within the frame) */
        uint32_t ihl = 6 + rnd_below(10);
        if (ihl * 4 > frame)
            return frame;
        p[0] = (uint8_t)(0x40 | ihl);
        uint32_t ntl = 20 + rnd_below(ihl * 4 - 20);
        set_tl(p, ntl);
        refill(p, frame, 0);
        return frame;
    }
    if (k < 95) { /* version or total_len garbage */
        if (rnd_below(2))
            p[0] = (uint8_t)((rnd_below(16) << 4) | (p[0] & 15));
        else
            set_tl(p, rnd_below(0x10000));
        refill(p, frame, 0);
        return frame;
    }
    /* a stale L4 checksum with a correct header */
    if (l4_fld(proto) && !frag_of(p) && tl >= ihl4 + l4_min(proto))
        p[ihl4 + l4_fld(proto)] ^= (uint8_t)(1 + rnd_below(255));
    return frame;
}

/* ------------------------------------------------------------ fixtures */

#define POOL_CAP (16u << 20)
static uint8_t pool_in[POOL_CAP], pool_out[POOL_CAP];

static void write_tx(void)
{
    FILE *f = open_out("stack_tx_cases.bin");
    uint32_t at = 0, kinds[4] = {0, 0, 0, 0};
    memset(pool_in, 0, POOL_CAP);
    memset(pool_out, 0, POOL_CAP);
    for (uint32_t i = 0; i < ncap; i++) {
        const uint8_t *fr = cap_bytes + cap_off[i];
        uint32_t len = cap_len[i];
        if (at + len + 64 > POOL_CAP)
            break;
        memcpy(pool_out + at, fr, len);
        memcpy(pool_in + at, fr, len);
        uint8_t *p = pool_in + at;
        uint32_t junk = rnd_below(3);
        p[10] = junk == 0 ? 0 : (uint8_t)rnd();
        p[11] = junk == 0 ? 0 : (uint8_t)rnd();
        uint32_t ihl4 = ihl4_of(p), tl = tl_of(p);
        uint8_t proto = p[9];
        int frag = frag_of(p);
        if (!frag && l4_fld(proto) && tl >= ihl4 + l4_min(proto)) {
            p[ihl4 + l4_fld(proto)] = junk == 0 ? 0 : (uint8_t)rnd();
            p[ihl4 + l4_fld(proto) + 1] = junk == 0 ? 0 : (uint8_t)rnd();
        }
        uint32_t kind = frag ? 3 : proto == 6 ? 0 : proto == 17 ? 1 : 2;
        kinds[kind]++;
        put_u32(f, at);
        put_u32(f, len);
        put_u32(f, api_flags(fr, len));
        put_u32(f, ((uint32_t)proto << 8) | (uint32_t)frag);
        at += len + (rnd_below(4) == 0 ? rnd_below(16) : 0);
    }
    fclose(f);
    FILE *fi = open_out("stack_tx_in.bin");
    fwrite(pool_in, 1, at + 64, fi);
    fclose(fi);
    FILE *fo = open_out("stack_tx_out.bin");
    fwrite(pool_out, 1, at + 64, fo);
    fclose(fo);
    fprintf(stderr, "stack_tx: %u frames (tcp %u, udp %u, icmp/other %u, fragments %u), %u bytes\n", ncap,
            kinds[0], kinds[1], kinds[2], kinds[3], at);
}

static void write_rx(int n_derived, int n_random)
{
    FILE *f = open_out("ipv4_rx_cases.bin");
    uint32_t at = 0, made = 0, skipped = 0;
    int counts[20] = {0};
    static uint8_t work[20000];
    uint32_t base_frames = ncap;
    for (int i = 0; i < n_derived + n_random; i++) {
        uint32_t frame;
        if (i < n_derived) {
            uint32_t src = (uint32_t)i < base_frames ? (uint32_t)i : rnd_below(base_frames);
            frame = cap_len[src];
            memcpy(work, cap_bytes + cap_off[src], frame);
            if ((uint32_t)i >= base_frames && (i % 4 != 0 || !gate_edit(work, frame)))
                frame = damage(work, frame, sizeof work - 64);
        } else {
            frame = make_packet(work, 3000);
        }
        if (!ref_defined(work, frame)) {
            skipped++;
            continue;
        }
        if (at + frame + 64 > POOL_CAP)
            break;
        uint32_t gate;
        int32_t v = ref_rx(work, frame, &gate);
        memcpy(pool_in + at, work, frame);
        put_u32(f, at);
        put_u32(f, frame);
        put_u32(f, (uint32_t)v);
        put_u32(f, api_flags(work, frame));
        put_u32(f, gate | (frame >= 20 ? (uint32_t)work[9] << 8 : 0u));
        counts[-v < 20 && v <= 0 ? -v : 19]++;
        made++;
        at += frame + (rnd_below(4) == 0 ? rnd_below(16) : 0);
    }
    fclose(f);
    FILE *fp = open_out("ipv4_rx_pool.bin");
    fwrite(pool_in, 1, at + 64, fp);
    fclose(fp);
    fprintf(stderr, "ipv4_rx: %u cases (%u undefined in the reference skipped):", made, skipped);
    for (int k = 0; k < 20; k++)
        if (counts[k])
            fprintf(stderr, " %d:%d", -k, counts[k]);
    fprintf(stderr, "\n");
}

int main(int argc, char **argv)
{
    outdir = argc > 1 ? argv[1] : "tests/golden";
    stack_init();
    gen_tx(900);
    write_tx();
    write_rx(3000, 1200);
    return 0;
}
