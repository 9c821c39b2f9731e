/*
 * stack_gen.h -- TEST INFRASTRUCTURE ONLY.  Shared by oracle/stack_gen.c and
 * the oracle/stack_tap_*.c translation units, which compile the reference's
 * own ipv4.c / tcp_out.c / icmpv4.c in place (by #include) to reach their
 * static functions.  Built by `make -C oracle stack`; never linked into the
 * product.
 */
#ifndef TCSUM_STACK_GEN_H
#define TCSUM_STACK_GEN_H

#include "icmpv4.h"
#include "ipaddr.h"
#include "netif.h"
#include "pktbuf.h"
#include "tcp.h"

/* Which of the reference's receive functions produced an rx verdict. */
#define TAP_GATE_IPV4 1u /* ipv4_in itself: pktbuf_set_cont / is_pkt_ok / resize (ipv4.c:475-505) */
#define TAP_GATE_FRAG 2u /* a fragment: queued for reassembly, ipv4_in returns OK (ipv4.c:506-509) */
#define TAP_GATE_L4 3u   /* ip_normal_in's return: tcp_in / udp_in / icmpv4_in / raw_in (ipv4.c:420-470) */

/* ipv4_in (ipv4.c:472-515) step by step, every step the reference's own code,
 * returning what ip_normal_in returns instead of discarding it
 * (ipv4.c:512-514); *gate says which stage decided. */
net_err_t tap_ipv4_rx(netif_t *netif, pktbuf_t *buf, unsigned *gate);

/* tcp_out.c:10-31 send_out (static there). */
net_err_t tap_tcp_send_out(tcp_hdr_t *out, pktbuf_t *buf, ipaddr_t *dest, ipaddr_t *src);

/* icmpv4.c:45-52 icmpv4_out (static there). */
net_err_t tap_icmpv4_out(ipaddr_t *dest, ipaddr_t *src, pktbuf_t *buf);

#endif
