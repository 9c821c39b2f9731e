/*
 * stack_tap_ipv4.c -- TEST INFRASTRUCTURE ONLY (oracle/Makefile target `stack`).
 *
 * The reference's net/src/ipv4.c is compiled here, unmodified and in place
 * (the #include below resolves to /root/reference/net/src/ipv4.c through the
 * Makefile's -I), so that stack_gen can run its receive steps one by one.
 * Nothing of ipv4.c is restated: tap_ipv4_rx only sequences the reference's
 * own functions the way ipv4_in does, and keeps the value ip_normal_in
 * returns, which ipv4_in throws away (ipv4.c:512-514).
 */
#include "ipv4.c"

#include "stack_gen.h"

net_err_t tap_ipv4_rx(netif_t *netif, pktbuf_t *buf, unsigned *gate)
{
    *gate = TAP_GATE_IPV4;
    net_err_t err = pktbuf_set_cont(buf, sizeof(ipv4_hdr_t)); /* ipv4.c:475 */
    if (err < 0)
        return err;
    ipv4_pkt_t *pkt = (ipv4_pkt_t *)pktbuf_data(buf);
    err = is_pkt_ok(pkt, buf->total_size, netif); /* ipv4.c:482 */
    if (err != NET_ERR_OK)
        return err;
    iphdr_ntohs(pkt); /* ipv4.c:489 */
    err = pktbuf_resize(buf, pkt->hdr.total_len); /* ipv4.c:490 */
    if (err < 0)
        return err;
    ipaddr_t dest_ip, src_ip;
    ipaddr_from_buf(&dest_ip, pkt->hdr.dest_ip);
    ipaddr_from_buf(&src_ip, pkt->hdr.src_ip);
    if (!ipaddr_is_match(&dest_ip, &netif->ipaddr, &netif->netmask)) /* ipv4.c:501 */
        return NET_ERR_UNREACHABLE;
    if (pkt->hdr.frag_offset || pkt->hdr.more) { /* ipv4.c:506 */
        *gate = TAP_GATE_FRAG;
        return NET_ERR_OK;
    }
    *gate = TAP_GATE_L4;
    return ip_normal_in(netif, buf, &src_ip, &dest_ip); /* ipv4.c:512 */
}
