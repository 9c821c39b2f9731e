/*
 * stack_tap_tx.c -- TEST INFRASTRUCTURE ONLY (oracle/Makefile target `stack`).
 *
 * The reference's net/src/tcp_out.c and net/src/icmpv4.c are compiled here,
 * unmodified and in place (#include through the Makefile's -I), to expose
 * their static transmit functions to stack_gen: send_out (tcp_out.c:10-31)
 * and icmpv4_out (icmpv4.c:45-52).  The two files share no static names.
 */
#include "tcp_out.c"
#include "icmpv4.c"

#include "stack_gen.h"

net_err_t tap_tcp_send_out(tcp_hdr_t *out, pktbuf_t *buf, ipaddr_t *dest, ipaddr_t *src)
{
    return send_out(out, buf, dest, src);
}

net_err_t tap_icmpv4_out(ipaddr_t *dest, ipaddr_t *src, pktbuf_t *buf)
{
    return icmpv4_out(dest, src, buf);
}
