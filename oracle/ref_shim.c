/*
 * ref_shim.c -- calls the REFERENCE's checksum_peso (net/src/tools.c:56) on a
 * contiguous segment, for bench.py's cpu_baseline leg ("kind": "reference").
 *
 * TEST INFRASTRUCTURE ONLY.  Compiled by oracle/Makefile together with the
 * unmodified reference sources into oracle/_ref/libtcpref.so.
 *
 * The segment is exposed to the reference as a pktbuf_t whose 127-byte blocks
 * (net/net/net_cfg.h:31) point straight into the segment -- the layout the
 * stack's own pktbuf_alloc produces, without a copy -- so the time measured
 * is the reference's block walk + checksum16 loop, as it runs in-stack
 * (tcp_out.c:20, udp.c:321).  One chain per thread, re-aimed per segment.
 */
#include <string.h>

#include "ipaddr.h"
#include "list.h"
#include "pktbuf.h"
#include "tools.h"

#define SHIM_MAX_BLKS 4096 /* up to 520,192-byte segments */

static __thread pktblk_t shim_blks[SHIM_MAX_BLKS];
static __thread pktbuf_t shim_buf;
static __thread int shim_ready;

/* Aim the thread's block chain at `seg`: the first ceil(len/127) blocks get
 * their size/data and are linked, the list is cut after the last one.  Only
 * the fields the stack's own pktbuf_alloc would have set are written, so
 * re-aiming costs a few stores per block for any mix of lengths (the payload
 * arrays are never touched: data points into the segment). */
static pktbuf_t *aim_chain(const uint8_t *seg, int len)
{
    if (!shim_ready) {
        memset(shim_blks, 0, sizeof shim_blks);
        for (int i = 1; i < SHIM_MAX_BLKS; ++i)
            shim_blks[i].node.pre = &shim_blks[i - 1].node;
        shim_ready = 1;
    }
    int left = len, k = 0;
    while (left > 0 && k < SHIM_MAX_BLKS) {
        int take = left > PKTBUF_BLK_SIZE ? PKTBUF_BLK_SIZE : left;
        pktblk_t *b = &shim_blks[k];
        b->size = take;
        b->data = (uint8_t *)seg + (len - left);
        b->node.next = k + 1 < SHIM_MAX_BLKS ? &shim_blks[k + 1].node : (node_t *)0;
        left -= take;
        ++k;
    }
    memset(&shim_buf, 0, sizeof shim_buf);
    if (k) {
        shim_blks[k - 1].node.next = (node_t *)0;
        shim_buf.blk_list.first = &shim_blks[0].node;
        shim_buf.blk_list.last = &shim_blks[k - 1].node;
    }
    shim_buf.blk_list.count = k;
    shim_buf.total_size = len - left;
    shim_buf.ref = 1;
    return &shim_buf;
}

/* Same shape as orc_peso_fn (oracle/csum_oracle.h). */
uint16_t tcpref_peso(const uint8_t *seg, uint32_t len, const uint8_t dest[4],
                     const uint8_t src[4], uint8_t protocol)
{
    ipaddr_t d, s;
    d.type = IPADDR_V4;
    s.type = IPADDR_V4;
    memcpy(d.addr, dest, 4);
    memcpy(s.addr, src, 4);
    return checksum_peso(aim_chain(seg, (int)len), &d, &s, protocol);
}

/* The reference's flat routine, exported under a distinct name so that a
 * process which also loads the product library never interposes the two. */
uint16_t tcpref_checksum16(int offset, void *buf, uint16_t len, uint32_t pre_sum,
                           int complement)
{
    return checksum16(offset, buf, len, pre_sum, complement);
}
