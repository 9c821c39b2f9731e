/*
 * tcsum_cpu_double.c -- a CPU stand-in for the libtcsum.so entry points the
 * patched stack calls (net_csum_gpu.c, the drop-in checksum symbols), backed
 * by the oracle (oracle/csum_oracle.c).  TEST CODE ONLY: it lets the
 * integration programs run in the build container, which has no GPU -- in
 * particular under ThreadSanitizer (integration/Makefile `tsan`), where the
 * question is the stack-side code's thread safety, not the checksums' source.
 * The GPU programs link the real libtcsum.so instead; nothing here is ever
 * part of the product.
 *
 * The three drop-in symbols keep the reference's cursor side effects
 * (pktbuf.c:646-670 moves the cursor by len; checksum_peso resets it and
 * leaves it at the end, tools.c:72-73) by reading the bytes through the
 * reference's own pktbuf_read, which walks the same move_forward.
 */
#include <stdlib.h>
#include <string.h>

#include "csum_oracle.h"
#include "ipaddr.h"
#include "pktbuf.h"
#include "tcsum.h"

int tcsum_device_count(void) { return 1; }
int tcsum_plat_init(int device) { return TCSUM_OK; }
int tcsum_queue_server(int device, int enable) { return TCSUM_OK; }
void *tcsum_host_alloc(size_t bytes) { return calloc(1, bytes ? bytes : 1); }
void tcsum_host_free(void *p) { free(p); }

int tcsum_host_batch_ipv4(int device, const void *host_arena, uint64_t arena_bytes, const tcsum_pkt_t *pkts,
                          uint32_t n, uint32_t *out, uint8_t *flags)
{
    for (uint32_t i = 0; i < n; i++)
        if (pkts[i].offset + pkts[i].len > arena_bytes)
            return TCSUM_ERR_PARAM;
    orc_batch_ipv4((const uint8_t *)host_arena, (const orc_pkt_t *)pkts, n, out, flags, 1);
    return TCSUM_OK;
}

int tcsum_host_batch_ipv4_tx_fill(int device, void *host_arena, uint64_t arena_bytes, const tcsum_pkt_t *pkts,
                                  uint32_t n, uint32_t *out, uint8_t *flags)
{
    for (uint32_t i = 0; i < n; i++)
        if (pkts[i].offset + pkts[i].len > arena_bytes)
            return TCSUM_ERR_PARAM;
    orc_batch_ipv4_tx_fill((uint8_t *)host_arena, (const orc_pkt_t *)pkts, n, flags, 1);
    if (out)
        orc_batch_ipv4((const uint8_t *)host_arena, (const orc_pkt_t *)pkts, n, out, (uint8_t *)0, 1);
    return TCSUM_OK;
}

uint16_t checksum16(int offset, void *buf, uint16_t len, uint32_t pre_sum, int complement)
{
    return orc_checksum16(offset, buf, len, pre_sum, complement);
}

uint16_t pktbuf_checksum16(pktbuf_t *buf, int len, int pre_sum, int complement)
{
    if (buf->total_size - buf->pos < len)
        return 0; /* pktbuf.c:650-655 */
    if (len <= 0) { /* no block is walked: the u16 pre_sum, complemented or not (pktbuf.c:657-669) */
        const uint16_t s = (uint16_t)pre_sum;
        return complement ? (uint16_t)~s : s;
    }
    uint8_t *tmp = (uint8_t *)malloc(len ? (size_t)len : 1u);
    if (!tmp || (len && pktbuf_read(buf, tmp, len) != NET_ERR_OK)) {
        free(tmp);
        return 0;
    }
    uint16_t v = orc_flat_checksum16(tmp, (uint64_t)len, pre_sum, complement);
    free(tmp);
    return v;
}

uint16_t checksum_peso(pktbuf_t *buf, const ipaddr_t *dest, const ipaddr_t *src, uint8_t protocol)
{
    const int len = buf->total_size;
    uint8_t *tmp = (uint8_t *)malloc(len ? (size_t)len : 1u);
    if (!tmp)
        return 0;
    pktbuf_reset_access(buf);
    if (len && pktbuf_read(buf, tmp, len) != NET_ERR_OK) {
        free(tmp);
        return 0;
    }
    uint16_t v = orc_checksum_peso(tmp, (uint32_t)len, dest->addr, src->addr, protocol);
    free(tmp);
    return v;
}
