/*
 * tcsum_legacy.h -- the drop-in half of the C ABI: the reference's three
 * checksum entry points with their exact names and signatures.
 *
 *   checksum16         replaces net/src/tools.c:24-54   (decl net/net/tools.h:45)
 *   checksum_peso      replaces net/src/tools.c:56-75   (decl net/net/tools.h:47)
 *   pktbuf_checksum16  replaces net/src/pktbuf.c:646-670 (decl net/net/pktbuf.h:229)
 *
 * Inside the stack these are reached through the stack's own tools.h /
 * pktbuf.h declarations; the stack does not include this header (see
 * INTEGRATION.md).  This header restates the reference's types under tcsum_
 * names with an identical memory layout (net/net/list.h:9-34,
 * net/net/pktbuf.h:15-41, net/net/ipaddr.h:12-22 on LP64) for callers outside
 * the stack and for the library's own build; the pointer parameters are
 * ABI-identical to the reference's.
 *
 * Semantics kept bit-for-bit, including side effects:
 *   - pktbuf_checksum16 starts at the buffer's cursor, returns 0 when len
 *     exceeds the bytes left (pktbuf.c:650-655), and advances the cursor by
 *     len (pos / curr_blk / blk_offset, pktbuf.c:665);
 *   - checksum_peso resets the cursor, sums the pseudo-header in memory order
 *     with htons((uint16_t)total_size), and leaves the cursor at the end.
 *   - checksum16 keeps the u32 accumulator wrap for pre_sum near 2^32.
 * Deviations (undefined behaviour in the reference, defined here):
 *   - checksum16 with len == 0 and odd offset sums nothing (the reference
 *     decrements the u16 len to 65535 and reads past the buffer, tools.c:33);
 *   - a zero-size block reached at an odd offset is skipped for the same
 *     reason; a buf with ref == 0 aborts (the reference spins in assert,
 *     net/net/debug.h:33-39).
 * All arithmetic runs on the GPU; a process without a usable gfx950 device
 * gets a message on stderr and abort() from the first call -- there is no CPU
 * fallback.
 */
#ifndef TCSUM_LEGACY_H
#define TCSUM_LEGACY_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TCSUM_PKTBUF_BLK_SIZE 127 /* net/net/net_cfg.h:31 (layout only) */

typedef struct tcsum_node {           /* node_t, list.h:9-12 */
    struct tcsum_node *pre;
    struct tcsum_node *next;
} tcsum_node_t;

typedef struct tcsum_list {           /* list_t, list.h:30-34 */
    tcsum_node_t *first;
    tcsum_node_t *last;
    int count;
} tcsum_list_t;

typedef struct tcsum_pktblk {         /* pktblk_t, pktbuf.h:15-23 */
    tcsum_node_t node;
    int size;
    uint8_t *data;
    uint8_t payload[TCSUM_PKTBUF_BLK_SIZE];
} tcsum_pktblk_t;

typedef struct tcsum_pktbuf {         /* pktbuf_t, pktbuf.h:26-41 */
    int total_size;
    tcsum_list_t blk_list;
    int ref;
    tcsum_node_t node;
    int pos;
    tcsum_pktblk_t *curr_blk;
    uint8_t *blk_offset;
} tcsum_pktbuf_t;

typedef struct tcsum_ipaddr {         /* ipaddr_t, ipaddr.h:12-22 */
    int type;                         /* IPADDR_V4 == 0 */
    union {
        uint32_t q_addr;
        uint8_t addr[4];
    };
} tcsum_ipaddr_t;

uint16_t checksum16(int offset, void *buf, uint16_t len, uint32_t pre_sum, int complement);

uint16_t checksum_peso(tcsum_pktbuf_t *buf, const tcsum_ipaddr_t *dest,
                       const tcsum_ipaddr_t *src, uint8_t protocol);

uint16_t pktbuf_checksum16(tcsum_pktbuf_t *buf, int len, int pre_sum, int complement);

#ifdef __cplusplus
}
#endif
#endif /* TCSUM_LEGACY_H */
