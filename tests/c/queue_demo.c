/*
 * queue_demo.c -- INTEGRATION.md §4a as a plain C program: the stack's netif
 * queues handed to libtcsum.so as host-queue batches.
 *
 * TEST INFRASTRUCTURE.  Built by tests/c/Makefile into tests/c/build/; run by
 * tests/test_gpu_hostq.py::test_c_netif_queue_demo.  For queues of 50 frames
 * (NETIF_OUTQ_SIZE / NETIF_INQ_SIZE, net_cfg.h:39-40), with and without the
 * queue server:
 *   tx: Ethernet frames (14-B link header + IPv4 + TCP/UDP/ICMP) are built
 *       with their checksum fields holding garbage in a tcsum_host_alloc
 *       arena; tcsum_host_batch_ipv4_tx_fill fills them in place; the bytes
 *       must equal the CPU oracle's tx fill of the same frames;
 *   rx: the filled frames verify OK (tcsum_host_batch_ipv4_rx_verify); one
 *       flipped payload bit per damaged frame turns exactly those frames into
 *       NET_ERR_BROKEN (-13), the oracle agreeing frame by frame.
 * Exit 0 when everything matches.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "csum_oracle.h"
#include "tcsum.h"

#define QUEUE 50    /* NETIF_OUTQ_SIZE, NETIF_INQ_SIZE (net_cfg.h:39-40) */
#define L2 14       /* sizeof(ether_hdr_t), ether.h:25 */
#define ROUNDS 200  /* queues per mode */

static uint64_t rng = 7;
static uint64_t next(void) { return rng = orc_splitmix64(rng); }

/* One frame at f: link header, IPv4 header (IHL 5), L4 header + payload. */
static uint32_t build_frame(uint8_t *f)
{
    const uint64_t r = next();
    const int proto = (int[]){6, 17, 1}[r % 3];
    const uint32_t l4 = (proto == 6 ? 20 : proto == 17 ? 8 : 8) + (uint32_t)((r >> 8) % 1461);
    const uint32_t total = 20 + l4;
    for (uint32_t i = 0; i < L2 + total; i += 8) {
        const uint64_t w = next();
        memcpy(f + i, &w, L2 + total - i < 8 ? L2 + total - i : 8);
    }
    uint8_t *ip = f + L2;
    ip[0] = 0x45;
    ip[2] = (uint8_t)(total >> 8);
    ip[3] = (uint8_t)total;
    ip[6] = ip[7] = 0; /* not a fragment */
    ip[9] = (uint8_t)proto;
    if (proto == 17) { /* the UDP length field */
        ip[20 + 4] = (uint8_t)(l4 >> 8);
        ip[20 + 5] = (uint8_t)l4;
    }
    if (proto != 1) { /* nonzero ports (tcp_in.c:93, udp.c:337) */
        ip[20 + 0] |= 0x80;
        ip[20 + 2] |= 0x80;
    }
    if (proto == 6) { /* data offset 5, ACK (tcp_in.c:87-103) */
        ip[20 + 12] = 0x50;
        ip[20 + 13] = 0x10;
    }
    return L2 + total; /* checksum fields keep their random bytes: the fill zeroes them first */
}

static int run(const char *mode)
{
    const size_t cap = QUEUE * (L2 + 20 + 20 + 1460 + 16);
    uint8_t *tx = tcsum_host_alloc(cap);  /* the pinned tx arena of INTEGRATION.md §4a */
    uint8_t *ref = malloc(cap);
    if (!tx || !ref)
        return 2;
    for (int round = 0; round < ROUNDS; round++) {
        tcsum_pkt_t pk[QUEUE];
        orc_pkt_t opk[QUEUE];
        uint64_t at = (uint64_t)(round % 7); /* odd arena offsets too */
        for (int i = 0; i < QUEUE; i++) {
            const uint32_t len = build_frame(tx + at);
            pk[i].offset = at + L2;
            pk[i].len = len - L2;
            pk[i].rsv = 0;
            opk[i].offset = pk[i].offset;
            opk[i].len = pk[i].len;
            opk[i].rsv = 0;
            at += len;
        }
        memcpy(ref, tx, at);
        /* tx: fill in place, compare with the oracle's fill */
        if (tcsum_host_batch_ipv4_tx_fill(0, tx, at, pk, QUEUE, NULL, NULL) != TCSUM_OK)
            return fprintf(stderr, "%s: tx fill failed\n", mode), 1;
        uint8_t oflags[QUEUE];
        orc_batch_ipv4_tx_fill(ref, opk, QUEUE, oflags, 1);
        if (memcmp(tx, ref, at) != 0)
            return fprintf(stderr, "%s round %d: tx bytes differ from the oracle\n", mode, round), 1;
        /* rx: damage some frames, verify the queue */
        int damaged[QUEUE] = {0};
        for (int i = 0; i < QUEUE; i++)
            if (next() % 4 == 0 && pk[i].len > 40) {
                tx[pk[i].offset + 20 + 20 + (next() % (pk[i].len - 40))] ^= (uint8_t)(1u << (next() % 8));
                damaged[i] = 1;
            }
        memcpy(ref, tx, at);
        int8_t v[QUEUE], ov[QUEUE];
        uint8_t of[QUEUE];
        if (tcsum_host_batch_ipv4_rx_verify(0, tx, at, pk, QUEUE, v, NULL, NULL) != TCSUM_OK)
            return fprintf(stderr, "%s: rx verify failed\n", mode), 1;
        orc_batch_ipv4_rx_verify(ref, opk, QUEUE, ov, of, 1);
        for (int i = 0; i < QUEUE; i++) {
            if (v[i] != ov[i])
                return fprintf(stderr, "%s round %d frame %d: verdict %d, oracle %d\n", mode, round, i, v[i], ov[i]), 1;
            if ((v[i] == TCSUM_ERR_BROKEN) != damaged[i] && !(damaged[i] && v[i] == TCSUM_OK))
                return fprintf(stderr, "%s round %d frame %d: verdict %d, damaged %d\n", mode, round, i, v[i],
                               damaged[i]),
                       1;
        }
    }
    tcsum_host_free(tx);
    free(ref);
    printf("%s: %d queues of %d frames: tx fill == oracle, rx verdicts == oracle\n", mode, ROUNDS, QUEUE);
    return 0;
}

int main(void)
{
    if (tcsum_plat_init(0) != TCSUM_OK) { /* net_plat_init hook (plat/net_plat.c:7) */
        fprintf(stderr, "no gfx950 device\n");
        return 2;
    }
    int rc = run("launch per queue");
    if (rc)
        return rc;
    if (tcsum_queue_server(0, 1) != TCSUM_OK)
        return 2;
    rc = run("queue server");
    if (tcsum_queue_server(0, 0) != TCSUM_OK)
        return 2;
    return rc;
}
