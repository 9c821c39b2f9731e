/*
 * dropin_stack.c -- the reference stack's own pktbuf/tools objects + libtcsum.so.
 *
 * TEST INFRASTRUCTURE.  Built by `make -C oracle dropin` into
 * oracle/_ref/dropin_stack: the reference's net/src/{tools,pktbuf,...}.c are
 * compiled in place, their checksum16 / checksum_peso / pktbuf_checksum16 are
 * made local with objcopy (what INTEGRATION.md's #ifndef NET_CHECKSUM_GPU does
 * to the sources), and the program links libtcsum.so, so every checksum call
 * below resolves to the GPU library while buffers, lists, cursors and
 * pktbuf_seek are the reference's own code.
 *
 * It replays tests/golden/{pktbuf,peso}_cases.bin (outputs of the reference's
 * own routines) and checks result AND cursor after every call.  Exit status 0
 * when all match.  Usage: dropin_stack <tests/golden dir>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ipaddr.h"
#include "list.h"
#include "pktbuf.h"
#include "tools.h"

#define MAXBLK 2048
static pktblk_t blks[MAXBLK];
static pktbuf_t buf;

static void *slurp(const char *dir, const char *name, size_t *len)
{
    char path[1024];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE *f = fopen(path, "rb");
    if (!f) {
        perror(path);
        exit(2);
    }
    fseek(f, 0, SEEK_END);
    *len = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    void *p = malloc(*len ? *len : 1);
    if (fread(p, 1, *len, f) != *len)
        exit(2);
    fclose(f);
    return p;
}

/* A chain with the recorded block sizes over the pool bytes, linked with the
 * reference's list code; cursor set by the reference's pktbuf_reset_access. */
static pktbuf_t *chain(const uint8_t *data, const uint32_t *sizes, uint32_t nblk)
{
    memset(&buf, 0, sizeof buf);
    list_init(&buf.blk_list);
    buf.ref = 1;
    for (uint32_t i = 0; i < nblk; i++) {
        pktblk_t *b = &blks[i];
        memset(b, 0, sizeof *b);
        b->size = (int)sizes[i];
        b->data = (uint8_t *)data;
        data += sizes[i];
        list_insert_last(&buf.blk_list, &b->node);
        buf.total_size += b->size;
    }
    pktbuf_reset_access(&buf);
    return &buf;
}

static uint32_t cursor_blk(pktbuf_t *b, uint32_t nblk)
{
    for (uint32_t i = 0; i < nblk; i++)
        if (b->curr_blk == &blks[i])
            return i;
    return 0xFFFFFFFFu;
}

int main(int argc, char **argv)
{
    const char *dir = argc > 1 ? argv[1] : "tests/golden";
    size_t n_pool, n_pk, n_pkb, n_pe, n_peb;
    const uint8_t *pool = slurp(dir, "pool.bin", &n_pool);
    const uint32_t *pk = slurp(dir, "pktbuf_cases.bin", &n_pk);
    const uint32_t *pkb = slurp(dir, "pktbuf_blocks.bin", &n_pkb);
    const uint32_t *pe = slurp(dir, "peso_cases.bin", &n_pe);
    const uint32_t *peb = slurp(dir, "peso_blocks.bin", &n_peb);
    int bad = 0, done = 0;

    /* pktbuf_cases.bin: 12 u32 per case (tests/golden_io.py PKTBUF) */
    for (size_t k = 0; k < n_pk / 48; k++) {
        const uint32_t *c = pk + 12 * k;
        pktbuf_t *b = chain(pool + c[0], pkb + c[2], c[3]);
        if (c[4])
            pktbuf_seek(b, (int)c[4]);
        uint16_t got = pktbuf_checksum16(b, (int)c[5], (int)c[6], (int)c[7]);
        uint32_t blk = cursor_blk(b, c[3]);
        uint32_t boff = blk == 0xFFFFFFFFu ? 0 : (uint32_t)(b->blk_offset - blks[blk].data);
        if (got != c[8] || (uint32_t)b->pos != c[9] || blk != c[10] ||
            (blk != 0xFFFFFFFFu && boff != c[11])) {
            if (bad < 5)
                fprintf(stderr, "pktbuf case %zu: got %04x pos %d blk %u, want %04x pos %u blk %u\n", k, got,
                        b->pos, blk, c[8], c[9], c[10]);
            bad++;
        }
        done++;
    }
    /* peso_cases.bin: 10 u32 per case (tests/golden_io.py PESO) */
    for (size_t k = 0; k < n_pe / 40; k++) {
        const uint32_t *c = pe + 10 * k;
        pktbuf_t *b = chain(pool + c[0], peb + c[2], c[3]);
        ipaddr_t src, dst;
        memset(&src, 0, sizeof src);
        memset(&dst, 0, sizeof dst);
        memcpy(src.addr, &c[4], 4);
        memcpy(dst.addr, &c[5], 4);
        uint16_t got = checksum_peso(b, &dst, &src, (uint8_t)c[6]);
        if (got != c[7] || (uint32_t)b->pos != c[8] || cursor_blk(b, c[3]) != 0xFFFFFFFFu) {
            if (bad < 5)
                fprintf(stderr, "peso case %zu: got %04x want %04x\n", k, got, c[7]);
            bad++;
        }
        done++;
    }
    /* checksum16 on an IPv4 header, the way is_pkt_ok calls it (ipv4.c:243) */
    uint8_t h[20] = {0x45, 0x00, 0x00, 0x73, 0x00, 0x00, 0x40, 0x00, 0x40, 0x11,
                     0x00, 0x00, 0xc0, 0xa8, 0x00, 0x01, 0xc0, 0xa8, 0x00, 0xc7};
    if (checksum16(0, h, 20, 0, 1) != 0x61B8)
        bad++;
    done++;
    printf("dropin_stack: %d/%d calls match the reference (reference pktbuf + libtcsum.so)\n", done - bad,
           done);
    return bad ? 1 : 0;
}
