/*
 * golden_gen.c -- writes tests/golden/* from the REFERENCE's own checksum code.
 *
 * TEST INFRASTRUCTURE ONLY.  Built by oracle/Makefile (target `golden`) in the
 * build container, linked against the unmodified reference sources compiled
 * where they lie under /root/reference (net/src/{tools,pktbuf,mblock,list,
 * locker,debug,ipaddr}.c + plat/sys_plat.c).  The binary goes to oracle/_ref/;
 * only the data files it writes are committed.
 *
 * Every expected value below is the return value of the reference's
 *   checksum16        (net/src/tools.c:24)
 *   pktbuf_checksum16 (net/src/pktbuf.c:646)
 *   checksum_peso     (net/src/tools.c:56)
 * on the recorded inputs.  pktbuf_free is never called: on Linux it
 * self-deadlocks (pktbuf.c:203 -> :44 on a non-recursive mutex), so
 * the pool is re-initialised with pktbuf_init() before each case instead.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ipaddr.h"
#include "list.h"
#include "pktbuf.h"
#include "tools.h"

static uint64_t rng_state = 20240807ull;
static uint64_t sm64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static uint64_t rnd(void) { return sm64(rng_state++); }
static uint32_t rnd_below(uint32_t n) { return n ? (uint32_t)(rnd() % n) : 0; }

#define POOL_RANDOM 0u
#define POOL_ZERO 131072u
#define POOL_FF 196608u
#define POOL_PATTERN 262144u
#define POOL_SIZE 327680u
static uint8_t pool[POOL_SIZE];

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

/* ------------------------------------------------------------------ pools */

static void make_pool(void)
{
    for (uint32_t i = 0; i < POOL_ZERO; i++)
        pool[i] = (uint8_t)(sm64(0xC0FFEEull + (i >> 3)) >> (8 * (i & 7)));
    memset(pool + POOL_ZERO, 0, 65536);
    memset(pool + POOL_FF, 0xFF, 65536);
    for (uint32_t i = 0; i < 65536; i++)
        pool[POOL_PATTERN + i] = (uint8_t)(i * 7 + 3);
    FILE *f = open_out("pool.bin");
    fwrite(pool, 1, POOL_SIZE, f);
    fclose(f);
}

/* ---------------------------------------------------- hand-built chains */
/* For ranges larger than the reference pool (12,700 B) a pktbuf is built by
 * hand: blocks of PKTBUF_BLK_SIZE whose `data` points straight into caller
 * memory, linked with the reference's own list code -- the same layout
 * pktbuf_alloc(size, tail) would produce, minus the copy. */
#define MAX_HAND_BLKS 2048
static pktblk_t hand_blks[MAX_HAND_BLKS];
static pktbuf_t hand_buf;

static pktbuf_t *hand_chain(const uint8_t *data, int len)
{
    memset(&hand_buf, 0, sizeof hand_buf);
    list_init(&hand_buf.blk_list);
    hand_buf.ref = 1;
    int i = 0;
    while (len > 0) {
        int take = len > PKTBUF_BLK_SIZE ? PKTBUF_BLK_SIZE : len;
        pktblk_t *b = &hand_blks[i++];
        memset(b, 0, sizeof *b);
        b->size = take;
        b->data = (uint8_t *)data;
        list_insert_last(&hand_buf.blk_list, &b->node);
        hand_buf.total_size += take;
        data += take;
        len -= take;
    }
    pktbuf_reset_access(&hand_buf);
    return &hand_buf;
}

static uint16_t ref_peso_flat(const uint8_t *data, int len, const uint8_t dst[4],
                              const uint8_t src[4], uint8_t proto)
{
    ipaddr_t d, s;
    memset(&d, 0, sizeof d);
    memset(&s, 0, sizeof s);
    memcpy(d.addr, dst, 4);
    memcpy(s.addr, src, 4);
    pktbuf_t *b = hand_chain(data, len);
    return checksum_peso(b, &d, &s, proto);
}

static uint16_t ref_pktbuf_flat(const uint8_t *data, int len, int pre, int comp)
{
    pktbuf_t *b = hand_chain(data, len);
    return pktbuf_checksum16(b, len, pre, comp);
}

/* ----------------------------------------------------------------- KATs */

static void kats(void)
{
    FILE *f = open_out("kat.json");
    uint8_t h[20] = {0x45, 0x00, 0x00, 0x73, 0x00, 0x00, 0x40, 0x00, 0x40, 0x11,
                     0x00, 0x00, 0xc0, 0xa8, 0x00, 0x01, 0xc0, 0xa8, 0x00, 0xc7};
    uint16_t k1 = checksum16(0, h, 20, 0, 1);
    memcpy(h + 10, &k1, 2);
    uint16_t k1v = checksum16(0, h, 20, 0, 1);
    uint8_t b[999];
    for (int i = 0; i < 999; i++)
        b[i] = (uint8_t)(i * 7 + 3);
    uint16_t k2 = ref_pktbuf_flat(b, 999, 0, 1);
    uint16_t k2f = checksum16(0, b, 999, 0, 1);
    uint8_t src[4] = {192, 168, 74, 2}, dst[4] = {192, 168, 74, 3};
    uint16_t k3 = ref_peso_flat(b, 999, dst, src, 6);
    uint8_t z[4] = {0, 0, 0, 0}, ff[2] = {0xff, 0xff};
    uint16_t k4 = checksum16(0, z, 4, 0, 1);
    uint16_t k5 = checksum16(0, ff, 2, 0, 1);
    fprintf(f,
            "{\n"
            " \"KAT-1\": {\"hex\": \"450000730000400040110000c0a80001c0a800c7\", \"call\": "
            "\"checksum16(0,h,20,0,1)\", \"expected\": %u, \"reverify\": %u},\n"
            " \"KAT-2\": {\"pattern\": \"b[i]=(i*7+3)&255, i<999\", \"call\": "
            "\"pktbuf_checksum16(buf,999,0,1)\", \"expected\": %u, \"flat\": %u},\n"
            " \"KAT-3\": {\"pattern\": \"KAT-2 bytes\", \"src\": \"192.168.74.2\", \"dst\": "
            "\"192.168.74.3\", \"proto\": 6, \"call\": \"checksum_peso\", \"expected\": %u},\n"
            " \"KAT-4\": {\"hex\": \"00000000\", \"call\": \"checksum16(0,b,4,0,1)\", "
            "\"expected\": %u},\n"
            " \"KAT-5\": {\"hex\": \"ffff\", \"call\": \"checksum16(0,b,2,0,1)\", \"expected\": %u}\n"
            "}\n",
            k1, k1v, k2, k2f, k3, k4, k5);
    fclose(f);
    /* SURVEY.md §8(c) values, measured on the same reference code. */
    if (k1 != 0x61B8 || k1v != 0 || k2 != 0x8EE9 || k2f != 0x8EE9 || k3 != 0x4AD0 ||
        k4 != 0xFFFF || k5 != 0x0000) {
        fprintf(stderr, "KAT mismatch: %04x %04x %04x %04x %04x %04x %04x\n", k1, k1v,
                k2, k2f, k3, k4, k5);
        exit(3);
    }
}

/* ---------------------------------------------------- flat checksum16 */

static void flat_cases(int n)
{
    FILE *f = open_out("flat_cases.bin");
    static const uint32_t fixed_len[] = {0, 1, 2, 3, 4, 5, 19, 20, 21, 127, 128, 1500, 65534, 65535};
    for (int i = 0; i < n; i++) {
        uint32_t len, region, off;
        uint32_t r = rnd_below(100);
        if (i < (int)(sizeof fixed_len / sizeof fixed_len[0]) * 2)
            len = fixed_len[i % (sizeof fixed_len / sizeof fixed_len[0])];
        else if (r < 60)
            len = rnd_below(301);
        else if (r < 85)
            len = 300 + rnd_below(2701);
        else if (r < 97)
            len = 3000 + rnd_below(17001);
        else
            len = 20000 + rnd_below(45536);
        uint32_t g = rnd_below(100);
        region = g < 80 ? POOL_RANDOM : g < 87 ? POOL_ZERO : g < 94 ? POOL_FF : POOL_PATTERN;
        uint32_t span = region == POOL_RANDOM ? 131072u : 65536u;
        off = region + rnd_below(span - len + 1);
        int offset = (int)rnd_below(400) - 5;
        uint32_t p = rnd_below(100), pre;
        if (p < 50)
            pre = rnd_below(0x10000);
        else if (p < 80)
            pre = (uint32_t)rnd();
        else {
            static const uint32_t sp[] = {0, 0xFFFF, 0x10000, 0xFFFFFFFFu, 0x80000000u, 0xFFFF0000u};
            pre = sp[rnd_below(6)];
        }
        uint32_t comp = (uint32_t)(rnd() & 1);
        if (len == 0 && (offset & 1))
            offset++; /* odd offset with len 0 reads 64 KiB past the buffer (tools.c:33) */
        uint16_t e = checksum16(offset, pool + off, (uint16_t)len, pre, (int)comp);
        put_u32(f, off);
        put_u32(f, len);
        put_u32(f, (uint32_t)offset);
        put_u32(f, pre);
        put_u32(f, comp);
        put_u32(f, e);
    }
    fclose(f);
}

/* ----------------------------------------------- pktbuf-based cases */

static uint32_t blk_sizes_total;

/* Build a pktbuf the way the stack does: pktbuf_alloc (head-inserted blocks,
 * first one partial), optional pktbuf_add_header, then pktbuf_write. */
static pktbuf_t *stack_buf(uint32_t total, uint32_t data_off)
{
    pktbuf_init();
    uint32_t h = 0;
    int cont = 0;
    if (total > 1 && rnd_below(100) < 60) {
        cont = (int)(rnd() & 1);
        h = 1 + rnd_below(cont ? 127 : (total < 300 ? total - 1 : 300));
        if (h >= total)
            h = total - 1;
    }
    pktbuf_t *b = pktbuf_alloc((int)(total - h));
    if (!b)
        return NULL;
    if (h && pktbuf_add_header(b, (int)h, cont) != NET_ERR_OK)
        return NULL;
    pktbuf_reset_access(b);
    if (total && pktbuf_write(b, pool + data_off, (int)total) != NET_ERR_OK)
        return NULL;
    pktbuf_reset_access(b);
    return b;
}

static uint32_t write_blocks(FILE *fb, pktbuf_t *b, pktblk_t **order, uint32_t *nblk)
{
    uint32_t first = blk_sizes_total, k = 0;
    for (pktblk_t *p = pktbuf_first_blk(b); p; p = pktblk_blk_next(p)) {
        put_u32(fb, (uint32_t)p->size);
        order[k++] = p;
        blk_sizes_total++;
    }
    *nblk = k;
    return first;
}

static void cursor_of(pktbuf_t *b, pktblk_t **order, uint32_t nblk, uint32_t *idx,
                      uint32_t *boff)
{
    *idx = 0xFFFFFFFFu;
    *boff = 0;
    for (uint32_t k = 0; k < nblk; k++)
        if (order[k] == b->curr_blk) {
            *idx = k;
            *boff = (uint32_t)(b->blk_offset - order[k]->data);
        }
}

static void pktbuf_cases(int n)
{
    FILE *f = open_out("pktbuf_cases.bin");
    FILE *fb = open_out("pktbuf_blocks.bin");
    pktblk_t *order[PKTBUF_BLK_CNT + 1];
    blk_sizes_total = 0;
    int made = 0;
    while (made < n) {
        uint32_t total = 1 + rnd_below(rnd_below(4) == 0 ? 12000 : 3000);
        uint32_t data_off = rnd_below(131072 - total);
        pktbuf_t *b = stack_buf(total, data_off);
        if (!b)
            continue;
        uint32_t seek = rnd_below(100) < 70 ? 0 : rnd_below(total);
        if (seek && pktbuf_seek(b, (int)seek) != NET_ERR_OK)
            continue;
        int remain = (int)(total - seek);
        uint32_t lr = rnd_below(100);
        int len = lr < 60 ? remain
                  : lr < 85 ? (int)rnd_below((uint32_t)remain + 1)
                  : lr < 95 ? remain + 1 + (int)rnd_below(50)
                            : -(int)rnd_below(5);
        uint32_t pr = rnd_below(100);
        int pre = pr < 60 ? (int)rnd_below(0x10000) : pr < 80 ? (int)rnd() : 0;
        int comp = (int)(rnd() & 1);
        uint32_t nblk, idx, boff;
        uint32_t first = write_blocks(fb, b, order, &nblk);
        uint16_t e = pktbuf_checksum16(b, len, pre, comp);
        cursor_of(b, order, nblk, &idx, &boff);
        put_u32(f, data_off);
        put_u32(f, total);
        put_u32(f, first);
        put_u32(f, nblk);
        put_u32(f, seek);
        put_u32(f, (uint32_t)len);
        put_u32(f, (uint32_t)pre);
        put_u32(f, (uint32_t)comp);
        put_u32(f, e);
        put_u32(f, (uint32_t)b->pos);
        put_u32(f, idx);
        put_u32(f, boff);
        made++;
    }
    fclose(f);
    fclose(fb);
}

static void peso_cases(int n, int nbig)
{
    FILE *f = open_out("peso_cases.bin");
    FILE *fb = open_out("peso_blocks.bin");
    pktblk_t *order[MAX_HAND_BLKS];
    blk_sizes_total = 0;
    int made = 0;
    static const uint32_t big_len[] = {65536, 65535, 65534, 65537, 100000, 131071, 131072, 1500, 9000};
    while (made < n + nbig) {
        int big = made >= n;
        uint32_t total;
        if (big)
            total = made - n < 9 ? big_len[made - n] : 12000 + rnd_below(131072 - 12000);
        else
            total = rnd_below(100) < 3 ? 1 + rnd_below(3) : 1 + rnd_below(rnd_below(3) ? 3000 : 12000);
        uint32_t data_off = rnd_below(131072 - total + 1);
        pktbuf_t *b = big ? hand_chain(pool + data_off, (int)total) : stack_buf(total, data_off);
        if (!b)
            continue;
        uint8_t src[4], dst[4];
        uint64_t r = rnd();
        memcpy(src, &r, 4);
        memcpy(dst, (uint8_t *)&r + 4, 4);
        uint32_t pp = rnd_below(100);
        uint8_t proto = pp < 45 ? 6 : pp < 90 ? 17 : (uint8_t)rnd();
        ipaddr_t d, s;
        memset(&d, 0, sizeof d);
        memset(&s, 0, sizeof s);
        memcpy(d.addr, dst, 4);
        memcpy(s.addr, src, 4);
        uint32_t nblk, idx, boff;
        uint32_t first = write_blocks(fb, b, order, &nblk);
        uint16_t e = checksum_peso(b, &d, &s, proto);
        cursor_of(b, order, nblk, &idx, &boff);
        put_u32(f, data_off);
        put_u32(f, total);
        put_u32(f, first);
        put_u32(f, nblk);
        fwrite(src, 1, 4, f);
        fwrite(dst, 1, 4, f);
        put_u32(f, proto);
        put_u32(f, e);
        put_u32(f, (uint32_t)b->pos);
        put_u32(f, idx);
        made++;
    }
    fclose(f);
    fclose(fb);
}

/* ------------------------------------------------------------ IPv4 packets */
/* The per-packet definitions of tcsum_batch_ipv4 / _tx_fill (include/tcsum.h)
 * on random, often malformed packets, with every checksum value taken from the
 * reference's own checksum16 / checksum_peso / pktbuf_checksum16.  Which
 * fields the fill writes on a malformed packet is this API's definition (the
 * reference never transmits one): the decisions on packets the reference
 * does transmit, and every rx verdict, come from the reference stack itself
 * (oracle/stack_gen.c: stack_tx_*.bin, ipv4_rx_*.bin). */

#define IPV4_POOL_CAP (12u << 20)
static uint8_t ipool[IPV4_POOL_CAP];

#define F_BAD_VERSION 0x01u
#define F_BAD_HDRLEN 0x02u
#define F_BAD_TOTLEN 0x04u
#define F_PROTO_OTHER 0x08u
#define F_SHORT 0x10u
#define F_FRAGMENT 0x20u
#define F_L4_SHORT 0x40u

static int l4_field(uint8_t proto, uint32_t *field, uint32_t *min_len)
{
    switch (proto) {
    case 6: *field = 16; *min_len = 20; return 1; /* tcp.h:71  (sizeof tcp_hdr_t = 20) */
    case 17: *field = 6; *min_len = 8; return 1;  /* udp.h:24  (sizeof udp_hdr_t = 8) */
    case 1: *field = 2; *min_len = 4; return 1;   /* icmpv4.h:28 (sizeof icmpv4_hdr_t = 4) */
    default: return 0;
    }
}

static void ref_pair(const uint8_t *p, uint32_t frame, uint32_t *ip, uint32_t *l4, uint32_t *flags)
{
    *ip = *l4 = *flags = 0;
    if (frame < 20) {
        *flags = F_SHORT;
        return;
    }
    uint32_t ver = p[0] >> 4, ihl4 = (uint32_t)(p[0] & 15) * 4;
    uint32_t tl = ((uint32_t)p[2] << 8) | p[3];
    if (ver != 4)
        *flags |= F_BAD_VERSION;
    if (ihl4 < 20 || ihl4 > frame)
        *flags |= F_BAD_HDRLEN;
    if (tl < 20 || tl > frame || tl < ihl4)
        *flags |= F_BAD_TOTLEN;
    if ((p[6] & 0x20) || (((p[6] & 0x1F) << 8) | p[7]))
        *flags |= F_FRAGMENT;
    uint32_t hl = ihl4 < 20 ? 20 : ihl4;
    if (hl > frame)
        hl = frame;
    uint32_t end = tl < hl ? hl : tl;
    if (end > frame)
        end = frame;
    *ip = checksum16(0, (void *)p, (uint16_t)hl, 0, 1);
    uint8_t proto = p[9];
    uint32_t fld, minl;
    if (l4_field(proto, &fld, &minl) && end - hl < minl)
        *flags |= F_L4_SHORT;
    if (proto == 6 || proto == 17)
        *l4 = ref_peso_flat(p + hl, (int)(end - hl), p + 16, p + 12, proto);
    else if (proto == 1)
        *l4 = ref_pktbuf_flat(p + hl, (int)(end - hl), 0, 1);
    else
        *flags |= F_PROTO_OTHER;
}

static uint32_t ref_tx_fill(uint8_t *p, uint32_t frame)
{
    uint32_t ip, l4, flags;
    ref_pair(p, frame, &ip, &l4, &flags);
    if (flags & (F_SHORT | F_BAD_VERSION | F_BAD_HDRLEN | F_BAD_TOTLEN))
        return flags;
    uint32_t hl = (uint32_t)(p[0] & 15) * 4, tl = ((uint32_t)p[2] << 8) | p[3];
    uint8_t proto = p[9];
    uint32_t fld, minl;
    if (!(flags & (F_FRAGMENT | F_L4_SHORT)) && l4_field(proto, &fld, &minl)) {
        uint8_t *l4p = p + hl;
        l4p[fld] = l4p[fld + 1] = 0;
        uint16_t v = proto == 1 ? ref_pktbuf_flat(l4p, (int)(tl - hl), 0, 1)
                                : ref_peso_flat(l4p, (int)(tl - hl), p + 16, p + 12, proto);
        memcpy(l4p + fld, &v, 2);
    }
    p[10] = p[11] = 0;
    uint16_t h = checksum16(0, p, (uint16_t)hl, 0, 1);
    memcpy(p + 10, &h, 2);
    return flags;
}

/* A random packet: mostly well formed, with the odd broken field. */
static uint32_t make_packet(uint8_t *p, uint32_t max_frame)
{
    uint32_t fr = rnd_below(100);
    uint32_t frame = fr < 2 ? rnd_below(20) : fr < 12 ? 20 + rnd_below(100)
                                                      : 64 + rnd_below(max_frame - 64 + 1);
    for (uint32_t k = 0; k < frame; k++)
        p[k] = (uint8_t)rnd();
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
    uint32_t fg = rnd_below(100); /* fragments: MF and/or offset */
    p[6] = fg < 85 ? 0x40 : (uint8_t)rnd(); /* DF, or random flag/offset bits */
    p[7] = fg < 85 ? 0 : (uint8_t)rnd();
    uint32_t pr = rnd_below(100);
    p[9] = pr < 42 ? 6 : pr < 84 ? 17 : pr < 92 ? 1 : (uint8_t)rnd();
    p[10] = p[11] = 0;
    return frame;
}

static void ipv4_cases(int n)
{
    FILE *f = open_out("ipv4_cases.bin");
    uint32_t at = 0;
    for (int i = 0; i < n; i++) {
        uint8_t *p = ipool + at;
        if (at + 9000 + 64 > IPV4_POOL_CAP)
            break;
        uint32_t frame = make_packet(p, 9000);
        if (frame >= 20 && rnd_below(2)) { /* rx-style: header checksum already filled */
            uint32_t hl = (uint32_t)(p[0] & 15) * 4;
            hl = hl < 20 ? 20 : hl;
            uint16_t c = checksum16(0, p, (uint16_t)hl, 0, 1);
            memcpy(p + 10, &c, 2);
        }
        uint32_t ip, l4, flags;
        ref_pair(p, frame, &ip, &l4, &flags);
        put_u32(f, at);
        put_u32(f, frame);
        put_u32(f, ip);
        put_u32(f, l4);
        put_u32(f, flags);
        at += frame + (rnd_below(4) == 0 ? rnd_below(16) : 0); /* mostly packed, some gaps */
    }
    fclose(f);
    FILE *fp = open_out("ipv4_pool.bin");
    fwrite(ipool, 1, at + 64, fp);
    fclose(fp);
}

/* tx: packets as the stack hands them over (fields arbitrary -- the fill zeroes
 * them); expected = the whole pool after the reference's fill. */
static void ipv4_tx_cases(int n)
{
    uint32_t *offs = (uint32_t *)malloc(sizeof(uint32_t) * 2 * (size_t)n);
    uint32_t at = 0;
    for (int i = 0; i < n; i++) {
        uint8_t *p = ipool + at;
        uint32_t frame = make_packet(p, 3000);
        if (frame >= 20 && rnd_below(3) == 0) { /* stale values in the fields */
            p[10] = (uint8_t)rnd();
            p[11] = (uint8_t)rnd();
        }
        offs[2 * i] = at;
        offs[2 * i + 1] = frame;
        at += frame + (rnd_below(4) == 0 ? rnd_below(16) : 0);
    }
    const uint32_t total = at + 64;
    FILE *fin = open_out("ipv4_tx_in.bin");
    fwrite(ipool, 1, total, fin);
    fclose(fin);
    FILE *f = open_out("ipv4_tx_cases.bin");
    for (int i = 0; i < n; i++) {
        uint32_t flags = ref_tx_fill(ipool + offs[2 * i], offs[2 * i + 1]);
        put_u32(f, offs[2 * i]);
        put_u32(f, offs[2 * i + 1]);
        put_u32(f, flags);
    }
    fclose(f);
    FILE *fo = open_out("ipv4_tx_out.bin");
    fwrite(ipool, 1, total, fo);
    fclose(fo);
    free(offs);
}

int main(int argc, char **argv)
{
    outdir = argc > 1 ? argv[1] : "tests/golden";
    tools_init();
    pktbuf_init();
    make_pool();
    kats();
    flat_cases(6000);
    pktbuf_cases(1500);
    peso_cases(1200, 48);
    ipv4_cases(500);
    ipv4_tx_cases(400);
    printf("golden vectors written to %s\n", outdir);
    return 0;
}
