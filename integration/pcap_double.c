/*
 * pcap_double.c -- link-time test double for libpcap (see pcap_double.h).
 * TEST CODE, built by integration/Makefile into the integration test programs
 * only.  It implements exactly the libpcap entry points the reference's pcap
 * driver calls (plat/sys_plat.c:436-618, plat/netif_pcap.c:9-92), with the
 * reference's vendored npcap/Include/pcap.h for their types.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <time.h>

#include <pcap.h>

#include "pcap_double.h"

struct pcap {
    char err[PCAP_ERRBUF_SIZE];
    int active;
    int have_mac;
    uint8_t mac[6];             /* from the filter pcap_device_open compiles */
    struct pcap_pkthdr hdr;
    uint8_t *data;              /* the frame pcap_next_ex handed out last */
};

typedef struct frame {
    struct frame *next;
    uint32_t len;
    uint8_t bytes[];
} frame_t;

static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t fed_cv = PTHREAD_COND_INITIALIZER;
static pthread_cond_t inj_cv = PTHREAD_COND_INITIALIZER;
static frame_t *rx_head, *rx_tail;
static uint32_t rx_pending;
static frame_t **inj;
static uint32_t inj_n, inj_cap;
static int inject_fail;
static uint64_t arp_replies, filtered, inject_failures;
static char dev_ip[64] = "192.168.74.2";
static uint8_t peer_mac[6] = {0x02, 0x00, 0x5e, 0x10, 0x00, 0x01};

static frame_t *frame_new(const uint8_t *p, uint32_t len)
{
    frame_t *f = (frame_t *)malloc(sizeof *f + (len ? len : 1));
    if (!f) {
        fprintf(stderr, "pcap_double: out of memory\n");
        abort();
    }
    f->next = NULL;
    f->len = len;
    memcpy(f->bytes, p, len);
    return f;
}

static void rx_push_locked(frame_t *f)
{
    if (rx_tail)
        rx_tail->next = f;
    else
        rx_head = f;
    rx_tail = f;
    rx_pending++;
    pthread_cond_broadcast(&fed_cv);
}

/* ------------------------------------------------------------ test side */

void pcapd_setup(const char *device_ip, const uint8_t mac[6])
{
    pthread_mutex_lock(&mu);
    snprintf(dev_ip, sizeof dev_ip, "%s", device_ip);
    memcpy(peer_mac, mac, 6);
    pthread_mutex_unlock(&mu);
}

void pcapd_feed(const uint8_t *p, uint32_t len)
{
    frame_t *f = frame_new(p, len);
    pthread_mutex_lock(&mu);
    rx_push_locked(f);
    pthread_mutex_unlock(&mu);
}

uint32_t pcapd_pending(void)
{
    pthread_mutex_lock(&mu);
    uint32_t n = rx_pending;
    pthread_mutex_unlock(&mu);
    return n;
}

uint32_t pcapd_injected_count(void)
{
    pthread_mutex_lock(&mu);
    uint32_t n = inj_n;
    pthread_mutex_unlock(&mu);
    return n;
}

const uint8_t *pcapd_injected(uint32_t i, uint32_t *len)
{
    pthread_mutex_lock(&mu);
    const frame_t *f = i < inj_n ? inj[i] : NULL;
    pthread_mutex_unlock(&mu);
    if (!f)
        return NULL;
    *len = f->len;
    return f->bytes;
}

void pcapd_reset_injected(void)
{
    pthread_mutex_lock(&mu);
    for (uint32_t i = 0; i < inj_n; i++)
        free(inj[i]);
    inj_n = 0;
    pthread_mutex_unlock(&mu);
}

int pcapd_wait_injected(uint32_t count, int ms)
{
    struct timespec until;
    clock_gettime(CLOCK_REALTIME, &until);
    until.tv_sec += ms / 1000;
    until.tv_nsec += (long)(ms % 1000) * 1000000L;
    if (until.tv_nsec >= 1000000000L) {
        until.tv_sec++;
        until.tv_nsec -= 1000000000L;
    }
    pthread_mutex_lock(&mu);
    int rc = 0;
    while (inj_n < count && rc == 0)
        rc = pthread_cond_timedwait(&inj_cv, &mu, &until);
    const int ok = inj_n >= count;
    pthread_mutex_unlock(&mu);
    return ok ? 0 : -1;
}

void pcapd_fail_inject(int n)
{
    pthread_mutex_lock(&mu);
    inject_fail = n;
    pthread_mutex_unlock(&mu);
}

uint64_t pcapd_arp_replies(void) { return __atomic_load_n(&arp_replies, __ATOMIC_RELAXED); }
uint64_t pcapd_filtered(void) { return __atomic_load_n(&filtered, __ATOMIC_RELAXED); }
uint64_t pcapd_inject_failures(void) { return __atomic_load_n(&inject_failures, __ATOMIC_RELAXED); }

/* ------------------------------------------------------------ the peer */

/* An ARP request among the injected frames gets its reply on the wire: the
 * peer claims every address (the reference's own reply layout, arp.c:354-367). */
static void answer_arp_locked(const uint8_t *f, uint32_t len)
{
    if (len < 42 || f[12] != 0x08 || f[13] != 0x06 || f[20] != 0 || f[21] != 1)
        return;
    if (memcmp(f + 28, f + 38, 4) == 0)
        return; /* a gratuitous request (arp_make_gratuitous): nobody answers */
    uint8_t r[60];
    memset(r, 0, sizeof r);
    memcpy(r, f + 6, 6);          /* to the requester */
    memcpy(r + 6, peer_mac, 6);
    r[12] = 0x08, r[13] = 0x06;
    memcpy(r + 14, f + 14, 6);    /* htype, ptype, hwlen, plen */
    r[20] = 0, r[21] = 2;         /* reply */
    memcpy(r + 22, peer_mac, 6);  /* sender: the peer, at the address asked for */
    memcpy(r + 28, f + 38, 4);
    memcpy(r + 32, f + 22, 6);    /* target: the requester */
    memcpy(r + 38, f + 28, 4);
    rx_push_locked(frame_new(r, sizeof r));
    __atomic_fetch_add(&arp_replies, 1, __ATOMIC_RELAXED);
}

/* ------------------------------------------------------------ libpcap */

int pcap_findalldevs(pcap_if_t **list, char *errbuf)
{
    pcap_if_t *d = (pcap_if_t *)calloc(1, sizeof *d);
    struct pcap_addr *a = (struct pcap_addr *)calloc(1, sizeof *a);
    struct sockaddr_in *sin = (struct sockaddr_in *)calloc(1, sizeof *sin);
    if (!d || !a || !sin) {
        snprintf(errbuf, PCAP_ERRBUF_SIZE, "out of memory");
        free(d), free(a), free(sin);
        return -1;
    }
    sin->sin_family = AF_INET;
    pthread_mutex_lock(&mu);
    inet_pton(AF_INET, dev_ip, &sin->sin_addr);
    pthread_mutex_unlock(&mu);
    a->addr = (struct sockaddr *)sin;
    d->name = strdup("tcsum-wire0");
    d->description = strdup("pcap test double (integration/pcap_double.c)");
    d->addresses = a;
    *list = d;
    return 0;
}

void pcap_freealldevs(pcap_if_t *list)
{
    while (list) {
        pcap_if_t *next = list->next;
        for (struct pcap_addr *a = list->addresses; a;) {
            struct pcap_addr *an = a->next;
            free(a->addr);
            free(a);
            a = an;
        }
        free(list->name);
        free(list->description);
        free(list);
        list = next;
    }
}

int pcap_lookupnet(const char *dev, bpf_u_int32 *net, bpf_u_int32 *mask, char *errbuf)
{
    *net = 0;
    *mask = 0;
    return 0;
}

pcap_t *pcap_create(const char *dev, char *errbuf)
{
    pcap_t *p = (pcap_t *)calloc(1, sizeof *p);
    if (!p)
        snprintf(errbuf, PCAP_ERRBUF_SIZE, "out of memory");
    return p;
}

int pcap_set_snaplen(pcap_t *p, int n) { return 0; }
int pcap_set_promisc(pcap_t *p, int on) { return 0; }
int pcap_set_timeout(pcap_t *p, int ms) { return 0; }
int pcap_set_immediate_mode(pcap_t *p, int on) { return 0; }
int pcap_activate(pcap_t *p)
{
    p->active = 1;
    return 0;
}
int pcap_setnonblock(pcap_t *p, int nb, char *errbuf) { return 0; }
char *pcap_geterr(pcap_t *p) { return p->err; }

/* The filter is the one pcap_device_open builds (sys_plat.c:598-603):
 * "(ether dst M or ether broadcast) and (not ether src M)". */
int pcap_compile(pcap_t *p, struct bpf_program *fp, const char *expr, int optimize, bpf_u_int32 net)
{
    unsigned m[6];
    if (sscanf(expr, "(ether dst %x:%x:%x:%x:%x:%x", &m[0], &m[1], &m[2], &m[3], &m[4], &m[5]) != 6) {
        snprintf(p->err, sizeof p->err, "pcap_double: filter not understood: %s", expr);
        return -1;
    }
    for (int i = 0; i < 6; i++)
        p->mac[i] = (uint8_t)m[i];
    p->have_mac = 1;
    memset(fp, 0, sizeof *fp);
    return 0;
}

int pcap_setfilter(pcap_t *p, struct bpf_program *fp) { return p->have_mac ? 0 : -1; }

static int passes(const pcap_t *p, const frame_t *f)
{
    static const uint8_t bcast[6] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff};
    if (!p->have_mac)
        return 1;
    if (f->len < 14)
        return 1; /* a runt: the filter cannot match ether fields; let the stack see it */
    return (memcmp(f->bytes, p->mac, 6) == 0 || memcmp(f->bytes, bcast, 6) == 0) &&
           memcmp(f->bytes + 6, p->mac, 6) != 0;
}

/* recv_thread's read (netif_pcap.c:19): 1 with a frame, 0 when none came
 * within a few milliseconds (libpcap's read timeout). */
int pcap_next_ex(pcap_t *p, struct pcap_pkthdr **hdr, const u_char **data)
{
    struct timespec until;
    clock_gettime(CLOCK_REALTIME, &until);
    until.tv_nsec += 5000000L;
    if (until.tv_nsec >= 1000000000L) {
        until.tv_sec++;
        until.tv_nsec -= 1000000000L;
    }
    pthread_mutex_lock(&mu);
    for (;;) {
        while (!rx_head) {
            if (pthread_cond_timedwait(&fed_cv, &mu, &until) == ETIMEDOUT && !rx_head) {
                pthread_mutex_unlock(&mu);
                return 0;
            }
        }
        frame_t *f = rx_head;
        rx_head = f->next;
        if (!rx_head)
            rx_tail = NULL;
        rx_pending--;
        if (!passes(p, f)) {
            __atomic_fetch_add(&filtered, 1, __ATOMIC_RELAXED);
            free(f);
            continue;
        }
        pthread_mutex_unlock(&mu);
        free(p->data);
        p->data = (uint8_t *)f; /* the bytes stay valid until the next call */
        gettimeofday(&p->hdr.ts, NULL);
        p->hdr.caplen = p->hdr.len = f->len;
        *hdr = &p->hdr;
        *data = f->bytes;
        return 1;
    }
}

/* xmit_thread's send (netif_pcap.c:62; the patched driver's inject loop). */
int pcap_inject(pcap_t *p, const void *buf, size_t len)
{
    frame_t *f = frame_new((const uint8_t *)buf, (uint32_t)len);
    pthread_mutex_lock(&mu);
    if (inject_fail > 0) {
        inject_fail--;
        __atomic_fetch_add(&inject_failures, 1, __ATOMIC_RELAXED);
        pthread_mutex_unlock(&mu);
        free(f);
        snprintf(p->err, sizeof p->err, "pcap_double: injected send failure");
        return -1;
    }
    if (inj_n == inj_cap) {
        inj_cap = inj_cap ? 2 * inj_cap : 1024;
        inj = (frame_t **)realloc(inj, inj_cap * sizeof *inj);
        if (!inj) {
            fprintf(stderr, "pcap_double: out of memory\n");
            abort();
        }
    }
    inj[inj_n++] = f;
    answer_arp_locked(f->bytes, f->len);
    pthread_cond_broadcast(&inj_cv);
    pthread_mutex_unlock(&mu);
    return (int)len;
}

void pcap_close(pcap_t *p)
{
    if (p) {
        free(p->data);
        free(p);
    }
}
