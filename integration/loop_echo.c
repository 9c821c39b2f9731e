/*
 * loop_echo.c -- BASELINE configs[0] ("app/echo over loopback") on the
 * reference stack patched by integration/net_checksum_gpu.patch.  Built with
 * -DNET_CHECKSUM_GPU (_build/loop_echo): every checksum the stack stores or
 * tests goes through libtcsum.so's batched fill (loop_xmit) and batched sums
 * (do_netif_in).  Built without it (_build/loop_echo_cpu): the reference's
 * own CPU checksum, i.e. configs[0] as the reference runs it.
 *
 * TEST PROGRAM.  Built by integration/Makefile into integration/_build/ from a
 * patched copy of /root/reference; run by tests/test_integration.py on the
 * GPU box.  Echo servers and clients use the reference's own socket API
 * (net_api.h), bound to INADDR_ANY on the loop netif 127.0.0.1/8 (loop.c:41-60;
 * the reference's tcp_echo_server binds netdev0_ip, tcp_echo_server.c:27,
 * which is the pcap netif this image cannot open).
 *
 * Exit 0 when every UDP datagram and every TCP byte comes back intact and the
 * engine's counters show that the frames were filled and checked on the GPU.
 * The one platform fix: sys_mutex_create is made recursive here (the Makefile
 * weakens the Linux definition), as pktbuf_free takes the pktbuf lock twice
 * (pktbuf.c:203 -> :44) and deadlocks on a default pthread mutex.
 *
 * Options: --udp-only; --rounds N (UDP datagrams, default 200); --tcp-bytes N
 * (default 65536); --ref-udp-server: the UDP server is the reference's own
 * app/echo/udp_echo_server.c, compiled unchanged (it binds INADDR_ANY,
 * udp_echo_server.c:22, and echoes at most 125 bytes, :31-33, so datagrams
 * are 1-125 B).  Both phases print their wall time: round trips per second
 * for UDP, MB/s for TCP (configs[0]'s only numbers).
 */
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <time.h>

#include "net.h"
#include "net_api.h"
#include "app/echo/udp_echo_server.h"
#include "net_csum_gpu.h"
#include "sys_plat.h"
#ifdef NET_CHECKSUM_GPU
#include "tcsum.h"
#endif

sys_mutex_t sys_mutex_create(void)
{
    pthread_mutex_t *m = (pthread_mutex_t *)malloc(sizeof *m);
    pthread_mutexattr_t a;
    pthread_mutexattr_init(&a);
    pthread_mutexattr_settype(&a, PTHREAD_MUTEX_RECURSIVE);
    pthread_mutex_init(m, &a);
    pthread_mutexattr_destroy(&a);
    return m;
}

#define UDP_PORT 7
#define TCP_PORT 8
static int UDP_ROUNDS = 200, UDP_MAX = 1400, TCP_BYTES = 64 * 1024;
#define TCP_INFLIGHT 2100 /* below the reference's 4-KiB window (TCP_RBUF / TCP_SBUF, net_cfg.h) */

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void udp_server(void *arg)
{
    int s = socket(AF_INET, SOCK_DGRAM, 0);
    struct sockaddr_in a;
    memset(&a, 0, sizeof a);
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = INADDR_ANY;
    a.sin_port = htons(UDP_PORT);
    if (s < 0 || bind(s, (const struct sockaddr *)&a, sizeof a) < 0) {
        fprintf(stderr, "udp server: socket/bind failed\n");
        return;
    }
    for (;;) {
        static char buf[2048];
        struct sockaddr_in c;
        x_socklen_t len = sizeof c;
        ssize_t n = recvfrom(s, buf, sizeof buf, 0, (struct sockaddr *)&c, &len);
        if (n <= 0)
            continue;
        sendto(s, buf, (size_t)n, 0, (struct sockaddr *)&c, len);
    }
}

static void tcp_server(void *arg)
{
    int s = socket(AF_INET, SOCK_STREAM, 0);
    struct sockaddr_in a;
    memset(&a, 0, sizeof a);
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = INADDR_ANY;
    a.sin_port = htons(TCP_PORT);
    if (s < 0 || bind(s, (const struct sockaddr *)&a, sizeof a) < 0 || listen(s, 5) < 0) {
        fprintf(stderr, "tcp server: socket/bind/listen failed\n");
        return;
    }
    for (;;) {
        struct sockaddr_in c;
        x_socklen_t len = sizeof c;
        int cl = accept(s, (struct sockaddr *)&c, &len);
        if (cl < 0)
            continue;
        static char buf[1024];
        ssize_t n;
        while ((n = recv(cl, buf, sizeof buf, 0)) > 0)
            send(cl, buf, (size_t)n, 0);
        close(cl);
    }
}

static int set_timeout(int s, int ms)
{
    struct x_timeval tv = {ms / 1000, (ms % 1000) * 1000};
    return setsockopt(s, SOL_SOCKET, SO_RCVTIMEO, (const char *)&tv, sizeof tv);
}

static void fill(uint8_t *p, int n, int seed)
{
    for (int i = 0; i < n; i++)
        p[i] = (uint8_t)(seed * 131 + i * 7 + (i >> 8));
}

static int udp_echo(void)
{
    int s = socket(AF_INET, SOCK_DGRAM, 0);
    if (s < 0)
        return fprintf(stderr, "udp client: socket failed\n"), 1;
    set_timeout(s, 2000);
    struct sockaddr_in to;
    memset(&to, 0, sizeof to);
    to.sin_family = AF_INET;
    to.sin_addr.s_addr = inet_addr("127.0.0.1");
    to.sin_port = htons(UDP_PORT);
    static uint8_t out[1500], in[2048];
    const double t0 = now_s();
    long bytes = 0;
    for (int r = 0; r < UDP_ROUNDS; r++) {
        int n = 1 + (r * 37) % UDP_MAX; /* the loop netif has mtu 0: no fragmentation (ipv4.c:616) */
        bytes += n;
        fill(out, n, r);
        if (sendto(s, out, (size_t)n, 0, (const struct sockaddr *)&to, sizeof to) != n)
            return fprintf(stderr, "udp round %d: sendto failed\n", r), 1;
        struct sockaddr_in from;
        x_socklen_t len = sizeof from;
        ssize_t got = recvfrom(s, in, sizeof in, 0, (struct sockaddr *)&from, &len);
        if (got != n || memcmp(in, out, (size_t)n) != 0)
            return fprintf(stderr, "udp round %d: sent %d bytes, echo %ld\n", r, n, (long)got), 1;
        if (r % 50 == 0)
            printf("udp round %d ok\n", r);
    }
    const double dt = now_s() - t0;
    close(s);
    printf("udp: %d datagrams (1-%d B) echoed intact\n", UDP_ROUNDS, UDP_MAX);
    printf("timing udp: %d round trips, %ld bytes each way, %.3f s: %.0f round trips/s, %.3f MB/s\n", UDP_ROUNDS,
           bytes, dt, UDP_ROUNDS / dt, bytes / dt / 1e6);
    return 0;
}

static int tcp_echo(void)
{
    int s = socket(AF_INET, SOCK_STREAM, 0);
    if (s < 0)
        return fprintf(stderr, "tcp client: socket failed\n"), 1;
    struct sockaddr_in to;
    memset(&to, 0, sizeof to);
    to.sin_family = AF_INET;
    to.sin_addr.s_addr = inet_addr("127.0.0.1");
    to.sin_port = htons(TCP_PORT);
    if (connect(s, (const struct sockaddr *)&to, sizeof to) < 0)
        return fprintf(stderr, "tcp client: connect failed\n"), 1;
    uint8_t *out = (uint8_t *)malloc((size_t)TCP_BYTES), *in = (uint8_t *)malloc((size_t)TCP_BYTES);
    if (!out || !in)
        return fprintf(stderr, "tcp client: out of memory\n"), 1;
    fill(out, TCP_BYTES, 99);
    int sent = 0, got = 0;
    const double t0 = now_s();
    while (got < TCP_BYTES) {
        /* at most TCP_INFLIGHT bytes sent and not yet echoed: with more, the
         * client can block in send() on a peer whose own send() waits for the
         * client to read -- both windows at 0, which the reference's TCP only
         * leaves by its retransmission timer (seconds per stall) */
        if (sent < TCP_BYTES && sent - got < TCP_INFLIGHT) {
            int chunk = TCP_BYTES - sent < 700 ? TCP_BYTES - sent : 700;
            ssize_t k = send(s, out + sent, (size_t)chunk, 0);
            if (k <= 0)
                return fprintf(stderr, "tcp: send failed at %d\n", sent), 1;
            sent += (int)k;
        }
        ssize_t k = recv(s, in + got, (size_t)(TCP_BYTES - got), 0);
        if (k <= 0)
            return fprintf(stderr, "tcp: recv failed at %d of %d\n", got, TCP_BYTES), 1;
        got += (int)k;
    }
    const double dt = now_s() - t0;
    if (memcmp(in, out, (size_t)TCP_BYTES) != 0) {
        /* where, and how: the reference's TCP occasionally hands a stretch of
         * the stream back out of place (CPU build too, no GPU involved) */
        int first = -1, ndiff = 0, last = -1;
        for (int i = 0; i < TCP_BYTES; i++)
            if (in[i] != out[i]) {
                if (first < 0)
                    first = i;
                last = i;
                ndiff++;
            }
        int shift = 0; /* the received bytes at `first` found at out[first + d], |d| <= 64 KiB */
        for (int d = -65536; d <= 65536 && !shift; d++)
            if (d && first + d >= 0 && first + d + 64 <= TCP_BYTES && first + 64 <= TCP_BYTES &&
                memcmp(in + first, out + first + d, 64) == 0)
                shift = d;
        fprintf(stderr, "tcp: got  ");
        for (int i = first; i < first + 16; i++)
            fprintf(stderr, " %02x", in[i]);
        fprintf(stderr, "\ntcp: sent ");
        for (int i = first; i < first + 16; i++)
            fprintf(stderr, " %02x", out[i]);
        fprintf(stderr, "\n");
        fprintf(stderr, "tcp: echoed bytes differ: %d bytes differ in [%d, %d]; the bytes at %d are the "
                        "sent stream's at offset %+d (0: not found)\n", ndiff, first, last, first, shift);
        /* the transfer itself completed: its time still says what the path costs */
        printf("timing tcp: %d bytes each way, %.3f s: %.3f MB/s (echo corrupted by the reference's TCP)\n",
               TCP_BYTES, dt, TCP_BYTES / dt / 1e6);
        return 1;
    }
    close(s);
    printf("tcp: %d bytes echoed intact\n", TCP_BYTES);
    printf("timing tcp: %d bytes each way, %.3f s: %.3f MB/s\n", TCP_BYTES, dt, TCP_BYTES / dt / 1e6);
    return 0;
}

static void print_engine(void)
{
#ifdef NET_CHECKSUM_GPU
    net_csum_gpu_stats_t st;
    net_csum_gpu_stats(&st);
    printf("engine: tx %llu frames in %llu batches, rx %llu frames in %llu batches, "
           "%llu with a filled header checksum, %llu checksum tests answered from a batch\n",
           (unsigned long long)st.tx_frames, (unsigned long long)st.tx_batches,
           (unsigned long long)st.rx_frames, (unsigned long long)st.rx_batches,
           (unsigned long long)st.rx_ip_filled, (unsigned long long)st.rx_used);
    // frames per batch (tx coalescing, net_csum_gpu.h): 1, 2-3, 4-7, 8-15, 16-31, >= 32
    printf("batch sizes: tx [1 %llu | 2-3 %llu | 4-7 %llu | 8-15 %llu | 16-31 %llu | 32+ %llu], "
           "rx [1 %llu | 2-3 %llu | 4-7 %llu | 8-15 %llu | 16-31 %llu | 32+ %llu], %llu flushes\n",
           (unsigned long long)st.tx_hist[0], (unsigned long long)st.tx_hist[1], (unsigned long long)st.tx_hist[2],
           (unsigned long long)st.tx_hist[3], (unsigned long long)st.tx_hist[4], (unsigned long long)st.tx_hist[5],
           (unsigned long long)st.rx_hist[0], (unsigned long long)st.rx_hist[1], (unsigned long long)st.rx_hist[2],
           (unsigned long long)st.rx_hist[3], (unsigned long long)st.rx_hist[4], (unsigned long long)st.rx_hist[5],
           (unsigned long long)st.tx_flushes);
#else
    printf("engine: none (the reference's own CPU checksum, configs[0])\n");
#endif
}

static const char *volatile stage = "start";
static void watchdog(int sig)
{
    printf("watchdog: no progress for 60 s at stage '%s'\n", stage);
    print_engine();
    _exit(3);
}

int main(int argc, char **argv)
{
    setvbuf(stdout, NULL, _IONBF, 0);
    signal(SIGALRM, watchdog);
    alarm(60);
    int do_tcp = 1, ref_server = 0;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "--udp-only"))
            do_tcp = 0;
        else if (!strcmp(argv[i], "--ref-udp-server"))
            ref_server = 1, UDP_MAX = 125;
        else if (!strcmp(argv[i], "--rounds") && i + 1 < argc)
            UDP_ROUNDS = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--tcp-bytes") && i + 1 < argc)
            TCP_BYTES = atoi(argv[++i]);
    }
#ifdef NET_CHECKSUM_GPU
    if (tcsum_device_count() < 1) /* net_init ignores net_plat_init's result (net.c:22) */
        return fprintf(stderr, "no gfx950 device: the GPU build cannot run here\n"), 2;
#endif
    stage = "net_init";
    if (net_init() != NET_ERR_OK) /* net_plat_init -> net_csum_gpu_init (HIP device, pinned staging) */
        return fprintf(stderr, "net_init failed\n"), 2;
    stage = "net_start";
    net_start();
    if (ref_server)
        udp_echo_server_start(UDP_PORT); /* the reference's app/echo server, unchanged */
    else
        sys_thread_create(udp_server, (void *)0);
    if (do_tcp)
        sys_thread_create(tcp_server, (void *)0);
    sys_sleep(100);
    stage = "udp";
    int rc = udp_echo();
    stage = "tcp";
    if (!rc && do_tcp)
        rc = tcp_echo();
    alarm(0);
    print_engine();
#ifdef NET_CHECKSUM_GPU
    net_csum_gpu_stats_t st;
    net_csum_gpu_stats(&st);
    if (!rc && (st.tx_frames < 2 * UDP_ROUNDS || st.rx_frames < 2 * UDP_ROUNDS ||
                st.rx_ip_filled != st.rx_frames || st.rx_used < 4 * UDP_ROUNDS)) {
        fprintf(stderr, "the frames did not all go through the GPU fill and sums\n");
        rc = 1;
    }
#endif
    fflush(stdout);
    _exit(rc); /* the stack's threads never return; skip exit-time teardown under them */
}
