/*
 * batch_demo.c -- a plain C host (the reference stack's language) driving the
 * batch C ABI: HIP runtime C API for buffers, libtcsum.so for the sums, and the
 * CPU oracle (liboracle.so) only as the checker; the tx fill is also captured
 * in a hipGraph through the C API.
 *
 * TEST INFRASTRUCTURE.  Built by tests/c/Makefile into tests/c/build/; run by
 * tests/test_gpu_parity.py::test_c_host_batch_demo.  Exit 0 when every result
 * matches.
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "csum_oracle.h"
#include "tcsum.h"

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                \
            return 2;                                                                              \
        }                                                                                          \
    } while (0)

static uint64_t rng = 20240807u;
static uint64_t next(void) { return rng = orc_splitmix64(rng); }

int main(void)
{
    const uint32_t n = 20000;
    /* TCP/UDP segments of 1..9000 bytes packed back to back (odd offsets too) */
    tcsum_peso_t *segs = calloc(n, sizeof *segs);
    uint64_t at = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint64_t r = next();
        segs[i].offset = at;
        segs[i].len = 1 + (uint32_t)(r % 9000);
        memcpy(segs[i].src, &r, 4);
        memcpy(segs[i].dst, (uint8_t *)&r + 4, 4);
        segs[i].protocol = (r >> 40) & 1 ? 17 : 6;
        at += segs[i].len;
    }
    const uint64_t bytes = at;
    uint8_t *host = malloc(bytes + 64);
    for (uint64_t i = 0; i < bytes; i += 8) {
        uint64_t r = next();
        memcpy(host + i, &r, 8);
    }

    if (tcsum_plat_init(0) != TCSUM_OK) { /* net_plat_init hook */
        fprintf(stderr, "no gfx950 device\n");
        return 2;
    }
    void *d_arena, *d_segs, *d_out;
    CHECK(hipMalloc(&d_arena, bytes + 64));
    CHECK(hipMalloc(&d_segs, sizeof(tcsum_peso_t) * n));
    CHECK(hipMalloc(&d_out, sizeof(uint16_t) * n));
    CHECK(hipMemcpy(d_arena, host, bytes + 64, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_segs, segs, sizeof(tcsum_peso_t) * n, hipMemcpyHostToDevice));

    int rc = tcsum_batch_peso(d_arena, d_segs, n, d_out, bytes, NULL);
    if (rc != TCSUM_OK) {
        fprintf(stderr, "tcsum_batch_peso: %d\n", rc);
        return 2;
    }
    CHECK(hipDeviceSynchronize());
    uint16_t *got = malloc(sizeof(uint16_t) * n), *want = malloc(sizeof(uint16_t) * n);
    CHECK(hipMemcpy(got, d_out, sizeof(uint16_t) * n, hipMemcpyDeviceToHost));
    orc_batch_peso(host, (const orc_peso_t *)segs, n, want, 8);
    uint32_t bad = 0;
    for (uint32_t i = 0; i < n; i++)
        bad += got[i] != want[i];

    /* the same batch from pinned host memory, end to end */
    uint8_t *pinned = tcsum_host_alloc(bytes + 64);
    memcpy(pinned, host, bytes + 64);
    memset(got, 0, sizeof(uint16_t) * n);
    rc = tcsum_host_batch_peso(0, pinned, bytes, segs, n, got);
    for (uint32_t i = 0; i < n; i++)
        bad += rc != TCSUM_OK || got[i] != want[i];
    tcsum_host_free(pinned);

    /* a tx fill captured in a hipGraph (the deferred-store form with scratch
     * the caller owns) and replayed twice over the same IPv4 packets, laid
     * over the segments: IHL 5, total_len = segment length */
    const uint32_t m = n;
    tcsum_pkt_t *pk = calloc(m, sizeof *pk);
    uint8_t *ip = malloc(bytes + 64);
    memcpy(ip, host, bytes + 64);
    uint32_t m_ok = 0;
    for (uint32_t i = 0; i < m; i++) {
        uint8_t *h = ip + segs[i].offset;
        pk[i].offset = segs[i].offset;
        pk[i].len = segs[i].len;
        if (segs[i].len < 40)
            continue;
        h[0] = 0x45;
        h[2] = (uint8_t)(segs[i].len >> 8);
        h[3] = (uint8_t)segs[i].len;
        h[6] = 0x40;
        h[7] = 0;
        h[9] = segs[i].protocol;
        m_ok++;
    }
    uint8_t *ip_want = malloc(bytes + 64);
    memcpy(ip_want, ip, bytes + 64);
    uint8_t *fl = malloc(m);
    orc_batch_ipv4_tx_fill(ip_want, (const orc_pkt_t *)pk, m, fl, 8);
    void *d_pk, *d_scratch;
    CHECK(hipMalloc(&d_pk, sizeof(tcsum_pkt_t) * m));
    CHECK(hipMalloc(&d_scratch, 8ull * m));
    CHECK(hipMemcpy(d_pk, pk, sizeof(tcsum_pkt_t) * m, hipMemcpyHostToDevice));
    hipStream_t st;
    hipGraph_t graph;
    hipGraphExec_t exec;
    CHECK(hipStreamCreate(&st));
    CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    rc = tcsum_batch_ipv4_tx_fill_scratch(d_arena, d_pk, m, NULL, NULL, d_scratch, 8ull * m, bytes, st);
    CHECK(hipStreamEndCapture(st, &graph));
    if (rc != TCSUM_OK) {
        fprintf(stderr, "tcsum_batch_ipv4_tx_fill_scratch under capture: %d\n", rc);
        return 2;
    }
    CHECK(hipGraphInstantiate(&exec, graph, NULL, NULL, 0));
    uint8_t *filled = malloc(bytes + 64);
    uint64_t graph_bad = 0;
    for (int rep = 0; rep < 2; rep++) {
        CHECK(hipMemcpy(d_arena, ip, bytes + 64, hipMemcpyHostToDevice));
        CHECK(hipGraphLaunch(exec, st));
        CHECK(hipStreamSynchronize(st));
        CHECK(hipMemcpy(filled, d_arena, bytes + 64, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < bytes; i++)
            graph_bad += filled[i] != ip_want[i];
    }
    bad += graph_bad != 0;
    CHECK(hipGraphExecDestroy(exec));
    CHECK(hipGraphDestroy(graph));
    CHECK(hipStreamDestroy(st));
    hipFree(d_pk);
    hipFree(d_scratch);
    printf("batch_demo: hipGraph tx fill over %u IPv4 packets (%u with headers), 2 replays: %llu bytes differ\n", m,
           m_ok, (unsigned long long)graph_bad);

    printf("batch_demo: %u segments, %llu bytes, %u mismatches (device-resident + end-to-end + graph)\n", n,
           (unsigned long long)bytes, bad);
    hipFree(d_arena);
    hipFree(d_segs);
    hipFree(d_out);
    return bad ? 1 : 0;
}
