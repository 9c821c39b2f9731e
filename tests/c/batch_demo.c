/*
 * batch_demo.c -- a plain C host (the reference stack's language) driving the
 * batch C ABI: HIP runtime C API for buffers, libtcsum.so for the sums, and the
 * CPU oracle (liboracle.so) only as the checker.
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

    printf("batch_demo: %u segments, %llu bytes, %u mismatches (device-resident + end-to-end)\n", n,
           (unsigned long long)bytes, bad);
    hipFree(d_arena);
    hipFree(d_segs);
    hipFree(d_out);
    return bad ? 1 : 0;
}
