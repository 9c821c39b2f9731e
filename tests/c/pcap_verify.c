/* tests/c/pcap_verify.c -- a plain C host of INTEGRATION.md §4b: verify every
 * frame of a libpcap savefile with the stack's rx rules, on the GPU.
 *
 *   pcap_verify FILE [VERDICTS_OUT]
 *
 * Reads FILE into pinned memory (tcsum_host_alloc), indexes it
 * (tcsum_pcap_index), runs tcsum_host_batch_ipv4_rx_verify over the file in
 * place, keeps ether_in's verdict for frames that never reach ipv4_in, and
 * prints one count per net_err_t value.  With VERDICTS_OUT, the per-frame
 * verdicts (int8) are written there for the test to compare. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tcsum.h"
#include "tcsum_pcap.h"

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s FILE [VERDICTS_OUT]\n", argv[0]);
        return 2;
    }
    FILE *fp = fopen(argv[1], "rb");
    if (!fp || fseek(fp, 0, SEEK_END) != 0) {
        perror(argv[1]);
        return 2;
    }
    const long bytes = ftell(fp);
    rewind(fp);
    uint8_t *file = tcsum_host_alloc(bytes > 0 ? (size_t)bytes : 1);
    if (!file || fread(file, 1, (size_t)bytes, fp) != (size_t)bytes) {
        fprintf(stderr, "cannot read %s into pinned memory\n", argv[1]);
        return 2;
    }
    fclose(fp);

    uint32_t n = 0;
    int rc = tcsum_pcap_index(file, (uint64_t)bytes, NULL, NULL, 0, &n);
    if (rc != TCSUM_OK && rc != TCSUM_ERR_MEM) {
        fprintf(stderr, "tcsum_pcap_index: %d\n", rc);
        return 1;
    }
    tcsum_pkt_t *pk = malloc((n ? n : 1) * sizeof *pk);
    int8_t *l2 = malloc(n ? n : 1), *v = malloc(n ? n : 1);
    if (!pk || !l2 || !v)
        return 2;
    if ((rc = tcsum_pcap_index(file, (uint64_t)bytes, pk, l2, n, &n)) != TCSUM_OK) {
        fprintf(stderr, "tcsum_pcap_index: %d\n", rc);
        return 1;
    }
    if ((rc = tcsum_host_batch_ipv4_rx_verify(0, file, (uint64_t)bytes, pk, n, v, NULL, NULL)) != TCSUM_OK) {
        fprintf(stderr, "tcsum_host_batch_ipv4_rx_verify: %d\n", rc);
        return 1;
    }
    unsigned count[256] = {0};
    for (uint32_t i = 0; i < n; ++i) {
        if (l2[i] != TCSUM_OK)
            v[i] = l2[i]; /* TCSUM_PCAP_ARP, TCSUM_ERR_SIZE, TCSUM_ERR_NOT_SUPPORT */
        count[(uint8_t)v[i]]++;
    }
    printf("%u frames:", n);
    for (int k = -128; k < 128; ++k)
        if (count[(uint8_t)k])
            printf(" %d:%u", k, count[(uint8_t)k]);
    printf("\n");
    if (argc > 2) {
        FILE *out = fopen(argv[2], "wb");
        if (!out || fwrite(v, 1, n, out) != n) {
            perror(argv[2]);
            return 2;
        }
        fclose(out);
    }
    free(pk);
    free(l2);
    free(v);
    tcsum_host_free(file);
    return 0;
}
