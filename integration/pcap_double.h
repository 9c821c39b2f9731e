/*
 * pcap_double.h -- a link-time test double for the libpcap calls of the
 * reference's pcap driver (plat/sys_plat.c:436-618 pcap_device_open and
 * friends; plat/netif_pcap.c:9-67 recv_thread / xmit_thread).  TEST CODE:
 * linked only into the integration test programs (integration/Makefile),
 * never into libtcsum.so.
 *
 * Behind the double is one in-memory "wire":
 *   - frames the test feeds are handed out by pcap_next_ex (recv_thread), in
 *     order, after the BPF filter pcap_device_open installs (its own filter
 *     string is parsed: ether dst = the netif's MAC or broadcast, and not
 *     ether src = that MAC);
 *   - every frame xmit_thread passes to pcap_inject is kept, in order;
 *   - an ARP request among them is answered on the wire (a peer that owns
 *     every address), so replies the stack queues behind ARP resolution
 *     (arp.c:406-460) go out instead of holding packet buffers.
 */
#ifndef TCSUM_PCAP_DOUBLE_H
#define TCSUM_PCAP_DOUBLE_H

#include <stdint.h>

/* The device pcap_findalldevs reports: its IPv4 address (the `ip` of the
 * reference's pcap_data_t, sys_plat.c:441-477) and the MAC of the peer that
 * answers ARP requests. */
void pcapd_setup(const char *device_ip, const uint8_t peer_mac[6]);

/* A frame on the wire, for pcap_next_ex. */
void pcapd_feed(const uint8_t *frame, uint32_t len);

/* Frames fed and not yet taken by pcap_next_ex (filtered ones count as taken). */
uint32_t pcapd_pending(void);

/* Frames pcap_inject was given so far, and frame i of them (valid until
 * pcapd_reset_injected). */
uint32_t pcapd_injected_count(void);
const uint8_t *pcapd_injected(uint32_t i, uint32_t *len);
void pcapd_reset_injected(void);

/* Wait until at least `count` frames were injected; 0 when they were, -1
 * after `ms` milliseconds without. */
int pcapd_wait_injected(uint32_t count, int ms);

/* Make the next `n` pcap_inject calls fail (-1, with pcap_geterr's text), as
 * a send error of the real library would. */
void pcapd_fail_inject(int n);

/* Counters: ARP requests answered, frames dropped by the filter, inject
 * failures reported. */
uint64_t pcapd_arp_replies(void);
uint64_t pcapd_filtered(void);
uint64_t pcapd_inject_failures(void);

#endif
