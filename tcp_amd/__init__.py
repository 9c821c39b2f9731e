"""tcp_amd -- MI355X-native Internet-checksum engine for the wj9806/tcp stack.

The product is tcp_amd/libtcsum.so (C ABI: include/tcsum.h,
include/tcsum_legacy.h, include/tcsum_debug.h); this package is its Python
face.  Synthetic batches and load probes come from libtcsum_bench.so
(include/tcsum_synth.h).
"""
from .csum import (LAYOUT_ORDERED, LAYOUT_SHUFFLED, LAYOUT_UNKNOWN, OP_IPV4, OP_IPV4_RX_VERIFY, OP_IPV4_TX_FILL,
                   OP_IPV4_TX_OFFLOAD, OP_PESO, OP_SEGMENTS, OP_SEGMENTS_COMP, PESO_DTYPE, PKT_DTYPE, SEG_DTYPE, batch,
                   batch_ipv4, batch_ipv4_rx_verify, batch_ipv4_tx_fill,
                   batch_ipv4_tx_offload, tx_apply_batch, batch_peso, batch_segments,
                   checksum16, checksum_peso, descs_to_device, device_count, host_batch_peso, host_batch_peso_multi,
                   HostArena, host_register, host_unregister, host_batch_ipv4, host_batch_ipv4_rx_verify, host_batch_ipv4_tx_fill,
                   pick_geometry, route, ipv4_route, debug, last_shards, flat_ipv4, debug_get, debug_set, pktbuf_checksum16, plat_init, probe_ipv4, probe_read, probe_segments, probe_tile, probe_txfloor, txfloor_prepare, queue_server, release, call_server, synth_fill,
                   synth_ipv4, to_host, to_host_tensor)
from .pktbuf import IpAddr, PktBuf
from . import pcap, workload

__all__ = [
    "checksum16", "checksum_peso", "pktbuf_checksum16", "batch", "batch_segments", "batch_peso", "batch_ipv4",
    "batch_ipv4_tx_fill", "batch_ipv4_tx_offload", "tx_apply_batch", "batch_ipv4_rx_verify",
    "host_batch_peso", "host_batch_peso_multi", "HostArena", "host_register", "host_unregister", "host_batch_ipv4", "host_batch_ipv4_tx_fill", "host_batch_ipv4_rx_verify",
    "synth_fill", "synth_ipv4", "descs_to_device", "device_count", "pick_geometry", "route", "ipv4_route", "debug", "last_shards", "flat_ipv4",
    "debug_get", "debug_set", "to_host", "to_host_tensor",
    "plat_init", "probe_ipv4", "probe_read", "probe_segments", "probe_tile", "probe_txfloor", "txfloor_prepare", "queue_server", "release", "call_server", "PktBuf", "IpAddr", "SEG_DTYPE", "PESO_DTYPE", "PKT_DTYPE", "pcap", "workload",
]
