"""ctypes binding of libtcsum.so (the C ABI declared in include/*.h).

The libraries are loaded from this package directory only; if one is missing
the import of any compute entry point raises -- there is no CPU fallback.
libtcsum.so is the product; libtcsum_bench.so (include/tcsum_synth.h) holds
the synthetic-data and load-probe kernels the tests and bench.py use.
"""
from __future__ import annotations

import ctypes
import os

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libtcsum.so")

# Return codes (net_err_t values, net/net/net_err.h:8-29)
OK = 0
ERR_SYS = -1
ERR_MEM = -2
ERR_SIZE = -5
ERR_PARAM = -7
ERR_NOT_SUPPORT = -11
ERR_BROKEN = -13
PCAP_ARP = 1  # tcsum_pcap_index l2 verdict: the frame goes to arp_in

# (name, restype, argtypes) for every symbol include/*.h declares
_V, _U16, _U32, _U64, _I, _SZ = (ctypes.c_void_p, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64,
                                  ctypes.c_int, ctypes.c_size_t)
SIGNATURES = {
    # tcsum.h
    "tcsum_batch": (_I, [_I, _V, _V, _U32, _V, _V, _V, _V, _V]),
    "tcsum_batch_segments": (_I, [_V, _V, _U32, _V, _I, _U64, _V]),
    "tcsum_batch_peso": (_I, [_V, _V, _U32, _V, _U64, _V]),
    "tcsum_batch_ipv4": (_I, [_V, _V, _U32, _V, _V, _U64, _V]),
    "tcsum_batch_ipv4_tx_fill": (_I, [_V, _V, _U32, _V, _V, _U64, _V]),
    "tcsum_batch_ipv4_tx_fill_scratch": (_I, [_V, _V, _U32, _V, _V, _V, _U64, _U64, _V]),
    "tcsum_batch_ipv4_rx_verify": (_I, [_V, _V, _U32, _V, _V, _V, _U64, _V]),
    "tcsum_batch_ipv4_tx_offload": (_I, [_V, _V, _U32, _V, _V, _U64, _V]),
    "tcsum_tx_apply": (_I, [_V, _U32, _U32, ctypes.c_uint8]),
    "tcsum_tx_apply_batch": (_I, [_V, _U64, _V, _U32, _V, _V]),
    "tcsum_host_batch_peso": (_I, [_I, _V, _U64, _V, _U32, _V]),
    "tcsum_host_batch_peso_multi": (_I, [_V, _I, _V, _U64, _V, _U32, _V]),
    "tcsum_host_batch_ipv4": (_I, [_I, _V, _U64, _V, _U32, _V, _V]),
    "tcsum_host_batch_ipv4_tx_fill": (_I, [_I, _V, _U64, _V, _U32, _V, _V]),
    "tcsum_host_batch_ipv4_rx_verify": (_I, [_I, _V, _U64, _V, _U32, _V, _V, _V]),
    "tcsum_host_batch_ipv4_multi": (_I, [_V, _I, _V, _U64, _V, _U32, _V, _V]),
    "tcsum_host_batch_ipv4_tx_fill_multi": (_I, [_V, _I, _V, _U64, _V, _U32, _V, _V]),
    "tcsum_host_batch_ipv4_rx_verify_multi": (_I, [_V, _I, _V, _U64, _V, _U32, _V, _V, _V]),
    "tcsum_queue_server": (_I, [_I, _I]),
    "tcsum_call_server": (_I, [_I, _I]),
    "tcsum_plat_init": (_I, [_I]),
    "tcsum_host_alloc": (_V, [_SZ]),
    "tcsum_host_free": (None, [_V]),
    "tcsum_host_register": (_I, [_V, _SZ]),
    "tcsum_host_unregister": (_I, [_V]),
    "tcsum_device_count": (_I, []),
    "tcsum_pick_geometry": (None, [_U64, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "tcsum_version": (ctypes.c_char_p, []),
    "tcsum_release": (_I, [_I]),
    # tcsum_legacy.h
    "checksum16": (_U16, [_I, _V, _U16, _U32, _I]),
    "checksum_peso": (_U16, [_V, _V, _V, ctypes.c_uint8]),
    "pktbuf_checksum16": (_U16, [_V, _I, _I, _I]),
    # tcsum_debug.h (tests and measurement only)
    "tcsum_debug_set": (_I, [ctypes.c_char_p, ctypes.c_int64]),
    "tcsum_debug_get": (ctypes.c_int64, [ctypes.c_char_p]),
    "tcsum_debug_route": (None, [_U64, ctypes.POINTER(ctypes.c_int32)]),
    "tcsum_debug_ipv4_route": (None, [_U64, _I, ctypes.POINTER(ctypes.c_int32)]),
    "tcsum_debug_plan_host_peso": (ctypes.c_int64, [_V, _U32, _U64, _V, _U32, _V]),
    "tcsum_debug_shards": (_I, [_V, _I]),
}

# tcsum_synth.h: libtcsum_bench.so (synthetic batches, load probes)
BENCH_LIB_PATH = os.path.join(PKG, "libtcsum_bench.so")
BENCH_SIGNATURES = {
    "tcsum_synth_fill": (_I, [_V, _U64, _U64, _U64, _V]),
    "tcsum_synth_ipv4": (_I, [_V, _V, _U32, _U64, _V]),
    "tcsum_probe_read": (_I, [_V, _U64, _V, _V]),
    "tcsum_probe_tile": (_I, [_V, _U64, _I, _I, _I, _V, _V]),
    "tcsum_probe_segments": (_I, [_V, _V, _U32, _U64, _V, _V]),
    "tcsum_probe_ipv4": (_I, [_V, _V, _U32, _U64, _I, _V, _V]),
    "tcsum_probe_flat": (_I, [_V, _V, _U32, _U64, _I, _I, _I, _V, _U64, _V, _V]),
    "tcsum_flat_ipv4": (_I, [_I, _V, _V, _U32, _U64, _V, _V, _V, _V]),
    "tcsum_probe_ipv4_shape": (_I, [_V, _V, _U32, _I, _I, _I, _V, _V, _V]),
    "tcsum_probe_window": (_I, [_V, _U64, _I, _I, _I, _V, _V, _U64, _V, _V]),
    "tcsum_probe_txfloor_windows": (_U32, [_U64]),
    "tcsum_probe_txfloor_prepare": (_I, [_V, _U64, _V, _U32, _U64, _V, _U64, _V, _U64, _V, _U64, _V]),
    "tcsum_probe_txfloor": (_I, [_V, _U64, _V, _V, _U32, _V, _I, _V, _V]),
}

# tcsum_pcap.h: the capture-file helper, libtcsum_pcap.so (host-only)
PCAP_LIB_PATH = os.path.join(PKG, "libtcsum_pcap.so")
PCAP_SIGNATURES = {
    "tcsum_pcap_index": (_I, [_V, _U64, _V, _V, _U32, ctypes.POINTER(_U32)]),
}

_lib = None
_bench_lib = None
_pcap_lib = None


def lib() -> ctypes.CDLL:
    """The loaded product library; raises if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                " (there is no CPU fallback)")
        # PyTorch ships its own HIP runtime under the same SONAME
        # (libamdhip64.so.7): load it first so this library binds to that one
        # copy -- loaded the other way round, torch's own init fails
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def bench_lib() -> ctypes.CDLL:
    """The measurement / synthetic-data library (include/tcsum_synth.h)."""
    global _bench_lib
    if _bench_lib is None:
        lib()  # its dependency, bound to torch's HIP runtime first
        if not os.path.exists(BENCH_LIB_PATH):
            raise RuntimeError(f"{BENCH_LIB_PATH} is missing: build it with __graft_entry__.build()")
        L = ctypes.CDLL(BENCH_LIB_PATH)
        for name, (res, args) in BENCH_SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _bench_lib = L
    return _bench_lib


def pcap_lib() -> ctypes.CDLL:
    """The capture-file helper library (include/tcsum_pcap.h)."""
    global _pcap_lib
    if _pcap_lib is None:
        if not os.path.exists(PCAP_LIB_PATH):
            raise RuntimeError(f"{PCAP_LIB_PATH} is missing: build it with __graft_entry__.build()")
        L = ctypes.CDLL(PCAP_LIB_PATH)
        for name, (res, args) in PCAP_SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _pcap_lib = L
    return _pcap_lib


def check(rc: int, what: str) -> None:
    if rc != OK:
        extra = ""
        if rc in (ERR_SYS, ERR_MEM):
            v = lib().tcsum_debug_get(b"last_sys_error")  # step * 1000 + hipError_t (tcsum_debug.h)
            extra = f" (last failed HIP call: step {v // 1000}, hipError_t {v % 1000})"
        raise RuntimeError(f"{what} failed with net_err_t {rc}{extra}")
