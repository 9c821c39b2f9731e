"""ctypes view of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, ``__graft_entry__.smoke()`` and
bench.py's ``cpu_baseline`` leg, and there only as the checker or the timed
CPU baseline.  The product path (``tcp_amd``) never imports this module.

Every function restates a reference routine; see oracle/csum_oracle.h for the
file:line anchors (net/src/tools.c:24-75, net/src/pktbuf.c:646-670).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_LIB_PATH = os.path.join(HERE, "_ref", "libtcpref.so")
REF_O3_LIB_PATH = os.path.join(HERE, "_ref", "libtcpref_o3.so")  # -O3 -march=x86-64-v3

# numpy views of the batch descriptors (identical to include/tcsum.h)
SEG_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("pre_sum", "<u4")])
PESO_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("src", "u1", 4),
                       ("dst", "u1", 4), ("protocol", "u1"), ("rsv", "u1", 3)])
PKT_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("rsv", "<u4")])
assert SEG_DTYPE.itemsize == 16 and PESO_DTYPE.itemsize == 24 and PKT_DTYPE.itemsize == 16

_lib = None


def build(force: bool = False) -> None:
    """Compile liboracle.so with gcc (and oracle/_ref when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE] + (["-B"] if force else []) + ["all"], check=True)


def build_ref() -> bool:
    """Compile oracle/_ref from the reference sources (golden generators, the
    reference CPU baseline, and the drop-in link test against libtcsum.so);
    False when /root/reference is absent (the GPU box uses the prebuilt files)."""
    if not os.path.isdir("/root/reference/net/src"):
        return False
    subprocess.run(["make", "-s", "-C", HERE, "ref", "stack", "dropin"], check=True)
    return True


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.c_void_p
        L.orc_checksum16.argtypes = [ctypes.c_int, u8p, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_int]
        L.orc_checksum16.restype = ctypes.c_uint16
        L.orc_pieces_checksum16.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_pieces_checksum16.restype = ctypes.c_uint16
        L.orc_flat_checksum16.argtypes = [u8p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
        L.orc_flat_checksum16.restype = ctypes.c_uint16
        L.orc_pseudo_sum.argtypes = [u8p, u8p, ctypes.c_uint8, ctypes.c_uint32]
        L.orc_pseudo_sum.restype = ctypes.c_uint16
        L.orc_checksum_peso.argtypes = [u8p, ctypes.c_uint32, u8p, u8p, ctypes.c_uint8]
        L.orc_checksum_peso.restype = ctypes.c_uint16
        L.orc_ipv4_pair.argtypes = [u8p, ctypes.c_uint32, u8p, u8p, u8p]
        L.orc_ipv4_pair.restype = None
        L.orc_batch_segments.argtypes = [u8p, u8p, ctypes.c_uint32, u8p, ctypes.c_int, ctypes.c_int]
        L.orc_batch_peso.argtypes = [u8p, u8p, ctypes.c_uint32, u8p, ctypes.c_int]
        L.orc_batch_ipv4.argtypes = [u8p, u8p, ctypes.c_uint32, u8p, u8p, ctypes.c_int]
        for f in ("orc_batch_segments", "orc_batch_peso", "orc_batch_ipv4"):
            getattr(L, f).restype = None
        L.orc_ipv4_tx_fill.argtypes = [u8p, ctypes.c_uint32]
        L.orc_ipv4_tx_fill.restype = ctypes.c_uint8
        L.orc_ipv4_rx_verify.argtypes = [u8p, ctypes.c_uint32, u8p]
        L.orc_ipv4_rx_verify.restype = ctypes.c_int8
        L.orc_batch_ipv4_tx_fill.argtypes = [u8p, u8p, ctypes.c_uint32, u8p, ctypes.c_int]
        L.orc_batch_ipv4_tx_fill.restype = None
        L.orc_batch_ipv4_rx_verify.argtypes = [u8p, u8p, ctypes.c_uint32, u8p, u8p, ctypes.c_int]
        L.orc_batch_ipv4_rx_verify.restype = None
        L.orc_synth_fill.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.orc_synth_fill.restype = None
        L.orc_time_peso.argtypes = [ctypes.c_void_p, u8p, u8p, ctypes.c_uint32, ctypes.c_int,
                                    ctypes.c_double, ctypes.POINTER(ctypes.c_uint64)]
        L.orc_time_peso.restype = ctypes.c_double
        L.orc_time_peso_rates.argtypes = [ctypes.c_void_p, u8p, u8p, ctypes.c_uint32, ctypes.c_int,
                                          ctypes.c_double, ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.POINTER(ctypes.c_double)]
        L.orc_time_peso_rates.restype = ctypes.c_double
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def _u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data.view(np.uint8).reshape(-1))
    return np.frombuffer(bytes(data), dtype=np.uint8).copy()


def checksum16(offset: int, data, length: int, pre_sum: int, complement: int) -> int:
    """tools.c:24-54."""
    a = _u8(data)
    assert length <= a.size
    return lib().orc_checksum16(offset, _ptr(a) if a.size else None, length, pre_sum & 0xFFFFFFFF,
                                complement)


def pieces_checksum16(pieces, length: int, pre_sum: int, complement: int) -> int:
    """pktbuf.c:646-670 over a list of byte pieces starting at the cursor."""
    arrs = [_u8(p) for p in pieces]
    class _P(ctypes.Structure):
        _fields_ = [("data", ctypes.c_void_p), ("size", ctypes.c_int)]

    arr = (_P * max(1, len(arrs)))()
    for i, a in enumerate(arrs):
        arr[i].data = _ptr(a) if a.size else None
        arr[i].size = a.size
    return lib().orc_pieces_checksum16(ctypes.addressof(arr), len(arrs), length, pre_sum, complement)


def flat_checksum16(data, pre_sum: int, complement: int) -> int:
    a = _u8(data)
    return lib().orc_flat_checksum16(_ptr(a) if a.size else None, a.size, pre_sum, complement)


def pseudo_sum(src, dst, protocol: int, length: int) -> int:
    s, d = _u8(src), _u8(dst)
    return lib().orc_pseudo_sum(_ptr(s), _ptr(d), protocol, length)


def checksum_peso(data, dest, src, protocol: int) -> int:
    """tools.c:56-75 over a contiguous L4 segment."""
    a, d, s = _u8(data), _u8(dest), _u8(src)
    return lib().orc_checksum_peso(_ptr(a) if a.size else None, a.size, _ptr(d), _ptr(s), protocol)


def ipv4_pair(pkt, frame_len: int | None = None):
    a = _u8(pkt)
    n = a.size if frame_len is None else frame_len
    ip = ctypes.c_uint16()
    l4 = ctypes.c_uint16()
    fl = ctypes.c_uint8()
    lib().orc_ipv4_pair(_ptr(a) if a.size else None, n, ctypes.addressof(ip), ctypes.addressof(l4),
                        ctypes.addressof(fl))
    return ip.value, l4.value, fl.value


def batch_segments(arena: np.ndarray, segs: np.ndarray, complement: int, nthreads: int = 8) -> np.ndarray:
    assert segs.dtype == SEG_DTYPE
    out = np.zeros(segs.size, np.uint16)
    lib().orc_batch_segments(_ptr(arena), _ptr(segs), segs.size, _ptr(out), complement, nthreads)
    return out


def batch_peso(arena: np.ndarray, segs: np.ndarray, nthreads: int = 8) -> np.ndarray:
    assert segs.dtype == PESO_DTYPE
    out = np.zeros(segs.size, np.uint16)
    lib().orc_batch_peso(_ptr(arena), _ptr(segs), segs.size, _ptr(out), nthreads)
    return out


def batch_ipv4(arena: np.ndarray, pkts: np.ndarray, nthreads: int = 8):
    assert pkts.dtype == PKT_DTYPE
    out = np.zeros(pkts.size, np.uint32)
    flags = np.zeros(pkts.size, np.uint8)
    lib().orc_batch_ipv4(_ptr(arena), _ptr(pkts), pkts.size, _ptr(out), _ptr(flags), nthreads)
    return out, flags


def batch_ipv4_tx_fill(arena: np.ndarray, pkts: np.ndarray, nthreads: int = 8) -> np.ndarray:
    """Fill the checksum fields in place (arena is modified); returns flags."""
    assert pkts.dtype == PKT_DTYPE and arena.flags["C_CONTIGUOUS"]
    flags = np.zeros(pkts.size, np.uint8)
    lib().orc_batch_ipv4_tx_fill(_ptr(arena), _ptr(pkts), pkts.size, _ptr(flags), nthreads)
    return flags


def batch_ipv4_rx_verify(arena: np.ndarray, pkts: np.ndarray, nthreads: int = 8):
    """(verdict int8 net_err_t, flags) per packet."""
    assert pkts.dtype == PKT_DTYPE
    verdict = np.zeros(pkts.size, np.int8)
    flags = np.zeros(pkts.size, np.uint8)
    lib().orc_batch_ipv4_rx_verify(_ptr(arena), _ptr(pkts), pkts.size, _ptr(verdict), _ptr(flags), nthreads)
    return verdict, flags


def synth_fill(byte_offset: int, nbytes: int, seed: int) -> np.ndarray:
    out = np.empty(nbytes, np.uint8)
    lib().orc_synth_fill(_ptr(out), byte_offset, nbytes, seed)
    return out


def time_peso(arena: np.ndarray, segs: np.ndarray, nthreads: int, min_seconds: float,
              kind: str = "reference", thread_rates: bool = False):
    """Bytes/s of a checksum_peso-shaped CPU routine over the batch.

    kind "reference" times the reference's own checksum_peso
    (oracle/_ref/libtcpref.so, built from /root/reference at the reference's
    -O2; "reference_o3": the same sources at -O3 -march=x86-64-v3) and raises
    FileNotFoundError when it was not built; kind "port" times this
    restatement.  Returns (bytes_per_second, kind, checksum_of_checksums),
    and with thread_rates=True a fourth item: each thread's own bytes/s.
    """
    L = lib()
    if kind in ("reference", "reference_o3"):
        path = REF_LIB_PATH if kind == "reference" else REF_O3_LIB_PATH
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} (the reference's checksum_peso) is not built: "
                                    "make -C oracle ref in the build container")
        ref = ctypes.CDLL(path)
        fn = ctypes.cast(ref.tcpref_peso, ctypes.c_void_p).value
    elif kind == "port":
        fn = ctypes.cast(L.orc_checksum_peso, ctypes.c_void_p).value
    else:
        raise ValueError(kind)
    cs = ctypes.c_uint64()
    per = (ctypes.c_double * max(1, min(256, nthreads)))()
    rate = L.orc_time_peso_rates(fn, _ptr(arena), _ptr(segs), segs.size, nthreads, min_seconds,
                                 ctypes.byref(cs), per)
    if thread_rates:
        return rate, kind, cs.value, list(per)[: max(1, min(256, nthreads))]
    return rate, kind, cs.value
