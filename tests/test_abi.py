"""CPU-side checks of the C ABI: the library builds, loads, and exports exactly
what include/*.h declares.  No compute call is made here (no GPU)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = ["tcsum.h", "tcsum_legacy.h", "tcsum_debug.h"]  # libtcsum.so
BENCH_HEADERS = ["tcsum_synth.h"]  # libtcsum_bench.so


@pytest.fixture(scope="module")
def libpath():
    from tcp_amd import build
    return build.build()


def declared_functions(headers=HEADERS):
    names = set()
    for h in headers:
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(\w+)\s*\([^;{]*\)\s*;", text, flags=re.M):
            if not m.group(0).lstrip().startswith(("typedef", "#")):
                names.add(m.group(1))
    return names


def test_headers_declare_the_drop_in_trio():
    names = declared_functions()
    assert {"checksum16", "checksum_peso", "pktbuf_checksum16"} <= names
    assert {"tcsum_batch_segments", "tcsum_batch_peso", "tcsum_batch_ipv4", "tcsum_host_batch_peso",
            "tcsum_plat_init", "tcsum_host_alloc", "tcsum_host_free", "tcsum_debug_set"} <= names
    assert {"tcsum_synth_fill", "tcsum_synth_ipv4", "tcsum_probe_read"} <= declared_functions(BENCH_HEADERS)


def _exports(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_every_declared_symbol_is_exported(libpath):
    """Each library exports exactly what its headers declare (export maps)."""
    from tcp_amd import _lib
    assert _exports(libpath) == declared_functions()
    assert _exports(_lib.BENCH_LIB_PATH) == declared_functions(BENCH_HEADERS)


def test_binding_table_matches_headers(libpath):
    from tcp_amd import _lib
    assert set(_lib.SIGNATURES) == declared_functions()
    assert set(_lib.BENCH_SIGNATURES) == declared_functions(BENCH_HEADERS)
    L = _lib.lib()  # loads libamdhip64 too; no device is touched
    for name in _lib.SIGNATURES:
        assert getattr(L, name)
    B = _lib.bench_lib()
    for name in _lib.BENCH_SIGNATURES:
        assert getattr(B, name)


LLVM = "/opt/rocm/lib/llvm/bin"


def code_object_kernels(path):
    """Demangled names of the gfx950 kernels in a library's code object."""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        fat, dev = os.path.join(d, "fat.bin"), os.path.join(d, "dev.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fat], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], check=True)
        syms = subprocess.run([f"{LLVM}/llvm-readelf", "--symbols", dev], capture_output=True, text=True,
                              check=True).stdout
    names = {ln.split()[-1] for ln in syms.splitlines() if ln.split() and ln.split()[-1].endswith(".kd")}
    out = subprocess.run(["c++filt"], input="\n".join(sorted(names)), capture_output=True, text=True).stdout
    return {n.replace(" [clone .kd]", "") for n in out.splitlines() if n}


@pytest.mark.skipif(not os.path.exists(f"{LLVM}/clang-offload-bundler"), reason="no ROCm llvm tools")
def test_product_code_object_holds_only_product_kernels(libpath):
    """libtcsum.so's code object: the kernels its router launches, the two
    resident servers and the drop-in one-shots -- no load probes, no
    synthetic-data kernels, no measurement-only shapes."""
    from tcp_amd import _lib
    prod = code_object_kernels(libpath)
    families = ("tcsum::k_segments<", "tcsum::k_segments_wg<", "tcsum::k_segments_wgx<16, 32, 4,",
                "tcsum::k_segments_pk<", "tcsum::k_ipv4<", "tcsum::k_tx_scatter<", "tcsum::k_server<",
                "tcsum::k_call(", "tcsum::k_inline16<", "tcsum::k_once<")
    # (a `true` template argument marks a measurement-only shape, except the
    # scatter's warming loads)
    stray = [k for k in prod if not any(f in k for f in families) or ("true>" in k and "k_tx_scatter<true>" not in k)]
    assert not stray, stray
    assert not any("k_probe" in k or "k_synth" in k or "k_segments_p<" in k or "k_segments_pp<" in k for k in prod)
    # the byte-window stream lost to k_ipv4 (profiles/r04/README.md) and is not
    # routed: measurement code, in libtcsum_bench.so only
    assert not any("k_flat_" in k for k in prod)
    bench = code_object_kernels(_lib.BENCH_LIB_PATH)
    assert any("k_probe_read" in k for k in bench) and any("k_synth_fill" in k for k in bench)
    assert any("k_flat_ipv4<2, 4, 3, 0>" in k for k in bench)  # every mode of tcsum_flat_ipv4


def test_environment_does_not_route(libpath):
    """Round 1-3's TCSUM_G / TCSUM_U / TCSUM_PACKED ... environment overrides
    are gone: a child process with them set gets the router's own choice."""
    code = ("import tcp_amd as tc; r = tc.route(1500); "
            "assert (r['lanes'], r['loads'], r['packed']) == (16, 6, 8), r; print('ok')")
    env = dict(os.environ, TCSUM_G="4", TCSUM_U="1", TCSUM_PACKED="0", TCSUM_XCD="1", TCSUM_P="2")
    r = subprocess.run([os.sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr


def test_product_reads_only_deployment_variables(libpath):
    """The only environment names in libtcsum.so are the two deployment
    choices a drop-in stack cannot make in code (device, call server); every
    tuning and route is a debug knob (include/tcsum_debug.h)."""
    import re
    names = set(re.findall(rb"TCSUM_[A-Z_0-9]+", open(libpath, "rb").read()))
    assert names <= {b"TCSUM_DEVICE", b"TCSUM_CALL_SERVER"}, names


def test_shuffled_route(libpath):
    """What a SHUFFLED batch (or a host chunk out of offset order) takes: the
    packed kernel, whose range-by-range path reads its descriptors with
    scalar loads, for K <= 8 ranges per workgroup (means from ~1.5 KiB), the
    per-range kernel for shorter ranges and whenever that path is off."""
    import tcp_amd as tc
    assert tc.route(1500)["shuffled_packed"] == 8 and tc.route(4000)["shuffled_packed"] == 3
    assert tc.route(576)["packed"] == 21 and tc.route(576)["shuffled_packed"] == 0
    assert tc.route(65536)["shuffled_packed"] == 0  # no packed kernel at all (TSO shape)
    with tc.debug(pk_early=0):
        assert tc.route(1500)["packed"] == 8 and tc.route(1500)["shuffled_packed"] == 0
    with tc.debug(packed=1):  # "packed" = 1 keeps the stream kernel for every SHUFFLED batch
        assert tc.route(576)["shuffled_packed"] == 21


def test_debug_knobs(libpath):
    import tcp_amd as tc
    assert tc.debug_get("lanes") == -1 and tc.debug_get("no_such_knob") == -2
    with tc.debug(lanes=32, loads=6):
        assert tc.route(1500)["lanes"] == 32 and tc.route(1500)["packed"] == 0
    assert tc.route(1500)["lanes"] == 16 and tc.debug_get("lanes") == -1
    from tcp_amd import _lib
    assert _lib.lib().tcsum_debug_set(b"no_such_knob", 1) == _lib.ERR_PARAM
    # read-only: no system failure yet in this process, and not settable
    assert tc.debug_get("last_sys_error") == 0
    assert _lib.lib().tcsum_debug_set(b"last_sys_error", 1) == _lib.ERR_PARAM


def test_capture_helper_is_a_library_of_its_own(libpath):
    """tcsum_pcap.h (capture files, not the checksum path) is exported by
    libtcsum_pcap.so, which has no GPU code, and not by the product library."""
    from tcp_amd import _lib
    names = declared_functions(["tcsum_pcap.h"])
    assert names == set(_lib.PCAP_SIGNATURES) == {"tcsum_pcap_index"}
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.PCAP_LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert names <= {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    prod = subprocess.run(["nm", "-D", "--defined-only", libpath], capture_output=True, text=True,
                          check=True).stdout
    assert "tcsum_pcap_index" not in prod
    deps = subprocess.run(["ldd", _lib.PCAP_LIB_PATH], capture_output=True, text=True).stdout
    assert "amdhip" not in deps and "libtcsum.so" not in deps
    assert getattr(_lib.pcap_lib(), "tcsum_pcap_index")


def test_descriptor_layouts():
    from tcp_amd import PESO_DTYPE, PKT_DTYPE, SEG_DTYPE
    from oracle import pyoracle
    assert SEG_DTYPE.itemsize == 16 and PESO_DTYPE.itemsize == 24 and PKT_DTYPE.itemsize == 16
    assert SEG_DTYPE == pyoracle.SEG_DTYPE and PESO_DTYPE == pyoracle.PESO_DTYPE
    assert PKT_DTYPE == pyoracle.PKT_DTYPE
    assert PESO_DTYPE.fields["protocol"][1] == 20


def test_pktbuf_mirror_layout():
    """tcsum_legacy.h restates net/net/pktbuf.h:15-41 (LP64)."""
    from tcp_amd.pktbuf import IpAddr, List, Node, PktBlk, PktBufStruct
    assert ctypes.sizeof(Node) == 16 and ctypes.sizeof(List) == 24
    assert PktBlk.size.offset == 16 and PktBlk.data.offset == 24 and PktBlk.payload.offset == 32
    assert PktBufStruct.blk_list.offset == 8 and PktBufStruct.ref.offset == 32
    assert PktBufStruct.pos.offset == 56 and PktBufStruct.curr_blk.offset == 64
    assert PktBufStruct.blk_offset.offset == 72 and ctypes.sizeof(PktBufStruct) == 80
    assert ctypes.sizeof(IpAddr) == 8


def test_pktbuf_cursor_walk_on_host():
    """The Python chain builder places the cursor the way pktbuf_seek does."""
    from tcp_amd import PktBuf
    b = PktBuf([b"abc", b"", b"defgh", b"i" * 200])
    assert b.s.total_size == 208
    assert b.cursor() == (0, 0, 0)
    b.seek(3)
    assert b.cursor() == (3, 1, 0)  # move_forward steps one block at a boundary
    b.seek(9)
    assert b.cursor() == (9, 3, 1)
    b.seek(2)
    assert b.cursor() == (2, 0, 2)


def test_geometry_choice(libpath):
    from tcp_amd import pick_geometry
    assert pick_geometry(1500) == (16, 6)
    assert pick_geometry(4500) == (32, 6)
    assert pick_geometry(40000) == (256, 16)
    assert pick_geometry(65536) == (1024, 4)
    assert pick_geometry(64) == (4, 1)
    shapes = {(4, 1), (4, 2), (8, 4), (16, 3), (16, 4), (16, 6), (16, 8), (32, 6), (256, 16), (1024, 4)}
    for n in range(0, 70000, 37):  # every choice is an instantiated kernel
        assert pick_geometry(n) in shapes


def test_ipv4_route_table(libpath):
    """k_ipv4's lane groups by mean packet length (csum_launch.h
    ipv4_short_shape; profiles/r06/ab21-ab25): narrow groups for short
    packets, configs[3]'s 32 x 6 (rx 16 x 6) untouched.  No device needed."""
    from tcp_amd import ipv4_route
    sums = {40: (2, 4), 64: (2, 4), 100: (4, 4), 200: (4, 4), 300: (8, 4), 600: (8, 6), 1000: (8, 3), 1500: (16, 4), 2000: (16, 3),
            3000: (16, 6), 4535: (32, 6), 9000: (32, 6)}
    rx = {40: (2, 4), 100: (2, 4), 200: (4, 4), 300: (4, 4), 600: (8, 6), 1000: (8, 3), 1500: (8, 3), 2000: (16, 3), 3000: (16, 6),
          4535: (16, 6), 9000: (16, 6)}
    for mean, want in sums.items():
        for mode in (0, 1, 3):  # sums, tx fill, tx offload
            assert ipv4_route(mean, mode) == want, (mean, mode)
    for mean, want in rx.items():
        assert ipv4_route(mean, 2) == want, mean
    shapes = {(2, 4), (4, 4), (8, 3), (8, 4), (8, 6), (16, 1), (16, 2), (16, 3), (16, 4), (16, 6), (16, 8), (32, 6),
              (64, 4), (64, 16)}
    for mean in range(0, 70000, 37):  # every routed shape is an instantiated k_ipv4
        for mode in range(4):
            assert ipv4_route(mean, mode) in shapes, (mean, mode)


def test_device_count_without_gpu(libpath):
    from tcp_amd import device_count
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    assert device_count() == 0


def test_product_never_imports_oracle():
    """The shipped path must not route through the checker."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "tcp_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                text = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"(from|import)\s+oracle|pyoracle|liboracle|libtcpref|orc_\w+\(", text), f


def test_batch_argument_errors_without_device(libpath):
    """Bad arguments come back as NET_ERR_PARAM before any device is touched."""
    from tcp_amd import _lib
    L = _lib.lib()
    assert L.tcsum_batch_peso(None, None, 4, None, 0, None) == _lib.ERR_PARAM
    assert L.tcsum_batch_segments(None, None, 4, None, 1, 0, None) == _lib.ERR_PARAM
    assert L.tcsum_batch_ipv4(None, None, 4, None, None, 0, None) == _lib.ERR_PARAM
    assert L.tcsum_batch_ipv4_tx_fill(None, None, 4, None, None, 0, None) == _lib.ERR_PARAM
    assert L.tcsum_batch_ipv4_tx_fill_scratch(ctypes.c_void_p(64), ctypes.c_void_p(64), 4, None, None,
                                              ctypes.c_void_p(64), 31, 0, None) == _lib.ERR_PARAM  # < 8 * n
    assert L.tcsum_batch_ipv4_tx_fill_scratch(ctypes.c_void_p(64), ctypes.c_void_p(64), 4, None, None,
                                              ctypes.c_void_p(66), 64, 0, None) == _lib.ERR_PARAM  # misaligned
    assert L.tcsum_batch_ipv4_rx_verify(None, None, 4, None, None, None, 0, None) == _lib.ERR_PARAM
    assert L.tcsum_batch_peso(None, None, 0, None, 0, None) == _lib.OK  # empty batch
    from tcp_amd.csum import Hint
    h = Hint(1500 * 4, 1, 0)
    v = ctypes.c_void_p(64)
    assert L.tcsum_batch(99, v, v, 4, v, None, None, ctypes.byref(h), None) == _lib.ERR_PARAM  # no such op
    assert L.tcsum_batch(2, v, v, 4, v, None, None, ctypes.byref(Hint(0, 7, 0)), None) == _lib.ERR_PARAM  # layout
    assert L.tcsum_batch(2, v, v, 4, v, None, None, ctypes.byref(Hint(0, 1, 5)), None) == _lib.ERR_PARAM  # rsv != 0
    assert L.tcsum_batch(2, v, v, 4, None, None, None, ctypes.byref(h), None) == _lib.ERR_PARAM  # no out
    assert L.tcsum_batch(6, v, v, 4, v, None, None, ctypes.byref(h), None) == _lib.ERR_PARAM  # rx: no verdict
    assert L.tcsum_batch(2, v, v, 0, None, None, None, None, None) == _lib.OK
    assert _lib.bench_lib().tcsum_synth_fill(ctypes.c_void_p(8), 16, 0, 1, None) == _lib.ERR_PARAM  # misaligned
    from tcp_amd import PESO_DTYPE
    seg = np.zeros(1, PESO_DTYPE)
    seg["offset"], seg["len"] = 10, 100
    host = np.zeros(64, np.uint8)
    out = np.zeros(1, np.uint16)
    rc = L.tcsum_host_batch_peso(0, host.ctypes.data, host.nbytes, seg.ctypes.data, 1, out.ctypes.data)
    assert rc == _lib.ERR_PARAM  # segment past the arena
    from tcp_amd import PKT_DTYPE
    pk = np.zeros(2, PKT_DTYPE)
    pk["offset"], pk["len"] = (0, 60), (20, 5)  # the second ends past a 64-byte arena
    out32, fl, vd = np.zeros(2, np.uint32), np.zeros(2, np.uint8), np.zeros(2, np.int8)
    a = host.ctypes.data
    assert L.tcsum_host_batch_ipv4(0, a, 64, pk.ctypes.data, 2, out32.ctypes.data, None) == _lib.ERR_PARAM
    assert L.tcsum_host_batch_ipv4_tx_fill(0, a, 64, pk.ctypes.data, 2, None, None) == _lib.ERR_PARAM
    assert L.tcsum_host_batch_ipv4_rx_verify(0, a, 64, pk.ctypes.data, 2, vd.ctypes.data, None,
                                             None) == _lib.ERR_PARAM
    assert L.tcsum_host_batch_ipv4_rx_verify(0, a, 64, pk.ctypes.data, 1, None, None, None) == _lib.ERR_PARAM
    assert L.tcsum_host_batch_ipv4(0, a, 64, pk.ctypes.data, 1, None, fl.ctypes.data) == _lib.ERR_PARAM
    assert L.tcsum_host_batch_ipv4_tx_fill(-1, a, 64, pk.ctypes.data, 1, None, None) == _lib.ERR_PARAM
    assert L.tcsum_host_batch_ipv4_tx_fill(0, a, 64, pk.ctypes.data, 0, None, None) == _lib.OK
    assert (host == 0).all()  # nothing touched
    assert L.tcsum_plat_init(99) == _lib.ERR_PARAM


def test_no_cpu_fallback(libpath):
    """Without a gfx950 device the drop-in symbols fail loudly (message + abort),
    and the batch/host entry points return NET_ERR_NOT_SUPPORT."""
    import sys
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    code = ("import sys; sys.path.insert(0, %r); import tcp_amd; "
            "print(tcp_amd.checksum16(0, b'\\xff\\xff', 2, 0, 1))" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "no CPU fallback" in r.stderr
    from tcp_amd import _lib, PESO_DTYPE
    L = _lib.lib()
    seg = np.zeros(1, PESO_DTYPE)
    seg["len"] = 10
    host = np.zeros(64, np.uint8)
    out = np.zeros(1, np.uint16)
    rc = L.tcsum_host_batch_peso(0, host.ctypes.data, host.nbytes, seg.ctypes.data, 1, out.ctypes.data)
    assert rc == _lib.ERR_NOT_SUPPORT
    assert L.tcsum_plat_init(0) == _lib.ERR_NOT_SUPPORT


def test_tx_apply_reproduces_the_reference_fill(libpath):
    """tcsum_tx_apply (the host half of the tx offload) stores exactly what the
    reference's tx path stores: the values are read back from the reference's
    filled frames (ipv4_tx_out.bin), the flags are the fixture's, and applying
    them to the unfilled frames must give the filled pool byte for byte --
    which fields are written, where, and for which packets not at all."""
    import golden_io as G
    from tcp_amd import PKT_DTYPE, tx_apply_batch
    from tcp_amd import _lib
    cases, pin, pout = G.ipv4_tx_cases()
    pk = G.pkt_descs(cases, PKT_DTYPE)
    off = pk["offset"].astype(np.int64)
    ln = pk["len"].astype(np.int64)
    ihl4 = np.where(ln >= 20, (pout[np.minimum(off, pout.size - 1)] & 0xF).astype(np.int64) * 4, 0)
    proto = pout[np.minimum(off + 9, pout.size - 1)]
    fld = np.select([proto == 6, proto == 17, proto == 1], [16, 6, 2], 0)

    def u16(pos):
        pos = np.clip(pos, 0, pout.size - 2)
        return pout[pos].astype(np.uint32) | (pout[pos + 1].astype(np.uint32) << 8)

    csums = u16(off + 10) | (u16(off + ihl4 + fld) << 16)
    host = pin.copy()
    tx_apply_batch(host, pk, csums, cases["flags"].astype(np.uint8))
    np.testing.assert_array_equal(host[: pout.size], pout)
    L = _lib.lib()
    assert L.tcsum_tx_apply(None, 20, 0, 0) == _lib.ERR_PARAM
    assert L.tcsum_batch_ipv4_tx_offload(None, None, 4, None, None, 0, None) == _lib.ERR_PARAM
    assert L.tcsum_batch_ipv4_tx_offload(None, None, 0, None, None, 0, None) == _lib.OK
    bad = np.zeros(1, PKT_DTYPE)
    bad["offset"], bad["len"] = host.size - 4, 20  # past the arena: nothing is touched
    before = host.copy()
    rc = L.tcsum_tx_apply_batch(host.ctypes.data, host.nbytes, bad.ctypes.data, 1,
                                np.zeros(1, np.uint32).ctypes.data, np.zeros(1, np.uint8).ctypes.data)
    assert rc == _lib.ERR_PARAM and (host == before).all()


def test_host_pool_concurrent_span_passes(libpath):
    """The host worker pool behind the host batches' parallel passes: eight
    callers at once (the *_multi shape), each a host-queue batch of 1M
    descriptors whose parallel pass finds the bad last one -- every call
    returns NET_ERR_PARAM, before any device is touched, with no hang or
    lost task."""
    import threading
    from tcp_amd import _lib
    L = _lib.lib()
    n = 1 << 20
    pk = np.zeros(n, dtype=np.dtype([("offset", "<u8"), ("len", "<u4"), ("rsv", "<u4")]))
    pk["offset"] = np.arange(n, dtype=np.uint64) * 16
    pk["len"] = 16
    pk["offset"][-1] = n * 16  # one packet past the arena
    arena = np.zeros(n * 16, np.uint8)
    out = np.zeros(n, np.uint32)
    rcs = []

    def caller():
        for _ in range(20):
            rcs.append(L.tcsum_host_batch_ipv4(0, arena.ctypes.data, arena.size, pk.ctypes.data, n,
                                               out.ctypes.data, None))

    th = [threading.Thread(target=caller) for _ in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th)
    assert rcs == [_lib.ERR_PARAM] * 160
