// csum_device.h -- the gfx950 device code both libraries compile: arithmetic
// helpers and the checksum kernels as templates.  libtcsum.so (csum_kernels.hip)
// instantiates the shapes its router can pick; libtcsum_bench.so
// (bench_kernels.hip) instantiates the load-only PROBE forms for measurement.
// Included by exactly one translation unit of each library.
//
// csum_kernels.hip -- gfx950 kernels for the Internet checksum (RFC 1071 sum as
// the wj9806/tcp stack computes it: net/src/tools.c:24-75, pktbuf.c:646-670).
//
// Arithmetic.  The reference adds the range as little-endian u16 words into a
// u32 and folds with end-around carry.  For a range of bytes b[0..n) whose
// byte parity starts at 0 that is
//     S = pre + sum_i b[i] * 256^(i & 1),   fold(S) = S == 0 ? 0 : 1 + (S-1) % 0xFFFF.
// 65536 == 1 (mod 0xFFFF), so any regrouping of the words gives the same
// fold, and folding never turns a non-zero sum into zero.  The kernels
//   * read the range as 16-byte-aligned chunks (global_load_dwordx4; an
//     aligned chunk never crosses a page, so touching a chunk's bytes outside
//     the range is safe and they are masked to zero),
//   * add each dword's two halves with one v_dot2_u32_u16 (d . {1,1} + acc),
//   * keep a u32 per lane, folded once per pass (never exact-overflows),
//   * reduce the G lanes that share a packet with DPP-free xor shuffles,
//   * and let the packet's first lane fold, rotate and complement.
// Address parity vs logical parity: the loads weight a byte by the parity of
// its ADDRESS; when the range starts at an odd address every byte is in the
// other half of its word, and the folded sum is the 8-bit rotation of the
// logical one (x*256 mod 0xFFFF), so one rotate fixes it.
//
// Lane mapping.  G lanes (4..64) share one packet and each issues U 16-byte
// loads per pass before adding anything, so a wave keeps 64*U*16 bytes in
// flight (8 KiB at U=8).  64/G packets ride in one wave; 4 waves per 256-thread
// workgroup; no LDS and no barriers -- the reduction stays inside a wave.
#pragma once

#include "csum_launch.h"

#include <tuple>
#include <type_traits>

namespace tcsum {

// Launch kernel `k` and return the status of THIS launch: hipLaunchKernel's
// own return value.  `k<<<...>>>(...); return hipGetLastError();` instead
// reads the calling thread's last-error slot, which any earlier runtime call
// on that thread may have left set -- a caller's own failed call, or a
// hipStreamQuery that answered hipErrorNotReady -- and a launch that
// succeeded was then reported as failed (round 4's intermittent
// TCSUM_ERR_SYS from tcsum_host_batch_peso, profiles/history/DESIGN_rounds1-5.md §5).  The arguments
// are converted to the kernel's parameter types first, as a <<<>>> call
// would convert them.
template <typename... P, typename... A>
inline hipError_t launch(void (*k)(P...), dim3 grid, dim3 block, size_t shmem, hipStream_t stream, A... a)
{
    static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
    std::tuple<std::remove_cv_t<P>...> v{static_cast<std::remove_cv_t<P>>(a)...};
    void *args[sizeof...(P)];
    std::apply([&args](auto &...x) {
        size_t i = 0;
        ((args[i++] = static_cast<void *>(&x)), ...);
    }, v);
    return hipLaunchKernel(reinterpret_cast<const void *>(k), grid, block, args, shmem, stream);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// a.lo + a.hi + acc in one VALU op (v_dot2_u32_u16 with {1,1}).
__device__ __forceinline__ uint32_t add_halves(uint32_t acc, uint32_t d)
{
    const u16x2 one = {1, 1};
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, d), one, acc, false);
}

__device__ __forceinline__ uint32_t chunk_sum(uint32_t acc, u32x4 v)
{
    acc = add_halves(acc, v.x);
    acc = add_halves(acc, v.y);
    acc = add_halves(acc, v.z);
    return add_halves(acc, v.w);
}

// acc + d.lo * w.lo + d.hi * w.hi.  The operands are taken by value: clang
// (ROCm 7.2) miscompiles __builtin_bit_cast applied directly to an
// ext_vector element (v.y reads v.x), so never bit_cast `v.y` in place.
__device__ __forceinline__ uint32_t dot_halves(uint32_t acc, uint32_t d, uint32_t w)
{
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, d), __builtin_bit_cast(u16x2, w), acc, false);
}

// acc + w.lo * (sum of the chunk's low halves) + w.hi * (high halves), w in
// {0x00010001, 0}: adds the chunk or nothing, without a branch.
__device__ __forceinline__ uint32_t chunk_sum_w(uint32_t acc, u32x4 v, uint32_t w)
{
    acc = dot_halves(acc, v.x, w);
    acc = dot_halves(acc, v.y, w);
    acc = dot_halves(acc, v.z, w);
    return dot_halves(acc, v.w, w);
}

// Four independent accumulators, one per dword of the chunk: the dot2 ops of
// one chunk do not wait on each other (a single chain put an s_nop between
// every two of them), and the last chunk to arrive costs one dot2 latency,
// not four, in the wave's tail.
struct Acc4 {
    uint32_t x, y, z, w;
};
__device__ __forceinline__ void acc4_add(Acc4 &a, u32x4 v, uint32_t w)
{
    a.x = dot_halves(a.x, v.x, w);
    a.y = dot_halves(a.y, v.y, w);
    a.z = dot_halves(a.z, v.z, w);
    a.w = dot_halves(a.w, v.w, w);
}
__device__ __forceinline__ uint32_t acc4_total(const Acc4 &a) { return (a.x + a.y) + (a.z + a.w); }

// Keep only bytes [lo, hi) of a chunk (positions 0..16).
__device__ __forceinline__ u32x4 mask_chunk(u32x4 v, int lo, int hi);

// Bytes [a, b) of a dword (0 <= a, b <= 4); empty when b <= a.
__device__ __forceinline__ uint32_t byte_mask(int a, int b)
{
    const uint64_t hi = (1ull << (8 * b)) - 1ull;
    const uint64_t lo = (1ull << (8 * a)) - 1ull;
    return (uint32_t)(hi & ~lo);
}

__device__ __forceinline__ int clamp4(int x) { return x < 0 ? 0 : (x > 4 ? 4 : x); }

__device__ __forceinline__ u32x4 mask_chunk(u32x4 v, int lo, int hi)
{
    v.x &= byte_mask(clamp4(lo), clamp4(hi));
    v.y &= byte_mask(clamp4(lo - 4), clamp4(hi - 4));
    v.z &= byte_mask(clamp4(lo - 8), clamp4(hi - 8));
    v.w &= byte_mask(clamp4(lo - 12), clamp4(hi - 12));
    return v;
}

// Sum of the chunk's bytes [lo, hi) (positions 0..16 inside the chunk).
__device__ __forceinline__ uint32_t chunk_sum_masked(uint32_t acc, u32x4 v, int lo, int hi)
{
    acc = add_halves(acc, v.x & byte_mask(clamp4(lo), clamp4(hi)));
    acc = add_halves(acc, v.y & byte_mask(clamp4(lo - 4), clamp4(hi - 4)));
    acc = add_halves(acc, v.z & byte_mask(clamp4(lo - 8), clamp4(hi - 8)));
    return add_halves(acc, v.w & byte_mask(clamp4(lo - 12), clamp4(hi - 12)));
}

// One end-around step: keeps x == 0 iff input == 0, x mod 0xFFFF, x <= 0x1FFFE.
__device__ __forceinline__ uint32_t fold_step(uint32_t x) { return (x & 0xFFFFu) + (x >> 16); }

// tools.c:47-51 closed form.
__device__ __forceinline__ uint32_t fold16(uint32_t x)
{
    x = fold_step(x);
    x = fold_step(x);
    return fold_step(x);
}

__device__ __forceinline__ uint32_t rot8(uint32_t x) { return ((x & 0xFFu) << 8) | (x >> 8); }

__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

template <bool NT>
__device__ __forceinline__ u32x4 load16(const u32x4 *p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

// Keep every load issued so far above this point: the optimizer may neither
// sink them into a later loop (IR level: memory clobber) nor reorder their
// consumers before them (machine scheduler barrier).  Without it hipcc moved
// the first pass of data loads behind an s_waitcnt vmcnt(0) on the header /
// edge loads -- one extra full memory latency per wave.
__device__ __forceinline__ void issue_fence()
{
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// x + (x of another lane selected by a DPP control), all lanes active.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_add(uint32_t x)
{
    return x + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}

// Sum over the G lanes that share a packet, in every lane of the group.
// Inside a 16-lane DPP row the butterfly is four DPP adds (quad_perm xor1,
// xor2; row_ror 4, 8: no LDS unit, no waits); only the cross-row steps
// (G = 8's xor 4, G >= 32) go through ds_bpermute.
template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t x)
{
    x = dpp_add<0xB1>(x); // quad_perm [1,0,3,2]: lane ^ 1
    if constexpr (G >= 4)
        x = dpp_add<0x4E>(x); // quad_perm [2,3,0,1]: lane ^ 2
    if constexpr (G == 8)
        x += __shfl_xor(x, 4, 64);
    if constexpr (G >= 16) {
        x = dpp_add<0x124>(x); // row_ror:4 -- quad sums of lanes i, i-4
        x = dpp_add<0x128>(x); // row_ror:8 -- + lanes i-8, i-12: the row sum
    }
    if constexpr (G >= 32)
        x += __shfl_xor(x, 16, 64);
    if constexpr (G >= 64)
        x += __shfl_xor(x, 32, 64);
    return x;
}

// XCD-grouped block order.  The dispatcher hands consecutive workgroups to
// the 8 XCDs round-robin (MI355X_MICROARCH.md, workgroup dispatch), so with the
// identity map the results of neighbouring packets -- one 128-byte line of
// `out` -- are written by 4..16 workgroups on different XCDs, each L2 writing
// its own partial copy of the line back to HBM, and the 16-byte chunk two
// packed packets share is fetched by two L2s.  Remapped, every run of `xg`
// consecutive logical blocks sits on one XCD (hardware blocks b, b+8, ...),
// while the set of blocks in flight -- the HBM window the chip streams
// through -- stays the same.  Bijective: a last, incomplete group of 8*xg
// blocks keeps the identity map.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb, uint32_t xg)
{
    if (xg <= 1)
        return b;
    const uint32_t sg = 8u * xg;
    if (b >= nb - nb % sg)
        return b;
    const uint32_t r = b % sg;
    return b - r + (r & 7u) * xg + (r >> 3);
}

// Descriptor prefetch (k_segments_pk's range-by-range path: aux >> 8, the
// distance pfd in logical workgroups, 0 = off).  A workgroup's data loads wait on its descriptors,
// and those come from HBM: one memory latency per workgroup with nothing of
// its own in flight.  Lanes 0-1 of wave 0 touch the descriptor lines of the
// workgroup pfd logical blocks ahead (a multiple of the XCD run's superblock
// lands on this XCD, about one workgroup lifetime later), so that its
// descriptor loads hit this XCD's L2.  The loaded word is consumed at the
// very end (an impossible store), so the compiler keeps the load and no wave
// waits for it earlier.  `lines`: the descriptor bytes one workgroup reads.
__device__ __forceinline__ uint32_t prefetch_descs(const void *__restrict__ descs, uint64_t first_ahead,
                                                   uint64_t ndesc, uint32_t dsz, uint32_t lines, uint32_t lane)
{
    if (first_ahead >= ndesc || lane >= lines)
        return 0u;
    const uint64_t last = dsz * (ndesc - 1u);
    uint64_t o = dsz * first_ahead + 128u * lane;
    o = (o < last ? o : last) & ~uint64_t(3);
    return *reinterpret_cast<const uint32_t *>(static_cast<const uint8_t *>(descs) + o);
}

// ---------------------------------------------------------------- segments
//
// One descriptor per range.  MODE_SEG: pktbuf_checksum16 (u16 pre_sum);
// MODE_EXACT: checksum16 (u32 pre_sum, u32 wrap, len <= 65535);
// MODE_PESO: checksum_peso with the pseudo-header built here (tools.c:58-70).

struct SegDesc {
    uint64_t off;
    uint32_t len, pre, src, dst, proto;
};

// Unconditional: a dead lane (seg >= n) reads descriptor 0 and gets len 0, so
// no load sits behind a branch.
template <int MODE>
__device__ __forceinline__ SegDesc load_desc(const void *__restrict__ descs, uint32_t seg, bool live)
{
    SegDesc d;
    const uint32_t i = live ? seg : 0u;
    if constexpr (MODE == MODE_PESO) {
        // 24 B = 16 + 8: two loads (the array is 8-byte aligned)
        const uint8_t *x = static_cast<const uint8_t *>(descs) + 24ull * i;
        const u32x4 a = *reinterpret_cast<const u32x4 *>(x);
        const uint2 b = *reinterpret_cast<const uint2 *>(x + 16);
        d.off = (uint64_t)a.x | ((uint64_t)a.y << 32);
        d.len = a.z;
        d.src = a.w;
        d.dst = b.x;
        d.proto = b.y & 0xFFu;
        d.pre = 0;
    } else {
        const u32x4 a = *(reinterpret_cast<const u32x4 *>(descs) + i);
        d.off = (uint64_t)a.x | ((uint64_t)a.y << 32);
        d.len = a.z;
        d.pre = a.w;
        d.src = d.dst = d.proto = 0;
    }
    d.len = live ? d.len : 0u;
    return d;
}

// A valid, 16-byte aligned chunk of zeros in the code object: lanes with no
// bytes to read load from here, so every load is unconditional (no branch
// around a load -> the compiler can count vmcnt exactly instead of vmcnt(0)).
__device__ u32x4 g_zero_chunk = {0u, 0u, 0u, 0u};

// One range's loads in flight for this lane (G lanes per range).  Lane 0
// takes the first chunk and lane 1 the last, masked; the interior chunks
// [1, nch-1) are whole, so the unrolled loop has no divergent branch: lanes
// past the end re-read the last interior chunk (same lines as a live lane,
// merged) and add it with weight 0.
template <int U>
struct Frame {
    const u32x4 *ibase;
    uint64_t e; // range end in bytes from the first chunk
    uint32_t s0, ni, ilast, eidx;
    bool has_edge;
    u32x4 ev;
    u32x4 v[U];
};

template <int G, int U>
__device__ __forceinline__ void frame_issue(Frame<U> &f, const uint8_t *__restrict__ arena, uint64_t off,
                                            uint32_t len, uint32_t gl)
{
    const uint8_t *p = arena + off; // derived from the kernel argument: global_load, not flat_load
    f.s0 = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 15u);
    const u32x4 *base = reinterpret_cast<const u32x4 *>(p - f.s0);
    f.e = (uint64_t)len + f.s0;
    const uint32_t nch = len ? (uint32_t)((f.e + 15) >> 4) : 0u;
    f.ni = nch > 2 ? nch - 2 : 0u;
    f.eidx = gl == 0 ? 0u : (nch ? nch - 1u : 0u);
    f.has_edge = gl < 2 && nch > 0 && (gl == 0 || nch >= 2);
    const u32x4 *ebase = nch ? base : &g_zero_chunk;
    f.ibase = f.ni ? base + 1 : &g_zero_chunk;
    f.ilast = f.ni ? f.ni - 1u : 0u;
    // the edge chunks with the DEFAULT policy, the interior nontemporal: a
    // packed range shares its first and last 128-B line with its neighbours,
    // and a line fetched by a default-policy load stays in L2 until the
    // neighbour's wave (same XCD, xcd_block) reads it -- configs[1] fetched
    // 1.2 % more than the algorithmic bytes with nt edges, 0.05 % without,
    // and ran 5 % faster (profiles/r01/ab_edge_policy.txt)
    f.ev = load16<false>(ebase + (nch ? f.eidx : 0u));
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t j = u * G + gl;
        f.v[u] = load16<true>(f.ibase + (j < f.ni ? j : f.ilast));
    }
}

template <int G, int U, bool EXACT>
__device__ __forceinline__ uint32_t frame_consume(Frame<U> &f, uint32_t gl)
{
    uint32_t acc;
    {
        const uint64_t c = 16ull * f.eidx;
        const int lo = f.has_edge && f.eidx == 0 ? (int)f.s0 : 0;
        const int hi = f.has_edge ? (int)(f.e - c < 16 ? f.e - c : 16) : 0;
        acc = chunk_sum_masked(0u, f.ev, lo, hi);
    }
    // pass 0: the loads frame_issue put in flight
    {
        Acc4 p{0u, 0u, 0u, 0u};
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc4_add(p, f.v[u], (uint32_t)(u * G) + gl < f.ni ? 0x00010001u : 0u);
        const uint32_t part = acc4_total(p); // <= 4 * 16 * 131070 < 2^23
        acc = EXACT ? acc + part : fold_step(acc + part);
    }
    // later passes load and sum inside one iteration: nothing vector-sized is
    // carried around the loop, so its registers are pass 0's (a loop-carried
    // f.v made hipcc keep two copies: 68 -> 52 VGPRs at U=6, 8 waves/SIMD)
    for (uint32_t b0 = G * U; b0 < f.ni; b0 += G * U) {
        u32x4 w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j = b0 + u * G + gl;
            w[u] = load16<true>(f.ibase + (j < f.ni ? j : f.ilast));
        }
        Acc4 p{0u, 0u, 0u, 0u};
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j = b0 + u * G + gl;
            acc4_add(p, w[u], j < f.ni ? 0x00010001u : 0u);
        }
        const uint32_t part = acc4_total(p);
        acc = EXACT ? acc + part : fold_step(acc + part);
    }
    return acc;
}

// This lane's share of the word sum of arena[off, off+len).  `issued` runs
// right after the first loads are in flight.
template <int G, int U, bool EXACT, class Issued>
__device__ __forceinline__ uint32_t sum_range(const uint8_t *__restrict__ arena, uint64_t off, uint32_t len,
                                              uint32_t gl, Issued &&issued)
{
    Frame<U> f;
    frame_issue<G, U>(f, arena, off, len, gl);
    issued();
    issue_fence();
    return frame_consume<G, U, EXACT>(f, gl);
}

// checksum_peso's pseudo-header words, folded (tools.c:58-70): src, dst,
// {0, proto}, htons((uint16_t)len).  Depends on the descriptor only, so the
// kernels compute it while the range's bytes are in flight.
__device__ __forceinline__ uint32_t peso_pseudo16(const SegDesc &d)
{
    uint32_t q = add_halves(0u, d.src);
    q = add_halves(q, d.dst);
    q += d.proto << 8;
    q += bswap16(d.len & 0xFFFFu);
    return fold16(q);
}

// Computed now, inside the load shadow: the empty asm pins the value here,
// so the compiler cannot sink the arithmetic into the tail behind the last load.
__device__ __forceinline__ uint32_t pinned(uint32_t x)
{
    asm volatile("" : "+v"(x));
    return x;
}

// The packet's first lane turns the group's sum into the reference's u16.
// MODE_PESO: q16 = peso_pseudo16(d) (ignored by the other modes).
template <int MODE>
__device__ __forceinline__ uint16_t finalize(uint32_t acc, uintptr_t start, const SegDesc &d, uint32_t aux,
                                             uint32_t q16)
{
    uint32_t r;
    if constexpr (MODE == MODE_EXACT) {
        // tools.c:27-53: u32 accumulator from pre_sum; acc is the exact word
        // sum (< 2^31 for len <= 65535).  The host stages the bytes so that
        // address parity == logical parity (aux bit 1).
        uint32_t s;
        if (((start ^ (aux >> 1)) & 1u) == 0) {
            s = d.pre + acc;
        } else { // not reached from the C ABI; mod-0xFFFF result
            const uint32_t f = rot8(fold16(acc));
            s = fold_step(f + fold16(d.pre));
        }
        s = fold16(s);
        r = (aux & 1u) ? (~s & 0xFFFFu) : s;
    } else {
        uint32_t f = fold16(acc);
        if (start & 1u)
            f = rot8(f);
        if constexpr (MODE == MODE_SEG) {
            const uint32_t t = fold_step(f + (d.pre & 0xFFFFu)); // pktbuf.c:657
            r = (aux & 1u) ? (~t & 0xFFFFu) : t;
        } else {
            r = ~fold_step(f + q16) & 0xFFFFu; // pktbuf_checksum16(..., 1), tools.c:73
        }
    }
    return (uint16_t)r;
}

// The descriptors of this wave's PER lane groups' ranges (k_segments_pk's
// range-by-range path, and the per-range kernel with aux bit 7; 64 / PER
// lanes per group), read with scalar loads -- all issued before any is used --
// and each group's own picked into x.  Ranges past kw read the workgroup's
// last descriptor (a group past kw takes no range).
template <int MODE, uint32_t PER>
__device__ __forceinline__ void pk_wave_descs(const void *__restrict__ descs, uint32_t first, uint32_t kw,
                                              uint32_t (&x)[6])
{
    constexpr uint32_t DW = MODE == MODE_PESO ? 6u : 4u; // dwords per descriptor
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t gi = (threadIdx.x & 63u) / (64u / PER);
    uint32_t sd[PER][DW];
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        const uint32_t r = wv * PER + j < kw ? wv * PER + j : kw - 1u;
        const uint32_t *q = reinterpret_cast<const uint32_t *>(descs) + (uint64_t)DW * (first + r);
#pragma unroll
        for (uint32_t i = 0; i < DW; ++i)
            sd[j][i] = q[i];
    }
    // pinned in scalar registers: otherwise the compiler folds the per-group
    // choice into one vector load from a chosen address -- the L2 round trip
    // this is here to avoid
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j)
#pragma unroll
        for (uint32_t i = 0; i < DW; ++i)
            asm volatile("" : "+s"(sd[j][i]));
#pragma unroll
    for (uint32_t i = 0; i < DW; ++i) {
        uint32_t v = sd[0][i];
#pragma unroll
        for (uint32_t j = 1; j < PER; ++j)
            v = gi == j ? sd[j][i] : v;
        x[i] = v;
    }
}

// A descriptor from the dwords pk_wave_descs picked (len 0 unless live).
template <int MODE>
__device__ __forceinline__ SegDesc desc_of(const uint32_t (&x)[6], bool live)
{
    SegDesc d{0, 0, 0, 0, 0, 0};
    d.off = (uint64_t)x[0] | ((uint64_t)x[1] << 32);
    d.len = live ? x[2] : 0u;
    if constexpr (MODE == MODE_PESO) {
        d.src = x[3];
        d.dst = x[4];
        d.proto = x[5] & 0xFFu;
    } else {
        d.pre = x[3];
    }
    return d;
}

// One wave-slice of packets per wave, one launch-wide pass.
//
// Results leave through the workgroup's LAST wave: each wave puts its packets'
// u16 into LDS and bumps an LDS counter; the wave that brings it to 4 stores
// all 256/G results with one coalesced store and the other three end at once.
// With every wave storing its own 4 results (an 8-byte partial store each) the
// headline ran 1.1 % slower -- as slow as its loads plus the stores' tail in
// every wave; with the gathered store it matches the same kernel with no
// store at all (profiles/r02/ab_store.txt).  A nontemporal store cost 4 %.
constexpr uint32_t kSegScalarDesc = 1u << 7; // aux of k_segments: descriptors by scalar loads

template <int G, int U, int MODE, int T = 256>
__global__ __launch_bounds__(T) void k_segments(const uint8_t *__restrict__ arena,
                                                const void *__restrict__ descs, uint32_t n,
                                                uint16_t *__restrict__ out, uint32_t aux, uint32_t xg)
{
    static_assert(G >= 4 && G <= 64 && (G & (G - 1)) == 0 && T >= 64 && T <= 1024 && T % 64 == 0 && T / G <= 64,
                  "G, T");
    constexpr uint32_t PER = T / G; // ranges per workgroup
    __shared__ uint16_t res[PER];
    __shared__ uint32_t arrived;
    if (threadIdx.x == 0)
        arrived = 0;
    __syncthreads();
    const uint32_t gl = threadIdx.x & (G - 1);
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x, xg);
    const uint32_t seg = blk * PER + threadIdx.x / G; // no 32-bit wrap for any n
    const bool live = seg < n;
    SegDesc d;
    if constexpr (G >= 8 && G <= 16) {
        // aux bit 7 (debug knob "seg_sdesc", on unless 0): each wave reads its
        // 4 or 8 groups' descriptors with scalar loads instead of every lane
        // loading its own: shuffled 576-B ranges 329 -> 304 us, 1,000 B 256
        // -> 249, 200 B 625 -> 606, packed 576 B 293 -> 272 (with 32 or 64
        // lanes per range, 1-2 ranges a wave: +0.5 %, not taken;
        // profiles/r05/seg_sdesc/)
        if ((aux & kSegScalarDesc) != 0u) {
            const uint32_t first = blk * PER, kw = n - first < PER ? n - first : PER;
            uint32_t x[6] = {0u, 0u, 0u, 0u, 0u, 0u};
            pk_wave_descs<MODE, 64u / G>(descs, first, kw, x);
            d = desc_of<MODE>(x, live);
        } else {
            d = load_desc<MODE>(descs, seg, live);
        }
    } else {
        d = load_desc<MODE>(descs, seg, live);
    }
    // descriptor prefetch (aux >> 8, k_segments_pk's fallback's): issued after
    // this workgroup's own descriptor load, so that load's wait is not its
    uint32_t pf = 0;
    if (const uint32_t pfd = MODE == MODE_EXACT ? 0u : aux >> 8; pfd != 0u && threadIdx.x < 64u)
        pf = prefetch_descs(descs, (uint64_t)(blk + pfd) * PER, n, MODE == MODE_PESO ? 24u : 16u,
                            (PER * (MODE == MODE_PESO ? 24u : 16u) + 127u) / 128u + 1u, threadIdx.x);
    uint32_t q16 = 0;
    uint32_t acc = sum_range<G, U, MODE == MODE_EXACT>(arena, d.off, d.len, gl, [&] {
        if constexpr (MODE == MODE_PESO)
            q16 = pinned(peso_pseudo16(d));
    });
    acc = group_sum<G>(acc);
    if (gl == 0)
        res[threadIdx.x / G] = finalize<MODE>(acc, reinterpret_cast<uintptr_t>(arena + d.off), d, aux, q16);
    uint32_t order = 0;
    if ((threadIdx.x & 63u) == 0) // release: this wave's res[] entries before the count
        order = __hip_atomic_fetch_add(&arrived, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    order = __builtin_amdgcn_readfirstlane(order);
    if (order == T / 64u - 1u) { // the last wave: every entry is in LDS
        const uint32_t l = threadIdx.x & 63u;
        const uint32_t sl = blk * PER + l;
        if (l < PER && sl < n)
            out[sl] = res[l];
    }
    asm volatile("" ::"v"(pf)); // keeps the prefetch load alive (its value is not used)
}

// One range per workgroup: all four waves on one range (G = 256), for ranges
// of tens of KiB (TSO).  Each wave's share of a 64-KiB range is one pass of
// U loads per lane -- the short-lived, one-pass shape of the fastest plain
// read (profiles/r01/probe_variants.txt) -- and the waves' sums meet in LDS.
template <int U, int MODE>
__global__ __launch_bounds__(256) void k_segments_wg(const uint8_t *__restrict__ arena,
                                                     const void *__restrict__ descs, uint32_t n,
                                                     uint16_t *__restrict__ out, uint32_t aux, uint32_t xg)
{
    __shared__ uint32_t part[4];
    const uint32_t gl = threadIdx.x;
    const uint32_t seg = xcd_block(blockIdx.x, gridDim.x, xg); // grid == n: one range per workgroup
    const bool live = seg < n;
    const SegDesc d = load_desc<MODE>(descs, seg, live);
    uint32_t q16 = 0;
    uint32_t acc = sum_range<256, U, MODE == MODE_EXACT>(arena, d.off, d.len, gl, [&] {
        if constexpr (MODE == MODE_PESO)
            q16 = pinned(peso_pseudo16(d));
    });
    acc = group_sum<64>(acc); // < 2^23 (folded lanes) or exact
    if ((gl & 63u) == 0)
        part[gl >> 6] = acc;
    __syncthreads();
    if (gl == 0 && live)
        out[seg] = finalize<MODE>(part[0] + part[1] + part[2] + part[3], reinterpret_cast<uintptr_t>(arena + d.off),
                                  d, aux, q16);
}

// One range per workgroup of W waves, with the lane -> chunk map as a
// parameter (measured against k_segments_wg for configs[2],
// scripts/env_ab.py, profiles/r03/ab_tso_shapes*.txt): GL = 0 interleaves the whole workgroup (load u of
// lane t is interior chunk u * 64W + t: each load instruction of the
// workgroup covers 64W contiguous chunks, k_segments_wg's map); GL > 0 cuts
// the range into sub-ranges of GL * U chunks, one per GL-lane group, each
// walked like one headline packet (k_segments<16, 6>: load u of lane l is
// chunk u * GL + l of its sub-range).  A pass covers 64W * U chunks; longer
// ranges take more passes.  Edges as in frame_issue: lane 0 loads the first
// chunk and lane 1 the last with the default policy, masked; every interior
// chunk is nontemporal and whole.
// PROBE: the same loads with the sums, the reduction and the store replaced
// by an XOR fold into a sink (`out`) stored on a 2^-32 fluke
// (tcsum_probe_segments for this geometry).
template <int W, int GL, int U, int MODE, bool PROBE = false>
__global__ __launch_bounds__(W * 64) void k_segments_wgx(const uint8_t *__restrict__ arena,
                                                         const void *__restrict__ descs, uint32_t n,
                                                         uint16_t *__restrict__ out, uint32_t aux, uint32_t xg)
{
    static_assert(MODE != MODE_EXACT, "the exact u32 sum stays on k_segments");
    constexpr uint32_t T = W * 64u, CPP = T * U;
    __shared__ uint32_t part[W];
    const uint32_t t = threadIdx.x;
    const uint32_t seg = xcd_block(blockIdx.x, gridDim.x, xg); // grid == n
    const bool live = seg < n;
    const SegDesc d = load_desc<MODE>(descs, seg, live);
    const uint8_t *p = arena + d.off;
    const uint32_t s0 = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 15u);
    const u32x4 *base = reinterpret_cast<const u32x4 *>(p - s0);
    const uint64_t e = (uint64_t)d.len + s0;
    const uint32_t nch = d.len ? (uint32_t)((e + 15) >> 4) : 0u;
    const uint32_t ni = nch > 2 ? nch - 2 : 0u;
    const u32x4 *ib = ni ? base + 1 : &g_zero_chunk;
    const uint32_t ilast = ni ? ni - 1u : 0u;
    const uint32_t eidx = t == 0 ? 0u : (nch ? nch - 1u : 0u);
    const bool has_edge = t < 2 && nch > 0 && (t == 0 || nch >= 2);
    const u32x4 ev = load16<false>((nch ? base : &g_zero_chunk) + (nch ? eidx : 0u));
    const uint32_t lane_off = GL ? (t / GL) * (GL * U) + (t % GL) : t;
    constexpr uint32_t ustep = GL ? GL : T;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t j = lane_off + u * ustep;
        v[u] = load16<true>(ib + (j < ni ? j : ilast));
    }
    if constexpr (PROBE) {
        issue_fence();
        u32x4 x = ev;
#pragma unroll
        for (int u = 0; u < U; ++u)
            x ^= v[u];
        for (uint32_t b0 = CPP; b0 < ni; b0 += CPP) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t j = b0 + lane_off + u * ustep;
                x ^= load16<true>(ib + (j < ni ? j : ilast));
            }
        }
        const uint32_t f = x.x ^ x.y ^ x.z ^ x.w;
        if (f == 0x9E3779B9u)
            reinterpret_cast<uint32_t *>(out)[0] = f;
        return;
    }
    uint32_t q16 = 0;
    if constexpr (MODE == MODE_PESO)
        q16 = pinned(peso_pseudo16(d));
    issue_fence();
    uint32_t acc;
    {
        const uint64_t c = 16ull * eidx;
        const int lo = has_edge && eidx == 0 ? (int)s0 : 0;
        const int hi = has_edge ? (int)(e - c < 16 ? e - c : 16) : 0;
        acc = chunk_sum_masked(0u, ev, lo, hi);
    }
    {
        Acc4 pa{0u, 0u, 0u, 0u};
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc4_add(pa, v[u], lane_off + u * ustep < ni ? 0x00010001u : 0u);
        acc = fold_step(acc + acc4_total(pa));
    }
    for (uint32_t b0 = CPP; b0 < ni; b0 += CPP) {
        u32x4 w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j = b0 + lane_off + u * ustep;
            w[u] = load16<true>(ib + (j < ni ? j : ilast));
        }
        Acc4 pa{0u, 0u, 0u, 0u};
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc4_add(pa, w[u], b0 + lane_off + u * ustep < ni ? 0x00010001u : 0u);
        acc = fold_step(acc + acc4_total(pa));
    }
    acc = group_sum<64>(acc); // < 2^23
    if ((t & 63u) == 0)
        part[t >> 6] = acc;
    __syncthreads();
    if (t == 0 && live) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < W; ++w)
            s += part[w]; // < 16 * 2^23
        out[seg] = finalize<MODE>(s, reinterpret_cast<uintptr_t>(p), d, aux, q16);
    }
}

// ---------------------------------------------------------------- packed stream
//
// Ranges laid out one after another in the arena (a batch of MTU segments
// packed back to back: offset[i+1] == offset[i] + len[i]; or with padding
// between them) are one byte stream.  k_segments_pk gives a workgroup of W
// waves K consecutive ranges and streams the region from the first range's
// first byte to the last range's end in the TSO kernel's load shape -- 32-lane
// groups each walking a contiguous sub-range, U loads per lane -- instead of
// giving every range its own lane group; a region longer than one pass
// (W * 64 * U chunks) is walked pass by pass, the next pass's loads in flight
// while the current one is combined.
//
// Per-range sums come from prefix sums.  Chunk c of the region (16-B aligned,
// address order) has the full word sum f(c); with E(c) = the sum of f over the
// chunks before c, the word sum of the region's bytes before byte x (counted
// from the first chunk) is
//     P(x) = E(x / 16) + (word sum of bytes [0, x % 16) of chunk x / 16),
// and range r's sum is P(end_r) - P(start_r): exact u32 arithmetic (a pass of
// <= 64 KiB sums to < 2^31 and P wraps mod 2^32 consistently), so bytes that
// belong to no range -- padding, the neighbouring regions' bytes in the first
// and last chunk -- cancel, and no chunk is masked.  Any layout works as long
// as every range lies inside the region: gaps, overlaps, duplicates, ranges of
// 0..16 bytes.  The address-parity weighting and the odd-start rotation are
// k_segments'.
//
// E is a scan in the load order: within a sub-range load u of lane l is chunk
// u*32 + l, so E = (sub-ranges before) + (loads u' < u of this sub-range) +
// (lanes l' < l of load u) -- a 32-lane DPP scan per load, the half-wave
// totals by readlane.  Every lane writes, per chunk, its sub-range prefix and
// the chunk itself to LDS; after one barrier, lane r of wave w (range 64w + r,
// whose descriptor it loaded while the bytes were in flight) adds the
// sub-range prefixes and the bytes before its start and end from the LDS copy
// of their chunks.  The waves place their loads from the first and last
// descriptor only (scalar loads), so the data loads wait on one descriptor
// latency, as in the per-range kernels.
//
// A workgroup whose region is longer than 64 passes, one of whose ranges lies
// outside it (a shuffled batch) or is 128 KiB or longer (its word sum could
// reach 2^32, where the u32 prefixes stop being exact), sums range by range with the widest lane
// groups that give every range one: always correct, only slower.
__device__ __forceinline__ uint32_t scan32(uint32_t x)
{
    // inclusive scan inside each 32-lane half: row_shr 1, 2, 4, 8 (16-lane
    // rows), then row_bcast:15 adds row 0's total into row 1 (and 2's into 3)
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    return x;
}

// Word sum of the chunk's bytes [0, b), b = 0..16.
__device__ __forceinline__ uint32_t chunk_prefix_sum(u32x4 v, uint32_t b)
{
    const int bits = (int)(8u * b);
    const uint32_t m0 = bits >= 32 ? ~0u : (1u << bits) - 1u;
    const uint32_t m1 = bits >= 64 ? ~0u : bits <= 32 ? 0u : (1u << (bits - 32)) - 1u;
    const uint32_t m2 = bits >= 96 ? ~0u : bits <= 64 ? 0u : (1u << (bits - 64)) - 1u;
    const uint32_t m3 = bits >= 128 ? ~0u : bits <= 96 ? 0u : (1u << (bits - 96)) - 1u;
    uint32_t acc = add_halves(0u, v.x & m0);
    acc = add_halves(acc, v.y & m1);
    acc = add_halves(acc, v.z & m2);
    return add_halves(acc, v.w & m3);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t x, uint32_t lane)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, (int)lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), (int)lane);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

constexpr uint32_t kPkWaves = 4, kPkLoads = 3; // 4 waves x 64 lanes x 3 loads x 16 B = 12 KiB per pass
constexpr uint32_t kPkMaxRanges = 64; // ranges per wave of the workgroup (lane r of wave w: range 64w + r)

// off and len of descriptor i (the same 12 bytes lead both layouts); called
// with a workgroup-uniform index, so it is a scalar load
template <int MODE>
__device__ __forceinline__ void desc_span(const void *__restrict__ descs, uint32_t i, uint64_t &off, uint32_t &len)
{
    const uint8_t *x = static_cast<const uint8_t *>(descs) + (MODE == MODE_PESO ? 24ull : 16ull) * i;
    const uint2 o = *reinterpret_cast<const uint2 *>(x);
    off = (uint64_t)o.x | ((uint64_t)o.y << 32);
    len = *reinterpret_cast<const uint32_t *>(x + 8);
}

// The per-range path for a workgroup whose ranges are not one region:
// groups of G lanes, G the widest power of two with one group per range.
// HAVE0: the lane's first range's descriptor may have been read already
// (e0, when have0: k_segments_pk's scalar reads, K <= 32).  (Loading each
// round's successor descriptor ahead, for K > 32, measured no gain:
// profiles/r05/pk_early/pk_tiny3.txt.)
template <int MODE, int G, int UL = 4, bool HAVE0 = false>
__device__ __forceinline__ void pk_ranges(const uint8_t *__restrict__ arena, const void *__restrict__ descs,
                                          uint16_t *__restrict__ out, uint32_t aux, uint32_t first, uint32_t kw,
                                          uint32_t T, const SegDesc &e0, bool have0)
{
    const uint32_t t = threadIdx.x, gl = t & (G - 1u);
    for (uint32_t r = t / G; r < kw; r += T / G) {
        const SegDesc e = HAVE0 && have0 && r == t / G ? e0 : load_desc<MODE>(descs, first + r, true);
        uint32_t q = 0;
        uint32_t acc = sum_range<G, UL, false>(arena, e.off, e.len, gl, [&] {
            if constexpr (MODE == MODE_PESO)
                q = pinned(peso_pseudo16(e));
        });
        acc = group_sum<G>(acc);
        if (gl == 0)
            out[first + r] = finalize<MODE>(acc, reinterpret_cast<uintptr_t>(arena + e.off), e, aux, q);
    }
}

constexpr uint32_t kPkMaxPasses = 64; // longer regions go range by range
constexpr uint32_t kPkEarly = 1u << 7; // aux: the range-by-range path's descriptors by scalar loads (pk_wave_descs)

// Lanes per range on k_segments_pk's range-by-range path for kw ranges.
__device__ __forceinline__ uint32_t pk_group(uint32_t T, uint32_t kw)
{
    const uint32_t lanes_per = T / kw;
    return lanes_per >= 64 ? 64u : lanes_per >= 32 ? 32u : lanes_per >= 16 || kw <= 22u ? 16u : 8u;
}

// A workgroup of k_segments_pk whose kw ranges are not one region: G lanes
// per range, G the widest power of two that gives every range a group
// (pk_group).  e0: this lane's first range's descriptor when have0.
template <int MODE>
__device__ __forceinline__ void pk_fallback(const uint8_t *__restrict__ arena, const void *__restrict__ descs,
                                            uint16_t *__restrict__ out, uint32_t aux, uint32_t first, uint32_t kw,
                                            uint32_t T, const SegDesc &e0, bool have0)
{
    // K was chosen so that K mean-length ranges fill a 12-KiB pass: a range is
    // about 12 KiB / K, and each group's pass is sized to hold one, as the
    // per-range kernel would size it (32 x 3 = 1.5 KiB at K = 8; 16 x 6 for
    // K = 9..11, 16 x 4 = 1 KiB for 12..16, 16 x 3 = 768 B for 17..22 -- a
    // second round for the ranges past 16 -- 8 x 4 = 512 B for 23..29, 8 x 3
    // for 30..54, 4 x 3 in one round for 55..64, 4 x 2 = 128 B for 65..127,
    // 4 x 1 for more; profiles/r05/pk_early/pk_mid*.txt, pk_tiny*.txt,
    // profiles/r06/ab16/, ab17/, ab19/)
    // (One round of narrower groups instead -- 8 x 6 for 17..32 ranges, 4 x 6
    // for 33..64 -- measured 1.08-1.15x slower on shuffled 200-576-B ranges,
    // profiles/r06/ab2/pk_one_round_ab.txt.)
    const uint32_t lanes_per = T / kw;
    if (lanes_per >= 64)
        pk_ranges<MODE, 64, 4, true>(arena, descs, out, aux, first, kw, T, e0, have0);
    else if (lanes_per >= 32)
        pk_ranges<MODE, 32, 3, true>(arena, descs, out, aux, first, kw, T, e0, have0);
    else if (lanes_per >= 16 && kw >= 12u) // ranges of ~1 KiB and less: 1-KiB passes
        pk_ranges<MODE, 16, 4, true>(arena, descs, out, aux, first, kw, T, e0, have0);
    else if (lanes_per >= 16)
        pk_ranges<MODE, 16, 6, true>(arena, descs, out, aux, first, kw, T, e0, have0);
    else if (kw <= 22u) // 17..22 ranges of ~560..720 B: 16 lanes x 3 loads, a second round for the last few
        pk_ranges<MODE, 16, 3, true>(arena, descs, out, aux, first, kw, T, e0, have0);
    // ~190..223 B: one round of 4-lane groups, 3 loads each -- just enough
    // for the interior chunks (shuffled 200-B ranges 628 -> 544 us,
    // profiles/r06/ab17/); ~224..415 B: 8 x 3, one or two rounds (250-B
    // 547 -> 504 us, 320-B 451 -> 424, 400-B 386 -> 371, profiles/r06/ab19/;
    // past ~415 B 3 loads leave a second pass: 480-B ranges lost 20 %).
    // With 5 or 6 loads, or 8-lane groups for 17..22 ranges, one round lost
    // 2-8 % (ab17/).
    else if (kw >= 55u && kw <= 64u)
        pk_ranges<MODE, 4, 3>(arena, descs, out, aux, first, kw, T, e0, false);
    else if (kw >= 30u && kw <= 64u) // (8-lane groups: the early descriptors' layout for 30..32)
        pk_ranges<MODE, 8, 3, true>(arena, descs, out, aux, first, kw, T, e0, have0);
    else if (kw <= 32u) // 23..29 ranges, ~420..530 B: 512-B passes
        pk_ranges<MODE, 8, 4, true>(arena, descs, out, aux, first, kw, T, e0, have0);
    else if (kw < 128u) // ~96..190 B: 4 lanes x 2 loads (128 B), 64 ranges a round
        pk_ranges<MODE, 4, 2>(arena, descs, out, aux, first, kw, T, e0, have0);
    else // shorter: 4 lanes x 1 load, as the per-range kernel takes them (pick_geometry:
         // at most 4 interior chunks); the spare second load slot was the gap to it
         // (shuffled 64-B ranges 887 -> 769 us, 40-B 1,536 -> 1,325: profiles/r06/ab16/)
        pk_ranges<MODE, 4, 1>(arena, descs, out, aux, first, kw, T, e0, have0);
}


template <int MODE, int W = kPkWaves, int U = kPkLoads, bool PROBE = false>
__global__ __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(8))) void k_segments_pk(
    const uint8_t *__restrict__ arena, const void *__restrict__ descs, uint32_t n, uint16_t *__restrict__ out,
    uint32_t aux, uint32_t xg, uint32_t K)
{
    static_assert(MODE != MODE_EXACT, "the exact u32 sum stays on k_segments");
    static_assert(W <= 16, "the sub-range totals are scanned by 32 lanes");
    constexpr uint32_t T = W * 64u, CH = T * U, SR = 32u * U; // chunks per pass, per sub-range
    __shared__ u32x4 dat[CH];            // the pass's chunks, for the boundary bytes
    __shared__ uint32_t ex[CH];          // per chunk: its sub-range's word sum before it
    __shared__ uint32_t subtot[2 * W];   // per sub-range (32 lanes x U loads)
    __shared__ uint32_t region_ok[W];     // per wave: its ranges lie in the region
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x, xg);
    const uint32_t first = blk * K;
    const uint32_t kw = n - first < K ? n - first : K; // >= 1: grid = ceil(n / K)
    // the region: from the first range's first byte to the last range's end
    uint64_t r0, offl;
    uint32_t len0, lenl;
    // scalar loads: their short latency is what the data loads wait on
    // (fetching the two descriptors with vector loads instead cut the read
    // traffic from 1.0165x to 1.0018x the algorithmic bytes but ran 11 %
    // slower, profiles/r03/packed/ab_vdesc_w8.txt)
    desc_span<MODE>(descs, first, r0, len0);
    desc_span<MODE>(descs, first + kw - 1u, offl, lenl);

    const uint64_t rend = offl + lenl;
    const uint8_t *p = arena + r0;
    const uint32_t s0 = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 15u);
    // [r0, rend) runs from a byte of the first range to a byte of the last, so
    // it lies inside the arena whatever the ranges between do: its chunks are
    // safe to load before the ranges are known to lie inside it
    const bool span_ok = len0 != 0 && lenl != 0 && rend > r0 &&
                         rend - r0 <= (uint64_t)kPkMaxPasses * CH * 16u - s0;
    if (!PROBE && !span_ok) {
        // workgroup-uniform, known from the two scalar descriptors: range by
        // range at once (a shuffled batch's usual case), before any stream
        // load or the region check's own descriptor loads -- so its ranges'
        // descriptors and then their bytes are the only waits.  The
        // descriptor lines of the workgroup aux >> 8 logical blocks ahead are
        // touched on the way (a shuffled batch's workgroups all come here:
        // 258.0 -> 250.7 us for configs[1]'s ranges shuffled; on the region
        // path the same prefetch cost 1.6-9 %, profiles/r05/pk_layouts_pf.txt)
        uint32_t pf = 0;
        if (const uint32_t pfd = aux >> 8; pfd != 0u && w == 0) // wave-uniform
            pf = prefetch_descs(descs, (uint64_t)(blk + pfd) * K, n, MODE == MODE_PESO ? 24u : 16u,
                                (K * (MODE == MODE_PESO ? 24u : 16u) + 127u) / 128u + 1u, lane);
        // aux bit 7 (debug knob "pk_early"), K <= 32 (one range per lane
        // group): each wave reads the descriptors of its lane groups' ranges
        // with scalar loads -- lines the span's loads just brought into the
        // scalar cache -- instead of every lane's vector load going to the L2
        // for them, and each group picks its own
        const uint32_t G = pk_group(T, kw);
        const bool early = (aux & kPkEarly) != 0u && kw <= 32u; // workgroup-uniform
        SegDesc e0{0, 0, 0, 0, 0, 0};
        if (early) {
            uint32_t x[6] = {0u, 0u, 0u, 0u, 0u, 0u};
            // per = 64 / G ranges per wave, every load issued before any is used
            if (G == 64u)
                pk_wave_descs<MODE, 1>(descs, first, kw, x);
            else if (G == 32u)
                pk_wave_descs<MODE, 2>(descs, first, kw, x);
            else if (G == 16u)
                pk_wave_descs<MODE, 4>(descs, first, kw, x);
            else
                pk_wave_descs<MODE, 8>(descs, first, kw, x);
            e0 = desc_of<MODE>(x, true);
        }
        pk_fallback<MODE>(arena, descs, out, aux, first, kw, T, e0, early);
        asm volatile("" ::"v"(pf)); // keeps the prefetch load alive (its value is not used)
        return;
    }
    bool ranges = !span_ok; // workgroup-uniform: sum range by range instead
    const uint32_t span = span_ok ? (uint32_t)(rend - r0) : 0u;
    const uint32_t nch = span_ok ? (s0 + span + 15u) >> 4 : 0u;
    const uint32_t npass = (nch + CH - 1u) / CH;
    const uint32_t sub = t >> 5, l = t & 31u, hf = (t >> 5) & 1u;
    const u32x4 *base = span_ok ? reinterpret_cast<const u32x4 *>(p - s0) : &g_zero_chunk;
    u32x4 v[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
        const uint32_t c = sub * SR + u * 32u + l;
        v[u] = load16<true>(base + (c < nch ? c : (nch ? nch - 1u : 0u)));
    }
    issue_fence();
    // every wave: its share of the K descriptors (lane r: range 64w + r),
    // whether each lies in the region, and its start and end in bytes from the
    // first chunk
    const uint32_t rr = w * 64u + lane;
    const bool mine = rr < kw;
    const bool has = w * 64u < kw; // wave-uniform
    SegDesc d{0, 0, 0, 0, 0, 0};
    uint32_t xs = 0, xe = 0, q16 = 0;
    if (has) {
        d = load_desc<MODE>(descs, first + rr, mine);
        // P wraps mod 2^32 across passes, so a difference is exact only for a
        // range whose word sum stays below 2^32: < 128 KiB (<= 65536 words)
        const bool inside = !mine || (d.off >= r0 && d.off + d.len <= rend && d.len < (1u << 17));
        const bool ok = __ballot(!inside) == 0;
        xs = ok ? s0 + (uint32_t)(d.off - r0) : 0u;
        xe = ok ? xs + d.len : 0u;
        if constexpr (MODE == MODE_PESO)
            q16 = peso_pseudo16(d);
        if (lane == 0)
            region_ok[w] = ok ? 1u : 0u;
    } else if (lane == 0) {
        region_ok[w] = 1u;
    }
    if constexpr (PROBE) { // measurement: the same loads, no arithmetic
        u32x4 z = v[0];
#pragma unroll
        for (uint32_t u = 1; u < U; ++u)
            z ^= v[u];
        const uint32_t f = z.x ^ z.y ^ z.z ^ z.w ^ q16 ^ xe;
        if (f == 0x9E3779B9u)
            reinterpret_cast<uint32_t *>(out)[0] = f;
        return;
    }
    uint32_t run = 0, ps = 0, pe = 0; // word sum of the passes before; P(start), P(end)
    for (uint32_t pass = 0; !ranges && pass < npass; ++pass) { // workgroup-uniform
        const uint32_t cb = pass * CH;
        // every wave: chunk sums, their scans over each 32-lane half; per chunk
        // the word sum of its sub-range before it, and the chunk itself
        uint32_t a = 0; // this lane's half-wave: chunks of loads u' < u
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t c = sub * SR + u * 32u + l;
            const uint32_t f = chunk_sum_w(0u, v[u], cb + c < nch ? 0x00010001u : 0u); // < 2^20
            const uint32_t sc = scan32(f);
            ex[c] = a + (sc - f);
            dat[c] = v[u];
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)sc, 31);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)sc, 63);
            a += hf ? hi : lo;
        }
        if (l == 0)
            subtot[sub] = a;
        if (pass + 1u < npass) { // the next pass's bytes stream during the barrier and the prefix sums
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) {
                const uint32_t c = cb + CH + sub * SR + u * 32u + l;
                v[u] = load16<true>(base + (c < nch ? c : nch - 1u));
            }
        }
        __syncthreads();
        if (pass == 0) {
            bool all = true;
#pragma unroll
            for (uint32_t i = 0; i < W; ++i)
                all = all && region_ok[i] != 0u;
            if (!all) {
                ranges = true;
                break;
            }
        }
        if (has) {
            // P(x) = passes before + sub-ranges before + ex[chunk] + the chunk's
            // bytes before x; the end of the region (x = 16 * nch) is byte 16 of
            // the last chunk
            const uint32_t st = lane < 2u * W ? subtot[lane] : 0u;
            const uint32_t si = scan32(st);
            const uint32_t sx = si - st;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint32_t x = k ? xe : xs;
                uint32_t cx = x >> 4, bx = x & 15u;
                if (cx == nch) {
                    cx = nch - 1u;
                    bx = 16u;
                }
                const bool here = cx >= cb && cx < cb + CH;
                const uint32_t lc = here ? cx - cb : 0u;
                const uint32_t sp = (uint32_t)__shfl((int)sx, (int)(lc / SR), 64);
                const uint32_t px = run + sp + ex[lc] + chunk_prefix_sum(dat[lc], bx);
                if (k)
                    pe = here ? px : pe;
                else
                    ps = here ? px : ps;
            }
            run += (uint32_t)__builtin_amdgcn_readlane((int)si, 31);
        }
        if (pass + 1u < npass)
            __syncthreads(); // the next pass overwrites dat / ex / subtot
    }
    if (ranges) { // a range outside the region, found by the descriptor check
        // (e0 is not carried here: it would stay live through the region path)
        pk_fallback<MODE>(arena, descs, out, aux, first, kw, T, SegDesc{0, 0, 0, 0, 0, 0}, false);
        return;
    }
    if (mine)
        out[first + rr] = finalize<MODE>(pe - ps, reinterpret_cast<uintptr_t>(arena + d.off), d, aux, q16);
}

// ---------------------------------------------------------------- IPv4
//
// Both checksums of a captured IPv4 packet in one pass over its bytes, in one
// of three modes:
//   IP_SUMS  header + L4 values (ipv4.c:243 / tcp_in.c:80 / udp.c:410 /
//            icmpv4.c:36) and is_pkt_ok flags;
//   IP_TX    the stack's tx fill, in place: checksum fields read as zero,
//            values stored into them (ipv4.c:643,656, tcp_out.c:19-20,
//            udp.c:320-321, icmpv4.c:45-58); with IP_OPT_NO_STORE the same
//            values go to `out` only (tx offload: the host applies them);
//   IP_RX    the stack's rx gates: net_err_t verdict per packet
//            (ipv4.c:475-515, is_pkt_ok ipv4.c:220-250, tcp_in.c:69-85,
//            udp.c:386-415, icmpv4.c:29-43,71-77).
// The 20 fixed header bytes come from two or three aligned chunks realigned
// with v_alignbyte; the data pass splits every chunk between the header range
// [0,hl), the L4 range [hl,end) and the 2-byte checksum fields.
enum IpMode : int { IP_SUMS = 0, IP_TX = 1, IP_RX = 2 };
// k_ipv4 `opts` bits (runtime, uniform over the grid)
constexpr uint32_t IP_OPT_NO_STORE = 1u; // IP_TX: compute the fill's values, leave the packets alone
// IP_TX, deferred stores (launch_ipv4 mode 4): the values go to `out` and each
// packet's store positions to a side array (through the verdict pointer, which
// tx never uses); k_tx_scatter then writes them into the packets in a second,
// short launch (profiles/history/DESIGN_rounds1-5.md §6, tx fill)
constexpr uint32_t IP_OPT_DEFER = 2u;
// launch_ipv4 mode 3: IP_TX kernels with IP_OPT_NO_STORE
constexpr int IP_TX_OFFLOAD = 3;
// launch_ipv4 mode 4: the tx fill as k_ipv4<IP_TX> with IP_OPT_DEFER + k_tx_scatter
constexpr int IP_TX_SPLIT = 4;

// One 16-byte LDS-DMA per lane (global_load_lds_dwordx4, nontemporal):
// lane l's chunk lands at slot[l] -- the wave-uniform slot base plus 16 * l.
__device__ __forceinline__ void lds_dma16(const u32x4 *src, u32x4 *slot)
{
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src),
                                     (__attribute__((address_space(3))) void *)(slot), 16, 0, 2);
}

// k_ipv4 PIPE 5's LDS: per wave of a 256-thread workgroup, U slots of 64
// chunks (U KiB), this wave's returned.
template <int U>
__device__ __forceinline__ u32x4 *ipv4_lds_ring()
{
    __shared__ u32x4 ring[4][U * 64];
    return ring[threadIdx.x >> 6];
}

// The 20 fixed header bytes at byte s0 (0..15) of the three aligned chunks
// h0, h1, h2, as five dwords: hd[k] = bytes [s0 + 4k, s0 + 4k + 4).  Two
// stages of selects on named scalars pick dwords q = s0 >> 2 .. q + 5, then
// v_alignbyte shifts by s0 & 3.  (Written over an array, w[q + k], clang
// turned the selects back into a dynamically indexed alloca and promoted it
// to 20 KiB of LDS per workgroup: ds_write/ds_read on every packet.)
struct Hdr5 {
    uint32_t d0, d1, d2, d3, d4;
};
__device__ __forceinline__ Hdr5 header_dwords(u32x4 h0, u32x4 h1, u32x4 h2, uint32_t s0)
{
    const bool b1 = s0 & 4u, b2 = s0 & 8u;
    const uint32_t y0 = b1 ? h0.y : h0.x, y1 = b1 ? h0.z : h0.y, y2 = b1 ? h0.w : h0.z, y3 = b1 ? h1.x : h0.w;
    const uint32_t y4 = b1 ? h1.y : h1.x, y5 = b1 ? h1.z : h1.y, y6 = b1 ? h1.w : h1.z, y7 = b1 ? h2.x : h1.w;
    const uint32_t x0 = b2 ? y2 : y0, x1 = b2 ? y3 : y1, x2 = b2 ? y4 : y2;
    const uint32_t x3 = b2 ? y5 : y3, x4 = b2 ? y6 : y4, x5 = b2 ? y7 : y5;
    const uint32_t r = s0 & 3u;
    return Hdr5{__builtin_amdgcn_alignbyte(x1, x0, r), __builtin_amdgcn_alignbyte(x2, x1, r),
                __builtin_amdgcn_alignbyte(x3, x2, r), __builtin_amdgcn_alignbyte(x4, x3, r),
                __builtin_amdgcn_alignbyte(x5, x4, r)};
}

// Sum of the chunk's bytes that fall in [r0, r1) (offsets from the chunk base c;
// all positions are bytes from the packet's first chunk, < 2^17).
__device__ __forceinline__ uint32_t region_sum(u32x4 v, int c, int r0, int r1)
{
    const int lo = r0 - c, hi = r1 - c;
    const int a = lo < 0 ? 0 : (lo > 16 ? 16 : lo);
    const int b = hi < 0 ? 0 : (hi > 16 ? 16 : hi);
    return chunk_sum_masked(0u, v, a, b);
}

// L4 checksum field offset and minimum header length by protocol
// (tcp.h:71, udp.h:24, icmpv4.h:28); 0 when the protocol has none here.
__device__ __forceinline__ uint32_t l4_field(uint32_t proto, uint32_t &min_len)
{
    min_len = proto == 6 ? 20u : proto == 17 ? 8u : proto == 1 ? 4u : 0u;
    return proto == 6 ? 16u : proto == 17 ? 6u : proto == 1 ? 2u : 0u;
}

// What the fixed IPv4 header (and, rx, the TCP/UDP header words) decide
// before any sum: the is_pkt_ok flags, the header and L4 byte ranges, the
// checksum field this mode treats specially, the folded pseudo-header and
// (rx) every sum-free gate.  Shared by k_ipv4 and the byte-window stream
// k_flat_ipv4 so that both decide exactly alike.
struct IpHdr {
    uint32_t fl;     // TCSUM_PKT_* (SHORT is set at the end)
    uint32_t hl;     // header bytes summed: IHL*4, clamped to [20, frame]
    uint32_t end;    // L4 range end: total_len clamped to [hl, frame]
    uint32_t proto;
    uint32_t fld;    // the L4 checksum field's offset in the L4 header (0: none)
    uint32_t pseudo; // TCP/UDP pseudo-header, folded (tools.c:58-70)
    uint32_t vcodes; // rx: three int8 gate codes + (stored header checksum != 0) << 24
    bool bad;        // SHORT / BAD_*: nothing stored, no field
    bool field_on;   // the L4 field this mode zeroes (tx) or tests (rx)
};

// hd: the 20 fixed header bytes; l4words(ihl4): the Hdr5 of the 16 bytes at
// packet offset ihl4 (the TCP/UDP header's first bytes; called for rx only).
template <int IPM, class L4Words>
__device__ __forceinline__ IpHdr ip_parse(const Hdr5 &hd, uint32_t frame, bool big_enough, L4Words &&l4words)
{
    IpHdr h;
    const uint32_t b0h = hd.d0 & 0xFFu;
    const uint32_t version = b0h >> 4;
    const uint32_t ihl4 = (b0h & 0xFu) << 2;
    const uint32_t tl = (((hd.d0 >> 16) & 0xFFu) << 8) | (hd.d0 >> 24);
    const uint32_t b6 = (hd.d1 >> 16) & 0xFFu, b7 = hd.d1 >> 24;
    const bool frag = (b6 & 0x20u) || (((b6 & 0x1Fu) << 8) | b7);
    const uint32_t proto = (hd.d2 >> 8) & 0xFFu;
    const uint32_t stored_ip = hd.d2 >> 16;
    uint32_t fl = 0;
    if (version != 4)
        fl |= TCSUM_PKT_BAD_VERSION;
    if (ihl4 < 20 || ihl4 > frame)
        fl |= TCSUM_PKT_BAD_HDRLEN;
    if (tl < 20 || tl > frame || tl < ihl4)
        fl |= TCSUM_PKT_BAD_TOTLEN;
    if (frag)
        fl |= TCSUM_PKT_FRAGMENT;
    uint32_t hl = ihl4 < 20 ? 20u : ihl4;
    hl = hl > frame ? frame : hl;
    uint32_t end = tl < hl ? hl : tl;
    end = end > frame ? frame : end;
    uint32_t min_l4;
    const uint32_t fld = l4_field(proto, min_l4);
    if (fld && end - hl < min_l4)
        fl |= TCSUM_PKT_L4_SHORT;
    const bool bad = !big_enough ||
                     (fl & (TCSUM_PKT_BAD_VERSION | TCSUM_PKT_BAD_HDRLEN | TCSUM_PKT_BAD_TOTLEN));
    // the L4 checksum field this mode treats specially (tx: zero + store;
    // rx: is it zero?) -- none for fragments, short L4, or ICMP on rx
    const bool field_on = IPM != IP_SUMS && !bad && !frag && fld && !(fl & TCSUM_PKT_L4_SHORT) &&
                          !(IPM == IP_RX && proto == 1);
    // The L4 pseudo-header (tools.c:58-70), folded now: src, dst (packet bytes
    // 12..19), {0, proto}, the L4 length; kept as one register past the data pass
    uint32_t pseudo = 0;
    if (proto == 6 || proto == 17)
        pseudo = fold16(add_halves(add_halves(0u, hd.d3), hd.d4) + (proto << 8) + bswap16((end - hl) & 0xFFFFu));
    if (big_enough && proto != 6 && proto != 17 && proto != 1)
        fl |= TCSUM_PKT_PROTO_OTHER;

    // rx: every gate that needs no sum, decided now, in the reference's order
    // (the verdict at the end only places the two checksum tests between them):
    //   pre  -- ipv4_in before the header checksum test (ipv4.c:475, 222-240)
    //   mid  -- the L4 input before its checksum test (tcp_in.c:70-74 and
    //           pktbuf_remove_header, udp.c:386-403, icmpv4.c:68)
    //   post -- the L4 input after it (tcp_in.c:87-103)
    // packed as three int8 in one register.
    uint32_t vcodes = 0;
    if constexpr (IPM == IP_RX) {
        int vpre = 0, vmid = 0, vpost = 0;
        if (!big_enough)
            vpre = TCSUM_ERR_SIZE; // pktbuf_set_cont(buf, 20), ipv4.c:475
        else if (version != 4)
            vpre = TCSUM_ERR_NOT_SUPPORT; // ipv4.c:222-226
        else if (ihl4 < 20 || tl < 20 || frame < tl)
            vpre = TCSUM_ERR_SIZE; // ipv4.c:228-240
        else if (frag)
            vmid = 0; // ipv4.c:506-509: queued for reassembly, OK past the header test
        else if (proto == 6 || proto == 17) { // TCP: pktbuf_remove_header + tcp_in (ipv4.c:450-452); UDP: udp_in
            // the header words: L4 bytes 0-3 (ports) and 12-15 (data offset, flags)
            uint32_t ports = 0, oflags = 0;
            if (tl >= ihl4 + 8u) {
                const Hdr5 l4h = l4words(ihl4);
                ports = l4h.d0;
                oflags = l4h.d3;
            }
            const uint32_t sport = ports & 0xFFFFu, dport = ports >> 16, fword = oflags & 0xFFFFu;
            if (proto == 6) {
                if (ihl4 > tl)
                    vmid = TCSUM_ERR_SIZE; // the reference runs off its block list (pktbuf.c:264-281)
                else if (tl - ihl4 < 20)
                    vmid = TCSUM_ERR_SYS; // pktbuf_set_cont fails: tcp_in returns -1, tcp_in.c:70-74
                else if (tl - ihl4 < (((oflags & 0xFFu) >> 4) << 2))
                    vpost = TCSUM_ERR_SIZE; // tcp_in.c:87-91
                else if (sport == 0 || dport == 0 || fword == 0)
                    vpost = TCSUM_ERR_BROKEN; // tcp_in.c:93-103
            } else {
                if (tl < ihl4 + 8)
                    vmid = TCSUM_ERR_SIZE; // pktbuf_set_cont(buf, 8 + ihl), udp.c:386-391
                else if (dport == 0)
                    vmid = TCSUM_ERR_UNREACHABLE; // no socket has port 0: udp.c:337-340, :399-403
            }
        } else if (proto == 1) { // icmpv4_in, ipv4.c:427; its checksum test cannot fail (A10)
            vmid = tl < ihl4 + 4 ? TCSUM_ERR_SIZE : 0; // pktbuf_set_cont(buf, ihl + 4), icmpv4.c:68
        } // other protocols: raw_in, no checksum (ipv4.c:460-469)
        vcodes = (uint32_t)(uint8_t)vpre | ((uint32_t)(uint8_t)vmid << 8) | ((uint32_t)(uint8_t)vpost << 16) |
                 (stored_ip != 0 ? 1u << 24 : 0u);
    }
    h.fl = fl;
    h.hl = hl;
    h.end = end;
    h.proto = proto;
    h.fld = fld;
    h.pseudo = pseudo;
    h.vcodes = vcodes;
    h.bad = bad;
    h.field_on = field_on;
    return h;
}

// The packet's results from its header sum and L4 sum (acc_h, acc_l: word
// sums by address parity, any grouping -- fold16 keeps "zero iff all bytes
// zero"), odd = the packet's start address parity, acc_f (rx): nonzero iff
// the stored L4 checksum field is.  Stores out / flags / verdict, and the tx
// fill's fields (in place, or their positions for k_tx_scatter with
// IP_OPT_DEFER).
template <int IPM>
__device__ __forceinline__ void ip_finish(const IpHdr &ih, uint32_t fl, bool big_enough, uint32_t odd,
                                          uint32_t acc_h, uint32_t acc_l, uint32_t acc_f, uint8_t *pp, uint32_t pk,
                                          uint32_t *__restrict__ out, uint8_t *__restrict__ flags_out,
                                          int8_t *__restrict__ verdict_out, uint32_t opts)
{
    uint32_t ip = 0, l4 = 0;
    if (!big_enough) {
        fl = TCSUM_PKT_SHORT;
    } else {
        uint32_t fh = fold16(acc_h);
        uint32_t f4 = fold16(acc_l);
        if (odd) {
            fh = rot8(fh);
            f4 = rot8(f4);
        }
        ip = ~fh & 0xFFFFu;
        if (ih.proto == 6 || ih.proto == 17)
            l4 = ~fold_step(f4 + ih.pseudo) & 0xFFFFu;
        else if (ih.proto == 1)
            l4 = ~f4 & 0xFFFFu;
    }
    if constexpr (IPM == IP_TX) {
        if (opts & IP_OPT_DEFER) // bit 16: the IPv4 field; low 16: the L4 field's offset (0: none)
            reinterpret_cast<uint32_t *>(verdict_out)[pk] = ih.bad ? 0u : (1u << 16) | (ih.field_on ? ih.hl + ih.fld : 0u);
        else if (!ih.bad && !(opts & IP_OPT_NO_STORE)) { // stored in host order, like the struct fields
            pp[10] = (uint8_t)ip;
            pp[11] = (uint8_t)(ip >> 8);
            if (ih.field_on) {
                pp[ih.hl + ih.fld] = (uint8_t)l4;
                pp[ih.hl + ih.fld + 1] = (uint8_t)(l4 >> 8);
            }
        }
    }
    if constexpr (IPM == IP_RX) {
        // The first gate that rejects, in the reference's order: ipv4_in /
        // is_pkt_ok, then the L4 input ip_normal_in dispatches to
        // (ipv4.c:420-470), up to socket lookup.  Pinned by the reference
        // stack's own verdicts (tests/golden/ipv4_rx_*, oracle/stack_gen.c).
        const uint32_t vcodes = ih.vcodes;
        const int vpre = (int8_t)(vcodes & 0xFFu), vmid = (int8_t)((vcodes >> 8) & 0xFFu);
        const int vpost = (int8_t)((vcodes >> 16) & 0xFFu);
        int v8;
        if (vpre)
            v8 = vpre;
        else if ((vcodes >> 24) && ip != 0)
            v8 = TCSUM_ERR_BROKEN; // ipv4.c:241-249
        else if (vmid)
            v8 = vmid;
        else if (acc_f != 0 && l4 != 0)
            v8 = TCSUM_ERR_BROKEN; // tcp_in.c:77-85, udp.c:407-415 (field_on: TCP/UDP only)
        else
            v8 = vpost;
        verdict_out[pk] = (int8_t)v8;
    }
    if (out)
        out[pk] = ip | (l4 << 16);
    if (flags_out)
        flags_out[pk] = (uint8_t)fl;
}

// Packet `pk` (one per G-lane group; pk >= n: a dead group that reads
// descriptor 0 and writes nothing).  Every lane of the wave must call it: the
// group reduction crosses lanes.
// SKEW (measurement): the data pass starts SKEW bytes past the packet's
// 128-B line instead of on it, for packets that start that far in (0: the
// route)
// PIPE (measurement): 1 = each later pass's loads are issued before the
// previous pass is summed (two passes in flight per lane group, more
// registers); 2 = rolling -- each load slot is reissued for the next pass as
// soon as its chunk is taken, so a multi-pass packet keeps U loads in flight
// per lane with no more registers than one pass; 3 = no header loads, the
// header chunks taken from the lanes whose first data-pass load holds them;
// 4 = the descriptors by scalar loads, a wave's 2 or 4 at once;
// 5 = a multi-pass packet's next pass streamed into LDS by LDS-DMA
// (global_load_lds_dwordx4, one 1-KiB wave-instruction per load slot) while
// the current pass is summed from registers: two passes in flight with no
// second register set (ipv4_lds_ring; 256-thread workgroups).
// H1: the third header chunk (whose first dword alone the sums / tx modes
// use) loaded as that one dword, so no dead part of a 16-byte header load
// is a register the compiler reuses -- with a vmcnt wait for the header
// loads -- before the data pass's loads are issued.
template <int G, int U, int IPM, int SKEW = 0, int PIPE = 0, bool H1 = false>
__device__ __forceinline__ void ipv4_packet(uint8_t *__restrict__ arena, const tcsum_pkt_t *__restrict__ pkts,
                                            uint32_t pk, uint32_t n, uint32_t *__restrict__ out,
                                            uint8_t *__restrict__ flags_out, int8_t *__restrict__ verdict_out,
                                            uint32_t opts)
{
    const uint32_t gl = threadIdx.x & (G - 1);
    const bool live = pk < n;

    // unconditional loads throughout (dead lanes read descriptor 0 / the zero chunk)
    u32x4 dv;
    if constexpr (PIPE == 4) {
        // the wave's packets' descriptors by scalar loads (16 B each, the
        // pktbuf_checksum16 layout), each lane group picking its own
        static_assert(G >= 16, "at most 4 descriptors a wave");
        const uint32_t firstp = pk - threadIdx.x / G; // the workgroup's first packet
        const uint32_t kwp = n > firstp ? (n - firstp < 256u / G ? n - firstp : 256u / G) : 1u;
        uint32_t x[6] = {0u, 0u, 0u, 0u, 0u, 0u};
        pk_wave_descs<MODE_SEG, 64u / G>(pkts, n > firstp ? firstp : 0u, kwp, x);
        dv.x = x[0];
        dv.y = x[1];
        dv.z = x[2];
        dv.w = x[3];
    } else {
        dv = *reinterpret_cast<const u32x4 *>(pkts + (live ? pk : 0u));
    }
    const uint64_t off = (uint64_t)dv.x | ((uint64_t)dv.y << 32);
    const uint32_t frame = live ? dv.z : 0u;
    const bool big_enough = frame >= 20;
    uint8_t *pp = arena + off;
    const uintptr_t start = reinterpret_cast<uintptr_t>(pp);
    const uint32_t s0 = (uint32_t)(start & 15u);
    const u32x4 *base = reinterpret_cast<const u32x4 *>(pp - s0);

    // IPv4 bytes past 65,535 (the largest total_len) never count: bound the
    // loads there, so every position below fits comfortably in 32 bits
    const uint32_t frame_ld = frame < 65600u ? frame : 65600u;
    const uint32_t nch = big_enough ? (frame_ld + s0 + 15) >> 4 : 0u;

    // fixed header: bytes [s0, s0 + 20) of base[0..2]
    const u32x4 *hb = big_enough ? base : &g_zero_chunk;
    const uint32_t h1i = big_enough ? 1u : 0u;
    // header loads: default cache policy (nontemporal like the data pass that
    // loads the same chunks: no different in time or traffic,
    // profiles/r02/ab_hdr_nt_*.txt)
    auto hload = [](const u32x4 *q) { return load16<false>(q); };
    u32x4 h0 = u32x4(0u), h1 = u32x4(0u), h2 = u32x4(0u), c2 = u32x4(0u), c3 = u32x4(0u);
    if constexpr (PIPE == 3) {
        // (PIPE 3: no header loads -- the chunks come from the data pass below)
    } else if constexpr (IPM == IP_RX) {
        h0 = hload(hb);
        h1 = hload(hb + h1i);
        // chunks 2 and 3 as well: an IHL-5 packet's TCP/UDP ports, data offset
        // and flags (L4 bytes 0-3, 12-13) lie in chunks 1..3
        c2 = hload(nch > 2 ? base + 2 : &g_zero_chunk);
        c3 = hload(nch > 3 && s0 >= 12 ? base + 3 : &g_zero_chunk);
        h2 = s0 > 12 ? c2 : u32x4(0u);
    } else if constexpr (H1) {
        h0 = hload(hb);
        h1 = hload(hb + h1i);
        const uint32_t h2x = *reinterpret_cast<const uint32_t *>(hb + (big_enough ? (s0 > 12 ? 2u : 1u) : 0u));
        h2 = u32x4(0u);
        h2.x = s0 > 12 ? h2x : 0u;
    } else {
        h0 = hload(hb);
        h1 = hload(hb + h1i);
        const u32x4 h2v = hload(hb + (big_enough ? (s0 > 12 ? 2u : 1u) : 0u));
        h2 = s0 > 12 ? h2v : u32x4(0u);
    }
    // The data pass counts chunks from the packet's 128-B line, not from its
    // 16-B chunk: the G*U-chunk span of each pass then ends on a line
    // boundary, so no line is split between two passes (a split line is
    // fetched once per pass: the nontemporal first fetch is gone from L2 by
    // the time the next pass, a memory latency later, wants the other half).
    // Chunks of that line before the packet are loaded (same line, same page)
    // but fall outside every byte range below.
    // (SKEW: only for packets that start at least SKEW bytes into their line,
    // so the pass never begins before the packet's own line)
    const uint32_t s127 = (uint32_t)(start & 127u);
    const uint32_t sl = SKEW && s127 >= (uint32_t)SKEW ? s127 - (uint32_t)SKEW : s127;
    const uint32_t dch = big_enough ? (frame_ld + sl + 15) >> 4 : 0u;
    const u32x4 *dbase = dch ? reinterpret_cast<const u32x4 *>(pp - sl) : &g_zero_chunk;
    const uint32_t dlast = dch ? dch - 1u : 0u;

    // first pass of data loads before the header is consumed: its latency
    // overlaps them (vmcnt counts in issue order)
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t idx = u * G + gl;
        v[u] = load16<true>(dbase + (idx < dch ? idx : dlast));
    }
    // PIPE 5: the wave's LDS slots -- load slot u of lane l at ring[u][l] --
    // and pass 1's chunks into them, in flight with pass 0's
    [[maybe_unused]] u32x4 *ring = nullptr;
    if constexpr (PIPE == 5) {
        ring = ipv4_lds_ring<U>();
        if (dch > (uint32_t)(G * U)) { // group-uniform: this packet has a second pass
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t idx = (uint32_t)(G * U + u * G) + gl;
                lds_dma16(dbase + (idx < dch ? idx : dlast), ring + u * 64);
            }
        }
    }
    issue_fence();
    if constexpr (PIPE == 3) {
        // the header chunks from the lanes of the group whose first-pass load
        // holds them: packet chunk j is pass chunk (sl >> 4) + j <= 10 < G,
        // i.e. load 0 of lane (sl >> 4) + j; zero past the packet
        static_assert(G >= 16 && SKEW == 0, "the header chunks lie in the first 11 lanes of the group");
        const int gb = (int)((threadIdx.x & 63u) & ~(uint32_t)(G - 1));
        auto hc = [&](uint32_t j) {
            const int src = gb + (int)((sl >> 4) + j);
            u32x4 r;
            r.x = (uint32_t)__shfl((int)v[0].x, src, 64);
            r.y = (uint32_t)__shfl((int)v[0].y, src, 64);
            r.z = (uint32_t)__shfl((int)v[0].z, src, 64);
            r.w = (uint32_t)__shfl((int)v[0].w, src, 64);
            return j < nch ? r : u32x4(0u);
        };
        h0 = hc(0);
        h1 = hc(1);
        if constexpr (IPM == IP_RX) {
            c2 = hc(2);
            c3 = s0 >= 12 ? hc(3) : u32x4(0u);
            h2 = s0 > 12 ? c2 : u32x4(0u);
        } else {
            h2 = s0 > 12 ? hc(2) : u32x4(0u);
        }
    }

    const Hdr5 hd = header_dwords(h0, h1, h2, s0);
    // rx: the TCP/UDP header words (L4 bytes 0-3: ports; 12-15: data offset,
    // flags) from the 32 bytes at chunk (s0 + ihl4) / 16: chunks 1..3 already
    // in registers for IHL 5, two more loads otherwise
    // (the lambda captures by value: a reference capture takes the chunks'
    // addresses, and clang then kept them in scratch memory)
    const IpHdr ih = ip_parse<IPM>(hd, frame, big_enough, [=](uint32_t ihl4) {
        const uint32_t o = s0 + ihl4, cw = o >> 4;
        u32x4 wa, wb;
        if (ihl4 == 20) {
            wa = cw == 1 ? h1 : c2;
            wb = cw == 1 ? c2 : c3;
        } else {
            wa = load16<false>(base + cw);
            wb = load16<false>(cw + 1 < nch ? base + cw + 1 : &g_zero_chunk);
        }
        return header_dwords(wa, wb, u32x4(0u), o & 15u);
    });
    uint32_t fl = ih.fl;
    const bool field_on = ih.field_on;
    const uint32_t hl = ih.hl, end = ih.end, fld = ih.fld;

    // byte ranges, from the data pass's line base (end <= tl <= 65535 whenever
    // it matters; clamp so a huge bogus frame cannot overflow)
    const int h_end = (int)(hl < 65600u ? hl : 65600u) + (int)sl;
    const int l_end = (int)(end < 65600u ? end : 65600u) + (int)sl;
    const int f0 = field_on ? (int)(hl + fld) + (int)sl : -64;
    const int i0 = (int)sl + 10; // IPv4 header checksum field

    uint32_t acc_h = 0, acc_l = 0, acc_f = 0;
    // one pass of U chunks per lane starting at chunk b0 (pass 0: the loads
    // already in flight; later passes load and sum inside one iteration, so
    // no vector registers are carried around the loop -- see frame_consume)
    auto pass = [&](const u32x4 (&vv)[U], uint32_t b0) {
        uint32_t ph = 0, pl = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t idx = b0 + u * G + gl;
            const bool valid = idx < dch;
            const int c = (int)(16u * idx);
            const bool inner = valid && c >= h_end && c + 16 <= l_end && (f0 + 2 <= c || f0 >= c + 16);
            if (valid && !inner) { // header chunks, the field chunk(s), the last chunk: rare
                uint32_t th = region_sum(vv[u], c, (int)sl, h_end);
                uint32_t tl4 = region_sum(vv[u], c, h_end, l_end);
                if (field_on) {
                    const uint32_t tf = region_sum(vv[u], c, f0, f0 + 2);
                    if (IPM == IP_TX)
                        tl4 -= tf; // tcp_out.c:19 / udp.c:320 / icmpv4.c:58 zero it first
                    else
                        acc_f += tf;
                }
                if (IPM == IP_TX)
                    th -= region_sum(vv[u], c, i0, i0 + 2); // ipv4.c:643
                ph += th;
                pl += tl4;
            }
            pl = chunk_sum_w(pl, vv[u], inner ? 0x00010001u : 0u);
        }
        acc_h += ph; // header <= 60 bytes: no overflow
        acc_l = fold_step(acc_l + pl);
    };
    if constexpr (PIPE == 2) {
        for (uint32_t b0 = 0; b0 < dch; b0 += G * U) {
            const bool more = b0 + G * U < dch; // group-uniform
            uint32_t ph = 0, pl = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const u32x4 x = v[u];
                { // unconditional (the last pass reloads its last chunk): a branch here
                  // makes the compiler wait for every load in flight at the join
                    const uint32_t nidx = more ? b0 + G * U + u * G + gl : dlast;
                    v[u] = load16<true>(dbase + (nidx < dch ? nidx : dlast));
                }
                const uint32_t idx = b0 + u * G + gl;
                const bool valid = idx < dch;
                const int c = (int)(16u * idx);
                const bool inner = valid && c >= h_end && c + 16 <= l_end && (f0 + 2 <= c || f0 >= c + 16);
                if (valid && !inner) {
                    uint32_t th = region_sum(x, c, (int)sl, h_end);
                    uint32_t tl4 = region_sum(x, c, h_end, l_end);
                    if (field_on) {
                        const uint32_t tf = region_sum(x, c, f0, f0 + 2);
                        if (IPM == IP_TX)
                            tl4 -= tf;
                        else
                            acc_f += tf;
                    }
                    if (IPM == IP_TX)
                        th -= region_sum(x, c, i0, i0 + 2);
                    ph += th;
                    pl += tl4;
                }
                pl = chunk_sum_w(pl, x, inner ? 0x00010001u : 0u);
            }
            acc_h += ph;
            acc_l = fold_step(acc_l + pl);
        }
    } else if constexpr (PIPE == 5) {
        if (dch)
            pass(v, 0u);
        const uint32_t ln = threadIdx.x & 63u;
        for (uint32_t b0 = G * U; b0 < dch; b0 += G * U) { // group-divergent: a done group's lanes idle
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // this pass's DMA has landed
            u32x4 w[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                w[u] = ring[u * 64 + ln];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // read out before the slots are refilled
            if (b0 + G * U < dch) { // the next pass streams in while this one is summed
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t idx = b0 + (uint32_t)(G * U + u * G) + gl;
                    lds_dma16(dbase + (idx < dch ? idx : dlast), ring + u * 64);
                }
            }
            pass(w, b0);
        }
    } else if constexpr (PIPE == 1) {
        u32x4 nx[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t idx = G * U + u * G + gl;
            nx[u] = load16<true>(dbase + (idx < dch ? idx : dlast));
        }
        if (dch)
            pass(v, 0u);
        for (uint32_t b0 = G * U; b0 < dch; b0 += G * U) {
            u32x4 cur[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                cur[u] = nx[u];
                const uint32_t idx = b0 + G * U + u * G + gl;
                nx[u] = load16<true>(dbase + (idx < dch ? idx : dlast));
            }
            pass(cur, b0);
        }
    } else {
        if (dch)
            pass(v, 0u);
        for (uint32_t b0 = G * U; b0 < dch; b0 += G * U) {
            u32x4 w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t idx = b0 + u * G + gl;
                w[u] = load16<true>(dbase + (idx < dch ? idx : dlast));
            }
            pass(w, b0);
        }
    }
    acc_h = group_sum<G>(acc_h);
    acc_l = group_sum<G>(acc_l);
    if (IPM == IP_RX)
        acc_f = group_sum<G>(acc_f);

    if (live && gl == 0)
        ip_finish<IPM>(ih, fl, big_enough, (uint32_t)(start & 1u), acc_h, acc_l, acc_f, pp, pk, out, flags_out,
                       verdict_out, opts);
}

template <int G, int U, int IPM, int T = 256, int SKEW = 0, int PIPE = 0, bool H1 = false>
__global__ __launch_bounds__(T) void k_ipv4(uint8_t *__restrict__ arena, const tcsum_pkt_t *__restrict__ pkts,
                                            uint32_t n, uint32_t *__restrict__ out,
                                            uint8_t *__restrict__ flags_out, int8_t *__restrict__ verdict_out,
                                            uint32_t opts, uint32_t xg)
{
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x, xg);
    ipv4_packet<G, U, IPM, SKEW, PIPE, H1>(arena, pkts, blk * (uint32_t)(T / G) + threadIdx.x / G, n, out,
                                           flags_out, verdict_out, opts); // no 32-bit wrap for any n
}

// k_ipv4 with two data passes in flight per lane group (measurement)
template <int G, int U, int IPM>
__global__ __launch_bounds__(256) void k_ipv4_db(uint8_t *__restrict__ arena, const tcsum_pkt_t *__restrict__ pkts,
                                                 uint32_t n, uint32_t *__restrict__ out,
                                                 uint8_t *__restrict__ flags_out, int8_t *__restrict__ verdict_out,
                                                 uint32_t opts, uint32_t xg)
{
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x, xg);
    ipv4_packet<G, U, IPM, 0, 1>(arena, pkts, blk * (256u / G) + threadIdx.x / G, n, out, flags_out, verdict_out,
                                    opts);
}

// k_ipv4 with the packets handed out inside the workgroup: M * (256 / G)
// consecutive packets per workgroup, each lane group taking the next one
// (an LDS counter) as soon as its own is summed, so a group whose packet was
// short does not idle until the workgroup's longest packet is done.
template <int G, int U, int IPM, int M, int OCC = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC ? OCC : 1))) void k_ipv4_dyn(uint8_t *__restrict__ arena, const tcsum_pkt_t *__restrict__ pkts,
                                                  uint32_t n, uint32_t *__restrict__ out,
                                                  uint8_t *__restrict__ flags_out, int8_t *__restrict__ verdict_out,
                                                  uint32_t opts, uint32_t xg)
{
    constexpr uint32_t NG = 256u / G, PER = NG * (uint32_t)M;
    __shared__ uint32_t next;
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x, xg);
    const uint64_t first = (uint64_t)blk * PER;
    const uint32_t lim = n - first < PER ? (uint32_t)(n - first) : PER; // >= 1: grid = ceil(n / PER)
    if (threadIdx.x == 0)
        next = NG;
    __syncthreads();
    const uint32_t gl = threadIdx.x & (G - 1u), lead = threadIdx.x & 63u & ~(G - 1u);
    uint32_t k = threadIdx.x / G;
    while (k < lim) { // group-uniform; the group reductions stay inside the group
        ipv4_packet<G, U, IPM>(arena, pkts, (uint32_t)(first + k), n, out, flags_out, verdict_out, opts);
        uint32_t c = 0;
        if (gl == 0)
            c = atomicAdd(&next, 1u);
        k = (uint32_t)__shfl((int)c, (int)lead, 64);
    }
}

// k_ipv4 held to OCC waves per SIMD (the sums form takes 66 VGPRs, i.e. 7
// waves; rx 74, 6): measurement (libtcsum_bench.so, tcsum_probe_ipv4_shape)
template <int G, int U, int IPM, int OCC, int PIPE = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) void k_ipv4_occ(
    uint8_t *__restrict__ arena, const tcsum_pkt_t *__restrict__ pkts, uint32_t n, uint32_t *__restrict__ out,
    uint8_t *__restrict__ flags_out, int8_t *__restrict__ verdict_out, uint32_t opts, uint32_t xg)
{
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x, xg);
    ipv4_packet<G, U, IPM, 0, PIPE>(arena, pkts, blk * (256u / G) + threadIdx.x / G, n, out, flags_out, verdict_out,
                                    opts);
}

// Two packets per wave streamed as ONE run of chunks (measurement, round 6):
// the wave's 64 lanes walk packet A's chunks (from its 128-B line) and then
// packet B's in passes of 64 x U, so the pair takes ceil((chunks A + chunks
// B) / 64U) passes where k_ipv4's two 32-lane groups take the longer
// packet's ceil(chunks / 32U) -- on configs[3] 2.00 passes a wave against
// 2.44.  Lanes 0..31 load and parse A's header, 32..63 B's (as k_ipv4<32>'s
// groups do); the stream's per-packet bounds are read out to scalars; each
// lane keeps a header and an L4 sum per packet; lane 0 finishes A, lane 32 B.
template <int U, int IPM>
__device__ __forceinline__ void ipv4_pair(uint8_t *__restrict__ arena, const tcsum_pkt_t *__restrict__ pkts,
                                          uint32_t pa, uint32_t n, uint32_t *__restrict__ out,
                                          uint8_t *__restrict__ flags_out, int8_t *__restrict__ verdict_out,
                                          uint32_t opts)
{
    const uint32_t ln = threadIdx.x & 63u;
    const uint32_t pk = pa + (ln >> 5); // this lane's home packet: A (lanes 0..31) or B
    const bool live = pk < n;
    const u32x4 dv = *reinterpret_cast<const u32x4 *>(pkts + (live ? pk : 0u));
    const uint64_t off = (uint64_t)dv.x | ((uint64_t)dv.y << 32);
    const uint32_t frame = live ? dv.z : 0u;
    const bool big_enough = frame >= 20;
    uint8_t *pp = arena + off;
    const uintptr_t start = reinterpret_cast<uintptr_t>(pp);
    const uint32_t s0 = (uint32_t)(start & 15u);
    const u32x4 *base = reinterpret_cast<const u32x4 *>(pp - s0);
    const uint32_t frame_ld = frame < 65600u ? frame : 65600u;
    const uint32_t nch = big_enough ? (frame_ld + s0 + 15) >> 4 : 0u;
    const uint32_t sl = (uint32_t)(start & 127u);
    const uint32_t dch = big_enough ? (frame_ld + sl + 15) >> 4 : 0u;
    // the pair's stream: A's chunks [0, dA), then B's [dA, dA + dB)
    const uint32_t dA = (uint32_t)__builtin_amdgcn_readlane((int)dch, 0);
    const uint32_t dB = (uint32_t)__builtin_amdgcn_readlane((int)dch, 32);
    const uint32_t total = dA + dB;
    const uint64_t lineA = readlane64((uint64_t)(start - sl), 0), lineB = readlane64((uint64_t)(start - sl), 32);
    const u32x4 *la = reinterpret_cast<const u32x4 *>(lineA);
    const u32x4 *lb = reinterpret_cast<const u32x4 *>(lineB);
    auto chunk_at = [&](uint32_t c) -> const u32x4 * { // unconditional: past the end, the last chunk again
        if (total == 0u)
            return &g_zero_chunk;
        const uint32_t cc = c < total ? c : total - 1u;
        return cc < dA ? la + cc : lb + (cc - dA);
    };

    // fixed header of the home packet: bytes [s0, s0 + 20) of base[0..2]
    const u32x4 *hb = big_enough ? base : &g_zero_chunk;
    const uint32_t h1i = big_enough ? 1u : 0u;
    auto hload = [](const u32x4 *q) { return load16<false>(q); };
    u32x4 h0, h1, h2 = u32x4(0u), c2 = u32x4(0u), c3 = u32x4(0u);
    if constexpr (IPM == IP_RX) {
        h0 = hload(hb);
        h1 = hload(hb + h1i);
        c2 = hload(nch > 2 ? base + 2 : &g_zero_chunk);
        c3 = hload(nch > 3 && s0 >= 12 ? base + 3 : &g_zero_chunk);
        h2 = s0 > 12 ? c2 : u32x4(0u);
    } else {
        h0 = hload(hb);
        h1 = hload(hb + h1i);
        const u32x4 h2v = hload(hb + (big_enough ? (s0 > 12 ? 2u : 1u) : 0u));
        h2 = s0 > 12 ? h2v : u32x4(0u);
    }
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        v[u] = load16<true>(chunk_at((uint32_t)(u * 64) + ln));
    issue_fence();

    const Hdr5 hd = header_dwords(h0, h1, h2, s0);
    const IpHdr ih = ip_parse<IPM>(hd, frame, big_enough, [=](uint32_t ihl4) {
        const uint32_t o = s0 + ihl4, cw = o >> 4;
        u32x4 wa, wb;
        if (ihl4 == 20) {
            wa = cw == 1 ? h1 : c2;
            wb = cw == 1 ? c2 : c3;
        } else {
            wa = load16<false>(base + cw);
            wb = load16<false>(cw + 1 < nch ? base + cw + 1 : &g_zero_chunk);
        }
        return header_dwords(wa, wb, u32x4(0u), o & 15u);
    });
    // the home packet's byte ranges from its line base, then both packets' in scalars
    const int h_end = (int)(ih.hl < 65600u ? ih.hl : 65600u) + (int)sl;
    const int l_end = (int)(ih.end < 65600u ? ih.end : 65600u) + (int)sl;
    const int f0 = ih.field_on ? (int)(ih.hl + ih.fld) + (int)sl : -64;
    const int hA = __builtin_amdgcn_readlane(h_end, 0), hB = __builtin_amdgcn_readlane(h_end, 32);
    const int lA = __builtin_amdgcn_readlane(l_end, 0), lB = __builtin_amdgcn_readlane(l_end, 32);
    const int fA = __builtin_amdgcn_readlane(f0, 0), fB = __builtin_amdgcn_readlane(f0, 32);
    const int sA = __builtin_amdgcn_readlane((int)sl, 0), sB = __builtin_amdgcn_readlane((int)sl, 32);
    const bool onA = __builtin_amdgcn_readlane((int)ih.field_on, 0) != 0;
    const bool onB = __builtin_amdgcn_readlane((int)ih.field_on, 32) != 0;

    uint32_t ahA = 0, alA = 0, afA = 0, ahB = 0, alB = 0, afB = 0;
    auto pass = [&](const u32x4 (&vv)[U], uint32_t b0) {
        uint32_t phA = 0, plA = 0, phB = 0, plB = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t ci = b0 + (uint32_t)(u * 64) + ln;
            const bool valid = ci < total;
            const bool isA = ci < dA;
            const int c = (int)(16u * (isA ? ci : ci - dA));
            const int hs = isA ? sA : sB, he = isA ? hA : hB, le = isA ? lA : lB, fo = isA ? fA : fB;
            const bool on = isA ? onA : onB;
            const bool inner = valid && c >= he && c + 16 <= le && (fo + 2 <= c || fo >= c + 16);
            if (valid && !inner) { // header chunks, the field chunk(s), the last chunk: rare
                uint32_t th = region_sum(vv[u], c, hs, he);
                uint32_t tl4 = region_sum(vv[u], c, he, le);
                if (on) {
                    const uint32_t tf = region_sum(vv[u], c, fo, fo + 2);
                    if (IPM == IP_TX)
                        tl4 -= tf;
                    else if (isA)
                        afA += tf;
                    else
                        afB += tf;
                }
                if (IPM == IP_TX)
                    th -= region_sum(vv[u], c, hs + 10, hs + 12);
                phA += isA ? th : 0u;
                plA += isA ? tl4 : 0u;
                phB += isA ? 0u : th;
                plB += isA ? 0u : tl4;
            }
            const uint32_t w = chunk_sum_w(0u, vv[u], inner ? 0x00010001u : 0u); // < 2^19
            plA += isA ? w : 0u;
            plB += isA ? 0u : w;
        }
        ahA += phA;
        ahB += phB;
        alA = fold_step(alA + plA);
        alB = fold_step(alB + plB);
    };
    if (total)
        pass(v, 0u);
    for (uint32_t b0 = 64u * U; b0 < total; b0 += 64u * U) { // wave-uniform
        u32x4 w[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            w[u] = load16<true>(chunk_at(b0 + (uint32_t)(u * 64) + ln));
        pass(w, b0);
    }
    ahA = group_sum<64>(ahA);
    alA = group_sum<64>(alA);
    ahB = group_sum<64>(ahB);
    alB = group_sum<64>(alB);
    if (IPM == IP_RX) {
        afA = group_sum<64>(afA);
        afB = group_sum<64>(afB);
    }
    const bool home_b = ln >= 32u;
    if (live && (ln & 31u) == 0u)
        ip_finish<IPM>(ih, ih.fl, big_enough, (uint32_t)(start & 1u), home_b ? ahB : ahA, home_b ? alB : alA,
                       home_b ? afB : afA, pp, pk, out, flags_out, verdict_out, opts);
}

// ipv4_pair over the batch: 8 packets per 256-thread workgroup, as k_ipv4<32>
template <int U, int IPM>
__global__ __launch_bounds__(256) void k_ipv4_pair(uint8_t *__restrict__ arena, const tcsum_pkt_t *__restrict__ pkts,
                                                   uint32_t n, uint32_t *__restrict__ out,
                                                   uint8_t *__restrict__ flags_out, int8_t *__restrict__ verdict_out,
                                                   uint32_t opts, uint32_t xg)
{
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x, xg);
    ipv4_pair<U, IPM>(arena, pkts, (blk * 4u + (threadIdx.x >> 6)) * 2u, n, out, flags_out, verdict_out, opts);
}

// The deferred tx stores (IP_OPT_DEFER): one lane per packet writes the values
// k_ipv4 left in `csums` at the positions it left in `pos` (bit 16: the IPv4
// header field; low 16 bits: the L4 field's offset, 0 for none).  All the
// packets' field writes then reach memory in one short burst instead of one at
// a time through the read stream (u16 or nontemporal stores: no different;
// system-scope write-through stores: slower; profiles/r02/ab_tx_split*.txt).
// WARM (the packets in HBM): each lane first loads the dword under each of its
// fields and only then stores the 2 bytes.  A 2-B store into a line L2 does
// not hold cost ~140 us per 2M fields after the fill's read; into a line the
// load brought in, ~100 us including the load (profiles/r06/ab7/).  The loads
// stay inside the packet's own dwords; the stored bytes are the same.  Not for
// host memory (`store` across PCIe): a read there is a round trip.
template <bool WARM>
__global__ __launch_bounds__(256) void k_tx_scatter(uint8_t *__restrict__ arena, const tcsum_pkt_t *__restrict__ pkts,
                                                    uint32_t n, const uint32_t *__restrict__ csums,
                                                    const uint32_t *__restrict__ pos)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t q = pos[i];
    if (!q)
        return;
    const uint32_t v = csums[i];
    uint8_t *pp = arena + pkts[i].offset;
    const uint32_t f = q & 0xFFFFu;
    // WARM: the dwords holding bytes 10-11 and f..f+1 (f >= 22: both inside
    // the packet's first bytes), loaded before the stores; an empty asm after
    // the stores takes their value, so the loads are kept and the stores do
    // not wait for them (no side effect of the loaded bytes)
    uint32_t w0 = 0, w1 = 0;
    if constexpr (WARM) {
        const uint32_t m = (uint32_t)(reinterpret_cast<uintptr_t>(pp) & 3u);
        w0 = *reinterpret_cast<const uint32_t *>(pp + 8 - m);
        w1 = *reinterpret_cast<const uint32_t *>(pp + (((f ? f : 8u) + m) & ~3u) - m); // no L4 field: w0's again
    }
    pp[10] = (uint8_t)v; // ipv4.c:643,656, host order like the struct field
    pp[11] = (uint8_t)(v >> 8);
    if (f) { // tcp_out.c:19-20 / udp.c:320-321 / icmpv4.c:45-58
        pp[f] = (uint8_t)(v >> 16);
        pp[f + 1] = (uint8_t)(v >> 24);
    }
    if constexpr (WARM)
        asm volatile("" ::"v"(w0), "v"(w1));
}


// ---------------------------------------------------------------- byte-window stream (IPv4)
//
// k_ipv4 gives every packet its own lane group, so a pass of a 64..9000-B
// packet ends wherever the packet ends: lanes idle in the last pass, and the
// loads in flight follow the packet lengths.  k_flat_ipv4 cuts the batch's
// BYTES instead: workgroup w streams window w, a fixed WB-byte stretch of the
// arena (W waves x 64 lanes x U 16-B loads, the TSO kernel's load shape:
// 32-lane groups walking contiguous sub-ranges), whatever packets lie there,
// and sums each packet's part of it from prefix sums as k_segments_pk does:
//
//     P(x) = word sum of the window's bytes before x,
//     part(window, [A, B)) = P(min(B, end)) - P(max(A, start)),
//
// exact in u32 (a window sums to < 2^31), so padding and the neighbours'
// bytes cancel.  A packet belongs to the window its first byte lies in (its
// "owner"); the windows its later bytes reach add their parts to one 64-bit
// word per owner window with a single atomic -- folded part in the low half,
// an arrival count in the high half -- and the last to arrive finishes the
// packet (fold keeps "zero iff all bytes zero", and any regrouping of the
// words is allowed, so the folded parts add up to the packet's fold).  Every
// participant parses the packet's header itself (from the window's LDS copy
// of its chunks, or from memory for a header outside the window), so nothing
// else crosses workgroups.
//
// Which packets a window holds comes from k_flat_plan, one pass over the
// descriptors before the stream: wfirst[w] = the first packet starting at or
// after window w's first byte.  It also checks that the batch IS a stream --
// descriptors in arena order, packets disjoint, the whole span inside the
// grid the host sized from the byte hint -- and otherwise marks the plan
// (plan->bad = this call's generation number), and every workgroup then sums
// its share of the packets one by one (ipv4_packet), as k_ipv4 would.
struct FlatPlan {
    uint64_t base; // absolute address of window 0: the first packet's 128-B line
    uint64_t end;  // absolute end of the stream (the last packet's loaded bytes)
    uint32_t bad;  // == the call's generation: not a stream, per-packet mode
    uint32_t rsv;
};
constexpr uint32_t kFlatMaxFrame = 65600; // bytes of a frame the IPv4 kernels load (k_ipv4: frame_ld)

template <uint32_t WB>
__global__ __launch_bounds__(256) void k_flat_plan(const uint8_t *__restrict__ arena,
                                                   const tcsum_pkt_t *__restrict__ pkts, uint32_t n, uint32_t nw,
                                                   FlatPlan *__restrict__ plan, uint32_t *__restrict__ wfirst,
                                                   unsigned long long *__restrict__ slot, uint32_t gen)
{
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t < nw)
        slot[t] = 0ull;
    if (t > n)
        return;
    const uint64_t a0 = reinterpret_cast<uintptr_t>(arena);
    const uint64_t base = (a0 + pkts[0].offset) & ~127ull;
    if (t == 0)
        plan->base = base;
    const uint64_t cover = (uint64_t)nw * WB;
    bool bad = false;
    uint64_t lo; // the windows whose first packet is t: (window of packet t-1's start, window of t's start]
    if (t == 0) {
        lo = 0;
    } else {
        const uint64_t sp = a0 + pkts[t - 1].offset;
        lo = sp >= base ? (sp - base) / WB + 1u : ~0ull;
    }
    uint64_t hi = nw;
    if (t < n) {
        const tcsum_pkt_t d = pkts[t];
        const uint64_t st = a0 + d.offset;
        if (st < base) {
            bad = true;
        } else {
            hi = (st - base) / WB;
            if (t + 1u < n && a0 + pkts[t + 1].offset < st + d.len) // arena order, disjoint
                bad = true;
            if (t + 1u == n) {
                const uint64_t e = st + (d.len < kFlatMaxFrame ? d.len : kFlatMaxFrame);
                plan->end = e;
                if (e - base > cover)
                    bad = true;
            }
        }
    }
    if (!bad && lo <= hi) {
        if (hi - lo > nw)
            bad = true;
        else
            for (uint64_t w = lo; w <= hi && w <= nw; ++w)
                wfirst[w] = t;
    }
    if (bad)
        plan->bad = gen;
}

// A 16-B chunk through the scalar data cache (reads only): the load waits on
// lgkmcnt, not on the vector loads issued before it, so a value a workgroup
// needs right after its window arrives can be fetched beside the window.
// The wait is inside: the wave stalls only until this load returns, while
// its window's vector loads stay in flight.  p must be uniform and 4-B
// aligned.
__device__ __forceinline__ u32x4 sload16(const void *p)
{
    u32x4 v;
    asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
    return v;
}

// Byte `i` (0..15) of a chunk (selects on named dwords: no dynamic indexing)
__device__ __forceinline__ uint32_t chunk_byte(u32x4 v, uint32_t i)
{
    const uint32_t q = i >> 2;
    const uint32_t d = q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
    return (d >> (8u * (i & 3u))) & 0xFFu;
}

// PROBE (measurement builds, libtcsum_bench.so): 1 = the plan read and the
// window's loads only (XOR-folded into a sink stored on a 2^-32 fluke); 2 =
// + the scans and the LDS copy, no packets; 3 = everything but the atomic
// (a crossing packet is finished by each window with its own part: wrong
// values, the cost without the combine).
template <int IPM, int W, int U, int PROBE = 0>
__global__ __launch_bounds__(W * 64) void k_flat_ipv4(uint8_t *__restrict__ arena,
                                                      const tcsum_pkt_t *__restrict__ pkts, uint32_t n,
                                                      uint32_t *__restrict__ out, uint8_t *__restrict__ flags_out,
                                                      int8_t *__restrict__ verdict_out, uint32_t opts, uint32_t xg,
                                                      const FlatPlan *__restrict__ plan,
                                                      const uint32_t *__restrict__ wfirst,
                                                      unsigned long long *__restrict__ slot, uint32_t gen)
{
    static_assert(2 * W <= 32, "the sub-range totals are scanned by 32 lanes");
    constexpr uint32_t T = W * 64u, CH = T * U, SR = 32u * U, WB = 16u * CH;
    // the window's chunks (headers, boundary bytes), then kHalo chunks past
    // its end (the headers of packets that start in its last bytes), then the
    // straddler's first kHalo chunks: every chunk a packet's parse reads is
    // one LDS read (max. chunk 5: s0 + IHL*4 + the L4 field's 2 bytes <= 92)
    constexpr uint32_t kHalo = 6;
    __shared__ u32x4 dat[CH + 2 * kHalo];
    __shared__ uint32_t ex[CH]; // per chunk: its sub-range's word sum before it; slot 0 of a sub-range: its total
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x, xg);
    const uint64_t a0 = reinterpret_cast<uintptr_t>(arena);
    if (plan->bad == gen) {
        // not a stream: this workgroup's share of the packets, one by one
        const uint32_t lo = (uint32_t)((uint64_t)n * blk / gridDim.x);
        const uint32_t hi = (uint32_t)((uint64_t)n * (blk + 1u) / gridDim.x);
        constexpr uint32_t G = 16, PER = T / G; // 2 loads per lane: the stream's register budget
        for (uint32_t p0 = lo; p0 < hi; p0 += PER) // workgroup-uniform
            ipv4_packet<G, 2, IPM>(arena, pkts, p0 + t / G, hi, out, flags_out, verdict_out, opts);
        return;
    }
    const uint64_t base = plan->base, send = plan->end;
    const uint64_t wlo = base + (uint64_t)blk * WB;
    if (wlo >= send) // past the stream (the grid is sized from the byte hint)
        return;
    // the window's loads: chunk c of the window is load u of lane l of
    // sub-range c / SR; chunks past the stream re-read its last chunk (their
    // bytes belong to no packet)
    const int64_t rel0 = (int64_t)(wlo - a0); // from the arena pointer: global_load, not flat_load
    const u32x4 *wbase = reinterpret_cast<const u32x4 *>(arena + rel0);
    const uint64_t nchx = (send - wlo + 15u) >> 4; // chunks to the stream's end
    const uint32_t nchw = nchx >= CH ? CH : (uint32_t)nchx;
    const uint32_t sub = t >> 5, l = t & 31u, hf = (t >> 5) & 1u;
    u32x4 v[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
        const uint32_t c = sub * SR + u * 32u + l;
        v[u] = load16<true>(wbase + (c < nchw ? c : nchw - 1u));
    }
    // the halo: wave 0's first lanes, default policy (the next window's
    // workgroup streams the same line at about the same time, on the same XCD)
    u32x4 hv = u32x4(0u);
    if (wv == 0 && lane < kHalo) {
        const uint64_t c = CH + lane;
        hv = load16<false>(wbase + (c < nchx ? c : nchx - 1u));
    }
    issue_fence();
    if constexpr (PROBE == 1) {
        u32x4 z = v[0];
#pragma unroll
        for (uint32_t u = 1; u < U; ++u)
            z ^= v[u];
        if ((z.x ^ z.y ^ z.z ^ z.w) == 0x9E3779B9u)
            out[0] = z.x;
        return;
    }
    // the packets: the straddler from the left (if any) and those starting here
    const uint32_t pf = wfirst[blk], pl = wfirst[blk + 1u];
    const uint32_t j0 = pf > 0 ? pf - 1u : 0u;
    const uint32_t m = pl - j0;
    // The straddler's header lies before this window: its descriptor and first
    // 96 bytes through the scalar cache now, while the window is in flight
    // (fetched after the barrier they put a whole memory latency into every
    // workgroup's tail: 687 -> 1169 us on configs[3], profiles/r04/flat/).
    // (six named chunks, not an array: captured into the fetch lambda below,
    // an array went to scratch memory)
    u32x4 sh0 = u32x4(0u), sh1 = u32x4(0u), sh2 = u32x4(0u), sh3 = u32x4(0u), sh4 = u32x4(0u), sh5 = u32x4(0u);
    if (pf > 0 && wv == 0) { // wave-uniform: wave 0 takes the packets
        const u32x4 sd = sload16(pkts + (pf - 1u));
        const uint64_t ss = a0 + ((uint64_t)sd.x | ((uint64_t)sd.y << 32));
        const uint32_t sfl = sd.z < kFlatMaxFrame ? sd.z : kFlatMaxFrame;
        if (sd.z >= 20 && ss + sfl > wlo) { // a header to parse, and bytes in this window
            const uint64_t c0 = ss & ~15ull, se = ss + sfl; // the packet's own chunks only
            const int64_t r0 = (int64_t)(c0 - a0);
            sh0 = sload16(arena + r0);
            if (c0 + 16u < se)
                sh1 = sload16(arena + r0 + 16);
            if (c0 + 32u < se)
                sh2 = sload16(arena + r0 + 32);
            if (c0 + 48u < se)
                sh3 = sload16(arena + r0 + 48);
            if (c0 + 64u < se)
                sh4 = sload16(arena + r0 + 64);
            if (c0 + 80u < se)
                sh5 = sload16(arena + r0 + 80);
        }
    }
    // packet i of the window goes to lane i % 64 of wave 0: the packet phase
    // is instruction-bound, not load-bound (one pass of it per wave per
    // window), so the other waves leave after the scans
    // (profiles/r04/flat/: packets spread over all W waves cost 4x the issue
    // slots and ran at 2x the stream's time)
    const uint32_t i0 = lane;
    u32x4 dv0 = u32x4(0u);
    if (wv == 0 && i0 < m)
        dv0 = *reinterpret_cast<const u32x4 *>(pkts + j0 + i0);

    // chunk sums, scans over each 32-lane half, the chunks and prefixes into LDS
    {
        uint32_t a = 0;
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t c = sub * SR + u * 32u + l;
            const uint32_t f = chunk_sum(0u, v[u]); // < 2^19
            const uint32_t sc = scan32(f);
            if (u != 0 || l != 0)
                ex[c] = a + (sc - f);
            dat[c] = v[u];
            const uint32_t lo32 = (uint32_t)__builtin_amdgcn_readlane((int)sc, 31);
            const uint32_t hi32 = (uint32_t)__builtin_amdgcn_readlane((int)sc, 63);
            a += hf ? hi32 : lo32;
        }
        if (l == 0)
            ex[sub * SR] = a; // the sub-range's total (its first chunk's prefix is 0)
    }
    if (wv == 0 && lane < 2u * kHalo) { // the halo and the straddler's chunks
        const uint32_t k = lane >= kHalo ? lane - kHalo : lane;
        const u32x4 sk = k == 0 ? sh0 : k == 1 ? sh1 : k == 2 ? sh2 : k == 3 ? sh3 : k == 4 ? sh4 : sh5;
        dat[CH + lane] = lane < kHalo ? hv : sk;
    }
    __syncthreads();
    if constexpr (PROBE == 2) {
        if (ex[(t * 37u) % CH] == 0x9E3779B9u && dv0.x == 1u)
            out[0] = 1u;
        return;
    }
    if (wv != 0)
        return;
    // the sub-ranges' exclusive prefixes (lane k: sub-range k)
    const uint32_t st = lane < 2u * W ? ex[lane * SR] : 0u;
    const uint32_t si = scan32(st);
    const uint32_t sx = si - st;
    const uint32_t wtot = (uint32_t)__builtin_amdgcn_readlane((int)si, 31);
    // P(x), x = 0..WB bytes from the window's start; called by every lane of
    // the wave (the shuffle), x = 0 for lanes without a packet
    auto prefix = [=](uint32_t x) -> uint32_t {
        const uint32_t c = x >> 4, b = x & 15u;
        const uint32_t cc = c < CH ? c : CH - 1u;
        const uint32_t sp = (uint32_t)__shfl((int)sx, (int)(cc / SR), 64);
        if (c >= CH)
            return wtot;
        uint32_t e = sp + (cc % SR ? ex[cc] : 0u);
        if (b)
            e += chunk_prefix_sum(dat[cc], b);
        return e;
    };
    const uint64_t whi = wlo + WB;
    const uint32_t rounds = (m + 63u) / 64u; // wave-uniform
    for (uint32_t r = 0; r < rounds; ++r) {
        const uint32_t i = r * 64u + i0;
        const bool act = i < m;
        const u32x4 dv = r == 0 ? dv0 : (act ? *reinterpret_cast<const u32x4 *>(pkts + j0 + i) : u32x4(0u));
        const uint32_t j = j0 + i;
        const uint64_t off = (uint64_t)dv.x | ((uint64_t)dv.y << 32);
        const uint32_t frame = act ? dv.z : 0u;
        const uint64_t s = a0 + off;
        const uint32_t frame_ld = frame < kFlatMaxFrame ? frame : kFlatMaxFrame;
        const uint64_t ee = s + frame_ld;
        // this window takes part: the packet starts here, or (packet j0 = pf - 1)
        // reaches in from the left
        const bool straddler = i == 0 && pf > 0;
        const bool part_of = act && (!straddler || ee > wlo);
        const bool owner = act && s >= wlo && s < whi;
        const bool big_enough = frame >= 20;
        const uint32_t s0 = (uint32_t)(s & 15u);
        const uint64_t hc = s >> 4; // the packet's first chunk (absolute)
        const uint32_t nchp = big_enough ? (frame_ld + s0 + 15u) >> 4 : 0u; // the packet's chunks
        // chunk k (< kHalo) of the packet: an owner's from the window's copy
        // (and the halo), the straddler's from its prefetched header
        const uint32_t hb = straddler ? CH + kHalo : owner ? (uint32_t)(hc - (wlo >> 4)) : 0u;
        auto fetch = [=](uint32_t k) -> u32x4 {
            return part_of && k < nchp ? dat[hb + k] : u32x4(0u);
        };
        const u32x4 h0 = fetch(0), h1 = fetch(1);
        const u32x4 h2 = s0 > 12 ? fetch(2) : u32x4(0u);
        const Hdr5 hd = header_dwords(h0, h1, h2, s0);
        // rx: the TCP/UDP header's first 16 bytes, fetched before the parse (a
        // fetch inside its callback kept the closure in scratch memory)
        u32x4 wa = u32x4(0u), wb = u32x4(0u);
        const uint32_t ol4 = s0 + ((hd.d0 & 0xFu) << 2);
        if (IPM == IP_RX) {
            wa = fetch(ol4 >> 4);
            wb = fetch((ol4 >> 4) + 1u);
        }
        const IpHdr ih = ip_parse<IPM>(hd, frame, big_enough,
                                       [=](uint32_t) { return header_dwords(wa, wb, u32x4(0u), ol4 & 15u); });
        // the L4 range's part in this window
        const uint64_t A = s + ih.hl, B = s + ih.end;
        const uint32_t xa = A <= wlo ? 0u : A >= whi ? WB : (uint32_t)(A - wlo);
        const uint32_t xb = B <= wlo ? 0u : B >= whi ? WB : (uint32_t)(B - wlo);
        const bool sums = part_of && big_enough;
        uint32_t part = prefix(sums ? xb : 0u) - prefix(sums ? xa : 0u);
        // the L4 checksum field: its bytes (tx subtracts those in this window:
        // the fill reads it as zero; rx tests whether it is zero)
        uint32_t acc_f = 0;
        if (sums && ih.field_on) {
#pragma unroll
            for (uint32_t k = 0; k < 2; ++k) {
                const uint32_t q = s0 + ih.hl + ih.fld + k; // from the packet's first chunk
                const uint32_t b = chunk_byte(fetch(q >> 4), q & 15u);
                const uint64_t F = s + ih.hl + ih.fld + k;
                if (IPM == IP_TX && F >= wlo && F < whi)
                    part -= b << (8u * (uint32_t)(F & 1u));
                acc_f |= b;
            }
        }
        if (!part_of || (!big_enough && !owner))
            continue;
        // windows this packet's bytes reach: its owner's and the ones after it
        const uint64_t ws = (s - base) / WB;
        const uint32_t kwin = frame_ld ? (uint32_t)((ee - 1u - base) / WB - ws + 1u) : 1u;
        uint32_t acc_l = part;
        if (PROBE != 3 && big_enough && kwin > 1u) {
            const uint32_t fp = fold16(part);
            const unsigned long long old =
                atomicAdd(&slot[ws], (1ull << 32) | (unsigned long long)fp);
            if ((uint32_t)(old >> 32) + 1u != kwin)
                continue; // another window finishes the packet
            acc_l = (uint32_t)old + fp;
        }
        // the finisher: the header sum from the packet's first chunks
        uint32_t acc_h = 0;
        if (big_enough) {
            const int h_end = (int)(s0 + ih.hl);
#pragma unroll
            for (uint32_t k = 0; k < 5; ++k) {
                if ((int)(16u * k) < h_end) {
                    const u32x4 hk = fetch(k);
                    uint32_t th = region_sum(hk, (int)(16u * k), (int)s0, h_end);
                    if (IPM == IP_TX)
                        th -= region_sum(hk, (int)(16u * k), (int)s0 + 10, (int)s0 + 12); // ipv4.c:643
                    acc_h += th;
                }
            }
        }
        ip_finish<IPM>(ih, ih.fl, big_enough, (uint32_t)(s & 1u), acc_h, acc_l, acc_f, arena + off, j, out,
                       flags_out, verdict_out, opts);
    }
}

} // namespace tcsum
