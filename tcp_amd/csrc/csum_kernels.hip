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
#include "csum_launch.h"

#include <stdlib.h>
#include <string.h>

#include <mutex>

namespace tcsum {

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

// One wave-slice of packets per wave, one launch-wide pass.
//
// Results leave through the workgroup's LAST wave: each wave puts its packets'
// u16 into LDS and bumps an LDS counter; the wave that brings it to 4 stores
// all 256/G results with one coalesced store and the other three end at once.
// With every wave storing its own 4 results (an 8-byte partial store each) the
// headline ran 1.1 % slower -- as slow as its loads plus the stores' tail in
// every wave; with the gathered store it matches the same kernel with no
// store at all (profiles/r02/ab_store.txt).  A nontemporal store cost 4 %.
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
    const SegDesc d = load_desc<MODE>(descs, seg, live);
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
// scripts/wg_shape_ab.py): GL = 0 interleaves the whole workgroup (load u of
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
template <int MODE, int G, int UL = 4>
__device__ __forceinline__ void pk_ranges(const uint8_t *__restrict__ arena, const void *__restrict__ descs,
                                          uint16_t *__restrict__ out, uint32_t aux, uint32_t first, uint32_t kw,
                                          uint32_t T)
{
    const uint32_t t = threadIdx.x, gl = t & (G - 1u);
    for (uint32_t r = t / G; r < kw; r += T / G) {
        const SegDesc e = load_desc<MODE>(descs, first + r, true);
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
    if (ranges) { // G lanes per range: the widest power of two that gives every range a group
        const uint32_t lanes_per = T / kw;
        if (lanes_per >= 64)
            pk_ranges<MODE, 64>(arena, descs, out, aux, first, kw, T);
        else if (lanes_per >= 32)
            pk_ranges<MODE, 32, 3>(arena, descs, out, aux, first, kw, T);
        else if (lanes_per >= 16)
            pk_ranges<MODE, 16>(arena, descs, out, aux, first, kw, T);
        else
            pk_ranges<MODE, 8>(arena, descs, out, aux, first, kw, T);
        return;
    }
    if (mine)
        out[first + rr] = finalize<MODE>(pe - ps, reinterpret_cast<uintptr_t>(arena + d.off), d, aux, q16);
}

// Persistent form: a resident grid walks the batch; each wave prefetches its
// next descriptor while the current packets' bytes are in flight, so the
// descriptor -> data dependence costs one latency per wave, not per packet.
template <int G, int U, int MODE>
__global__ __launch_bounds__(256) void k_segments_p(const uint8_t *__restrict__ arena,
                                                    const void *__restrict__ descs, uint32_t n,
                                                    uint16_t *__restrict__ out, uint32_t aux)
{
    constexpr uint32_t PER_WAVE = 64 / G;
    const uint32_t gl = threadIdx.x & (G - 1);
    const uint32_t wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t step = gridDim.x * 4u * PER_WAVE;
    uint32_t seg = wave * PER_WAVE + ((threadIdx.x & 63u) / G);
    SegDesc d = load_desc<MODE>(descs, seg, seg < n);
    for (uint32_t first = wave * PER_WAVE; first < n; first += step) { // wave-uniform
        const uint32_t nseg = seg + step;
        SegDesc nd{0, 0, 0, 0, 0, 0};
        uint32_t acc = sum_range<G, U, MODE == MODE_EXACT>(arena, d.off, d.len, gl,
                                                           [&] { nd = load_desc<MODE>(descs, nseg, nseg < n); });
        acc = group_sum<G>(acc);
        if (seg < n && gl == 0)
            out[seg] = finalize<MODE>(acc, reinterpret_cast<uintptr_t>(arena + d.off), d, aux,
                                      MODE == MODE_PESO ? peso_pseudo16(d) : 0u);
        seg = nseg;
        d = nd;
    }
}

// Pipelined persistent form: each wave keeps TWO ranges' loads in flight.
// Descriptors run two ranges ahead and are issued before the data loads that
// need the previous one, so with in-order vmcnt every wait is a counted one:
//   order: d[i+2], L[i+1], (wait L[i]) sum, store
// and the bytes of range i+1 stream while range i is summed.  The loop is
// unrolled by two with two named frames: copying a frame whose loads are in
// flight would force a wait on them (a v_mov of a pending register).
template <int G, int U, int MODE>
__device__ __forceinline__ void finish_range(Frame<U> &f, const SegDesc &d, uint32_t seg, uint32_t n,
                                             uint32_t gl, const uint8_t *__restrict__ arena,
                                             uint16_t *__restrict__ out, uint32_t aux)
{
    uint32_t acc = frame_consume<G, U, MODE == MODE_EXACT>(f, gl);
    acc = group_sum<G>(acc);
    if (seg < n && gl == 0)
        out[seg] = finalize<MODE>(acc, reinterpret_cast<uintptr_t>(arena + d.off), d, aux,
                                  MODE == MODE_PESO ? peso_pseudo16(d) : 0u);
}

template <int G, int U, int MODE>
__global__ __launch_bounds__(256) void k_segments_pp(const uint8_t *__restrict__ arena,
                                                     const void *__restrict__ descs, uint32_t n,
                                                     uint16_t *__restrict__ out, uint32_t aux)
{
    constexpr uint32_t PER_WAVE = 64 / G;
    const uint32_t gl = threadIdx.x & (G - 1);
    const uint32_t wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t step = gridDim.x * 4u * PER_WAVE;
    uint32_t seg = wave * PER_WAVE + ((threadIdx.x & 63u) / G);
    uint32_t first = wave * PER_WAVE; // wave-uniform loop control
    Frame<U> fa, fb;
    SegDesc d0 = load_desc<MODE>(descs, seg, seg < n);
    SegDesc d1 = load_desc<MODE>(descs, seg + step, seg + step < n);
    frame_issue<G, U>(fa, arena, d0.off, d0.len, gl);
    while (first < n) {
        // fa in flight for d0, d1 loading
        const SegDesc d2 = load_desc<MODE>(descs, seg + 2 * step, seg + 2 * step < n);
        frame_issue<G, U>(fb, arena, d1.off, d1.len, gl);
        issue_fence();
        finish_range<G, U, MODE>(fa, d0, seg, n, gl, arena, out, aux);
        seg += step;
        first += step;
        if (first >= n)
            break;
        // fb in flight for d1, d2 loading
        const SegDesc d3 = load_desc<MODE>(descs, seg + 2 * step, seg + 2 * step < n);
        frame_issue<G, U>(fa, arena, d2.off, d2.len, gl);
        issue_fence();
        finish_range<G, U, MODE>(fb, d1, seg, n, gl, arena, out, aux);
        seg += step;
        first += step;
        // back to: fa in flight for d0 := d2, d1 := d3 loading (descriptor
        // copies wait only for themselves: they were issued before fa's loads)
        d0 = d2;
        d1 = d3;
    }
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
// short launch (tx fill)
constexpr uint32_t IP_OPT_DEFER = 2u;
// launch_ipv4 mode 3: IP_TX kernels with IP_OPT_NO_STORE
constexpr int IP_TX_OFFLOAD = 3;
// launch_ipv4 mode 4: the tx fill as k_ipv4<IP_TX> with IP_OPT_DEFER + k_tx_scatter
constexpr int IP_TX_SPLIT = 4;

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

// Packet `pk` (one per G-lane group; pk >= n: a dead group that reads
// descriptor 0 and writes nothing).  Every lane of the wave must call it: the
// group reduction crosses lanes.
template <int G, int U, int IPM>
__device__ __forceinline__ void ipv4_packet(uint8_t *__restrict__ arena, const tcsum_pkt_t *__restrict__ pkts,
                                            uint32_t pk, uint32_t n, uint32_t *__restrict__ out,
                                            uint8_t *__restrict__ flags_out, int8_t *__restrict__ verdict_out,
                                            uint32_t opts)
{
    const uint32_t gl = threadIdx.x & (G - 1);
    const bool live = pk < n;

    // unconditional loads throughout (dead lanes read descriptor 0 / the zero chunk)
    const u32x4 dv = *reinterpret_cast<const u32x4 *>(pkts + (live ? pk : 0u));
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
    const u32x4 h0 = hload(hb);
    const u32x4 h1 = hload(hb + h1i);
    u32x4 h2, c2 = u32x4(0u), c3 = u32x4(0u);
    if constexpr (IPM == IP_RX) {
        // chunks 2 and 3 as well: an IHL-5 packet's TCP/UDP ports, data offset
        // and flags (L4 bytes 0-3, 12-13) lie in chunks 1..3
        c2 = hload(nch > 2 ? base + 2 : &g_zero_chunk);
        c3 = hload(nch > 3 && s0 >= 12 ? base + 3 : &g_zero_chunk);
        h2 = s0 > 12 ? c2 : u32x4(0u);
    } else {
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
    const uint32_t sl = (uint32_t)(start & 127u);
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
    issue_fence();

    const Hdr5 hd = header_dwords(h0, h1, h2, s0);
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
            // the header words (L4 bytes 0-3: ports; 12-15: data offset,
            // flags) from the 32 bytes at chunk (s0 + ihl4) / 16: chunks 1..3
            // already in registers for IHL 5, two more loads otherwise
            uint32_t ports = 0, oflags = 0;
            if (tl >= ihl4 + 8u) {
                const uint32_t o = s0 + ihl4, cw = o >> 4;
                u32x4 wa, wb;
                if (ihl4 == 20) {
                    wa = cw == 1 ? h1 : c2;
                    wb = cw == 1 ? c2 : c3;
                } else {
                    wa = load16<false>(base + cw);
                    wb = load16<false>(cw + 1 < nch ? base + cw + 1 : &g_zero_chunk);
                }
                const Hdr5 l4h = header_dwords(wa, wb, u32x4(0u), o & 15u);
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
    acc_h = group_sum<G>(acc_h);
    acc_l = group_sum<G>(acc_l);
    if (IPM == IP_RX)
        acc_f = group_sum<G>(acc_f);

    if (live && gl == 0) {
        uint32_t ip = 0, l4 = 0;
        if (!big_enough) {
            fl = TCSUM_PKT_SHORT;
        } else {
            const bool odd = start & 1u;
            uint32_t fh = fold16(acc_h);
            uint32_t f4 = fold16(acc_l);
            if (odd) {
                fh = rot8(fh);
                f4 = rot8(f4);
            }
            ip = ~fh & 0xFFFFu;
            if (proto == 6 || proto == 17)
                l4 = ~fold_step(f4 + pseudo) & 0xFFFFu;
            else if (proto == 1)
                l4 = ~f4 & 0xFFFFu;
        }
        if constexpr (IPM == IP_TX) {
            if (opts & IP_OPT_DEFER) // bit 16: the IPv4 field; low 16: the L4 field's offset (0: none)
                reinterpret_cast<uint32_t *>(verdict_out)[pk] = bad ? 0u : (1u << 16) | (field_on ? hl + fld : 0u);
            else if (!bad && !(opts & IP_OPT_NO_STORE)) { // stored in host order, like the struct fields
                pp[10] = (uint8_t)ip;
                pp[11] = (uint8_t)(ip >> 8);
                if (field_on) {
                    pp[hl + fld] = (uint8_t)l4;
                    pp[hl + fld + 1] = (uint8_t)(l4 >> 8);
                }
            }
        }
        if constexpr (IPM == IP_RX) {
            // The first gate that rejects, in the reference's order: ipv4_in /
            // is_pkt_ok, then the L4 input ip_normal_in dispatches to
            // (ipv4.c:420-470), up to socket lookup.  Pinned by the reference
            // stack's own verdicts (tests/golden/ipv4_rx_*, oracle/stack_gen.c).
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
}

template <int G, int U, int IPM, int T = 256>
__global__ __launch_bounds__(T) void k_ipv4(uint8_t *__restrict__ arena, const tcsum_pkt_t *__restrict__ pkts,
                                            uint32_t n, uint32_t *__restrict__ out,
                                            uint8_t *__restrict__ flags_out, int8_t *__restrict__ verdict_out,
                                            uint32_t opts, uint32_t xg)
{
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x, xg);
    ipv4_packet<G, U, IPM>(arena, pkts, blk * (uint32_t)(T / G) + threadIdx.x / G, n, out, flags_out, verdict_out,
                           opts); // no 32-bit wrap for any n
}

// The deferred tx stores (IP_OPT_DEFER): one lane per packet writes the values
// k_ipv4 left in `csums` at the positions it left in `pos` (bit 16: the IPv4
// header field; low 16 bits: the L4 field's offset, 0 for none).  All the
// packets' field writes then reach memory in one short burst instead of one at
// a time through the read stream (u16 or nontemporal stores: no different;
// system-scope write-through stores: slower; profiles/r02/ab_tx_split*.txt).
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
    pp[10] = (uint8_t)v; // ipv4.c:643,656, host order like the struct field
    pp[11] = (uint8_t)(v >> 8);
    const uint32_t f = q & 0xFFFFu;
    if (f) { // tcp_out.c:19-20 / udp.c:320-321 / icmpv4.c:45-58
        pp[f] = (uint8_t)(v >> 16);
        pp[f + 1] = (uint8_t)(v >> 24);
    }
}

// k_ipv4's loads and nothing else (measurement: tcsum_probe_ipv4): the 16-B
// descriptor, the two or three default-policy header chunks (four for rx),
// the line-aligned nontemporal data pass -- same lanes, same clamping, same
// XCD order -- folded by XOR into a sink stored on a 2^-32 fluke.  The rate
// the IPv4 kernels would run at if their arithmetic and stores were free.
// PM_TX adds exactly the deferred tx fill's writes (the ceiling for a kernel
// that must write): every packet's 8 bytes of scratch -- a value word and the
// field positions k_ipv4<IP_TX> derives from the header (same rules) -- and
// then k_tx_scatter, the product's own scatter, writing the fields.  The
// values are the XOR fold, so the packets' checksum fields end up junk.
enum ProbeMode : int { PM_SUMS = 0, PM_RX = 1, PM_TX = 2 };
template <int G, int U, int PM>
__global__ __launch_bounds__(256) void k_probe_ipv4(const uint8_t *__restrict__ arena,
                                                    const tcsum_pkt_t *__restrict__ pkts, uint32_t n,
                                                    uint32_t *__restrict__ sink, uint32_t xg,
                                                    uint32_t *__restrict__ vals, uint32_t *__restrict__ posv)
{
    constexpr bool RX = PM == PM_RX;
    const uint32_t gl = threadIdx.x & (G - 1);
    const uint32_t pk = xcd_block(blockIdx.x, gridDim.x, xg) * (256u / G) + threadIdx.x / G;
    const bool live = pk < n;
    const u32x4 dv = *reinterpret_cast<const u32x4 *>(pkts + (live ? pk : 0u));
    const uint64_t off = (uint64_t)dv.x | ((uint64_t)dv.y << 32);
    const uint32_t frame = live ? dv.z : 0u;
    const bool big_enough = frame >= 20;
    const uint8_t *pp = arena + off;
    const uintptr_t start = reinterpret_cast<uintptr_t>(pp);
    const uint32_t s0 = (uint32_t)(start & 15u);
    const u32x4 *base = reinterpret_cast<const u32x4 *>(pp - s0);
    const uint32_t frame_ld = frame < 65600u ? frame : 65600u;
    const uint32_t nch = big_enough ? (frame_ld + s0 + 15) >> 4 : 0u;
    const u32x4 *hb = big_enough ? base : &g_zero_chunk;
    const u32x4 h0 = load16<false>(hb);
    const u32x4 h1 = load16<false>(hb + (big_enough ? 1u : 0u));
    u32x4 h2;
    if constexpr (RX) {
        const u32x4 c2 = load16<false>(nch > 2 ? base + 2 : &g_zero_chunk);
        const u32x4 c3 = load16<false>(nch > 3 && s0 >= 12 ? base + 3 : &g_zero_chunk);
        h2 = c2 ^ c3;
    } else {
        h2 = load16<false>(hb + (big_enough ? (s0 > 12 ? 2u : 1u) : 0u));
    }
    const uint32_t sl = (uint32_t)(start & 127u);
    const uint32_t dch = big_enough ? (frame_ld + sl + 15) >> 4 : 0u;
    const u32x4 *dbase = dch ? reinterpret_cast<const u32x4 *>(pp - sl) : &g_zero_chunk;
    const uint32_t dlast = dch ? dch - 1u : 0u;
    u32x4 x = h0 ^ h1 ^ h2;
    for (uint32_t b0 = 0; b0 < (dch ? dch : 1u); b0 += G * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t idx = b0 + u * G + gl;
            x ^= load16<true>(dbase + (idx < dch ? idx : dlast));
        }
    }
    const uint32_t acc = x.x ^ x.y ^ x.z ^ x.w;
    if constexpr (PM == PM_TX) {
        // the positions k_ipv4<IP_TX> stores with IP_OPT_DEFER (ipv4_packet)
        const Hdr5 hd = header_dwords(h0, h1, h2, s0);
        const uint32_t b0h = hd.d0 & 0xFFu, ihl4 = (b0h & 0xFu) << 2;
        const uint32_t tl = (((hd.d0 >> 16) & 0xFFu) << 8) | (hd.d0 >> 24);
        const uint32_t b6 = (hd.d1 >> 16) & 0xFFu, b7 = hd.d1 >> 24;
        const bool frag = (b6 & 0x20u) || (((b6 & 0x1Fu) << 8) | b7);
        const uint32_t proto = (hd.d2 >> 8) & 0xFFu;
        const bool bad = !big_enough || (b0h >> 4) != 4 || ihl4 < 20 || ihl4 > frame || tl < 20 || tl > frame ||
                         tl < ihl4;
        uint32_t hl = ihl4 < 20 ? 20u : ihl4;
        hl = hl > frame ? frame : hl;
        uint32_t end = tl < hl ? hl : tl;
        end = end > frame ? frame : end;
        uint32_t min_l4;
        const uint32_t fld = l4_field(proto, min_l4);
        const bool field_on = !bad && !frag && fld && end - hl >= min_l4;
        if (live && gl == 0) {
            vals[pk] = acc;
            posv[pk] = bad ? 0u : (1u << 16) | (field_on ? hl + fld : 0u);
        }
    } else if (acc == 0x9E3779B9u) {
        sink[0] = acc;
    }
}

// ---------------------------------------------------------------- queue server
//
// A resident grid that serves small host-queue batches without a launch and
// a stream sync per batch (tcsum_queue_server, include/tcsum.h).  The host
// posts one job at a time into pinned, coherent memory (SrvHost: job fields,
// then `req`); workgroup 0 polls `req` over PCIe with one lane and s_sleep,
// copies the job into device memory (SrvCtl, agent-scope atomics) and bumps
// SrvCtl::seq; the other workgroups poll that word (relaxed, s_sleep), take
// ONE system-scope acquire (their L1/L2 may hold host lines from the last
// job), and every workgroup sums its share of the packets.  Each workgroup
// drains its stores, releases them at system scope (results and tx bytes live
// in host memory) and adds to SrvCtl::arrivals; the last arriver writes
// SrvHost::done.  Exit: workgroup 0 alone decides -- host `quit`, or no job
// for `idle_ticks` of the 100 MHz real-time clock -- and publishes
// SrvCtl::quit; every other workgroup also gives up after 8x that without a
// word, so every wave reaches an exit.  A job posted while the grid is
// leaving is never lost: the host sees the stream idle with done != req and
// relaunches (csum_api.cpp).
template <int G, int U>
__global__ __launch_bounds__(256) void k_server(SrvHost *__restrict__ h, SrvCtl *__restrict__ d, uint32_t last,
                                                uint64_t idle_ticks)
{
    __shared__ uint32_t s_go;
    const bool lead = threadIdx.x == 0;
    uint32_t jobs = 0;
    uint64_t t_last = __builtin_amdgcn_s_memrealtime();
    // phase stamps (100 MHz) of job j in tr[(j % 256) * 8 + k], measurement only
    uint64_t *tr = reinterpret_cast<uint64_t *>(__hip_atomic_load(&h->trace, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    auto stamp = [&](int k) {
        if (tr)
            __hip_atomic_store(tr + (jobs % 256u) * 8u + k, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    };
    for (;;) {
        if (lead) {
            uint32_t go = 0;
            if (blockIdx.x == 0) {
                for (;;) {
                    const uint32_t r = __hip_atomic_load(&h->req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    if (r != last) {
                        stamp(0);
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); // system: the host's job and data
                        // all job words in flight together: one PCIe round trip, not seven
                        const uint32_t jop = __hip_atomic_load(&h->op, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        const uint32_t jn = __hip_atomic_load(&h->n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        uint64_t jp[5];
#pragma unroll
                        for (int k = 0; k < 5; ++k)
                            jp[k] = __hip_atomic_load(&h->ptr[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        __hip_atomic_store(&d->op, jop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&d->n, jn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                        for (int k = 0; k < 5; ++k)
                            __hip_atomic_store(&d->ptr[k], jp[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        __hip_atomic_store(&d->seq, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        stamp(1);
                        go = r;
                        break;
                    }
                    if (__hip_atomic_load(&h->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ||
                        __builtin_amdgcn_s_memrealtime() - t_last > idle_ticks) {
                        __hip_atomic_store(&d->quit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(4);
                }
            } else {
                for (;;) {
                    const uint32_t sq = __hip_atomic_load(&d->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (sq != 0u && sq != last) { // 0: zeroed at launch, nothing posted yet
                        if (blockIdx.x == 1)
                            stamp(2);
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); // system: SrvCtl + the host's data
                        go = sq;
                        break;
                    }
                    if (__hip_atomic_load(&d->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                        __builtin_amdgcn_s_memrealtime() - t_last > 8 * idle_ticks)
                        break;
                    __builtin_amdgcn_s_sleep(8);
                }
            }
            s_go = go;
        }
        __syncthreads();
        const uint32_t go = s_go;
        if (!go)
            return;
        const uint32_t op = __hip_atomic_load(&d->op, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t n = __hip_atomic_load(&d->n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint64_t q[5];
#pragma unroll
        for (int k = 0; k < 5; ++k)
            q[k] = __hip_atomic_load(&d->ptr[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint8_t *arena = reinterpret_cast<uint8_t *>(q[0]);
        const tcsum_pkt_t *pkts = reinterpret_cast<const tcsum_pkt_t *>(q[1]);
        uint32_t *out = reinterpret_cast<uint32_t *>(q[2]);
        uint8_t *flags = reinterpret_cast<uint8_t *>(q[3]);
        int8_t *verdict = reinterpret_cast<int8_t *>(q[4]);
        constexpr uint32_t PER = 256u / G;
        const uint32_t stride = gridDim.x * PER;
        for (uint32_t first = blockIdx.x * PER; first < n; first += stride) { // workgroup-uniform
            const uint32_t pk = first + threadIdx.x / G;
            if (op == IP_TX)
                ipv4_packet<G, U, IP_TX>(arena, pkts, pk, n, out, flags, verdict, 0u);
            else if (op == IP_RX)
                ipv4_packet<G, U, IP_RX>(arena, pkts, pk, n, out, flags, verdict, 0u);
            else
                ipv4_packet<G, U, IP_SUMS>(arena, pkts, pk, n, out, flags, verdict, 0u);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // every storing wave drains
        __syncthreads();
        if (lead) {
            if (blockIdx.x == 0)
                stamp(3);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); // system: this workgroup's results / tx bytes
            if (blockIdx.x == 0)
                stamp(4);
            const uint32_t old = __hip_atomic_fetch_add(&d->arrivals, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old == (jobs + 1u) * gridDim.x - 1u) {
                stamp(5);
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");
                __hip_atomic_store(&h->done, go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                stamp(6);
            }
            ++jobs;
        }
        last = go;
        t_last = __builtin_amdgcn_s_memrealtime();
    }
}

// ---------------------------------------------------------------- call server
//
// One resident wave serving the synchronous drop-in calls (csum_api.cpp,
// tcsum_call_server): instead of a kernel launch plus a stream sync per call
// (~17 us), the host copies the call's bytes into pinned staging, writes the
// job into a pinned CallBox and spins on the result word; the wave polls the
// box (both 16-byte job words in one PCIe round trip, s_sleep between polls),
// sums the range with all 64 lanes exactly like k_segments, and stores
// result << 32 | seq with one system-scope release.  A job is taken only when
// both job words carry its sequence number: the host stores them last, w1
// before w0, so a read that sees the new number in both saw every field.
// Exit: a QUIT job, or no job for idle_ticks of the 100 MHz clock -- every
// path leaves the loop, so the wave always finishes.

// The box's four 16-byte job words, system-scope loads all in flight (one
// PCIe round trip)
__device__ __forceinline__ void load_job(const CallBox *p, u32x4 &a, u32x4 &b, u32x4 &c, u32x4 &e)
{
    asm volatile("global_load_dwordx4 %0, %4, off sc0 sc1\n\t"
                 "global_load_dwordx4 %1, %4, off offset:16 sc0 sc1\n\t"
                 "global_load_dwordx4 %2, %4, off offset:32 sc0 sc1\n\t"
                 "global_load_dwordx4 %3, %4, off offset:48 sc0 sc1\n\t"
                 "s_waitcnt vmcnt(0)"
                 : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(e)
                 : "v"(p)
                 : "memory");
}

__global__ __launch_bounds__(64) void k_call(CallBox *__restrict__ box, const uint8_t *__restrict__ stage,
                                             uint32_t last, uint64_t idle_ticks)
{
    constexpr int G = 64, U = 16; // 16 KiB per pass: a 1500-B call is one PCIe round trip
    const uint32_t gl = threadIdx.x;
    uint64_t t_last = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        u32x4 a, b, c, e;
        for (;;) {
            load_job(box, a, b, c, e);
            const uint32_t sa = __builtin_amdgcn_readfirstlane(a.x), sb = __builtin_amdgcn_readfirstlane(b.w),
                           sc = __builtin_amdgcn_readfirstlane(c.w), se = __builtin_amdgcn_readfirstlane(e.w);
            if (sa != last && sa != 0u && sa == sb && sa == sc && sa == se)
                break;
            if (__builtin_amdgcn_s_memrealtime() - t_last > idle_ticks)
                return;
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); // system: the staged bytes
        last = __builtin_amdgcn_readfirstlane(a.x);
        const uint32_t ctl = __builtin_amdgcn_readfirstlane(a.y);
        if (ctl & CALL_QUIT)
            return;
        SegDesc d;
        d.off = (ctl & CALL_ODD) ? 1u : 0u;
        d.len = __builtin_amdgcn_readfirstlane(a.z);
        d.pre = __builtin_amdgcn_readfirstlane(a.w);
        d.src = __builtin_amdgcn_readfirstlane(b.x);
        d.dst = __builtin_amdgcn_readfirstlane(b.y);
        d.proto = __builtin_amdgcn_readfirstlane(b.z) & 0xFFu;
        const uint32_t mode = ctl & CALL_MODE_MASK;
        uint32_t acc;
        uintptr_t start = reinterpret_cast<uintptr_t>(stage + d.off);
        if (ctl & CALL_INLINE) {
            // <= 24 bytes that came with the job: the host zeroed the rest of
            // w2/w3 and put the bytes at offset (ctl & CALL_ODD), so the
            // exact word sum of the six dwords is the range's (no PCIe trip)
            acc = 0;
            acc = dot_halves(acc, __builtin_amdgcn_readfirstlane(c.x), 0x00010001u);
            acc = dot_halves(acc, __builtin_amdgcn_readfirstlane(c.y), 0x00010001u);
            acc = dot_halves(acc, __builtin_amdgcn_readfirstlane(c.z), 0x00010001u);
            acc = dot_halves(acc, __builtin_amdgcn_readfirstlane(e.x), 0x00010001u);
            acc = dot_halves(acc, __builtin_amdgcn_readfirstlane(e.y), 0x00010001u);
            acc = dot_halves(acc, __builtin_amdgcn_readfirstlane(e.z), 0x00010001u);
            start = d.off; // the byte parity the sum was taken at
        } else {
            if (mode == MODE_EXACT)
                acc = sum_range<G, U, true>(stage, d.off, d.len, gl, [] {});
            else
                acc = sum_range<G, U, false>(stage, d.off, d.len, gl, [] {});
            acc = group_sum<G>(acc);
        }
        if (gl == 0) {
            const uint32_t comp = (ctl & CALL_COMPLEMENT) ? 1u : 0u;
            uint16_t r;
            if (mode == MODE_EXACT)
                r = finalize<MODE_EXACT>(acc, start, d, comp | ((uint32_t)d.off << 1), 0u);
            else if (mode == MODE_PESO)
                r = finalize<MODE_PESO>(acc, start, d, 0u, peso_pseudo16(d));
            else
                r = finalize<MODE_SEG>(acc, start, d, comp, 0u);
            __hip_atomic_store(&box->res, ((uint64_t)r << 32) | last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        t_last = __builtin_amdgcn_s_memrealtime();
    }
}

// ---------------------------------------------------------------- synthetic

__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void k_synth_fill(uint8_t *__restrict__ arena, uint64_t nbytes,
                                                    uint64_t word_base, uint64_t seed)
{
    const uint64_t units = (nbytes + 15) / 16;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < units; i += (uint64_t)gridDim.x * 256ull) {
        const uint64_t w0 = splitmix64(seed + word_base + 2 * i);
        const uint64_t w1 = splitmix64(seed + word_base + 2 * i + 1);
        if (16 * i + 16 <= nbytes) {
            uint64_t *p = reinterpret_cast<uint64_t *>(arena + 16 * i);
            p[0] = w0;
            p[1] = w1;
        } else {
            for (uint64_t b = 16 * i; b < nbytes; ++b)
                arena[b] = (uint8_t)((b - 16 * i < 8 ? w0 : w1) >> (8 * (b & 7)));
        }
    }
}

__global__ __launch_bounds__(256) void k_synth_ipv4(uint8_t *__restrict__ arena,
                                                    const tcsum_pkt_t *__restrict__ pkts,
                                                    uint32_t n, uint64_t seed)
{
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t len = pkts[i].len;
    if (len < 20)
        return;
    uint8_t *p = arena + pkts[i].offset;
    const uint64_t h = splitmix64(seed ^ (0x1000000ull + i));
    const uint64_t a = splitmix64(h);
    const uint32_t tl = len > 0xFFFFu ? 0xFFFFu : len;
    p[0] = 0x45;
    p[1] = 0;
    p[2] = (uint8_t)(tl >> 8);
    p[3] = (uint8_t)tl;
    p[4] = (uint8_t)(h >> 8);
    p[5] = (uint8_t)h;
    p[6] = 0x40;
    p[7] = 0;
    p[8] = 64;
    p[9] = (h >> 20) & 1u ? 17 : 6;
    p[10] = 0;
    p[11] = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        p[12 + k] = (uint8_t)(a >> (8 * k));
    // L4 header fields the receive gates read (tcp_in.c:87-103, udp.c:337):
    // nonzero ports; TCP data offset 5 with ACK (+ PSH half the time); UDP
    // length.  The rest of the L4 bytes stay the synthetic stream.
    if (len < 40u) // room for a TCP header (the configs start at 64 B)
        return;
    const uint64_t b = splitmix64(a);
    const uint32_t sport = 1u + (uint32_t)(b % 65535u), dport = 1u + (uint32_t)((b >> 20) % 65535u);
    p[20] = (uint8_t)(sport >> 8);
    p[21] = (uint8_t)sport;
    p[22] = (uint8_t)(dport >> 8);
    p[23] = (uint8_t)dport;
    if (p[9] == 6) {
        p[32] = 0x50;
        p[33] = (b >> 40) & 1u ? 0x18 : 0x10;
    } else {
        const uint32_t ul = tl - 20u;
        p[24] = (uint8_t)(ul >> 8);
        p[25] = (uint8_t)ul;
    }
}

// ---------------------------------------------------------------- read probe
//
// The "achievable" side of the roofline: a plain streaming read of the same
// bytes with the same load shape (nontemporal dwordx4, one contiguous
// 64*U-chunk tile per wave), XOR-folded so the loads stay live; a store only
// happens if the fold hits a magic value.
template <int U, bool NT = true>
__global__ __launch_bounds__(256) void k_probe_read(const u32x4 *__restrict__ p, uint64_t nchunks,
                                                    uint32_t *__restrict__ sink, uint32_t xg)
{
    const uint64_t wave = (xcd_block(blockIdx.x, gridDim.x, xg) * 256ull + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t base = wave * 64ull * U;
    uint32_t acc = 0;
    u32x4 v[U];
    // unconditional loads, index clamped to the last chunk (as the checksum
    // kernels do): a bounds test per load would put each one behind its own
    // exec-mask branch
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t idx = base + u * 64ull + lane;
        v[u] = load16<NT>(p + (idx < nchunks ? idx : nchunks - 1));
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
        acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    if (acc == 0x9E3779B9u)
        sink[0] = acc;
}

// The same plain read in the product's own tile shape: G lanes share a
// "unit" of G*U consecutive chunks (lane gl loads chunks u*G + gl, u < U),
// 256/G units per workgroup, workgroups in the product's XCD-grouped order --
// k_segments / k_ipv4 minus descriptors, edge masking and sums (G = 256: one
// unit per workgroup, k_segments_wg's shape).  The ceiling the product kernel
// is compared with, on the same bytes.
// DEP: each unit first reads a 16-B "descriptor" (its own first chunk, so no
// extra bytes) and issues the tile's loads only behind it, as the product
// kernels wait for their descriptor before the data loads.
template <int G, int U, bool DEP>
__global__ __launch_bounds__(256) void k_probe_tile(const u32x4 *__restrict__ p, uint64_t nchunks,
                                                    uint32_t *__restrict__ sink, uint32_t xg)
{
    const uint64_t blk = xcd_block(blockIdx.x, gridDim.x, xg);
    const uint32_t gl = threadIdx.x & (G - 1);
    uint64_t base = (blk * (256u / G) + threadIdx.x / G) * (uint64_t)(G * U);
    if constexpr (DEP) {
        const u32x4 d = p[base < nchunks ? base : nchunks - 1];
        uint32_t zero;
        asm volatile("v_and_b32 %0, 0, %1" : "=v"(zero) : "v"(d.x)); // 0, but only once d is here
        base += zero;
    }
    uint32_t acc = 0;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { // unconditional, clamped (see k_probe_read)
        const uint64_t idx = base + (uint64_t)(u * G) + gl;
        v[u] = load16<true>(p + (idx < nchunks ? idx : nchunks - 1));
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
        acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    if (acc == 0x9E3779B9u)
        sink[0] = acc;
}

// The product's own load shape and nothing else: k_segments / k_segments_wg
// on the real checksum_peso descriptors -- descriptor, then the range's
// default-policy edge chunks and nontemporal interior chunks, same lanes, same
// XCD order -- with the sums, the group reduction and the result store
// replaced by an XOR fold (stored only on a 2^-32 fluke).  What the kernel
// would run at if its arithmetic were free.
template <int G, int U>
__global__ __launch_bounds__(256) void k_probe_desc(const uint8_t *__restrict__ arena,
                                                    const void *__restrict__ descs, uint32_t n,
                                                    uint32_t *__restrict__ sink, uint32_t xg, uint32_t pace)
{
    const uint32_t gl = threadIdx.x & (G - 1);
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x, xg);
    const uint32_t seg = G == 256 ? blk : blk * (256u / G) + threadIdx.x / G;
    if (pace) { // measurement (TCSUM_PROBE_PACE): hold the wave back before its first load
        uint32_t k = pace & 0xFFu;
        if (pace & 0x100u)
            k *= (threadIdx.x >> 6) + 1u; // staggered by wave in the workgroup
        if (pace & 0x200u)
            k *= (blockIdx.x & 3u); // staggered by workgroup
        for (uint32_t i = 0; i < k; ++i)
            __builtin_amdgcn_s_sleep(1);
    }
    const SegDesc d = load_desc<MODE_PESO>(descs, seg, seg < n);
    Frame<U> f;
    frame_issue<G, U>(f, arena, d.off, d.len, gl);
    issue_fence();
    uint32_t acc = f.ev.x ^ f.ev.y ^ f.ev.z ^ f.ev.w;
#pragma unroll
    for (int u = 0; u < U; ++u)
        acc ^= f.v[u].x ^ f.v[u].y ^ f.v[u].z ^ f.v[u].w;
    for (uint32_t b0 = G * U; b0 < f.ni; b0 += G * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j = b0 + u * G + gl;
            const u32x4 w = load16<true>(f.ibase + (j < f.ni ? j : f.ilast));
            acc ^= w.x ^ w.y ^ w.z ^ w.w;
        }
    }
    if (acc == 0x9E3779B9u)
        sink[0] = acc;
}

hipError_t launch_probe_desc(const void *arena, const void *descs, uint32_t n, uint64_t mean_len, uint32_t *sink,
                             hipStream_t stream)
{
    if (n == 0)
        return hipSuccess;
    const Geometry g = pick_geometry(mean_len);
    const uint32_t xg = (uint32_t)g.xcd;
    const uint8_t *a = static_cast<const uint8_t *>(arena);
    if (g.packed > 0) { // k_segments_pk's loads (the default shape)
        const uint32_t K = (uint32_t)g.packed < kPkMaxRanges * kPkWaves ? (uint32_t)g.packed
                                                                          : kPkMaxRanges * kPkWaves;
        if ((n + K - 1) / K >= (1u << 24))
            return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_segments_pk<MODE_PESO, kPkWaves, kPkLoads, true>), dim3((n + K - 1) / K),
                           dim3(kPkWaves * 64), 0, stream, a, descs, n, reinterpret_cast<uint16_t *>(sink), 0u, xg,
                           K);
        return hipGetLastError();
    }
    if (g.lanes == 1024 && g.loads == 4) { // k_segments_wgx<16, 32, 4>'s loads
        if (n >= (1u << 22))
            return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_segments_wgx<16, 32, 4, MODE_PESO, true>), dim3(n), dim3(1024), 0, stream, a, descs, n,
                           reinterpret_cast<uint16_t *>(sink), 0u, xg);
        return hipGetLastError();
    }
    const char *pe = getenv("TCSUM_PROBE_PACE");
    const uint32_t pace = pe ? (uint32_t)strtoul(pe, nullptr, 0) : 0u;
#define TCSUM_PD(GG, UU)                                                                                     \
    if (g.lanes == GG && g.loads == UU) {                                                                    \
        const uint32_t per_block = GG == 256 ? 1u : 256u / GG;                                               \
        if ((n + per_block - 1) / per_block >= (1u << 24))                                                   \
            return hipErrorInvalidValue;                                                                     \
        hipLaunchKernelGGL((k_probe_desc<GG, UU>), dim3((n + per_block - 1) / per_block), dim3(256), 0, stream, a, \
                           descs, n, sink, xg, pace);                                                        \
        return hipGetLastError();                                                                            \
    }
    TCSUM_PD(16, 3) TCSUM_PD(16, 4) TCSUM_PD(16, 6) TCSUM_PD(16, 8) TCSUM_PD(32, 4) TCSUM_PD(32, 6)
    TCSUM_PD(8, 4) TCSUM_PD(256, 16)
#undef TCSUM_PD
    return hipErrorInvalidValue;
}

hipError_t launch_probe_tile(const void *p, uint64_t nbytes, int G, int U, uint32_t *sink, hipStream_t stream)
{
    const uint64_t nchunks = nbytes / 16;
    if (nchunks == 0)
        return hipSuccess;
    const uint32_t xg = (uint32_t)pick_geometry(1500).xcd; // the product's order (TCSUM_XCD applies too)
    const dim3 grid((uint32_t)((nchunks + 256ull * U - 1) / (256ull * U)));
    const u32x4 *q = static_cast<const u32x4 *>(p);
    const char *dep_s = getenv("TCSUM_PROBE_DEP");
    const bool dep = dep_s && atoi(dep_s);
#define TCSUM_PT(GG, UU)                                                                         \
    if (G == GG && U == UU) {                                                                  \
        if (dep)                                                                               \
            hipLaunchKernelGGL((k_probe_tile<GG, UU, true>), grid, dim3(256), 0, stream, q, nchunks, sink, xg); \
        else                                                                                   \
            hipLaunchKernelGGL((k_probe_tile<GG, UU, false>), grid, dim3(256), 0, stream, q, nchunks, sink, xg); \
        return hipGetLastError();                                                              \
    }
    TCSUM_PT(16, 4) TCSUM_PT(16, 6) TCSUM_PT(16, 8) TCSUM_PT(32, 4) TCSUM_PT(32, 6) TCSUM_PT(32, 8)
    TCSUM_PT(64, 4) TCSUM_PT(64, 8) TCSUM_PT(256, 4) TCSUM_PT(256, 8) TCSUM_PT(256, 16)
#undef TCSUM_PT
    return hipErrorInvalidValue;
}

hipError_t launch_probe_read(const void *p, uint64_t nbytes, uint32_t *sink, hipStream_t stream)
{
    const uint64_t nchunks = nbytes / 16;
    if (nchunks == 0)
        return hipSuccess;
    int U = 4; // the fastest plain read of those measured (profiles/r01/probe_variants.txt)
    if (const char *s = getenv("TCSUM_PROBE_U"))
        U = atoi(s);
    uint32_t xg = 1; // dispatch order: measured faster for the plain read (profiles/r01/xcd_tune.txt)
    if (const char *s = getenv("TCSUM_PROBE_XCD"))
        xg = (uint32_t)atoi(s);
    const uint64_t per_block = 4ull * 64 * (uint64_t)U;
    const dim3 grid((uint32_t)((nchunks + per_block - 1) / per_block));
    const u32x4 *q = static_cast<const u32x4 *>(p);
    if (const char *s = getenv("TCSUM_PROBE_NT"); s && atoi(s) == 0) { // measurement: default-policy loads
        switch (U) {
        case 4: hipLaunchKernelGGL((k_probe_read<4, false>), grid, dim3(256), 0, stream, q, nchunks, sink, xg); break;
        case 16: hipLaunchKernelGGL((k_probe_read<16, false>), grid, dim3(256), 0, stream, q, nchunks, sink, xg); break;
        default: hipLaunchKernelGGL((k_probe_read<8, false>), grid, dim3(256), 0, stream, q, nchunks, sink, xg); break;
        }
        return hipGetLastError();
    }
    switch (U) {
    case 1: hipLaunchKernelGGL(k_probe_read<1>, grid, dim3(256), 0, stream, q, nchunks, sink, xg); break;
    case 2: hipLaunchKernelGGL(k_probe_read<2>, grid, dim3(256), 0, stream, q, nchunks, sink, xg); break;
    case 4: hipLaunchKernelGGL(k_probe_read<4>, grid, dim3(256), 0, stream, q, nchunks, sink, xg); break;
    case 16: hipLaunchKernelGGL(k_probe_read<16>, grid, dim3(256), 0, stream, q, nchunks, sink, xg); break;
    default: hipLaunchKernelGGL(k_probe_read<8>, grid, dim3(256), 0, stream, q, nchunks, sink, xg); break;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------- dispatch

// Workgroups of `kernel` that fit on the device at once (occupancy API x CUs),
// cached per kernel: a persistent grid larger than this runs a tail of
// non-resident blocks after the rest.
template <class K>
static uint32_t resident_blocks(K kernel)
{
    static uint32_t blocks = 0;
    if (blocks == 0) {
        int dev = 0, cus = 256, per_cu = 0;
        if (hipGetDevice(&dev) == hipSuccess)
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu < 1)
            per_cu = 1;
        if (per_cu > 8)
            per_cu = 8;
        blocks = (uint32_t)(cus * per_cu);
    }
    return blocks;
}

// Measured on MI355X (scripts/tune.py; profiles/r01/tune*.txt, one process,
// interleaved rounds).  Interior chunks per range c (edges excluded):
//   c <= ~136 (<= ~2 KiB, e.g. MTU): 16 lanes, U = ceil(c/16) loads -> one
//       pass with almost no idle slots (1500 B: G=16, U=6, 95% of the read
//       probe on the same bytes);
//   ~2 KiB .. 32 KiB (mixed 64-9000 B, mean 4.5 KiB): 32 lanes x 6 loads,
//       several passes (95-97% of the probe; re-measured with the XCD order);
//   >= 32 KiB (TSO): one range per WORKGROUP, 16 loads per lane -- a 64-KiB
//       range is one pass of every wave (profiles/r01/tso_wg.txt: 2343 us
//       against 2385 us for one range per wave, 1.02x the read probe).
// The resident-grid variants (persist 1, 2) measured slower on all three.
Geometry pick_geometry(uint64_t mean_len)
{
    // xcd: 64 workgroups per XCD run (scripts/xcd_tune.py, profiles/r01/xcd_tune.txt:
    // 2-4 % on every config, flat from 32 to 512)
    Geometry g{32, 4, 0, 64};
    const uint64_t chunks = mean_len / 16 + 1;
    const uint64_t interior = chunks > 2 ? chunks - 2 : 0;
    if (chunks >= 3072) {
        // >= 48 KiB (TSO): one range per 16-wave workgroup, 32-lane groups on
        // 2-KiB sub-ranges, 4 loads per lane: a 64-KiB range is one pass of
        // the workgroup -- 3.6 % faster than k_segments_wg on configs[2]
        // (profiles/r03/ab_tso_shapes2*.txt: 2,242 against 2,326 us)
        g.lanes = 1024;
        g.loads = 4;
    } else if (chunks >= 2048) {
        g.lanes = 256; // one range per workgroup (k_segments_wg): 1.8 % over G=64 on configs[2]
        g.loads = 16;
    } else if (interior > 128) {
        g.lanes = 32;
        g.loads = 6; // 1.0-1.5 % over 4 and 8 on every mixed variant (profiles/r01/geom_tune_mixed.txt)
    } else if (interior > 32) {
        g.lanes = 16;
        const uint64_t u = (interior + 15) / 16; // 3..8
        g.loads = u <= 3 ? 3 : u <= 4 ? 4 : u <= 6 ? 6 : 8;
    } else if (interior > 8) {
        g.lanes = 8;
        g.loads = 4;
    } else {
        g.lanes = 4;
        g.loads = interior > 4 ? 2 : 1;
    }
    if (const char *s = getenv("TCSUM_G"))
        g.lanes = atoi(s);
    if (const char *s = getenv("TCSUM_U"))
        g.loads = atoi(s);
    if (const char *s = getenv("TCSUM_P"))
        g.persist = atoi(s);
    if (const char *s = getenv("TCSUM_XCD"))
        g.xcd = atoi(s);
    // packed stream (k_segments_pk) for checksum_peso / pktbuf_checksum16
    // batches of ranges up to ~4 KiB: K ranges of this mean length fill one
    // 12-KiB pass of a 4-wave workgroup (1500 B: K = 8).  One-process A/Bs on
    // 1.5-GB batches (profiles/r03/ab_pk_layouts.txt): packed 1500-B ranges
    // 0.98 of k_segments<16,6>'s time, 576 B 0.73, 200 B 0.48, 64 B 0.70,
    // 4000 B 0.94, ragged 64..2936 B 0.96, with 0..63-B gaps 1.00; with
    // K < 3 (mean > ~4 KiB) it lost (9000 B 1.04, ragged 64..9000 B 1.20), and
    // a shuffled batch (ranges outside the region: range by range) costs 1.13.
    // TCSUM_PACKED=0 turns it off; TCSUM_PK_W / TCSUM_PK_U pick another
    // shape (measurement).
    // (a forced per-range geometry -- TCSUM_G / TCSUM_U / TCSUM_P -- keeps it off
    // unless TCSUM_PACKED=1 asks for it)
    const char *pks = getenv("TCSUM_PACKED");
    const bool forced = getenv("TCSUM_G") || getenv("TCSUM_U") || getenv("TCSUM_P");
    if ((pks ? atoi(pks) != 0 : !forced) && mean_len > 0) {
        const char *pw = getenv("TCSUM_PK_W");
        const char *pu = getenv("TCSUM_PK_U");
        const uint64_t w = pw ? (uint64_t)atoi(pw) : kPkWaves;
        const uint64_t pass = 16ull * 64u * w * (pu ? (uint64_t)atoi(pu) : kPkLoads);
        const uint64_t k = (pass - 15u) / mean_len;
        const uint64_t kmax = (uint64_t)kPkMaxRanges * w;
        if (k >= 3)
            g.packed = (int)(k > kmax ? kmax : k);
    }
    return g;
}

template <int MODE>
static hipError_t seg_u(int G, int U, int persist, uint32_t xg, uint32_t n, const void *arena, const void *descs,
                        uint16_t *out, uint32_t aux, hipStream_t s)
{
#define TCSUM_SEG(GG, UU)                                                                            \
    if (G == GG && U == UU) {                                                                      \
        const uint32_t per_block = 256u / GG;                                                      \
        uint32_t blocks = (n + per_block - 1) / per_block;                                         \
        if (persist == 2) {                                                                        \
            const uint32_t rb = resident_blocks(k_segments_pp<GG, UU, MODE>);                     \
            hipLaunchKernelGGL((k_segments_pp<GG, UU, MODE>), dim3(blocks < rb ? blocks : rb),     \
                               dim3(256), 0, s, static_cast<const uint8_t *>(arena), descs, n, out, \
                               aux);                                                               \
        } else if (persist == 1) {                                                                 \
            const uint32_t rb = resident_blocks(k_segments_p<GG, UU, MODE>);                      \
            hipLaunchKernelGGL((k_segments_p<GG, UU, MODE>), dim3(blocks < rb ? blocks : rb),      \
                               dim3(256), 0, s, static_cast<const uint8_t *>(arena), descs, n, out, \
                               aux);                                                               \
        } else {                                                                                   \
            hipLaunchKernelGGL((k_segments<GG, UU, MODE>), dim3(blocks), dim3(256), 0, s,          \
                               static_cast<const uint8_t *>(arena), descs, n, out, aux, xg);       \
        }                                                                                          \
        return hipGetLastError();                                                                  \
    }
#define TCSUM_SEG_U(GG)                                                                              \
    TCSUM_SEG(GG, 1) TCSUM_SEG(GG, 2) TCSUM_SEG(GG, 3) TCSUM_SEG(GG, 4) TCSUM_SEG(GG, 6)             \
        TCSUM_SEG(GG, 8) TCSUM_SEG(GG, 16)
    TCSUM_SEG_U(4)
    TCSUM_SEG_U(8)
    TCSUM_SEG_U(16)
    TCSUM_SEG_U(32)
    TCSUM_SEG_U(64)
#undef TCSUM_SEG_U
#undef TCSUM_SEG
    if (G == 1024) { // one range per 16-wave workgroup, 2 KiB sub-ranges (TSO)
        if (U != 4)
            return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_segments_wgx<16, 32, 4, MODE>), dim3(n), dim3(1024), 0, s,
                           static_cast<const uint8_t *>(arena), descs, n, out, aux, xg);
        return hipGetLastError();
    }
    if (G == 256) { // one range per workgroup
        const dim3 grid(n);
        const uint8_t *a = static_cast<const uint8_t *>(arena);
        // TCSUM_WGX=W/GL/U: k_segments_wgx's shapes (checksum_peso batches)
        if (const char *x = MODE == MODE_PESO ? getenv("TCSUM_WGX") : nullptr) {
            int w = 0, gl = -1, u = 0;
            if (sscanf(x, "%d%*[/x,]%d%*[/x,]%d", &w, &gl, &u) != 3)
                return hipErrorInvalidValue;
#define TCSUM_WGX(WW, GG, UU)                                                                                \
    if (w == WW && gl == GG && u == UU) {                                                                    \
        hipLaunchKernelGGL((k_segments_wgx<WW, GG, UU, MODE_PESO>), grid, dim3(WW * 64), 0, s, a, descs, n, out, aux, \
                           xg);                                                                              \
        return hipGetLastError();                                                                            \
    }
            TCSUM_WGX(4, 0, 16) TCSUM_WGX(8, 0, 8) TCSUM_WGX(16, 0, 4) TCSUM_WGX(4, 16, 16) TCSUM_WGX(8, 16, 8)
            TCSUM_WGX(16, 16, 4) TCSUM_WGX(16, 16, 6) TCSUM_WGX(8, 64, 8) TCSUM_WGX(16, 64, 4)
            TCSUM_WGX(4, 16, 6) TCSUM_WGX(4, 16, 8) TCSUM_WGX(4, 0, 8) TCSUM_WGX(4, 0, 4)
            TCSUM_WGX(16, 64, 2) TCSUM_WGX(8, 64, 4) TCSUM_WGX(4, 64, 4) TCSUM_WGX(16, 32, 4) TCSUM_WGX(16, 128, 4)
            TCSUM_WGX(16, 256, 4) TCSUM_WGX(16, 64, 3) TCSUM_WGX(8, 64, 2)
#undef TCSUM_WGX
            return hipErrorInvalidValue;
        }
        switch (U) {
        case 4: hipLaunchKernelGGL((k_segments_wg<4, MODE>), grid, dim3(256), 0, s, a, descs, n, out, aux, xg); break;
        case 8: hipLaunchKernelGGL((k_segments_wg<8, MODE>), grid, dim3(256), 0, s, a, descs, n, out, aux, xg); break;
        case 16: hipLaunchKernelGGL((k_segments_wg<16, MODE>), grid, dim3(256), 0, s, a, descs, n, out, aux, xg); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

// The AQL dispatch packet counts work-items in 32 bits: one launch may carry
// at most 2^24 - 1 workgroups of 256 threads.  Larger batches are split into
// several launches over consecutive descriptor ranges.
static constexpr uint64_t kMaxBlocks = (1u << 24) - 1;

hipError_t launch_segments(Mode mode, Geometry g, const void *arena, const void *descs, uint32_t n,
                           uint16_t *out, uint32_t aux, hipStream_t stream)
{
    if (n == 0)
        return hipSuccess;
    {
        const uint32_t lanes = mode == MODE_EXACT ? 64u : (uint32_t)g.lanes;
        // ranges per launch: 2^32 - 1 work-items (256 / G ranges per 256-thread
        // block; one range per block of 256 or 1024 threads)
        const uint64_t per_launch = g.packed > 0 && mode != MODE_EXACT ? ((1ull << 22) - 1) * (uint64_t)g.packed
                                    : lanes >= 1024 ? (1ull << 22) - 1
                                    : lanes >= 256 ? kMaxBlocks
                                                   : kMaxBlocks * (256u / (lanes ? lanes : 64u));
        if (n > per_launch) {
            const size_t dsz = mode == MODE_PESO ? sizeof(tcsum_peso_t) : sizeof(tcsum_seg_t);
            for (uint64_t i0 = 0; i0 < n; i0 += per_launch) {
                const uint32_t m = (uint32_t)(n - i0 < per_launch ? n - i0 : per_launch);
                const hipError_t e = launch_segments(mode, g, arena, static_cast<const uint8_t *>(descs) + i0 * dsz,
                                                     m, out + i0, aux, stream);
                if (e != hipSuccess)
                    return e;
            }
            return hipSuccess;
        }
    }
    if (g.packed > 0 && mode != MODE_EXACT) {
        const uint32_t K = (uint32_t)g.packed; // <= 64 per wave: capped by pick_geometry
        const uint8_t *a = static_cast<const uint8_t *>(arena);
        // TCSUM_PK_W / TCSUM_PK_U: the shapes the parity tests cover besides
        // the default (measurement otherwise)
        const char *pw = getenv("TCSUM_PK_W");
        const char *pu = getenv("TCSUM_PK_U");
        const int W = pw ? atoi(pw) : (int)kPkWaves, Ul = pu ? atoi(pu) : (int)kPkLoads;
        const uint32_t xgc = (uint32_t)g.xcd;
#define TCSUM_PK(WW, UU)                                                                                        \
    if (W == WW && Ul == UU) {                                                                                  \
        const uint32_t Kc = K < 64u * WW ? K : 64u * WW;                                                        \
        const dim3 gr((n + Kc - 1) / Kc), bl(WW * 64);                                                          \
        if (mode == MODE_SEG)                                                                                   \
            hipLaunchKernelGGL((k_segments_pk<MODE_SEG, WW, UU>), gr, bl, 0, stream, a, descs, n, out, aux, xgc, Kc); \
        else                                                                                                    \
            hipLaunchKernelGGL((k_segments_pk<MODE_PESO, WW, UU>), gr, bl, 0, stream, a, descs, n, out, aux, xgc, Kc); \
        return hipGetLastError();                                                                               \
    }
        TCSUM_PK(4, 3) TCSUM_PK(8, 3) TCSUM_PK(16, 2)
#undef TCSUM_PK
        return hipErrorInvalidValue;
    }
    if (mode == MODE_EXACT) {
        hipLaunchKernelGGL((k_segments<64, 8, MODE_EXACT>), dim3((n + 3) / 4), dim3(256), 0, stream,
                           static_cast<const uint8_t *>(arena), descs, n, out, aux, 1u);
        return hipGetLastError();
    }
    if (mode == MODE_SEG)
        return seg_u<MODE_SEG>(g.lanes, g.loads, g.persist, (uint32_t)g.xcd, n, arena, descs, out, aux, stream);
    return seg_u<MODE_PESO>(g.lanes, g.loads, g.persist, (uint32_t)g.xcd, n, arena, descs, out, aux, stream);
}

template <int IPM>
static hipError_t ipv4_u(int G, int U, dim3 grid, uint8_t *arena, const tcsum_pkt_t *pkts, uint32_t n,
                         uint32_t *out, uint8_t *flags, int8_t *verdict, uint32_t opts, uint32_t xg,
                         hipStream_t s)
{
#define TCSUM_IP(GG, UU)                                                                             \
    if (G == GG && U == UU) {                                                                      \
        hipLaunchKernelGGL((k_ipv4<GG, UU, IPM>), grid, dim3(256), 0, s, arena, pkts, n, out, flags, \
                           verdict, opts, xg);                                                     \
        return hipGetLastError();                                                                  \
    }
#define TCSUM_IP_U(GG)                                                                               \
    TCSUM_IP(GG, 1) TCSUM_IP(GG, 2) TCSUM_IP(GG, 3) TCSUM_IP(GG, 4) TCSUM_IP(GG, 6) TCSUM_IP(GG, 8)  \
        TCSUM_IP(GG, 16)
    TCSUM_IP_U(16)
    TCSUM_IP_U(32)
    TCSUM_IP_U(64)
#undef TCSUM_IP_U
#undef TCSUM_IP
    return hipErrorInvalidValue;
}

// Stream-ordered scratch for the deferred tx fill, from a pool of the
// library's own per device that keeps up to 1 GiB between calls: the default
// pool hands its memory back at every synchronization, and mapping it again
// cost a synchronized 1M-packet fill ~190 us (profiles/r02/tx_sync_probe.txt).
// The pool is the one of the device the caller's stream belongs to (the
// calling thread's current device only for the null stream).
static std::mutex g_scratch_mu;
static hipMemPool_t g_scratch_pools[64] = {};

static hipError_t scratch_alloc(void **p, size_t bytes, hipStream_t stream)
{
    int dev = 0;
    hipError_t e = stream ? hipStreamGetDevice(stream, &dev) : hipGetDevice(&dev);
    if (e != hipSuccess)
        return e;
    hipMemPool_t pool = nullptr;
    if (dev >= 0 && dev < 64) {
        std::lock_guard<std::mutex> lk(g_scratch_mu);
        if (!g_scratch_pools[dev]) {
            hipMemPoolProps props = {};
            props.allocType = hipMemAllocationTypePinned;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = dev;
            if (hipMemPoolCreate(&g_scratch_pools[dev], &props) == hipSuccess) {
                uint64_t keep = 1ull << 30;
                (void)hipMemPoolSetAttribute(g_scratch_pools[dev], hipMemPoolAttrReleaseThreshold, &keep);
            } else {
                g_scratch_pools[dev] = nullptr;
            }
        }
        pool = g_scratch_pools[dev];
    }
    return pool ? hipMallocFromPoolAsync(p, bytes, pool, stream) : hipMallocAsync(p, bytes, stream);
}

// tcsum_release: hand the pool's kept memory back (the caller has synchronized
// every stream that allocated from it).
hipError_t scratch_trim(int dev)
{
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    if (dev < 0 || dev >= 64 || !g_scratch_pools[dev])
        return hipSuccess;
    return hipMemPoolTrimTo(g_scratch_pools[dev], 0);
}

// The tx fill with its stores deferred (IP_OPT_DEFER + k_tx_scatter): the
// values are computed from `arena` and stored into `store`, the same packets
// at another address (the same arena, or the host memory an HBM copy was
// made from: the scatter's stores then cross PCIe as posted writes).
// `side`: 8 * n bytes of scratch (positions [n], then the values [n] when the
// caller wants no `out`).
static hipError_t tx_split_in(Geometry g, dim3 grid, uint32_t xg, uint8_t *arena, uint8_t *store,
                              const tcsum_pkt_t *pkts, uint32_t n, uint32_t *out, uint8_t *flags, uint32_t *side,
                              hipStream_t stream)
{
    uint32_t *vals = out ? out : side + n;
    hipError_t e = ipv4_u<IP_TX>(g.lanes, g.loads, grid, arena, pkts, n, vals, flags,
                                 reinterpret_cast<int8_t *>(side), IP_OPT_DEFER, xg, stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_tx_scatter, dim3((n + 255) / 256), dim3(256), 0, stream, store, pkts, n, vals, side);
        e = hipGetLastError();
    }
    return e;
}

static hipError_t tx_split(Geometry g, dim3 grid, uint32_t xg, uint8_t *arena, uint8_t *store,
                           const tcsum_pkt_t *pkts, uint32_t n, uint32_t *out, uint8_t *flags, hipStream_t stream)
{
    uint32_t *side = nullptr;
    hipError_t e = scratch_alloc(reinterpret_cast<void **>(&side), (size_t)n * (out ? 4u : 8u), stream);
    if (e != hipSuccess)
        return e;
    e = tx_split_in(g, grid, xg, arena, store, pkts, n, out, flags, side, stream);
    const hipError_t f = hipFreeAsync(side, stream);
    return e != hipSuccess ? e : f;
}

hipError_t launch_ipv4_tx_scratch(Geometry g, uint8_t *arena, const tcsum_pkt_t *pkts, uint32_t n, uint32_t *out,
                                  uint8_t *flags, uint32_t *scratch, hipStream_t stream)
{
    if (n == 0)
        return hipSuccess;
    g.lanes = g.lanes < 16 ? 16 : g.lanes > 64 ? 64 : g.lanes; // launch_ipv4's rules
    const uint64_t per_launch = kMaxBlocks * (256u / (uint32_t)g.lanes);
    if (n > per_launch) { // each part uses the scratch of its own packets
        for (uint64_t i0 = 0; i0 < n; i0 += per_launch) {
            const uint32_t m = (uint32_t)(n - i0 < per_launch ? n - i0 : per_launch);
            const hipError_t e = launch_ipv4_tx_scratch(g, arena, pkts + i0, m, out ? out + i0 : nullptr,
                                                        flags ? flags + i0 : nullptr, scratch + 2 * i0, stream);
            if (e != hipSuccess)
                return e;
        }
        return hipSuccess;
    }
    const uint64_t per_block = 256u / (uint32_t)g.lanes;
    return tx_split_in(g, dim3((uint32_t)((n + per_block - 1) / per_block)), (uint32_t)g.xcd, arena, arena, pkts,
                       n, out, flags, scratch, stream);
}

hipError_t launch_ipv4_tx_to(Geometry g, uint8_t *arena, uint8_t *store, const tcsum_pkt_t *pkts, uint32_t n,
                             uint32_t *out, uint8_t *flags, hipStream_t stream)
{
    if (n == 0)
        return hipSuccess;
    g.lanes = g.lanes < 16 ? 16 : g.lanes > 64 ? 64 : g.lanes; // launch_ipv4's rules
    const uint64_t per_launch = kMaxBlocks * (256u / (uint32_t)g.lanes);
    if (n > per_launch) {
        for (uint64_t i0 = 0; i0 < n; i0 += per_launch) {
            const uint32_t m = (uint32_t)(n - i0 < per_launch ? n - i0 : per_launch);
            const hipError_t e = launch_ipv4_tx_to(g, arena, store, pkts + i0, m, out ? out + i0 : nullptr,
                                                   flags ? flags + i0 : nullptr, stream);
            if (e != hipSuccess)
                return e;
        }
        return hipSuccess;
    }
    const uint64_t per_block = 256u / (uint32_t)g.lanes;
    return tx_split(g, dim3((uint32_t)((n + per_block - 1) / per_block)), (uint32_t)g.xcd, arena, store, pkts, n,
                    out, flags, stream);
}

hipError_t launch_ipv4(int ip_mode, Geometry g, uint8_t *arena, const tcsum_pkt_t *pkts, uint32_t n,
                       uint32_t *out, uint8_t *flags, int8_t *verdict, hipStream_t stream)
{
    if (n == 0)
        return hipSuccess;
    if (g.lanes < 16)
        g.lanes = 16;
    if (g.lanes > 64) // k_ipv4 keeps a packet inside one wave (no workgroup-per-packet form)
        g.lanes = 64;
    // rx keeps more registers live through the data pass (the gate codes, the
    // field sum): with 16 lanes per packet instead of 32 it measured 3.8 %
    // faster on configs[3] (profiles/r02/geom_rx.txt); the other modes keep 32
    if (ip_mode == IP_RX && g.lanes == 32 && !getenv("TCSUM_G"))
        g.lanes = 16;
    const uint64_t per_launch = kMaxBlocks * (256u / (uint32_t)g.lanes);
    if (n > per_launch) { // see kMaxBlocks
        for (uint64_t i0 = 0; i0 < n; i0 += per_launch) {
            const uint32_t m = (uint32_t)(n - i0 < per_launch ? n - i0 : per_launch);
            const hipError_t e = launch_ipv4(ip_mode, g, arena, pkts + i0, m, out ? out + i0 : nullptr,
                                             flags ? flags + i0 : nullptr, verdict ? verdict + i0 : nullptr, stream);
            if (e != hipSuccess)
                return e;
        }
        return hipSuccess;
    }
    const uint64_t per_block = 256u / (uint32_t)g.lanes;
    const dim3 grid((uint32_t)((n + per_block - 1) / per_block));
    const uint32_t xg = (uint32_t)g.xcd;
    switch (ip_mode) {
    case IP_TX:
        return ipv4_u<IP_TX>(g.lanes, g.loads, grid, arena, pkts, n, out, flags, verdict, 0u, xg, stream);
    case IP_TX_SPLIT: // the fill with its stores deferred to k_tx_scatter
        return tx_split(g, grid, xg, arena, arena, pkts, n, out, flags, stream);
    case IP_TX_OFFLOAD: // the tx values into `out` only; the packets are not written
        return ipv4_u<IP_TX>(g.lanes, g.loads, grid, arena, pkts, n, out, flags, verdict, IP_OPT_NO_STORE, xg,
                             stream);
    case IP_RX:
        return ipv4_u<IP_RX>(g.lanes, g.loads, grid, arena, pkts, n, out, flags, verdict, 0u, xg, stream);
    default:
        return ipv4_u<IP_SUMS>(g.lanes, g.loads, grid, arena, pkts, n, out, flags, verdict, 0u, xg, stream);
    }
}

hipError_t launch_probe_ipv4(const void *arena, const tcsum_pkt_t *pkts, uint32_t n, uint64_t mean_len, int mode,
                             uint32_t *sink, hipStream_t stream)
{
    if (n == 0)
        return hipSuccess;
    if (mode < PM_SUMS || mode > PM_TX)
        return hipErrorInvalidValue;
    Geometry g = pick_geometry(mean_len); // launch_ipv4's geometry rules
    if (g.lanes < 16)
        g.lanes = 16;
    if (g.lanes > 64)
        g.lanes = 64;
    if (mode == PM_RX && g.lanes == 32 && !getenv("TCSUM_G"))
        g.lanes = 16;
    const uint32_t per_block = 256u / (uint32_t)g.lanes;
    const uint64_t blocks = ((uint64_t)n + per_block - 1) / per_block;
    if (blocks > kMaxBlocks)
        return hipErrorInvalidValue;
    const uint8_t *a = static_cast<const uint8_t *>(arena);
    const uint32_t xg = (uint32_t)g.xcd;
    // PM_TX: the deferred fill's scratch (values, positions), from its pool
    uint32_t *side = nullptr;
    if (mode == PM_TX) {
        const hipError_t e = scratch_alloc(reinterpret_cast<void **>(&side), (size_t)n * 8u, stream);
        if (e != hipSuccess)
            return e;
    }
    uint32_t *vals = side, *posv = side ? side + n : nullptr;
    hipError_t e = hipErrorInvalidValue;
#define TCSUM_PI(GG, UU)                                                                                     \
    if (e == hipErrorInvalidValue && g.lanes == GG && g.loads == UU) {                                       \
        if (mode == PM_RX)                                                                                   \
            hipLaunchKernelGGL((k_probe_ipv4<GG, UU, PM_RX>), dim3((uint32_t)blocks), dim3(256), 0, stream, a,   \
                               pkts, n, sink, xg, vals, posv);                                              \
        else if (mode == PM_TX)                                                                              \
            hipLaunchKernelGGL((k_probe_ipv4<GG, UU, PM_TX>), dim3((uint32_t)blocks), dim3(256), 0, stream, a,   \
                               pkts, n, sink, xg, vals, posv);                                              \
        else                                                                                                 \
            hipLaunchKernelGGL((k_probe_ipv4<GG, UU, PM_SUMS>), dim3((uint32_t)blocks), dim3(256), 0, stream, a, \
                               pkts, n, sink, xg, vals, posv);                                              \
        e = hipGetLastError();                                                                               \
    }
    TCSUM_PI(16, 3) TCSUM_PI(16, 4) TCSUM_PI(16, 6) TCSUM_PI(16, 8) TCSUM_PI(32, 4) TCSUM_PI(32, 6)
    TCSUM_PI(64, 16)
#undef TCSUM_PI
    if (mode == PM_TX) {
        if (e == hipSuccess) { // the product's scatter, on the probe's values and positions
            hipLaunchKernelGGL(k_tx_scatter, dim3((n + 255) / 256), dim3(256), 0, stream, const_cast<uint8_t *>(a),
                               pkts, n, vals, posv);
            e = hipGetLastError();
        }
        const hipError_t f = hipFreeAsync(side, stream);
        e = e != hipSuccess ? e : f;
    }
    return e;
}

hipError_t launch_server(SrvHost *h, SrvCtl *d, uint32_t last, uint64_t idle_ticks, int wgs, hipStream_t stream)
{
    hipError_t e = hipMemsetAsync(d, 0, sizeof(SrvCtl), stream); // re-initialise every polled word
    if (e != hipSuccess)
        return e;
    // 64 lanes x 16 loads per frame: a frame of up to 16 KiB is one pass -- one
    // PCIe round trip for its bytes (the server's frames live in host memory)
    hipLaunchKernelGGL((k_server<64, 16>), dim3((uint32_t)(wgs > 0 ? wgs : 1)), dim3(256), 0, stream, h, d, last,
                       idle_ticks);
    return hipGetLastError();
}

// checksum16 on <= kCallInline bytes with the bytes in the kernel arguments
// (the call server's inline job, as a one-shot launch): no PCIe read of a
// descriptor or of staged bytes before the sum -- ipv4.c:243,656's 20-byte
// header checks.  w: the bytes at offset `odd`, zero-padded to 24.
template <int MODE>
__global__ __launch_bounds__(64) void k_inline16(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4,
                                                 uint32_t w5, uint32_t odd, uint32_t len, uint32_t pre,
                                                 uint32_t comp, uint16_t *__restrict__ out)
{
    if (threadIdx.x != 0)
        return;
    uint32_t acc = 0; // the exact word sum of the six dwords is the range's
    acc = dot_halves(acc, w0, 0x00010001u);
    acc = dot_halves(acc, w1, 0x00010001u);
    acc = dot_halves(acc, w2, 0x00010001u);
    acc = dot_halves(acc, w3, 0x00010001u);
    acc = dot_halves(acc, w4, 0x00010001u);
    acc = dot_halves(acc, w5, 0x00010001u);
    SegDesc d;
    d.off = odd;
    d.len = len;
    d.pre = pre;
    d.src = d.dst = d.proto = 0u;
    if constexpr (MODE == MODE_EXACT)
        *out = finalize<MODE_EXACT>(acc, odd, d, comp | (odd << 1), 0u);
    else
        *out = finalize<MODE_SEG>(acc, odd, d, comp, 0u);
}

// One staged range (the drop-in symbols' launch path) with its descriptor in
// the kernel arguments instead of pinned memory: one PCIe read less before
// the bytes.  The call server's staged job as a one-shot launch.
template <int MODE>
__global__ __launch_bounds__(64) void k_once(const uint8_t *__restrict__ stage, uint32_t off, uint32_t len,
                                             uint32_t pre, uint32_t src, uint32_t dst, uint32_t proto, uint32_t comp,
                                             uint16_t *__restrict__ out)
{
    constexpr int G = 64, U = 16; // 16 KiB per pass
    const uint32_t gl = threadIdx.x;
    SegDesc d;
    d.off = off;
    d.len = len;
    d.pre = pre;
    d.src = src;
    d.dst = dst;
    d.proto = proto;
    uint32_t acc = sum_range<G, U, MODE == MODE_EXACT>(stage, off, len, gl, [] {});
    acc = group_sum<G>(acc);
    if (gl == 0) {
        const uintptr_t start = reinterpret_cast<uintptr_t>(stage + off);
        if constexpr (MODE == MODE_EXACT)
            *out = finalize<MODE_EXACT>(acc, start, d, comp | ((off & 1u) << 1), 0u);
        else if constexpr (MODE == MODE_PESO)
            *out = finalize<MODE_PESO>(acc, start, d, 0u, peso_pseudo16(d));
        else
            *out = finalize<MODE_SEG>(acc, start, d, comp, 0u);
    }
}

hipError_t launch_once(Mode mode, const uint8_t *stage, uint32_t off, uint32_t len, uint32_t pre, uint32_t src,
                       uint32_t dst, uint32_t proto, int complement, uint16_t *out, hipStream_t stream)
{
    const uint32_t comp = complement ? 1u : 0u;
    if (mode == MODE_EXACT)
        hipLaunchKernelGGL(k_once<MODE_EXACT>, dim3(1), dim3(64), 0, stream, stage, off, len, pre, src, dst, proto,
                           comp, out);
    else if (mode == MODE_PESO)
        hipLaunchKernelGGL(k_once<MODE_PESO>, dim3(1), dim3(64), 0, stream, stage, off, len, pre, src, dst, proto,
                           comp, out);
    else
        hipLaunchKernelGGL(k_once<MODE_SEG>, dim3(1), dim3(64), 0, stream, stage, off, len, pre, src, dst, proto,
                           comp, out);
    return hipGetLastError();
}

hipError_t launch_inline16(Mode mode, const void *bytes, uint32_t len, uint32_t odd, uint32_t pre, int complement,
                           uint16_t *out, hipStream_t stream)
{
    if (len + odd > kCallInline || (mode != MODE_EXACT && mode != MODE_SEG))
        return hipErrorInvalidValue;
    uint32_t w[6] = {0u, 0u, 0u, 0u, 0u, 0u};
    if (len)
        memcpy(reinterpret_cast<uint8_t *>(w) + odd, bytes, len);
    if (mode == MODE_EXACT)
        hipLaunchKernelGGL(k_inline16<MODE_EXACT>, dim3(1), dim3(64), 0, stream, w[0], w[1], w[2], w[3], w[4], w[5],
                           odd, len, pre, complement ? 1u : 0u, out);
    else
        hipLaunchKernelGGL(k_inline16<MODE_SEG>, dim3(1), dim3(64), 0, stream, w[0], w[1], w[2], w[3], w[4], w[5],
                           odd, len, pre, complement ? 1u : 0u, out);
    return hipGetLastError();
}

hipError_t launch_call_server(CallBox *box, const uint8_t *stage, uint32_t last, uint64_t idle_ticks,
                              hipStream_t stream)
{
    hipLaunchKernelGGL(k_call, dim3(1), dim3(64), 0, stream, box, stage, last, idle_ticks);
    return hipGetLastError();
}

hipError_t launch_synth_fill(void *arena, uint64_t nbytes, uint64_t byte_base, uint64_t seed,
                             hipStream_t stream)
{
    if (nbytes == 0)
        return hipSuccess;
    const uint64_t units = (nbytes + 15) / 16;
    uint64_t blocks = (units + 255) / 256;
    if (blocks > 65536)
        blocks = 65536;
    hipLaunchKernelGGL(k_synth_fill, dim3((uint32_t)blocks), dim3(256), 0, stream,
                       static_cast<uint8_t *>(arena), nbytes, byte_base / 8, seed);
    return hipGetLastError();
}

hipError_t launch_synth_ipv4(void *arena, const tcsum_pkt_t *pkts, uint32_t n, uint64_t seed,
                             hipStream_t stream)
{
    if (n == 0)
        return hipSuccess;
    hipLaunchKernelGGL(k_synth_ipv4, dim3((n + 255) / 256), dim3(256), 0, stream,
                       static_cast<uint8_t *>(arena), pkts, n, seed);
    return hipGetLastError();
}

} // namespace tcsum
