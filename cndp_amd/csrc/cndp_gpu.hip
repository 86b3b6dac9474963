// cndp_gpu.hip -- MI355X (gfx950) device runtime and kernels of libcndp_gpu.so.
//
// Kernels (one packet per lane, wave64, no MFMA -- pure integer/byte work):
//   k_classify_fast<MODE>  l3fwd / hash modes: fixed-offset header fields
//                          (Eth + IPv4 at 14) loaded straight into VGPRs,
//                          Toeplitz by byte-sliced tables in LDS, DIR-24-8
//                          gather, per-block LDS bin counters.
//   k_classify_cnet        cnet mode: each lane's 64-byte header window is
//                          staged in LDS (17-dword rows: conflict-free for
//                          equal offsets across lanes), cne_get_ptype parse
//                          from LDS with variable offsets, IPv4 checksum,
//                          DIR-24-8 / trie gathers.
//   k_lookup4<W>/k_lookup6<W>  bulk FIB lookups (cne_fib[6]_lookup_bulk).
//   k_bin_ids, k_part_*    stable partition into per-edge streams.
// Reference behaviour each kernel restates is cited inline (CNDP v25.08.0).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <vector>

#include "fib_internal.h"
#include "node_internal.h"
#include "../../include/cndp_gpu.h"

#define CNDP_VERSION "cndp_amd 0.1 (gfx950)"

#define HIP_TRY(expr)                                                                            \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "cndp_gpu: %s failed: %s (%s:%d)\n", #expr, hipGetErrorString(e_),   \
                    __FILE__, __LINE__);                                                         \
            return e_ == hipErrorNoDevice || e_ == hipErrorInvalidDevice ? -ENODEV : -EIO;       \
        }                                                                                        \
    } while (0)

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu); }
__device__ __forceinline__ uint32_t alignb(uint32_t hi, uint32_t lo, uint32_t s)
{
    return __builtin_amdgcn_alignbyte(hi, lo, s);
}

// lo16(x) + hi16(x) + acc in one v_dot2_u32_u16 (x . (1, 1) + acc)
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t hsum2(uint32_t x, uint32_t acc)
{
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, x), (u16x2_t){1, 1}, acc, false);
}

// global address space for buffer pointers (see gp() below)
#ifndef GP_GLOBAL
#define GP_GLOBAL 1 /* 0: generic pointers (A/B builds) */
#endif
#if GP_GLOBAL
#define GAS __attribute__((address_space(1)))
#else
#define GAS
#endif

// bounded global byte read (bytes past the slab end read as 0)
__device__ __forceinline__ uint32_t gbyte(const uint8_t *p, uint64_t avail, uint64_t o)
{
    return o < avail ? (uint32_t)((const GAS uint8_t *)p)[o] : 0u;
}
// 4 bytes at o assembled little-endian, bounded
__device__ __forceinline__ uint32_t gld32(const uint8_t *p, uint64_t avail, uint64_t o)
{
    return gbyte(p, avail, o) | (gbyte(p, avail, o + 1) << 8) | (gbyte(p, avail, o + 2) << 16) |
           (gbyte(p, avail, o + 3) << 24);
}

// DIR-24-8 4B lookup, dir24_8.h:131-135
__device__ __forceinline__ uint32_t lpm4(const uint32_t *__restrict__ t24,
                                         const uint32_t *__restrict__ t8, uint32_t ip)
{
    uint32_t e = t24[ip >> 8];
    if (e & 1u)
        e = t8[(e >> 1) * 256u + (ip & 0xffu)];
    return e >> 1;
}

// DIR-24-8 4B lookup through the /16 directory (same result as lpm4)
__device__ __forceinline__ uint32_t lpm4d(const uint32_t *__restrict__ d16,
                                          const uint32_t *__restrict__ pages,
                                          const uint32_t *__restrict__ t8, uint32_t ip)
{
    uint32_t e = d16[ip >> 16];
    if (e & 1u)
        e = pages[(e >> 1) * 256u + ((ip >> 8) & 0xffu)];
    if (e & 1u)
        e = t8[(e >> 1) * 256u + (ip & 0xffu)];
    return e >> 1;
}

// Toeplitz byte table access: T[b][v] at tab[b * 256 + v]
template <typename TP>
__device__ __forceinline__ uint32_t tz4(TP tab, uint32_t b, uint32_t x)
{
    // the 4 stream bytes b..b+3 held little-endian in x (byte b = x & 0xff)
    return tab[(b + 0) * 256 + (x & 0xffu)] ^ tab[(b + 1) * 256 + ((x >> 8) & 0xffu)] ^
           tab[(b + 2) * 256 + ((x >> 16) & 0xffu)] ^ tab[(b + 3) * 256 + (x >> 24)];
}

// the same from the nibble tables N[q][u] (tab[q * 16 + u], TABN_OFF in the
// global table): 8 reads a word instead of 4, but a wave's 32 lanes read at
// most 16 distinct dwords of one 16-dword row, so no LDS bank conflicts
template <typename TP>
__device__ __forceinline__ uint32_t tz4n(TP tab, uint32_t b, uint32_t x)
{
    uint32_t h = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t v = (x >> (8 * j)) & 0xffu, q = 2 * (b + j);
        h ^= tab[q * 16 + (v >> 4)] ^ tab[(q + 1) * 16 + (v & 15u)];
    }
    return h;
}

#define CNDP_RW_MAX_NH CNDP_IP4_REWRITE_MAX_NH       // CNE_GRAPH_IP4_REWRITE_MAX_NH
#define CNDP_RW_MAX_LEN CNDP_IP4_REWRITE_MAX_LEN     // CNE_GRAPH_IP4_REWRITE_MAX_LEN
#define CNDP_RW_MAX_PORTS CNDP_IP4_REWRITE_MAX_PORTS // CNE_MAX_ETHPORTS
// struct cndp_rw_nh = struct ip4_rewrite_nh_header (node_internal.h)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4))); // dword-aligned 16-B load
typedef uint32_t u32x3a4 __attribute__((ext_vector_type(3), aligned(4)));
typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

struct KArgs {
    const uint8_t *slab;
    uint64_t slab_len;
    uint64_t stride;
    const uint64_t *offsets;
    uint32_t data_off;
    uint32_t n;
    uint32_t buf_len;
    uint32_t reta_mask;
    const uint32_t *tbl24;
    const uint32_t *tbl8;
    const uint32_t *tbl24_6;
    const uint32_t *tbl8_6;
    const uint32_t *dir16; // /16 directory (nullptr = plain tbl24 path)
    const uint32_t *pages;
    const uint32_t *ttab; // 36 x 256 Toeplitz byte tables (global)
    const uint16_t *reta;
    uint32_t *nh;
    uint32_t *hash;
    uint16_t *queue;
    uint8_t *edge;
    unsigned long long *bins;
    uint32_t n_bins;
    uint32_t *ptype;   // optional: packet_type per frame
    uint32_t *rxmeta;  // optional (cnet): eth_rx lengths + ol_flags, packed (cndp_gpu.h)
    uint32_t *iplen;   // node queue (cnet): 1 << 16 | IPv4 total_length / IPv6 payload_len
                       // of the frames the fast path parsed (the rest left 0)
    u32x4 *win;        // node queue (zero-copy cnet): each frame's first 64 bytes as parsed
                       // (4 x 16 B per frame), the source of the cnet_metadata addresses
    uint32_t *spec_nh; // cnet speculation model: input-node result of every frame a
                       // ptype-node group could send to ip4/ip6_input (else ~0)
    uint32_t *spec_flags; // 2048-bit set of the type signatures seen (speculation model)
    uint16_t *spec_t16;   // speculation model: packet_type & 0xFFFF of every frame
    // cnet fast / general split (k_cnet_stream -> k_classify_cnet): frames the
    // fast kernel leaves to the general parse, and their count
    uint32_t *wl;
    uint32_t *wl_n;
    // speculation bookkeeping, folded into k_classify_cnet's last block to
    // finish (spec_classes): nullptr spec_meta = no speculation model
    uint32_t *spec_meta;   // sp_small + 1 (meta[-1] = the node state)
    uint8_t *spec_cls;     // class id per signature (2048)
    uint32_t *spec_ticket; // k_classify_cnet's block arrivals, 9 words 32 apart (0 between launches)
    uint32_t *spec_bar;    // k_spec_fallback's barrier words, reset by spec_classes
    uint8_t *spec_tile;    // per 64-frame tile: 0x80 | edge when every frame has that edge, else 0
    uint32_t *spec_cwl;    // CNDP_TUNE_SPEC_LISTS: chunks with a non-canonical tile ([0] = count)
    uint32_t *spec_cflag;  //   and a flag per chunk so each is listed once
    uint32_t *spec_hint;   // pinned host words (device view): the last call's worklist size class, uniform flag
    uint32_t spec_B;       // graph burst size
    uint32_t wl_fold;      // k_cnet_defer's last block parses the worklist and runs spec_classes
    uint32_t tail_lo;      // with wl_fold: the first frame of the last SPEC_TAIL bursts
    uint32_t spec_allow;   // batch shortcuts allowed (CNDP_TUNE_SPEC_SCAN auto)
    // canonical tiles' types as 2-bit codes (CNDP_TUNE_SPEC_TYPES): per tile 16 B,
    // the ballots of "IPv6" and "UDP" over its frames, tile word SPEC_TW_CODES and
    // no spec_t16 stores; frames >= spec_keep_lo always store their types
    uint8_t *spec_c2;
    uint32_t spec_codes;
    uint32_t spec_keep_lo;
    // fused ip4_rewrite (k_classify_tile<..., RW = true>)
    const struct cndp_rw_nh *rw_tbl;
    uint16_t *tx_edge;
    uint32_t rw_parts; // 16-B parts of each rewritten frame written back
};

#define FAST_THREADS 256
#define SPEC_CH_K 4 // graph bursts per speculation chunk (SPEC_CH)
// meta word (spec_meta index) of CNDP_TUNE_SPEC_LISTS:
// what the fast kernel saw of the groups that could move
// the node state off a common edge (ptype.c:122-130: a group's 4th type
// becomes the state when the 3rd equals it or when its p_nxt edge is the
// state's): bits 0-7 = the edges of such 4th types (fast-parsed, not bound
// for their low byte's input node, 3rd type different), bit 8 = a 4th type
// that equals the 3rd or is not known to the fast kernel.  k_spec_fallback
// clears it for the next call.
#define SPEC_MX 135
#define SPEC_PTRS 151 // meta[151..154] (8-B aligned): the chunk list's and its flags' device pointers
#define SPEC_ALLOW_LISTS 2u // KArgs::spec_allow bit: this call lists (spec_cwl / spec_cflag set)
// a packet ip4_lookup hands to ip4_rewrite (edge 0, ip4_lookup.c:150)
__device__ __forceinline__ bool nh_ready_rw(uint32_t v) { return v != 0xFFFFFFFFu && (v >> 16) == 0u; }
#define TAB4_POS 12 /* Toeplitz positions for the IPv4 L4 tuple */
#define TAB_POS 36  /* ... for the IPv6 L4 tuple */
#define TABN_OFF (TAB_POS * 256) /* nibble tables N[q][u] (72 x 16) follow the byte tables */
#define TAB_WORDS (TABN_OFF + 2 * TAB_POS * 16)

// Bins (identical to oracle.c classify_one)
template <int MODE>
__device__ __forceinline__ uint32_t bin_of(uint32_t nh, uint32_t edge, uint32_t q, uint32_t nb)
{
    if (MODE == CNDP_MODE_HASH)
        return q < nb ? q : nb + 1;
    if (MODE == CNDP_MODE_L3FWD) {
        if (edge == 0)
            return (nh & 0xffffu) < nb ? (nh & 0xffffu) : nb + 1;
        return (edge == 1 || edge == 0xFFu) ? nb : nb + 1;
    }
    if (edge == 1)
        return (nh & 0xffffffu) < nb ? (nh & 0xffffffu) : nb + 1;
    return (edge == 0 || edge == 0x80u) ? nb : nb + 1;
}

// IPv6 flow hash when the tables are not all in LDS (l3fwd/hash modes);
// addresses at ip+8 / ip+24, ports at ip+40 (no extension headers there).
__device__ uint32_t hash_v6_global(const uint8_t *p, uint64_t avail, uint32_t ip, bool l4,
                                   const uint32_t *__restrict__ ttab)
{
    const GAS uint32_t *gt = (const GAS uint32_t *)ttab;
    uint32_t h = 0;
    for (uint32_t k = 0; k < 8; k++)
        h ^= tz4(gt, 4 * k, gld32(p, avail, ip + 8 + 4 * k));
    if (l4)
        h ^= tz4(gt, 32, gld32(p, avail, ip + 40));
    return h;
}

// ---------------------------------------------------------------------------
// l3fwd / hash classify: pktdev_rx.c:24-34 + pkt_cls.c:19-31 + ip4_lookup.c
// :108-154 (+ build-defined Toeplitz / RSS queue).  Header fields sit at fixed
// offsets (Ethernet 14 B, no VLAN parse in this chain), so each lane loads
// bytes 12..39 of its frame into VGPRs and never touches them again.
// Variants (runtime-selected, see cndp_gpu_set_tuning):
//   NT  frames read / outputs written with the non-temporal hint, so the
//       once-touched stream does not evict the DIR-24-8 table from the
//       Infinity Cache / L2 (the random 10% of lookups then stay on-die);
//   U   packets per lane per loop trip (U = 2 issues both frames' loads
//       before the first dependent LPM gather: more bytes in flight).
// ---------------------------------------------------------------------------

// Every buffer a kernel touches is device memory or host memory mapped for
// the device (hipMalloc, hipHostMalloc, hipHostRegister): global, never LDS or
// scratch.  Pointers that reach a load or store through integer arithmetic,
// __shfl or an opaque copy lose that to the compiler, which then emits FLAT
// instructions: a FLAT access counts in both vmcnt and lgkmcnt, so every
// later wait for an LDS result (the Toeplitz tables, the tile) waits for the
// frame loads in flight as well.  gp() restores the global address space.
template <typename T>
__device__ __forceinline__ GAS T *gp(T *p)
{
    return (GAS T *)p;
}
template <typename T>
__device__ __forceinline__ const GAS T *gp(const T *p)
{
    return (const GAS T *)p;
}

template <bool NT>
__device__ __forceinline__ u32x4 ldg4(const uint8_t *p)
{
    if (NT)
        return __builtin_nontemporal_load(gp((const u32x4 *)p));
    return *gp((const u32x4 *)p);
}
template <bool NT>
__device__ __forceinline__ u32x2 ldg2(const uint8_t *p)
{
    if (NT)
        return __builtin_nontemporal_load(gp((const u32x2 *)p));
    return *gp((const u32x2 *)p);
}
template <bool NT, typename T>
__device__ __forceinline__ void stg(T *p, T v)
{
    if (NT)
        __builtin_nontemporal_store(v, gp(p));
    else
        *p = v;
}

struct FastHdr {
    const uint8_t *p;
    uint64_t avail;
    uint32_t w3, w5, w6, w7, w8, w9;
};

template <bool NT>
__device__ __forceinline__ void fast_load(const KArgs &a, uint64_t i, FastHdr &h)
{
    const uint64_t base = (a.offsets ? a.offsets[i] : i * a.stride) + a.data_off;
    h.p = a.slab + base;
    h.avail = base < a.slab_len ? a.slab_len - base : 0;
    if (h.avail >= 48 && (base & 15u) == 0) {
        const u32x4 q0 = ldg4<NT>(h.p + 0);
        const u32x4 q1 = ldg4<NT>(h.p + 16);
        const u32x2 q2 = ldg2<NT>(h.p + 32);
        h.w3 = q0.w;
        h.w5 = q1.y;
        h.w6 = q1.z;
        h.w7 = q1.w;
        h.w8 = q2.x;
        h.w9 = q2.y;
    } else if (h.avail >= 40 && (base & 3u) == 0) {
        const uint32_t *d = (const uint32_t *)h.p;
        h.w3 = d[3];
        h.w5 = d[5];
        h.w6 = d[6];
        h.w7 = d[7];
        h.w8 = d[8];
        h.w9 = d[9];
    } else {
        h.w3 = gld32(h.p, h.avail, 12);
        h.w5 = gld32(h.p, h.avail, 20);
        h.w6 = gld32(h.p, h.avail, 24);
        h.w7 = gld32(h.p, h.avail, 28);
        h.w8 = gld32(h.p, h.avail, 32);
        h.w9 = gld32(h.p, h.avail, 36);
    }
}

// ip4_lookup.c:109-145 for one frame: the FIB value, or CNDP_NH_INVALID when
// pkt_cls would not send the frame to ip4_lookup (ethertype != IPv4)
template <int MODE>
__device__ __forceinline__ uint32_t fast_lpm(const KArgs &a, const FastHdr &h)
{
    if (MODE != CNDP_MODE_L3FWD || bswap16(h.w3 & 0xffffu) != 0x0800u)
        return CNDP_NH_INVALID;
    const uint32_t ip = bswap32(alignb(h.w8, h.w7, 2));
    return a.dir16 ? lpm4d(a.dir16, a.pages, a.tbl8, ip) : lpm4(a.tbl24, a.tbl8, ip);
}

// 5-tuple Toeplitz of one frame (build-defined: L4 tuple for TCP/UDP
// non-fragments, else L3), tables T[b][v] in LDS for the IPv4 tuple
template <int MODE>
__device__ __forceinline__ uint32_t fast_hash(const KArgs &a, const FastHdr &h, const uint32_t *s_t)
{
    const uint32_t et = bswap16(h.w3 & 0xffffu);
    uint32_t hs = 0;
    if (et == 0x0800u) {
        const uint32_t ihl = (h.w3 >> 16) & 0xfu;
        const uint32_t proto = h.w5 >> 24;
        const uint32_t frag = bswap16(h.w5 & 0xffffu) & 0x3fffu;
        const uint32_t src = alignb(h.w7, h.w6, 2);
        const uint32_t dst = alignb(h.w8, h.w7, 2);
        hs = tz4(s_t, 0, src) ^ tz4(s_t, 4, dst);
        if (ihl >= 5 && (proto == 6u || proto == 17u) && frag == 0) {
            const uint32_t ports = ihl == 5 ? alignb(h.w9, h.w8, 2) : gld32(h.p, h.avail, 14 + 4 * ihl);
            hs ^= tz4(s_t, 8, ports);
        }
    } else if (et == 0x86DDu) {
        const uint32_t nx = h.w5 & 0xffu; // ip6 next header: frame byte 20
        hs = hash_v6_global(h.p, h.avail, 14, nx == 6u || nx == 17u, a.ttab);
    }
    return hs;
}

// queue, bins and the output stores of one frame
template <int MODE, bool NT>
__device__ __forceinline__ void fast_emit(const KArgs &a, uint64_t i, uint32_t et, uint32_t nh, uint32_t hs,
                                          const uint16_t *s_reta, uint32_t *s_bins, bool count)
{
    uint32_t edge;
    if (MODE == CNDP_MODE_HASH)
        edge = 0;
    else
        edge = et == 0x0800u ? ((nh >> 16) & 0xffu) : 0xFFu;
    const uint32_t q = s_reta[hs & a.reta_mask];
    if (a.ptype) // pktdev_rx.c:24-34 l3_ptype
        stg<NT>(a.ptype + i, et == 0x0800u ? 0x90u : et == 0x86DDu ? 0xE0u : 0u);
    if (a.nh)
        stg<NT>(a.nh + i, nh);
    if (a.hash)
        stg<NT>(a.hash + i, hs);
    if (a.queue)
        stg<NT>(a.queue + i, (uint16_t)q);
    if (a.edge)
        stg<NT>(a.edge + i, (uint8_t)edge);
    if (count)
        atomicAdd(&s_bins[bin_of<MODE>(nh, edge, q, a.n_bins)], 1u);
}

template <int MODE, bool NT, bool PRE = false>
__device__ __forceinline__ void fast_finish(const KArgs &a, uint64_t i, const FastHdr &h,
                                            const uint32_t *s_t, const uint16_t *s_reta,
                                            uint32_t *s_bins, bool count, uint32_t nh_pre = 0)
{
    const uint32_t et = bswap16(h.w3 & 0xffffu);
    uint32_t nh = PRE ? nh_pre : CNDP_NH_INVALID;
    if (MODE == CNDP_MODE_L3FWD && !PRE && et == 0x0800u) { // issue the gather first
        const uint32_t ip = bswap32(alignb(h.w8, h.w7, 2));
        nh = a.dir16 ? lpm4d(a.dir16, a.pages, a.tbl8, ip) : lpm4(a.tbl24, a.tbl8, ip);
    }
    const uint32_t hs = fast_hash<MODE>(a, h, s_t);
    fast_emit<MODE, NT>(a, i, et, nh, hs, s_reta, s_bins, count);
}

template <int MODE, bool NT, int U>
__global__ __launch_bounds__(FAST_THREADS) void k_classify_fast(KArgs a)
{
    __shared__ uint32_t s_t[TAB4_POS * 256];
    __shared__ uint16_t s_reta[CNDP_RETA_MAX];
    __shared__ uint32_t s_bins[CNDP_BINS_MAX + 2];

    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < TAB4_POS * 256; k += FAST_THREADS)
        s_t[k] = a.ttab[k];
    for (uint32_t k = tid; k <= a.reta_mask; k += FAST_THREADS)
        s_reta[k] = a.reta[k];
    const bool count = a.bins != nullptr;
    if (count)
        for (uint32_t k = tid; k < a.n_bins + 2; k += FAST_THREADS)
            s_bins[k] = 0;
    __syncthreads();

    const uint64_t step = (uint64_t)gridDim.x * FAST_THREADS;
    uint64_t i = (uint64_t)blockIdx.x * FAST_THREADS + tid;
    if (U == 2) {
        for (; i + step < a.n; i += 2 * step) {
            FastHdr h0, h1;
            fast_load<NT>(a, i, h0);
            fast_load<NT>(a, i + step, h1);
            fast_finish<MODE, NT>(a, i, h0, s_t, s_reta, s_bins, count);
            fast_finish<MODE, NT>(a, i + step, h1, s_t, s_reta, s_bins, count);
        }
    }
    for (; i < a.n; i += step) {
        FastHdr h0;
        fast_load<NT>(a, i, h0);
        fast_finish<MODE, NT>(a, i, h0, s_t, s_reta, s_bins, count);
    }
    if (count) {
        __syncthreads();
        for (uint32_t k = tid; k < a.n_bins + 2; k += FAST_THREADS)
            if (s_bins[k])
                atomicAdd(&a.bins[k], (unsigned long long)s_bins[k]);
    }
}


// ---------------------------------------------------------------------------
// Wave-tile variant for packed 64-byte slots (stride 64): each wave owns a
// tile of 64 consecutive frames = 4 KiB of contiguous HBM.  The wave reads
// it with 4 fully coalesced 1-KiB loads (16 B/lane), writes the 16-B chunks
// to its LDS tile with the row swizzle  part' = part ^ ((frame >> 2) & 3),
// and each lane then reads its own frame's parts 0..2 with ds_read_b128 /
// ds_read_b64 -- conflict-free for the b128 lane groups.  The next tile's
// four loads are issued before the current tile is parsed, so each wave
// keeps 4 KiB in flight while it computes.
// ---------------------------------------------------------------------------
#define TILE_WAVES (FAST_THREADS / 64)

template <int MODE, int SCHED, bool NTS, bool RW = false, bool LNT = false>
__global__ __launch_bounds__(FAST_THREADS) void k_classify_tile(KArgs a, uint64_t n_tiles)
{
    __shared__ uint32_t s_t[TAB4_POS * 256];
    __shared__ uint16_t s_reta[CNDP_RETA_MAX];
    __shared__ uint32_t s_bins[CNDP_BINS_MAX + 2];
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[TILE_WAVES][256];
    __shared__ struct cndp_rw_nh s_rw[RW ? CNDP_RW_MAX_NH : 1];
    __shared__ uint32_t s_rwc[2][TILE_WAVES];

    const uint32_t tid = threadIdx.x;
    if (RW)
        for (uint32_t k = tid; k < sizeof(s_rw) / 4; k += FAST_THREADS)
            ((uint32_t *)s_rw)[k] = ((const uint32_t *)a.rw_tbl)[k];
    uint32_t rw_par = 0;
    for (uint32_t k = tid; k < TAB4_POS * 256; k += FAST_THREADS)
        s_t[k] = a.ttab[k];
    for (uint32_t k = tid; k <= a.reta_mask; k += FAST_THREADS)
        s_reta[k] = a.reta[k];
    const bool count = a.bins != nullptr;
    if (count)
        for (uint32_t k = tid; k < a.n_bins + 2; k += FAST_THREADS)
            s_bins[k] = 0;
    __syncthreads();

    const uint32_t lane = tid & 63u, wv = tid >> 6;
    u32x4 *tile = s_tile[wv];
    const uint8_t *base = a.slab + a.data_off;
    const uint64_t wstep = (uint64_t)gridDim.x * TILE_WAVES;
    uint64_t t = (uint64_t)blockIdx.x * TILE_WAVES + wv;
    // swizzled destination of the chunk this lane loads in instruction k:
    // chunk c = 64k + lane -> frame c>>2 (= 16k + lane>>2), part c&3
    const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
    u32x4 r0, r1, r2, r3;
    if (t < n_tiles) {
        const u32x4 *g = (const u32x4 *)(base + t * 4096u);
        r0 = ldg4<LNT>((const uint8_t *)(g + lane));
        r1 = ldg4<LNT>((const uint8_t *)(g + 64 + lane));
        r2 = ldg4<LNT>((const uint8_t *)(g + 128 + lane));
        r3 = ldg4<LNT>((const uint8_t *)(g + 192 + lane));
    }
    for (; t < n_tiles; t += wstep) {
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t f = 16u * k + fr_in_k;
            const u32x4 v = k == 0 ? r0 : k == 1 ? r1 : k == 2 ? r2 : r3;
            tile[f * 4u + (part ^ ((f >> 2) & 3u))] = v;
        }
        __builtin_amdgcn_wave_barrier();
        const uint64_t tn = t + wstep;
        if (SCHED == 0 && tn < n_tiles) { // prefetch the next tile while this one is parsed
            const u32x4 *g = (const u32x4 *)(base + tn * 4096u);
            r0 = ldg4<LNT>((const uint8_t *)(g + lane));
            r1 = ldg4<LNT>((const uint8_t *)(g + 64 + lane));
            r2 = ldg4<LNT>((const uint8_t *)(g + 128 + lane));
            r3 = ldg4<LNT>((const uint8_t *)(g + 192 + lane));
        }
        const uint32_t sw = (lane >> 2) & 3u;
        const u32x4 p0 = tile[lane * 4u + (0u ^ sw)];
        const u32x4 p1 = tile[lane * 4u + (1u ^ sw)];
        const u32x4 p2 = tile[lane * 4u + (2u ^ sw)];
        __builtin_amdgcn_wave_barrier();
        const uint64_t i = t * 64u + lane;
        FastHdr h;
        h.p = base + i * 64u;
        h.avail = a.slab_len - (a.data_off + i * 64u);
        h.w3 = p0.w;
        h.w5 = p1.y;
        h.w6 = p1.z;
        h.w7 = p1.w;
        h.w8 = p2.x;
        h.w9 = p2.y;
        if (SCHED == 0) {
            fast_finish<MODE, NTS>(a, i, h, s_t, s_reta, s_bins, count);
        } else if (SCHED == 2) {
            // first FIB gather (directory or tbl24) issued before the next
            // tile's loads, the second after them: the wave waits for
            // max(frame latency, both gathers) instead of their sum, and the
            // Toeplitz work runs while all three are in flight.  Both the
            // gather and the prefetch are unconditional (any ip indexes the
            // directory / tbl24 in bounds; the last tile re-reads itself), so
            // the compiler's in-order vmcnt bookkeeping can leave the prefetch
            // in flight when it waits for the gather.  Frames needing global
            // byte loads for the hash (IPv6, IPv4 options) are hashed after.
            const uint32_t et = bswap16(h.w3 & 0xffffu);
            const uint32_t dst = alignb(h.w8, h.w7, 2), ip = bswap32(dst);
            uint32_t e = 0;
            if (MODE == CNDP_MODE_L3FWD)
                e = a.dir16 ? a.dir16[ip >> 16] : a.tbl24[ip >> 8];
            {
                const uint64_t tp = tn < n_tiles ? tn : t;
                const u32x4 *g = (const u32x4 *)(base + tp * 4096u);
                r0 = ldg4<LNT>((const uint8_t *)(g + lane));
                r1 = ldg4<LNT>((const uint8_t *)(g + 64 + lane));
                r2 = ldg4<LNT>((const uint8_t *)(g + 128 + lane));
                r3 = ldg4<LNT>((const uint8_t *)(g + 192 + lane));
            }
            uint32_t hs = 0;
            bool slow = et == 0x86DDu;
            if (et == 0x0800u) {
                const uint32_t ihl = (h.w3 >> 16) & 0xfu;
                const uint32_t proto = h.w5 >> 24;
                const uint32_t frag = bswap16(h.w5 & 0xffffu) & 0x3fffu;
                hs = tz4(s_t, 0, alignb(h.w7, h.w6, 2)) ^ tz4(s_t, 4, dst);
                if (ihl >= 5 && (proto == 6u || proto == 17u) && frag == 0) {
                    if (ihl == 5)
                        hs ^= tz4(s_t, 8, alignb(h.w9, h.w8, 2));
                    else
                        slow = true;
                }
            }
            uint32_t nh = CNDP_NH_INVALID;
            if (MODE == CNDP_MODE_L3FWD && et == 0x0800u) {
                if (a.dir16 && (e & 1u))
                    e = a.pages[(e >> 1) * 256u + ((ip >> 8) & 0xffu)];
                if (e & 1u)
                    e = a.tbl8[(e >> 1) * 256u + (ip & 0xffu)];
                nh = e >> 1;
            }
            if (slow)
                hs = fast_hash<MODE>(a, h, s_t);
            if (RW) {
                // ip4_rewrite fused (ip4_rewrite.c:40-247): the block's 4 waves
                // hold the 4 tiles of one 256-packet graph burst; the burst's
                // rewrite stream is its edge-0 packets in order
                const bool f = nh_ready_rw(nh);
                const unsigned long long m = __ballot(f);
                const uint32_t below = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                uint32_t *cw = s_rwc[rw_par];
                rw_par ^= 1u;
                if (lane == 0)
                    cw[wv] = (uint32_t)__popcll(m);
                __syncthreads();
                uint32_t pre = 0, tot = 0;
#pragma unroll
                for (uint32_t k = 0; k < TILE_WAVES; k++) {
                    pre += k < wv ? cw[k] : 0u;
                    tot += cw[k];
                }
                uint32_t tx = 0xFFFFu;
                if (f) {
                    const uint32_t pos = pre + below, nh16 = nh & 0xffffu;
                    const struct cndp_rw_nh *e = &s_rw[nh16 < CNDP_RW_MAX_NH ? nh16 : 0];
                    const uint32_t len = nh16 < CNDP_RW_MAX_NH ? e->rewrite_len : 0u;
                    const uint32_t lenc = len < CNDP_RW_MAX_LEN ? len : CNDP_RW_MAX_LEN;
                    tx = nh16 < CNDP_RW_MAX_NH ? e->tx_node : 0u;
                    uint32_t *fd = (uint32_t *)tile;
                    const uint32_t sw = (lane >> 2) & 3u;
#define RW_DW(d) fd[((lane * 4u + (((d) >> 2) ^ sw)) << 2) | ((d) & 3u)]
                    const uint32_t d5 = RW_DW(5u), d6 = RW_DW(6u);
                    const uint32_t ttl = (d5 >> 16) & 0xffu, ck = d6 & 0xffffu;
                    const uint32_t *src = (const uint32_t *)e->rewrite_data;
                    for (uint32_t d = 0; d * 4 < lenc; d++) {
                        const uint32_t nb = lenc - d * 4;
                        const uint32_t keep = nb >= 4 ? 0u : (0xffffffffu << (nb * 8));
                        RW_DW(d) = (RW_DW(d) & keep) | (src[d] & ~keep);
                    }
                    uint32_t nck;
                    if (pos < (tot & ~3u)) {
                        const uint32_t c32 = ck + 1u;
                        nck = ((c32 & 0xffffu) + (c32 >> 16)) & 0xffffu;
                    } else {
                        const uint32_t c16 = (ck + 1u) & 0xffffu;
                        nck = (c16 + (c16 >= 0xffffu ? 1u : 0u)) & 0xffffu;
                    }
                    RW_DW(5u) = (RW_DW(5u) & 0xff00ffffu) | (((ttl - 1u) & 0xffu) << 16);
                    RW_DW(6u) = (RW_DW(6u) & 0xffff0000u) | nck;
#undef RW_DW
                }
                __builtin_amdgcn_wave_barrier();
                // write back the rewritten frames' first rw_parts 16-B parts
                // rw_parts == 4 with whole-tile write-back (CNDP_TUNE_RW_WB):
                // every frame of a tile holding a rewrite goes back as full
                // coalesced 1-KiB stores (unchanged frames rewrite their own bytes)
                const bool whole = a.rw_parts > 4u && m != 0ull;
#pragma unroll
                for (uint32_t k = 0; k < 4; k++) {
                    const uint32_t fk = 16u * k + fr_in_k;
                    if (whole || (part < a.rw_parts && ((m >> fk) & 1ull)))
                        *(u32x4 *)(const_cast<uint8_t *>(base) + (t * 64u + fk) * 64u + part * 16u) =
                            tile[fk * 4u + (part ^ ((fk >> 2) & 3u))];
                }
                __builtin_amdgcn_wave_barrier();
                a.tx_edge[i] = (uint16_t)tx;
            }
            fast_emit<MODE, NTS>(a, i, et, nh, hs, s_reta, s_bins, count);
        } else {
            // finish the dependent tbl24 -> tbl8 gathers first: vmcnt drains in
            // issue order, so a prefetch issued before them would be waited for
            const uint32_t nh = fast_lpm<MODE>(a, h);
            if (tn < n_tiles) {
                const u32x4 *g = (const u32x4 *)(base + tn * 4096u);
                r0 = ldg4<LNT>((const uint8_t *)(g + lane));
                r1 = ldg4<LNT>((const uint8_t *)(g + 64 + lane));
                r2 = ldg4<LNT>((const uint8_t *)(g + 128 + lane));
                r3 = ldg4<LNT>((const uint8_t *)(g + 192 + lane));
            }
            fast_finish<MODE, NTS, true>(a, i, h, s_t, s_reta, s_bins, count, nh);
        }
    }
    // ragged tail (frames past the last whole tile): per-lane path
    const uint64_t done = n_tiles * 64u;
    for (uint64_t i = done + (uint64_t)blockIdx.x * FAST_THREADS + tid; i < a.n;
         i += (uint64_t)gridDim.x * FAST_THREADS) {
        FastHdr h;
        fast_load<false>(a, i, h);
        fast_finish<MODE, false>(a, i, h, s_t, s_reta, s_bins, count);
    }
    if (count) {
        __syncthreads();
        for (uint32_t k = tid; k < a.n_bins + 2; k += FAST_THREADS)
            if (s_bins[k])
                atomicAdd(&a.bins[k], (unsigned long long)s_bins[k]);
    }
}


// ---------------------------------------------------------------------------
// Streamed wave-tile kernel (CNDP_TUNE_TILE 5, l3fwd / hash, packed 64-B slots).
// The per-tile work is cut into four stages that run one loop trip apart,
// so every FIB gather has a whole trip to come back and nothing waits on
// the newest frame loads:
//   A  tile c    LDS-stage the frames, parse, Toeplitz; gather 1 (/16
//                directory, or tbl24 without it)
//   B  tile c-1  gather 2 (directory page, or tbl8 without the directory)
//   C  tile c-2  gather 3 (tbl8 behind a page)
//   D  tile c-3  queue, bins and the result stores
// Frame tiles are loaded two trips ahead into two alternating register
// sets (the trip is unrolled by two).  Each trip issues its loads in the
// order  gathers(C, B, A) -> frame tile c+2 -> stores(D), so the vmcnt wait
// at the top of the next trip -- for the gathers and tile c+1 -- leaves
// tile c+2 and the stores in flight: a wave always has one to two 4-KiB
// tiles outstanding and never idles on an L2 round trip.
// ---------------------------------------------------------------------------
struct StreamLane { // one lane's packet in flight between stages
    uint32_t et, ip, hs;
    uint32_t e;   // FIB entry so far
    uint32_t raw; // the gather issued for it last trip (may still be in flight)
    bool sel;     // raw replaces e (resolved by the consumer, not at issue)
};

// c: tile of stage A, cn: the tile whose frames this trip loads, cd: stage D's
// tile (its stores only when dD); an index >= n_tiles stands for none
template <int MODE, bool NTS, bool LNT, int P>
__device__ __forceinline__ void stream_trip(const KArgs &a, uint64_t n_tiles, uint64_t c, uint64_t cn, uint64_t cd,
                                            bool dD, uint32_t lane, u32x4 *tile, u32x4 (&r)[2][4],
                                            StreamLane &sb, StreamLane &sc, StreamLane &sd, const uint32_t *s_t,
                                            const uint16_t *s_reta, uint32_t *s_bins, bool count)
{
    // Every load below is issued unconditionally (a safe index when its
    // result is not needed; past the wave's last tile the frame loads re-read
    // the slab's last tile, an L2 hit): the compiler's static vmcnt
    // bookkeeping then sees the same issue order on every path and waits only
    // for what is older than the newest frame tile.
    const uint8_t *base = a.slab + a.data_off;
    const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
    // D: tile c-3 -- its final entry came back with last trip's gather 3
    uint32_t nhD = CNDP_NH_INVALID;
    const uint32_t etD = sd.et, hsD = sd.hs;
    if (MODE == CNDP_MODE_L3FWD && etD == 0x0800u)
        nhD = (sd.sel ? sd.raw : sd.e) >> 1;
    StreamLane nd = sc, nc = sb, nb;
    if (MODE == CNDP_MODE_L3FWD) {
        // C: tile c-2 -- gather 3 (tbl8 behind a directory page)
        const uint32_t ec = sc.sel ? sc.raw : sc.e;
        nd.e = ec;
        nd.sel = a.dir16 && (ec & 1u);
        nd.raw = a.tbl8[nd.sel ? (ec >> 1) * 256u + (sc.ip & 0xffu) : 0u];
        // B: tile c-1 -- gather 2 (directory page, or tbl8 without the directory)
        const uint32_t eb = sb.sel ? sb.raw : 0u; // gather 1 was issued for IPv4 frames only
        nc.e = eb;
        nc.sel = (eb & 1u) != 0u;
        const uint32_t *t2 = a.dir16 ? a.pages : a.tbl8;
        const uint32_t i2 = a.dir16 ? (eb >> 1) * 256u + ((sb.ip >> 8) & 0xffu) : (eb >> 1) * 256u + (sb.ip & 0xffu);
        nc.raw = t2[nc.sel ? i2 : 0u];
    }
    // A: tile c -- stage, parse, hash, gather 1
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        const uint32_t f = 16u * k + fr_in_k;
        tile[f * 4u + (part ^ ((f >> 2) & 3u))] = r[P][k];
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t sw = (lane >> 2) & 3u;
    const u32x4 p0 = tile[lane * 4u + (0u ^ sw)];
    const u32x4 p1 = tile[lane * 4u + (1u ^ sw)];
    const u32x4 p2 = tile[lane * 4u + (2u ^ sw)];
    __builtin_amdgcn_wave_barrier();
    FastHdr h;
    const uint64_t i = (c < n_tiles ? c : n_tiles - 1u) * 64u + lane;
    h.p = base + i * 64u;
    h.avail = a.slab_len - (a.data_off + i * 64u);
    h.w3 = p0.w;
    h.w5 = p1.y;
    h.w6 = p1.z;
    h.w7 = p1.w;
    h.w8 = p2.x;
    h.w9 = p2.y;
    const uint32_t et = bswap16(h.w3 & 0xffffu);
    const uint32_t dst = alignb(h.w8, h.w7, 2);
    nb.et = et;
    nb.ip = bswap32(dst);
    nb.e = 0;
    nb.sel = et == 0x0800u; // non-IPv4: no lookup, no further gathers
    nb.raw = 0;
    if (MODE == CNDP_MODE_L3FWD)
        nb.raw = a.dir16 ? a.dir16[nb.ip >> 16] : a.tbl24[nb.ip >> 8];
    nb.hs = 0;
    bool slow = et == 0x86DDu;
    if (et == 0x0800u) {
        const uint32_t ihl = (h.w3 >> 16) & 0xfu;
        const uint32_t proto = h.w5 >> 24;
        const uint32_t frag = bswap16(h.w5 & 0xffffu) & 0x3fffu;
        nb.hs = tz4(s_t, 0, alignb(h.w7, h.w6, 2)) ^ tz4(s_t, 4, dst);
        if (ihl >= 5 && (proto == 6u || proto == 17u) && frag == 0) {
            if (ihl == 5)
                nb.hs ^= tz4(s_t, 8, alignb(h.w9, h.w8, 2));
            else
                slow = true;
        }
    }
    if (slow) // IPv6 tuple / IPv4 options: bytes past the staged 48
        nb.hs = fast_hash<MODE>(a, h, s_t);
    // frame tile c+2 into the register set just consumed
    {
        const u32x4 *g = (const u32x4 *)(base + (cn < n_tiles ? cn : n_tiles - 1u) * 4096u);
        r[P][0] = ldg4<LNT>((const uint8_t *)(g + lane));
        r[P][1] = ldg4<LNT>((const uint8_t *)(g + 64 + lane));
        r[P][2] = ldg4<LNT>((const uint8_t *)(g + 128 + lane));
        r[P][3] = ldg4<LNT>((const uint8_t *)(g + 192 + lane));
    }
    // D: the stores of tile c-3
    if (dD)
        fast_emit<MODE, NTS>(a, cd * 64u + lane, etD, nhD, hsD, s_reta, s_bins, count);
    sd = nd;
    sc = nc;
    sb = nb;
}

template <int MODE, bool NTS, bool LNT>
__global__ __launch_bounds__(FAST_THREADS) void k_classify_stream(KArgs a, uint64_t n_tiles)
{
    __shared__ uint32_t s_t[TAB4_POS * 256];
    __shared__ uint16_t s_reta[CNDP_RETA_MAX];
    __shared__ uint32_t s_bins[CNDP_BINS_MAX + 2];
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[TILE_WAVES][256];

    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < TAB4_POS * 256; k += FAST_THREADS)
        s_t[k] = a.ttab[k];
    for (uint32_t k = tid; k <= a.reta_mask; k += FAST_THREADS)
        s_reta[k] = a.reta[k];
    const bool count = a.bins != nullptr;
    if (count)
        for (uint32_t k = tid; k < a.n_bins + 2; k += FAST_THREADS)
            s_bins[k] = 0;
    __syncthreads();

    const uint32_t lane = tid & 63u, wv = tid >> 6;
    u32x4 *tile = s_tile[wv];
    const uint8_t *base = a.slab + a.data_off;
    const uint64_t wstep = (uint64_t)gridDim.x * TILE_WAVES;
    const uint64_t t0 = (uint64_t)blockIdx.x * TILE_WAVES + wv;
    const uint64_t nt_w = t0 < n_tiles ? (n_tiles - t0 + wstep - 1) / wstep : 0; // this wave's tiles
    u32x4 r[2][4];
#pragma unroll
    for (uint32_t s = 0; s < 2; s++) {
        const uint64_t ts = t0 + s * wstep;
        const u32x4 *g = (const u32x4 *)(base + (ts < n_tiles ? ts : n_tiles - 1u) * 4096u);
        r[s][0] = ldg4<LNT>((const uint8_t *)(g + lane));
        r[s][1] = ldg4<LNT>((const uint8_t *)(g + 64 + lane));
        r[s][2] = ldg4<LNT>((const uint8_t *)(g + 128 + lane));
        r[s][3] = ldg4<LNT>((const uint8_t *)(g + 192 + lane));
    }
    StreamLane sb = {0, 0, 0, 0, 0, false}, sc = sb, sd = sb;
    const uint64_t trips = nt_w ? nt_w + 3 : 0;
    for (uint64_t j = 0; j < trips; j += 2) {
        stream_trip<MODE, NTS, LNT, 0>(a, n_tiles, t0 + j * wstep, t0 + (j + 2) * wstep, t0 + (j - 3) * wstep,
                                       j >= 3 && j - 3 < nt_w, lane, tile, r, sb, sc, sd, s_t, s_reta, s_bins, count);
        if (j + 1 < trips)
            stream_trip<MODE, NTS, LNT, 1>(a, n_tiles, t0 + (j + 1) * wstep, t0 + (j + 3) * wstep,
                                           t0 + (j - 2) * wstep, j >= 2 && j - 2 < nt_w, lane, tile, r, sb, sc, sd,
                                           s_t, s_reta, s_bins, count);
    }
    // ragged tail (frames past the last whole tile): per-lane path
    const uint64_t done = n_tiles * 64u;
    for (uint64_t i = done + (uint64_t)blockIdx.x * FAST_THREADS + tid; i < a.n;
         i += (uint64_t)gridDim.x * FAST_THREADS) {
        FastHdr h;
        fast_load<false>(a, i, h);
        fast_finish<MODE, false>(a, i, h, s_t, s_reta, s_bins, count);
    }
    if (count) {
        __syncthreads();
        for (uint32_t k = tid; k < a.n_bins + 2; k += FAST_THREADS)
            if (s_bins[k])
                atomicAdd(&a.bins[k], (unsigned long long)s_bins[k]);
    }
}


// The same stages with the block's tiles (blockIdx + k * gridDim) handed to
// its BW waves by an LDS counter (CNDP_TUNE_STREAM_BAL): one BW * 64-thread
// block a CU, so the CU's waves share one pool and the ones the SQ's
// oldest-first arbitration favours take more tiles -- no wave is left with a
// static share after the others have finished.  Each wave's first three
// tiles are static; every trip draws the index it will load two trips
// later, a trip ahead of its use (the LDS atomic's return is waited for with
// the trip's other LDS traffic).
#define STREAM_BW 8
template <int MODE, bool NTS, bool LNT>
__global__ __launch_bounds__(STREAM_BW * 64) void k_classify_stream_bal(KArgs a, uint64_t n_tiles)
{
    __shared__ uint32_t s_t[TAB4_POS * 256];
    __shared__ uint16_t s_reta[CNDP_RETA_MAX];
    __shared__ uint32_t s_bins[CNDP_BINS_MAX + 2];
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[STREAM_BW][256];
    __shared__ uint32_t s_next;
    constexpr uint32_t NT = STREAM_BW * 64;

    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < TAB4_POS * 256; k += NT)
        s_t[k] = a.ttab[k];
    for (uint32_t k = tid; k <= a.reta_mask; k += NT)
        s_reta[k] = a.reta[k];
    const bool count = a.bins != nullptr;
    if (count)
        for (uint32_t k = tid; k < a.n_bins + 2; k += NT)
            s_bins[k] = 0;
    if (tid == 0)
        s_next = 3u * STREAM_BW;
    const uint32_t lane = tid & 63u, wv = tid >> 6;
    u32x4 *tile = s_tile[wv];
    const uint8_t *base = a.slab + a.data_off;
    const uint64_t G = gridDim.x, b = blockIdx.x;
    const uint64_t NONE = ~0ull;
    // the block's tiles, G apart (in the static schedule's round order instead,
    // k_cnet_defer's BAL mapping, C3 is 1 % slower)
    const uint64_t nk = b < n_tiles ? (n_tiles - b + G - 1) / G : 0;
    auto tile_of = [&](uint64_t k) { return k < nk ? b + k * G : NONE; };
    // the wave's first three tiles, static; two of them loaded now
    uint64_t q0 = tile_of(wv), q1 = tile_of(wv + STREAM_BW), q2 = tile_of(wv + 2u * STREAM_BW);
    u32x4 r[2][4];
#pragma unroll
    for (uint32_t s = 0; s < 2; s++) {
        const uint64_t ts = s ? q1 : q0;
        const u32x4 *g = (const u32x4 *)(base + (ts < n_tiles ? ts : n_tiles - 1u) * 4096u);
        r[s][0] = ldg4<LNT>((const uint8_t *)(g + lane));
        r[s][1] = ldg4<LNT>((const uint8_t *)(g + 64 + lane));
        r[s][2] = ldg4<LNT>((const uint8_t *)(g + 128 + lane));
        r[s][3] = ldg4<LNT>((const uint8_t *)(g + 192 + lane));
    }
    __syncthreads();
    // the index after q2, drawn a trip ahead (lane 0's LDS atomic)
    auto draw = [&](uint64_t prev) -> uint32_t {
        uint32_t v = 0;
        if (prev != NONE && lane == 0)
            v = atomicAdd(&s_next, 1u);
        return v;
    };
    uint32_t kv = draw(q2);
    uint64_t h1 = NONE, h2 = NONE, h3 = NONE; // the tiles of stages B, C, D
    StreamLane sb = {0, 0, 0, 0, 0, false}, sc = sb, sd = sb;
    for (;;) {
        if (q0 == NONE && h1 == NONE && h2 == NONE && h3 == NONE) // wave-uniform
            break;
        stream_trip<MODE, NTS, LNT, 0>(a, n_tiles, q0, q2, h3, h3 != NONE, lane, tile, r, sb, sc, sd, s_t, s_reta,
                                       s_bins, count);
        {
            const uint64_t qn = q2 == NONE ? NONE : tile_of(__builtin_amdgcn_readfirstlane(kv));
            kv = draw(qn);
            h3 = h2;
            h2 = h1;
            h1 = q0;
            q0 = q1;
            q1 = q2;
            q2 = qn;
        }
        if (q0 == NONE && h1 == NONE && h2 == NONE && h3 == NONE)
            break;
        stream_trip<MODE, NTS, LNT, 1>(a, n_tiles, q0, q2, h3, h3 != NONE, lane, tile, r, sb, sc, sd, s_t, s_reta,
                                       s_bins, count);
        {
            const uint64_t qn = q2 == NONE ? NONE : tile_of(__builtin_amdgcn_readfirstlane(kv));
            kv = draw(qn);
            h3 = h2;
            h2 = h1;
            h1 = q0;
            q0 = q1;
            q1 = q2;
            q2 = qn;
        }
    }
    // ragged tail (frames past the last whole tile): per-lane path
    const uint64_t done = n_tiles * 64u;
    for (uint64_t i = done + (uint64_t)blockIdx.x * NT + tid; i < a.n; i += (uint64_t)gridDim.x * NT) {
        FastHdr h;
        fast_load<false>(a, i, h);
        fast_finish<MODE, false>(a, i, h, s_t, s_reta, s_bins, count);
    }
    if (count) {
        __syncthreads();
        for (uint32_t k = tid; k < a.n_bins + 2; k += NT)
            if (s_bins[k])
                atomicAdd(&a.bins[k], (unsigned long long)s_bins[k]);
    }
}

// ---------------------------------------------------------------------------
// cnet classify: eth_rx (cne_get_ptype) -> ptype -> ip4_input / ip6_input.
// ---------------------------------------------------------------------------
#define CNET_THREADS 512
#define WIN_DW 16      /* 64-byte window per lane */
#define ROW_DW 17      /* padded row: lane L dword k sits in bank (L + k) % 32 */

struct Win {
    const uint32_t *row; // LDS row, bytes 0..63 of the frame (zero past avail)
    const uint8_t *g;
    uint64_t avail;
    __device__ __forceinline__ uint32_t ld32(uint32_t o) const
    {
        if (o + 4 <= 64) {
            const uint32_t lo = row[o >> 2], hi = row[(o >> 2) + 1];
            return alignb(hi, lo, o & 3u);
        }
        return gld32(g, avail, o);
    }
    __device__ __forceinline__ uint32_t b8(uint32_t o) const
    {
        return o < 64 ? (row[o >> 2] >> ((o & 3u) * 8)) & 0xffu : gbyte(g, avail, o);
    }
    __device__ __forceinline__ uint32_t raw16(uint32_t o) const { return ld32(o) & 0xffffu; }
    __device__ __forceinline__ uint32_t be16(uint32_t o) const { return bswap16(ld32(o) & 0xffffu); }
    __device__ __forceinline__ uint32_t be32(uint32_t o) const { return bswap32(ld32(o)); }
};

#define BE16C(x) ((uint32_t)((((x) & 0xffu) << 8) | (((x) >> 8) & 0xffu)))

struct Lens {
    uint32_t l2, l3, l4; // outer lengths (cne_net_hdr_lens); unset ones stay 0
};

__device__ __forceinline__ uint32_t pt_l3_ip(uint32_t vihl)
{
    return vihl == 0x45u ? 0x10u : (vihl >= 0x46u && vihl <= 0x4fu) ? 0x30u : 0u;
}
__device__ __forceinline__ uint32_t pt_l4(uint32_t p)
{
    // independent selects ORed (a ternary chain compiles to a branch tree)
    return (p == 17u ? 0x200u : 0u) | (p == 6u ? 0x100u : 0u) | (p == 132u ? 0x400u : 0u);
}
__device__ __forceinline__ bool v6_ext(uint32_t p)
{
    return p == 0u || p == 43u || p == 44u || p == 50u || p == 51u || p == 60u;
}


// pktmbuf_ptype.c:426-468 (skip_ip6_ext); returns -1 past 5 headers
template <class W>
__device__ int skip_v6_ext(const W &w, uint32_t proto, uint32_t &off, int &frag)
{
    frag = 0;
    for (int i = 0; i < 5; i++) {
        if (proto == 0u || proto == 43u || proto == 60u) {
            const uint32_t x = w.ld32(off);
            proto = x & 0xffu;
            off += (((x >> 8) & 0xffu) + 1u) * 8u;
        } else if (proto == 44u) {
            proto = w.b8(off);
            off += 8;
            frag = 1;
            return (int)proto;
        } else if (proto == 59u) {
            return 0;
        } else {
            return (int)proto;
        }
    }
    return -1;
}

// cne_get_ptype, pktmbuf_ptype.c:472-744, all layers (CNE_PTYPE_ALL_MASK).
// Only l2_len / l3_len are consumed downstream (eth_rx.c:56-60 + the input
// nodes), so the inner-header lengths are not tracked; the ptype bits are.
template <class W>
__device__ uint32_t get_ptype(const W &w, Lens &ln)
{
    uint32_t pt = 0x1u, off = 14, proto = w.raw16(12);
    int ret;
    ln.l2 = 14;
    ln.l3 = 0;
    ln.l4 = 0;
    if (proto == BE16C(0x0806u))
        return 0x3u;
    if (proto != BE16C(0x0800u)) {
        if (proto == BE16C(0x8100u)) {
            pt = 0x6u;
            proto = w.raw16(off + 2);
            off += 4;
            ln.l2 += 4;
        } else if (proto == BE16C(0x88A8u)) {
            pt = 0x7u;
            proto = w.raw16(off + 6);
            off += 8;
            ln.l2 += 8;
        } else if (proto == BE16C(0x8847u) || proto == BE16C(0x8848u)) {
            return pt; // :541-556 never sets the MPLS bits
        }
    }
    if (proto == BE16C(0x0800u)) {
        const uint32_t ip = off;
        const uint32_t x0 = w.ld32(ip);
        pt |= pt_l3_ip(x0 & 0xffu);
        ln.l3 = (x0 & 0xfu) * 4u;
        off += ln.l3;
        const uint32_t x6 = w.ld32(ip + 6);
        if ((x6 & 0xffffu) & BE16C(0x3fffu))
            return pt | 0x300u;
        proto = (x6 >> 24) & 0xffu; // byte ip+9
        pt |= pt_l4(proto);
    } else if (proto == BE16C(0x86DDu)) {
        int frag = 0;
        proto = w.b8(off + 6);
        ln.l3 = 40;
        off += 40;
        pt |= v6_ext(proto) ? 0xc0u : 0x40u;
        if ((pt & 0xf0u) == 0xc0u) {
            ret = skip_v6_ext(w, proto, off, frag);
            if (ret < 0)
                return pt;
            proto = (uint32_t)ret;
            ln.l3 = off - ln.l2;
        }
        if (proto == 0u)
            return pt;
        if (frag)
            return pt | 0x300u;
        pt |= pt_l4(proto);
    }
    const uint32_t l4t = pt & 0xf00u;
    if (l4t == 0x200u) {
        ln.l4 = 8;
        const uint32_t dport = w.raw16(ln.l2 + ln.l3 + 2);
        if (dport == BE16C(2152u))
            pt |= 0x8000u;
        else if (dport == BE16C(2123u))
            pt |= 0x7000u;
        return pt;
    }
    if (l4t == 0x100u) {
        ln.l4 = (w.b8(ln.l2 + ln.l3 + 12) & 0xf0u) >> 2; // TCP data offset
        return pt;
    }
    if (l4t == 0x400u) {
        ln.l4 = 12;
        return pt;
    }

    // tunnels (:372-411)
    if (proto == 47u) {
        const uint32_t x = w.ld32(off);
        const uint32_t flags = bswap16(x & 0xffffu) >> 12;
        const uint32_t olen = flags == 0 ? 4 : (flags == 1 || flags == 2 || flags == 8) ? 8
                            : (flags == 3 || flags == 9 || flags == 10)           ? 12
                            : flags == 11                                         ? 16
                                                                                  : 0;
        if (olen) {
            proto = x >> 16;
            off += olen;
            pt |= proto == BE16C(0x6558u) ? 0x4000u : 0x2000u;
        }
    } else if (proto == 4u) {
        proto = BE16C(0x0800u);
        pt |= 0x1000u;
    } else if (proto == 41u) {
        proto = BE16C(0x86DDu);
        pt |= 0x1000u;
    }
    // inner headers (:617-744); note the reference compares IP protocol
    // numbers against htobe16() ethertypes here, so proto 8 / 129 alias
    // IPv4 / VLAN -- reproduced as is.
    if (proto == BE16C(0x6558u)) {
        pt |= 0x10000u;
        proto = w.raw16(off + 12);
        off += 14;
    }
    if (proto == BE16C(0x8100u)) {
        pt = (pt & ~0xf0000u) | 0x20000u;
        proto = w.raw16(off + 2);
        off += 4;
    } else if (proto == BE16C(0x88A8u)) {
        pt = (pt & ~0xf0000u) | 0x30000u;
        proto = w.raw16(off + 6);
        off += 8;
    }
    if (proto == BE16C(0x0800u)) {
        const uint32_t x0 = w.ld32(off);
        const uint32_t v = x0 & 0xffu;
        pt |= v == 0x45u ? 0x100000u : (v >= 0x46u && v <= 0x4fu) ? 0x200000u : 0u;
        const uint32_t x6 = w.ld32(off + 6);
        off += (x0 & 0xfu) * 4u;
        if ((x6 & 0xffffu) & BE16C(0x3fffu))
            return pt | 0x3000000u;
        const uint32_t p4 = (x6 >> 24) & 0xffu;
        pt |= p4 == 17u ? 0x2000000u : p4 == 6u ? 0x1000000u : p4 == 132u ? 0x4000000u : 0u;
    } else if (proto == BE16C(0x86DDu)) {
        int frag = 0;
        proto = w.b8(off + 6);
        off += 40;
        pt |= v6_ext(proto) ? 0x500000u : 0x300000u;
        if ((pt & 0xf00000u) == 0x500000u) {
            ret = skip_v6_ext(w, proto, off, frag);
            if (ret < 0)
                return pt;
            proto = (uint32_t)ret;
        }
        if (proto == 0u)
            return pt;
        if (frag)
            return pt | 0x3000000u;
        pt |= proto == 17u ? 0x2000000u : proto == 6u ? 0x1000000u : proto == 132u ? 0x4000000u : 0u;
    }
    return pt;
}

// eth_rx.c:43-60 packed: tx_offload l2:7 | l3:9 | l4:8, ol_flags >> 32 in bits 29..31
__device__ __forceinline__ uint32_t rx_meta(const Lens &ln, uint32_t w0, uint32_t w1, uint32_t et_raw)
{
    uint32_t m = (ln.l2 & 0x7fu) | ((ln.l3 & 0x1ffu) << 7) | ((ln.l4 & 0xffu) << 16);
    if (et_raw == BE16C(0x86DDu))
        m |= 1u << 31;                                   // CNE_MBUF_TYPE_IPv6
    if (w0 == 0xffffffffu && (w1 & 0xffffu) == 0xffffu)
        m |= 1u << 30;                                   // CNE_MBUF_TYPE_BCAST
    else if (w0 & 1u)
        m |= 1u << 29;                                   // CNE_MBUF_TYPE_MCAST
    return m;
}

// lib/cnet/ptype/ptype.c:32-46 (indexed by ptype & 0xffff)
__host__ __device__ __forceinline__ constexpr uint32_t cnet_edge(uint32_t pt)
{
    // branch-free: bitwise ORs of the compares, selects (it runs in the
    // speculation walks once per group)
    const uint32_t l = pt & 0xffffu;
    uint32_t e = l == 0x0003u ? 2u : 0u;                                             // FRAME_PUNT
    e = ((l == 0x0211u) | (l == 0x0111u) | (l == 0x0231u) | (l == 0x0291u)) ? 3u : e; // IP4_INPUT
    e = ((l == 0x0241u) | (l == 0x0141u) | (l == 0x02c1u) | (l == 0x02e1u)) ? 4u : e; // IP6_INPUT
    e = ((l == 0x8211u) | (l == 0x8241u)) ? 5u : e;                                  // GTPU_INPUT
    return e;                                                                         // else PKT_DROP
}

__device__ __forceinline__ uint32_t spec_sig(uint32_t l) { return ((l & 0xffu) << 3) | cnet_edge(l); }

// low bytes shared by types of different p_nxt (the others all go to pkt_drop)
#define SPEC_LOWS 7
__host__ __device__ __forceinline__ constexpr uint32_t spec_lowslot(uint32_t low)
{
    return low == 0x03u ? 0u : low == 0x11u ? 1u : low == 0x31u ? 2u : low == 0x91u ? 3u
         : low == 0x41u ? 4u : low == 0xc1u ? 5u : low == 0xe1u ? 6u : SPEC_LOWS;
}

// The edge every frame of a canonical tile (k_cnet_defer's tile words) has
// for its low byte: 0x11 (IPv4) -> ip4_input, 0x41 (IPv6) -> ip6_input; a
// canonical tile holds no other low byte.  0xFF: none.
__device__ __forceinline__ uint32_t spec_canon(uint32_t low) { return low == 0x11u ? 3u : low == 0x41u ? 4u : 0xFFu; }

// cnet_edge and the speculation summary bit of a type, by (high-byte class
// hi, low byte): a 5 x 256 table of u16 built at compile time and copied to
// LDS by the kernels that use it.  hi = 0..3 for high bytes 0x00, 0x01,
// 0x02, 0x82 (the only ones any p_nxt entry other than pkt_drop has,
// ptype.c:32-46), 4 for every other.  Entry = p_nxt << 6 | em bit, the em
// bit being 6 * spec_lowslot(low) + p_nxt, or 63 (masked off) outside the
// slots.  One LDS read + ~6 ops instead of the compare chains.
#define CNET_LUT_N (5 * 256)
struct alignas(16) CnetLut {
    uint16_t v[CNET_LUT_N];
};
constexpr CnetLut make_cnet_lut()
{
    CnetLut t{};
    for (uint32_t hi = 0; hi < 5; hi++)
        for (uint32_t k = 0; k < 256; k++) {
            const uint32_t hb = hi == 0 ? 0x00u : hi == 1 ? 0x01u : hi == 2 ? 0x02u : 0x82u;
            const uint32_t e = hi < 4 ? cnet_edge((hb << 8) | k) : 0u, q = spec_lowslot(k);
            t.v[hi * 256 + k] = (uint16_t)((e << 6) | (q < SPEC_LOWS ? 6 * q + e : 63u));
        }
    return t;
}
__constant__ CnetLut g_cnet_lut = make_cnet_lut();
static_assert(make_cnet_lut().v[2 * 256 + 0x11] == (3u << 6 | 9u), "cnet LUT");
static_assert(make_cnet_lut().v[3 * 256 + 0x41] == (5u << 6 | 29u), "cnet LUT");
static_assert(make_cnet_lut().v[0 * 256 + 0x03] == (2u << 6 | 2u), "cnet LUT");
static_assert(make_cnet_lut().v[4 * 256 + 0x55] == 63u, "cnet LUT");
__device__ __forceinline__ void cnet_lut_fill(uint16_t *lut, uint32_t tid, uint32_t nthr)
{
    for (uint32_t k = tid; k < CNET_LUT_N / 2; k += nthr) // two entries per 4-B copy
        ((uint32_t *)lut)[k] = ((const uint32_t *)g_cnet_lut.v)[k];
}
// the same copy in two halves for 256-thread blocks: the loads at a kernel's
// start, in flight with its other first loads, the LDS stores later
struct LutRegs {
    uint32_t v[3];
};
__device__ __forceinline__ LutRegs cnet_lut_load256(uint32_t tid)
{
    static_assert(CNET_LUT_N / 2 <= 3 * 256, "three words a thread");
    LutRegs r;
#pragma unroll
    for (uint32_t j = 0; j < 3; j++) {
        const uint32_t k = tid + 256u * j;
        r.v[j] = k < CNET_LUT_N / 2 ? ((const uint32_t *)g_cnet_lut.v)[k] : 0u;
    }
    return r;
}
__device__ __forceinline__ void cnet_lut_store256(uint16_t *lut, uint32_t tid, const LutRegs &r)
{
#pragma unroll
    for (uint32_t j = 0; j < 3; j++) {
        const uint32_t k = tid + 256u * j;
        if (k < CNET_LUT_N / 2)
            ((uint32_t *)lut)[k] = r.v[j];
    }
}
__device__ __forceinline__ uint32_t cnet_lut_x(const uint16_t *lut, uint32_t l)
{
    const uint32_t h = (l >> 8) & 0xffu;
    const uint32_t hi = h < 3u ? h : h == 0x82u ? 3u : 4u;
    return lut[hi * 256u + (l & 0xffu)];
}
__device__ __forceinline__ uint32_t cnet_edge_l(const uint16_t *lut, uint32_t l) { return cnet_lut_x(lut, l) >> 6; }

// Burst / chunk maps store their target states tagged with the target's
// signature class (state | class << 16; SPEC_UNCH = keep the state), so map
// composition never recomputes a signature.
__device__ __forceinline__ uint32_t spec_tag(uint32_t st, const uint8_t *class_id)
{
    return st == 0xFFFFFFFFu ? st : (st & 0xffffu) | ((uint32_t)class_id[spec_sig(st)] << 16);
}

// OR the signature bit of each active lane into a 64-word LDS bitmap with one
// LDS atomic per distinct word in the wave
__device__ __forceinline__ void spec_mark(uint32_t *s_f, bool on, uint32_t g)
{
    const uint32_t w = g >> 5, bit = 1u << (g & 31u);
    bool todo = on;
    while (__any(todo)) {
        const uint32_t lead = __shfl(w, __ffsll((unsigned long long)__ballot(todo)) - 1);
        const bool mine = todo && w == lead;
        const unsigned long long mm = __ballot(mine);
        uint32_t v = mine ? bit : 0u;
        for (int o = 32; o > 0; o >>= 1)
            v |= __shfl_xor(v, o);
        if (mine && (uint32_t)__lane_id() == (uint32_t)(__ffsll(mm) - 1))
            atomicOr(&s_f[lead], v);
        todo = todo && !mine;
    }
}


__device__ __forceinline__ void spec_classes(uint32_t t, uint32_t *flags, uint8_t *class_id, uint32_t *meta,
                             const uint16_t *__restrict__ pt, uint32_t n, uint32_t B, uint64_t nb,
                             uint32_t allow_skip, uint32_t *wl_n, uint32_t *bar, uint32_t *hint);

// The speculation classes pass, folded into k_classify_cnet (no launch of its
// own): every block takes an arrival ticket once its flag ORs (device
// atomics) and, if it parsed frames, its type stores have left -- each wave's
// vmcnt(0), a block barrier, then a release fence by a block that stored --
// and the block that draws the last ticket acquires and runs spec_classes
// with its wave 0.  The ticket is two-level (MI355X_MICROARCH.md fanin: one
// word takes ~88 returning atomics per µs, 512 blocks would queue ~6 µs on
// it): block b counts on word b % 8, the last of each group on word 8
// (words 128 B apart).
__device__ __forceinline__ void cnet_spec_tail(const KArgs &a, bool stored)
{
    __shared__ uint32_t s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (stored)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const uint32_t G = gridDim.x, g = blockIdx.x & 7u, ng = G < 8u ? G : 8u;
        const uint32_t in_g = (G - g + 7u) / 8u; // blocks of group g
        bool last = __hip_atomic_fetch_add(&a.spec_ticket[32u * g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                    in_g - 1u;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent"); // pass the group's releases on
            last = __hip_atomic_fetch_add(&a.spec_ticket[32u * 8u], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   ng - 1u;
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last || threadIdx.x >= 64)
        return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (threadIdx.x < 9)
        a.spec_ticket[32u * threadIdx.x] = 0; // for the next launch (kernel boundary)
    const uint64_t nb = ((uint64_t)a.n + a.spec_B - 1) / a.spec_B;
    spec_classes(threadIdx.x, a.spec_flags, a.spec_cls, a.spec_meta, a.spec_t16, a.n, a.spec_B, nb, a.spec_allow,
                 a.wl_n, a.spec_bar, a.spec_hint);
}

// cne_get_ptype + eth_rx + ptype + ip4_input / ip6_input for frame i, one
// lane, over the lane's LDS row (ROW_DW words; row[WIN_DW] must be 0)
__device__ __forceinline__ void cnet_general(const KArgs &a, uint64_t i, uint32_t *row, const uint32_t *s_t,
                                             const uint16_t *s_reta, uint32_t *s_bins, uint32_t *s_sf, bool count)
{
    const uint64_t base = (a.offsets ? a.offsets[i] : i * a.stride) + a.data_off;
    const uint8_t *p = a.slab + base;
    const uint64_t avail = base < a.slab_len ? a.slab_len - base : 0;
    // stage the 64-byte header window (bounded) into this lane's LDS row
    if (avail >= 64 && (base & 15u) == 0) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 q = *(const uint4 *)(p + 16 * k);
            row[4 * k + 0] = q.x;
            row[4 * k + 1] = q.y;
            row[4 * k + 2] = q.z;
            row[4 * k + 3] = q.w;
        }
    } else {
        for (int k = 0; k < WIN_DW; k++)
            row[k] = gld32(p, avail, 4u * (uint32_t)k);
    }
    const Win w{row, p, avail};
    if (a.win) // the node queue's metadata source (k_mq_cnet_post)
        for (int k = 0; k < 4; k++)
            a.win[4 * i + k] = (u32x4){row[4 * k], row[4 * k + 1], row[4 * k + 2], row[4 * k + 3]};
    Lens ln;
    const uint32_t pt = get_ptype(w, ln);
    if (a.ptype)
        a.ptype[i] = pt;
    if (a.rxmeta)
        a.rxmeta[i] = rx_meta(ln, row[0], row[1], row[3] & 0xffffu);
    const uint32_t l3 = pt & 0xf0u, l4t = pt & 0xf00u;
    const uint32_t ip = ln.l2;
    const bool l4ok = l4t == 0x100u || l4t == 0x200u;
    uint32_t h = 0, nh = CNDP_NH_INVALID, edge;
    if (l3 != 0u && !(l3 & 0x40u)) {
        h = tz4(s_t, 0, w.ld32(ip + 12)) ^ tz4(s_t, 4, w.ld32(ip + 16));
        if (l4ok)
            h ^= tz4(s_t, 8, w.ld32(ip + ln.l3));
    } else if (l3 & 0x40u) {
#pragma unroll
        for (uint32_t k = 0; k < 8; k++)
            h ^= tz4(s_t, 4 * k, w.ld32(ip + 8 + 4 * k));
        if (l4ok)
            h ^= tz4(s_t, 32, w.ld32(ip + ln.l3));
    }
    const uint32_t pe = cnet_edge(pt);
    // with the speculation model, frames of the types a quiet 4-group can
    // carry into ip4/ip6_input get the input node's result as well
    const uint32_t lb = pt & 0xffu;
    const bool alt4 = a.spec_nh && (lb == 0x11u || lb == 0x31u || lb == 0x91u);
    const bool alt6 = a.spec_nh && (lb == 0x41u || lb == 0xc1u || lb == 0xe1u);
    bool has = false;
    if (pe == 3u || alt4) {
        // ip4_input.c:121-140: total_length < buf_len && cksum == 0
        const uint32_t x0 = w.ld32(ip);
        const uint32_t hl = (x0 & 0xfu);
        uint32_t sum = 0;
        for (uint32_t k = 0; k < hl; k++) {
            const uint32_t x = k == 0 ? x0 : w.ld32(ip + 4 * k);
            sum += (x & 0xffffu) + (x >> 16);
        }
        sum = (sum >> 16) + (sum & 0xffffu);
        sum = (sum >> 16) + (sum & 0xffffu);
        const bool ok = bswap16(x0 >> 16) < a.buf_len && ((~sum) & 0xffffu) == 0u;
        const uint32_t dip = ok ? w.be32(ip + 16) : 0u;
        nh = a.dir16 ? lpm4d(a.dir16, a.pages, a.tbl8, dip) : lpm4(a.tbl24, a.tbl8, dip);
        has = true;
    } else if (pe == 4u || alt6) {
        // ip6_input.c:115-135: payload_len < buf_len, else dip = ::
        const bool ok = w.be16(ip + 4) < a.buf_len;
        uint32_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
        if (ok) {
            d0 = w.ld32(ip + 24);
            d1 = w.ld32(ip + 28);
            d2 = w.ld32(ip + 32);
            d3 = w.ld32(ip + 36);
        }
        // trie.h:126-134
        uint32_t e = a.tbl24_6[((d0 & 0xffu) << 16) | (d0 & 0xff00u) | ((d0 >> 16) & 0xffu)];
        uint32_t j = 3;
        while ((e & 1u) && j < 16) {
            const uint32_t wd = j < 4 ? d0 : j < 8 ? d1 : j < 12 ? d2 : d3;
            const uint32_t byte = (wd >> ((j & 3u) * 8)) & 0xffu;
            e = a.tbl8_6[(e >> 1) * 256u + byte];
            j++;
        }
        nh = e >> 1;
        has = true;
    }
    if (a.spec_nh) {
        if (has && (!a.nh || (pe != 3u && pe != 4u)))
            a.spec_nh[i] = nh;
        a.spec_t16[i] = (uint16_t)pt;
        spec_mark(s_sf, true, spec_sig(pt & 0xffffu));
    }
    if (pe == 3u || pe == 4u) {
        edge = nh >> 24;
    } else {
        nh = CNDP_NH_INVALID;
        edge = 0x80u | pe;
    }
    const uint32_t q = s_reta[h & a.reta_mask];
    if (a.nh)
        a.nh[i] = nh;
    if (a.hash)
        a.hash[i] = h;
    if (a.queue)
        a.queue[i] = (uint16_t)q;
    if (a.edge)
        a.edge[i] = (uint8_t)edge;
    if (count)
        atomicAdd(&s_bins[bin_of<CNDP_MODE_CNET>(nh, edge, q, a.n_bins)], 1u);
}

template <bool WL>
__global__ __launch_bounds__(CNET_THREADS) void k_classify_cnet(KArgs a)
{
    __shared__ uint32_t s_t[TAB_POS * 256];
    __shared__ uint32_t s_win[CNET_THREADS * ROW_DW];
    __shared__ uint16_t s_reta[CNDP_RETA_MAX];
    __shared__ uint32_t s_bins[CNDP_BINS_MAX + 2];
    __shared__ uint32_t s_sf[64]; // type signatures seen (speculation model)

    const uint32_t tid = threadIdx.x;
    // WL: nothing left for this block -- it only takes its arrival ticket
    if (WL && (uint64_t)blockIdx.x * CNET_THREADS >= *a.wl_n) {
        if (a.spec_meta)
            cnet_spec_tail(a, false);
        return;
    }
    if (tid < 64)
        s_sf[tid] = 0;
    for (uint32_t k = tid; k < TAB_POS * 256; k += CNET_THREADS)
        s_t[k] = a.ttab[k];
    for (uint32_t k = tid; k <= a.reta_mask; k += CNET_THREADS)
        s_reta[k] = a.reta[k];
    const bool count = a.bins != nullptr;
    if (count)
        for (uint32_t k = tid; k < a.n_bins + 2; k += CNET_THREADS)
            s_bins[k] = 0;
    __syncthreads();

    uint32_t *row = s_win + tid * ROW_DW;
    row[WIN_DW] = 0;
    const uint64_t step = (uint64_t)gridDim.x * CNET_THREADS;
    // WL: the frames k_cnet_stream left to the general parse (a.wl[0 .. *a.wl_n))
    const uint64_t n_it = WL ? (uint64_t)*a.wl_n : a.n;
    for (uint64_t j = (uint64_t)blockIdx.x * CNET_THREADS + tid; j < n_it; j += step) {
        const uint64_t i = WL ? (uint64_t)a.wl[j] : j;
        cnet_general(a, i, row, s_t, s_reta, s_bins, s_sf, count);
    }
    if (count || a.spec_flags)
        __syncthreads();
    if (count)
        for (uint32_t k = tid; k < a.n_bins + 2; k += CNET_THREADS)
            if (s_bins[k])
                atomicAdd(&a.bins[k], (unsigned long long)s_bins[k]);
    if (a.spec_flags && tid < 64 && s_sf[tid])
        atomicOr(&a.spec_flags[tid], s_sf[tid]);
    if (a.spec_meta)
        cnet_spec_tail(a, true);
}

// ---------------------------------------------------------------------------
// cnet classify, wave-tile form (default for CNDP_MODE_CNET).  Same outputs as
// k_classify_cnet, restructured for latency:
//  * a wave owns 64 consecutive packets; their 64-B windows are fetched 4
//    lanes per frame (one 16-B load each, so a wave instruction covers 16
//    whole windows) into the swizzled LDS tile, for any stride / offsets;
//  * per tile: parse from LDS, issue the first FIB gather (/16 directory,
//    tbl24 or IPv6 tbl24), then the next tile's window loads, then the
//    Toeplitz hash from the LDS tables while both are in flight, then the
//    rest of the gather chain;
//  * IPv4 and IPv6 lanes share one hash loop and one gather-chain loop, so
//    a mixed wave pays max(v4, v6) steps instead of their sum.
// Frames that are not 16-B aligned or have < 64 bytes before the slab end
// are staged with bounded byte loads (zero past the end), like Win.
// ---------------------------------------------------------------------------
// the balanced k_cnet_defer (CNDP_TUNE_STREAM_BAL): one block of this many
// threads a CU, all of the CU's waves sharing one LDS counter
#ifndef CD_BAL_THREADS
#define CD_BAL_THREADS 1024
#endif
#ifndef CT_THREADS
#define CT_THREADS 512
#endif
#define CT_WAVES (CT_THREADS / 64)

// frame base (bytes from slab) of packet i, or ~0 when i >= n
__device__ __forceinline__ uint64_t ct_base(const KArgs &a, uint64_t i, uint64_t off_i)
{
    if (i >= a.n)
        return ~0ull;
    return (a.offsets ? off_i : i * a.stride) + a.data_off;
}

__device__ __forceinline__ bool ct_fast(const KArgs &a, uint64_t base)
{
    // base + 64 <= slab_len (base = ~0 fails it) and 16-B aligned; bitwise
    // ANDs so the test stays straight-line
    return (a.slab_len >= 64) & (base <= a.slab_len - 64) & ((((uintptr_t)a.slab + base) & 15u) == 0);
}

// ---------------------------------------------------------------------------
// Streamed cnet kernel (CNDP_TUNE_CNET_TILE 2): the wave-tile
// kernel's fast path only -- Ethernet + IPv4 IHL 5 unfragmented or IPv6
// without extension headers, carrying TCP / UDP / SCTP, 64 readable aligned
// bytes -- with every other frame appended to a worklist that the general
// per-lane kernel (k_classify_cnet<true>) finishes afterwards.  Without the
// general parse the kernel is small enough to keep two window tiles in
// flight: each loop trip resolves its whole FIB gather chain before it issues
// the window loads of the tile two ahead, so the in-order vmcnt waits of the
// chain only ever include loads issued a trip earlier.
// ---------------------------------------------------------------------------
// element i of a per-frame output through a 32-bit byte offset (a scalar base
// + zero-extended VGPR offset: one store, no 64-bit address per lane); the
// deferred kernel runs only for n < 2^30, so i * 4 fits
__device__ __forceinline__ GAS uint32_t &at32(uint32_t *p, uint32_t i)
{
    return *(GAS uint32_t *)((GAS char *)gp(p) + (uint32_t)(i << 2));
}
__device__ __forceinline__ GAS uint16_t &at16(uint16_t *p, uint32_t i)
{
    return *(GAS uint16_t *)((GAS char *)gp(p) + (uint32_t)(i << 1));
}

struct CsOff { // this lane's frame offsets for tiles t, t+1, t+2 and the load for t+3
    uint64_t o0, o1, o2, o3;
};

template <bool LNT>
__device__ __forceinline__ void cs_issue(const KArgs &a, uint32_t tt, uint32_t n_tiles, uint64_t off,
                                         uint32_t lane, u32x4 (&r)[4])
{
    const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
    const uint64_t my_base = tt < n_tiles ? ct_base(a, tt * 64u + lane, off) : ~0ull;
    // each lane resolves its own frame's load address once; frames off the
    // fast path load a dummy chunk of the (aligned, 36 KiB) Toeplitz table
    // instead, so every load is unconditional
    const uint64_t my_src = ct_fast(a, my_base) ? (uint64_t)(uintptr_t)(a.slab + my_base) : (uint64_t)(uintptr_t)a.ttab;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t src = __shfl(my_src, 16 * k + (int)fr_in_k) + part * 16u;
        r[k] = ldg4<LNT>((const uint8_t *)(uintptr_t)src);
    }
}

// ---------------------------------------------------------------------------
// Deferred-chain cnet kernel (CNDP_TUNE_CNET_TILE 3, the default): k_cnet_stream's fast
// path (worklist for the rest) in two stages one loop trip apart.
//   A  tile c    stage, parse, Toeplitz, first FIB gather
//   B  tile c-1  the rest of its FIB chain, then its results
// A trip issues B's chain -> A's first gather -> offsets of c+3 -> windows of
// c+2 -> B's stores.  B's chain waits only behind loads issued a trip
// earlier, never behind the window loads of the same trip.
// ---------------------------------------------------------------------------
struct CdLane {
    uint32_t ptf;  // pt (16) | do4 << 16 | do6 << 17 | fast << 18 | p_nxt edge << 19
    uint32_t h, e, rx;
    uint32_t ipl; // META: 1 << 16 | the IP length field (KArgs::iplen)
    // the chain's key bytes after the first gather, next byte lowest: v6
    // address bytes 3..15 (trie.h:127-134); v4 dip bits 15:8 then 7:0 with
    // the /16 directory, bits 7:0 without (dir24_8.h:135-140)
    uint32_t q0, q1, q2, q3;
};

// a non-canonical tile of the fast kernel (CNDP_TUNE_SPEC_LISTS), looked at
// once the wave's loop is done so the loop holds no registers for it: its
// chunks listed, and SPEC_MX bits 0..7 from its groups -- lane 4q + 3 looks at
// group q (bursts of a multiple of 4).  A group whose 4th frame is off the
// common edge moves the node state to that edge unless its 3rd type equals
// the 4th (then to any edge: bit 8).  The loop already set bit 8 for a group
// whose 4th frame, or whose 3rd beside an off-edge 4th, was not parsed there;
// without it both types here are the fast kernel's own, stored by this lane.
// The list's device pointers sit in meta (SPEC_PTRS).
__device__ __forceinline__ void spec_odd_tile(const KArgs &a, uint32_t tt, uint32_t lane, uint32_t *s_mx)
{
    if (lane == 0) {
        uint32_t *const cwl = *(uint32_t *const *)(a.spec_meta + SPEC_PTRS);
        uint32_t *const cflag = *(uint32_t *const *)(a.spec_meta + SPEC_PTRS + 2);
        const uint32_t per = SPEC_CH_K * a.spec_B, f0 = tt * 64u, f1 = f0 + 63u < a.n ? f0 + 63u : a.n - 1u;
        for (uint32_t c = f0 / per; c <= f1 / per; c++)
            if (atomicExch(&cflag[c], 1u) == 0u)
                cwl[1u + atomicAdd(&cwl[0], 1u)] = c;
    }
    const uint32_t i = tt * 64u + lane;
    const bool in = i < a.n;
    const uint32_t pt = in ? (uint32_t)at16(a.spec_t16, i) : 0u;
    const uint32_t p2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)pt, 0xAA, 0xf, 0xf, true); // lane 4q + 2
    const uint32_t pe = cnet_edge(pt);
    if ((lane & 3u) == 3u && in && pe != 3u && pe != 4u)
        atomicOr(s_mx, p2 == pt ? 1u << 8 : 1u << pe);
}

// The per-frame output pointers, read from the kernarg segment where they are
// used (an opaque copy of the segment pointer per trip keeps the compiler from
// hoisting them): a scalar load each instead of SGPRs held across the loop,
// which the kernel does not have (spilled to VGPR lanes otherwise).
#ifndef CD_RELOAD
#define CD_RELOAD 1
#endif
#define KAS __attribute__((address_space(4)))
__device__ __forceinline__ const KAS KArgs &kargs_fresh(const KArgs &a)
{
#if CD_RELOAD
    const KAS KArgs *p = (const KAS KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *p;
#else
    return *(const KAS KArgs *)&a;
#endif
}

#ifndef CD_PIN
#define CD_PIN 1
#endif
// timing-only ablations (tools/abbuild.sh -DCD_ABL=<bits>; wrong results,
// but every index stays in bounds): 1 no Toeplitz, 2 no chain levels, 4 no
// first gather (and so no chain), 8 at most CD_V6CAP IPv6 tbl8 levels, 16 no result
// stores but the edge, 32 five IPv6 levels every lane, all within one line of the
// first tbl8 group (the walk's dependent latency without its distinct lines)
#ifndef CD_ABL
#define CD_ABL 0
#endif
#ifndef CD_V6CAP
#define CD_V6CAP 2 // CD_ABL bit 8: IPv6 tbl8 levels walked at most
#endif
// CD_NIB 1: k_cnet_defer's Toeplitz from the nibble tables (4.5 KiB of LDS,
// conflict-free reads) instead of the byte tables (36 KiB, random banks)
#ifndef CD_NIB
#define CD_NIB 0
#endif
#define CD_TAB_WORDS (CD_NIB ? 2 * TAB_POS * 16 : TAB_POS * 256)
// CD_STAMP 1 (diagnostic builds only): s_memtime stamps around cd_trip's
// stages, summed per wave into cd_stamps (cndp_gpu_debug_stamps reads them)
#ifndef CD_STAMP
#define CD_STAMP 0
#endif
#if CD_STAMP
#define CD_STAMP_WAVES 8192
__device__ unsigned long long cd_stamps[CD_STAMP_WAVES * 16];
// k_spec_local_t per block (start, inputs in, tables filled, end, path) and
// k_spec_fallback's block 0 (start, end) at [SP_STAMP_BLOCKS * 16]
#define SP_STAMP_BLOCKS 4096
__device__ unsigned long long sp_stamps[SP_STAMP_BLOCKS * 16 + 8];
#define SP_TS(k, v)                                                                              \
    do {                                                                                         \
        if (threadIdx.x == 0 && blockIdx.x < SP_STAMP_BLOCKS)                                    \
            sp_stamps[blockIdx.x * 16u + (k)] = (v);                                              \
    } while (0)
#define CD_TS(k)                                                                                 \
    do {                                                                                         \
        const uint64_t now_ = __builtin_amdgcn_s_memtime();                                      \
        acc[k] += now_ - acc[7];                                                                 \
        acc[7] = now_;                                                                           \
    } while (0)
#else
#define SP_TS(k, v) ((void)0)
#define CD_TS(k) ((void)0)
#endif
// CD_HSKIP 1: no Toeplitz in a call that stores neither the hash nor the queue
#ifndef CD_HSKIP
#define CD_HSKIP 1
#endif
template <class T> __device__ __forceinline__ const GAS T *sgpr_pin(const T *p)
{
    const GAS T *g = (const GAS T *)p;
#if CD_PIN
    asm volatile("" : "+s"(g));
#endif
    return g;
}

struct SigCache { // wave-uniform: 4 signatures already marked, round-robin slot
    uint32_t s0, s1, s2, s3, next;
};

// the four packet types a canonical tile holds (spec_canon): Ethernet + IPv4 /
// IPv6 (0x11 / 0x41) with TCP / UDP (0x100 / 0x200, pktmbuf_ptype.h), coded as
// IPv6 bit | UDP bit; SPEC_TW_CODES marks a tile whose types went out coded
#define SPEC_TW_CODES 3u
__device__ __forceinline__ bool spec_code_type(uint32_t pt)
{
    return pt == 0x111u || pt == 0x211u || pt == 0x141u || pt == 0x241u;
}

// tA: stage A's tile, tB: stage B's (the previous trip's A), tW: the tile
// whose windows this trip loads, tO: the tile whose offsets it loads;
// CD_NONE for none
#define CD_NONE 0xFFFFFFFFu
template <bool LNT, bool META, bool CODES, int P>
__device__ __forceinline__ void cd_trip(const KArgs &a, uint32_t n_tiles, uint32_t tA, uint32_t tB, uint32_t tW,
                                        uint32_t tO, uint32_t lane, u32x4 *tile, u32x4 (&r)[2][4], CsOff &off,
                                        CdLane &sb, const uint32_t *s_t, const uint16_t *s_reta, uint32_t *s_bins,
                                        uint32_t *s_sf, bool count, SigCache &sc, uint32_t *s_mx, uint64_t *acc)
{
    const uint32_t fr_in_k = lane >> 2, part = lane & 3u;
    // B: tile c-1 -- the rest of its chain (v4: page / tbl8, v6: tbl8 levels, trie.h:127-134)
    const bool bv = tB != CD_NONE;
    const uint32_t ib = tB * 64u + lane;
    uint32_t eb = sb.e;
    {
        // one branch-free body for both families: the key bytes stream out of
        // q0..q3, the level count and the table pair are fixed per lane
        const bool d6 = (sb.ptf & (1u << 17)) != 0u, d4 = (sb.ptf & (1u << 16)) != 0u;
        uint32_t rem = d6 ? ((CD_ABL & 8) ? (uint32_t)CD_V6CAP : (CD_ABL & 32) ? 5u : 13u) : (a.dir16 ? 2u : 1u);
        const uint32_t g6 = eb >> 1; // (CD_ABL & 32)
        // the table pointers pinned in SGPRs before the per-lane select:
        // otherwise the select is of their kernarg addresses and the pointer
        // itself a vector load each trip, waited for at the chain's first level
        const GAS uint32_t *const t6 = sgpr_pin(a.tbl8_6), *const t8 = sgpr_pin(a.tbl8);
        const GAS uint32_t *const t4 = sgpr_pin(a.dir16 ? a.pages : a.tbl8);
        bool more = bv & (d4 | d6) & ((eb & 1u) != 0u);
        const GAS uint32_t *tb = d6 ? t6 : t4;
        const GAS uint32_t *const tb2 = d6 ? t6 : t8;
        uint32_t q0 = sb.q0, q1 = sb.q1, q2 = sb.q2, q3 = sb.q3;
        while (!(CD_ABL & 2) && __any(more)) {
            uint32_t idx = ((eb >> 1) << 8) | (q0 & 0xffu);
            if (CD_ABL & 32)
                idx = d6 ? (g6 << 8) | (eb & 7u) : idx;
            if (more)
                eb = tb[idx];
            tb = tb2;
            q0 = alignb(q1, q0, 1);
            q1 = alignb(q2, q1, 1);
            q2 = alignb(q3, q2, 1);
            q3 >>= 8;
            rem--;
            more = more & (((eb & 1u) != 0u) | ((CD_ABL & 32) && d6)) & (rem != 0u);
        }
    }
    CD_TS(0); // B's chain
    // A: tile c
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t f = 16u * k + fr_in_k;
        tile[f * 4u + (part ^ ((f >> 2) & 3u))] = r[P][k];
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t i = tA * 64u + lane;
    const bool live = tA != CD_NONE && i < a.n;
    const uint64_t base = live ? ct_base(a, i, off.o0) : ~0ull;
    const uint32_t sw = (lane >> 2) & 3u;
    uint32_t W[16];
    {
        const u32x4 c0 = tile[lane * 4u + (0u ^ sw)], c1 = tile[lane * 4u + (1u ^ sw)];
        const u32x4 c2 = tile[lane * 4u + (2u ^ sw)], c3 = tile[lane * 4u + (3u ^ sw)];
        W[0] = c0.x; W[1] = c0.y; W[2] = c0.z; W[3] = c0.w;
        W[4] = c1.x; W[5] = c1.y; W[6] = c1.z; W[7] = c1.w;
        W[8] = c2.x; W[9] = c2.y; W[10] = c2.z; W[11] = c2.w;
        W[12] = c3.x; W[13] = c3.y; W[14] = c3.z; W[15] = c3.w;
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t et = W[3] & 0xffffu;
    const uint32_t p4 = W[5] >> 24, p6 = W[5] & 0xffu;
    // straight-line tests (bitwise &, not &&: no branch tree)
    const uint32_t l4b4 = pt_l4(p4), l4b6 = pt_l4(p6);
    const bool f4 = (et == BE16C(0x0800u)) & (((W[3] >> 16) & 0xffu) == 0x45u) &
                    (((W[5] & 0xffffu) & BE16C(0x3fffu)) == 0u) & (l4b4 != 0u);
    const bool f6 = (et == BE16C(0x86DDu)) & (l4b6 != 0u);
    const bool fast = live & ct_fast(a, base) & (f4 | f6);
    {
        const bool slow = live && !fast;
        const unsigned long long m = __ballot(slow);
        if (m) {
            const KAS KArgs &o = kargs_fresh(a);
            uint32_t w0 = 0;
            if (lane == (uint32_t)(__ffsll(m) - 1))
                w0 = atomicAdd(o.wl_n, (uint32_t)__popcll(m));
            w0 = __shfl(w0, __ffsll(m) - 1);
            if (slow)
                // write-through (agent-scope) store: k_cnet_defer's last block
                // may read it without a release by this one (cnet_defer_tail)
                __hip_atomic_store(&o.wl[w0 + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))], (uint32_t)i,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    CdLane na;
    na.ptf = 0;
    na.h = 0;
    na.rx = 0;
    na.q0 = na.q1 = na.q2 = na.q3 = 0;
    uint32_t idx0 = 0;
    const uint32_t *tb0 = a.tbl24_6;
    if (fast) {
        const uint32_t proto = f4 ? p4 : p6;
        uint32_t pt = (f4 ? 0x11u : 0x41u) | (f4 ? l4b4 : l4b6);
        // pktmbuf_ptype.c: UDP dport 2152 / 2123 (GTP)
        const uint32_t dport = f4 ? (W[9] & 0xffffu) : (W[14] & 0xffffu);
        const bool udp = proto == 17u, gtpu = udp & (dport == BE16C(2152u)), gtpc = udp & (dport == BE16C(2123u));
        pt |= gtpu ? 0x8000u : gtpc ? 0x7000u : 0u;
        // cnet_edge(pt) for these shapes (ptype.c:32-46): TCP / UDP go to the
        // family's input node, GTP-U to gtpu_input, GTP-C and SCTP to pkt_drop
        const uint32_t pe = (proto == 6u) | (udp & !gtpc) ? (gtpu ? 5u : f4 ? 3u : 4u) : 0u;
        const bool l4ok = proto == 6u || proto == 17u;
        Lens lens{14u, f4 ? 20u : 40u, 0u};
        if (META && a.rxmeta) { // l4_len: UDP 8, SCTP 12, TCP data offset (pktmbuf_ptype.c:596-615)
            lens.l4 = proto == 17u ? 8u : proto == 132u ? 12u
                    : f4 ? ((W[11] >> 16) & 0xf0u) >> 2
                         : (gbyte(a.slab + base, a.slab_len - base, 66) & 0xf0u) >> 2;
            na.rx = rx_meta(lens, W[0], W[1], et);
        }
        if (META && a.iplen) // at mtod + l2_len 2 / 4 (ip4_input.c:121-124, ip6_input.c:121-124)
            na.ipl = (1u << 16) | bswap16(f4 ? (W[4] & 0xffffu) : (W[4] >> 16));
        if (META && a.win) { // the node queue's metadata source (k_mq_cnet_post)
            u32x4 *dw = a.win + 4ull * i;
#pragma unroll
            for (int k = 0; k < 4; k++)
                dw[k] = (u32x4){W[4 * k], W[4 * k + 1], W[4 * k + 2], W[4 * k + 3]};
        }
        uint32_t flags = 0;
        // Toeplitz, one instruction stream for both families: the v6 words
        // are V[0..7] + L4 V[8], the v4 ones V[1..2] + L4 V[3] (a zero word
        // adds nothing); positions past the v4 tuple only when the wave has v6.
        // Skipped when the call asks for neither the hash nor the queue
        // (launch-uniform; the bins of cnet mode do not use the queue).
        if (!CD_HSKIP || a.hash || a.queue) {
            uint32_t V[9];
#pragma unroll
            for (int k = 0; k < 9; k++)
                V[k] = alignb(W[6 + k], W[5 + k], 2);
            const bool any6 = __any(f6);
#pragma unroll
            for (int k = 0; k < 9; k++) {
                if (k >= 3 && !any6)
                    break;
                uint32_t u = k < 2 ? (f4 ? V[k + 1] : V[k]) : k == 2 ? (f4 ? (l4ok ? V[3] : 0u) : V[2])
                           : k < 8 ? (f4 ? 0u : V[k]) : (f4 || !l4ok ? 0u : V[8]);
                if (!(CD_ABL & 1))
                    na.h ^= CD_NIB ? tz4n(s_t, 4 * k, u) : tz4(s_t, 4 * k, u);
            }
        }
        // both families' input-node pieces, straight-line, then selects: the
        // waves of an IMIX batch hold both families, and a branch per family
        // ran both bodies anyway (plus the exec-mask saves and zero fills)
        const bool do4 = f4 & ((pe == 3u) | (a.spec_nh != nullptr)); // ip4_input.c:121-140
        const bool do6 = !f4 & ((pe == 4u) | (a.spec_nh != nullptr)); // ip6_input.c:115-135
        const uint32_t dst = alignb(W[8], W[7], 2);
        // the header's 10 16-bit words (bytes 14..33) are W[3]'s high half,
        // both halves of W[4..7] and W[8]'s low half: four packed dot
        // products with (1, 1) add the pairs (cne_ip.h:131-214)
        uint32_t sum = (W[3] >> 16) + (W[8] & 0xffffu);
#pragma unroll
        for (int k = 4; k < 8; k++)
            sum = hsum2(W[k], sum);
        sum = (sum >> 16) + (sum & 0xffffu);
        sum = (sum >> 16) + (sum & 0xffffu);
        const bool ok4 = (bswap16(W[4] & 0xffffu) < a.buf_len) & (((~sum) & 0xffffu) == 0u);
        const uint32_t d4 = ok4 ? bswap32(dst) : 0u;
        const bool ok6 = bswap16(W[4] >> 16) < a.buf_len;
        const uint32_t d0 = ok6 ? alignb(W[10], W[9], 2) : 0u, d1 = ok6 ? alignb(W[11], W[10], 2) : 0u;
        const uint32_t d2 = ok6 ? alignb(W[12], W[11], 2) : 0u, d3 = ok6 ? alignb(W[13], W[12], 2) : 0u;
        const uint32_t q04 = ok4 ? dst >> (a.dir16 ? 16 : 24) : 0u; // network bytes 2, 3
        na.q0 = do4 ? q04 : do6 ? alignb(d1, d0, 3) : 0u;
        na.q1 = do6 ? alignb(d2, d1, 3) : 0u;
        na.q2 = do6 ? alignb(d3, d2, 3) : 0u;
        na.q3 = do6 ? d3 >> 24 : 0u;
        flags = do4 ? 1u << 16 : do6 ? 1u << 17 : 0u;
        const uint32_t i4 = a.dir16 ? d4 >> 16 : d4 >> 8;
        const uint32_t i6 = ((d0 & 0xffu) << 16) | (d0 & 0xff00u) | ((d0 >> 16) & 0xffu); // trie.h:126
        idx0 = do4 ? i4 : do6 ? i6 : 0u;
        if (do4)
            tb0 = a.dir16 ? a.dir16 : a.tbl24;
        na.ptf = pt | flags | (1u << 18) | (pe << 19);
    }
    CD_TS(1); // A's tile, parse, hash
    // (the ablation's stand-in has bit 0 clear: no chain level follows it)
    na.e = (CD_ABL & 4) ? (idx0 & 0xffu) << 1 : tb0[idx0]; // first gather, unconditional
    // offsets one tile further, then the windows of tile c+2 (issued after
    // the first gather: the next trip's wait for the gather leaves them in
    // flight when no lane of the wave needs a further level)
    {
        const uint32_t i3 = tO * 64u + lane;
        off.o3 = a.offsets && tO < n_tiles && i3 < a.n ? a.offsets[i3] : 0;
        cs_issue<LNT>(a, tW, n_tiles, off.o2, lane, r[P]);
    }
    CD_TS(2); // gather, offsets and windows issued
    // B's results
    {
        const KAS KArgs &o = kargs_fresh(a);
        const uint32_t pt = sb.ptf & 0xffffu, pe = sb.ptf >> 19;
        const bool bf = bv && (sb.ptf & (1u << 18));
        const bool din = (sb.ptf & (3u << 16)) != 0u;
        uint32_t nh = CNDP_NH_INVALID, edge = 0x80u | pe;
        if (din && (pe == 3u || pe == 4u)) {
            nh = eb >> 1;
            edge = nh >> 24;
        }
        if (o.spec_nh) {
            if (bf && din && (!o.nh || (pe != 3u && pe != 4u)))
                at32(o.spec_nh, ib) = eb >> 1;
            if (!CODES && bf) {
                // the last SPEC_TAIL bursts' types are read by spec_classes in
                // this kernel's last block when it folds: write-through stores
                if (a.wl_fold && ib >= a.tail_lo)
                    __hip_atomic_store(&at16(o.spec_t16, ib), (uint16_t)pt, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                else
                    __builtin_nontemporal_store((uint16_t)pt, &at16(o.spec_t16, ib));
            }
            const uint32_t sg = ((pt & 0xffu) << 3) | pe; // spec_sig(pt)
            // sc: signatures this wave already put in the block's flag set
            // (wave-uniform; the set only grows within a call): only a frame of
            // another signature marks (IMIX: the first trips only; the mark is
            // a loop of cross-lane reductions)
            const bool on = bf && sg != sc.s0 && sg != sc.s1 && sg != sc.s2 && sg != sc.s3;
            const unsigned long long mo = __ballot(on);
            if (mo) {
                spec_mark(s_sf, on, sg);
                const uint32_t ns = (uint32_t)__builtin_amdgcn_readlane((int)sg, (int)(__ffsll(mo) - 1));
                const uint32_t k = sc.next & 3u;
                sc.s0 = k == 0u ? ns : sc.s0;
                sc.s1 = k == 1u ? ns : sc.s1;
                sc.s2 = k == 2u ? ns : sc.s2;
                sc.s3 = k == 3u ? ns : sc.s3;
                sc.next++;
            }
            bool codes = false;
            if (o.spec_tile && bv) {
                // the tile's word for the speculation passes (spec_canon): 1 when
                // every frame has its low byte's common edge -- parsed here (low
                // byte 0x11 / 0x41) and bound for ip4_input / ip6_input, not GTP
                // or pkt_drop, nor left to the general parse
                const bool odd = ib < a.n && !(bf && (pe == 3u || pe == 4u));
                const uint64_t om = __ballot(odd);
                // such a tile's types are IPv4 / IPv6 x TCP / UDP: with
                // a.spec_codes (the previous call was a uniform batch, whose
                // passes never read a canonical tile's types) they go out as two
                // ballots, 16 B a tile, instead of 128 B of types (k_spec_expand
                // writes the types should this batch need them after all)
                codes = CODES && om == 0ull && (tB + 1u) * 64u <= a.spec_keep_lo &&
                        __ballot(ib < a.n && !spec_code_type(pt)) == 0ull;
                if (codes) {
                    const uint64_t m6 = __ballot((pt & 0xf0u) == 0x40u), mu = __ballot((pt & 0xf00u) == 0x200u);
                    if (lane == 0)
                        __builtin_nontemporal_store((u32x4){(uint32_t)m6, (uint32_t)(m6 >> 32), (uint32_t)mu,
                                                            (uint32_t)(mu >> 32)},
                                                    (u32x4 *)(a.spec_c2 + 16u * tB));
                }
                if (lane == 0)
                    o.spec_tile[tB] = codes ? (uint8_t)SPEC_TW_CODES : (uint8_t)(om == 0ull);
                if (om && (a.spec_allow & SPEC_ALLOW_LISTS)) { // wave-uniform, rare
                    // groups (lanes 4q + 3) whose 4th frame was not parsed here, or
                    // is off the common edge beside a 3rd not parsed here (spec_odd_tile)
                    const uint64_t nf = __ballot(ib < a.n && !bf), m3 = 0x8888888888888888ull;
                    if (lane == 0 && ((nf & m3) | (om & m3 & (nf << 1))))
                        atomicOr(s_mx, 1u << 8);
                }
            }
            if (CODES && bf && !codes) {
                if (a.wl_fold && ib >= a.tail_lo)
                    __hip_atomic_store(&at16(o.spec_t16, ib), (uint16_t)pt, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                else
                    __builtin_nontemporal_store((uint16_t)pt, &at16(o.spec_t16, ib));
            }
        }
        CD_TS(4); // B's speculation words (types, tile word, signature flags)
        if (bf) {
            const uint32_t q = s_reta[sb.h & a.reta_mask];
            if (META && o.ptype)
                __builtin_nontemporal_store(pt, &at32(o.ptype, ib));
            if (META && o.rxmeta)
                __builtin_nontemporal_store(sb.rx, &at32(o.rxmeta, ib));
            if (META && o.iplen)
                __builtin_nontemporal_store(sb.ipl, &at32(o.iplen, ib));
            // non-temporal stores: the outputs are written once and must not
            // push the FIB tables of the gather chains out of L2 (C4 -4.5%)
            if (!(CD_ABL & 16) && o.nh)
                __builtin_nontemporal_store(nh, &at32(o.nh, ib));
            if (!(CD_ABL & 16) && o.hash)
                __builtin_nontemporal_store(sb.h, &at32(o.hash, ib));
            if (!(CD_ABL & 16) && o.queue)
                __builtin_nontemporal_store((uint16_t)q, &at16(o.queue, ib));
            if (o.edge)
                __builtin_nontemporal_store((uint8_t)edge, &o.edge[ib]);
            if (count)
                atomicAdd(&s_bins[bin_of<CNDP_MODE_CNET>(nh, edge, q, a.n_bins)], 1u);
        }
    }
    sb = na;
    off.o0 = off.o1;
    off.o1 = off.o2;
    off.o2 = off.o3;
    CD_TS(3); // B's results stored
}

// With a.wl_fold, k_cnet_defer ends the way k_classify_cnet<true> does, so
// that nothing runs between it and the speculation passes: every block takes
// an arrival ticket (cnet_spec_tail's two-level ticket, after its type /
// worklist stores and flag ORs have left), and the last one parses the
// worklist -- the frames off the fast path, appended by every block -- with
// 256 lanes over LDS rows in the tile area, then runs spec_classes with wave
// 0.  The host folds when the previous call left no worklist (spec_hint[0]);
// any worklist is still handled here, by one block.
// NT threads a block; NL of them parse (rows of ROW_DW dwords in the tile area)
template <uint32_t NT, uint32_t NL>
__device__ __forceinline__ void cnet_defer_tail(const KArgs &a, uint32_t *rows, const uint32_t *s_t,
                                             const uint16_t *s_reta, uint32_t *s_bins, uint32_t *s_sf, bool count)
{
    __shared__ uint32_t s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint32_t tid = threadIdx.x;
    if (tid == 0) {
        // no release: what the last block reads of this one's stores -- the
        // worklist, the last SPEC_TAIL bursts' types -- was stored write-through
        // and the signature flags are device atomics; vmcnt(0) saw them done
        const uint32_t G = gridDim.x, g = blockIdx.x & 7u, ng = G < 8u ? G : 8u;
        const uint32_t in_g = (G - g + 7u) / 8u; // blocks of group g
        bool last = __hip_atomic_fetch_add(&a.spec_ticket[32u * g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                    in_g - 1u;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent"); // pass the group's releases on
            last = __hip_atomic_fetch_add(&a.spec_ticket[32u * 8u], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   ng - 1u;
        }
        s_last = last;
    }
    __syncthreads();
#if CD_STAMP
    if ((threadIdx.x & 63u) == 0 && blockIdx.x * CT_WAVES + (threadIdx.x >> 6) < CD_STAMP_WAVES)
        cd_stamps[(blockIdx.x * CT_WAVES + (threadIdx.x >> 6)) * 16u + 14u] =
            __builtin_amdgcn_s_memrealtime() | ((uint64_t)s_last << 63); // ticket taken (bit 63: the last block)
#endif
    if (!s_last)
        return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const uint32_t n_wl = __hip_atomic_load(a.wl_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n_wl) { // block-uniform
        if (tid < 64)
            s_sf[tid] = 0;
        if (count)
            for (uint32_t k = tid; k < a.n_bins + 2; k += NT)
                s_bins[k] = 0;
        __syncthreads();
        if (tid < NL) {
            uint32_t *row = rows + tid * ROW_DW;
            row[WIN_DW] = 0;
            for (uint32_t j = tid; j < n_wl; j += NL) // entries other blocks stored write-through
                cnet_general(a, __hip_atomic_load(&a.wl[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), row, s_t,
                             s_reta, s_bins, s_sf, count);
        }
        __syncthreads();
        if (count)
            for (uint32_t k = tid; k < a.n_bins + 2; k += NT)
                if (s_bins[k])
                    atomicAdd(&a.bins[k], (unsigned long long)s_bins[k]);
        if (a.spec_flags && tid < 64 && s_sf[tid])
            atomicOr(&a.spec_flags[tid], s_sf[tid]);
        // wave 0 reads the other waves' type stores and flag ORs
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    if (tid >= 64)
        return;
    if (tid < 9)
        a.spec_ticket[32u * tid] = 0; // for the next launch (kernel boundary)
    const uint64_t nb = ((uint64_t)a.n + a.spec_B - 1) / a.spec_B;
    spec_classes(tid, a.spec_flags, a.spec_cls, a.spec_meta, a.spec_t16, a.n, a.spec_B, nb, a.spec_allow, a.wl_n,
                 a.spec_bar, a.spec_hint);
}

// META: ptype / rxmeta outputs requested (without them the kernel keeps
// 14 VGPRs and 18 spilled SGPRs fewer).  BAL (CNDP_TUNE_STREAM_BAL): the
// block's tiles are handed to its waves by an LDS counter instead of each
// wave taking tiles t0, t0 + wstep, ... -- each
// wave's first four are static, then every trip draws the tile it will
// read the offsets of next trip (the LDS atomic's return is waited for with
// the trip's other LDS traffic); the waves the SQ favours take more tiles.
template <bool LNT, bool META, bool CODES, bool BAL>
__global__ __launch_bounds__(BAL ? CD_BAL_THREADS : CT_THREADS) void k_cnet_defer(KArgs a, uint32_t n_tiles)
{
    constexpr uint32_t NTH = BAL ? CD_BAL_THREADS : CT_THREADS, NWV = NTH / 64u;
    __shared__ uint32_t s_t[CD_TAB_WORDS];
    __shared__ __attribute__((aligned(16))) u32x4 s_tile[NWV][256];
    __shared__ uint16_t s_reta[CNDP_RETA_MAX];
    __shared__ uint32_t s_bins[CNDP_BINS_MAX + 2];
    __shared__ uint32_t s_sf[64];
    __shared__ uint32_t s_mx;   // SPEC_MX bits of this block
    __shared__ uint32_t s_next; // BAL: the block's next tile index

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u, wv = tid >> 6;
    u32x4 *tile = s_tile[wv];
    const uint32_t G = gridDim.x, bk = blockIdx.x;
    const uint32_t wstep = G * NWV;
    const uint32_t t0 = bk * NWV + wv;
    const uint32_t nt_w = t0 < n_tiles ? (n_tiles - t0 + wstep - 1) / wstep : 0;
    // BAL: the block's tiles are the static schedule's tiles of its waves, in
    // round order -- index k is round k / NWV, wave k % NWV -- so the
    // block's waves work on neighbouring tiles at any time (tiles G apart
    // instead: C5 11 % slower, the windows of one CU spread over many pages);
    // they form a prefix of k, nk of them (the waves' static counts)
    uint32_t nk = 0;
    if (BAL) {
        const uint32_t tb0 = bk * NWV;
        for (uint32_t w = 0; w < NWV; w++)
            nk += tb0 + w < n_tiles ? (n_tiles - tb0 - w + wstep - 1) / wstep : 0;
    }
    auto tile_k = [&](uint32_t k) -> uint32_t {
        return k < nk ? (k / NWV) * wstep + bk * NWV + k % NWV : CD_NONE;
    };
    // the wave's k-th tile while its sequence is static
    auto seq = [&](uint32_t k) -> uint32_t {
        if (BAL)
            return tile_k(wv + k * NWV);
        return k < nt_w ? t0 + k * wstep : CD_NONE;
    };
    uint32_t q0 = seq(0), q1 = seq(1), q2 = seq(2), q3 = seq(3);
    // the first offsets, then the first two frame tiles, in flight while the
    // tables are copied to LDS
    CsOff off{0, 0, 0, 0};
    if (a.offsets) {
#pragma unroll
        for (uint32_t s = 0; s < 3; s++) {
            const uint32_t ts = s == 0 ? q0 : s == 1 ? q1 : q2, is = ts * 64u + lane;
            const uint64_t o = ts < n_tiles && is < a.n ? a.offsets[is] : 0;
            if (s == 0)
                off.o0 = o;
            else if (s == 1)
                off.o1 = o;
            else
                off.o2 = o;
        }
    }
    if (tid < 64)
        s_sf[tid] = 0;
    if (tid == 0) {
        s_mx = 0;
        s_next = 4u * NWV;
    }
    for (uint32_t k = tid; k < CD_TAB_WORDS; k += NTH)
        s_t[k] = a.ttab[(CD_NIB ? TABN_OFF : 0) + k];
    u32x4 r[2][4];
    cs_issue<LNT>(a, q0, n_tiles, off.o0, lane, r[0]);
    cs_issue<LNT>(a, q1, n_tiles, off.o1, lane, r[1]);
    for (uint32_t k = tid; k <= a.reta_mask; k += NTH)
        s_reta[k] = a.reta[k];
    const bool count = a.bins != nullptr;
    if (count)
        for (uint32_t k = tid; k < a.n_bins + 2; k += NTH)
            s_bins[k] = 0;
#if CD_STAMP
    const uint64_t rt_entry = __builtin_amdgcn_s_memrealtime(); // after the prologue's issue
#endif
    __syncthreads();
    // BAL: the index after q3, drawn by lane 0 a trip ahead
    uint32_t kv = 0, kst = 4;
    auto draw = [&]() {
        if (BAL && q3 != CD_NONE && lane == 0)
            kv = atomicAdd(&s_next, 1u);
    };
    auto next = [&]() -> uint32_t {
        if (BAL) {
            if (q3 == CD_NONE)
                return CD_NONE;
            return tile_k((uint32_t)__builtin_amdgcn_readfirstlane((int)kv));
        }
        return seq(kst++);
    };
    draw();
    CdLane sb;
    sb.ptf = sb.h = sb.e = sb.rx = 0;
    sb.q0 = sb.q1 = sb.q2 = sb.q3 = 0;
    SigCache sig_cache{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u};
    uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#if CD_STAMP
    acc[7] = __builtin_amdgcn_s_memtime();
    acc[6] = acc[7];
    const uint64_t rt_loop = __builtin_amdgcn_s_memrealtime();
#endif
    uint32_t tb = CD_NONE, trips = 0; // stage B's tile
    for (;;) {
        if (q0 == CD_NONE && tb == CD_NONE) // wave-uniform
            break;
        cd_trip<LNT, META, CODES, 0>(a, n_tiles, q0, tb, q2, q3, lane, tile, r, off, sb, s_t, s_reta, s_bins, s_sf,
                                     count, sig_cache, &s_mx, acc);
        {
            const uint32_t qn = next();
            tb = q0;
            q0 = q1;
            q1 = q2;
            q2 = q3;
            q3 = qn;
            draw();
            trips++;
        }
        if (q0 == CD_NONE && tb == CD_NONE)
            break;
        cd_trip<LNT, META, CODES, 1>(a, n_tiles, q0, tb, q2, q3, lane, tile, r, off, sb, s_t, s_reta, s_bins, s_sf,
                                     count, sig_cache, &s_mx, acc);
        {
            const uint32_t qn = next();
            tb = q0;
            q0 = q1;
            q1 = q2;
            q2 = q3;
            q3 = qn;
            draw();
            trips++;
        }
    }
    (void)trips; // (CD_STAMP)
#if CD_STAMP
    if (lane == 0 && blockIdx.x * NWV + wv < CD_STAMP_WAVES) {
        unsigned long long *o = cd_stamps + (blockIdx.x * NWV + wv) * 16u;
        for (int k = 0; k < 4; k++)
            o[k] = acc[k];
        o[4] = acc[7] - acc[6]; // the loop
        o[5] = trips;
        o[6] = acc[4];
        o[8] = rt_entry; // s_memrealtime (100 MHz): prologue issued, loop start, loop end
        o[9] = rt_loop;
        o[10] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    if ((a.spec_allow & SPEC_ALLOW_LISTS) && a.spec_tile) {
        // the non-canonical tiles: the wave's own (its own tile words and
        // types), or with BAL a static share of the block's once every wave
        // of the block is done (workgroup-scope release / acquire)
        uint32_t ns = nt_w;
        if (BAL) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __syncthreads();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            ns = nk > wv ? (nk - wv + NWV - 1) / NWV : 0;
        } else {
            __threadfence_block();
        }
        for (uint32_t j0 = 0; j0 < ns; j0 += 64u) {
            const uint32_t j = j0 + lane;
            uint64_t om = __ballot(j < ns && a.spec_tile[seq(j)] == 0u);
            while (om) {
                const uint32_t jj = j0 + (uint32_t)(__ffsll((unsigned long long)om) - 1);
                om &= om - 1ull;
                spec_odd_tile(a, seq(jj), lane, &s_mx);
            }
        }
    }
#if CD_STAMP
    if (lane == 0 && blockIdx.x * NWV + wv < CD_STAMP_WAVES)
        cd_stamps[(blockIdx.x * NWV + wv) * 16u + 12u] = __builtin_amdgcn_s_memrealtime(); // odd tiles done
#endif
    if (count || a.spec_flags || (a.spec_allow & SPEC_ALLOW_LISTS))
        __syncthreads();
    if (count)
        for (uint32_t k = tid; k < a.n_bins + 2; k += NTH)
            if (s_bins[k])
                atomicAdd(&a.bins[k], (unsigned long long)s_bins[k]);
    if (a.spec_flags && tid < 64 && s_sf[tid])
        atomicOr(&a.spec_flags[tid], s_sf[tid]);
    if ((a.spec_allow & SPEC_ALLOW_LISTS) && tid == 0 && s_mx)
        atomicOr(&a.spec_meta[SPEC_MX], s_mx);
#if CD_STAMP
    if (lane == 0 && blockIdx.x * NWV + wv < CD_STAMP_WAVES)
        cd_stamps[(blockIdx.x * NWV + wv) * 16u + 13u] = __builtin_amdgcn_s_memrealtime(); // flushes issued
#endif
    if (a.wl_fold)
        // (the general parse takes the byte tables: from LDS, or global memory
        // when LDS holds the nibble tables)
        cnet_defer_tail<NTH, 256>(a, (uint32_t *)&s_tile[0][0], CD_NIB ? a.ttab : s_t, s_reta, s_bins, s_sf,
                                         count);
#if CD_STAMP
    if (lane == 0 && blockIdx.x * NWV + wv < CD_STAMP_WAVES)
        cd_stamps[(blockIdx.x * NWV + wv) * 16u + 11u] = __builtin_amdgcn_s_memrealtime(); // the wave's end
#endif
}

// ---------------------------------------------------------------------------
// cnet ptype-node speculation (ptype.c:48-210) as a post-pass over the
// per-packet ptypes the classify kernel wrote.  In each graph burst of B
// packets the node walks 4-packet groups against its state last_type: a
// group whose four low bytes equal last_type's (the uint8_t fix_spec,
// :109-110) goes whole to p_nxt[last_type]; any other group goes packet by
// packet to p_nxt[type] and moves last_type to the group's 4th type when the
// 3rd equals it or p_nxt agrees; the tail goes per packet.  The state only
// matters through its signature sig = (low byte, p_nxt), and a group either
// keeps it or replaces it by its 4th type, so each burst is a map
// sig -> {unchanged | new state}.  Bursts are resolved with a chunked scan of
// those maps over the signatures present in the batch (<= SPEC_KMAX; more
// falls back to one sequential thread), then every burst is replayed from
// its true start state and the frames whose node edge differs from
// p_nxt[own type] get that edge's result (spec_nh) and their bins moved.
// ---------------------------------------------------------------------------
#define SPEC_KMAX 64
#define SPEC_UNCH 0xFFFFFFFFu

// meta[0] = K, meta[1 + k] = signature of class k; class_id[sig] = k or 0xFF
// (64 threads: thread t owns flag word t, classes numbered in signature order).
//
// Batch-level shortcut, meta[SPEC_SKIP]: when no low byte among the
// signatures present (the entering state's included) carries two p_nxt
// edges, a quiet group's speculated edge p_nxt[last_type] is every one of
// its frames' own edge, so the node routes exactly like the per-frame result
// already written -- only the final last_type is left to find.  A
// "universal" group (low bytes not all equal, 3rd type == 4th) sets the state
// to its 4th type whatever it was, so the final state is the walk from the
// batch's last universal group to its end.  The wave looks for one in the
// last SPEC_TAIL bursts; found, it stores the final state and sets
// meta[SPEC_SKIP], and the table / scan / replay passes return at once.
#define SPEC_SKIP 129
#define SPEC_FULL 130 // k_spec_local left a chunk unresolved: run the full passes
#define SPEC_IN 131   // the node state entering this batch (meta[-1] becomes the final one)
#define SPEC_NOLOCAL 132 // one low byte only: no universal group exists, k_spec_local is skipped
#define SPEC_UNIF 133 // every type has the entering state's low byte: k_spec_local's uniform pass only
#define SPEC_ERR 134  // a k_spec_fallback wait expired (the host reads spec_hint[3])
#define SPEC_HINT 900 // the hint words last written to host memory
#define SPEC_TAIL 16
// a type another block of the running kernel stored (write-through, agent
// scope): read at agent scope too, never from a line an XCD's L2 may hold
// from before (spec_classes runs in the last block of the kernel whose other
// blocks wrote the batch's last types)
__device__ __forceinline__ uint32_t spec_ld(const uint16_t *pt, uint64_t i)
{
    return __hip_atomic_load(pt + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void spec_step(uint32_t l0, uint32_t l1, uint32_t l2, uint32_t l3, uint32_t &cur)
{
    const uint32_t low = cur & 0xffu;
    const bool quiet = (l0 & 0xffu) == low && (l1 & 0xffu) == low && (l2 & 0xffu) == low && (l3 & 0xffu) == low;
    if (!quiet && (l2 == l3 || cnet_edge(cur) == cnet_edge(l3)))
        cur = l3;
}

// Run by wave 0 of the last block of k_classify_cnet to finish (after every
// block's flag ORs and type stores, see there).  It also clears the signature
// flags, the worklist count and k_spec_fallback's barrier words for the next
// call (the flags and the count were read before), which saves per-call
// memsets.
__device__ __forceinline__ void spec_classes(uint32_t t, uint32_t *flags, uint8_t *class_id, uint32_t *meta,
                             const uint16_t *__restrict__ pt, uint32_t n, uint32_t B, uint64_t nb,
                             uint32_t allow_skip, uint32_t *wl_n, uint32_t *bar, uint32_t *hint)
{
    // every load first (one memory round trip for the wave), then the stores
    const uint32_t wl_cnt = wl_n ? __hip_atomic_load(wl_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const uint32_t prev = meta[-1], hint_h0 = meta[SPEC_HINT], hint_h1 = meta[SPEC_HINT + 1];
    const uint32_t f = __hip_atomic_load(&flags[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t s_in = prev & 0xffffu, g0 = spec_sig(s_in); // the node state entering the batch
    if (t == 0) {
        meta[SPEC_IN] = s_in;
        meta[SPEC_FULL] = 0;
        bar[0] = bar[1] = bar[2] = bar[3] = 0; // k_spec_fallback's ticket and phase counts
    }
    const uint32_t w = f | (t == (g0 >> 5) ? 1u << (g0 & 31u) : 0u), cnt = (uint32_t)__popc(w);
    flags[t] = 0;
    if (wl_n && t == 0)
        *wl_n = 0;
    uint32_t pre = cnt; // inclusive wave prefix
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(pre, o);
        if ((int)t >= o)
            pre += v;
    }
    // lane t's 32 class ids (signatures 32t..32t+31) packed into two 16-B stores
    uint32_t k = pre - cnt, cw[8];
#pragma unroll
    for (uint32_t j = 0; j < 32; j++) {
        const bool on = (w >> j) & 1u;
        const uint32_t id = on && k < SPEC_KMAX ? k : 0xFFu;
        if (j % 4 == 0)
            cw[j / 4] = 0;
        cw[j / 4] |= id << (8 * (j % 4));
        k += on;
    }
    *(u32x4 *)(class_id + 32 * t) = (u32x4){cw[0], cw[1], cw[2], cw[3]};
    *(u32x4 *)(class_id + 32 * t + 16) = (u32x4){cw[4], cw[5], cw[6], cw[7]};
    k = pre - cnt;
    for (uint32_t ww = w; ww && k < SPEC_KMAX; ww &= ww - 1u, k++)
        meta[1 + k] = t * 32 + (uint32_t)__ffs(ww) - 1u;
    if (t == 63)
        meta[0] = pre;
    // flag word t holds the 8 edge bits of low bytes 4t..4t+3: one edge each?
    bool one = true;
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
        const uint32_t e8 = (w >> (8 * q)) & 0xffu;
        one = one && (e8 & (e8 - 1u)) == 0u;
    }
    uint32_t skip = 0;
    // every type with one low byte (e.g. all IPv4 + L2 ether): no group can
    // be universal, so k_spec_local would resolve nothing -- go straight to
    // the full passes
    uint32_t lows = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; q++)
        lows += ((w >> (8 * q)) & 0xffu) != 0u;
    for (int o = 32; o > 0; o >>= 1)
        lows += __shfl_xor(lows, o);
    // Uniform batch (auto mode, bursts <= 256): lows <= 1 counts the entering
    // state's low byte too, so every type shares it.  Each full group is then
    // quiet (ptype.c:109-110), goes whole to p_nxt[last_type] and never moves
    // the state (the per-packet tail, :171-187, does not either): the final
    // state is the entering one, and only frames of full groups whose own
    // edge differs get re-routed -- by k_spec_local's uniform pass, or by
    // nobody when no other signature is present.
    const bool unif = allow_skip && lows <= 1u && B <= 256u;
    if (t == 0) {
        meta[SPEC_NOLOCAL] = lows <= 1u;
        meta[SPEC_UNIF] = 0;
        if (lows <= 1u && !unif)
            meta[SPEC_FULL] = 1;
    }
    if (unif) {
        const uint32_t own = t == (g0 >> 5) ? 1u << (g0 & 31u) : 0u;
        skip = __ballot((w & ~own) != 0u) == 0ull;
        if (t == 0)
            meta[SPEC_UNIF] = !skip;
    } else if (allow_skip && __ballot(!one) == 0ull) {
        int64_t ub = -1; // the last universal group: burst ub, group ug
        uint32_t ug = 0;
        for (uint64_t q = 0; q < SPEC_TAIL && q < nb && ub < 0; q++) {
            const uint64_t b = nb - 1 - q, b0 = b * B;
            const uint32_t ng = (uint32_t)((uint64_t)n - b0 < B ? (uint64_t)n - b0 : B) >> 2;
            int best = -1;
            for (uint32_t j = t; j < ng; j += 64) {
                const uint32_t l0 = spec_ld(pt, b0 + 4 * j), l1 = spec_ld(pt, b0 + 4 * j + 1);
                const uint32_t l2 = spec_ld(pt, b0 + 4 * j + 2), l3 = spec_ld(pt, b0 + 4 * j + 3);
                const uint32_t v = l0 & 0xffu;
                const bool allq = (l1 & 0xffu) == v && (l2 & 0xffu) == v && (l3 & 0xffu) == v;
                if (!allq && l2 == l3)
                    best = (int)j;
            }
            for (int o = 32; o > 0; o >>= 1)
                best = max(best, __shfl_xor(best, o));
            if (best >= 0) {
                ub = (int64_t)b;
                ug = (uint32_t)best;
            }
        }
        if (ub >= 0) {
            skip = 1;
            if (t == 0) { // walk from it to the batch end
                uint32_t cur = spec_ld(pt, (uint64_t)ub * B + 4 * ug + 3);
                uint32_t j = ug + 1;
                for (uint64_t b = (uint64_t)ub; b < nb; b++, j = 0) {
                    const uint64_t b0 = b * B;
                    const uint32_t ng = (uint32_t)((uint64_t)n - b0 < B ? (uint64_t)n - b0 : B) >> 2;
                    for (; j < ng; j++)
                        spec_step(spec_ld(pt, b0 + 4 * j), spec_ld(pt, b0 + 4 * j + 1), spec_ld(pt, b0 + 4 * j + 2),
                                  spec_ld(pt, b0 + 4 * j + 3), cur);
                }
                meta[-1] = cur;
            }
        }
    }
    if (t == 0) {
        meta[SPEC_SKIP] = skip;
        if (hint) {
            // host-visible launch-size hint for the next call (pinned, mapped):
            // the worklist size class and the uniform flag, written only when
            // they change (a write to host memory delays the kernel's end)
            const uint32_t h0 = wl_cnt ? 32u - (uint32_t)__clz(wl_cnt) : 0u, h1 = meta[SPEC_UNIF];
            if (hint_h0 != h0 || hint_h1 != h1) {
                meta[SPEC_HINT] = h0;
                meta[SPEC_HINT + 1] = h1;
                __hip_atomic_store(&hint[0], h0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&hint[1], h1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// the 4 types of the group at packet j (16-B load when the burst size keeps
// groups 16-B aligned)
__device__ __forceinline__ void spec_group(const uint16_t *__restrict__ pt, uint64_t j, bool vec, uint32_t &l0,
                                           uint32_t &l1, uint32_t &l2, uint32_t &l3)
{
    if (vec) {
        const u32x2 q = *(const u32x2 *)(pt + j);
        l0 = q.x & 0xffffu;
        l1 = q.x >> 16;
        l2 = q.y & 0xffffu;
        l3 = q.y >> 16;
    } else {
        l0 = pt[j];
        l1 = pt[j + 1];
        l2 = pt[j + 2];
        l3 = pt[j + 3];
    }
}

// one burst's effect on a state of signature sig: SPEC_UNCH or the new state
__device__ uint32_t spec_burst_map(const uint16_t *__restrict__ pt, uint64_t b0, uint32_t cnt, uint32_t sig,
                                   bool vec)
{
    uint32_t low = sig >> 3, E = sig & 7u, c = SPEC_UNCH;
    for (uint32_t g = 0; g + 4 <= cnt; g += 4) {
        uint32_t l0, l1, l2, l3;
        spec_group(pt, b0 + g, vec, l0, l1, l2, l3);
        const bool quiet = (l0 & 0xffu) == low && (l1 & 0xffu) == low && (l2 & 0xffu) == low && (l3 & 0xffu) == low;
        if (!quiet && (l2 == l3 || E == cnet_edge(l3))) {
            c = l3;
            low = l3 & 0xffu;
            E = cnet_edge(l3);
        }
    }
    return c;
}

#define SPEC_STAGE 1024
// Wave-parallel shortcuts for a burst of <= 256 packets (lane g = group g),
// types staged in st as type | p_nxt << 16:
//  * a "universal" group (low bytes not all equal, 3rd type == 4th) moves
//    every state to its 4th type, so after the last one the walk no longer
//    depends on where it started;
//  * a "uniform" burst (every group: equal low bytes v, 3rd == 4th) leaves a
//    state with low byte v alone and sends any other to group 0's 4th type.
struct SpecGroups {
    unsigned long long U; // universal groups
    bool uniform;
    uint32_t v, first;    // uniform: the low byte, group 0's 4th type
};

__device__ __forceinline__ SpecGroups spec_groups(const uint32_t *st, uint32_t ng, uint32_t lane)
{
    SpecGroups r;
    bool allq = true, eq23 = false;
    uint32_t v = 0;
    if (lane < ng) {
        const u32x4 x = *(const u32x4 *)(st + 4 * lane);
        v = x.x & 0xffu;
        allq = (x.y & 0xffu) == v && (x.z & 0xffu) == v && (x.w & 0xffu) == v;
        eq23 = (x.z & 0xffffu) == (x.w & 0xffffu);
    }
    r.U = __ballot(lane < ng && !allq && eq23);
    const uint32_t v0 = __shfl(v, 0);
    const unsigned long long ok = __ballot(lane >= ng || (allq && eq23 && v == v0));
    r.uniform = ng > 0 && ok == ~0ull;
    r.v = v0;
    r.first = st[3] & 0xffffu;
    return r;
}

// walk groups [g0, g1) from a state given as (low byte, p_nxt, type)
__device__ __forceinline__ void spec_walk(const uint32_t *st, uint32_t g0, uint32_t g1, uint32_t &low, uint32_t &E,
                                          uint32_t &cur)
{
    for (uint32_t g = g0; g < g1; g++) {
        const u32x4 x = *(const u32x4 *)(st + 4 * g);
        const bool quiet = (x.x & 0xffu) == low && (x.y & 0xffu) == low && (x.z & 0xffu) == low &&
                           (x.w & 0xffu) == low;
        if (!quiet && ((x.z & 0xffffu) == (x.w & 0xffffu) || E == (x.w >> 16))) {
            cur = x.w & 0xffffu;
            low = x.w & 0xffu;
            E = x.w >> 16;
        }
    }
}

// one wave per burst: the burst's types are staged through LDS (1024 at a
// time) and lane k runs the group walk for signature class k
__global__ __launch_bounds__(256) void k_spec_tables(const uint16_t *__restrict__ pt, uint32_t n, uint32_t B,
                                                     uint64_t nb, const uint32_t *meta, const uint8_t *class_id,
                                                     uint32_t *T)
{
    __shared__ __attribute__((aligned(16))) uint32_t s_pt[4][SPEC_STAGE];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t b = (uint64_t)blockIdx.x * 4 + wv;
    const uint32_t K = meta[0];
    if (b >= nb || K > SPEC_KMAX || meta[SPEC_SKIP])
        return;
    uint32_t *st = s_pt[wv];
    const uint64_t b0 = b * B;
    const uint32_t cnt = (uint32_t)((uint64_t)n - b0 < B ? (uint64_t)n - b0 : B);
    const uint32_t sig = lane < K ? meta[1 + lane] : 0u;
    uint32_t low = sig >> 3, E = sig & 7u, c = SPEC_UNCH;
    for (uint32_t c0 = 0; c0 + 4 <= cnt; c0 += SPEC_STAGE) {
        const uint32_t m = cnt - c0 < SPEC_STAGE ? cnt - c0 : SPEC_STAGE;
        for (uint32_t k = lane; k < m; k += 64) { // type | p_nxt << 16, computed in parallel
            const uint32_t l = pt[b0 + c0 + k];
            st[k] = l | (cnet_edge(l) << 16);
        }
        __builtin_amdgcn_wave_barrier();
        if (cnt <= 256) { // one stage holds the burst: try the shortcuts
            const uint32_t ng = m >> 2;
            const SpecGroups sg = spec_groups(st, ng, lane);
            if (sg.U) { // every class ends where the walk from the last universal group ends
                const uint32_t u = 63u - (uint32_t)__clzll(sg.U);
                uint32_t cu = st[4 * u + 3] & 0xffffu, lu = cu & 0xffu, Eu = st[4 * u + 3] >> 16;
                spec_walk(st, u + 1, ng, lu, Eu, cu);
                c = cu;
                break;
            }
            if (sg.uniform) {
                c = low == sg.v ? SPEC_UNCH : sg.first;
                break;
            }
        }
        uint32_t cur = c;
        spec_walk(st, 0, m >> 2, low, E, cur);
        c = cur;
        __builtin_amdgcn_wave_barrier();
    }
    if (lane < K)
        T[b * SPEC_KMAX + lane] = spec_tag(c, class_id);
}

// Burst maps are composed with a two-level LDS scan, a map being
// SPEC_KFAST registers when at most that many signatures occur and
// SPEC_KMAX otherwise; the composition "E then L" sends a class k through E,
// then through L.
#define SPEC_KFAST 8
#define SPEC_BLK 256

// the map width of the scans for K signature classes (kfast = SPEC_KFAST, or
// 0 to force the wide maps; kmax = SPEC_KMAX, or 0 to force the sequential
// walk -- CNDP_TUNE_SPEC_SCAN)
__device__ __forceinline__ uint32_t spec_kf(uint32_t K, uint32_t kfast) { return K <= kfast ? SPEC_KFAST : SPEC_KMAX; }

// the 2 KiB class table into LDS with one 16-B load per thread (threads >= 128 idle)
__device__ __forceinline__ void spec_cls_stage(uint8_t *s_cls, const uint8_t *class_id, uint32_t tid, uint32_t nthr)
{
    for (uint32_t k = tid; k < 128; k += nthr)
        ((u32x4 *)s_cls)[k] = ((const u32x4 *)class_id)[k];
}

// plain state st after the tagged map m (in memory)
__device__ __forceinline__ uint32_t spec_apply(const uint32_t *m, const uint8_t *cls, uint32_t st)
{
    const uint32_t nx = m[cls[spec_sig(st)]];
    return nx == SPEC_UNCH ? st : nx & 0xffffu;
}

// tagged state st after the tagged map m (an LDS row)
__device__ __forceinline__ uint32_t spec_apply_t(const uint32_t *m, uint32_t st)
{
    const uint32_t nx = m[st >> 16];
    return nx == SPEC_UNCH ? st : nx;
}

// per block of SPEC_BLK bursts or chunks: inclusive scan of their maps (P),
// and the block's total map (Bt).  KF = the map width: SPEC_KFAST when at
// most that many signatures occur, else SPEC_KMAX (P and Bt rows are KF
// words; s_m rows KF + 1, so a row store by 64 lanes hits 64 banks).
template <uint32_t KF>
__device__ __forceinline__ void spec_scan_a_body(uint32_t *s_m, uint64_t nb, uint32_t K, const uint32_t *T,
                                                 uint32_t *P, uint32_t *Bt, uint64_t vb)
{
    const uint32_t t = threadIdx.x;
    const uint64_t b = vb * SPEC_BLK + t;
    uint32_t *row = s_m + t * (KF + 1);
    uint32_t m[KF];
#pragma unroll
    for (uint32_t k = 0; k < KF; k++)
        m[k] = b < nb && k < K ? T[b * SPEC_KMAX + k] : SPEC_UNCH;
    for (uint32_t d = 1; d < SPEC_BLK; d <<= 1) {
#pragma unroll
        for (uint32_t k = 0; k < KF; k++)
            row[k] = m[k];
        __syncthreads();
        if (t >= d) {
            const uint32_t *e = row - d * (KF + 1); // earlier map, then ours
#pragma unroll
            for (uint32_t k = 0; k < KF; k++) {
                const uint32_t ek = e[k];
                m[k] = k >= K ? SPEC_UNCH : ek == SPEC_UNCH ? row[k] : spec_apply_t(row, ek);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (uint32_t k = 0; k < KF; k++) { // unrolled: m stays in registers
        if (b < nb && k < K)
            P[b * KF + k] = m[k];
        if (t == SPEC_BLK - 1 && k < K)
            __hip_atomic_store(&Bt[vb * KF + k], m[k], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT); // sc1: read by the last block to arrive
    }
}

// block start states: Hillis-Steele over the block totals, W at a time with
// the composed map of the earlier windows carried along, and the final
// state (threads >= W only keep the barriers)
template <uint32_t KF, uint32_t W>
__device__ __forceinline__ void spec_scan_c_body(uint32_t *s_m, uint32_t *s_carry, uint64_t nblk, uint32_t K,
                                                 const uint8_t *class_id, const uint32_t *Bt, uint32_t *Sblk,
                                                 uint32_t *state)
{
    const uint32_t t = threadIdx.x;
    const bool act = t < W;
    uint32_t *row = s_m + t * (KF + 1);
    if (t < KF)
        s_carry[t] = SPEC_UNCH;
    const uint32_t s0 = spec_tag(state[SPEC_IN + 1] & 0xffffu, class_id); // state = meta - 1
    __syncthreads();
    for (uint64_t w0 = 0; w0 < nblk; w0 += W) {
        const uint64_t k0 = w0 + t;
        uint32_t m[KF];
#pragma unroll
        for (uint32_t k = 0; k < KF; k++)
            m[k] = act && k0 < nblk && k < K ? __hip_atomic_load((uint32_t *)&Bt[k0 * KF + k], __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT)
                                             : SPEC_UNCH;
        const uint32_t dmax = nblk - w0 < W ? (uint32_t)(nblk - w0) : W;
        for (uint32_t d = 1; d < dmax; d <<= 1) {
            if (act)
#pragma unroll
                for (uint32_t k = 0; k < KF; k++)
                    row[k] = m[k];
            __syncthreads();
            if (act && t >= d) {
                const uint32_t *e = row - d * (KF + 1);
#pragma unroll
                for (uint32_t k = 0; k < KF; k++) {
                    const uint32_t ek = e[k];
                    m[k] = k >= K ? SPEC_UNCH : ek == SPEC_UNCH ? row[k] : spec_apply_t(row, ek);
                }
            }
            __syncthreads();
        }
        if (act)
#pragma unroll
            for (uint32_t k = 0; k < KF; k++)
                row[k] = m[k];
        __syncthreads();
        // state entering block k0: the carry, then this window's blocks before k0
        if (act) {
            uint32_t st = spec_apply_t(s_carry, s0);
            if (t > 0)
                st = spec_apply_t(row - (KF + 1), st);
            if (k0 < nblk)
                Sblk[k0] = st; // tagged: the consumers index P rows with it
        }
        __syncthreads();
        if (t < KF) { // carry = carry then this window's total (entry t reads only entry t)
            const uint32_t *tot = s_m + (dmax - 1) * (KF + 1);
            const uint32_t ck = s_carry[t];
            s_carry[t] = t >= K ? SPEC_UNCH : ck == SPEC_UNCH ? tot[t] : spec_apply_t(tot, ck);
        }
        __syncthreads();
    }
    if (t == 0)
        *state = spec_apply_t(s_carry, s0) & 0xffffu;
}

// Both scan levels in one launch: every block scans its SPEC_BLK items
// (bursts or chunks) into P and writes its total to Bt with write-through
// (sc1) stores; after every wave's vmcnt(0) and a block barrier one lane adds
// to an arrival ticket (agent scope), and the block that draws the last
// ticket (acquire fence, sc1 loads of Bt) composes the totals into the block
// start states Sblk and the final state -- MI355X_MICROARCH.md hand-off row 1,
// no release fence (which writes back the XCD's dirty L2) on any block.  With
// more than SPEC_KMAX signatures (the parser's ptypes give fewer; a guard, not
// a path) that block's thread 0 walks the bursts sequentially instead
// (S = the state entering every burst).  gated: only when k_spec_local left
// a chunk unresolved (meta[SPEC_FULL]).
__global__ __launch_bounds__(SPEC_BLK) void k_spec_scan(uint64_t nitems, const uint32_t *meta, const uint32_t *T,
                                                      uint32_t *P, uint32_t *Bt, const uint8_t *class_id,
                                                      uint32_t *Sblk, uint32_t *state, uint32_t *ticket,
                                                      const uint16_t *__restrict__ pt, uint32_t n, uint32_t B,
                                                      uint64_t nb, uint32_t *S, uint32_t kfast, uint32_t kmax,
                                                      uint32_t gated)
{
    __shared__ uint32_t s_m[SPEC_BLK * (SPEC_KMAX + 1)];
    __shared__ uint32_t s_carry[SPEC_KMAX];
    __shared__ uint32_t s_last;
    const uint32_t K = meta[0];
    if (meta[SPEC_SKIP] || (gated && !meta[SPEC_FULL]))
        return;
    if (K <= kfast)
        spec_scan_a_body<SPEC_KFAST>(s_m, nitems, K, T, P, Bt, blockIdx.x);
    else if (K <= kmax)
        spec_scan_a_body<SPEC_KMAX>(s_m, nitems, K, T, P, Bt, blockIdx.x);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u;
    __syncthreads();
    if (!s_last)
        return;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (K <= kfast) {
        spec_scan_c_body<SPEC_KFAST, SPEC_BLK>(s_m, s_carry, gridDim.x, K, class_id, Bt, Sblk, state);
    } else if (K <= kmax) {
        spec_scan_c_body<SPEC_KMAX, SPEC_BLK>(s_m, s_carry, gridDim.x, K, class_id, Bt, Sblk, state);
    } else if (threadIdx.x == 0) {
        uint32_t st = meta[SPEC_IN] & 0xffffu;
        for (uint64_t b = 0; b < nb; b++) {
            S[b] = st;
            const uint64_t b0 = b * B;
            const uint32_t cnt = (uint32_t)((uint64_t)n - b0 < B ? (uint64_t)n - b0 : B);
            const uint32_t c = spec_burst_map(pt, b0, cnt, spec_sig(st), false);
            if (c != SPEC_UNCH)
                st = c;
        }
        *state = st;
    }
    if (threadIdx.x == 0)
        *ticket = 0; // for the next launch (kernel boundary)
}

// the plain state entering burst / chunk j of a scan block: the block's
// tagged start state sb, then the block's earlier items (inclusive prefix of
// item j - 1, kf-word rows of P)
__device__ __forceinline__ uint32_t spec_enter(const uint32_t *P, uint64_t j, uint32_t kf, uint32_t sb)
{
    if (j % SPEC_BLK == 0)
        return sb & 0xffffu;
    const uint32_t nx = P[(j - 1) * kf + (sb >> 16)];
    return (nx == SPEC_UNCH ? sb : nx) & 0xffffu;
}

// lbins != nullptr: the bin moves go to a block's LDS counters (flushed by
// the caller) -- the uniform pass moves every frame from the same few bins,
// and same-address global atomics serialize
// The one word a fix reads: the frame's own input-node result when its own
// edge is ip4/ip6_input (nh, or spec_nh without an nh output), else the
// speculated destination's when that is an input node (spec_nh), else none.
__device__ __forceinline__ uint32_t spec_fix_load(const KArgs &a, uint64_t i, uint32_t own_l, uint32_t dst)
{
    const uint32_t own = cnet_edge(own_l);
    if (own == 3u || own == 4u)
        return a.nh ? a.nh[i] : a.spec_nh[i];
    return dst == 3u || dst == 4u ? a.spec_nh[i] : 0u;
}

__device__ void spec_fix_v(const KArgs &a, uint64_t i, uint32_t own_l, uint32_t dst, uint32_t v, int *lbins)
{
    const uint32_t own = cnet_edge(own_l);
    const bool own_in = own == 3u || own == 4u;
    const uint32_t old_nh = own_in ? v : CNDP_NH_INVALID;
    const uint32_t old_edge = own_in ? old_nh >> 24 : 0x80u | own;
    const uint32_t nh = dst == 3u || dst == 4u ? v : CNDP_NH_INVALID;
    const uint32_t edge = dst == 3u || dst == 4u ? nh >> 24 : 0x80u | dst;
    if (a.nh)
        a.nh[i] = nh;
    if (a.edge)
        a.edge[i] = (uint8_t)edge;
    if (a.bins && lbins) {
        atomicAdd(&lbins[bin_of<CNDP_MODE_CNET>(old_nh, old_edge, 0, a.n_bins)], -1);
        atomicAdd(&lbins[bin_of<CNDP_MODE_CNET>(nh, edge, 0, a.n_bins)], 1);
    } else if (a.bins) {
        atomicAdd(&a.bins[bin_of<CNDP_MODE_CNET>(old_nh, old_edge, 0, a.n_bins)], ~0ull); // -1
        atomicAdd(&a.bins[bin_of<CNDP_MODE_CNET>(nh, edge, 0, a.n_bins)], 1ull);
    }
}

__device__ __forceinline__ void spec_fix(const KArgs &a, uint64_t i, uint32_t own_l, uint32_t dst,
                                         int *lbins = nullptr)
{
    spec_fix_v(a, i, own_l, dst, spec_fix_load(a, i, own_l, dst), lbins);
}

// one wave per burst: start state from the scan, types staged through LDS;
// every lane walks the groups (uniform, broadcast LDS reads) and remembers
// the state at the groups it owns (g % 64 == lane), then fixes those groups
__global__ __launch_bounds__(256) void k_spec_emit(KArgs a, uint32_t B, uint64_t nb, uint32_t kfast, uint32_t kmax,
                                                   const uint32_t *meta, const uint8_t *class_id, const uint32_t *P,
                                                   const uint32_t *Sblk, const uint32_t *S)
{
    __shared__ __attribute__((aligned(16))) uint32_t s_pt[4][SPEC_STAGE];
    __shared__ uint8_t s_q[4][SPEC_STAGE / 4];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t b = (uint64_t)blockIdx.x * 4 + wv;
    if (b >= nb || meta[SPEC_SKIP])
        return;
    uint32_t *st = s_pt[wv];
    const uint64_t b0 = b * B;
    const uint32_t cnt = (uint32_t)((uint64_t)a.n - b0 < B ? (uint64_t)a.n - b0 : B);
    uint32_t s0;
    if (meta[0] > kmax) {
        s0 = S[b];
    } else { // block start state through the block's earlier bursts (exclusive prefix)
        const uint64_t blk = b / SPEC_BLK;
        s0 = spec_enter(P, b, spec_kf(meta[0], kfast), Sblk[blk]);
    }
    uint32_t low = s0 & 0xffu, E = cnet_edge(s0);
    uint8_t *sq = s_q[wv];
    for (uint32_t c0 = 0; c0 + 4 <= cnt; c0 += SPEC_STAGE) {
        const uint32_t m = cnt - c0 < SPEC_STAGE ? cnt - c0 : SPEC_STAGE;
        for (uint32_t k = lane; k < m; k += 64) {
            const uint32_t l = a.spec_t16[b0 + c0 + k];
            st[k] = l | (cnet_edge(l) << 16);
        }
        __builtin_amdgcn_wave_barrier();
        if (cnt <= 256) {
            // lane g finds the state entering group g on its own: from the last
            // universal group before it, or (uniform burst) directly, or from
            // the burst start -- then marks its group
            const uint32_t ng = m >> 2;
            const SpecGroups sg = spec_groups(st, ng, lane);
            if (lane < ng) {
                uint32_t l = low, e = E, cur = 0;
                const unsigned long long before = sg.U & ((1ull << lane) - 1ull);
                if (before) {
                    const uint32_t u = 63u - (uint32_t)__clzll(before);
                    l = st[4 * u + 3] & 0xffu;
                    e = st[4 * u + 3] >> 16;
                    spec_walk(st, u + 1, lane, l, e, cur);
                } else if (sg.uniform) {
                    if (lane > 0 && low != sg.v) {
                        l = sg.first & 0xffu;
                        e = st[3] >> 16;
                    }
                } else {
                    spec_walk(st, 0, lane, l, e, cur);
                }
                const u32x4 x = *(const u32x4 *)(st + 4 * lane);
                const bool quiet = (x.x & 0xffu) == l && (x.y & 0xffu) == l && (x.z & 0xffu) == l &&
                                   (x.w & 0xffu) == l;
                sq[lane] = quiet ? (uint8_t)(0x80u | e) : (uint8_t)0;
            }
        } else {
            // the node walk (uniform over the wave): per group, quiet under the
            // state (0x80 | p_nxt[state]) or not (0)
            for (uint32_t g = 0; g + 4 <= m; g += 4) {
                const u32x4 x = *(const u32x4 *)(st + g);
                const bool quiet = (x.x & 0xffu) == low && (x.y & 0xffu) == low && (x.z & 0xffu) == low &&
                                   (x.w & 0xffu) == low;
                if (lane == 0)
                    sq[g >> 2] = quiet ? (uint8_t)(0x80u | E) : (uint8_t)0;
                if (!quiet && ((x.z & 0xffffu) == (x.w & 0xffffu) || E == (x.w >> 16))) {
                    low = x.w & 0xffu;
                    E = x.w >> 16;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        for (uint32_t gi = lane; gi * 4 + 4 <= m; gi += 64) {
            const uint32_t q = sq[gi];
            if (q & 0x80u)
                for (uint32_t j = 0; j < 4; j++) {
                    const uint32_t x = st[gi * 4 + j];
                    if ((x >> 16) != (q & 7u))
                        spec_fix(a, b0 + c0 + gi * 4 + j, x & 0xffffu, q & 7u);
                }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------------------
// Chunked speculation passes for graph bursts of B <= 256 packets (<= 64
// groups, one group per lane): one wave per chunk of SPEC_CH bursts, the
// chunk's types staged in LDS by one batch of loads.
//   spec_ctable_chunk  the chunk's map (its bursts' maps composed), lane k =
//                   signature class k -- the scans then run over chunks;
//   spec_cemit_chunk   from the chunk's entering state, burst after burst: lane
//                   g finds the state entering group g, fixes its frames if
//                   the group is quiet under it, and lane ng-1 hands the
//                   burst's exit state to the next burst.
// ---------------------------------------------------------------------------
#define SPEC_CH SPEC_CH_K // measured: 4 beats 1 and 16 (occupancy vs per-wave latency)
#ifndef SPEC_LQ
#define SPEC_LQ 4 // chunks per wave of k_spec_local_t (grid-stride, next chunk prefetched; 4 beats 1, 2, 8)
#endif
#ifndef SPEC_WPB
#define SPEC_WPB 4 // waves (chunks) per block of k_spec_local (measured: 4 beats 8 and 16)
#endif

// stage the types of bursts [c0, c1) as type | p_nxt << 16, burst j at
// st + (j - c0) * spec_bstride(B) (16-B aligned groups for any B)
__device__ __forceinline__ uint32_t spec_bstride(uint32_t B) { return (B + 3u) & ~3u; }

// em: bit 6 * spec_lowslot(low) + edge for every staged type (slots < SPEC_LOWS)
__device__ __forceinline__ unsigned long long spec_em(uint32_t l, uint32_t e)
{
    const uint32_t q = spec_lowslot(l & 0xffu);
    return q < SPEC_LOWS ? 1ull << (6 * q + e) : 0ull;
}

template <int CH>
__device__ __forceinline__ unsigned long long spec_stage_chunk(const uint16_t *__restrict__ pt, uint32_t n,
                                                               uint32_t B, uint64_t c0, uint64_t c1, uint32_t lane,
                                                               uint32_t *st, const uint16_t *lut)
{
    unsigned long long em = 0;
    const uint32_t bs = spec_bstride(B);
    if ((B & 7u) == 0) {
        // bursts are contiguous in LDS too (bs == B): 16-B loads of 8 types,
        // every load of the chunk issued before the first is used
        const uint64_t p0 = c0 * B, p1 = c1 * B < n ? c1 * B : n;
        const uint32_t m = (uint32_t)(p1 - p0);
        constexpr uint32_t R = CH * 256 / 512 > 0 ? CH * 256 / 512 : 1;
        u32x4 v[R];
#pragma unroll
        for (uint32_t r = 0; r < R; r++) {
            const uint32_t idx = (r * 64u + lane) * 8u;
            v[r] = idx + 8u <= m ? *(const u32x4 *)(pt + p0 + idx) : (u32x4){0, 0, 0, 0};
        }
#pragma unroll
        for (uint32_t r = 0; r < R; r++) {
            const uint32_t idx = (r * 64u + lane) * 8u;
            if (idx >= m)
                continue;
            uint32_t w[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
            if (idx + 8u > m) // the batch's last partial vector
                for (uint32_t q = 0; q < 4; q++) {
                    const uint32_t lo = idx + 2 * q < m ? pt[p0 + idx + 2 * q] : 0u;
                    const uint32_t hi = idx + 2 * q + 1 < m ? pt[p0 + idx + 2 * q + 1] : 0u;
                    w[q] = lo | (hi << 16);
                }
            uint32_t o[8];
#pragma unroll
            for (uint32_t q = 0; q < 8; q++) {
                const uint32_t l = (w[q >> 1] >> (16 * (q & 1u))) & 0xffffu, x = cnet_lut_x(lut, l);
                o[q] = l | ((x >> 6) << 16);
                if (idx + q < m)
                    em |= 1ull << (x & 63u);
            }
            *(u32x4 *)(st + idx) = (u32x4){o[0], o[1], o[2], o[3]};
            *(u32x4 *)(st + idx + 4) = (u32x4){o[4], o[5], o[6], o[7]};
        }
    } else {
        for (uint64_t j = c0; j < c1; j++) {
            const uint64_t p0 = j * B;
            const uint32_t cnt = (uint32_t)((uint64_t)n - p0 < B ? (uint64_t)n - p0 : B);
            uint32_t *d = st + (j - c0) * bs;
            for (uint32_t k = lane; k < cnt; k += 64) {
                const uint32_t l = pt[p0 + k], x = cnet_lut_x(lut, l);
                d[k] = l | ((x >> 6) << 16);
                em |= 1ull << (x & 63u);
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    return em & ~(1ull << 63); // bit 63: types outside the slots
}

// Edge-consistency summary of a chunk (em OR-reduced over the wave).  Only
// the low bytes in spec_lowslot() carry types of different p_nxt
// (ptype.c:32-46; every other type goes to pkt_drop), so per slot the chunk
// records which edges its frames have: slot r = bit 3 present, bits 0..2 its
// edge; bit 31 = a slot with two edges.  A chunk where each slot has at most
// one edge cannot re-route a frame unless the entering state disagrees.
__device__ __forceinline__ uint32_t spec_summary(unsigned long long em)
{
    for (int o = 32; o > 0; o >>= 1)
        em |= __shfl_xor(em, o);
    uint32_t sm = 0;
#pragma unroll
    for (uint32_t r = 0; r < SPEC_LOWS; r++) {
        const uint32_t v = (uint32_t)(em >> (6 * r)) & 0x3fu;
        if (v & (v - 1u))
            sm |= 1u << 31;
        else if (v)
            sm |= (8u | (31u - (uint32_t)__clz(v))) << (4 * r);
    }
    return sm;
}

// true when no frame of a chunk with summary sm can leave by another edge
// from the entering state s0
__device__ __forceinline__ bool spec_chunk_quiet(uint32_t sm, uint32_t s0)
{
    const uint32_t q0 = spec_lowslot(s0 & 0xffu);
    const uint32_t slot = q0 < SPEC_LOWS ? (sm >> (4 * q0)) & 0xfu : 0u;
    return !(sm >> 31) && (!(slot & 8u) || (slot & 7u) == cnet_edge(s0));
}

// chunk c's map (lane k = signature class k) and its edge summary into T
template <int CH>
__device__ __forceinline__ void spec_ctable_chunk(const uint16_t *__restrict__ pt, uint32_t n, uint32_t B, uint64_t nb, uint64_t nch,
                                  uint64_t c, uint32_t K, const uint32_t *meta, uint32_t *T, uint32_t *st,
                                  const uint16_t *s_lut, const uint8_t *s_cls)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t c0 = c * CH, c1 = c0 + CH < nb ? c0 + CH : nb;
    unsigned long long em = spec_stage_chunk<CH>(pt, n, B, c0, c1, lane, st, s_lut);
    const uint32_t sig = lane < K ? meta[1 + lane] : 0u;
    uint32_t cm = SPEC_UNCH;
    for (uint64_t bb = c0; bb < c1; bb++) {
        const uint32_t *sb = st + (bb - c0) * spec_bstride(B);
        const uint64_t b0 = bb * B;
        const uint32_t cnt = (uint32_t)((uint64_t)n - b0 < B ? (uint64_t)n - b0 : B);
        const uint32_t ng = cnt >> 2;
        const SpecGroups sg = spec_groups(sb, ng, lane);
        uint32_t mp = SPEC_UNCH;
        if (sg.U) {
            const uint32_t u = 63u - (uint32_t)__clzll(sg.U);
            uint32_t cu = sb[4 * u + 3] & 0xffffu, lu = cu & 0xffu, Eu = sb[4 * u + 3] >> 16;
            spec_walk(sb, u + 1, ng, lu, Eu, cu);
            mp = cu;
        } else if (sg.uniform) {
            mp = (sig >> 3) == sg.v ? SPEC_UNCH : sg.first;
        } else {
            uint32_t low = sig >> 3, E = sig & 7u;
            spec_walk(sb, 0, ng, low, E, mp);
        }
        // cm = this burst after the chunk so far (tagged states)
        // tag with the class (LDS tables, not two dependent global loads)
        mp = lane < K && mp != SPEC_UNCH ? mp | ((uint32_t)s_cls[((mp & 0xffu) << 3) | cnet_edge_l(s_lut, mp)] << 16)
                                          : SPEC_UNCH;
        const uint32_t nx = __shfl(mp, (int)(cm == SPEC_UNCH ? 0u : cm >> 16));
        cm = cm == SPEC_UNCH ? mp : nx == SPEC_UNCH ? cm : nx;
    }
    if (lane < K)
        T[c * SPEC_KMAX + lane] = cm;
    const uint32_t sm = spec_summary(em);
    if (lane == 0)
        T[nch * SPEC_KMAX + c] = sm;
}

template <int CH>
__device__ __forceinline__ void spec_replay(const KArgs &a, uint32_t B, uint64_t c0, uint64_t c1, uint32_t s0, uint32_t lane,
                            const uint32_t *st, int *lbins = nullptr);
template <int CH>
__device__ __forceinline__ void spec_replay_walk(const KArgs &a, uint32_t B, uint64_t c0, uint64_t c1, uint32_t s0,
                                                 uint32_t lane, const uint32_t *st, uint32_t &fm, uint32_t &fe);
template <int CH>
__device__ __forceinline__ void spec_replay_fix(const KArgs &a, uint32_t B, uint64_t c0, uint32_t lane,
                                                const uint32_t *st, uint32_t fm, uint32_t fe, int *lbins = nullptr);

// replay chunk c from its entering state (the scan's block start, then the
// block's earlier chunks) unless its summary says no frame can move
template <int CH>
__device__ __forceinline__ void spec_cemit_chunk(const KArgs &a, uint32_t B, uint64_t nb, uint64_t nch, uint64_t c,
                                 const uint32_t *meta, const uint32_t *P, const uint32_t *Sblk, const uint32_t *S,
                                 const uint32_t *T, uint32_t kfast, uint32_t kmax, uint32_t *st,
                                 const uint16_t *s_lut)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t c0 = c * CH, c1 = c0 + CH < nb ? c0 + CH : nb;
    uint32_t s0;
    if (meta[0] > kmax) {
        s0 = S[c0];
    } else {
        const uint64_t blk = c / SPEC_BLK;
        s0 = spec_enter(P, c, spec_kf(meta[0], kfast), Sblk[blk]);
    }
    // spec_ctable_chunk wrote the chunk's summary
    if (meta[0] <= SPEC_KMAX && spec_chunk_quiet(T[nch * SPEC_KMAX + c], s0))
        return; // no frame of this chunk can leave by another edge
    spec_stage_chunk<CH>(a.spec_t16, a.n, B, c0, c1, lane, st, s_lut);
    spec_replay<CH>(a, B, c0, c1, s0, lane, st);
}

// replay the staged chunk [c0, c1) from its entering state s0: lane g finds
// the state entering group g, fixes the group's frames if it is quiet under
// that state, and lane ng-1 hands the burst's exit state to the next burst
template <int CH>
__device__ __forceinline__ void spec_replay(const KArgs &a, uint32_t B, uint64_t c0, uint64_t c1, uint32_t s0, uint32_t lane,
                            const uint32_t *st, int *lbins)
{
    uint32_t fm, fe;
    spec_replay_walk<CH>(a, B, c0, c1, s0, lane, st, fm, fe);
    SP_TS(8, __builtin_amdgcn_s_memrealtime());
    spec_replay_fix<CH>(a, B, c0, lane, st, fm, fe, lbins);
}

// the walk: fm = frames to fix (bit 4 * burst + j), fe = each burst's edge (3 bits)
// A type is plain when its p_nxt is its low byte's common edge (spec_canon).
// A group of four plain types entered in a plain state moves no frame: quiet,
// its low bytes are the state's and their edge is the state's p_nxt.  The
// state entering group g is the 4th type of the last group before g that set
// it (a universal group always does), or the burst's entering state, so it
// can be other than plain only when a group in [last universal before g, g)
// has a 4th type that is not, or with no universal group before g, when the
// entering state is not.  Only those lanes, the lanes holding a type that is
// not plain and the last lane (the burst's exit state) walk.
template <int CH>
__device__ __forceinline__ void spec_replay_walk(const KArgs &a, uint32_t B, uint64_t c0, uint64_t c1, uint32_t s0,
                                                 uint32_t lane, const uint32_t *st, uint32_t &fm, uint32_t &fe)
{
    static_assert(CH <= 8, "fix masks: 4 frames and 3 edge bits per burst");
    fm = 0;
    fe = 0;
    for (uint64_t bb = c0; bb < c1; bb++) {
        const uint32_t *sb = st + (bb - c0) * spec_bstride(B);
        const uint64_t b0 = bb * B;
        const uint32_t cnt = (uint32_t)((uint64_t)a.n - b0 < B ? (uint64_t)a.n - b0 : B);
        const uint32_t ng = cnt >> 2;
        const SpecGroups sg = spec_groups(sb, ng, lane);
        const uint32_t low0 = s0 & 0xffu;
        uint32_t nxt = s0; // the state after this lane's group
        bool need = false;
        {
            u32x4 y = lane < ng ? *(const u32x4 *)(sb + 4 * lane) : (u32x4){0x30011u, 0x30011u, 0x30011u, 0x30011u};
            const bool p0 = spec_canon(y.x & 0xffu) == (y.x >> 16), p1 = spec_canon(y.y & 0xffu) == (y.y >> 16);
            const bool p2 = spec_canon(y.z & 0xffu) == (y.z >> 16), p3 = spec_canon(y.w & 0xffu) == (y.w >> 16);
            const unsigned long long O = __ballot(!p3), below = (1ull << lane) - 1ull, ub = sg.U & below;
            const uint32_t lu = ub ? 63u - (uint32_t)__clzll(ub) : 0u;
            const bool s0p = spec_canon(low0) == cnet_edge(s0);
            need = !(p0 && p1 && p2 && p3) || ((O & below) >> lu) != 0ull || (!s0p && ub == 0ull) ||
                   lane + 1u == ng;
        }
#if CD_STAMP
        if (bb == c0) { // the first burst: the longest walk (groups) and the lanes that walk
            const unsigned long long bef = sg.U & ((1ull << lane) - 1ull);
            uint32_t wl = lane < ng && need ? lane - (bef ? 64u - (uint32_t)__clzll(bef) : 0u) : 0u;
            for (int o = 32; o > 0; o >>= 1)
                wl = max(wl, (uint32_t)__shfl_xor((int)wl, o));
            SP_TS(15, (uint64_t)wl | ((uint64_t)__popcll(__ballot(lane < ng && need)) << 32));
            SP_TS(14, __builtin_amdgcn_s_memrealtime());
        }
#endif
        if (lane < ng && need) {
            // the state entering group `lane`
            uint32_t cur = s0, l = low0, e = cnet_edge(s0);
            const unsigned long long before = sg.U & ((1ull << lane) - 1ull);
            if (before) {
                const uint32_t u = 63u - (uint32_t)__clzll(before);
                cur = sb[4 * u + 3] & 0xffffu;
                l = cur & 0xffu;
                e = sb[4 * u + 3] >> 16;
                spec_walk(sb, u + 1, lane, l, e, cur);
            } else if (sg.uniform) {
                if (lane > 0 && low0 != sg.v) {
                    cur = sg.first;
                    l = cur & 0xffu;
                    e = sb[3] >> 16;
                }
            } else {
                spec_walk(sb, 0, lane, l, e, cur);
            }
            const u32x4 x = *(const u32x4 *)(sb + 4 * lane);
            const bool quiet = (x.x & 0xffu) == l && (x.y & 0xffu) == l && (x.z & 0xffu) == l && (x.w & 0xffu) == l;

            nxt = cur;
            if (!quiet && ((x.z & 0xffffu) == (x.w & 0xffffu) || e == (x.w >> 16)))
                nxt = x.w & 0xffffu;
            if (quiet) { // the group goes whole to p_nxt[state]: mark the frames that move
                const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (uint32_t j = 0; j < 4; j++)
                    fm |= (uint32_t)((xs[j] >> 16) != e) << (4u * (uint32_t)(bb - c0) + j);
                fe |= e << (3u * (uint32_t)(bb - c0));
            }
        }
        s0 = ng ? __shfl(nxt, (int)ng - 1) : s0;
        SP_TS(10 + (uint32_t)(bb - c0), __builtin_amdgcn_s_memrealtime());
    }
}

// the fixes after the walk, a burst at a time: its reads first, then its
// writes (bursts without a fix cost nothing)
template <int CH>
__device__ __forceinline__ void spec_replay_fix(const KArgs &a, uint32_t B, uint64_t c0, uint32_t lane,
                                                const uint32_t *st, uint32_t fm, uint32_t fe, int *lbins)
{
#pragma unroll 1
    for (uint32_t bq = 0; bq < (uint32_t)CH; bq++) {
        const uint32_t m4 = (fm >> (4u * bq)) & 0xfu, dst = (fe >> (3u * bq)) & 7u;
        if (__ballot(m4 != 0u) == 0ull)
            continue;
        const uint32_t *sg = st + bq * spec_bstride(B) + lane * 4u;
        const uint64_t i0 = (c0 + bq) * B + lane * 4u;
        uint32_t v[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; j++)
            v[j] = (m4 >> j) & 1u ? spec_fix_load(a, i0 + j, sg[j] & 0xffffu, dst) : 0u;
#pragma unroll
        for (uint32_t j = 0; j < 4; j++)
            if ((m4 >> j) & 1u)
                spec_fix_v(a, i0 + j, sg[j] & 0xffffu, dst, v[j], lbins);
    }
}

// ---------------------------------------------------------------------------
// Local resolution (bursts <= 256, the default): the state entering chunk c
// is the walk from the last universal group before it, and for IMIX-like
// traffic one sits in the previous chunk's last burst.  k_spec_local finds it
// there, stages chunk c and replays it when its summary says a frame could
// leave by another edge; the last chunk's wave also walks the final state.  A
// chunk whose previous chunk holds no universal group (long single-type runs)
// is left to the table / scan / replay passes, which run only then
// (meta[SPEC_FULL]) and replay only the chunks left (done[c] == 0).
// ---------------------------------------------------------------------------
// group `lane` of the burst at packet b0 (cnt packets) as two words
__device__ __forceinline__ void spec_group_regs(const uint16_t *__restrict__ pt, uint64_t b0, uint32_t cnt,
                                                uint32_t lane, uint32_t &q0, uint32_t &q1)
{
    q0 = q1 = 0;
    if (4 * lane + 4 <= cnt) {
        if ((b0 & 3u) == 0) {
            const u32x2 v = *(const u32x2 *)(pt + b0 + 4 * lane);
            q0 = v.x;
            q1 = v.y;
        } else {
            const uint16_t *g = pt + b0 + 4 * lane;
            q0 = (uint32_t)g[0] | ((uint32_t)g[1] << 16);
            q1 = (uint32_t)g[2] | ((uint32_t)g[3] << 16);
        }
    }
}

// walk groups [g0, ng) of a burst held one group per lane (ptype.c:95-130):
// g0 and ng are wave-uniform, so the walk is a scalar loop (v_readlane) with
// the 4th types' p_nxt looked up for all groups at once
__device__ __forceinline__ void spec_walk_regs(uint32_t q0, uint32_t q1, uint32_t g0, uint32_t ng,
                                               const uint16_t *lut, uint32_t &cur)
{
    const uint32_t v = q0 & 0xffu;
    const bool allq = ((q0 >> 16) & 0xffu) == v && (q1 & 0xffu) == v && ((q1 >> 16) & 0xffu) == v;
    const uint32_t gq = (allq ? v : 0x1FFu) | ((q1 & 0xffffu) == (q1 >> 16) ? 0x200u : 0u);
    const uint32_t d = (q1 >> 16) | (cnet_edge_l(lut, q1 >> 16) << 16);
    uint32_t c = __builtin_amdgcn_readfirstlane(cur);
    uint32_t E = __builtin_amdgcn_readfirstlane(cnet_edge_l(lut, c));
    for (uint32_t g = g0; g < ng; g++) {
        const uint32_t qg = (uint32_t)__builtin_amdgcn_readlane((int)gq, (int)g);
        const uint32_t dg = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)g);
        if ((qg & 0x1FFu) != (c & 0xffu) && ((qg & 0x200u) || E == (dg >> 16))) {
            c = dg & 0xffffu;
            E = dg >> 16;
        }
    }
    cur = c;
}

// the node state after bursts [b_lo, b_hi): the walk from the last universal
// group in them to their end; false when they hold none
// pre: the groups of burst b_hi - 1 are already in (pq0, pq1) (loaded by
// the caller ahead of its barrier)
__device__ __forceinline__ bool spec_lookback(const uint16_t *__restrict__ pt, uint32_t n, uint32_t B, uint64_t b_lo, uint64_t b_hi,
                              uint32_t lane, const uint16_t *lut, uint32_t &s_out, bool pre = false,
                              uint32_t pq0 = 0, uint32_t pq1 = 0)
{
    for (uint64_t j = b_hi; j-- > b_lo;) {
        const uint64_t b0 = j * B;
        const uint32_t cnt = (uint32_t)((uint64_t)n - b0 < B ? (uint64_t)n - b0 : B), ng = cnt >> 2;
        uint32_t q0, q1;
        if (pre && j + 1 == b_hi) {
            q0 = pq0;
            q1 = pq1;
        } else {
            spec_group_regs(pt, b0, cnt, lane, q0, q1);
        }
        const uint32_t v = q0 & 0xffu;
        const bool allq = ((q0 >> 16) & 0xffu) == v && (q1 & 0xffu) == v && ((q1 >> 16) & 0xffu) == v;
        const unsigned long long U = __ballot(lane < ng && !allq && (q1 & 0xffffu) == (q1 >> 16));
        if (U) {
            const uint32_t u = 63u - (uint32_t)__clzll(U);
            uint32_t cur = __shfl(q1, (int)u) >> 16;
            spec_walk_regs(q0, q1, u + 1, ng, lut, cur);
            for (uint64_t k = j + 1; k < b_hi; k++) {
                const uint64_t k0 = k * B;
                const uint32_t kc = (uint32_t)((uint64_t)n - k0 < B ? (uint64_t)n - k0 : B);
                spec_group_regs(pt, k0, kc, lane, q0, q1);
                spec_walk_regs(q0, q1, 0, kc >> 2, lut, cur);
            }
            s_out = cur;
            return true;
        }
    }
    return false;
}

// raise meta[SPEC_FULL]: read first, so that a batch where every chunk is
// unresolved (single-type traffic, C5) does not serialize one atomic per wave
// on one word (that cost C5 0.4 ms)
__device__ __forceinline__ void spec_flag_full(uint32_t *meta)
{
    if (!__hip_atomic_load(&meta[SPEC_FULL], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        __hip_atomic_store(&meta[SPEC_FULL], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// uniform batch (spec_classes): every frame of a full group of bursts
// [c0, c1) leaves by edge E, the entering state's p_nxt; fix those whose own
// edge differs.  Tail frames (a burst's last cnt % 4) keep their own edge.
// A wave takes one chunk and issues all its type loads (16 B = 8 types
// each) before the first is used (4 chunks per wave measured slower on C5)
template <int CH>
__device__ __forceinline__ void spec_uniform_range(const KArgs &a, uint32_t B, uint64_t c0, uint64_t c1, uint32_t lane,
                                                   uint32_t T, int *lbins)
{
    // T: the node state; 8 types all equal to it need no cnet_edge (4 compares)
    const uint32_t E = cnet_edge(T), TT = T | (T << 16);
    constexpr uint32_t U = CH * 256 / 512 > 0 ? CH * 256 / 512 : 1;
    const uint32_t p0 = (uint32_t)(c0 * B), p1 = (uint32_t)(c1 * B < a.n ? c1 * B : a.n);
    const bool vec = (B & 7u) == 0;
    u32x4 v[U];
#pragma unroll
    for (uint32_t r = 0; r < U; r++) {
        const uint32_t i0 = p0 + (r * 64u + lane) * 8u;
        v[r] = vec && i0 + 8u <= p1 ? *(const u32x4 *)(a.spec_t16 + i0) : (u32x4){0, 0, 0, 0};
    }
    // B <= 256 here (spec_classes), so a wave's range is <= U * 512 types
#pragma unroll
    for (uint32_t r = 0; r < U; r++) {
        const uint32_t i0 = p0 + (r * 64u + lane) * 8u;
        const bool full8 = vec && i0 + 8u <= p1;
        u32x4 x = v[r];
        const bool same = (i0 >= p1) | (full8 & (x.x == TT) & (x.y == TT) & (x.z == TT) & (x.w == TT));
        if (__all(same)) // wave-uniform skip
            continue;
        if (!same && !full8) { // ragged end, or bursts not a multiple of 8
            uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
            for (uint32_t q = 0; q < 8; q++)
                w[q >> 1] |= (i0 + q < p1 ? (uint32_t)a.spec_t16[i0 + q] : 0u) << (16 * (q & 1u));
            x = (u32x4){w[0], w[1], w[2], w[3]};
        }
        // frames of this vector whose own edge differs, then one fix site
        uint32_t m = 0;
        if (!same) {
            const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (uint32_t q = 0; q < 8; q++)
                m |= (uint32_t)((i0 + q < p1) & (cnet_edge((w[q >> 1] >> (16 * (q & 1u))) & 0xffffu) != E)) << q;
        }
        const uint64_t lo = ((uint64_t)x.y << 32) | x.x, hi = ((uint64_t)x.w << 32) | x.z;
        while (m) {
            const uint32_t q = (uint32_t)__ffs(m) - 1u;
            m &= m - 1u;
            const uint32_t i = i0 + q, l = (uint32_t)((q < 4 ? lo : hi) >> (16 * (q & 3u))) & 0xffffu;
            const uint32_t b0 = i / B * B, bend = b0 + B < a.n ? b0 + B : a.n;
            if (b0 + ((i - b0) & ~3u) + 4u <= bend) // a full group
                spec_fix(a, i, l, E, lbins);
        }
    }
}

// a chunk whose entering state s0 is known, from its types: the edge
// summary from registers (16-B loads of 8 when the bursts allow), then --
// when a frame could leave by another edge -- staged in LDS and replayed
template <int CH>
__device__ __forceinline__ void spec_chunk_load(const KArgs &a, uint32_t B, uint64_t c0, uint64_t c1, uint32_t lane,
                                                u32x4 (&v)[CH * 256 / 512 > 0 ? CH * 256 / 512 : 1]);
template <int CH>
__device__ __forceinline__ void spec_chunk_types_v(const KArgs &a, uint32_t B, uint64_t c0, uint64_t c1, uint32_t s0,
                                                   uint32_t lane, uint32_t *st, const uint16_t *s_lut, int *lbins,
                                                   const u32x4 (&v)[CH * 256 / 512 > 0 ? CH * 256 / 512 : 1]);
template <int CH>
__device__ __forceinline__ void spec_chunk_types(const KArgs &a, uint32_t B, uint64_t c0, uint64_t c1, uint32_t s0,
                                                 uint32_t lane, uint32_t *st, const uint16_t *s_lut, int *lbins)
{
    if ((B & 7u) != 0) {
        const unsigned long long em = spec_stage_chunk<CH>(a.spec_t16, a.n, B, c0, c1, lane, st, s_lut);
        if (!spec_chunk_quiet(spec_summary(em), s0))
            spec_replay<CH>(a, B, c0, c1, s0, lane, st, lbins);
        return;
    }
    constexpr uint32_t R = CH * 256 / 512 > 0 ? CH * 256 / 512 : 1;
    u32x4 v[R];
    spec_chunk_load<CH>(a, B, c0, c1, lane, v);
    spec_chunk_types_v<CH>(a, B, c0, c1, s0, lane, st, s_lut, lbins, v);
}

// the types of chunk [c0, c1) as 16-B loads of 8 (bursts of a multiple of 8)
template <int CH>
__device__ __forceinline__ void spec_chunk_load(const KArgs &a, uint32_t B, uint64_t c0, uint64_t c1, uint32_t lane,
                                                u32x4 (&v)[CH * 256 / 512 > 0 ? CH * 256 / 512 : 1])
{
    constexpr uint32_t R = CH * 256 / 512 > 0 ? CH * 256 / 512 : 1;
    const uint64_t p0 = c0 * B, p1 = c1 * B < a.n ? c1 * B : a.n;
    const uint32_t m = (uint32_t)(p1 - p0);
#pragma unroll
    for (uint32_t r = 0; r < R; r++) {
        const uint32_t idx = (r * 64u + lane) * 8u;
        v[r] = idx + 8u <= m ? *(const u32x4 *)(a.spec_t16 + p0 + idx) : (u32x4){0, 0, 0, 0};
    }
}

// spec_chunk_types for bursts of a multiple of 8 from the loaded types v
template <int CH>
__device__ __forceinline__ void spec_chunk_types_v(const KArgs &a, uint32_t B, uint64_t c0, uint64_t c1, uint32_t s0,
                                                   uint32_t lane, uint32_t *st, const uint16_t *s_lut, int *lbins,
                                                   const u32x4 (&v)[CH * 256 / 512 > 0 ? CH * 256 / 512 : 1])
{
    constexpr uint32_t R = CH * 256 / 512 > 0 ? CH * 256 / 512 : 1;
    const uint64_t p0 = c0 * B, p1 = c1 * B < a.n ? c1 * B : a.n;
    const uint32_t m = (uint32_t)(p1 - p0);
    // the summary and the LDS staging (spec_stage_chunk's layout) from the
    // same registers: a replay does not load the types a second time
    unsigned long long em = 0;
#pragma unroll
    for (uint32_t r = 0; r < R; r++) {
        const uint32_t idx = (r * 64u + lane) * 8u;
        if (idx >= m)
            continue;
        uint32_t w[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
        if (idx + 8u > m) // the batch's last partial vector
            for (uint32_t q = 0; q < 4; q++) {
                const uint32_t lo = idx + 2 * q < m ? a.spec_t16[p0 + idx + 2 * q] : 0u;
                const uint32_t hi = idx + 2 * q + 1 < m ? a.spec_t16[p0 + idx + 2 * q + 1] : 0u;
                w[q] = lo | (hi << 16);
            }
        uint32_t o[8];
#pragma unroll
        for (uint32_t q = 0; q < 8; q++) {
            const uint32_t l = (w[q >> 1] >> (16 * (q & 1u))) & 0xffffu, x = cnet_lut_x(s_lut, l);
            o[q] = l | ((x >> 6) << 16);
            if (idx + q < m)
                em |= 1ull << (x & 63u);
        }
        *(u32x4 *)(st + idx) = (u32x4){o[0], o[1], o[2], o[3]};
        *(u32x4 *)(st + idx + 4) = (u32x4){o[4], o[5], o[6], o[7]};
    }
    __builtin_amdgcn_wave_barrier();
    SP_TS(7, __builtin_amdgcn_s_memrealtime());
    if (!spec_chunk_quiet(spec_summary(em & ~(1ull << 63)), s0))
        spec_replay<CH>(a, B, c0, c1, s0, lane, st, lbins);
    SP_TS(9, __builtin_amdgcn_s_memrealtime());
}

template <int CH, int WPB>
__global__ __launch_bounds__(WPB * 64) void k_spec_local(KArgs a, uint32_t B, uint64_t nb, uint64_t nch, uint32_t *meta,
                                                    uint8_t *done)
{
    __shared__ __attribute__((aligned(16))) uint32_t s_pt[WPB][CH * 256];
    __shared__ __attribute__((aligned(16))) uint16_t s_lut[CNET_LUT_N];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t c = (uint64_t)blockIdx.x * WPB + wv;
    if (meta[SPEC_UNIF]) { // block-uniform; wave c takes chunks [c*W, c*W + W), the rest return
        const uint64_t u0 = c * CH, u1 = u0 + CH;
        static_assert(WPB * CH * 256 >= CNDP_BINS_MAX + 2, "bin counters must fit the staging tile");
        int *lbins = (int *)&s_pt[0][0]; // n_bins + 2 <= CNDP_BINS_MAX + 2 ints fit the staging tile
        const uint32_t nb2 = a.bins ? a.n_bins + 2u : 0u;
        for (uint32_t k = threadIdx.x; k < nb2; k += WPB * 64u)
            lbins[k] = 0;
        __syncthreads();
        if (u0 < nb)
            spec_uniform_range<CH>(a, B, u0, u1 < nb ? u1 : nb, lane, meta[SPEC_IN] & 0xffffu, lbins);
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nb2; k += WPB * 64u)
            if (lbins[k])
                atomicAdd(&a.bins[k], (unsigned long long)(long long)lbins[k]);
        return;
    }
    if (meta[SPEC_SKIP] || meta[SPEC_NOLOCAL]) // block-uniform: before the barrier
        return;
    const uint64_t c0 = c * CH, c1 = c0 + CH < nb ? c0 + CH : nb;
    // the chunk's types (16-B loads of 8) are issued first, so that they
    // overlap the table fill and the look-back
    constexpr uint32_t R = CH * 256 / 512 > 0 ? CH * 256 / 512 : 1;
    const bool pre = (B & 7u) == 0 && c < nch;
    const uint64_t p0 = c0 * B, p1 = c1 * B < a.n ? c1 * B : a.n;
    const uint32_t m = pre ? (uint32_t)(p1 - p0) : 0u;
    u32x4 v[R];
#pragma unroll
    for (uint32_t r = 0; r < R; r++) {
        const uint32_t idx = (r * 64u + lane) * 8u;
        v[r] = idx + 8u <= m ? *(const u32x4 *)(a.spec_t16 + p0 + idx) : (u32x4){0, 0, 0, 0};
    }
    // and the previous chunk's last burst, where the look-back starts
    uint32_t pq0 = 0, pq1 = 0;
    const bool prev = c > 0 && c < nch;
    if (prev) {
        const uint64_t b0 = (c0 - 1) * B; // a full burst: only the batch's last burst is short
        spec_group_regs(a.spec_t16, b0, B, lane, pq0, pq1);
    }
    cnet_lut_fill(s_lut, threadIdx.x, WPB * 64);
    __syncthreads();
    if (c >= nch)
        return;
    if (c == nch - 1) { // the final node state (meta[-1]; the entering one is meta[SPEC_IN])
        uint32_t sf = 0;
        if (spec_lookback(a.spec_t16, a.n, B, c0, c1, lane, s_lut, sf)) {
            if (lane == 0)
                meta[-1] = sf;
        } else if (lane == 0) {
            spec_flag_full(meta);
        }
    }
    uint32_t s0 = meta[SPEC_IN] & 0xffffu;
    if (c > 0 && !spec_lookback(a.spec_t16, a.n, B, c0 - CH, c0, lane, s_lut, s0, true, pq0, pq1)) {
        if (lane == 0) {
            done[c] = 0;
            spec_flag_full(meta);
        }
        return;
    }
    uint32_t *st = s_pt[wv];
    if (pre) { // summary from the registers; stage in LDS only to replay
        unsigned long long em = 0;
#pragma unroll
        for (uint32_t r = 0; r < R; r++) {
            const uint32_t idx = (r * 64u + lane) * 8u;
            if (idx >= m)
                continue;
            uint32_t w[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
            if (idx + 8u > m) // the batch's last partial vector
                for (uint32_t q = 0; q < 4; q++) {
                    const uint32_t lo = idx + 2 * q < m ? a.spec_t16[p0 + idx + 2 * q] : 0u;
                    const uint32_t hi = idx + 2 * q + 1 < m ? a.spec_t16[p0 + idx + 2 * q + 1] : 0u;
                    w[q] = lo | (hi << 16);
                }
#pragma unroll
            for (uint32_t q = 0; q < 8; q++)
                if (idx + q < m)
                    em |= 1ull << (cnet_lut_x(s_lut, (w[q >> 1] >> (16 * (q & 1u))) & 0xffffu) & 63u);
        }
        if (!spec_chunk_quiet(spec_summary(em & ~(1ull << 63)), s0)) {
            spec_stage_chunk<CH>(a.spec_t16, a.n, B, c0, c1, lane, st, s_lut);
            spec_replay<CH>(a, B, c0, c1, s0, lane, st);
        }
    } else {
        const unsigned long long em = spec_stage_chunk<CH>(a.spec_t16, a.n, B, c0, c1, lane, st, s_lut);
        if (!spec_chunk_quiet(spec_summary(em), s0))
            spec_replay<CH>(a, B, c0, c1, s0, lane, st);
    }
    if (lane == 0)
        done[c] = 1;
}

// k_spec_local over the main kernel's tile words (k_cnet_defer wrote one per
// 64 frames; spec_canon).  The pass is latency-bound -- a few dependent loads
// per wave, next to no traffic -- and the types of a chunk are read only when
// its tiles cannot rule out a re-routed frame:
//   uniform batch  the wave's share of tiles: a canonical tile's frames all
//                  have spec_canon(T), so when that is E only the other tiles
//                  are looked at (frame by frame); otherwise every chunk goes
//                  through spec_uniform_range as without tile words;
//   chunk lists    (the fast kernel listed the chunks holding a frame off its
//                  low byte's common edge, and no group can move the state
//                  off a common edge): a listed chunk a block, a burst a wave,
//                  each burst's entering state from the look-back over the
//                  bursts before it, replayed side by side;
//   otherwise      per chunk: the entering state from the look-back, then
//                  quiet when every tile is canonical and the state agrees
//                  with its low byte's common edge (or has another low byte),
//                  else replayed by the wave that looked.
// Any grid is correct (chunks, bursts and tiles are strided over the blocks
// and waves): the host sizes it from the previous call's hint -- a wave per
// SPEC_LQ chunks, or a small grid when that call was a uniform batch.

// chunk c's tile words (lane < tiles covering it: <= 17 for B <= 256) and
// the burst before it (its groups, one per lane)
__device__ __forceinline__ void spec_chunk_pre(const KArgs &a, uint32_t B, uint64_t nch, uint64_t c, uint32_t lane,
                                               uint32_t &tw, uint32_t &pq0, uint32_t &pq1)
{
    tw = 1u;
    pq0 = pq1 = 0u;
    if (c < nch) {
        const uint64_t p0 = c * SPEC_CH * B, e1 = (c + 1) * SPEC_CH * B, p1 = e1 < a.n ? e1 : a.n;
        const uint64_t tl0 = p0 >> 6, ntl = ((p1 - 1) >> 6) - tl0 + 1;
        if (lane < ntl)
            tw = a.spec_tile[tl0 + lane];
        if (c > 0) // a full burst: only the batch's last burst is short
            spec_group_regs(a.spec_t16, (c * SPEC_CH - 1) * B, B, lane, pq0, pq1);
    }
}

// k_spec_local_t's body: bid / nblk stand for blockIdx.x / gridDim.x; LDS:
// s_bins (CNDP_BINS_MAX + 2 ints), s_lut (CNET_LUT_N), s_stw (this wave's
// CH * 256 staged types)
template <int CH>
__device__ __forceinline__ void spec_local_body(const KArgs &a, uint32_t B, uint64_t nb, uint64_t nch, uint32_t *meta,
                                                uint8_t *done, uint32_t bid, uint32_t nblk, int *s_bins,
                                                uint16_t *s_lut, uint32_t *s_stw)
{
    static_assert(CH == SPEC_CH, "spec_chunk_pre");
    static_assert(CH == 4, "a listed chunk is replayed a burst a wave by a 4-wave block");
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    // wave-uniform in SGPRs (the chunk index and all that derives from it)
    const uint64_t wid = (uint64_t)bid * 4 + __builtin_amdgcn_readfirstlane(wv), W = (uint64_t)nblk * 4;
    // the prologue's inputs in one round trip: every meta word it decides on,
    // the chunk list's count and this block's entry (read past the count and
    // ignored there) -- independent loads, waited for together
    const LutRegs lr = cnet_lut_load256(threadIdx.x);
    const uint32_t unif = meta[SPEC_UNIF], s_in = meta[SPEC_IN] & 0xffffu;
    const uint32_t m_stop = meta[SPEC_SKIP] | meta[SPEC_NOLOCAL], mx = meta[SPEC_MX], K = meta[0];
    const uint32_t sig = lane < SPEC_KMAX ? meta[1 + lane] : 0u;
    const uint32_t *const cwl = a.spec_cwl ? a.spec_cwl : meta;
    const uint32_t nl_w = cwl[0], lc_w = a.spec_cwl && bid < nch ? cwl[1 + bid] : 0u;
    SP_TS(0, __builtin_amdgcn_s_memrealtime());
    asm volatile("" ::"s"(unif), "s"(s_in), "s"(m_stop), "s"(mx), "s"(K), "v"(sig), "s"(nl_w), "s"(lc_w));
    SP_TS(1, __builtin_amdgcn_s_memrealtime());
    SP_TS(4, unif ? 1u : m_stop ? 2u : 5u);
    SP_TS(2, 0u);
    SP_TS(3, 0u);
    SP_TS(6, 0u);
    SP_TS(7, 0u);
    SP_TS(8, 0u);
    SP_TS(9, 0u);
    SP_TS(10, 0u);
    SP_TS(11, 0u);
    SP_TS(12, 0u);
    SP_TS(13, 0u);
    SP_TS(14, 0u);
    SP_TS(15, 0u);
    if (unif) { // block-uniform
        const uint32_t T = s_in, E = cnet_edge(T);
        const bool tcan = spec_canon(T & 0xffu) == E;
        const uint64_t n_tiles = ((uint64_t)a.n + 63u) >> 6, tpw = (n_tiles + W - 1) / W;
        const uint64_t t_lo = wid * tpw, t_hi = t_lo + tpw < n_tiles ? t_lo + tpw : n_tiles;
        // the tile words of the wave's first 64 tiles, before the barrier
        uint32_t tw = tcan && t_lo + lane < t_hi ? a.spec_tile[t_lo + lane] : 0u;
        int *lbins = s_bins;
        const uint32_t nb2 = a.bins ? a.n_bins + 2u : 0u;
        for (uint32_t k = threadIdx.x; k < nb2; k += 256u)
            lbins[k] = 0;
        __syncthreads();
        if (tcan) {
            for (uint64_t t0 = t_lo; t0 < t_hi; t0 += 64) {
                if (t0 != t_lo)
                    tw = t0 + lane < t_hi ? a.spec_tile[t0 + lane] : 1u;
                unsigned long long m = __ballot(t0 + lane < t_hi && tw == 0u);
                while (m) { // the few other tiles: the wave takes their frames one per lane
                    const uint32_t k = (uint32_t)__ffsll(m) - 1u;
                    m &= m - 1ull;
                    const uint64_t i = (t0 + k) * 64u + lane;
                    if (i < a.n) {
                        const uint32_t l = a.spec_t16[i];
                        const uint64_t b0 = i / B * B, bend = b0 + B < a.n ? b0 + B : a.n;
                        if (cnet_edge(l) != E && b0 + ((i - b0) & ~3ull) + 4u <= bend) // a full group
                            spec_fix(a, i, l, E, lbins);
                    }
                }
            }
        } else {
            for (uint64_t c = wid; c < nch; c += W) {
                const uint64_t u0 = c * CH, u1 = u0 + CH < nb ? u0 + CH : nb;
                spec_uniform_range<CH>(a, B, u0, u1, lane, T, lbins);
            }
        }
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nb2; k += 256u)
            if (lbins[k])
                atomicAdd(&a.bins[k], (unsigned long long)(long long)lbins[k]);
        return;
    }
    // CNDP_TUNE_SPEC_LISTS: when no group of the batch can take the node state
    // off its low byte's common edge (SPEC_MX, the entering state, the other
    // low bytes present), a frame can leave by another edge only inside a
    // chunk the fast kernel listed, so only those are looked at (grid-uniform)
    // (SPEC_UNIF implies no SPEC_SKIP; SPEC_NOLOCAL without it: nothing here)
    if (m_stop)
        return;
    bool lists = false;
    if (a.spec_cwl) {
        const uint32_t M = mx & 0xffu, e_in = cnet_edge(s_in), cn = spec_canon(s_in & 0xffu);
        lists = !(mx >> 8) && (cn == 0xFFu || cn == e_in) && !((M >> e_in) & 1u);
        if (lists) { // a state of another low byte whose edge is in M could take such a 4th type
            const bool clash = lane < K && lane < SPEC_KMAX && (sig >> 3) != 0x11u && (sig >> 3) != 0x41u &&
                               ((M >> (sig & 7u)) & 1u);
            lists = K <= SPEC_KMAX && __ballot(clash) == 0ull;
        }
    }
    // lists: block k < nl takes listed chunk k (one of its bursts a wave),
    // block nl walks the final state; the others leave before the table fill
    // (most of the grid, block-uniform)
    const uint32_t nl = lists ? nl_w : 0u;
    SP_TS(4, lists ? (bid <= nl ? 4u : 3u) : 5u);
    SP_TS(5, nl);
    if (lists && bid > nl)
        return;
    // without the lists: the first SPEC_LQ chunks' tile words and previous
    // bursts, all in flight during the table fill (one round trip for the
    // wave's chunks at the host's grid; a ring of SPEC_LQ at a smaller one)
    uint32_t tws[SPEC_LQ], q0s[SPEC_LQ], q1s[SPEC_LQ];
#pragma unroll
    for (int k = 0; k < SPEC_LQ; k++) {
        tws[k] = 1u;
        q0s[k] = q1s[k] = 0u;
        if (!lists)
            spec_chunk_pre(a, B, nch, wid + k * W, lane, tws[k], q0s[k], q1s[k]);
    }
    // lists: this wave's burst of the block's chunk -- its types and the groups
    // of the burst before -- in flight during the table fill
    constexpr uint32_t LR = CH * 256 / 512 > 0 ? CH * 256 / 512 : 1;
    const bool lvec = (B & 7u) == 0;
    u32x4 lv[LR];
    uint32_t lq0 = 0u, lq1 = 0u;
    auto burst_pre = [&](uint64_t lb) {
        lq0 = lq1 = 0u;
        if (lb < nb) {
            if (lvec)
                spec_chunk_load<CH>(a, B, lb, lb + 1, lane, lv);
            if (lb > 0)
                spec_group_regs(a.spec_t16, (lb - 1) * B, B, lane, lq0, lq1);
        }
    };
    if (lists && bid < nl)
        burst_pre((uint64_t)lc_w * CH + wv);
    cnet_lut_store256(s_lut, threadIdx.x, lr);
    const uint32_t nb2 = a.bins ? a.n_bins + 2u : 0u;
    for (uint32_t k = threadIdx.x; k < nb2; k += 256u)
        s_bins[k] = 0;
    __syncthreads();
    SP_TS(2, __builtin_amdgcn_s_memrealtime());
    if (lists) {
        // every burst of a listed chunk at once: burst b's entering state is the
        // walk from the last universal group before it (spec_lookback over the
        // bursts [b - 2 CH, b), the chunk's own earlier ones included: they hold
        // the same types the node walked), so the chunk's bursts replay side by
        // side.  A chunk with a burst whose state is not found there is left
        // whole to the full passes (done[c] = 0), none of it replayed here.
        for (uint64_t k = bid; k <= nl; k += nblk) {
            if (k == nl) { // the final node state (meta[-1]): the walk in the last chunk
                if (wv == 0) {
                    const uint64_t l0 = (nch - 1) * CH, l1 = l0 + CH < nb ? l0 + CH : nb;
                    uint32_t sf = 0;
                    if (spec_lookback(a.spec_t16, a.n, B, l0, l1, lane, s_lut, sf)) {
                        if (lane == 0)
                            meta[-1] = sf;
                    } else if (lane == 0) {
                        spec_flag_full(meta);
                    }
                }
                continue;
            }
            const uint64_t c = k == bid ? (uint64_t)lc_w : (uint64_t)a.spec_cwl[1 + k];
            const uint64_t lb = c * CH + wv;
            if (k != bid)
                burst_pre(lb);
            uint32_t s0 = s_in;
            bool ok = true;
            if (lb < nb && lb > 0)
                ok = spec_lookback(a.spec_t16, a.n, B, lb >= 2 * CH ? lb - 2 * CH : 0, lb, lane, s_lut, s0, true, lq0,
                                   lq1);
            SP_TS(6, __builtin_amdgcn_s_memrealtime());
            if (!__syncthreads_and(ok)) { // block-uniform
                if (threadIdx.x == 0) { // left to the full passes (done[] of the others is not read)
                    done[c] = 0;
                    spec_flag_full(meta);
                }
                continue;
            }
            if (threadIdx.x == 0)
                done[c] = 1;
            if (lb < nb) {
                if (lvec)
                    spec_chunk_types_v<CH>(a, B, lb, lb + 1, s0, lane, s_stw, s_lut, a.bins ? s_bins : nullptr, lv);
                else
                    spec_chunk_types<CH>(a, B, lb, lb + 1, s0, lane, s_stw, s_lut, a.bins ? s_bins : nullptr);
                __builtin_amdgcn_wave_barrier();
            }
        }
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nb2; k += 256u)
            if (s_bins[k])
                atomicAdd(&a.bins[k], (unsigned long long)(long long)s_bins[k]);
        SP_TS(3, __builtin_amdgcn_s_memrealtime());
        return;
    }
    for (uint64_t c = wid; c < nch; c += W) {
        const uint32_t ctw = tws[0], cq0 = q0s[0], cq1 = q1s[0];
#pragma unroll
        for (int k = 0; k + 1 < SPEC_LQ; k++) {
            tws[k] = tws[k + 1];
            q0s[k] = q0s[k + 1];
            q1s[k] = q1s[k + 1];
        }
        // the ring's next chunk, in flight meanwhile
        spec_chunk_pre(a, B, nch, c + SPEC_LQ * W, lane, tws[SPEC_LQ - 1], q0s[SPEC_LQ - 1], q1s[SPEC_LQ - 1]);
        const uint64_t c0 = c * CH, c1 = c0 + CH < nb ? c0 + CH : nb;
        if (c == nch - 1) { // the final node state (meta[-1]; the entering one is meta[SPEC_IN])
            uint32_t sf = 0;
            if (spec_lookback(a.spec_t16, a.n, B, c0, c1, lane, s_lut, sf)) {
                if (lane == 0)
                    meta[-1] = sf;
            } else if (lane == 0) {
                spec_flag_full(meta);
            }
        }
        const bool odd = __ballot(ctw == 0u) != 0ull; // a non-canonical tile
        uint32_t s0 = s_in;
        if (c > 0 && !spec_lookback(a.spec_t16, a.n, B, c0 - CH, c0, lane, s_lut, s0, true, cq0, cq1)) {
            if (lane == 0) {
                done[c] = 0;
                spec_flag_full(meta);
            }
            continue;
        }
        const uint32_t cn = spec_canon(s0 & 0xffu);
        if (odd || (cn != 0xFFu && cn != cnet_edge_l(s_lut, s0))) {
            // its types decide: read (one more round trip, this wave only) and
            // replayed here
            spec_chunk_types<CH>(a, B, c0, c1, s0, lane, s_stw, s_lut, a.bins ? s_bins : nullptr);
            __builtin_amdgcn_wave_barrier();
        }
        if (lane == 0)
            done[c] = 1;
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nb2; k += 256u)
        if (s_bins[k])
            atomicAdd(&a.bins[k], (unsigned long long)(long long)s_bins[k]);
    SP_TS(3, __builtin_amdgcn_s_memrealtime());
}

template <int CH>
__global__ __launch_bounds__(256) void k_spec_local_t(KArgs a, uint32_t B, uint64_t nb, uint64_t nch, uint32_t *meta,
                                                      uint8_t *done)
{
    __shared__ int s_bins[CNDP_BINS_MAX + 2]; // the uniform pass's / listed chunks' bin moves
    __shared__ __attribute__((aligned(16))) uint16_t s_lut[CNET_LUT_N];
    __shared__ __attribute__((aligned(16))) uint32_t s_st[4][CH * 256]; // a listed chunk's types
    spec_local_body<CH>(a, B, nb, nch, meta, done, blockIdx.x, gridDim.x, s_bins, s_lut, s_st[threadIdx.x >> 6]);
}

// CNDP_TUNE_SPEC_TYPES: the types of the tiles k_cnet_defer coded
// (SPEC_TW_CODES: IPv6 bit and UDP bit per frame, 16 B a tile) written out
// as spec_t16, when this batch's speculation passes read them after all.
// They do not when the batch resolved by its last universal group
// (meta[SPEC_SKIP]: nothing runs) or is uniform with an entering state on its
// low byte's common edge (k_spec_local_t's uniform pass reads the types of the
// other tiles only) -- the case the host codes for, a uniform batch before --
// and the kernel returns at once.
__global__ __launch_bounds__(256) void k_spec_expand(KArgs a, uint32_t n_tiles, const uint32_t *meta)
{
    if (meta[SPEC_SKIP])
        return;
    if (meta[SPEC_UNIF]) {
        const uint32_t T = meta[SPEC_IN] & 0xffffu;
        if (spec_canon(T & 0xffu) == cnet_edge(T))
            return;
    }
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t t = blockIdx.x * 4u + (threadIdx.x >> 6); t < n_tiles; t += gridDim.x * 4u) {
        if (a.spec_tile[t] != SPEC_TW_CODES) // wave-uniform
            continue;
        const u32x4 c = *(const u32x4 *)(a.spec_c2 + 16u * t);
        const uint32_t w6 = lane < 32u ? c.x : c.y, wu = lane < 32u ? c.z : c.w;
        const uint32_t b = lane & 31u, i = t * 64u + lane;
        if (i < a.n)
            a.spec_t16[i] = (uint16_t)((((w6 >> b) & 1u) ? 0x41u : 0x11u) | (((wu >> b) & 1u) ? 0x200u : 0x100u));
    }
}

// k_spec_fallback's work is handed out in ticket order, so it never assumes
// that its blocks are co-resident (other kernels, other contexts' queues and
// other graphs' launches may hold CUs).  bar[0] is the ticket counter; the
// tickets run tables [0, nT), scan rows [nT, nT + nA), the composition
// nT + nA, and the replay after it.  A phase's items wait only for the
// earlier phase's completion count (bar[1..3]), and every ticket of that
// phase was drawn before any ticket that waits on it -- by a block that is
// running -- so the waits always end, whatever the grid and whoever else is
// on the chip (the decoupled-lookback argument).  spec_classes zeroes
// bar[0..3] every call.  A wait is bounded all the same (wait_ticks of the
// 100 MHz s_memrealtime clock; 0 = fault injection, every wait expires): an
// expiry stores meta[SPEC_ERR] and the host-visible hint word [3], the
// waiting block leaves, and the host reports -EIO (cndp_gpu_classify
// at the context's next cnet call, cndp_gpu_mq_poll for the batch,
// CNDP_STAT_SPEC_ERR) -- never silent edges.
#define SPEC_ERR 134
#define SPEC_HINT_ERR 3 // spec_hint[3]: a k_spec_fallback wait expired (sticky until the host takes it)

// the block's completion of one work item: every wave's stores drained, then
// one release-add on the phase's counter
__device__ __forceinline__ void spec_item_done(uint32_t *ctr)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// wait until *ctr reaches want (lane 0 polls, relaxed loads + s_sleep, then
// acquires); false for the whole block when the wait expired (reported)
__device__ __forceinline__ bool spec_item_wait(const uint32_t *ctr, uint32_t want, uint32_t wait_ticks,
                                               uint32_t *meta, uint32_t *hint, uint32_t *s_flag)
{
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t ok = wait_ticks != 0u; // 0: fault injection, every wait expires
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (ok && __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)wait_ticks) {
                ok = 0u;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!ok) {
            __hip_atomic_store(&meta[SPEC_ERR], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (hint)
                __hip_atomic_store(&hint[SPEC_HINT_ERR], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        *s_flag = ok;
    }
    __syncthreads();
    return *s_flag != 0u;
}

// k_spec_fallback's body: bid stands for blockIdx.x; LDS: s_m (the scan's rows, which the
// tables / replay staging reuse), s_carry, s_lut, s_cls, s_tk (ticket / wait word).  Block 0
// also empties the fast kernel's chunk list for the next call.
template <int CH>
__device__ __forceinline__ void spec_fallback_body(const KArgs &a, uint32_t B, uint64_t nb, uint64_t nch,
                                                   uint32_t *meta, const uint8_t *class_id, uint32_t *T, uint32_t *P,
                                                   uint32_t *Bt, uint32_t *Sblk, uint32_t *S, const uint8_t *done,
                                                   uint32_t *bar, uint32_t kfast, uint32_t kmax, uint32_t gated,
                                                   uint32_t wait_ticks, uint32_t bid, uint32_t nblk, uint32_t *s_m,
                                                   uint32_t *s_carry, uint16_t *s_lut, uint8_t *s_cls, uint32_t *s_tk)
{
    static_assert(SPEC_BLK * (SPEC_KMAX + 1) >= 4 * CH * 256, "staging fits the scan rows");
    // what this launch decides on, in one round trip: SPEC_FULL / SPEC_SKIP
    // and (block 0) the chunk list's count with its first 256 entries (read
    // past the count and ignored there)
#if CD_STAMP
    if (bid == 0 && threadIdx.x == 0)
        sp_stamps[SP_STAMP_BLOCKS * 16] = __builtin_amdgcn_s_memrealtime();
#endif
    const uint32_t m_full = meta[SPEC_FULL], m_skip = meta[SPEC_SKIP];
    const bool clean = bid == 0 && a.spec_cwl;
    const uint32_t nl = clean ? a.spec_cwl[0] : 0u;
    const uint32_t e0 = clean && threadIdx.x < nch ? a.spec_cwl[1 + threadIdx.x] : 0u;
    if (clean) { // the fast kernel's chunk list and SPEC_MX, empty for the next call
        if (threadIdx.x < nl)
            a.spec_cflag[e0] = 0u;
        for (uint32_t k = threadIdx.x + 256u; k < nl; k += 256u)
            a.spec_cflag[a.spec_cwl[1 + k]] = 0u;
        __syncthreads();
        if (threadIdx.x == 0) {
            a.spec_cwl[0] = 0u;
            meta[SPEC_MX] = 0u;
        }
    }
    const bool full = !gated || m_full;
#if CD_STAMP
    if (bid == 0 && threadIdx.x == 0) {
        sp_stamps[SP_STAMP_BLOCKS * 16 + 1] = __builtin_amdgcn_s_memrealtime();
        sp_stamps[SP_STAMP_BLOCKS * 16 + 2] = (uint64_t)full << 32;
    }
#endif
    if (m_skip || !full) // grid-uniform
        return;
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t K = meta[0];
    uint32_t *st = s_m + wv * (CH * 256);
    cnet_lut_fill(s_lut, threadIdx.x, 256);
    spec_cls_stage(s_cls, class_id, threadIdx.x, 256);
    // the items: table / replay rows of 4 chunks (a chunk a wave), item i
    // takes rows i, i + nT, ...; scan rows of SPEC_BLK chunks likewise
    const uint64_t nrow = (nch + 3) / 4, nblk_s = (nch + SPEC_BLK - 1) / SPEC_BLK;
    const uint32_t nT = (uint32_t)(nrow < nblk ? nrow : nblk), nA = (uint32_t)(nblk_s < nblk ? nblk_s : nblk);
    const uint32_t t_a = nT, t_c = nT + nA, t_e = t_c + 1u, t_end = t_e + nT;
    const bool all = !gated || meta[SPEC_NOLOCAL];
    uint32_t *hint = a.spec_hint;
    for (;;) {
        __syncthreads(); // s_tk of the previous item read by every wave
        if (threadIdx.x == 0)
            *s_tk = __hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const uint32_t tk = *s_tk;
        if (tk >= t_end)
            return;
        if (tk < t_a) { // every chunk's map over the signature classes
            if (K <= SPEC_KMAX)
                for (uint64_t r = tk; r < nrow; r += nT) {
                    const uint64_t c = r * 4 + wv;
                    if (c < nch)
                        spec_ctable_chunk<CH>(a.spec_t16, a.n, B, nb, nch, c, K, meta, T, st, s_lut, s_cls);
                    __builtin_amdgcn_wave_barrier();
                }
            spec_item_done(&bar[1]);
        } else if (tk < t_c) { // the chunk maps composed, a block of SPEC_BLK chunks a row
            if (!spec_item_wait(&bar[1], nT, wait_ticks, meta, hint, s_tk))
                return;
            for (uint64_t vb = tk - t_a; vb < nblk_s; vb += nA) {
                if (K <= kfast)
                    spec_scan_a_body<SPEC_KFAST>(s_m, nch, K, T, P, Bt, vb);
                else if (K <= kmax)
                    spec_scan_a_body<SPEC_KMAX>(s_m, nch, K, T, P, Bt, vb);
                __syncthreads();
            }
            spec_item_done(&bar[2]);
        } else if (tk == t_c) { // the block totals into block start states and the final node state
            if (!spec_item_wait(&bar[2], nA, wait_ticks, meta, hint, s_tk))
                return;
            uint32_t *state = meta - 1;
            if (K <= kfast) {
                spec_scan_c_body<SPEC_KFAST, SPEC_BLK>(s_m, s_carry, nblk_s, K, class_id, Bt, Sblk, state);
            } else if (K <= kmax) {
                spec_scan_c_body<SPEC_KMAX, SPEC_BLK>(s_m, s_carry, nblk_s, K, class_id, Bt, Sblk, state);
            } else if (threadIdx.x == 0) {
                uint32_t s = meta[SPEC_IN] & 0xffffu;
                for (uint64_t b = 0; b < nb; b++) {
                    S[b] = s;
                    const uint64_t b0 = b * B;
                    const uint32_t cnt = (uint32_t)((uint64_t)a.n - b0 < B ? (uint64_t)a.n - b0 : B);
                    const uint32_t m = spec_burst_map(a.spec_t16, b0, cnt, spec_sig(s), false);
                    if (m != SPEC_UNCH)
                        s = m;
                }
                *state = s;
            }
            spec_item_done(&bar[3]);
        } else { // replay each chunk the local pass did not resolve, from its entering state
            if (!spec_item_wait(&bar[3], 1u, wait_ticks, meta, hint, s_tk))
                return;
            for (uint64_t r = tk - t_e; r < nrow; r += nT) {
                const uint64_t c = r * 4 + wv;
                if (c < nch && (all || !done[c]))
                    spec_cemit_chunk<CH>(a, B, nb, nch, c, meta, P, Sblk, S, T, kfast, kmax, st, s_lut);
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
}

// The general resolution, for what the local pass leaves (meta[SPEC_FULL]) or
// for everything (gated == 0, CNDP_TUNE_SPEC_SCAN forced): one launch of 4-wave
// blocks whose work items come in ticket order (above), three phases --
//   tables  every chunk's map over the signature classes and its summary,
//   scan    the chunk maps composed (blocks of SPEC_BLK chunks, then one item
//           composes the block totals into block start states and the final
//           node state; more than SPEC_KMAX classes: that item's thread 0
//           walks the bursts in order instead),
//   replay  each chunk the local pass did not resolve, from its entering state.
// With nothing left to resolve it returns at once.  Any grid gives the same
// results; the host launches a block per CU.
template <int CH>
__global__ __launch_bounds__(256) void k_spec_fallback(KArgs a, uint32_t B, uint64_t nb, uint64_t nch, uint32_t *meta,
                                                       const uint8_t *class_id, uint32_t *T, uint32_t *P,
                                                       uint32_t *Bt, uint32_t *Sblk, uint32_t *S, const uint8_t *done,
                                                       uint32_t *bar, uint32_t kfast, uint32_t kmax, uint32_t gated,
                                                       uint32_t wait_ticks)
{
    __shared__ __attribute__((aligned(16))) uint32_t s_m[SPEC_BLK * (SPEC_KMAX + 1)];
    __shared__ uint32_t s_carry[SPEC_KMAX];
    __shared__ __attribute__((aligned(16))) uint16_t s_lut[CNET_LUT_N];
    __shared__ __attribute__((aligned(16))) uint8_t s_cls[2048];
    __shared__ uint32_t s_tk;
    spec_fallback_body<CH>(a, B, nb, nch, meta, class_id, T, P, Bt, Sblk, S, done, bar, kfast, kmax, gated,
                           wait_ticks, blockIdx.x, gridDim.x, s_m, s_carry, s_lut, s_cls, &s_tk);
}

// ---------------------------------------------------------------------------
// bulk lookups (cne_fib_lookup_bulk / cne_fib6_lookup_bulk semantics)
// ---------------------------------------------------------------------------
// Completion of a lookup whose next hops go to mapped host memory: every
// block makes its stores visible to the host, the last one raises the flag
// the calling thread spins on (no stream synchronize: its wake-up cost as
// much as the lookups).  flag == nullptr: no completion.
struct LkDone {
    uint32_t *ticket, *flag;
    uint32_t seq;
};

__device__ __forceinline__ void lk_complete(const LkDone &d)
{
    if (!d.flag)
        return;
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = atomicAdd(d.ticket, 1u);
        if (t == gridDim.x - 1) {
            *d.ticket = 0u; // ready for the next call (stream order)
            __threadfence_system();
            __hip_atomic_store(d.flag, d.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <typename E>
__global__ __launch_bounds__(256) void k_lookup4(const E *__restrict__ t24, const E *__restrict__ t8,
                                                 const uint32_t *__restrict__ ips,
                                                 uint64_t *__restrict__ nh, uint32_t n, LkDone d)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) {
        const uint32_t ip = ips[i];
        uint64_t e = (uint64_t)t24[ip >> 8];
        if (e & 1u)
            e = (uint64_t)t8[(e >> 1) * 256u + (ip & 0xffu)];
        nh[i] = e >> 1;
    }
    lk_complete(d);
}

template <typename E>
__global__ __launch_bounds__(256) void k_lookup6(const E *__restrict__ t24, const E *__restrict__ t8,
                                                 const uint8_t *__restrict__ ips,
                                                 uint64_t *__restrict__ nh, uint32_t n, LkDone d)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) {
        const uint8_t *ip = ips + (uint64_t)i * 16u;
        uint64_t e = (uint64_t)t24[((uint32_t)ip[0] << 16) | ((uint32_t)ip[1] << 8) | ip[2]];
        uint32_t j = 3;
        while ((e & 1u) && j < 16)
            e = (uint64_t)t8[(e >> 1) * 256u + ip[j++]];
        nh[i] = e >> 1;
    }
    lk_complete(d);
}

// ---------------------------------------------------------------------------
// per-packet bin ids and the stable partition (per-edge streams)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bin_ids(uint32_t mode, const uint32_t *__restrict__ nh,
                                                 const uint8_t *__restrict__ edge,
                                                 const uint16_t *__restrict__ queue, uint32_t n,
                                                 uint32_t nb, uint16_t *__restrict__ out)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n)
        return;
    uint32_t b;
    if (mode == CNDP_MODE_HASH)
        b = bin_of<CNDP_MODE_HASH>(0, 0, queue[i], nb);
    else if (mode == CNDP_MODE_L3FWD)
        b = bin_of<CNDP_MODE_L3FWD>(nh[i], edge[i], 0, nb);
    else
        b = bin_of<CNDP_MODE_CNET>(nh[i], edge[i], 0, nb);
    out[i] = (uint16_t)b;
}

#define PART_TILE 1024u
#define PART_THREADS 256u

// pass 1: per-tile histogram, stored bin-major: hist[bin * tiles + tile]
__global__ __launch_bounds__(PART_THREADS) void k_part_hist(const uint16_t *__restrict__ bin_of,
                                                            uint32_t n, uint32_t nbt,
                                                            uint32_t tiles, uint32_t *hist)
{
    __shared__ uint32_t h[CNDP_BINS_MAX + 2];
    for (uint32_t k = threadIdx.x; k < nbt; k += PART_THREADS)
        h[k] = 0;
    __syncthreads();
    const uint32_t t0 = blockIdx.x * PART_TILE;
    for (uint32_t k = threadIdx.x; k < PART_TILE; k += PART_THREADS) {
        const uint32_t i = t0 + k;
        if (i < n)
            atomicAdd(&h[bin_of[i]], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nbt; k += PART_THREADS)
        hist[(uint64_t)k * tiles + blockIdx.x] = h[k];
}

// pass 2: exclusive scan of hist (bin-major) -> tile offsets; bin_start
__global__ __launch_bounds__(1024) void k_part_scan(uint32_t *hist, uint32_t total,
                                                    uint32_t tiles, uint32_t nbt,
                                                    uint32_t *bin_start)
{
    __shared__ uint32_t s_carry;
    __shared__ uint32_t s_wave[16];
    if (threadIdx.x == 0)
        s_carry = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    for (uint32_t base = 0; base < total; base += 1024u) {
        const uint32_t k = base + threadIdx.x;
        const uint32_t v = k < total ? hist[k] : 0u;
        // inclusive wave scan
        uint32_t x = v;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (lane >= d)
                x += y;
        }
        if (lane == 63)
            s_wave[wv] = x;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            for (int q = 0; q < 16; q++) {
                const uint32_t t = s_wave[q];
                s_wave[q] = acc;
                acc += t;
            }
        }
        __syncthreads();
        const uint32_t excl = s_carry + s_wave[wv] + x - v;
        if (k < total) {
            hist[k] = excl;
            if (k % tiles == 0)
                bin_start[k / tiles] = excl;
        }
        __syncthreads();
        if (threadIdx.x == 1023)
            s_carry = excl + v;
        __syncthreads();
    }
    if (threadIdx.x == 0)
        bin_start[nbt] = s_carry;
}

// pass 3: stable scatter.  Within a tile, waves go in order; within a wave
// the rank among same-bin lanes comes from ballots over the lane's peers.
__global__ __launch_bounds__(PART_THREADS) void k_part_scatter(const uint16_t *__restrict__ bin_of,
                                                               uint32_t n, uint32_t nbt,
                                                               uint32_t tiles,
                                                               const uint32_t *__restrict__ off,
                                                               uint32_t *__restrict__ order)
{
    __shared__ uint32_t cur[CNDP_BINS_MAX + 2];
    for (uint32_t k = threadIdx.x; k < nbt; k += PART_THREADS)
        cur[k] = off[(uint64_t)k * tiles + blockIdx.x];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t lt_mask = lane ? (~0ULL >> (64 - lane)) : 0ULL;
    const uint32_t t0 = blockIdx.x * PART_TILE;
    for (uint32_t chunk = 0; chunk < PART_TILE; chunk += PART_THREADS) {
        // process the 4 waves of this chunk strictly in order
        for (uint32_t turn = 0; turn < PART_THREADS / 64u; turn++) {
            if (wv == turn) {
                const uint32_t i = t0 + chunk + threadIdx.x;
                const bool valid = i < n;
                const uint32_t b = valid ? bin_of[i] : 0xFFFFFFFFu;
                uint64_t todo = __ballot(valid);
                uint32_t dst = 0;
                while (todo) {
                    const uint32_t leader = (uint32_t)__builtin_ctzll(todo);
                    const uint32_t lb = __shfl(b, leader, 64);
                    const uint64_t peers = __ballot(valid && b == lb);
                    const uint32_t cnt = (uint32_t)__builtin_popcountll(peers);
                    uint32_t basev = 0;
                    if (lane == leader)
                        basev = cur[lb];
                    basev = __shfl(basev, leader, 64);
                    if (b == lb && valid)
                        dst = basev + (uint32_t)__builtin_popcountll(peers & lt_mask);
                    if (lane == leader)
                        cur[lb] = basev + cnt;
                    todo &= ~peers;
                }
                if (valid)
                    order[dst] = i;
            }
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
#define CNDP_MAX_REGIONS 16
struct cndp_gpu_ctx {
    int dev;
    uint32_t *mq_iplen; // set by the node queue around its classify calls (KArgs::iplen)
    u32x4 *mq_win;      // ... and KArgs::win (zero-copy cnet: the windows the metadata comes from)
    uint8_t key[CNDP_RSS_KEY_LEN];
    uint32_t *d_ttab;     // 36 x 256
    uint16_t *d_reta;
    uint32_t reta_size;
    struct cne_fib *fib4;
    struct cne_fib6 *fib6;
    uint32_t *d_part;     // partition scratch
    size_t part_cap;
    int num_cu;
    int tune_nt;          // CNDP_TUNE_NT
    int tune_unroll;      // CNDP_TUNE_UNROLL
    int tune_bpc;         // CNDP_TUNE_BLOCKS_PER_CU
    int tune_tile;        // CNDP_TUNE_TILE
    int tune_dir16;       // CNDP_TUNE_DIR16
    int tune_cnet_tile;   // CNDP_TUNE_CNET_TILE
    int tune_lnt;         // CNDP_TUNE_LOAD_NT
    int tune_spec_scan;   // CNDP_TUNE_SPEC_SCAN
    int tune_cnet_fold;   // CNDP_TUNE_CNET_FOLD: 0 hint, 1 always, 2 never
    int tune_spec_grid;   // CNDP_TUNE_SPEC_GRID: 0 hint, 1 shrunk (2 blocks), 2 full
    int tune_spec_wait_us; // CNDP_TUNE_SPEC_WAIT: k_spec_fallback wait bound (us), -1 = fault injection
    int tune_host_window;  // CNDP_TUNE_HOST_WINDOW: classify_host moves 64-B windows of strided frames
    int tune_spec_lists;  // CNDP_TUNE_SPEC_LISTS: 1 chunk lists from the fast kernel (default), 0 off
    int sf_clean, wl_clean; // signature flags / worklist count known zero (no memset needed)
    uint32_t host_chunk;  // CNDP_TUNE_HOST_CHUNK: packets per pipelined host chunk
    int tune_rw_wb;       // CNDP_TUNE_RW_WB: fused rewrite write-back 0 auto, 1 frame, 2 tile
    uint32_t spec_burst;  // CNDP_TUNE_CNET_SPEC: ptype-node speculation burst (0 = off)
    int spec_reset;       // the node state (last_type) restarts at 0 on the next cnet call
    int mbuf_hash;        // CNDP_TUNE_MBUF_HASH: cndp_gpu_l3fwd_mbufs also writes m->hash
    // Stream order of the context's scratch (speculation state, worklist,
    // partition scratch): a call on another stream than the last user's
    // records ev_scratch on that stream and waits for it, so calls on
    // different streams never overlap on the shared scratch.
    hipEvent_t ev_scratch;
    hipStream_t scratch_stream;
    int scratch_used;
    int scratch_armed;    // ev_scratch already recorded (cndp_gpu_stream_release)
    // host regions registered through this context (zero-copy mbuf queues),
    // each holding `refs` references on the process-wide registration
    struct {
        uint8_t *host, *dev;
        uint64_t len;
        int refs;
    } reg[CNDP_MAX_REGIONS];
    int n_reg;
    uint32_t *sp_small;   // [0] last_type, [1..65] class meta, [66..129] signature flags
    uint32_t *cs_wl;      // k_cnet_stream worklist ([0] = count, then frame indices)
    uint64_t cs_wl_cap;
    uint8_t *sp_class;    // class id per signature (2048)
    uint32_t *sp_pt, *sp_nh, *sp_S, *sp_T, *sp_U; // sp_pt: the u16 types (speculation model)
    uint8_t *sp_done;     // per chunk: resolved by k_spec_local
    uint32_t *sp_cwl;     // chunks the fast kernel lists ([0] = count), CNDP_TUNE_SPEC_LISTS
    uint32_t *sp_cflag;   // per chunk: listed this call (cleared by k_spec_fallback)
    uint8_t *sp_tile;     // per 64-frame tile: the main kernel's canonical-tile word
    uint8_t *sp_c2;       // per 64-frame tile: 16 B of type codes (CNDP_TUNE_SPEC_TYPES)
    int tune_spec_types;  // CNDP_TUNE_SPEC_TYPES: 0 auto, 1 always the types, 2 always codes
    int tune_stream_bal;  // CNDP_TUNE_STREAM_BAL: 1 static, 2 LDS-balanced, 0 auto
    uint32_t *sp_hint, *sp_hint_d; // pinned, mapped: [0] bit length of the last worklist count, [1] last batch
                                   // uniform, [2] the last call ran the full speculation passes
    uint64_t sp_n_cap, sp_b_cap;
    // host-batch pipeline (cndp_gpu_classify_host): device mirrors, grown on demand
    hipStream_t hs[3];    // copy-in, classify, copy-out
    uint8_t *h_slab;      // device mirror of the host slab (same byte offsets)
    uint64_t h_slab_cap;
    uint64_t *h_off;
    uint64_t h_off_cap;
    uint8_t *h_out;       // nh | hash | queue | edge | bins
    uint64_t h_out_cap;
    // mbuf shim staging: pinned host windows / results and their device twins
    uint8_t *m_hwin, *m_dwin;
    uint32_t *m_hres, *m_dres; // nh[cap] | hash[cap]
    uint32_t m_cap;
    // ip4_rewrite node state (ip4_rewrite_priv.h:15-51)
    struct cndp_rw_nh rw_tbl[CNDP_RW_MAX_NH];
    uint16_t rw_next[CNDP_RW_MAX_PORTS];
    struct cndp_rw_nh *d_rw_tbl;
    int rw_dirty;
    int rw_local;         // the ctx-level rewrite API was used: do not follow the node table
    uint64_t rw_gen_seen; // generation of the process-global table (node.c) last copied
    uint32_t rw_parts;    // 16-B parts a rewrite touches: ceil(max(26, longest rewrite) / 16)
};

static const uint8_t ms_default_key[CNDP_RSS_KEY_LEN] = {
    0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
    0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
    0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};

// 32-bit key window starting at key bit s (MSB-first bit order)
static uint32_t key_window(const uint8_t *key, uint32_t s)
{
    uint64_t v = 0;
    for (uint32_t k = 0; k < 5; k++) {
        const uint32_t byte = s / 8 + k;
        v = (v << 8) | (byte < CNDP_RSS_KEY_LEN ? key[byte] : 0u);
    }
    return (uint32_t)(v >> (8 - (s % 8)));
}

// T[b][v] = XOR of the windows of the set bits of byte v at stream byte b
// (linearity of cne_softrss, cne_thash.h:150-163)
static void build_ttab(const uint8_t *key, uint32_t *tab)
{
    for (uint32_t b = 0; b < TAB_POS; b++) {
        uint32_t wbit[8];
        for (uint32_t k = 0; k < 8; k++)
            wbit[k] = key_window(key, 8 * b + k);
        for (uint32_t v = 0; v < 256; v++) {
            uint32_t h = 0;
            for (uint32_t k = 0; k < 8; k++)
                if (v & (0x80u >> k))
                    h ^= wbit[k];
            tab[b * 256 + v] = h;
        }
    }
    // N[q][u]: the 4 stream bits of nibble q (q = 2b high, 2b + 1 low nibble of
    // byte b), so T[b][v] = N[2b][v >> 4] ^ N[2b + 1][v & 15]
    for (uint32_t q = 0; q < 2 * TAB_POS; q++)
        for (uint32_t u = 0; u < 16; u++) {
            uint32_t h = 0;
            for (uint32_t k = 0; k < 4; k++)
                if (u & (0x8u >> k))
                    h ^= key_window(key, 4 * q + k);
            tab[TABN_OFF + q * 16 + u] = h;
        }
}

static int set_device(int dev)
{
    HIP_TRY(hipSetDevice(dev));
    return 0;
}

// order this call after the previous scratch user if it ran on another stream.
// The event is recorded on the previous user's stream only then, not after
// every call: a record is a system-scope release in the stream (the L2 is
// written back for the host to see), ~6 us in front of every cnet call's
// first kernel (a device-scope release measured the same).  Recorded late,
// it also covers whatever that stream ran since, which only orders more.
// So a stream given to a call that used the scratch must outlive the next
// call on another stream (cndp_gpu.h); the library's own streams (node
// queues, the host path's) clear the context's record when they go.
// A caller that destroys such a stream first hands it back with
// cndp_gpu_stream_release, which records the event on it there and then
// (scratch_armed): the next call waits on that record instead of touching the
// stream.
static int scratch_acquire(cndp_gpu_ctx_t *c, hipStream_t s)
{
    if (c->scratch_used && (c->scratch_armed || s != c->scratch_stream)) {
        if (!c->scratch_armed)
            HIP_TRY(hipEventRecord(c->ev_scratch, c->scratch_stream));
        HIP_TRY(hipStreamWaitEvent(s, c->ev_scratch, 0));
    }
    return 0;
}
static int scratch_release(cndp_gpu_ctx_t *c, hipStream_t s)
{
    c->scratch_stream = s;
    c->scratch_used = 1;
    c->scratch_armed = 0;
    return 0;
}

extern "C" int cndp_gpu_stream_release(cndp_gpu_ctx_t *c, void *stream)
{
    if (!c)
        return -EINVAL;
    if (!c->scratch_used || c->scratch_armed || c->scratch_stream != (hipStream_t)stream)
        return 0;
    int r;
    if ((r = set_device(c->dev)))
        return r;
    HIP_TRY(hipEventRecord(c->ev_scratch, c->scratch_stream));
    c->scratch_armed = 1;
    c->scratch_stream = nullptr;
    return 0;
}

extern "C" int cndp_gpu_init(int device, cndp_gpu_ctx_t **out)
{
    if (!out)
        return -EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return -ENODEV;
    if (device < 0)
        HIP_TRY(hipGetDevice(&device));
    if (device >= ndev)
        return -ENODEV;
    int r = set_device(device);
    if (r)
        return r;
    cndp_gpu_ctx_t *c = (cndp_gpu_ctx_t *)calloc(1, sizeof(*c));
    if (!c)
        return -ENOMEM;
    c->dev = device;
    c->tune_nt = 1;
    c->tune_unroll = 1;
    c->tune_bpc = 0; // auto: 2 for the streamed tile kernel, 4 otherwise
    c->tune_tile = 1;
    c->tune_dir16 = 1;
    c->tune_cnet_tile = 1;
    c->tune_lnt = 1;
    c->tune_spec_lists = 1;
    c->tune_spec_wait_us = 1000000; // 1 s: the waits end by construction, this only bounds a fault
    c->tune_host_window = 1;
    c->host_chunk = 1u << 20;
    c->spec_burst = 256;
    c->tune_rw_wb = 2;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess)
        c->num_cu = prop.multiProcessorCount;
    if (c->num_cu <= 0)
        c->num_cu = 256;
    if (hipMalloc((void **)&c->d_ttab, TAB_WORDS * 4) != hipSuccess ||
        hipMalloc((void **)&c->d_reta, CNDP_RETA_MAX * 2) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_scratch, hipEventDisableTiming) != hipSuccess) {
        cndp_gpu_fini(c);
        return -ENOMEM;
    }
    r = cndp_gpu_set_rss(c, nullptr, 0, nullptr, 0, 16);
    if (r) {
        cndp_gpu_fini(c);
        return r;
    }
    *out = c;
    return 0;
}

extern "C" void cndp_gpu_fini(cndp_gpu_ctx_t *c)
{
    if (!c)
        return;
    hipSetDevice(c->dev);
    hipDeviceSynchronize(); // nothing in flight may still use the scratch below
    while (c->n_reg > 0) // references this context holds on registered regions
        cndp_gpu_host_unregister(c, c->reg[0].host);
    if (c->ev_scratch)
        hipEventDestroy(c->ev_scratch);
    for (int k = 0; k < 3; k++)
        if (c->hs[k])
            hipStreamDestroy(c->hs[k]);
    if (c->h_slab)
        hipFree(c->h_slab);
    if (c->h_off)
        hipFree(c->h_off);
    if (c->h_out)
        hipFree(c->h_out);
    if (c->m_hwin)
        hipHostFree(c->m_hwin);
    if (c->m_hres)
        hipHostFree(c->m_hres);
    if (c->m_dwin)
        hipFree(c->m_dwin);
    if (c->m_dres)
        hipFree(c->m_dres);
    if (c->d_rw_tbl)
        hipFree(c->d_rw_tbl);
    void *sp[] = {c->sp_small, c->sp_class, c->sp_pt,   c->sp_nh,  c->sp_S,    c->sp_T,
                  c->sp_U,     c->sp_done,  c->sp_tile, c->sp_cwl, c->sp_cflag, c->sp_c2};
    for (void *q : sp)
        if (q)
            hipFree(q);
    if (c->sp_hint)
        hipHostFree(c->sp_hint);
    if (c->d_ttab)
        hipFree(c->d_ttab);
    if (c->d_reta)
        hipFree(c->d_reta);
    if (c->d_part)
        hipFree(c->d_part);
    if (c->cs_wl)
        hipFree(c->cs_wl);
    free(c);
}

extern "C" int cndp_gpu_device(const cndp_gpu_ctx_t *c) { return c ? c->dev : -EINVAL; }

extern "C" int cndp_gpu_set_rss(cndp_gpu_ctx_t *c, const uint8_t *key, uint32_t key_len,
                                const uint16_t *reta, uint32_t reta_size, uint32_t nb_queues)
{
    if (!c)
        return -EINVAL;
    if (key && key_len != CNDP_RSS_KEY_LEN)
        return -EINVAL;
    uint16_t rt[CNDP_RETA_MAX];
    if (reta) {
        if (reta_size == 0 || reta_size > CNDP_RETA_MAX || (reta_size & (reta_size - 1)))
            return -EINVAL;
        memcpy(rt, reta, reta_size * 2);
    } else {
        if (nb_queues == 0)
            return -EINVAL;
        reta_size = 128;
        for (uint32_t i = 0; i < reta_size; i++)
            rt[i] = (uint16_t)(i % nb_queues);
    }
    memcpy(c->key, key ? key : ms_default_key, CNDP_RSS_KEY_LEN);
    uint32_t *tab = (uint32_t *)malloc(TAB_WORDS * 4);
    if (!tab)
        return -ENOMEM;
    build_ttab(c->key, tab);
    int r = set_device(c->dev);
    if (!r && (hipMemcpy(c->d_ttab, tab, TAB_WORDS * 4, hipMemcpyHostToDevice) != hipSuccess ||
               hipMemcpy(c->d_reta, rt, reta_size * 2, hipMemcpyHostToDevice) != hipSuccess))
        r = -EIO;
    free(tab);
    if (!r)
        c->reta_size = reta_size;
    return r;
}

extern "C" int cndp_gpu_set_fib(cndp_gpu_ctx_t *c, struct cne_fib *f4, struct cne_fib6 *f6)
{
    if (!c)
        return -EINVAL;
    if (f4 && f4->t.nh_sz != 2)
        return -ENOTSUP;
    if (f6 && f6->t.nh_sz != 2)
        return -ENOTSUP;
    c->fib4 = f4;
    c->fib6 = f6;
    return 0;
}

// ---- table mirror -----------------------------------------------------------
extern "C" void cndp_tbl_dev_free(struct cndp_tbl *t)
{
    if (!t)
        return;
    // lookup staging exists once a lookup ran (even one whose mirror sync failed)
    for (uint32_t k = 0; k < CNDP_LK_SLOTS; k++) {
        struct cndp_tbl::cndp_lk_slot &sl = t->lk[k];
        if (sl.stream)
            hipStreamDestroy((hipStream_t)sl.stream);
        if (sl.host)
            hipHostFree(sl.host);
        if (sl.ticket)
            hipFree(sl.ticket);
        memset(&sl, 0, sizeof(sl));
    }
    if (t->paint_host)
        hipHostFree(t->paint_host);
    t->paint_host = nullptr;
    t->paint_cap = 0;
    if (t->dev_id < 0)
        return;
    int cur = 0;
    hipGetDevice(&cur);
    hipSetDevice(t->dev_id);
    if (t->dev_tbl24)
        hipFree(t->dev_tbl24);
    if (t->dev_tbl8)
        hipFree(t->dev_tbl8);
    if (t->dev_dir16)
        hipFree(t->dev_dir16);
    if (t->dev_pages)
        hipFree(t->dev_pages);
    if (t->lk_stream)
        hipStreamDestroy((hipStream_t)t->lk_stream);
    if (t->lk_dbuf)
        hipFree(t->lk_dbuf);
    t->lk_stream = nullptr;
    t->lk_dbuf = nullptr;
    for (uint32_t k = 0; k < t->n_old; k++)
        hipFree(t->dev_old[k]);
    free(t->dev_old);
    t->dev_old = nullptr;
    t->n_old = t->cap_old = 0;
    hipSetDevice(cur);
    t->dev_dir16 = t->dev_pages = nullptr;
    t->dev_cap_pages = 0;
    t->dev_tbl24 = t->dev_tbl8 = nullptr;
    t->dev_id = -1;
    t->dev_groups = 0;
}

// ---- /16 directory maintenance (host) ---------------------------------------
static int dir16_page_alloc(struct cndp_tbl *t)
{
    if (t->n_free)
        return (int)t->page_free[--t->n_free];
    if (t->page_hwm == t->cap_pages) {
        const uint32_t ncap = t->cap_pages ? t->cap_pages * 2 : 64;
        uint32_t *np = (uint32_t *)realloc(t->pages, (size_t)ncap * 256 * 4);
        uint32_t *nf = (uint32_t *)realloc(t->page_free, (size_t)ncap * 4);
        if (!np || !nf) {
            if (np)
                t->pages = np;
            if (nf)
                t->page_free = nf;
            return -ENOMEM;
        }
        t->pages = np;
        t->page_free = nf;
        t->cap_pages = ncap;
    }
    return (int)t->page_hwm++;
}

// refresh the directory entries of /16 blocks [k0, k1]
static int dir16_update(struct cndp_tbl *t, uint32_t k0, uint32_t k1)
{
    if (!t->dir16) {
        t->dir16 = (uint32_t *)calloc(65536, 4);
        t->page_of = (int32_t *)malloc(65536 * 4);
        if (!t->dir16 || !t->page_of)
            return -ENOMEM;
        for (uint32_t k = 0; k < 65536; k++)
            t->page_of[k] = -1;
        k0 = 0;
        k1 = 65535;
        t->dd_lo = t->dp_lo = ~0ULL;
        t->dd_hi = t->dp_hi = 0;
    }
    const uint32_t *t24 = (const uint32_t *)t->tbl24;
    for (uint32_t k = k0; k <= k1; k++) {
        const uint32_t *e = t24 + (size_t)k * 256;
        const uint32_t v = e[0];
        bool uni = !(v & 1u);
        for (uint32_t b = 1; uni && b < 256; b++)
            uni = e[b] == v;
        uint32_t nd;
        if (uni) {
            if (t->page_of[k] >= 0) {
                t->page_free[t->n_free++] = (uint32_t)t->page_of[k];
                t->page_of[k] = -1;
                t->n_pages_used--;
            }
            nd = v;
        } else {
            if (t->page_of[k] < 0) {
                const int pg = dir16_page_alloc(t);
                if (pg < 0)
                    return pg;
                t->page_of[k] = pg;
                t->n_pages_used++;
            }
            const uint64_t pe = (uint64_t)t->page_of[k] * 256;
            memcpy(t->pages + pe, e, 256 * 4);
            if (pe < t->dp_lo)
                t->dp_lo = pe;
            if (pe + 256 > t->dp_hi)
                t->dp_hi = pe + 256;
            nd = ((uint32_t)t->page_of[k] << 1) | 1u;
        }
        if (t->dir16[k] != nd || t->dd_hi == 0) {
            t->dir16[k] = nd;
            if (k < t->dd_lo)
                t->dd_lo = k;
            if ((uint64_t)k + 1 > t->dd_hi)
                t->dd_hi = (uint64_t)k + 1;
        }
    }
    return 0;
}

// Device buffers replaced by a sync (caller holds dev_lock): a launch that
// took an address under dev_lock (tbl_acquire) may still be on its way, so a
// replaced buffer is kept while any view of the table is held.  Once none is,
// every kept buffer goes: no thread can take a new view without dev_lock, and
// hipFree waits for the device, so the launches already enqueued have finished
// reading them.  Swept at every retire and at the start of every sync (each
// launch that reads the table syncs first), so a retired DUMMY tbl8 pool or
// /16 page array does not stay in HBM until the next growth.
static int tbl_dev_sweep(struct cndp_tbl *t)
{
    if (t->n_old && __atomic_load_n(&t->views, __ATOMIC_ACQUIRE) == 0) {
        const uint32_t n = t->n_old;
        t->n_old = 0;
        for (uint32_t k = 0; k < n; k++)
            HIP_TRY(hipFree(t->dev_old[k]));
    }
    return 0;
}

static int tbl_dev_retire(struct cndp_tbl *t, void *p)
{
    if (!p)
        return 0;
    if (t->n_old == t->cap_old) {
        const uint32_t cap = t->cap_old ? 2 * t->cap_old : 8;
        void **n = (void **)realloc(t->dev_old, cap * sizeof(void *));
        if (!n)
            return -ENOMEM;
        t->dev_old = n;
        t->cap_old = cap;
    }
    t->dev_old[t->n_old++] = p;
    return tbl_dev_sweep(t);
}

// the /16 directory after tbl24 entries [r[k].lo, r[k].hi) changed (the
// merged change log, or the one bounding range)
static int dir16_sync(struct cndp_tbl *t, hipStream_t s, const struct cndp_range *rg, uint32_t nr)
{
    for (uint32_t k = 0; k < nr || (!t->dir16 && k == 0); k++) {
        const uint64_t lo = k < nr ? rg[k].lo : 0, hi = k < nr ? rg[k].hi : 0;
        if (hi > lo || !t->dir16) {
            int r = dir16_update(t, (uint32_t)(lo >> 8), (uint32_t)((hi ? hi - 1 : 0) >> 8));
            if (r)
                return r;
        }
    }
    if (!t->dev_dir16) {
        HIP_TRY(hipMalloc(&t->dev_dir16, 65536 * 4));
        t->dd_lo = 0;
        t->dd_hi = 65536;
    }
    if (!t->dev_pages || t->dev_cap_pages < t->cap_pages) {
        int r = tbl_dev_retire(t, t->dev_pages);
        if (r)
            return r;
        t->dev_pages = nullptr;
        const uint32_t cap = t->cap_pages > 64 ? t->cap_pages : 64;
        HIP_TRY(hipMalloc(&t->dev_pages, (size_t)cap * 256 * 4));
        t->dev_cap_pages = cap;
        t->dp_lo = 0;
        t->dp_hi = (uint64_t)t->page_hwm * 256;
    }
    if (t->dd_hi > t->dd_lo)
        HIP_TRY(hipMemcpyAsync((uint32_t *)t->dev_dir16 + t->dd_lo, t->dir16 + t->dd_lo,
                               (t->dd_hi - t->dd_lo) * 4, hipMemcpyHostToDevice, s));
    if (t->dp_hi > t->dp_lo)
        HIP_TRY(hipMemcpyAsync((uint32_t *)t->dev_pages + t->dp_lo, t->pages + t->dp_lo,
                               (t->dp_hi - t->dp_lo) * 4, hipMemcpyHostToDevice, s));
    t->dd_lo = t->dp_lo = ~0ULL;
    t->dd_hi = t->dp_hi = 0;
    return 0;
}

// ---------------------------------------------------------------------------
// Device painter of the FIB mirror (SURVEY §8(f) row 4, dir24_8.c:249-453):
// the entry ranges a route change touched since the last sync, merged, are
// cut into maximal runs of one value -- filled on the device from a 24-B
// command -- and the short runs between them, copied from a payload.  The
// commands and payload sit in pinned mapped host memory the kernel reads, one
// block per command; the ranges are disjoint, so the blocks need no order.
// ---------------------------------------------------------------------------
struct TblCmd {
    uint64_t first;  // entry index in tbl24 / tbl8
    uint32_t count;  // entries
    uint32_t op;     // bit 0: tbl8 (else tbl24); bit 1: copy (arg = payload byte offset), else fill (arg = value)
    uint64_t arg;
};
#define PAINT_RUN_MIN 8u      // a run this long is filled, shorter ones are copied
#define PAINT_FILL_MAX 65536u // entries per fill command (large ranges spread over blocks)

template <typename T>
__global__ __launch_bounds__(256) void k_tbl_paint(const TblCmd *cmds, uint32_t n, const uint8_t *payload, T *t24,
                                                   T *t8)
{
    for (uint32_t c = blockIdx.x; c < n; c += gridDim.x) {
        const TblCmd k = cmds[c];
        T *const dst = ((k.op & 1u) ? t8 : t24) + k.first;
        if (k.op & 2u) {
            const T *const src = (const T *)(payload + k.arg);
            for (uint32_t i = threadIdx.x; i < k.count; i += blockDim.x)
                dst[i] = src[i];
        } else {
            const T v = (T)k.arg;
            for (uint32_t i = threadIdx.x; i < k.count; i += blockDim.x)
                dst[i] = v;
        }
    }
}

static inline uint64_t host_ent(const uint8_t *base, uint32_t nh_sz, uint64_t i)
{
    switch (nh_sz) {
    case 0:
        return base[i];
    case 1:
        return ((const uint16_t *)(const void *)base)[i];
    case 2:
        return ((const uint32_t *)(const void *)base)[i];
    default:
        return ((const uint64_t *)(const void *)base)[i];
    }
}

// merge a table's logged ranges (sorted, touching ones joined) in place;
// returns how many remain
static uint32_t paint_merge(struct cndp_range *r, uint32_t n)
{
    std::sort(r, r + n, [](const cndp_range &a, const cndp_range &b) { return a.lo < b.lo; });
    uint32_t m = 0;
    for (uint32_t k = 0; k < n; k++) {
        if (m && r[k].lo <= r[m - 1].hi) {
            if (r[k].hi > r[m - 1].hi)
                r[m - 1].hi = r[k].hi;
        } else {
            r[m++] = r[k];
        }
    }
    return m;
}

// the commands of one table's merged ranges, appended to cmds / payload
static void paint_plan(const struct cndp_tbl *t, uint32_t which, const uint8_t *img, const struct cndp_range *r,
                       uint32_t n, std::vector<TblCmd> &cmds, std::vector<uint8_t> &payload)
{
    const uint32_t esz = 1u << t->nh_sz;
    auto copy = [&](uint64_t lo, uint64_t hi) {
        if (hi <= lo)
            return;
        const uint64_t off = (payload.size() + 7u) & ~7ull;
        payload.resize(off + (hi - lo) * esz);
        memcpy(payload.data() + off, img + lo * esz, (hi - lo) * esz);
        // long copies spread over blocks like fills
        for (uint64_t f = lo; f < hi; f += PAINT_FILL_MAX) {
            const uint64_t c = hi - f < PAINT_FILL_MAX ? hi - f : PAINT_FILL_MAX;
            cmds.push_back(TblCmd{f, (uint32_t)c, which | 2u, off + (f - lo) * esz});
        }
    };
    for (uint32_t k = 0; k < n; k++) {
        uint64_t i = r[k].lo, cs = i; // cs: start of the pending copy segment
        while (i < r[k].hi) {
            const uint64_t v = host_ent(img, t->nh_sz, i);
            uint64_t j = i + 1;
            while (j < r[k].hi && host_ent(img, t->nh_sz, j) == v)
                j++;
            if (j - i >= PAINT_RUN_MIN) {
                copy(cs, i);
                for (uint64_t f = i; f < j; f += PAINT_FILL_MAX) {
                    const uint64_t c = j - f < PAINT_FILL_MAX ? j - f : PAINT_FILL_MAX;
                    cmds.push_back(TblCmd{f, (uint32_t)c, which, v});
                }
                cs = j;
            }
            i = j;
        }
        copy(cs, r[k].hi);
    }
}

// paint the logged changes of the tables whose mirror is not new (paint24 /
// paint8) on the device; returns 1 when it did, 0 when the bounding-range
// copy is cheaper, < 0 on error.  Caller holds dev_lock.
static int tbl_dev_paint(struct cndp_tbl *t, hipStream_t s, bool paint24, bool paint8)
{
    std::vector<TblCmd> cmds;
    std::vector<uint8_t> payload;
    const uint32_t esz = 1u << t->nh_sz;
    if (paint24)
        paint_plan(t, 0, t->tbl24, t->log24, paint_merge(t->log24, t->n_log24), cmds, payload);
    if (paint8)
        paint_plan(t, 1, t->tbl8, t->log8, paint_merge(t->log8, t->n_log8), cmds, payload);
    const uint64_t cmd_bytes = cmds.size() * sizeof(TblCmd), bytes = cmd_bytes + payload.size();
    const uint64_t span = ((paint24 && t->d24_hi > t->d24_lo) ? (t->d24_hi - t->d24_lo) * esz : 0) +
                          ((paint8 && t->d8_hi > t->d8_lo) ? (t->d8_hi - t->d8_lo) * esz : 0);
    if (cmds.empty() || bytes >= span)
        return 0;
    if (bytes > t->paint_cap) {
        if (t->paint_host)
            HIP_TRY(hipHostFree(t->paint_host));
        t->paint_host = nullptr;
        t->paint_cap = 0;
        const uint64_t cap = bytes > (1u << 16) ? bytes + bytes / 2 : (1u << 16);
        HIP_TRY(hipHostMalloc(&t->paint_host, cap, hipHostMallocMapped));
        t->paint_cap = cap;
    }
    uint8_t *h = (uint8_t *)t->paint_host;
    memcpy(h, cmds.data(), cmd_bytes);
    if (!payload.empty())
        memcpy(h + cmd_bytes, payload.data(), payload.size());
    void *hd = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&hd, t->paint_host, 0));
    const TblCmd *dc = (const TblCmd *)hd;
    const uint8_t *dp = (const uint8_t *)hd + cmd_bytes;
    const uint32_t n = (uint32_t)cmds.size(), g = n < 1024u ? n : 1024u;
    switch (t->nh_sz) {
    case 0:
        hipLaunchKernelGGL(k_tbl_paint<uint8_t>, dim3(g), dim3(256), 0, s, dc, n, dp, (uint8_t *)t->dev_tbl24,
                           (uint8_t *)t->dev_tbl8);
        break;
    case 1:
        hipLaunchKernelGGL(k_tbl_paint<uint16_t>, dim3(g), dim3(256), 0, s, dc, n, dp, (uint16_t *)t->dev_tbl24,
                           (uint16_t *)t->dev_tbl8);
        break;
    case 2:
        hipLaunchKernelGGL(k_tbl_paint<uint32_t>, dim3(g), dim3(256), 0, s, dc, n, dp, (uint32_t *)t->dev_tbl24,
                           (uint32_t *)t->dev_tbl8);
        break;
    default:
        hipLaunchKernelGGL(k_tbl_paint<uint64_t>, dim3(g), dim3(256), 0, s, dc, n, dp, (uint64_t *)t->dev_tbl24,
                           (uint64_t *)t->dev_tbl8);
        break;
    }
    HIP_TRY(hipGetLastError());
    t->sync_bytes += bytes;
    t->sync_cmds += n;
    return 1;
}

// caller holds t->dev_lock
static int tbl_dev_sync_locked(struct cndp_tbl *t, void *stream)
{
    if (!t || !t->tbl24)
        return -EINVAL;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        return -ENODEV;
    const size_t esz = (size_t)1 << t->nh_sz;
    const uint32_t groups = t->cap_groups + 1;
    if (t->dev_id >= 0 && t->dev_id != dev)
        return -EXDEV; // a FIB mirror lives on one device
    int rs = tbl_dev_sweep(t); // buffers retired while views were held
    if (rs)
        return rs;
    hipStream_t s = (hipStream_t)stream;
    // a mirror (or tbl8 pool) allocated by this sync is copied whole
    bool paint24 = t->dev_id >= 0, paint8 = t->dev_id >= 0 && t->dev_groups == groups;
    if (t->dev_id < 0) {
        HIP_TRY(hipMalloc(&t->dev_tbl24, (size_t)CNDP_TBL24_ENT * esz));
        HIP_TRY(hipMalloc(&t->dev_tbl8, (size_t)groups * CNDP_TBL8_GRP * esz));
        t->dev_id = dev;
        t->dev_groups = groups;
        t->d24_lo = 0;
        t->d24_hi = CNDP_TBL24_ENT;
        t->d8_lo = 0;
        t->d8_hi = (uint64_t)groups * CNDP_TBL8_GRP;
    } else if (t->dev_groups != groups) { // pool grew (DUMMY FIBs)
        void *n8 = nullptr;
        HIP_TRY(hipMalloc(&n8, (size_t)groups * CNDP_TBL8_GRP * esz));
        int r = tbl_dev_retire(t, t->dev_tbl8);
        if (r) {
            hipFree(n8);
            return r;
        }
        t->dev_tbl8 = n8;
        t->dev_groups = groups;
        t->d8_lo = 0;
        t->d8_hi = (uint64_t)groups * CNDP_TBL8_GRP;
    }
    // CNDP_FIB_PAINT=0: always the bounding-range copy (A/B of the painter)
    const char *pe = getenv("CNDP_FIB_PAINT");
    const bool paint_on = !pe || atoi(pe) != 0;
    paint24 = paint_on && paint24 && t->n_log24 <= CNDP_TBL_LOG && t->d24_hi > t->d24_lo;
    if (paint24) // merged once here: the painter and the /16 directory walk the same ranges
        t->n_log24 = paint_merge(t->log24, t->n_log24);
    paint8 = paint_on && paint8 && t->n_log8 <= CNDP_TBL_LOG && t->d8_hi > t->d8_lo;
    int painted = 0;
    if (paint24 || paint8) {
        painted = tbl_dev_paint(t, s, paint24, paint8);
        if (painted < 0)
            return painted;
    }
    if (t->d24_hi > t->d24_lo && !(painted && paint24)) {
        HIP_TRY(hipMemcpyAsync((uint8_t *)t->dev_tbl24 + t->d24_lo * esz, t->tbl24 + t->d24_lo * esz,
                               (t->d24_hi - t->d24_lo) * esz, hipMemcpyHostToDevice, s));
        t->sync_bytes += (t->d24_hi - t->d24_lo) * esz;
    }
    if (t->d8_hi > t->d8_lo && !(painted && paint8)) {
        HIP_TRY(hipMemcpyAsync((uint8_t *)t->dev_tbl8 + t->d8_lo * esz, t->tbl8 + t->d8_lo * esz,
                               (t->d8_hi - t->d8_lo) * esz, hipMemcpyHostToDevice, s));
        t->sync_bytes += (t->d8_hi - t->d8_lo) * esz;
    }
    // (the /16 directory exists for 4-B DIR-24-8 tables only: a trie table
    // without one is not dirty -- that test made every cnet call wait here)
    const bool has_dir16 = !t->is_trie && t->nh_sz == 2;
    const bool dirty = t->d24_hi > t->d24_lo || t->d8_hi > t->d8_lo || (has_dir16 && !t->dev_dir16);
    if (has_dir16) {
        // the directory scans only the changed tbl24 ranges when they were logged
        const struct cndp_range whole = {t->d24_lo, t->d24_hi};
        const bool logged = paint24 && t->dir16;
        int r = dir16_sync(t, s, logged ? t->log24 : &whole, logged ? t->n_log24 : 1u);
        if (r)
            return r;
    }
    // the host image (and the painter's staging) may change right after we
    // return: finish the copies and the paint
    if (dirty)
        HIP_TRY(hipStreamSynchronize(s));
    t->d24_lo = t->d8_lo = ~0ULL;
    t->d24_hi = t->d8_hi = 0;
    t->n_log24 = t->n_log8 = 0;
    return 0;
}

extern "C" int cndp_tbl_dev_sync(struct cndp_tbl *t, void *stream)
{
    if (!t || !t->tbl24)
        return -EINVAL;
    pthread_mutex_lock(&t->dev_lock);
    const int r = tbl_dev_sync_locked(t, stream);
    pthread_mutex_unlock(&t->dev_lock);
    return r;
}

static inline uint32_t blocks_for(uint64_t n, uint32_t threads)
{
    return (uint32_t)((n + threads - 1) / threads);
}

// the device tables one launch reads, taken under dev_lock right after the
// sync (tbl_view inside a locked section, or tbl_acquire, which also holds a
// view so the buffers outlive a replacement until tbl_release)
struct TblView {
    const void *t24, *t8;
    uint32_t nh_sz;
    const uint32_t *d16, *pages; // the /16 directory (4-B DIR-24-8 images), or null
};
static inline TblView tbl_view(const struct cndp_tbl *t)
{
    const bool dir = t->dev_dir16 && t->dev_pages;
    return TblView{t->dev_tbl24, t->dev_tbl8, t->nh_sz, dir ? (const uint32_t *)t->dev_dir16 : nullptr,
                   dir ? (const uint32_t *)t->dev_pages : nullptr};
}
static int tbl_acquire(struct cndp_tbl *t, hipStream_t s, TblView *v)
{
    pthread_mutex_lock(&t->dev_lock);
    const int r = tbl_dev_sync_locked(t, s);
    if (!r) {
        *v = tbl_view(t);
        __atomic_add_fetch(&t->views, 1u, __ATOMIC_RELAXED);
    }
    pthread_mutex_unlock(&t->dev_lock);
    return r;
}
static inline void tbl_release(struct cndp_tbl *t)
{
    __atomic_sub_fetch(&t->views, 1u, __ATOMIC_RELEASE);
}
static int tbl_lookup4_launch(TblView v, const uint32_t *ips, uint64_t *nh, uint32_t n, hipStream_t s,
                              LkDone d = LkDone{nullptr, nullptr, 0});
static int tbl_lookup6_launch(TblView v, const uint8_t *ips, uint64_t *nh, uint32_t n, hipStream_t s,
                              LkDone d = LkDone{nullptr, nullptr, 0});

extern "C" int cndp_tbl_lookup4_dev(struct cndp_tbl *t, const uint32_t *ips, uint64_t *nh,
                                    uint32_t n, void *stream)
{
    TblView v{};
    int r = tbl_acquire(t, (hipStream_t)stream, &v);
    if (r)
        return r;
    r = tbl_lookup4_launch(v, ips, nh, n, (hipStream_t)stream);
    tbl_release(t);
    return r;
}

extern "C" int cndp_tbl_lookup6_dev(struct cndp_tbl *t, const uint8_t *ips, uint64_t *nh, uint32_t n,
                                    void *stream)
{
    TblView v{};
    int r = tbl_acquire(t, (hipStream_t)stream, &v);
    if (r)
        return r;
    r = tbl_lookup6_launch(v, ips, nh, n, (hipStream_t)stream);
    tbl_release(t);
    return r;
}

static int tbl_lookup4_launch(TblView v, const uint32_t *ips, uint64_t *nh, uint32_t n, hipStream_t s,
                              LkDone d)
{
    if (n == 0)
        return 0;
    const uint32_t g = blocks_for(n, 256);
    switch (v.nh_sz) {
    case 0:
        hipLaunchKernelGGL(k_lookup4<uint8_t>, dim3(g), dim3(256), 0, s, (const uint8_t *)v.t24,
                           (const uint8_t *)v.t8, ips, nh, n, d);
        break;
    case 1:
        hipLaunchKernelGGL(k_lookup4<uint16_t>, dim3(g), dim3(256), 0, s,
                           (const uint16_t *)v.t24, (const uint16_t *)v.t8, ips, nh, n, d);
        break;
    case 2:
        hipLaunchKernelGGL(k_lookup4<uint32_t>, dim3(g), dim3(256), 0, s,
                           (const uint32_t *)v.t24, (const uint32_t *)v.t8, ips, nh, n, d);
        break;
    default:
        hipLaunchKernelGGL(k_lookup4<uint64_t>, dim3(g), dim3(256), 0, s,
                           (const uint64_t *)v.t24, (const uint64_t *)v.t8, ips, nh, n, d);
        break;
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

static int tbl_lookup6_launch(TblView v, const uint8_t *ips, uint64_t *nh, uint32_t n, hipStream_t s,
                              LkDone d)
{
    if (n == 0)
        return 0;
    const uint32_t g = blocks_for(n, 256);
    switch (v.nh_sz) {
    case 1:
        hipLaunchKernelGGL(k_lookup6<uint16_t>, dim3(g), dim3(256), 0, s,
                           (const uint16_t *)v.t24, (const uint16_t *)v.t8, ips, nh, n, d);
        break;
    case 2:
        hipLaunchKernelGGL(k_lookup6<uint32_t>, dim3(g), dim3(256), 0, s,
                           (const uint32_t *)v.t24, (const uint32_t *)v.t8, ips, nh, n, d);
        break;
    default:
        hipLaunchKernelGGL(k_lookup6<uint64_t>, dim3(g), dim3(256), 0, s,
                           (const uint64_t *)v.t24, (const uint64_t *)v.t8, ips, nh, n, d);
        break;
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

// Host-array lookups (cne_fib_lookup_bulk / cne_fib6_lookup_bulk).  The
// reference lookup reads the table in place and cannot fail
// (cne_fib.c:111-116); callers like examples/cndpfwd/l3-fwd.c:85 call it per
// burst from every forwarding thread on one FIB and ignore the return code.
// So: the mirror's own device (not the caller's current one), and on any
// failure every next hop is set to the FIB default before the negative
// errno is returned.  A small call (the per-burst case) takes one of the
// table's staging slots for itself -- its own stream, pinned and mapped
// staging that the kernel reads and writes in place, and a completion flag
// the kernel raises there, which the caller spins on (no stream
// synchronize: its wake-up cost as much as the lookups) -- and holds the
// table lock only to sync the mirror and take the table addresses, so calls
// from different threads overlap.  Larger calls move keys and next hops by
// DMA through device scratch, under the table lock.
#define LK_MAPPED_MAX 16384u   // lookups per round through mapped staging
#define LK_DMA_CHUNK (1u << 20) // lookups per round through device scratch
#define LK_FLAG_OFF ((size_t)LK_MAPPED_MAX * (16 + 8)) // the completion flag, after the staging
#define LK_WAIT_S 10             // a mapped lookup not done by then is an error

static uint64_t now_ns();

// spin on the mapped lookup's completion flag; on a timeout, the stream's
// own status says why
static int lk_wait(const uint32_t *flag, uint32_t seq, hipStream_t s)
{
    const uint64_t t0 = now_ns();
    for (uint32_t spin = 0; __atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq; spin++) {
        if ((spin & 255u) == 255u && now_ns() - t0 > LK_WAIT_S * 1000000000ull) {
            HIP_TRY(hipStreamSynchronize(s));
            return __atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq ? 0 : -EIO;
        }
        __builtin_ia32_pause();
    }
    return 0;
}

// a free staging slot, the calling thread's usual one first
static struct cndp_tbl::cndp_lk_slot *lk_slot_take(struct cndp_tbl *t)
{
    static std::atomic<uint32_t> next_home{0};
    static thread_local uint32_t home = next_home.fetch_add(1u) % CNDP_LK_SLOTS;
    for (uint32_t spin = 0;; spin++) {
        for (uint32_t k = 0; k < CNDP_LK_SLOTS; k++) {
            struct cndp_tbl::cndp_lk_slot *sl = &t->lk[(home + k) % CNDP_LK_SLOTS];
            if (!__atomic_load_n(&sl->busy, __ATOMIC_RELAXED) && !__atomic_exchange_n(&sl->busy, 1, __ATOMIC_ACQUIRE))
                return sl;
        }
        if ((spin & 63u) == 63u)
            sched_yield();
        else
            __builtin_ia32_pause();
    }
}

static void lk_slot_give(struct cndp_tbl::cndp_lk_slot *sl)
{
    __atomic_store_n(&sl->busy, 0, __ATOMIC_RELEASE);
}

// the slot's stream, staging and ticket on the current device (first use)
static int lk_slot_init(struct cndp_tbl::cndp_lk_slot *sl)
{
    if (!sl->stream) {
        hipStream_t st = nullptr;
        HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        sl->stream = st;
    }
    if (!sl->host) {
        void *h = nullptr, *d = nullptr;
        HIP_TRY(hipHostMalloc(&h, LK_FLAG_OFF + 64, hipHostMallocMapped));
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
            hipHostFree(h);
            return -EIO;
        }
        *(volatile uint32_t *)((uint8_t *)h + LK_FLAG_OFF) = 0u;
        sl->host = (uint8_t *)h;
        sl->hdev = (uint8_t *)d;
        sl->seq = 0;
    }
    if (!sl->ticket) {
        HIP_TRY(hipMalloc((void **)&sl->ticket, sizeof(uint32_t)));
        HIP_TRY(hipMemsetAsync(sl->ticket, 0, sizeof(uint32_t), (hipStream_t)sl->stream));
    }
    return 0;
}

static int lookup_mapped(struct cndp_tbl *t, const uint8_t *ips, uint32_t key_sz, uint64_t *nh, uint32_t n, int v6)
{
    struct cndp_tbl::cndp_lk_slot *sl = lk_slot_take(t);
    int r = lk_slot_init(sl);
    hipStream_t s = (hipStream_t)sl->stream;
    TblView v{};
    bool held = false;
    if (!r) // waits for its copies when the image was dirty
        held = (r = tbl_acquire(t, s, &v)) == 0;
    if (!r) {
        uint8_t *hk = sl->host, *hn = sl->host + (size_t)LK_MAPPED_MAX * key_sz;
        memcpy(hk, ips, (size_t)n * key_sz);
        const uint8_t *dk = sl->hdev;
        uint64_t *dn = (uint64_t *)(sl->hdev + (size_t)LK_MAPPED_MAX * key_sz);
        sl->seq = sl->seq + 1u ? sl->seq + 1u : 1u; // never the flag's initial 0
        const LkDone d{sl->ticket, (uint32_t *)(sl->hdev + LK_FLAG_OFF), sl->seq};
        r = v6 ? tbl_lookup6_launch(v, dk, dn, n, s, d) : tbl_lookup4_launch(v, (const uint32_t *)dk, dn, n, s, d);
        tbl_release(t);
        held = false;
        if (!r)
            r = lk_wait((const uint32_t *)(sl->host + LK_FLAG_OFF), sl->seq, s);
        if (!r)
            memcpy(nh, hn, (size_t)n * 8);
    }
    if (held)
        tbl_release(t);
    lk_slot_give(sl);
    return r;
}

// caller holds t->dev_lock
static int lookup_dma_locked(struct cndp_tbl *t, const uint8_t *ips, uint32_t key_sz, uint64_t *nh, uint32_t n,
                             int v6)
{
    if (!t->lk_stream) {
        hipStream_t st = nullptr;
        HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        t->lk_stream = st;
    }
    hipStream_t s = (hipStream_t)t->lk_stream;
    int r = tbl_dev_sync_locked(t, s);
    if (r)
        return r;
    const TblView v = tbl_view(t);
    if (!t->lk_dbuf)
        HIP_TRY(hipMalloc((void **)&t->lk_dbuf, (size_t)LK_DMA_CHUNK * (16 + 8)));
    for (uint32_t i0 = 0; i0 < n; i0 += LK_DMA_CHUNK) {
        const uint32_t c = n - i0 < LK_DMA_CHUNK ? n - i0 : LK_DMA_CHUNK;
        uint8_t *dk = t->lk_dbuf;
        uint64_t *dn = (uint64_t *)(t->lk_dbuf + (size_t)LK_DMA_CHUNK * key_sz);
        HIP_TRY(hipMemcpyAsync(dk, ips + (size_t)i0 * key_sz, (size_t)c * key_sz, hipMemcpyHostToDevice, s));
        r = v6 ? tbl_lookup6_launch(v, dk, dn, c, s) : tbl_lookup4_launch(v, (const uint32_t *)dk, dn, c, s);
        if (r)
            return r;
        HIP_TRY(hipMemcpyAsync(nh + i0, dn, (size_t)c * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    return 0;
}

static int lookup_host_common(struct cndp_tbl *t, const void *ips, size_t key_sz, uint64_t *nh, uint32_t n,
                              int v6)
{
    int r = 0, ndev = 0, cur = -1;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        r = -ENODEV;
    } else if (n) {
        hipGetDevice(&cur);
        pthread_mutex_lock(&t->dev_lock);
        const int dev = t->dev_id >= 0 ? t->dev_id : (cur >= 0 ? cur : 0);
        if (dev != cur && hipSetDevice(dev) != hipSuccess)
            r = -ENODEV;
        if (!r && n > LK_MAPPED_MAX)
            r = lookup_dma_locked(t, (const uint8_t *)ips, (uint32_t)key_sz, nh, n, v6);
        pthread_mutex_unlock(&t->dev_lock);
        if (!r && n <= LK_MAPPED_MAX)
            r = lookup_mapped(t, (const uint8_t *)ips, (uint32_t)key_sz, nh, n, v6);
        if (cur >= 0 && dev != cur)
            hipSetDevice(cur);
    }
    if (r) // the caller may ignore the code: leave it the default next hop
        for (uint32_t i = 0; i < n; i++)
            nh[i] = t->def_nh;
    return r;
}

extern "C" int cndp_tbl_lookup4_host(struct cndp_tbl *t, const uint32_t *ips, uint64_t *nh, uint32_t n)
{
    return lookup_host_common(t, ips, 4, nh, n, 0);
}

extern "C" int cndp_tbl_lookup6_host(struct cndp_tbl *t, const uint8_t *ips, uint64_t *nh, uint32_t n)
{
    return lookup_host_common(t, ips, 16, nh, n, 1);
}

// ---- classify ---------------------------------------------------------------
static int validate_batch(const cndp_gpu_ctx_t *c, const struct cndp_batch *b)
{
    if (!c || !b)
        return -EINVAL;
    if (b->mode != CNDP_MODE_L3FWD && b->mode != CNDP_MODE_CNET && b->mode != CNDP_MODE_HASH)
        return -EINVAL;
    if (b->n && !b->slab)
        return -EINVAL;
    if (b->bins && b->n_bins > CNDP_BINS_MAX)
        return -EINVAL;
    if (b->mode != CNDP_MODE_HASH && !c->fib4)
        return -EINVAL;
    if (b->mode == CNDP_MODE_CNET && !c->fib6)
        return -EINVAL;
    return 0;
}

// scratch of the ptype-speculation pass, grown on demand
static int spec_scratch(cndp_gpu_ctx_t *c, uint64_t n, uint64_t nb)
{
    if (!c->sp_small) {
        HIP_TRY(hipMalloc((void **)&c->sp_small, 1024 * 4));
        HIP_TRY(hipMemset(c->sp_small, 0, 1024 * 4));
        HIP_TRY(hipMalloc((void **)&c->sp_class, 2048));
        HIP_TRY(hipHostMalloc((void **)&c->sp_hint, 64, hipHostMallocMapped));
        memset(c->sp_hint, 0, 64);
        HIP_TRY(hipHostGetDevicePointer((void **)&c->sp_hint_d, c->sp_hint, 0));
    }
    if (n > c->sp_n_cap) {
        if (c->sp_pt)
            HIP_TRY(hipFree(c->sp_pt));
        if (c->sp_nh)
            HIP_TRY(hipFree(c->sp_nh));
        if (c->sp_tile)
            HIP_TRY(hipFree(c->sp_tile));
        if (c->sp_c2)
            HIP_TRY(hipFree(c->sp_c2));
        c->sp_pt = c->sp_nh = nullptr;
        c->sp_tile = c->sp_c2 = nullptr;
        c->sp_n_cap = 0;
        const uint64_t cap = n + (n >> 3) + 1024;
        HIP_TRY(hipMalloc((void **)&c->sp_pt, cap * 2));
        HIP_TRY(hipMalloc((void **)&c->sp_nh, cap * 4));
        HIP_TRY(hipMalloc((void **)&c->sp_tile, cap / 64 + 1));
        HIP_TRY(hipMalloc((void **)&c->sp_c2, (cap / 64 + 1) * 16));
        c->sp_n_cap = cap;
    }
    if (nb > c->sp_b_cap) {
        if (c->sp_S)
            HIP_TRY(hipFree(c->sp_S));
        if (c->sp_T)
            HIP_TRY(hipFree(c->sp_T));
        if (c->sp_U)
            HIP_TRY(hipFree(c->sp_U));
        if (c->sp_done)
            HIP_TRY(hipFree(c->sp_done));
        if (c->sp_cwl)
            HIP_TRY(hipFree(c->sp_cwl));
        if (c->sp_cflag)
            HIP_TRY(hipFree(c->sp_cflag));
        c->sp_S = c->sp_T = c->sp_U = c->sp_cwl = c->sp_cflag = nullptr;
        c->sp_done = nullptr;
        c->sp_b_cap = 0;
        const uint64_t cap = nb + (nb >> 3) + 64;
        HIP_TRY(hipMalloc((void **)&c->sp_S, cap * 4));
        HIP_TRY(hipMalloc((void **)&c->sp_done, cap));
        // the chunk list and its flags start empty; k_spec_fallback empties them again
        HIP_TRY(hipMalloc((void **)&c->sp_cwl, (cap + 1) * 4));
        HIP_TRY(hipMemset(c->sp_cwl, 0, (cap + 1) * 4));
        HIP_TRY(hipMalloc((void **)&c->sp_cflag, cap * 4));
        HIP_TRY(hipMemset(c->sp_cflag, 0, cap * 4));
        const uint64_t ptrs[2] = {(uint64_t)(uintptr_t)c->sp_cwl, (uint64_t)(uintptr_t)c->sp_cflag};
        HIP_TRY(hipMemcpy(c->sp_small + 1 + SPEC_PTRS, ptrs, sizeof(ptrs), hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc((void **)&c->sp_T, cap * SPEC_KMAX * 4));
        // inclusive burst prefixes + block totals + block start states
        HIP_TRY(hipMalloc((void **)&c->sp_U, (cap * SPEC_KMAX + (cap / SPEC_BLK + 2) * (SPEC_KMAX + 1)) * 4));
        c->sp_b_cap = cap;
    }
    return 0;
}

static int classify_cnet(cndp_gpu_ctx_t *c, const struct cndp_batch *b, KArgs &a, hipStream_t s);
static int classify_l3(cndp_gpu_ctx_t *c, const struct cndp_batch *b, KArgs &a, hipStream_t s, uint16_t *rw_tx,
                       bool *fused);

static int classify_launch(cndp_gpu_ctx_t *c, const struct cndp_batch *b, void *stream, uint16_t *rw_tx,
                           bool *fused, const TblView *v4, const TblView *v6);

// rw_tx != nullptr asks for ip4_rewrite fused into the wave-tile kernel
// (256-packet bursts); *fused says whether that kernel ran
static int classify_impl(cndp_gpu_ctx_t *c, const struct cndp_batch *b, void *stream, uint16_t *rw_tx,
                         bool *fused)
{
    int r = validate_batch(c, b);
    if (r)
        return r;
    r = set_device(c->dev);
    if (r)
        return r;
    // the tables this call's launches read, held until they are enqueued
    struct cndp_tbl *t4 = b->mode != CNDP_MODE_HASH ? &c->fib4->t : nullptr;
    struct cndp_tbl *t6 = b->mode == CNDP_MODE_CNET ? &c->fib6->t : nullptr;
    TblView v4{}, v6{};
    if (t4 && (r = tbl_acquire(t4, (hipStream_t)stream, &v4)))
        return r;
    if (t6 && (r = tbl_acquire(t6, (hipStream_t)stream, &v6))) {
        tbl_release(t4);
        return r;
    }
    r = b->n ? classify_launch(c, b, stream, rw_tx, fused, t4 ? &v4 : nullptr, t6 ? &v6 : nullptr) : 0;
    if (t4)
        tbl_release(t4);
    if (t6)
        tbl_release(t6);
    return r;
}

static int classify_launch(cndp_gpu_ctx_t *c, const struct cndp_batch *b, void *stream, uint16_t *rw_tx,
                           bool *fused, const TblView *v4, const TblView *v6)
{
    int r;
    KArgs a;
    memset(&a, 0, sizeof(a));
    a.slab = (const uint8_t *)b->slab;
    a.slab_len = b->slab_len;
    a.stride = b->stride;
    a.offsets = b->offsets;
    a.data_off = b->data_off;
    a.n = b->n;
    a.buf_len = b->buf_len;
    a.reta_mask = c->reta_size - 1;
    if (v4) {
        a.tbl24 = (const uint32_t *)v4->t24;
        a.tbl8 = (const uint32_t *)v4->t8;
        if (c->tune_dir16 && v4->d16) {
            a.dir16 = v4->d16;
            a.pages = v4->pages;
        }
    }
    if (v6) {
        a.tbl24_6 = (const uint32_t *)v6->t24;
        a.tbl8_6 = (const uint32_t *)v6->t8;
    }
    a.ttab = c->d_ttab;
    a.reta = c->d_reta;
    a.nh = b->nh;
    a.hash = b->hash;
    a.queue = b->queue;
    a.edge = b->edge;
    a.bins = (unsigned long long *)b->bins;
    a.n_bins = b->n_bins;
    a.ptype = b->ptype;
    a.rxmeta = b->mode == CNDP_MODE_CNET ? b->rxmeta : nullptr;
    a.iplen = b->mode == CNDP_MODE_CNET && b->rxmeta ? c->mq_iplen : nullptr;
    a.win = b->mode == CNDP_MODE_CNET && b->rxmeta ? c->mq_win : nullptr;
    hipStream_t s = (hipStream_t)stream;
    if (b->mode == CNDP_MODE_CNET) {
        if ((r = scratch_acquire(c, s)))
            return r;
        r = classify_cnet(c, b, a, s);
        const int r2 = scratch_release(c, s);
        return r ? r : r2;
    }
    return classify_l3(c, b, a, s, rw_tx, fused);
}

static int classify_cnet(cndp_gpu_ctx_t *c, const struct cndp_batch *b, KArgs &a, hipStream_t s)
{
    int r;
    {
        uint32_t g = blocks_for(b->n, CNET_THREADS);
        const uint32_t cap = (uint32_t)c->num_cu * 2u;
        if (g > cap)
            g = cap;
        const uint32_t B = c->spec_burst;
        if (B && (r = spec_scratch(c, b->n, ((uint64_t)b->n + B - 1) / B)))
            return r;
        if (c->spec_reset && c->sp_small) { // CNDP_TUNE_CNET_SPEC was set: a new graph
            HIP_TRY(hipMemsetAsync(c->sp_small, 0, 4, s));
            c->spec_reset = 0;
        }
        if (B) {
            a.spec_t16 = (uint16_t *)c->sp_pt;
            a.spec_nh = c->sp_nh;
            a.spec_flags = c->sp_small + 66;
            if (!c->sf_clean) // spec_classes of the previous call clears them
                HIP_TRY(hipMemsetAsync(a.spec_flags, 0, 64 * 4, s));
            c->sf_clean = 0;
            // sp_small: [0] node state, [1..] meta, [66..129] flags, [140] k_spec_scan's
            // ticket, [142..143] k_spec_fallback's barrier, [512 + 32 g] k_classify_cnet's tickets
            a.spec_meta = c->sp_small + 1;
            a.spec_cls = c->sp_class;
            a.spec_ticket = c->sp_small + 512;
            a.spec_bar = c->sp_small + 142;
            a.spec_B = B;
            a.spec_allow = c->tune_spec_scan == 0 ? 1u : 0u;
            a.spec_hint = c->sp_hint_d;
        }
        // the deferred kernel indexes frames in 32 bits and its outputs by 32-bit
        // byte offsets (at32: n < 2^30)
        if (c->tune_cnet_tile && b->n < (1u << 30)) {
            // fast kernel, then the general parse of the frames it left
            if ((uint64_t)b->n + 1 > c->cs_wl_cap) {
                if (c->cs_wl)
                    HIP_TRY(hipFree(c->cs_wl));
                c->cs_wl = nullptr;
                c->cs_wl_cap = 0;
                const uint64_t wcap = (uint64_t)b->n + (b->n >> 3) + 1024;
                HIP_TRY(hipMalloc((void **)&c->cs_wl, wcap * 4));
                c->cs_wl_cap = wcap;
                c->wl_clean = 0;
            }
            a.wl_n = c->cs_wl;
            a.wl = c->cs_wl + 1;
            if (!c->wl_clean) // else spec_classes of the previous call cleared it
                HIP_TRY(hipMemsetAsync(a.wl_n, 0, 4, s));
            c->wl_clean = 0;
            const uint64_t n_tiles = ((uint64_t)b->n + 63u) / 64u;
            // the schedule (CNDP_TUNE_STREAM_BAL): balanced -- one CD_BAL_THREADS block a
            // CU, all its waves sharing the block's tiles -- for strided frames (C5 2.5 %
            // faster), static 512-thread blocks, two a CU, for frames at offsets (IMIX:
            // C4 0.8-3 % slower balanced)
            const bool bal = c->tune_lnt && (c->tune_stream_bal == 2 || (c->tune_stream_bal == 0 && !b->offsets));
            const uint32_t nthr = bal ? CD_BAL_THREADS : CT_THREADS;
            uint64_t gd = (n_tiles + nthr / 64u - 1) / (nthr / 64u);
            const uint32_t bpc = c->tune_bpc ? (uint32_t)c->tune_bpc : bal ? 1u : 2u;
            if (gd > (uint64_t)c->num_cu * bpc)
                gd = (uint64_t)c->num_cu * bpc;
            // [load_nt][meta out][codes] (codes with non-temporal loads only: load_nt 0
            // is an A/B knob, and the codes only save stores)
            static void (*const dfns[2][2][2])(KArgs, uint32_t) = {
                {{k_cnet_defer<false, false, false, false>, k_cnet_defer<false, false, false, false>},
                 {k_cnet_defer<false, true, false, false>, k_cnet_defer<false, true, false, false>}},
                {{k_cnet_defer<true, false, false, false>, k_cnet_defer<true, false, true, false>},
                 {k_cnet_defer<true, true, false, false>, k_cnet_defer<true, true, true, false>}}};
            // the LDS-balanced schedule (CNDP_TUNE_STREAM_BAL), non-temporal loads: [meta out][codes]
            static void (*const bfns[2][2])(KArgs, uint32_t) = {
                {k_cnet_defer<true, false, false, true>, k_cnet_defer<true, false, true, true>},
                {k_cnet_defer<true, true, false, true>, k_cnet_defer<true, true, true, true>}};
            const bool meta_out = a.ptype != nullptr || a.rxmeta != nullptr;
            a.spec_tile = B ? c->sp_tile : nullptr; // written by this kernel only
            // chunk lists (CNDP_TUNE_SPEC_LISTS): groups must be lane quads of the
            // tiles (bursts of a multiple of 4) and the chunked passes run (B <= 256)
            if (B && B <= 256 && (B & 3u) == 0 && c->tune_spec_lists && c->tune_spec_scan == 0) {
                a.spec_cwl = c->sp_cwl;
                a.spec_cflag = c->sp_cflag;
                a.spec_allow |= SPEC_ALLOW_LISTS;
            }
            // the previous call left no worklist: the main kernel's last block
            // takes this call's (if any) and the classes pass, no second launch.
            // The hint is a pinned word an earlier call's kernel wrote, maybe
            // not yet this call's predecessor: either branch gives the same
            // results (CNDP_TUNE_CNET_FOLD forces one, the tests run both)
            a.wl_fold = 0;
            const bool fold = c->tune_cnet_fold == 1 ||
                              (c->tune_cnet_fold == 0 && c->sp_hint && ((volatile uint32_t *)c->sp_hint)[0] == 0u);
            if (B && fold) {
                const uint64_t nb = ((uint64_t)b->n + B - 1) / B;
                const uint64_t t0 = nb > SPEC_TAIL ? (nb - SPEC_TAIL) * B : 0;
                a.wl_fold = 1;
                a.tail_lo = (uint32_t)t0;
            }
            // canonical tiles' types as codes (CNDP_TUNE_SPEC_TYPES): auto after a
            // uniform batch, whose passes read none of them
            if (a.spec_tile && B <= 256) {
                const uint64_t nb = ((uint64_t)b->n + B - 1) / B;
                a.spec_c2 = c->sp_c2;
                a.spec_keep_lo = nb > SPEC_TAIL ? (uint32_t)((nb - SPEC_TAIL) * B) : 0u;
                a.spec_codes = c->tune_spec_types == 2 ||
                               (c->tune_spec_types == 0 && c->sp_hint && ((volatile uint32_t *)c->sp_hint)[1]);
            }
            if (!c->tune_lnt)
                a.spec_codes = 0;
            hipLaunchKernelGGL(bal ? bfns[meta_out ? 1 : 0][a.spec_codes ? 1 : 0]
                                   : dfns[c->tune_lnt ? 1 : 0][meta_out ? 1 : 0][a.spec_codes ? 1 : 0],
                               dim3((uint32_t)gd), dim3(nthr), 0, s, a, (uint32_t)n_tiles);
            if (!a.wl_fold)
                hipLaunchKernelGGL(k_classify_cnet<true>, dim3(g), dim3(CNET_THREADS), 0, s, a);
            if (a.spec_codes) // the coded types, should the passes read them after all
                hipLaunchKernelGGL(k_spec_expand, dim3((uint32_t)c->num_cu * 2u), dim3(256), 0, s, a,
                                   (uint32_t)n_tiles, (const uint32_t *)(c->sp_small + 1));
        } else {
            hipLaunchKernelGGL(k_classify_cnet<false>, dim3(g), dim3(CNET_THREADS), 0, s, a);
        }
        if (B) {
            const uint64_t nb = ((uint64_t)b->n + B - 1) / B;
            uint32_t *state = c->sp_small, *meta = c->sp_small + 1;
            uint32_t *ticket = c->sp_small + 140; // k_spec_scan's arrival count (0 between launches)
            c->sf_clean = 1; // spec_classes (k_classify_cnet's last block) clears them
            c->wl_clean = a.wl_n != nullptr;
            const uint32_t gw = (uint32_t)((nb + 3) / 4); // one wave per burst
            const uint32_t kfast = c->tune_spec_scan == 0 ? SPEC_KFAST : 0u;
            const uint32_t kmax = c->tune_spec_scan == 2 ? 0u : SPEC_KMAX;
            if (B <= 256) { // chunked passes (SPEC_CH bursts per wave)
                const uint64_t nch = (nb + SPEC_CH - 1) / SPEC_CH;
                // auto mode: the local pass first, the general one only for what it leaves
                const uint32_t gated = c->tune_spec_scan == 0 ? 1u : 0u;
                const uint64_t nblk = (nch + SPEC_BLK - 1) / SPEC_BLK;
                uint32_t *P = c->sp_U, *Bt = c->sp_U + nch * SPEC_KMAX, *Sblk = Bt + nblk * SPEC_KMAX;
                if (gated && a.spec_tile) { // the main kernel wrote tile words
                    uint32_t gl = (uint32_t)((nch + 4 * SPEC_LQ - 1) / (4 * SPEC_LQ)); // SPEC_LQ chunks per wave
                    // the previous call was a uniform batch: a wave per 64+ tiles
                    // (any grid gives the same results; CNDP_TUNE_SPEC_GRID forces
                    // a 2-block grid or the full one)
                    const bool shrink = c->tune_spec_grid == 1 ||
                                        (c->tune_spec_grid == 0 && c->sp_hint && ((volatile uint32_t *)c->sp_hint)[1]);
                    const uint32_t cap = c->tune_spec_grid == 1 ? 2u : (uint32_t)c->num_cu * 4u;
                    if (shrink && gl > cap)
                        gl = cap;
                    hipLaunchKernelGGL(k_spec_local_t<SPEC_CH>, dim3(gl), dim3(256), 0, s, a, B, nb, nch, meta,
                                       c->sp_done);
                } else if (gated) {
                    auto lo = k_spec_local<SPEC_CH, SPEC_WPB>;
                    const uint32_t gl = (uint32_t)((nch + SPEC_WPB - 1) / SPEC_WPB);
                    hipLaunchKernelGGL(lo, dim3(gl), dim3(SPEC_WPB * 64), 0, s, a, B, nb, nch, meta, c->sp_done);
                }
                // the general resolution: a block a CU (ticket-ordered items, so
                // correct whichever blocks get a CU; mostly it returns at once)
                hipLaunchKernelGGL(k_spec_fallback<SPEC_CH>, dim3((uint32_t)c->num_cu), dim3(256), 0, s, a, B, nb,
                                   nch, meta, (const uint8_t *)c->sp_class, c->sp_T, P, Bt, Sblk, c->sp_S,
                                   (const uint8_t *)c->sp_done, a.spec_bar, kfast, kmax, gated,
                                   c->tune_spec_wait_us < 0 ? 0u : (uint32_t)c->tune_spec_wait_us * 100u);
            } else {
                hipLaunchKernelGGL(k_spec_tables, dim3(gw), dim3(256), 0, s, (const uint16_t *)a.spec_t16, b->n, B,
                                   nb, (const uint32_t *)meta, (const uint8_t *)c->sp_class, c->sp_T);
                const uint64_t nblk = (nb + SPEC_BLK - 1) / SPEC_BLK;
                uint32_t *P = c->sp_U, *Bt = c->sp_U + nb * SPEC_KMAX, *Sblk = Bt + nblk * SPEC_KMAX;
                hipLaunchKernelGGL(k_spec_scan, dim3((uint32_t)nblk), dim3(SPEC_BLK), 0, s, nb,
                                   (const uint32_t *)meta, (const uint32_t *)c->sp_T, P, Bt,
                                   (const uint8_t *)c->sp_class, Sblk, state, ticket,
                                   (const uint16_t *)a.spec_t16, b->n, B, nb, c->sp_S, kfast, kmax, 0u);
                hipLaunchKernelGGL(k_spec_emit, dim3(gw), dim3(256), 0, s, a, B, nb, kfast, kmax,
                                   (const uint32_t *)meta, (const uint8_t *)c->sp_class, (const uint32_t *)P,
                                   (const uint32_t *)Sblk, (const uint32_t *)c->sp_S);
            }
        }
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

static int classify_l3(cndp_gpu_ctx_t *c, const struct cndp_batch *b, KArgs &a, hipStream_t s, uint16_t *rw_tx,
                       bool *fused)
{
    {
        uint32_t g = blocks_for(b->n, FAST_THREADS);
        // auto: 2 blocks per CU for the streamed kernel, 4 for the others
        // (the fused rewrite runs the split-gather tile kernel)
        const uint32_t bpc = c->tune_bpc ? (uint32_t)c->tune_bpc : !rw_tx ? 2u : 4u;
        const uint32_t cap = (uint32_t)c->num_cu * bpc;
        if (g > cap)
            g = cap;
        // wave-tile path: packed 64-B slots, 16-B aligned, whole tiles in bounds
        const uint64_t n_tiles = b->n / 64u;
        const bool tile_ok = c->tune_tile && !b->offsets && b->stride == 64 &&
                             (((uintptr_t)b->slab + b->data_off) & 15u) == 0 && n_tiles > 0 &&
                             b->data_off + n_tiles * 4096u <= b->slab_len;
        const int mi = b->mode == CNDP_MODE_L3FWD ? 0 : 1, nti = c->tune_nt ? 1 : 0, li = c->tune_lnt ? 1 : 0;
        if (tile_ok) {
            uint32_t gt = (uint32_t)((n_tiles + TILE_WAVES - 1) / TILE_WAVES);
            if (gt > cap)
                gt = cap;
            typedef void (*tile_fn)(KArgs, uint64_t);
            if (rw_tx && b->mode == CNDP_MODE_L3FWD && b->n % 256u == 0 && c->d_rw_tbl) {
                // ip4_rewrite fused into the split-gather tile kernel (the rewrite is
                // applied to the frame tile already in LDS)
                static const tile_fn rfns[2][2] = {
                    {k_classify_tile<CNDP_MODE_L3FWD, 2, false, true, false>,
                     k_classify_tile<CNDP_MODE_L3FWD, 2, false, true, true>},
                    {k_classify_tile<CNDP_MODE_L3FWD, 2, true, true, false>,
                     k_classify_tile<CNDP_MODE_L3FWD, 2, true, true, true>}};
                a.rw_tbl = c->d_rw_tbl;
                a.tx_edge = rw_tx;
                a.rw_parts = c->tune_rw_wb == 1 ? 4u : c->tune_rw_wb == 2 ? 5u : c->rw_parts;
                *fused = true;
                hipLaunchKernelGGL(rfns[nti][li], dim3(gt), dim3(FAST_THREADS), 0, s, a, n_tiles);
                HIP_TRY(hipGetLastError());
                return 0;
            }
            if (c->tune_stream_bal != 1) {
                // one STREAM_BW-wave block a CU, the block's tiles shared by an LDS counter
                static const tile_fn bfns[2][2][2] = {
                    {{k_classify_stream_bal<CNDP_MODE_L3FWD, false, false>,
                      k_classify_stream_bal<CNDP_MODE_L3FWD, false, true>},
                     {k_classify_stream_bal<CNDP_MODE_L3FWD, true, false>,
                      k_classify_stream_bal<CNDP_MODE_L3FWD, true, true>}},
                    {{k_classify_stream_bal<CNDP_MODE_HASH, false, false>,
                      k_classify_stream_bal<CNDP_MODE_HASH, false, true>},
                     {k_classify_stream_bal<CNDP_MODE_HASH, true, false>,
                      k_classify_stream_bal<CNDP_MODE_HASH, true, true>}}};
                uint32_t gb = (uint32_t)c->num_cu * (c->tune_bpc ? (uint32_t)c->tune_bpc : 1u);
                if ((uint64_t)gb > n_tiles)
                    gb = (uint32_t)n_tiles;
                hipLaunchKernelGGL(bfns[mi][nti][li], dim3(gb), dim3(STREAM_BW * 64), 0, s, a, n_tiles);
                HIP_TRY(hipGetLastError());
                return 0;
            }
            static const tile_fn sfns[2][2][2] = {
                {{k_classify_stream<CNDP_MODE_L3FWD, false, false>, k_classify_stream<CNDP_MODE_L3FWD, false, true>},
                 {k_classify_stream<CNDP_MODE_L3FWD, true, false>, k_classify_stream<CNDP_MODE_L3FWD, true, true>}},
                {{k_classify_stream<CNDP_MODE_HASH, false, false>, k_classify_stream<CNDP_MODE_HASH, false, true>},
                 {k_classify_stream<CNDP_MODE_HASH, true, false>, k_classify_stream<CNDP_MODE_HASH, true, true>}}};
            hipLaunchKernelGGL(sfns[mi][nti][li], dim3(gt), dim3(FAST_THREADS), 0, s, a, n_tiles);
            HIP_TRY(hipGetLastError());
            return 0;
        }
        // any layout (strided UMEM frames, IMIX offsets, unaligned slabs): per lane
        typedef void (*fast_fn)(KArgs);
        static const fast_fn ffns[2][2] = {{k_classify_fast<CNDP_MODE_L3FWD, false, 1>, k_classify_fast<CNDP_MODE_L3FWD, true, 1>},
                                           {k_classify_fast<CNDP_MODE_HASH, false, 1>, k_classify_fast<CNDP_MODE_HASH, true, 1>}};
        hipLaunchKernelGGL(ffns[mi][nti], dim3(g), dim3(FAST_THREADS), 0, s, a);
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

// a k_spec_fallback wait of an earlier call expired (its edges are not the
// node's): taken once, the node state restarts at 0
static bool spec_err_take(cndp_gpu_ctx_t *c)
{
    if (!c->sp_hint || !__atomic_load_n(&c->sp_hint[SPEC_HINT_ERR], __ATOMIC_ACQUIRE))
        return false;
    __atomic_store_n(&c->sp_hint[SPEC_HINT_ERR], 0u, __ATOMIC_RELAXED);
    c->spec_reset = 1;
    return true;
}

extern "C" int cndp_gpu_classify(cndp_gpu_ctx_t *c, const struct cndp_batch *b, void *stream)
{
    if (c && b && b->mode == CNDP_MODE_CNET && spec_err_take(c))
        return -EIO;
    return classify_impl(c, b, stream, nullptr, nullptr);
}

// grow a device buffer to at least `need` bytes (contents not kept)
static int grow(void **buf, uint64_t *cap, uint64_t need)
{
    if (*cap >= need && *buf)
        return 0;
    if (*buf)
        HIP_TRY(hipFree(*buf));
    *buf = nullptr;
    *cap = 0;
    const uint64_t sz = need + (need >> 3) + 4096;
    HIP_TRY(hipMalloc(buf, sz));
    *cap = sz;
    return 0;
}

// Host-memory batch (AF_XDP UMEM / loopback socket buffers).  The slab is
// mirrored into device memory at the same byte offsets, streamed in 64 MiB
// segments in byte order on the copy-in stream; packet chunk k is classified
// on the compute stream as soon as every segment it can read has landed --
// its frame bases plus CNDP_HOST_REACH bytes, the farthest any parse reads
// (Ethernet + 2 VLAN tags + IPv4 options + tunnel + inner headers + 5 IPv6
// extension headers of at most 2 KiB each) -- and its results go back on the
// copy-out stream.  The kernel therefore sees exactly the bytes the device-
// resident path sees: results are identical to cndp_gpu_classify.
//
// Windows only (CNDP_TUNE_HOST_WINDOW, default): the l3fwd and hash parses
// read nothing past a frame's first 64 bytes (Ethernet + IPv4 + the L4
// ports), so for frames at a stride wider than that -- the AF_XDP UMEM's
// 2 KiB frames with data at +256 -- each chunk's windows go H2D as one
// strided 2-D copy (source pitch = the stride, 64-B rows) into packed 64-B
// slots, and the streamed wave-tile kernel classifies those: 64 of every
// 2048 bytes cross PCIe.  Same bytes in every window, so the same results.
#define CNDP_HOST_SEG (64ull << 20)
#define CNDP_HOST_REACH (16ull << 10)
#define CNDP_HOST_WIN 64ull

extern "C" int cndp_gpu_classify_host(cndp_gpu_ctx_t *c, const struct cndp_batch *hb)
{
    int r = validate_batch(c, hb);
    if (r)
        return r;
    if ((r = set_device(c->dev)))
        return r;
    const uint64_t n = hb->n;
    const uint64_t o_nh = 0, o_hash = o_nh + n * 4, o_q = o_hash + n * 4, o_e = o_q + ((n * 2 + 15) & ~15ull),
                   o_b = o_e + ((n + 15) & ~15ull), o_pt = o_b + ((uint64_t)hb->n_bins + 2) * 8,
                   o_rm = o_pt + n * 4, out_bytes = o_rm + n * 4;
    for (int k = 0; k < 3; k++)
        if (!c->hs[k])
            HIP_TRY(hipStreamCreateWithFlags(&c->hs[k], hipStreamNonBlocking));
    hipStream_t cs = c->hs[0], ks = c->hs[1], ds = c->hs[2];
    const bool win = c->tune_host_window && hb->mode != CNDP_MODE_CNET && !hb->offsets && n &&
                     hb->stride > CNDP_HOST_WIN && (uint64_t)hb->data_off + CNDP_HOST_WIN <= hb->stride &&
                     (n - 1) * hb->stride + hb->data_off + CNDP_HOST_WIN <= hb->slab_len;
    if ((r = grow((void **)&c->h_slab, &c->h_slab_cap, win ? n * CNDP_HOST_WIN : hb->slab_len ? hb->slab_len : 1)) ||
        (r = grow((void **)&c->h_out, &c->h_out_cap, out_bytes)) ||
        (hb->offsets && (r = grow((void **)&c->h_off, &c->h_off_cap, n * 8 + 8))))
        return r;
    uint64_t *d_bins = hb->bins ? (uint64_t *)(c->h_out + o_b) : nullptr;
    if (hb->bins)
        HIP_TRY(hipMemcpyAsync(d_bins, hb->bins, ((uint64_t)hb->n_bins + 2) * 8, hipMemcpyHostToDevice, cs));
    uint64_t C = c->host_chunk;
    if (hb->mode == CNDP_MODE_CNET && c->spec_burst) // chunks hold whole graph bursts
        C = C < c->spec_burst ? c->spec_burst : C - C % c->spec_burst;
    const uint64_t n_chunks = n ? (n + C - 1) / C : 0;
    const uint64_t n_segs = (hb->slab_len + CNDP_HOST_SEG - 1) / CNDP_HOST_SEG;
    uint64_t seg_done = 0; // segments issued so far
    hipEvent_t ev_in = nullptr, ev_k = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&ev_k, hipEventDisableTiming));
    r = -EIO;
    for (uint64_t k = 0; k < n_chunks; k++) {
        const uint64_t i0 = k * C, cnt = (n - i0) < C ? (n - i0) : C;
        if (win) { // this chunk's windows, packed
            struct cndp_batch cb = *hb;
            if (hipMemcpy2DAsync(c->h_slab + i0 * CNDP_HOST_WIN, CNDP_HOST_WIN,
                                 (const uint8_t *)hb->slab + i0 * hb->stride + hb->data_off, hb->stride, CNDP_HOST_WIN,
                                 cnt, hipMemcpyHostToDevice, cs) != hipSuccess ||
                hipEventRecord(ev_in, cs) != hipSuccess || hipStreamWaitEvent(ks, ev_in, 0) != hipSuccess)
                goto out;
            cb.n = (uint32_t)cnt;
            cb.slab = c->h_slab + i0 * CNDP_HOST_WIN;
            cb.slab_len = (n - i0) * CNDP_HOST_WIN;
            cb.stride = (uint32_t)CNDP_HOST_WIN;
            cb.data_off = 0;
            cb.nh = hb->nh ? (uint32_t *)(c->h_out + o_nh) + i0 : nullptr;
            cb.hash = hb->hash ? (uint32_t *)(c->h_out + o_hash) + i0 : nullptr;
            cb.queue = hb->queue ? (uint16_t *)(c->h_out + o_q) + i0 : nullptr;
            cb.edge = hb->edge ? c->h_out + o_e + i0 : nullptr;
            cb.bins = d_bins;
            cb.ptype = hb->ptype ? (uint32_t *)(c->h_out + o_pt) + i0 : nullptr;
            cb.rxmeta = nullptr;
            if ((r = cndp_gpu_classify(c, &cb, ks)))
                goto out;
            r = -EIO;
            if (hipEventRecord(ev_k, ks) != hipSuccess || hipStreamWaitEvent(ds, ev_k, 0) != hipSuccess)
                goto out;
            if (hb->nh && hipMemcpyAsync(hb->nh + i0, cb.nh, cnt * 4, hipMemcpyDeviceToHost, ds) != hipSuccess)
                goto out;
            if (hb->hash && hipMemcpyAsync(hb->hash + i0, cb.hash, cnt * 4, hipMemcpyDeviceToHost, ds) != hipSuccess)
                goto out;
            if (hb->queue && hipMemcpyAsync(hb->queue + i0, cb.queue, cnt * 2, hipMemcpyDeviceToHost, ds) != hipSuccess)
                goto out;
            if (hb->edge && hipMemcpyAsync(hb->edge + i0, cb.edge, cnt, hipMemcpyDeviceToHost, ds) != hipSuccess)
                goto out;
            if (hb->ptype && hipMemcpyAsync(hb->ptype + i0, cb.ptype, cnt * 4, hipMemcpyDeviceToHost, ds) != hipSuccess)
                goto out;
            continue;
        }
        // byte span this chunk's parse can reach
        uint64_t hi;
        if (hb->offsets) {
            hi = 0;
            for (uint64_t i = i0; i < i0 + cnt; i++)
                hi = hb->offsets[i] > hi ? hb->offsets[i] : hi;
        } else {
            hi = (i0 + cnt - 1) * hb->stride;
        }
        hi += (uint64_t)hb->data_off + CNDP_HOST_REACH;
        const uint64_t seg_need = hi / CNDP_HOST_SEG + 1 < n_segs ? hi / CNDP_HOST_SEG + 1 : n_segs;
        for (; seg_done < seg_need; seg_done++) {
            const uint64_t lo = seg_done * CNDP_HOST_SEG;
            const uint64_t len = hb->slab_len - lo < CNDP_HOST_SEG ? hb->slab_len - lo : CNDP_HOST_SEG;
            if (hipMemcpyAsync(c->h_slab + lo, (const uint8_t *)hb->slab + lo, len, hipMemcpyHostToDevice, cs) !=
                hipSuccess)
                goto out;
        }
        if (hb->offsets && hipMemcpyAsync(c->h_off + i0, hb->offsets + i0, cnt * 8, hipMemcpyHostToDevice, cs) !=
                               hipSuccess)
            goto out;
        if (hipEventRecord(ev_in, cs) != hipSuccess || hipStreamWaitEvent(ks, ev_in, 0) != hipSuccess)
            goto out;
        struct cndp_batch cb = *hb;
        cb.n = (uint32_t)cnt;
        cb.slab = c->h_slab;
        if (hb->offsets)
            cb.offsets = c->h_off + i0;
        else
            cb.data_off = hb->data_off; // packet i0 sits at i0 * stride: shift the slab view instead
        cb.nh = hb->nh ? (uint32_t *)(c->h_out + o_nh) + i0 : nullptr;
        cb.hash = hb->hash ? (uint32_t *)(c->h_out + o_hash) + i0 : nullptr;
        cb.queue = hb->queue ? (uint16_t *)(c->h_out + o_q) + i0 : nullptr;
        cb.edge = hb->edge ? c->h_out + o_e + i0 : nullptr;
        cb.bins = d_bins;
        cb.ptype = hb->ptype ? (uint32_t *)(c->h_out + o_pt) + i0 : nullptr;
        cb.rxmeta = hb->rxmeta ? (uint32_t *)(c->h_out + o_rm) + i0 : nullptr;
        if (!hb->offsets) {
            // frames of this chunk start at byte i0 * stride of the mirror
            cb.slab = c->h_slab + i0 * hb->stride;
            cb.slab_len = hb->slab_len > i0 * hb->stride ? hb->slab_len - i0 * hb->stride : 0;
        }
        if ((r = cndp_gpu_classify(c, &cb, ks)))
            goto out;
        r = -EIO;
        if (hipEventRecord(ev_k, ks) != hipSuccess || hipStreamWaitEvent(ds, ev_k, 0) != hipSuccess)
            goto out;
        if (hb->nh && hipMemcpyAsync(hb->nh + i0, cb.nh, cnt * 4, hipMemcpyDeviceToHost, ds) != hipSuccess)
            goto out;
        if (hb->hash && hipMemcpyAsync(hb->hash + i0, cb.hash, cnt * 4, hipMemcpyDeviceToHost, ds) != hipSuccess)
            goto out;
        if (hb->queue && hipMemcpyAsync(hb->queue + i0, cb.queue, cnt * 2, hipMemcpyDeviceToHost, ds) != hipSuccess)
            goto out;
        if (hb->edge && hipMemcpyAsync(hb->edge + i0, cb.edge, cnt, hipMemcpyDeviceToHost, ds) != hipSuccess)
            goto out;
        if (hb->ptype && hipMemcpyAsync(hb->ptype + i0, cb.ptype, cnt * 4, hipMemcpyDeviceToHost, ds) != hipSuccess)
            goto out;
        if (hb->rxmeta &&
            hipMemcpyAsync(hb->rxmeta + i0, cb.rxmeta, cnt * 4, hipMemcpyDeviceToHost, ds) != hipSuccess)
            goto out;
    }
    if (n_chunks == 0) { // still bind / sync the FIB images like the device path
        struct cndp_batch cb = *hb;
        cb.n = 0;
        if ((r = cndp_gpu_classify(c, &cb, ks)))
            goto out;
        r = -EIO;
    }
    if (hb->bins) {
        if (hipEventRecord(ev_k, ks) != hipSuccess || hipStreamWaitEvent(ds, ev_k, 0) != hipSuccess)
            goto out;
        if (hipMemcpyAsync(hb->bins, d_bins, ((uint64_t)hb->n_bins + 2) * 8, hipMemcpyDeviceToHost, ds) !=
            hipSuccess)
            goto out;
    }
    if (hipStreamSynchronize(ds) != hipSuccess || hipStreamSynchronize(ks) != hipSuccess ||
        hipStreamSynchronize(cs) != hipSuccess)
        goto out;
    r = 0;
out:
    if (r) {
        hipStreamSynchronize(cs);
        hipStreamSynchronize(ks);
        hipStreamSynchronize(ds);
    }
    hipEventDestroy(ev_in);
    hipEventDestroy(ev_k);
    return r;
}

// ---------------------------------------------------------------------------
// ip4_rewrite (ip4_rewrite.c:40-247) and the cndpfwd loopback MAC swap
// (examples/cndpfwd/main.h:303-315), in place on the device frame slab.
// A block owns whole graph bursts: the rewrite stream of a burst is its
// edge-0 packets in order; the first (count & ~3) of them take the 4-wide
// loop's checksum update (end-around carry, :97-104), the rest the tail
// loop's (:214-216).  Frames whose first 28 bytes are 4-B aligned and in
// the slab are rewritten as 7 dwords; others byte by byte.
// ---------------------------------------------------------------------------
struct RwArgs {
    uint8_t *slab;
    uint64_t slab_len, stride;
    const uint64_t *offsets;
    uint32_t data_off, n, burst;
    const uint32_t *nh;
    const struct cndp_rw_nh *tbl;
    uint16_t *tx_edge;
};

__device__ __forceinline__ bool rw_bound(uint32_t v) { return v != CNDP_NH_INVALID && (v >> 16) == 0u; }

// block-wide count of `f` and this thread's exclusive prefix (256 threads)
__device__ __forceinline__ uint32_t block_scan(bool f, uint32_t *s_w, uint32_t &total)
{
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const unsigned long long m = __ballot(f);
    const uint32_t below = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    __syncthreads();
    if (lane == 0)
        s_w[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t pre = 0;
    total = 0;
    for (uint32_t k = 0; k < 4; k++) {
        pre += k < wv ? s_w[k] : 0u;
        total += s_w[k];
    }
    return pre + below;
}

__device__ __forceinline__ void rw_byte(uint8_t *slab, uint64_t len, uint64_t o, uint32_t v)
{
    if (o < len)
        slab[o] = (uint8_t)v;
}

__global__ __launch_bounds__(256) void k_ip4_rewrite(RwArgs a)
{
    __shared__ struct cndp_rw_nh s_tbl[CNDP_RW_MAX_NH];
    __shared__ uint32_t s_w[4];
    for (uint32_t k = threadIdx.x; k < sizeof(s_tbl) / 4; k += 256)
        ((uint32_t *)s_tbl)[k] = ((const uint32_t *)a.tbl)[k];
    __syncthreads();
    const uint64_t n_bursts = ((uint64_t)a.n + a.burst - 1) / a.burst;
    for (uint64_t b = blockIdx.x; b < n_bursts; b += gridDim.x) {
        const uint64_t b0 = b * a.burst, b1 = b0 + a.burst < a.n ? b0 + a.burst : a.n;
        uint32_t cnt = 0;
        for (uint64_t c0 = b0; c0 < b1; c0 += 256) {
            const uint64_t i = c0 + threadIdx.x;
            uint32_t tot;
            block_scan(i < b1 && rw_bound(a.nh[i]), s_w, tot);
            cnt += tot;
        }
        const uint32_t vec = cnt & ~3u;
        uint32_t run = 0;
        for (uint64_t c0 = b0; c0 < b1; c0 += 256) {
            const uint64_t i = c0 + threadIdx.x;
            const uint32_t v = i < b1 ? a.nh[i] : CNDP_NH_INVALID;
            const bool f = i < b1 && rw_bound(v);
            uint32_t tot;
            const uint32_t pos = run + block_scan(f, s_w, tot);
            run += tot;
            if (i >= b1)
                continue;
            if (!f) {
                if (a.tx_edge)
                    a.tx_edge[i] = 0xFFFFu;
                continue;
            }
            const uint64_t base = (a.offsets ? a.offsets[i] : i * a.stride) + a.data_off;
            const uint32_t nh16 = v & 0xffffu;
            const uint32_t len = nh16 < CNDP_RW_MAX_NH ? s_tbl[nh16].rewrite_len : 0u;
            const uint32_t tx = nh16 < CNDP_RW_MAX_NH ? s_tbl[nh16].tx_node : 0u;
            const uint8_t *data = s_tbl[nh16 < CNDP_RW_MAX_NH ? nh16 : 0].rewrite_data;
            const uint32_t lenc = len < CNDP_RW_MAX_LEN ? len : CNDP_RW_MAX_LEN;
            uint8_t *p = a.slab + base;
            const bool fast = base + 28 <= a.slab_len && (((uintptr_t)p) & 3u) == 0;
            uint32_t ttl, ck;
            if (fast) {
                uint32_t d[7];
#pragma unroll
                for (int k = 0; k < 7; k++)
                    d[k] = ((const uint32_t *)p)[k];
                ttl = (d[5] >> 16) & 0xffu;
                ck = d[6] & 0xffffu;
                for (uint32_t k = 0; k < lenc && k < 28; k++) {
                    const uint32_t sh = (k & 3u) * 8u;
                    d[k >> 2] = (d[k >> 2] & ~(0xffu << sh)) | ((uint32_t)data[k] << sh);
                }
                uint32_t nck;
                if (pos < vec) {
                    const uint32_t c32 = ck + 1u;
                    nck = ((c32 & 0xffffu) + (c32 >> 16)) & 0xffffu;
                } else {
                    uint32_t c16 = (ck + 1u) & 0xffffu;
                    nck = (c16 + (c16 >= 0xffffu ? 1u : 0u)) & 0xffffu;
                }
                d[5] = (d[5] & 0xff00ffffu) | (((ttl - 1u) & 0xffu) << 16);
                d[6] = (d[6] & 0xffff0000u) | nck;
#pragma unroll
                for (int k = 0; k < 7; k++)
                    ((uint32_t *)p)[k] = d[k];
                for (uint32_t k = 28; k < lenc; k++)
                    rw_byte(a.slab, a.slab_len, base + k, data[k]);
            } else {
                ttl = base + 22 < a.slab_len ? p[22] : 0u;
                ck = (base + 24 < a.slab_len ? p[24] : 0u) | ((base + 25 < a.slab_len ? (uint32_t)p[25] : 0u) << 8);
                for (uint32_t k = 0; k < lenc; k++)
                    rw_byte(a.slab, a.slab_len, base + k, data[k]);
                uint32_t nck;
                if (pos < vec) {
                    const uint32_t c32 = ck + 1u;
                    nck = ((c32 & 0xffffu) + (c32 >> 16)) & 0xffffu;
                } else {
                    uint32_t c16 = (ck + 1u) & 0xffffu;
                    nck = (c16 + (c16 >= 0xffffu ? 1u : 0u)) & 0xffffu;
                }
                rw_byte(a.slab, a.slab_len, base + 22, ttl - 1u);
                rw_byte(a.slab, a.slab_len, base + 24, nck & 0xffu);
                rw_byte(a.slab, a.slab_len, base + 25, nck >> 8);
            }
            if (a.tx_edge)
                a.tx_edge[i] = (uint16_t)tx;
        }
    }
}

__global__ __launch_bounds__(256) void k_mac_swap(uint8_t *slab, uint64_t slab_len, uint64_t stride,
                                                  const uint64_t *offsets, uint32_t data_off, uint32_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t base = (offsets ? offsets[i] : i * stride) + data_off;
        if (base + 12 > slab_len)
            continue;
        uint8_t *p = slab + base;
        if ((((uintptr_t)p) & 3u) == 0) {
            uint32_t *d = (uint32_t *)p;
            const uint32_t d0 = d[0], d1 = d[1], d2 = d[2];
            d[0] = alignb(d2, d1, 2);          // bytes 6..9
            d[1] = (d2 >> 16) | (d0 << 16);    // bytes 10, 11, 0, 1
            d[2] = alignb(d1, d0, 2);          // bytes 2..5
        } else {
            for (int k = 0; k < 6; k++) {
                const uint8_t t = p[k];
                p[k] = p[6 + k];
                p[6 + k] = t;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// pktmbuf shim: the l3fwd-graph chain pktdev_rx (ptype) -> pkt_cls ->
// ip4_lookup over an array of pktmbuf_t pointers (host memory), with every
// field those nodes write into the mbuf written back the same way.
// pktmbuf_t layout (pktmbuf.h:102-204): buf_addr @8, hash @16, data_off @24,
// buf_len @28, data_len @30, packet_type @32, udata64 @56.
// ---------------------------------------------------------------------------
#define MB_BUF_ADDR 8
#define MB_HASH 16
#define MB_DATA_OFF 24
#define MB_BUF_LEN 28
#define MB_PTYPE 32
#define MB_UDATA64 56

static int mbuf_stage_grow(cndp_gpu_ctx_t *c, uint32_t n)
{
    if (c->m_cap >= n)
        return 0;
    const uint32_t cap = n < 4096 ? 4096 : n + (n >> 2);
    if (c->m_hwin)
        hipHostFree(c->m_hwin);
    if (c->m_hres)
        hipHostFree(c->m_hres);
    if (c->m_dwin)
        hipFree(c->m_dwin);
    if (c->m_dres)
        hipFree(c->m_dres);
    c->m_hwin = nullptr;
    c->m_hres = c->m_dres = nullptr;
    c->m_dwin = nullptr;
    c->m_cap = 0;
    HIP_TRY(hipHostMalloc((void **)&c->m_hwin, (size_t)cap * 64, 0));
    HIP_TRY(hipHostMalloc((void **)&c->m_hres, (size_t)cap * 8, 0));
    HIP_TRY(hipMalloc((void **)&c->m_dwin, (size_t)cap * 64));
    HIP_TRY(hipMalloc((void **)&c->m_dres, (size_t)cap * 8));
    c->m_cap = cap;
    return 0;
}

extern "C" int cndp_gpu_l3fwd_mbufs(cndp_gpu_ctx_t *c, void *const *mbufs, uint32_t n, uint16_t *edges,
                                    void *stream)
{
    if (!c || (n && (!mbufs || !edges)) || !c->fib4)
        return -EINVAL;
    int r = set_device(c->dev);
    if (r)
        return r;
    if (n == 0)
        return 0;
    if ((r = mbuf_stage_grow(c, n)))
        return r;
    // gather the 64-byte header window of each frame (bytes past the
    // segment buffer are zero, like the slab-end rule of the device path)
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t *m = (const uint8_t *)mbufs[i];
        const uint8_t *buf = *(uint8_t *const *)(m + MB_BUF_ADDR);
        const uint16_t doff = *(const uint16_t *)(m + MB_DATA_OFF);
        const uint16_t blen = *(const uint16_t *)(m + MB_BUF_LEN);
        uint8_t *w = c->m_hwin + (size_t)i * 64;
        const uint32_t avail = blen > doff ? (uint32_t)(blen - doff) : 0u;
        if (avail >= 64) {
            memcpy(w, buf + doff, 64);
        } else {
            memcpy(w, buf + doff, avail);
            memset(w + avail, 0, 64 - avail);
        }
    }
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipMemcpyAsync(c->m_dwin, c->m_hwin, (size_t)n * 64, hipMemcpyHostToDevice, s));
    struct cndp_batch b;
    memset(&b, 0, sizeof(b));
    b.mode = CNDP_MODE_L3FWD;
    b.n = n;
    b.slab = c->m_dwin;
    b.slab_len = (uint64_t)n * 64;
    b.stride = 64;
    b.buf_len = 1984;
    b.nh = c->m_dres;
    b.hash = c->m_dres + c->m_cap;
    if ((r = cndp_gpu_classify(c, &b, s)))
        return r;
    HIP_TRY(hipMemcpyAsync(c->m_hres, c->m_dres, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(c->m_hres + c->m_cap, c->m_dres + c->m_cap, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (uint32_t i = 0; i < n; i++) {
        uint8_t *m = (uint8_t *)mbufs[i];
        const uint8_t *w = c->m_hwin + (size_t)i * 64;
        const uint32_t et = ((uint32_t)w[12] << 8) | w[13];
        // pktdev_rx.c:24-34 l3_ptype
        *(uint32_t *)(m + MB_PTYPE) = et == 0x0800u ? 0x90u : et == 0x86DDu ? 0xE0u : 0u;
        if (c->mbuf_hash) // no reference node writes m->hash: opt-in (CNDP_TUNE_MBUF_HASH)
            *(uint32_t *)(m + MB_HASH) = c->m_hres[c->m_cap + i];
        const uint32_t val = c->m_hres[i];
        if (val == CNDP_NH_INVALID) { // pkt_cls.c: not IPv4 -> pkt_drop
            edges[i] = CNDP_MBUF_EDGE_CLS_DROP;
            continue;
        }
        // ip4_lookup.c:108-154: priv1 {nh, ttl, cksum} in udata64, edge = val >> 16
        const uint64_t nh16 = val & 0xffffu, ttl = w[22], cksum = (uint64_t)w[24] | ((uint64_t)w[25] << 8);
        *(uint64_t *)(m + MB_UDATA64) = nh16 | (ttl << 16) | (cksum << 32);
        edges[i] = (uint16_t)(val >> 16);
    }
    return 0;
}

// ip4_rewrite_set_next (ip4_rewrite.c:252-263)
extern "C" int cndp_gpu_ip4_rewrite_set_next(cndp_gpu_ctx_t *c, uint16_t port_id, uint16_t next_index)
{
    if (!c || port_id >= CNDP_RW_MAX_PORTS)
        return -EINVAL;
    if (!c->rw_local) { // from now on this context keeps a table of its own
        memset(c->rw_tbl, 0, sizeof(c->rw_tbl));
        c->rw_local = 1;
        c->rw_dirty = 1;
    }
    c->rw_next[port_id] = next_index;
    return 0;
}

// cne_node_ip4_rewrite_add (ip4_rewrite.c:265-295): same checks, same order
extern "C" int cndp_gpu_ip4_rewrite_add(cndp_gpu_ctx_t *c, uint16_t next_hop, const uint8_t *rewrite_data,
                                        uint8_t rewrite_len, uint16_t dst_port)
{
    if (!c)
        return -EINVAL;
    if (next_hop >= CNDP_RW_MAX_NH)
        return -EINVAL;
    if (rewrite_len > CNDP_RW_MAX_LEN)
        return -EINVAL;
    if (dst_port >= CNDP_RW_MAX_PORTS || !c->rw_next[dst_port])
        return -EINVAL;
    if (rewrite_len && !rewrite_data)
        return -EINVAL;
    struct cndp_rw_nh *e = &c->rw_tbl[next_hop];
    if (rewrite_len)
        memcpy(e->rewrite_data, rewrite_data, rewrite_len);
    e->tx_node = c->rw_next[dst_port];
    e->rewrite_len = rewrite_len;
    e->enabled = 1;
    c->rw_dirty = 1;
    return 0;
}

static int rw_sync(cndp_gpu_ctx_t *c, hipStream_t s)
{
    // a context without a table of its own follows the node table that
    // cne_node_ip4_rewrite_add fills (node.c), like the reference node does
    if (!c->rw_local && cndp_node_rw_gen() != c->rw_gen_seen) {
        c->rw_gen_seen = cndp_node_rw_snapshot(c->rw_tbl);
        c->rw_dirty = 1;
    }
    if (!c->d_rw_tbl) {
        HIP_TRY(hipMalloc((void **)&c->d_rw_tbl, sizeof(c->rw_tbl)));
        c->rw_dirty = 1;
    }
    if (c->rw_dirty) {
        uint32_t mx = 26; // TTL and checksum end at byte 26
        for (int k = 0; k < CNDP_RW_MAX_NH; k++)
            mx = c->rw_tbl[k].rewrite_len > mx ? c->rw_tbl[k].rewrite_len : mx;
        c->rw_parts = (mx + 15) / 16;
        HIP_TRY(hipMemcpyAsync(c->d_rw_tbl, c->rw_tbl, sizeof(c->rw_tbl), hipMemcpyHostToDevice, s));
        HIP_TRY(hipStreamSynchronize(s)); // the host table may change after we return
        c->rw_dirty = 0;
    }
    return 0;
}

extern "C" int cndp_gpu_ip4_rewrite(cndp_gpu_ctx_t *c, const struct cndp_batch *b, uint32_t burst,
                                    uint16_t *tx_edge, void *stream)
{
    if (!c || !b || burst == 0 || (b->n && (!b->slab || !b->nh)))
        return -EINVAL;
    int r = set_device(c->dev);
    if (r)
        return r;
    hipStream_t s = (hipStream_t)stream;
    if ((r = rw_sync(c, s)))
        return r;
    if (b->n == 0)
        return 0;
    RwArgs a;
    a.slab = (uint8_t *)b->slab;
    a.slab_len = b->slab_len;
    a.stride = b->stride;
    a.offsets = b->offsets;
    a.data_off = b->data_off;
    a.n = b->n;
    a.burst = burst;
    a.nh = b->nh;
    a.tbl = c->d_rw_tbl;
    a.tx_edge = tx_edge;
    const uint64_t n_bursts = ((uint64_t)b->n + burst - 1) / burst;
    uint64_t g = n_bursts;
    const uint64_t cap = (uint64_t)c->num_cu * 8u;
    if (g > cap)
        g = cap;
    hipLaunchKernelGGL(k_ip4_rewrite, dim3((uint32_t)g), dim3(256), 0, s, a);
    HIP_TRY(hipGetLastError());
    return 0;
}

// classify (l3fwd) + ip4_rewrite: one fused wave-tile kernel for packed
// 64-B slots in 256-packet bursts, otherwise the two kernels back to back
extern "C" int cndp_gpu_classify_rewrite(cndp_gpu_ctx_t *c, const struct cndp_batch *b, uint32_t burst,
                                         uint16_t *tx_edge, void *stream)
{
    if (!c || !b || b->mode != CNDP_MODE_L3FWD || burst == 0 || (b->n && (!b->nh || !tx_edge)))
        return -EINVAL;
    int r = set_device(c->dev);
    if (r)
        return r;
    if ((r = rw_sync(c, (hipStream_t)stream)))
        return r;
    bool fused = false;
    if ((r = classify_impl(c, b, stream, burst == 256 ? tx_edge : nullptr, &fused)))
        return r;
    return fused ? 0 : cndp_gpu_ip4_rewrite(c, b, burst, tx_edge, stream);
}

extern "C" int cndp_gpu_mac_swap(cndp_gpu_ctx_t *c, const struct cndp_batch *b, void *stream)
{
    if (!c || !b || (b->n && !b->slab))
        return -EINVAL;
    int r = set_device(c->dev);
    if (r)
        return r;
    if (b->n == 0)
        return 0;
    uint32_t g = blocks_for(b->n, 256);
    const uint32_t cap = (uint32_t)c->num_cu * 8u;
    if (g > cap)
        g = cap;
    hipLaunchKernelGGL(k_mac_swap, dim3(g), dim3(256), 0, (hipStream_t)stream, (uint8_t *)b->slab, b->slab_len,
                       b->stride, b->offsets, b->data_off, b->n);
    HIP_TRY(hipGetLastError());
    return 0;
}

// Device frame memory (cndp_gpu.h): the HBM a NIC's peer DMA or a host copy
// fills with frames and the classify kernels read in place.  Uncached
// (hipDeviceMallocUncached, MTYPE UC): no GPU L2 line of it can go stale under
// a peer's writes, and the kernels' sparse 64-B window reads (C4 IMIX, C5
// 1536-B strides) allocate no L2 lines -- DESIGN.md §6 (round 4) measures them
// faster than from hipMalloc memory.  CNDP_FRAMES_CACHED takes plain hipMalloc.
extern "C" int cndp_gpu_frames_alloc(int device, uint64_t bytes, uint32_t flags, void **dptr)
{
    if (dptr)
        *dptr = nullptr;
    if (!dptr || !bytes || (flags & ~CNDP_FRAMES_CACHED))
        return -EINVAL;
    int cur = -1;
    if (device >= 0 && (hipGetDevice(&cur) != hipSuccess || set_device(device)))
        return -ENODEV;
    const hipError_t e = (flags & CNDP_FRAMES_CACHED) ? hipMalloc(dptr, bytes)
                                                      : hipExtMallocWithFlags(dptr, bytes, hipDeviceMallocUncached);
    if (cur >= 0 && cur != device)
        hipSetDevice(cur); // the caller's current device is left as it was
    if (e != hipSuccess) {
        *dptr = nullptr;
        fprintf(stderr, "cndp_gpu: frames alloc of %llu B failed: %s\n", (unsigned long long)bytes,
                hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? -ENOMEM : -EIO;
    }
    return 0;
}

extern "C" int cndp_gpu_frames_free(void *dptr)
{
    if (dptr)
        HIP_TRY(hipFree(dptr));
    return 0;
}

// Pin + map host memory (an AF_XDP UMEM region, a socket buffer pool) so the
// device reads frames from it in place (zero-copy ingest) and DMA runs at
// full rate.  *dev_ptr is the device-side address of `ptr`.
// hipHostRegister is per process, while every graph node holds its own
// context: the registration is shared and reference counted.  A region
// already registered through another context (or by the application itself,
// hipHostRegister) is recorded with its device address and never
// unregistered by a context that did not register it; the last reference
// registered here unregisters it.
struct HostRegion {
    uint8_t *host, *dev;
    uint64_t len;
    int refs;
    bool owned; // registered by this library (else by the application)
};
static pthread_mutex_t g_reg_lock = PTHREAD_MUTEX_INITIALIZER;
static HostRegion g_reg[64];
static int g_nreg;

extern "C" int cndp_gpu_host_register(cndp_gpu_ctx_t *c, void *ptr, uint64_t len, void **dev_ptr)
{
    if (!c || !ptr || !len)
        return -EINVAL;
    int r = set_device(c->dev);
    if (r)
        return r;
    pthread_mutex_lock(&g_reg_lock);
    int gi = -1, ci = -1;
    for (int k = 0; k < g_nreg; k++)
        if (g_reg[k].host == (uint8_t *)ptr)
            gi = k;
    for (int k = 0; k < c->n_reg; k++)
        if (c->reg[k].host == (uint8_t *)ptr)
            ci = k;
    if (gi >= 0 && len > g_reg[gi].len) {
        r = -EEXIST; // a different (larger) range at the same address
    } else if (ci < 0 && c->n_reg == CNDP_MAX_REGIONS) {
        r = -ENOSPC;
    } else if (gi < 0) {
        if (g_nreg == (int)(sizeof(g_reg) / sizeof(g_reg[0]))) {
            r = -ENOSPC;
        } else {
            const hipError_t e = hipHostRegister(ptr, len, hipHostRegisterMapped | hipHostRegisterPortable);
            void *d = nullptr;
            if (e == hipSuccess || e == hipErrorHostMemoryAlreadyRegistered) {
                if (hipHostGetDevicePointer(&d, ptr, 0) != hipSuccess) {
                    if (e == hipSuccess)
                        hipHostUnregister(ptr);
                    r = e == hipSuccess ? -EIO : -EEXIST; // registered by the application, unmapped
                }
            } else {
                fprintf(stderr, "cndp_gpu: hipHostRegister failed: %s\n", hipGetErrorString(e));
                r = -ENOMEM;
            }
            if (!r) {
                gi = g_nreg++;
                g_reg[gi] = HostRegion{(uint8_t *)ptr, (uint8_t *)d, len, 0, e == hipSuccess};
            }
        }
    }
    if (!r) {
        g_reg[gi].refs++;
        if (ci < 0) {
            ci = c->n_reg++;
            c->reg[ci].host = g_reg[gi].host;
            c->reg[ci].dev = g_reg[gi].dev;
            c->reg[ci].len = g_reg[gi].len;
            c->reg[ci].refs = 0;
        }
        c->reg[ci].refs++;
        if (dev_ptr)
            *dev_ptr = g_reg[gi].dev;
    }
    pthread_mutex_unlock(&g_reg_lock);
    return r;
}

extern "C" int cndp_gpu_host_unregister(cndp_gpu_ctx_t *c, void *ptr)
{
    if (!c || !ptr)
        return -EINVAL;
    pthread_mutex_lock(&g_reg_lock);
    int ci = -1, gi = -1, r = 0;
    for (int k = 0; k < c->n_reg; k++)
        if (c->reg[k].host == (uint8_t *)ptr)
            ci = k;
    for (int k = 0; k < g_nreg; k++)
        if (g_reg[k].host == (uint8_t *)ptr)
            gi = k;
    if (ci < 0 || gi < 0) {
        r = -ENOENT;
    } else {
        if (--c->reg[ci].refs == 0)
            c->reg[ci] = c->reg[--c->n_reg];
        if (--g_reg[gi].refs == 0) {
            if (g_reg[gi].owned && hipHostUnregister(ptr) != hipSuccess)
                r = -ENOENT;
            g_reg[gi] = g_reg[--g_nreg];
        }
    }
    pthread_mutex_unlock(&g_reg_lock);
    return r;
}

extern "C" int cndp_gpu_bin_ids(cndp_gpu_ctx_t *c, uint32_t mode, const uint32_t *nh,
                                const uint8_t *edge, const uint16_t *queue, uint32_t n,
                                uint32_t n_bins, uint16_t *bin_of_out, void *stream)
{
    if (!c || !bin_of_out || n_bins > CNDP_BINS_MAX)
        return -EINVAL;
    if (mode == CNDP_MODE_HASH ? !queue : (!nh || !edge))
        return -EINVAL;
    if (mode > CNDP_MODE_HASH)
        return -EINVAL;
    int r = set_device(c->dev);
    if (r)
        return r;
    if (n == 0)
        return 0;
    hipLaunchKernelGGL(k_bin_ids, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, mode,
                       nh, edge, queue, n, n_bins, bin_of_out);
    HIP_TRY(hipGetLastError());
    return 0;
}

extern "C" int cndp_gpu_bin_partition(cndp_gpu_ctx_t *c, const uint16_t *bin_of, uint32_t n,
                                      uint32_t n_bins, uint32_t *bin_start, uint32_t *order,
                                      void *stream)
{
    if (!c || !bin_start || n_bins > CNDP_BINS_MAX || (n && (!bin_of || !order)))
        return -EINVAL;
    int r = set_device(c->dev);
    if (r)
        return r;
    const uint32_t nbt = n_bins + 2;
    const uint32_t tiles = n ? blocks_for(n, PART_TILE) : 1;
    const size_t need = (size_t)nbt * tiles;
    if (need > c->part_cap) {
        if (c->d_part)
            HIP_TRY(hipFree(c->d_part));
        c->d_part = nullptr;
        c->part_cap = 0;
        HIP_TRY(hipMalloc((void **)&c->d_part, need * 4));
        c->part_cap = need;
    }
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(bin_start, 0, (size_t)(nbt + 1) * 4, s));
        return 0;
    }
    if ((r = scratch_acquire(c, s)))
        return r;
    hipLaunchKernelGGL(k_part_hist, dim3(tiles), dim3(PART_THREADS), 0, s, bin_of, n, nbt, tiles,
                       c->d_part);
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(1024), 0, s, c->d_part, (uint32_t)need, tiles, nbt,
                       bin_start);
    hipLaunchKernelGGL(k_part_scatter, dim3(tiles), dim3(PART_THREADS), 0, s, bin_of, n, nbt, tiles,
                       c->d_part, order);
    HIP_TRY(hipGetLastError());
    return scratch_release(c, s);
}

// ---------------------------------------------------------------------------
// Asynchronous node path over pktmbuf_t bursts (cndp_gpu_mq_*, cndp_gpu.h).
//
// Bursts fill the open batch slot on the host; a full slot -- or, at poll
// time, a partly filled one when nothing is in flight or it has waited
// max_delay_us -- is launched on the queue's stream.  Every host buffer a
// slot uses is pinned and mapped, so the kernels read their inputs and write
// their outputs in host memory directly: no DMA calls per batch.
//   zero-copy (conf.umem): the host only copies the burst's mbuf pointers.
//     The kernels read each mbuf's header (buf_addr, data_off, ...) and its
//     frame in the registered region over PCIe, and write the fields the
//     replaced nodes write straight into the mbuf.
//   staged: the host gathers each frame's bytes (and header fields) into the
//     slot's pinned staging; the kernels read that and return compact
//     records, which poll writes into the mbufs.
// The batch's last kernel ends with a completion flag: each block makes its
// host writes visible system-wide (__threadfence_system), the last block to
// arrive (device ticket) stores the batch sequence number into the slot's
// pinned flag.  poll is a plain acquire load of that flag -- no HIP call.
// ---------------------------------------------------------------------------
#define MQ_FREE 0
#define MQ_OPEN 1
#define MQ_FLIGHT 2
#define MQ_DONE 3
#define MQ_BURST 256u       // CNE_GRAPH_BURST_SIZE (cne_graph.h:30)
#define MQ_W4_AT 20u        // ip4_lookup reads bytes 22..33 (ttl, checksum, dst): the window 20..35
#define MQ_W4 16u
#define MQ_W4R_AT 12u       // ip4_lookup with CNDP_MQ_F_RX_PARSE: the ethertype too, the window 12..35
#define MQ_W4R 24u
#define MQ_SWAP 16u         // mac swap: staged bytes (it touches 0..11)
#define MQ_RW_STAGE 64u     // ip4_rewrite: staged bytes (rewrite data <= 56, TTL / checksum at 22..25)
#define MQ_RUNS_MAX 512u    // cnet: runs of equal-size bursts per batch
#define MQ_EDGE_NONE 0xFFFFu // zero-copy: an mbuf or frame outside every registered region
#define MQ_SHORT 128u       // cnet staged bytes of a frame whose parse stays in its first 128
#define MQ_PF 32u           // mbufs prefetched ahead in the host loops (8 / 16 / 32 swept: tools/pf_sweep.sh)
#define MQ_ADDR_MASK ((1ull << 56) - 1ull) // frame word: device address | readable bytes (<= 255) << 56
#define MQ_RW_TAIL 1ull     // ip4_rewrite: the frame takes the tail loop's checksum rule
#define MQ_MD_LEN 40u       // struct cnet_metadata {faddr, laddr} (cnet_meta.h:20-25, cne_inet.h:37-45)
#define CNDP_MQ_POOLS 4u    // cnet device headers: pools whose pktmbuf_metadata is the default m + 64
#define MQ_AF_INET 2u
#define MQ_AF_INET6 10u

// Staged cnet: whether a frame's bytes past its first MQ_SHORT can matter.
// cne_get_ptype (pktmbuf_ptype.c:472-615) stops early for ARP and MPLS, and
// after Ethernet (at most one VLAN / QinQ tag), IPv4 (any IHL; a fragment
// stops there) or IPv6 without extension headers, and TCP / UDP / SCTP: it
// reads below l2 (<= 22) + l3 (<= 60) + 13 < 128, and so do the input nodes
// (ip4_input.c / ip6_input.c: the IP header) and the flow hash (the tuple).
// Every other frame -- extension headers, tunnels, and the protocols the
// inner-header walk picks up by their raw value -- gets the whole buffer (up
// to stage_max), so the staged bytes never change a result.
static inline bool mq_short_reach(const uint8_t *f, uint32_t room)
{
    if (room <= MQ_SHORT)
        return true; // the whole buffer fits anyway
    uint32_t et = ((uint32_t)f[12] << 8) | f[13], l2 = 14;
    if (et == 0x0806u || et == 0x8847u || et == 0x8848u) // ARP, MPLS
        return true;
    if (et == 0x8100u) {
        et = ((uint32_t)f[16] << 8) | f[17];
        l2 = 18;
    } else if (et == 0x88A8u) {
        et = ((uint32_t)f[20] << 8) | f[21];
        l2 = 22;
    }
    uint32_t proto;
    if (et == 0x0800u) {
        if (((((uint32_t)f[l2 + 6] << 8) | f[l2 + 7]) & 0x3fffu) != 0)
            return true; // a fragment: no L4 read
        proto = f[l2 + 9];
    } else if (et == 0x86DDu) {
        proto = f[l2 + 6];
    } else {
        return false;
    }
    return proto == 6u || proto == 17u || proto == 132u;
}

// pktmbuf_t fields (pktmbuf.h:102-204)
#define MB_LPORT 26
#define MB_DATA_LEN 30
#define MB_TX_OFFLOAD 40
#define MB_OL_FLAGS 48

struct MqTables {
    const uint32_t *t24, *t8, *d16, *pages, *t24_6, *t8_6;
    uint32_t buf_len;
};

// Per-mbuf inputs are host-filled pinned arrays (read by the kernels over
// PCIe as coalesced runs): the host has each mbuf's header line in cache
// anyway -- the node that hands the burst over just touched it -- so it
// resolves the frame address there and the kernels read only frame bytes in
// place (one PCIe read per frame instead of three dependent ones).
struct MqArgs {
    uint32_t n;
    uint32_t zc;            // zero-copy: frames read and fields written in the registered regions
    const uint64_t *mb;     // zc: device address of each mbuf (0: outside every region); rewrite: MQ_RW_TAIL
    const uint64_t *off;    // zc ip4 / swap / rewrite: frame word (device address | readable << 56, 0: none)
                            // zc cnet: frame offset in the batch's region; staged: offset in the staging
    const u32x2 *lens;      // cnet: {data_len | room << 16, buf_len | data_off << 16}
    const uint64_t *priv;   // rewrite: node_mbuf_priv1 (udata64) as ip4_lookup left it
    const uint64_t *md;     // cnet zc: device address of pktmbuf_metadata(m) (0: poll writes it)
    const uint8_t *slab;    // cnet zc: the batch's region (device view); staged: the staging
    uint64_t slab_len;
    uint16_t *edges;        // out: next edge per mbuf (pinned host)
    uint64_t *priv1;        // out (staged ip4_lookup, and zc with hostwb): node_mbuf_priv1 (pkt_cls drops: packet_type)
    u32x4 *rec;             // out (staged cnet, and zc with hostwb): {ptype, rxmeta, data_len | edge << 16 | node << 24, hash}
    u32x4 *rec_md;          // out (zc cnet, hostwb): per mbuf the source and destination address (2 x 16 B)
    uint32_t hostwb;        // zc cnet / ip4_lookup, CNDP_MQ_F_HOST_WRITEBACK: results as records, poll writes the mbufs
    // cnet classify outputs (device)
    const uint32_t *ptype, *rxmeta, *hash;
    const uint8_t *edge8;
    uint32_t *iplen;        // cnet: the IP length fields the parse read (0: read the frame); cleared here
    const u32x4 *win;       // cnet: each fast-parsed or general-parsed frame's first 64 bytes
    const struct cndp_rw_nh *rw; // rewrite: next-hop table (device)
    uint32_t lport, want_hash;
    uint32_t rxparse;       // ip4_lookup, CNDP_MQ_F_RX_PARSE: pktdev_rx's soft parse + pkt_cls first
    const uint32_t *bstart; // CNDP_MQ_F_REWRITE: each submitted burst's first mbuf, then n
    uint32_t devhdr;        // zc, CNDP_MQ_F_DEVICE_HEADERS: the kernels read each mbuf's header
    uint32_t nrg;           //   themselves; ip4_lookup: its frame lies in one of the nrg registered
    struct {                //   regions (host address range, device = host + delta); cnet: rg[0]
        uint64_t host, len; //   is the batch's region
        int64_t delta;
    } rg[CNDP_MAX_REGIONS];
    // cnet with device headers (k_mq_cnet_hdr): the frame offsets, length
    // fields and metadata addresses it derives (device arrays, the metadata
    // addresses also into the pinned array poll reads); pktmbuf_metadata is
    // m + 64 for the mbufs of md_pool[0..n_pool) (all of them with md_all)
    uint64_t *w_off;
    u32x2 *w_lens;
    uint64_t *w_md, *w_mdh;
    uint32_t n_pool, md_all;
    uint64_t md_pool[CNDP_MQ_POOLS];
    MqTables tb;
    uint32_t *ticket;       // device arrival counter of this slot
    uint32_t *flag;         // device view of the slot's pinned completion flag
    uint32_t seq;           // value the flag takes when the batch is done
};

// every block: its host writes visible, then the last block raises the flag
__device__ __forceinline__ void mq_complete(const MqArgs &a)
{
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = atomicAdd(a.ticket, 1u);
        if (t == gridDim.x - 1) {
            *a.ticket = 0u; // ready for the slot's next batch (stream order)
            __threadfence_system();
            __hip_atomic_store(a.flag, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// a zero-copy frame word: the frame's device address and how many bytes
// from there lie inside its registered region (capped at 255)
__device__ __forceinline__ uint8_t *mq_frame(uint64_t w, uint32_t &avail)
{
    avail = (uint32_t)(w >> 56);
    return (uint8_t *)(uintptr_t)(w & MQ_ADDR_MASK);
}

// node-queue kernels: one wave per block, so a batch spreads over 4x the CUs
// (in place, each mbuf costs a PCIe round trip; more CUs keep more in flight)
#define MQ_TPB 64u

// ip4_rewrite_node_process's work on one frame p (avail readable bytes) from
// its node_mbuf_priv1 pv (ip4_rewrite.c:85-110, :201-216): the next hop's
// rewrite data at mtod, TTL = priv1.ttl - 1 and the checksum from
// priv1.cksum + htons(0x0100) -- the 4-wide loop's u32 end-around carry, or
// with `tail` the tail loop's u16 `chksum += chksum >= 0xffff`.  Returns the
// next hop's tx_node; next hops past the reference's 64-entry array act as
// unset entries (no data, tx node 0).
__device__ __forceinline__ uint32_t mq_rewrite_frame(uint8_t *p, uint32_t avail, uint64_t pv, bool tail,
                                                     const struct cndp_rw_nh *rw)
{
    const uint32_t nh = (uint32_t)(pv & 0xffffu), ttl = (uint32_t)(pv >> 16) & 0xffffu;
    const uint32_t ck32 = (uint32_t)(pv >> 32);
    const bool set = nh < CNDP_RW_MAX_NH;
    const struct cndp_rw_nh *e = &rw[set ? nh : 0u];
    const uint32_t hdr = set ? *(const uint32_t *)e : 0u; // rewrite_len | tx_node << 16
    uint32_t len = hdr & 0xffffu;
    len = len < CNDP_RW_MAX_LEN ? len : CNDP_RW_MAX_LEN;
    const uint32_t *src = (const uint32_t *)e->rewrite_data;
    if (len == 12u && len <= avail && (((uintptr_t)p) & 3u) == 0) { // the usual MAC pair: one store
        *(u32x3a4 *)p = (u32x3a4){src[0], src[1], src[2]};
    } else if (len <= avail && (((uintptr_t)p) & 3u) == 0 && (len & 3u) == 0) {
        for (uint32_t k = 0; k < len / 4; k++)
            ((uint32_t *)p)[k] = src[k];
    } else {
        for (uint32_t k = 0; k < len && k < avail; k++)
            p[k] = e->rewrite_data[k];
    }
    uint32_t nck;
    if (!tail) {
        const uint32_t c32 = ck32 + 1u;
        nck = ((c32 & 0xffffu) + (c32 >> 16)) & 0xffffu;
    } else {
        const uint32_t c16 = (ck32 + 1u) & 0xffffu;
        nck = (c16 + (c16 >= 0xffffu ? 1u : 0u)) & 0xffffu;
    }
    if (avail > 22)
        p[22] = (uint8_t)(ttl - 1u);
    if (avail > 25 && (((uintptr_t)p) & 1u) == 0) {
        *(uint16_t *)(p + 24) = (uint16_t)nck;
    } else {
        if (avail > 24)
            p[24] = (uint8_t)nck;
        if (avail > 25)
            p[25] = (uint8_t)(nck >> 8);
    }
    return hdr >> 16;
}

// the same with the frame's bytes 20..27 already in registers (the lookup's
// one-load window, p 4-aligned, avail > 35): the new TTL and checksum go out
// with the bytes around them unchanged as one 8-B store at p + 20, and the
// usual 12-B rewrite data as one 12-B store -- two PCIe writes per frame
// instead of five (each store of a lane is a transaction of its own in place)
__device__ __forceinline__ uint32_t mq_rewrite_frame_w(uint8_t *p, uint32_t avail, uint64_t pv, bool tail,
                                                       const struct cndp_rw_nh *rw, uint32_t w20, uint32_t w24)
{
    const uint32_t nh = (uint32_t)(pv & 0xffffu), ttl = (uint32_t)(pv >> 16) & 0xffffu;
    const uint32_t ck32 = (uint32_t)(pv >> 32);
    const bool set = nh < CNDP_RW_MAX_NH;
    const struct cndp_rw_nh *e = &rw[set ? nh : 0u];
    const uint32_t hdr = set ? *(const uint32_t *)e : 0u; // rewrite_len | tx_node << 16
    uint32_t len = hdr & 0xffffu;
    len = len < CNDP_RW_MAX_LEN ? len : CNDP_RW_MAX_LEN;
    const uint32_t *src = (const uint32_t *)e->rewrite_data;
    if (len == 12u) {
        *(u32x3a4 *)p = (u32x3a4){src[0], src[1], src[2]};
    } else if (len <= avail && (len & 3u) == 0) {
        for (uint32_t k = 0; k < len / 4; k++)
            ((uint32_t *)p)[k] = src[k];
    } else {
        for (uint32_t k = 0; k < len && k < avail; k++)
            p[k] = e->rewrite_data[k];
    }
    uint32_t nck;
    if (!tail) {
        const uint32_t c32 = ck32 + 1u;
        nck = ((c32 & 0xffffu) + (c32 >> 16)) & 0xffffu;
    } else {
        const uint32_t c16 = (ck32 + 1u) & 0xffffu;
        nck = (c16 + (c16 >= 0xffffu ? 1u : 0u)) & 0xffffu;
    }
    // rewrite data longer than 20 bytes covers some of bytes 20..27: those
    // bytes are the data's (the reference then writes TTL / checksum over it)
    if (len > 20u) {
        const uint32_t m20 = len >= 24u ? ~0u : (1u << (8u * (len - 20u))) - 1u;
        w20 = (src[5] & m20) | (w20 & ~m20);
        if (len > 24u) {
            const uint32_t m24 = len >= 28u ? ~0u : (1u << (8u * (len - 24u))) - 1u;
            w24 = (src[6] & m24) | (w24 & ~m24);
        }
    }
    *(u32x2a4 *)(p + 20) = (u32x2a4){(w20 & 0xff00ffffu) | (((ttl - 1u) & 0xffu) << 16),
                                     (w24 & 0xffff0000u) | nck};
    return hdr >> 16;
}

// ip4_lookup_node_process_vec, per packet (ip4_lookup.c:108-154): dip at
// mtod + 14 + 16, priv1 = {nh = val & 0xffff, ttl, hdr_checksum}, edge = val >> 16
// one mbuf through the queue's ip4_lookup mode: the frame's readable
// window, with CNDP_MQ_F_RX_PARSE the soft parse and pkt_cls first, then the
// lookup and node_mbuf_priv1 (written into the mbuf, or the record when
// staged).  Zero-copy also hands back the frame (mtod) and its readable bytes
// (<= 255) for a rewrite.
#define MQ_L3_NONE 0u   // the mbuf or its frame is outside every registered region
#define MQ_L3_CLS 1u    // pkt_cls sent it to pkt_drop (not IPv4)
#define MQ_L3_LOOKED 2u // ip4_lookup ran: val
struct MqL3 {
    uint32_t st, val;
    uint64_t priv1;
    uint8_t *frame;
    uint32_t favail;
    uint32_t w20, w24; // zero-copy, one-load window: frame bytes 20..27 (else w20 = w24 = 0, q16 false)
    bool q16;
};
__device__ __forceinline__ MqL3 mq_l3_one(const MqArgs &a, uint32_t i)
{
    MqL3 r{MQ_L3_NONE, 0u, 0ull, nullptr, 0u, 0u, 0u, false};
    const uint64_t w = a.devhdr ? 0u : a.off[i];
    const uint8_t *p; // bytes 20..35 of the frame
    uint32_t avail;   // readable bytes from p
    uint32_t eavail;  // readable bytes from the ethertype (frame byte 12, p - 8)
    uint64_t m = 0;
    if (a.zc && a.devhdr) {
        m = a.mb[i];
        const uint8_t *dm = (const uint8_t *)(uintptr_t)m;
        const uint64_t buf = m ? *gp((const uint64_t *)(dm + MB_BUF_ADDR)) : 0u;
        const uint32_t doff = m ? *gp((const uint16_t *)(dm + MB_DATA_OFF)) : 0u;
        const uint64_t fh = buf + doff; // pktmbuf_mtod, a host address
        uint64_t fo = ~0ull, rlen = 0;
        int64_t delta = 0;
        for (uint32_t k = 0; k < a.nrg; k++) // the frame's registered region
            if (fh - a.rg[k].host < a.rg[k].len) {
                fo = fh - a.rg[k].host;
                rlen = a.rg[k].len;
                delta = a.rg[k].delta;
                break;
            }
        if (m == 0 || fo == ~0ull)
            return r;
        r.frame = (uint8_t *)(uintptr_t)(fh + delta);
        r.favail = rlen - fo < 255u ? (uint32_t)(rlen - fo) : 255u;
        p = r.frame + MQ_W4_AT;
        avail = rlen - fo > MQ_W4_AT + 16 ? 16u : (uint32_t)(rlen - fo > MQ_W4_AT ? rlen - fo - MQ_W4_AT : 0);
        eavail = rlen - fo > MQ_W4R_AT + 2 ? 2u : (uint32_t)(rlen - fo > MQ_W4R_AT ? rlen - fo - MQ_W4R_AT : 0);
    } else if (a.zc) {
        m = a.mb[i];
        uint32_t fa;
        uint8_t *f = mq_frame(w, fa);
        if (m == 0 || f == nullptr)
            return r;
        r.frame = f;
        r.favail = fa;
        p = f + MQ_W4_AT;
        avail = fa > MQ_W4_AT ? fa - MQ_W4_AT : 0u;
        eavail = fa > MQ_W4R_AT ? fa - MQ_W4R_AT : 0u;
    } else { // staged: the window from MQ_W4R_AT with the soft parse, else from MQ_W4_AT
        p = a.slab + w + (a.rxparse ? MQ_W4_AT - MQ_W4R_AT : 0u);
        avail = MQ_W4;
        eavail = 2u;
    }
    if (a.rxparse) {
        // pktdev_rx's eth_pkt_parse_cb (pktdev_rx.c:24-34, :88-100):
        // packet_type = l3_ptype(ether_type, 0); then pkt_cls
        // (pkt_cls.c:19-31): only IPv4 (0x90) goes on to ip4_lookup
        const uint8_t *e = p - (MQ_W4_AT - MQ_W4R_AT);
        const uint32_t et = eavail >= 2 ? ((uint32_t)gbyte(e, eavail, 0) << 8) | gbyte(e, eavail, 1) : 0u;
        const uint32_t pt = et == 0x0800u ? 0x90u : et == 0x86DDu ? 0xE0u : 0u;
        if (a.zc && !a.hostwb)
            *gp((uint32_t *)(m + MB_PTYPE)) = pt;
        if (pt != 0x90u) {
            if (a.hostwb) // the record of a frame pkt_cls drops carries its packet_type
                a.priv1[i] = pt;
            r.st = MQ_L3_CLS;
            return r;
        }
    }
    uint32_t ttl, ck, dip;
    if (avail >= 16 && (((uintptr_t)p) & 3u) == 0 && (((uintptr_t)p) & 63u) <= 48u) {
        // ttl, checksum and dst in one load inside one 64-B line: the
        // frame's only PCIe read when it is read in place
        const u32x4a4 q = *(const GAS u32x4a4 *)p;
        ttl = (q.x >> 16) & 0xffu;
        ck = q.y & 0xffffu;
        dip = bswap32(alignb(q.w, q.z, 2));
        r.w20 = q.x;
        r.w24 = q.y;
        r.q16 = a.zc != 0;
    } else {
        ttl = gbyte(p, avail, 2);
        ck = gbyte(p, avail, 4) | (gbyte(p, avail, 5) << 8);
        dip = (gbyte(p, avail, 10) << 24) | (gbyte(p, avail, 11) << 16) | (gbyte(p, avail, 12) << 8) |
              gbyte(p, avail, 13);
    }
    r.val = a.tb.d16 ? lpm4d(a.tb.d16, a.tb.pages, a.tb.t8, dip) : lpm4(a.tb.t24, a.tb.t8, dip);
    r.priv1 = (uint64_t)(r.val & 0xffffu) | ((uint64_t)ttl << 16) | ((uint64_t)ck << 32);
    if (a.zc && !a.hostwb)
        *gp((uint64_t *)(m + MB_UDATA64)) = r.priv1;
    else // staged, or CNDP_MQ_F_HOST_WRITEBACK: a coalesced record poll writes into the mbuf
        a.priv1[i] = r.priv1;
    r.st = MQ_L3_LOOKED;
    return r;
}

__global__ __launch_bounds__(MQ_TPB) void k_mq_ip4_lookup(MqArgs a)
{
    for (uint32_t i = blockIdx.x * MQ_TPB + threadIdx.x; i < a.n; i += gridDim.x * MQ_TPB) {
        const MqL3 r = mq_l3_one(a, i);
        a.edges[i] = (uint16_t)(r.st == MQ_L3_NONE  ? MQ_EDGE_NONE
                                : r.st == MQ_L3_CLS ? CNDP_MQ_EDGE_CLS_DROP
                                                    : r.val >> 16);
    }
    mq_complete(a);
}

// CNDP_MQ_F_REWRITE: one block per submitted burst (<= MQ_BURST mbufs), the
// lookup of every mbuf, then ip4_rewrite_node_process (ip4_rewrite.c:40-247)
// over the ones ip4_lookup sent to it, in burst order: a block-wide rank among
// them picks the 4-wide loop's checksum rule for the first (count & ~3) and
// the tail loop's for the rest, as when ip4_rewrite gets the burst's stream in
// one call; the rewrite goes into the frame where it lies (zero-copy only).
#define MQ_L3_TPB MQ_BURST
__global__ __launch_bounds__(MQ_L3_TPB) void k_mq_l3fwd_burst(MqArgs a)
{
    __shared__ uint32_t s_w[MQ_L3_TPB / 64];
    const uint32_t i0 = a.bstart[blockIdx.x], i1 = a.bstart[blockIdx.x + 1];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint32_t i = i0 + t;
    const bool in = i < i1;
    MqL3 r{MQ_L3_NONE, 0u, 0ull, nullptr, 0u, 0u, 0u, false};
    if (in)
        r = mq_l3_one(a, i);
    const bool to_rw = in && r.st == MQ_L3_LOOKED && (r.val >> 16) == 0u; // CNE_NODE_IP4_LOOKUP_NEXT_REWRITE
    const unsigned long long bal = __ballot(to_rw);
    if (lane == 0)
        s_w[wv] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t before = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull)), total = 0;
    for (uint32_t k = 0; k < MQ_L3_TPB / 64; k++) {
        before += k < wv ? s_w[k] : 0u;
        total += s_w[k];
    }
    if (in) {
        uint32_t e;
        if (r.st == MQ_L3_NONE)
            e = MQ_EDGE_NONE;
        else if (r.st == MQ_L3_CLS)
            e = CNDP_MQ_EDGE_CLS_DROP;
        else if (!to_rw)
            e = CNDP_MQ_EDGE_LOOKUP_DROP;
        else if (r.q16)
            e = mq_rewrite_frame_w(r.frame, r.favail, r.priv1, before >= (total & ~3u), a.rw, r.w20, r.w24);
        else
            e = mq_rewrite_frame(r.frame, r.favail, r.priv1, before >= (total & ~3u), a.rw);
        a.edges[i] = (uint16_t)e;
    }
    mq_complete(a);
}

// cndpfwd _loopback_test (examples/cndpfwd/main.c:317-339): MAC_SWAP =
// swap_mac_addresses (main.h:303-315) at pktmbuf_mtod of every mbuf, then tx.
// Zero-copy: in the frame where it lies; staged: in the staged window, which
// poll copies back.  Every mbuf leaves by edge 0 (tx).
__global__ __launch_bounds__(MQ_TPB) void k_mq_mac_swap(MqArgs a)
{
    for (uint32_t i = blockIdx.x * MQ_TPB + threadIdx.x; i < a.n; i += gridDim.x * MQ_TPB) {
        uint8_t *p;
        uint32_t avail;
        if (a.zc) {
            p = mq_frame(a.off[i], avail);
        } else {
            p = (uint8_t *)a.slab + a.off[i];
            avail = MQ_SWAP;
        }
        const bool ok = p != nullptr && avail >= 12;
        if (ok) {
            if ((((uintptr_t)p) & 3u) == 0) {
                uint32_t *d = (uint32_t *)p;
                const uint32_t d0 = d[0], d1 = d[1], d2 = d[2];
                d[0] = alignb(d2, d1, 2);       // bytes 6..9
                d[1] = (d2 >> 16) | (d0 << 16); // bytes 10, 11, 0, 1
                d[2] = alignb(d1, d0, 2);       // bytes 2..5
            } else {
                for (int k = 0; k < 6; k++) {
                    const uint8_t t = p[k];
                    p[k] = p[6 + k];
                    p[6 + k] = t;
                }
            }
        }
        a.edges[i] = ok || !a.zc ? (uint16_t)0 : (uint16_t)MQ_EDGE_NONE;
    }
    mq_complete(a);
}

// ip4_rewrite_node_process (ip4_rewrite.c:40-247) per packet of the node's
// bursts: the next hop's rewrite data at mtod (:85), TTL = priv1.ttl - 1 and
// the checksum from priv1.cksum + htons(0x0100) -- in the 4-wide loop with
// the u32 end-around carry (:97-104, :109-110), in the tail loop as a u16
// with `chksum += chksum >= 0xffff` (:209-216); the host marks which frames
// of each burst the tail loop takes (the last nb_objs % 4).  edge = the next
// hop's tx_node (ip4_rewrite_set_next / cne_node_ip4_rewrite_add); next hops
// past the reference's 64-entry array act as unset entries (no data, edge 0).
__global__ __launch_bounds__(MQ_TPB) void k_mq_ip4_rewrite(MqArgs a)
{
    for (uint32_t i = blockIdx.x * MQ_TPB + threadIdx.x; i < a.n; i += gridDim.x * MQ_TPB) {
        const bool tail = (a.mb[i] & MQ_RW_TAIL) != 0u;
        uint8_t *p;
        uint32_t avail;
        uint64_t pv;
        if (a.devhdr) { // the mbuf's device address | tail flag: its header read here
            const uint64_t m = a.mb[i] & ~MQ_RW_TAIL;
            uint64_t fh = 0, fo = ~0ull, rlen = 0;
            int64_t delta = 0;
            if (m) {
                const uint8_t *dm = (const uint8_t *)(uintptr_t)m;
                fh = *gp((const uint64_t *)(dm + MB_BUF_ADDR)) + *gp((const uint16_t *)(dm + MB_DATA_OFF));
                for (uint32_t k = 0; k < a.nrg; k++) // the frame's registered region
                    if (fh - a.rg[k].host < a.rg[k].len) {
                        fo = fh - a.rg[k].host;
                        rlen = a.rg[k].len;
                        delta = a.rg[k].delta;
                        break;
                    }
            }
            if (fo == ~0ull) {
                a.edges[i] = (uint16_t)MQ_EDGE_NONE;
                continue;
            }
            pv = *gp((const uint64_t *)((const uint8_t *)(uintptr_t)m + MB_UDATA64)); // node_mbuf_priv1
            p = (uint8_t *)(uintptr_t)(fh + delta);
            avail = rlen - fo < 255u ? (uint32_t)(rlen - fo) : 255u;
            a.edges[i] = (uint16_t)mq_rewrite_frame(p, avail, pv, tail, a.rw);
            continue;
        }
        pv = a.priv[i];
        if (a.zc) {
            p = mq_frame(a.off[i], avail);
            if (p == nullptr) {
                a.edges[i] = (uint16_t)MQ_EDGE_NONE;
                continue;
            }
        } else {
            p = (uint8_t *)a.slab + a.off[i];
            avail = MQ_RW_STAGE;
        }
        a.edges[i] = (uint16_t)mq_rewrite_frame(p, avail, pv, tail, a.rw);
    }
    mq_complete(a);
}

// A frame an input node takes is re-evaluated here when the batch-wide
// classify could not see its case: eth_rx's pktmbuf_adj_offset(l2_len) was
// skipped (l2_len > data_len: the node then reads its IP header at the frame
// start, pktmbuf.h:955-984) or its buf_len differs from the batch's (the
// length test, ip4_input.c:121-140 / ip6_input.c:121-135).
__device__ uint32_t mq_input_at(const uint8_t *slab, uint64_t slab_len, uint64_t o, bool v6, const MqTables &t,
                                uint32_t buf_len)
{
    if (!v6) {
        const uint32_t x0 = gld32(slab, slab_len, o);
        const uint32_t hl = x0 & 0xfu;
        uint32_t sum = 0;
        for (uint32_t k = 0; k < hl; k++) {
            const uint32_t x = k == 0 ? x0 : gld32(slab, slab_len, o + 4 * k);
            sum += (x & 0xffffu) + (x >> 16);
        }
        sum = (sum >> 16) + (sum & 0xffffu);
        sum = (sum >> 16) + (sum & 0xffffu);
        const bool ok = bswap16(x0 >> 16) < buf_len && ((~sum) & 0xffffu) == 0u;
        const uint32_t dip = ok ? bswap32(gld32(slab, slab_len, o + 16)) : 0u;
        return t.d16 ? lpm4d(t.d16, t.pages, t.t8, dip) : lpm4(t.t24, t.t8, dip);
    }
    const bool ok = ((gbyte(slab, slab_len, o + 4) << 8) | gbyte(slab, slab_len, o + 5)) < buf_len;
    uint32_t e = t.t24_6[ok ? (gbyte(slab, slab_len, o + 24) << 16) | (gbyte(slab, slab_len, o + 25) << 8) |
                                  gbyte(slab, slab_len, o + 26)
                            : 0u];
    for (uint32_t j = 3; (e & 1u) && j < 16; j++)
        e = t.t8_6[(e >> 1) * 256u + (ok ? gbyte(slab, slab_len, o + 24 + j) : 0u)];
    return e >> 1;
}

// the 4 frame bytes at o (< 61) of a saved 64-B window, little-endian
__device__ __forceinline__ uint32_t mq_win32(const u32x4 *w, uint32_t o)
{
    const uint32_t *d = (const uint32_t *)w;
    const uint32_t k = o >> 2, s = o & 3u;
    return s ? alignb(d[k + 1], d[k], s) : d[k];
}

// ipv4_save_metadata / ipv6_save_metadata (ip4_input.c:33-48, ip6_input.c:32-48)
// for a frame whose IP header sits at byte ip of its window: faddr / laddr
// {cin_family, cin_len, ..., address} at pktmbuf_metadata(m); cin_port and
// the rest of the address union are left as they were, as there.
__device__ void mq_save_md(uint8_t *d, const u32x4 *w, const uint8_t *fr, uint64_t favail, uint32_t ip, bool v6)
{
    const uint32_t na = v6 ? 4u : 1u, s_at = ip + (v6 ? 8u : 12u), d_at = ip + (v6 ? 24u : 16u);
    uint32_t sa[4], da[4];
    const bool inwin = d_at + 4u * na <= 64u;
    for (uint32_t k = 0; k < na; k++) {
        sa[k] = inwin ? mq_win32(w, s_at + 4 * k) : gld32(fr, favail, s_at + 4 * k);
        da[k] = inwin ? mq_win32(w, d_at + 4 * k) : gld32(fr, favail, d_at + 4 * k);
    }
    const uint32_t fl = v6 ? (MQ_AF_INET6 | (16u << 8)) : (MQ_AF_INET | (4u << 8));
    if ((((uintptr_t)d) & 3u) == 0) {
        *(uint16_t *)d = (uint16_t)fl;
        *(uint16_t *)(d + 20) = (uint16_t)fl;
        if (v6) {
            *(u32x4a4 *)(d + 4) = (u32x4a4){sa[0], sa[1], sa[2], sa[3]};
            *(u32x4a4 *)(d + 24) = (u32x4a4){da[0], da[1], da[2], da[3]};
        } else {
            *(uint32_t *)(d + 4) = sa[0];
            *(uint32_t *)(d + 24) = da[0];
        }
    } else {
        d[0] = d[20] = (uint8_t)fl;
        d[1] = d[21] = (uint8_t)(fl >> 8);
        for (uint32_t k = 0; k < 4 * na; k++) {
            d[4 + k] = (uint8_t)(sa[k >> 2] >> (8 * (k & 3u)));
            d[24 + k] = (uint8_t)(da[k >> 2] >> (8 * (k & 3u)));
        }
    }
}

// cnet results per mbuf.  Frames an input node took get data_len =
// total_length (ip4_input.c:121-124) or payload_len (ip6_input.c:121-124),
// read at mtod after eth_rx's pktmbuf_adj_offset(l2_len) (eth_rx.c:62), and
// their cnet_metadata addresses (ipv4/ipv6_save_metadata).  Which input node:
// ip4_input for the low ptype bytes of its p_nxt entries (0x11, 0x31, 0x91),
// ip6_input for 0x41, 0xc1, 0xe1 -- the ptype node's speculation only sends a
// frame to the edge of a type with the same low byte (ptype.c:109-110).
// Zero-copy: the eth_rx fields (eth_rx.c:35-63), data_len and the metadata go
// straight into the mbuf; staged: into records for poll.
// cnet with CNDP_MQ_F_DEVICE_HEADERS: what mq_fill derives on the host from
// each mbuf's header line, read here instead (one 32-B read per mbuf: pooldata,
// buf_addr, data_off, buf_len, data_len, pktmbuf.h:102-112) -- the frame's
// offset in the batch's region (its end when outside), the length fields, and
// the metadata address when the mbuf's pool keeps it at m + 64
// (pktmbuf_metadata's default, pktmbuf.h:1209-1220); else 0, and poll writes
// the metadata through conf.metadata
__global__ __launch_bounds__(MQ_TPB) void k_mq_cnet_hdr(MqArgs a)
{
    const uint64_t host = a.rg[0].host, len = a.rg[0].len;
    for (uint32_t i = blockIdx.x * MQ_TPB + threadIdx.x; i < a.n; i += gridDim.x * MQ_TPB) {
        const uint64_t m = a.mb[i];
        uint64_t fo = len, md = 0;
        u32x2 l = {0u, 0u};
        if (m) {
            const u32x4 h0 = *gp((const u32x4 *)(uintptr_t)m);        // pooldata, buf_addr
            const u32x4 h1 = *gp((const u32x4 *)(uintptr_t)(m + 16)); // hash, meta_index, data_off .. data_len
            const uint64_t pool = (uint64_t)h0.x | ((uint64_t)h0.y << 32);
            const uint64_t buf = (uint64_t)h0.z | ((uint64_t)h0.w << 32);
            const uint32_t doff = h1.z & 0xffffu, blen = h1.w & 0xffffu, dlen = h1.w >> 16;
            const uint32_t room = blen > doff ? blen - doff : 0u;
            const uint64_t f = buf + doff; // pktmbuf_mtod, a host address
            if (f - host < len)
                fo = f - host;
            l.x = dlen | (room << 16);
            l.y = blen | (doff << 16);
            bool def = a.md_all != 0u;
            for (uint32_t k = 0; k < a.n_pool; k++)
                def = def || pool == a.md_pool[k];
            md = def ? m + 64u : 0u;
        }
        a.w_off[i] = fo;
        a.w_lens[i] = l;
        if (a.w_md) {
            a.w_md[i] = md;
            a.w_mdh[i] = md; // pinned: poll's writeback reads it
        }
    }
    __threadfence_system();
}

__global__ __launch_bounds__(MQ_TPB) void k_mq_cnet_post(MqArgs a)
{
    for (uint32_t i = blockIdx.x * MQ_TPB + threadIdx.x; i < a.n; i += gridDim.x * MQ_TPB) {
        const uint32_t pt = a.ptype[i], rm = a.rxmeta[i], e8 = a.edge8[i];
        const u32x2 ln = a.lens[i];
        uint32_t ipl = 0;
        if (a.iplen) { // consumed: the next batch's fast path writes only its own frames
            ipl = a.iplen[i];
            if (ipl)
                a.iplen[i] = 0u;
        }
        const uint32_t dl = ln.x & 0xffffu, room = ln.x >> 16, blen = ln.y & 0xffffu, doff = ln.y >> 16;
        const uint32_t l2 = rm & 0x7fu;
        const bool adj = l2 <= dl && l2 <= room;
        const uint64_t fo = a.off[i];
        uint32_t node, e, dlen = adj ? dl - l2 : dl;
        bool v6 = false;
        if (e8 & 0x80u) {
            node = CNDP_MQ_NODE_PTYPE;
            e = e8 & 0x7fu;
        } else {
            const uint32_t low = pt & 0xffu;
            v6 = low == 0x41u || low == 0xc1u || low == 0xe1u;
            node = v6 ? CNDP_MQ_NODE_IP6 : CNDP_MQ_NODE_IP4;
            e = e8;
            const uint64_t o = fo + (adj ? l2 : 0u);
            const uint64_t lo = o + (v6 ? 4u : 2u);
            if (adj && ipl) // the parse's read of the same field (no second read of the frame)
                dlen = ipl & 0xffffu;
            else if ((lo & 1u) == 0 && lo + 2 <= a.slab_len) // one read (one PCIe read in place)
                dlen = bswap16(*(const uint16_t *)(a.slab + lo));
            else
                dlen = (gbyte(a.slab, a.slab_len, lo) << 8) | gbyte(a.slab, a.slab_len, lo + 1);
            if (!adj || blen != a.tb.buf_len)
                e = mq_input_at(a.slab, a.slab_len, o, v6, a.tb, blen) >> 24;
        }
        const uint32_t h = a.want_hash ? a.hash[i] : 0u;
        if (a.zc && a.hostwb) {
            // the record staged mode writes, plus the addresses ipv4/ipv6_save_metadata
            // copy (from the saved window, or the frame when past it)
            const uint64_t m = a.mb[i];
            if (m != 0 && fo < a.slab_len) {
                u32x4 r;
                r.x = pt;
                r.y = rm;
                r.z = dlen | (e << 16) | (node << 24);
                r.w = h;
                a.rec[i] = r;
                if (node != CNDP_MQ_NODE_PTYPE && a.rec_md) {
                    const uint32_t ip = adj ? l2 : 0u, na = v6 ? 4u : 1u;
                    const uint32_t s_at = ip + (v6 ? 8u : 12u), d_at = ip + (v6 ? 24u : 16u);
                    const bool inwin = d_at + 4u * na <= 64u;
                    const u32x4 *w = a.win + 4ull * i;
                    const uint8_t *fr = a.slab + fo;
                    const uint64_t fav = a.slab_len - fo;
                    uint32_t sa[4] = {0u, 0u, 0u, 0u}, da[4] = {0u, 0u, 0u, 0u};
                    for (uint32_t k = 0; k < na; k++) {
                        sa[k] = inwin ? mq_win32(w, s_at + 4 * k) : gld32(fr, fav, s_at + 4 * k);
                        da[k] = inwin ? mq_win32(w, d_at + 4 * k) : gld32(fr, fav, d_at + 4 * k);
                    }
                    a.rec_md[2 * i] = (u32x4){sa[0], sa[1], sa[2], sa[3]};
                    a.rec_md[2 * i + 1] = (u32x4){da[0], da[1], da[2], da[3]};
                }
                a.edges[i] = (uint16_t)((node << 8) | e);
            } else {
                a.edges[i] = (uint16_t)MQ_EDGE_NONE;
            }
        } else if (a.zc) {
            const uint64_t m = a.mb[i];
            if (m != 0 && fo < a.slab_len) {
                // data_off, lport, buf_len, data_len, packet_type in one 12-B store
                u32x3a4 w;
                w.x = (adj ? doff + l2 : doff) | (a.lport << 16);
                w.y = blen | ((dlen & 0xffffu) << 16);
                w.z = pt;
                *(u32x3a4 *)(m + MB_DATA_OFF) = w;
                u32x4 tol; // tx_offload = l2 | l3 << 7 | l4 << 16, ol_flags = MCAST/BCAST/IPv6 bits 61..63
                tol.x = rm & 0xffffffu;
                tol.y = 0u;
                tol.z = 0u;
                tol.w = (rm >> 29) << 29;
                *(u32x4 *)(m + MB_TX_OFFLOAD) = tol;
                if (a.want_hash)
                    *(uint32_t *)(m + MB_HASH) = h;
                if (node != CNDP_MQ_NODE_PTYPE && a.md && a.md[i])
                    mq_save_md((uint8_t *)(uintptr_t)a.md[i], a.win + 4ull * i, a.slab + fo, a.slab_len - fo,
                               adj ? l2 : 0u, v6);
                a.edges[i] = (uint16_t)((node << 8) | e);
            } else {
                a.edges[i] = (uint16_t)MQ_EDGE_NONE;
            }
        } else {
            u32x4 r;
            r.x = pt;
            r.y = rm;
            r.z = dlen | (e << 16) | (node << 24);
            r.w = h;
            a.rec[i] = r;
            a.edges[i] = (uint16_t)((node << 8) | e);
        }
    }
    mq_complete(a);
}

struct MqSlot {
    int state;
    int failed;            // its launch failed: every mbuf comes back with CNDP_MQ_EDGE_NONE
    uint32_t n, polled, buf_len, seq;
    int32_t rg;            // cnet zero-copy: the region every frame of the batch lies in (-1: none yet)
    uint64_t t_open_ns;    // when the first mbuf went in
    uint64_t stage_used;   // staged bytes
    uint32_t nrun;         // cnet: runs of equal-size bursts (each ends with at most one short burst)
    uint32_t run_B[MQ_RUNS_MAX], run_n[MQ_RUNS_MAX];
    uint8_t run_closed;
    uint32_t nb;           // CNDP_MQ_F_REWRITE: submitted bursts (their starts at h_bst)
    void **mb;             // host
    uint8_t *h, *hd;       // pinned + mapped block (host view, device view)
    uint8_t *d;            // device block (cnet classify outputs)
};

struct MqRegion {
    const uint8_t *host;
    uint64_t len;
    int64_t delta; // device address - host address
};

struct cndp_gpu_mq {
    cndp_gpu_ctx_t *c;
    struct cndp_mq_conf conf;
    hipStream_t s;
    int zc;                        // zero-copy (conf.umem was a registered region)
    MqRegion rg[CNDP_MAX_REGIONS]; // zero-copy: the context's regions when the queue was made
    int nrg, rg_last;
    uint32_t stage;                // staged bytes reserved per frame
    uint32_t *flags, *flags_d;     // pinned completion flags (host / device view)
    uint32_t *tickets;             // device, one per slot
    // byte offsets inside each slot's pinned block (H) and device block (D)
    uint64_t h_mb, h_off, h_len, h_md, h_edge, h_rec, h_rmd, h_stage, h_bst, h_bytes;
    int hostwb;                    // zc cnet / ip4_lookup with CNDP_MQ_F_HOST_WRITEBACK
    uint64_t d_nh, d_edge, d_pt, d_rm, d_hash, d_ipl, d_win, d_off, d_len, d_md, d_bytes;
    int devhdr;                    // zc with CNDP_MQ_F_DEVICE_HEADERS (ip4_lookup, cnet)
    // cnet device headers: pools seen whose conf.metadata(m) is m + 64 (and
    // those whose is not), learnt from the first mbuf of a burst
    uint32_t n_pool, n_pool_ext;
    uint64_t pool[CNDP_MQ_POOLS], pool_ext[CNDP_MQ_POOLS];
    uint32_t head, open, in_flight, seq; // head: oldest slot not fully polled
    uint32_t pending;
    int err;                       // a launch error not yet reported (returned by the next submit)
    uint64_t n_batches, n_mbufs;   // launched so far (cndp_gpu_mq_stat)
    MqSlot slot[CNDP_MQ_DEPTH_MAX];
};

static uint64_t now_ns()
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

static inline uint64_t al64(uint64_t x) { return (x + 63u) & ~63ull; }

// the registered region holding [p, p + need), or -1
static inline int mq_region(cndp_gpu_mq_t *q, const void *p, uint64_t need)
{
    const uint8_t *x = (const uint8_t *)p;
    const MqRegion *r = &q->rg[q->rg_last];
    if (q->nrg && x >= r->host && x + need <= r->host + r->len)
        return q->rg_last;
    for (int k = 0; k < q->nrg; k++)
        if (x >= q->rg[k].host && x + need <= q->rg[k].host + q->rg[k].len) {
            q->rg_last = k;
            return k;
        }
    return -1;
}

// zero-copy frame word of host address f (0: outside every region)
static inline uint64_t mq_frame_word(cndp_gpu_mq_t *q, const uint8_t *f)
{
    const int k = mq_region(q, f, 1);
    if (k < 0)
        return 0;
    const uint64_t left = (uint64_t)(q->rg[k].host + q->rg[k].len - f);
    return ((uint64_t)(intptr_t)(f + q->rg[k].delta) & MQ_ADDR_MASK) | ((left < 255u ? left : 255u) << 56);
}

extern "C" int cndp_gpu_mq_create(cndp_gpu_ctx_t *c, const struct cndp_mq_conf *conf, cndp_gpu_mq_t **out)
{
    if (!c || !conf || !out)
        return -EINVAL;
    *out = nullptr;
    struct cndp_mq_conf k = *conf;
    if (k.mode != CNDP_MQ_IP4_LOOKUP && k.mode != CNDP_MQ_CNET && k.mode != CNDP_MQ_MAC_SWAP &&
        k.mode != CNDP_MQ_IP4_REWRITE)
        return -EINVAL;
    if (k.flags & ~(CNDP_MQ_F_HASH | CNDP_MQ_F_NO_METADATA | CNDP_MQ_F_DEVICE_HEADERS | CNDP_MQ_F_RX_PARSE |
                    CNDP_MQ_F_REWRITE | CNDP_MQ_F_HOST_WRITEBACK))
        return -EINVAL;
    // host writeback: cnet and ip4_lookup; cnet's poll reads the header fields
    // it adjusts, so its headers stay on the host, while ip4_lookup's poll only
    // stores (packet_type, udata64), so its headers may be the device's
    if ((k.flags & CNDP_MQ_F_HOST_WRITEBACK) &&
        ((k.mode != CNDP_MQ_CNET && k.mode != CNDP_MQ_IP4_LOOKUP) ||
         (k.mode == CNDP_MQ_CNET && (k.flags & CNDP_MQ_F_DEVICE_HEADERS))))
        return -EINVAL;
    if ((k.flags & (CNDP_MQ_F_RX_PARSE | CNDP_MQ_F_REWRITE)) && k.mode != CNDP_MQ_IP4_LOOKUP)
        return -EINVAL;
    if ((k.flags & CNDP_MQ_F_REWRITE) && !k.umem) // the rewrite goes into the frame where it lies
        return -EINVAL;
    k.batch = k.batch ? k.batch : 8192u;
    k.depth = k.depth ? k.depth : 4u;
    k.max_delay_us = k.max_delay_us ? k.max_delay_us : 50u;
    k.stage_max = k.stage_max ? k.stage_max : 2048u;
    if (k.batch < MQ_BURST || k.batch > (1u << 24) || k.depth < 2 || k.depth > CNDP_MQ_DEPTH_MAX ||
        k.stage_max < 64 || k.stage_max > 65535)
        return -EINVAL;
    if (k.mode == CNDP_MQ_IP4_LOOKUP ? !c->fib4 : k.mode == CNDP_MQ_CNET ? (!c->fib4 || !c->fib6) : false)
        return -EINVAL;
    int r = set_device(c->dev);
    if (r)
        return r;
    cndp_gpu_mq_t *q = (cndp_gpu_mq_t *)calloc(1, sizeof(*q));
    if (!q)
        return -ENOMEM;
    q->c = c;
    q->conf = k;
    if (k.umem) {
        // zero-copy: every region the context holds (the UMEMs of all the
        // graph's ports), conf.umem among them
        bool named = false;
        for (int j = 0; j < c->n_reg; j++) {
            q->rg[q->nrg].host = c->reg[j].host;
            q->rg[q->nrg].len = c->reg[j].len;
            q->rg[q->nrg].delta = (int64_t)((intptr_t)c->reg[j].dev - (intptr_t)c->reg[j].host);
            q->nrg++;
            named = named || c->reg[j].host == (uint8_t *)k.umem;
        }
        if (!named) {
            free(q);
            return -EINVAL; // not registered with cndp_gpu_host_register
        }
        q->zc = 1;
    }
    const uint64_t B = k.batch;
    const bool cnet = k.mode == CNDP_MQ_CNET, rw = k.mode == CNDP_MQ_IP4_REWRITE;
    const bool zc = q->zc != 0;
    q->stage = zc ? 0u
             : cnet ? (uint32_t)al64(k.stage_max)
             : k.mode == CNDP_MQ_IP4_LOOKUP ? ((k.flags & CNDP_MQ_F_RX_PARSE) ? 32u : MQ_W4)
             : k.mode == CNDP_MQ_MAC_SWAP ? MQ_SWAP : MQ_RW_STAGE;
    q->h_mb = 0;                                          // zc: mbuf device addresses; rewrite: tail flags
    q->h_off = al64(B * 8);                               // frame words / offsets
    q->h_len = q->h_off + al64(B * 8);                    // cnet: length fields; rewrite: priv1
    q->h_md = q->h_len + (cnet || rw ? al64(B * 8) : 0);  // cnet zc: metadata addresses
    q->h_edge = q->h_md + (cnet && zc ? al64(B * 8) : 0);
    q->hostwb = zc && (k.flags & CNDP_MQ_F_HOST_WRITEBACK);
    q->h_rec = q->h_edge + al64(B * 2);                   // staged (and host writeback): records
    q->h_rmd = q->h_rec + ((zc && !q->hostwb) || rw || k.mode == CNDP_MQ_MAC_SWAP ? 0 : al64(B * (cnet ? 16 : 8)));
    q->h_stage = q->h_rmd + (q->hostwb && cnet ? B * 32 : 0); // cnet host writeback: metadata addresses
    q->h_bst = q->h_stage + B * q->stage;                 // CNDP_MQ_F_REWRITE: burst starts
    q->h_bytes = q->h_bst + ((k.flags & CNDP_MQ_F_REWRITE) ? al64((B + 1) * 4) : 0);
    q->d_nh = 0;
    q->d_edge = q->d_nh + al64(B * 4);
    q->d_pt = q->d_edge + al64(B);
    q->d_rm = q->d_pt + al64(B * 4);
    q->d_hash = q->d_rm + al64(B * 4);
    q->d_ipl = q->d_hash + al64(B * 4);
    q->d_win = q->d_ipl + al64(B * 4);
    q->devhdr = zc && (k.flags & CNDP_MQ_F_DEVICE_HEADERS) && k.mode != CNDP_MQ_MAC_SWAP;
    q->d_off = q->d_win + (zc ? B * 64 : 0);
    q->d_len = q->d_off + (cnet && q->devhdr ? al64(B * 8) : 0);
    q->d_md = q->d_len + (cnet && q->devhdr ? al64(B * 8) : 0);
    q->d_bytes = cnet ? q->d_md + (q->devhdr ? al64(B * 8) : 0) : 64;
    r = -ENOMEM;
    if (hipStreamCreateWithFlags(&q->s, hipStreamNonBlocking) != hipSuccess)
        goto fail;
    if (hipHostMalloc((void **)&q->flags, CNDP_MQ_DEPTH_MAX * 64, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void **)&q->flags_d, q->flags, 0) != hipSuccess ||
        hipMalloc((void **)&q->tickets, CNDP_MQ_DEPTH_MAX * 4) != hipSuccess ||
        hipMemset(q->tickets, 0, CNDP_MQ_DEPTH_MAX * 4) != hipSuccess)
        goto fail;
    memset(q->flags, 0, CNDP_MQ_DEPTH_MAX * 64);
    for (uint32_t j = 0; j < k.depth; j++) {
        MqSlot *sl = &q->slot[j];
        sl->mb = (void **)malloc(B * sizeof(void *));
        if (!sl->mb || hipHostMalloc((void **)&sl->h, q->h_bytes, hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer((void **)&sl->hd, sl->h, 0) != hipSuccess ||
            hipMalloc((void **)&sl->d, q->d_bytes) != hipSuccess ||
            hipMemset(sl->d, 0, q->d_bytes) != hipSuccess) // iplen starts cleared
            goto fail;
    }
    // the clears done before the queue's own (non-blocking) stream first runs
    if (hipDeviceSynchronize() != hipSuccess)
        goto fail;
    *out = q;
    return 0;
fail:
    cndp_gpu_mq_free(q);
    return r;
}

extern "C" void cndp_gpu_mq_free(cndp_gpu_mq_t *q)
{
    if (!q)
        return;
    hipSetDevice(q->c->dev);
    if (q->s)
        hipStreamSynchronize(q->s);
    for (uint32_t j = 0; j < CNDP_MQ_DEPTH_MAX; j++) {
        MqSlot *sl = &q->slot[j];
        free(sl->mb);
        if (sl->h)
            hipHostFree(sl->h);
        if (sl->d)
            hipFree(sl->d);
    }
    if (q->flags)
        hipHostFree(q->flags);
    if (q->tickets)
        hipFree(q->tickets);
    if (q->s) {
        // the context's last scratch user may be this stream (scratch_acquire
        // would record on it): drained above, so nothing is left to order
        if (q->c->scratch_used && q->c->scratch_stream == q->s)
            q->c->scratch_used = 0;
        hipStreamDestroy(q->s);
    }
    free(q);
}

extern "C" uint32_t cndp_gpu_mq_pending(const cndp_gpu_mq_t *q) { return q ? q->pending : 0u; }

// the slot being filled, opened on demand (nullptr: every slot is busy)
static MqSlot *mq_open_slot(cndp_gpu_mq_t *q)
{
    MqSlot *sl = &q->slot[q->open];
    if (sl->state == MQ_OPEN)
        return sl;
    if (sl->state != MQ_FREE)
        return nullptr;
    sl->state = MQ_OPEN;
    sl->failed = 0;
    sl->n = sl->polled = 0;
    sl->nrun = 0;
    sl->run_closed = 0;
    sl->nb = 0;
    sl->stage_used = 0;
    sl->buf_len = 0;
    sl->rg = -1;
    return sl;
}

// the node kernels' tables, from views taken with tbl_acquire (v6 may be null)
static MqTables mq_tables(const cndp_gpu_ctx_t *c, const TblView &v4, const TblView *v6, uint32_t buf_len)
{
    MqTables t;
    memset(&t, 0, sizeof(t));
    t.t24 = (const uint32_t *)v4.t24;
    t.t8 = (const uint32_t *)v4.t8;
    if (c->tune_dir16 && v4.d16) {
        t.d16 = v4.d16;
        t.pages = v4.pages;
    }
    if (v6) {
        t.t24_6 = (const uint32_t *)v6->t24;
        t.t8_6 = (const uint32_t *)v6->t8;
    }
    t.buf_len = buf_len;
    return t;
}

static int rw_sync(cndp_gpu_ctx_t *c, hipStream_t s);

static int mq_launch_kernels(cndp_gpu_mq_t *q, MqSlot *sl, uint32_t slot_i)
{
    cndp_gpu_ctx_t *c = q->c;
    int r = set_device(c->dev);
    if (r)
        return r;
    hipStream_t s = q->s;
    const uint32_t n = sl->n;
    const bool cnet = q->conf.mode == CNDP_MQ_CNET, zc = q->zc != 0;
    uint8_t *HD = sl->hd, *D = sl->d;
    MqArgs a;
    memset(&a, 0, sizeof(a));
    a.n = n;
    a.zc = zc;
    a.mb = (const uint64_t *)(HD + q->h_mb);
    a.off = (const uint64_t *)(HD + q->h_off);
    a.lens = (const u32x2 *)(HD + q->h_len);
    a.priv = (const uint64_t *)(HD + q->h_len);
    a.md = zc && cnet && !(q->conf.flags & CNDP_MQ_F_NO_METADATA) ? (const uint64_t *)(HD + q->h_md) : nullptr;
    if (zc && cnet) {
        const MqRegion &g = q->rg[sl->rg >= 0 ? sl->rg : 0];
        a.slab = g.host + g.delta;
        a.slab_len = g.len;
    } else {
        a.slab = HD + q->h_stage;
        a.slab_len = sl->stage_used ? sl->stage_used : 64;
    }
    a.edges = (uint16_t *)(HD + q->h_edge);
    a.priv1 = (uint64_t *)(HD + q->h_rec);
    a.rec = (u32x4 *)(HD + q->h_rec);
    a.hostwb = (uint32_t)q->hostwb;
    a.rec_md = q->hostwb && cnet && !(q->conf.flags & CNDP_MQ_F_NO_METADATA) ? (u32x4 *)(HD + q->h_rmd) : nullptr;
    a.lport = q->conf.lport;
    a.want_hash = (q->conf.flags & CNDP_MQ_F_HASH) != 0;
    a.ticket = q->tickets + slot_i;
    a.flag = q->flags_d + slot_i * 16u;
    sl->seq = ++q->seq;
    a.seq = sl->seq;
    const uint32_t g = blocks_for(n, MQ_TPB);
    if (q->conf.mode == CNDP_MQ_MAC_SWAP) {
        hipLaunchKernelGGL(k_mq_mac_swap, dim3(g), dim3(MQ_TPB), 0, s, a);
    } else if (q->conf.mode == CNDP_MQ_IP4_REWRITE) {
        if ((r = rw_sync(c, s)))
            return r;
        a.rw = c->d_rw_tbl;
        if (q->devhdr) { // frames in any registered region
            a.devhdr = 1;
            a.nrg = (uint32_t)q->nrg;
            for (int k = 0; k < q->nrg; k++) {
                a.rg[k].host = (uint64_t)(uintptr_t)q->rg[k].host;
                a.rg[k].len = q->rg[k].len;
                a.rg[k].delta = q->rg[k].delta;
            }
        }
        hipLaunchKernelGGL(k_mq_ip4_rewrite, dim3(g), dim3(MQ_TPB), 0, s, a);
    } else if (!cnet) {
        TblView v4{};
        if ((r = tbl_acquire(&c->fib4->t, s, &v4)))
            return r;
        a.tb = mq_tables(c, v4, nullptr, 0);
        a.rxparse = (q->conf.flags & CNDP_MQ_F_RX_PARSE) != 0;
        const bool fuse = (q->conf.flags & CNDP_MQ_F_REWRITE) != 0;
        if (fuse) {
            if ((r = rw_sync(c, s))) {
                tbl_release(&c->fib4->t);
                return r;
            }
            a.rw = c->d_rw_tbl;
            ((uint32_t *)(sl->h + q->h_bst))[sl->nb] = n;
            a.bstart = (const uint32_t *)(HD + q->h_bst);
        }
        if (q->devhdr) { // frames in any registered region
            a.devhdr = 1;
            a.nrg = (uint32_t)q->nrg;
            for (int k = 0; k < q->nrg; k++) {
                a.rg[k].host = (uint64_t)(uintptr_t)q->rg[k].host;
                a.rg[k].len = q->rg[k].len;
                a.rg[k].delta = q->rg[k].delta;
            }
        }
        if (fuse)
            hipLaunchKernelGGL(k_mq_l3fwd_burst, dim3(sl->nb), dim3(MQ_L3_TPB), 0, s, a);
        else
            hipLaunchKernelGGL(k_mq_ip4_lookup, dim3(g), dim3(MQ_TPB), 0, s, a);
        tbl_release(&c->fib4->t);
    } else {
        // one classify per run of equal-size graph bursts, the ptype node's
        // speculation run with that burst size, its state carried in the
        // context from run to run and batch to batch
        if (q->devhdr) { // the headers read on the device first (k_mq_cnet_hdr)
            const MqRegion &br = q->rg[sl->rg >= 0 ? sl->rg : 0];
            a.devhdr = 1;
            a.nrg = 1;
            a.rg[0].host = (uint64_t)(uintptr_t)br.host;
            a.rg[0].len = br.len;
            a.rg[0].delta = br.delta;
            a.w_off = (uint64_t *)(D + q->d_off);
            a.w_lens = (u32x2 *)(D + q->d_len);
            a.w_md = a.md ? (uint64_t *)(D + q->d_md) : nullptr;
            a.w_mdh = (uint64_t *)(HD + q->h_md);
            a.md_all = q->conf.metadata == nullptr;
            a.n_pool = q->n_pool;
            for (uint32_t k = 0; k < q->n_pool; k++)
                a.md_pool[k] = q->pool[k];
            hipLaunchKernelGGL(k_mq_cnet_hdr, dim3(g), dim3(MQ_TPB), 0, s, a);
            a.off = a.w_off;
            a.lens = a.w_lens;
            a.md = a.w_md;
        }
        const uint32_t saved_B = c->spec_burst;
        uint32_t i0 = 0;
        for (uint32_t k = 0; k < sl->nrun && !r; k++) {
            struct cndp_batch b;
            memset(&b, 0, sizeof(b));
            b.mode = CNDP_MODE_CNET;
            b.n = sl->run_n[k];
            b.slab = a.slab;
            b.slab_len = a.slab_len;
            b.offsets = a.off + i0;
            b.buf_len = sl->buf_len;
            b.nh = (uint32_t *)(D + q->d_nh) + i0;
            b.edge = D + q->d_edge + i0;
            b.ptype = (uint32_t *)(D + q->d_pt) + i0;
            b.rxmeta = (uint32_t *)(D + q->d_rm) + i0;
            b.hash = a.want_hash ? (uint32_t *)(D + q->d_hash) + i0 : nullptr;
            c->spec_burst = saved_B ? sl->run_B[k] : 0u;
            c->mq_iplen = (uint32_t *)(D + q->d_ipl) + i0;
            c->mq_win = a.md ? (u32x4 *)(D + q->d_win) + 4ull * i0 : nullptr;
            r = classify_impl(c, &b, s, nullptr, nullptr); // a speculation error is the poll's (mq_poll)
            c->mq_iplen = nullptr;
            c->mq_win = nullptr;
            i0 += sl->run_n[k];
        }
        c->spec_burst = saved_B;
        if (r)
            return r;
        a.ptype = (const uint32_t *)(D + q->d_pt);
        a.rxmeta = (const uint32_t *)(D + q->d_rm);
        a.hash = (const uint32_t *)(D + q->d_hash);
        a.edge8 = D + q->d_edge;
        a.iplen = (uint32_t *)(D + q->d_ipl);
        a.win = (const u32x4 *)(D + q->d_win);
        TblView v4{}, v6{};
        if ((r = tbl_acquire(&c->fib4->t, s, &v4)))
            return r;
        if ((r = tbl_acquire(&c->fib6->t, s, &v6))) {
            tbl_release(&c->fib4->t);
            return r;
        }
        a.tb = mq_tables(c, v4, &v6, sl->buf_len);
        hipLaunchKernelGGL(k_mq_cnet_post, dim3(g), dim3(MQ_TPB), 0, s, a);
        tbl_release(&c->fib4->t);
        tbl_release(&c->fib6->t);
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

// launch the open slot; on failure its mbufs come back from poll with
// CNDP_MQ_EDGE_NONE (each mbuf keeps exactly one owner) and the error is
// returned
static int mq_launch(cndp_gpu_mq_t *q)
{
    const uint32_t slot_i = q->open;
    MqSlot *sl = &q->slot[slot_i];
    if (sl->state != MQ_OPEN || sl->n == 0)
        return 0;
    const int r = mq_launch_kernels(q, sl, slot_i);
    if (r) {
        // kernels of the batch's earlier runs may be enqueued and still read
        // the slot's staging: let them finish before its mbufs go back; the
        // speculation state they advanced part way restarts from 0
        (void)hipStreamSynchronize(q->s);
        if (q->conf.mode == CNDP_MQ_CNET)
            q->c->spec_reset = 1;
        sl->failed = 1;
        sl->state = MQ_DONE;
        uint16_t *ed = (uint16_t *)(sl->h + q->h_edge);
        for (uint32_t i = 0; i < sl->n; i++)
            ed[i] = (uint16_t)MQ_EDGE_NONE;
    } else {
        sl->state = MQ_FLIGHT;
        q->in_flight++;
    }
    q->n_batches++;
    q->n_mbufs += sl->n;
    q->open = (q->open + 1) % q->conf.depth;
    return r;
}

extern "C" int cndp_gpu_mq_flush(cndp_gpu_mq_t *q)
{
    if (!q)
        return -EINVAL;
    return mq_launch(q);
}

// eth_rx's metadata address of m: pktmbuf_metadata (pktmbuf.h:1209-1220)
// through the node's hook, else its default m + sizeof(pktmbuf_t)
static inline uint8_t *mq_md_host(const cndp_gpu_mq_t *q, uint8_t *m)
{
    return q->conf.metadata ? (uint8_t *)q->conf.metadata(m) : m + 64;
}

// cnet device headers: whether m's pool keeps pktmbuf_metadata at m + 64, from
// conf.metadata on the first mbuf of a burst whose pool (pooldata, word 0 of
// the header) is new -- one header read per burst, not per mbuf.  A pool not
// in either list (both full) has its mbufs' metadata written by poll.
static void mq_learn_pool(cndp_gpu_mq_t *q, void *m)
{
    const uint64_t pool = *(const uint64_t *)m;
    for (uint32_t k = 0; k < q->n_pool; k++)
        if (q->pool[k] == pool)
            return;
    for (uint32_t k = 0; k < q->n_pool_ext; k++)
        if (q->pool_ext[k] == pool)
            return;
    if ((uint8_t *)q->conf.metadata(m) == (uint8_t *)m + 64) {
        if (q->n_pool < CNDP_MQ_POOLS)
            q->pool[q->n_pool++] = pool;
    } else if (q->n_pool_ext < CNDP_MQ_POOLS) {
        q->pool_ext[q->n_pool_ext++] = pool;
    }
}

// one burst of k mbufs into the open slot sl (room checked by the caller)
static void mq_fill(cndp_gpu_mq_t *q, MqSlot *sl, void *const *mbufs, uint32_t k)
{
    const uint32_t mode = q->conf.mode;
    const bool cnet = mode == CNDP_MQ_CNET, rw = mode == CNDP_MQ_IP4_REWRITE, zc = q->zc != 0;
    const bool want_md = cnet && zc && !(q->conf.flags & CNDP_MQ_F_NO_METADATA);
    const bool devhdr = q->devhdr != 0;
    uint8_t *H = sl->h;
    uint64_t *hmb = (uint64_t *)(H + q->h_mb), *hoff = (uint64_t *)(H + q->h_off);
    uint64_t *hlen = (uint64_t *)(H + q->h_len), *hmd = (uint64_t *)(H + q->h_md);
    const uint32_t vec = k & ~3u; // ip4_rewrite: the 4-wide loop's share of the burst
    if (devhdr) { // the kernels read the headers (CNDP_MQ_F_DEVICE_HEADERS): pointers only
        // cnet: the default metadata (m + 64) must lie in the mbuf's region too
        const uint64_t need = want_md ? 64u + 64u + MQ_MD_LEN : 64u;
        if (want_md && q->conf.metadata && k)
            mq_learn_pool(q, mbufs[0]);
        for (uint32_t i = 0; i < k; i++) {
            uint8_t *m = (uint8_t *)mbufs[i];
            const int km = mq_region(q, m, need);
            sl->mb[sl->n + i] = m;
            hmb[sl->n + i] = km < 0 ? 0u : (uint64_t)(intptr_t)(m + q->rg[km].delta);
            if (rw && km >= 0 && i >= vec) // ip4_rewrite's tail loop (bit 0: mbufs are 64-B aligned)
                hmb[sl->n + i] |= MQ_RW_TAIL;
            if (cnet && sl->rg < 0 && km >= 0) {
                // the batch's region is its first frame's (as on the host-header
                // path), which the host reads from that one header: mbuf headers
                // may sit in another registered region than their buffers
                const uint8_t *f = *(uint8_t *const *)(m + MB_BUF_ADDR) + *(const uint16_t *)(m + MB_DATA_OFF);
                sl->rg = mq_region(q, f, 1);
            }
        }
        return;
    }
    for (uint32_t i = 0; i < k; i++) {
        // the mbuf headers MQ_PF ahead, the frames of the ones half as far
        // (their buf_addr already in cache) where the host copies frame bytes
        if (i + MQ_PF < k)
            __builtin_prefetch((const uint8_t *)mbufs[i + MQ_PF], 1);
        if (!zc && i + MQ_PF / 2 < k) {
            const uint8_t *pm = (const uint8_t *)mbufs[i + MQ_PF / 2];
            __builtin_prefetch(*(uint8_t *const *)(pm + MB_BUF_ADDR) + *(const uint16_t *)(pm + MB_DATA_OFF));
        }
        uint8_t *m = (uint8_t *)mbufs[i];
        uint8_t *buf = *(uint8_t *const *)(m + MB_BUF_ADDR);
        const uint16_t doff = *(const uint16_t *)(m + MB_DATA_OFF);
        const uint16_t blen = *(const uint16_t *)(m + MB_BUF_LEN);
        const uint16_t dlen = *(const uint16_t *)(m + MB_DATA_LEN);
        const uint32_t room = blen > doff ? (uint32_t)(blen - doff) : 0u;
        const uint32_t j = sl->n + i;
        uint8_t *f = buf + doff; // pktmbuf_mtod
        sl->mb[j] = m;
        if (cnet) {
            u32x2 l;
            l.x = (uint32_t)dlen | (room << 16);
            l.y = (uint32_t)blen | ((uint32_t)doff << 16);
            ((u32x2 *)hlen)[j] = l;
        }
        if (rw) {
            hmb[j] = i >= vec ? MQ_RW_TAIL : 0u;
            hlen[j] = *(const uint64_t *)(m + MB_UDATA64); // node_mbuf_priv1
        }
        if (zc) {
            if (!rw) {
                const int km = mq_region(q, m, 64);
                hmb[j] = km < 0 ? 0u : (uint64_t)(intptr_t)(m + q->rg[km].delta);
            }
            if (cnet) {
                // frame offset in the batch's region (the first frame's);
                // outside it: the region's end, which reads as zero bytes
                const int kf = mq_region(q, f, 1);
                if (sl->rg < 0 && kf >= 0)
                    sl->rg = kf;
                const MqRegion &g = q->rg[sl->rg >= 0 ? sl->rg : 0];
                hoff[j] = kf >= 0 && kf == sl->rg ? (uint64_t)(f - g.host) : g.len;
                if (want_md) {
                    uint8_t *md = mq_md_host(q, m);
                    const int kd = md ? mq_region(q, md, MQ_MD_LEN) : -1;
                    hmd[j] = kd < 0 ? 0u : (uint64_t)(intptr_t)(md + q->rg[kd].delta);
                }
            } else {
                hoff[j] = mq_frame_word(q, f);
            }
        } else {
            // staged copy of the bytes the nodes can read (bounded by the buffer)
            uint32_t at = 0, want;
            if (cnet) {
                const uint32_t cap = q->conf.stage_max > MQ_SHORT && mq_short_reach(f, room) ? MQ_SHORT
                                                                                             : q->conf.stage_max;
                want = room < cap ? room : cap;
            } else if (mode == CNDP_MQ_IP4_LOOKUP) {
                const bool rxp = (q->conf.flags & CNDP_MQ_F_RX_PARSE) != 0;
                at = rxp ? MQ_W4R_AT : MQ_W4_AT;
                want = rxp ? MQ_W4R : MQ_W4;
            } else {
                want = q->stage;
            }
            const uint32_t cp = room > at ? (room - at < want ? room - at : want) : 0u;
            uint8_t *dst = H + q->h_stage + sl->stage_used;
            memcpy(dst, f + at, cp);
            const uint64_t span = cnet ? al64(want ? want : 1) : (uint64_t)((want + 15u) & ~15u);
            memset(dst + cp, 0, span - cp);
            hoff[j] = sl->stage_used;
            sl->stage_used += span;
        }
    }
}

extern "C" int cndp_gpu_mq_submit(cndp_gpu_mq_t *q, void *const *mbufs, uint32_t n)
{
    if (!q || (n && !mbufs))
        return -EINVAL;
    if (q->err) { // a launch failed after the previous call accepted its mbufs
        const int e = q->err;
        q->err = 0;
        return e;
    }
    const bool cnet = q->conf.mode == CNDP_MQ_CNET;
    uint32_t done = 0;
    while (done < n) {
        MqSlot *sl = mq_open_slot(q);
        if (!sl)
            break;
        // one graph burst (<= 256 mbufs) at a time, never split across batches
        const uint32_t k = n - done < MQ_BURST ? n - done : MQ_BURST;
        bool full = sl->n + k > q->conf.batch;
        if (cnet && !full && sl->nrun == MQ_RUNS_MAX && !(sl->run_closed == 0 && k <= sl->run_B[sl->nrun - 1]))
            full = true;
        if (full) {
            const int r = mq_launch(q);
            if (r) {
                if (done)
                    q->err = r;
                return done ? (int)done : r;
            }
            continue;
        }
        if (sl->n == 0) {
            sl->t_open_ns = now_ns();
            // the batch's buf_len for the input nodes' length test; frames with
            // another one are re-evaluated by k_mq_cnet_post
            if (cnet)
                sl->buf_len = *(const uint16_t *)((const uint8_t *)mbufs[done] + MB_BUF_LEN);
        }
        if (q->conf.flags & CNDP_MQ_F_REWRITE) // this burst's first mbuf (the kernel's block)
            ((uint32_t *)(sl->h + q->h_bst))[sl->nb++] = sl->n;
        mq_fill(q, sl, mbufs + done, k);
        if (cnet) { // runs of equal-size bursts, each closed by a shorter one
            if (sl->nrun && !sl->run_closed && k == sl->run_B[sl->nrun - 1]) {
                sl->run_n[sl->nrun - 1] += k;
            } else if (sl->nrun && !sl->run_closed && k < sl->run_B[sl->nrun - 1]) {
                sl->run_n[sl->nrun - 1] += k;
                sl->run_closed = 1;
            } else {
                sl->run_B[sl->nrun] = k;
                sl->run_n[sl->nrun] = k;
                sl->nrun++;
                sl->run_closed = 0;
            }
        }
        sl->n += k;
        done += k;
        q->pending += k;
        if (sl->n + MQ_BURST > q->conf.batch) { // no room for another full burst
            const int r = mq_launch(q);
            if (r) { // this call's mbufs are in the failed slot: poll returns them
                q->err = r;
                return (int)done;
            }
        }
    }
    return (int)done;
}

// ipv4/ipv6_save_metadata on the host (ip4_input.c:33-48, ip6_input.c:32-48)
// from the frame at the input node's mtod
static void mq_save_md_host(uint8_t *md, const uint8_t *ip, bool v6)
{
    const uint8_t fam = v6 ? (uint8_t)MQ_AF_INET6 : (uint8_t)MQ_AF_INET, alen = v6 ? 16 : 4;
    md[0] = md[20] = fam;
    md[1] = md[21] = alen;
    memcpy(md + 4, ip + (v6 ? 8 : 12), alen);
    memcpy(md + 24, ip + (v6 ? 24 : 16), alen);
}

// one finished slot's results into its mbufs where the kernels did not
// write them (staged: every field; zero-copy cnet: metadata the device could
// not reach; zero-copy with host writeback: every field, from records)
static void mq_writeback(cndp_gpu_mq_t *q, MqSlot *sl, uint32_t i0, uint32_t i1)
{
    const uint32_t mode = q->conf.mode;
    const uint16_t *ed = (const uint16_t *)(sl->h + q->h_edge);
    if (mode == CNDP_MQ_IP4_LOOKUP && (q->hostwb || !q->zc)) {
        // node_mbuf_priv1 (ip4_lookup.c:144-154) and, with the soft parse,
        // packet_type: staged from the staged ethertype, host writeback from
        // the record (pkt_cls's drops carry their packet_type there)
        const uint64_t *priv1 = (const uint64_t *)(sl->h + q->h_rec);
        const uint64_t *ho = (const uint64_t *)(sl->h + q->h_off);
        const bool rxp = (q->conf.flags & CNDP_MQ_F_RX_PARSE) != 0;
        for (uint32_t i = i0; i < i1; i++) {
            if (i + MQ_PF < i1)
                __builtin_prefetch((uint8_t *)sl->mb[i + MQ_PF] + MB_UDATA64, 1);
            if (ed[i] == MQ_EDGE_NONE) // zero-copy: outside every registered region, untouched
                continue;
            uint8_t *m = (uint8_t *)sl->mb[i];
            const bool cls_drop = ed[i] == CNDP_MQ_EDGE_CLS_DROP;
            if (rxp) {
                uint32_t pt;
                if (q->hostwb) {
                    pt = cls_drop ? (uint32_t)priv1[i] : 0x90u;
                } else {
                    const uint8_t *e = sl->h + q->h_stage + ho[i];
                    const uint32_t et = ((uint32_t)e[0] << 8) | e[1];
                    pt = et == 0x0800u ? 0x90u : et == 0x86DDu ? 0xE0u : 0u;
                }
                *(uint32_t *)(m + MB_PTYPE) = pt;
                if (cls_drop) // pkt_cls dropped it: ip4_lookup never saw it
                    continue;
            }
            *(uint64_t *)(m + MB_UDATA64) = priv1[i];
        }
        return;
    }
    if (q->hostwb) {
        const uint32_t *rec = (const uint32_t *)(sl->h + q->h_rec);
        const uint8_t *rmd = sl->h + q->h_rmd;
        const bool wh = (q->conf.flags & CNDP_MQ_F_HASH) != 0;
        const bool md_on = !(q->conf.flags & CNDP_MQ_F_NO_METADATA);
        const uint16_t lport = q->conf.lport;
        for (uint32_t i = i0; i < i1; i++) {
            if (i + MQ_PF < i1)
                __builtin_prefetch(sl->mb[i + MQ_PF], 1);
            if (ed[i] == MQ_EDGE_NONE) // outside every registered region: untouched
                continue;
            uint8_t *m = (uint8_t *)sl->mb[i];
            const uint32_t pt = rec[4 * i], rm = rec[4 * i + 1], w2 = rec[4 * i + 2];
            // eth_rx mbuf_update (eth_rx.c:35-63), then the input node's data_len
            *(uint32_t *)(m + MB_PTYPE) = pt;
            *(uint64_t *)(m + MB_OL_FLAGS) = (uint64_t)(rm >> 29) << 61;
            *(uint64_t *)(m + MB_TX_OFFLOAD) = (uint64_t)(rm & 0xffffffu);
            *(uint16_t *)(m + MB_LPORT) = lport;
            const uint16_t l2 = (uint16_t)(rm & 0x7fu);
            uint16_t doff = *(uint16_t *)(m + MB_DATA_OFF);
            const uint16_t dlen0 = *(uint16_t *)(m + MB_DATA_LEN);
            const uint16_t blen = *(const uint16_t *)(m + MB_BUF_LEN);
            if (l2 <= dlen0 && (uint32_t)l2 + doff <= blen) // pktmbuf_adj_offset
                *(uint16_t *)(m + MB_DATA_OFF) = (uint16_t)(doff + l2);
            *(uint16_t *)(m + MB_DATA_LEN) = (uint16_t)(w2 & 0xffffu);
            if (wh)
                *(uint32_t *)(m + MB_HASH) = rec[4 * i + 3];
            const uint32_t node = w2 >> 24;
            if (md_on && (node == CNDP_MQ_NODE_IP4 || node == CNDP_MQ_NODE_IP6)) {
                uint8_t *md = mq_md_host(q, m);
                if (md) { // ipv4/ipv6_save_metadata (ip4_input.c:33-48, ip6_input.c:32-48)
                    const bool v6 = node == CNDP_MQ_NODE_IP6;
                    const uint8_t fam = v6 ? (uint8_t)MQ_AF_INET6 : (uint8_t)MQ_AF_INET, alen = v6 ? 16 : 4;
                    md[0] = md[20] = fam;
                    md[1] = md[21] = alen;
                    memcpy(md + 4, rmd + 32ull * i, alen);
                    memcpy(md + 24, rmd + 32ull * i + 16, alen);
                }
            }
        }
        return;
    }
    if (q->zc) {
        if (mode != CNDP_MQ_CNET || (q->conf.flags & CNDP_MQ_F_NO_METADATA))
            return;
        const uint64_t *hmd = (const uint64_t *)(sl->h + q->h_md);
        for (uint32_t i = i0; i < i1; i++) {
            const uint32_t node = ed[i] >> 8;
            if (hmd[i] || ed[i] == MQ_EDGE_NONE || (node != CNDP_MQ_NODE_IP4 && node != CNDP_MQ_NODE_IP6))
                continue;
            uint8_t *m = (uint8_t *)sl->mb[i], *md = mq_md_host(q, m);
            if (md) // the mbuf fields are final: mtod is the input node's
                mq_save_md_host(md, *(uint8_t **)(m + MB_BUF_ADDR) + *(const uint16_t *)(m + MB_DATA_OFF),
                                node == CNDP_MQ_NODE_IP6);
        }
        return;
    }
    const uint8_t *R = sl->h + q->h_rec;
    const uint64_t *ho = (const uint64_t *)(sl->h + q->h_off);
    if (mode == CNDP_MQ_MAC_SWAP || mode == CNDP_MQ_IP4_REWRITE) { // the changed bytes back into the frame
        const uint32_t span = mode == CNDP_MQ_MAC_SWAP ? 12u : MQ_RW_STAGE;
        for (uint32_t i = i0; i < i1; i++) {
            uint8_t *m = (uint8_t *)sl->mb[i];
            uint8_t *buf = *(uint8_t **)(m + MB_BUF_ADDR);
            const uint16_t doff = *(const uint16_t *)(m + MB_DATA_OFF);
            const uint16_t blen = *(const uint16_t *)(m + MB_BUF_LEN);
            const uint32_t room = blen > doff ? (uint32_t)(blen - doff) : 0u;
            memcpy(buf + doff, sl->h + q->h_stage + ho[i], room < span ? room : span);
        }
        return;
    }
    const uint32_t *rec = (const uint32_t *)R;
    const u32x2 *lens = (const u32x2 *)(sl->h + q->h_len); // data_off at submit (staging offset 0)
    const bool wh = (q->conf.flags & CNDP_MQ_F_HASH) != 0;
    const bool md_on = !(q->conf.flags & CNDP_MQ_F_NO_METADATA);
    const uint16_t lport = q->conf.lport;
    for (uint32_t i = i0; i < i1; i++) {
        if (i + MQ_PF < i1)
            __builtin_prefetch(sl->mb[i + MQ_PF], 1);
        uint8_t *m = (uint8_t *)sl->mb[i];
        const uint32_t pt = rec[4 * i], rm = rec[4 * i + 1], w2 = rec[4 * i + 2];
        // eth_rx mbuf_update (eth_rx.c:35-63)
        *(uint32_t *)(m + MB_PTYPE) = pt;
        *(uint64_t *)(m + MB_OL_FLAGS) = (uint64_t)(rm >> 29) << 61;
        *(uint64_t *)(m + MB_TX_OFFLOAD) = (uint64_t)(rm & 0xffffffu);
        *(uint16_t *)(m + MB_LPORT) = lport;
        const uint16_t l2 = (uint16_t)(rm & 0x7fu);
        uint16_t doff = *(uint16_t *)(m + MB_DATA_OFF);
        const uint16_t dlen0 = *(uint16_t *)(m + MB_DATA_LEN);
        const uint16_t blen = *(const uint16_t *)(m + MB_BUF_LEN);
        if (l2 <= dlen0 && (uint32_t)l2 + doff <= blen) // pktmbuf_adj_offset
            doff = (uint16_t)(doff + l2);
        *(uint16_t *)(m + MB_DATA_OFF) = doff;
        *(uint16_t *)(m + MB_DATA_LEN) = (uint16_t)(w2 & 0xffffu); // adjusted, or the IP header's
        if (wh)
            *(uint32_t *)(m + MB_HASH) = rec[4 * i + 3];
        const uint32_t node = w2 >> 24;
        if (md_on && (node == CNDP_MQ_NODE_IP4 || node == CNDP_MQ_NODE_IP6)) {
            // the addresses from the staged copy of the frame (read in
            // sequence, not the frame's own line again); the IP header sits
            // where the adjusted data_off put it
            uint8_t *md = mq_md_host(q, m);
            const uint8_t *st = sl->h + q->h_stage + ((const uint64_t *)(sl->h + q->h_off))[i];
            if (md)
                mq_save_md_host(md, st + (doff - (uint16_t)(lens[i].y >> 16)),
                                node == CNDP_MQ_NODE_IP6);
        }
    }
}

extern "C" int cndp_gpu_mq_poll(cndp_gpu_mq_t *q, void **mbufs, uint16_t *edges, uint32_t max)
{
    if (!q || (max && (!mbufs || !edges)))
        return -EINVAL;
    // adaptive batching: a partly filled batch goes out once it has waited
    // max_delay_us, or earlier when the GPU is idle and the batch is half
    // full or half that old -- not at the first poll after any burst: under
    // a steady stream that launched a batch every few graph bursts, and the
    // launches (several us of host time each) became the host's largest
    // per-mbuf cost (a failed launch is reported by the next submit; its
    // mbufs come back below with CNDP_MQ_EDGE_NONE)
    MqSlot *op = &q->slot[q->open];
    if (op->state == MQ_OPEN && op->n) {
        const uint64_t age = now_ns() - op->t_open_ns, dmax = (uint64_t)q->conf.max_delay_us * 1000u;
        const bool idle = q->in_flight == 0 && (op->n >= q->conf.batch / 2u || age >= dmax / 2u);
        if (idle || age >= dmax) {
            const int r = mq_launch(q);
            if (r)
                q->err = r;
        }
    }
    uint32_t got = 0;
    while (got < max) {
        const uint32_t hi = q->head;
        MqSlot *sl = &q->slot[hi];
        if (sl->state == MQ_FLIGHT) {
            if (__atomic_load_n(&q->flags[hi * 16u], __ATOMIC_ACQUIRE) != sl->seq)
                break;
            sl->state = MQ_DONE;
            q->in_flight--;
            // a speculation wait of this batch expired (its flag was raised
            // after k_spec_fallback's error store): its edges are not the
            // node's, so it comes back like a failed launch
            if (q->conf.mode == CNDP_MQ_CNET && spec_err_take(q->c)) {
                sl->failed = 1;
                uint16_t *ed = (uint16_t *)(sl->h + q->h_edge);
                for (uint32_t i = 0; i < sl->n; i++)
                    ed[i] = (uint16_t)MQ_EDGE_NONE;
                q->err = -EIO;
            }
        }
        if (sl->state != MQ_DONE)
            break;
        const uint32_t take = sl->n - sl->polled < max - got ? sl->n - sl->polled : max - got;
        if (!sl->failed)
            mq_writeback(q, sl, sl->polled, sl->polled + take);
        memcpy(mbufs + got, sl->mb + sl->polled, (size_t)take * sizeof(void *));
        memcpy(edges + got, (const uint16_t *)(sl->h + q->h_edge) + sl->polled, (size_t)take * 2);
        sl->polled += take;
        got += take;
        q->pending -= take;
        if (sl->polled == sl->n) {
            sl->state = MQ_FREE;
            q->head = (q->head + 1) % q->conf.depth;
        }
    }
    return (int)got;
}

extern "C" int64_t cndp_gpu_mq_stat(const cndp_gpu_mq_t *q, int key)
{
    if (!q)
        return -EINVAL;
    switch (key) {
    case CNDP_MQ_STAT_BATCHES:
        return (int64_t)q->n_batches;
    case CNDP_MQ_STAT_MBUFS:
        return (int64_t)q->n_mbufs;
    default:
        return -EINVAL;
    }
}

// The oldest batch's completion flag (the load poll makes), spun on: no HIP
// event per batch (an event record cost as much host time as a launch).
// Bounded: a batch not done within CNDP_MQ_WAIT_S seconds is an error.
#define CNDP_MQ_WAIT_S 30
extern "C" int cndp_gpu_mq_wait(cndp_gpu_mq_t *q)
{
    if (!q)
        return -EINVAL;
    const uint32_t hi = q->head;
    MqSlot *sl = &q->slot[hi];
    if (sl->state != MQ_FLIGHT)
        return 0;
    const uint64_t t0 = now_ns();
    for (uint32_t spin = 0; __atomic_load_n(&q->flags[hi * 16u], __ATOMIC_ACQUIRE) != sl->seq; spin++) {
        if ((spin & 255u) == 255u) {
            if (now_ns() - t0 > CNDP_MQ_WAIT_S * 1000000000ull)
                return -ETIMEDOUT;
            sched_yield();
        } else {
            __builtin_ia32_pause();
        }
    }
    return 0;
}

extern "C" int64_t cndp_gpu_get_stat(cndp_gpu_ctx_t *c, int key)
{
    if (!c || (key != CNDP_STAT_CNET_WORKLIST && key != CNDP_STAT_CNET_UNIFORM && key != CNDP_STAT_SPEC_ERR))
        return -EINVAL;
    if (!c->sp_hint)
        return 0;
    return ((volatile uint32_t *)c->sp_hint)[key == CNDP_STAT_CNET_WORKLIST ? 0
                                             : key == CNDP_STAT_CNET_UNIFORM ? 1
                                                                             : SPEC_HINT_ERR];
}

extern "C" int cndp_gpu_set_tuning(cndp_gpu_ctx_t *c, int key, int value)
{
    if (!c)
        return -EINVAL;
    switch (key) {
    case CNDP_TUNE_NT:
        c->tune_nt = value ? 1 : 0;
        return 0;
    case CNDP_TUNE_UNROLL:
        if (value != 1)
            return -EINVAL;
        c->tune_unroll = value;
        return 0;
    case CNDP_TUNE_BLOCKS_PER_CU:
        if (value < 0 || value > 64)
            return -EINVAL;
        c->tune_bpc = value;
        return 0;
    case CNDP_TUNE_TILE:
        if (value < 0 || value > 1)
            return -EINVAL;
        c->tune_tile = value;
        return 0;
    case CNDP_TUNE_DIR16:
        c->tune_dir16 = value ? 1 : 0;
        return 0;
    case CNDP_TUNE_CNET_TILE:
        if (value < 0 || value > 1)
            return -EINVAL;
        c->tune_cnet_tile = value;
        return 0;
    case CNDP_TUNE_LOAD_NT:
        c->tune_lnt = value ? 1 : 0;
        return 0;
    case CNDP_TUNE_SPEC_SCAN:
        if (value < 0 || value > 2)
            return -EINVAL;
        c->tune_spec_scan = value;
        return 0;
    case CNDP_TUNE_RW_WB:
        if (value < 0 || value > 2)
            return -EINVAL;
        c->tune_rw_wb = value;
        return 0;
    case CNDP_TUNE_CNET_SPEC:
        if (value < 0)
            return -EINVAL;
        c->spec_burst = (uint32_t)value;
        c->spec_reset = 1; // a new graph: ctx->last_type starts at 0 again (stream-ordered, next call)
        return 0;
    case CNDP_TUNE_MBUF_HASH:
        c->mbuf_hash = value ? 1 : 0;
        return 0;
    case CNDP_TUNE_CNET_FOLD:
        if (value < 0 || value > 2)
            return -EINVAL;
        c->tune_cnet_fold = value;
        return 0;
    case CNDP_TUNE_SPEC_GRID:
        if (value < 0 || value > 2)
            return -EINVAL;
        c->tune_spec_grid = value;
        return 0;
    case CNDP_TUNE_SPEC_LISTS:
        if (value < 0 || value > 1)
            return -EINVAL;
        c->tune_spec_lists = value;
        return 0;
    case CNDP_TUNE_SPEC_TYPES:
        if (value < 0 || value > 2)
            return -EINVAL;
        c->tune_spec_types = value;
        return 0;
    case CNDP_TUNE_STREAM_BAL:
        if (value < 0 || value > 2)
            return -EINVAL;
        c->tune_stream_bal = value;
        return 0;
    case CNDP_TUNE_HOST_WINDOW:
        c->tune_host_window = value ? 1 : 0;
        return 0;
    case CNDP_TUNE_SPEC_WAIT:
        if (value == 0 || value < -1 || value > 40000000)
            return -EINVAL;
        c->tune_spec_wait_us = value;
        return 0;
    case CNDP_TUNE_HOST_CHUNK:
        if (value < 1024)
            return -EINVAL;
        c->host_chunk = (uint32_t)value;
        return 0;
    default:
        return -EINVAL;
    }
}

#if CD_STAMP
// diagnostic builds: the per-wave stage sums of the last k_cnet_defer launch
// (8 words a wave: chain, parse, issue, stores, loop, trips)
extern "C" int cndp_gpu_debug_stamps(unsigned long long *out, uint32_t n)
{
    if (n > CD_STAMP_WAVES * 16)
        n = CD_STAMP_WAVES * 16;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(cd_stamps), (size_t)n * 8));
    return 0;
}

extern "C" int cndp_gpu_debug_spec_stamps(unsigned long long *out, uint32_t n)
{
    if (n > SP_STAMP_BLOCKS * 16 + 8)
        n = SP_STAMP_BLOCKS * 16 + 8;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(sp_stamps), (size_t)n * 8));
    return 0;
}
#endif

extern "C" const char *cndp_gpu_version(void) { return CNDP_VERSION; }
