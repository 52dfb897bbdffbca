// f16x3 implicit-GEMM convolution (the main-path conv arithmetic), deep-pipelined:
// forward, stride-1 backward-data (the same kernel on the gradient with flipped
// weights), backward-filter, and the 7x7/s2 stem.
//
// f16x3 arithmetic: every operand v is split as hi = f16(v), lo = f16(v - hi) and
//     v_a * v_b ≈ hi_a*hi_b + hi_a*lo_b + lo_a*hi_b
// (3 fp16 MFMAs, fp32 accumulation, the dropped lo*lo and lo's own rounding cost
// ~2^-22 relative per product).  All three products go into ONE fp32
// accumulator — fp32-class with the same rounding as separate ones, and half the
// accumulator registers, which is what pays for the 256x256 tiles below.  lo is
// stored unscaled, so it is exact only while v - hi is an fp16 normal
// (|v| >= 2^-3): operands with no natural scale are scaled by a power of two —
// weights per output channel (max|w| -> [2^13, 2^14), inverse applied in the
// epilogue), gradients per tensor from max|dy| — and activations keep an
// absolute error floor of 2^-25 below 2^-3, negligible next to fp32 rounding of
// the sums they feed.
//
// Operands arrive PRE-SPLIT in the "packed split" layout written by their
// producers (bn_apply / bn_relu_maxpool with split_passes=3, hkp_split_pack_x3,
// hkp_weight_pack_x3):
//     xs[pixel][C/32][ hi(32 ch) | lo(32 ch) ]        fp16, 128 B per (pixel, group)
//     ws[k][tap][C/32][ hi(32 ch) | lo(32 ch) ]       (+ ws_scale[k]: 2^-e_k)
// so the 32 channels of one filter tap of one GEMM row are one 128-B cache line
// holding both planes — the same bytes as the fp32 tensor.
//
// Forward kernel (conv_x3_kernel<BN, STEM, PAIR, MFD, SK, P>): tile 256 pixels x
// BN output channels, 8 waves as 4x2 (wave tile 64 x BN/2).  A K-step stages one
// 128-B line per GEMM row (32 channels hi|lo; P = 1: 64 plain fp16 channels) into
// a 2- or 3-stage LDS ring by LDS-DMA (global_load_lds_dwordx4: no VGPR round
// trip, no ds_write), NST-1 K-steps in flight ahead of the compute, retired by a
// counted s_waitcnt vmcnt + raw s_barrier (never __syncthreads inside the loop:
// its fence would drain the DMA queue).  LDS rows are unpadded (the DMA writes
// lane-linear 1 KiB pieces); an XOR swizzle of the 16-B chunk index with
// (row>>1)&7, applied to the per-lane DMA SOURCE address and to the ds_read
// address, makes the fragment reads conflict-free (0 conflicts measured).  K
// order: channel group outer, filter tap inner (a pixel line is re-read by the
// next taps while in L2).  Out-of-image taps / rows past M load a zero line.
// MFMA bodies: 16x16x32 (MFD 16) or 32x32x16 (MFD 32), software-pipelined (next
// fragments read during the current MFMAs, one ds_read per MFMA gap, one barrier
// per K-step).  Epilogue: NHWC fp32 (or fp16) store (x weight scale, x gradient
// scale, + addend) + BN tile partials per 128-row tile.
//
// Operand layouts (P): 3 = the packed f16x3 split above (fp32-accurate, the
// default arithmetic); 1 = plain fp16 NHWC activations and KRSC weights (each
// output channel scaled by a power of two) — BASELINE config C4's "fp16 with
// MFMA", the same kernel with 2 MFMAs per 64 channels instead of 3 per 32.
// Intermediate precisions on the packed layout (inference; DESIGN "precision
// modes"), 2 MFMAs per 32 channels: P = 2 keeps hi_x*hi_w + lo_x*hi_w (the
// weights rounded to fp16 after their per-channel power-of-two scale, the
// activation exact to ~2^-22), P = 4 keeps hi_x*hi_w + hi_x*lo_w (the activation
// rounded to fp16, the weights exact).
//
// Replaces the cuDNN convs of src/resnet.py:20-37,77,86,137,184-188 and their
// backward under loss.backward() (train.py:35).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace hkp {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __attribute__((aligned(256))) uint4 g_x3_zero_line[8];   // 128 B of zeros (static, zero-initialised)
// 128 B of all-ones bytes: a NaN in fp32 and in fp16.  The halo body's
// out-of-image lines when it applies the input's BN itself (X3Args::in_ss):
// relu(NaN * s + t) = 0 for any s, t, as a zero-padded post-ReLU input.
__device__ __attribute__((aligned(256))) uint4 g_x3_nan_line[8] = {
    {~0u, ~0u, ~0u, ~0u}, {~0u, ~0u, ~0u, ~0u}, {~0u, ~0u, ~0u, ~0u}, {~0u, ~0u, ~0u, ~0u},
    {~0u, ~0u, ~0u, ~0u}, {~0u, ~0u, ~0u, ~0u}, {~0u, ~0u, ~0u, ~0u}, {~0u, ~0u, ~0u, ~0u}};

struct X3Args {
    const _Float16* xs;
    const _Float16* ws;
    const float* wscale;   // per output channel inverse weight scale [K] (nullable: 1)
    float* y;              // fp32 output, or
    _Float16* y16 = nullptr;   // fp16 output (plain-fp16 path, autocast semantics)
    float* part;
    const unsigned* amax;  // max|input| bits: the input was scaled by pow2_scale_for(amax) (dgrad)
    const float* add;      // addend of the output (dgrad: the residual-branch gradient), nullable
    int N, H, W, C, K, R, S, stride, pad, dil, Ho, Wo;
    int M, nks, cch, n_tiles, RS;
    long plane;            // STEM: halves between the hi and lo image planes
    // phase output (strided dgrad): output pixel (n, ho, wo) of this launch is
    // written at (n, ho*ost + oy, wo*ost + ox) of an [N][OH][OW][K] tensor; ost = 0: dense
    int ost = 0, OH = 0, OW = 0, oy = 0, ox = 0;
    // stream-K (sk_units > 0): the grid's blocks split tiles x K-steps into equal
    // unit ranges; a tile split between blocks is summed by its last-arriving
    // block from per-segment fp32 slabs (sk_ws) — sk_cnt[tile] arrival counters,
    // zero on entry and left zero
    int mt0 = 0;           // m-tile offset of this launch (the split-K tail launch of conv_x3_tail_kernel)
    long sk_units = 0;
    float* sk_ws = nullptr;
    unsigned* sk_cnt = nullptr;
    // the stream-K grid sk_combine works in when it is not the launch's grid: its
    // block count (0: gridDim.x) and this block's index in it (after the XCD remap)
    int sk_grid = 0, sk_b = 0;
    // split-K tail (every group's range inside one m-tile): one slab per group
    // (slot gg * n_tiles + nt) instead of the stream-K grid's two
    int sk_one = 0;
    // A3 launches with the split-K tail appended (conv_x3_a3_kernel): blocks
    // [0, main_blocks) run the full rounds' tiles, the rest the tail's segments —
    // tail_groups groups of n_tiles blocks over tail_units (m-tile, K-step) units
    // from m-tile tail_mt0 (the one-launch form of conv_x3_tail_kernel)
    int main_blocks = 0, tail_groups = 0, tail_mt0 = 0;
    long tail_units = 0;
    unsigned long long* stamps = nullptr;   // debug: per-block phase clocks (hkp_debug_x3_stamps)
    // first-round stagger: blocks b < stagger_blocks with (b >> 3) & 1 (half the CUs
    // of every XCD) wait stagger_ticks (s_memrealtime, 100 MHz) before starting, so
    // the CUs' epilogues (HBM-bound stores) do not all coincide with each other
    int stagger_blocks = 0, stagger_ticks = 0;
    // fused BN apply of the output (P 1, hkp_conv2d_fwd_f16_bn): out = [relu](y*s + t
    // [+ res | + res*rs + rt]) on the fp16-rounded y, bn_apply_f16's arithmetic
    const float* ep_ss = nullptr;          // [2K] scale | shift
    const _Float16* ep_res = nullptr;      // residual [M][K] fp16, nullable
    const float* ep_rss = nullptr;         // residual scale | shift [2K], nullable (raw residual)
    int ep_relu = 0;
    // fused input BN (the halo body, inference): xs is the producer conv's raw
    // NHWC output (fp32 for P 3, fp16 for P 1) and the A operand is
    // relu(x * s + t) — bn_apply's arithmetic — split into hi | lo (P 3) in LDS
    const float* in_ss = nullptr;          // [2C] scale | shift
    // epilogue output stores (A/B: hkp_debug_x3_store): 0 each site's own flavour,
    // 1 plain, 2 nontemporal, 3 sc1 (written through, not kept in the XCD's L2), 4 sc0 sc1
    int st_kind = 0;
    // A/B (hkp_debug_x3_prio): static wave priority in the A3 K loop — 0 none, 1
    // s_setprio 1 on waves 4-7 (the second wave on each SIMD), 2 on waves 0-3
    int prio = 0;
#ifdef HKP_AB_KNOBS
    // A/B probe (hkp_debug_x3_a_wrap): the one-tile and DUO bodies read the A operand of row
    // m from row m % a_wrap (0: off) — wrong outputs, but an L2-resident A stream —
    // to time a conv's K loop without the activation lines' HBM / MALL latency
    int a_wrap = 0;
#endif
};

// One 16-B epilogue output store of flavour `kind` (X3Args::st_kind); dflt: the
// site's own flavour for kind 0 (1 plain, 2 nontemporal).  Measured per site
// (tools/conv_ab.py / infer_ab.py --stores, profiles/r05_store_ab.log): the fp32
// ring-body tile nontemporal (C2 +0.8 %); the plain-fp16 tile plain (C4: nt -0.4 %,
// sc1 -1.6 % end to end, although nt wins 4-7 % per conv in isolation), the fused
// BN epilogue nontemporal
typedef unsigned x3u32x4 __attribute__((ext_vector_type(4)));
template <typename V>
__device__ __forceinline__ void x3_st16(V* p, const V& val, int kind, int dflt) {
    static_assert(sizeof(V) == 16, "16-B store");
    x3u32x4 v;
    __builtin_memcpy(&v, &val, 16);
    x3u32x4* q = (x3u32x4*)p;
    const int k = kind ? kind : dflt;
    if (k == 2) {
        __builtin_nontemporal_store(v, q);
    } else if (k == 3) {
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(q), "v"(v) : "memory");
    } else if (k == 4) {
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(q), "v"(v) : "memory");
    } else {
        *q = v;
    }
}

// debug phase stamps (s_memrealtime, 100 MHz) of one-tile conv blocks: slot k of
// block b at stamps[b * 8 + k]; written by lane 0 of wave 0
__device__ __forceinline__ void x3_stamp(const X3Args& a, int k) {
    if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 8 + k] = __builtin_amdgcn_s_memrealtime();
}
// debug: where the block runs — slot 6: HW_REG_HW_ID (CU / SH / SE ids), slot 7: HW_REG_XCC_ID
__device__ __forceinline__ void x3_stamp_where(const X3Args& a) {
    if (a.stamps && threadIdx.x == 0) {
        a.stamps[blockIdx.x * 8 + 6] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        a.stamps[blockIdx.x * 8 + 7] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
    }
}

// 2^e putting max|x| in [2^13, 2^14) (1 for 0 / non-finite): exact scaling
__device__ __forceinline__ float pow2_scale_of(float m) {
    if (!(m > 0.f) || !(m < INFINITY)) return 1.f;
    int e;
    frexpf(m, &e);
    e = 14 - e;
    e = e < -100 ? -100 : (e > 100 ? 100 : e);
    return ldexpf(1.f, e);
}

// raw workgroup barrier (no vmcnt(0) drain: LDS-DMA stays in flight across it) +
// compiler fence so no LDS access is moved across it
__device__ __forceinline__ void lds_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// workgroup barrier for LDS traffic only: this wave's LDS ops retired, no
// vmcnt(0) — __syncthreads() would also wait for every global store of the
// epilogue to complete (~2-5 us under the other CUs' output writes)
__device__ __forceinline__ void lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    lds_barrier();
}

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// LDS-DMA through a raw buffer resource: address = base + soffset + voffset; a
// voffset >= num_records (soffset is not range-checked) loads zeros — the
// out-of-image taps and the rows past M cost one v_cndmask instead of a 64-bit
// address select, and the per-K-step tap offset rides in the scalar soffset.
typedef int i32x4 __attribute__((ext_vector_type(4)));
extern "C" __device__ void hkp_raw_buffer_load_lds(i32x4 rsrc, __attribute__((address_space(3))) void* lds, int size,
                                                   int voffset, int soffset, int offset,
                                                   int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");
__device__ __forceinline__ i32x4 buffer_rsrc(const void* base, unsigned bytes) {
    const unsigned long long p = (unsigned long long)base;
    i32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)p);
    r[1] = __builtin_amdgcn_readfirstlane((int)(unsigned)(p >> 32) & 0xFFFF);   // stride 0
    r[2] = __builtin_amdgcn_readfirstlane((int)bytes);                          // num_records
    r[3] = 0x00020000;                                                            // gfx9 raw-buffer config
    return r;
}
__device__ __forceinline__ void blds16(i32x4 rsrc, unsigned voff, unsigned soff, char* lds_wave_base) {
    hkp_raw_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)lds_wave_base, 16, (int)voff, (int)soff, 0, 0);
}

// schedule NM MFMAs and NR ds_reads of one basic block as evenly spread
// groups: MFMA first, then one read after every NM/NR MFMAs
template <int NM, int NR>
__device__ __forceinline__ void interleave() {
    constexpr int per = NM >= NR ? NM / NR : 1;
    constexpr int nr = NM >= NR ? NR : NM;          // reads paired with MFMA groups
#pragma unroll
    for (int k = 0; k < nr; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, per, 0);   // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);     // ds_read
    }
    if constexpr (NR > nr) __builtin_amdgcn_sched_group_barrier(0x100, NR - nr, 0);
    if constexpr (NM > per * nr) __builtin_amdgcn_sched_group_barrier(0x008, NM - per * nr, 0);
}

// LDS ring depth of a conv_x3 tile config (32-channel / 128-B stages): 256x256
// tiles 2 (B fragments refilled per column instead), two blocks per CU (PAIR:
// 256x64 tiles and the stem) 2, otherwise 3.  The whole 160 KiB at most (the
// stream-K flag reuses the drained ring).
constexpr int x3_nst(int BN, bool PAIR) { return (BN == 256 || PAIR) ? 2 : 3; }

// the ring, or (P = 1) the staged fp16 output tile if that is larger (256x256: 132 KiB)
constexpr int x3_lds_bytes(int BN, bool PAIR, int P) {
    return P == 1 && 256 * (BN + 8) * 2 > x3_nst(BN, PAIR) * (256 + BN) * 128 ? 256 * (BN + 8) * 2
                                                                              : x3_nst(BN, PAIR) * (256 + BN) * 128;
}
// A3 (conv_x3_a3_kernel): the 256x256 16x16x32 body with separate A and B rings —
// A (the activation lines) 3 stages deep, so a stage's DMA has two K-steps to
// land instead of one (the 1x1 convs of config C4 stream every A line from HBM),
// B (the weights, L2-resident) 2 stages: 5 x 32 KiB = the whole 160 KiB; the
// epilogue's scratch and column scales reuse the drained ring.
constexpr int X3_A3_LDS = 5 * 256 * 128;
// ... with BM-row A stages (A3_192: 192-row tiles, 136 KiB; A3_160: 125 KiB, with a
// 1 KiB sink for the A DMA pieces past row 160 — 20 pieces over 8 waves, 3 each)
constexpr int x3_a3_lds(int BM, int BN = 256) { return 3 * BM * 128 + 2 * BN * 128 + (BM % 64 ? 1024 : 0); }
// waves in M of a BM-row tile (8 waves): 4 (64- / 48-row wave tiles), 2 for 160 rows
// (40-row wave tiles do not split into 16-row MFMA tiles; 80 x 64 instead)
constexpr int x3_wm(int BM) { return BM == 160 ? 2 : 4; }

// BN-partials scratch (x3_bn_partials_w: [2][WM][BN] floats) past the ring, so
// the epilogue needs no barrier before it, then the tile's BN column scales
// (loaded during the pipeline fill: a global load in the epilogue waited ~4 us
// behind the other CUs' output writes); the two-blocks-per-CU tiles (PAIR) have
// no LDS to spare: they reuse the ring after a barrier and load scales late
constexpr int x3_red_bytes(int BN, bool PAIR) { return PAIR ? 0 : 2 * 4 * BN * 4 + BN * 4; }

// ---- stream-K bookkeeping (X3Args::sk_units) ----
__device__ __forceinline__ long sk_start(long b, long U, int G) { return b * U / G; }
// the block whose unit range holds unit u: the largest b with sk_start(b) <= u
__device__ __forceinline__ int sk_block_of(long u, long U, int G) { return (int)(((u + 1) * G + U - 1) / U) - 1; }

typedef f32x4 __attribute__((address_space(1))) gf32x4;
typedef unsigned __attribute__((address_space(1))) gu32;

// A partial tile segment: publish this block's accumulators as an fp32 slab,
// count the arrival; the last-arriving segment's block reads every slab of the
// tile in segment order (fixed summation order: the result does not depend on
// which block arrives last) and returns true with the sum in its accumulators.
// Stream-K is column-grouped: the grid is NG groups of n_tiles blocks; group g
// runs units [g*U/NG, (g+1)*U/NG) of the (m-tile, K-step) sequence, block
// g*n_tiles + nt of it for column tile nt — the n_tiles blocks of a group are
// adjacent after the XCD remap and read the same A lines at the same time (one
// L2 fetch), as the data-parallel grid's neighbouring tiles do.
// Slab of group gg's block for tile (mt, nt): slot 2*(gg*n_tiles + nt) + (0: mt
// is the group's first m-tile, 1: its last).  Hand-off per
// cdna_hip_programming.md §6 Guideline 16 (split-K counter form): every wave
// drains its stores, barrier, one lane releases at agent scope and adds to the
// counter; the last arriver acquires at agent scope before any wave reads a
// slab, and re-zeroes the counter.
template <int NV4, typename Get, typename Set>
__device__ __forceinline__ bool sk_combine(const X3Args& a, int T, int tid, char* flag_lds, Get&& get, Set&& set) {
    const long U = a.sk_units;
    const int NT = a.n_tiles, NG = (a.sk_grid ? a.sk_grid : (int)gridDim.x) / NT;
    const int mt = T / NT, nt = T - mt * NT;
    const long t0 = (long)mt * a.nks;
    const int b0 = sk_block_of(t0, U, NG), nseg = sk_block_of(t0 + a.nks - 1, U, NG) - b0 + 1;
    auto slab = [&](int gg) {
        const int which = sk_start(gg, U, NG) >= t0 ? 0 : 1;
        return (gf32x4*)a.sk_ws + (long)(a.sk_one ? gg * NT + nt : 2 * (gg * NT + nt) + which) * NV4 * 512;
    };
    gf32x4* mine = slab((a.sk_grid ? a.sk_b : xcd_remap(blockIdx.x, gridDim.x)) / NT);
#pragma unroll
    for (int v = 0; v < NV4; ++v) mine[v * 512 + tid] = get(v);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        gu32* cnt = (gu32*)a.sk_cnt + T;
        const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == (unsigned)(nseg - 1);
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        *(volatile int*)flag_lds = last;
    }
    __syncthreads();
    if (!*(volatile int*)flag_lds) return false;
    // 8 loads in flight per chunk (the accumulators leave few free registers;
    // double-buffered chunks, or a chunk index computed at run time, put the
    // 256x256 accumulators into scratch)
    static_assert(NV4 % 8 == 0 || NV4 < 8, "sk_combine chunks");
    constexpr int CW = NV4 < 8 ? NV4 : 8;
    for (int sg = 0; sg < nseg; ++sg) {
        const gf32x4* p = slab(b0 + sg);
#pragma unroll
        for (int v0 = 0; v0 < NV4; v0 += CW) {
            f32x4 x[CW];
#pragma unroll
            for (int v = 0; v < CW; ++v) x[v] = p[(v0 + v) * 512 + tid];
#pragma unroll
            for (int v = 0; v < CW; ++v) set(v0 + v, sg == 0 ? x[v] : get(v0 + v) + x[v]);
        }
    }
    return true;
}

// NHWC offset of output (row m, channel n) of a launch (-1: row past M); strided
// dgrad writes one output phase per launch
__device__ __forceinline__ long x3_out_off(const X3Args& a, int m, int n) {
    if (m >= a.M) return -1;
    long pix = m;
    if (a.ost) {
        const int hw = a.Ho * a.Wo, ni = m / hw, rem = m - ni * hw;
        const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
        pix = ((long)ni * a.OH + ho * a.ost + a.oy) * a.OW + wo * a.ost + a.ox;
    }
    return pix * a.K + n;
}

// One output element: y (fp32) or y16 (fp16, the plain-fp16 path), scaled, +
// the addend (dgrad's residual-branch gradient)
__device__ __forceinline__ void x3_store(const X3Args& a, long off, float v, float av) {
    if (off < 0) return;
    v = a.add ? v + av : v;
    if (a.y16) a.y16[off] = (_Float16)v;
    else a.y[off] = v;
}

// The MFMAs of one 128-B stage row pair (A fragment a0/a1, B fragment b0/b1 =
// the row's chunks 0-3 / 4-7) for operand layout P:
//   P = 3 (packed f16x3 split, chunks = hi32 | lo32):  hi*hi + hi*lo + lo*hi
//   P = 2 / 4 (packed split): two of those three products (see the header)
//   P = 1 (plain fp16, chunks = channels 0-31 | 32-63): two k-slices
// operand layout of P: the packed hi|lo split (P 2, 3, 4) or plain fp16 (P 1)
constexpr bool x3_packed(int P) { return P != 1; }
// fp16 MFMAs per 128-B stage row pair
constexpr int x3_nprod(int P) { return P == 3 ? 3 : 2; }

template <int P, typename V, typename Acc, typename Mfma>
__device__ __forceinline__ void x3_products(Acc& acc, const V& a0, const V& a1, const V& b0, const V& b1, Mfma&& mfma) {
    if constexpr (P == 3) {
        acc = mfma(a0, b0, acc);
        acc = mfma(a0, b1, acc);
        acc = mfma(a1, b0, acc);
    } else if constexpr (P == 2) {         // weights at fp16: (hi_x + lo_x) * hi_w
        acc = mfma(a0, b0, acc);
        acc = mfma(a1, b0, acc);
    } else if constexpr (P == 4) {         // activation at fp16: hi_x * (hi_w + lo_w)
        acc = mfma(a0, b0, acc);
        acc = mfma(a0, b1, acc);
    } else {
        acc = mfma(a0, b0, acc);
        acc = mfma(a1, b1, acc);
    }
}

// BN tile partials of the tile in the accumulators: per 128-row half, the
// column sum and the sum of squares about the half's mean (Chan-mergeable in
// bn_finalize).  VAL(i, j, r) / ROW(i, r) address the accumulator element and
// its output row; COLS per wave column block, LGRP lanes per column group.
template <int BN, int NI, int NJ, int NR, int CW, int SHF, typename Val, typename Row>
__device__ __forceinline__ void x3_bn_partials(const X3Args& a, char* smem, int m0, int n0, int wm, int wn, int lane,
                                               int tid, Val&& val, Row&& row) {
    constexpr int WM = 4;
    __syncthreads();                       // every wave done reading the ring
    float* red = (float*)smem;             // [WM][BN] column sums, then [2][BN] half-tile means
    float* tmean = red + WM * BN;
    float colsum[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < NR; ++r) s += (row(i, r) < a.M) ? val(i, j, r) : 0.f;
        for (int o = SHF; o < 64; o <<= 1) s += __shfl_xor(s, o);
        colsum[j] = s;
    }
    if (lane < CW) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) red[wm * BN + wn * NJ * CW + j * CW + lane] = colsum[j];
    }
    __syncthreads();
    const long tile128 = (long)(m0 >> 7);
    for (int e = tid; e < 2 * BN; e += 512) {
        const int h = e / BN, c = e - h * BN;
        const int cnt = min(128, a.M - (m0 + 128 * h));
        if (cnt > 0) {
            const float s = red[(2 * h) * BN + c] + red[(2 * h + 1) * BN + c];
            tmean[h * BN + c] = s / (float)cnt;
            a.part[((tile128 + h) * a.K + n0 + c) * 2 + 0] = s;
        }
    }
    __syncthreads();
    const float* mu_h = tmean + (wm >> 1) * BN;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const float mu = mu_h[wn * NJ * CW + j * CW + (lane % CW)];
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const float d = val(i, j, r) - mu;
                q += (row(i, r) < a.M) ? d * d : 0.f;
            }
        for (int o = SHF; o < 64; o <<= 1) q += __shfl_xor(q, o);
        colsum[j] = q;
    }
    __syncthreads();
    if (lane < CW) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) red[wm * BN + wn * NJ * CW + j * CW + lane] = colsum[j];
    }
    __syncthreads();
    for (int e = tid; e < 2 * BN; e += 512) {
        const int h = e / BN, c = e - h * BN;
        if (a.M - (m0 + 128 * h) > 0)
            a.part[((tile128 + h) * a.K + n0 + c) * 2 + 1] = red[(2 * h) * BN + c] + red[(2 * h + 1) * BN + c];
    }
}

// BN tile partials, one barrier, VALU-lean (a wave64 VALU op costs 4 cycles;
// the first version's ~1700 per wave, mostly row masks and selects, took ~6 us
// per tile): each lane reduces its own NI*NR rows of a column to (sum, M2 about
// its own mean) in registers — on f32x4 vectors (packed fp32 ops), without row
// masks when all 64 rows of the wave are valid (every tile but the last) — the
// lane groups of a column merge pairwise by Chan's formula over log2(64/CW)
// shuffle steps (sums and M2s are symmetric in the pair, so both lanes get the
// same bits), and the two waves of a 128-row half merge through a small LDS
// scratch (red: [2][WM][BN] floats, outside anything still being read):
//   n = na + nb,  sum = sa + sb,  M2 = M2a + M2b + (mb - ma)^2 * na*nb / n.
// Same quantities as x3_bn_partials (sum, M2 about the half-tile mean).
// A wave covers 16 * NI rows (WM = 4 waves: NI = 4 for the 256-row tiles, 3 for the
// 192-row A3 tiles), so a partial tile (a half tile) holds 32 * NI rows: 128 / 96.
// WMP = 2 (the 160-row A3 tiles, NI = 5): a wave's 80 rows are a whole partial tile,
// written from its lanes after the shuffle merge (no LDS, no WIDE form).
// VEC(i, j): the f32x4 of accumulator rows ROW(i, 0..3) of column block j.
// SC(j): the column's output scale (a power of two: sums scale by it, M2 by its
// square, exactly) when VEC is the unscaled accumulator.
//
// WIDE (full 256-row tiles; scratch of 33 * BN floats that is free once every
// wave is past its last fragment read, e.g. the drained ring): the lanes' (sum,
// M2) go to LDS as they are, and one thread per (128-row half, column) merges
// the four row groups of each wave and then the half's two waves — the order
// and the formulas of the shuffle tree below (equal counts: Chan's factor is
// the constant n/2, the 1/n scalings powers of two), so the partials are the
// same bits, without its 34 dependent lane shuffles and per-merge divisions.
__device__ __forceinline__ void x3_chan_merge(float& s, float& q, float s2, float q2, float inv_n, float f) {
    const float d = s2 * inv_n - s * inv_n;
    s = s + s2;
    q = (q + q2) + d * d * f;
}

template <int BN, int NI, int NJ, int CW, int SHF, int WMP = 4, typename Vec, typename Row, typename Sc>
__device__ __forceinline__ void x3_bn_partials_w(const X3Args& a, float* red, int m0, int n0, int wm, int wn,
                                                 int lane, Vec&& vec, Row&& row, Sc&& sc_of,
                                                 float* wide = nullptr) {
    constexpr int WROWS = 16 * NI;                                   // rows per wave
    if constexpr (CW == 16 && SHF == 16 && WMP == 4 && (NI == 4 || NI == 3)) {
        if (wide != nullptr && m0 + 4 * WROWS <= a.M) {              // block-uniform
            const int q = lane >> 4, r16 = lane & 15;
            constexpr float inv = 1.f / (NI * 4);
            float ls[NJ], lq[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                f32x4 s4 = vec(0, j);
#pragma unroll
                for (int i = 1; i < NI; ++i) s4 += vec(i, j);
                const float s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
                const f32x4 mu = {s * inv, s * inv, s * inv, s * inv};
                f32x4 q4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = 0; i < NI; ++i) {
                    const f32x4 d = vec(i, j) - mu;
                    q4 += d * d;
                }
                ls[j] = s;
                lq[j] = (q4[0] + q4[1]) + (q4[2] + q4[3]);
            }
            lds_sync();                                              // the scratch is free
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int c = wn * NJ * CW + j * CW + r16;
                wide[(wm * 4 + q) * BN + c] = ls[j];
                wide[16 * BN + (wm * 4 + q) * BN + c] = lq[j];
                if (wm == 0 && q == 0) wide[32 * BN + c] = sc_of(j);
            }
            lds_sync();
            for (int t = threadIdx.x; t < 2 * BN; t += blockDim.x) {
                const int h = t / BN, c = t - h * BN;
                float S[2], Q[2];
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    const int w4 = (2 * h + v) * 4;
                    float s[4], qq[4];
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        s[g] = wide[(w4 + g) * BN + c];
                        qq[g] = wide[16 * BN + (w4 + g) * BN + c];
                    }
                    // groups of n1 = 4 * NI rows: Chan's factor n_a n_b / n = n1 / 2, ...
                    constexpr float n1 = 4.f * NI;
                    x3_chan_merge(s[0], qq[0], s[1], qq[1], 1.f / n1, n1 / 2);   // lane pairs l, l ^ 16
                    x3_chan_merge(s[2], qq[2], s[3], qq[3], 1.f / n1, n1 / 2);
                    x3_chan_merge(s[0], qq[0], s[2], qq[2], 1.f / (2 * n1), n1); // then l, l ^ 32
                    S[v] = s[0];
                    Q[v] = qq[0];
                }
                x3_chan_merge(S[0], Q[0], S[1], Q[1], 1.f / (16 * NI), 8.f * NI);   // even wave, odd wave
                const float sc = wide[32 * BN + c];
                const long tile128 = (long)(m0 / (2 * WROWS)) + h;
                a.part[(tile128 * a.K + n0 + c) * 2 + 0] = S[0] * sc;
                a.part[(tile128 * a.K + n0 + c) * 2 + 1] = Q[0] * (sc * sc);
            }
            return;
        }
    }
    float* rs = red;                                                 // [WM][BN] wave sums
    float* rq = red + 4 * BN;                                        // [WM][BN] wave M2
    const int nw = min(WROWS, max(0, a.M - (m0 + WROWS * wm)));    // valid rows of this wave (a prefix)
    float ls[NJ], lq[NJ], ln;
    if (nw == WROWS) {                                               // every row valid: no masks
        ln = (float)(NI * 4);
        constexpr float inv = 1.f / (NI * 4);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            f32x4 s4 = vec(0, j);
#pragma unroll
            for (int i = 1; i < NI; ++i) s4 += vec(i, j);
            const float s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
            const f32x4 mu = {s * inv, s * inv, s * inv, s * inv};
            f32x4 q4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const f32x4 d = vec(i, j) - mu;
                q4 += d * d;
            }
            ls[j] = s;
            lq[j] = (q4[0] + q4[1]) + (q4[2] + q4[3]);
        }
    } else {
        ln = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) ln += (row(i, r) < a.M) ? 1.f : 0.f;
        const float linv = ln > 0.f ? 1.f / ln : 0.f;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) s += (row(i, r) < a.M) ? vec(i, j)[r] : 0.f;
            const float mu = s * linv;
            float q = 0.f;
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float d = vec(i, j)[r] - mu;
                    q += (row(i, r) < a.M) ? d * d : 0.f;
                }
            ls[j] = s;
            lq[j] = q;
        }
    }
    // pairwise Chan merge across the lane groups of a column (counts ride along)
    for (int o = SHF; o < 64; o <<= 1) {
        const float nb = __shfl_xor(ln, o);
        const float nt = ln + nb;
        const float f = nt > 0.f ? ln * nb / nt : 0.f;
        const float ia = ln > 0.f ? 1.f / ln : 0.f, ib = nb > 0.f ? 1.f / nb : 0.f;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const float sb = __shfl_xor(ls[j], o), qb = __shfl_xor(lq[j], o);
            const float d = sb * ib - ls[j] * ia;
            ls[j] = ls[j] + sb;
            lq[j] = (lq[j] + qb) + d * d * f;
        }
        ln = nt;
    }
    if constexpr (WMP == 2) {              // 2 waves in M (160-row tiles): a wave IS a partial tile
        if (nw == 0 || lane >= CW) return;
        const long pt = (long)(m0 / WROWS) + wm;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int c = wn * NJ * CW + j * CW + lane;
            const float sc = sc_of(j);
            a.part[(pt * a.K + n0 + c) * 2 + 0] = ls[j] * sc;
            a.part[(pt * a.K + n0 + c) * 2 + 1] = lq[j] * (sc * sc);
        }
        return;
    }
    if (lane < CW) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int c = wn * NJ * CW + j * CW + lane;
            rs[wm * BN + c] = ls[j];
            rq[wm * BN + c] = lq[j];
        }
    }
    lds_sync();
    const int nb = min(WROWS, max(0, a.M - (m0 + WROWS * (wm | 1))));   // valid rows of the odd wave of the half
    if ((wm & 1) || nw == 0 || lane >= CW) return;
    const long tile128 = (long)(m0 / (2 * WROWS)) + (wm >> 1);
    const float ia = 1.f / (float)nw, ib = nb > 0 ? 1.f / (float)nb : 0.f;
    const float f = (float)nw * (float)nb / (float)(nw + nb);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int c = wn * NJ * CW + j * CW + lane;
        const float sa = rs[wm * BN + c], qa = rq[wm * BN + c];
        const float sb = rs[(wm + 1) * BN + c], qb = rq[(wm + 1) * BN + c];
        const float d = sb * ib - sa * ia;
        const float sum = nb > 0 ? sa + sb : sa;
        const float m2 = nb > 0 ? (qa + qb) + d * d * f : qa;
        const float sc = sc_of(j);
        a.part[(tile128 * a.K + n0 + c) * 2 + 0] = sum * sc;
        a.part[(tile128 * a.K + n0 + c) * 2 + 1] = m2 * (sc * sc);
    }
}

// fp16 output tile staged in LDS ([256][BN + 8] halves: the 16-B row pad makes
// the fragment-layout ds_write_b16s conflict-free) and written as whole 16-B
// row chunks: 8x fewer store instructions than per-element fp16 stores, full
// 128-B lines — the epilogue of the short-K 1x1 convs of config C4 is most of
// their time.
template <int BN>
__device__ __forceinline__ void x3_store_tile_f16(const X3Args& a, const char* smem, int m0, int n0, int tid) {
    constexpr int CH = BN / 8, PITCH = BN + 8;
#pragma unroll 4
    for (int e = tid; e < 256 * CH; e += 512) {
        const int row = e / CH, cc = e - row * CH;
        const int m = m0 + row;
        if (m < a.M)
            x3_st16((uint4*)(a.y16 + (long)m * a.K + n0 + cc * 8), *(const uint4*)(smem + (row * PITCH + cc * 8) * 2), a.st_kind, 1);
    }
}

// BN-apply epilogue of the fp16 tile (hkp_conv2d_fwd_f16_bn): the staged fp16 y
// chunk, x scale + shift, + the residual chunk (raw or scaled + shifted), ReLU —
// bn_apply_f16's arithmetic on the same fp16 y, so the fused path returns what
// conv + hkp_bn_apply_f16 would with the same scale/shift.  ssl: LDS [4][BN]
// (scale, shift, residual scale, residual shift of the tile's columns).  A
// thread always handles the same 8 channels (512 % (BN/8) == 0).
template <int BN>
struct X3Res {
    static constexpr int NPT = 256 * (BN / 8) / 512;     // 16-B chunks per thread
    f16x8 r[NPT];
};
// the residual chunks this thread's store loop will use, loaded before the tile
// is staged (the loads of a whole tile in flight at once: a per-chunk load in
// the store loop exposed its HBM latency ~4 times per tile)
template <int BN>
__device__ __forceinline__ X3Res<BN> x3_ep_res_load(const X3Args& a, int m0, int n0, int tid) {
    constexpr int CH = BN / 8;
    X3Res<BN> res;
    const int cc = tid % CH;
#pragma unroll
    for (int u = 0; u < X3Res<BN>::NPT; ++u) {
        const int row = (tid + 512 * u) / CH, m = m0 + row;
        res.r[u] = f16x8{};
        if (a.ep_res && m < a.M)
            res.r[u] = __builtin_nontemporal_load((const f16x8*)(a.ep_res + (long)m * a.K + n0 + cc * 8));
    }
    return res;
}

template <int BN>
__device__ __forceinline__ void x3_store_tile_f16_bn(const X3Args& a, const char* smem, const float* ssl,
                                                     const X3Res<BN>& res, int m0, int n0, int tid) {
    constexpr int CH = BN / 8, PITCH = BN + 8;
    static_assert(512 % CH == 0, "fixed channels per thread");
    const int cc = tid % CH;
    float sa[8], sb[8], ra[8], rb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        sa[e] = ssl[cc * 8 + e];
        sb[e] = ssl[BN + cc * 8 + e];
        ra[e] = ssl[2 * BN + cc * 8 + e];
        rb[e] = ssl[3 * BN + cc * 8 + e];
    }
    const bool hres = a.ep_res != nullptr, rsc = a.ep_rss != nullptr, relu = a.ep_relu != 0;
#pragma unroll
    for (int u = 0; u < X3Res<BN>::NPT; ++u) {
        const int row = (tid + 512 * u) / CH;
        const int m = m0 + row;
        if (m >= a.M) continue;
        const long off = (long)m * a.K + n0 + cc * 8;
        const f16x8 v = *(const f16x8*)(smem + (row * PITCH + cc * 8) * 2);
        const f16x8 r = res.r[u];
        f16x8 h;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float o = __fadd_rn(__fmul_rn((float)v[k], sa[k]), sb[k]);
            if (hres) o = rsc ? __fadd_rn(o, __fadd_rn(__fmul_rn((float)r[k], ra[k]), rb[k])) : __fadd_rn(o, (float)r[k]);
            if (relu) o = o > 0.f ? o : 0.f;
            h[k] = (_Float16)o;
        }
        x3_st16((f16x8*)(a.y16 + off), h, a.st_kind, 2);
    }
}

// the fused epilogue's per-column parameters: thread tid < 2*BN holds scale (tid
// < BN) or shift of column tid % BN, and the residual's; loaded before the tile
// is staged (their latency hides behind it), written to LDS after
struct X3EpSS {
    float v0 = 0.f, v1 = 0.f;
};
template <int BN>
__device__ __forceinline__ X3EpSS x3_ep_load(const X3Args& a, int n0, int tid) {
    X3EpSS r;
    if (a.ep_ss && tid < 2 * BN) {
        const int h = tid / BN, c = tid - h * BN;
        r.v0 = a.ep_ss[h * a.K + n0 + c];
        r.v1 = a.ep_rss ? a.ep_rss[h * a.K + n0 + c] : 0.f;
    }
    return r;
}
template <int BN>
__device__ __forceinline__ void x3_ep_store(float* ssl, const X3EpSS& r, int tid) {
    if (tid < 2 * BN) {
        ssl[tid] = r.v0;
        ssl[2 * BN + tid] = r.v1;
    }
}

// Mainloop + epilogue of the 16x16x32-MFMA bodies: one k32 step per half of a
// 128-B stage row (LDS ring, DMA issue and the swizzled rows exactly as the
// 32x32 path).  Wave tile 64 x BN/2 = UM x UN 16x16 tiles.
// Fragment read: lane reads row (lane & 15) of a 16-row tile, 16-B chunk
// (lane >> 4) (first half) / 4 + (lane >> 4) (second half): with the
// (row >> 1) & 7 chunk swizzle every ds_read_b128 lane group covers the 64 banks
// once.  Output fragment: lane holds column (lane & 15), rows 4 * (lane >> 4) + 0..3.
// Pipeline per K-step t (NST 3): [issue DMA t+NST-1] wait own DMA of t+1 (+ this
// wave's reads of t), barrier, [read A frags of t+1] then per column block j:
// [MFMAs of t with B_j] [refill B_j with t+1's].  NST 2 (256x256; 256x64 pairs):
// A single-buffered, t+2's DMA issued right after the barrier into t's buffer.
template <int BN, int NST, int STAGE, int GL, int P, bool A3, int GA, int BM, typename Issue, typename IssueA,
          typename IssueB>
__device__ __forceinline__ void conv_x3_mf16_body(const X3Args& a, char* smem, int tile, int ks, int nks, bool partial,
                                                  int m0, int n0, int wm, int wn, int lane, int tid,
                                                  Issue& issue_next, IssueA& issue_a, IssueB& issue_b) {
    constexpr int WM = x3_wm(BM), WN = 8 / WM, ROW = 128;
    constexpr int UM = BM / (WM * 16), UN = BN / (WN * 16);
    constexpr int NMC = x3_nprod(P) * UM;           // MFMAs per column block per K-step
    static_assert(BM == 256 || (A3 && (BM == 192 || BM == 160) && P != 1),
                  "192- / 160-row tiles: the A3 body, packed operands");
    constexpr bool PAIRB = BN == 64 && NST == 2;    // the 256x64 two-blocks-per-CU tiles
    static_assert(!A3 || (BN == 256 && NST == 2) || (BN == 128 && BM == 160), "A3: 256-wide tiles (128: 160 rows)");
    // PAIRB and A3 have no LDS past the ring: the epilogue's scratch is the drained
    // ring and the column scales are loaded in the epilogue
    constexpr bool RINGSCR = PAIRB || A3;
    constexpr int RED_OFF = RINGSCR ? 0 : x3_lds_bytes(BN, PAIRB, P);
    constexpr int LDS_ALL = A3 ? x3_a3_lds(BM, BN) : x3_lds_bytes(BN, PAIRB, P) + x3_red_bytes(BN, PAIRB);
    float* const scl = (float*)(smem + RED_OFF + 2 * 4 * BN * 4);   // [BN] column scales (!RINGSCR)
    float sclv = 1.f;                              // issued before the fill, stored after it
    if constexpr (!RINGSCR) {
        if (tid < BN) sclv = (a.wscale ? a.wscale[n0 + tid] : 1.f) * (a.amax ? 1.f / pow2_scale_for(a.amax) : 1.f);
    }
    auto store_scl = [&]() {
        if constexpr (!RINGSCR) {
            if (tid < BN) scl[tid] = sclv;
        }
    };
    const int r16 = lane & 15, q = lane >> 4;
    const int sw = (r16 >> 1) & 7;                 // the DMA's swizzle of every row ≡ r16 (mod 16)
    const int fo_h = r16 * ROW + ((q ^ sw) << 4), fo_l = r16 * ROW + (((4 + q) ^ sw) << 4);
    // A3: A stages at [0, 3*BM*ROW), B stages past them, each its own ring
    const int a_base = (wm * UM * 16) * ROW, b_base = ((A3 ? 0 : BM) + wn * UN * 16) * ROW;

    f32x4 acc[UM][UN];
#pragma unroll
    for (int i = 0; i < UM; ++i)
#pragma unroll
        for (int j = 0; j < UN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    struct FA {
        f16x8 h[UM], l[UM];
    };
    f16x8 bh[UN], bl[UN];
    auto read_a = [&](FA& f, const char* st) {
#pragma unroll
        for (int i = 0; i < UM; ++i) {
            f.h[i] = *(const f16x8*)(st + a_base + i * 16 * ROW + fo_h);
            f.l[i] = *(const f16x8*)(st + a_base + i * 16 * ROW + fo_l);
        }
    };
    auto read_b = [&](int j, const char* st) {
        bh[j] = *(const f16x8*)(st + b_base + j * 16 * ROW + fo_h);
        bl[j] = *(const f16x8*)(st + b_base + j * 16 * ROW + fo_l);
    };
    auto mfma = [](const f16x8& x, const f16x8& y, const f32x4& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(x, y, c, 0, 0, 0);
    };
    auto mma_col = [&](const FA& f, int j) {
#pragma unroll
        for (int i = 0; i < UM; ++i) x3_products<P>(acc[i][j], f.h[i], f.l[i], bh[j], bl[j], mfma);
    };

    // The next stage's DMA (GL pieces per wave) is issued inside the K-step's
    // MFMA stream, one piece per column block, instead of as a burst after the
    // barrier (a piece costs ~60 issue cycles, MI355X_MICROARCH.md; the burst
    // left every SIMD without an MFMA to issue right after each barrier).  The
    // last K-steps issue nothing (peeled: no branch inside the scheduled region).
    auto sched_kstep = [&](const bool dma) {
#pragma unroll
        for (int j = 0; j < UN; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, NMC, 0);     // column j's MFMAs
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);       // refill B_j
            if (dma && j * ((GL + UN - 1) / UN) < GL)
                __builtin_amdgcn_sched_group_barrier(0x020, (GL + UN - 1) / UN, 0);   // DMA pieces
        }
    };
    // the same with NP DMA pieces in the step (A3: B only, or A and B)
    auto sched_kstep_n = [&](auto np) {
        constexpr int NP = decltype(np)::value;
#pragma unroll
        for (int j = 0; j < UN; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, NMC, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            if (NP > 0 && j * ((NP + UN - 1) / UN) < NP)
                __builtin_amdgcn_sched_group_barrier(0x020, (NP + UN - 1) / UN, 0);
        }
    };
    if constexpr (A3) {
        // A3: the NST 2 schedule below with A one stage further ahead.  Issue order
        // per K-step t (after its barrier): B(t+2) into B's slot of t, then A(t+3)
        // into A's slot of t (both read into registers during step t-1); so at step
        // t's top, waiting until only A(t+2) is in flight (vmcnt GA) retires A(t+1)
        // and B(t+1).  Prologue order A0 B0 A1 B1 A2.
        constexpr int GB = GL - GA;
        const char* const bring = smem + 3 * BM * ROW;
        issue_a();
        issue_b();
        if (nks > 1) {
            issue_a();
            issue_b();
        }
        if (nks > 2) issue_a();
        if (nks > 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL + GA) : "memory");
        else if (nks > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        x3_stamp(a, 1);
        const int wv = wm * 2 + wn;
        if (a.prio == 1 && wv >= 4) __builtin_amdgcn_s_setprio(1);
        if (a.prio == 2 && wv < 4) __builtin_amdgcn_s_setprio(1);
        FA fa;
        read_a(fa, smem);
#pragma unroll
        for (int j = 0; j < UN; ++j) read_b(j, bring);
        int ca = 0, cb = 0;
        // one K-step: NP DMA pieces issued (GL: B(t+2) and A(t+3); GB: B only; 0),
        // WA: A(t+2) may stay in flight at the top
        auto kstep = [&](auto np, auto wa) {
            constexpr int NP = decltype(np)::value;
            if constexpr (decltype(wa)::value) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(GA) : "memory");
            else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            lds_barrier();
            ca = ca == 2 ? 0 : ca + 1;
            cb ^= 1;
            const char* sta = smem + ca * (BM * ROW);
            const char* stb = bring + cb * (BN * ROW);
            if constexpr (NP > 0) issue_b();
            if constexpr (NP == GL) issue_a();
#pragma unroll
            for (int j = 0; j < UN; ++j) {
                mma_col(fa, j);
                read_b(j, stb);
            }
            read_a(fa, sta);
            sched_kstep_n(np);
            __builtin_amdgcn_sched_group_barrier(0x100, 2 * UM, 0);      // next A frags
            __builtin_amdgcn_sched_barrier(0);
        };
        using IGL = std::integral_constant<int, GL>;
        using IGB = std::integral_constant<int, GB>;
        using I0 = std::integral_constant<int, 0>;
        int t = 0;
        for (; t + 3 < nks; ++t) kstep(IGL{}, std::true_type{});
        if (t + 2 < nks) {
            kstep(IGB{}, std::true_type{});
            ++t;
        }
        if (t + 1 < nks) kstep(I0{}, std::false_type{});
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < UN; ++j) mma_col(fa, j);
        if (a.prio) __builtin_amdgcn_s_setprio(0);
    } else if constexpr (NST == 2) {
        // 2-stage ring (256x256 tiles; 256x64 at two blocks per CU), A single-buffered
        // (registers: 128 acc + 32 A + 64 B): per K-step t — wait own DMA of t+1,
        // barrier, then per column j [MFMAs of t with B_j] [refill B_j with t+1's]
        // [a DMA piece of t+2 into t's buffer, read before the barrier], then A of
        // t+1 (its latency covered by the SIMD's other wave)
        issue_next();
        if (nks > 1) issue_next();
        store_scl();
        if (nks > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        x3_stamp(a, 1);
        FA fa;
        read_a(fa, smem);
#pragma unroll
        for (int j = 0; j < UN; ++j) read_b(j, smem);
        int cur = 0;
        auto kstep = [&](const bool dma) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            lds_barrier();
            cur ^= 1;
            const char* st = smem + cur * STAGE;
            if (dma) issue_next();
#pragma unroll
            for (int j = 0; j < UN; ++j) {
                mma_col(fa, j);
                read_b(j, st);
            }
            read_a(fa, st);
            sched_kstep(dma);
            __builtin_amdgcn_sched_group_barrier(0x100, 2 * UM, 0);      // next A frags
            __builtin_amdgcn_sched_barrier(0);
        };
        int t = 0;
        for (; t + 2 < nks; ++t) kstep(true);
        if (t + 1 < nks) kstep(false);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < UN; ++j) mma_col(fa, j);
    } else {
        // 3-stage ring (256x128 tiles), the 2-stage body's schedule with two
        // stages of DMA lead: A single-buffered, per K-step t — wait own DMA of
        // t+1 (t+2 stays in flight), barrier, then per column j [MFMAs of t with
        // B_j] [refill B_j with t+1's] [a DMA piece of t+3 into t's buffer: t's
        // fragments were all read during step t-1], then A of t+1.  (The burst
        // of t+2's DMA before the barrier, with A double-buffered, left every SIMD
        // without an MFMA to issue after each barrier.)
        static_assert(NST == 3, "stage t+3 goes into stage t's buffer");
        for (int s = 0; s < NST; ++s)
            if (s < nks) issue_next();
        store_scl();
        {
            const int after = std::min(nks, NST) - 1;         // stages in flight past stage 0
            if (after >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GL) : "memory");
            else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        lds_barrier();
        x3_stamp(a, 1);
        FA fa;
        read_a(fa, smem);
#pragma unroll
        for (int j = 0; j < UN; ++j) read_b(j, smem);
        int cur = 0;
        auto kstep = [&](const int t, const bool dma) {
            if (t + 2 < nks) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(GL) : "memory");
            else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            lds_barrier();
            cur = cur == NST - 1 ? 0 : cur + 1;
            const char* st = smem + cur * STAGE;
            if (dma) issue_next();
#pragma unroll
            for (int j = 0; j < UN; ++j) {
                mma_col(fa, j);
                read_b(j, st);
            }
            read_a(fa, st);
            sched_kstep(dma);
            __builtin_amdgcn_sched_group_barrier(0x100, 2 * UM, 0);      // next A frags
            __builtin_amdgcn_sched_barrier(0);
        };
        int t = 0;
        for (; t + 3 < nks; ++t) kstep(t, true);
        for (; t + 1 < nks; ++t) kstep(t, false);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < UN; ++j) mma_col(fa, j);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA in flight into the ring past here
    x3_stamp(a, 2);

    if constexpr (BM == 256) {             // (the 192- / 160-row grids run whole tiles)
        if (partial) {                     // stream-K: fold the tile's segments
            auto get = [&](int v) -> f32x4 { return acc[v / UN][v % UN]; };
            auto set = [&](int v, f32x4 y) { acc[v / UN][v % UN] = y; };
            if (!sk_combine<UM * UN>(a, tile, tid, smem, get, set)) return;
        }
    }
    const int rbase = m0 + wm * UM * 16 + 4 * q;
    // column scale (weight scale x gradient scale): the prefetched LDS copy, or
    // (PAIRB, A3) loaded now
    auto col_scale = [&](int c) -> float {
        if constexpr (RINGSCR) return (a.wscale ? a.wscale[n0 + c] : 1.f) * (a.amax ? 1.f / pow2_scale_for(a.amax) : 1.f);
        else return scl[c];
    };
    if constexpr (P == 1) {                // fp16 output: partials, scale, LDS-staged store
        float sc[UN];
#pragma unroll
        for (int j = 0; j < UN; ++j) sc[j] = col_scale(wn * UN * 16 + j * 16 + r16);
        if (a.part) {
            if constexpr (RINGSCR) lds_sync();         // the scratch is the ring
            x3_bn_partials_w<BN, UM, UN, 16, 16, WM>(
                a, (float*)(smem + RED_OFF), m0, n0, wm, wn, lane, [&](int i, int j) { return acc[i][j]; },
                [&](int i, int r) { return rbase + i * 16 + r; }, [&](int j) { return sc[j]; }, (float*)smem);
        }
        const X3EpSS eps = x3_ep_load<BN>(a, n0, tid);
        X3Res<BN> eres;
        if (a.ep_ss) eres = x3_ep_res_load<BN>(a, m0, n0, tid);
        lds_sync();                        // the ring is free
        x3_stamp(a, 3);
        _Float16* t = (_Float16*)smem;
        constexpr int PITCH = BN + 8;
        constexpr int SS_OFF = 256 * PITCH * 2;
        static_assert(SS_OFF + 4 * BN * 4 <= LDS_ALL, "epilogue LDS");
#pragma unroll
        for (int i = 0; i < UM; ++i)
#pragma unroll
            for (int j = 0; j < UN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    t[(wm * UM * 16 + i * 16 + 4 * q + r) * PITCH + wn * UN * 16 + j * 16 + r16] =
                        (_Float16)(acc[i][j][r] * sc[j]);
        if (a.ep_ss) x3_ep_store<BN>((float*)(smem + SS_OFF), eps, tid);
        lds_sync();
        x3_stamp(a, 4);
        if (a.ep_ss) x3_store_tile_f16_bn<BN>(a, smem, (const float*)(smem + SS_OFF), eres, m0, n0, tid);
        else x3_store_tile_f16<BN>(a, smem, m0, n0, tid);
        x3_stamp(a, 5);
        return;
    }
    // ---- epilogue (fp32 output): BN partials, then the scaled tile ----
    float sc[UN];
#pragma unroll
    for (int j = 0; j < UN; ++j) sc[j] = col_scale(wn * UN * 16 + j * 16 + r16);
    if (a.part) {
        if constexpr (RINGSCR) lds_sync();             // the scratch is the ring
        x3_bn_partials_w<BN, UM, UN, 16, 16, WM>(
            a, (float*)(smem + RED_OFF), m0, n0, wm, wn, lane, [&](int i, int j) { return acc[i][j]; },
            [&](int i, int r) { return rbase + i * 16 + r; }, [&](int j) { return sc[j]; }, (float*)smem);
    }
    x3_stamp(a, 3);
    {
        // The output tile is staged through the (drained) ring as fp32 rows and
        // written as whole 16-B row chunks — 32 store instructions per thread,
        // full 128-B lines (a phase output row of the strided dgrad is still 4
        // contiguous channels per chunk; the addend is read the same way).  The
        // fragment-layout stores (128 4-B stores per thread, 64-B pieces) of
        // every CU at once took ~34 us per C2 layer4 tile (10 %): more than a
        // wave's 63 outstanding memory ops, so the waves stalled on their
        // completion instead of ending and letting the next block start.
        // 256-wide tiles stage half the rows per pass (128 KiB).
        constexpr int PASSES = BN == 256 ? 2 : 1, RPP = BM / PASSES, PITCH = BN + 4, C4 = BN / 4;
        static_assert(RPP * PITCH * 4 <= LDS_ALL, "staging");
        float* t = (float*)smem;
        lds_sync();                                    // every wave done with the ring and the partials' scratch
#pragma unroll
        for (int h = 0; h < PASSES; ++h) {
            if (PASSES == 1 || (wm * UM * 16) / RPP == h) {          // the pass holding this wave's rows
#pragma unroll
                for (int i = 0; i < UM; ++i)
#pragma unroll
                    for (int j = 0; j < UN; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            t[(wm * UM * 16 + i * 16 + 4 * q + r - h * RPP) * PITCH + wn * UN * 16 + j * 16 + r16] =
                                acc[i][j][r] * sc[j];
            }
            lds_sync();
            if (!a.add && !a.ost) {
#pragma unroll 4
                for (int e = tid; e < RPP * C4; e += 512) {
                    const int row = e / C4, c4 = e - row * C4;
                    const int m = m0 + h * RPP + row;
                    if (m < a.M)
                        // nontemporal (in-process A/B, profiles/r05_store_ab.log: C2 1825.7 ->
                        // 1841.1 img/s; C3 training 464.6 both)
                        x3_st16((f32x4*)(a.y + (long)m * a.K + n0 + c4 * 4), *(const f32x4*)(t + row * PITCH + c4 * 4),
                                a.st_kind, 2);
                }
            } else {
#pragma unroll 2
                for (int e = tid; e < RPP * C4; e += 512) {
                    const int row = e / C4, c4 = e - row * C4;
                    const long off = x3_out_off(a, m0 + h * RPP + row, n0 + c4 * 4);
                    if (off >= 0) {
                        f32x4 v = *(const f32x4*)(t + row * PITCH + c4 * 4);
                        if (a.add) {
                            const f32x4 ad = *(const f32x4*)(a.add + off);
#pragma unroll
                            for (int k = 0; k < 4; ++k) v[k] = v[k] + ad[k];
                        }
                        *(f32x4*)(a.y + off) = v;
                    }
                }
            }
            if (h + 1 < PASSES) lds_sync();            // the next pass overwrites the rows just read
        }
    }
    x3_stamp(a, 4);
    x3_stamp(a, 5);
}

// STEM: the 7x7/s2 stem on the zero-padded NHWC4 image planes of
// hkp_stem_pack_x3 (a.H/a.W = padded size, stride 2, pad 0, R = 7, S = 1: one
// K-step per filter row = 8 taps x 4 channels; logical chunk j of a row holds
// padded pixels 2wo+2j, 2wo+2j+1 from the hi plane (j < 4) or the lo plane).
// MFD: MFMA shape, 32 = v_mfma_f32_32x32x16_f16 (two k16 slices per 128-B
// stage), 16 = v_mfma_f32_16x16x32_f16 (one k32 step per stage half; same cycles
// per FLOP, lower power per FLOP, so the chip holds a higher clock under load —
// MI355X_MICROARCH.md "DVFS give-back" item 7).
// P: operand layout and products (x3_products) — 3 packed f16x3 split, 2 / 4
// packed split with two of its three products, 1 plain fp16.
template <int BN, bool STEM, bool PAIR, int MFD, int P, bool A3 = false, int BM = 256>
__device__ __forceinline__ void conv_x3_tile(const X3Args& a, char* smem, int tile, int ks, int nks, bool partial) {
    constexpr int WM = x3_wm(BM), WN = 8 / WM;
    constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
    constexpr int ROW = 128;                       // bytes per LDS row (one packed line)
    constexpr int CPR = ROW / 16;                  // 16-B chunks per row
    constexpr int RPI = 1024 / ROW;                // rows per DMA wave-instruction
    constexpr int NST = x3_nst(BN, PAIR);          // LDS ring depth
    constexpr int STAGE = (BM + BN) * ROW;
    constexpr int GA = (BM / RPI + 7) / 8;         // A DMA instructions per wave per stage (rounded up)
    constexpr bool A_SINK = BM / RPI % 8 != 0;    // pieces past row BM load the zero line into a sink
    constexpr int GBT = BN / RPI;                  // B DMA instructions per stage (all waves)
    constexpr int GB = GBT >= 8 ? GBT / 8 : 1;     // per wave (GBT < 8: waves duplicate, same bytes)
    constexpr int GL = GA + GB;                    // DMA instructions per wave per stage
    static_assert(MFD == 16 || MFD == 32, "bad conv_x3 MFMA shape");
    static_assert(P == 3 || ((P == 1 || P == 2 || P == 4) && !STEM), "bad conv_x3 operand layout");
    static_assert(!(MFD == 32 && BN == 256), "256x256 tiles run the 16x16x32 body");
    static_assert(NST * STAGE <= 160 * 1024, "LDS");
    static_assert(!A3 || ((BN == 256 || (BN == 128 && BM == 160)) && !STEM && !PAIR && MFD == 16),
                  "A3: the 16x16x32 body on 256-wide tiles (128-wide: 160 rows)");
    static_assert(BM == 256 || (A3 && (BM == 192 || BM == 160) && x3_packed(P)), "192- / 160-row tiles: A3, packed");
    static_assert(!A_SINK || A3, "the A sink is the A3 body's");

    const int mt = tile / a.n_tiles, nt = tile - mt * a.n_tiles;
    const int m0 = (mt + a.mt0) * BM, n0 = nt * BN;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w / WN, wn = w % WN;

    // swizzled physical chunk of a logical chunk in row r
    auto swz = [](int row) { return (row >> 1) & 7; };
    // halves offset, inside a packed line, of logical chunk L
    auto lofs = [&](int L) -> long {
        if constexpr (STEM) return (L >> 2) * a.plane + (L & 3) * 8;
        else return L * 8;
    };

    // ---- DMA source bookkeeping (rows this lane feeds) ----
    // Per row: the image-space origin (hb, wb) of its receptive field packed as
    // two int16, and the unsigned 32-bit element offset of that (possibly
    // padded-out) origin pixel from xbase = a.xs - pad*(W+1)*cstride (the
    // furthest a padded-out origin reaches before a.xs); a tap adds a
    // wave-uniform offset.  Rows past M get an origin that is never in-bounds.  B
    // rows: 32-bit offsets from a.ws.  (64-bit pointers here pushed the 256x256
    // kernels past 256 VGPRs; the spill reload inside the DMA issue waited
    // vmcnt(0) on every K-step.  The host checks the operand sizes fit.)
    const int cstride = STEM ? 4 : a.cch * 64;     // halves per pixel
    const long xbias = (long)a.pad * (a.W + 1) * cstride;
    const _Float16* xbase = a.xs - xbias;
    int a_org[GA];
    unsigned a_off[GA];
#pragma unroll
    for (int i = 0; i < GA; ++i) {
        const int row = RPI * (w * GA + i) + lane / CPR;
        const int Lc = (lane % CPR) ^ swz(row);
        const long L = lofs(Lc);
#ifdef HKP_AB_KNOBS
        const int m = a.a_wrap ? (m0 + row) % a.a_wrap : m0 + row;
#else
        const int m = m0 + row;
#endif
        int hb = -16384, wb = -16384;
        long off = 0;
        if (m < a.M && (!A_SINK || RPI * (w * GA + i) < BM)) {
            const int hw = a.Ho * a.Wo;
            const int n = m / hw, rem = m - n * hw;
            const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
            hb = ho * a.stride - a.pad;
            wb = wo * a.stride - a.pad;
            off = (((long)n * a.H + hb) * a.W + wb) * cstride + L;
        }
        a_org[i] = (int)(((unsigned)hb << 16) | ((unsigned)wb & 0xFFFFu));
        a_off[i] = (unsigned)(off + xbias);
    }
    const int bline = a.RS * a.cch * 64;           // halves per weight row (output channel)
    int b_off[GB], b_dst[GB];
#pragma unroll
    for (int j = 0; j < GB; ++j) {
        const int bi = (w * GB + j) % GBT;
        const int row = RPI * bi + lane / CPR;
        const int Lc = (lane % CPR) ^ swz(row);
        b_off[j] = (n0 + row) * bline + (STEM ? Lc * 8 : (int)lofs(Lc));
        b_dst[j] = (BM + RPI * bi) * ROW;
    }
    const _Float16* zero = (const _Float16*)g_x3_zero_line;

    // staging state of the next K-step to issue (wave-uniform, advanced per issue)
    // (a stream-K segment starts at K-step ks: channel group outer, tap inner)
    int q_buf = 0;
    int q_cc = ks / a.RS;
    int q_tap = ks - q_cc * a.RS;
    int q_rr = q_tap / a.S, q_ss = q_tap - q_rr * a.S;
    auto issue_next = [&]() {
        char* st = smem + q_buf * STAGE;
        const int dh = q_rr * a.dil, dw = q_ss * a.dil;
        const long toff = ((long)dh * a.W + dw) * cstride + q_cc * 64;
#pragma unroll
        for (int i = 0; i < GA; ++i) {
            const int hb = a_org[i] >> 16, wb = (int)(short)(a_org[i] & 0xFFFF);
            const bool in = (unsigned)(hb + dh) < (unsigned)a.H && (unsigned)(wb + dw) < (unsigned)a.W;
            glds16(in ? xbase + ((unsigned long)a_off[i] + toff) : zero, st + (RPI * (w * GA + i)) * ROW);
        }
        const int boff = (q_tap * a.cch + q_cc) * 64;
#pragma unroll
        for (int j = 0; j < GB; ++j) glds16(a.ws + (unsigned)(b_off[j] + boff), st + b_dst[j]);
        q_buf = q_buf == NST - 1 ? 0 : q_buf + 1;
        if (++q_ss == a.S) {
            q_ss = 0;
            ++q_rr;
        }
        if (++q_tap == a.RS) {
            q_tap = 0;
            q_rr = 0;
            ++q_cc;
        }
    };

    // A3: A and B stages in rings of their own (3 and 2 deep), A issued one K-step
    // ahead of B — each with its own (channel group, tap) position
    int qa_buf = 0, qa_cc = q_cc, qa_tap = q_tap, qa_rr = q_rr, qa_ss = q_ss;
    int qb_buf = 0, qb_cc = q_cc, qb_tap = q_tap;
    // issue_a(): the next A stage, then the advance to the stage after it
    auto issue_a = [&]() {
        {
            char* st = smem + qa_buf * (BM * ROW);
            const int dh = qa_rr * a.dil, dw = qa_ss * a.dil;
            const long toff = ((long)dh * a.W + dw) * cstride + qa_cc * 64;
#pragma unroll
            for (int i = 0; i < GA; ++i) {
                const int hb = a_org[i] >> 16, wb = (int)(short)(a_org[i] & 0xFFFF);
                const bool in = (unsigned)(hb + dh) < (unsigned)a.H && (unsigned)(wb + dw) < (unsigned)a.W;
                const int prow = RPI * (w * GA + i);
                char* dst = st + prow * ROW;
                if constexpr (A_SINK) dst = prow < BM ? dst : smem + (3 * BM + 2 * BN) * ROW;   // wave-uniform
                glds16(in ? xbase + ((unsigned long)a_off[i] + toff) : zero, dst);
            }
        }
        qa_buf = qa_buf == 2 ? 0 : qa_buf + 1;
        if (++qa_ss == a.S) {
            qa_ss = 0;
            ++qa_rr;
        }
        if (++qa_tap == a.RS) {
            qa_tap = 0;
            qa_rr = 0;
            ++qa_cc;
        }
    };
    auto issue_b = [&]() {
        char* st = smem + 3 * (BM * ROW) + qb_buf * (BN * ROW) - BM * ROW;   // b_dst counts from row BM
        const int boff = (qb_tap * a.cch + qb_cc) * 64;
#pragma unroll
        for (int j = 0; j < GB; ++j) glds16(a.ws + (unsigned)(b_off[j] + boff), st + b_dst[j]);
        qb_buf ^= 1;
        if (++qb_tap == a.RS) {
            qb_tap = 0;
            ++qb_cc;
        }
    };

    if constexpr (MFD == 16) {
        conv_x3_mf16_body<BN, NST, STAGE, GL, P, A3, GA, BM>(a, smem, tile, ks, nks, partial, m0, n0, wm, wn, lane,
                                                             tid, issue_next, issue_a, issue_b);
        return;
    } else {
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // fragment reads: lane reads row (lane&31) of each 32-row tile; logical chunk
    // of k16 slice u (of 2 per row half): 2u + kh (first half) / 4 + 2u + kh
    const int frow = lane & 31, kh = lane >> 5;
    int foff[2][2];
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
#pragma unroll
        for (int u = 0; u < 2; ++u) foff[pl][u] = frow * ROW + ((((CPR / 2) * pl + 2 * u + kh) ^ swz(frow)) << 4);
    const int a_base = (wm * TM * 32) * ROW, b_base = (BM + wn * TN * 32) * ROW;

    struct Frag {
        f16x8 ah[TM], al[TM], bh[TN], bl[TN];
    };
    auto read_frag = [&](Frag& f, const char* st, int u) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            f.ah[i] = *(const f16x8*)(st + a_base + i * 32 * ROW + foff[0][u]);
            f.al[i] = *(const f16x8*)(st + a_base + i * 32 * ROW + foff[1][u]);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            f.bh[j] = *(const f16x8*)(st + b_base + j * 32 * ROW + foff[0][u]);
            f.bl[j] = *(const f16x8*)(st + b_base + j * 32 * ROW + foff[1][u]);
        }
    };
    auto mfma = [](const f16x8& x, const f16x8& y, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(x, y, c, 0, 0, 0);
    };
    auto mma = [&](const Frag& f) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) x3_products<P>(acc[i][j], f.ah[i], f.al[i], f.bh[j], f.bl[j], mfma);
    };
    constexpr int NR = 2 * (TM + TN), NM = x3_nprod(P) * TM * TN;   // ds_reads / MFMAs per k16 slice

    // prologue: NST-1 stages in flight, stage 0 landed everywhere
    issue_next();
    for (int s = 1; s < NST - 1; ++s)
        if (s < nks) issue_next();
    {
        const int after = std::min(nks - 1, NST - 2);   // stages issued after stage 0
        if (after >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();
    Frag f0, f1;
    int cur = 0;
    read_frag(f0, smem, 0);

    // wait for this wave's DMA of stage t+1, given that the stages up to
    // min(nks-1, t+NST-1) have been issued; lgkmcnt(0) retires this wave's
    // fragment reads of the buffer the next DMA will overwrite
    auto wait_next = [&](int t) {
        const int after = std::min(nks - 1, t + NST - 1) - (t + 1);
        if (after >= 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(GL) : "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    };

    // one barrier per K-step, placed between its two k16 halves:
    //   [issue DMA t+NST-1] [read frags u=1 of t] [MFMA u=0 of t]
    //   wait own DMA of t+1, barrier (t+1 landed everywhere; t-1 fully read)
    //   [read frags u=0 of t+1] [MFMA u=1 of t]
    // DMA t+NST-1 overwrites the buffer of t-1, whose reads retired before the
    // previous barrier.  Each half is one basic block so the ds_reads can be
    // interleaved one per MFMA gap.  The last K-step is peeled so the loop body
    // has no branch around the MFMAs (a join of two differently scheduled acc
    // writers costs a full accumulator copy).
    for (int t = 0; t + 1 < nks; ++t) {
        const char* st = smem + cur * STAGE;
        if (t + NST - 1 < nks) issue_next();
        read_frag(f1, st, 1);
        mma(f0);
        interleave<NM, NR>();
        __builtin_amdgcn_sched_barrier(0);       // every MFMA of this half ahead of the wait
        wait_next(t);
        lds_barrier();
        cur = cur == NST - 1 ? 0 : cur + 1;
        mma(f1);
        read_frag(f0, smem + cur * STAGE, 0);
        interleave<NM, NR>();
        __builtin_amdgcn_sched_barrier(0);
    }
    read_frag(f1, smem + cur * STAGE, 1);
    mma(f0);
    mma(f1);

    if (!STEM && partial) {                // stream-K: fold the tile's segments
        auto get = [&](int v) -> f32x4 {
            const f32x16& x = acc[(v >> 2) / TN][(v >> 2) % TN];
            const int q4 = (v & 3) * 4;
            return f32x4{x[q4], x[q4 + 1], x[q4 + 2], x[q4 + 3]};
        };
        auto set = [&](int v, f32x4 y) {
            f32x16& x = acc[(v >> 2) / TN][(v >> 2) % TN];
            const int q4 = (v & 3) * 4;
            x[q4] = y[0]; x[q4 + 1] = y[1]; x[q4 + 2] = y[2]; x[q4 + 3] = y[3];
        };
        if (!sk_combine<TM * TN * 4>(a, tile, tid, smem, get, set)) return;
    }
    const float ginv = a.amax ? 1.f / pow2_scale_for(a.amax) : 1.f;   // exact (power of two)
    const int rbase = m0 + wm * TM * 32 + 4 * kh;
    if constexpr (P == 1) {                // fp16 output: scale, partials, LDS-staged store
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const float sc = (a.wscale ? a.wscale[n0 + wn * TN * 32 + j * 32 + frow] : 1.f) * ginv;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] *= sc;
        }
        if (a.part)
            x3_bn_partials<BN, TM, TN, 16, 32, 32>(
                a, smem, m0, n0, wm, wn, lane, tid, [&](int i, int j, int r) { return acc[i][j][r]; },
                [&](int i, int r) { return rbase + i * 32 + (r & 3) + 8 * (r >> 2); });
        const X3EpSS eps = x3_ep_load<BN>(a, n0, tid);
        X3Res<BN> eres;
        if (a.ep_ss) eres = x3_ep_res_load<BN>(a, m0, n0, tid);
        __syncthreads();
        _Float16* t = (_Float16*)smem;
        constexpr int PITCH = BN + 8;
        constexpr int SS_OFF = 256 * PITCH * 2;
        static_assert(SS_OFF + 4 * BN * 4 <= x3_lds_bytes(BN, PAIR, P) + x3_red_bytes(BN, PAIR), "epilogue LDS");
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    t[(wm * TM * 32 + i * 32 + 4 * kh + (r & 3) + 8 * (r >> 2)) * PITCH + wn * TN * 32 + j * 32 +
                      frow] = (_Float16)acc[i][j][r];
        if (a.ep_ss) x3_ep_store<BN>((float*)(smem + SS_OFF), eps, tid);
        __syncthreads();
        if (a.ep_ss) x3_store_tile_f16_bn<BN>(a, smem, (const float*)(smem + SS_OFF), eres, m0, n0, tid);
        else x3_store_tile_f16<BN>(a, smem, m0, n0, tid);
        return;
    }

    // ---- epilogue: NHWC store (x scales, + addend) + BN partials per 128-row tile ----
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * TN * 32 + j * 32 + frow;
        const float sc = (a.wscale ? a.wscale[n] : 1.f) * ginv;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            // output offsets of the fragment's 16 rows (-1: past M), then all its
            // addend loads in flight at once (one exposed latency per fragment)
            long off[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) off[r] = x3_out_off(a, rbase + i * 32 + (r & 3) + 8 * (r >> 2), n);
            float av[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) av[r] = (a.add && off[r] >= 0) ? a.add[off[r]] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[i][j][r] *= sc;
                x3_store(a, off[r], acc[i][j][r], av[r]);
            }
        }
    }
    if (a.part == nullptr) return;
    x3_bn_partials<BN, TM, TN, 16, 32, 32>(
        a, smem, m0, n0, wm, wn, lane, tid, [&](int i, int j, int r) { return acc[i][j][r]; },
        [&](int i, int r) { return rbase + i * 32 + (r & 3) + 8 * (r >> 2); });
    }
}

// One tile per block (blocks remapped XCD-aware), or (SK) column-grouped
// stream-K: group g runs units [g*U/NG, (g+1)*U/NG) of the m-tile-major
// (m-tile, K-step) sequence, one tile segment after another (sk_combine).
// Separate instantiations (SK): the stream-K loop's live state would otherwise
// raise the register allocation of the one-tile kernels.  PAIR = two blocks per
// CU (256x64 tiles, the stem: 80 KiB each): one block's prologue / epilogue
// overlaps the other's main loop.
// the first-round stagger of X3Args (one wave-uniform wait at block start)
__device__ __forceinline__ void x3_stagger(const X3Args& a) {
    const int b = blockIdx.x;
    if (a.stagger_ticks > 0 && b < a.stagger_blocks && ((b >> 3) & 1)) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)a.stagger_ticks) __builtin_amdgcn_s_sleep(2);
    }
}

template <int BN, bool STEM, bool PAIR, int MFD, bool SK, int P>
__global__ __launch_bounds__(512, PAIR ? 2 : 1) void conv_x3_kernel(X3Args a) {
    __shared__ __attribute__((aligned(1024))) char smem[x3_lds_bytes(BN, PAIR, P) + x3_red_bytes(BN, PAIR)];
    if constexpr (!SK) x3_stagger(a);
    x3_stamp(a, 0);
    const int G = gridDim.x, b = xcd_remap(blockIdx.x, G);
    if constexpr (!SK) {
        conv_x3_tile<BN, STEM, PAIR, MFD, P>(a, smem, b, 0, a.nks, false);
        return;
    }
    // column-grouped stream-K (sk_combine): group g = b / n_tiles, column tile b % n_tiles
    const int NT = a.n_tiles, NG = G / NT, g = b / NT, nt = b - g * NT;
    if (g >= NG) return;                   // grid is NG * n_tiles; never taken
    const long U = a.sk_units, u0 = sk_start(g, U, NG), u1 = sk_start(g + 1, U, NG);
    for (long u = u0; u < u1;) {
        const int mt = (int)(u / a.nks);
        const long t0 = (long)mt * a.nks;
        const int ks = (int)(u - t0), ke = (int)min((long)a.nks, u1 - t0);
        if (u != u0) __syncthreads();      // the previous segment is done with the LDS ring
        conv_x3_tile<BN, STEM, PAIR, MFD, P>(a, smem, mt * NT + nt, ks, ke - ks, ks != 0 || ke != a.nks);
        u = t0 + ke;
    }
}

// One 256x256 tile per block on the A3 body (3-stage A ring, 2-stage B ring);
// with a.main_blocks > 0 the blocks past it run the grid's split-K tail (the
// segments of conv_x3_tail_kernel) in the same launch: they are dispatched as the
// full rounds' tiles finish, without the second launch's gap — and, in training,
// ahead of a side-stream wgrad that would otherwise take the freed CUs first.
template <int P>
__device__ __forceinline__ void conv_x3_a3_grid(const X3Args& a, char* smem) {
    x3_stagger(a);
    x3_stamp(a, 0);
    const int b = blockIdx.x;
    if (a.tail_groups == 0 || b < a.main_blocks) {
        conv_x3_tile<256, false, false, 16, P, true>(
            a, smem, xcd_remap(b, a.tail_groups ? a.main_blocks : gridDim.x), 0, a.nks, false);
        return;
    }
    X3Args t = a;
    const int NT = a.n_tiles, G = a.tail_groups * NT;
    t.mt0 = a.tail_mt0;
    t.sk_units = a.tail_units;
    t.sk_grid = G;
    t.sk_b = xcd_remap(b - a.main_blocks, G);
    const int g = t.sk_b / NT, nt = t.sk_b - g * NT;
    const long U = t.sk_units, u0 = sk_start(g, U, a.tail_groups), u1 = sk_start(g + 1, U, a.tail_groups);
    const int mt = (int)(u0 / a.nks);
    const int ks = (int)(u0 - (long)mt * a.nks), ke = (int)(u1 - (long)mt * a.nks);
    conv_x3_tile<256, false, false, 16, P, true>(t, smem, mt * NT + nt, ks, ke - ks, true);
}

template <int P>
__global__ __launch_bounds__(512, 1) void conv_x3_a3_kernel(X3Args a) {
    __shared__ __attribute__((aligned(1024))) char smem[X3_A3_LDS];
    conv_x3_a3_grid<P>(a, smem);
}

// The A3 body on 192 x 256 tiles (HKP_TILE_192_A3, packed operands): a grid whose
// 256-row tiles leave most CUs idle in a single partial round — the B=8 shard's
// layer3, 150 m-tiles on 256 CUs — runs ceil(M / 192) blocks in the same one
// round, each 3/4 of a tile (200 m-tiles: 0.78 of the CUs instead of 0.59).
// Waves 4 x 2 as in A3 (48 x 128 each, 96 accumulators), the A ring 3 stages of
// 192 lines; BN partials per 96-row half tile (hkp_bn_finalize tile_rows 96).
template <int P>
__global__ __launch_bounds__(512, 1) void conv_x3_a3_192_kernel(X3Args a) {
    __shared__ __attribute__((aligned(1024))) char smem[x3_a3_lds(192)];
    x3_stamp(a, 0);
    conv_x3_tile<256, false, false, 16, P, true, 192>(a, smem, xcd_remap(blockIdx.x, gridDim.x), 0, a.nks, false);
}

// ... on 160 x 256 tiles (HKP_TILE_160_A3): 240 m-tiles for the B=8 shard's layer3,
// 0.94 of the CUs, each 5/8 of a 256-row tile.  Waves 2 x 4 (80 x 64 each, 80
// accumulators); a wave's rows are one 80-row BN partial tile.
template <int P>
__global__ __launch_bounds__(512, 1) void conv_x3_a3_160_kernel(X3Args a) {
    __shared__ __attribute__((aligned(1024))) char smem[x3_a3_lds(160)];
    x3_stamp(a, 0);
    conv_x3_tile<256, false, false, 16, P, true, 160>(a, smem, xcd_remap(blockIdx.x, gridDim.x), 0, a.nks, false);
}

// ... on 160 x 128 tiles (HKP_TILE_160_A3 with Cout % 256 != 0, Cout % 128 == 0): the
// B=8 shard's layer2 (128 channels: 150 256x128 tiles -> 240 160x128); waves 2 x 4
// of 80 x 32, a 2-stage ring of 128 weight rows
template <int P>
__global__ __launch_bounds__(512, 1) void conv_x3_a3_160x128_kernel(X3Args a) {
    __shared__ __attribute__((aligned(1024))) char smem[x3_a3_lds(160, 128)];
    x3_stamp(a, 0);
    conv_x3_tile<128, false, false, 16, P, true, 160>(a, smem, xcd_remap(blockIdx.x, gridDim.x), 0, a.nks, false);
}

// Split-K tail: the m-tiles of the last, partly filled round of a one-tile grid,
// each cut into S equal K segments — one block per segment, a single round —
// summed by the tile's last-arriving segment in segment order (sk_combine; the
// launch is laid out as a column-grouped stream-K grid of NG = tiles x S groups,
// so every group's unit range lies inside one tile).  The stream-K kernel's
// segment loop is what made the 256x256 stream-K body spill; a block here runs
// exactly one segment (a two-segment form that balanced C2 layer4's 176 tail
// tiles over all 256 CUs spilled outside the K loop and measured no faster than
// the plain partial round, whose CUs run at a higher clock).  C2 layer3 on
// 256x256 tiles: 600 tiles = 2 rounds + 88 tiles, which run as 176 half tiles.
template <int BN, int P>
__global__ __launch_bounds__(512, 1) void conv_x3_tail_kernel(X3Args a) {
    __shared__ __attribute__((aligned(1024))) char smem[x3_lds_bytes(BN, false, P) + x3_red_bytes(BN, false)];
    const int G = gridDim.x, b = xcd_remap(blockIdx.x, G);
    const int NT = a.n_tiles, NG = G / NT, g = b / NT, nt = b - g * NT;
    const long U = a.sk_units, u0 = sk_start(g, U, NG), u1 = sk_start(g + 1, U, NG);
    const int mt = (int)(u0 / a.nks);
    const int ks = (int)(u0 - (long)mt * a.nks), ke = (int)(u1 - (long)mt * a.nks);
    conv_x3_tile<BN, false, false, 16, P>(a, smem, mt * NT + nt, ks, ke - ks, true);
}

// ---------------------------------------------------------------------------
// Halo-tile body (conv_x3_halo_kernel<P>) for stride-1 3x3 convs with pad =
// dilation = 1 whose output tiles exactly into 8 x 32 pixel patches (Ho % 8 ==
// 0, Wo % 32 == 0): layer1 of every R-net here (64 channels at 120x160 in
// C2-C4, 240x320 in C5), forward and stride-1 dgrad.  The one-tile kernels
// stage, per K-step, a tap-shifted 256-row A window — every input line is
// fetched from L2 nine times, and at Cin = 64 (2 channel groups x 9 taps) the
// 256x64 tile is bound by that operand stream, not by its MFMAs.  Here a tile is
// an 8 x 32 patch of one image: per channel group its (8+2) x (32+2) = 340
// input lines are staged ONCE by LDS-DMA into a halo image and the nine taps
// read their fragments from it (tile row m = pixel (m/32, m%32) reads halo line
// (m/32 + r) * 34 + m%32 + s for tap (r, s)); only the 64-row weight stage
// streams per K-step (a 3-slot ring).  A tile moves 2 x 42.5 + 18 x 8 = 229 KB
// from L2 instead of 18 x 40 = 720 KB.  Lines past the image are zero lines.
// The 16-B chunk swizzle (halo_swz: line & 6) is keyed on the halo line, so any
// 16 consecutive lines a fragment read touches are conflict-free, as in the ring.
// Two blocks per CU (72 KB each): one block's halo reload / epilogue overlaps the
// other's MFMAs.  256 x 64 tile, 8 waves 4 x 2 (wave tile 64 x 32), 16x16x32
// MFMAs; epilogue = the one-tile kernels' (BN tile partials from the
// accumulators, LDS-staged 16-B row chunks), rows remapped to the patch pixels.
constexpr int HALO_PH = 8, HALO_PW = 32, HALO_LW = HALO_PW + 2, HALO_NL = (HALO_PH + 2) * HALO_LW;   // 340 lines
constexpr int HALO_GA = 6;                                   // halo DMA instructions per wave (48 x 8 lines >= 340)
constexpr int HALO_ABYTES = 8 * HALO_GA * 8 * 128;           // 48 KiB: halo image (+ 44 dummy lines)
constexpr int HALO_NSTB = 3, HALO_BSTAGE = 64 * 128;         // weight ring: 3 x 8 KiB
constexpr int HALO_LDS = HALO_ABYTES + HALO_NSTB * HALO_BSTAGE;

// 16-B chunk swizzle of halo line L: physical chunk = logical ^ (L & 6).  A
// fragment read covers 16 consecutive lines from ANY start (the tap offsets and
// the 34-line patch rows put it anywhere), so the ring bodies' (row >> 1) & 7 —
// conflict-free only from a 4-aligned start — cost ~3 extra LDS cycles per
// ds_read_b128 here (0.30 of the halo kernels' LDS cycles, PMC r04); keyed on
// bits 1-2 of L alone, every ds_read_b128 lane group of a read from any start
// line hits 16 distinct 16-B bank slots (bit 0 of L picks the 128-B half, and the
// group's two q values differ in bit 0 of the chunk).
__device__ __forceinline__ int halo_swz(int L) { return L & 6; }

static bool halo_shape(int stride, int r, int s, int pad, int dil, int ho, int wo, int k) {
    return stride == 1 && r == 3 && s == 3 && pad == 1 && dil == 1 && ho % HALO_PH == 0 && wo % HALO_PW == 0 &&
           k % 64 == 0;
}

// BNIN: the input is the producer's raw output and its BN + ReLU (+ the f16x3
// split, P 3) is applied to each channel group's halo image in LDS after it
// lands (X3Args::in_ss) — the bn_apply pass between the two convs disappears.
// Each lane transforms whole 8-channel pieces: P 3 reads the piece's two fp32
// chunks and writes its hi and lo chunks in place (the four pieces of a line are
// four adjacent lanes of one wave instruction, so every read of the line precedes
// its writes); P 1 rewrites one fp16 chunk.  Out-of-image lines are NaN lines
// (relu(NaN*s + t) = 0).
template <int P, bool BNIN>
__device__ __forceinline__ void x3_halo_bnin(const X3Args& a, char* smem, int g, int tid) {
    constexpr int ROW = 128;
    constexpr int PIECES = P == 1 ? 8 : 4;                       // 8-channel pieces per line
    constexpr int LPI = 512 / PIECES;                            // lines per block-wide pass
    constexpr int NL = 8 * HALO_GA * 8;                          // halo lines incl. the dummies (384)
    const int j = tid % PIECES;
    const int c0 = g * (P == 1 ? 64 : 32) + 8 * j;
    float sa[8], sb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        sa[e] = a.in_ss[c0 + e];
        sb[e] = a.in_ss[a.C + c0 + e];
    }
#pragma unroll
    for (int L0 = 0; L0 < NL; L0 += LPI) {
        const int L = L0 + tid / PIECES;
        const int sw = halo_swz(L);
        char* line = smem + L * ROW;
        if constexpr (P == 1) {
            f16x8* ch = (f16x8*)(line + ((j ^ sw) << 4));
            const f16x8 v = *ch;
            f16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float x = __fadd_rn(__fmul_rn((float)v[e], sa[e]), sb[e]);
                o[e] = (_Float16)(x > 0.f ? x : 0.f);
            }
            *ch = o;
        } else {
            const f32x4 v0 = *(const f32x4*)(line + (((2 * j) ^ sw) << 4));
            const f32x4 v1 = *(const f32x4*)(line + (((2 * j + 1) ^ sw) << 4));
            f16x8 h, l;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float y = e < 4 ? v0[e] : v1[e - 4];
                float x = __fadd_rn(__fmul_rn(y, sa[e]), sb[e]);
                x = x > 0.f ? x : 0.f;
                const _Float16 hv = (_Float16)x;
                h[e] = hv;
                l[e] = (_Float16)(x - (float)hv);
            }
            *(f16x8*)(line + ((j ^ sw) << 4)) = h;
            *(f16x8*)(line + (((4 + j) ^ sw) << 4)) = l;
        }
    }
}

template <int P, bool BNIN>
__device__ __forceinline__ void conv_x3_halo_body(const X3Args& a, char* smem) {
    constexpr int BM = 256, BN = 64, WM = 4, WN = 2, ROW = 128;
    constexpr int UM = BM / (WM * 16), UN = BN / (WN * 16);     // 4 x 2 16x16 sub-tiles per wave
    static_assert(256 * (BN + 4) * 4 <= HALO_LDS && 8 * BN * 4 <= HALO_LDS, "epilogue staging");
    static_assert(!BNIN || P == 3 || P == 1, "fused input BN: f16x3 or plain fp16");

    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mt = tile / a.n_tiles, nt = tile - mt * a.n_tiles;
    const int pwn = a.Wo / HALO_PW, tpi = (a.Ho / HALO_PH) * pwn;
    const int img = mt / tpi, rem = mt - img * tpi;
    const int h0 = (rem / pwn) * HALO_PH, w0 = (rem - (rem / pwn) * pwn) * HALO_PW;
    const int m0 = mt * BM, n0 = nt * BN;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w / WN, wn = w % WN;
    const int cstride = a.cch * 64;                             // halves per pixel
    const int nks = a.nks;                                      // 9 taps x channel groups
    const _Float16* zero = (const _Float16*)(BNIN ? g_x3_nan_line : g_x3_zero_line);

    // ---- halo DMA: instruction i of wave w fills lines 8 (w*GA + i) .. +7 ----
    unsigned h_off[HALO_GA];                                    // element offsets from a.xs (or ~0u: zero line)
#pragma unroll
    for (int i = 0; i < HALO_GA; ++i) {
        const int L = 8 * (w * HALO_GA + i) + lane / 8;
        const int Lc = (lane % 8) ^ halo_swz(L);
        const int hl = L / HALO_LW, wl = L - hl * HALO_LW;
        const int hi = h0 - 1 + hl, wi = w0 - 1 + wl;
        const bool in = L < HALO_NL && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
        h_off[i] = in ? (unsigned)((((long)img * a.H + hi) * a.W + wi) * cstride + Lc * 8) : ~0u;
    }
    auto issue_halo = [&](int g) {
#pragma unroll
        for (int i = 0; i < HALO_GA; ++i)
            glds16(h_off[i] != ~0u ? a.xs + ((unsigned long)h_off[i] + g * 64) : zero,
                   smem + 8 * (w * HALO_GA + i) * ROW);
    };
    // ---- weight stage DMA: one instruction per wave, rows 8w .. 8w+7 ----
    const int brow = 8 * w + lane / 8;
    const int bline = a.RS * a.cch * 64;
    const unsigned b_off = (unsigned)((n0 + brow) * bline + (((lane % 8) ^ ((brow >> 1) & 7)) * 8));
    auto issue_b = [&](int t) {
        const int g = t / 9, u = t - g * 9;
        glds16(a.ws + (b_off + (unsigned)((u * a.cch + g) * 64)),
               smem + HALO_ABYTES + (t % HALO_NSTB) * HALO_BSTAGE + 8 * w * ROW);
    };

    // ---- fragment addressing ----
    const int r16 = lane & 15, q = lane >> 4;
    int lb[UM];                                                 // halo line of tap (0, 0) for sub-tile i
#pragma unroll
    for (int i = 0; i < UM; ++i) {
        const int m = wm * 64 + 16 * i + r16;
        lb[i] = (m >> 5) * HALO_LW + (m & 31);
    }
    const int sw = (r16 >> 1) & 7;                              // B rows: 16-row tiles, as the ring's
    const int fb_h = (wn * 32 + r16) * ROW + ((q ^ sw) << 4), fb_l = (wn * 32 + r16) * ROW + (((4 + q) ^ sw) << 4);

    f32x4 acc[UM][UN];
#pragma unroll
    for (int i = 0; i < UM; ++i)
#pragma unroll
        for (int j = 0; j < UN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto mfma = [](const f16x8& x, const f16x8& y, const f32x4& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(x, y, c, 0, 0, 0);
    };

    // column scale (weight scale x gradient scale), issued before the pipeline
    const float ginv = a.amax ? 1.f / pow2_scale_for(a.amax) : 1.f;
    float scv[UN];
#pragma unroll
    for (int j = 0; j < UN; ++j) scv[j] = (a.wscale ? a.wscale[n0 + wn * 32 + 16 * j + r16] : 1.f) * ginv;

    // prologue: halo of group 0, weight stages 0 and 1
    issue_halo(0);
    issue_b(0);
    if (nks > 1) issue_b(1);
    if (nks > 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if constexpr (BNIN) {
        x3_halo_bnin<P, BNIN>(a, smem, 0, tid);
        lds_sync();
    }
    for (int t = 0; t < nks; ++t) {
        const int g = t / 9, u = t - g * 9;
        const int toff = (u / 3) * HALO_LW + (u - (u / 3) * 3);
        // fragments of step t
        f16x8 ah[UM], al[UM], bh[UN], bl[UN];
#pragma unroll
        for (int i = 0; i < UM; ++i) {
            const int L = lb[i] + toff;
            const int ls = halo_swz(L);
            ah[i] = *(const f16x8*)(smem + L * ROW + ((q ^ ls) << 4));
            al[i] = *(const f16x8*)(smem + L * ROW + (((4 + q) ^ ls) << 4));
        }
        const char* bst = smem + HALO_ABYTES + (t % HALO_NSTB) * HALO_BSTAGE;
#pragma unroll
        for (int j = 0; j < UN; ++j) {
            bh[j] = *(const f16x8*)(bst + j * 16 * ROW + fb_h);
            bl[j] = *(const f16x8*)(bst + j * 16 * ROW + fb_l);
        }
        // weight stage t+2 goes into the slot step t-1 read (every wave is past
        // this step's barrier, so done reading it)
        if (t + 2 < nks) issue_b(t + 2);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < UM; ++i)
#pragma unroll
            for (int j = 0; j < UN; ++j) x3_products<P>(acc[i][j], ah[i], al[i], bh[j], bl[j], mfma);
        if (t + 1 >= nks) break;
        if (u == 8) {
            // the group's last tap: every wave done with the halo, then the next
            // group's halo (the youngest DMA: wait for everything)
            lds_barrier();
            issue_halo(g + 1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if constexpr (BNIN) {
                lds_barrier();                                   // the whole halo landed
                x3_halo_bnin<P, BNIN>(a, smem, g + 1, tid);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
        } else if (t + 2 < nks) {
            asm volatile("s_waitcnt vmcnt(1)" ::: "memory");     // stage t+1 landed, t+2 in flight
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        lds_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---- epilogue: BN tile partials (rows all valid: exact patch tiling), then
    // the scaled tile staged through the drained LDS and written as 16-B row
    // chunks; tile row m -> pixel (img, h0 + m/32, w0 + m%32) ----
    const int rbase = m0 + wm * UM * 16 + 4 * q;
    lds_sync();                                                  // every wave done with the halo / ring
    if (a.part) {
        x3_bn_partials_w<BN, UM, UN, 16, 16>(
            a, (float*)smem, m0, n0, wm, wn, lane, [&](int i, int j) { return acc[i][j]; },
            [&](int i, int r) { return rbase + i * 16 + r; }, [&](int j) { return scv[j]; }, (float*)smem);
        lds_sync();
    }
    auto out_pix = [&](int row) { return ((long)img * a.Ho + h0 + (row >> 5)) * a.Wo + w0 + (row & 31); };
    if constexpr (P == 1) {
        constexpr int PITCH = BN + 8, CH = BN / 8;
        _Float16* st = (_Float16*)smem;
#pragma unroll
        for (int i = 0; i < UM; ++i)
#pragma unroll
            for (int j = 0; j < UN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    st[(wm * UM * 16 + i * 16 + 4 * q + r) * PITCH + wn * 32 + j * 16 + r16] =
                        (_Float16)(acc[i][j][r] * scv[j]);
        lds_sync();
#pragma unroll 4
        for (int e = tid; e < BM * CH; e += 512) {
            const int row = e / CH, cc = e - row * CH;
            x3_st16((uint4*)(a.y16 + out_pix(row) * a.K + n0 + cc * 8), *(const uint4*)(smem + (row * PITCH + cc * 8) * 2), a.st_kind, 1);
        }
    } else {
        constexpr int PITCH = BN + 4, C4 = BN / 4;
        float* st = (float*)smem;
#pragma unroll
        for (int i = 0; i < UM; ++i)
#pragma unroll
            for (int j = 0; j < UN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    st[(wm * UM * 16 + i * 16 + 4 * q + r) * PITCH + wn * 32 + j * 16 + r16] = acc[i][j][r] * scv[j];
        lds_sync();
#pragma unroll 4
        for (int e = tid; e < BM * C4; e += 512) {
            const int row = e / C4, c4 = e - row * C4;
            const long off = out_pix(row) * a.K + n0 + c4 * 4;
            f32x4 v = *(const f32x4*)(st + row * PITCH + c4 * 4);
            if (a.add) {
                const f32x4 ad = *(const f32x4*)(a.add + off);
#pragma unroll
                for (int k = 0; k < 4; ++k) v[k] = v[k] + ad[k];
            }
            *(f32x4*)(a.y + off) = v;
        }
    }
}

template <int P>
__global__ __launch_bounds__(512, 2) void conv_x3_halo_kernel(X3Args a) {
    __shared__ __attribute__((aligned(1024))) char smem[HALO_LDS];
    conv_x3_halo_body<P, false>(a, smem);
}

// the same with the input's BN + ReLU applied to each halo image (X3Args::in_ss)
template <int P>
__global__ __launch_bounds__(512, 2) void conv_x3_halo_bnin_kernel(X3Args a) {
    __shared__ __attribute__((aligned(1024))) char smem[HALO_LDS];
    conv_x3_halo_body<P, true>(a, smem);
}

// ---------------------------------------------------------------------------
// Stem patch body (conv_x3_stem_patch_kernel): the 7x7/s2 stem on the padded
// NHWC4 hi | lo image planes of hkp_stem_pack_x3, a tile = an 8 x 32 patch of
// output pixels.  The one-tile stem (conv_x3_kernel<64, STEM, PAIR>) stages per
// filter row a 256-line im2col window — pixels 2wo .. 2wo+7 of one padded row for
// every output pixel, each input pixel fetched ~4x per row and 7 rows deep: 224 KB
// of L2 -> LDS traffic per tile, the stem's bound (C2 288 us for 629 MB of output).
// Here the patch's (2*8+5) x (2*32+6) = 21 x 70 padded pixels of both planes
// (23 KB) and all 7 filter rows of the 64 weight rows (56 KB) are staged ONCE by
// LDS-DMA and the 7 K-steps read their fragments from them with no barrier between:
// output pixel (i, j), filter row r, chunk q (taps 2q, 2q+1 x 4 channels) is the
// 16 B at patch row 2i + r, pixel 2j + 2q — 16 consecutive pixels of a fragment
// read 256 contiguous bytes (every bank once).  B lines keep the ring bodies'
// (row >> 1) & 7 chunk swizzle.  256 x 64 tile, 8 waves 4 x 2 (wave tile 64 x 32),
// 16x16x32 MFMAs, 80 KiB: two blocks per CU, one's epilogue beside the other's
// MFMAs; epilogue = the halo body's (BN tile partials, LDS-staged fp32 row chunks).
constexpr int STEM_PH = 8, STEM_PW = 32, STEM_PR = 2 * STEM_PH + 5, STEM_PC = 2 * STEM_PW + 6;   // 21 x 70 pixels
constexpr int STEM_PLANE = STEM_PR * STEM_PC * 8;                // bytes per plane (4 ch fp16 per pixel)
constexpr int STEM_BBYTES = 7 * 64 * 128;                        // 7 filter rows x 64 weight lines
constexpr int STEM_PCH = 2 * STEM_PLANE / 16;                    // patch 16-B chunks (1470)
constexpr int STEM_PGA = (STEM_PCH + 511) / 512;                 // patch DMA instructions per wave (3)
constexpr int STEM_LDS = STEM_BBYTES + 8 * STEM_PGA * 1024;      // B, then the patch (+ dummy chunks): 80 KiB

HKP_AB_KNOB(int, g_stem_pair, 0);                               // hkp_debug_stem_pair
static bool stem_patch_shape(int ho, int wo, int k) {
    return !g_stem_pair && ho % STEM_PH == 0 && wo % STEM_PW == 0 && k % 64 == 0;
}

// SRC: 0 the padded hi | lo planes of hkp_stem_pack_x3 (DMA), 1 the fp32 NCHW image,
// 2 the uint8 NHWC (BGR) batch — for 1 / 2 the patch is built in LDS from the image
// itself (hkp_stem_pack_x3's arithmetic: x = u8 / 255 for uint8, hi = f16(x),
// lo = f16(x - hi), zeros outside the image and in channels C..3), so the planes
// are never written (a.H / a.W / a.C: the image's height, width, channels)
template <int SRC>
__global__ __launch_bounds__(512, 2) void conv_x3_stem_patch_kernel(X3Args a) {
    __shared__ __attribute__((aligned(1024))) char smem[STEM_LDS];
    constexpr int BM = 256, BN = 64, WM = 4, WN = 2, ROW = 128;
    constexpr int UM = BM / (WM * 16), UN = BN / (WN * 16);     // 4 x 2 16x16 sub-tiles per wave
    static_assert(256 * (BN + 4) * 4 <= STEM_LDS && STEM_PGA * 512 >= STEM_PCH, "stem patch LDS");
    x3_stamp(a, 0);
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mt = tile / a.n_tiles, nt = tile - mt * a.n_tiles;
    const int pwn = a.Wo / STEM_PW, tpi = (a.Ho / STEM_PH) * pwn;
    const int img = mt / tpi, rem = mt - img * tpi;
    const int h0 = (rem / pwn) * STEM_PH, w0 = (rem - (rem / pwn) * pwn) * STEM_PW;
    const int m0 = mt * BM, n0 = nt * BN;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w / WN, wn = w % WN;

    // ---- staging: the weight lines (7 instructions per wave: LDS row R = r*64 + n
    // holds logical chunk p ^ ((n >> 1) & 7) at physical chunk p), then the patch
    // (chunk c: plane c / (PLANE/16), patch row, 16-B column — 35 per row, the 70
    // padded pixels of a patch row are contiguous in the plane) ----
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        const int R = 8 * (w * 7 + i) + lane / 8;
        const int r = R >> 6, n = R & 63;
        const int Lc = (lane % 8) ^ ((n >> 1) & 7);
        glds16(a.ws + ((long)(n0 + n) * 7 + r) * 64 + Lc * 8, smem + 8 * (w * 7 + i) * ROW);
    }
    if constexpr (SRC == 0) {
        const _Float16* zero = (const _Float16*)g_x3_zero_line;
        const long prow0 = ((long)img * a.H + 2 * h0) * a.W + 2 * w0;   // padded pixel of patch (0, 0)
#pragma unroll
        for (int i = 0; i < STEM_PGA; ++i) {
            const int c = 512 * i + 64 * w + lane;               // instruction i of wave w: chunks 512 i + 64 w + lane
            const int pl = c >= STEM_PLANE / 16 ? 1 : 0, cc = c - pl * (STEM_PLANE / 16);
            const int pr = cc / (STEM_PC / 2), pc = cc - pr * (STEM_PC / 2);
            const _Float16* src = c < STEM_PCH ? a.xs + pl * a.plane + (prow0 + (long)pr * a.W) * 4 + pc * 8 : zero;
            glds16(src, smem + STEM_BBYTES + (512 * i + 64 * w) * 16);
        }
    } else {
        // padded pixel (pr, pc) of the patch = image pixel (2 h0 + pr - 3, 2 w0 + pc - 3);
        // every load of the thread's pixels issued before the first conversion
        constexpr int NPX = STEM_PR * STEM_PC, IT = (NPX + 511) / 512;
        f32x4 v[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int px = tid + 512 * it;
            const int pr = px / STEM_PC, pc = px - pr * STEM_PC;
            const int h = 2 * h0 + pr - 3, wi = 2 * w0 + pc - 3;
            const bool in = px < NPX && (unsigned)h < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
            v[it] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (in && c < a.C) {
                    if constexpr (SRC == 2)
                        v[it][c] = __fdiv_rn((float)((const uint8_t*)a.xs)[(((long)img * a.H + h) * a.W + wi) * a.C + c], 255.f);
                    else
                        v[it][c] = ((const float*)a.xs)[(((long)img * a.C + c) * a.H + h) * a.W + wi];
                }
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int px = tid + 512 * it;
            if (px >= NPX) break;
            h16x4 hv, lv;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const _Float16 hh = (_Float16)v[it][c];
                hv[c] = hh;
                lv[c] = (_Float16)(v[it][c] - (float)hh);
            }
            *(h16x4*)(smem + STEM_BBYTES + px * 8) = hv;
            *(h16x4*)(smem + STEM_BBYTES + STEM_PLANE + px * 8) = lv;
        }
    }

    // ---- fragment addressing ----
    const int r16 = lane & 15, q = lane >> 4;
    int aoff[UM];                                               // patch byte offset of sub-tile i's pixel, filter row 0, chunk q
#pragma unroll
    for (int i = 0; i < UM; ++i) {
        const int m = wm * 64 + 16 * i + r16;
        aoff[i] = STEM_BBYTES + ((2 * (m >> 5)) * STEM_PC + 2 * (m & 31) + 2 * q) * 8;
    }
    const int sw = (r16 >> 1) & 7;
    const int fb_h = (wn * 32 + r16) * ROW + ((q ^ sw) << 4), fb_l = (wn * 32 + r16) * ROW + (((4 + q) ^ sw) << 4);

    f32x4 acc[UM][UN];
#pragma unroll
    for (int i = 0; i < UM; ++i)
#pragma unroll
        for (int j = 0; j < UN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto mfma = [](const f16x8& x, const f16x8& y, const f32x4& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(x, y, c, 0, 0, 0);
    };
    float scv[UN];
#pragma unroll
    for (int j = 0; j < UN; ++j) scv[j] = a.wscale ? a.wscale[n0 + wn * 32 + 16 * j + r16] : 1.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    x3_stamp(a, 1);
    // 7 K-steps (filter rows) from the resident patch and weights: no barriers
    f16x8 ah[UM], al[UM], bh[UN], bl[UN];
    auto read_frags = [&](int r) {
#pragma unroll
        for (int i = 0; i < UM; ++i) {
            ah[i] = *(const f16x8*)(smem + aoff[i] + r * STEM_PC * 8);
            al[i] = *(const f16x8*)(smem + aoff[i] + r * STEM_PC * 8 + STEM_PLANE);
        }
#pragma unroll
        for (int j = 0; j < UN; ++j) {
            bh[j] = *(const f16x8*)(smem + r * 64 * ROW + j * 16 * ROW + fb_h);
            bl[j] = *(const f16x8*)(smem + r * 64 * ROW + j * 16 * ROW + fb_l);
        }
    };
#pragma unroll
    for (int r = 0; r < 7; ++r) {
        read_frags(r);
#pragma unroll
        for (int i = 0; i < UM; ++i)
#pragma unroll
            for (int j = 0; j < UN; ++j) x3_products<3>(acc[i][j], ah[i], al[i], bh[j], bl[j], mfma);
    }
    x3_stamp(a, 2);

    // ---- epilogue: BN tile partials (rows all valid: exact patch tiling), the
    // scaled tile staged through the LDS and written as 16-B row chunks; tile row
    // m -> output pixel (img, h0 + m/32, w0 + m%32) ----
    const int rbase = m0 + wm * UM * 16 + 4 * q;
    lds_sync();                                                  // every wave done with the patch and weights
    if (a.part) {
        x3_bn_partials_w<BN, UM, UN, 16, 16>(
            a, (float*)smem, m0, n0, wm, wn, lane, [&](int i, int j) { return acc[i][j]; },
            [&](int i, int r) { return rbase + i * 16 + r; }, [&](int j) { return scv[j]; }, (float*)smem);
        lds_sync();
    }
    x3_stamp(a, 3);
    constexpr int PITCH = BN + 4, C4 = BN / 4;
    float* st = (float*)smem;
#pragma unroll
    for (int i = 0; i < UM; ++i)
#pragma unroll
        for (int j = 0; j < UN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                st[(wm * UM * 16 + i * 16 + 4 * q + r) * PITCH + wn * 32 + j * 16 + r16] = acc[i][j][r] * scv[j];
    lds_sync();
    x3_stamp(a, 4);
#pragma unroll 4
    for (int e = tid; e < BM * C4; e += 512) {
        const int row = e / C4, c4 = e - row * C4;
        const long off = (((long)img * a.Ho + h0 + (row >> 5)) * a.Wo + w0 + (row & 31)) * a.K + n0 + c4 * 4;
        x3_st16((f32x4*)(a.y + off), *(const f32x4*)(st + row * PITCH + c4 * 4), a.st_kind, 2);
    }
    x3_stamp(a, 5);
}


// ---------------------------------------------------------------------------
// DUO body (conv_x3_duo_kernel<1>): plain-fp16 (P 1, config C4) convs on 256 x 128
// tiles run by TWO 4-wave blocks per CU.  The one-tile 256x256 bodies hold a
// whole CU, so each tile's pipeline fill, BN partials, fp16 staging and stores
// run with the CU's matrix pipes idle — on C4's short-K 1x1 GEMMs (8-16 K-steps
// per tile) about half of a tile's time (DESIGN "C4's 1x1 GEMMs").  Here two
// independent blocks share the CU: one block's fill and epilogue run beside the
// other's K loop, and their vmcnt / barriers are separate (a persistent body's
// epilogue stores, by contrast, shared vmcnt with its next tile's DMA).
// Per block: 4 waves as 2 x 2, wave tile 128 x 64 (8 x 4 16x16x32 MFMA tiles,
// 128 accumulator registers); a 3-stage LDS ring of HALF lines — a stage holds
// 32 channels (64 B) of every A row (256) and B row (128): 24 KiB — so three
// stages (72 KiB, which also holds the fp16 epilogue tile) fit twice per CU.
// K order: channel group (64 channels), tap, half; a half-line is one k32 step,
// one MFMA per (16-row, 16-column) pair.  64-B rows: lane l of a DMA piece writes
// row l/4, 16-B chunk l%4; the chunk swizzle (4 - (row >> 2)) & 3 makes every
// ds_read_b128 lane group of the fragment reads (rows r16 = lane & 15, chunk
// lane >> 4) hit 16 distinct 16-B bank groups.  Epilogue: BN partials per
// 128-row half straight from one wave's accumulators (a wave holds a whole
// half: no LDS merge), then the fp16 tile staged in the drained ring and written
// as 16-B row chunks, optionally through the fused BN + residual + ReLU
// (hkp_conv2d_fwd_f16_bn) — the 256x256 body's arithmetic, element for element.
constexpr int DUO_BM = 256, DUO_BN = 128, DUO_ROW = 64, DUO_NST = 3;
// first-round arrivals per CU (key: XCC id x the HW_ID's SE / SH / CU bits): the
// second block to arrive on a CU starts late, so the two blocks sharing it run
// half a block apart (see conv_x3_duo_kernel); parity of a running count, never reset
__device__ unsigned g_duo_cu_cnt[8 * 128];
constexpr int DUO_STAGE = (DUO_BM + DUO_BN) * DUO_ROW;                 // 24 KiB
constexpr int DUO_LDS = DUO_NST * DUO_STAGE;                           // 72 KiB: two blocks per CU
static_assert(DUO_BM * (DUO_BN + 8) * 2 + 4 * DUO_BN * 4 <= DUO_LDS, "DUO epilogue staging");

__device__ __forceinline__ int duo_swz(int row) { return (4 - ((row >> 2) & 3)) & 3; }

// BN partials (sum, M2 about the half's mean) of one wave's 128-row half of the
// tile: each lane reduces its 32 rows of a column, then lanes l, l^16, l^32, l^48
// (the column's four row groups) merge by Chan's formula — equal counts, so the
// factors are constants and the result is symmetric in each pair (all four lanes
// hold the same bits).  Rows past M (the last tile) take the counted form.
template <int UM, int UN>
__device__ __forceinline__ void duo_bn_partials(const X3Args& a, const f32x4 (&acc)[UM][UN], const float (&sc)[UN],
                                                int m0h, int ncol0, int lane) {
    const int q = lane >> 4, r16 = lane & 15;
    const long tile128 = (long)(m0h >> 7);
    if (m0h + 128 <= a.M) {                                  // block-uniform
#pragma unroll
        for (int j = 0; j < UN; ++j) {
            f32x4 s4 = acc[0][j];
#pragma unroll
            for (int i = 1; i < UM; ++i) s4 += acc[i][j];
            float s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
            constexpr float inv = 1.f / (UM * 4);
            const f32x4 mu = {s * inv, s * inv, s * inv, s * inv};
            f32x4 q4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < UM; ++i) {
                const f32x4 d = acc[i][j] - mu;
                q4 += d * d;
            }
            float m2 = (q4[0] + q4[1]) + (q4[2] + q4[3]);
            x3_chan_merge(s, m2, __shfl_xor(s, 16), __shfl_xor(m2, 16), 1.f / (UM * 4), UM * 2.f);
            x3_chan_merge(s, m2, __shfl_xor(s, 32), __shfl_xor(m2, 32), 1.f / (UM * 8), UM * 4.f);
            if (q == 0) {
                const int c = ncol0 + 16 * j + r16;
                a.part[(tile128 * a.K + c) * 2 + 0] = s * sc[j];
                a.part[(tile128 * a.K + c) * 2 + 1] = m2 * (sc[j] * sc[j]);
            }
        }
        return;
    }
    if (m0h >= a.M) return;
    float ln = 0.f;
#pragma unroll
    for (int i = 0; i < UM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) ln += (m0h + 16 * i + 4 * q + r < a.M) ? 1.f : 0.f;
    const float linv = ln > 0.f ? 1.f / ln : 0.f;
#pragma unroll
    for (int j = 0; j < UN; ++j) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < UM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) s += (m0h + 16 * i + 4 * q + r < a.M) ? acc[i][j][r] : 0.f;
        const float mu = s * linv;
        float m2 = 0.f;
#pragma unroll
        for (int i = 0; i < UM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float d = acc[i][j][r] - mu;
                m2 += (m0h + 16 * i + 4 * q + r < a.M) ? d * d : 0.f;
            }
        float n = ln;
        for (int o = 16; o < 64; o <<= 1) {
            const float nb = __shfl_xor(n, o), sb = __shfl_xor(s, o), qb = __shfl_xor(m2, o);
            const float nt = n + nb;
            const float f = nt > 0.f ? n * nb / nt : 0.f;
            const float ia = n > 0.f ? 1.f / n : 0.f, ib = nb > 0.f ? 1.f / nb : 0.f;
            const float d = sb * ib - s * ia;
            s = s + sb;
            m2 = (m2 + qb) + d * d * f;
            n = nt;
        }
        if (q == 0) {
            const int c = ncol0 + 16 * j + r16;
            a.part[(tile128 * a.K + c) * 2 + 0] = s * sc[j];
            a.part[(tile128 * a.K + c) * 2 + 1] = m2 * (sc[j] * sc[j]);
        }
    }
}

template <int P>
__global__ __launch_bounds__(256, 2) void conv_x3_duo_kernel(X3Args a) {
    static_assert(P == 1, "DUO: the plain-fp16 operand layout");
    __shared__ __attribute__((aligned(1024))) char smem[DUO_LDS];
    constexpr int BM = DUO_BM, BN = DUO_BN, ROW = DUO_ROW, NST = DUO_NST, STAGE = DUO_STAGE;
    constexpr int UM = 8, UN = 4;                    // 16x16 tiles per wave (wave tile 128 x 64)
    constexpr int GA = 4, GB = 2, GL = GA + GB;      // DMA pieces (16 rows each) per wave per stage

    x3_stamp(a, 0);
    x3_stamp_where(a);
    // Co-resident blocks of a one-round-per-tile grid start together and, doing the
    // same work, stay in phase: both fill, both run the K loop, both run the
    // epilogue — nothing overlaps.  In the first round the second block to arrive
    // on each CU waits about half a block's lifetime (X3Args::stagger_ticks), so
    // from then on one block's fill and epilogue run beside the other's K loop.
    if (a.stagger_ticks > 0 && blockIdx.x < (unsigned)a.stagger_blocks) {
        __shared__ int late;
        if (threadIdx.x == 0) {
            const unsigned hw = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
            const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
            const unsigned key = (xcc & 7) * 128 + ((hw >> 8) & 127);
            late = (int)(atomicAdd(&g_duo_cu_cnt[key], 1u) & 1u);
        }
        __syncthreads();
        if (late) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)a.stagger_ticks) __builtin_amdgcn_s_sleep(8);
        }
    }
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mt = tile / a.n_tiles, nt = tile - mt * a.n_tiles;
    const int m0 = mt * BM, n0 = nt * BN;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w >> 1, wn = w & 1;
    const int nst = 2 * a.nks;                       // half-line stages

    // ---- DMA sources (the one-tile bodies' bookkeeping, 64-B rows) ----
    const int cstride = a.cch * 64;                  // halves per pixel
    const long xbias = (long)a.pad * (a.W + 1) * cstride;
    const _Float16* xbase = a.xs - xbias;
    const _Float16* zero = (const _Float16*)g_x3_zero_line;
    int a_org[GA];
    unsigned a_off[GA];
#pragma unroll
    for (int i = 0; i < GA; ++i) {
        const int row = 64 * w + 16 * i + (lane >> 2);
        const int Lc = (lane & 3) ^ duo_swz(row);
#ifdef HKP_AB_KNOBS
        const int m = a.a_wrap ? (m0 + row) % a.a_wrap : m0 + row;
#else
        const int m = m0 + row;
#endif
        int hb = -16384, wb = -16384;
        long off = 0;
        if (m < a.M) {
            const int hw = a.Ho * a.Wo;
            const int n = m / hw, rem = m - n * hw;
            const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
            hb = ho * a.stride - a.pad;
            wb = wo * a.stride - a.pad;
            off = (((long)n * a.H + hb) * a.W + wb) * cstride + Lc * 8;
        }
        a_org[i] = (int)(((unsigned)hb << 16) | ((unsigned)wb & 0xFFFFu));
        a_off[i] = (unsigned)(off + xbias);
    }
    const int bline = a.RS * a.cch * 64;             // halves per weight row
    int b_off[GB];
#pragma unroll
    for (int j = 0; j < GB; ++j) {
        const int row = 32 * w + 16 * j + (lane >> 2);
        b_off[j] = (n0 + row) * bline + ((lane & 3) ^ duo_swz(row)) * 8;
    }
    // staging position of the next stage to issue: (channel group, tap, half)
    int q_buf = 0, q_cc = 0, q_tap = 0, q_rr = 0, q_ss = 0, q_half = 0;
    auto issue = [&]() {
        char* st = smem + q_buf * STAGE;
        const int dh = q_rr * a.dil, dw = q_ss * a.dil;
        const long toff = ((long)dh * a.W + dw) * cstride + q_cc * 64 + q_half * 32;
#pragma unroll
        for (int i = 0; i < GA; ++i) {
            const int hb = a_org[i] >> 16, wb = (int)(short)(a_org[i] & 0xFFFF);
            const bool in = (unsigned)(hb + dh) < (unsigned)a.H && (unsigned)(wb + dw) < (unsigned)a.W;
            glds16(in ? xbase + ((unsigned long)a_off[i] + toff) : zero, st + (64 * w + 16 * i) * ROW);
        }
        const int boff = (q_tap * a.cch + q_cc) * 64 + q_half * 32;
#pragma unroll
        for (int j = 0; j < GB; ++j) glds16(a.ws + (unsigned)(b_off[j] + boff), st + (BM + 32 * w + 16 * j) * ROW);
        q_buf = q_buf == NST - 1 ? 0 : q_buf + 1;
        if (++q_half == 2) {
            q_half = 0;
            if (++q_ss == a.S) {
                q_ss = 0;
                ++q_rr;
            }
            if (++q_tap == a.RS) {
                q_tap = 0;
                q_rr = 0;
                ++q_cc;
            }
        }
    };

    // ---- fragments: lane reads row r16 of a 16-row tile, logical chunk q ----
    const int r16 = lane & 15, q = lane >> 4;
    const int fo = r16 * ROW + ((q ^ duo_swz(r16)) << 4);
    const int a_base = (wm * 128) * ROW + fo, b_base = (BM + wn * 64) * ROW + fo;
    f32x4 acc[UM][UN];
#pragma unroll
    for (int i = 0; i < UM; ++i)
#pragma unroll
        for (int j = 0; j < UN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    f16x8 fa[UM], fb[UN];
    auto read_a = [&](const char* st) {
#pragma unroll
        for (int i = 0; i < UM; ++i) fa[i] = *(const f16x8*)(st + a_base + i * 16 * ROW);
    };
    auto read_b = [&](int j, const char* st) { fb[j] = *(const f16x8*)(st + b_base + j * 16 * ROW); };
    auto mma_col = [&](int j) {
#pragma unroll
        for (int i = 0; i < UM; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    };

    // column scales (weight scale), issued before the fill
    float sc[UN];
#pragma unroll
    for (int j = 0; j < UN; ++j) sc[j] = a.wscale ? a.wscale[n0 + wn * 64 + 16 * j + r16] : 1.f;

    // ---- pipeline (the 3-stage ring schedule of conv_x3_mf16_body): per stage t —
    // wait own DMA of t+1 (t+2 stays in flight), barrier, DMA of t+3 into t's
    // buffer (its fragments were read during step t-1) spread over the columns,
    // per column j [MFMAs of t with B_j] [read B_j of t+1], then A of t+1 ----
    for (int s = 0; s < NST; ++s)
        if (s < nst) issue();
    {
        const int after = min(nst, NST) - 1;
        if (after >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GL) : "memory");
        else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();
    x3_stamp(a, 1);
    read_a(smem);
#pragma unroll
    for (int j = 0; j < UN; ++j) read_b(j, smem);
    int cur = 0;
    auto kstep = [&](const int t, const bool dma) {
        if (t + 2 < nst) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(GL) : "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        lds_barrier();
        cur = cur == NST - 1 ? 0 : cur + 1;
        const char* st = smem + cur * STAGE;
        if (dma) issue();
#pragma unroll
        for (int j = 0; j < UN; ++j) {
            mma_col(j);
            read_b(j, st);
        }
        read_a(st);
#pragma unroll
        for (int j = 0; j < UN; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, UM, 0);     // column j's MFMAs
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);      // refill B_j
            if (dma && j * ((GL + UN - 1) / UN) < GL)
                __builtin_amdgcn_sched_group_barrier(0x020, (GL + UN - 1) / UN, 0);   // DMA pieces
        }
        __builtin_amdgcn_sched_group_barrier(0x100, UM, 0);         // next A frags
        __builtin_amdgcn_sched_barrier(0);
    };
    int t = 0;
    for (; t + 3 < nst; ++t) kstep(t, true);
    for (; t + 1 < nst; ++t) kstep(t, false);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int j = 0; j < UN; ++j) mma_col(j);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA in flight into the ring past here
    x3_stamp(a, 2);

    // ---- epilogue: BN partials of this wave's 128-row half, then the fp16 tile ----
    if (a.part) duo_bn_partials<UM, UN>(a, acc, sc, m0 + 128 * wm, n0 + wn * 64, lane);
    x3_stamp(a, 3);
    constexpr int PITCH = BN + 8, CH = BN / 8, SS_OFF = BM * PITCH * 2;
    constexpr int NT = 256, NPT = BM * CH / NT;              // 16-B chunks per thread
    static_assert(NT % CH == 0, "a thread keeps its 8 channels");
    const int cc = tid % CH;
    // fused BN epilogue: per-column parameters and the residual chunks in flight
    // before the tile is staged (their latency hides behind it)
    float ep0 = 0.f, ep1 = 0.f;
    f16x8 res[NPT];
    if (a.ep_ss) {
        const int h = tid / BN, c = tid - h * BN;                // tid < 2 * BN: all 256 threads
        ep0 = a.ep_ss[h * a.K + n0 + c];
        ep1 = a.ep_rss ? a.ep_rss[h * a.K + n0 + c] : 0.f;
#pragma unroll
        for (int u = 0; u < NPT; ++u) {
            const int row = (tid + NT * u) / CH, m = m0 + row;
            res[u] = f16x8{};
            if (a.ep_res && m < a.M)
                res[u] = __builtin_nontemporal_load((const f16x8*)(a.ep_res + (long)m * a.K + n0 + cc * 8));
        }
    }
    lds_sync();                                              // every wave done reading the ring
    _Float16* tl = (_Float16*)smem;
#pragma unroll
    for (int i = 0; i < UM; ++i)
#pragma unroll
        for (int j = 0; j < UN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                tl[(wm * 128 + i * 16 + 4 * q + r) * PITCH + wn * 64 + j * 16 + r16] = (_Float16)(acc[i][j][r] * sc[j]);
    float* ssl = (float*)(smem + SS_OFF);                    // [4][BN]: scale, shift, residual scale, shift
    if (a.ep_ss) {
        ssl[tid] = ep0;
        ssl[2 * BN + tid] = ep1;
    }
    lds_sync();
    x3_stamp(a, 4);
    if (!a.ep_ss) {
#pragma unroll 4
        for (int u = 0; u < NPT; ++u) {
            const int row = (tid + NT * u) / CH, m = m0 + row;
            if (m < a.M)
                x3_st16((uint4*)(a.y16 + (long)m * a.K + n0 + cc * 8), *(const uint4*)(smem + (row * PITCH + cc * 8) * 2), a.st_kind, 1);
        }
        x3_stamp(a, 5);
        return;
    }
    float sa[8], sb[8], ra[8], rb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        sa[e] = ssl[cc * 8 + e];
        sb[e] = ssl[BN + cc * 8 + e];
        ra[e] = ssl[2 * BN + cc * 8 + e];
        rb[e] = ssl[3 * BN + cc * 8 + e];
    }
    const bool hres = a.ep_res != nullptr, rsc = a.ep_rss != nullptr, relu = a.ep_relu != 0;
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
        const int row = (tid + NT * u) / CH, m = m0 + row;
        if (m >= a.M) continue;
        const f16x8 v = *(const f16x8*)(smem + (row * PITCH + cc * 8) * 2);
        const f16x8 rv = res[u];
        f16x8 h;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float o = __fadd_rn(__fmul_rn((float)v[k], sa[k]), sb[k]);
            if (hres) o = rsc ? __fadd_rn(o, __fadd_rn(__fmul_rn((float)rv[k], ra[k]), rb[k])) : __fadd_rn(o, (float)rv[k]);
            if (relu) o = o > 0.f ? o : 0.f;
            h[k] = (_Float16)o;
        }
        x3_st16((f16x8*)(a.y16 + (long)m * a.K + n0 + cc * 8), h, a.st_kind, 2);
    }
    x3_stamp(a, 5);
}

// ---------------------------------------------------------------------------
// operand packing

__device__ __forceinline__ void split_store(float v, _Float16* hi_p) {   // hi at p, lo at p + 32
    const _Float16 h = (_Float16)v;
    hi_p[0] = h;
    hi_p[32] = (_Float16)(v - (float)h);
}

// block max |x| over a row of n elements addressed by idx(i); result broadcast
template <typename F>
__device__ __forceinline__ float block_absmax(int n, F&& val) {
    __shared__ float red[8];
    float m = 0.f;
    for (int i = threadIdx.x; i < n; i += blockDim.x) m = fmaxf(m, fabsf(val(i)));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    float r = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r = fmaxf(r, red[i]);
    __syncthreads();
    return r;
}

// w[k][tap][c] fp32 (KRSC) * 2^e_k → ws[k][tap][c/32][hi32|lo32]; one block per k.
// Element e → 2e - (c&31) (lo 32 halves later); wscale[k] = 2^-e_k.
__global__ __launch_bounds__(256) void weight_pack_x3_kernel(int rsc, const float* __restrict__ w,
                                                            _Float16* __restrict__ ws, float* __restrict__ wscale) {
    const int k = blockIdx.x;
    const float* row = w + (long)k * rsc;
    const float sc = pow2_scale_of(block_absmax(rsc, [&](int i) { return row[i]; }));
    for (int i = threadIdx.x; i < rsc; i += blockDim.x) {
        const long e = (long)k * rsc + i;
        split_store(row[i] * sc, ws + 2 * e - (e & 31));
    }
    if (threadIdx.x == 0) wscale[k] = 1.f / sc;
}

// w[k][tap][c] fp32 (KRSC) * 2^e_k → fp16 KRSC (the plain-fp16 conv's operand:
// 64-channel 128-B lines); one block per k, wscale[k] = 2^-e_k
__global__ __launch_bounds__(256) void weight_pack_f16_kernel(int rsc, const float* __restrict__ w,
                                                             _Float16* __restrict__ out, float* __restrict__ wscale) {
    const int k = blockIdx.x;
    const float* row = w + (long)k * rsc;
    const float sc = pow2_scale_of(block_absmax(rsc, [&](int i) { return row[i]; }));
    for (int i = threadIdx.x; i < rsc; i += blockDim.x) out[(long)k * rsc + i] = (_Float16)(row[i] * sc);
    if (threadIdx.x == 0) wscale[k] = 1.f / sc;
}

// flipped dgrad weight, packed: row c (forward input channel) holds element
// (r', s', k) = w[k][R-1-r'][S-1-s'][c] * 2^e_c; one block per c
__global__ __launch_bounds__(256) void weight_flip_pack_x3_kernel(int K, int R, int S, int C,
                                                                 const float* __restrict__ w,
                                                                 _Float16* __restrict__ out,
                                                                 float* __restrict__ wscale) {
    const int c = blockIdx.x;
    const int n = R * S * K;
    auto val = [&](int i) {
        const int k = i % K, t = i / K, sp = t % S, rp = t / S;
        return w[(((long)k * R + (R - 1 - rp)) * S + (S - 1 - sp)) * C + c];
    };
    const float sc = pow2_scale_of(block_absmax(n, val));
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const long e = (long)c * n + i;
        split_store(val(i) * sc, out + 2 * e - (e & 31));
    }
    if (threadIdx.x == 0) wscale[c] = 1.f / sc;
}

// x * 2^e (e from amax; 1 without) → packed split [P][C/32][hi32|lo32]
__global__ __launch_bounds__(256) void split_pack_x3_kernel(long n4, const f32x4* __restrict__ x,
                                                           const unsigned* __restrict__ amax,
                                                           _Float16* __restrict__ out) {
    const float sc = pow2_scale_for(amax);
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        f32x4 v = x[i];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] *= sc;
        store_split4(v, i, out, 3);
    }
}

// ---------------------------------------------------------------------------
// Weight gradient on packed split operands:
//     dW[k][tap][c] = sum_p dy[p][k] * x[pixel(p, tap)][c]        (p: output pixels)
// GEMM rows = Cout (dy side, KA per tile), columns = (tap, c) flattened (x side,
// 256 per tile = 8 channel groups, one per wave for staging), reduction over
// output pixels, split-K over pixel ranges into fixed-order fp32 slabs
// [split][K][R*S*C] (summed by wg_x3_reduce_kernel — deterministic).
// Both LDS images are pixel-major per channel group: line (group, pixel) =
// 128 B [hi32|lo32], 32 pixels per K-step, written by LDS-DMA; the MFMA
// fragments (8 consecutive pixels of one channel per lane) come from
// ds_read_b64_tr_b16 transposed reads.  Swizzle: 16-B chunk ^= ((pixel>>1)&1)<<2
// makes every 32-lane half of a transposed read cover all 64 banks once.
typedef short s16x4 __attribute__((ext_vector_type(4)));

struct WgX3Args {
    const _Float16* xs;     // packed x  [N*H*W][C/32][64]
    const _Float16* dys;    // packed, scaled dy [M][K/32][64]
    const unsigned* amax;   // the scale dy was split with (pow2_scale_for), nullable
    float* ws;              // slabs [splits][K][RSC]
    int N, H, W, C, K, R, S, stride, pad, dil, Ho, Wo;
    int M, RSC, r_tiles, mps, tiles;
};

// ds_read_b64_tr_b16 as inline asm: the builtin makes hipcc drain the whole
// LDS-DMA queue (vmcnt(0)) before every transposed read, since it cannot tell
// the read from the in-flight DMA's destination.  The caller waits lgkmcnt
// itself before the MFMAs that consume the result (explicit waits below, each
// followed by sched_barrier(0) so no MFMA is scheduled ahead of it).
template <int OFF>
__device__ __forceinline__ s16x4 ds_tr16(unsigned lds_addr) {
    s16x4 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(lds_addr), "i"(OFF));
    return r;
}

__device__ __forceinline__ unsigned lds_addr_of(const char* p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}

__device__ __forceinline__ f16x8 cat_tr(s16x4 lo, s16x4 hi) {
    const auto v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(f16x8, v);
}

// KA = 256 (Cout % 256 == 0): a 256x256 tile, 96 MAC per staged byte instead of
// 64 (KA 128) — the 256x128 body is bound by operand delivery, not the MFMAs
// (MFMA-busy scales with the intensity: 0.25 at KA 64, 0.42 at KA 128).  Its
// stage holds PX = 16 pixels (one MFMA k-slice) so three stages fit in 96 KB.
// The PX = 16 body runs a 4-stage ring (128 KB, inside the epilogue's 132 KB) and
// issues each stage's DMA as GL = TM pieces placed after the MFMAs of one row
// (address math branch-free: one wrap per stage, Wo >= PX, see wg_x3_plan), so
// the per-lane address VALU runs in the MFMA shadow instead of between the
// barrier and the first MFMA of every stage.
template <int KA>
__global__ __launch_bounds__(512, 1) void wgrad_x3_kernel(WgX3Args a) {
    constexpr int BR = 256, GX = BR / 32, GD = KA / 32;
    constexpr int PX = KA == 256 ? 16 : 32;                  // pixels per stage
    constexpr int NS = PX == 16 ? 4 : 3;                     // LDS ring depth
    constexpr int ROW = 128, STAGE = (GX + GD) * PX * ROW;
    constexpr int NX = PX / 8, ND = GD * PX / 64, GL = NX + ND;
    constexpr int TM = KA / 64, TN = 2;
    static_assert(ND >= 1 && (KA == 64 || KA == 128 || KA == 256), "KA must be 64, 128 or 256");
    // the epilogue stages the slab tile (KA x 256 fp32, pitch 264) in passes of
    // 128 rows through the drained ring: at least 132 KiB
    constexpr int EPI_ROWS = KA < 128 ? KA : 128, EPI_PITCH = BR + 8;
    constexpr int LDS = NS * STAGE > EPI_ROWS * EPI_PITCH * 4 ? NS * STAGE : EPI_ROWS * EPI_PITCH * 4;
    __shared__ __attribute__((aligned(1024))) char smem[LDS];

    const int bid = xcd_remap(blockIdx.x, gridDim.x);       // same pixel range → same XCD
    const int split = bid / a.tiles, tile = bid - split * a.tiles;
    const int kt = tile / a.r_tiles, rt = tile - kt * a.r_tiles;
    const int k0 = kt * KA, r0 = rt * BR;
    const int p_begin = split * a.mps;
    const int p_end = min(a.M, p_begin + a.mps);
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);

    // ---- staging bookkeeping ----
    const int Lx = ((lane & 7) ^ (((lane >> 4) & 1) << 2)) * 8;   // logical chunk (halves) this lane fetches
    const int mg = r0 + 32 * w;                                   // first column of this wave's x group
    const bool gvalid = mg < a.RSC;
    const int tap = gvalid ? mg / a.C : 0;
    const int cg = gvalid ? (mg - tap * a.C) >> 5 : 0;
    const int rr = tap / a.S, ss = tap - rr * a.S;
    const int dh = rr * a.dil - a.pad, dw = ss * a.dil - a.pad;
    const int xstride = a.C * 2, dstride = a.K * 2;
    const _Float16* xg = a.xs + cg * 64 + Lx;
    const _Float16* zero = (const _Float16*)g_x3_zero_line;
    int xn[NX], xho[NX], xwo[NX];
    const int hw = a.Ho * a.Wo;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
        const int p = p_begin + 8 * i + (lane >> 3);
        xn[i] = p / hw;
        const int rem = p - xn[i] * hw;
        xho[i] = rem / a.Wo;
        xwo[i] = rem - xho[i] * a.Wo;
    }
    const _Float16* dg[ND];
    int dpp[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
        const int line = 8 * (w * ND + j) + (lane >> 3);
        dpp[j] = line % PX;
        dg[j] = a.dys + (k0 >> 5) * 64 + (line / PX) * 64 + Lx;
    }

    auto issue = [&](int t) {
        char* st = smem + (t % NS) * STAGE;
        const int pb = p_begin + PX * t;
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const int p = pb + 8 * i + (lane >> 3);
            const int hi = xho[i] * a.stride + dh, wi = xwo[i] * a.stride + dw;
            const bool in = gvalid && p < p_end && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
            const long pix = ((long)xn[i] * a.H + hi) * a.W + wi;
            glds16(in ? xg + pix * xstride : zero, st + (w * PX + 8 * i) * ROW);
            xwo[i] += PX;                                    // this slot's pixel for the next K-step
            while (xwo[i] >= a.Wo) {
                xwo[i] -= a.Wo;
                if (++xho[i] == a.Ho) {
                    xho[i] = 0;
                    ++xn[i];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < ND; ++j) {
            const int p = pb + dpp[j];
            glds16(p < p_end ? dg[j] + (long)p * dstride : zero, st + (GX * PX + 8 * (w * ND + j)) * ROW);
        }
    };

    // one DMA piece of stage t (PX == 16 body): k < NX an x slot, else a dy slot.
    // The x slot's pixel advances by PX per stage with at most one row wrap
    // (Wo >= PX): selects, no branches, so the piece can sit between MFMAs.
    auto piece = [&](int t, const int k) {
        char* st = smem + (t & (NS - 1)) * STAGE;
        const int pb = p_begin + PX * t;
        // 32-bit byte offsets (wg_x3_plan: both operands < 4 GiB for KA 256), the
        // validity as a mask and the zero line as a select: no branch
        if (k < NX) {
            const int i = k;
            const int p = pb + 8 * i + (lane >> 3);
            const int hi = xho[i] * a.stride + dh, wi = xwo[i] * a.stride + dw;
            const bool in = gvalid & (p < p_end) & ((unsigned)hi < (unsigned)a.H) & ((unsigned)wi < (unsigned)a.W);
            const unsigned off = (((unsigned)xn[i] * a.H + hi) * a.W + wi) * (unsigned)(xstride * 2);
            const char* src = in ? (const char*)xg : (const char*)zero;
            glds16(src + (in ? off : 0u), st + (w * PX + 8 * i) * ROW);
            const int w2 = xwo[i] + PX;
            const bool wrap = w2 >= a.Wo;
            xwo[i] = wrap ? w2 - a.Wo : w2;
            const int h2 = xho[i] + (wrap ? 1 : 0);
            const bool wrap2 = h2 == a.Ho;
            xho[i] = wrap2 ? 0 : h2;
            xn[i] += wrap2 ? 1 : 0;
        } else {
            const int j = k - NX;
            const int p = pb + dpp[j];
            const bool in = p < p_end;
            const char* src = in ? (const char*)dg[j] : (const char*)zero;
            glds16(src + (in ? (unsigned)p * (unsigned)(dstride * 2) : 0u), st + (GX * PX + 8 * (w * ND + j)) * ROW);
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // transposed-read addressing: 16-lane group G reads 4 pixel rows (q) x 16
    // channels (column block cb = G&1); lane 4q+p supplies row q, channels 4p..4p+3
    const int wk = w & 1, wr = w >> 1;
    const int h = lane >> 5, cb = (lane >> 4) & 1, q = (lane >> 2) & 3, pq = lane & 3;
    int toff[2];
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
        toff[pl] = (8 * h + q) * ROW + (((4 * pl + 2 * cb + (pq >> 1)) ^ (((q >> 1) & 1) << 2)) << 4) + 8 * (pq & 1);
    const int a_line = (GX + wk * TM) * PX * ROW;     // dy groups of this wave
    const int b_line = (wr * TN) * PX * ROW;          // x groups of this wave

    struct Frag {
        f16x8 dh[TM], dl[TM], xh[TN], xl[TN];
    };
    // per-lane LDS byte addresses of the two planes' transposed-read blocks
    const unsigned lds0 = lds_addr_of(smem);
    const unsigned ta0 = lds0 + a_line + toff[0], ta1 = lds0 + a_line + toff[1];
    const unsigned tb0 = lds0 + b_line + toff[0], tb1 = lds0 + b_line + toff[1];
    auto read_frag = [&](Frag& f, int buf, const int s) {
        const unsigned so = buf * STAGE;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            // immediate offsets: tile i (32 rows), half s (16 rows), second read +4 rows
            if (s == 0) {
                f.dh[i] = cat_tr(ds_tr16<0>(ta0 + so + i * PX * ROW), ds_tr16<4 * ROW>(ta0 + so + i * PX * ROW));
                f.dl[i] = cat_tr(ds_tr16<0>(ta1 + so + i * PX * ROW), ds_tr16<4 * ROW>(ta1 + so + i * PX * ROW));
            } else {
                f.dh[i] = cat_tr(ds_tr16<16 * ROW>(ta0 + so + i * PX * ROW),
                                 ds_tr16<20 * ROW>(ta0 + so + i * PX * ROW));
                f.dl[i] = cat_tr(ds_tr16<16 * ROW>(ta1 + so + i * PX * ROW),
                                 ds_tr16<20 * ROW>(ta1 + so + i * PX * ROW));
            }
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            if (s == 0) {
                f.xh[j] = cat_tr(ds_tr16<0>(tb0 + so + j * PX * ROW), ds_tr16<4 * ROW>(tb0 + so + j * PX * ROW));
                f.xl[j] = cat_tr(ds_tr16<0>(tb1 + so + j * PX * ROW), ds_tr16<4 * ROW>(tb1 + so + j * PX * ROW));
            } else {
                f.xh[j] = cat_tr(ds_tr16<16 * ROW>(tb0 + so + j * PX * ROW),
                                 ds_tr16<20 * ROW>(tb0 + so + j * PX * ROW));
                f.xl[j] = cat_tr(ds_tr16<16 * ROW>(tb1 + so + j * PX * ROW),
                                 ds_tr16<20 * ROW>(tb1 + so + j * PX * ROW));
            }
        }
    };
    auto mma = [&](const Frag& f) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.dh[i], f.xh[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.dh[i], f.xl[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.dl[i], f.xh[j], acc[i][j], 0, 0, 0);
            }
    };
    // same software pipeline as conv_x3_kernel<*, 2> (see there); 4*(TM+TN)
    // transposed b64 reads per half, two per MFMA gap.  The reads are inline
    // asm: every consumer MFMA sits behind an explicit lgkmcnt wait + sched_barrier.
    constexpr int NR = 4 * (TM + TN), NM = 3 * TM * TN;
    const int nsteps = p_end > p_begin ? (p_end - p_begin + PX - 1) / PX : 0;
    if constexpr (PX == 16) {
        // one dy fragment set, refilled row by row right after its MFMAs issue
        // (128 accumulators + 32 dy + 2x16 x registers): per stage t
        // [wait own DMA t+1 and this wave's reads, barrier | t+1's x fragments |
        //  rows i = 0..TM-1: t's MFMAs, one DMA piece of stage t+3, t+1's row i]
        struct XF {
            f16x8 xh[TN], xl[TN];
        };
        f16x8 dh[TM], dl[TM];
        XF x0, x1;
        auto read_d = [&](const int i, const unsigned so) {
            dh[i] = cat_tr(ds_tr16<0>(ta0 + so + i * PX * ROW), ds_tr16<4 * ROW>(ta0 + so + i * PX * ROW));
            dl[i] = cat_tr(ds_tr16<0>(ta1 + so + i * PX * ROW), ds_tr16<4 * ROW>(ta1 + so + i * PX * ROW));
        };
        auto read_x = [&](XF& x, const unsigned so) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                x.xh[j] = cat_tr(ds_tr16<0>(tb0 + so + j * PX * ROW), ds_tr16<4 * ROW>(tb0 + so + j * PX * ROW));
                x.xl[j] = cat_tr(ds_tr16<0>(tb1 + so + j * PX * ROW), ds_tr16<4 * ROW>(tb1 + so + j * PX * ROW));
            }
        };
        auto mma_row = [&](const int i, const XF& x) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(dh[i], x.xh[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(dh[i], x.xl[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(dl[i], x.xh[j], acc[i][j], 0, 0, 0);
            }
        };
        static_assert(PX != 16 || GL == TM, "one DMA piece per MFMA row");
        if (nsteps > 0) {
            // prologue: stages 0..NS-2 (past the end: zero lines, never read)
#pragma unroll
            for (int u = 0; u < NS - 1; ++u)
#pragma unroll
                for (int k = 0; k < GL; ++k) piece(u, k);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * GL) : "memory");
            lds_barrier();
            read_x(x0, 0);
#pragma unroll
            for (int i = 0; i < TM; ++i) read_d(i, 0);
            // step t: wait for stage t+1 (stage t+2's pieces stay in flight), barrier,
            // read t+1's fragments row by row beside t's MFMAs, and issue stage
            // t+3's pieces (into the buffer stage t-1 used: every wave finished
            // reading it before this step's barrier) one per MFMA row.  Stages past
            // the end load zero lines into buffers no later stage reads, so every
            // non-final step is the same branch-free code.
            auto step = [&](const int t, const XF& xa, XF& xb) {
                asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NS - 3) * GL) : "memory");
                lds_barrier();
                __builtin_amdgcn_sched_barrier(0);
                const unsigned so = ((t + 1) & (NS - 1)) * STAGE;
                read_x(xb, so);
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    mma_row(i, xa);
                    piece(t + NS - 1, i);
                    read_d(i, so);
                    __builtin_amdgcn_sched_barrier(0);
                }
            };
            auto last = [&](const XF& xa) {
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // + the dummy DMAs
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < TM; ++i) mma_row(i, xa);
            };
            int t = 0;
            for (; t + 2 < nsteps; t += 2) {
                step(t, x0, x1);
                step(t + 1, x1, x0);
            }
            // the x fragments' reads retire before the join's register copies read
            // them (asm reads are untracked; tools/trcheck.py)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if (t + 1 < nsteps) {
                step(t, x0, x1);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                x0 = x1;                                     // one last() call site
            }
            last(x0);
        }
    } else if (nsteps > 0) {
        int q_t = 0;
        auto issue_next = [&]() { issue(q_t++); };
        issue_next();
        if (nsteps > 1) issue_next();
        if (nsteps > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        Frag f0, f1;
        int cur = 0;
        read_frag(f0, 0, 0);
        auto step = [&](const bool ISSUE, const bool NEXT) {
            const int bcur = cur;
            if (ISSUE) issue_next();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // f0 (read last half) landed
            __builtin_amdgcn_sched_barrier(0);
            read_frag(f1, bcur, 1);
            mma(f0);
#pragma unroll
            for (int k = 0; k < NR / 2; ++k) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x001, 2, 0);   // the asm reads count as ALU
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NM - NR / 2, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (NEXT) {
                if (ISSUE) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(GL) : "memory");
                else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                lds_barrier();
                __builtin_amdgcn_sched_barrier(0);
                cur = cur == 2 ? 0 : cur + 1;
                mma(f1);
                read_frag(f0, cur, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#pragma unroll
                for (int k = 0; k < NR / 2; ++k) {
                    __builtin_amdgcn_sched_group_barrier(0x001, 2, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x008, NM - 1 - NR / 2, 0);
                __builtin_amdgcn_sched_barrier(0);
            } else {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                mma(f1);
            }
        };
        int t = 0;
        for (; t + 2 < nsteps; ++t) step(true, true);
        if (t + 1 < nsteps) {
            step(false, true);
            ++t;
        }
        step(false, false);
    }

    // ---- epilogue: the slab tile staged through the drained ring in passes of
    // EPI_ROWS output-channel rows and written as 16-B row chunks (whole 128-B
    // lines, 32-64 stores per thread).  Per-element stores from the fragments
    // (128 per thread, past a wave's 63 outstanding memory ops) stalled every
    // wave on their completion while all CUs wrote their slabs at once.
    const float inv = 1.f / pow2_scale_for(a.amax);
    float* out = a.ws + (long)split * a.K * a.RSC;
    float* t = (float*)smem;
    constexpr int PASSES = KA / EPI_ROWS, C4 = BR / 4;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    lds_barrier();                                             // every wave done with the ring
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
        // wave rows: k_local = wk*TM*32 + i*32 + 8*(r>>2) + 4*h + (r&3) in [ps*EPI_ROWS, +EPI_ROWS)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int kb = wk * TM * 32 + i * 32;
            if (kb / EPI_ROWS != ps) continue;                 // wave-uniform
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    t[(kb - ps * EPI_ROWS + 8 * (r >> 2) + 4 * h + (r & 3)) * EPI_PITCH + wr * 64 + j * 32 + (lane & 31)] =
                        acc[i][j][r] * inv;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        lds_barrier();
        const int mcols = min(BR, a.RSC - r0);                 // multiple of 4 (RSC = R*S*C, C % 32 == 0)
#pragma unroll 4
        for (int e = tid; e < EPI_ROWS * C4; e += 512) {
            const int row = e / C4, c4 = e - row * C4;
            if (c4 * 4 < mcols)
                *(f32x4*)(out + (long)(k0 + ps * EPI_ROWS + row) * a.RSC + r0 + c4 * 4) =
                    *(const f32x4*)(t + row * EPI_PITCH + c4 * 4);
        }
        if (ps + 1 < PASSES) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            lds_barrier();
        }
    }
}

// Weight gradient of a 3x3, stride-1, pad-1, dilation-1 conv from one staged halo
// (round 6; the small-channel layers).  The tiled body above stages a pixel's x
// line once per 256-column group — for C = 64 three groups, the third 1/4 used —
// so its K-step moves 40 KiB per 64x256 tile and runs at MFMA busy 0.25.  Here a
// block owns 64 output channels x all 9 taps x 64 input channels (576 slab
// columns); a K-step is one patch of 4 output rows x 16 columns (Ho % 4 == 0,
// Wo % 16 == 0), staged as its 6 x 18 input halo x 2 channel groups (every tap
// of every row of the patch reads from it) beside the patch's dy lines: 43 KiB
// for 64 pixels.  16x16x32 MFMAs over two 32-pixel k-slices (patch rows 0-1,
// 2-3): wave w owns K rows 32*(w&1).. (2 m-tiles) x input channels 16*(w>>1)..
// of every tap (9 n-tiles, 72 accumulators); the x fragment of tap (r, s) for
// patch row i is staged row i + r read s lines further.  Both operands come from
// ds_read_b64_tr_b16 (8 consecutive pixels of one channel per lane).  Swizzle:
// 16-B chunk ^= 2*(((j>>1)&1) | ((j>>3)&1)<<1) for line j of a run, so the 8
// lines a 32-lane half of a transposed read touches ({a..a+3} u {a+8..a+11}, any
// shift a) fall on 8 distinct 32-B bank slots.  3-stage ring, one barrier per
// K-step; slabs [split][K][R*S*C] as wgrad_x3_kernel's (same reduce), the pixel
// ranges whole patches.
constexpr int WGH_LX = 18, WGH_XL = 12 * WGH_LX, WGH_SL = WGH_XL + 128, WGH_STAGE = WGH_SL * 128, WGH_NS = 3;
constexpr int WGH_PITCH = 580;                       // epilogue rows: 576 slab columns + 4 (conflict-free stores)
// s_waitcnt lgkmcnt(N) for a compile-time N (after unrolling)
__device__ __forceinline__ void wait_lgkm(const int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory"); break;
        default: asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory"); break;
    }
}
__global__ __launch_bounds__(512, 1) void wgrad_x3_halo_kernel(WgX3Args a) {
    constexpr int ROW = 128, LX = WGH_LX, XL = WGH_XL, STAGE = WGH_STAGE, NS = WGH_NS;
    // DMA pieces per stage: XP x pieces as slots 0-3 of the 8 waves (piece w + 8 i;
    // past XP the sink), the 16 dy pieces as slots 4-5 (piece w + 8 (i - 4))
    constexpr int XP = XL / 8, XS = 4, SLOTS = XS + 2;
    static_assert(XP <= 8 * XS, "x pieces");
    constexpr int SINK = NS * STAGE;
    static_assert(XL % 8 == 0 && 32 * WGH_PITCH * 4 <= SINK, "wgrad halo LDS");
    __shared__ __attribute__((aligned(1024))) char smem[SINK + 1024];

    const int bid = xcd_remap(blockIdx.x, gridDim.x);       // same pixel range → same XCD
    const int split = bid / a.tiles, tile = bid - split * a.tiles;
    const int kt = tile / a.r_tiles, ct = tile - kt * a.r_tiles;
    const int k0 = kt * 64, c0 = ct * 64;
    const int HP = a.Ho / 4, WP = a.Wo / 16, npatch = a.N * HP * WP;
    const int P0 = split * a.mps;                            // this split's patches [P0, P1)
    const int P1 = min(npatch, P0 + a.mps);
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    auto xsw = [](int j) { return (((j >> 1) & 1) | (((j >> 3) & 1) << 1)) << 1; };

    // ---- DMA sources: raw-buffer loads (an offset past num_records loads zeros:
    // halo lines outside the image, patches past the range, the sink pieces; the
    // operands are under 2 GiB, wg_halo_shape, so bit 31 marks them).  Stride 1,
    // pad 1: input pixel of halo line (staged row R, column j) of the patch at
    // output pixel p (its top-left) is p + (R - 1) W + j - 1, so a lane's byte
    // offset is the stage's p * 4C plus a constant ----
    const i32x4 xr = buffer_rsrc(a.xs, (unsigned)((long)a.N * a.H * a.W * a.C * 4));
    const i32x4 dr = buffer_rsrc(a.dys, (unsigned)((long)a.M * a.K * 4));
    int xk[XS];                 // byte offset from the stage's p * 4C (signed)
    int xg[XS];                 // halo edge of the line: top row | bottom row << 1 | left column << 2 | right << 3
#pragma unroll
    for (int i = 0; i < XS; ++i) {
        const int pc = min(w + 8 * i, XP - 1);               // past XP: a valid line, loaded into the sink
        const int L = 8 * pc + (lane >> 3), run = L / LX, j = L - run * LX;
        const int R = run >> 1, cg = run & 1;
        xk[i] = ((R - 1) * a.W + j - 1) * (a.C * 4) + ((c0 / 32 + cg) * 64 + ((lane & 7) ^ xsw(j)) * 8) * 2;
        xg[i] = (R == 0 ? 1 : 0) | (R == 5 ? 2 : 0) | (j == 0 ? 4 : 0) | (j == LX - 1 ? 8 : 0);
    }
    int dk[2];                  // dy: byte offset from the stage's p * 4K (line: K group | patch row | column)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int L = 8 * (w + 8 * i) + (lane >> 3), pr = (L >> 4) & 3, cc = L & 15;
        dk[i] = (pr * a.W + cc) * (a.K * 4) + ((k0 / 32 + (L >> 6)) * 64 + ((lane & 7) ^ xsw(L & 31)) * 8) * 2;
    }
    // the patch being issued: index, top-left output pixel, patch row / column (wave-uniform)
    int q_P = P0, q_hp, q_wp, q_p;
    {
        const int n = P0 / (HP * WP), rem = P0 - n * (HP * WP);
        q_hp = rem / WP;
        q_wp = rem - q_hp * WP;
        q_p = (n * a.Ho + 4 * q_hp) * a.Wo + 16 * q_wp;
    }
    int q_t = 0, q_em = 0, q_bad = 0;
    auto begin_issue = [&]() {
        q_em = (q_hp == 0 ? 1 : 0) | (q_hp == HP - 1 ? 2 : 0) | (q_wp == 0 ? 4 : 0) | (q_wp == WP - 1 ? 8 : 0);
        q_bad = q_P >= P1 ? 1 : 0;
    };
    auto piece = [&](const int i) {
        char* st = smem + (q_t % NS) * STAGE;
        if (i < XS) {
            // branch-free: an invalid line gets bit 31 (past num_records) or'd in
            const int pc = w + 8 * i;                        // wave-uniform
            const unsigned bad = (unsigned)q_bad | (unsigned)((xg[i] & q_em) != 0) | (unsigned)(pc >= XP);
            blds16(xr, (unsigned)(q_p * (a.C * 4) + xk[i]) | (bad << 31), 0, pc < XP ? st + pc * 1024 : smem + SINK);
        } else {
            blds16(dr, (unsigned)(q_p * (a.K * 4) + dk[i - XS]) | ((unsigned)q_bad << 31), 0,
                   st + XL * ROW + (w + 8 * (i - XS)) * 1024);
        }
    };
    auto end_issue = [&]() {                                 // the next patch
        ++q_t;
        ++q_P;
        q_p += 16;
        if (++q_wp == WP) {
            q_wp = 0;
            q_p += 3 * a.Wo;
            q_hp = q_hp + 1 == HP ? 0 : q_hp + 1;
        }
    };
    auto issue = [&]() {
        begin_issue();
#pragma unroll
        for (int i = 0; i < SLOTS; ++i) piece(i);
        end_issue();
    };

    f32x4 acc[2][9];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // ---- transposed-read addresses (stage-relative bytes, k-slice 0): 16-lane
    // group G reads patch row G >> 1 (+2 in k-slice 1), pixels 8 (G & 1) + q (+4 the
    // second read) of 16 channels; lane 4q + pp supplies row q, channels 4pp..4pp+3 ----
    const int G = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int kh = w & 1, cb4 = w >> 1, cg = cb4 >> 1, cbl = cb4 & 1;
    unsigned a_ad[2][2];        // dy: [m-tile][plane]; line 8G + q of the wave's K group (+4: same swizzle)
    {
        const int j = 8 * G + q;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int pl = 0; pl < 2; ++pl)
                a_ad[mi][pl] = (unsigned)((XL + 64 * kh + j) * ROW + ((((pl * 4 + mi * 2 + (pp >> 1)) ^ xsw(j))) << 4) +
                                          8 * (pp & 1));
    }
    unsigned b_ad[3][2][2];     // x: [tap column s][read half][plane], staged row G >> 1 (+ k-slice * 2 + r)
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
            const int j = 8 * (G & 1) + q + s + 4 * h2;
            const int run = (G >> 1) * 2 + cg;
#pragma unroll
            for (int pl = 0; pl < 2; ++pl)
                b_ad[s][h2][pl] = (unsigned)((run * LX + j) * ROW + ((((pl * 4 + cbl * 2 + (pp >> 1)) ^ xsw(j))) << 4) +
                                             8 * (pp & 1));
        }
    const unsigned lds0 = lds_addr_of(smem);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) a_ad[mi][pl] += lds0;
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
            for (int pl = 0; pl < 2; ++pl) b_ad[s][h2][pl] += lds0;

    // Per K-step t (stage t in LDS): 18 tap-slices v = 9 * k-slice + tap, each's x
    // fragments read two ahead, k-slice 1's dy fragments in two halves at v = 3 and
    // 6; after v = 15 the step's one barrier (stage t+1 landed everywhere, stage
    // t-1 read by everyone), then stage t+1's k-slice-0 dy and first x fragments
    // read beside v = 16-17, and stage t+NS-1's DMA pieces (into stage t-1's
    // buffer) issued between them — the barrier and the next stage's first LDS
    // latency sit behind this wave's own MFMAs.  lgkmcnt counts this wave's
    // transposed reads in issue order (at most 15 outstanding: waits of 8 and 12).
    // A step with no stage after it reads none (an asm read whose result is never
    // used leaves its registers free to the compiler while it is in flight).
    const int nsteps = P1 - P0;
    f16x8 dfa[2][2], dfb[2][2], xfr[3][2];
    auto read_d = [&](f16x8 (&d)[2][2], const int mi, const unsigned so) {
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
            d[mi][pl] = cat_tr(ds_tr16<0>(a_ad[mi][pl] + so), ds_tr16<4 * ROW>(a_ad[mi][pl] + so));
    };
    auto read_x = [&](const int v, const unsigned so) {
        const int kk = v / 9, tap = v - 9 * (v / 9), r = tap / 3, s = tap - 3 * (tap / 3);
        const unsigned ro = so + (unsigned)((2 * kk + r) * 2 * LX * ROW);
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
            xfr[v % 3][pl] = cat_tr(ds_tr16<0>(b_ad[s][0][pl] + ro), ds_tr16<0>(b_ad[s][1][pl] + ro));
    };
    auto mfma_v = [&](const f16x8 (&d)[2][2], const int v) {
        const int tap = v % 9;
        const f16x8* xf = xfr[v % 3];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
            acc[mi][tap] = __builtin_amdgcn_mfma_f32_16x16x32_f16(d[mi][0], xf[0], acc[mi][tap], 0, 0, 0);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
            acc[mi][tap] = __builtin_amdgcn_mfma_f32_16x16x32_f16(d[mi][0], xf[1], acc[mi][tap], 0, 0, 0);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
            acc[mi][tap] = __builtin_amdgcn_mfma_f32_16x16x32_f16(d[mi][1], xf[0], acc[mi][tap], 0, 0, 0);
    };
    if (nsteps > 0) {
#pragma unroll
        for (int u = 0; u < NS - 1; ++u) issue();           // stages past the end: zero lines, never read
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * SLOTS) : "memory");
        lds_barrier();
        __builtin_amdgcn_sched_barrier(0);
        read_d(dfa, 0, 0u);
        read_d(dfa, 1, 0u);
        read_x(0, 0u);
        read_x(1, 0u);
        unsigned so = 0;
        auto step = [&](const bool next) {
            const unsigned sn = so == (unsigned)((NS - 1) * STAGE) ? 0u : so + STAGE;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                read_x(v + 2, so);
                if (v == 3) read_d(dfb, 0, so + 32 * ROW);
                if (v == 6) read_d(dfb, 1, so + 32 * ROW);
                wait_lgkm(v >= 3 && v <= 8 ? 12 : 8);
                __builtin_amdgcn_sched_barrier(0);
                mfma_v(v < 9 ? dfa : dfb, v);
                __builtin_amdgcn_sched_barrier(0);
            }
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 3) * SLOTS) : "memory");   // stage t+1
            lds_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if (next) {
                read_d(dfa, 0, sn);
                read_d(dfa, 1, sn);
                wait_lgkm(12);                                          // x of v = 16
            } else {
                wait_lgkm(4);
            }
            __builtin_amdgcn_sched_barrier(0);
            mfma_v(dfb, 16);
            __builtin_amdgcn_sched_barrier(0);
            if (next) read_x(0, sn);
            begin_issue();
            piece(0);
            piece(1);
            piece(2);
            wait_lgkm(next ? 12 : 0);                                   // x of v = 17
            __builtin_amdgcn_sched_barrier(0);
            mfma_v(dfb, 17);
            __builtin_amdgcn_sched_barrier(0);
            if (next) read_x(1, sn);
#pragma unroll
            for (int i = 3; i < SLOTS; ++i) piece(i);
            end_issue();
            __builtin_amdgcn_sched_barrier(0);
            so = sn;
        };
        for (int t = 0; t + 1 < nsteps; ++t) step(true);
        step(false);
    }

    // ---- epilogue: the 64 x 576 slab tile through the drained ring in two passes
    // of 32 K rows (one per wave row), stored as 16-B row chunks ----
    const float inv = 1.f / pow2_scale_for(a.amax);
    float* out = a.ws + (long)split * a.K * a.RSC;
    float* T = (float*)smem;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // + the DMAs past the end
    lds_barrier();
#pragma unroll
    for (int ps = 0; ps < 2; ++ps) {
        if (kh == ps) {
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int tap = 0; tap < 9; ++tap)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        T[(16 * mi + 4 * G + e) * WGH_PITCH + tap * 64 + 16 * cb4 + (lane & 15)] = acc[mi][tap][e] * inv;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        lds_barrier();
        for (int e = tid; e < 32 * 144; e += 512) {
            const int row = e / 144, c4 = e - row * 144, tap = c4 >> 4, cc = (c4 & 15) * 4;
            *(f32x4*)(out + (long)(k0 + 32 * ps + row) * a.RSC + tap * a.C + c0 + cc) =
                *(const f32x4*)(T + row * WGH_PITCH + tap * 64 + cc);
        }
        if (ps == 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            lds_barrier();
        }
    }
}

// dw[i] = sum_split ws[split][i], fixed order
// Sum of the split-K slabs [splits][n4] (fixed order, deterministic).  G = 1: a
// thread per float4 element, its slabs summed left to right with 16 loads in
// flight; G = 4 (8 loads in flight per thread) (many splits: the small layers' wgrads split over up to ~75
// pixel ranges): the four waves of a block take the same 64 elements, wave g
// summing slabs g, g+4, g+8, ... left to right, and the four partial sums are
// added in wave order through LDS — 4x fewer dependent load round trips per
// element.
template <int G>
__global__ __launch_bounds__(256) void wg_x3_reduce_kernel(long n4, int splits, const f32x4* __restrict__ ws,
                                                          f32x4* __restrict__ dw) {
    constexpr int B = G == 1 ? 16 : 8;      // slab loads in flight per thread
    auto sum_from = [&](long i, int k0, int step) {
        f32x4 s = {0.f, 0.f, 0.f, 0.f};
        bool first = true;
        for (int k = k0; k < splits; k += B * step) {
            f32x4 v[B];
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (k + u * step < splits) v[u] = __builtin_nontemporal_load(&ws[(long)(k + u * step) * n4 + i]);
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (k + u * step < splits) {
                    if (first) s = v[u];
                    else
#pragma unroll
                        for (int e = 0; e < 4; ++e) s[e] += v[u][e];
                    first = false;
                }
        }
        return s;
    };
    if constexpr (G == 1) {
        const long stride = (long)gridDim.x * blockDim.x;
        for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) dw[i] = sum_from(i, 0, 1);
    } else {
        static_assert(G == 4, "wg_x3_reduce_kernel: G is 1 or 4");
        __shared__ f32x4 part[G][64];
        const int g = threadIdx.x >> 6, l = threadIdx.x & 63;
        for (long b0 = (long)blockIdx.x * 64; b0 < n4; b0 += (long)gridDim.x * 64) {
            const long i = b0 + l;
            if (i < n4 && g < splits) part[g][l] = sum_from(i, g, G);
            __syncthreads();
            if (g == 0 && i < n4) {
                f32x4 s = part[0][l];
                for (int q = 1; q < G && q < splits; ++q)
#pragma unroll
                    for (int e = 0; e < 4; ++e) s[e] += part[q][l][e];
                dw[i] = s;
            }
            __syncthreads();
        }
    }
}

// wgrad_x3_halo_kernel's shapes: 3x3, stride 1, pad = dilation = 1, C and K
// multiples of 64 up to 128 (the layers it was measured on), whole 4x16-pixel
// patches, operands under 2 GiB (32-bit byte offsets); d->tile == -1 keeps the
// tiled body (A/B, tests)
static bool wg_halo_shape(const hkp_conv_desc* d, int ho, int wo) {
    return d->tile != -1 && d->r == 3 && d->s == 3 && d->stride == 1 && d->pad == 1 && d->dilation == 1 &&
           d->k % 64 == 0 && d->c % 64 == 0 && d->k <= 128 && d->c <= 128 && wo % 16 == 0 && ho % 4 == 0 &&
           ho == d->h &&
           wo == d->w && (long)d->n * d->h * d->w * d->c * 4 < (1L << 31) && (long)d->n * ho * wo * d->k * 4 < (1L << 31);
}

// ka = 0: the halo body (r_tiles = its 64-channel column tiles, mps = patches per split)
static void wg_x3_plan(const hkp_conv_desc* d, long M, int wo, int* splits, int* mps, int* ka, int* r_tiles) {
    if (wg_halo_shape(d, (int)(M / ((long)d->n * wo)), wo)) {
        const long tiles = (long)(d->k / 64) * (d->c / 64), np = M / 64;   // 4x16-pixel patches
        // one 130 KiB block per CU: one round of 256, or the caller's CU budget
        long sp = std::max(1L, (d->tile > 0 ? d->tile : 256) / tiles);
        sp = std::min(sp, np);
        const long per = (np + sp - 1) / sp;
        *ka = 0;
        *r_tiles = d->c / 64;
        *mps = (int)per;                                   // patches per split
        *splits = (int)((np + per - 1) / per);
        return;
    }
    // KA 256's 16-pixel stages advance each x slot with at most one row wrap
    // (and 32-bit byte offsets into both operands)
    const bool ka256 = d->k % 256 == 0 && wo >= 16 && (long)d->n * d->h * d->w * d->c * 4 < (1L << 32) &&
                       M * d->k * 4 < (1L << 32);
    *ka = ka256 ? 256 : d->k % 128 == 0 ? 128 : 64;
    const long rsc = (long)d->r * d->s * d->c;
    *r_tiles = (int)((rsc + 255) / 256);
    const long tiles = (long)(d->k / *ka) * *r_tiles;
    // One 512-thread block per CU at a time: pick the split count whose block
    // count best fills whole rounds of 256 CUs (few rounds, few slabs to reduce),
    // with at least 16 K-steps (512 pixels) per block.
    const long max_sp = std::max(1L, (M + 511) / 512);
    long sp = 1;
    double best = -1.0;
    for (long c = 1; c <= max_sp && d->tile <= 0; ++c) {
        const long blocks = tiles * c;
        const long rounds = (blocks + 255) / 256;
        if (rounds > 4) break;
        const double fill = (double)blocks / (256.0 * rounds);
        const double score = fill - 0.03 * rounds;            // prefer fewer rounds / slabs at equal fill
        if (score > best + 1e-9) {
            best = score;
            sp = c;
        }
    }
    if (d->tile > 0) sp = std::max(1L, std::min<long>(max_sp, d->tile / tiles));   // the caller's CU budget
    long m = (M + sp - 1) / sp;
    m = (m + 31) / 32 * 32;
    *splits = (int)((M + m - 1) / m);
    *mps = (int)m;
}


// Stem operand: the image → zero-padded NHWC4 planes [2][N][Hp][Wp][4] (hi, then
// lo = f16(x-hi)); padded pixel (hp, wp) = input (hp-3, wp-3).  U8: the image is
// the uint8 HWC batch cv2.imread gives ([N][H][W][C], BGR) and x = u8 / 255 in
// fp32 — ToTensor (dataset.py:16) fused into the stem's operand pack.
template <bool U8>
__global__ __launch_bounds__(256) void stem_pack_x3_kernel(int N, int C, int H, int W, int Hp, int Wp,
                                                          const void* __restrict__ src, _Float16* __restrict__ out) {
    const long total = (long)N * Hp * Wp;
    const long plane = total * 4;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < total; p += stride) {
        const int wp = (int)(p % Wp);
        const long t = p / Wp;
        const int hp = (int)(t % Hp);
        const int n = (int)(t / Hp);
        const int h = hp - 3, w = wp - 3;
        const bool in = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        f32x4 v;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (!(in && c < C)) {
                v[c] = 0.f;
            } else if constexpr (U8) {
                const uint8_t u = ((const uint8_t*)src)[(((long)n * H + h) * W + w) * C + c];
                v[c] = __fdiv_rn((float)u, 255.f);
            } else {
                v[c] = ((const float*)src)[(((long)n * C + c) * H + h) * W + w];
            }
        }
        h16x4 hv, lv;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const _Float16 hh = (_Float16)v[c];
            hv[c] = hh;
            lv[c] = (_Float16)(v[c] - (float)hh);
        }
        *(h16x4*)(out + p * 4) = hv;
        *(h16x4*)(out + plane + p * 4) = lv;
    }
}

// Stem weight OIHW [K][C][7][7] * 2^e_k → [K][r][hi32|lo32], 32 = 8 taps (s; 7 = 0)
// x 4 channels (C..3 = 0); one block per k, wscale[k] = 2^-e_k
__global__ __launch_bounds__(256) void stem_weight_pack_x3_kernel(int C, const float* __restrict__ w,
                                                                 _Float16* __restrict__ out,
                                                                 float* __restrict__ wscale) {
    const int k = blockIdx.x;
    const float* wk = w + (long)k * C * 49;
    const float sc = pow2_scale_of(block_absmax(C * 49, [&](int i) { return wk[i]; }));
    for (int e = threadIdx.x; e < 7 * 32; e += blockDim.x) {
        const int c = e & 3, s = (e >> 2) & 7, r = e >> 5;
        const float v = (s < 7 && c < C) ? wk[(c * 7 + r) * 7 + s] * sc : 0.f;
        split_store(v, out + ((long)k * 7 + r) * 64 + s * 4 + c);
    }
    if (threadIdx.x == 0) wscale[k] = 1.f / sc;
}

static bool stem_x3_shape(const hkp_conv_desc* d) {
    return d && d->in_layout == HKP_LAYOUT_NCHW && d->c >= 1 && d->c <= 4 && d->r == 7 && d->s == 7 &&
           d->stride == 2 && d->pad == 3 && d->dilation == 1 && d->k % 64 == 0;
}

// Compute units (one 512-thread conv block per CU at a time); cached per process.
static int x3_cus() {
    static int n = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                      hipSuccess || v <= 0)
            v = 256;
        return v;
    }();
    return n;
}

// stream-K: per-tile arrival counters in the first X3_SK_CNT_BYTES of the
// workspace, then two fp32 slabs per block (a block splits at most its first
// and its last tile): 2 * CUs * BN * 1 KiB (256 x BN floats per slab)
constexpr long X3_SK_CNT_BYTES = 64 << 10;
static long x3_sk_ws_bytes(int bn) { return X3_SK_CNT_BYTES + 2L * x3_cus() * bn * 1024; }

// stream-K overhead per block in tile times: every block writes up to two
// fp32 slabs and most reduce a tile from two (~0.4 MB per CU, all CUs at once),
// plus a second pipeline fill — so it shrinks with the K depth nks of a tile.
// Fitted to in-process A/Bs on the box (column-grouped stream-K vs one tile per
// block): t4 nks 144 0.34, t3 / layer3 nks 72 0.46 / 0.48, t2 nks 36 0.63,
// t1 / layer1 nks 18 1.18 / 1.46 tile-times: 0.2 + 19 / nks.
static double sk_over(int nks) { return 0.2 + 19.0 / nks; }

// Tile width (and data-parallel vs stream-K) for Cout = k over m_tiles 256-row
// tiles: data-parallel costs ceil(blocks / CUs) rounds of one tile each,
// stream-K blocks / CUs + the overhead above; minimise rounds x the measured
// per-column tile cost (256x256: 0.9, 256x128: 1.0, 256x64: 1.25 — wider tiles
// reuse each A line more).  E.g. C2 layer4 (600 m-tiles, Cout 512): 1200
// 256x256 tiles = 4.69 rounds, data-parallel (5 rounds); training layer4 (150
// m-tiles): 600 256x128 tiles stream-K (2.34 + 0.25 rounds) beats 3 rounds of
// 256x128 (data-parallel's best).  Measured on C2 layer4: 256x256 1.70 ms vs
// 256x128 1.82 ms; on C2 layer3 (Cout 256, 600 m-tiles) 256x256 loses to round
// quantisation (0.53 vs 0.47 ms).  No stream-K with 256x256 tiles (the one-tile
// 256x256 kernel sits at 255 VGPRs; the stream-K loop would spill).
// Split-K tail (conv_x3_tail_kernel) for a one-tile grid of m_tiles x nt tiles:
// the group count NG = tm*S of the tail grid (0: no tail) — each of the tm
// m-tiles past the last full round in S equal K segments, one per group — and its
// cost in tile times, 1/S + 0.08 (a segment's fill, slab hand-off and combine)
// per round of segments.  C2 layer3 on 256x256 tiles (88 tail tiles): S = 2,
// ~0.58 instead of 1; training t4: S = 5.  C2 layer4 (88 tail m-tiles x 2
// columns) has no S >= 2 that beats one plain round.  (A fractional tail — every
// CU's group a fraction of a tile, two segments per block — was built in round 5
// and measured slower end to end: DESIGN "Fractional split-K tail".)
// (Multi-round tails — S segments per tail m-tile past one round, one slab per
// segment — measured slower in round 5: the B=8 shard's layer3 0.138 -> 0.164 ms
// at S = 3, C2 layer3 0.384 -> 0.418 ms at S = 5; profiles/r05_multi_*.  The tail
// on 256x128 grids of >= 2 rounds (C2 layer2) measured neutral: C2 1753.0 vs 1755.5
// img/s, C4 / C3 unchanged; profiles/r05_tail128_*_v2.)
HKP_AB_KNOB(int, g_x3_split_tail, 0);                 // hkp_debug_x3_split_tail
static long x3_tail_groups(long m_tiles, int nt, int nks, double* cost = nullptr) {
    const long G = x3_cus(), tiles = m_tiles * nt, tr = tiles % G;
    const long tm = m_tiles - tiles / G * G / nt;
    double best = 1.0;
    long ng = 0;
    if (tr > 0) {
        for (int S = 2; S <= 8 && nks / S >= 4 && tm * S * nt <= G; ++S)
            if (1.0 / S + 0.08 < best - 1e-9) {
                best = 1.0 / S + 0.08;
                ng = tm * S;
            }
    }
    if (cost) *cost = tr > 0 ? best : 0.0;
    return ng;
}

struct X3Plan {
    int bn;
    bool sk;
};
static X3Plan x3_plan(int k, long m_tiles, int nks, bool sk_ok, double over) {
    const int G = x3_cus();
    X3Plan best{64, false};
    double best_cost = 1e300;
    for (int bn : {256, 128, 64}) {
        if (k % bn) continue;
        const long tiles = m_tiles * (k / bn);
        const double col = bn * (bn == 256 ? 0.9 : bn == 128 ? 1.0 : 1.25);
        double tail = (tiles % G) ? 1.0 : 0.0;             // the last, partly filled round
        if (bn == 256 && sk_ok) x3_tail_groups(m_tiles, k / bn, nks, &tail);
        const double dp = ((double)(tiles / G) + tail) * col;
        if (dp < best_cost - 1e-9) {
            best_cost = dp;
            best = {bn, false};
        }
        const int ng = G / (k / bn);       // column-grouped stream-K: groups of k/bn blocks
        if (sk_ok && bn != 256 && ng > 0 && m_tiles % ng && tiles * 4 <= X3_SK_CNT_BYTES) {
            const double skc = ((double)m_tiles / ng + over) * col;
            if (skc < best_cost - 1e-9) {
                best_cost = skc;
                best = {bn, true};
            }
        }
    }
    return best;
}

// The kernel a launch runs (conv_x3_kernel<bn, STEM, pair, mfd, sk, P>):
//   256x256                 16x16x32 body, 2-stage ring (C2 layer4 1.79 -> 1.62 ms
//                           vs the 32x32x16 body: same cycles per FLOP at lower
//                           power, so the chip holds a higher clock —
//                           MI355X_MICROARCH.md DVFS item 7)
//   256x128, >= 2 rounds    16x16x32 body, 3-stage ring (C2 layer3 +6 %, layer2 +5 %)
//   256x128, one round      32x32x16 body (the 16x16 body's longer fill lost 8-11 %;
//                           round 5: AUTO on packed f16x3 runs the 16x16 body here
//                           and 256x64 pairs for >= 1 round — x3_choose)
//   256x64                  16x16x32 body, two blocks per CU (layer1 0.223 -> 0.166 ms)
//   stream-K 256x128 / 64   16x16x32 / 32x32x16 bodies (training t4 fwd +3-6 %, t3 +6 %)
// hkp_conv_desc.tile (HKP_TILE_*) forces one of them — every body is reachable
// for the parity tests; results agree to fp32 summation order.
struct X3Choice {
    int bn, mfd;
    bool pair, sk;
    bool halo = false;                 // conv_x3_halo_kernel<P>
    bool a3 = false;                   // conv_x3_a3_kernel<P> (256x256, 3-stage A ring)
    bool duo = false;                  // conv_x3_duo_kernel<1> (256x128, two 4-wave blocks per CU)
    int bm = 256;                      // rows per tile (192 / 160: conv_x3_a3_192 / _160_kernel<P>)
};
// halo: 0 the halo-tile body cannot take the shape, 1 it can (HKP_TILE_HALO
// forces it), 2 it is also the default (64 input channels: measured faster;
// at 128 channels it ties the ring bodies, which then stay)
static X3Choice x3_choose_base(int k, long m_tiles, int nks, bool sk_ok, int policy, int halo);
static X3Choice x3_choose(int k, long m_tiles, int nks, bool sk_ok, int policy, int halo, int P);
// AUTO (= AUTO_A3): the planner's choice, its 256x256 one-tile grids on the A3
// body (measured in-process on one box: C2 1721 -> 1741 img/s, C4 2616 -> 2657;
// per conv -1...-4 % on the 1x1 and 3x3 shapes of C4, -1 % on C2's layer3/4;
// HKP_TILE_256 / 256_TAIL keep the 2-stage body)
// DUO (the plain-fp16 256x128 two-blocks-per-CU body) where forced and legal;
// other operand layouts plan as AUTO
HKP_AB_KNOB(int, g_x3_pair128, 1);                    // hkp_debug_x3_pair128
static X3Choice x3_choose(int k, long m_tiles, int nks, bool sk_ok, int policy, int halo, int P) {
    if (policy == HKP_TILE_DUO) {
        if (P == 1 && k % DUO_BN == 0) {
            X3Choice c{DUO_BN, 16, false, false};
            c.duo = true;
            return c;
        }
        policy = HKP_TILE_AUTO;
    }
    // the overlapped dgrad's A3 request (Policy.dgrad_overlap_tile) on a 64- or
    // 128-channel output, which A3 cannot take: plan it as AUTO (the rules below)
    if (policy == HKP_TILE_256_A3 && P == 3 && k % 256 != 0 && g_x3_pair128) policy = HKP_TILE_AUTO;
    // 192-row A3 tiles: packed operands with 256-divisible outputs; AUTO otherwise
    if (policy == HKP_TILE_192_A3 && (!x3_packed(P) || k % 256 != 0)) policy = HKP_TILE_AUTO;
    if (policy == HKP_TILE_160_A3 && (!x3_packed(P) || k % 128 != 0)) policy = HKP_TILE_AUTO;
    if (policy != HKP_TILE_AUTO_A3 && policy != HKP_TILE_AUTO) return x3_choose_base(k, m_tiles, nks, sk_ok, policy, halo);
    X3Choice c = x3_choose_base(k, m_tiles, nks, sk_ok, HKP_TILE_AUTO, halo);
    if (c.bn == 256 && !c.sk && !c.halo && !c.pair) c.a3 = true;
    // AUTO, plain fp16: the DUO body where it measured faster than the one-tile
    // bodies (tools/conv_ab.py, in-process, profiles/r05_duo_*): K-depth 64 (one
    // K-step: C4's layer1 1x1 expansions, 64 -> 256: -12 %, all fill and epilogue)
    // and 128-wide outputs (layer2: -4...-10 % against the one-block 256x128 body);
    // the long-K 256-wide shapes stay on A3 (DUO +10...+33 %: its half-line stream
    // moves 1.5x the operand bytes per MAC).  AUTO_A3 keeps the round-4 planner.
    if (policy == HKP_TILE_AUTO && P == 1 && !c.halo && k % DUO_BN == 0 && (nks == 1 || k == DUO_BN)) {
        X3Choice d{DUO_BN, 16, false, false};
        d.duo = true;
        return d;
    }
    // AUTO, packed f16x3, one-tile grids: the 256x64 two-blocks-per-CU tiles (one
    // block's fill and epilogue overlap the other's K loop) for short-K convs (the
    // 1x1 downsamples, K-depth <= 256 channels: C2 128 -> 256 0.061 -> 0.052 ms;
    // B=8 256 -> 512 0.061 -> 0.040 and 128 -> 256 0.021 -> 0.019) and where the
    // cost table picks 256x128 tiles over at least a round of them (C2 layer2 3x3
    // 0.140 -> 0.125 ms, its stride-2 conv1 0.086 -> 0.073, the 64 -> 128 downsample
    // 0.033 -> 0.025); a one-round 256x128 grid on the 16x16x32 body (the B=8 shard's
    // layer2 0.053 -> 0.040 ms: the 32x32x16 body's shorter fill no longer wins).
    // Stream-K plans stay (B=8 layer3: 0.128 ms vs 0.138 on pairs), and so do grids
    // of more than 3 rounds of 256x256 tiles, where the longer grid's steady state
    // favours the larger tiles (C2 256 -> 512 downsample at 4.7 rounds: even; config
    // C5 at 1280x960, 4.7-37 rounds: its 128-wide 3x3 1.05x, its 1x1s 1.04-1.27x
    // slower on pairs).  tools/conv_ab.py, profiles/r05_l2_conv_ab*.log
    if (policy == HKP_TILE_AUTO && P == 3 && !c.halo && !c.sk && g_x3_pair128) {
        const bool small = (double)m_tiles * k <= 3.0 * 256 * x3_cus();
        if (small && (nks <= 8 || (c.bn == 128 && m_tiles * (k / 128) >= x3_cus()))) return {64, 16, true, false};
        if (c.bn == 128 && m_tiles * (k / 128) < x3_cus()) c.mfd = 16;
    }
    return c;
}
static X3Choice x3_choose_base(int k, long m_tiles, int nks, bool sk_ok, int policy, int halo) {
    // the halo-tile body wherever the shape allows it, unless a tile body is forced
    if ((halo >= 1 && policy == HKP_TILE_HALO) ||
        (halo == 2 && (policy == HKP_TILE_AUTO || policy == HKP_TILE_256_TAIL || policy == HKP_TILE_256_A3 ||
                       policy == HKP_TILE_192_A3 || policy == HKP_TILE_160_A3))) {
        X3Choice c{64, 16, true, false};
        c.halo = true;
        return c;
    }
    switch (policy) {
        case HKP_TILE_256:
            if (k % 256 == 0) return {256, 16, false, false};
            break;
        case HKP_TILE_128_MF16:
            if (k % 128 == 0) return {128, 16, false, false};
            break;
        case HKP_TILE_128_MF32:
            if (k % 128 == 0) return {128, 32, false, false};
            break;
        case HKP_TILE_64_PAIR:
            return {64, 16, true, false};
        case HKP_TILE_256_TAIL:            // 256x256, the partial last round as split-K segments
            if (k % 256 == 0) return {256, 16, false, false};
            break;
        case HKP_TILE_256_A3:              // the same on the A3 body
            if (k % 256 == 0) return {256, 16, false, false, false, true};
            break;
        case HKP_TILE_192_A3:              // 192x256 / 160x256 (160x128) tiles on the A3 body
        case HKP_TILE_160_A3:              // (x3_choose checked the operands)
            if (k % 256 == 0 || (policy == HKP_TILE_160_A3 && k % 128 == 0)) {
                X3Choice c{k % 256 == 0 ? 256 : 128, 16, false, false, false, true};
                c.bm = policy == HKP_TILE_192_A3 ? 192 : 160;
                return c;
            }
            break;
        default:
            break;
    }
    const bool sk = sk_ok && policy != HKP_TILE_NO_SK && policy != HKP_TILE_256_TAIL && policy != HKP_TILE_256_A3;
    const X3Plan pl = x3_plan(k, m_tiles, nks, sk, policy == HKP_TILE_SK ? 0.0 : sk_over(nks));
    if (pl.sk) return {pl.bn, pl.bn == 128 ? 16 : 32, false, true};
    if (pl.bn == 256) return {256, 16, false, false};
    if (pl.bn == 128) return {128, (double)m_tiles * (k / 128) >= 2.0 * x3_cus() ? 16 : 32, false, false};
    return {64, 16, true, false};
}

static const X3Choice X3_STEM{64, 16, true, false};

static int x3_kernel_name(const X3Choice& c, bool stem, int P, char* buf, int len) {
    if (c.halo) return snprintf(buf, len, "conv_x3_halo_kernel<%d>", P);
    if (c.duo) return snprintf(buf, len, "conv_x3_duo_kernel<%d>", P);
    if (c.a3)
        return snprintf(buf, len, c.bm == 192                  ? "conv_x3_a3_192_kernel<%d>"
                                  : c.bm == 160 && c.bn == 128 ? "conv_x3_a3_160x128_kernel<%d>"
                                  : c.bm == 160                ? "conv_x3_a3_160_kernel<%d>"
                                                               : "conv_x3_a3_kernel<%d>", P);
    return snprintf(buf, len, "conv_x3_kernel<%d, %s, %s, %d, %s, %d>", c.bn, stem ? "true" : "false",
                    c.pair ? "true" : "false", c.mfd, c.sk ? "true" : "false", P);
}

// the A3 grid (conv_x3_a3_kernel<P>)
template <int P>
static void launch_a3(dim3 grid, hipStream_t st, const X3Args& a) {
    hipLaunchKernelGGL(conv_x3_a3_kernel<P>, grid, dim3(512), 0, st, a);
}

template <int P>
static void launch_x3_p(const X3Choice& c, dim3 grid, hipStream_t st, const X3Args& a) {
    if (c.a3)
        launch_a3<P>(grid, st, a);
    else if (c.sk && c.bn == 128)
        hipLaunchKernelGGL((conv_x3_kernel<128, false, false, 16, true, P>), grid, dim3(512), 0, st, a);
    else if (c.sk)
        hipLaunchKernelGGL((conv_x3_kernel<64, false, false, 32, true, P>), grid, dim3(512), 0, st, a);
    else if (c.bn == 256)
        hipLaunchKernelGGL((conv_x3_kernel<256, false, false, 16, false, P>), grid, dim3(512), 0, st, a);
    else if (c.bn == 128 && c.mfd == 16)
        hipLaunchKernelGGL((conv_x3_kernel<128, false, false, 16, false, P>), grid, dim3(512), 0, st, a);
    else if (c.bn == 128)
        hipLaunchKernelGGL((conv_x3_kernel<128, false, false, 32, false, P>), grid, dim3(512), 0, st, a);
    else
        hipLaunchKernelGGL((conv_x3_kernel<64, false, true, 16, false, P>), grid, dim3(512), 0, st, a);
}

// a.RS, a.cch (128-B lines per pixel), a.M ... set by the caller; P = operand
// layout (3 packed f16x3 split, 1 plain fp16)
HKP_AB_KNOB(unsigned long long*, g_x3_stamps, nullptr);   // hkp_debug_x3_stamps
HKP_AB_KNOB(int, g_x3_stagger_ns, 0);                 // hkp_debug_x3_stagger
HKP_AB_KNOB(int, g_x3_store, 0);                      // hkp_debug_x3_store
HKP_AB_KNOB(int, g_duo_stagger_ns, -1);               // hkp_debug_duo_stagger
HKP_AB_KNOB(int, g_x3_prio, 0);                       // hkp_debug_x3_prio
HKP_AB_KNOB(int, g_x3_a_wrap, 0);                     // hkp_debug_x3_a_wrap

// the halo-tile body takes this launch (shape, plain dense output, no fused
// epilogue, 32-bit halo offsets)
// lines: 128-B input lines per pixel (32 channels each for P 3, 64 for P 1)
static int x3_halo_level(bool ok, int lines, int P) {
    return !ok ? 0 : lines * (x3_packed(P) ? 32 : 64) <= 64 ? 2 : 1;
}

static bool x3_halo_ok(const X3Args& a, int k) {
    return halo_shape(a.stride, a.R, a.S, a.pad, a.dil, a.Ho, a.Wo, k) && a.ost == 0 && a.ep_ss == nullptr &&
           a.mt0 == 0 && a.plane == 0 && (long)a.N * a.H * a.W * a.cch * 64L + 64 < (1L << 32);
}

// run f with std::integral_constant<int, P> for a runtime operand layout P
template <typename F>
static void x3_dispatch_p(int P, F&& f) {
    switch (P) {
        case 3: f(std::integral_constant<int, 3>{}); break;
        case 1: f(std::integral_constant<int, 1>{}); break;
        case 2: f(std::integral_constant<int, 2>{}); break;
        case 4: f(std::integral_constant<int, 4>{}); break;
        default: break;
    }
}

static void launch_x3(int k, long m_tiles, int policy, int P, hipStream_t st, X3Args& a, void* ws = nullptr,
                      int64_t ws_bytes = 0) {
    a.stamps = g_x3_stamps;
    a.st_kind = g_x3_store;
    a.prio = g_x3_prio;
#ifdef HKP_AB_KNOBS
    a.a_wrap = g_x3_a_wrap;
#endif
    a.stagger_ticks = g_x3_stagger_ns / 10;
    a.stagger_blocks = x3_cus();
    const bool sk_ok = ws && ws_bytes >= x3_sk_ws_bytes(256);
    const int nks = a.RS * a.cch;
    const X3Choice c = x3_choose(k, m_tiles, nks, sk_ok, policy, x3_halo_level(x3_halo_ok(a, k), a.cch, P), P);
    a.n_tiles = k / c.bn;
    a.nks = nks;
    a.sk_units = 0;
    if (c.duo) {
        // first-round stagger of the second block on each CU: half a block's
        // lifetime, ~(fill + epilogue + K loop) / 2 — hkp_debug_duo_stagger overrides
        // (ns; 0 = off, < 0 = this estimate)
        const long blocks = m_tiles * a.n_tiles;
        const int ns = g_duo_stagger_ns < 0 ? 5500 + 450 * 2 * nks : g_duo_stagger_ns;
        a.stagger_ticks = blocks > 2L * x3_cus() ? ns / 10 : 0;
        a.stagger_blocks = 2 * x3_cus();
        hipLaunchKernelGGL(conv_x3_duo_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, st, a);
        return;
    }
    if (c.halo) {
        const dim3 gh((unsigned)(m_tiles * a.n_tiles));
        if (a.in_ss) {
            if (P == 3) hipLaunchKernelGGL(conv_x3_halo_bnin_kernel<3>, gh, dim3(512), 0, st, a);
            else hipLaunchKernelGGL(conv_x3_halo_bnin_kernel<1>, gh, dim3(512), 0, st, a);
        } else {
            x3_dispatch_p(P, [&](auto pc) { hipLaunchKernelGGL(conv_x3_halo_kernel<pc.value>, gh, dim3(512), 0, st, a); });
        }
        return;
    }
    if (c.bm != 256) {                     // one tile per block, no split-K tail
        const long mt = ((long)a.M + c.bm - 1) / c.bm;
        const dim3 gm((unsigned)(mt * a.n_tiles));
        x3_dispatch_p(P, [&](auto pc) {
            if constexpr (x3_packed(pc.value)) {
                if (c.bm == 192) hipLaunchKernelGGL(conv_x3_a3_192_kernel<pc.value>, gm, dim3(512), 0, st, a);
                else if (c.bn == 128) hipLaunchKernelGGL(conv_x3_a3_160x128_kernel<pc.value>, gm, dim3(512), 0, st, a);
                else hipLaunchKernelGGL(conv_x3_a3_160_kernel<pc.value>, gm, dim3(512), 0, st, a);
            }
        });
        return;
    }
    dim3 grid((unsigned)(m_tiles * a.n_tiles));
    if (c.sk) {
        a.sk_units = m_tiles * a.nks;
        a.sk_cnt = (unsigned*)ws;
        a.sk_ws = (float*)((char*)ws + X3_SK_CNT_BYTES);
        // at least one unit per group: an empty group range inside a tile's group
        // span would be counted as a segment that never arrives
        const long ng = std::min<long>(x3_cus() / a.n_tiles, a.sk_units);
        grid = dim3((unsigned)(ng * a.n_tiles));
    }
    // split-K tail for the 256x256 one-tile grid (auto, or forced by HKP_TILE_256_TAIL)
    const long tiles = m_tiles * a.n_tiles;
    const long G = x3_cus();
    const long rm = tiles / G * G / a.n_tiles;              // m-tiles of the full rounds
    const long tm = m_tiles - rm;
    long NG = (!c.sk && c.bn == 256 && sk_ok &&
               (policy == HKP_TILE_AUTO || policy == HKP_TILE_256_TAIL || policy == HKP_TILE_256_A3 ||
                policy == HKP_TILE_AUTO_A3))
                  ? x3_tail_groups(m_tiles, a.n_tiles, nks)
                  : 0;
    // one round, every group non-empty and inside one tile (NG = tm * S), one slab
    // per block and the counters in the workspace
    if (NG > 0 && !(tm > 0 && NG % tm == 0 && NG * a.n_tiles <= G && tm * nks >= NG &&
                    NG * a.n_tiles * 256L * 1024 + X3_SK_CNT_BYTES <= ws_bytes && tm * a.n_tiles * 4 <= X3_SK_CNT_BYTES))
        NG = 0;
    const bool tail = NG > 0;
    a.sk_one = tail;
    // one launch: the full rounds, then the tail's segments
    if (tail && c.a3 && !g_x3_split_tail) {
        X3Args t = a;
        t.main_blocks = (int)(rm * a.n_tiles);
        t.tail_groups = (int)NG;
        t.tail_mt0 = (int)rm;
        t.tail_units = tm * nks;
        t.sk_cnt = (unsigned*)ws;
        t.sk_ws = (float*)((char*)ws + X3_SK_CNT_BYTES);
        const dim3 g1((unsigned)((rm + NG) * a.n_tiles));
        x3_dispatch_p(P, [&](auto pc) { launch_a3<pc.value>(g1, st, t); });
        return;
    }
    if (tail) {
        if (rm > 0) {
            dim3 g0((unsigned)(rm * a.n_tiles));
            x3_dispatch_p(P, [&](auto pc) { launch_x3_p<pc.value>(c, g0, st, a); });     // (A3 body, A/B only)
        }
        X3Args t = a;
        t.mt0 = (int)rm;
        t.sk_units = tm * nks;
        t.sk_cnt = (unsigned*)ws;
        t.sk_ws = (float*)((char*)ws + X3_SK_CNT_BYTES);
        const dim3 gt((unsigned)(NG * a.n_tiles));
        x3_dispatch_p(P, [&](auto pc) { hipLaunchKernelGGL((conv_x3_tail_kernel<256, pc.value>), gt, dim3(512), 0, st, t); });
        return;
    }
    x3_dispatch_p(P, [&](auto pc) { launch_x3_p<pc.value>(c, grid, st, a); });
}

}  // namespace hkp

using namespace hkp;

extern "C" int hkp_weight_pack_x3(int32_t k, int32_t rsc, int32_t c, const float* w, uint16_t* w_split,
                                  float* w_inv_scale, hkp_stream_t stream) {
    HKP_CHECK_ARG(k > 0 && c > 0 && c % 32 == 0 && rsc > 0 && rsc % c == 0 && w && w_split && w_inv_scale,
                  "hkp_weight_pack_x3: bad args");
    hipLaunchKernelGGL(weight_pack_x3_kernel, dim3(k), dim3(256), 0, as_stream(stream), rsc, w, (_Float16*)w_split,
                       w_inv_scale);
    HKP_LAUNCH_CHECK("hkp_weight_pack_x3");
    return HKP_OK;
}

extern "C" int hkp_weight_pack_f16(int32_t k, int32_t rsc, const float* w, uint16_t* w_f16, float* w_inv_scale,
                                   hkp_stream_t stream) {
    HKP_CHECK_ARG(k > 0 && rsc > 0 && w && w_f16 && w_inv_scale, "hkp_weight_pack_f16: bad args");
    hipLaunchKernelGGL(weight_pack_f16_kernel, dim3(k), dim3(256), 0, as_stream(stream), rsc, w, (_Float16*)w_f16,
                       w_inv_scale);
    HKP_LAUNCH_CHECK("hkp_weight_pack_f16");
    return HKP_OK;
}

extern "C" int64_t hkp_conv_x3_sk_workspace_bytes(void) { return x3_sk_ws_bytes(256); }

// the kernels address operands with 32-bit element offsets (see conv_x3_tile):
// the input ([n][h][w][cstride] halves, plus a padded-out margin of up to 64
// rows) and the weights ([k][rs][cstride]) must fit
static bool x3_offsets_fit(long n, long h, long w, long cstride, long k, long rs) {
    return (n * h * w + 64 * (w + 65)) * cstride < (1L << 32) && k * rs * cstride < (1L << 31);
}

static int check_tile(const hkp_conv_desc* d, const char* who) {
    HKP_CHECK_ARG(d->tile >= HKP_TILE_AUTO && d->tile <= HKP_TILE_160_A3, "%s: unknown tile policy %d", who,
                  d->tile);
    HKP_CHECK_ARG(d->tile != HKP_TILE_RESERVED_7 && d->tile != HKP_TILE_RESERVED_8 && d->tile != HKP_TILE_RESERVED_14,
                  "%s: tile policy %d is retired (a persistent conv body, measured slower)", who, d->tile);
    return HKP_OK;
}

// forward launch shared by the f16x3 (P 3) and plain-fp16 (P 1) entry points
static int conv_fwd_x3_common(const hkp_conv_desc* d, const uint16_t* xs, const uint16_t* ws, const float* wsc,
                              float* y, uint16_t* y16, float* part, void* sk_ws, int64_t sk_bytes, int P,
                              hkp_stream_t stream, const char* who, const X3Args* ep = nullptr) {
    int ho, wo;
    int rc = hkp_conv_out_hw(d, &ho, &wo);
    if (rc) return rc;
    rc = check_tile(d, who);
    if (rc) return rc;
    HKP_CHECK_ARG(xs && ws && (x3_packed(P) ? y != nullptr && y16 == nullptr : y == nullptr && y16 != nullptr),
                  "%s: null tensor (the packed split writes fp32 y, P 1 fp16 y)", who);
    HKP_CHECK_ARG(d->in_layout == HKP_LAYOUT_NHWC, "%s: NHWC only", who);
    const int cg = x3_packed(P) ? 32 : 64;
    HKP_CHECK_ARG(d->c % cg == 0 && d->k % 64 == 0, "%s: need Cin%%%d==0, Cout%%64==0 (c=%d k=%d)", who, cg, d->c,
                  d->k);
    const long M = (long)d->n * ho * wo;
    HKP_CHECK_ARG(M < (1L << 31) && x3_offsets_fit(d->n, d->h, d->w, d->c / cg * 64, d->k, d->r * d->s), "%s: too large",
                  who);
    X3Args a;
    a.xs = (const _Float16*)xs; a.ws = (const _Float16*)ws; a.wscale = wsc;
    a.y = y; a.y16 = (_Float16*)y16; a.part = part; a.amax = nullptr; a.add = nullptr; a.plane = 0;
    a.N = d->n; a.H = d->h; a.W = d->w; a.C = d->c; a.K = d->k; a.R = d->r; a.S = d->s;
    a.stride = d->stride; a.pad = d->pad; a.dil = d->dilation; a.Ho = ho; a.Wo = wo;
    a.M = (int)M; a.cch = d->c / cg; a.RS = d->r * d->s;
    int policy = d->tile;
    if (ep) {
        a.ep_ss = ep->ep_ss; a.ep_res = ep->ep_res; a.ep_rss = ep->ep_rss; a.ep_relu = ep->ep_relu;
        a.in_ss = ep->in_ss;
    }
    if (a.in_ss) {
        // the fused input BN runs where the unfused conv would run the halo-tile body,
        // so its output is the unfused path's, bit for bit
        HKP_CHECK_ARG(P == 3 || P == 1, "%s: fused input BN needs f16x3 or plain fp16", who);
        const bool sk_ok = sk_ws && sk_bytes >= x3_sk_ws_bytes(256);
        const X3Choice c = x3_choose(d->k, (M + 255) / 256, a.RS * a.cch, sk_ok, d->tile,
                                     x3_halo_level(x3_halo_ok(a, d->k), a.cch, P), P);
        HKP_CHECK_ARG(c.halo,
                      "%s: the fused input BN needs a launch on the halo-tile body (stride-1 3x3, pad = dil = 1, "
                      "Ho %% 8 == 0, Wo %% 32 == 0)", who);
    }
    launch_x3(d->k, (M + 255) / 256, policy, P, as_stream(stream), a, sk_ws, sk_bytes);
    HKP_LAUNCH_CHECK(who);
    return HKP_OK;
}

extern "C" int hkp_conv2d_fwd_x3(const hkp_conv_desc* d, const uint16_t* x_split, const uint16_t* w_split,
                                 const float* w_inv_scale, float* y, float* stat_partials, void* sk_workspace,
                                 int64_t sk_ws_bytes, hkp_stream_t stream) {
    HKP_CHECK_ARG(d && y, "hkp_conv2d_fwd_x3: null argument");
    return conv_fwd_x3_common(d, x_split, w_split, w_inv_scale, y, nullptr, stat_partials, sk_workspace, sk_ws_bytes,
                              3, stream, "hkp_conv2d_fwd_x3");
}

extern "C" int hkp_conv2d_fwd_x3_bnin(const hkp_conv_desc* d, const float* x_raw, const float* in_scale_shift,
                                      const uint16_t* w_split, const float* w_inv_scale, float* y, float* stat_partials,
                                      void* sk_workspace, int64_t sk_ws_bytes, hkp_stream_t stream) {
    HKP_CHECK_ARG(d && y && x_raw && in_scale_shift, "hkp_conv2d_fwd_x3_bnin: null argument");
    X3Args ep;
    ep.in_ss = in_scale_shift;
    return conv_fwd_x3_common(d, (const uint16_t*)x_raw, w_split, w_inv_scale, y, nullptr, stat_partials, sk_workspace,
                              sk_ws_bytes, 3, stream, "hkp_conv2d_fwd_x3_bnin", &ep);
}

extern "C" int hkp_conv2d_fwd_f16_bnin(const hkp_conv_desc* d, const uint16_t* x_raw_f16, const float* in_scale_shift,
                                       const uint16_t* w_f16, const float* w_inv_scale, uint16_t* y_f16,
                                       float* stat_partials, void* sk_workspace, int64_t sk_ws_bytes,
                                       hkp_stream_t stream) {
    HKP_CHECK_ARG(d && y_f16 && x_raw_f16 && in_scale_shift, "hkp_conv2d_fwd_f16_bnin: null argument");
    X3Args ep;
    ep.in_ss = in_scale_shift;
    return conv_fwd_x3_common(d, x_raw_f16, w_f16, w_inv_scale, nullptr, y_f16, stat_partials, sk_workspace,
                              sk_ws_bytes, 1, stream, "hkp_conv2d_fwd_f16_bnin", &ep);
}

extern "C" int hkp_conv2d_fwd_x3_products(const hkp_conv_desc* d, const uint16_t* x_split, const uint16_t* w_split,
                                          const float* w_inv_scale, int32_t products, float* y, float* stat_partials,
                                          void* sk_workspace, int64_t sk_ws_bytes, hkp_stream_t stream) {
    HKP_CHECK_ARG(d && y, "hkp_conv2d_fwd_x3_products: null argument");
    HKP_CHECK_ARG(products == HKP_X3_ALL || products == HKP_X3_W16 || products == HKP_X3_X16,
                  "hkp_conv2d_fwd_x3_products: unknown product set %d", products);
    const int P = products == HKP_X3_ALL ? 3 : products == HKP_X3_W16 ? 2 : 4;
    return conv_fwd_x3_common(d, x_split, w_split, w_inv_scale, y, nullptr, stat_partials, sk_workspace, sk_ws_bytes,
                              P, stream, "hkp_conv2d_fwd_x3_products");
}

extern "C" int hkp_conv2d_fwd_f16(const hkp_conv_desc* d, const uint16_t* x_f16, const uint16_t* w_f16,
                                  const float* w_inv_scale, uint16_t* y_f16, float* stat_partials,
                                  void* sk_workspace, int64_t sk_ws_bytes, hkp_stream_t stream) {
    HKP_CHECK_ARG(d && y_f16, "hkp_conv2d_fwd_f16: null argument");
    return conv_fwd_x3_common(d, x_f16, w_f16, w_inv_scale, nullptr, y_f16, stat_partials, sk_workspace, sk_ws_bytes,
                              1, stream, "hkp_conv2d_fwd_f16");
}

extern "C" int hkp_conv2d_fwd_f16_bn(const hkp_conv_desc* d, const uint16_t* x_f16, const uint16_t* w_f16,
                                     const float* w_inv_scale, const float* scale_shift, const uint16_t* res_f16,
                                     const float* res_scale_shift, int32_t relu, uint16_t* out_f16,
                                     void* sk_workspace, int64_t sk_ws_bytes, hkp_stream_t stream) {
    HKP_CHECK_ARG(d && out_f16 && scale_shift, "hkp_conv2d_fwd_f16_bn: null argument");
    HKP_CHECK_ARG(!res_scale_shift || res_f16, "hkp_conv2d_fwd_f16_bn: res_scale_shift needs a residual");
    X3Args ep;
    ep.ep_ss = scale_shift;
    ep.ep_res = (const _Float16*)res_f16;
    ep.ep_rss = res_scale_shift;
    ep.ep_relu = relu ? 1 : 0;
    return conv_fwd_x3_common(d, x_f16, w_f16, w_inv_scale, nullptr, out_f16, nullptr, sk_workspace, sk_ws_bytes, 1,
                              stream, "hkp_conv2d_fwd_f16_bn", &ep);
}

extern "C" int hkp_split_pack_x3(int64_t n, int32_t c, const float* x, const uint32_t* amax_bits,
                                 uint16_t* x_split, hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && c > 0 && c % 32 == 0 && n % c == 0 && x && x_split, "hkp_split_pack_x3: bad args");
    long g = (n / 4 + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(split_pack_x3_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), (long)(n / 4),
                       (const f32x4*)x, (const unsigned*)amax_bits, (_Float16*)x_split);
    HKP_LAUNCH_CHECK("hkp_split_pack_x3");
    return HKP_OK;
}

extern "C" int hkp_weight_flip_pack_x3(const hkp_conv_desc* d, const float* w, uint16_t* wf_split,
                                       float* wf_inv_scale, hkp_stream_t stream) {
    HKP_CHECK_ARG(d && w && wf_split && wf_inv_scale, "hkp_weight_flip_pack_x3: null argument");
    HKP_CHECK_ARG(d->k % 32 == 0, "hkp_weight_flip_pack_x3: need Cout%%32==0 (k=%d)", d->k);
    hipLaunchKernelGGL(weight_flip_pack_x3_kernel, dim3(d->c), dim3(256), 0, as_stream(stream), d->k, d->r, d->s,
                       d->c, w, (_Float16*)wf_split, wf_inv_scale);
    HKP_LAUNCH_CHECK("hkp_weight_flip_pack_x3");
    return HKP_OK;
}

extern "C" int hkp_conv2d_bwd_data_x3(const hkp_conv_desc* d, const uint16_t* dy_split, const uint16_t* wf_split,
                                      const float* wf_inv_scale, const uint32_t* dy_amax_bits, const float* add,
                                      float* dx, void* sk_workspace, int64_t sk_ws_bytes, hkp_stream_t stream) {
    int ho, wo;
    int rc = hkp_conv_out_hw(d, &ho, &wo);
    if (rc) return rc;
    HKP_CHECK_ARG(dy_split && wf_split && dx, "hkp_conv2d_bwd_data_x3: null tensor");
    HKP_CHECK_ARG(d->in_layout == HKP_LAYOUT_NHWC && d->stride == 1,
                  "hkp_conv2d_bwd_data_x3: stride-1 NHWC convs only (strided ones use hkp_conv2d_bwd_data)");
    HKP_CHECK_ARG(d->c % 64 == 0 && d->k % 32 == 0, "hkp_conv2d_bwd_data_x3: need Cin%%64==0, Cout%%32==0");
    const int padp = d->dilation * (d->r - 1) - d->pad;
    HKP_CHECK_ARG(padp >= 0 && d->dilation * (d->s - 1) - d->pad == padp, "hkp_conv2d_bwd_data_x3: padding");
    const long M = (long)d->n * d->h * d->w;
    HKP_CHECK_ARG(M < (1L << 31) && x3_offsets_fit(d->n, ho, wo, d->k / 32 * 64, d->c, d->r * d->s),
                  "hkp_conv2d_bwd_data_x3: too large");
    X3Args a;
    a.xs = (const _Float16*)dy_split; a.ws = (const _Float16*)wf_split; a.wscale = wf_inv_scale;
    a.y = dx; a.part = nullptr; a.amax = (const unsigned*)dy_amax_bits; a.add = add; a.plane = 0;
    a.N = d->n; a.H = ho; a.W = wo; a.C = d->k; a.K = d->c; a.R = d->r; a.S = d->s;
    a.stride = 1; a.pad = padp; a.dil = d->dilation; a.Ho = d->h; a.Wo = d->w;
    a.M = (int)M; a.cch = d->k / 32; a.RS = d->r * d->s;
    launch_x3(d->c, (M + 255) / 256, d->tile, 3, as_stream(stream), a, sk_workspace, sk_ws_bytes);
    HKP_LAUNCH_CHECK("hkp_conv2d_bwd_data_x3");
    return HKP_OK;
}

// Strided dgrad as stride-1 convs, one per output phase (py, px) of dx: dx pixel
// (2a+py, 2b+px) receives the taps r = r_max - 2r' (r ≡ py + pad mod 2) at dy row
// a + o_min + r', o_min = (py + pad - r_max) / 2 (likewise for columns); a phase
// no tap reaches (e.g. odd pixels of a 1x1 stride-2 conv) is dx = add (or 0).
static int phase_taps(int R, int pad, int stride, int ph, int* r_max, int* o_min) {
    int rm = -1;
    for (int r = R - 1; r >= 0; --r)
        if ((((ph + pad - r) % stride) + stride) % stride == 0) {
            rm = r;
            break;
        }
    if (rm < 0) return 0;
    *r_max = rm;
    *o_min = (ph + pad - rm) / stride;
    return rm / stride + 1;
}

__global__ __launch_bounds__(256) void phase_fill_kernel(long total, int C4, int Ha, int Wa, int OH, int OW, int ost,
                                                        int oy, int ox, const f32x4* __restrict__ add,
                                                        f32x4* __restrict__ dx) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int c4 = (int)(i % C4);
        long p = i / C4;
        const int b = (int)(p % Wa);
        p /= Wa;
        const int a = (int)(p % Ha);
        const long n = p / Ha;
        const long off = ((n * OH + (long)a * ost + oy) * OW + (long)b * ost + ox) * C4 + c4;
        dx[off] = add ? add[off] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
}

extern "C" int hkp_phase_taps(int32_t r, int32_t pad, int32_t stride, int32_t phase) {
    int rm, om;
    if (r <= 0 || stride <= 0 || phase < 0 || phase >= stride) return -1;
    return phase_taps(r, pad, stride, phase, &rm, &om);
}

extern "C" int hkp_conv2d_bwd_data_x3_strided(const hkp_conv_desc* d, const uint16_t* dy_split,
                                              const uint16_t* const* phase_split, const float* const* phase_inv_scale,
                                              const uint32_t* dy_amax_bits, const float* add, float* dx,
                                              void* sk_workspace, int64_t sk_ws_bytes, hkp_stream_t stream) {
    int ho, wo;
    int rc = hkp_conv_out_hw(d, &ho, &wo);
    if (rc) return rc;
    HKP_CHECK_ARG(dy_split && phase_split && phase_inv_scale && dx, "hkp_conv2d_bwd_data_x3_strided: null tensor");
    HKP_CHECK_ARG(d->in_layout == HKP_LAYOUT_NHWC && d->stride == 2 && d->dilation == 1,
                  "hkp_conv2d_bwd_data_x3_strided: stride-2, dilation-1 NHWC convs only");
    HKP_CHECK_ARG(d->c % 64 == 0 && d->k % 32 == 0, "hkp_conv2d_bwd_data_x3_strided: need Cin%%64==0, Cout%%32==0");
    HKP_CHECK_ARG((long)d->n * d->h * d->w < (1L << 31) && x3_offsets_fit(d->n, ho, wo, d->k / 32 * 64, d->c,
                                                                         d->r * d->s),
                  "hkp_conv2d_bwd_data_x3_strided: too large");
    hipStream_t st = as_stream(stream);
    for (int py = 0; py < 2; ++py)
        for (int px = 0; px < 2; ++px) {
            const int ph = py * 2 + px;
            const int Ha = (d->h - py + 1) / 2, Wa = (d->w - px + 1) / 2;
            if (Ha <= 0 || Wa <= 0) continue;
            int rmx = 0, omy = 0, smx = 0, omx = 0;
            const int R2 = phase_taps(d->r, d->pad, 2, py, &rmx, &omy);
            const int S2 = phase_taps(d->s, d->pad, 2, px, &smx, &omx);
            if (R2 == 0 || S2 == 0) {
                HKP_CHECK_ARG(phase_split[ph] == nullptr, "hkp_conv2d_bwd_data_x3_strided: phase %d has no taps", ph);
                const long total = (long)d->n * Ha * Wa * (d->c / 4);
                long g = (total + 255) / 256;
                if (g > 8192) g = 8192;
                hipLaunchKernelGGL(phase_fill_kernel, dim3((unsigned)g), dim3(256), 0, st, total, d->c / 4, Ha, Wa,
                                   d->h, d->w, 2, py, px, (const f32x4*)add, (f32x4*)dx);
                HKP_LAUNCH_CHECK("hkp_conv2d_bwd_data_x3_strided(fill)");
                continue;
            }
            HKP_CHECK_ARG(phase_split[ph] && phase_inv_scale[ph], "hkp_conv2d_bwd_data_x3_strided: phase %d weights",
                          ph);
            X3Args a;
            a.xs = (const _Float16*)dy_split; a.ws = (const _Float16*)phase_split[ph]; a.wscale = phase_inv_scale[ph];
            a.y = dx; a.part = nullptr; a.amax = (const unsigned*)dy_amax_bits; a.add = add; a.plane = 0;
            a.N = d->n; a.H = ho; a.W = wo; a.C = d->k; a.K = d->c; a.R = R2; a.S = S2;
            a.stride = 1; a.pad = -omy; a.dil = 1; a.Ho = Ha; a.Wo = Wa;
            a.M = d->n * Ha * Wa; a.cch = d->k / 32; a.RS = R2 * S2;
            a.ost = 2; a.OH = d->h; a.OW = d->w; a.oy = py; a.ox = px;
            // the column offset: the kernel applies one pad to both axes
            HKP_CHECK_ARG(omx == omy, "hkp_conv2d_bwd_data_x3_strided: row/column phase offsets differ (%d, %d)",
                          omy, omx);
            launch_x3(d->c, ((long)a.M + 255) / 256, d->tile, 3, st, a, sk_workspace, sk_ws_bytes);
            HKP_LAUNCH_CHECK("hkp_conv2d_bwd_data_x3_strided");
        }
    return HKP_OK;
}

extern "C" int64_t hkp_conv_bwd_filter_x3_workspace(const hkp_conv_desc* d) {
    int ho, wo;
    if (hkp_conv_out_hw(d, &ho, &wo) != HKP_OK) return -1;
    int sp, mps, ka, rt;
    wg_x3_plan(d, (long)d->n * ho * wo, wo, &sp, &mps, &ka, &rt);
    return (int64_t)sp * d->k * d->r * d->s * d->c * (int64_t)sizeof(float);
}

extern "C" int hkp_conv2d_bwd_filter_x3(const hkp_conv_desc* d, const uint16_t* x_split, const uint16_t* dy_split,
                                        const uint32_t* dy_amax_bits, float* dw, void* workspace, int64_t ws_bytes,
                                        hkp_stream_t stream) {
    int ho, wo;
    int rc = hkp_conv_out_hw(d, &ho, &wo);
    if (rc) return rc;
    HKP_CHECK_ARG(x_split && dy_split && dw && workspace, "hkp_conv2d_bwd_filter_x3: null tensor");
    HKP_CHECK_ARG(d->in_layout == HKP_LAYOUT_NHWC, "hkp_conv2d_bwd_filter_x3: NHWC convs only");
    HKP_CHECK_ARG(d->k % 64 == 0 && d->c % 32 == 0, "hkp_conv2d_bwd_filter_x3: need Cout%%64==0, Cin%%32==0");
    const long M = (long)d->n * ho * wo;
    HKP_CHECK_ARG(M < (1L << 31), "hkp_conv2d_bwd_filter_x3: too large");
    int sp, mps, ka, rt;
    wg_x3_plan(d, M, wo, &sp, &mps, &ka, &rt);
    const long n = (long)d->k * d->r * d->s * d->c;
    HKP_CHECK_ARG(ws_bytes >= sp * n * (long)sizeof(float), "hkp_conv2d_bwd_filter_x3: workspace %ld < %ld",
                  (long)ws_bytes, sp * n * (long)sizeof(float));
    WgX3Args a;
    a.xs = (const _Float16*)x_split; a.dys = (const _Float16*)dy_split; a.amax = (const unsigned*)dy_amax_bits;
    a.ws = (float*)workspace;
    a.N = d->n; a.H = d->h; a.W = d->w; a.C = d->c; a.K = d->k; a.R = d->r; a.S = d->s;
    a.stride = d->stride; a.pad = d->pad; a.dil = d->dilation; a.Ho = ho; a.Wo = wo;
    a.M = (int)M; a.RSC = d->r * d->s * d->c; a.r_tiles = rt; a.mps = mps;
    a.tiles = (d->k / (ka ? ka : 64)) * rt;
    hipStream_t st = as_stream(stream);
    const unsigned grid = (unsigned)(a.tiles * sp);
    if (ka == 0) hipLaunchKernelGGL(wgrad_x3_halo_kernel, dim3(grid), dim3(512), 0, st, a);
    else if (ka == 256) hipLaunchKernelGGL(wgrad_x3_kernel<256>, dim3(grid), dim3(512), 0, st, a);
    else if (ka == 128) hipLaunchKernelGGL(wgrad_x3_kernel<128>, dim3(grid), dim3(512), 0, st, a);
    else hipLaunchKernelGGL(wgrad_x3_kernel<64>, dim3(grid), dim3(512), 0, st, a);
    HKP_LAUNCH_CHECK("hkp_conv2d_bwd_filter_x3");
    if (sp > 16) {
        long g = (n / 4 + 63) / 64;
        if (g > 4096) g = 4096;
        hipLaunchKernelGGL(wg_x3_reduce_kernel<4>, dim3((unsigned)g), dim3(256), 0, st, n / 4, sp,
                           (const f32x4*)workspace, (f32x4*)dw);
    } else {
        long g = (n / 4 + 255) / 256;
        if (g > 4096) g = 4096;
        hipLaunchKernelGGL(wg_x3_reduce_kernel<1>, dim3((unsigned)g), dim3(256), 0, st, n / 4, sp,
                           (const f32x4*)workspace, (f32x4*)dw);
    }
    HKP_LAUNCH_CHECK("hkp_conv2d_bwd_filter_x3 (reduce)");
    return HKP_OK;
}

extern "C" int64_t hkp_stem_pack_x3_elems(const hkp_conv_desc* d) {
    int ho, wo;
    if (!stem_x3_shape(d) || hkp_conv_out_hw(d, &ho, &wo) != HKP_OK) return -1;
    return 2L * d->n * (2L * ho + 6) * (2L * wo + 6) * 4;
}

static int stem_pack(const hkp_conv_desc* d, const void* src, bool u8, uint16_t* x_split, hkp_stream_t stream,
                     const char* who) {
    int ho, wo;
    int rc = hkp_conv_out_hw(d, &ho, &wo);
    if (rc) return rc;
    HKP_CHECK_ARG(stem_x3_shape(d), "%s: needs the 7x7/s2/p3 NCHW stem with C<=4, Cout%%64==0", who);
    HKP_CHECK_ARG(src && x_split, "%s: null tensor", who);
    const int hp = 2 * ho + 6, wp = 2 * wo + 6;
    long g = ((long)d->n * hp * wp + 255) / 256;
    if (g > 8192) g = 8192;
    if (u8)
        hipLaunchKernelGGL(stem_pack_x3_kernel<true>, dim3((unsigned)g), dim3(256), 0, as_stream(stream), d->n, d->c,
                           d->h, d->w, hp, wp, src, (_Float16*)x_split);
    else
        hipLaunchKernelGGL(stem_pack_x3_kernel<false>, dim3((unsigned)g), dim3(256), 0, as_stream(stream), d->n, d->c,
                           d->h, d->w, hp, wp, src, (_Float16*)x_split);
    HKP_LAUNCH_CHECK(who);
    return HKP_OK;
}

extern "C" int hkp_stem_pack_x3(const hkp_conv_desc* d, const float* x_nchw, uint16_t* x_split, hkp_stream_t stream) {
    return stem_pack(d, x_nchw, false, x_split, stream, "hkp_stem_pack_x3");
}

extern "C" int hkp_stem_pack_x3_u8(const hkp_conv_desc* d, const uint8_t* img_nhwc, uint16_t* x_split,
                                   hkp_stream_t stream) {
    return stem_pack(d, img_nhwc, true, x_split, stream, "hkp_stem_pack_x3_u8");
}

extern "C" int hkp_stem_weight_pack_x3(int32_t k, int32_t c, const float* w_oihw, uint16_t* w_split,
                                       float* w_inv_scale, hkp_stream_t stream) {
    HKP_CHECK_ARG(k > 0 && c >= 1 && c <= 4 && w_oihw && w_split && w_inv_scale, "hkp_stem_weight_pack_x3: bad args");
    hipLaunchKernelGGL(stem_weight_pack_x3_kernel, dim3(k), dim3(256), 0, as_stream(stream), c, w_oihw,
                       (_Float16*)w_split, w_inv_scale);
    HKP_LAUNCH_CHECK("hkp_stem_weight_pack_x3");
    return HKP_OK;
}

extern "C" int hkp_conv2d_fwd_stem_x3(const hkp_conv_desc* d, const uint16_t* x_split, const uint16_t* w_split,
                                      const float* w_inv_scale, float* y, float* stat_partials, hkp_stream_t stream) {
    int ho, wo;
    int rc = hkp_conv_out_hw(d, &ho, &wo);
    if (rc) return rc;
    HKP_CHECK_ARG(stem_x3_shape(d), "hkp_conv2d_fwd_stem_x3: needs the 7x7/s2/p3 NCHW stem with C<=4, Cout%%64==0");
    HKP_CHECK_ARG(x_split && w_split && y, "hkp_conv2d_fwd_stem_x3: null tensor");
    const long M = (long)d->n * ho * wo;
    HKP_CHECK_ARG(M < (1L << 31) && x3_offsets_fit(d->n, 2L * ho + 6, 2L * wo + 6, 8, d->k, 7),
                  "hkp_conv2d_fwd_stem_x3: too large");
    X3Args a;
    a.xs = (const _Float16*)x_split; a.ws = (const _Float16*)w_split; a.wscale = w_inv_scale;
    a.y = y; a.part = stat_partials; a.amax = nullptr; a.add = nullptr;
    a.N = d->n; a.H = 2 * ho + 6; a.W = 2 * wo + 6; a.C = 4; a.K = d->k; a.R = 7; a.S = 1;
    a.stride = 2; a.pad = 0; a.dil = 1; a.Ho = ho; a.Wo = wo;
    a.M = (int)M; a.cch = 1; a.RS = 7; a.nks = 7;
    a.plane = (long)d->n * a.H * a.W * 4;
    a.n_tiles = d->k / 64;
    a.stamps = g_x3_stamps;
    a.st_kind = g_x3_store;
    const long m_tiles = (M + 255) / 256;
    if (stem_patch_shape(ho, wo, d->k) && d->tile != HKP_TILE_64_PAIR) {
        // the patch body (patch-divisible outputs: 480x640 and 960x1280 images);
        // HKP_TILE_64_PAIR keeps the one-tile stem (A/B, parity tests)
        hipLaunchKernelGGL(conv_x3_stem_patch_kernel<0>, dim3(m_tiles * a.n_tiles), dim3(512), 0, as_stream(stream), a);
        HKP_LAUNCH_CHECK("hkp_conv2d_fwd_stem_x3");
        return HKP_OK;
    }
    // two blocks per CU (7 K-steps per tile: prologue / epilogue dominate one
    // block), 16x16x32 body on a 2-stage ring (the layer1 256x64 pair's body)
    hipLaunchKernelGGL((conv_x3_kernel<64, true, true, 16, false, 3>), dim3(m_tiles * a.n_tiles), dim3(512), 0,
                       as_stream(stream), a);
    HKP_LAUNCH_CHECK("hkp_conv2d_fwd_stem_x3");
    return HKP_OK;
}

// the stem straight from the image (conv_x3_stem_patch_kernel<1 | 2>): no packed
// planes, where the patch body takes the shape (hkp_stem_x3_image_ok)
extern "C" int32_t hkp_stem_x3_image_ok(const hkp_conv_desc* d) {
    int ho, wo;
    if (!stem_x3_shape(d) || hkp_conv_out_hw(d, &ho, &wo) != HKP_OK) return 0;
    return stem_patch_shape(ho, wo, d->k) && d->tile != HKP_TILE_64_PAIR && (long)d->n * ho * wo < (1L << 31) ? 1 : 0;
}

extern "C" int hkp_conv2d_fwd_stem_x3_image(const hkp_conv_desc* d, const void* image, int32_t image_u8,
                                            const uint16_t* w_split, const float* w_inv_scale, float* y,
                                            float* stat_partials, hkp_stream_t stream) {
    HKP_CHECK_ARG(hkp_stem_x3_image_ok(d), "hkp_conv2d_fwd_stem_x3_image: shape not on the patch body "
                                           "(hkp_stem_x3_image_ok; use hkp_stem_pack_x3 + hkp_conv2d_fwd_stem_x3)");
    HKP_CHECK_ARG(image && w_split && y, "hkp_conv2d_fwd_stem_x3_image: null tensor");
    int ho, wo;
    hkp_conv_out_hw(d, &ho, &wo);
    X3Args a;
    a.xs = (const _Float16*)image; a.ws = (const _Float16*)w_split; a.wscale = w_inv_scale;
    a.y = y; a.part = stat_partials; a.amax = nullptr; a.add = nullptr;
    a.N = d->n; a.H = d->h; a.W = d->w; a.C = d->c; a.K = d->k; a.R = 7; a.S = 1;
    a.stride = 2; a.pad = 0; a.dil = 1; a.Ho = ho; a.Wo = wo;
    a.M = d->n * ho * wo; a.cch = 1; a.RS = 7; a.nks = 7; a.plane = 0;
    a.n_tiles = d->k / 64;
    a.stamps = g_x3_stamps;
    a.st_kind = g_x3_store;
    const dim3 grid((unsigned)(((long)a.M + 255) / 256 * a.n_tiles));
    if (image_u8) hipLaunchKernelGGL(conv_x3_stem_patch_kernel<2>, grid, dim3(512), 0, as_stream(stream), a);
    else hipLaunchKernelGGL(conv_x3_stem_patch_kernel<1>, grid, dim3(512), 0, as_stream(stream), a);
    HKP_LAUNCH_CHECK("hkp_conv2d_fwd_stem_x3_image");
    return HKP_OK;
}

// rows per BN statistic tile of a packed forward conv (see hulkkp.h)
extern "C" int32_t hkp_conv_x3_stat_tile_rows(const hkp_conv_desc* d, int32_t op) {
    HKP_CHECK_ARG(d, "hkp_conv_x3_stat_tile_rows: null descriptor");
    const bool packed = op == HKP_KOP_FWD_X3 || op == HKP_KOP_FWD_X3_W16 || op == HKP_KOP_FWD_X3_X16;
    if (packed && d->tile == HKP_TILE_192_A3 && d->k % 256 == 0) return 96;
    if (packed && d->tile == HKP_TILE_160_A3 && d->k % 128 == 0) return 80;
    return 128;
}

// the kernel symbol a launch with this descriptor runs (see hulkkp.h)
extern "C" int32_t hkp_conv_kernel_name(const hkp_conv_desc* d, int32_t op, int32_t stream_k_ok, char* buf,
                                        int32_t len) {
    HKP_CHECK_ARG(d && buf && len > 0, "hkp_conv_kernel_name: bad args");
    int ho, wo;
    int rc = hkp_conv_out_hw(d, &ho, &wo);
    if (rc) return rc;
    if (op != HKP_KOP_WGRAD_X3) {          // a wgrad's d->tile is its CU budget
        rc = check_tile(d, "hkp_conv_kernel_name");
        if (rc) return rc;
    }
    const bool sk = stream_k_ok != 0;
    switch (op) {
        case HKP_KOP_FWD_X3:
        case HKP_KOP_FWD_X3_W16:
        case HKP_KOP_FWD_X3_X16:
        case HKP_KOP_FWD_F16: {
            const int P = op == HKP_KOP_FWD_X3 ? 3 : op == HKP_KOP_FWD_X3_W16 ? 2 : op == HKP_KOP_FWD_X3_X16 ? 4 : 1;
            const long m = (long)d->n * ho * wo;
            const int cg = x3_packed(P) ? 32 : 64;
            const int nks = d->r * d->s * (d->c / cg);
            const bool halo = halo_shape(d->stride, d->r, d->s, d->pad, d->dilation, ho, wo, d->k) &&
                              (long)d->n * d->h * d->w * (d->c / cg * 64L) + 64 < (1L << 32);
            return x3_kernel_name(x3_choose(d->k, (m + 255) / 256, nks, sk, d->tile, x3_halo_level(halo, d->c / cg, P), P),
                                  false, P, buf, len);
        }
        case HKP_KOP_DGRAD_X3: {
            const long m = (long)d->n * d->h * d->w;
            const int nks = d->r * d->s * (d->k / 32);
            const int padp = d->dilation * (d->r - 1) - d->pad;
            const bool halo = halo_shape(d->stride, d->r, d->s, padp, d->dilation, d->h, d->w, d->c) &&
                              (long)d->n * ho * wo * (d->k / 32 * 64L) + 64 < (1L << 32);
            return x3_kernel_name(x3_choose(d->c, (m + 255) / 256, nks, sk, d->tile, x3_halo_level(halo, d->k / 32, 3), 3),
                                  false, 3, buf, len);
        }
        case HKP_KOP_STEM_X3:
            if (stem_patch_shape(ho, wo, d->k) && d->tile != HKP_TILE_64_PAIR)
                return snprintf(buf, len, "conv_x3_stem_patch_kernel<0>");
            return x3_kernel_name(X3_STEM, true, 3, buf, len);
        case HKP_KOP_STEM_X3_IMAGE:
        case HKP_KOP_STEM_X3_IMAGE_U8:
            HKP_CHECK_ARG(hkp_stem_x3_image_ok(d), "hkp_conv_kernel_name: the image stem needs the patch body's shape");
            return snprintf(buf, len, "conv_x3_stem_patch_kernel<%d>", op == HKP_KOP_STEM_X3_IMAGE ? 1 : 2);
        case HKP_KOP_WGRAD_X3: {
            HKP_CHECK_ARG(d->k % 64 == 0, "hkp_conv_kernel_name: wgrad needs Cout%%64==0");
            int sp, mps, ka, rt;
            wg_x3_plan(d, (long)d->n * ho * wo, wo, &sp, &mps, &ka, &rt);
            if (ka == 0) return snprintf(buf, len, "wgrad_x3_halo_kernel");
            return snprintf(buf, len, "wgrad_x3_kernel<%d>", ka);
        }
        default:
            HKP_CHECK_ARG(false, "hkp_conv_kernel_name: unknown op %d", op);
    }
    return HKP_ERR_BAD_ARG;
}

#ifdef HKP_AB_KNOBS   // the A/B instruments (tools/ab_lib build only; include/hulkkp_ab.h)
// Debug: forward conv launches record per-block phase clocks into buf (8 slots of
// s_memrealtime per block: start, pipeline filled, K loop done, BN partials
// done, fp16 tile staged, stores issued; 0 where a body records none); NULL
// turns it off.  Not thread-safe; for tools/ only.
extern "C" void hkp_debug_x3_stamps(uint64_t* buf) { g_x3_stamps = (unsigned long long*)buf; }

// Debug / tuning (tools/ only, not thread-safe): the first-round stagger of the
// one-tile forward conv launches, in ns (0 = off; X3Args::stagger_ticks).
extern "C" void hkp_debug_x3_stagger(int32_t ns) { g_x3_stagger_ns = ns > 0 ? ns : 0; }

// Debug / A/B (tools/ only, not thread-safe): nonzero runs an A3 grid's split-K
// tail as its own conv_x3_tail_kernel launch instead of inside the A3 launch.
extern "C" void hkp_debug_x3_split_tail(int32_t on) { g_x3_split_tail = on != 0; }
extern "C" void hkp_debug_stem_pair(int32_t on) { g_stem_pair = on != 0; }
extern "C" void hkp_debug_x3_pair128(int32_t on) { g_x3_pair128 = on != 0; }

// Debug / A/B (tools/ only, not thread-safe): the flavour of the forward convs'
// epilogue output stores (X3Args::st_kind: 0 each site's own, 1 plain, 2
// nontemporal, 3 sc1, 4 sc0 sc1).
extern "C" void hkp_debug_x3_store(int32_t kind) { g_x3_store = kind >= 0 && kind <= 4 ? kind : 0; }

// Debug / A/B (tools/ only, not thread-safe): the DUO body's first-round stagger of
// the second block on each CU, in ns (0 = off; < 0 = the planner's estimate).
extern "C" void hkp_debug_duo_stagger(int32_t ns) { g_duo_stagger_ns = ns; }

// Debug / A/B (tools/ only, not thread-safe): static wave priority in the A3 body's
// K loop (X3Args::prio: 0 none, 1 waves 4-7, 2 waves 0-3 at s_setprio 1).
extern "C" void hkp_debug_x3_prio(int32_t mode) { g_x3_prio = mode >= 0 && mode <= 2 ? mode : 0; }

// A/B probe (tools/ only, not thread-safe): the one-tile and DUO conv bodies read A row m
// from row m % rows (0 = off) — an L2-resident activation stream, wrong outputs
extern "C" void hkp_debug_x3_a_wrap(int32_t rows) { g_x3_a_wrap = rows > 0 ? rows : 0; }
#endif

