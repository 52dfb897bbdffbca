// Batched f16x3 weight packing: every conv weight of a network packed in two
// launches per optimizer step (the f16x3 conv operands of conv_x3.hip).
//
// One training step changes every parameter, so every conv needs its forward
// operand (hkp_weight_pack_x3: per output channel k) and, for the stride-1
// convs, its dgrad operand (hkp_weight_flip_pack_x3: the transposed, flipped
// filter, per forward INPUT channel c) repacked.  Packed one conv at a time that
// is ~70 launches of a few blocks each (R34) and a strided gather for the flip;
// here:
//   launch A  units: forward-pack rows (one block per k: load the RSC row into
//             registers, max, scale, store — one HBM read) and flip-max tiles
//             (64 channels x 8 k x all taps: per-channel column maxima over 8
//             filters into a workspace);
//   launch B  flip-pack tiles (8 channels x 1024 (tap, k) rows): per-channel max
//             over the workspace column partials → scale, then a transpose
//             through LDS so that both the fp32 reads (one 32-B sector per row)
//             and the packed 128-B [hi32|lo32] lines are written whole.
// Outputs are bit-identical to the per-conv kernels (same power-of-two scales,
// same split).  Kind 2 packs one output phase of a stride-2 conv's dgrad operand
// (hkp_conv2d_bwd_data_x3_strided): the flipped filter's taps of that phase, with
// the whole flipped filter's per-channel scales.  Jobs travel by value in the
// kernel arguments, 32 per launch.
#include "common.h"

namespace hkp {

constexpr int PK_MAXJ = 32;
constexpr int PK_FLIP_ROWS = 1024;  // (tap, k) rows per flip-pack tile (4 per thread)
constexpr int PK_KCHUNK = 8;        // filters per flip-max tile
constexpr int PK_RV = 5;            // float4 per thread held in registers (rows <= 5120)

struct PackJob {
    const float* w;
    _Float16* out;
    float* inv;
    float* part;   // flip: [k/8][c] column maxima
    int kind, k, rs, c;
    // flipped operands: row tap (r', s') of the output reads w tap
    // (rmx - tstep*r', smx - tstep*s'); R2 x S2 taps (kind 1: the whole filter,
    // tstep 1; kind 2: one output phase of a stride-2 conv, tstep 2)
    int S, R2, S2, rmx, smx, tstep;
};

struct PackTable {
    PackJob j[PK_MAXJ];
    int ubeg[PK_MAXJ + 1];   // first unit of each job in this launch's grid
    int n;
};

__device__ __forceinline__ float pk_scale(float m) {   // = conv_x3.hip pow2_scale_of
    if (!(m > 0.f) || !(m < INFINITY)) return 1.f;
    int e;
    frexpf(m, &e);
    e = 14 - e;
    e = e < -100 ? -100 : (e > 100 ? 100 : e);
    return ldexpf(1.f, e);
}

__device__ __forceinline__ float amax4(const f32x4& v) {
    return fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
}

__device__ __forceinline__ float block_max256(float m, float* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

__device__ __forceinline__ int find_job(const PackTable& t, int b) {
    int j = 0;
    while (j + 1 < t.n && b >= t.ubeg[j + 1]) ++j;
    return j;
}

// forward pack of row k: ws[k][tap][c/32][hi|lo] = split(w[k][tap][c] * 2^e_k)
__device__ void fwd_row(const PackJob& J, int k, float* red) {
    const int n4 = J.rs * J.c / 4;
    const f32x4* row = (const f32x4*)J.w + (long)k * n4;
    f32x4 v[PK_RV];
    float m = 0.f;
#pragma unroll
    for (int q = 0; q < PK_RV; ++q) {
        const int i = threadIdx.x + 256 * q;
        if (i < n4) {
            v[q] = row[i];
            m = fmaxf(m, amax4(v[q]));
        }
    }
    for (int i = threadIdx.x + 256 * PK_RV; i < n4; i += 256) m = fmaxf(m, amax4(row[i]));
    const float sc = pk_scale(block_max256(m, red));
    const long e0 = (long)k * n4;
#pragma unroll
    for (int q = 0; q < PK_RV; ++q) {
        const int i = threadIdx.x + 256 * q;
        if (i < n4) store_split4(v[q] * sc, e0 + i, J.out, 3);
    }
    for (int i = threadIdx.x + 256 * PK_RV; i < n4; i += 256) store_split4(row[i] * sc, e0 + i, J.out, 3);
    if (threadIdx.x == 0) J.inv[k] = 1.f / sc;
}

// flip-max tile u: channels [64*(u % (c/64)), +64) over filters [8*(u / (c/64)), +8)
__device__ void flip_max_tile(const PackJob& J, int u, float* red) {
    const int cg = J.c / 64, g = u % cg, q = u / cg;
    const int c4 = J.c / 4, cl = threadIdx.x & 15, rl = threadIdx.x >> 4;
    const f32x4* src = (const f32x4*)J.w + (long)q * PK_KCHUNK * J.rs * c4 + g * 16 + cl;
    f32x4 m = {0.f, 0.f, 0.f, 0.f};
    for (int r = rl; r < PK_KCHUNK * J.rs; r += 16) {
        const f32x4 v = src[(long)r * c4];
#pragma unroll
        for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], fabsf(v[e]));
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        m[e] = fmaxf(m[e], __shfl_xor(m[e], 16));
        m[e] = fmaxf(m[e], __shfl_xor(m[e], 32));
    }
    if ((threadIdx.x & 63) < 16) {
#pragma unroll
        for (int e = 0; e < 4; ++e) red[(threadIdx.x >> 6) * 64 + cl * 4 + e] = m[e];
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const int t = threadIdx.x;
        J.part[(long)q * J.c + g * 64 + t] = fmaxf(fmaxf(red[t], red[64 + t]), fmaxf(red[128 + t], red[192 + t]));
    }
}

__global__ __launch_bounds__(256) void weight_pack_a_kernel(const PackTable t) {
    __shared__ float red[256];
    const int jb = find_job(t, blockIdx.x);
    const PackJob& J = t.j[jb];
    const int u = blockIdx.x - t.ubeg[jb];
    if (J.kind == 0) fwd_row(J, u, red);
    else flip_max_tile(J, u, red);   // kinds 1 and 2: scale from the whole filter column
}

// flip-pack tile u: channels [8*(u % (c/8)), +8), rows [1024*(u / (c/8)), +1024) of
// the flipped [c][tap'][k] operand, tap' = rs-1-tap
__global__ __launch_bounds__(256) void weight_pack_b_kernel(const PackTable t) {
    __shared__ float tile[8][PK_FLIP_ROWS];
    __shared__ float red[4][8];
    __shared__ float scl[8];
    const int jb = find_job(t, blockIdx.x);
    const PackJob& J = t.j[jb];
    const int u = blockIdx.x - t.ubeg[jb];
    const int cg = J.c / 8, g = u % cg, p = u / cg, c0 = 8 * g;
    const int n = J.R2 * J.S2 * J.k, K = J.k, tid = threadIdx.x;
    // channel scales from the column partials of launch A
    {
        const int cc = tid & 7;
        float m = 0.f;
        for (int q = tid >> 3; q < K / PK_KCHUNK; q += 32) m = fmaxf(m, J.part[(long)q * J.c + c0 + cc]);
        m = fmaxf(m, __shfl_xor(m, 8));
        m = fmaxf(m, __shfl_xor(m, 16));
        m = fmaxf(m, __shfl_xor(m, 32));
        if ((tid & 63) < 8) red[tid >> 6][cc] = m;
        __syncthreads();
        if (tid < 8) {
            const float sc = pk_scale(fmaxf(fmaxf(red[0][tid], red[1][tid]), fmaxf(red[2][tid], red[3][tid])));
            scl[tid] = sc;
            if (p == 0) J.inv[c0 + tid] = 1.f / sc;
        }
    }
    // gather: row r = tap'*K + k reads w[k][src tap of tap'][c0..c0+8) (one 32-B sector)
    f32x4 a[4], b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int r = p * PK_FLIP_ROWS + tid + 256 * q;
        if (r < n) {
            const int tp = r / K, k = r - tp * K, rp = tp / J.S2, sp = tp - rp * J.S2;
            const int src = (J.rmx - J.tstep * rp) * J.S + (J.smx - J.tstep * sp);
            const f32x4* s = (const f32x4*)(J.w + ((long)k * J.rs + src) * J.c + c0);
            a[q] = s[0];
            b[q] = s[1];
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            tile[e][tid + 256 * q] = a[q][e];
            tile[4 + e][tid + 256 * q] = b[q][e];
        }
    }
    __syncthreads();
    // scatter: channel cc, 8 consecutive rows per thread → whole packed lines
    const int cc = tid >> 5;
    const float sc = scl[cc];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int r8 = (tid & 31) * 8 + 256 * q, rr = p * PK_FLIP_ROWS + r8;
        if (rr < n) {
            const long e4 = ((long)(c0 + cc) * n + rr) / 4;
            f32x4 v0, v1;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v0[e] = tile[cc][r8 + e] * sc;
                v1[e] = tile[cc][r8 + 4 + e] * sc;
            }
            store_split4(v0, e4, J.out, 3);
            store_split4(v1, e4 + 1, J.out, 3);
        }
    }
}

// taps of output phase ph of a stride-2 conv along an axis of R taps (conv_x3.hip)
static int pk_phase_taps(int R, int pad, int ph, int* r_max) {
    for (int r = R - 1; r >= 0; --r)
        if ((((ph + pad - r) % 2) + 2) % 2 == 0) {
            *r_max = r;
            return r / 2 + 1;
        }
    return 0;
}

static void flip_geometry(const hkp_pack_job& j, PackJob& d) {
    if (j.kind == 2) {
        d.S = j.s;
        d.R2 = pk_phase_taps(j.r, j.pad, j.phase >> 1, &d.rmx);
        d.S2 = pk_phase_taps(j.s, j.pad, j.phase & 1, &d.smx);
        d.tstep = 2;
    } else {   // whole flipped filter; rs taps as one axis
        d.S = 1; d.R2 = j.rs; d.S2 = 1; d.rmx = j.rs - 1; d.smx = 0; d.tstep = 1;
    }
}

static int units_a(const hkp_pack_job& j) { return j.kind == 0 ? j.k : (j.c / 64) * (j.k / PK_KCHUNK); }
static int units_b(const hkp_pack_job& j) {
    if (j.kind == 0) return 0;
    PackJob d;
    flip_geometry(j, d);
    return (j.c / 8) * cdiv((long)d.R2 * d.S2 * j.k, PK_FLIP_ROWS);
}
static long part_floats(const hkp_pack_job& j) { return j.kind == 0 ? 0 : (long)(j.k / PK_KCHUNK) * j.c; }

}  // namespace hkp

using namespace hkp;

extern "C" int64_t hkp_weight_pack_x3_batch_ws_bytes(int32_t njobs, const hkp_pack_job* jobs) {
    if (njobs < 0 || (njobs > 0 && !jobs)) return -1;
    long f = 0;
    for (int i = 0; i < njobs; ++i) f += part_floats(jobs[i]);
    return f * 4;
}

extern "C" int hkp_weight_pack_x3_batch(int32_t njobs, const hkp_pack_job* jobs, void* workspace, int64_t ws_bytes,
                                        hkp_stream_t stream) {
    HKP_CHECK_ARG(njobs >= 0 && (njobs == 0 || jobs), "hkp_weight_pack_x3_batch: bad job list");
    long need = 0;
    for (int i = 0; i < njobs; ++i) {
        const hkp_pack_job& j = jobs[i];
        HKP_CHECK_ARG(j.w && j.out && j.inv_scale && j.kind >= 0 && j.kind <= 2 && j.k > 0 && j.rs > 0 && j.c > 0,
                      "hkp_weight_pack_x3_batch: job %d: bad fields", i);
        if (j.kind == 2) {
            int rm;
            HKP_CHECK_ARG(j.r > 0 && j.s > 0 && j.r * j.s == j.rs && j.phase >= 0 && j.phase < 4 &&
                              pk_phase_taps(j.r, j.pad, j.phase >> 1, &rm) > 0 &&
                              pk_phase_taps(j.s, j.pad, j.phase & 1, &rm) > 0,
                          "hkp_weight_pack_x3_batch: job %d: phase %d of r=%d s=%d pad=%d has no taps", i, j.phase,
                          j.r, j.s, j.pad);
        }
        if (j.kind == 0)
            HKP_CHECK_ARG(j.c % 32 == 0, "hkp_weight_pack_x3_batch: job %d: forward pack needs c%%32==0 (c=%d)", i,
                          j.c);
        else
            HKP_CHECK_ARG(j.c % 64 == 0 && j.k % 32 == 0,
                          "hkp_weight_pack_x3_batch: job %d: flip/phase pack needs c%%64==0, k%%32==0 (c=%d k=%d)", i,
                          j.c, j.k);
        HKP_CHECK_ARG((long)j.k * j.rs * j.c < (1L << 31), "hkp_weight_pack_x3_batch: job %d too large", i);
        need += part_floats(j);
    }
    HKP_CHECK_ARG(need == 0 || (workspace && ws_bytes >= need * 4),
                  "hkp_weight_pack_x3_batch: workspace of %ld bytes needed", need * 4);
    hipStream_t st = as_stream(stream);
    for (int pass = 0; pass < 2; ++pass) {
        float* part = (float*)workspace;
        for (int j0 = 0; j0 < njobs; j0 += PK_MAXJ) {
            PackTable t;
            t.n = 0;
            int units = 0;
            float* part_here = part;
            for (int i = j0; i < njobs && i < j0 + PK_MAXJ; ++i) {
                const hkp_pack_job& s = jobs[i];
                const int u = pass == 0 ? units_a(s) : units_b(s);
                float* pj = part_here;
                part_here += part_floats(s);
                if (u == 0) continue;
                PackJob& d = t.j[t.n];
                d.w = s.w; d.out = (_Float16*)s.out; d.inv = s.inv_scale; d.part = pj;
                d.kind = s.kind; d.k = s.k; d.rs = s.rs; d.c = s.c;
                flip_geometry(s, d);
                t.ubeg[t.n++] = units;
                units += u;
            }
            for (int i = j0; i < njobs && i < j0 + PK_MAXJ; ++i) part += part_floats(jobs[i]);
            if (units == 0) continue;
            t.ubeg[t.n] = units;
            if (pass == 0) hipLaunchKernelGGL(weight_pack_a_kernel, dim3(units), dim3(256), 0, st, t);
            else hipLaunchKernelGGL(weight_pack_b_kernel, dim3(units), dim3(256), 0, st, t);
            HKP_LAUNCH_CHECK("hkp_weight_pack_x3_batch");
        }
    }
    return HKP_OK;
}
