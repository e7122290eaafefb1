// spmm.hip - CSR SpMM (DGL gspmm 'mul'/'sum') for gfx950.
//
// Replaces dgl.ops.gspmm(g, 'mul', 'sum', lhs, rhs) at model.py:106, 4184,
// 4196, 4037 and its reverse-graph backward:
//     y[r] = sum_{p in row r} rhs[eid(p)] * x[col[p]]          (fp32)
//
// Design:
//  * One feature row of x is D fp32 = D/4 float4; LPR = D/4 lanes cover it
//    with one 16-B load each, so a wave64 holds G = 64/LPR rows.
//  * Row tier: each LPR-lane group owns one output row.  Rows are visited in
//    degree-descending order (igr_plan_fill), so the G rows of a wave have
//    ~equal degree (no intra-wave imbalance) and the heaviest rows start
//    first (no tail).  A group loads LPR (col, val) pairs with one coalesced
//    load, broadcasts them with ds_bpermute, and keeps 8 row gathers in
//    flight; the next block of (col, val) is prefetched under the gathers.
//  * Chunk tier: rows longer than split_threshold are cut into fixed-size
//    chunks; one wave per chunk, each group taking its own LPR-edge slice of
//    every 64-edge block, then a cross-group xor reduction, and a partial row written to a workspace.
//    A second kernel sums each row's partials in chunk order.  No atomics:
//    results are bitwise reproducible run to run.
//  * Both tiers run in ONE launch (chunk blocks first, heaviest work first).
//  * The row epilogue fuses the LightGCN/IGCN layer mean and the backward's
//    "+ g/(L+1)" (igr_epilogue).
//  * CSR structure and edge values are plain loads (non-temporal loads and
//    stores measured 1-3 % slower / neutral on MI355X, scripts/tune_spmm.py).
#include <algorithm>
#include <mutex>

#include "common.h"

namespace igr {

struct Epi {
    float *y;
    int64_t ldy;
    float alpha, beta;
    const float *add;
    int64_t ld_add;
    float *acc;
    int64_t ld_acc;
    int acc_mode;
    float acc_div;
    int skip_y;
    const float *row_scale;
    const uint32_t *row_mask, *col_mask;
};

__device__ __forceinline__ bool bit_set(const uint32_t *__restrict__ m, int64_t i) {
    return (m[i >> 5] >> (i & 31)) & 1u;
}

#ifndef IGR_SPMM_NT_STORE
#define IGR_SPMM_NT_STORE 0
#endif

__device__ __forceinline__ void store_row4(const Epi &e, int64_t r, int f, float4 s) {
    float4 y = s;
    if (e.alpha != 1.f) y = f4_scale(e.alpha, y);
    if (e.add) {
        float4 a = *reinterpret_cast<const float4 *>(e.add + r * e.ld_add + f);
        y = f4_fma(e.beta, a, y);
    }
    if (e.row_scale) y = f4_scale(e.row_scale[r], y);
    if (!e.skip_y) {
        float4 *yp = reinterpret_cast<float4 *>(e.y + r * e.ldy + f);
#if IGR_SPMM_NT_STORE
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v yv = {y.x, y.y, y.z, y.w};
        __builtin_nontemporal_store(yv, reinterpret_cast<f4v *>(yp));
#else
        *yp = y;
#endif
    }
    if (e.acc_mode) {
        float4 *ap = reinterpret_cast<float4 *>(e.acc + r * e.ld_acc + f);
        float4 a = (e.acc_mode == 2) ? f4_add(*ap, y) : y;
        if (e.acc_div != 1.f) a = f4_div(a, e.acc_div);
        *ap = a;
    }
}

__device__ __forceinline__ void store_row1(const Epi &e, int64_t r, int f, float s) {
    float y = e.alpha * s;
    if (e.add) y = fmaf(e.beta, e.add[r * e.ld_add + f], y);
    if (e.row_scale) y *= e.row_scale[r];
    if (!e.skip_y) e.y[r * e.ldy + f] = y;
    if (e.acc_mode) {
        float a = (e.acc_mode == 2) ? e.acc[r * e.ld_acc + f] + y : y;
        e.acc[r * e.ld_acc + f] = a / e.acc_div;
    }
}

// Edge-weight policies (template argument W of the kernels): the weight of
// CSR position p of row r with source column c.
// drops(): the policy zeroes edges at run time (in-kernel dropout); the launch
// then takes the MASK variant, whose zero-weight edges skip their row gather.
struct W_One {  // rhs == NULL: unit weights
    bool drops() const { return false; }
    __device__ __forceinline__ float operator()(int64_t, int, int) const { return 1.f; }
};
struct W_Val {  // rhs by edge id == CSR position
    const float *val;
    bool drops() const { return false; }
    __device__ __forceinline__ float operator()(int64_t p, int, int) const { return ld_stream(val + p); }
};
struct W_ValEid {  // rhs by edge id, edge id = edge_id[p] (multigraph / reverse graph)
    const float *val;
    const int64_t *eid;
    bool drops() const { return false; }
    __device__ __forceinline__ float operator()(int64_t p, int, int) const { return val[ld_stream(eid + p)]; }
};
struct W_ValHead {  // per-head rhs [nnz, h] by edge id (CSR position or edge_id[p]), head j
    const float *val;
    const int64_t *eid;
    int64_t h, j;
    bool drops() const { return false; }
    __device__ __forceinline__ float operator()(int64_t p, int, int) const {
        return val[(eid ? ld_stream(eid + p) : p) * h + j];
    }
};
// Key of an edge for the dropout draw: its (row, column) in the frame the
// mask was drawn for (a coalesced graph has one edge per pair), so the reverse
// graph regenerates the forward's mask from its own (column, row) without
// reading an edge-id permutation.
__device__ __forceinline__ uint64_t edge_key(uint32_t r, uint32_t c) {
    return mix64(((uint64_t)r << 32) | c);
}

// Row / column scaled weights with fused dropout (igr_spmm_scaled_f32):
//   w = rs[r] * cs[c], then dropped (0) or divided by keep, the mask drawn from
//   uniform24(seed, offset, edge_key(forward row, forward column)); swap = this
//   graph is the reverse of the mask's frame.
struct W_Scaled {
    const float *rs, *cs;
    float keep;
    uint64_t seed, offset;
    const int64_t *offset_dev;  // + *offset_dev (a device step counter: hipGraph replays draw fresh masks)
    int swap;
    bool drops() const { return keep < 1.f; }
    __device__ __forceinline__ float operator()(int64_t, int c, int r) const {
        float w = rs ? rs[r] : 1.f;
        if (cs) w *= cs[c];
        if (keep < 1.f) {
            const uint64_t k = swap ? edge_key((uint32_t)c, (uint32_t)r) : edge_key((uint32_t)r, (uint32_t)c);
            const uint64_t off = offset + (offset_dev ? (uint64_t)*offset_dev : 0);
            // random_tensor = keep + U; mask = floor(random_tensor) (model.py:4019-4021)
            w = (floorf(keep + uniform24(seed, off, k)) != 0.f) ? w / keep : 0.f;
        }
        return w;
    }
};

#ifndef IGR_SPMM_UNROLL
#define IGR_SPMM_UNROLL 16
#endif
#ifndef IGR_SPMM_MIN_WAVES
#define IGR_SPMM_MIN_WAVES 1
#endif

// Accumulate the first n edges of a block whose (col, val) pairs live in lanes
// gbase .. gbase+n-1 of the caller's own lane group (shuffles never leave the
// group, so divergence between groups is harmless).  Steps of U edges issue
// all U row gathers before their FMAs; the last partial step masks its
// out-of-range slots (no load is issued for them).
// MASK: a column with cl < 0 (masked out when the pair was loaded) adds
// nothing and its row is not read.
template <int U, bool MASK>
__device__ __forceinline__ float4 gather_block(float4 acc, int cl, float vl, int gbase, int n,
                                               const float *__restrict__ xs, int64_t ldx) {
    int k = 0;
    for (; k + U <= n; k += U) {
        float4 xv[U];
        float wv[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int c = shfl_i(cl, gbase + k + j);
            wv[j] = shfl_f(vl, gbase + k + j);
            if (MASK) {
                xv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (c >= 0) xv[j] = *reinterpret_cast<const float4 *>(xs + (int64_t)c * ldx);
            } else {
                xv[j] = *reinterpret_cast<const float4 *>(xs + (int64_t)c * ldx);
            }
        }
#pragma unroll
        for (int j = 0; j < U; ++j) acc = f4_fma(wv[j], xv[j], acc);
    }
    if (k < n) {
        float4 xv[U];
        float wv[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            if (k + j < n) {
                const int c = shfl_i(cl, gbase + k + j);
                wv[j] = shfl_f(vl, gbase + k + j);
                xv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (!MASK || c >= 0) xv[j] = *reinterpret_cast<const float4 *>(xs + (int64_t)c * ldx);
            }
        }
#pragma unroll
        for (int j = 0; j < U; ++j)
            if (k + j < n) acc = f4_fma(wv[j], xv[j], acc);
    }
    return acc;
}

// One round of NB (col, val) blocks of LPR edges each (n <= NB*LPR edges):
// edge j lives in block j / LPR, lane gbase + j % LPR - both compile-time, so
// all n row gathers are issued before their FMAs (narrow rows, d = 32, where a
// single LPR-edge block would leave only 8 gathers in flight per group).
template <int NB, int LPR, bool MASK>
__device__ __forceinline__ float4 gather_round(float4 acc, const int (&cl)[NB], const float (&vl)[NB], int gbase,
                                               int n, const float *__restrict__ xs, int64_t ldx) {
    constexpr int BE = NB * LPR;
    float4 xv[BE];
    float wv[BE];
#pragma unroll
    for (int j = 0; j < BE; ++j) {
        if (j < n) {
            const int c = shfl_i(cl[j / LPR], gbase + j % LPR);
            wv[j] = shfl_f(vl[j / LPR], gbase + j % LPR);
            xv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (!MASK || c >= 0) xv[j] = *reinterpret_cast<const float4 *>(xs + (int64_t)c * ldx);
        }
    }
#pragma unroll
    for (int j = 0; j < BE; ++j)
        if (j < n) acc = f4_fma(wv[j], xv[j], acc);
    return acc;
}

// (col, val) of CSR position p; with MASK, masked-out columns and zero-weight
// edges come back as -1
template <bool MASK, class W>
__device__ __forceinline__ void load_pair(const int32_t *__restrict__ col, const W &wfn, int64_t p, int r,
                                          const uint32_t *__restrict__ cmask, int &c, float &w) {
    c = ld_stream(col + p);
    w = wfn(p, c, r);
    // a dropped edge (w == 0) adds an exact 0 (the accumulator is never -0), so
    // skipping its gather leaves every sum bitwise unchanged
    if (MASK && ((cmask && !bit_set(cmask, c)) || w == 0.f)) {
        c = -1;
        w = 0.f;
    }
}

template <int D, class W, bool MASK>
__global__ __launch_bounds__(256, IGR_SPMM_MIN_WAVES) void spmm_main(
    const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col, W wfn,
    const float *__restrict__ x, int64_t ldx, const int32_t *__restrict__ order, int64_t n_order,
    const int32_t *__restrict__ chunk_row, const int64_t *__restrict__ chunk_beg, int64_t n_chunks,
    int64_t chunk_edges, float *__restrict__ ws, int64_t chunk_blocks, Epi epi) {
    constexpr int LPR = D / 4;   // lanes per feature row
    constexpr int G = 64 / LPR;  // groups per wave
    constexpr int U = IGR_SPMM_UNROLL < LPR ? IGR_SPMM_UNROLL : LPR;  // gathers in flight per group
    const int lane = threadIdx.x & 63;
    const int grp = lane / LPR;
    const int sub = lane - grp * LPR;
    const int wib = threadIdx.x >> 6;
    const float *xs = x + sub * 4;

    if ((int64_t)blockIdx.x < chunk_blocks) {
        // ---------------- chunk tier: one wave per chunk of a long row
        const int64_t c = (int64_t)blockIdx.x * 4 + wib;
        if (c >= n_chunks) return;
        const int r = chunk_row[c];
        if (epi.row_mask && !bit_set(epi.row_mask, r)) return;  // wave-uniform
        const int64_t b = chunk_beg[c];
        const int64_t e = min(b + chunk_edges, row_ptr[r + 1]);
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        int64_t base = b;
        int n = (int)min((int64_t)64, e - base);
        int cl = 0;
        float vl = 0.f;
        if (lane < n) load_pair<MASK>(col, wfn, base + lane, r, epi.col_mask, cl, vl);
        while (n > 0) {
            const int64_t nb = base + 64;
            const int nn = (int)min((int64_t)64, e - nb);
            int cl2 = 0;
            float vl2 = 0.f;
            if (lane < nn) load_pair<MASK>(col, wfn, nb + lane, r, epi.col_mask, cl2, vl2);
            // group grp takes edges [grp*LPR, grp*LPR + LPR) of this 64-edge block,
            // i.e. exactly the (col, val) pairs its own lanes loaded
            const int m = min(max(n - grp * LPR, 0), LPR);
            acc = gather_block<U, MASK>(acc, cl, vl, grp * LPR, m, xs, ldx);
            base = nb;
            n = nn;
            cl = cl2;
            vl = vl2;
        }
#pragma unroll
        for (int s = LPR; s < 64; s <<= 1) {
            acc.x += shfl_xor_f(acc.x, s);
            acc.y += shfl_xor_f(acc.y, s);
            acc.z += shfl_xor_f(acc.z, s);
            acc.w += shfl_xor_f(acc.w, s);
        }
        if (grp == 0) *reinterpret_cast<float4 *>(ws + c * D + sub * 4) = acc;
        return;
    }

    // ---------------- row tier: one LPR-lane group per row
    const int64_t w = ((int64_t)blockIdx.x - chunk_blocks) * 4 + wib;
    const int64_t i = w * G + grp;
    if (i >= n_order) return;
    const int r = order[i];
    // a skipped row's group leaves; shuffles never cross groups, so this is safe
    if (epi.row_mask && !bit_set(epi.row_mask, r)) return;
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    const int gbase = grp * LPR;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    constexpr int NB = LPR >= 16 ? 1 : 16 / LPR;  // (col, val) blocks per round
    if constexpr (NB > 1) {
        constexpr int BE = NB * LPR;
        int64_t base = b;
        int n = (int)min((int64_t)BE, e - base);
        int cl[NB];
        float vl[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            cl[k] = 0;
            vl[k] = 0.f;
            if (k * LPR + sub < n) load_pair<MASK>(col, wfn, base + k * LPR + sub, r, epi.col_mask, cl[k], vl[k]);
        }
        while (n > 0) {
            const int64_t nb = base + BE;
            const int nn = (int)min((int64_t)BE, e - nb);
            int cl2[NB];
            float vl2[NB];
#pragma unroll
            for (int k = 0; k < NB; ++k) {  // next round's pairs, under this round's gathers
                cl2[k] = 0;
                vl2[k] = 0.f;
                if (k * LPR + sub < nn)
                    load_pair<MASK>(col, wfn, nb + k * LPR + sub, r, epi.col_mask, cl2[k], vl2[k]);
            }
            acc = gather_round<NB, LPR, MASK>(acc, cl, vl, gbase, n, xs, ldx);
            base = nb;
            n = nn;
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                cl[k] = cl2[k];
                vl[k] = vl2[k];
            }
        }
        store_row4(epi, r, sub * 4, acc);
        return;
    }
    int64_t base = b;
    int n = (int)min((int64_t)LPR, e - base);
    int cl = 0;
    float vl = 0.f;
    if (sub < n) load_pair<MASK>(col, wfn, base + sub, r, epi.col_mask, cl, vl);
    while (n > 0) {
        const int64_t nb = base + LPR;
        const int nn = (int)min((int64_t)LPR, e - nb);
        int cl2 = 0;
        float vl2 = 0.f;
        if (sub < nn) load_pair<MASK>(col, wfn, nb + sub, r, epi.col_mask, cl2, vl2);
        acc = gather_block<U, MASK>(acc, cl, vl, gbase, n, xs, ldx);
        base = nb;
        n = nn;
        cl = cl2;
        vl = vl2;
    }
    store_row4(epi, r, sub * 4, acc);
}

// Sum each split row's chunk partials, then the epilogue.  One workgroup per
// split row: its 4*G lane groups ("slots") sum chunks slot, slot + 4G, ... in
// order, then the slots are added in a fixed tree through LDS, so the result
// is the same on every run whatever the chunk count (a row of 10^6 edges has
// ~2000 chunks; a single group would walk them serially).
template <int D, int NT>
__global__ __launch_bounds__(NT) void spmm_combine(const int32_t *__restrict__ split_row,
                                                   const int64_t *__restrict__ split_ptr,
                                                   int64_t n_split, const float *__restrict__ ws,
                                                   Epi epi) {
    constexpr int LPR = D / 4;
    constexpr int S = (NT / 64) * (64 / LPR);  // slots per workgroup
    __shared__ float4 red[S][LPR];
    const int slot = threadIdx.x / LPR;
    const int sub = threadIdx.x - slot * LPR;
    const int64_t i = blockIdx.x;
    if (i >= n_split) return;
    if (epi.row_mask && !bit_set(epi.row_mask, split_row[i])) return;  // block-uniform
    // 8 independent partial sums per slot keep 8 loads in flight (a hub row's
    // slots each walk ~100+ partials); combined in a fixed tree: deterministic
    constexpr int V = 8;
    float4 a[V];
#pragma unroll
    for (int j = 0; j < V; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t c = split_ptr[i] + slot;
    const int64_t e = split_ptr[i + 1];
    for (; c + (V - 1) * S < e; c += V * S) {
#pragma unroll
        for (int j = 0; j < V; ++j)
            a[j] = f4_add(a[j], *reinterpret_cast<const float4 *>(ws + (c + j * S) * D + sub * 4));
    }
    for (; c < e; c += S) a[0] = f4_add(a[0], *reinterpret_cast<const float4 *>(ws + c * D + sub * 4));
    red[slot][sub] = f4_add(f4_add(f4_add(a[0], a[1]), f4_add(a[2], a[3])),
                            f4_add(f4_add(a[4], a[5]), f4_add(a[6], a[7])));
    __syncthreads();
#pragma unroll
    for (int w = S / 2; w >= 1; w >>= 1) {
        if (slot < w) red[slot][sub] = f4_add(red[slot][sub], red[slot + w][sub]);
        __syncthreads();
    }
    if (slot == 0) store_row4(epi, split_row[i], sub * 4, red[0][sub]);
}

// The same with a wave per split row, four rows per workgroup, for graphs whose split rows
// mostly have few chunks (a small graph with a low split threshold: thousands of split
// rows of 2-3 chunks, for which a workgroup with LDS and barriers per row is the cost).
// A wave's 64 / (D / 4) slots take alternate chunks and are added in a fixed xor tree.
// A row of more than kWaveChunks chunks (a hub row; rows come heaviest first, so these
// fill the first workgroups) is instead added by the whole workgroup as in spmm_combine:
// the test is uniform over the workgroup.
constexpr int kWaveChunks = 32;

template <int D>
__global__ __launch_bounds__(256) void spmm_combine_wave(const int32_t *__restrict__ split_row,
                                                         const int64_t *__restrict__ split_ptr,
                                                         int64_t n_split, const float *__restrict__ ws, Epi epi) {
    constexpr int LPR = D / 4;
    constexpr int S = 64 / LPR;         // slots of a wave
    constexpr int SB = 4 * S;           // slots of the workgroup
    __shared__ float4 red[SB][LPR];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
#pragma unroll 1
    for (int q = 0; q < 4; ++q) {
        const int64_t i = (int64_t)blockIdx.x * 4 + q;
        if (i >= n_split) break;  // uniform
        const int64_t b = split_ptr[i], e = split_ptr[i + 1];
        const int32_t r = split_row[i];
        if (epi.row_mask && !bit_set(epi.row_mask, r)) continue;  // uniform
        if (e - b > kWaveChunks) {
            // the whole workgroup on this row: 8 independent sums per slot, then a fixed tree
            const int slot = threadIdx.x / LPR;
            const int sub = threadIdx.x - slot * LPR;
            constexpr int V = 8;
            float4 a[V];
#pragma unroll
            for (int j = 0; j < V; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            int64_t c = b + slot;
            for (; c + (V - 1) * SB < e; c += V * SB) {
#pragma unroll
                for (int j = 0; j < V; ++j)
                    a[j] = f4_add(a[j], *reinterpret_cast<const float4 *>(ws + (c + j * SB) * D + sub * 4));
            }
            for (; c < e; c += SB) a[0] = f4_add(a[0], *reinterpret_cast<const float4 *>(ws + c * D + sub * 4));
            __syncthreads();  // red may still be read for the previous heavy row
            red[slot][sub] = f4_add(f4_add(f4_add(a[0], a[1]), f4_add(a[2], a[3])),
                                    f4_add(f4_add(a[4], a[5]), f4_add(a[6], a[7])));
            __syncthreads();
#pragma unroll
            for (int w = SB / 2; w >= 1; w >>= 1) {
                if (slot < w) red[slot][sub] = f4_add(red[slot][sub], red[slot + w][sub]);
                __syncthreads();
            }
            if (slot == 0) store_row4(epi, r, sub * 4, red[0][sub]);
        } else if (wave == q) {
            const int slot = lane / LPR;
            const int sub = lane - slot * LPR;
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int64_t c = b + slot; c < e; c += S)
                a = f4_add(a, *reinterpret_cast<const float4 *>(ws + c * D + sub * 4));
#pragma unroll
            for (int m = LPR; m < 64; m <<= 1) {
                a.x += shfl_xor_f(a.x, m);
                a.y += shfl_xor_f(a.y, m);
                a.z += shfl_xor_f(a.z, m);
                a.w += shfl_xor_f(a.w, m);
            }
            if (slot == 0) store_row4(epi, r, sub * 4, a);
        }
    }
}

// Any d / alignment: one wave per row, lanes over features.
template <class W>
__global__ __launch_bounds__(256) void spmm_generic(int64_t n_rows, int d,
                                                    const int64_t *__restrict__ row_ptr,
                                                    const int32_t *__restrict__ col, W wfn,
                                                    const float *__restrict__ x, int64_t ldx,
                                                    Epi epi) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= n_rows) return;
    if (epi.row_mask && !bit_set(epi.row_mask, r)) return;
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    for (int f = lane; f < d; f += 64) {
        float s = 0.f;
        for (int64_t p = b; p < e; ++p) {
            if (epi.col_mask && !bit_set(epi.col_mask, col[p])) continue;
            s = fmaf(wfn(p, col[p], (int)r), x[(int64_t)col[p] * ldx + f], s);
        }
        store_row1(epi, r, f, s);
    }
}

template <int D, class W>
static void launch_fast(const igr_csr *g, const float *x, int64_t ldx, const W &wfn, const Epi &epi,
                        float *ws, hipStream_t st) {
    constexpr int G = 64 / (D / 4);
    const int64_t chunk_blocks = (g->n_chunks + 3) / 4;
    const int64_t row_blocks = (g->n_order + 4 * G - 1) / (4 * G);
    const int64_t blocks = chunk_blocks + row_blocks;
    if (blocks > 0) {
        if (epi.col_mask || wfn.drops())
            hipLaunchKernelGGL((spmm_main<D, W, true>), dim3((unsigned)blocks), dim3(256), 0, st, g->row_ptr,
                               g->col_idx, wfn, x, ldx, g->order, g->n_order, g->chunk_row, g->chunk_beg,
                               g->n_chunks, g->chunk_edges, ws, chunk_blocks, epi);
        else
            hipLaunchKernelGGL((spmm_main<D, W, false>), dim3((unsigned)blocks), dim3(256), 0, st, g->row_ptr,
                               g->col_idx, wfn, x, ldx, g->order, g->n_order, g->chunk_row, g->chunk_beg,
                               g->n_chunks, g->chunk_edges, ws, chunk_blocks, epi);
    }
    if (g->n_split > 0) {
        // rows of ~64+ chunks on average (the feature graph's general rows: 10^3-10^4
        // chunks) take 1024-thread workgroups, 4x the partial loads in flight;
        // the choice depends on the graph only, so results stay reproducible
        if (g->n_chunks >= 64 * g->n_split)
            hipLaunchKernelGGL((spmm_combine<D, 1024>), dim3((unsigned)g->n_split), dim3(1024), 0, st, g->split_row,
                               g->split_ptr, g->n_split, ws, epi);
        else if (g->n_chunks <= 8 * g->n_split)  // mostly short split rows; hub rows inside take the workgroup
            hipLaunchKernelGGL((spmm_combine_wave<D>), dim3((unsigned)((g->n_split + 3) / 4)), dim3(256), 0, st,
                               g->split_row, g->split_ptr, g->n_split, ws, epi);
        else
            hipLaunchKernelGGL((spmm_combine<D, 256>), dim3((unsigned)g->n_split), dim3(256), 0, st, g->split_row,
                               g->split_ptr, g->n_split, ws, epi);
    }
}

// Validate the epilogue / shapes, pick the fast (d in {32,64,128,256}, 16-B
// aligned) or the generic kernel, and launch with the weight policy W.
template <class W>
static int run_spmm(const char *fn, const igr_csr *g, int32_t d, const float *x, int64_t ldx, const W &wfn,
                    float *y, int64_t ldy, const igr_epilogue *epi_in, float *workspace, void *stream) {
    if (!g) return arg_error(fn, "graph is NULL");
    if (d <= 0) return arg_error(fn, "d must be positive");
    if (g->n_rows < 0 || g->n_cols < 0 || g->nnz < 0) return arg_error(fn, "negative sizes");
    if (g->n_rows == 0) return IGR_OK;
    if (!g->row_ptr || (g->nnz > 0 && !g->col_idx)) return arg_error(fn, "missing CSR arrays");
    if (g->nnz > 0 && !x) return arg_error(fn, "x is NULL");
    if (ldx < d || ldy < d) return arg_error(fn, "leading dimension smaller than d");
    if (g->n_order + g->n_split != g->n_rows)
        return arg_error(fn, "schedule does not cover every row (n_order + n_split != n_rows)");
    if (g->n_chunks > 0 && !workspace) return arg_error(fn, "workspace required for split rows");
    Epi e{};
    e.y = y;
    e.ldy = ldy;
    e.alpha = 1.f;
    e.beta = 0.f;
    e.acc_div = 1.f;
    if (epi_in) {
        e.alpha = epi_in->alpha;
        e.beta = epi_in->beta;
        e.add = epi_in->add;
        e.ld_add = epi_in->ld_add;
        e.acc = epi_in->acc;
        e.ld_acc = epi_in->ld_acc;
        e.acc_mode = epi_in->acc_mode;
        e.acc_div = epi_in->acc_div;
        e.skip_y = epi_in->skip_y;
        e.row_scale = epi_in->row_scale;
        e.row_mask = epi_in->row_mask;
        e.col_mask = epi_in->col_mask;
        if (e.acc_mode < 0 || e.acc_mode > 2) return arg_error(fn, "acc_mode must be 0, 1 or 2");
        if (e.acc_mode && (!e.acc || e.ld_acc < d)) return arg_error(fn, "bad acc");
        if (e.add && e.ld_add < d) return arg_error(fn, "bad ld_add");
        if (e.acc_div == 0.f) return arg_error(fn, "acc_div is 0");
    }
    if (!e.skip_y && !y) return arg_error(fn, "y is NULL");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    bool fast = (d == 32 || d == 64 || d == 128 || d == 256) && (ldx % 4 == 0) && (ldy % 4 == 0) &&
                aligned16(x) && aligned16(y) && aligned16(workspace);
    if (e.add) fast = fast && aligned16(e.add) && e.ld_add % 4 == 0;
    if (e.acc_mode) fast = fast && aligned16(e.acc) && e.ld_acc % 4 == 0;
    if (fast) {
        if (!g->order && g->n_order > 0) return arg_error(fn, "missing schedule");
        switch (d) {
            case 32: launch_fast<32>(g, x, ldx, wfn, e, workspace, st); break;
            case 64: launch_fast<64>(g, x, ldx, wfn, e, workspace, st); break;
            case 128: launch_fast<128>(g, x, ldx, wfn, e, workspace, st); break;
            default: launch_fast<256>(g, x, ldx, wfn, e, workspace, st); break;
        }
    } else {
        const unsigned blocks = (unsigned)((g->n_rows + 3) / 4);
        hipLaunchKernelGGL((spmm_generic<W>), dim3(blocks), dim3(256), 0, st, g->n_rows, d, g->row_ptr, g->col_idx,
                           wfn, x, ldx, e);
    }
    return launch_status(fn);
}

// The uniforms W_Scaled draws, per CSR position of g (explicit-values path:
// AttIGCN's per-edge dropout; tests).  One wave per row, lanes over its edges.
// With val: the dropout itself in the same pass, by edge id - out[e] = val[e] / keep where
// floor(keep + U) is 1, else 0 (model.py:4019-4027), the expression of edge_dropout_kernel.
__global__ __launch_bounds__(256) void uniforms_kernel(int64_t n_rows, const int64_t *__restrict__ row_ptr,
                                                       const int32_t *__restrict__ col,
                                                       const int64_t *__restrict__ eid, uint64_t seed, uint64_t offset,
                                                       const int64_t *__restrict__ offset_dev, int swap,
                                                       const float *__restrict__ val, float keep,
                                                       float *__restrict__ out, RowPlan plan, int planned) {
    // planned: a wave takes one chunk of a split row or one whole unsplit row (a hub row
    // is otherwise one wave's loop); else wave w takes row w
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    int64_t r, b, e;
    if (planned) {
        if (w >= plan.n_chunks + plan.n_order) return;
        if (w < plan.n_chunks) {
            r = plan.chunk_row[w];
            b = plan.chunk_beg[w];
            e = min(b + plan.chunk_edges, row_ptr[r + 1]);
        } else {
            r = plan.order[w - plan.n_chunks];
            b = row_ptr[r];
            e = row_ptr[r + 1];
        }
    } else {
        r = w;
        if (r >= n_rows) return;
        b = row_ptr[r];
        e = row_ptr[r + 1];
    }
    const uint64_t off = offset + (offset_dev ? (uint64_t)*offset_dev : 0);
    for (int64_t p = b + (threadIdx.x & 63); p < e; p += 64) {
        const uint32_t c = (uint32_t)col[p];
        const float u = uniform24(seed, off, swap ? edge_key(c, (uint32_t)r) : edge_key((uint32_t)r, c));
        if (!val) {
            out[p] = u;
        } else {
            const int64_t e = eid ? eid[p] : p;
            out[e] = floorf(keep + u) != 0.f ? val[e] / keep : 0.f;
        }
    }
}

}  // namespace igr

using namespace igr;

extern "C" int igr_spmm_f32(const igr_csr *g, int32_t d, const float *x, int64_t ldx,
                            const float *rhs, float *y, int64_t ldy, const igr_epilogue *epi,
                            float *workspace, void *stream) {
    return guarded("igr_spmm_f32", [&]() -> int {
        const char *fn = "igr_spmm_f32";
        if (!g) return arg_error(fn, "graph is NULL");
        if (!rhs) return run_spmm(fn, g, d, x, ldx, W_One{}, y, ldy, epi, workspace, stream);
        if (g->edge_id) return run_spmm(fn, g, d, x, ldx, W_ValEid{rhs, g->edge_id}, y, ldy, epi, workspace, stream);
        return run_spmm(fn, g, d, x, ldx, W_Val{rhs}, y, ldy, epi, workspace, stream);
    });
}

// ---------------------------------------------------------------------------
// igr_spmm_noalloc_f32: igr_spmm_f32 for callers that cannot allocate device
// memory (code under hipGraph capture, tight serving loops, harnesses that
// forbid hipMalloc).  The chunk tier's partial rows, which igr_spmm_f32 takes
// as a caller-allocated `workspace`, live in a file-scope device array instead.
// Every GPU the library runs on holds its own copy of the array (16 MiB) until
// the process ends.  `scratch` is only a host-side stand-in for that array: its
// per-device address comes from hipGetSymbolAddress, looked up once per device
// (on the entry point's first call there, with that device current) and used
// for every kernel argument afterwards.
static __device__ __align__(256) float scratch[IGR_SPMM_NOALLOC_MAX_FLOATS];

namespace igr {
constexpr int kMaxDevices = 64;
static std::mutex g_scratch_mu;
static float *g_scratch_ptr[kMaxDevices];  // per device, filled on first use

// The scratch array of the device that owns `owned` (a device pointer of the call: the
// output).  hipGetSymbolAddress resolves the array for the CURRENT device, so that device
// must be the pointer's: a launch on another GPU's stream with this GPU's array would fault.
static int scratch_for_device_of(const char *fn, const void *owned, float **out) {
    int dev = -1;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) {
        set_error(std::string(fn) + ": hipGetDevice: " + hipGetErrorString(e));
        return IGR_ERR_HIP;
    }
    if (dev < 0 || dev >= kMaxDevices) return arg_error(fn, "device index out of range");
    hipPointerAttribute_t at{};
    e = hipPointerGetAttributes(&at, owned);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // the failed query must not surface as a later launch error
        return arg_error(fn, std::string("the output is not memory HIP knows (") + hipGetErrorString(e) + ")");
    }
    if (at.type != hipMemoryTypeDevice && at.type != hipMemoryTypeManaged)
        return arg_error(fn, "the output is not device memory");
    if (at.device != dev)
        return arg_error(fn, "the output lives on device " + std::to_string(at.device) + " but device " +
                                 std::to_string(dev) + " is current: make the output's device current before the "
                                 "call (each GPU has its own scratch array)");
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    if (!g_scratch_ptr[dev]) {
        void *p = nullptr;
        e = hipGetSymbolAddress(&p, HIP_SYMBOL(scratch));
        if (e != hipSuccess || !p) {
            set_error(std::string(fn) + ": hipGetSymbolAddress(scratch): " + hipGetErrorString(e));
            return IGR_ERR_HIP;
        }
        g_scratch_ptr[dev] = static_cast<float *>(p);
    }
    *out = g_scratch_ptr[dev];
    return IGR_OK;
}
}  // namespace igr

extern "C" int igr_spmm_noalloc_f32(const igr_csr *g, int32_t d, const float *x, int64_t ldx,
                                    const float *rhs, float *y, int64_t ldy, const igr_epilogue *epi,
                                    void *stream) {
    return guarded("igr_spmm_noalloc_f32", [&]() -> int {
        const char *fn = "igr_spmm_noalloc_f32";
        if (!g) return arg_error(fn, "graph is NULL");
        if (d <= 0) return arg_error(fn, "d must be positive");
        if (g->n_chunks < 0) return arg_error(fn, "negative n_chunks");
        if (g->n_chunks > 0 && g->n_chunks > (int64_t)IGR_SPMM_NOALLOC_MAX_FLOATS / d)
            return arg_error(fn, "split rows need n_chunks * d = " + std::to_string(g->n_chunks) + " * " +
                                     std::to_string(d) + " floats of scratch, more than the static " +
                                     std::to_string((int64_t)IGR_SPMM_NOALLOC_MAX_FLOATS) +
                                     " (IGR_SPMM_NOALLOC_MAX_FLOATS); use igr_spmm_f32 with a workspace");
        float *ws = nullptr;
        // every partial row the combine kernel reads is written by the main kernel
        // of the same call, so nothing in the array has to start at zero
        if (g->n_chunks > 0) {
            const void *owned = y ? (const void *)y : (epi ? (const void *)epi->acc : nullptr);
            if (!owned) return arg_error(fn, "no output (y is NULL and the epilogue has no acc)");
            const int rc = scratch_for_device_of(fn, owned, &ws);
            if (rc != IGR_OK) return rc;
        }
        if (!rhs) return run_spmm(fn, g, d, x, ldx, W_One{}, y, ldy, epi, ws, stream);
        if (g->edge_id) return run_spmm(fn, g, d, x, ldx, W_ValEid{rhs, g->edge_id}, y, ldy, epi, ws, stream);
        return run_spmm(fn, g, d, x, ldx, W_Val{rhs}, y, ldy, epi, ws, stream);
    });
}

extern "C" int igr_spmm_scaled_f32(const igr_csr *g, int32_t d, const float *x, int64_t ldx,
                                   const float *row_scale, const float *col_scale, float keep, uint64_t seed,
                                   uint64_t offset, const int64_t *offset_dev, int32_t transposed, float *y,
                                   int64_t ldy,
                                   const igr_epilogue *epi, float *workspace, void *stream) {
    return guarded("igr_spmm_scaled_f32", [&]() -> int {
        const char *fn = "igr_spmm_scaled_f32";
        if (!g) return arg_error(fn, "graph is NULL");
        if (!(keep > 0.f && keep <= 1.f)) return arg_error(fn, "keep must be in (0, 1]");
        if (keep < 1.f && (g->n_rows > 4294967295LL || g->n_cols > 4294967295LL))
            return arg_error(fn, "dropout keys need row / column ids below 2^32");
        return run_spmm(fn, g, d, x, ldx, W_Scaled{row_scale, col_scale, keep, seed, offset, offset_dev, transposed ? 1 : 0}, y,
                        ldy, epi, workspace, stream);
    });
}

extern "C" int igr_spmm_heads_f32(const igr_csr *g, int32_t h, int32_t d, const float *x, int64_t ldx,
                                  const float *rhs, float *y, int64_t ldy, float *workspace, void *stream) {
    return guarded("igr_spmm_heads_f32", [&]() -> int {
        const char *fn = "igr_spmm_heads_f32";
        if (!g || h <= 0) return arg_error(fn, "bad graph / h");
        if (g->nnz > 0 && !rhs) return arg_error(fn, "rhs is NULL");
        if (ldx < (int64_t)h * d || ldy < (int64_t)h * d) return arg_error(fn, "leading dimension < h*d");
        // one launch per head: each gathers only its d-column slice of x (the
        // slices of a small table stay L2-resident)
        for (int32_t j = 0; j < h; ++j) {
            const int rc = run_spmm(fn, g, d, x ? x + (int64_t)j * d : nullptr, ldx,
                                    W_ValHead{rhs, g->edge_id, h, j}, y ? y + (int64_t)j * d : nullptr, ldy,
                                    nullptr, workspace, stream);
            if (rc != IGR_OK) return rc;
        }
        return IGR_OK;
    });
}

extern "C" int igr_dropout_uniforms(const igr_csr *g, uint64_t seed, uint64_t offset, const int64_t *offset_dev,
                                    int32_t transposed, float *out, void *stream) {
    return guarded("igr_dropout_uniforms", [&]() -> int {
        if (!g || !out) return arg_error("igr_dropout_uniforms", "graph / out NULL");
        if (g->n_rows <= 0 || g->nnz <= 0) return IGR_OK;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        if (g->n_rows > 4294967295LL || g->n_cols > 4294967295LL)
            return arg_error("igr_dropout_uniforms", "dropout keys need row / column ids below 2^32");
        const bool planned = use_row_plan(g);
        const int64_t waves = planned ? g->n_chunks + g->n_order : g->n_rows;
        hipLaunchKernelGGL(uniforms_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, g->n_rows,
                           g->row_ptr, g->col_idx, g->edge_id, seed, offset, offset_dev, transposed ? 1 : 0,
                           (const float *)nullptr, 1.f, out, row_plan_of(g), planned ? 1 : 0);
        return launch_status("igr_dropout_uniforms");
    });
}

extern "C" int igr_edge_dropout_counter_f32(const igr_csr *g, const float *val, float p, uint64_t seed, uint64_t offset,
                                            const int64_t *offset_dev, int32_t transposed, float *out, void *stream) {
    return guarded("igr_edge_dropout_counter_f32", [&]() -> int {
        const char *fn = "igr_edge_dropout_counter_f32";
        if (!g || !val || !out) return arg_error(fn, "NULL pointer");
        if (!(p >= 0.f && p < 1.f)) return arg_error(fn, "p must be in [0, 1)");
        if (g->n_rows == 0 || g->nnz == 0) return IGR_OK;
        if (g->n_rows > 4294967295LL || g->n_cols > 4294967295LL)
            return arg_error(fn, "dropout keys need row / column ids below 2^32");
        const float keep = (float)(1.0 - (double)p);
        const bool planned = use_row_plan(g);
        const int64_t waves = planned ? g->n_chunks + g->n_order : g->n_rows;
        hipLaunchKernelGGL(uniforms_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0,
                           reinterpret_cast<hipStream_t>(stream), g->n_rows, g->row_ptr, g->col_idx, g->edge_id, seed,
                           offset, offset_dev, transposed ? 1 : 0, val, keep, out, row_plan_of(g), planned ? 1 : 0);
        return launch_status(fn);
    });
}

// ---------------------------------------------------------------------------
// igr_spmv_f32: y[r] = sum_{p in row r} w(p) x[col[p]] for ONE value per node (IMCGAE's two
// repeated blocks stay rank one through every layer, model.py:4326-4337, so they follow from
// one scalar per node and layer).  4 bytes gathered per edge from a vector that fits L2, so
// the work is the streamed CSR: 16 lanes share a row (lane l takes edges l, l + 16, ...; a
// fixed xor tree adds the 16 partial sums), rows the schedule split (hub rows) take a whole
// workgroup each.  Fixed summation orders: the same bits on every run.
namespace igr {

__global__ __launch_bounds__(256) void spmv_rows_kernel(int64_t n_list, const int32_t *__restrict__ list,
                                                        const int64_t *__restrict__ row_ptr,
                                                        const int32_t *__restrict__ col,
                                                        const int64_t *__restrict__ eid,
                                                        const float *__restrict__ rhs, const float *__restrict__ x,
                                                        float *__restrict__ y) {
    const int64_t grp = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    if (grp >= n_list) return;  // whole 16-lane groups leave together; the shuffles stay inside a group
    const int l = threadIdx.x & 15;
    const int64_t r = list ? list[grp] : grp;
    const int64_t beg = row_ptr[r], end = row_ptr[r + 1];
    float s = 0.f;
    for (int64_t p = beg + l; p < end; p += 16) {
        const float w = rhs ? rhs[eid ? eid[p] : p] : 1.f;
        s += w * x[col[p]];
    }
    s += shfl_xor_f(s, 8);
    s += shfl_xor_f(s, 4);
    s += shfl_xor_f(s, 2);
    s += shfl_xor_f(s, 1);
    if (l == 0) y[r] = s;
}

__global__ __launch_bounds__(256) void spmv_split_kernel(const int32_t *__restrict__ split_row,
                                                         const int64_t *__restrict__ row_ptr,
                                                         const int32_t *__restrict__ col,
                                                         const int64_t *__restrict__ eid,
                                                         const float *__restrict__ rhs, const float *__restrict__ x,
                                                         float *__restrict__ y) {
    __shared__ float part[256];
    const int t = threadIdx.x;
    const int64_t r = split_row[blockIdx.x];
    const int64_t beg = row_ptr[r], end = row_ptr[r + 1];
    float s = 0.f;
    for (int64_t p = beg + t; p < end; p += 256) {
        const float w = rhs ? rhs[eid ? eid[p] : p] : 1.f;
        s += w * x[col[p]];
    }
    part[t] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) part[t] += part[t + o];
        __syncthreads();
    }
    if (t == 0) y[r] = part[0];
}

}  // namespace igr

extern "C" int igr_spmv_f32(const igr_csr *g, const float *x, const float *rhs, float *y, void *stream) {
    return guarded("igr_spmv_f32", [&]() -> int {
        const char *fn = "igr_spmv_f32";
        if (!g) return arg_error(fn, "graph is NULL");
        if (g->n_rows <= 0) return IGR_OK;
        if (!y || !g->row_ptr || (g->nnz > 0 && (!x || !g->col_idx))) return arg_error(fn, "NULL pointer");
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        // the schedule's two lists cover every row once: unsplit rows (16 lanes each), split rows
        // (a workgroup each); without a schedule every row takes 16 lanes
        const bool planned = g->order && g->n_order > 0 && g->n_order + g->n_split == g->n_rows &&
                             (g->n_split == 0 || g->split_row) && g->n_split <= 2147483647;
        const int64_t n_list = planned ? g->n_order : g->n_rows;
        const int64_t blocks = (n_list * 16 + 255) / 256;
        if (blocks > 2147483647) return arg_error(fn, "too many rows");
        hipLaunchKernelGGL(spmv_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, n_list,
                           planned ? g->order : nullptr, g->row_ptr, g->col_idx, g->edge_id, rhs, x, y);
        if (planned && g->n_split > 0)
            hipLaunchKernelGGL(spmv_split_kernel, dim3((unsigned)g->n_split), dim3(256), 0, st, g->split_row,
                               g->row_ptr, g->col_idx, g->edge_id, rhs, x, y);
        return launch_status(fn);
    });
}
