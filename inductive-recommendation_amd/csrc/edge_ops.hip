// edge_ops.hip - per-edge kernels of the attention inductive layer and the
// feature-matrix value updates (gfx950).
//
//   igr_sddmm_dot_f32         AttIGCN.masked_mm            model.py:4246-4255
//   igr_segment_reduce_f32    gspmm copy_rhs max/sum       model.py:4270, 4273
//   igr_att_softmax_f32(+bwd) edge softmax + head mean     model.py:4270-4275
//   igr_edge_dropout_f32      NGCF.dropout_sp_mat          model.py:4016-4028
//   igr_feat_values_f32       IGCN.update_feat_mat         model.py:4127-4130
#include <cmath>

#include "common.h"

namespace igr {

// ---------------------------------------------------------------- SDDMM
// One wave per (destination row, head block).  A launch pass gathers TOT
// floats of each source row: all h*d of them, or - head split, when one
// head's slice of v fits an XCD's L2 but the whole table does not - the d of
// one head, with the grid ordered head-major (blockIdx / row_blocks = head) so
// the waves running together share one L2-resident slice.  LPE = TOT/4 lanes
// read a source row with a float4 each; EPW = 64/LPE lane groups per wave each
// take U consecutive edges of a 64-edge block whose columns came with one
// coalesced load (broadcast by ds_bpermute).  All U row gathers are issued
// before any dot.  Head sums: each lane holds U partial dots; a butterfly
// reduce-scatter over the head's hs = d/4 lanes (masks U/2 .. 1: every step
// halves the values a lane holds) leaves lane j with edge j's sum over its U
// lanes - hs - 1 shuffles for U edges instead of U*log2(hs) - then plain xor
// steps (masks U .. hs/2) finish heads wider than U lanes.  The U writer lanes
// of a head store U consecutive outputs.
#ifndef IGR_SDDMM_U
#define IGR_SDDMM_U 2
#endif
template <int TOT, int HS>
__global__ __launch_bounds__(256) void sddmm_dot_kernel(
    int64_t n_rows, int h, int d, const int64_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const int64_t *__restrict__ eid, const float *__restrict__ u,
    int64_t ld_u, const float *__restrict__ v, int64_t ld_v, float *__restrict__ out, int64_t row_blocks) {
    constexpr int LPE = TOT / 4;
    constexpr int EPW = 64 / LPE;
    constexpr int U = HS < IGR_SDDMM_U ? HS : IGR_SDDMM_U;  // edges per group per trip
    constexpr int TRIP = U * EPW;                            // edges per trip (divides 64)
    const int64_t hb = (int64_t)blockIdx.x / row_blocks;     // head block (0 unless head split)
    const int64_t r = ((int64_t)blockIdx.x - hb * row_blocks) * 4 + (threadIdx.x >> 6);
    if (r >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int eg = lane / LPE;
    const int sub = lane - eg * LPE;
    const int lh = sub % HS;  // lane within its head segment
    const int64_t f0 = hb * TOT;  // first feature of this pass
    const int head = (int)(f0 / d) + sub / HS;
    const float4 uq = *reinterpret_cast<const float4 *>(u + r * ld_u + f0 + sub * 4);
    const float *vs = v + f0 + sub * 4;
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    for (int64_t base = b; base < e; base += 64) {
        const int n = (int)min((int64_t)64, e - base);
        const int cl = lane < n ? col[base + lane] : 0;
        for (int t = 0; t < n; t += TRIP) {
            const int k0 = t + eg * U;  // this group's first edge in the block
            float4 vk[U];
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int c = shfl_i(cl, (k0 + j) & 63);
                vk[j] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (k0 + j < n) vk[j] = *reinterpret_cast<const float4 *>(vs + (int64_t)c * ld_v);
            }
            float sv[U];
#pragma unroll
            for (int j = 0; j < U; ++j) sv[j] = uq.x * vk[j].x + uq.y * vk[j].y + uq.z * vk[j].z + uq.w * vk[j].w;
#pragma unroll
            for (int m = U / 2, cnt = U; m >= 1; m >>= 1, cnt >>= 1) {
                const bool hi = (lh & m) != 0;
#pragma unroll
                for (int i = 0; i < cnt / 2; ++i) {
                    const float keep = hi ? sv[i + cnt / 2] : sv[i];
                    const float send = hi ? sv[i] : sv[i + cnt / 2];
                    sv[i] = keep + shfl_xor_f(send, m);
                }
            }
            float tot = sv[0];
#pragma unroll
            for (int m = U; m < HS; m <<= 1) tot += shfl_xor_f(tot, m);
            const int k = k0 + (lh & (U - 1));
            if (lh < U && k < n) out[(eid ? eid[base + k] : base + k) * h + head] = tot;
        }
    }
}

// Any shape: one thread per (edge, head).
__global__ void sddmm_dot_generic(int64_t n_rows, int h, int d, const int64_t *__restrict__ row_ptr,
                                  const int32_t *__restrict__ col, const int64_t *__restrict__ eid,
                                  const float *__restrict__ u, int64_t ld_u,
                                  const float *__restrict__ v, int64_t ld_v, float *__restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    for (int64_t t = lane; t < (e - b) * h; t += 64) {
        const int64_t p = b + t / h;
        const int j = (int)(t % h);
        const float *a = u + r * ld_u + (int64_t)j * d;
        const float *c = v + (int64_t)col[p] * ld_v + (int64_t)j * d;
        float s = 0.f;
        for (int k = 0; k < d; ++k) s = fmaf(a[k], c[k], s);
        out[(eid ? eid[p] : p) * h + j] = s;
    }
}

// ---------------------------------------------------------------- wave reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += shfl_xor_f(v, m);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, shfl_xor_f(v, m));
    return v;
}

// ---------------------------------------------------------------- copy_rhs reduce
__global__ __launch_bounds__(256) void segment_reduce_kernel(int64_t n_rows, int h,
                                                             const int64_t *__restrict__ row_ptr,
                                                             const int64_t *__restrict__ eid,
                                                             const float *__restrict__ x, int reduce,
                                                             float *__restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    for (int j = 0; j < h; ++j) {
        float a = reduce ? -INFINITY : 0.f;
        for (int64_t p = b + lane; p < e; p += 64) {
            const float t = x[(eid ? eid[p] : p) * h + j];
            a = reduce ? fmaxf(a, t) : a + t;
        }
        a = reduce ? wave_max(a) : wave_sum(a);
        if (lane == 0) out[r * h + j] = (b == e) ? 0.f : a;
    }
}

// ---------------------------------------------------------------- attention edge softmax
constexpr int kMaxHeads = 8;

// z = (alpha - m) / sqrt_d / 10, computed as the two divisions the reference writes.
__device__ __forceinline__ float att_exp(float a, float m, float sqrt_d) {
    return expf((a - m) / sqrt_d / 10.f);
}

// Edges whose keep value is 0 (dropped by dropout_sp_mat, model.py:4016-4028,
// which REMOVES them from the reference's graph) take no part in the row max /
// sum and get weight 0.
__device__ __forceinline__ bool kept(const float *__restrict__ keep, int64_t e) {
    return keep == nullptr || keep[e] != 0.f;
}

__global__ __launch_bounds__(256) void att_softmax_kernel(
    int64_t n_rows, int h, const int64_t *__restrict__ row_ptr, const int64_t *__restrict__ eid,
    const float *__restrict__ alpha, const float *__restrict__ keep, float sqrt_d, float *__restrict__ w,
    float *__restrict__ row_max, float *__restrict__ row_sum) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    float m[kMaxHeads], s[kMaxHeads];
#pragma unroll
    for (int j = 0; j < kMaxHeads; ++j) {
        m[j] = -INFINITY;
        s[j] = 0.f;
    }
    for (int64_t p = b + lane; p < e; p += 64) {
        const int64_t ed = eid ? eid[p] : p;
        if (!kept(keep, ed)) continue;
        const float *a = alpha + ed * h;
#pragma unroll
        for (int j = 0; j < kMaxHeads; ++j)
            if (j < h) m[j] = fmaxf(m[j], a[j]);
    }
#pragma unroll
    for (int j = 0; j < kMaxHeads; ++j)
        if (j < h) m[j] = wave_max(m[j]);
    for (int64_t p = b + lane; p < e; p += 64) {
        const int64_t ed = eid ? eid[p] : p;
        if (!kept(keep, ed)) continue;
        const float *a = alpha + ed * h;
#pragma unroll
        for (int j = 0; j < kMaxHeads; ++j)
            if (j < h) s[j] += att_exp(a[j], m[j], sqrt_d);
    }
#pragma unroll
    for (int j = 0; j < kMaxHeads; ++j)
        if (j < h) s[j] = wave_sum(s[j]);
    if (lane == 0 && b < e) {
        for (int j = 0; j < h; ++j) {
            if (row_max) row_max[r * h + j] = m[j];
            if (row_sum) row_sum[r * h + j] = s[j];
        }
    }
    for (int64_t p = b + lane; p < e; p += 64) {
        const int64_t ed = eid ? eid[p] : p;
        if (!kept(keep, ed)) {
            w[ed] = 0.f;
            continue;
        }
        const float *a = alpha + ed * h;
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < kMaxHeads; ++j)
            if (j < h) acc += att_exp(a[j], m[j], sqrt_d) / s[j];
        w[ed] = acc / (float)h;
    }
}

// d alpha[e,j] = a_ej (g_e/h - S_j) / (sqrt_d * 10),  S_j = sum_e a_ej g_e / h,
// a_ej = softmax weight of head j.  The path through the row max carries an
// exactly-zero gradient (softmax is shift invariant) and is omitted.
__global__ __launch_bounds__(256) void att_softmax_bwd_kernel(
    int64_t n_rows, int h, const int64_t *__restrict__ row_ptr, const int64_t *__restrict__ eid,
    const float *__restrict__ alpha, const float *__restrict__ keep, float sqrt_d, const float *__restrict__ row_max,
    const float *__restrict__ row_sum, const float *__restrict__ dw, float *__restrict__ dalpha) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    if (b == e) return;
    float m[kMaxHeads], s[kMaxHeads], S[kMaxHeads];
#pragma unroll
    for (int j = 0; j < kMaxHeads; ++j) {
        m[j] = (j < h) ? row_max[r * h + j] : 0.f;
        s[j] = (j < h) ? row_sum[r * h + j] : 1.f;
        S[j] = 0.f;
    }
    const float inv_h = 1.f / (float)h;
    for (int64_t p = b + lane; p < e; p += 64) {
        const int64_t ed = eid ? eid[p] : p;
        if (!kept(keep, ed)) continue;
        const float g = dw[ed] * inv_h;
#pragma unroll
        for (int j = 0; j < kMaxHeads; ++j)
            if (j < h) S[j] += att_exp(alpha[ed * h + j], m[j], sqrt_d) / s[j] * g;
    }
#pragma unroll
    for (int j = 0; j < kMaxHeads; ++j)
        if (j < h) S[j] = wave_sum(S[j]);
    const float c = sqrt_d * 10.f;
    for (int64_t p = b + lane; p < e; p += 64) {
        const int64_t ed = eid ? eid[p] : p;
        const bool k = kept(keep, ed);
        const float g = dw[ed] * inv_h;
#pragma unroll
        for (int j = 0; j < kMaxHeads; ++j)
            if (j < h) {
                const float a = k ? att_exp(alpha[ed * h + j], m[j], sqrt_d) / s[j] : 0.f;
                dalpha[ed * h + j] = a * (g - S[j]) / c;
            }
    }
}

// ---------------------------------------------------------------- grouped softmax (H heads, 16 lanes per row)
#ifndef IGR_SOFTMAX_R
#define IGR_SOFTMAX_R 4  // register-cached edges per lane at H <= 4 (H = 8: half); swept 2/4/8/16 on MI355X
#endif
// The feature graph's rows are short (a user row ~20 edges, an item row ~200):
// a wave per row leaves most lanes idle and pays a 64-lane reduction per head
// three times.  Here 16 lanes take a row (4 rows per wave); each lane keeps the
// alpha rows of its first R edges in registers (one read of alpha; edges past
// 16R, if any, are re-read), the exps are computed once, and the row max / sum
// are 4-step xor reductions inside the 16 lanes.
template <int H>
__device__ __forceinline__ void load_heads(const float *__restrict__ alpha, int64_t ed, float (&a)[H]) {
    if constexpr (H % 4 == 0) {
#pragma unroll
        for (int q = 0; q < H / 4; ++q) {
            const float4 v = *reinterpret_cast<const float4 *>(alpha + ed * H + 4 * q);
            a[4 * q] = v.x;
            a[4 * q + 1] = v.y;
            a[4 * q + 2] = v.z;
            a[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < H; ++j) a[j] = alpha[ed * H + j];
    }
}

template <int LPR>
__device__ __forceinline__ float gmax(float v) {
#pragma unroll
    for (int o = LPR / 2; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

template <int LPR>
__device__ __forceinline__ float gsum(float v) {
#pragma unroll
    for (int o = LPR / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int H, int R, int LPR>
__global__ __launch_bounds__(256) void att_softmax_g16_kernel(
    int64_t n_rows, const int64_t *__restrict__ row_ptr, const int64_t *__restrict__ eid,
    const float *__restrict__ alpha, const float *__restrict__ keep, float sqrt_d, float *__restrict__ w,
    float *__restrict__ row_max, float *__restrict__ row_sum, const int32_t *__restrict__ order) {
    // n_rows rows, or with `order` the n_rows rows it lists (the unsplit rows of the graph's
    // schedule, heaviest first; att_softmax_block_kernel takes the split ones)
    const int64_t idx = (int64_t)blockIdx.x * (256 / LPR) + threadIdx.x / LPR;
    const int sub = threadIdx.x % LPR;
    const bool live = idx < n_rows;  // every lane stays for the group shuffles
    const int64_t r = live ? (order ? (int64_t)order[idx] : idx) : 0;
    const int64_t b = live ? row_ptr[r] : 0, e = live ? row_ptr[r + 1] : 0;
    float a[R][H];
    bool k[R];
    float m[H], sm[H];
#pragma unroll
    for (int j = 0; j < H; ++j) m[j] = -INFINITY;
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const int64_t p = b + sub + LPR * t;
        k[t] = false;
        if (p < e) {
            const int64_t ed = eid ? eid[p] : p;
            k[t] = kept(keep, ed);
            if (k[t]) {
                load_heads<H>(alpha, ed, a[t]);
#pragma unroll
                for (int j = 0; j < H; ++j) m[j] = fmaxf(m[j], a[t][j]);
            }
        }
    }
    for (int64_t p = b + sub + LPR * R; p < e; p += LPR) {  // past the register cache
        const int64_t ed = eid ? eid[p] : p;
        if (!kept(keep, ed)) continue;
        float x[H];
        load_heads<H>(alpha, ed, x);
#pragma unroll
        for (int j = 0; j < H; ++j) m[j] = fmaxf(m[j], x[j]);
    }
#pragma unroll
    for (int j = 0; j < H; ++j) {
        m[j] = gmax<LPR>(m[j]);
        sm[j] = 0.f;
    }
#pragma unroll
    for (int t = 0; t < R; ++t)
        if (k[t]) {
#pragma unroll
            for (int j = 0; j < H; ++j) {
                a[t][j] = att_exp(a[t][j], m[j], sqrt_d);
                sm[j] += a[t][j];
            }
        }
    for (int64_t p = b + sub + LPR * R; p < e; p += LPR) {
        const int64_t ed = eid ? eid[p] : p;
        if (!kept(keep, ed)) continue;
        float x[H];
        load_heads<H>(alpha, ed, x);
#pragma unroll
        for (int j = 0; j < H; ++j) sm[j] += att_exp(x[j], m[j], sqrt_d);
    }
#pragma unroll
    for (int j = 0; j < H; ++j) sm[j] = gsum<LPR>(sm[j]);
    if (!live || b == e) return;
    if (sub == 0) {
#pragma unroll
        for (int j = 0; j < H; ++j) {
            if (row_max) row_max[r * H + j] = m[j];
            if (row_sum) row_sum[r * H + j] = sm[j];
        }
    }
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const int64_t p = b + sub + LPR * t;
        if (p < e) {
            const int64_t ed = eid ? eid[p] : p;
            float acc = 0.f;
            if (k[t]) {
#pragma unroll
                for (int j = 0; j < H; ++j) acc += a[t][j] / sm[j];
                acc /= (float)H;
            }
            w[ed] = acc;
        }
    }
    for (int64_t p = b + sub + LPR * R; p < e; p += LPR) {
        const int64_t ed = eid ? eid[p] : p;
        if (!kept(keep, ed)) {
            w[ed] = 0.f;
            continue;
        }
        float x[H];
        load_heads<H>(alpha, ed, x);
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < H; ++j) acc += att_exp(x[j], m[j], sqrt_d) / sm[j];
        w[ed] = acc / (float)H;
    }
}

template <int H, int R, int LPR>
__global__ __launch_bounds__(256) void att_softmax_bwd_g16_kernel(
    int64_t n_rows, const int64_t *__restrict__ row_ptr, const int64_t *__restrict__ eid,
    const float *__restrict__ alpha, const float *__restrict__ keep, float sqrt_d, const float *__restrict__ row_max,
    const float *__restrict__ row_sum, const float *__restrict__ dw, float *__restrict__ dalpha,
    const int32_t *__restrict__ order) {
    const int64_t idx = (int64_t)blockIdx.x * (256 / LPR) + threadIdx.x / LPR;
    const int sub = threadIdx.x % LPR;
    const bool live = idx < n_rows;
    const int64_t r = live ? (order ? (int64_t)order[idx] : idx) : 0;
    const int64_t b = live ? row_ptr[r] : 0, e = live ? row_ptr[r + 1] : 0;
    float m[H], s[H], S[H];
#pragma unroll
    for (int j = 0; j < H; ++j) {
        m[j] = live && b < e ? row_max[r * H + j] : 0.f;
        s[j] = live && b < e ? row_sum[r * H + j] : 1.f;
        S[j] = 0.f;
    }
    const float inv_h = 1.f / (float)H;
    float a[R][H], g[R];
    bool k[R];
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const int64_t p = b + sub + LPR * t;
        k[t] = false;
        g[t] = 0.f;
        if (p < e) {
            const int64_t ed = eid ? eid[p] : p;
            g[t] = dw[ed] * inv_h;
            k[t] = kept(keep, ed);
            if (k[t]) {
                load_heads<H>(alpha, ed, a[t]);
#pragma unroll
                for (int j = 0; j < H; ++j) {
                    a[t][j] = att_exp(a[t][j], m[j], sqrt_d) / s[j];
                    S[j] += a[t][j] * g[t];
                }
            }
        }
    }
    for (int64_t p = b + sub + LPR * R; p < e; p += LPR) {
        const int64_t ed = eid ? eid[p] : p;
        if (!kept(keep, ed)) continue;
        const float gg = dw[ed] * inv_h;
        float x[H];
        load_heads<H>(alpha, ed, x);
#pragma unroll
        for (int j = 0; j < H; ++j) S[j] += att_exp(x[j], m[j], sqrt_d) / s[j] * gg;
    }
#pragma unroll
    for (int j = 0; j < H; ++j) S[j] = gsum<LPR>(S[j]);
    if (!live || b == e) return;
    const float c = sqrt_d * 10.f;
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const int64_t p = b + sub + LPR * t;
        if (p < e) {
            const int64_t ed = eid ? eid[p] : p;
#pragma unroll
            for (int j = 0; j < H; ++j) dalpha[ed * H + j] = k[t] ? a[t][j] * (g[t] - S[j]) / c : 0.f;
        }
    }
    for (int64_t p = b + sub + LPR * R; p < e; p += LPR) {
        const int64_t ed = eid ? eid[p] : p;
        const bool kk = kept(keep, ed);
        const float gg = dw[ed] * inv_h;
        float x[H];
        if (kk) load_heads<H>(alpha, ed, x);
#pragma unroll
        for (int j = 0; j < H; ++j) dalpha[ed * H + j] = kk ? att_exp(x[j], m[j], sqrt_d) / s[j] * (gg - S[j]) / c : 0.f;
    }
}

// ---------------------------------------------------------------- split rows: a workgroup per row
// A hub row (an item most users rated, a general-feature row) is thousands of edges long:
// as one lane group's loop it outlasts the rest of the launch.  The rows the graph's
// schedule splits (degree above its threshold) go to these kernels instead, a whole
// workgroup each: per-thread partials over a strided walk of the row, a fixed xor tree
// inside each wave, then the waves' results combined in wave order through LDS - the
// same value in every thread, the same bits on every run.  (MovieLens-1M-shaped feature
// graph, 4 heads, no register cache: 31.5 us at 512 threads, 38.4 at 256, 72.8 at 1024; a
// wave each for the split rows up to 1024 edges and workgroups for the longer ones: 63 us.)
// Also tried: a wave each for the split rows up to 256 edges (whole row in registers) and
// workgroups for the longer ones only - forward 37 us against 38, backward 43 against 37.
#ifndef IGR_SOFTMAX_BLOCK_R
#define IGR_SOFTMAX_BLOCK_R 4
#endif
constexpr int kSoftmaxBlockR = IGR_SOFTMAX_BLOCK_R;  // register-cached edges per thread
#ifndef IGR_SOFTMAX_BLOCK
#define IGR_SOFTMAX_BLOCK 512
#endif
constexpr int kSoftmaxBlock = IGR_SOFTMAX_BLOCK;

template <int H, int NT, bool MAX>
__device__ __forceinline__ void block_reduce(float (&v)[H], float (*red)[H]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < H; ++j) v[j] = MAX ? gmax<64>(v[j]) : gsum<64>(v[j]);
    __syncthreads();  // red may still be read from the previous reduction
    if (lane == 0) {
#pragma unroll
        for (int j = 0; j < H; ++j) red[wave][j] = v[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < H; ++j) {
        float a = red[0][j];
#pragma unroll
        for (int k = 1; k < NT / 64; ++k) a = MAX ? fmaxf(a, red[k][j]) : a + red[k][j];
        v[j] = a;
    }
}

template <int H, int NT, int R>
__global__ __launch_bounds__(NT) void att_softmax_block_kernel(
    int64_t n_split, const int32_t *__restrict__ split_row, const int64_t *__restrict__ row_ptr,
    const int64_t *__restrict__ eid, const float *__restrict__ alpha, const float *__restrict__ keep, float sqrt_d,
    float *__restrict__ w, float *__restrict__ row_max, float *__restrict__ row_sum) {
    __shared__ float red[NT / 64][H];
    const int64_t r = split_row[blockIdx.x];
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    // the first NT * R edges of the row stay in registers (one read of alpha, all of a
    // thread's loads in flight together); a longer row re-reads its tail in every pass
    float a[R][H], m[H], sm[H];
    int64_t ed[R];
    bool k[R];
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const int64_t p = b + threadIdx.x + (int64_t)NT * t;
        ed[t] = p < e ? (eid ? eid[p] : p) : -1;
    }
#pragma unroll
    for (int t = 0; t < R; ++t) {
        k[t] = ed[t] >= 0 && kept(keep, ed[t]);
        if (k[t]) load_heads<H>(alpha, ed[t], a[t]);
    }
#pragma unroll
    for (int j = 0; j < H; ++j) m[j] = -INFINITY;
#pragma unroll
    for (int t = 0; t < R; ++t)
        if (k[t]) {
#pragma unroll
            for (int j = 0; j < H; ++j) m[j] = fmaxf(m[j], a[t][j]);
        }
    for (int64_t p = b + threadIdx.x + (int64_t)NT * R; p < e; p += NT) {
        const int64_t ee = eid ? eid[p] : p;
        if (!kept(keep, ee)) continue;
        float x[H];
        load_heads<H>(alpha, ee, x);
#pragma unroll
        for (int j = 0; j < H; ++j) m[j] = fmaxf(m[j], x[j]);
    }
    block_reduce<H, NT, true>(m, red);
#pragma unroll
    for (int j = 0; j < H; ++j) sm[j] = 0.f;
#pragma unroll
    for (int t = 0; t < R; ++t)
        if (k[t]) {
#pragma unroll
            for (int j = 0; j < H; ++j) {
                a[t][j] = att_exp(a[t][j], m[j], sqrt_d);
                sm[j] += a[t][j];
            }
        }
    for (int64_t p = b + threadIdx.x + (int64_t)NT * R; p < e; p += NT) {
        const int64_t ee = eid ? eid[p] : p;
        if (!kept(keep, ee)) continue;
        float x[H];
        load_heads<H>(alpha, ee, x);
#pragma unroll
        for (int j = 0; j < H; ++j) sm[j] += att_exp(x[j], m[j], sqrt_d);
    }
    block_reduce<H, NT, false>(sm, red);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int j = 0; j < H; ++j) {
            if (row_max) row_max[r * H + j] = m[j];
            if (row_sum) row_sum[r * H + j] = sm[j];
        }
    }
#pragma unroll
    for (int t = 0; t < R; ++t)
        if (ed[t] >= 0) {
            float acc = 0.f;
            if (k[t]) {
#pragma unroll
                for (int j = 0; j < H; ++j) acc += a[t][j] / sm[j];
                acc /= (float)H;
            }
            w[ed[t]] = acc;
        }
    for (int64_t p = b + threadIdx.x + (int64_t)NT * R; p < e; p += NT) {
        const int64_t ee = eid ? eid[p] : p;
        if (!kept(keep, ee)) {
            w[ee] = 0.f;
            continue;
        }
        float x[H];
        load_heads<H>(alpha, ee, x);
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < H; ++j) acc += att_exp(x[j], m[j], sqrt_d) / sm[j];
        w[ee] = acc / (float)H;
    }
}

template <int H, int NT, int R>
__global__ __launch_bounds__(NT) void att_softmax_bwd_block_kernel(
    int64_t n_split, const int32_t *__restrict__ split_row, const int64_t *__restrict__ row_ptr,
    const int64_t *__restrict__ eid, const float *__restrict__ alpha, const float *__restrict__ keep, float sqrt_d,
    const float *__restrict__ row_max, const float *__restrict__ row_sum, const float *__restrict__ dw,
    float *__restrict__ dalpha) {
    __shared__ float red[NT / 64][H];
    const int64_t r = split_row[blockIdx.x];
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    float m[H], s[H], S[H];
#pragma unroll
    for (int j = 0; j < H; ++j) {
        m[j] = row_max[r * H + j];
        s[j] = row_sum[r * H + j];
        S[j] = 0.f;
    }
    const float inv_h = 1.f / (float)H;
    float a[R][H], g[R];
    int64_t ed[R];
    bool k[R];
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const int64_t p = b + threadIdx.x + (int64_t)NT * t;
        ed[t] = p < e ? (eid ? eid[p] : p) : -1;
    }
#pragma unroll
    for (int t = 0; t < R; ++t) {
        k[t] = ed[t] >= 0 && kept(keep, ed[t]);
        g[t] = ed[t] >= 0 ? dw[ed[t]] * inv_h : 0.f;
        if (k[t]) load_heads<H>(alpha, ed[t], a[t]);
    }
#pragma unroll
    for (int t = 0; t < R; ++t)
        if (k[t]) {
#pragma unroll
            for (int j = 0; j < H; ++j) {
                a[t][j] = att_exp(a[t][j], m[j], sqrt_d) / s[j];
                S[j] += a[t][j] * g[t];
            }
        }
    for (int64_t p = b + threadIdx.x + (int64_t)NT * R; p < e; p += NT) {
        const int64_t ee = eid ? eid[p] : p;
        if (!kept(keep, ee)) continue;
        const float gg = dw[ee] * inv_h;
        float x[H];
        load_heads<H>(alpha, ee, x);
#pragma unroll
        for (int j = 0; j < H; ++j) S[j] += att_exp(x[j], m[j], sqrt_d) / s[j] * gg;
    }
    block_reduce<H, NT, false>(S, red);
    const float c = sqrt_d * 10.f;
#pragma unroll
    for (int t = 0; t < R; ++t)
        if (ed[t] >= 0) {
#pragma unroll
            for (int j = 0; j < H; ++j) dalpha[ed[t] * H + j] = k[t] ? a[t][j] * (g[t] - S[j]) / c : 0.f;
        }
    for (int64_t p = b + threadIdx.x + (int64_t)NT * R; p < e; p += NT) {
        const int64_t ee = eid ? eid[p] : p;
        const bool kk = kept(keep, ee);
        const float gg = dw[ee] * inv_h;
        float x[H];
        if (kk) load_heads<H>(alpha, ee, x);
#pragma unroll
        for (int j = 0; j < H; ++j) dalpha[ee * H + j] = kk ? att_exp(x[j], m[j], sqrt_d) / s[j] * (gg - S[j]) / c : 0.f;
    }
}

// ---------------------------------------------------------------- split rows by chunks (with a workspace)
// With a workspace the split rows go chunk by chunk instead, a wave per chunk of the
// schedule, so a row of any length is spread over the chip (a workgroup per row walks a
// 2 M-edge hub row for milliseconds).  Forward: (1) per chunk the max m_c and
// s_c = sum exp((a - m_c) / t) per head; (2) per split row m = max_c m_c and
// s = sum_c s_c exp((m_c - m) / t), the chunks in order across the lanes and a fixed xor
// tree (t = sqrt_d * 10, the temperature of att_exp); (3) per chunk the weights.  Backward:
// per-chunk sums of a * g, their per-row totals written back over every chunk slot of the
// row, then per chunk the gradient.  Slots: 2 H floats per chunk forward, H backward.
template <int H>
__global__ __launch_bounds__(256) void att_softmax_chunk_stats_kernel(
    RowPlan plan, const int64_t *__restrict__ row_ptr, const int64_t *__restrict__ eid,
    const float *__restrict__ alpha, const float *__restrict__ keep, float sqrt_d, float *__restrict__ ws) {
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= plan.n_chunks) return;
    const int lane = threadIdx.x & 63;
    const int64_t b = plan.chunk_beg[c], e = min(b + plan.chunk_edges, row_ptr[plan.chunk_row[c] + 1]);
    float m[H], sm[H];
#pragma unroll
    for (int j = 0; j < H; ++j) m[j] = -INFINITY;
    for (int64_t p = b + lane; p < e; p += 64) {
        const int64_t ee = eid ? eid[p] : p;
        if (!kept(keep, ee)) continue;
        float x[H];
        load_heads<H>(alpha, ee, x);
#pragma unroll
        for (int j = 0; j < H; ++j) m[j] = fmaxf(m[j], x[j]);
    }
#pragma unroll
    for (int j = 0; j < H; ++j) {
        m[j] = gmax<64>(m[j]);
        sm[j] = 0.f;
    }
    for (int64_t p = b + lane; p < e; p += 64) {
        const int64_t ee = eid ? eid[p] : p;
        if (!kept(keep, ee)) continue;
        float x[H];
        load_heads<H>(alpha, ee, x);
#pragma unroll
        for (int j = 0; j < H; ++j) sm[j] += att_exp(x[j], m[j], sqrt_d);
    }
#pragma unroll
    for (int j = 0; j < H; ++j) sm[j] = gsum<64>(sm[j]);
    if (lane == 0) {
#pragma unroll
        for (int j = 0; j < H; ++j) {
            ws[c * (2 * H) + j] = m[j];
            ws[c * (2 * H) + H + j] = sm[j];
        }
    }
}

template <int H>
__global__ __launch_bounds__(256) void att_softmax_row_stats_kernel(
    int64_t n_split, const int32_t *__restrict__ split_row, const int64_t *__restrict__ split_ptr,
    const float *__restrict__ ws, float sqrt_d, float *__restrict__ row_max, float *__restrict__ row_sum) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n_split) return;
    const int lane = threadIdx.x & 63;
    const int64_t b = split_ptr[i], e = split_ptr[i + 1];
    float m[H], sm[H];
#pragma unroll
    for (int j = 0; j < H; ++j) m[j] = -INFINITY;
    for (int64_t c = b + lane; c < e; c += 64) {
#pragma unroll
        for (int j = 0; j < H; ++j) m[j] = fmaxf(m[j], ws[c * (2 * H) + j]);
    }
#pragma unroll
    for (int j = 0; j < H; ++j) {
        m[j] = gmax<64>(m[j]);
        sm[j] = 0.f;
    }
    for (int64_t c = b + lane; c < e; c += 64) {
#pragma unroll
        for (int j = 0; j < H; ++j) {
            const float mc = ws[c * (2 * H) + j];
            if (mc != -INFINITY) sm[j] += ws[c * (2 * H) + H + j] * att_exp(mc, m[j], sqrt_d);  // a chunk with no kept edge adds nothing
        }
    }
#pragma unroll
    for (int j = 0; j < H; ++j) sm[j] = gsum<64>(sm[j]);
    if (lane == 0) {
        const int64_t r = split_row[i];
#pragma unroll
        for (int j = 0; j < H; ++j) {
            row_max[r * H + j] = m[j];
            row_sum[r * H + j] = sm[j];
        }
    }
}

template <int H>
__global__ __launch_bounds__(256) void att_softmax_chunk_write_kernel(
    RowPlan plan, const int64_t *__restrict__ row_ptr, const int64_t *__restrict__ eid,
    const float *__restrict__ alpha, const float *__restrict__ keep, float sqrt_d,
    const float *__restrict__ row_max, const float *__restrict__ row_sum, float *__restrict__ w) {
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= plan.n_chunks) return;
    const int lane = threadIdx.x & 63;
    const int64_t r = plan.chunk_row[c];
    const int64_t b = plan.chunk_beg[c], e = min(b + plan.chunk_edges, row_ptr[r + 1]);
    float m[H], sm[H];
#pragma unroll
    for (int j = 0; j < H; ++j) {
        m[j] = row_max[r * H + j];
        sm[j] = row_sum[r * H + j];
    }
    for (int64_t p = b + lane; p < e; p += 64) {
        const int64_t ee = eid ? eid[p] : p;
        if (!kept(keep, ee)) {
            w[ee] = 0.f;
            continue;
        }
        float x[H];
        load_heads<H>(alpha, ee, x);
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < H; ++j) acc += att_exp(x[j], m[j], sqrt_d) / sm[j];
        w[ee] = acc / (float)H;
    }
}

template <int H>
__global__ __launch_bounds__(256) void att_softmax_bwd_chunk_sums_kernel(
    RowPlan plan, const int64_t *__restrict__ row_ptr, const int64_t *__restrict__ eid,
    const float *__restrict__ alpha, const float *__restrict__ keep, float sqrt_d,
    const float *__restrict__ row_max, const float *__restrict__ row_sum, const float *__restrict__ dw,
    float *__restrict__ ws) {
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= plan.n_chunks) return;
    const int lane = threadIdx.x & 63;
    const int64_t r = plan.chunk_row[c];
    const int64_t b = plan.chunk_beg[c], e = min(b + plan.chunk_edges, row_ptr[r + 1]);
    float m[H], s[H], S[H];
#pragma unroll
    for (int j = 0; j < H; ++j) {
        m[j] = row_max[r * H + j];
        s[j] = row_sum[r * H + j];
        S[j] = 0.f;
    }
    const float inv_h = 1.f / (float)H;
    for (int64_t p = b + lane; p < e; p += 64) {
        const int64_t ee = eid ? eid[p] : p;
        if (!kept(keep, ee)) continue;
        const float gg = dw[ee] * inv_h;
        float x[H];
        load_heads<H>(alpha, ee, x);
#pragma unroll
        for (int j = 0; j < H; ++j) S[j] += att_exp(x[j], m[j], sqrt_d) / s[j] * gg;
    }
#pragma unroll
    for (int j = 0; j < H; ++j) S[j] = gsum<64>(S[j]);
    if (lane == 0) {
#pragma unroll
        for (int j = 0; j < H; ++j) ws[c * H + j] = S[j];
    }
}

// ws[c, :] <- the sum over the row's chunks of ws[c', :], for every chunk c of the row
template <int H>
__global__ __launch_bounds__(256) void att_softmax_bwd_row_sums_kernel(int64_t n_split,
                                                                       const int64_t *__restrict__ split_ptr,
                                                                       float *__restrict__ ws) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n_split) return;
    const int lane = threadIdx.x & 63;
    const int64_t b = split_ptr[i], e = split_ptr[i + 1];
    float S[H];
#pragma unroll
    for (int j = 0; j < H; ++j) S[j] = 0.f;
    for (int64_t c = b + lane; c < e; c += 64) {
#pragma unroll
        for (int j = 0; j < H; ++j) S[j] += ws[c * H + j];
    }
#pragma unroll
    for (int j = 0; j < H; ++j) S[j] = gsum<64>(S[j]);  // every lane holds the total before any slot is overwritten
    for (int64_t c = b + lane; c < e; c += 64) {
#pragma unroll
        for (int j = 0; j < H; ++j) ws[c * H + j] = S[j];
    }
}

template <int H>
__global__ __launch_bounds__(256) void att_softmax_bwd_chunk_write_kernel(
    RowPlan plan, const int64_t *__restrict__ row_ptr, const int64_t *__restrict__ eid,
    const float *__restrict__ alpha, const float *__restrict__ keep, float sqrt_d,
    const float *__restrict__ row_max, const float *__restrict__ row_sum, const float *__restrict__ dw,
    const float *__restrict__ ws, float *__restrict__ dalpha) {
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= plan.n_chunks) return;
    const int lane = threadIdx.x & 63;
    const int64_t r = plan.chunk_row[c];
    const int64_t b = plan.chunk_beg[c], e = min(b + plan.chunk_edges, row_ptr[r + 1]);
    float m[H], s[H], S[H];
#pragma unroll
    for (int j = 0; j < H; ++j) {
        m[j] = row_max[r * H + j];
        s[j] = row_sum[r * H + j];
        S[j] = ws[c * H + j];
    }
    const float inv_h = 1.f / (float)H, cc = sqrt_d * 10.f;
    for (int64_t p = b + lane; p < e; p += 64) {
        const int64_t ee = eid ? eid[p] : p;
        const bool kk = kept(keep, ee);
        const float gg = dw[ee] * inv_h;
        float x[H];
        if (kk) load_heads<H>(alpha, ee, x);
#pragma unroll
        for (int j = 0; j < H; ++j) dalpha[ee * H + j] = kk ? att_exp(x[j], m[j], sqrt_d) / s[j] * (gg - S[j]) / cc : 0.f;
    }
}

// gspmm copy_rhs sum / max with 16 lanes per row and all H heads per lane
// (the segment_reduce_kernel above takes a wave per row and a pass per head).
template <int H, int LPR>
__global__ __launch_bounds__(256) void segment_reduce_g16_kernel(int64_t n_rows, const int64_t *__restrict__ row_ptr,
                                                                 const int64_t *__restrict__ eid,
                                                                 const float *__restrict__ x, int reduce,
                                                                 float *__restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * (256 / LPR) + threadIdx.x / LPR;
    const int sub = threadIdx.x % LPR;
    const bool live = r < n_rows;
    const int64_t b = live ? row_ptr[r] : 0, e = live ? row_ptr[r + 1] : 0;
    float a[H];
#pragma unroll
    for (int j = 0; j < H; ++j) a[j] = reduce ? -INFINITY : 0.f;
    for (int64_t p = b + sub; p < e; p += LPR) {
        float v[H];
        load_heads<H>(x, eid ? eid[p] : p, v);
#pragma unroll
        for (int j = 0; j < H; ++j) a[j] = reduce ? fmaxf(a[j], v[j]) : a[j] + v[j];
    }
#pragma unroll
    for (int j = 0; j < H; ++j) a[j] = reduce ? gmax<LPR>(a[j]) : gsum<LPR>(a[j]);
    if (live && sub == 0) {
#pragma unroll
        for (int j = 0; j < H; ++j) out[r * H + j] = (b == e) ? 0.f : a[j];
    }
}

// ---------------------------------------------------------------- value kernels
__global__ void edge_dropout_kernel(int64_t n, const float *__restrict__ val,
                                    const float *__restrict__ rand, float keep,
                                    float *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        // random_tensor = (1 - p) + U; mask = floor(random_tensor) (model.py:4019-4021)
        const bool k = floorf(keep + rand[i]) != 0.f;
        out[i] = k ? val[i] / keep : 0.f;
    }
}

__global__ void feat_values_kernel(int64_t n_rows, const float *__restrict__ row_sum, float ex,
                                   float *__restrict__ out) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_rows;
         r += (int64_t)gridDim.x * blockDim.x) {
        const float x = row_sum[r];
        // torch.pow(t, -0.5) lowers to rsqrt (1 / sqrt); other exponents to pow
        const float v = (ex == -0.5f) ? 1.f / sqrtf(x) : powf(x, ex);
        out[r] = v;
    }
}

// The per-edge form: thread per edge, its row found by bisection of row_ptr (a thread per
// row would walk a hub row's edges alone: 12 ms for a 2 M-edge row).
__global__ void feat_values_edges_kernel(int64_t n_rows, const int64_t *__restrict__ row_ptr,
                                         const float *__restrict__ row_sum, float ex, float *__restrict__ out) {
    const int64_t nnz = row_ptr[n_rows];
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = n_rows;  // the last row with row_ptr[r] <= p
        while (hi - lo > 1) {
            const int64_t mid = (lo + hi) >> 1;
            if (row_ptr[mid] <= p) lo = mid;
            else hi = mid;
        }
        const float x = row_sum[lo];
        out[p] = (ex == -0.5f) ? 1.f / sqrtf(x) : powf(x, ex);
    }
}

static unsigned grid_for(int64_t n, int block) {
    int64_t g = (n + block - 1) / block;
    if (g > 8192) g = 8192;
    return (unsigned)(g < 1 ? 1 : g);
}

static bool pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }

// Rows long enough on average that 64 lanes per row beat 16 (a 16-lane group
// walking ~200 edges serially leaves the chip latency-bound: ML-1M's feature
// graph; the synthetic feature graph's ~37-edge rows stay on 16 lanes).
#ifndef IGR_WIDE_ROW_DEG
#define IGR_WIDE_ROW_DEG 96
#endif
static bool wide_rows(const igr_csr *g) { return g->nnz >= (int64_t)IGR_WIDE_ROW_DEG * g->n_rows; }

// The graph's schedule lists its unsplit rows (order) and its split rows (split_row), and
// some row is split: the row kernels then take the two lists separately.
static bool split_plan(const igr_csr *g) {
    return g->n_split > 0 && g->split_row && (g->n_order == 0 || g->order) && g->n_order + g->n_split == g->n_rows;
}

struct SddmmArgs {
    const igr_csr *g;
    int h, d;
    const float *u;
    int64_t ld_u;
    const float *v;
    int64_t ld_v;
    float *out;
    int64_t row_blocks;
    unsigned grid;
    hipStream_t st;
};

template <int T, int HS>
static void launch_sddmm(const SddmmArgs &a) {
    if constexpr (HS <= T / 4)  // a head segment lies inside one edge group
        hipLaunchKernelGGL((sddmm_dot_kernel<T, HS>), dim3(a.grid), dim3(256), 0, a.st, a.g->n_rows, a.h, a.d,
                           a.g->row_ptr, a.g->col_idx, a.g->edge_id, a.u, a.ld_u, a.v, a.ld_v, a.out,
                           a.row_blocks);
}

// TOT floats per pass; d/4 = lanes per head (a power of two <= TOT/4, checked by the caller)
template <int T>
static void launch_sddmm_t(const SddmmArgs &a) {
    switch (a.d / 4) {
        case 1: launch_sddmm<T, 1>(a); break;
        case 2: launch_sddmm<T, 2>(a); break;
        case 4: launch_sddmm<T, 4>(a); break;
        case 8: launch_sddmm<T, 8>(a); break;
        case 16: launch_sddmm<T, 16>(a); break;
        case 32: launch_sddmm<T, 32>(a); break;
        default: launch_sddmm<T, 64>(a); break;
    }
}

}  // namespace igr

using namespace igr;

extern "C" int igr_sddmm_dot_f32(const igr_csr *g, int32_t h, int32_t d, const float *u,
                                 int64_t ld_u, const float *v, int64_t ld_v, float *out,
                                 void *stream) {
    return guarded("igr_sddmm_dot_f32", [&]() -> int {
        const char *fn = "igr_sddmm_dot_f32";
        if (!g || h <= 0 || d <= 0) return arg_error(fn, "bad graph / h / d");
        if (ld_u < (int64_t)h * d || ld_v < (int64_t)h * d) return arg_error(fn, "leading dimension < h*d");
        if (g->n_rows == 0 || g->nnz == 0) return IGR_OK;
        // one head: the same sums as the shared-source kernel (one d-float source row per edge),
        // whose gathers are unconditional and whose lane sums are DPP adds
        if (h == 1 && (d == 32 || d == 64 || d == 128 || d == 256) && ld_u % 4 == 0 && ld_v % 4 == 0 &&
            ld_v <= 2147483647 && aligned16(u) && aligned16(v))
            return igr_sddmm_shared_f32(g, 1, d, u, ld_u, v, ld_v, out, stream);
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const int64_t row_blocks = (g->n_rows + 3) / 4;
        const unsigned blocks = (unsigned)row_blocks;
        const bool vec = (d % 4 == 0) && pow2(d / 4) && ld_u % 4 == 0 && ld_v % 4 == 0 &&
                         aligned16(u) && aligned16(v);
        // head split: one head's slice of v fits an XCD's 4 MB L2, the whole table does not
        constexpr double kL2 = 3.0 * (1 << 20);
        const double slice = (double)g->n_cols * d * 4;
#ifndef IGR_SDDMM_SPLIT
#define IGR_SDDMM_SPLIT 1
#endif
        const bool split = IGR_SDDMM_SPLIT && vec && h > 1 && slice <= kL2 && slice * h > kL2 &&
                           (d == 32 || d == 64 || d == 128 || d == 256);
        const int tot = split ? d : h * d;
        const unsigned grid = split ? (unsigned)(row_blocks * h) : blocks;
        const SddmmArgs a{g, h, d, u, ld_u, v, ld_v, out, row_blocks, grid, st};
        if (vec && tot == 64) launch_sddmm_t<64>(a);
        else if (vec && tot == 128) launch_sddmm_t<128>(a);
        else if (vec && tot == 256) launch_sddmm_t<256>(a);
        else if (vec && tot == 32) launch_sddmm_t<32>(a);
        else
            hipLaunchKernelGGL(sddmm_dot_generic, dim3(blocks), dim3(256), 0, st, g->n_rows, h, d,
                               g->row_ptr, g->col_idx, g->edge_id, u, ld_u, v, ld_v, out);
        return launch_status(fn);
    });
}

extern "C" int igr_segment_reduce_f32(const igr_csr *g, int32_t h, const float *x, int32_t reduce,
                                      float *out, void *stream) {
    return guarded("igr_segment_reduce_f32", [&]() -> int {
        const char *fn = "igr_segment_reduce_f32";
        if (!g || h <= 0) return arg_error(fn, "bad graph / h");
        if (reduce != 0 && reduce != 1) return arg_error(fn, "reduce must be 0 (sum) or 1 (max)");
        if (g->n_rows == 0) return IGR_OK;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const bool wide = wide_rows(g);
        const dim3 g16((unsigned)((g->n_rows + 15) / 16)), g64((unsigned)((g->n_rows + 3) / 4));
        const bool vec = (reinterpret_cast<uintptr_t>(x) & 15u) == 0;
#define IGR_SR(HH)                                                                                                \
    if (wide)                                                                                                     \
        hipLaunchKernelGGL((segment_reduce_g16_kernel<HH, 64>), g64, dim3(256), 0, st, g->n_rows, g->row_ptr,     \
                           g->edge_id, x, reduce, out);                                                           \
    else                                                                                                          \
        hipLaunchKernelGGL((segment_reduce_g16_kernel<HH, 16>), g16, dim3(256), 0, st, g->n_rows, g->row_ptr,     \
                           g->edge_id, x, reduce, out)
        if (h == 1) IGR_SR(1);
        else if (h == 2) IGR_SR(2);
        else if (h == 4 && vec) IGR_SR(4);
        else if (h == 8 && vec) IGR_SR(8);
        else
            hipLaunchKernelGGL(segment_reduce_kernel, dim3((unsigned)((g->n_rows + 3) / 4)), dim3(256),
                               0, st, g->n_rows, h, g->row_ptr, g->edge_id, x, reduce, out);
#undef IGR_SR
        return launch_status(fn);
    });
}

extern "C" int igr_att_softmax_f32(const igr_csr *g, int32_t h, const float *alpha, const float *keep,
                                   float sqrt_d, float *w, float *row_max, float *row_sum, void *stream) {
    return igr_att_softmax_ws_f32(g, h, alpha, keep, sqrt_d, w, row_max, row_sum, nullptr, 0, stream);
}

extern "C" int64_t igr_att_softmax_workspace_size(const igr_csr *g, int32_t h) {
    if (!g || h <= 0 || g->n_chunks <= 0) return 0;
    return g->n_chunks * (int64_t)(2 * h) * (int64_t)sizeof(float);
}

extern "C" int igr_att_softmax_ws_f32(const igr_csr *g, int32_t h, const float *alpha, const float *keep,
                                      float sqrt_d, float *w, float *row_max, float *row_sum, float *workspace,
                                      int64_t workspace_bytes, void *stream) {
    return guarded("igr_att_softmax_ws_f32", [&]() -> int {
        const char *fn = "igr_att_softmax_ws_f32";
        if (!g || h <= 0 || h > kMaxHeads) return arg_error(fn, "h must be in [1, 8]");
        if (workspace && workspace_bytes < igr_att_softmax_workspace_size(g, h))
            return arg_error(fn, "workspace smaller than igr_att_softmax_workspace_size");
        // the chunked path hands the row max / sum from its second launch to its third
        const bool chunked = workspace != nullptr && row_max != nullptr && row_sum != nullptr && has_row_plan(g) &&
                             g->n_chunks > 0 && g->split_ptr != nullptr;
        if (g->n_rows == 0) return IGR_OK;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const bool wide = wide_rows(g);
        // with a schedule that splits rows: the unsplit rows by lane groups, heaviest first,
        // and every split row by a workgroup of its own
        const bool planned = split_plan(g);
        const int64_t nr = planned ? g->n_order : g->n_rows;
        const int32_t *order = planned ? g->order : nullptr;
        const dim3 g16((unsigned)((nr + 15) / 16)), g64((unsigned)((nr + 3) / 4));
        const bool vec = (reinterpret_cast<uintptr_t>(alpha) & 15u) == 0;
#define IGR_SM(HH, RR)                                                                                            \
    do {                                                                                                          \
        if (nr > 0) {                                                                                             \
            if (wide)                                                                                             \
                hipLaunchKernelGGL((att_softmax_g16_kernel<HH, RR, 64>), g64, dim3(256), 0, st, nr, g->row_ptr,  \
                                   g->edge_id, alpha, keep, sqrt_d, w, row_max, row_sum, order);                 \
            else                                                                                                  \
                hipLaunchKernelGGL((att_softmax_g16_kernel<HH, RR, 16>), g16, dim3(256), 0, st, nr, g->row_ptr,  \
                                   g->edge_id, alpha, keep, sqrt_d, w, row_max, row_sum, order);                 \
        }                                                                                                         \
        if (planned && chunked) {                                                                                 \
            const dim3 gc((unsigned)((g->n_chunks + 3) / 4)), gs((unsigned)((g->n_split + 3) / 4));               \
            hipLaunchKernelGGL((att_softmax_chunk_stats_kernel<HH>), gc, dim3(256), 0, st, row_plan_of(g),        \
                               g->row_ptr, g->edge_id, alpha, keep, sqrt_d, workspace);                           \
            hipLaunchKernelGGL((att_softmax_row_stats_kernel<HH>), gs, dim3(256), 0, st, g->n_split,              \
                               g->split_row, g->split_ptr, workspace, sqrt_d, row_max, row_sum);                  \
            hipLaunchKernelGGL((att_softmax_chunk_write_kernel<HH>), gc, dim3(256), 0, st, row_plan_of(g),        \
                               g->row_ptr, g->edge_id, alpha, keep, sqrt_d, row_max, row_sum, w);                 \
        } else if (planned)                                                                                       \
            hipLaunchKernelGGL((att_softmax_block_kernel<HH, kSoftmaxBlock, kSoftmaxBlockR>),                     \
                               dim3((unsigned)g->n_split), dim3(kSoftmaxBlock), 0, st, g->n_split, g->split_row,  \
                               g->row_ptr, g->edge_id, alpha, keep, sqrt_d, w, row_max, row_sum);                 \
    } while (0)
        if (h == 1) IGR_SM(1, IGR_SOFTMAX_R);
        else if (h == 2) IGR_SM(2, IGR_SOFTMAX_R);
        else if (h == 4 && vec) IGR_SM(4, IGR_SOFTMAX_R);
        else if (h == 8 && vec) IGR_SM(8, (IGR_SOFTMAX_R + 1) / 2);
        else  // other head counts: every row by one wave
            hipLaunchKernelGGL(att_softmax_kernel, dim3((unsigned)((g->n_rows + 3) / 4)), dim3(256), 0,
                               st, g->n_rows, h, g->row_ptr, g->edge_id, alpha, keep, sqrt_d, w, row_max,
                               row_sum);
#undef IGR_SM
        return launch_status(fn);
    });
}

extern "C" int igr_att_softmax_bwd_f32(const igr_csr *g, int32_t h, const float *alpha,
                                       const float *keep, float sqrt_d, const float *row_max,
                                       const float *row_sum, const float *dw, float *dalpha, void *stream) {
    return igr_att_softmax_bwd_ws_f32(g, h, alpha, keep, sqrt_d, row_max, row_sum, dw, dalpha, nullptr, 0, stream);
}

extern "C" int igr_att_softmax_bwd_ws_f32(const igr_csr *g, int32_t h, const float *alpha, const float *keep,
                                          float sqrt_d, const float *row_max, const float *row_sum, const float *dw,
                                          float *dalpha, float *workspace, int64_t workspace_bytes, void *stream) {
    return guarded("igr_att_softmax_bwd_ws_f32", [&]() -> int {
        const char *fn = "igr_att_softmax_bwd_ws_f32";
        if (!g || h <= 0 || h > kMaxHeads) return arg_error(fn, "h must be in [1, 8]");
        if (!row_max || !row_sum) return arg_error(fn, "row_max / row_sum required");
        if (workspace && workspace_bytes < igr_att_softmax_workspace_size(g, h) / 2)
            return arg_error(fn, "workspace smaller than half of igr_att_softmax_workspace_size");
        const bool chunked = workspace != nullptr && has_row_plan(g) && g->n_chunks > 0 && g->split_ptr != nullptr;
        if (g->n_rows == 0) return IGR_OK;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const bool wide = wide_rows(g);
        const bool planned = split_plan(g);
        const int64_t nr = planned ? g->n_order : g->n_rows;
        const int32_t *order = planned ? g->order : nullptr;
        const dim3 g16((unsigned)((nr + 15) / 16)), g64((unsigned)((nr + 3) / 4));
        const bool vec = (reinterpret_cast<uintptr_t>(alpha) & 15u) == 0;
#define IGR_SMB(HH, RR)                                                                                           \
    do {                                                                                                          \
        if (nr > 0) {                                                                                             \
            if (wide)                                                                                             \
                hipLaunchKernelGGL((att_softmax_bwd_g16_kernel<HH, RR, 64>), g64, dim3(256), 0, st, nr,          \
                                   g->row_ptr, g->edge_id, alpha, keep, sqrt_d, row_max, row_sum, dw, dalpha,     \
                                   order);                                                                       \
            else                                                                                                  \
                hipLaunchKernelGGL((att_softmax_bwd_g16_kernel<HH, RR, 16>), g16, dim3(256), 0, st, nr,          \
                                   g->row_ptr, g->edge_id, alpha, keep, sqrt_d, row_max, row_sum, dw, dalpha,     \
                                   order);                                                                       \
        }                                                                                                         \
        if (planned && chunked) {                                                                                 \
            const dim3 gc((unsigned)((g->n_chunks + 3) / 4)), gs((unsigned)((g->n_split + 3) / 4));               \
            hipLaunchKernelGGL((att_softmax_bwd_chunk_sums_kernel<HH>), gc, dim3(256), 0, st, row_plan_of(g),     \
                               g->row_ptr, g->edge_id, alpha, keep, sqrt_d, row_max, row_sum, dw, workspace);     \
            hipLaunchKernelGGL((att_softmax_bwd_row_sums_kernel<HH>), gs, dim3(256), 0, st, g->n_split,           \
                               g->split_ptr, workspace);                                                          \
            hipLaunchKernelGGL((att_softmax_bwd_chunk_write_kernel<HH>), gc, dim3(256), 0, st, row_plan_of(g),    \
                               g->row_ptr, g->edge_id, alpha, keep, sqrt_d, row_max, row_sum, dw, workspace,      \
                               dalpha);                                                                           \
        } else if (planned)                                                                                       \
            hipLaunchKernelGGL((att_softmax_bwd_block_kernel<HH, kSoftmaxBlock, kSoftmaxBlockR>),                 \
                               dim3((unsigned)g->n_split), dim3(kSoftmaxBlock), 0, st, g->n_split, g->split_row,  \
                               g->row_ptr, g->edge_id, alpha, keep, sqrt_d, row_max, row_sum, dw, dalpha);        \
    } while (0)
        if (h == 1) IGR_SMB(1, IGR_SOFTMAX_R);
        else if (h == 2) IGR_SMB(2, IGR_SOFTMAX_R);
        else if (h == 4 && vec) IGR_SMB(4, IGR_SOFTMAX_R);
        else if (h == 8 && vec) IGR_SMB(8, (IGR_SOFTMAX_R + 1) / 2);
        else
            hipLaunchKernelGGL(att_softmax_bwd_kernel, dim3((unsigned)((g->n_rows + 3) / 4)), dim3(256),
                               0, st, g->n_rows, h, g->row_ptr, g->edge_id, alpha, keep, sqrt_d, row_max,
                               row_sum, dw, dalpha);
#undef IGR_SMB
        return launch_status(fn);
    });
}

extern "C" int igr_edge_dropout_f32(int64_t n, const float *val, const float *rand, float p,
                                    float *out, void *stream) {
    return guarded("igr_edge_dropout_f32", [&]() -> int {
        if (!(p >= 0.f && p < 1.f)) return arg_error("igr_edge_dropout_f32", "p must be in [0, 1)");
        if (n <= 0) return IGR_OK;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const float keep = (float)(1.0 - (double)p);
        hipLaunchKernelGGL(edge_dropout_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, n, val,
                           rand, keep, out);
        return launch_status("igr_edge_dropout_f32");
    });
}

extern "C" int igr_feat_values_f32(int64_t n_rows, const int64_t *row_ptr, const float *row_sum,
                                   float exponent, float *out, void *stream) {
    return guarded("igr_feat_values_f32", [&]() -> int {
        if (n_rows <= 0) return IGR_OK;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        if (row_ptr)  // per edge; the edge count is row_ptr[n_rows], read on the device
            hipLaunchKernelGGL(feat_values_edges_kernel, dim3(grid_for(n_rows * 16, 256)), dim3(256), 0, st, n_rows,
                               row_ptr, row_sum, exponent, out);
        else
            hipLaunchKernelGGL(feat_values_kernel, dim3(grid_for(n_rows, 256)), dim3(256), 0, st, n_rows, row_sum,
                               exponent, out);
        return launch_status("igr_feat_values_f32");
    });
}
