// spmm_rows.hip - SpMM restricted to a set of rows, and its transpose (push).
//
// The training step only reads the representation at the batch rows
// (rep[users], rep[n_users + pos/neg], model.py:4048-4049), so the LAST
// propagation layer of IGCN / LightGCN.get_rep (model.py:4196, 106) is needed
// only there, and the FIRST layer of its backward only pushes from there:
//   igr_spmm_rows_f32: out[i] = scale (sum_{p in row rows[i]} w(p) x[col[p]]
//                                      + add_g[rows[i]] + add_i[i])
//   igr_spmm_push_f32: dst[col[p]] += scale w(p) src[i]  for p in row rows[i]
//                      (+ dst[rows[i]] += scale src[i] with self_add)
// rows may repeat (both are linear in the selected rows).
// One workgroup per selected row: its 256/(d/4) lane groups stride the row's
// edges in 16-edge blocks, so a hub row is spread over the whole workgroup.
// rows_f32 reduces the groups through LDS in a fixed order (deterministic);
// push_f32 adds with float atomics (order of adds not fixed).
#include "common.h"

namespace igr {

template <int D>
__global__ __launch_bounds__(256) void spmm_rows_kernel(const int64_t *__restrict__ row_ptr,
                                                        const int32_t *__restrict__ col,
                                                        const float *__restrict__ val,
                                                        const int64_t *__restrict__ rows, int64_t n_sel,
                                                        const float *__restrict__ x, int64_t ldx,
                                                        const float *__restrict__ add_g, int64_t ld_g,
                                                        const float *__restrict__ add_i, int64_t ld_i,
                                                        float *__restrict__ out, int64_t ldo, float scale) {
    constexpr int LPR = D / 4;
    constexpr int NG = 256 / LPR;  // lane groups per workgroup
    __shared__ float4 red[NG][LPR];
    const int grp = threadIdx.x / LPR;
    const int sub = threadIdx.x - grp * LPR;
    const int64_t i = blockIdx.x;
    if (i >= n_sel) return;
    const int64_t r = rows[i];
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    // group g takes edges b + g, b + g + NG, ... (loads independent, NG in flight per step)
    for (int64_t p = b + grp; p < e; p += NG) {
        const float w = val ? val[p] : 1.f;
        const float4 xv = *reinterpret_cast<const float4 *>(x + (int64_t)col[p] * ldx + sub * 4);
        acc = f4_fma(w, xv, acc);
    }
    red[grp][sub] = acc;
    __syncthreads();
#pragma unroll
    for (int s = NG / 2; s >= 1; s >>= 1) {
        if (grp < s) red[grp][sub] = f4_add(red[grp][sub], red[grp + s][sub]);
        __syncthreads();
    }
    if (grp == 0) {
        float4 v = red[0][sub];
        if (add_g) v = f4_add(v, *reinterpret_cast<const float4 *>(add_g + r * ld_g + sub * 4));
        if (add_i) v = f4_add(v, *reinterpret_cast<const float4 *>(add_i + i * ld_i + sub * 4));
        *reinterpret_cast<float4 *>(out + i * ldo + sub * 4) = f4_scale(scale, v);
    }
}

template <int D>
__global__ __launch_bounds__(256) void spmm_push_kernel(const int64_t *__restrict__ row_ptr,
                                                        const int32_t *__restrict__ col,
                                                        const float *__restrict__ val,
                                                        const int64_t *__restrict__ rows, int64_t n_sel,
                                                        const float *__restrict__ src, int64_t lds,
                                                        float *__restrict__ dst, int64_t ldd, float scale,
                                                        int self_add) {
    constexpr int LPR = D / 4;
    constexpr int NG = 256 / LPR;
    const int grp = threadIdx.x / LPR;
    const int sub = threadIdx.x - grp * LPR;
    const int64_t i = blockIdx.x;
    if (i >= n_sel) return;
    const int64_t r = rows[i];
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    const float4 sv = f4_scale(scale, *reinterpret_cast<const float4 *>(src + i * lds + sub * 4));
    if (self_add && grp == 0) {
        float *o = dst + r * ldd + sub * 4;
        atomicAdd(o + 0, sv.x);
        atomicAdd(o + 1, sv.y);
        atomicAdd(o + 2, sv.z);
        atomicAdd(o + 3, sv.w);
    }
    for (int64_t p = b + grp; p < e; p += NG) {
        const float w = val ? val[p] : 1.f;
        float *o = dst + (int64_t)col[p] * ldd + sub * 4;
        atomicAdd(o + 0, w * sv.x);
        atomicAdd(o + 1, w * sv.y);
        atomicAdd(o + 2, w * sv.z);
        atomicAdd(o + 3, w * sv.w);
    }
}

// Launch kernel template K at d in {32, 64, 128, 256}; false for other widths.
#define IGR_ROWS_DISPATCH(K, d, grid, st, ...)                                                        \
    [&]() -> bool {                                                                                  \
        switch (d) {                                                                                 \
            case 32: hipLaunchKernelGGL((K<32>), grid, dim3(256), 0, st, __VA_ARGS__); return true;   \
            case 64: hipLaunchKernelGGL((K<64>), grid, dim3(256), 0, st, __VA_ARGS__); return true;   \
            case 128: hipLaunchKernelGGL((K<128>), grid, dim3(256), 0, st, __VA_ARGS__); return true; \
            case 256: hipLaunchKernelGGL((K<256>), grid, dim3(256), 0, st, __VA_ARGS__); return true; \
            default: return false;                                                                   \
        }                                                                                            \
    }()

}  // namespace igr

using namespace igr;

extern "C" int igr_spmm_rows_f32(const igr_csr *g, int32_t d, const int64_t *rows, int64_t n_sel, const float *x,
                                 int64_t ldx, const float *rhs, const float *add_g, int64_t ld_g, const float *add_i,
                                 int64_t ld_i, float scale, float *out, int64_t ldo, void *stream) {
    return guarded("igr_spmm_rows_f32", [&]() -> int {
        const char *fn = "igr_spmm_rows_f32";
        if (!g || !rows) return arg_error(fn, "graph / rows NULL");
        if (g->edge_id && rhs) return arg_error(fn, "rhs by edge id with an edge_id permutation is not supported");
        if (ldx < d || ldo < d || ldx % 4 || ldo % 4 || !aligned16(x) || !aligned16(out))
            return arg_error(fn, "x / out must be 16-byte aligned with leading dims >= d, multiple of 4");
        if ((add_g && (ld_g < d || ld_g % 4 || !aligned16(add_g))) || (add_i && (ld_i < d || ld_i % 4 || !aligned16(add_i))))
            return arg_error(fn, "add_g / add_i must be 16-byte aligned with leading dims >= d, multiple of 4");
        if (n_sel <= 0) return IGR_OK;
        if (n_sel > 2147483647) return arg_error(fn, "too many rows");
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        if (!IGR_ROWS_DISPATCH(spmm_rows_kernel, d, dim3((unsigned)n_sel), st, g->row_ptr, g->col_idx, rhs, rows, n_sel,
                                           x, ldx, add_g, ld_g, add_i, ld_i, out, ldo, scale))
            return arg_error(fn, "d must be 32, 64, 128 or 256");
        return launch_status(fn);
    });
}

extern "C" int igr_spmm_push_f32(const igr_csr *g, int32_t d, const int64_t *rows, int64_t n_sel, const float *src,
                                 int64_t lds, const float *rhs, float scale, int32_t self_add, float *dst, int64_t ldd,
                                 void *stream) {
    return guarded("igr_spmm_push_f32", [&]() -> int {
        const char *fn = "igr_spmm_push_f32";
        if (!g || !rows) return arg_error(fn, "graph / rows NULL");
        if (g->edge_id && rhs) return arg_error(fn, "rhs by edge id with an edge_id permutation is not supported");
        if (lds < d || ldd < d || lds % 4 || !aligned16(src)) return arg_error(fn, "bad src / dst layout");
        if (self_add && g->n_rows > g->n_cols) return arg_error(fn, "self_add needs a square graph");
        if (n_sel <= 0) return IGR_OK;
        if (n_sel > 2147483647) return arg_error(fn, "too many rows");
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        if (!IGR_ROWS_DISPATCH(spmm_push_kernel, d, dim3((unsigned)n_sel), st, g->row_ptr, g->col_idx, rhs, rows, n_sel,
                                           src, lds, dst, ldd, scale, (int)self_add))
            return arg_error(fn, "d must be 32, 64, 128 or 256");
        return launch_status(fn);
    });
}
