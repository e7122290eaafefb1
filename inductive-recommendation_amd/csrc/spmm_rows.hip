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
#include <algorithm>

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

// ------------------------------------------------------------------ masked pull
// The transpose of spmm_rows without atomics: mark the selected rows in a
// bitmap (n/32 words: 137 KB at 1.1M rows, L2-resident), sum repeated rows
// into one slot each (agg; igr_rowset_sum_f32 in rowsort.hip: sorted, fixed
// order), then every output row c streams its column
// indices, tests their bits and gathers agg only on hits:
//   out[c] = scale (sum_{p in row c, col[p] marked} rhs[p] agg[slot[col[p]]]
//                   + self_add * [c marked] agg[slot[c]])
// Run on the reverse graph this is dst = A^T G (+ G) for G = the selected rows'
// gradients; every summation order is fixed (bitwise reproducible).
namespace igr {

// LDS filter of the marked set: bit (r mod 2^19), 64 KB - two 1024-thread
// workgroups per CU hold it in LDS, so the per-edge probe never leaves the CU;
// only filter hits (the marked rows plus ~n_sel/2^19 false positives) probe
// the exact bitmap in L2.
constexpr int kFilterLog2 = 19;
constexpr uint32_t kFilterMask = (1u << kFilterLog2) - 1;
constexpr int kFilterWords = (1 << kFilterLog2) / 32;

__global__ void rowset_mark_kernel(int64_t n, const int64_t *__restrict__ rows, uint32_t *__restrict__ bits,
                                   uint32_t *__restrict__ filter) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t r = rows[i];
    atomicOr(bits + (r >> 5), 1u << (r & 31));
    const uint32_t h = (uint32_t)r & kFilterMask;
    atomicOr(filter + (h >> 5), 1u << (h & 31));
}

// bits |= every column of the selected rows (and the row ids themselves when
// self_mark); one wave per selected row
__global__ __launch_bounds__(256) void rowset_mark_neighbors_kernel(int64_t n, const int64_t *__restrict__ rows,
                                                                    const int64_t *__restrict__ row_ptr,
                                                                    const int32_t *__restrict__ col,
                                                                    uint32_t *__restrict__ bits, int self_mark) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const int lane = threadIdx.x & 63;
    const int64_t r = rows[i];
    if (self_mark && lane == 0) atomicOr(bits + (r >> 5), 1u << (r & 31));
    for (int64_t p = row_ptr[r] + lane; p < row_ptr[r + 1]; p += 64) {
        const uint32_t c = (uint32_t)col[p];
        atomicOr(bits + (c >> 5), 1u << (c & 31));
    }
}

// Byte-map form of the marking: plain idempotent byte stores instead of
// same-word atomics (a batch's ~10^6 neighbour marks land on ~3*10^4 bitmap
// words), then one pass packs the bytes into the bitmap and re-zeroes them.
__global__ __launch_bounds__(256) void rowset_mark_neighbors_bytes_kernel(int64_t n, const int64_t *__restrict__ rows,
                                                                          const int64_t *__restrict__ row_ptr,
                                                                          const int32_t *__restrict__ col,
                                                                          uint8_t *__restrict__ bytes, int self_mark) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const int lane = threadIdx.x & 63;
    const int64_t r = rows[i];
    if (self_mark && lane == 0) bytes[r] = 1;
    for (int64_t p = row_ptr[r] + lane; p < row_ptr[r + 1]; p += 64) bytes[col[p]] = 1;
}

// bits[w] |= the 32 bytes of word w (one thread per word); the bytes go back to 0
__global__ void pack_bytes_kernel(int64_t n, uint8_t *__restrict__ bytes, uint32_t *__restrict__ bits) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w * 32 >= n) return;
    uint32_t m = 0;
    if (w * 32 + 32 <= n) {
        uint4 *q = reinterpret_cast<uint4 *>(bytes + w * 32);
        const uint4 a = q[0], b = q[1];
        const uint32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) m |= (((v[k] >> (8 * j)) & 0xffu) ? 1u : 0u) << (4 * k + j);
        if (m) {
            q[0] = make_uint4(0, 0, 0, 0);
            q[1] = make_uint4(0, 0, 0, 0);
        }
    } else {
        for (int64_t k = w * 32; k < n; ++k) {
            if (bytes[k]) {
                m |= 1u << (k - w * 32);
                bytes[k] = 0;
            }
        }
    }
    if (m) bits[w] |= m;
}

__global__ void bitmap_set_kernel(int64_t n, const int64_t *__restrict__ idx, uint32_t *__restrict__ bits) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t r = idx[i];
    atomicOr(bits + (r >> 5), 1u << (r & 31));
}

__global__ void rowset_clear_kernel(int64_t n, const int64_t *__restrict__ rows, uint32_t *__restrict__ bits,
                                    uint32_t *__restrict__ filter) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t r = rows[i];
    bits[r >> 5] = 0u;  // every bit set in these words belongs to a selected row
    filter[((uint32_t)r & kFilterMask) >> 5] = 0u;
}

template <int D>
__global__ __launch_bounds__(1024) void spmm_pull_marked_kernel(
    int64_t n_rows, const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
    const float *__restrict__ val, const uint32_t *__restrict__ bits, const uint32_t *__restrict__ filter,
    int exact_filter, const int32_t *__restrict__ slot, const float *__restrict__ agg, int64_t ld_agg,
    float *__restrict__ out, int64_t ldo, float scale, int self_add, const uint32_t *__restrict__ row_mask) {
    constexpr int LPR = D / 4;  // lanes per row, one float4 each
    constexpr int RPB = 1024 / LPR;  // rows per workgroup pass
    constexpr int U = 4;  // blocks of LPR edges per trip (independent loads in flight)
    __shared__ uint32_t sf[kFilterWords];
    for (int k = threadIdx.x; k < kFilterWords / 4; k += 1024)
        reinterpret_cast<uint4 *>(sf)[k] = reinterpret_cast<const uint4 *>(filter)[k];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int sub = lane & (LPR - 1);
    const int gbase = lane - sub;  // first lane of this row's group within the wave
    const uint64_t gmask = LPR == 64 ? ~0ull : ((1ull << LPR) - 1);
    // persistent: the grid strides over row passes (every wave runs the same trip count)
    for (int64_t r0 = (int64_t)blockIdx.x * RPB; r0 < n_rows; r0 += (int64_t)gridDim.x * RPB) {
        const int64_t r = r0 + threadIdx.x / LPR;
        // rows outside row_mask are neither read nor written (trip count 0)
        const bool live = r < n_rows && (!row_mask || ((row_mask[r >> 5] >> (r & 31)) & 1u));
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        int64_t b = 0, e = 0;
        if (live) {
            b = row_ptr[r];
            e = row_ptr[r + 1];
            if (self_add && ((bits[r >> 5] >> (r & 31)) & 1u))
                acc = *reinterpret_cast<const float4 *>(agg + (int64_t)slot[r] * ld_agg + sub * 4);
        }
        int64_t len = e - b;  // uniform trip count across the wave (shuffles need every lane)
        for (int o = 32; o >= 1; o >>= 1) len = max(len, (int64_t)__shfl_xor((long long)len, o, 64));
        for (int64_t k = 0; k < len; k += LPR * U) {
            int cu[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t p = b + k + u * LPR + sub;
                cu[u] = p < e ? col[p] : -1;
            }
            bool hu[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t h = (uint32_t)cu[u] & kFilterMask;
                hu[u] = cu[u] >= 0 && ((sf[h >> 5] >> (h & 31)) & 1u);
            }
            if (!exact_filter) {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (hu[u]) hu[u] = (bits[cu[u] >> 5] >> (cu[u] & 31)) & 1u;
            }
            // hit lanes fetch their slot and edge value in parallel
            int su[U];
            float vu[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                su[u] = hu[u] ? slot[cu[u]] : 0;
                vu[u] = hu[u] ? (val ? val[b + k + u * LPR + sub] : 1.f) : 0.f;
            }
            // hits applied in CSR order (block u, then lane j): fixed summation order
#pragma unroll
            for (int u = 0; u < U; ++u) {
                uint64_t hit = (__ballot(hu[u]) >> gbase) & gmask;
                while (__builtin_amdgcn_readfirstlane((int)(__ballot(hit != 0) != 0))) {
                    // each group walks its own hits two at a time (both agg rows in flight)
                    const int j1 = hit ? __builtin_ctzll(hit) : 0;
                    const uint64_t rest = hit & (hit - 1);
                    const int j2 = rest ? __builtin_ctzll(rest) : j1;
                    const int s1 = __shfl(su[u], gbase + j1, 64), s2 = __shfl(su[u], gbase + j2, 64);
                    const float w1 = __shfl(vu[u], gbase + j1, 64), w2 = __shfl(vu[u], gbase + j2, 64);
                    if (hit) {
                        const float4 a1 = *reinterpret_cast<const float4 *>(agg + (int64_t)s1 * ld_agg + sub * 4);
                        if (rest) {
                            const float4 a2 =
                                *reinterpret_cast<const float4 *>(agg + (int64_t)s2 * ld_agg + sub * 4);
                            acc = f4_fma(w1, a1, acc);
                            acc = f4_fma(w2, a2, acc);
                            hit = rest & (rest - 1);
                        } else {
                            acc = f4_fma(w1, a1, acc);
                            hit = 0;
                        }
                    }
                }
            }
        }
        if (live) *reinterpret_cast<float4 *>(out + r * ldo + sub * 4) = f4_scale(scale, acc);
    }
}

}  // namespace igr

static unsigned blocks_for(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

extern "C" int igr_rowset_mark(int64_t n_sel, const int64_t *rows, uint32_t *bits, uint32_t *filter, void *stream) {
    return guarded("igr_rowset_mark", [&]() -> int {
        if (n_sel <= 0) return IGR_OK;
        if (!rows || !bits || !filter) return arg_error("igr_rowset_mark", "NULL pointer");
        if (n_sel > 2147483647) return arg_error("igr_rowset_mark", "too many rows");
        hipLaunchKernelGGL(rowset_mark_kernel, dim3(blocks_for(n_sel, 256)), dim3(256), 0,
                           reinterpret_cast<hipStream_t>(stream), n_sel, rows, bits, filter);
        return launch_status("igr_rowset_mark");
    });
}

extern "C" int igr_rowset_mark_neighbors(const igr_csr *g, int64_t n_sel, const int64_t *rows, uint32_t *bits,
                                         int32_t self_mark, uint8_t *scratch, void *stream) {
    return guarded("igr_rowset_mark_neighbors", [&]() -> int {
        if (!g) return arg_error("igr_rowset_mark_neighbors", "graph is NULL");
        if (n_sel <= 0) return IGR_OK;
        if (!rows || !bits) return arg_error("igr_rowset_mark_neighbors", "NULL pointer");
        if (self_mark && g->n_rows != g->n_cols)
            return arg_error("igr_rowset_mark_neighbors", "self_mark needs a square graph");
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        if (scratch) {
            if (!aligned16(scratch)) return arg_error("igr_rowset_mark_neighbors", "scratch must be 16-byte aligned");
            hipLaunchKernelGGL(rowset_mark_neighbors_bytes_kernel, dim3(blocks_for(n_sel, 4)), dim3(256), 0, st,
                               n_sel, rows, g->row_ptr, g->col_idx, scratch, self_mark ? 1 : 0);
            hipLaunchKernelGGL(pack_bytes_kernel, dim3(blocks_for((g->n_cols + 31) / 32, 256)), dim3(256), 0, st,
                               g->n_cols, scratch, bits);
        } else {
            hipLaunchKernelGGL(rowset_mark_neighbors_kernel, dim3(blocks_for(n_sel, 4)), dim3(256), 0, st, n_sel,
                               rows, g->row_ptr, g->col_idx, bits, self_mark ? 1 : 0);
        }
        return launch_status("igr_rowset_mark_neighbors");
    });
}

extern "C" int igr_bitmap_set(int64_t n, const int64_t *idx, uint32_t *bits, void *stream) {
    return guarded("igr_bitmap_set", [&]() -> int {
        if (n <= 0) return IGR_OK;
        if (!idx || !bits) return arg_error("igr_bitmap_set", "NULL pointer");
        hipLaunchKernelGGL(bitmap_set_kernel, dim3(blocks_for(n, 256)), dim3(256), 0,
                           reinterpret_cast<hipStream_t>(stream), n, idx, bits);
        return launch_status("igr_bitmap_set");
    });
}

extern "C" int igr_rowset_clear(int64_t n_sel, const int64_t *rows, uint32_t *bits, uint32_t *filter,
                                void *stream) {
    return guarded("igr_rowset_clear", [&]() -> int {
        if (n_sel <= 0) return IGR_OK;
        if (!rows || !bits || !filter) return arg_error("igr_rowset_clear", "NULL pointer");
        hipLaunchKernelGGL(rowset_clear_kernel, dim3(blocks_for(n_sel, 256)), dim3(256), 0,
                           reinterpret_cast<hipStream_t>(stream), n_sel, rows, bits, filter);
        return launch_status("igr_rowset_clear");
    });
}

extern "C" int igr_spmm_pull_marked_f32(const igr_csr *g, int32_t d, const uint32_t *bits, const uint32_t *filter,
                                        const int32_t *slot, const float *agg, int64_t ld_agg, const float *rhs,
                                        float scale, int32_t self_add, const uint32_t *row_mask, float *out,
                                        int64_t ldo, void *stream) {
    return guarded("igr_spmm_pull_marked_f32", [&]() -> int {
        const char *fn = "igr_spmm_pull_marked_f32";
        if (!g || !bits || !filter || !slot) return arg_error(fn, "graph / bits / filter / slot NULL");
        if (g->edge_id && rhs) return arg_error(fn, "rhs by edge id with an edge_id permutation is not supported");
        if (self_add && g->n_rows > g->n_cols) return arg_error(fn, "self_add needs a square graph");
        if (ld_agg < d || ldo < d || ld_agg % 4 || ldo % 4 || !aligned16(agg) || !aligned16(out))
            return arg_error(fn, "agg / out must be 16-byte aligned with leading dims >= d, multiple of 4");
        if (g->n_rows <= 0) return IGR_OK;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const int64_t n = g->n_rows;
        // the filter is exact when every column index fits in it
        const int exact = g->n_cols <= (int64_t(1) << kFilterLog2);
        // persistent grid: two 1024-thread workgroups (2 x 64 KB of filter) per CU
        static int cus = 0;
        if (cus <= 0) {
            int dev = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
                cus = 256;
        }
#define IGR_PULL(DD)                                                                                               \
    hipLaunchKernelGGL((spmm_pull_marked_kernel<DD>),                                                             \
                       dim3((unsigned)std::min<int64_t>(2 * (int64_t)cus, blocks_for(n, 1024 / (DD / 4)))),       \
                       dim3(1024), 0, st, n, g->row_ptr, g->col_idx, rhs, bits, filter, exact, slot, agg, ld_agg, \
                       out, ldo, scale, (int)self_add, row_mask)
        switch (d) {
            case 32: IGR_PULL(32); break;
            case 64: IGR_PULL(64); break;
            case 128: IGR_PULL(128); break;
            case 256: IGR_PULL(256); break;
            default: return arg_error(fn, "d must be 32, 64, 128 or 256");
        }
#undef IGR_PULL
        return launch_status(fn);
    });
}
