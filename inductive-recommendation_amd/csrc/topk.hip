// topk.hip - the eval ranking: train-item mask + per-user top-k of the score rows.
//
// BasicTrainer.eval (trainer.py:146-182): scores = rep[users] . rep[items]^T
// (igr_gemm_f32), scores[u, train items of u] = -inf, then topk(k = max topks)
// per user.  Here:
//   igr_mask_scores_f32: scores[r, cols[p]] = -inf for p in [row_ptr[r], row_ptr[r+1])
//   igr_topk_f32:        per row the k largest scores, sorted (value desc, index asc)
// One workgroup per row.  The k-th largest value is found by an 8-bit radix
// select on the order-preserving uint32 key of the float (4 histogram passes
// over the row, each restricted to the prefix chosen so far); if several
// elements share that key, a second radix select on the index picks the
// smallest indices among them, so the result is deterministic.  One pass then
// collects exactly k (key, index) pairs into LDS and a bitonic sort orders them.
#include "common.h"

namespace igr {

constexpr int kTopkThreads = 256;
constexpr int kTopkMax = 1024;  // k <= kTopkMax (LDS sort buffer)

// -0.0 and +0.0 compare equal (as in torch / numpy): f + 0.0f maps -0.0 to +0.0
__device__ __forceinline__ uint32_t order_key(float f) {
    const uint32_t u = __float_as_uint(f + 0.0f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Radix select: among row elements with pred(j) true, the `need`-th largest of
// kfn(j).  Returns the key and sets *left = how many elements equal to it are
// still needed (1 .. need).  hist: 256 LDS ints; shared scalars in sh[0..1].
template <class KeyFn, class Pred>
__device__ uint32_t radix_select(int64_t n, KeyFn kfn, Pred pred, int need, int *hist, int *sh, int *left) {
    uint32_t prefix = 0, pmask = 0;
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int b = threadIdx.x; b < 256; b += kTopkThreads) hist[b] = 0;
        __syncthreads();
        for (int64_t j = threadIdx.x; j < n; j += kTopkThreads) {
            if (!pred(j)) continue;
            const uint32_t key = kfn(j);
            if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 0xff], 1);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int acc = 0, digit = 0;
            for (int b = 255; b >= 0; --b) {
                if (acc + hist[b] >= need) {
                    digit = b;
                    break;
                }
                acc += hist[b];
            }
            sh[0] = digit;
            sh[1] = need - acc;
        }
        __syncthreads();
        prefix |= (uint32_t)sh[0] << shift;
        pmask |= 0xffu << shift;
        need = sh[1];
        __syncthreads();
    }
    *left = need;
    return prefix;
}

__global__ __launch_bounds__(kTopkThreads) void topk_kernel(int64_t n_rows, int64_t n_cols,
                                                            const float *__restrict__ scores, int64_t ld, int k,
                                                            float *__restrict__ out_val, int64_t *__restrict__ out_idx) {
    __shared__ int hist[256];
    __shared__ int sh[4];
    __shared__ uint32_t skey[kTopkMax];
    __shared__ int32_t sidx[kTopkMax];
    const int64_t r = blockIdx.x;
    if (r >= n_rows) return;
    const float *row = scores + r * ld;
    auto vkey = [&](int64_t j) { return order_key(row[j]); };
    auto all = [](int64_t) { return true; };
    int left;
    const uint32_t T = radix_select(n_cols, vkey, all, k, hist, sh, &left);
    // among elements equal to T, the `left` smallest indices (largest ~index)
    bool all_ties = true;  // accept every tie unless more than `left` exist
    uint32_t TI = 0u;
    {
        if (threadIdx.x == 0) sh[2] = 0;
        __syncthreads();
        int cnt = 0;
        for (int64_t j = threadIdx.x; j < n_cols; j += kTopkThreads) cnt += (vkey(j) == T);
        atomicAdd(&sh[2], cnt);
        __syncthreads();
        const int ties = sh[2];
        __syncthreads();
        if (ties > left) {
            all_ties = false;
            int dummy;
            TI = radix_select(
                n_cols, [](int64_t j) { return ~(uint32_t)j; }, [&](int64_t j) { return vkey(j) == T; }, left, hist,
                sh, &dummy);
        }
    }
    // collect exactly k elements: key > T, or key == T (all of them, or those with ~index >= TI)
    if (threadIdx.x == 0) sh[3] = 0;
    __syncthreads();
    for (int64_t j = threadIdx.x; j < n_cols; j += kTopkThreads) {
        const uint32_t key = vkey(j);
        const bool take = key > T || (key == T && (all_ties || ~(uint32_t)j >= TI));
        if (take) {
            const int s = atomicAdd(&sh[3], 1);
            if (s < kTopkMax) {
                skey[s] = key;
                sidx[s] = (int32_t)j;
            }
        }
    }
    __syncthreads();
    int m = 1;
    while (m < k) m <<= 1;
    for (int s = k + threadIdx.x; s < m; s += kTopkThreads) {  // pad: sorts after every real element
        skey[s] = 0u;
        sidx[s] = 0x7fffffff;
    }
    __syncthreads();
    // bitonic sort, descending by key, ascending by index among equal keys
    for (int size = 2; size <= m; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = threadIdx.x; t < m / 2; t += kTopkThreads) {
                const int i = 2 * stride * (t / stride) + (t % stride);
                const int j = i + stride;
                const bool desc = ((i & size) == 0);
                const uint32_t ki = skey[i], kj = skey[j];
                const int32_t ii = sidx[i], ij = sidx[j];
                const bool i_first = ki > kj || (ki == kj && ii < ij);  // i ranks before j
                if (desc != i_first) {
                    skey[i] = kj;
                    skey[j] = ki;
                    sidx[i] = ij;
                    sidx[j] = ii;
                }
            }
            __syncthreads();
        }
    }
    for (int s = threadIdx.x; s < k; s += kTopkThreads) {
        if (out_val) out_val[r * k + s] = row[sidx[s]];  // the row's own bits
        out_idx[r * k + s] = sidx[s];
    }
}

__global__ void mask_scores_kernel(int64_t n_rows, const int64_t *__restrict__ row_ptr,
                                   const int32_t *__restrict__ cols, float *__restrict__ scores, int64_t ld) {
    const int64_t r = blockIdx.x;
    if (r >= n_rows) return;
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    for (int64_t p = b + threadIdx.x; p < e; p += blockDim.x) scores[r * ld + cols[p]] = -__builtin_huge_valf();
}

}  // namespace igr

using namespace igr;

extern "C" int igr_mask_scores_f32(int64_t n_rows, const int64_t *row_ptr, const int32_t *cols, float *scores,
                                   int64_t ld, void *stream) {
    return guarded("igr_mask_scores_f32", [&]() -> int {
        if (n_rows <= 0) return IGR_OK;
        if (!row_ptr || !scores) return arg_error("igr_mask_scores_f32", "NULL pointer");
        if (n_rows > 2147483647) return arg_error("igr_mask_scores_f32", "too many rows");
        hipLaunchKernelGGL(mask_scores_kernel, dim3((unsigned)n_rows), dim3(256), 0,
                           reinterpret_cast<hipStream_t>(stream), n_rows, row_ptr, cols, scores, ld);
        return launch_status("igr_mask_scores_f32");
    });
}

extern "C" int igr_topk_f32(int64_t n_rows, int64_t n_cols, const float *scores, int64_t ld, int32_t k,
                            float *out_val, int64_t *out_idx, void *stream) {
    return guarded("igr_topk_f32", [&]() -> int {
        const char *fn = "igr_topk_f32";
        if (k < 1 || k > kTopkMax) return arg_error(fn, "k must be in [1, 1024]");
        if (n_cols < k) return arg_error(fn, "k larger than the number of columns");
        if (n_cols > 2147483647) return arg_error(fn, "too many columns");
        if (ld < n_cols) return arg_error(fn, "ld < n_cols");
        if (n_rows <= 0) return IGR_OK;
        if (!scores || !out_idx) return arg_error(fn, "NULL pointer");
        if (n_rows > 2147483647) return arg_error(fn, "too many rows");
        hipLaunchKernelGGL(topk_kernel, dim3((unsigned)n_rows), dim3(kTopkThreads), 0,
                           reinterpret_cast<hipStream_t>(stream), n_rows, n_cols, scores, ld, (int)k, out_val,
                           out_idx);
        return launch_status(fn);
    });
}
